#!/usr/bin/env python3
"""Golden BattleState JSON pinned by the REFERENCE's own client class (build container only).

BattleState JSON written by footsies_gym_amd.battle_state for oracle arenas in varied
situations is parsed by the reference's FootsiesBattleState.from_json and written back
with its .json() (footsies_gym/state.py:78-137); the dataclass constructors reject any
missing or unknown field, so a successful round trip pins the schema (names, nesting,
types).  Output (committed): tests/golden/battle_state_golden.json.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(HERE, "_gym_stub"))
sys.path.insert(0, "/root/reference/footsies-gym")

from footsies_gym.state import FootsiesBattleState  # noqa: E402

from footsies_gym_amd import _abi, battle_state  # noqa: E402
from oracle import binding  # noqa: E402


def main():
    o = binding.Oracle(64, p2_mode=_abi.FS_P2_EXTERNAL, base_seed=9, autoreset_mode=_abi.FS_AUTORESET_NEXT_STEP)
    rng = np.random.default_rng(9)
    a1 = rng.integers(0, 8, 64)
    a2 = rng.integers(0, 8, 64)
    cases = []
    for t in range(900):
        a1 = np.where(rng.random(64) < 0.9, a1, rng.integers(0, 8, 64))
        a2 = np.where(rng.random(64) < 0.9, a2, rng.integers(0, 8, 64))
        o.step(a1.astype(np.uint8), a2.astype(np.uint8))
        if t % 150 == 149:
            st = o.state()
            for i in (0, 17, 40):
                ours = battle_state.dumps(battle_state.battle_state(st, i))
                ref = FootsiesBattleState.from_json(ours).json()
                cases.append({"ours": ours, "reference": ref})
    with open(os.path.join(HERE, "battle_state_golden.json"), "w") as f:
        json.dump(cases, f)
    print("wrote", len(cases), "cases")


if __name__ == "__main__":
    main()
