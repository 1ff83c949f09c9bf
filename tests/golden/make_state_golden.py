#!/usr/bin/env python3
"""Golden FootsiesState values from the REFERENCE's own client class (build container only).

For every BattleState of tests/golden/battle_state_golden.json (JSON written by
footsies_gym_amd.battle_state for oracle arenas), the reference's
FootsiesState.from_battle_state(FootsiesBattleState.from_json(...)) (footsies_gym/state.py:7-76)
is recorded as its field values and its str().  Output (committed): tests/golden/state_golden.json.
"""
import dataclasses
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "_gym_stub"))
sys.path.insert(0, "/root/reference/footsies-gym")

from footsies_gym.state import FootsiesBattleState, FootsiesState  # noqa: E402


def main():
    with open(os.path.join(HERE, "battle_state_golden.json")) as f:
        cases = json.load(f)
    out = []
    for i, c in enumerate(cases):
        s = FootsiesState.from_battle_state(FootsiesBattleState.from_json(c["ours"]))
        out.append({"case": i, "fields": dataclasses.asdict(s), "str": str(s)})
    with open(os.path.join(HERE, "state_golden.json"), "w") as f:
        json.dump(out, f)
    print("wrote", len(out), "cases")


if __name__ == "__main__":
    main()
