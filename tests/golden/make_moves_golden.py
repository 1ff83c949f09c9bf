#!/usr/bin/env python3
"""tests/golden/moves_golden.json from the REFERENCE's own `footsies_gym.moves` (build
container only; imported with the throwaway gymnasium stub, as make_golden.py does).

Records the move table (moves.py:12-28), the id -> index map (moves.py:41-42) and, for every
move and every frame 0 .. duration + 1, the reference's in_startup / in_active / in_recovery
answers (moves.py:30-38) as one 3-bit code per frame (bit 0 startup, 1 active, 2 recovery).
make_golden.py calls write() when it regenerates the FE vectors.
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REF_PY = "/root/reference/footsies-gym"


def table(ref_moves):
    return {
        "id_to_index": {str(k): v for k, v in ref_moves.FOOTSIES_MOVE_ID_TO_INDEX.items()},
        "moves": [[m.name, m.value.id, m.value.duration, m.value.startup, m.value.active, m.value.recovery]
                  for m in ref_moves.FootsiesMove],
        "phases": {m.name: [int(m.in_startup(f)) | (int(m.in_active(f)) << 1) | (int(m.in_recovery(f)) << 2)
                            for f in range(m.value.duration + 2)] for m in ref_moves.FootsiesMove},
    }


def write(ref_moves):
    with open(os.path.join(HERE, "moves_golden.json"), "w") as f:
        json.dump(table(ref_moves), f, indent=1)


if __name__ == "__main__":
    sys.path.insert(0, os.path.join(HERE, "_gym_stub"))
    sys.path.insert(0, REF_PY)
    import footsies_gym.moves as ref_moves  # noqa: E402
    write(ref_moves)
    print("wrote moves_golden.json")
