"""The move table of the reference's `footsies_gym.moves` (moves.py:5-42) for code written against
it: `FootsiesMove` members carry (id, duration, startup, active, recovery) as `FootsiesMoveInfo`,
and the index <-> move maps follow the observation's move index order.

Every value comes from the game's own frame data (data/f00.json, extracted from the reference's
assets): duration = the action's frameCount, and for attacks startup / active / recovery = the
frames before, inside and after the windows of its non-proximity hitboxes.
tests/test_tables.py re-derives them from data/f00.json.
"""
from dataclasses import dataclass
from enum import Enum

from ._abi import MOVES


@dataclass(frozen=True)
class FootsiesMoveInfo:
    id: int
    duration: int
    startup: int
    active: int
    recovery: int


# (startup, active, recovery) of the attacks; every other action has none
_ATTACK_FRAMES = {"N_ATTACK": (4, 2, 16), "B_ATTACK": (3, 3, 15), "N_SPECIAL": (11, 4, 29), "B_SPECIAL": (2, 6, 47)}

FootsiesMove = Enum("FootsiesMove", [(name, FootsiesMoveInfo(mid, dur, *_ATTACK_FRAMES.get(name, (0, 0, 0))))
                                     for name, mid, dur in MOVES])


# the reference's phase tests (moves.py:31-38), by frame of the move
def _in_recovery(self, frame: int) -> bool:
    return frame >= (self.value.startup + self.value.active)


def _in_active(self, frame: int) -> bool:
    return self.value.startup <= frame < (self.value.startup + self.value.active)


def _in_startup(self, frame: int) -> bool:
    return frame < self.value.startup


FootsiesMove.in_recovery = _in_recovery
FootsiesMove.in_active = _in_active
FootsiesMove.in_startup = _in_startup

FOOTSIES_MOVE_INDEX_TO_MOVE = list(FootsiesMove)
FOOTSIES_MOVE_ID_TO_INDEX = {m.value.id: i for i, m in enumerate(FOOTSIES_MOVE_INDEX_TO_MOVE)}

__all__ = ["FootsiesMove", "FootsiesMoveInfo", "FOOTSIES_MOVE_INDEX_TO_MOVE", "FOOTSIES_MOVE_ID_TO_INDEX"]
