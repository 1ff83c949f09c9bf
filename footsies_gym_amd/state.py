"""The reference package's state module (footsies_gym/state.py): ``FootsiesState`` (the game's
EnvironmentState as the client decodes it, state.py:7-76) beside the BattleState classes, which
live in ``battle_state`` and are re-exported here under the reference's module path."""
import dataclasses

from .battle_state import FootsiesBattleState, FootsiesFighterState

__all__ = ["FootsiesState", "FootsiesBattleState", "FootsiesFighterState"]


def _action_bools(a):
    """A 3-bit input (Left 1, Right 2, Attack 4) as the (left, right, attack) tuple (state.py:26-36)."""
    a = int(a)
    return ((a & 1) != 0, (a & 2) != 0, (a & 4) != 0)


@dataclasses.dataclass
class FootsiesState:
    """The environment state of FOOTSIES (EnvironmentState.cs:12-26), with the field names and the
    most-recent-action decoding of the reference's FootsiesState (state.py:7-36)."""

    p1Vital: int
    p2Vital: int
    p1Guard: int
    p2Guard: int
    p1Move: int
    p2Move: int
    p1MoveFrame: int
    p2MoveFrame: int
    p1Position: float
    p2Position: float
    globalFrame: int
    p1MostRecentAction: "tuple[bool, bool, bool]"
    p2MostRecentAction: "tuple[bool, bool, bool]"
    p1Hitstun: int
    p2Hitstun: int

    def __post_init__(self):
        self.p1MostRecentAction = _action_bools(self.p1MostRecentAction)
        self.p2MostRecentAction = _action_bools(self.p2MostRecentAction)

    @staticmethod
    def from_battle_state(battle_state: FootsiesBattleState) -> "FootsiesState":
        """state.py:38-55: the fields a BattleState holds, input[0] as the most recent action."""
        p1, p2 = battle_state.p1State, battle_state.p2State
        return FootsiesState(
            p1Vital=p1.vitalHealth, p2Vital=p2.vitalHealth, p1Guard=p1.guardHealth, p2Guard=p2.guardHealth,
            p1Move=p1.currentActionID, p2Move=p2.currentActionID,
            p1MoveFrame=p1.currentActionFrame, p2MoveFrame=p2.currentActionFrame,
            p1Position=p1.position[0], p2Position=p2.position[0], globalFrame=battle_state.frameCount,
            p1MostRecentAction=p1.input[0], p2MostRecentAction=p2.input[0],
            p1Hitstun=p1.currentHitStunFrame, p2Hitstun=p2.currentHitStunFrame)

    @staticmethod
    def from_env_state(rec) -> "FootsiesState":
        """One ``fs_env_state`` record (``FootsiesSim.env_state()[i]``, the 15 fields of
        EnvironmentState.cs:12-26 that the game sends every frame)."""
        return FootsiesState(**{f: (float(rec[f]) if f.endswith("Position") else int(rec[f]))
                                for f in (fl.name for fl in dataclasses.fields(FootsiesState))})

    def __str__(self):
        """Detailed representation of the environment state (state.py:57-76)."""
        return f"""[P1]:
- Vital: {self.p1Vital}
- Guard: {self.p1Guard}
- Move: {self.p1Move}
- Move frame: {self.p1MoveFrame}
- Position: {self.p1Position}
[P2]:
- Vital: {self.p2Vital}
- Guard: {self.p2Guard}
- Move: {self.p2Move}
- Move frame: {self.p2MoveFrame}
- Position: {self.p2Position}
[Info]:
- Frame: {self.globalFrame}
- P1 most recent action: {self.p1MostRecentAction}
- P2 most recent action: {self.p2MostRecentAction}"""
