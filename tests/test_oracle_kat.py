"""Known-answer scenarios (tests/kat_scenarios.py) on the CPU oracle."""
import pytest

from footsies_gym_amd import _abi
from tests import kat_actors, kat_combat, kat_core, kat_geometry
from tests import kat_scenarios as kat


@pytest.mark.parametrize("name", sorted(kat.ALL))
def test_kat_oracle(oracle_lib, name):
    o = oracle_lib.Oracle(1, p2_mode=_abi.FS_P2_EXTERNAL, autoreset_mode=_abi.FS_AUTORESET_SAME_STEP)
    kat.ALL[name](o)


@pytest.mark.parametrize("name", sorted(kat_actors.ALL))
def test_kat_actors_oracle(oracle_lib, name):
    kat_actors.ALL[name](lambda p1, p2, seed: kat_actors.OracleActors(oracle_lib, p1, p2, seed))


@pytest.mark.parametrize("name", sorted(kat_combat.ALL))
def test_kat_combat_oracle(oracle_lib, name):
    kat_combat.ALL[name](kat_combat.OracleKat(oracle_lib))


@pytest.mark.parametrize("name", sorted(kat_core.ALL))
def test_kat_core_oracle(oracle_lib, name):
    """The sim-core paths pinned by hand-derived scenarios (tests/kat_core.py) on the oracle."""
    kat_core.ALL[name](kat_combat.OracleKat(oracle_lib))


@pytest.mark.parametrize("name", sorted(kat_geometry.ALL))
def test_kat_geometry_oracle(oracle_lib, name):
    """Fighters off the ground / facing the other way (tests/kat_geometry.py) on the oracle."""
    kat_geometry.ALL[name](kat_combat.OracleKat(oracle_lib))


def test_kat_core_covers_its_pin_table():
    from tests import kat_core as K
    assert set(K.ALL) == set(K.PINS)


def test_kat_bot_plans_oracle(oracle_lib):
    """The scripted bot's plan logic (tests/kat_bot.py: every distance bucket's draw and outcome
    map, the no-draw TwoHit rules, every plan's contents, the 1-call-old FightState) on the oracle."""
    from tests import kat_bot
    kat_bot.run(lambda n, p1: kat_bot.OracleBot(oracle_lib, n, p1))


def test_kat_bot_cases_cover_every_branch():
    """The sampled RNG states reach every outcome of every distance bucket (so the plan-logic KAT
    exercises each branch of AI:68-190), and the forced TwoHit rules hold with no draw."""
    from tests import kat_bot as K
    cov = K.coverage(K.build_cases())
    assert cov[("move", 0)] == {K.MP_FAR1, K.MP_FAR2}
    assert cov[("move", 1)] == {K.MP_MID1, K.MP_MID2, K.MP_FAR1, K.MP_FAR2, K.MP_NEUTRAL}
    assert cov[("move", 2)] == {K.MP_MID1, K.MP_MID2, K.MP_FALLBACK1, K.MP_FALLBACK2, K.MP_NEUTRAL}
    assert cov[("move", 3)] == cov[("move", 4)] == {K.MP_FALLBACK1, K.MP_FALLBACK2, K.MP_NEUTRAL}
    # d > 4 draws Random.Range(0, 4) and takes NoAttack for rand <= 3: always (AI:136-143), so
    # DelaySpecial is unreachable there -- but the draw is still taken
    assert cov[("attack", 0, False, False)] == {K.AP_NONE}
    assert cov[("attack", 1, False, False)] == {K.AP_NONE, K.AP_ONE_HIT, K.AP_DELAY_SPECIAL}
    assert cov[("attack", 1, False, True)] == {K.AP_TWO_HIT}
    assert cov[("attack", 0, False, True)] == {K.AP_NONE}  # N_ATTACK forces only at 3 < d <= 4
    assert cov[("attack", 2, False, False)] == {K.AP_NONE, K.AP_ONE_HIT, K.AP_TWO_HIT}
    assert cov[("attack", 3, False, False)] == {K.AP_ONE_HIT, K.AP_TWO_HIT, K.AP_IMMEDIATE_SPECIAL, K.AP_DELAY_SPECIAL}
    assert cov[("attack", 4, False, False)] == {K.AP_ONE_HIT, K.AP_TWO_HIT}
    for b in range(5):
        assert cov[("attack", b, True, False)] == {K.AP_TWO_HIT}
    # plan lengths as the C# builds them (AI:192-312)
    assert [len(K.move_plan(p)) for p in range(7)] == [30, 90, 56, 70, 33, 60, 63]
    assert [len(K.attack_plan(p)) for p in range(5)] == [30, 19, 23, 61, 121]
    assert K.move_plan(K.MP_FALLBACK2)[:4] == [K.L, 0, K.L, K.R]  # the "backward" dash is forward (AI:337-342)
    assert K.move_plan(K.MP_FALLBACK2, player1=True)[:4] == [K.R, 0, K.R, K.L]
