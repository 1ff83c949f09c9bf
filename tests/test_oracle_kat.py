"""Known-answer scenarios (tests/kat_scenarios.py) on the CPU oracle."""
import pytest

from footsies_gym_amd import _abi
from tests import kat_actors, kat_combat
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
