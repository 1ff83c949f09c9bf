"""FootsiesSim wrapped in the Oracle-style step interface used by the scenario/golden runners."""
from footsies_gym_amd import _abi

P2 = {_abi.FS_P2_EXTERNAL: "external", _abi.FS_P2_BOT: "bot", _abi.FS_P2_NOOP: "noop"}
AR = {_abi.FS_AUTORESET_SAME_STEP: "same_step", _abi.FS_AUTORESET_NEXT_STEP: "next_step"}


class SimBackend:
    def __init__(self, n, p2_mode=_abi.FS_P2_EXTERNAL, dense=True, autoreset=_abi.FS_AUTORESET_SAME_STEP, seed=0,
                 frame_delay=0):
        from footsies_gym_amd.simulator import FootsiesSim
        self.sim = FootsiesSim(n, p2_mode=P2[p2_mode], dense_reward=dense, autoreset_mode=AR[autoreset], seed=seed,
                               frame_delay=frame_delay)

    def reset(self):
        self.sim.reset()
        return self.sim.outputs_numpy()

    def step(self, a1, a2=None):
        self.sim.step(a1, a2 if self.sim.p2_mode == "external" else None)
        return self.sim.outputs_numpy()

    def env_state(self):
        return self.sim.env_state()

    def state(self):
        return self.sim.get_state()

    def set_state(self, st):
        self.sim.set_state(st)


def make(n, p2_mode, dense, autoreset, seed, frame_delay=0):
    return SimBackend(n, p2_mode, dense, autoreset, seed, frame_delay)
