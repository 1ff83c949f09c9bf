"""Test double: the wire server's backend interface over the CPU oracle (one arena), so the
protocol layer runs without a GPU.  Test infrastructure only; the product backend is
footsies_gym_amd.server.SimBackend (libfootsies.so)."""
import numpy as np

from footsies_gym_amd import _abi


class OracleBackend:
    def __init__(self, oracle_lib, p2_bot=True, seed=0):
        self.remote = not p2_bot
        self.o = oracle_lib.Oracle(1, p2_mode=_abi.FS_P2_BOT if p2_bot else _abi.FS_P2_EXTERNAL,
                                   autoreset_mode=_abi.FS_AUTORESET_NEXT_STEP, base_seed=seed)

    def env_state(self):
        return self.o.env_state()[0]

    def step(self, p1, p2):
        if p2 is None and self.remote:  # the handle's remote P2 is switched to the bot: no action arrived
            p2 = 0
        out = self.o.step(np.array([p1], np.uint8), None if p2 is None else np.array([p2], np.uint8))
        return bool(out["terminated"][0])

    def reset(self, hard):
        self.o.reset(flags=_abi.FS_RESET_HARD if hard else _abi.FS_RESET_IF_NEEDED)

    def seed(self, seed):
        self.o.reset(seeds=np.array([seed], np.uint64), flags=_abi.FS_RESET_SEED_ONLY)

    def get_state(self):
        return self.o.state()

    def set_state(self, st):
        assert self.o.set_state(st) == 0

    def set_p2_bot(self, bot):
        assert self.o.set_p2_mode(_abi.FS_P2_BOT if bot else _abi.FS_P2_EXTERNAL) == 0

    def close(self):
        self.o.close()
