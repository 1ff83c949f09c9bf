"""Test double: the FootsiesVectorEnv surface over the CPU oracle, so host-side layers
(the wrappers) can be checked without a GPU.  Test infrastructure only -- the product
FootsiesVectorEnv runs on libfootsies.so and has no CPU path."""
import numpy as np

from footsies_gym_amd import _abi
from footsies_gym_amd import spaces as sp
from footsies_gym_amd.simulator import encode_actions
from footsies_gym_amd.vector_env import obs_info_from_outputs, step_result_from_outputs

AR = {"same_step": _abi.FS_AUTORESET_SAME_STEP, "next_step": _abi.FS_AUTORESET_NEXT_STEP}


class OracleVectorEnv:
    def __init__(self, num_envs, oracle_lib, dense_reward=True, seed=0, autoreset_mode="next_step", frame_delay=0):
        self.num_envs = num_envs
        self.autoreset_mode = autoreset_mode
        self.ora = oracle_lib.Oracle(num_envs, p2_mode=_abi.FS_P2_BOT, dense_reward=dense_reward,
                                     autoreset_mode=AR[autoreset_mode], base_seed=seed, frame_delay=frame_delay)
        self.single_observation_space = sp.single_observation_space()
        self.single_action_space = sp.single_action_space()

    def _host(self, out):
        return {k: np.array(v, copy=True) for k, v in out.items()}

    def reset(self, *, seed=None, options=None):
        return obs_info_from_outputs(self._host(self.ora.reset()))

    def step(self, actions):
        out = self._host(self.ora.step(encode_actions(np.asarray(actions))))
        return step_result_from_outputs(out, self.autoreset_mode)

    def step_masked(self, actions, active):
        active = np.asarray(active, dtype=bool)
        out = self._host(self.ora.step(encode_actions(np.asarray(actions)), active=active.astype(np.uint8)))
        out["reward"][~active] = 0.0
        out["terminated"][~active] = 0
        out["truncated"][~active] = 0
        return step_result_from_outputs(out, self.autoreset_mode)

    def close(self):
        self.ora.close()
