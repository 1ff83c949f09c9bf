"""The Python drop-in surface without PyTorch (VERDICT r05 missing #5: the reference client needs only
gymnasium).  A child process with torch made unimportable runs the numpy FootsiesVectorEnv and the
single-arena FootsiesEnv on FootsiesSim's native backend -- outputs in pinned host memory the library
allocates (fs_host_alloc), host actions, the library's own stream -- and checks it against the CPU
oracle step by step; the parent runs the same steps on the torch-backed surface and requires the
child's observations, rewards and flags byte for byte."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N, STEPS, SINGLE = 1024, 300, 400

CHILD = r'''
import sys
sys.modules["torch"] = None  # torch is not importable in this process
sys.path.insert(0, %(root)r)
import numpy as np
from footsies_gym_amd import _lib
from footsies_gym_amd.vector_env import FootsiesVectorEnv, FootsiesEnv
from oracle import binding
from tests.oracle_vector_env import OracleVectorEnv
N, STEPS, SINGLE = %(n)d, %(steps)d, %(single)d
env = FootsiesVectorEnv(N, device=0, seed=3, autoreset_mode="next_step")
assert env.sim.backend == "native", env.sim.backend
ref = OracleVectorEnv(N, binding, seed=3, autoreset_mode="next_step")
obs, _ = env.reset()
robs, _ = ref.reset()
rng = np.random.default_rng(11)
rec = {"obs": [], "rew": [], "term": []}
terms = 0
for t in range(STEPS):
    a = rng.integers(0, 8, N)
    obs, rew, term, trunc, info = env.step(a)
    robs, rrew, rterm, rtrunc, rinfo = ref.step(a)
    for k in obs:
        assert np.array_equal(obs[k], robs[k]), (t, k)
    assert np.array_equal(rew, rrew) and np.array_equal(term, rterm) and np.array_equal(trunc, rtrunc), t
    terms += int(term.sum())
    rec["obs"].append(np.concatenate([obs[k].reshape(N, -1).astype(np.float64) for k in sorted(obs)], axis=1))
    rec["rew"].append(rew.copy())
    rec["term"].append(term.copy())
assert terms > 0
state = env.save_battle_state()
env.close()
one = FootsiesEnv(seed=5)
o, i = one.reset(seed=5)
singles = [sorted(o.items())]
for t in range(SINGLE):
    o, r, d, tr, i = one.step((bool(t %% 3 == 0), bool(t %% 5 == 1), bool(t %% 2)))
    singles.append((sorted(o.items()), r, d))
    if d:
        o, i = one.reset()
one.close()
np.savez(%(out)r, obs=np.stack(rec["obs"]), rew=np.stack(rec["rew"]), term=np.stack(rec["term"]), state=state,
         singles=np.array(repr(singles)))
print("images", _lib.runtime_images().split(), "torch" in sys.modules and sys.modules["torch"] is not None)
'''


def test_numpy_surface_runs_without_torch(tmp_path):
    out = str(tmp_path / "native.npz")
    code = CHILD % dict(root=ROOT, n=N, steps=STEPS, single=SINGLE, out=out)
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    last = r.stdout.strip().splitlines()[-1]
    assert last.endswith("False"), last  # torch never got into the child
    got = np.load(out)
    # the same steps on the torch-backed surface in this process
    from footsies_gym_amd.vector_env import FootsiesEnv, FootsiesVectorEnv
    env = FootsiesVectorEnv(N, device=0, seed=3, autoreset_mode="next_step")
    assert env.sim.backend == "torch"
    env.reset()
    rng = np.random.default_rng(11)
    for t in range(STEPS):
        obs, rew, term, trunc, info = env.step(rng.integers(0, 8, N))
        row = np.concatenate([obs[k].reshape(N, -1).astype(np.float64) for k in sorted(obs)], axis=1)
        assert row.tobytes() == got["obs"][t].tobytes(), t
        assert rew.tobytes() == got["rew"][t].tobytes() and term.tobytes() == got["term"][t].tobytes(), t
    assert env.save_battle_state().tobytes() == got["state"].tobytes()
    env.close()
    one = FootsiesEnv(seed=5)
    o, i = one.reset(seed=5)
    singles = [sorted(o.items())]
    for t in range(SINGLE):
        o, r, d, tr, i = one.step((bool(t % 3 == 0), bool(t % 5 == 1), bool(t % 2)))
        singles.append((sorted(o.items()), r, d))
        if d:
            o, i = one.reset()
    one.close()
    assert repr(singles) == str(got["singles"])


def test_native_backend_in_process_matches_torch_backend():
    """backend="native" forced beside torch: the same host outputs, bit for bit, as the torch-backed
    handle over 200 steps of host actions with terminals; the device-tensor APIs say they need torch."""
    from footsies_gym_amd.simulator import FootsiesSim
    a = FootsiesSim(777, p2_mode="external", seed=9, host_outputs=True, backend="native")
    b = FootsiesSim(777, p2_mode="external", seed=9, host_outputs=True)
    assert a.backend == "native" and b.backend == "torch"
    rng = np.random.default_rng(2)
    terms = 0
    for t in range(200):
        p1, p2 = rng.integers(0, 8, 777), rng.integers(0, 8, 777)
        oa, ob = a.step(p1, p2), b.step(p1, p2)
        for k in oa:
            assert oa[k].tobytes() == ob[k].numpy().tobytes(), (t, k)
        terms += int(oa["terminated"].sum())
    assert terms > 0
    for call in (lambda: a.hash_actions(4), lambda: a.alloc_trajectory(4), lambda: a.step_n(4)):
        with pytest.raises(RuntimeError, match="needs PyTorch"):
            call()
    # views of the pinned outputs a caller still holds outlive close(): the buffer is released with
    # the last of them, not under them
    va, vb = a.outputs_numpy(copy=False)["position"], b.outputs_numpy(copy=False)["position"]
    want = va.copy()
    a.close()
    b.close()
    import gc
    gc.collect()
    assert va.tobytes() == want.tobytes() and vb.tobytes() == want.tobytes()
