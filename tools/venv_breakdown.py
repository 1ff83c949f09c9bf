"""Where a numpy FootsiesVectorEnv.step goes at 65 536 arenas, without a profiler in the way:
the step call (+ stream wait), the D2H copy (outputs_numpy), the host conversion
(step_result_from_outputs), and the whole step with the device-resident outputs (one D2H copy a
step) against the pinned-host outputs (_host_outputs: the kernels write across the bus, no copy).
GPU box only."""
import sys
import time

sys.path.insert(0, "/root/repo")
import numpy as np  # noqa: E402
import torch  # noqa: E402
from footsies_gym_amd import vector_env as ve  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
WARM, STEPS = 400, 200
rng = np.random.default_rng(0)
a1 = rng.integers(0, 8, (WARM + STEPS, N)).astype(np.uint8)
a2 = rng.integers(0, 8, (WARM + STEPS, N)).astype(np.uint8)


def whole(host_outputs):
    k = [0]
    env = ve.FootsiesVectorEnv(N, device=0, opponent=lambda o, i: a2[k[0]], seed=0, _host_outputs=host_outputs)
    env.reset(seed=0)
    for j in range(WARM):
        k[0] = j
        env.step(a1[j])
    torch.cuda.synchronize()
    t = time.perf_counter()
    for j in range(WARM, WARM + STEPS):
        k[0] = j
        env.step(a1[j])
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / STEPS
    env.close()
    return dt


def parts():
    env = ve.FootsiesVectorEnv(N, device=0, opponent=lambda o, i: a2[0], seed=0)
    env.reset(seed=0)
    sim = env.sim
    for j in range(WARM):
        env.step(a1[j])
    torch.cuda.synchronize()
    ts = {"step+sync": 0.0, "d2h": 0.0, "convert": 0.0}
    for j in range(WARM, WARM + STEPS):
        t0 = time.perf_counter()
        sim.step(a1[j], a2[j])
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        host = sim.outputs_numpy(copy=False, _synced=True)
        t2 = time.perf_counter()
        ve.step_result_from_outputs(host, "same_step")
        t3 = time.perf_counter()
        ts["step+sync"] += t1 - t0
        ts["d2h"] += t2 - t1
        ts["convert"] += t3 - t2
    env.close()
    return {k: 1e3 * v / STEPS for k, v in ts.items()}


T = {}


def _tick(k, t0):
    t = time.perf_counter()
    T[k] = T.get(k, 0.0) + t - t0
    return t


def pieces_of(out):
    """step_result_from_outputs("same_step") restated with a clock between its pieces."""
    t = time.perf_counter()
    n = len(out["frame"])
    obs, info, (rewards, term, trunc) = ve._host_convert(out, "", None, n, True)
    t = _tick("main convert", t)
    idx = np.nonzero(term)[0]
    t = _tick("nonzero", t)
    fobs, finfo, _ = ve._host_convert(out, "final_", idx, len(idx), False, info_copies=False)
    t = _tick("final convert", t)
    final_obs = np.empty(len(term), dtype=object)
    final_info = np.empty(len(term), dtype=object)
    t = _tick("object arrays", t)
    g, m, mf, pos = (list(fobs[k]) for k in ("guard", "move", "move_frame", "position"))
    fr, a1, a2, h1, h2 = (list(finfo[k]) for k in ("frame", "p1_action", "p2_action", "p1_hitstun", "p2_hitstun"))
    t = _tick("row views", t)
    final_obs[idx] = [{"guard": a, "move": b, "move_frame": c, "position": d} for a, b, c, d in zip(g, m, mf, pos)]
    final_info[idx] = [{"frame": v0, "p1_action": v1, "p2_action": v2, "p1_hitstun": v3, "p2_hitstun": v4,
                        "guard": v5, "move": v6, "move_frame": v7, "position": v8}
                       for v0, v1, v2, v3, v4, v5, v6, v7, v8 in zip(fr, a1, a2, h1, h2, g, m, mf, pos)]
    t = _tick("dicts", t)
    info["final_observation"] = final_obs
    info["_final_observation"] = term.copy()
    info["final_info"] = final_info
    info["_final_info"] = term.copy()
    _tick("rest", t)
    return obs, rewards, term, trunc, info


def pieces(host_outputs):
    T.clear()
    env = ve.FootsiesVectorEnv(N, device=0, opponent=lambda o, i: a2[0], seed=0, _host_outputs=host_outputs)
    env.reset(seed=0)
    sim = env.sim
    for j in range(WARM):
        env.step(a1[j])
    torch.cuda.synchronize()
    t = time.perf_counter()
    for j in range(WARM, WARM + STEPS):
        t0 = time.perf_counter()
        sim.step(a1[j], a2[j])
        t0 = _tick("step call", t0)
        host = sim.outputs_numpy(copy=False, _synced=True)
        t0 = _tick("outputs_numpy (D2H / wait)", t0)
        pieces_of(host)
    dt = (time.perf_counter() - t) / STEPS
    env.close()
    return 1e3 * dt, {k: round(1e3 * v / STEPS, 4) for k, v in T.items()}


if __name__ == "__main__":
    print("N", N, "host threads", ve.host_threads())
    for r in range(2):
        print("round", r, "device outputs ms/step %.4f" % (1e3 * whole(False)),
              " host outputs ms/step %.4f" % (1e3 * whole(True)))
    print("parts (ms/step):", {k: round(v, 4) for k, v in parts().items()})
    for ho in (False, True):
        ms, tab = pieces(ho)
        print("pieces, host outputs" if ho else "pieces, device outputs", "ms/step %.4f" % ms, tab)
