#!/usr/bin/env python3
"""Time the reference's own client path: the unmodified reference FootsiesEnv (imported from
/root/reference with the throwaway gymnasium stub of tests/golden/) stepping against
footsies_gym_amd.server.FootsiesServer over localhost TCP (build container only: the reference
does not exist on the GPU box).

What is timed is the reference's per-step plumbing (FE:518-570 with FE:308-334): the 3-byte
action send, the 4-byte big-endian length + JSON EnvironmentState receive, json.loads,
FootsiesState construction, _extract_obs / _extract_info / the dense reward.  The game side is
the wire-compatible server in a separate process, backed by the CPU oracle (one arena, P2 = the
in-game bot), answering each action at once -- so this is an upper bound for the reference's
socket path: the real Unity game additionally paces Fight ticks at 50 x timeScale Hz (6.0 by
default: <= 300 env-steps/s per game process, FE:42-43, GameManager.cs:58, 177-182).

  python tools/time_reference_client.py [--seconds 10] [--out profiles/r04_reference_client.json]
"""
import argparse
import json
import multiprocessing as mp
import os
import platform
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
REF = "/root/reference/footsies-gym"


def serve(q, seed):
    sys.path.insert(0, ROOT)
    from footsies_gym_amd.server import FootsiesServer
    from oracle import binding
    from tests.oracle_server_backend import OracleBackend
    binding.build()
    srv = FootsiesServer("127.0.0.1", 0, 0, None, p2_no_state=True, backend=OracleBackend(binding, p2_bot=True,
                                                                                           seed=seed))
    q.put(srv.ports)
    srv.serve()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r04_reference_client.json"))
    a = ap.parse_args()
    if not os.path.isdir(REF):
        raise SystemExit("the reference is not here (build container only)")
    q = mp.get_context("spawn").Queue()
    proc = mp.get_context("spawn").Process(target=serve, args=(q, 0), daemon=True)
    proc.start()
    ports = q.get(timeout=120)
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden", "_gym_stub"))
    sys.path.insert(0, REF)
    import numpy as np
    from footsies_gym.envs.footsies import FootsiesEnv  # the reference client, unmodified
    env = FootsiesEnv(skip_instancing=True, game_address="127.0.0.1", game_port=ports["p1"],
                      remote_control_port=ports["rc"], dense_reward=True)
    rng = np.random.default_rng(0)
    acts = [tuple(bool(b) for b in row) for row in rng.integers(0, 2, (200000, 3))]
    env.reset(seed=0)
    for j in range(200):  # warm-up
        if env.step(acts[j])[2]:
            env.reset()
    steps, episodes, resets_s = 0, 0, 0.0
    t0 = time.perf_counter()
    j = 200
    while time.perf_counter() - t0 < a.seconds:
        for _ in range(500):
            term = env.step(acts[j % len(acts)])[2]
            j += 1
            steps += 1
            if term:
                episodes += 1
                r0 = time.perf_counter()
                env.reset()
                resets_s += time.perf_counter() - r0
    dt = time.perf_counter() - t0
    for s in (env.comm, env.remote_control_comm, env.opponent_comm):
        if s is not None:
            s.close()
    proc.terminate()
    res = {"value": steps / dt, "unit": "env-steps/s", "steps": steps, "seconds": round(dt, 2),
           "episodes": episodes, "reset_seconds_included": round(resets_s, 3),
           "client_cores": 1, "server_cores": 1, "host": platform.processor() or platform.machine(),
           "host_cpus": os.cpu_count(),
           "label": "build container, reference client + socket + JSON (unmodified FootsiesEnv from /root/reference "
                    "against FootsiesServer on the CPU oracle in a second process; P2 = in-game bot; resets after "
                    "terminals included)",
           "reference_ceiling_derived": "<= 300 env-steps/s per game process (50 Hz x timeScale 6.0; FE:42-43)",
           "command": "python tools/time_reference_client.py --seconds %g" % a.seconds}
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
