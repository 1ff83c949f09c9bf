#!/usr/bin/env python3
"""Traffic of the REFERENCE's own FootsiesEnv client against footsies_gym_amd.server
(build container only).

The unmodified FootsiesEnv (imported from /root/reference with the throwaway gymnasium
stub) connects to FootsiesServer -- backed here by the CPU oracle, since this container
has no GPU -- and plays scripted episodes through its public API: reset(seed=...),
step(), mid-episode reset() (the RESET command), save_battle_state() /
load_battle_state(), a custom opponent on the P2 port, set_opponent() switching P2 between
it and the in-game bot (the P2_BOT command), and frame_delay on the client side.  The server records every message it receives and sends; the transcript
is the fixture: tests replay the client half against the GPU-backed server and require
the server half back byte for byte.  Output (committed): tests/golden/wire_golden.json.gz.
"""
import base64
import gzip
import json
import os
import sys
import threading

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(HERE, "_gym_stub"))
sys.path.insert(0, "/root/reference/footsies-gym")

from footsies_gym.envs.footsies import FootsiesEnv  # noqa: E402

from footsies_gym_amd.server import FootsiesServer  # noqa: E402
from oracle import binding  # noqa: E402
from tests.oracle_server_backend import OracleBackend  # noqa: E402


def play(name, opponent, frame_delay, steps, seed, rng_seed, switch_every=0):
    transcript = []
    remote_p2 = opponent is not None
    srv = FootsiesServer("127.0.0.1", 0, 0, 0 if remote_p2 else None, p2_no_state=True,
                         backend=OracleBackend(binding, p2_bot=not remote_p2, seed=seed), transcript=transcript)
    th = threading.Thread(target=srv.serve, daemon=True)
    th.start()
    env = FootsiesEnv(skip_instancing=True, game_address="127.0.0.1", game_port=srv.ports["p1"],
                      remote_control_port=srv.ports["rc"], opponent_port=srv.ports.get("p2", 0),
                      opponent=opponent, frame_delay=frame_delay, dense_reward=True)
    rng = np.random.default_rng(rng_seed)
    log = {"rewards": [], "terminated": [], "frames": []}
    env.reset(seed=None)
    saved = None
    episodes = 0
    for t in range(steps):
        a = tuple(bool(b) for b in rng.integers(0, 2, 3))
        obs, r, term, trunc, info = env.step(a)
        log["rewards"].append(r)
        log["terminated"].append(bool(term))
        log["frames"].append(info["frame"])
        if term:
            episodes += 1
            env.reset(seed=int(rng.integers(0, 2**31)) if episodes % 2 else None)
        elif t % 97 == 50:
            env.reset()  # mid-episode: the RESET command
        elif remote_p2 and t % 61 == 20:
            saved = env.save_battle_state()
        elif remote_p2 and saved is not None and t % 61 == 40:
            env.load_battle_state(saved)
        if switch_every and t % switch_every == switch_every - 1:  # FE:458-480: P2_BOT both ways
            env.set_opponent(None if env.opponent is not None else opponent)
    env.close() if hasattr(env, "close") else None
    for s in (env.comm, env.remote_control_comm, env.opponent_comm):
        if s is not None:
            s.close()
    th.join(timeout=30)
    print(name, "messages:", len(transcript), "episodes:", episodes)
    return {"ports": sorted(srv.ports), "seed": seed, "remote_p2": remote_p2,
            "transcript": [[k, c, base64.b64encode(d).decode()] for k, c, d in transcript], "client": log}


def main():
    def opp(obs, info):
        return (info["frame"] % 7 < 3, info["frame"] % 5 == 1, info["frame"] % 11 == 0)
    cases = {
        "bot": play("bot", None, 0, 2500, 3, 1),
        "remote_delay2": play("remote_delay2", opp, 2, 2500, 4, 2),
        "remote_switch": play("remote_switch", opp, 0, 2500, 5, 3, switch_every=113),
    }
    with gzip.open(os.path.join(HERE, "wire_golden.json.gz"), "wt") as f:
        json.dump(cases, f)
    print("wrote wire_golden.json.gz")


if __name__ == "__main__":
    main()
