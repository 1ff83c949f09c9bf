"""Replay of tests/golden/wire_golden.json.gz (the reference FootsiesEnv client's traffic
against footsies_gym_amd.server, recorded by tests/golden/make_wire_golden.py)."""
import base64
import gzip
import json
import os
import threading

from footsies_gym_amd.server import FootsiesServer
from tests import wire_client

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = ("bot", "remote_delay2", "remote_switch")
_CACHE = {}


def load():
    if "w" not in _CACHE:
        with gzip.open(os.path.join(HERE, "golden", "wire_golden.json.gz"), "rt") as f:
            _CACHE["w"] = json.load(f)
    return _CACHE["w"]


def replay(name, make_backend):
    """make_backend(p2_bot, seed) -> a server backend.  Serves the recorded client half and
    checks every server message; returns the count."""
    case = load()[name]
    transcript = [(k, c, base64.b64decode(d)) for k, c, d in case["transcript"]]
    remote = case["remote_p2"]
    srv = FootsiesServer("127.0.0.1", 0, 0, 0 if remote else None, p2_no_state=True,
                         backend=make_backend(not remote, case["seed"]))
    th = threading.Thread(target=srv.serve, daemon=True)
    th.start()
    try:
        n = wire_client.replay(transcript, srv.ports)
    finally:
        srv.stop()
        th.join(timeout=30)
    assert n == sum(1 for k, _, _ in transcript if k == "send")
    return n
