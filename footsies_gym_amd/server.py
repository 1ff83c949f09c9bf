"""Wire-compatible FOOTSIES game server: the Unity game's side of the training sockets,
simulated by libfootsies.so, so an unmodified FootsiesEnv (FE) can drive it.

The game is the server on three TCP ports (GameManager.cs command line):
  * P1 (``--p1-port``, FE game_port 11000): after every emitted frame the game sends the
    EnvironmentState as UTF-8 JSON with a 4-byte big-endian length prefix
    (TrainingRemoteActor.cs:53-63, SocketHelper.cs:70-82) and, unless the battle is
    over, waits for a 3-byte action [left, right, attack], non-zero = pressed
    (TrainingRemoteActor.cs:93-117);
  * P2 (``--p2-port``, FE opponent_port 11001), when P2 is a remote actor: 3-byte actions,
    and states too unless ``--p2-no-state`` (FE passes it, FE:246-248);
  * remote control (``--remote-control-port``, 11002): length-prefixed JSON
    {"command": int, "value": str} (TrainingRemoteControl.cs:28-33, 78-110), handled
    before the frame like BattleCore.FixedUpdate (BattleCore.cs:138-170): RESET (1),
    STATE_SAVE (2, answered with the BattleState JSON, length-prefixed), STATE_LOAD (3),
    P2_BOT (4, value "True"/"False"), SEED (5).
A Fight frame runs once the P1 action (and a remote P2's) has arrived (TrainingManager
Ready, TrainingManager.cs:59-92).  After a terminal frame the game plays KO -> End ->
Stop -> Intro -> Fight on its own and emits state(-1) (BattleCore.cs:212-243, 262-291);
this server completes that sequence right after sending the terminal state, so a SEED
sent after a terminal step (a race in Unity) applies from the next RNG draw on.

One server is one game (one arena).  Run: python -m footsies_gym_amd.server --help.
"""
import argparse
import json
import select
import socket
import struct

import numpy as np

from . import battle_state

ENV_STATE_FIELDS = ("p1Vital", "p2Vital", "p1Guard", "p2Guard", "p1Move", "p1MoveFrame", "p2Move", "p2MoveFrame",
                    "p1Position", "p2Position", "globalFrame", "p1MostRecentAction", "p2MostRecentAction",
                    "p1Hitstun", "p2Hitstun")  # EnvironmentState.cs:12-26, JsonUtility field order
CMD_NONE, CMD_RESET, CMD_STATE_SAVE, CMD_STATE_LOAD, CMD_P2_BOT, CMD_SEED = 0, 1, 2, 3, 4, 5


def env_state_json(rec):
    """One fs_env_state record as the game's JSON (floats: shortest float32 round trip)."""
    parts = []
    for f in ENV_STATE_FIELDS:
        v = rec[f]
        parts.append('"%s":%s' % (f, str(np.float32(v)) if f.endswith("Position") else str(int(v))))
    return "{" + ",".join(parts) + "}"


def frame(payload):
    """SocketHelper.SendWithSizeSuffixAsync framing: 4-byte big-endian length + bytes."""
    return struct.pack("!I", len(payload)) + payload


def action_bits(msg):
    """TrainingRemoteActor.RequestTrainingInput (cs:108-111): 3 bytes -> Left|Right|Attack."""
    return (1 if msg[0] else 0) | (2 if msg[1] else 0) | (4 if msg[2] else 0)


class SimBackend:
    """The product backend: one arena of libfootsies.so (FootsiesSim on a GPU)."""

    def __init__(self, p2_bot=True, dense_reward=True, device=0, seed=0):
        from .simulator import FootsiesSim
        # (one arena: outputs written into pinned host memory, see FootsiesSim host_outputs)
        self.sim = FootsiesSim(1, p2_mode="bot" if p2_bot else "external", seed=seed, device=device,
                               dense_reward=dense_reward, autoreset_mode="next_step", host_outputs=True)

    def env_state(self):
        return self.sim.env_state()[0]

    def step(self, p1, p2):
        self.sim.step(np.array([p1], np.uint8), np.array([0 if p2 is None else p2], np.uint8)
                      if self.sim.p2_mode == "external" else None)
        return bool(self.sim.outputs_numpy(copy=False, _synced=True)["terminated"][0])  # (step waited)

    def reset(self, hard):
        self.sim.reset(hard=hard)

    def seed(self, seed):
        self.sim.reset(seeds=[np.uint64(seed & (2**64 - 1))], seed_only=True)

    def get_state(self):
        return self.sim.get_state()

    def set_state(self, st):
        self.sim.set_state(st)

    def set_p2_bot(self, bot):
        """P2_BOT (BattleCore.cs:158-167): TrainingManager.actorP2 becomes the game's P2 bot or the
        remote actor again (fs_set_p2_mode); each keeps its own state while the other plays."""
        self.sim.set_p2_mode("bot" if bot else "external")

    def close(self):
        self.sim.close()


def _listener(address, port):
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    s.bind((address, port))
    s.listen(1)
    return s


class FootsiesServer:
    """The game's socket protocol over a backend (default: SimBackend on the GPU)."""

    def __init__(self, address="localhost", p1_port=11000, remote_control_port=11002, p2_port=None,
                 p2_no_state=True, backend=None, p2_bot=None, dense_reward=True, device=0, seed=0,
                 remote_control_address=None, p2_address=None, transcript=None):
        self.p2_remote = p2_port is not None
        p2_bot = (not self.p2_remote) if p2_bot is None else p2_bot
        self.backend = backend if backend is not None else SimBackend(p2_bot, dense_reward, device, seed)
        self.p2_bot = p2_bot
        self.p2_no_state = p2_no_state
        self.listeners = {"p1": _listener(address, p1_port),
                          "rc": _listener(remote_control_address or address, remote_control_port)}
        if self.p2_remote:
            self.listeners["p2"] = _listener(p2_address or address, p2_port)
        self.transcript = transcript  # optional list of ("recv" | "send", channel, bytes)
        self.ports = {k: s.getsockname()[1] for k, s in self.listeners.items()}
        self.conn = {}
        self.buf = {k: b"" for k in ("p1", "p2", "rc")}
        self.running = True

    # -- plumbing -----------------------------------------------------------------------
    def _accept_all(self):
        pending = dict(self.listeners)
        while pending and self.running:
            r, _, _ = select.select(list(pending.values()), [], [], 0.2)
            for name, ls in list(pending.items()):
                if ls in r:
                    c, _ = ls.accept()
                    c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                    self.conn[name] = c
                    del pending[name]
        for ls in self.listeners.values():
            ls.close()

    def _send(self, name, msg):
        if self.transcript is not None:
            self.transcript.append(("send", name, msg))
        self.conn[name].sendall(msg)

    def _send_state(self):
        msg = frame(env_state_json(self.backend.env_state()).encode("utf-8"))
        self._send("p1", msg)
        if self.p2_remote and not self.p2_no_state and "p2" in self.conn:
            self._send("p2", msg)

    def _read(self, name):
        data = self.conn[name].recv(65536)
        if not data:
            raise ConnectionError(name)
        self.buf[name] += data

    def _take_action(self, name):
        if len(self.buf[name]) < 3:
            return None
        msg, self.buf[name] = self.buf[name][:3], self.buf[name][3:]
        if self.transcript is not None:
            self.transcript.append(("recv", name, msg))
        return action_bits(msg)

    def _take_command(self):
        b = self.buf["rc"]
        if len(b) < 4:
            return None
        n = struct.unpack("!I", b[:4])[0]
        if len(b) < 4 + n:
            return None
        self.buf["rc"] = b[4 + n:]
        if self.transcript is not None:
            self.transcript.append(("recv", "rc", b[:4 + n]))
        return json.loads(b[4:4 + n].decode("utf-8"))

    # -- the game -----------------------------------------------------------------------
    def _command(self, msg):
        """BattleCore.FixedUpdate's remote-control switch (BattleCore.cs:138-170)."""
        cmd, value = int(msg.get("command", CMD_NONE)), msg.get("value", "")
        if cmd == CMD_RESET:  # Stop -> Intro -> Fight: state(-1)
            self.backend.reset(hard=True)
            self._send_state()
        elif cmd == CMD_STATE_SAVE:
            doc = battle_state.dumps(battle_state.battle_state(self.backend.get_state(), 0))
            self._send("rc", frame(doc.encode("utf-8")))
        elif cmd == CMD_STATE_LOAD:
            st = self.backend.get_state()
            self.backend.set_state(battle_state.load_into(st, 0, value))
        elif cmd == CMD_P2_BOT:
            # TrainingRemoteControl.ProcessCommand (cs:100-102): value.ToLower() == "true".  Only a
            # game launched with a remote P2 is served: the reference client sends P2_BOT only then
            # (FE:468-470 raises before sending otherwise).
            if self.p2_remote:
                self.p2_bot = str(value).lower() == "true"
                self.backend.set_p2_bot(self.p2_bot)
        elif cmd == CMD_SEED:
            self.backend.seed(int(value))

    def serve(self):
        """Accept the agent's connections, start the game (state(-1)) and run until the agent
        disconnects or stop() is called."""
        self._accept_all()
        if not self.running:
            return
        self._send_state()  # game start: Stop -> Intro -> Fight emits state(-1)
        p1 = p2 = None
        try:
            while self.running:
                socks = [self.conn[k] for k in ("rc", "p1", "p2") if k in self.conn]
                r, _, _ = select.select(socks, [], [], 0.2)
                for name in ("rc", "p1", "p2"):
                    if name in self.conn and self.conn[name] in r:
                        self._read(name)
                while True:  # one command per FixedUpdate, in arrival order
                    msg = self._take_command()
                    if msg is None:
                        break
                    self._command(msg)
                if p1 is None:
                    p1 = self._take_action("p1")
                if self.p2_remote and p2 is None:
                    p2 = self._take_action("p2")
                remote_p2 = self.p2_remote and not self.p2_bot
                if p1 is not None and (p2 is not None or not remote_p2):
                    over = self.backend.step(p1, p2 if remote_p2 else None)
                    p1 = None
                    if remote_p2:
                        p2 = None
                    self._send_state()
                    if over:  # the game plays KO -> ... -> Fight by itself, then emits state(-1)
                        self.backend.reset(hard=False)
                        self._send_state()
        except ConnectionError:
            pass
        finally:
            for c in self.conn.values():
                c.close()
            self.backend.close()

    def stop(self):
        self.running = False


def main(argv=None):
    ap = argparse.ArgumentParser(description="FOOTSIES game server over libfootsies.so (the Unity game's "
                                             "training-socket protocol)")
    ap.add_argument("--p1-address", default="localhost")
    ap.add_argument("--p1-port", type=int, default=11000)
    ap.add_argument("--remote-control-address", default=None)
    ap.add_argument("--remote-control-port", type=int, default=11002)
    ap.add_argument("--p2-bot", action="store_true", help="P2 is the in-game bot (default without --p2-port)")
    ap.add_argument("--p2-address", default=None)
    ap.add_argument("--p2-port", type=int, default=None)
    ap.add_argument("--p2-no-state", action="store_true")
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--seed", type=int, default=0)
    # accepted for command-line compatibility with the game binary; no effect here
    for flag in ("--training", "--mute", "--synced-non-blocking", "--synced-blocking", "-batchmode", "-nographics",
                 "-force-gfx-direct", "-nolog", "--fast-forward"):
        ap.add_argument(flag, action="store_true")
    ap.add_argument("--fast-forward-speed", type=float, default=None)
    ap.add_argument("-logFile", default=None)
    for flag in ("--p1-bot", "--p1-spectator", "--p1-player", "--p2-player", "--p2-spectator", "--p1-no-state"):
        ap.add_argument(flag, action="store_true")
    a = ap.parse_args(argv)
    if a.p1_bot or a.p1_player or a.p2_player or a.p1_spectator or a.p2_spectator or a.p1_no_state:
        ap.error("only the training setup is served: P1 remote agent, P2 bot or remote agent")
    srv = FootsiesServer(a.p1_address, a.p1_port, a.remote_control_port, a.p2_port, a.p2_no_state,
                         p2_bot=True if a.p2_bot else None, device=a.device, seed=a.seed,
                         remote_control_address=a.remote_control_address, p2_address=a.p2_address)
    srv.serve()


if __name__ == "__main__":
    main()
