"""Raw client of the game's training-socket protocol (the byte-level behaviour of
FootsiesEnv's sockets, FE:261-334, 407-430), used to replay recorded traffic."""
import socket
import struct
import time


def connect(address, port, timeout=30.0):
    end = time.time() + timeout
    while True:
        s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        s.settimeout(timeout)
        try:
            s.connect((address, port))
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            return s
        except (ConnectionRefusedError, ConnectionAbortedError):
            s.close()
            if time.time() > end:
                raise
            time.sleep(0.05)


def recv_exact(s, n):
    out = b""
    while len(out) < n:
        chunk = s.recv(n - len(out))
        if not chunk:
            raise ConnectionError("server closed")
        out += chunk
    return out


def recv_message(s):
    """4-byte big-endian length + payload (FE:308-313)."""
    head = recv_exact(s, 4)
    return head + recv_exact(s, struct.unpack("!I", head)[0])


def replay(transcript, ports, address="127.0.0.1"):
    """Connect like FootsiesEnv._connect_to_game (P1, remote control, then P2) and replay a
    server transcript: "recv" events are sent to the server, "send" events are read back and
    compared byte for byte.  Returns the number of messages checked."""
    socks = {"p1": connect(address, ports["p1"]), "rc": connect(address, ports["rc"])}
    if "p2" in ports:
        socks["p2"] = connect(address, ports["p2"])
    checked = 0
    try:
        for i, (kind, chan, data) in enumerate(transcript):
            if kind == "recv":
                socks[chan].sendall(data)
            else:
                got = recv_message(socks[chan])
                assert got == data, (i, chan, got[:200], data[:200])
                checked += 1
    finally:
        for s in socks.values():
            s.close()
    return checked
