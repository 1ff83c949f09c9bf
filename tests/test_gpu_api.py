"""The HIP product path through its public surfaces: KATs, the reference-FE golden vectors,
fused multi-tick launches, state save/load, hashed actions, VectorEnv / FootsiesEnv."""
import numpy as np
import pytest

from footsies_gym_amd import _abi
from tests import golden_utils as gu
from tests import kat_combat, kat_core, kat_geometry
from tests import kat_scenarios as kat
from tests import wire_client, wire_replay
from tests import wrapper_replay as wr
from tests.gpu_backend import SimBackend, make
from tests.parity_utils import compare_outputs, compare_states, fused_kernel

P2_MODES = {"external": _abi.FS_P2_EXTERNAL, "bot": _abi.FS_P2_BOT, "noop": _abi.FS_P2_NOOP}

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", sorted(kat.ALL))
def test_kat_gpu(name):
    kat.ALL[name](SimBackend(1))


@pytest.mark.parametrize("name", sorted(kat_combat.ALL))
def test_kat_combat_gpu(name):
    kat_combat.ALL[name](SimBackend(1))


@pytest.mark.parametrize("name", sorted(kat_core.ALL))
def test_kat_core_gpu(name):
    """tests/kat_core.py (the sim-core paths round 3 pinned only by lockstep) through the HIP path."""
    kat_core.ALL[name](SimBackend(1))


@pytest.mark.parametrize("name", sorted(kat_geometry.ALL))
def test_kat_geometry_gpu(name):
    """tests/kat_geometry.py (the general-geometry tick: y != 0, flipped facings) through the HIP path."""
    kat_geometry.ALL[name](SimBackend(1))


@pytest.mark.parametrize("name", gu.CASES)
def test_golden_reference_fe_gpu(name):
    c = gu.case(gu.load(), name)
    gu.replay_next_step(c, make)
    gu.replay_same_step(c, make)


def test_step_n_trajectory_matches_single_steps(oracle_lib):
    """fs_step_n with a [n][N] trajectory == n fs_step calls == the oracle."""
    import torch
    from footsies_gym_amd.simulator import FootsiesSim
    N, T = 1000, 150
    a = FootsiesSim(N, p2_mode="external", seed=3)
    b = FootsiesSim(N, p2_mode="external", seed=3)
    p1, p2 = a.hash_actions(T, seed=77)
    traj = a.alloc_trajectory(T)
    a.step_n(T, p1, p2, trajectory=traj)
    torch.cuda.synchronize()
    tr = {k: v.cpu().numpy() for k, v in traj.items()}
    ora = oracle_lib.Oracle(N, p2_mode=_abi.FS_P2_EXTERNAL, base_seed=3)
    h1, h2 = p1.cpu().numpy(), p2.cpu().numpy()
    for t in range(T):
        b.step(p1[t], p2[t])
        got = b.outputs_numpy()
        exp = ora.step(h1[t], h2[t])
        compare_outputs(exp, got, step=t)
        compare_outputs(exp, {k: v[t] for k, v in tr.items()}, step=t)
    compare_states(ora.state(), a.get_state())
    compare_states(ora.state(), b.get_state())


@pytest.mark.parametrize("N,T,p2", [(1, 37, "external"), (33, 37, "bot"), (97, 64, "external"), (97, 1, "bot")])
def test_fused_ragged_sizes_match_oracle(oracle_lib, N, T, p2):
    """Fused launches over grids that are mostly idle lanes (1, 33, 97 arenas: one block, a
    part-filled wave; the LDS-DMA staging still runs in every thread) and odd tick counts (the
    loop's odd tail; one tick = the k_step path): every trajectory row and the final state equal
    the oracle's."""
    import torch
    from footsies_gym_amd.simulator import FootsiesSim
    sim = FootsiesSim(N, p2_mode=p2, seed=6)
    ora = oracle_lib.Oracle(N, p2_mode=P2_MODES[p2], base_seed=6)
    p1, p2a = sim.hash_actions(T, seed=91, p2=p2 == "external")
    traj = sim.alloc_trajectory(T)
    sim.step_n(T, p1, p2a if p2 == "external" else None, trajectory=traj)
    torch.cuda.synchronize()
    tr = {k: v.cpu().numpy() for k, v in traj.items()}
    h1 = p1.cpu().numpy()
    h2 = p2a.cpu().numpy() if p2 == "external" else None
    for t in range(T):
        exp = ora.step(h1[t], None if h2 is None else h2[t])
        compare_outputs(exp, {k: v[t] for k, v in tr.items()}, step=t)
    compare_states(ora.state(), sim.get_state())

@pytest.mark.parametrize("autoreset", ["same_step", "next_step"])
def test_frame_delay_paths_match_oracle(oracle_lib, autoreset):
    """frame_delay > 0 (FE:126-131, 532-535) through fs_step, fs_step_n with a trajectory
    and fs_step_n without one (launched tick by tick) == the oracle's FE deque."""
    import torch
    from footsies_gym_amd.simulator import FootsiesSim
    N, T, D = 777, 260, 5
    ar = {"same_step": _abi.FS_AUTORESET_SAME_STEP, "next_step": _abi.FS_AUTORESET_NEXT_STEP}[autoreset]
    kw = dict(p2_mode="external", seed=11, frame_delay=D, autoreset_mode=autoreset)
    a, b, c = FootsiesSim(N, **kw), FootsiesSim(N, **kw), FootsiesSim(N, **kw)
    p1, p2 = a.hash_actions(T, seed=0xD1A)
    traj = a.alloc_trajectory(T)
    a.step_n(T, p1, p2, trajectory=traj)
    c.step_n(T, p1, p2)
    torch.cuda.synchronize()
    tr = {k: v.cpu().numpy() for k, v in traj.items()}
    ora = oracle_lib.Oracle(N, p2_mode=_abi.FS_P2_EXTERNAL, base_seed=11, frame_delay=D, autoreset_mode=ar)
    h1, h2 = p1.cpu().numpy(), p2.cpu().numpy()
    terminals = 0
    for t in range(T):
        b.step(p1[t], p2[t])
        exp = ora.step(h1[t], h2[t])
        terminals += int(exp["terminated"].sum())
        compare_outputs(exp, b.outputs_numpy(), step=t)
        compare_outputs(exp, {k: v[t] for k, v in tr.items()}, step=t)
    compare_outputs(exp, c.outputs_numpy(), step=T - 1)
    assert terminals > 0
    # an explicit reset refills the queue: the next D observations repeat state(-1)
    b.reset(hard=True)
    ora.reset(flags=_abi.FS_RESET_HARD)
    for t in range(D + 3):
        b.step(h1[t], h2[t])
        compare_outputs(ora.step(h1[t], h2[t]), b.outputs_numpy(), step=T + t)


@pytest.mark.parametrize("p2", ["bot", "external"])
def test_step_masked_matches_oracle(oracle_lib, p2):
    """fs_step_masked: only active arenas tick; the others keep state and outputs."""
    from footsies_gym_amd.simulator import FootsiesSim
    N, T = 999, 300
    p2m = _abi.FS_P2_BOT if p2 == "bot" else _abi.FS_P2_EXTERNAL
    s = FootsiesSim(N, p2_mode=p2, seed=21)
    ora = oracle_lib.Oracle(N, p2_mode=p2m, base_seed=21)
    rng = np.random.default_rng(5)
    for t in range(T):
        a1 = rng.integers(0, 8, N).astype(np.uint8)
        a2 = rng.integers(0, 8, N).astype(np.uint8) if p2 == "external" else None
        active = rng.random(N) < (0.3 if t % 2 else 0.9)
        s.step(a1, a2, active=active)
        exp = ora.step(a1, a2, active=active.astype(np.uint8))
        compare_outputs(exp, s.outputs_numpy(), step=t)
    compare_states(ora.state(), s.get_state())


@pytest.mark.parametrize("name", wr.CASES)
def test_wrappers_match_reference_gpu(name):
    from footsies_gym_amd.vector_env import FootsiesVectorEnv
    wr.replay(name, lambda n, dense, seed, delay: FootsiesVectorEnv(n, opponent=None, dense_reward=dense, seed=seed,
                                                                    autoreset_mode="next_step", frame_delay=delay))


def test_battle_state_json_into_gpu_continues_like_oracle(oracle_lib):
    """Oracle arenas mid-episode -> BattleState JSON -> loaded into GPU arenas (which keep
    their own non-BattleState fields, copied from the oracle first) -> identical futures."""
    from footsies_gym_amd import battle_state as B
    from footsies_gym_amd.vector_env import FootsiesVectorEnv
    n = 300
    rng = np.random.default_rng(8)
    ora = oracle_lib.Oracle(n, p2_mode=_abi.FS_P2_EXTERNAL, base_seed=2)
    for _ in range(210):
        ora.step(rng.integers(0, 8, n), rng.integers(0, 8, n))
    snap = ora.state()
    venv = FootsiesVectorEnv(n, opponent=lambda o, i: np.zeros(n, np.uint8), seed=2)
    venv.load_battle_state(snap)  # the non-BattleState fields (recording, reward sum, ...)
    base = venv.save_battle_state()
    base["f"]["action_id"] = 0
    base["f"]["position_x"] = 0.0
    venv.load_battle_state(base)
    for i in range(n):
        venv.load_battle_state_json(B.dumps(B.battle_state(snap, i)), arena=i)
    compare_states(snap, venv.save_battle_state())
    for t in range(300):
        a1, a2 = rng.integers(0, 8, n).astype(np.uint8), rng.integers(0, 8, n).astype(np.uint8)
        venv.sim.step(a1, a2)
        compare_outputs(ora.step(a1, a2), venv.sim.outputs_numpy(), step=t)
    venv.close()


def test_single_env_battle_state_roundtrip():
    from footsies_gym_amd.vector_env import FootsiesEnv
    env = FootsiesEnv(opponent=lambda o, i: (False, True, False))
    env.reset()
    for t in range(77):
        env.step((t % 3 == 0, False, t % 5 == 0))
    saved = env.save_battle_state()
    after = [env.step((False, t % 2 == 0, False)) for t in range(40)]
    env.load_battle_state(saved)
    again = [env.step((False, t % 2 == 0, False)) for t in range(40)]
    for (o1, r1, d1, _, i1), (o2, r2, d2, _, i2) in zip(after, again):
        assert o1 == o2 and r1 == r2 and d1 == d2 and i1["frame"] == i2["frame"]
    env.close()


@pytest.mark.parametrize("name", wire_replay.CASES)
def test_wire_server_gpu_replays_reference_client_traffic(name):
    """The reference client's recorded traffic, served by the GPU-backed game server."""
    from footsies_gym_amd.server import SimBackend
    assert wire_replay.replay(name, lambda p2_bot, seed: SimBackend(p2_bot=p2_bot, seed=seed)) > 1000


def test_wire_server_p2_bot_toggle():
    """P2_BOT switches P2 between the remote actor and the in-game bot mid-battle."""
    import json
    import struct
    import threading
    from footsies_gym_amd.server import FootsiesServer
    srv = FootsiesServer("127.0.0.1", 0, 0, 0, seed=5)
    th = threading.Thread(target=srv.serve, daemon=True)
    th.start()
    p1 = wire_client.connect("127.0.0.1", srv.ports["p1"])
    rc = wire_client.connect("127.0.0.1", srv.ports["rc"])
    p2 = wire_client.connect("127.0.0.1", srv.ports["p2"])

    def state():
        return json.loads(wire_client.recv_message(p1)[4:])

    def command(c, v=""):
        m = json.dumps({"command": c, "value": v}).encode()
        rc.sendall(struct.pack("!I", len(m)) + m)

    s = state()
    assert s["globalFrame"] == -1
    p2_moves = {"remote": set(), "bot": set(), "remote again": set()}
    for phase, remote in (("remote", True), ("bot", False), ("remote again", True)):
        command(4, str(not remote))
        for t in range(150):
            p1.sendall(bytes([0, 0, 0]))
            if remote:
                p2.sendall(bytes([0, 0, 0]))
            s = state()
            if s["p1Vital"] == 0 or s["p2Vital"] == 0:
                s = state()  # the next episode's state(-1)
            p2_moves[phase].add(s["p2Move"])
    assert p2_moves["remote"] <= {0}  # an idle remote P2 only stands
    assert len(p2_moves["bot"]) > 1    # the bot moves
    assert 0 in p2_moves["remote again"]
    for x in (p1, rc, p2):
        x.close()
    srv.stop()
    th.join(timeout=30)


def test_policy_rollout_graph_matches_oracle(oracle_lib):
    """C5 loop: MLP actor + fs_step captured in a HIP graph; the actions it sampled, replayed
    through the oracle (same bot seeds), give the same outputs and state."""
    import torch
    from footsies_gym_amd.rollout import PolicyRollout, make_actor
    from footsies_gym_amd.simulator import FootsiesSim
    N = 2000
    sim = FootsiesSim(N, p2_mode="bot", seed=13)
    ora = oracle_lib.Oracle(N, p2_mode=_abi.FS_P2_BOT, base_seed=13)
    ro = PolicyRollout(sim, make_actor(device=torch.device("cuda", 0), seed=4))
    for a in ro.capture(7, warmup=3, log=True):
        ora.step(a.numpy())
    for _ in range(4):
        ro.replay()
        torch.cuda.synchronize()
        for a in ro.action_log.cpu().numpy():
            exp = ora.step(a)
    assert len(np.unique(ro.action_log.cpu().numpy())) == 8
    compare_outputs(exp, sim.outputs_numpy())
    compare_states(ora.state(), sim.get_state())


def test_game_binary_stand_in_with_reference_command_line():
    """bin/FOOTSIES started with the argument list FootsiesEnv._instantiate_game builds
    (FE:193-259, bot P2, no render) serves the same frames as a one-arena FootsiesSim."""
    import json
    import os
    import socket
    import subprocess
    from footsies_gym_amd.server import env_state_json
    from footsies_gym_amd.simulator import FootsiesSim
    ports = []
    for _ in range(2):
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            ports.append(s.getsockname()[1])
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    args = [os.path.join(root, "bin", "FOOTSIES"), "--mute", "--training", "--p1-address", "127.0.0.1", "--p1-port",
            str(ports[0]), "--remote-control-address", "127.0.0.1", "--remote-control-port", str(ports[1]),
            "-force-gfx-direct", "-batchmode", "-nographics", "--fast-forward", "--fast-forward-speed", "6.0",
            "--synced-non-blocking", "--p2-bot", "-nolog"]
    proc = subprocess.Popen(args, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
    try:
        p1 = wire_client.connect("127.0.0.1", ports[0], timeout=120)
        rc = wire_client.connect("127.0.0.1", ports[1], timeout=120)
        ref = FootsiesSim(1, p2_mode="bot", autoreset_mode="next_step", seed=0)
        got = wire_client.recv_message(p1)[4:].decode()
        assert got == env_state_json(ref.env_state()[0])
        rng = np.random.default_rng(3)
        for t in range(400):
            a = rng.integers(0, 2, 3)
            p1.sendall(bytes(int(x) for x in a))
            ref.step(np.array([a[0] | a[1] << 1 | a[2] << 2], np.uint8))
            assert wire_client.recv_message(p1)[4:].decode() == env_state_json(ref.env_state()[0]), t
            if ref.outputs_numpy()["terminated"][0]:
                ref.reset()
                assert json.loads(wire_client.recv_message(p1)[4:])["globalFrame"] == -1
        p1.close()
        rc.close()
        assert proc.wait(timeout=60) == 0, proc.stderr.read()
    finally:
        if proc.poll() is None:
            proc.kill()
            proc.wait()


def test_hashed_actions_match_host_stream(oracle_lib):
    """fs_hash_actions / in-kernel hashing == the splitmix64 stream of SURVEY.md §8(d)."""
    from footsies_gym_amd.simulator import FootsiesSim
    N = 3000
    s = FootsiesSim(N, p2_mode="external")
    p1, p2 = s.hash_actions(4, seed=0x5EED, t0=10)
    for t in range(4):
        assert np.array_equal(p1[t].cpu().numpy(), oracle_lib.hash_actions(0x5EED, N, 10 + t, 0))
        assert np.array_equal(p2[t].cpu().numpy(), oracle_lib.hash_actions(0x5EED, N, 10 + t, 1))
    # in-kernel hashed actions (no action arrays) follow the same stream
    ora = oracle_lib.Oracle(N, p2_mode=_abi.FS_P2_EXTERNAL)
    s2 = FootsiesSim(N, p2_mode="external")
    s2.step_n(25, None, None, action_seed=0x5EED)
    ora.step_n_hashed(25, 0x5EED)
    compare_states(ora.state(), s2.get_state())


def test_set_state_rejects_queue_index_past_its_plan():
    """A bot queue index at or past its plan's length is no state the bot can be in (the queue
    would be empty, exported as plan -1): fs_set_state rejects it, accepts the last input."""
    from footsies_gym_amd._lib import FootsiesError
    from footsies_gym_amd.simulator import FootsiesSim
    sim = FootsiesSim(4, p2_mode="bot", seed=0)
    st = sim.get_state()
    for plan_key, idx_key, plan, length in (("move_plan", "move_index", 2, 56),
                                            ("attack_plan", "attack_index", 4, 121)):
        bad = st.copy()
        bad[plan_key][1], bad[idx_key][1] = plan, length
        with pytest.raises(FootsiesError):
            sim.set_state(bad)
        ok = st.copy()
        ok[plan_key][1], ok[idx_key][1] = plan, length - 1
        sim.set_state(ok)
        got = sim.get_state()
        assert got[plan_key][1] == plan and got[idx_key][1] == length - 1
    sim.close()


@pytest.mark.parametrize("p2", ["bot", "external"])
def test_state_save_load_roundtrip(oracle_lib, p2):
    """fs_get_state -> fs_set_state into a fresh handle continues bit-identically."""
    from footsies_gym_amd.simulator import FootsiesSim
    N = 700
    a = FootsiesSim(N, p2_mode=p2, seed=1)
    rng = np.random.default_rng(0)
    for _ in range(300):
        a.step(rng.integers(0, 8, N), rng.integers(0, 8, N) if p2 == "external" else None)
    st = a.get_state()
    b = FootsiesSim(N, p2_mode=p2, seed=999)
    b.set_state(st)
    compare_states(st, b.get_state())
    for t in range(200):
        x1, x2 = rng.integers(0, 8, N), rng.integers(0, 8, N)
        a.step(x1, x2 if p2 == "external" else None)
        b.step(x1, x2 if p2 == "external" else None)
        oa, ob = a.outputs_numpy(), b.outputs_numpy()
        compare_outputs(oa, ob, step=t)


def test_device_actions_and_stream_interop():
    """Device-tensor actions produced by torch kernels on torch's stream need no sync."""
    import torch
    from footsies_gym_amd.simulator import FootsiesSim
    N = 4096
    a = FootsiesSim(N, p2_mode="external", seed=5)
    b = FootsiesSim(N, p2_mode="external", seed=5)
    g = torch.Generator(device="cuda").manual_seed(0)
    for _ in range(50):
        x1 = torch.randint(0, 8, (N,), device="cuda", dtype=torch.uint8, generator=g)
        x2 = torch.randint(0, 8, (N,), device="cuda", dtype=torch.uint8, generator=g)
        a.step(x1, x2)  # device path
        b.step(x1.cpu().numpy(), x2.cpu().numpy())  # host path
        oa = {k: v.clone() for k, v in a.outputs().items()}
        ob = b.outputs_numpy()
        compare_outputs(ob, {k: v.cpu().numpy() for k, v in oa.items()})


def test_vector_env_surface():
    from footsies_gym_amd import vector_env as ve
    from footsies_gym_amd.vector_env import FootsiesVectorEnv
    tuned = ve._HEAP_RETAINED
    env = FootsiesVectorEnv(64, seed=0)
    assert ve._HEAP_RETAINED == tuned  # the glibc tuning is opt-in (retain_host_heap=True)
    obs, info = env.reset(seed=42)
    assert obs["guard"].shape == (64, 2) and obs["guard"].dtype == np.int64
    assert (obs["position"][:, 0] == -2).all() and (info["frame"] == -1).all()
    assert env.observation_space.contains(obs)
    total_eps = 0
    rng = np.random.default_rng(0)
    for _ in range(400):
        obs, rew, term, trunc, info = env.step(rng.integers(0, 2, (64, 3)).astype(bool))
        assert rew.dtype == np.float64 and term.dtype == bool and not trunc.any()
        if term.any():
            total_eps += int(term.sum())
            i = int(np.nonzero(term)[0][0])
            assert info["final_observation"][i] is not None
            # final_info holds the final observation's own rows (FE:379), read-only
            fo, fi = info["final_observation"][i], info["final_info"][i]
            assert all(fi[k] is fo[k] and not fo[k].flags.writeable for k in fo)
            assert info["frame"][i] == -1  # same-step auto-reset: obs is the new episode's state(-1)
            assert obs["move"][i].tolist() == [0, 0]
        assert env.observation_space.contains(obs)
    assert total_eps > 0
    env.close()


def test_vector_env_custom_opponent_and_torch_output():
    import torch
    from footsies_gym_amd.vector_env import FootsiesVectorEnv
    calls = []

    def opponent(obs, info):
        calls.append(1)
        return np.full(16, 4, np.uint8)  # always attack
    env = FootsiesVectorEnv(16, opponent=opponent, output="torch")
    obs, _ = env.reset()
    o, r, te, tr, info = env.step(torch.zeros(16, dtype=torch.uint8, device="cuda"))
    assert calls and o["guard"].is_cuda and r.dtype == torch.float64
    env.close()


def test_single_env_adapter_matches_reference_api():
    from footsies_gym_amd.vector_env import FootsiesEnv
    env = FootsiesEnv(dense_reward=True)
    obs, info = env.reset(seed=0)
    assert obs == {"guard": (3, 3), "move": (0, 0), "move_frame": (0, 0), "position": (-2.0, 2.0)}
    assert info["frame"] == -1 and info["p1_action"] == (False, False, False)
    done = False
    n = 0
    while not done and n < 5000:
        obs, reward, done, trunc, info = env.step((False, False, True) if n % 2 else (False, True, False))
        assert isinstance(reward, float) and trunc is False
        n += 1
    assert done
    obs, info = env.reset()
    assert info["frame"] == -1
    env.close()


def test_pack_outputs_kernel_matches_host_packing():
    """fs_pack_outputs (one kernel) == parallel.pack_outputs (torch ops) byte for byte, and
    ShardedSim.gather's unpacking restores the outputs."""
    import torch
    from footsies_gym_amd import parallel
    from footsies_gym_amd.simulator import FootsiesSim
    sim = FootsiesSim(1003, p2_mode="external", seed=2)
    p1, p2 = sim.hash_actions(300, seed=9)
    terminals = 0
    for t in range(300):
        sim.step(p1[t], p2[t])
        if t >= 100:
            got = sim.pack_outputs()
            want = parallel.pack_outputs(sim.outputs(), torch)
            assert bool(torch.equal(got, want)), t
            terminals += int(sim.outputs()["terminated"].sum())
    assert terminals > 0  # terminal rows covered
    back = parallel.unpack_outputs(got, torch)
    for k, v in back.items():
        assert bool(torch.equal(v, sim.outputs()[k])), k


@pytest.mark.parametrize("n,kw", [
    (1003, dict(p2_mode="external")),
    (1003, dict(p2_mode="bot", dense_reward=False)),
    (1003, dict(p2_mode="external", autoreset_mode="next_step", float_mode="double")),
    (777, dict(p2_mode="bot", p1_mode="bot", autoreset_mode="next_step")),
    (3, dict(p2_mode="external")),  # few arenas: host actions travel in the kernel arguments
    (513, dict(p2_mode="external", frame_delay=2)),  # the delayed queue: fs_step + fs_pack_outputs
    (2049, dict(p2_mode="external", geom=True)),  # general-geometry tick: y, -0.0 y, flipped
    (1500, dict(p2_mode="bot", geom=True)),
])
def test_step_rec_equals_step_then_pack(n, kw):
    """fs_step_rec (k_step writes the 40-byte gather records itself) == fs_step followed by
    fs_pack_outputs, byte for byte, on twin handles over 400 steps with terminal and reset rows,
    and the outputs the handle keeps are the same as well.  `geom`: both handles first load the
    same arbitrary states with fighters off the ground (some at y = -0.0) and flipped facings, so
    the steps run env_step<..., GEOM> and its record stores (write_record under GEOM)."""
    import numpy as np
    import torch
    from footsies_gym_amd import parallel
    from footsies_gym_amd.simulator import FootsiesSim
    from tests.parity_utils import random_states
    kw = dict(kw)
    geom = kw.pop("geom", False)
    a, b = FootsiesSim(n, seed=4, **kw), FootsiesSim(n, seed=4, **kw)
    if geom:
        st = random_states(n, np.random.default_rng(77), p2=kw["p2_mode"], geom_frac=0.3)
        st["f"]["position_y"][::17, 0] = np.float32(-0.0)
        assert (st["f"]["position_y"] != 0).any() and (st["f"]["facing_flipped"] == 1).any()
        assert np.signbit(st["f"]["position_y"][::17, 0]).all()
        a.set_state(st)
        b.set_state(st)
    p1, p2 = a.hash_actions(400, seed=13)
    host = n <= 8
    terminals = 0
    for t in range(400):
        q1 = None if kw.get("p1_mode") == "bot" else p1[t]
        q2 = p2[t] if kw["p2_mode"] == "external" else None
        if host:
            b.step(q1.cpu().numpy(), q2.cpu().numpy())
        else:
            b.step(q1 if q1 is not None else None, q2)
        want = b.pack_outputs()
        got = a.step_records(q1, q2) if not host else _step_rec_host(a, q1, q2)
        assert bool(torch.equal(got, want)), (t, (got != want).nonzero()[:4].tolist())
        terminals += int(b.outputs()["terminated"].sum())
    assert terminals > 0
    for k, v in b.outputs().items():
        assert bool(torch.equal(v, a.outputs()[k])), k
    back = parallel.unpack_outputs(got, torch)
    for k, v in back.items():
        assert bool(torch.equal(v, b.outputs()[k])), k


def _step_rec_host(sim, q1, q2):
    """fs_step_rec with host action bytes (the few-arena inline-argument path)."""
    import ctypes as C
    import numpy as np
    import torch
    from footsies_gym_amd import _abi
    from footsies_gym_amd._lib import check, lib
    a1 = np.ascontiguousarray(q1.cpu().numpy())
    a2 = np.ascontiguousarray(q2.cpu().numpy())
    dst = torch.empty((sim.num_envs, _abi.FS_RECORD_BYTES), dtype=torch.uint8, device=sim.device)
    check(lib().fs_step_rec(sim._h, a1.ctypes.data, a2.ctypes.data, _abi.FS_ACT_HOST, C.c_void_p(dst.data_ptr())),
          sim._h)
    return dst


def test_step_rec_rejects_bad_destinations():
    import ctypes as C
    from footsies_gym_amd import _abi
    from footsies_gym_amd._lib import lib
    from footsies_gym_amd.simulator import FootsiesSim
    import torch
    s = FootsiesSim(16, p2_mode="bot")
    a = torch.zeros(16, dtype=torch.uint8, device=s.device)
    buf = torch.zeros(16 * 40 + 8, dtype=torch.uint8, device=s.device)
    assert lib().fs_step_rec(s._h, C.c_void_p(a.data_ptr()), None, _abi.FS_ACT_DEVICE, None) == _abi.FS_E_INVALID
    assert lib().fs_step_rec(s._h, C.c_void_p(a.data_ptr()), None, _abi.FS_ACT_DEVICE,
                             C.c_void_p(buf.data_ptr() + 4)) == _abi.FS_E_INVALID
    with pytest.raises(ValueError):
        s.step_records(a, dst=buf[:100])


@pytest.mark.parametrize("extra", [[], ["--global-envs", "4096", "--mode", "step"]])
def test_bench_json_contract(extra):
    """bench.py prints one JSON line with the driver's fields, the roofline and (1 GPU) the
    CPU baseline; --global-envs switches to strong scaling."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--envs", "4096", "--steps", "100", "--warmup", "10",
           "--chunk", "50", "--no-extras", "--cpu-seconds", "0.5", "--kernel-samples", "10"] + extra
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, check=True).stdout
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline", "step_gather_mode"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 100 and d["warmup"] == 10 and d["value"] > 0
    assert d["scaling"] == ("strong" if extra else "weak")
    r = d["roofline"]
    assert r["bound"] in ("hbm", "simd-issue") and 0 < r["frac"] < 1 and r["achieved"] == pytest.approx(r["frac"] * r["peak"])
    # the byte accounting: algorithmic (2 B in + 38 B out per env-step, 96 B of state per arena and
    # launch) and the packed layout's 2 B in + 40 B out beside it
    n, t = d["config"]["envs_per_gpu"], r["ticks_per_launch"]
    assert r["algorithmic_bytes_per_launch"] == n * (96 + 40 * t)
    packed = d["config"]["mode"] == "fused" and d["config"]["trajectory"].startswith("packed")
    assert r["layout_bytes_per_launch"] == n * (96 + (42 if packed else 40) * t)
    assert r["traffic_ratio"] is None or r["traffic_ratio"] == pytest.approx(r["traffic"] / r["algorithmic_bytes_per_launch"])
    assert d["cpu_baseline"]["kind"] == "port" and d["cpu_baseline"]["cores"] >= 1


def test_bench_extras_legs():
    """The side legs of the bench line at a small size: the bot opponent (C2), the per-arena actors
    (mixed P2 and by_example, the kActors kernels) each name the kernel that ran, and the
    VectorEnv leg times steady steps whatever --steps is."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--envs", "2048", "--steps", "20", "--warmup", "5",
           "--chunk", "20", "--roofline-ticks", "20", "--no-cpu-baseline", "--kernel-samples", "5"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=110, check=True).stdout
    d = json.loads([l for l in out.splitlines() if l.startswith("{")][-1])
    # (the side legs use the headline's trajectory layout, packed by default)
    assert d["p2_bot_mode"]["kernel"] == fused_kernel("fsk::k_step_n_packed<0, 1>", 2048) and d["p2_bot_mode"]["value"] > 0
    for leg in ("mixed_p2", "by_example"):
        assert d["actors_mode"][leg]["kernel"] == "fsk::k_step_n_packed<0, 3>", d["actors_mode"]
        assert d["actors_mode"][leg]["value"] > 0
    # the headline's fused trajectory is packed by default; the per-field layout is timed beside
    assert d["roofline"]["kernel"] == fused_kernel("fsk::k_step_n_packed<0, 0>", 2048)
    assert d["config"]["trajectory"].startswith("packed")
    assert d["fused_other_layout"]["kernel"] == fused_kernel("fsk::k_step_n<0, 0>", 2048)
    assert d["fused_other_layout"]["value"] > 0
    v = d["vector_env"]["numpy"]
    assert v["steps"] >= 200 and v["warmup_steps"] >= 200 and v["terminals_per_step"] > 0


def test_native_consumer_under_host_sanitizers():
    """tests/native/abi_lockstep: a C++ program on include/footsies.h, built with host-side
    ASan + UBSan over a sanitizer build of the library's host code, steps the GPU in lockstep
    with the linked-in oracle (bitwise state compare), checks determinism across handles, the
    packed gather records and the C-ABI's error paths."""
    import os
    import subprocess
    d = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native")
    b = subprocess.run(["make", "-C", d, "-j4"], capture_output=True, text=True, timeout=900)
    assert b.returncode == 0, b.stderr[-4000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1", UBSAN_OPTIONS="print_stacktrace=1",
               LSAN_OPTIONS="suppressions=" + os.path.join(d, "lsan.supp"))
    r = subprocess.run([os.path.join(d, "abi_lockstep")], env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-6000:])
    assert "all checks passed" in r.stdout


@pytest.mark.parametrize("p2", ["external", "bot"])
def test_long_fused_launches_split_like_one(monkeypatch, p2):
    """A fused call longer than one launch's 32-bit trajectory offsets allow runs as several
    launches over row ranges of the same buffers (fs_api.cpp step_chunked).  With the split
    forced at 3 ticks per launch, trajectories, actor samples and final states equal those of
    single launches: device actions, hashed actions and the in-kernel actor."""
    import torch
    from footsies_gym_amd.rollout import FusedPolicyRollout, make_actor
    from footsies_gym_amd.simulator import FootsiesSim
    N, T = 256, 37
    mk = lambda: FootsiesSim(N, p2_mode=p2, seed=11)  # noqa: E731
    one, split = mk(), mk()
    p1, q2 = one.hash_actions(T, seed=5, p2=(p2 == "external"))
    runs = []
    for sim, rows in ((one, None), (split, "1000")):
        if rows:
            monkeypatch.setenv("FOOTSIES_MAX_LAUNCH_ROWS", rows)
        got = []
        tr = sim.alloc_trajectory(T)
        sim.step_n(T, p1, q2, trajectory=tr)                  # device actions
        got.append(tr)
        if p2 == "bot":
            tr = sim.alloc_trajectory(T)
            sim.step_n(T, None, None, action_seed=9, trajectory=tr)  # hashed actions
            got.append(tr)
            ro = FusedPolicyRollout(sim, make_actor(device=sim.device, seed=2), seed=4)
            tr = sim.alloc_trajectory(T)
            acts, logp = ro.rollout(T, trajectory=tr)         # actor in the loop
            got += [tr, {"actions": acts, "logp": logp}]
        torch.cuda.synchronize()
        runs.append((got, sim.get_state()))
        monkeypatch.delenv("FOOTSIES_MAX_LAUNCH_ROWS", raising=False)
    for a, b in zip(runs[0][0], runs[1][0]):
        for k in a:
            assert torch.equal(a[k], b[k]), k
    compare_states(runs[0][1], runs[1][1])
    one.close()
    split.close()


def test_single_env_after_close_raises_game_closed_error():
    """The single-arena FootsiesEnv, like the reference's, refuses use after close()."""
    from footsies_gym_amd import FootsiesGameClosedError
    from footsies_gym_amd.vector_env import FootsiesEnv
    env = FootsiesEnv(seed=1)
    env.reset()
    env.step((False, True, False))
    env.close()
    env.close()  # idempotent
    with pytest.raises(FootsiesGameClosedError):
        env.step((False, False, True))
    with pytest.raises(FootsiesGameClosedError):
        env.reset()


@pytest.mark.parametrize("opponent,delay", [(None, 0), ("callable", 0), (None, 2)])
def test_single_env_step_equals_one_arena_vector_env(opponent, delay):
    """FootsiesEnv.step (its direct host conversion) == FootsiesVectorEnv(1, next-step auto-reset)
    through the batch path, step for step over terminations, with the bot or a remote P2."""
    from footsies_gym_amd.simulator import encode_actions
    from footsies_gym_amd.vector_env import FootsiesEnv, FootsiesVectorEnv
    seen = []

    def opp(obs, info):  # reads the agent's most recent single-arena dicts (FE:525-527)
        seen.append(obs["position"])
        return (False, obs["position"][0] < 0, True)
    single = FootsiesEnv(seed=3, opponent=None if opponent is None else opp, frame_delay=delay)

    def batch_opp(obs, info):  # the same P2 policy over the batch env's own (obs, info)
        return np.array([encode_actions([opp(*FootsiesEnv._py(obs, info))])[0]], np.uint8)
    wrapped = None if opponent is None else batch_opp
    venv = FootsiesVectorEnv(1, seed=3, autoreset_mode="next_step", opponent=wrapped, frame_delay=delay)
    rng = np.random.default_rng(5)
    o1, i1 = single.reset(seed=3)
    o2, i2 = FootsiesEnv._py(*venv.reset(seed=3))
    assert (o1, i1) == (o2, i2)
    dones = 0
    for t in range(3000):
        a = tuple(bool(b) for b in rng.integers(0, 2, 3))
        o1, r1, d1, tr1, i1 = single.step(a)
        obs, rew, term, trunc, info = venv.step(np.asarray([a]).reshape(1, 3))
        o2, i2 = FootsiesEnv._py(obs, info)
        assert (o1, r1, d1, tr1, i1) == (o2, float(rew[0]), bool(term[0]), False, i2), t
        if d1:
            dones += 1
            assert single.reset() == FootsiesEnv._py(*venv.reset())
    assert dones > 0
    if opponent is not None:
        assert seen
    single.close()
    venv.close()


@pytest.mark.parametrize("n,p2", [(1, "bot"), (5, "external")])
def test_host_outputs_equal_device_outputs(n, p2):
    """FootsiesSim(host_outputs=True) -- the kernels write the outputs into pinned host memory --
    gives the outputs of a device-output handle, step for step, over terminals and resets."""
    from footsies_gym_amd.simulator import FootsiesSim
    a, b = FootsiesSim(n, p2_mode=p2, seed=4), FootsiesSim(n, p2_mode=p2, seed=4, host_outputs=True)
    assert not b.outputs()["guard"].is_cuda
    compare_outputs(a.outputs_numpy(), b.outputs_numpy(), step=-1)
    rng = np.random.default_rng(9)
    terminals = 0
    for t in range(3000):
        a1, a2 = rng.integers(0, 8, n).astype(np.uint8), rng.integers(0, 8, n).astype(np.uint8)
        q2 = a2 if p2 == "external" else None
        a.step(a1, q2)
        b.step(a1, q2)
        oa, ob = a.outputs_numpy(), b.outputs_numpy()
        compare_outputs(oa, ob, step=t)
        terminals += int(oa["terminated"].sum())
        if t % 700 == 0:
            a.reset(hard=True)
            b.reset(hard=True)
            compare_outputs(a.outputs_numpy(), b.outputs_numpy(), step=t)
    assert terminals > 0
    compare_states(a.get_state(), b.get_state(), step=3000)
    a.close()
    b.close()


@pytest.mark.parametrize("p2", ["bot", "external"])
def test_host_outputs_read_straight_from_step(p2):
    """With host_outputs the tensors sim.step / sim.reset / sim.outputs return are pinned host
    memory the kernels write asynchronously; each of those calls waits for the handle's stream
    first, so reading them at once gives this tick's values (advisor r03: they could hold the
    previous tick's).  Read with no outputs_numpy call in between, against a device-output twin."""
    from footsies_gym_amd.simulator import FootsiesSim
    n = 7
    a, b = FootsiesSim(n, p2_mode=p2, seed=11), FootsiesSim(n, p2_mode=p2, seed=11, host_outputs=True)
    rng = np.random.default_rng(3)
    terminals = 0
    for t in range(600):
        a1, a2 = rng.integers(0, 8, n).astype(np.uint8), rng.integers(0, 8, n).astype(np.uint8)
        q2 = a2 if p2 == "external" else None
        a.step(a1, q2)
        out = b.step(a1, q2)  # read immediately: no sync by the caller
        got = {k: v.numpy().copy() for k, v in out.items()}
        compare_outputs(a.outputs_numpy(), got, step=t)
        terminals += int(got["terminated"].sum())
        if t % 250 == 249:
            a.reset(hard=True)
            got = {k: v.numpy().copy() for k, v in b.reset(hard=True).items()}
            compare_outputs(a.outputs_numpy(), got, step=t)
            compare_outputs(a.outputs_numpy(), {k: v.numpy().copy() for k, v in b.outputs().items()}, step=t)
    assert terminals > 0
    a.close()
    b.close()


def test_step_kernel_names_the_launched_kernel():
    """fs_step_kernel names the kernel launch_step picks (advisor r03: bench's roofline / PMC lookups
    hard-coded k_step_n<0, 0>, which is not what runs from 131 072 arenas on)."""
    import ctypes as C
    import os
    from footsies_gym_amd._lib import lib
    from footsies_gym_amd.simulator import FootsiesSim
    L = lib()
    a = FootsiesSim(64, p2_mode="external")
    name = lambda s, n, fl=0: L.fs_step_kernel(s.handle, n, fl).decode()  # noqa: E731
    assert name(a, 1) == "fsk::k_step<0, 0>"
    forced = os.environ.get("FOOTSIES_FUSED_LANES", "")
    assert name(a, 1000) == ("fsk::k_step_n1<0, 0>" if forced == "1" else fused_kernel("fsk::k_step_n<0, 0>", 64))
    assert name(a, 1000, 1) == "fsk::k_step_n_hashed<0, 0>" and name(a, 20, 2) == "fsk::k_step_n_policy<0, 0>"
    a.set_p2_mode("bot", np.arange(64) % 2 == 0)
    assert name(a, 1000) == "fsk::k_step_n<0, 3>"  # per-arena actors
    assert L.fs_step_kernel(a.handle, 0, 0) is None and L.fs_step_kernel(a.handle, 1, 8) is None
    a.close()
    b = FootsiesSim(64, p2_mode="bot", float_mode="double")
    assert name(b, 1) == "fsk::k_step<1, 1>"
    b.close()
    big = FootsiesSim(131072, p2_mode="external")
    if not forced:
        assert name(big, 1000) == "fsk::k_step_n1<0, 0>"  # two one-lane waves per SIMD on MI355X
    big.close()
    # packed launches with a remote P2 from four one-lane waves per SIMD on: the two-lane kernel
    # (fs_kernels.hip fused_one_lane); the scripted bot, and every per-field launch, keep the one-lane one
    for p2, want in (("external", "fsk::k_step_n_packed<0, 0>"), ("bot", "fsk::k_step_n1_packed<0, 1>")):
        huge = FootsiesSim(262144, p2_mode=p2)
        if not forced:
            assert name(huge, 1000, 4) == want, p2
            assert name(huge, 1000) == "fsk::k_step_n1<0, %d>" % (p2 == "bot"), p2
        huge.close()
