#!/usr/bin/env python3
"""bench.py -- env-steps/sec of the FOOTSIES hot path on MI355X (BASELINE.json's metric).

Workload (BASELINE.json configs[2], "C3"): 65 536 arenas per GPU, self-play with
synthetic random actions for both players (the splitmix64 stream of SURVEY.md
§8(d), generated into HBM by fs_hash_actions before the timed region).  One
"step" = one Fight tick of every arena with full per-step outputs (obs, reward,
terminated/truncated, info) written to HBM and auto-reset of finished episodes
-- exactly FootsiesEnv.step's work for all arenas.

Modes
  fused (default): fs_step_n, `--chunk` ticks per kernel launch, every tick's
                   outputs kept in a [chunk][N] rollout buffer in HBM.
  step:            fs_step, one kernel launch per tick (the VectorEnv.step path).
Both modes are timed and reported; `value` is the --mode one.

Multi-GPU: one process per GPU, arenas sharded per rank with no data-path collective
(`scaling: weak`); max-over-ranks timing.  `python bench.py --gpus N` starts the N ranks
itself (a torch.distributed.run child, started before this process touches the GPU);
under an outside launcher (WORLD_SIZE set) it is one of the ranks and checks that the
launcher's world size is N.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "env-steps/sec (whole node) at 65 536 envs; bit-exact vs Unity ref"
MI355X_SIMDS = 256 * 4  # CUs x SIMDs per CU (MI355X_MICROARCH.md)
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md, chip-level parameters (8.0 TB/s spec)
STATE_BYTES = 96        # per arena per launch: 48 B state read + 48 B written (fs_kernels.hip layout)
# per env-step, algorithmic (the useful bytes, whatever the layout): 2 B of actions in + 38 B of
# outputs out (include/footsies.h fs_outputs' fields).  The headline's packed layout
# (fs_step_n_packed, fs_packed_traj) writes those 38 B as two 16-B lane records + the 8-B reward,
# i.e. 40 B out: 38 useful + 2 pad bytes in P2's record -- 42 B moved per env-step, 5 % above this
# figure; `roofline.traffic_ratio` (PMC traffic / algorithmic bytes) reports the difference.
STEP_IO_BYTES = 40
PACKED_STEP_MOVED_BYTES = 42  # 2 B in + 40 B out per env-step in the packed layout (incl. the pad)
XGMI_LINK_GBPS = 153.0  # per xGMI link and direction (task brief: 7 links x ~153 GB/s per MI355X)
LEG_TICKS = 1000        # ticks per region (and per launch) of the fused side legs, whatever --steps is
VENV_STEPS = 200        # timed FootsiesVectorEnv steps, after a warm-up into steady state


LAYOUT_DEFAULT = "packed"
C4_GLOBAL_ENVS = 262144  # BASELINE.json configs[3]: 262 144 arenas sharded over the node's GPUs


def c4_split(world, rank, total=C4_GLOBAL_ENVS):
    """The c4_strong leg's shard of this rank: (arenas, arena_base).  A contiguous range of the
    global arena indices, so seeds and the hashed action rows (fs_config.arena_base) are those of
    the same arenas in one unsharded run; 262 144 / N per rank (strong scaling)."""
    if total % world:
        return None  # (no even split: the leg is skipped and the line says why)
    n = total // world
    return n, rank * n


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); default: the launcher's WORLD_SIZE, else 1")
    # SURVEY 8(d)'s C3 protocol: 200 warm-up steps, then 5 timed runs of 2 000 steps (median)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--envs", type=int, default=65536, help="arenas per GPU (weak scaling)")
    ap.add_argument("--global-envs", type=int, default=0,
                    help="strong scaling: this many arenas in total, split evenly over the ranks "
                         "(SURVEY 8(d) C4: 262144); overrides --envs")
    ap.add_argument("--mode", choices=["fused", "step"], default="fused")
    ap.add_argument("--chunk", type=int, default=1000, help="ticks per fs_step_n launch (fused mode; SURVEY 8(d) C3: n=1000)")
    ap.add_argument("--layout", choices=["packed", "fields"], default=LAYOUT_DEFAULT,
                    help="fused mode's trajectory: packed records (fs_step_n_packed, two stores per tick) or one "
                         "array per field (fs_step_n); the other layout is timed beside as a secondary leg")
    ap.add_argument("--seed", type=lambda s: int(s, 0), default=0x5EED)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target length of the cpu_baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--kernel-samples", type=int, default=50, help="launches timed back-to-back for roofline")
    ap.add_argument("--regions", type=int, default=5,
                    help="timed regions of exactly --steps steps each, back to back; value = the median region")
    ap.add_argument("--roofline-ticks", type=int, default=1000,
                    help="ticks per fs_step_n launch of the roofline block (the shape profiles/ covers)")
    ap.add_argument("--no-extras", action="store_true", help="skip the C2 bot-opponent and C5 policy-loop rates")
    ap.add_argument("--no-solo-group", action="store_true",
                    help="a plain one-GPU run stays without a process group (default: a one-rank RCCL group, so the "
                         "per-step gather legs run their collective at N = 1 too)")
    ap.add_argument("--no-c4", action="store_true",
                    help="skip the c4_strong leg (262 144 arenas split over the ranks, BASELINE configs[3])")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="process group for N>1 (nccl = RCCL; gloo only to rehearse several ranks on one GPU)")
    ap.add_argument("--dry-run", action="store_true",
                    help="rehearse the launch / barrier / max-over-ranks / JSON plumbing with a no-op CPU step "
                         "(no GPU, no simulator; the line says dry_run and is never a measurement)")
    return ap.parse_args()


def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args):
    """`--gpus N` (N > 1) without an outside launcher: start N ranks, one per GPU, as one
    torch.distributed.run child process and return its exit code.  Called before anything
    touches the GPU (this process never initialises HIP), and the ranks are children, not
    an exec of this process."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % args.gpus,
           "--master-addr=127.0.0.1", "--master-port=%d" % free_port(), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.run(cmd, env=env).returncode


def cpu_baseline(envs, seconds, seed):
    """The CPU oracle (scalar C port, OpenMP over host cores) on a bounded sample."""
    from oracle import binding
    from footsies_gym_amd import _abi
    binding.build()
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    binding.lib().or_set_threads(threads)
    threads = binding.lib().or_get_threads()
    o = binding.Oracle(envs, p2_mode=_abi.FS_P2_EXTERNAL, base_seed=0)
    o.step_n_hashed(5, seed)  # warm-up / page-in
    t = time.perf_counter()
    o.step_n_hashed(10, seed)
    probe = time.perf_counter() - t
    steps = int(max(10, min(200000, seconds / max(probe / 10, 1e-9))))
    t = time.perf_counter()
    o.step_n_hashed(steps, seed)
    dt = time.perf_counter() - t
    # the same port on one thread (SURVEY.md 8(d) asks for both), a short sample
    binding.lib().or_set_threads(1)
    t = time.perf_counter()
    o.step_n_hashed(2, seed)
    probe1 = time.perf_counter() - t
    steps1 = int(max(2, min(100000, 0.2 * seconds / max(probe1 / 2, 1e-9))))
    t = time.perf_counter()
    o.step_n_hashed(steps1, seed)
    dt1 = time.perf_counter() - t
    binding.lib().or_set_threads(threads)
    o.close()
    return {"value": envs * steps / dt, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": "%d arenas x %d steps, self-play splitmix64 actions, oracle/liboracle.so (OpenMP %d threads), "
                      "%.1f s" % (envs, steps, threads, dt),
            "single_thread": {"value": envs * steps1 / dt1, "cores": 1,
                              "sample": "%d arenas x %d steps, 1 thread, %.1f s" % (envs, steps1, dt1)}}


def fused_leg(torch, N, ticks, chunk, seed, device, rank, kind, layout="fields"):
    """A fused-mode leg on its own handle, set up untimed; returns (run(k0, n), kernel name, close).
    kind "bot" = config C2's opponent at this size: P1 random (HBM), P2 the in-kernel BattleAI.
    kind "mixed_p2" = the per-arena actors (kActors, BC:158-167 P2_BOT): a remote-P2 handle with P2
    switched to the bot in every other arena (FE:458-480 set_opponent), both players' rows read.
    kind "by_example" = the bot as P1 too (GameManager.cs:87, 185-189; FE:118), P2 the bot."""
    from footsies_gym_amd import _abi
    from footsies_gym_amd._lib import check, lib
    from footsies_gym_amd.simulator import FootsiesSim
    import numpy as np
    if kind == "bot":
        sim = FootsiesSim(N, device=device, p2_mode="bot", seed=0, arena_base=rank * N)
    elif kind == "mixed_p2":
        sim = FootsiesSim(N, device=device, p2_mode="external", seed=0, arena_base=rank * N)
        sim.set_p2_mode("bot", (np.arange(N) % 2 == 0).astype(np.uint8))
    elif kind == "by_example":
        sim = FootsiesSim(N, device=device, p2_mode="bot", p1_mode="bot", seed=0, arena_base=rank * N)
    else:
        raise ValueError(kind)
    ext = kind == "mixed_p2"
    p1, p2 = sim.hash_actions(ticks, seed=seed, p2=ext)
    # the headline's trajectory layout (packed records unless --layout fields)
    packed = layout == "packed"
    if packed:
        traj = sim.alloc_packed_trajectory(chunk)
        td = _abi.fs_packed_traj(lanes=traj["lanes"].data_ptr(), reward=traj["reward"].data_ptr(),
                                 final_lanes=traj["final_lanes"].data_ptr())
    else:
        traj = sim.alloc_trajectory(chunk)
        td = _abi.fs_outputs(**{k: traj[k].data_ptr() for k in _abi.OUTPUT_SPEC})
    h, L = sim.handle, lib()
    b1 = p1.data_ptr()
    b2 = p2.data_ptr() if ext else None

    def run(k0, n):
        k = k0
        while k < k0 + n:
            m = min(chunk, k0 + n - k)
            q2 = C.c_void_p(b2 + k * N) if ext else None
            if packed:
                rc = L.fs_step_n_packed(h, m, C.c_void_p(b1 + k * N), q2, C.byref(td))
            else:
                rc = L.fs_step_n(h, m, C.c_void_p(b1 + k * N), q2, 0, C.byref(td))
            if rc:
                check(rc, h)
            k += m
    kname = L.fs_step_kernel(h, chunk, _abi.FS_KERNEL_PACKED if packed else 0).decode()

    def close():
        sim.close()
    return run, kname, close


LEG_CONFIG = {
    "bot": "C2 opponent: P1 random actions, P2 = in-kernel BattleAI",
    "mixed_p2": "per-arena actors: P2 remote in odd arenas, switched to the bot in even ones (set_opponent / P2_BOT)",
    "by_example": "by_example: the BattleAI plays P1 and P2 (bot vs bot, the agent observes)",
}


def policy_loop_rate(torch, N, steps, device):
    """Config C5: a 2x64 MLP actor samples P1's action from the outputs every step (P2 = bot);
    blocks of steps are captured into one HIP graph and replayed."""
    from footsies_gym_amd.rollout import PolicyRollout, make_actor
    from footsies_gym_amd.simulator import FootsiesSim
    sim = FootsiesSim(N, device=device, p2_mode="bot", seed=0)
    ro = PolicyRollout(sim, make_actor(device=torch.device("cuda", device)))
    block = 25
    ro.capture(block)
    ro.replay(2)
    torch.cuda.synchronize(device)
    reps = max(1, steps // block)
    t = time.perf_counter()
    ro.replay(reps)
    torch.cuda.synchronize(device)
    dt = time.perf_counter() - t
    sim.close()
    return {"value": N * reps * block / dt, "ms_per_step": 1e3 * dt / (reps * block), "graph_steps": block,
            "config": "C5: %d arenas, Linear(8,64)-tanh-Linear(64,64)-tanh-Linear(64,8) actor, Gumbel-max "
                      "sampling + log-prob, fs_step per step, P2 = bot, HIP graph replay" % N}


def fused_policy_rate(torch, N, steps, device, ticks=100):
    """Config C5 fused: the same actor evaluated inside the simulator kernel (bf16 MFMAs,
    fs_step_n_policy), `ticks` policy-driven ticks per launch, P1's actions and log-probs
    stored per tick ([ticks][N] each, what a PPO rollout keeps); P2 = bot.  Timed with HIP
    events on torch's current stream, where FootsiesSim issues its launches."""
    from footsies_gym_amd.rollout import FusedPolicyRollout, make_actor
    from footsies_gym_amd.simulator import FootsiesSim
    sim = FootsiesSim(N, device=device, p2_mode="bot", seed=0)
    ro = FusedPolicyRollout(sim, make_actor(device=torch.device("cuda", device)), seed=1)
    acts = torch.empty((ticks, N), dtype=torch.uint8, device=torch.device("cuda", device))
    logp = torch.empty((ticks, N), dtype=torch.float32, device=torch.device("cuda", device))
    ro.rollout(ticks, acts, logp)
    torch.cuda.synchronize(device)
    reps = max(1, steps // ticks)
    stream = torch.cuda.current_stream(device)  # FootsiesSim issues on torch's current stream
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record(stream)
    for _ in range(reps):
        ro.rollout(ticks, acts, logp)
    t1.record(stream)
    torch.cuda.synchronize(device)
    dt = t0.elapsed_time(t1) / 1e3
    sim.close()
    return {"value": N * reps * ticks / dt, "ms_per_step": 1e3 * dt / (reps * ticks), "ticks_per_launch": ticks,
            "config": "C5 fused: %d arenas, the same actor in bf16 MFMA inside the tick loop (fs_step_n_policy), "
                      "inverse-CDF sampling + log-prob stored per tick, P2 = bot" % N}


def ppo_rate(torch, N, device, horizon=128, iterations=3):
    """Config C5 end to end: PPO iterations (fused rollout of `horizon` ticks with the in-kernel
    actor, then GAE and 2 epochs x 4 minibatches of fp32 Adam updates of actor and critic, then
    the new weights copied into the kernel's buffers); P2 = bot.  `value` with the fused
    learner kernel (fs_ppo_grad) at PPOTrainer's default split-bf16 precision, `fp32_learner`
    with its fp32-FMA precision, `torch_learner` with the same loss through torch autograd.  One
    untimed warm-up iteration each."""
    from footsies_gym_amd.ppo import PPOTrainer
    from footsies_gym_amd.simulator import FootsiesSim
    rates = {}
    for key, learner, prec in (("hip_split", "hip", "split_bf16"), ("hip", "hip", "fp32"), ("torch", "torch", "fp32")):
        sim = FootsiesSim(N, device=device, p2_mode="bot", seed=0)
        tr = PPOTrainer(sim, horizon=horizon, learner=learner, learner_precision=prec)
        tr.train(1)
        rates[key] = tr.train(iterations)
        sim.close()
    return {"value": rates["hip_split"], "fp32_learner": rates["hip"], "torch_learner": rates["torch"],
            "horizon": horizon, "iterations": iterations,
            "config": "C5 end to end: %d arenas, PPO (fused rollout of %d ticks + GAE + 2x4 Adam minibatch "
                      "updates of the 8-64-64-8 actor and critic, gradients by fs_ppo_grad with the split-bf16 "
                      "hidden layer), P2 = bot"
                      % (N, horizon)}


def ppo_dp_rate(torch, N, device, rank, world, timed, horizon=128, iterations=3):
    """Config C5 over the ranks as one job: data-parallel PPO, N arenas per rank (arena_base =
    rank x N, P2 = bot), split-bf16 learner; each of the epochs x minibatches updates averages the
    flat gradient buffer over the ranks (one all_reduce SUM over RCCL, parallel.allreduce_mean_)
    and the advantages are normalised with every rank's statistics.  One untimed warm-up
    iteration, then one timed region of `iterations` iterations (barrier + synchronize, max over
    ranks); value = all ranks' samples / that wall."""
    from footsies_gym_amd import _abi
    from footsies_gym_amd.ppo import PPOTrainer
    from footsies_gym_amd.simulator import FootsiesSim
    sim = FootsiesSim(N, device=device, p2_mode="bot", seed=0, arena_base=rank * N)
    tr = PPOTrainer(sim, horizon=horizon, group="default")
    tr.train(1)
    wall = timed(lambda k0, n: tr.train(n, sync=False), 0, iterations)
    updates = tr.epochs * tr.minibatches
    sim.close()
    return {"value": world * N * horizon * iterations / wall, "unit": "env-steps/s",
            "ms_per_iteration": 1e3 * wall / iterations, "horizon": horizon, "iterations": iterations,
            "envs_per_rank": N, "allreduces_per_iteration": updates,
            "allreduce_bytes": 4 * (_abi.FS_PPO_ACTOR_PARAMS + _abi.FS_PPO_CRITIC_PARAMS),
            "config": "C5 data-parallel: %d ranks x %d arenas (P2 = bot), PPO with the fused rollout of %d ticks, "
                      "GAE, %d Adam minibatch updates per iteration, each minibatch's gradient averaged over the "
                      "ranks (all_reduce of the flat gradient buffer) and the advantages normalised with every "
                      "rank's statistics" % (world, N, horizon, updates)}


def vector_env_rate(torch, N, steps, device, warm=400):
    """The drop-in surface itself at the C3 size: FootsiesVectorEnv.step with numpy (N,) int
    actions in and numpy obs / reward / info out (the D2H copy, the conversions and gymnasium
    0.29's per-arena final_observation / final_info dicts of every step included), P2 a callable
    opponent returning pre-drawn numpy actions; then the same env with output="torch": device
    actions in, device tensors out (zero-copy).  `warm` untimed steps first, so the timed steps
    run at the steady terminal rate (right after a reset no episode can end for tens of steps),
    and `steps` timed steps whatever the bench's --steps is; the terminal count of the timed
    steps is reported."""
    import numpy as np
    from footsies_gym_amd.vector_env import FootsiesVectorEnv
    rng = np.random.default_rng(0)
    a1 = rng.integers(0, 8, (warm + steps, N)).astype(np.uint8)
    a2 = rng.integers(0, 8, (warm + steps, N)).astype(np.uint8)
    out = {}
    for kind in ("numpy", "torch"):
        k = [0]
        # each step's action rows are sliced out of the pre-drawn tables before the clock starts
        # (as a policy hands the env a fresh tensor per step): a torch row index costs ~1 us of its own
        if kind == "numpy":
            acts, r2 = list(a1), list(a2)
        else:
            acts = list(torch.as_tensor(a1, device=torch.device("cuda", device)).unbind(0))
            r2 = list(torch.as_tensor(a2, device=torch.device("cuda", device)).unbind(0))
        opp = (lambda obs, info: r2[k[0]])
        env = FootsiesVectorEnv(N, device=device, opponent=opp, output=kind, seed=0, retain_host_heap=kind == "numpy")
        env.reset(seed=0)
        for j in range(warm):
            k[0] = j
            env.step(acts[j])
        torch.cuda.synchronize(device)
        terms = []
        t = time.perf_counter()
        for j in range(warm, warm + steps):
            k[0] = j
            terms.append(env.step(acts[j])[2])
        torch.cuda.synchronize(device)
        dt = time.perf_counter() - t
        env.close()
        nterm = int(sum(int(x.sum()) for x in terms))
        out[kind] = {"value": N * steps / dt, "ms_per_step": 1e3 * dt / steps, "steps": steps,
                     "warmup_steps": warm, "terminals_per_step": nterm / steps}
    out["config"] = ("FootsiesVectorEnv(%d, opponent=callable).step: numpy actions -> numpy obs/info dicts "
                     "(D2H + conversion every step, final_observation dicts for the terminated arenas; retain_host_heap=True, "
                     "the opt-in glibc tuning), and "
                     "output='torch' (device tensors in/out); steady state after the warm-up" % N)
    return out


def single_env_rate(torch, steps, device):
    """The one-arena drop-in: FootsiesEnv (the reference's own API: tuples in, dicts out) vs the
    in-game bot, `steps` steps with random actions, auto-reset by the caller after terminal steps
    as FE's users do.  Latency-bound by design (one launch and one D2H per step); reported beside
    the reference's own per-game-process ceiling (<= 300 env-steps/s)."""
    import numpy as np
    from footsies_gym_amd.vector_env import FootsiesEnv
    rng = np.random.default_rng(1)
    acts = [tuple(bool(b) for b in row) for row in rng.integers(0, 2, (steps + 20, 3))]
    env = FootsiesEnv(device=device, seed=0)
    env.reset(seed=0)
    for j in range(20):
        if env.step(acts[j])[2]:
            env.reset()
    torch.cuda.synchronize(device)
    t = time.perf_counter()
    for j in range(20, 20 + steps):
        if env.step(acts[j])[2]:
            env.reset()
    dt = time.perf_counter() - t
    env.close()
    return {"value": steps / dt, "ms_per_step": 1e3 * dt / steps, "steps": steps,
            "config": "FootsiesEnv (1 arena, reference API: (left, right, attack) tuple in, obs/info dicts out), "
                      "P2 = in-game bot"}


def pmc_traffic(kernel, envs, ticks):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary
    (profiles/*_traffic.json, written by tools/summarize_profile.py from separate
    FETCH_SIZE / WRITE_SIZE passes over this same bench command): FETCH_SIZE x 2
    (gfx950 correction, MI355X_MICROARCH.md HBM section) + WRITE_SIZE, KiB -> bytes.
    None when no summary for this kernel at this arena count / ticks per launch."""
    import glob
    best = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_traffic.json"))):
        with open(path) as f:
            doc = json.load(f)
        for k in doc.get("kernels", []):
            if k["kernel"] == kernel and k["envs"] == envs and k["ticks_per_launch"] == ticks:
                best = (k["traffic_bytes_per_launch"], os.path.relpath(path, ROOT))
    return best


def issue_profile(kernel, envs, ticks):
    """The step kernel's instruction-issue picture, per wave and per SIMD, from committed summaries
    of the same kernel at the same arena count:
    * profiles/*_sq.json (tools/pmc_table.py --json over tools/prof_pmc.sh passes): instructions
      and VALU issued per wave-tick, wave cycles per wave-tick (quad-cycles) and the quad-cycles
      parked in s_waitcnt; `wave_frac` = one wave's issued instructions over its quad-cycles;
    * profiles/*_issue_model.json (tools/issue_model.py): the SIMD level.  `issue_frac` = the
      kernel's env-step rate at its own occupancy (2 waves per SIMD at 65 536 arenas) over the
      plateau the same kernel reaches at 4 and 8 waves per SIMD (tools/occupancy_sweep.sh), where
      only the SIMDs' issue is near its limit: the share of the SIMD issue rate this instruction
      stream can use that it does use.  Beside it the VALU pipe time priced by
      tools/valu_probe's per-class SIMD costs (plain 32-bit ops 2.4 cycles at 2 waves, VOP3-only /
      DPP / VOPC / SGPR-operand kinds 4.7-5.6), an estimate (the probe shows the costs do not add).
    None when no SQ summary matches."""
    import glob
    best = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_sq.json"))):
        with open(path) as f:
            doc = json.load(f)
        kernels = doc.get("kernels", []) if isinstance(doc, dict) else []
        for k in kernels if isinstance(kernels, list) else []:  # (other summaries have other layouts)
            if (isinstance(k, dict) and k.get("kernel") == kernel and k.get("envs") == envs
                    and k.get("ticks_per_launch") == ticks):
                pw = k["per_wave_tick"]
                best = {"insts_per_wave_tick": round(k["insts_per_wave_tick"], 1),
                        "valu_per_wave_tick": round(pw.get("SQ_INSTS_VALU", 0.0), 1),
                        "salu_per_wave_tick": round(pw.get("SQ_INSTS_SALU", 0.0), 1),
                        "wave_quad_cycles_per_wave_tick": round(pw.get("SQ_WAVE_CYCLES", 0.0), 1),
                        "wait_quad_cycles_per_wave_tick": round(pw.get("SQ_WAIT_ANY", 0.0), 1),
                        "waves_per_simd": k.get("waves", 0) / MI355X_SIMDS,
                        # instructions issued over the wave's quad-cycles: one wave's issue ceiling in use
                        "wave_frac": k["wave_issue_frac"], "ticks_per_launch_profiled": k["ticks_per_launch"],
                        "source": os.path.relpath(path, ROOT)}
    if best is None:
        return None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_issue_model.json"))):
        with open(path) as f:
            m = json.load(f)
        if isinstance(m, dict) and m.get("kernel") == kernel and m.get("envs") == envs:
            best.update({"issue_frac": m.get("issue_frac"),
                         "rate_by_waves_per_simd": m.get("rate_by_waves_per_simd"),
                         "valu_pipe_frac_priced": m["valu_pipe_frac_priced"],
                         "valu_pipe_frac_if_all_fast": m["valu_pipe_frac_if_all_fast"],
                         "simd_cycles_per_valu_class": m["simd_cycles_per_valu"],
                         "model_source": os.path.relpath(path, ROOT)})
    return best


def short_launch_attribution(ticks):
    """The committed critical-path split of an isolated launch of `ticks` ticks
    (profiles/*_t<ticks>_attribution.json, tools/short_launch_attribution.py over the stamped
    timeline of tools/timeline_probe.py), or None."""
    import glob
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_t%d_attribution.json" % ticks)))
    if not paths:
        return None
    with open(paths[-1]) as f:
        doc = json.load(f)
    return dict(doc["critical_path"], span_us=doc["span_us"], source=os.path.relpath(paths[-1], ROOT))


def dry_run(args, world, rank):
    """The multi-rank plumbing without a GPU: the same regions (barrier on both sides, host wall
    clock, max over ranks), a no-op CPU step, one JSON line from rank 0 marked dry_run."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
    K, R, N = args.steps, max(1, args.regions), args.envs
    x = torch.zeros(64)
    walls, local = [], []
    for _ in range(R):
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(K):
            x.add_(1.0)
        local.append(time.perf_counter() - t0)
        if world > 1:
            dist.barrier()
        t = torch.tensor([local[-1]], dtype=torch.float64)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        walls.append(float(t.item()))
    wall = sorted(walls)[len(walls) // 2]
    c4n, c4b = c4_split(world, rank) or (0, -1)
    mine = torch.tensor([float(N), sorted(local)[len(local) // 2], float(c4n), float(c4b)], dtype=torch.float64)
    every = [torch.zeros(4, dtype=torch.float64) for _ in range(world)]
    if world > 1:
        dist.all_gather(every, mine)
    else:
        every = [mine]
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": sum(float(e[0]) for e in every) * K / wall, "unit": "env-steps/s",
                          "n_gpus": world, "steps": K, "warmup": args.warmup, "ms_per_step": 1e3 * wall / K,
                          "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dry_run": True,
                          "dtype": "none (dry run)", "data": "none (dry run: no-op CPU step, not a measurement)",
                          "config": {"workload": "dry run", "envs_per_gpu": N, "global_envs": N * world,
                                     "parallelism": "arena-shard x%d" % world},
                          "ranks": {"world_size": world, "backend": dist.get_backend() if world > 1 else None,
                                    "rank_walls_ms": [round(1e3 * float(e[1]), 4) for e in every]},
                          # the c4_strong leg's plan as every rank computed it (no simulator in a dry run)
                          "c4_strong": {"global_envs": C4_GLOBAL_ENVS, "scaling": "strong",
                                        "envs_per_rank": [int(e[2]) for e in every],
                                        "arena_base_per_rank": [int(e[3]) for e in every]}}))
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    if args.gpus is not None and args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if args.gpus is not None and args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # the driver's plain `python3 bench.py --gpus N`: start the N ranks (nothing has touched the GPU)
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    # under a launcher, --gpus may be left out (the launcher's world size is taken); given, it must agree
    if args.gpus is not None and world != args.gpus:
        raise SystemExit("bench.py --gpus %d, but the launcher started %d rank(s) (WORLD_SIZE)" % (args.gpus, world))
    args.gpus = world
    if args.dry_run:
        return dry_run(args, world, rank)
    import torch
    import torch.distributed as dist

    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; the modulo only matters when ranks are rehearsed on fewer devices
    local = local % max(1, torch.cuda.device_count())
    # a process group whenever a launcher started the ranks, a single one included (the driver's
    # torch.distributed.run at N = 1, or tests/test_gpu_rccl.py): RCCL then carries the barrier,
    # the max-over-ranks and the gather modes at every N
    solo_group_error = None
    grouped = world > 1 or "WORLD_SIZE" in os.environ
    if grouped:
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    elif args.dist_backend == "nccl" and not args.no_solo_group:
        # the plain one-GPU run (the driver's `bench.py --gpus 1`) joins a one-rank RCCL group too, so
        # the per-step gather legs run their collective at N = 1 as well (RCCL's own kernels and
        # copies at world size 1); a failure to form it leaves the run ungrouped and says so
        torch.cuda.set_device(local)
        try:
            dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % free_port(), rank=0, world_size=1,
                                    device_id=torch.device("cuda", local))
            grouped = True
        except Exception as e:  # noqa: BLE001 - reported, never fatal to the headline
            solo_group_error = "%s: %s" % (type(e).__name__, e)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    coll_dev = dev if args.dist_backend == "nccl" else torch.device("cpu")  # gloo reduces host tensors

    from footsies_gym_amd import _abi
    from footsies_gym_amd._lib import check, lib, library_info
    from footsies_gym_amd.simulator import FootsiesSim

    N, K, W = args.envs, args.steps, args.warmup
    if args.global_envs:
        if args.global_envs % world:
            raise SystemExit("--global-envs must be a multiple of the rank count")
        N = args.global_envs // world
    scaling = "strong" if args.global_envs else "weak"
    # arena_base = the shard's first global index: seeds and the hashed action stream are those of
    # the same arenas in one unsharded run (fs_config.arena_base), so every rank's work differs
    sim = FootsiesSim(N, device=local, p2_mode="external", seed=0, arena_base=rank * N)
    h = sim.handle
    L = lib()
    # synthetic inputs resident in HBM before timing: W warm-up rows, then R regions of K rows
    R = max(1, args.regions)
    p1, p2 = sim.hash_actions(W + R * K, seed=args.seed, t0=0)
    torch.cuda.synchronize(dev)
    chunk = max(1, min(args.chunk, K))
    packed = args.layout == "packed"
    alloc = sim.alloc_packed_trajectory if packed else sim.alloc_trajectory
    traj = alloc(chunk)  # zero-filled: the pages are resident before timing
    fs_step, fs_step_n, fs_step_n_packed = L.fs_step, L.fs_step_n, L.fs_step_n_packed
    layout_flag = _abi.FS_KERNEL_PACKED if packed else 0

    def make_runs(a1, a2, tr, ticks_per_launch, packed=packed, handle=None, n=None):
        h = handle if handle is not None else sim.handle
        N = n if n is not None else sim.num_envs
        b1, b2 = a1.data_ptr(), a2.data_ptr()
        if packed:
            td = _abi.fs_packed_traj(lanes=tr["lanes"].data_ptr(), reward=tr["reward"].data_ptr(),
                                     final_lanes=tr["final_lanes"].data_ptr())
        else:
            td = _abi.fs_outputs(**{k: tr[k].data_ptr() for k in _abi.OUTPUT_SPEC})
        # The calls' ctypes arguments (row pointers into the resident action rows, the trajectory
        # struct) are built here, before any timed region: a region holds the launch calls and the
        # synchronizes only (building them inline cost ~0.9 us per 20-tick region,
        # profiles/r05ag_region_args.txt).
        rows = a1.shape[0]
        q1 = [C.c_void_p(b1 + k * N) for k in range(rows)]
        q2 = [C.c_void_p(b2 + k * N) for k in range(rows)]
        tdr = C.byref(td)
        act = _abi.FS_ACT_DEVICE

        def run_step(k0, n):
            for k in range(k0, k0 + n):
                rc = fs_step(h, q1[k], q2[k], act)
                if rc:
                    check(rc, h)

        def run_fused(k0, n):
            k = k0
            while k < k0 + n:
                m = min(ticks_per_launch, k0 + n - k)
                if packed:
                    rc = fs_step_n_packed(h, m, q1[k], q2[k], tdr)
                else:
                    rc = fs_step_n(h, m, q1[k], q2[k], 0, tdr)
                if rc:
                    check(rc, h)
                k += m
        return run_step, run_fused

    run_step, run_fused = make_runs(p1, p2, traj, chunk)
    base1, base2 = p1.data_ptr(), p2.data_ptr()

    def barrier():
        if grouped and world > 1:  # (one rank has no one to wait for)
            dist.barrier()

    def timed(fn, k0, n):
        """One timed region of exactly n steps: barrier + synchronize on both sides, each rank's
        host wall clock from its synchronize before the launches to its synchronize after them,
        max over ranks.  Nothing else is issued inside the region; the closing barrier follows
        the clock, so the collective's own latency is not counted as work (the max over ranks
        holds the slowest rank's region)."""
        barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        fn(k0, n)
        torch.cuda.synchronize(dev)
        wall = time.perf_counter() - t0
        barrier()
        local_walls.append(wall)
        t = torch.tensor([wall], dtype=torch.float64, device=coll_dev)
        if grouped:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def rank_values(v, raw=False):
        """Every rank's value of v (this rank's median region wall), in rank order, in ms (raw: as given)."""
        t = torch.tensor([v], dtype=torch.float64, device=coll_dev)
        if world == 1:
            every = [t]
        else:
            every = [torch.zeros_like(t) for _ in range(world)]
            dist.all_gather(every, t)
        return [float(e.item()) if raw else round(1e3 * float(e.item()), 4) for e in every]

    def kernel_time(fn, lo, hi, launches, ticks_per_launch):
        """The kernel's launch-to-launch period with the queue pre-filled (a spin kernel holds the
        GPU while the host enqueues, so no host gap is timed): (average, median).  The average is
        one event pair around `launches` back-to-back launches; the median comes from a second
        pass with an event pair around each launch, whose records themselves add a few
        microseconds between kernels (measured: 27 vs 24 us at 20 ticks per launch).  Every
        launch reads action rows inside [lo, hi)."""
        def spin():
            try:
                torch.cuda._sleep(int(2e7))
            except Exception:
                pass
        start = lambda j: lo + (j * ticks_per_launch) % max(1, hi - lo - ticks_per_launch + 1)  # noqa: E731
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        spin()
        e0.record()
        for j in range(launches):
            fn(start(j), ticks_per_launch)
        e1.record()
        torch.cuda.synchronize(dev)
        avg = e0.elapsed_time(e1) / 1e3 / launches
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(launches)]
        spin()
        for j, (a, b) in enumerate(evs):
            a.record()
            fn(start(j), ticks_per_launch)
            b.record()
        torch.cuda.synchronize(dev)
        d = sorted(a.elapsed_time(b) / 1e3 for a, b in evs)
        return avg, d[len(d) // 2]

    # warm-up (untimed)
    if W:
        (run_fused if args.mode == "fused" else run_step)(0, W)
    torch.cuda.synchronize(dev)

    # R back-to-back regions of exactly K steps each (fresh action rows per region); the
    # median region is reported, every region's wall time is listed
    res = {}
    for mode, fn in (("fused", run_fused), ("step", run_step)):
        local_walls = []
        walls = [timed(fn, W + r * K, K) for r in range(R)]
        wall = sorted(walls)[len(walls) // 2]
        mine = sorted(local_walls)[len(local_walls) // 2]
        res[mode] = {"wall_s": wall, "region_walls_ms": [round(1e3 * w, 4) for w in walls],
                     "env_steps_per_s": world * N * K / wall, "ms_per_step": 1e3 * wall / K,
                     "rank_walls_ms": rank_values(mine)}
    # fused mode: the other trajectory layout over the same action rows, timed the same way and
    # reported beside (it continues the same handle's arenas)
    other_layout = None
    if args.mode == "fused":
        otraj = (sim.alloc_trajectory if packed else sim.alloc_packed_trajectory)(chunk)
        _, ofused = make_runs(p1, p2, otraj, chunk, packed=not packed)
        ofused(W, min(K, 3))
        torch.cuda.synchronize(dev)
        local_walls = []
        owalls = [timed(ofused, W + r * K, K) for r in range(R)]
        ow = sorted(owalls)[len(owalls) // 2]
        other_layout = {"trajectory": "one array per field (fs_step_n)" if packed else "packed records (fs_step_n_packed)",
                        "value": world * N * K / ow, "ms_per_step": 1e3 * ow / K,
                        "region_walls_ms": [round(1e3 * w, 4) for w in owalls],
                        "kernel": L.fs_step_kernel(h, chunk, 0 if packed else _abi.FS_KERNEL_PACKED).decode()}
        del otraj, ofused
    def leg_median(fn, k0, n):
        """A secondary leg: one untimed call (its kernels' first launch, staging buffers and the
        process group's first collective stay out of the timing), then R timed regions of n
        steps, the median reported as for the headline."""
        fn(k0, min(n, 3))
        torch.cuda.synchronize(dev)
        return sorted(timed(fn, k0, n) for _ in range(R))[R // 2]

    # P1/P2 actions handed over from host memory (FS_ACT_HOST: pinned staging + H2D copy per
    # step), the PCIe-inclusive rate of the per-step path; reported beside, never as `value`
    kh = min(K, 500)
    p1h, p2h = p1[W:W + kh].cpu().numpy(), p2[W:W + kh].cpu().numpy()

    def run_host(k0, n):
        for k in range(n):
            rc = fs_step(h, p1h[k % kh].ctypes.data, p2h[k % kh].ctypes.data, _abi.FS_ACT_HOST)
            if rc:
                check(rc, h)
    host_rate = N * kh / leg_median(run_host, 0, kh)
    # the per-step path with the multi-GPU exchange of SURVEY 8(e): every step's outputs written
    # as 40-B records by the step kernel itself (fs_step_rec; before r05: fs_step + a separate
    # fs_pack_outputs launch) and gathered over RCCL/xGMI
    kg = min(K, 500)
    rec = torch.empty((N, _abi.FS_RECORD_BYTES), dtype=torch.uint8, device=dev)
    gbuf = torch.empty((world * N, _abi.FS_RECORD_BYTES), dtype=torch.uint8, device=dev)
    fs_step_rec = L.fs_step_rec
    recp = C.c_void_p(rec.data_ptr())

    def run_step_gather(k0, n):
        for k in range(k0, k0 + n):
            rc = fs_step_rec(h, C.c_void_p(base1 + k * N), C.c_void_p(base2 + k * N), _abi.FS_ACT_DEVICE, recp)
            if rc:
                check(rc, h)
            if grouped and args.dist_backend == "nccl":
                dist.all_gather_into_tensor(gbuf, rec)
    gwall = leg_median(run_step_gather, W, kg)

    def run_step_gather_root(k0, n):  # the learner-only variant: grouped send / recv to rank 0
        from footsies_gym_amd.parallel import gather_records_to
        for k in range(k0, k0 + n):
            rc = fs_step_rec(h, C.c_void_p(base1 + k * N), C.c_void_p(base2 + k * N), _abi.FS_ACT_DEVICE, recp)
            if rc:
                check(rc, h)
            if grouped and args.dist_backend == "nccl":
                gather_records_to(rec, 0)
    grwall = leg_median(run_step_gather_root, W, kg)
    # The dominant kernel of the reported mode, back-to-back launches.  The roofline block is
    # measured at a fixed launch shape (--roofline-ticks ticks per fs_step_n launch, the shape
    # the committed rocprofv3 summaries under profiles/ cover), independent of --steps; the
    # kernel at the timed region's own launch shape is reported beside it.
    def roofline_at(ticks, fn, lo, hi, launches):
        kt_, kmed_ = kernel_time(fn, lo, hi, launches, ticks)
        b = N * (STATE_BYTES + ticks * STEP_IO_BYTES)
        return kt_, kmed_, b
    if args.mode == "fused":
        rt = max(1, args.roofline_ticks)
        if rt <= W + R * K and rt == chunk:
            rfn, rlo, rhi = run_fused, W, W + R * K
        else:
            q1, q2 = sim.hash_actions(rt, seed=args.seed ^ 0x5A5A, t0=0)
            rtraj = traj if rt == chunk else alloc(rt)
            _, rfn = make_runs(q1, q2, rtraj, rt)
            rlo, rhi = 0, rt
            torch.cuda.synchronize(dev)
        kt, kmed, bytes_per_launch = roofline_at(rt, rfn, rlo, rhi, max(5, args.kernel_samples // 10))
        ticks = rt
        st_kt, st_kmed, st_bytes = roofline_at(chunk, run_fused, W, W + R * K, max(5, args.kernel_samples // 5))
        kname = L.fs_step_kernel(h, rt, layout_flag).decode()  # the kernel this launch shape runs (k_step_n1 from 2 x 64 x SIMDs arenas)
    else:
        kt, kmed, bytes_per_launch = roofline_at(1, run_step, W, W + R * K, args.kernel_samples)
        st_kt, st_kmed, st_bytes = kt, kmed, bytes_per_launch
        ticks = 1
        kname = L.fs_step_kernel(h, 1, 0).decode()
    st_kname = L.fs_step_kernel(h, chunk if args.mode == "fused" else 1, layout_flag if args.mode == "fused" else 0).decode()
    achieved = bytes_per_launch / kt / 1e9
    tr = pmc_traffic(kname, N, ticks)
    st_ticks = chunk if args.mode == "fused" else 1
    st_tr = pmc_traffic(st_kname, N, st_ticks)
    issue = issue_profile(kname, N, ticks)
    # what binds the kernel: its SIMDs' instruction issue when the committed issue model puts the
    # kernel nearer that limit than HBM's (the C3 kernel: 0.90 of its issue plateau, ~0.3 of HBM)
    hbm_frac = achieved / HBM_PEAK_GBPS
    bound = "simd-issue" if issue and (issue.get("issue_frac") or 0.0) > hbm_frac else "hbm"
    other = "step" if args.mode == "fused" else "fused"
    out = {
        "metric": METRIC,
        "value": res[args.mode]["env_steps_per_s"],
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": K,
        "warmup": W,
        "ms_per_step": res[args.mode]["ms_per_step"],
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "int32+f32 (reward f64)",
        "data": "synthetic (splitmix64 self-play actions in HBM)",
        "library": library_info(),
        "config": {"workload": ("C4 strong: %d arenas over %d GPUs" % (N * world, world) if args.global_envs else
                                "C3: %d arenas/GPU" % N) + ", self-play random actions, P2 external, auto-reset same-step",
                   "envs_per_gpu": N, "global_envs": N * world, "mode": args.mode,
                   "ticks_per_launch": chunk if args.mode == "fused" else 1,
                   "trajectory": ("packed records (fs_step_n_packed)" if packed else "one array per field (fs_step_n)")
                   if args.mode == "fused" else None, "parallelism": "arena-shard x%d" % world},
        "ranks": {"world_size": dist.get_world_size() if grouped else 1,
                  "backend": dist.get_backend() if grouped else None,
                  "launcher": "WORLD_SIZE" in os.environ, "solo_group_error": solo_group_error,
                  "rank_walls_ms": res[args.mode]["rank_walls_ms"],
                  "note": "world_size / backend as the process group reports them (nccl = RCCL); each rank's "
                          "median region wall, before the max over ranks"},
        "timing": {"regions": R, "region_walls_ms": res[args.mode]["region_walls_ms"],
                   "note": "each region times exactly `steps` steps between barrier + synchronize pairs "
                           "(host wall clock, max over ranks); value = the median region"},
        "roofline": {"bound": bound, "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBPS, "traffic": tr[0] if tr else None,
                     "traffic_ratio": (tr[0] / bytes_per_launch) if tr else None,
                     "traffic_source": tr[1] if tr else None,
                     "layout_bytes_per_launch": (N * (STATE_BYTES + ticks * PACKED_STEP_MOVED_BYTES)
                                                 if args.mode == "fused" and packed else bytes_per_launch),
                     "kernel": kname, "ticks_per_launch": ticks, "avg_launch_us": kt * 1e6,
                     "median_launch_us": kmed * 1e6, "algorithmic_bytes_per_launch": bytes_per_launch,
                     "note": "avg_launch_us: back-to-back launch period (one HIP event pair over the launches), median_launch_us: per-launch event pairs (their records add a few us between kernels); achieved / peak / frac: the HBM roofline of the kernel's algorithmic bytes (per arena 96 B of state per launch, per env-step 2 B of actions in + 38 B of outputs out); the packed layout moves 2 B in + 40 B out per env-step (38 useful + 2 pad bytes in P2's 16-B record), layout_bytes_per_launch; traffic_ratio = PMC traffic / algorithmic bytes; `bound` "
                             "names what binds it: the SIMDs' instruction issue (issue.issue_frac, the rate over the "
                             "same kernel's plateau at 4-8 waves per SIMD) when a SIMD-level issue model of this "
                             "kernel is committed",
                     "issue": issue},
        "kernel_at_timed_shape": {"ticks_per_launch": chunk if args.mode == "fused" else 1,
                                  "avg_launch_us": st_kt * 1e6, "median_launch_us": st_kmed * 1e6,
                                  "algorithmic_bytes_per_launch": st_bytes,
                                  "frac": st_bytes / st_kt / 1e9 / HBM_PEAK_GBPS,
                                  "kernel": st_kname,
                                  "traffic": (st_tr or (None,))[0],
                                  "traffic_ratio": (st_tr[0] / st_bytes) if st_tr else None,
                                  "traffic_source": st_tr[1] if st_tr else None,
                                  "issue": issue_profile(st_kname, N, st_ticks),
                                  "attribution": short_launch_attribution(st_ticks)},
        other + "_mode": {"value": res[other]["env_steps_per_s"], "ms_per_step": res[other]["ms_per_step"]},
        "fused_other_layout": other_layout,
        "host_actions_step_mode": {"value": world * host_rate, "steps": kh,
                                   "note": "fs_step with FS_ACT_HOST (PCIe-inclusive action hand-over); this and "
                                           "the gather legs: one untimed call, then the median of `regions` regions"},
        "step_gather_mode": {"value": world * N * kg / gwall, "ms_per_step": 1e3 * gwall / kg, "steps": kg,
                             "bytes_gathered_per_step": world * N * _abi.FS_RECORD_BYTES,
                             "collective": bool(grouped and args.dist_backend == "nccl"),
                             "note": "fs_step_rec (records from the step kernel) + one all_gather_into_tensor of the 40-B "
                                     "(obs, reward, done) records over RCCL per step (at N = 1 in a one-rank RCCL group; "
                                     "none with --no-solo-group or --dist-backend gloo)"},
        "step_gather_root_mode": {"value": world * N * kg / grwall, "ms_per_step": 1e3 * grwall / kg, "steps": kg,
                                  "bytes_into_rank0_per_step": (world - 1) * N * _abi.FS_RECORD_BYTES,
                                  "note": "fs_step_rec + the records of every rank gathered to rank 0 "
                                          "only (grouped send / recv over RCCL, parallel.gather_records_to)"},
    }
    # BASELINE configs[3] (C4): 262 144 arenas split over the N ranks (strong scaling), so the
    # driver's plain `bench.py --gpus N` at N = 1, 2, 4, 8 records C4's scaling curve -- its N = 1
    # point is all 262 144 arenas on one GPU.  Each rank: a second handle over its contiguous global
    # range (arena_base, so seeds and hashed rows are the unsharded run's), the packed fused kernel
    # timed at the headline's launch shape (R regions of --steps) and in LEG_TICKS-tick launches
    # (R regions), barrier + max over ranks like the headline; no data-path collective.
    if not args.no_c4 and c4_split(world, rank) is None:
        out["c4_strong"] = {"skipped": "%d ranks do not split %d arenas evenly" % (world, C4_GLOBAL_ENVS)}
    elif not args.no_c4:
        c4n, c4b = c4_split(world, rank)
        try:
            sim4 = FootsiesSim(c4n, device=local, p2_mode="external", seed=0, arena_base=c4b)
            rows4 = max(W + R * K, (R + 1) * LEG_TICKS)
            a41, a42 = sim4.hash_actions(rows4, seed=args.seed, t0=0)
            ch4 = chunk if args.mode == "fused" else 1
            tr4 = sim4.alloc_packed_trajectory(max(ch4, LEG_TICKS))
            _, f4 = make_runs(a41, a42, tr4, ch4, packed=True, handle=sim4.handle, n=c4n)
            _, f4k = make_runs(a41, a42, tr4, LEG_TICKS, packed=True, handle=sim4.handle, n=c4n)
            torch.cuda.synchronize(dev)
            f4(0, max(1, W))
            torch.cuda.synchronize(dev)
            local_walls = []
            w4 = [timed(f4, W + r * K, K) for r in range(R)]
            wall4, mine4 = sorted(w4)[R // 2], sorted(local_walls)[R // 2]
            f4k(0, LEG_TICKS)
            torch.cuda.synchronize(dev)
            local_walls = []
            wk = [timed(f4k, (r + 1) * LEG_TICKS, LEG_TICKS) for r in range(R)]
            wallk, minek = sorted(wk)[R // 2], sorted(local_walls)[R // 2]
            kt4, km4 = kernel_time(f4k, LEG_TICKS, rows4, 5, LEG_TICKS)
            kts4, kms4 = kernel_time(f4, W, W + R * K, max(5, args.kernel_samples // 5), ch4)
            kname4 = L.fs_step_kernel(sim4.handle, LEG_TICKS, _abi.FS_KERNEL_PACKED).decode()
            skname4 = L.fs_step_kernel(sim4.handle, ch4, _abi.FS_KERNEL_PACKED).decode()
            b4 = c4n * (STATE_BYTES + LEG_TICKS * STEP_IO_BYTES)
            bs4 = c4n * (STATE_BYTES + ch4 * STEP_IO_BYTES)
            # (a 1000-tick call at 262 144 arenas is two launches -- 32-bit trajectory offsets,
            # fs_api.cpp kMaxPackedLaunchRows -- whose per-launch PMC summary is at ~500 ticks)
            per_call = -(-LEG_TICKS // max(1, (0xFFFFFFFF // 32) // c4n))
            tr4k = pmc_traffic(kname4, c4n, LEG_TICKS // per_call)
            if tr4k:
                tr4k = (tr4k[0] * per_call, tr4k[1])
            out["c4_strong"] = {
                "global_envs": C4_GLOBAL_ENVS, "scaling": "strong", "envs_per_gpu": c4n,
                "envs_per_rank": [c4n] * world, "arena_base_per_rank": [int(e) for e in rank_values(float(c4b), raw=True)],
                "value": C4_GLOBAL_ENVS * K / wall4, "unit": "env-steps/s", "ms_per_step": 1e3 * wall4 / K,
                "steps": K, "ticks_per_launch": ch4, "region_walls_ms": [round(1e3 * w, 4) for w in w4],
                "rank_walls_ms": rank_values(mine4), "kernel": skname4,
                "kernel_avg_launch_us": kts4 * 1e6, "kernel_median_launch_us": kms4 * 1e6,
                "frac": bs4 / kts4 / 1e9 / HBM_PEAK_GBPS,
                "launch_%d" % LEG_TICKS: {
                    "value": C4_GLOBAL_ENVS * LEG_TICKS / wallk, "ms_per_step": 1e3 * wallk / LEG_TICKS,
                    "ticks_per_launch": LEG_TICKS, "region_walls_ms": [round(1e3 * w, 4) for w in wk],
                    "rank_walls_ms": rank_values(minek), "kernel": kname4,
                    "avg_launch_us": kt4 * 1e6, "median_launch_us": km4 * 1e6,
                    "algorithmic_bytes_per_launch": b4, "achieved": b4 / kt4 / 1e9,
                    "frac": b4 / kt4 / 1e9 / HBM_PEAK_GBPS,
                    "traffic": tr4k[0] if tr4k else None, "traffic_ratio": (tr4k[0] / b4) if tr4k else None,
                    "traffic_source": tr4k[1] if tr4k else None},
                "config": "C4 strong: %d arenas over %d GPU(s), %d per GPU (arena_base = rank x %d), self-play "
                          "random actions, P2 external, packed trajectories (fs_step_n_packed)"
                          % (C4_GLOBAL_ENVS, world, c4n, c4n),
                "note": "value = all ranks' arenas x steps over the max-over-ranks median region of `steps` steps at "
                        "the headline's launch shape; launch_%d: the same in %d-tick launches; frac: the kernel's "
                        "algorithmic bytes per launch over its back-to-back launch period, against 8 TB/s"
                        % (LEG_TICKS, LEG_TICKS)}
            sim4.close()
            del a41, a42, tr4, f4, f4k
            torch.cuda.empty_cache()
        except Exception as e:  # noqa: BLE001 - the headline line must still print
            out["c4_strong"] = {"error": "%s: %s" % (type(e).__name__, e)}
    # the fused legs beside the headline, on every rank (barrier + max over ranks, like the
    # headline), at a fixed shape whatever --steps is: R regions of LEG_TICKS ticks in
    # LEG_TICKS-tick launches, the median reported
    if not args.no_extras:
        for key, kind in (("p2_bot_mode", "bot"), ("actors_mode.mixed_p2", "mixed_p2"),
                          ("actors_mode.by_example", "by_example")):
            try:
                run_leg, leg_kernel, close_leg = fused_leg(torch, N, LEG_TICKS * (R + 1), LEG_TICKS, args.seed, local,
                                                           rank, kind, layout=args.layout)
                lw = leg_median(run_leg, LEG_TICKS, LEG_TICKS)
                close_leg()
                v = {"value": world * N * LEG_TICKS / lw, "ms_per_step": 1e3 * lw / LEG_TICKS,
                     "ticks_per_launch": LEG_TICKS, "kernel": leg_kernel, "config": LEG_CONFIG[kind] +
                     ", %d arenas per GPU" % N}
            except Exception as e:  # noqa: BLE001 - the headline line must still print
                v = {"error": "%s: %s" % (type(e).__name__, e)}
            if "." in key:
                a, b = key.split(".")
                out.setdefault(a, {})[b] = v
            else:
                out[key] = v
    # the exchange alone: the same all_gather of the 40-B records with no simulation between
    # them, its received bytes per rank against the xGMI links that carry them (one link per
    # peer on a fully connected node; 7 links x ~153 GB/s per MI355X, the task brief -- the
    # figure is not in MI355X_MICROARCH.md)
    if grouped and args.dist_backend == "nccl" and world > 1:
        def run_gather(k0, n):
            for _ in range(n):
                dist.all_gather_into_tensor(gbuf, rec)
        gowall = leg_median(run_gather, 0, kg)
        recv = (world - 1) * N * _abi.FS_RECORD_BYTES
        out["step_gather_mode"]["xgmi"] = {
            "bytes_received_per_rank_per_step": recv,
            "gather_only_us_per_step": 1e6 * gowall / kg,
            "link_GBps_per_rank": recv / (gowall / kg) / 1e9,
            "in_step_GBps_per_rank": recv / (gwall / kg) / 1e9,
            "peak_GBps_per_rank": (world - 1) * XGMI_LINK_GBPS,
            "frac": recv / (gowall / kg) / 1e9 / ((world - 1) * XGMI_LINK_GBPS),
            "note": "all_gather_into_tensor of every rank's [N, 40] records, alone (gather_only) and inside the "
                    "fs_step + pack + gather step (in_step); peak = one ~153 GB/s xGMI link per peer"}
    # C5 at N > 1 as one training job: data-parallel PPO (ppo.PPOTrainer(group=...)), every rank
    # rolling out its own N arenas (arena_base = rank x N) and averaging each minibatch's gradient
    # over the ranks with one all_reduce; barrier + max over ranks around the iterations
    if world > 1 and not args.no_extras:
        try:
            out["ppo_dp"] = ppo_dp_rate(torch, N, local, rank, world, timed)
        except Exception as e:  # noqa: BLE001 - the headline line must still print
            out["ppo_dp"] = {"error": "%s: %s" % (type(e).__name__, e)}
    if world == 1 and not args.no_extras:
        try:
            out["policy_loop"] = policy_loop_rate(torch, N, min(K, 1000), local)
        except Exception as e:  # reported, never fatal to the headline measurement
            out["policy_loop"] = {"error": "%s: %s" % (type(e).__name__, e)}
        try:
            out["policy_loop_fused"] = fused_policy_rate(torch, N, 5 * chunk, local, ticks=chunk)
        except Exception as e:  # noqa: BLE001 - the headline line must still print
            out["policy_loop_fused"] = {"error": "%s: %s" % (type(e).__name__, e)}
        try:
            out["ppo_end_to_end"] = ppo_rate(torch, N, local)
        except Exception as e:  # noqa: BLE001 - the headline line must still print
            out["ppo_end_to_end"] = {"error": "%s: %s" % (type(e).__name__, e)}
        try:
            out["vector_env"] = vector_env_rate(torch, N, VENV_STEPS, local)
        except Exception as e:  # noqa: BLE001 - the headline line must still print
            out["vector_env"] = {"error": "%s: %s" % (type(e).__name__, e)}
        try:
            out["single_env"] = single_env_rate(torch, 500, local)
        except Exception as e:  # noqa: BLE001 - the headline line must still print
            out["single_env"] = {"error": "%s: %s" % (type(e).__name__, e)}
    sim.close()
    if grouped:
        barrier()
        dist.destroy_process_group()
    # the CPU baseline last, on rank 0 alone: at N > 1 the other ranks have left, so the oracle
    # has the host's cores to itself
    if rank == 0 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(N, args.cpu_seconds, args.seed)
    if rank == 0:
        print(json.dumps(out))


if __name__ == "__main__":
    main()
