import sys, time, torch
sys.path.insert(0, '/root/repo')
from footsies_gym_amd.simulator import FootsiesSim
from footsies_gym_amd.ppo import PPOTrainer
N = 65536
sim = FootsiesSim(N, device=0, p2_mode="bot", seed=0)
tr = PPOTrainer(sim, horizon=128)
feats, actions, rewards, dones = tr.collect()
def timeit(label, fn, reps=2):
    fn(); torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    print("%-40s %.1f ms" % (label, (time.perf_counter() - t) / reps * 1e3), flush=True)
timeit("fp32 update", lambda: tr.update(feats, actions, rewards, dones))
def bf16():
    with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
        tr.update(feats, actions, rewards, dones)
timeit("autocast bf16 update", bf16)
torch.backends.cuda.matmul.allow_tf32 = True
timeit("allow_tf32 update", lambda: tr.update(feats, actions, rewards, dones))
torch.backends.cuda.matmul.allow_tf32 = False
# weight-gradient GEMM shapes alone
M = 128 * N // 4
dH = torch.randn(M, 64, device="cuda"); X = torch.randn(M, 64, device="cuda")
timeit("dW = dH^T X  fp32 (2.1M x 64)", lambda: dH.t() @ X, reps=5)
timeit("dW via bmm chunks of 8192", lambda: torch.bmm(dH.view(-1, 8192, 64).transpose(1, 2), X.view(-1, 8192, 64)).sum(0), reps=5)
dHb, Xb = dH.bfloat16(), X.bfloat16()
timeit("dW bf16", lambda: dHb.t() @ Xb, reps=5)
timeit("dW bf16 bmm chunks 8192", lambda: torch.bmm(dHb.view(-1, 8192, 64).transpose(1, 2), Xb.view(-1, 8192, 64)).float().sum(0), reps=5)
