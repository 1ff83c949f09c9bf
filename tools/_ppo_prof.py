import sys, time, torch
sys.path.insert(0, '/root/repo')
from footsies_gym_amd.simulator import FootsiesSim
from footsies_gym_amd.ppo import PPOTrainer, gae
N=65536
sim = FootsiesSim(N, device=0, p2_mode="bot", seed=0)
tr = PPOTrainer(sim, horizon=128)
tr.train(1)
torch.cuda.synchronize()
def t(): torch.cuda.synchronize(); return time.perf_counter()
for it in range(2):
    a=t(); feats, actions, rewards, dones = tr.collect(); b=t()
    with torch.no_grad():
        values = tr.critic(feats).squeeze(-1); c=t()
        adv, ret = gae(rewards, values, dones, tr.gamma, tr.lam); d=t()
    tr.update(feats, actions, rewards, dones); e=t()
    print("collect %.1f ms, critic %.1f ms, gae %.1f ms, update(total incl. critic+gae again) %.1f ms" % ((b-a)*1e3,(c-b)*1e3,(d-c)*1e3,(e-d)*1e3), flush=True)
from torch.profiler import profile, ProfilerActivity
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
    tr.iterate(); torch.cuda.synchronize()
print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=25))
