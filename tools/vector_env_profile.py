"""cProfile of FootsiesVectorEnv.step with numpy actions in / numpy dicts out at 65 536 arenas
(the bench's vector_env numpy leg): where the ~0.8 ms per step goes on the host.  GPU box only."""
import cProfile, pstats, sys, time, io
sys.path.insert(0, "/root/repo")
import numpy as np, torch
from footsies_gym_amd.vector_env import FootsiesVectorEnv
N=65536
rng=np.random.default_rng(0)
acts=[rng.integers(0,8,N).astype(np.uint8) for _ in range(120)]
k=[0]
opp=lambda obs, info: acts[(k[0]+7)%120]
env=FootsiesVectorEnv(N, device=0, opponent=opp, output="numpy", seed=0)
env.reset(seed=0)
for j in range(20): k[0]=j; env.step(acts[j])
torch.cuda.synchronize()
pr=cProfile.Profile(); pr.enable()
t=time.perf_counter()
for j in range(20,120): k[0]=j; env.step(acts[j])
torch.cuda.synchronize()
dt=time.perf_counter()-t
pr.disable()
print("ms per step", dt/100*1e3)
s=io.StringIO(); pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(18); print(s.getvalue()[:5000])
