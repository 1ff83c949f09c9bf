"""Where FootsiesVectorEnv.step(output="torch") spends its ~8 us per step: the same 300 steps
timed through each layer -- the env, FootsiesSim.step, the bare ctypes fs_step call -- at the C3
size and at 256 arenas (where the kernel is short and the host side is the step's time).  GPU box
only; measurement support for DESIGN.md section 6."""
import ctypes as C
import sys
import time

sys.path.insert(0, "/root/repo")
import torch  # noqa: E402
from footsies_gym_amd import _abi  # noqa: E402
from footsies_gym_amd._lib import lib  # noqa: E402
from footsies_gym_amd.vector_env import FootsiesVectorEnv  # noqa: E402

STEPS = 300


WARM = int(sys.argv[1]) if len(sys.argv) > 1 else 50


def timed(fn):
    for j in range(50):
        fn(j)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for j in range(STEPS):
        fn(j)
    torch.cuda.synchronize()
    return 1e6 * (time.perf_counter() - t) / STEPS


def main():
    for n in (65536, 256):
        g = torch.Generator(device="cuda").manual_seed(0)
        a1 = torch.randint(0, 8, (STEPS + 50, n), dtype=torch.uint8, device="cuda", generator=g)
        a2 = torch.randint(0, 8, (STEPS + 50, n), dtype=torch.uint8, device="cuda", generator=g)
        rows1 = [a1[j] for j in range(STEPS + 50)]  # the row views made once (the env leg indexes per step)
        rows2 = [a2[j] for j in range(STEPS + 50)]
        k = [0]
        env = FootsiesVectorEnv(n, opponent=lambda o, i: a2[k[0]], output="torch", seed=0)
        env.reset(seed=0)
        for j in range(WARM):  # into the steady terminal rate (~130 auto-resets per step at 65 536)
            env.step(rows1[j % STEPS])

        def env_step(j):
            k[0] = j
            env.step(a1[j])
        res = {"env.step": timed(env_step)}
        sim = env.sim
        res["sim.step"] = timed(lambda j: sim.step(rows1[j], rows2[j]))
        L, h = lib(), sim.handle
        res["ctypes fs_step"] = timed(lambda j: L.fs_step(h, rows1[j].data_ptr(), rows2[j].data_ptr(),
                                                          _abi.FS_ACT_DEVICE))
        p1, p2 = rows1[0].data_ptr(), rows2[0].data_ptr()
        res["ctypes fs_step, same rows"] = timed(lambda j: L.fs_step(h, p1, p2, _abi.FS_ACT_DEVICE))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for j in range(STEPS):
            L.fs_step(h, p1, p2, _abi.FS_ACT_DEVICE)
        e1.record()
        torch.cuda.synchronize()
        res["device period (events)"] = 1e3 * e0.elapsed_time(e1) / STEPS
        env.close()
        print("N=%d warm=%d " % (n, WARM) + "  ".join("%s %.2f us" % kv for kv in res.items()), flush=True)


if __name__ == "__main__":
    main()
