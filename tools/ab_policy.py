#!/usr/bin/env python3
"""A/B timing of the fused policy kernel (fs_step_n_policy, C5 fused) across built libfootsies.so
variants (measurement only).

  python tools/ab_policy.py LIB [LIB ...] [--rounds R] [--envs N] [--ticks T]

Each library runs bench.py's fused_policy_rate leg in its own subprocess (FOOTSIES_LIB override),
rounds interleaved; per library the median rate over the rounds.
"""
import argparse
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CODE = r'''
import sys, torch
sys.path.insert(0, %(root)r)
import bench
r = bench.fused_policy_rate(torch, %(envs)d, 5 * %(ticks)d, 0, ticks=%(ticks)d)
print("RESULT %%.6e" %% r["value"])
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--ticks", type=int, default=1000)
    a = ap.parse_args()
    code = CODE % dict(root=ROOT, envs=a.envs, ticks=a.ticks)
    rates = {lib: [] for lib in a.libs}
    for r in range(a.rounds):
        for lib in a.libs:
            env = dict(os.environ, FOOTSIES_LIB=os.path.abspath(lib))
            p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
            line = [x for x in p.stdout.splitlines() if x.startswith("RESULT")]
            if p.returncode or not line:
                print("%s: error\n%s" % (lib, p.stderr[-800:]), flush=True)
                sys.exit(1)
            rates[lib].append(float(line[0].split()[1]))
            print("round %d %-45s C5 fused %.4e env-steps/s" % (r, lib, rates[lib][-1]), flush=True)
    base = None
    for lib, v in rates.items():
        med = sorted(v)[len(v) // 2]
        base = base or med
        print("%-45s C5 fused %.4e env-steps/s (%+.1f%%)" % (lib, med, 100 * (med / base - 1)), flush=True)


if __name__ == "__main__":
    main()
