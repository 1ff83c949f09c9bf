"""How much the unpinned float model matters: C3's hashed self-play stream
stepped by the CPU oracle under both float models, side by side, and compared every tick.

Mono's float evaluation precision is unknown (DESIGN §3 "Float model"): the C# float arithmetic of
UpdateMovement and the pushes (F:300, 305, 316; BC:492-498, 511-515) is either rounded to binary32
after every operation (FS_FLOAT_STRICT32, the default) or carried in binary64 temporaries and
rounded on store (FS_FLOAT_DOUBLE).  Both are built and bit-exact between oracle and kernel; this
measures how fast trajectories under the two models part.

Per tick it reports the fraction of arenas whose canonical state (fs_arena_state, every field)
differs, the fraction whose observation/info outputs differ (the terminal record only on a terminal
tick), the same excluding the positions (guard, move, frame, reward, termination ... -- what a
discrete policy or the episode boundaries see), and the fraction that have differed at least once;
per arena the first-divergence tick (its distribution) and whether it ever re-converged
(the round start re-places both fighters, BC:279-286).  Test infrastructure (oracle/ only).

    python tools/float_model_divergence.py --envs 65536 --ticks 2000 --out profiles/r06_float_model_divergence.json
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from footsies_gym_amd import _abi  # noqa: E402
from oracle import binding  # noqa: E402


def rows(a):
    """A structured / plain array as one byte row per arena."""
    a = np.ascontiguousarray(a)
    return a.view(np.uint8).reshape(a.shape[0], -1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--ticks", type=int, default=2000)
    ap.add_argument("--seed", type=lambda s: int(s, 0), default=0x5EED)
    ap.add_argument("--every", type=int, default=10, help="per-tick series sampled every this many ticks")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    binding.build()
    n, T = a.envs, a.ticks
    strict = binding.Oracle(n, p2_mode=_abi.FS_P2_EXTERNAL, float_mode=_abi.FS_FLOAT_STRICT32, base_seed=0)
    double = binding.Oracle(n, p2_mode=_abi.FS_P2_EXTERNAL, float_mode=_abi.FS_FLOAT_DOUBLE, base_seed=0)
    first = np.full(n, -1, dtype=np.int64)        # first tick whose state differs
    first_obs = np.full(n, -1, dtype=np.int64)    # first tick whose outputs differ
    reconverged = np.zeros(n, dtype=bool)         # differed once, equal again later
    first_disc = np.full(n, -1, dtype=np.int64)   # first tick whose non-position outputs differ
    field_first, max_dpos = {}, 0.0
    series = []
    t0 = time.perf_counter()
    for t in range(T):
        strict.step_n_hashed(1, a.seed)
        double.step_n_hashed(1, a.seed)
        ds = (rows(strict.state()) != rows(double.state())).any(axis=1)
        os_, od = strict.outputs(copy=False), double.outputs(copy=False)
        do = np.zeros(n, dtype=bool)       # this tick's observation / info / reward / flags differ
        disc = np.zeros(n, dtype=bool)     # ... in a field other than the positions
        term = (os_["terminated"] != 0) | (od["terminated"] != 0)
        for k in os_:
            if k.startswith("final_"):     # the terminal record: only meaningful on a terminal tick
                dk = term & (rows(os_[k].reshape(n, -1)) != rows(od[k].reshape(n, -1))).any(axis=1)
            else:
                dk = (rows(os_[k].reshape(n, -1)) != rows(od[k].reshape(n, -1))).any(axis=1)
            if dk.any():
                field_first.setdefault(k, t)
            do |= dk
            if k not in ("position", "final_position"):
                disc |= dk
        dp = np.abs(os_["position"].astype(np.float64) - od["position"].astype(np.float64)).max()
        max_dpos = max(max_dpos, float(dp))
        first[(first < 0) & ds] = t
        first_obs[(first_obs < 0) & do] = t
        first_disc[(first_disc < 0) & disc] = t
        reconverged |= (first >= 0) & ~ds
        if t % a.every == a.every - 1 or t == T - 1:
            series.append({"tick": t + 1, "state_differs": float(ds.mean()), "outputs_differ": float(do.mean()),
                           "discrete_outputs_differ": float(disc.mean()),
                           "ever_differed": float((first >= 0).mean())})
    dt = time.perf_counter() - t0
    strict.close()
    double.close()
    ever = first[first >= 0]
    pct = (lambda x: {str(p): int(np.percentile(x, p)) for p in (1, 10, 25, 50, 75, 90, 99)} if len(x) else None)
    hist_edges = [0, 10, 50, 100, 200, 500, 1000, 2000, 5000, 10 ** 9]
    res = {
        "what": "CPU oracle, FS_FLOAT_STRICT32 vs FS_FLOAT_DOUBLE, C3's splitmix64 self-play stream (P2 external, "
                "seed 0x%X), compared every tick; canonical state = every field of fs_arena_state" % a.seed,
        "envs": n, "ticks": T, "seconds": round(dt, 1),
        "final": series[-1],
        "arenas_ever_differed": float((first >= 0).mean()),
        "arenas_outputs_ever_differed": float((first_obs >= 0).mean()),
        "arenas_reconverged": float(reconverged.mean()),
        "first_divergence_tick_percentiles": pct(ever),
        "first_divergence_tick_histogram": {"edges": hist_edges[:-1] + ["inf"],
                                            "counts": np.histogram(ever, bins=hist_edges)[0].tolist()},
        "first_output_divergence_tick_percentiles": pct(first_obs[first_obs >= 0]),
        "arenas_discrete_outputs_ever_differed": float((first_disc >= 0).mean()),
        "first_discrete_divergence_tick_percentiles": pct(first_disc[first_disc >= 0]),
        "first_tick_each_output_field_differed": field_first,
        "max_abs_position_difference": max_dpos,
        "series": series,
        "refs": "F:300, 305, 316 (UpdateMovement), BC:492-498, 511-515 (pushes); DESIGN.md §3 Float model",
    }
    s = json.dumps(res, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")
    print(json.dumps({k: v for k, v in res.items() if k != "series"}, indent=1))


if __name__ == "__main__":
    main()
