"""Debug aid: lockstep HIP vs oracle with a full-state comparison every step; on the first
divergence print the recent history (actions + both canonical states) of that arena."""
import sys
import numpy as np
sys.path.insert(0, ".")
from footsies_gym_amd import _abi
from footsies_gym_amd.simulator import FootsiesSim
from oracle import binding
from tests.parity_utils import bits

p2 = sys.argv[1] if len(sys.argv) > 1 else "external"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 512
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 400
P2 = {"external": 0, "bot": 1, "noop": 2}[p2]
sim = FootsiesSim(n, p2_mode=p2, seed=11)
ora = binding.Oracle(n, p2_mode=P2, base_seed=11)
rng = np.random.default_rng(1)
hist = []
def flat(s, i):
    d = {}
    for k in s.dtype.names:
        if k == "f":
            for j in range(2):
                for fk in s["f"].dtype.names:
                    d["f%d.%s" % (j, fk)] = s["f"][fk][i, j]
        else:
            d[k] = s[k][i]
    return d
for t in range(steps):
    a1 = rng.integers(0, 8, n).astype(np.uint8)
    a2 = rng.integers(0, 8, n).astype(np.uint8)
    ora.step(a1, a2 if P2 == 0 else None)
    sim.step(a1, a2 if P2 == 0 else None)
    so, sg = ora.state(), sim.get_state()
    hist.append((a1, a2, so, sg))
    bad = set()
    for k in so.dtype.names:
        if k.startswith("pad"):
            continue
        if k == "f":
            for fk in so["f"].dtype.names:
                if fk.startswith("pad"):
                    continue
                m = np.any(bits(so["f"][fk]) != bits(sg["f"][fk]), axis=1)
                bad |= set(np.nonzero(m)[0].tolist())
        else:
            m = bits(so[k]) != bits(sg[k])
            if m.ndim > 1:
                m = m.any(axis=1)
            bad |= set(np.nonzero(m)[0].tolist())
    if bad:
        i = min(bad)
        print("first divergence at step", t, "arenas", sorted(bad)[:10])
        for tt in range(max(0, t - 6), t + 1):
            a1_, a2_, so_, sg_ = hist[tt]
            fo, fg = flat(so_, i), flat(sg_, i)
            diffs = {k: (fo[k], fg[k]) for k in fo if not k.startswith("pad") and (np.asarray(fo[k]) != np.asarray(fg[k])).any()}
            print("step", tt, "a1", a1_[i], "a2", a2_[i])
            print("   oracle:", {k: (v.tolist() if hasattr(v, 'tolist') else v) for k, v in fo.items() if not k.startswith('pad')})
            print("   diffs (oracle, gpu):", diffs)
        sys.exit(1)
print("no divergence in", steps, "steps")
