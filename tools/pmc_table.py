#!/usr/bin/env python3
"""Per-kernel averages of every PMC pass under a tools/prof_pmc.sh output directory.

  python tools/pmc_table.py gpurun_out/pmc11_fused [--ticks 100] [--waves 2048]

prints counter averages per dispatch and, with --ticks/--waves, per wave-tick.
--json OUT (with --ticks/--waves/--envs) also writes the per-wave-tick SQ table of the step
kernel and its wave-issue fraction: instructions issued per wave-tick / SQ_WAVE_CYCLES per
wave-tick (quad-cycles).  One wave issues at most one instruction per 4 cycles
(MI355X_MICROARCH.md, constants table, 'vector-instruction ISSUE cost'), so that quotient is
the fraction of its own issue ceiling a wave sustains; bench.py reports it beside the HBM
roofline of the same kernel.
"""
import json
import argparse
import csv
import glob
import os
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--ticks", type=int, default=0)
    ap.add_argument("--waves", type=int, default=0)
    ap.add_argument("--kernel", default="k_step")
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--json", default="")
    ap.add_argument("--command", default="")
    a = ap.parse_args()
    vals = {}
    for path in sorted(glob.glob(os.path.join(a.dir, "*", "run_counter_collection.csv"))):
        per = {}
        with open(path) as f:
            for r in csv.DictReader(f):
                if a.kernel not in r["Kernel_Name"]:
                    continue
                key = (re.sub(r"\(.*", "", r["Kernel_Name"]), r["Counter_Name"])
                per.setdefault(key, {}).setdefault(r["Dispatch_Id"], 0.0)
                per[key][r["Dispatch_Id"]] += float(r["Counter_Value"])
        for key, d in per.items():
            vals[key] = sum(d.values()) / len(d)
    for (k, c), v in sorted(vals.items()):
        extra = ""
        if a.ticks and a.waves and c.startswith("SQ_"):
            extra = "  per wave-tick %.1f" % (v / a.ticks / a.waves)
        print("%-28s %-24s %16.1f%s" % (k[-28:], c, v, extra))
    if a.json and a.ticks and a.waves:
        kernels = sorted({k for k, _ in vals})
        docs = []
        for k in kernels:
            per = {c: v / a.ticks / a.waves for (kk, c), v in vals.items() if kk == k and c.startswith("SQ_")}
            issued = sum(per.get(c, 0.0) for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS",
                                                    "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_SMEM",
                                                    "SQ_INSTS_BRANCH"))
            wc = per.get("SQ_WAVE_CYCLES")
            docs.append({"kernel": re.sub(r"^void ", "", k), "envs": a.envs, "ticks_per_launch": a.ticks,
                         "waves": a.waves, "per_wave_tick": per, "insts_per_wave_tick": issued,
                         "wave_issue_frac": issued / wc if wc else None})
        with open(a.json, "w") as f:
            json.dump({"command": a.command, "source": os.path.relpath(a.dir), "kernels": docs}, f, indent=1)


if __name__ == "__main__":
    main()
