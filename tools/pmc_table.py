#!/usr/bin/env python3
"""Per-kernel averages of every PMC pass under a tools/prof_pmc.sh output directory.

  python tools/pmc_table.py gpurun_out/pmc11_fused [--ticks 100] [--waves 2048]

prints counter averages per dispatch and, with --ticks/--waves, per wave-tick.
"""
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


if __name__ == "__main__":
    main()
