#!/usr/bin/env python3
"""Reduce a tools/prof_bench.sh output directory to the files committed under profiles/.

  python tools/summarize_profile.py gpurun_out/prof9 r01 --envs 65536 --chunk 100

writes profiles/<tag>_kernel_stats.csv (the --kernel-trace --stats summary of the
bench command, verbatim) and profiles/<tag>_traffic.json: per step kernel the average
launch duration from the trace pass and the per-launch FETCH_SIZE / WRITE_SIZE from
the PMC passes.  HBM bytes per launch = (2 x FETCH_SIZE + WRITE_SIZE) x 1024: both
counters are in KiB and gfx950's FETCH_SIZE reports half the bytes of a coalesced
read (MI355X_MICROARCH.md, HBM section).
"""
import argparse
import csv
import json
import os
import re
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    name = re.sub(r"^void ", "", name)
    return re.sub(r"\(.*$", "", name)


def counters(path):
    agg = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            agg.setdefault(short(r["Kernel_Name"]), {}).setdefault(int(r["Dispatch_Id"]), 0.0)
            agg[short(r["Kernel_Name"])][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    return {k: sum(v.values()) / len(v) for k, v in agg.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("tag")
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--chunk", type=int, default=100)
    ap.add_argument("--command", default="python3 bench.py --steps 400 --warmup 100 --no-cpu-baseline")
    a = ap.parse_args()
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    stats = os.path.join(a.dir, "trace", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(out, "%s_kernel_stats.csv" % a.tag))
    avg = {}
    with open(stats) as f:
        for r in csv.DictReader(f):
            avg[short(r["Name"])] = (float(r["AverageNs"]), int(r["Calls"]))
    fetch = counters(os.path.join(a.dir, "fetch", "run_counter_collection.csv"))
    write = counters(os.path.join(a.dir, "write", "run_counter_collection.csv"))
    kernels = []
    for k, (ns, calls) in sorted(avg.items()):
        if not re.match(r"fsk::k_step", k) or k not in fetch or k not in write:
            continue
        ticks = 1 if re.match(r"fsk::k_step<", k) else a.chunk
        kernels.append({"kernel": k, "envs": a.envs, "ticks_per_launch": ticks, "calls": calls,
                        "avg_duration_ns": ns, "fetch_size_kib": fetch[k], "write_size_kib": write[k],
                        "traffic_bytes_per_launch": (2 * fetch[k] + write[k]) * 1024})
    doc = {"command": a.command, "source": os.path.relpath(a.dir, ROOT), "kernels": kernels}
    with open(os.path.join(out, "%s_traffic.json" % a.tag), "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main()
