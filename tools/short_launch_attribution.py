#!/usr/bin/env python3
"""Where a short fused launch's time goes beyond its steady ticks (measurement).

  python tools/short_launch_attribution.py TIMELINE_JSON [--ticks 20] [--json OUT]

Reads tools/timeline_probe.py's per-wave s_memrealtime stamps (t0 entry, t1 after the prologue,
t2 after the tick loop, t3 after the final stores drained; HW_ID and XCC_ID) of one isolated launch
of `ticks` ticks and of the 1000-tick launch, and splits the launch's span (first wave entry to last
wave drained) along its critical path -- the wave that ends last -- into:
  dispatch_stagger  its entry after the launch's first wave entry (the XCDs start apart);
  prologue          its state loads and table staging;
  steady_ticks      ticks x the 1000-tick launch's median per-tick loop time;
  loop_ramp         the median wave's loop beyond steady_ticks (short-launch start-up);
  loop_tail         the last wave's loop beyond the median wave's (the younger wave of a SIMD pair
                    running its last ticks alone, skew between SIMDs);
  drain             its final state stores.
"""
import argparse
import collections
import json
import statistics


def analyse(doc, ticks):
    raw = doc["raw_%d" % ticks]
    t0 = min(r[0] for r in raw)
    us = lambda v: (v - t0) / 100.0  # noqa: E731  (100 MHz)
    last = max(raw, key=lambda r: r[3])
    loop = lambda r: (r[2] - r[1]) / 100.0  # noqa: E731
    steady = statistics.median(loop(r) for r in doc["raw_1000"]) / 1000.0
    med = statistics.median(loop(r) for r in raw)
    slot = lambda r: int(r[4]) & 15  # noqa: E731
    by_slot = collections.defaultdict(list)
    for r in raw:
        by_slot[slot(r)].append(loop(r))
    parts = {
        "dispatch_stagger_us": us(last[0]),
        "prologue_us": (last[1] - last[0]) / 100.0,
        "steady_ticks_us": ticks * steady,
        "loop_ramp_us": med - ticks * steady,
        "loop_tail_us": loop(last) - med,
        "drain_us": (last[3] - last[2]) / 100.0,
    }
    span = us(last[3])
    return {
        "ticks": ticks, "waves": len(raw), "span_us": round(span, 3),
        "critical_path": {k: round(v, 3) for k, v in parts.items()},
        "check_sum_us": round(sum(parts.values()), 3),
        "steady_us_per_tick": round(steady, 4),
        "excess_over_steady_us": round(span - ticks * steady, 3),
        "last_wave": {"xcc": int(last[5]) & 15, "se": (int(last[4]) >> 13) & 7, "cu": (int(last[4]) >> 8) & 31,
                      "simd": (int(last[4]) >> 4) & 3, "slot": slot(last)},
        "loop_us_median_by_wave_slot": {str(k): round(statistics.median(v), 3) for k, v in sorted(by_slot.items())},
        "xcc_first_entry_us": {str(k): round(v, 3) for k, v in sorted(
            {x: min(us(r[0]) for r in raw if int(r[5]) & 15 == x) for x in {int(r[5]) & 15 for r in raw}}.items())},
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("timeline")
    ap.add_argument("--ticks", type=int, default=20)
    ap.add_argument("--json")
    a = ap.parse_args()
    with open(a.timeline) as f:
        doc = json.load(f)
    res = analyse(doc, a.ticks)
    res["source"] = a.timeline
    res["shape"] = next(s for s in doc["shapes"] if s["ticks"] == a.ticks)
    s = json.dumps(res, indent=1)
    if a.json:
        with open(a.json, "w") as f:
            f.write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
