"""Per-kernel summary of a rocprofv3 kernel trace written in its SQLite (rocpd) format:
calls, total / average / min / max duration and share, like `--stats`' kernel_stats.csv.

    python tools/rocpd_stats.py gpurun_out/<dir>/<name>_results.db [--per N]

`--per N` adds the total divided by N (e.g. PPO iterations in the traced run)."""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--per", type=int, default=0)
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    rows = con.execute("select name, count(*), sum(duration), min(duration), max(duration) from kernels "
                       "group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    head = "%-70s %6s %11s %10s %10s %10s %6s" % ("kernel", "calls", "total_us", "avg_us", "min_us", "max_us", "%")
    if a.per:
        head += " %12s" % ("us/" + str(a.per))
    print(head)
    for name, n, tot, lo, hi in rows:
        line = "%-70s %6d %11.1f %10.2f %10.2f %10.2f %6.2f" % (name[:70], n, tot / 1e3, tot / n / 1e3, lo / 1e3,
                                                             hi / 1e3, 100.0 * tot / total)
        if a.per:
            line += " %12.1f" % (tot / 1e3 / a.per)
        print(line)
    print("all kernels: %.1f us" % (total / 1e3))


if __name__ == "__main__":
    main()
