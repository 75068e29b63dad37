"""Summarise rocprofv3 kernel statistics (kernel_stats.csv or a rocpd results.db):
per kernel calls, average and per-step microseconds, share of GPU time.
usage: python tools/kstats.py <kernel_stats.csv | results.db> [steps]"""
import csv
import re
import sqlite3
import sys


def load(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        return [(n, int(k), float(t) * 1e3) for n, k, t in
                c.execute("select name, total_calls, total_duration from top_kernels")]  # us -> ns
    return [(r["Name"], int(r["Calls"]), float(r["TotalDurationNs"])) for r in csv.DictReader(open(path))]


def main():
    rows = load(sys.argv[1])
    steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    tot = sum(t for _, _, t in rows)
    print(f"{'kernel':64s} {'calls':>6s} {'avg_us':>9s} {'per_step_us':>11s} {'pct':>6s}")
    for name, calls, t in sorted(rows, key=lambda r: -r[2]):
        short = re.sub(r"\(.*", "", name)[:64]
        print(f"{short:64s} {calls:6d} {t / calls / 1e3:9.1f} {t / 1e3 / steps:11.1f} {100 * t / tot:6.1f}")


if __name__ == "__main__":
    main()
