"""Per-kernel summary (calls, total/avg/min duration) from a rocprofv3 results database or
kernel_stats.csv.  Usage: python profiles/kstats.py <run_results.db | kernel_stats.csv> [top]"""
import csv
import sqlite3
import sys


def from_db(path):
    con = sqlite3.connect(path)
    rows = con.execute("select name, start, end from kernels").fetchall()
    agg = {}
    for name, s, e in rows:
        a = agg.setdefault(name, [0, 0.0, float("inf")])
        d = (e - s) / 1e3
        a[0] += 1
        a[1] += d
        a[2] = min(a[2], d)
    return [(n, c, t, t / c, m) for n, (c, t, m) in agg.items()]


def from_csv(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            c = int(r["Calls"])
            out.append((r["Name"], c, float(r["TotalDurationNs"]) / 1e3, float(r["AverageNs"]) / 1e3,
                        float(r["MinNs"]) / 1e3))
    return out


def main():
    path = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    rows = from_db(path) if path.endswith(".db") else from_csv(path)
    rows.sort(key=lambda r: -r[2])
    tot = sum(r[2] for r in rows)
    print(f"{'kernel':70s} {'calls':>6s} {'total_us':>10s} {'avg_us':>9s} {'min_us':>9s} {'pct':>6s}")
    for n, c, t, a, m in rows[:top]:
        print(f"{n[:70]:70s} {c:6d} {t:10.1f} {a:9.2f} {m:9.2f} {100 * t / tot:6.2f}")


if __name__ == "__main__":
    main()
