"""Per-dispatch durations of the small kernels of one bench trajectory (rocprofv3 --kernel-trace csv).

    python profiles/scripts/probes/ktrace_small.py <kernel_trace.csv> [pattern ...]
"""
import csv
import sys


def main():
    path = sys.argv[1]
    pats = sys.argv[2:] or ["k_gather_prior", "k_reduce", "k_leap_open", "k_scatter", "k_gram_sum", "k_fwd_fused",
                            "k_bwd_bf2", "k_gram_a", "k_gram_b", "k_contract"]
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # the last 400 dispatches of the trace: one or two trajectories of the timed region
    rows = rows[-400:]
    t0 = int(rows[0]["Start_Timestamp"])
    prev_end = None
    for r in rows:
        name = r["Kernel_Name"]
        if not any(p in name for p in pats):
            continue
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev_end) / 1e3 if prev_end else 0.0
        prev_end = e
        print(f"{(s - t0) / 1e3:10.1f} us  {((e - s) / 1e3):8.2f} us  gap {gap:7.2f}  grid {r.get('Grid_Size', '?'):>9}  "
              f"{name[:70]}")


if __name__ == "__main__":
    main()
