"""Per-kernel summary of a rocprofv3 --kernel-trace CSV, split into phases at each k_bwd_chain grid size (the one-chain
legs of probe_legs.py: the DeepONet leg's plan and config 4's half-shard plans launch different grids), with the idle
gap before each kernel.

    python profiles/scripts/diag/trace_summary.py gpurun_out/r05lt/t_kernel_trace.csv
"""
import collections
import csv
import re
import sys


def name(r):
    n = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("vihmc::", "").replace("void ", "")
    return n[:44]


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    # phase = the grid of the most recent k_bwd_chain launch
    phase, prev_end = None, None
    stats = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if "k_bwd_chain" in r["Kernel_Name"]:
            phase = "bwd_chain grid " + r["Grid_Size_X"]
        gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
        prev_end = e
        if phase is None:
            continue
        stats[phase][name(r)].append(((e - s) / 1e3, gap))
    for ph, ks in stats.items():
        n_chain = len(ks.get("k_bwd_chain", [])) or 1
        print(f"== phase {ph}: {n_chain} evaluations with the chain backward")
        print(f"{'kernel':44s} {'calls':>6s} {'avg_us':>8s} {'per_eval_us':>11s} {'gap_before_us':>13s}")
        tot = 0.0
        for k, v in sorted(ks.items(), key=lambda kv: -sum(x[0] for x in kv[1])):
            d = sum(x[0] for x in v)
            g = sum(min(x[1], 1000.0) for x in v)
            tot += d
            print(f"{k:44s} {len(v):6d} {d / len(v):8.2f} {d / n_chain:11.2f} {g / len(v):13.2f}")
        print(f"{'sum of kernel time per evaluation':44s} {'':6s} {'':8s} {tot / n_chain:11.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
