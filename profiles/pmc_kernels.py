"""Mean per launch of every counter in rocprofv3 --pmc CSV directories, per vihmc kernel (bare name).

Usage: python profiles/pmc_kernels.py <dir> [<dir> ...]
SQ_*_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles summed over waves (MI355X_MICROARCH.md, cycle
constants); SQ_VALU_MFMA_BUSY_CYCLES counts cycles. Derived lines: the share of wave cycles each wait class takes,
LDS bank-conflict cycles over LDS-array cycles, and MFMA busy over busy cycles.
"""
import csv
import glob
import re
import sys
from collections import defaultdict

NAME = re.compile(r"vihmc::(k_[A-Za-z0-9_]+)")


def main():
    vals = defaultdict(lambda: defaultdict(list))
    for d in sys.argv[1:]:
        for path in glob.glob(d.rstrip("/") + "/*counter_collection.csv"):
            with open(path) as f:
                for r in csv.DictReader(f):
                    m = NAME.search(r["Kernel_Name"])
                    if m:
                        vals[m.group(1)][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k in sorted(vals):
        c = {n: sum(v) / len(v) for n, v in vals[k].items()}
        print(f"{k}  ({max(len(v) for v in vals[k].values())} launches)")
        for n in sorted(c):
            print(f"  {n:28s} {c[n]:16.0f}")
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_LDS"):
                if n in c:
                    print(f"  {n + ' / wave cycles':42s} {c[n] / wc:.3f}")
        if c.get("SQ_LDS_IDX_ACTIVE") and "SQ_LDS_BANK_CONFLICT" in c:
            print(f"  {'LDS bank conflict / LDS active':42s} {c['SQ_LDS_BANK_CONFLICT'] / c['SQ_LDS_IDX_ACTIVE']:.3f}")


if __name__ == "__main__":
    main()
