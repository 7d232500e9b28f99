"""HBM traffic per launch of every vihmc kernel, from two rocprofv3 PMC passes of the bench command.

Usage: python profiles/traffic_from_pmc.py <fetch_dir> <write_dir> <out.json> [chains_per_gpu] [source-tag]
  <fetch_dir>: rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE  -- python3 bench.py ...
  <write_dir>: rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE  -- python3 bench.py ...
Kernels are keyed by their bare name (``vihmc::k_bwd_bf(vihmc::BwdArgs)`` -> ``k_bwd_bf``, template arguments
dropped), so k_contract_bf (side A) and k_contract_bf_b (side B) stay separate.
gfx950 correction (MI355X_MICROARCH.md, HBM/rocprofv3): FETCH_SIZE reports 1/2 of the bytes of wide
coalesced streaming reads -> doubled; WRITE_SIZE is exact for 16-B-per-lane stores. Both are KB.
bench.py reads profiles/traffic.json into roofline.traffic for the kernel it prices, when the chain count matches.
"""
import csv
import glob
import json
import re
import sys
from collections import defaultdict

NAME = re.compile(r"vihmc::(k_[A-Za-z0-9_]+)")


def per_kernel(d, counter):
    vals = defaultdict(list)
    for path in glob.glob(d.rstrip("/") + "/*counter_collection.csv"):
        with open(path) as f:
            for r in csv.DictReader(f):
                m = NAME.search(r["Kernel_Name"])
                if m and r["Counter_Name"] == counter:
                    vals[m.group(1)].append(float(r["Counter_Value"]))
    return vals


def main():
    fd, wd, out = sys.argv[1:4]
    C = int(sys.argv[4]) if len(sys.argv) > 4 else 16
    src = sys.argv[5] if len(sys.argv) > 5 else fd
    fa = per_kernel(fd, "FETCH_SIZE")
    wa = per_kernel(wd, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fa) & set(wa)):
        fetch = 2.0 * 1024.0 * sum(fa[k]) / len(fa[k])
        write = 1024.0 * sum(wa[k]) / len(wa[k])
        kernels[k] = {"launches_fetch": len(fa[k]), "launches_write": len(wa[k]), "fetch_bytes_per_launch": fetch,
                      "write_bytes_per_launch": write, "hbm_bytes_per_launch": fetch + write}
    res = {"chains_per_gpu": C, "source": src, "kernels": kernels,
           "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes over bench.py; FETCH x2 (gfx950)"}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
