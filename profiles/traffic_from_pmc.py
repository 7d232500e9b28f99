"""HBM traffic per launch of the roofline kernel, from two rocprofv3 PMC passes of the bench command.

Usage: python profiles/traffic_from_pmc.py <fetch_dir> <write_dir> <out.json> [chains_per_gpu] [kernel]
  <fetch_dir>: rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE  -- python3 bench.py ...
  <write_dir>: rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE  -- python3 bench.py ...
Side-A contraction launches are the k_contract_bf dispatches (bf16x6 side A, the default; side B runs
k_contract_bf_b) or k_contract_ws (fp32-MFMA side A, VIHMC_CONTRACT_BF16=0). The kernel name is matched as
a whole identifier, so k_contract_bf does not match k_contract_bf_b.
gfx950 correction (MI355X_MICROARCH.md, HBM/rocprofv3): FETCH_SIZE reports 1/2 of the bytes of wide
coalesced streaming reads -> doubled; WRITE_SIZE is exact for 16-B-per-lane stores. Both are KB.
bench.py reads the resulting JSON into roofline.traffic when its config matches.
"""
import csv
import glob
import json
import re
import sys

KERNEL = "k_contract_bf"


def side_a_values(d, counter):
    pat = re.compile(r"(^|[^A-Za-z0-9_])" + KERNEL + r"($|[^A-Za-z0-9_])")
    rows = []
    for path in glob.glob(d.rstrip("/") + "/*counter_collection.csv"):
        with open(path) as f:
            for r in csv.DictReader(f):
                if pat.search(r["Kernel_Name"]) and r["Counter_Name"] == counter:
                    rows.append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    rows.sort()
    return [v for _, v in rows]


def main():
    global KERNEL
    fd, wd, out = sys.argv[1:4]
    C = int(sys.argv[4]) if len(sys.argv) > 4 else 16
    if len(sys.argv) > 5:
        KERNEL = sys.argv[5]
    fa = side_a_values(fd, "FETCH_SIZE")
    wa = side_a_values(wd, "WRITE_SIZE")
    fetch = 2.0 * 1024.0 * sum(fa) / len(fa)
    write = 1024.0 * sum(wa) / len(wa)
    res = {"kernel": KERNEL + " (side A)", "chains_per_gpu": C, "contract_bf16x6": int(KERNEL == "k_contract_bf"), "launches_fetch": len(fa),
           "launches_write": len(wa), "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
           "hbm_bytes_per_launch": fetch + write,
           "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes over bench.py; FETCH x2 (gfx950)"}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
