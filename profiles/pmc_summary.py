"""Per-kernel PMC summary from profiles/pmc_passes.sh output.

Usage: python profiles/pmc_summary.py gpurun_out/<name>   (reads <name>_{a..e}/p_counter_collection.csv)
Ratios follow /opt/skills/guides/MI355X_MICROARCH.md: WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~=
WAVE_CYCLES (quad-cycles); MFMA util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 32 CUs * 4
SIMDs); FETCH_SIZE (KB) is doubled on gfx950 (guide's HBM/rocprofv3 section), WRITE_SIZE is not.
"""
import collections
import csv
import glob
import sys


def load(prefix):
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    calls = collections.defaultdict(set)
    for path in sorted(glob.glob(prefix + "_*/p_counter_collection.csv")):
        tag = path.split("/")[-2]
        with open(path) as f:
            for r in csv.DictReader(f):
                k = r["Kernel_Name"]
                vals[k][r["Counter_Name"]] += float(r["Counter_Value"])
                calls[(k, tag)].add(r["Dispatch_Id"])
    ncalls = collections.defaultdict(dict)
    for (k, tag), ids in calls.items():
        ncalls[k][tag] = len(ids)
    return vals, ncalls


def main():
    prefix = sys.argv[1].rstrip("/")
    vals, ncalls = load(prefix)
    order = sorted(vals, key=lambda k: -vals[k].get("SQ_WAVE_CYCLES", 0))
    for k in order[:8]:
        v = vals[k]
        wc = v.get("SQ_WAVE_CYCLES", 0) or 1
        print(k[:90])
        print("   calls/pass", dict(ncalls[k]))
        print("   wait_any %.2f  wait_inst %.2f  active %.2f  (of wave-cycles)" % (
            v.get("SQ_WAIT_ANY", 0) / wc, v.get("SQ_WAIT_INST_ANY", 0) / wc, v.get("SQ_ACTIVE_INST_ANY", 0) / wc))
        print("   active valu %.2f lds %.2f vmem %.2f  wait_inst_lds %.2f" % (
            v.get("SQ_ACTIVE_INST_VALU", 0) / wc, v.get("SQ_ACTIVE_INST_LDS", 0) / wc,
            v.get("SQ_ACTIVE_INST_VMEM", 0) / wc, v.get("SQ_WAIT_INST_LDS", 0) / wc))
        g = v.get("GRBM_GUI_ACTIVE", 0)
        na = ncalls[k].get(prefix.split("/")[-1] + "_a", 1) or 1
        nb = ncalls[k].get(prefix.split("/")[-1] + "_b", 1) or 1
        if g:
            simd_cycles = g / 2 / 8 * 1024   # GRBM_GUI_ACTIVE (summed over 8 XCDs) collected in passes a and b; 1024 SIMDs
            print("   mfma util %.2f  coexec %.2f" % (v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / simd_cycles,
                                                    v.get("SQ_VALU_MFMA_COEXEC_CYCLES", 0) / simd_cycles))
        ni = v.get("SQ_INSTS_MFMA", 0)
        if ni:
            print("   per MFMA: valu %.2f lds %.2f salu %.2f vmem_rd %.3f vmem_wr %.3f   mean waves %.1f" % (
                v.get("SQ_INSTS_VALU", 0) / ni - 1, v.get("SQ_INSTS_LDS", 0) / ni, v.get("SQ_INSTS_SALU", 0) / ni,
                v.get("SQ_INSTS_VMEM_RD", 0) / ni, v.get("SQ_INSTS_VMEM_WR", 0) / ni,
                v.get("SQ_LEVEL_WAVES", 0) / (v.get("SQ_BUSY_CYCLES", 1) or 1)))
        if v.get("SQ_LDS_IDX_ACTIVE"):
            print("   lds bank-conflict/idx %.2f" % (v["SQ_LDS_BANK_CONFLICT"] / v["SQ_LDS_IDX_ACTIVE"]))
        nd = ncalls[k].get(prefix.split("/")[-1] + "_d", 1) or 1
        ne = ncalls[k].get(prefix.split("/")[-1] + "_e", 1) or 1
        if "FETCH_SIZE" in v:
            print("   HBM fetch %.1f MB/dispatch (x2 gfx950)  write %.1f MB/dispatch" % (
                2 * v["FETCH_SIZE"] / 1024 / nd, v.get("WRITE_SIZE", 0) / 1024 / ne))


if __name__ == "__main__":
    main()
