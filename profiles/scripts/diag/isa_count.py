"""Static instruction mix per basic block of a gfx950 kernel (hipcc -S output).

Usage: python isa_count.py <file.s> [kernel-substring] [--loops]

For every kernel whose symbol contains the substring, prints per basic block (label) the number of MFMA,
VALU (v_* that are not MFMA), LDS (ds_*), VMEM (global_/buffer_), SALU (s_*) instructions and the VALU/MFMA
ratio; --loops keeps only blocks that are the target of a backward branch (loop bodies), which is where the
issue-port budget of an MFMA-paced kernel is spent. A static count: each block's instructions once per pass.
"""
import re
import sys


def kernels(lines):
    cur, body = None, []
    for ln in lines:
        m = re.match(r"^([A-Za-z_][\w.$]*):\s*(;.*)?$", ln)
        if m and not m.group(1).startswith(".") and "@function" not in ln:
            name = m.group(1)
            if cur is not None and not name.startswith("$") and name.startswith("_Z"):
                yield cur, body
                cur, body = name, []
                continue
            if cur is None and name.startswith("_Z"):
                cur, body = name, []
                continue
        if cur is not None:
            if ln.strip().startswith(".Lfunc_end"):
                yield cur, body
                cur, body = None, []
                continue
            body.append(ln)
    if cur is not None:
        yield cur, body


def classify(op):
    if op.startswith("v_mfma") or op.startswith("v_smfmac"):
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("global_") or op.startswith("buffer_") or op.startswith("flat_"):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    return None


def blocks(body):
    blk, name = [], "entry"
    order = []
    for ln in body:
        s = ln.strip()
        m = re.match(r"^(\.LBB[\w_]+):", s)
        if m:
            order.append((name, blk))
            name, blk = m.group(1), []
            continue
        if not s or s.startswith(";") or s.startswith("."):
            continue
        blk.append(s.split()[0])
        if s.split()[0].startswith("s_cbranch") or s.split()[0] == "s_branch":
            blk.append("->" + s.split()[-1])
    order.append((name, blk))
    return order


def main():
    path = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else ""
    loops_only = "--loops" in sys.argv
    lines = open(path).read().splitlines()
    for kname, body in kernels(lines):
        if sub not in kname:
            continue
        bl = blocks(body)
        names = [b[0] for b in bl]
        back = set()
        for i, (n, ins) in enumerate(bl):
            for x in ins:
                if x.startswith("->"):
                    t = x[2:]
                    if t in names and names.index(t) <= i:
                        back.add(t)
        print(f"== {kname}")
        tot = {"mfma": 0, "valu": 0, "lds": 0, "vmem": 0, "salu": 0, "wait": 0}
        for n, ins in bl:
            c = {"mfma": 0, "valu": 0, "lds": 0, "vmem": 0, "salu": 0, "wait": 0}
            for x in ins:
                k = classify(x)
                if k:
                    c[k] += 1
            for k in tot:
                tot[k] += c[k]
            if loops_only and n not in back:
                continue
            if sum(c.values()) == 0:
                continue
            r = c["valu"] / c["mfma"] if c["mfma"] else float("inf")
            tag = "loop" if n in back else ""
            print(f"  {n:28s} {tag:4s} mfma {c['mfma']:4d} valu {c['valu']:4d} lds {c['lds']:4d} vmem {c['vmem']:4d}"
                  f" salu {c['salu']:4d} wait {c['wait']:4d}  valu/mfma {r:5.2f}")
        r = tot["valu"] / tot["mfma"] if tot["mfma"] else float("inf")
        print(f"  total mfma {tot['mfma']} valu {tot['valu']} lds {tot['lds']} vmem {tot['vmem']} salu {tot['salu']}"
              f" valu/mfma {r:.2f}")


if __name__ == "__main__":
    main()
