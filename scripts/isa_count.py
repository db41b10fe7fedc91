"""Instruction counts per basic block of one kernel in a gfx950 assembly dump
(hipcc --cuda-device-only -S), for the ISA-level view of a hot loop.

usage:
  hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -munsafe-fp-atomics \
        -x hip --cuda-device-only -S csrc/bhtree.hip -o /tmp/bhtree.s
  python scripts/isa_count.py /tmp/bhtree.s 'bh_traverseILi0ELb0E' [--blocks]

Prints, per basic block (.LBB label), the counts of VALU (v_*; fp64 ones
apart), SALU (s_* minus branches / waitcnt), branches, LDS (ds_*), vector
memory (global_* / buffer_* / flat_*) and scalar memory (s_load / s_buffer)
instructions, and the loop back-edges (a branch to an earlier block), so that
the blocks of a loop body can be summed by hand or with --range A:B.
"""
import argparse
import re
import sys

FP64 = re.compile(r"^v_(\w+)_f64|^v_fma_f64|^v_rcp_f64|^v_rsq_f64|^v_sqrt_f64|^v_ldexp_f64|^v_div_\w+_f64|^v_cvt_f64")


def kernel_lines(path, key):
    lines = open(path).read().splitlines()
    start = None
    for i, l in enumerate(lines):
        if start is None and key in l and l.rstrip().endswith(":") is False and re.match(r"^_Z\S*:", l) and key in l.split(":")[0]:
            start = i
            continue
        if start is not None and (l.startswith(".Lfunc_end") or l.strip().startswith(".size")):
            return lines[start:i]
    if start is not None:
        return lines[start:]
    sys.exit(f"kernel matching {key!r} not found")


def classify(op):
    if op.startswith("v_"):
        return "valu64" if FP64.match(op) else "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith(("s_waitcnt", "s_nop", "s_barrier", "s_sleep")):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("kernel", help="substring of the mangled kernel name")
    ap.add_argument("--range", default="", help="sum blocks A:B (label numbers, inclusive)")
    a = ap.parse_args()
    body = kernel_lines(a.asm, a.kernel)
    blocks, order = {}, []
    cur = "entry"
    blocks[cur] = {"n": 0}
    order.append(cur)
    back = []
    for l in body[1:]:
        s = l.strip()
        m = re.match(r"^(\.LBB\d+_\d+):", s)
        if m:
            cur = m.group(1)
            blocks[cur] = {"n": 0}
            order.append(cur)
            continue
        if not s or s.startswith((";", ".", "//")):
            continue
        op = s.split()[0]
        k = classify(op)
        if k is None:
            continue
        b = blocks[cur]
        b[k] = b.get(k, 0) + 1
        b["n"] += 1
        if k == "branch":
            t = s.split()[-1]
            if t in blocks and order.index(t) <= order.index(cur):
                back.append((cur, t))
    keys = ["valu", "valu64", "salu", "branch", "lds", "vmem", "smem", "wait"]
    print(f"{'block':14s} " + " ".join(f"{k:>7s}" for k in keys))
    tot = {k: 0 for k in keys}
    for name in order:
        b = blocks[name]
        if b["n"] == 0:
            continue
        print(f"{name:14s} " + " ".join(f"{b.get(k, 0):7d}" for k in keys))
        for k in keys:
            tot[k] += b.get(k, 0)
    print(f"{'total':14s} " + " ".join(f"{tot[k]:7d}" for k in keys))
    print("back-edges:", ", ".join(f"{s}->{t}" for s, t in back))
    if a.range:
        lo, hi = (int(x) for x in a.range.split(":"))
        sel = [n for n in order if n.startswith(".LBB") and lo <= int(n.split("_")[-1]) <= hi]
        sums = {k: sum(blocks[n].get(k, 0) for n in sel) for k in keys}
        print(f"range {a.range}: " + " ".join(f"{k} {sums[k]}" for k in keys))


if __name__ == "__main__":
    main()
