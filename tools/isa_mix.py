#!/usr/bin/env python3
"""Instruction mix of a kernel's steady-state march loop (measurement aid, not product).

Reads gfx950 assembly (hipcc --cuda-device-only -S), takes one kernel (a substring of its
mangled name), finds its loops (a backward s_cbranch / s_branch to a label) and reports the
largest one's instruction classes: fp64 VALU (4 issue cycles per wave64 on SIMD-32), other
VALU incl. DPP moves and packed fp32 (2 cycles), LDS, vector memory, SALU, s_nop (with its
wait states), s_waitcnt. The fp64 / 32-bit split prices SQ_INSTS_VALU in cycles (bench.py).
  python tools/isa_mix.py /tmp/dppy_f64_2.s 'fused_dppy_kernelIdLi4ELi2ELi3ELi1ELb0E'
"""
import collections
import re
import sys


def kernel_lines(path, key):
    lines = open(path).read().splitlines()
    start = None
    for i, l in enumerate(lines):
        head = l.split(";")[0].strip()
        if head.endswith(":") and key in head and not head.startswith("."):
            start = i
            break
    if start is None:
        raise SystemExit(f"kernel {key} not found")
    out = []
    for l in lines[start + 1:]:
        if l.strip().startswith(".Lfunc_end"):
            break
        out.append(l)
    return out


def classify(ins):
    op = ins.split()[0]
    if op.startswith("s_nop"):
        return "s_nop"
    if op.startswith("s_waitcnt"):
        return "s_waitcnt"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_", "global_", "flat_")):
        return "vmem"
    if op.startswith("v_"):
        if "_dpp" in op or "row_" in ins or "wave_sh" in ins or "quad_perm" in ins:
            return "valu_dpp"
        if op.endswith("_f64") or "_f64_" in op:
            return "valu_f64"
        return "valu_32"
    return "other"


def main():
    path, key = sys.argv[1], sys.argv[2]
    body = kernel_lines(path, key)
    labels = {}
    ins = []  # (index, text)
    for l in body:
        s = l.strip()
        m = re.match(r"^(\.LBB\d+_\d+):", s)
        if m:
            labels[m.group(1)] = len(ins)
            continue
        if not s or s.startswith((";", ".", "//")):
            continue
        ins.append(s.split(";")[0].strip())
    loops = []
    for j, t in enumerate(ins):
        m = re.match(r"^s_(cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", t)
        if m and m.group(2) in labels and labels[m.group(2)] <= j:
            loops.append((labels[m.group(2)], j))
    if not loops:
        raise SystemExit("no loop")
    which = int(sys.argv[3]) if len(sys.argv) > 3 else None
    for k, (a, b) in enumerate(loops):
        print(f"  loop {k}: {b - a + 1} instructions")
    lo, hi = loops[which] if which is not None else max(loops, key=lambda p: p[1] - p[0])
    mix = collections.Counter()
    nop_states = 0
    for t in ins[lo:hi + 1]:
        c = classify(t)
        mix[c] += 1
        if c == "s_nop":
            m = re.match(r"s_nop\s+(\d+)", t)
            nop_states += 1 + (int(m.group(1)) if m else 0)
    total_valu = mix["valu_f64"] + mix["valu_32"] + mix["valu_dpp"]
    print(f"kernel {key}: {len(loops)} loops, largest {hi - lo + 1} instructions")
    for k in ("valu_f64", "valu_32", "valu_dpp", "lds", "vmem", "salu", "s_nop", "s_waitcnt", "other"):
        print(f"  {k:10s} {mix[k]:6d}")
    print(f"  s_nop wait states {nop_states}")
    cyc = 4 * mix["valu_f64"] + 2 * (mix["valu_32"] + mix["valu_dpp"])
    print(f"  VALU {total_valu}, SIMD-32 issue cycles {cyc} = {cyc / max(total_valu, 1):.3f} per VALU instruction")


if __name__ == "__main__":
    main()
