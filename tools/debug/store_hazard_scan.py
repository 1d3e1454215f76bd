"""Scan gfx950 ISA (compiler .s or llvm-objdump -d output) for a >8-byte buffer/global store
followed directly by a VALU instruction that writes one of its data VGPRs: the store-data
hazard that needs one wait state, which the compiler leaves out when the store's soffset is
an SGPR (ws_fused_dev.h buf_store_nt). Used by tests/test_isa_hazards.py."""
import re
import sys

_STORE = re.compile(r"(buffer|global)_store_dwordx[34]\b")


def _regs(tok):
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def _instr(line):
    line = line.split("//")[0].split(";")[0].strip()
    return "" if not line or line.endswith(":") or line.startswith(".") else line


def scan(lines):
    """Return [(line_no, store, next_instruction)] for every hazard in `lines`."""
    ins = [(i + 1, _instr(l)) for i, l in enumerate(lines)]
    ins = [(n, t) for n, t in ins if t]
    hits = []
    for k, (n, t) in enumerate(ins[:-1]):
        if not _STORE.match(t):
            continue
        # the data operand: buffer_store vdata, vaddr, ...; global_store vaddr, vdata, saddr
        ops = [o.rstrip(",") for o in t.split()[1:]]
        data = _regs(ops[1] if t.startswith("global_") and len(ops) > 1 else ops[0])
        nxt = ins[k + 1][1]
        if nxt.startswith("v_") and len(nxt.split()) > 1 and _regs(nxt.split()[1].rstrip(",")) & data:
            hits.append((n, t, nxt))
    return hits


if __name__ == "__main__":
    total = 0
    for path in sys.argv[1:]:
        for n, t, nxt in scan(open(path).read().splitlines()):
            total += 1
            print(f"{path}:{n}: {t}  ->  {nxt}")
    print(f"{total} hazard(s)")
