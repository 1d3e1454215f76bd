"""Debug aid: scan gfx950 ISA (.s) for a >8-byte buffer store followed directly by a VALU
instruction writing one of its data VGPRs (the store-data hazard that needs one wait state)."""
import re, sys

def regs(tok):
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)", tok)
    return {int(m.group(1))} if m else set()

hits = 0
for path in sys.argv[1:]:
    lines = [l.strip() for l in open(path)]
    for i, l in enumerate(lines):
        if not re.match(r"buffer_store_dwordx[34]|global_store_dwordx[34]", l):
            continue
        data = regs(l.split()[1].rstrip(","))
        j = i + 1
        while j < len(lines) and (not lines[j] or lines[j].startswith(";")):
            j += 1
        nxt = lines[j] if j < len(lines) else ""
        if nxt.startswith("v_"):
            dst = regs(nxt.split()[1].rstrip(","))
            if dst & data:
                hits += 1
                print(f"{path}:{i + 1}: {l}  ->  {nxt}")
print(f"{hits} hazard(s)")
