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


# ---------------------------------------------------------------------------------------
# Rule 2 (round 5): stores through an address that is undefined on some path.
#
# The bvort RK4 fp64 fault of rounds 2-3: the compiler lowered a switch over
# stores with the store pointer as a phi whose SGPR pair was `implicit-def` (undefined) on one
# edge, and the store's 64-bit VGPR address was then computed from that pair. No source-level
# index was out of range. This rule finds the pattern in DISASSEMBLED code (the built library's
# gfx950 code objects, where no implicit-def comments survive) by a forward may-be-undefined
# analysis over each kernel's control-flow graph:
#   * at entry every SGPR beyond the hardware-preloaded ones (user SGPRs, workgroup ids /
#     info, private segment offset: the kernel descriptor's COMPUTE_PGM_RSRC2) is undefined;
#     VGPRs are taken as defined (undefinedness is only tracked from SGPRs: VGPR merges of
#     exec-masked branches would otherwise flag every structurized if / else);
#   * an instruction's destinations become undefined iff one of its register sources is;
#   * at a join, a register is undefined if it is on ANY incoming path;
#   * a global / buffer / flat store whose address operands (vaddr, saddr, srsrc, soffset)
#     may be undefined is reported.
# ---------------------------------------------------------------------------------------
import struct

_REG = re.compile(r"^(?:(?P<k>[sv])(?P<n>\d+)|(?P<kk>[sv])\[(?P<a>\d+):(?P<b>\d+)\]|(?P<sp>vcc|vcc_lo|vcc_hi|m0))$")
_NO_DEST = re.compile(r"^(s_cmp|s_bitcmp|s_cbranch|s_branch|s_waitcnt|s_nop|s_endpgm|s_barrier|s_setprio|s_sleep|"
                      r"s_sendmsg|s_setreg|s_set_gpr_idx|s_trap|s_icache|s_dcache|s_ttrace|s_wait|s_delay|s_sethalt|"
                      r"s_setkill|s_cbranch|s_code_end|s_incperflevel|s_decperflevel|"
                      r"buffer_store|global_store|flat_store|scratch_store|ds_write|ds_store|exp|"
                      r"buffer_wbl2|buffer_inv|buffer_wbinvl1|s_store|s_scratch_store|s_buffer_store)")


def _regset(tok):
    """Registers named by one operand token ({'s4', 's5'}, {'v7'}, {'vcc'}) or empty."""
    tok = tok.strip().rstrip(",")
    if tok.startswith("-"):
        tok = tok[1:]
    tok = re.sub(r"^\|(.*)\|$", r"\1", tok)  # |v1| (abs)
    m = _REG.match(tok)
    if not m:
        return set()
    if m.group("k"):
        return {m.group("k") + m.group("n")}
    if m.group("kk"):
        return {f"{m.group('kk')}{i}" for i in range(int(m.group("a")), int(m.group("b")) + 1)}
    return {"vcc"}


def _dests_and_srcs(ins):
    """(destination registers, source registers) of one instruction (text)."""
    op, _, rest = ins.partition(" ")
    ops = [o for o in (x.strip() for x in rest.split(",")) if o]
    toks = [o.split()[0] if o.split() else o for o in ops]  # drop modifiers glued after a space
    regs = [_regset(t) for t in toks]
    if not regs or _NO_DEST.match(op):
        return set(), set().union(*regs) if regs else set()
    if op.startswith("v_cmp") and "_e64" not in op and not op.startswith("v_cmpx"):
        return {"vcc"}, set().union(*regs)  # VOPC e32: vcc = compare(src0, src1)
    dests = set(regs[0])
    srcs = set().union(*regs[1:]) if len(regs) > 1 else set()
    # two-destination VALU ops: v_add_co / v_sub_co / v_addc / v_subb / v_div_scale / v_mad_u64
    if re.match(r"v_(add|sub|subrev)(_co|c_co|b_co)?_u32|v_addc|v_subb|v_div_scale|v_mad_[iu]64", op) and len(regs) > 2 \
            and (toks[1].startswith("s") or toks[1].startswith("vcc")):
        dests |= regs[1]
        srcs = set().union(*regs[2:]) if len(regs) > 2 else set()
    return dests, srcs


def _store_addr_regs(ins):
    op, _, rest = ins.partition(" ")
    toks = [o.strip().split()[0] for o in rest.split(",") if o.strip()]
    if op.startswith("global_store") or op.startswith("global_atomic") or op.startswith("flat_store"):
        regs = set(_regset(toks[0])) if toks else set()
        if len(toks) > 2:
            regs |= _regset(toks[2])  # saddr (or 'off')
        return regs
    if op.startswith("buffer_store") or op.startswith("buffer_atomic"):
        regs = set()
        for t in toks[1:4]:  # vaddr (or off), srsrc, soffset
            regs |= _regset(t)
        return regs
    return None


_LINE = re.compile(r"^\s+(?P<ins>[a-z_][^/]*?)\s*//\s*(?P<addr>[0-9A-Fa-f]+):[^<]*(?:<(?P<tgt>[^>+]+)(?:\+0x(?P<off>[0-9a-fA-F]+))?>)?\s*$")
_FUNC = re.compile(r"^(?P<addr>[0-9a-fA-F]+) <(?P<name>[^>]+)>:$")


def parse_functions(lines):
    """{name: (start address, [(address, instruction, branch target address or None)])} from
    llvm-objdump -d output."""
    funcs, cur = {}, None
    for l in lines:
        m = _FUNC.match(l)
        if m:
            cur = m.group("name")
            funcs[cur] = (int(m.group("addr"), 16), [])
            continue
        m = _LINE.match(l)
        if m and cur is not None:
            tgt = None
            if m.group("tgt") and m.group("ins").startswith(("s_branch", "s_cbranch")):
                base = funcs.get(m.group("tgt"), (None,))[0]
                if base is not None:
                    tgt = base + int(m.group("off") or "0", 16)
            funcs[cur][1].append((int(m.group("addr"), 16), m.group("ins").strip(), tgt))
    return funcs


def undefined_address_stores(ins_list, npreload):
    """Stores of one kernel whose address may be undefined: [(address, instruction, regs)]."""
    if not ins_list:
        return []
    addrs = [a for a, _, _ in ins_list]
    index = {a: i for i, a in enumerate(addrs)}
    leaders = {0}
    for i, (a, t, tgt) in enumerate(ins_list):
        if t.startswith(("s_branch", "s_cbranch", "s_endpgm", "s_setpc", "s_swappc")):
            if i + 1 < len(ins_list):
                leaders.add(i + 1)
            if tgt is not None and tgt in index:
                leaders.add(index[tgt])
    starts = sorted(leaders)
    blocks = [(s, (starts[k + 1] if k + 1 < len(starts) else len(ins_list))) for k, s in enumerate(starts)]
    bid = {s: k for k, (s, _) in enumerate(blocks)}
    succ = []
    for s, e in blocks:
        a, t, tgt = ins_list[e - 1]
        out = []
        if tgt is not None and tgt in index:
            out.append(bid[index[tgt]])
        if not t.startswith(("s_branch", "s_endpgm", "s_setpc")) and e < len(ins_list):
            out.append(bid[e])
        succ.append(out)
    undef0 = {f"s{k}" for k in range(npreload, 106)} | {"vcc"}
    IN = [None] * len(blocks)
    IN[0] = set(undef0)
    work = [0]
    OUT = [None] * len(blocks)
    while work:
        b = work.pop()
        st = set(IN[b])
        s, e = blocks[b]
        for _, t, _ in ins_list[s:e]:
            d, src = _dests_and_srcs(t)
            if d:
                if src & st:
                    st |= d
                else:
                    st -= d
        OUT[b] = st
        for n in succ[b]:
            new = st if IN[n] is None else (IN[n] | st)
            if IN[n] is None or new != IN[n]:
                IN[n] = new
                work.append(n)
    hits = []
    for b, (s, e) in enumerate(blocks):
        if IN[b] is None:
            continue  # unreachable
        st = set(IN[b])
        for a, t, _ in ins_list[s:e]:
            regs = _store_addr_regs(t)
            if regs is not None and regs & st:
                hits.append((a, t, sorted(regs & st)))
            d, src = _dests_and_srcs(t)
            if d:
                if src & st:
                    st |= d
                else:
                    st -= d
    return hits


def kernel_preloads(path):
    """{kernel name: SGPRs the hardware preloads} from the kernel descriptors (<name>.kd
    symbols) of a gfx950 code object: user SGPRs + workgroup id x / y / z + workgroup info +
    private segment wave offset (COMPUTE_PGM_RSRC2, the AMDHSA kernel descriptor at +52)."""
    data = open(path, "rb").read()
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", data, shoff + i * shentsize) for i in range(shnum)]
    out = {}
    for sec in secs:
        if sec[1] != 2:  # SHT_SYMTAB
            continue
        strtab = secs[sec[6]]
        for k in range(sec[5] // 24):
            name_off, info, other, shndx, value, size = struct.unpack_from("<IBBHQQ", data, sec[4] + k * 24)
            end = data.index(b"\0", strtab[4] + name_off)
            name = data[strtab[4] + name_off:end].decode()
            if not name.endswith(".kd") or shndx == 0 or shndx >= len(secs):
                continue
            tsec = secs[shndx]
            rsrc2, = struct.unpack_from("<I", data, tsec[4] + (value - tsec[3]) + 52)
            n = ((rsrc2 >> 1) & 31) + sum((rsrc2 >> b) & 1 for b in (7, 8, 9, 10)) + (rsrc2 & 1)
            out[name[:-3]] = n
    return out


def scan_code_object(path, objdump):
    """Rule 2 over one gfx950 code object: [(kernel, address, store, undefined regs)], and the
    number of stores examined."""
    import subprocess
    pre = kernel_preloads(path)
    dis = subprocess.run([objdump, "-d", "--mcpu=gfx950", path], capture_output=True, text=True, check=True).stdout
    hits, stores = [], 0
    for name, (_, ins) in parse_functions(dis.splitlines()).items():
        if name not in pre:
            continue  # not a kernel entry
        stores += sum(_store_addr_regs(t) is not None for _, t, _ in ins)
        hits += [(name, a, t, r) for a, t, r in undefined_address_stores(ins, pre[name])]
    return hits, stores
