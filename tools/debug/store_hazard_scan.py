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
# edge; the store's 64-bit VGPR address was then computed from that pair, and the store wrote
# through whatever the SGPRs still held. No source-level index was out of range, and in the
# code object nothing shows it (the SGPRs hold a stale, valid-looking value). The compiler's
# assembly keeps the fact as `; implicit-def: $sgpr8_sgpr9` comments, so the rule runs on the
# gfx950 assembly the library was built from (the Makefile keeps it: -save-temps=obj, which
# leaves the instruction stream bit-identical), by a forward may-be-undefined analysis over
# each kernel's control-flow graph:
#   * an SGPR implicit-def makes its registers undefined from that point (SGPRs are
#     wave-uniform: the undefined edge is a path the whole wave takes; VGPR implicit-defs are
#     the exec-masked arms of divergent if / else and are not followed);
#   * an instruction's destinations become undefined iff one of its register sources is
#     (and defined again when all its sources are defined);
#   * at a join a register is undefined if it is on ANY incoming path;
#   * a global / buffer / flat store (or atomic) whose address operands (vaddr, saddr,
#     srsrc, soffset) may be undefined is reported.
# ---------------------------------------------------------------------------------------
_REG = re.compile(r"^(?:(?P<k>[sv])(?P<n>\d+)|(?P<kk>[sv])\[(?P<a>\d+):(?P<b>\d+)\]|(?P<sp>vcc|vcc_lo|vcc_hi))$")
_NO_DEST = re.compile(r"^(s_cmp|s_bitcmp|s_cbranch|s_branch|s_waitcnt|s_nop|s_endpgm|s_barrier|s_setprio|s_sleep|"
                      r"s_sendmsg|s_setreg|s_set_gpr_idx|s_trap|s_icache|s_dcache|s_ttrace|s_wait|s_delay|s_sethalt|"
                      r"s_setkill|s_code_end|s_incperflevel|s_decperflevel|s_sched|"
                      r"buffer_store|global_store|flat_store|scratch_store|ds_write|ds_store|exp\b|"
                      r"buffer_wbl2|buffer_inv|buffer_wbinvl1|s_store|s_scratch_store|s_buffer_store)")
_MIR = re.compile(r"\$(sgpr|vgpr)(\d+)")


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


def _operands(rest):
    return [o.strip().split()[0] for o in rest.split(",") if o.strip()]


def dests_and_srcs(ins):
    """(destination registers, source registers) of one instruction (text)."""
    op, _, rest = ins.partition(" ")
    toks = _operands(rest)
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
        srcs = set().union(*regs[2:])
    return dests, srcs


def store_addr_regs(ins):
    """Address registers of a global / buffer / flat store or atomic; None for other ops."""
    op, _, rest = ins.partition(" ")
    toks = _operands(rest)
    if op.startswith(("global_store", "global_atomic", "flat_store", "flat_atomic")):
        regs = set(_regset(toks[0])) if toks else set()
        if len(toks) > 2:
            regs |= _regset(toks[2])  # saddr (or 'off')
        return regs
    if op.startswith(("buffer_store", "buffer_atomic")):
        regs = set()
        for t in toks[1:4]:  # vaddr (or off), srsrc, soffset
            regs |= _regset(t)
        return regs
    return None


def parse_asm_kernels(lines):
    """{kernel: [item]} from compiler (-S) assembly; an item is ("label", name),
    ("undef", regs) for an implicit-def comment, or ("ins", text)."""
    kernels, cur = {}, None
    globl = set()
    for l in lines:
        st = l.strip()
        m = re.match(r"^\.globl\s+(\S+)", st)
        if m:
            globl.add(m.group(1))
            continue
        m = re.match(r"^([A-Za-z_.$][\w.$]*):", l)
        if m and not l.startswith("\t") and not l.startswith(" "):
            name = m.group(1)
            if name in globl and not name.startswith("."):
                cur = name
                kernels[cur] = []
                continue
            if cur is not None and name.startswith(".LBB"):
                kernels[cur].append(("label", name))
            continue
        if cur is None:
            continue
        if st.startswith("; %bb."):
            kernels[cur].append(("label", st[2:].split()[0]))  # fallthrough block
            continue
        if st.startswith("; implicit-def:"):
            # SGPRs only: an SGPR is wave-uniform, so "undefined on an edge" is a real path of
            # the whole wave (the round-3 store pointer). VGPR implicit-defs mark the two arms
            # of a divergent if / else writing one value (e.g. the 64-bit division expansion):
            # the exec-masked, structurized CFG has "neither arm" paths that no lane takes.
            regs = {"s" + n for k, n in _MIR.findall(st) if k == "sgpr"}
            if regs:
                kernels[cur].append(("undef", regs))
            continue
        if st.startswith(".Lfunc_end") or st.startswith(".size") or st.startswith("s_endpgm") and False:
            continue
        t = st.split(";")[0].strip()
        if not t or t.startswith(".") or t.endswith(":"):
            continue
        kernels[cur].append(("ins", t))
    return kernels


_IMM = re.compile(r"^-?(0x[0-9a-fA-F]+|\d+)$")


def _imm(tok):
    return int(tok, 0) if _IMM.match(tok) else None


def undefined_address_stores(items, max_contexts=8):
    """Stores of one kernel whose address may be undefined: [(item index, store, regs)].

    Path-sensitive in the one way the compiler's lowering needs: SGPRs set to constants
    (s_mov_b32 / s_mov_b64 of an immediate) are tracked per path, and a branch on vcc derived
    from such a constant mask (s_and[n2]_b64 vcc, exec, s[..]) follows only its feasible edge
    (exec assumed non-zero). That is how the compiler guards "defined on the other path":
    e.g. `s_mov_b64 s[2:3], -1; implicit-def s27; ... s_andn2_b64 vcc, exec, s[2:3];
    s_cbranch_vccnz` never reaches the use with s27 undefined. Up to max_contexts constant
    environments per block; beyond that they merge (constants that differ are dropped)."""
    blocks, labels, cur = [], {}, []
    for i, it in enumerate(items):
        if it[0] == "label":
            if cur:
                blocks.append(cur)
            cur = []
            labels[it[1]] = len(blocks)
            continue
        cur.append(i)
        if it[0] == "ins" and it[1].startswith(("s_branch", "s_cbranch", "s_endpgm", "s_setpc")):
            blocks.append(cur)
            cur = []
    if cur:
        blocks.append(cur)
    if not blocks:
        return []

    def step(taint, const, vcc, it):
        """Transfer one item; vcc: None unknown, 0 zero, 1 non-zero."""
        if it[0] == "undef":
            taint = taint | it[1]
            const = {k: v for k, v in const.items() if k not in it[1]}
            return taint, const, vcc
        if it[0] != "ins":
            return taint, const, vcc
        t = it[1]
        op, _, rest = t.partition(" ")
        toks = _operands(rest)
        d, src = dests_and_srcs(t)
        if d:
            taint = (taint | d) if (src & taint) else (taint - d)
            const = {k: v for k, v in const.items() if k not in d}
            if op in ("s_mov_b32", "s_mov_b64") and len(toks) == 2 and _imm(toks[1]) is not None:
                for r in d:
                    const[r] = _imm(toks[1])
            if "vcc" in d:
                vcc = None
                if op in ("s_and_b64", "s_andn2_b64") and len(toks) == 3 and toks[1] == "exec":
                    regs = sorted(_regset(toks[2]))
                    vals = [const.get(r) for r in regs]
                    if regs and all(v is not None for v in vals):
                        allone = all(v in (-1, 0xffffffff) for v in vals)
                        zero = all(v == 0 for v in vals)
                        if op == "s_and_b64":
                            vcc = 0 if zero else 1 if allone else None
                        else:
                            vcc = 0 if allone else 1 if zero else None
        return taint, const, vcc

    def successors(b, vcc):
        idx = blocks[b]
        last = items[idx[-1]] if idx else ("", "")
        out = []
        fall = b + 1 < len(blocks)
        if last[0] == "ins":
            op, _, rest = last[1].partition(" ")
            tgt = labels.get(rest.strip())
            if op.startswith("s_branch"):
                return [tgt] if tgt is not None else []
            if op.startswith(("s_endpgm", "s_setpc")):
                return []
            if op.startswith("s_cbranch") and tgt is not None:
                taken = fall_ok = True
                if op == "s_cbranch_vccnz" and vcc is not None:
                    taken, fall_ok = vcc == 1, vcc == 0
                elif op == "s_cbranch_vccz" and vcc is not None:
                    taken, fall_ok = vcc == 0, vcc == 1
                if taken:
                    out.append(tgt)
                if fall and fall_ok:
                    out.append(b + 1)
                return out
        return [b + 1] if fall else []

    # contexts per block: {frozenset(const items): taint}
    IN = [dict() for _ in blocks]
    IN[0][frozenset()] = frozenset()
    work = [(0, frozenset())]
    while work:
        b, key = work.pop()
        if key not in IN[b]:
            continue  # a context since merged into another (its work item is queued)
        taint, const, vcc = set(IN[b][key]), dict(key), None
        for i in blocks[b]:
            taint, const, vcc = step(taint, const, vcc, items[i])
        for n in successors(b, vcc):
            k2 = frozenset(const.items())
            ctx = IN[n]
            if k2 not in ctx and len(ctx) >= max_contexts:
                # merge everything into one context: keep only constants all contexts agree on
                common = None
                tall = set(taint)
                for kk, tt in ctx.items():
                    common = set(kk) if common is None else common & set(kk)
                    tall |= tt
                common = (common or set()) & set(k2)
                ctx.clear()
                ctx[frozenset(common)] = frozenset(tall)
                work.append((n, frozenset(common)))
                continue
            if k2 in ctx:
                merged = ctx[k2] | frozenset(taint)
                if merged == ctx[k2]:
                    continue
                ctx[k2] = merged
            else:
                # a key may have been collapsed by a merge: fold into the surviving context
                ctx[k2] = frozenset(taint)
            work.append((n, k2))
    hits, seen = [], set()
    for b, idx in enumerate(blocks):
        for key, t0 in IN[b].items():
            taint, const, vcc = set(t0), dict(key), None
            for i in idx:
                it = items[i]
                if it[0] == "ins" and i not in seen:
                    regs = store_addr_regs(it[1])
                    if regs is not None and regs & taint:
                        hits.append((i, it[1], sorted(regs & taint)))
                        seen.add(i)
                taint, const, vcc = step(taint, const, vcc, it)
    return hits


def scan_asm(lines):
    """Rule 2 over compiler assembly: ([(kernel, store, undefined regs)], stores examined)."""
    hits, stores = [], 0
    for name, items in parse_asm_kernels(lines).items():
        stores += sum(1 for it in items if it[0] == "ins" and store_addr_regs(it[1]) is not None)
        hits += [(name, t, r) for _, t, r in undefined_address_stores(items)]
    return hits, stores
