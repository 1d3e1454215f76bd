"""CPU tests over the BUILT device code (tools/debug/store_hazard_scan.py):

Rule 1: no >8-byte store in libws_hip.so is followed directly by a VALU write of its data
VGPRs (the hazard that corrupted fused_x2y pair stores at large grids; see ws_fused_dev.h
buf_store_nt). Extracts the gfx950 code objects with llvm-objdump --offloading and
disassembles them.

Rule 2 (round 5): no store's address may be undefined on some path -- derived from a register
the compiler marked `implicit-def` (the bvort RK4 fp64 fault of rounds 2-3: a store switch
lowered with an undefined SGPR pointer). Checked on the gfx950 assembly the
library was built from (the Makefile's -save-temps=obj), against the round-3 assembly as a
fixture (tests/fixtures/bvort_r3_rowregs_stage_f64.s: must be caught)."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools", "debug"))
from store_hazard_scan import scan, scan_asm  # noqa: E402

LIB = os.path.join(ROOT, "nvidia-jetson-workload_amd", "lib", "libws_hip.so")
OBJ = os.path.join(ROOT, "nvidia-jetson-workload_amd", "csrc", "_obj")
FIXTURE = os.path.join(ROOT, "tests", "fixtures", "bvort_r3_rowregs_stage_f64.s")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def test_scanner_flags_the_hazard():
    bad = ["buffer_store_dwordx4 v[0:3], v194, s[56:59], s10 offen nt", "v_add_u32_e32 v0, s8, v229"]
    ok = ["buffer_store_dwordx4 v[0:3], v194, s[56:59], 0 offen nt", "s_nop 0", "v_add_u32_e32 v0, s8, v229"]
    other = ["buffer_store_dwordx4 v[0:3], v194, s[56:59], s10 offen nt", "v_add_u32_e32 v4, s8, v229"]
    assert len(scan(bad)) == 1 and not scan(ok) and not scan(other)
    # global stores: vaddr first, vdata second (rewriting the address is no data hazard)
    gbad = ["global_store_dwordx4 v[0:1], v[12:15], off nt", "v_mov_b32_e32 v13, 0"]
    gaddr = ["global_store_dwordx4 v[0:1], v[12:15], off nt", "v_lshl_add_u64 v[0:1], s[14:15], 0, v[16:17]"]
    assert len(scan(gbad)) == 1 and not scan(gaddr)


@pytest.mark.skipif(not (os.path.exists(LIB) and os.path.exists(OBJDUMP)), reason="library or llvm-objdump absent")
def test_built_library_has_no_store_data_hazard(tmp_path):
    lib = tmp_path / "libws_hip.so"
    shutil.copy(LIB, lib)
    subprocess.run([OBJDUMP, "--offloading", str(lib)], cwd=tmp_path, check=True, capture_output=True)
    objs = sorted(p for p in tmp_path.iterdir() if "gfx950" in p.name)
    assert objs, "no gfx950 code object in the library"
    stores, hits = 0, []
    for p in objs:
        out = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", str(p)], capture_output=True, text=True, check=True)
        lines = out.stdout.splitlines()
        stores += sum("_store_dwordx4" in l for l in lines)
        hits += [(p.name, *h) for h in scan(lines)]
    assert stores > 0, "disassembly parsed no 16-byte stores"
    assert not hits, hits[:5]


def test_rule2_catches_the_round3_store_switch():
    """The round-3 bv_stage_kernel<double> (-DWS_BV_ROWREGS): its epilogue stores go through
    v[..] = lshl_add(index, 3, s[8:9]) with s[8:9] implicit-def on one edge."""
    with open(FIXTURE) as f:
        hits, stores = scan_asm(f.read().splitlines())
    assert stores == 13
    assert len(hits) == 4, hits
    assert all("global_store" in t for _, t, _ in hits)


def test_rule2_dataflow_basics():
    k = ["\t.globl\tk", "k:", "\ts_load_dwordx2 s[4:5], s[0:1], 0x0"]
    ok = k + ["\tv_lshl_add_u64 v[2:3], v[0:1], 3, s[4:5]", "\tglobal_store_dwordx2 v[2:3], v[6:7], off"]
    # an implicit-def of the base on a path that joins the store's block
    bad = k + ["\ts_cbranch_scc1 .LBB0_2", "; %bb.1:", "\t; implicit-def: $sgpr4_sgpr5", ".LBB0_2:",
               "\tv_lshl_add_u64 v[2:3], v[0:1], 3, s[4:5]", "\tglobal_store_dwordx2 v[2:3], v[6:7], off"]
    # redefined on every path before the store: clean
    redef = bad[:-2] + ["\ts_mov_b64 s[4:5], s[0:1]", "\tv_lshl_add_u64 v[2:3], v[0:1], 3, s[4:5]",
                        "\tglobal_store_dwordx2 v[2:3], v[6:7], off"]
    # undefined DATA (not the address) is not this hazard
    data = k + ["\t; implicit-def: $sgpr6_sgpr7", "\tv_mov_b64 v[6:7], s[6:7]", "\tglobal_store_dwordx2 v[2:3], v[6:7], off"]
    # a VGPR address merged from the two exec-masked arms of a divergent if / else (the
    # compiler's implicit-def of the VGPR phi): no lane reaches the store without a value
    vmerge = k + ["\t; implicit-def: $vgpr2_vgpr3", "\ts_and_saveexec_b64 s[8:9], vcc", "\ts_cbranch_execz .LBB0_2",
                  "; %bb.1:", "\tv_mov_b64 v[2:3], s[4:5]", ".LBB0_2:", "\tglobal_store_dwordx2 v[2:3], v[6:7], off"]
    assert scan_asm(ok)[0] == [] and scan_asm(redef)[0] == [] and scan_asm(data)[0] == [] and scan_asm(vmerge)[0] == []
    assert len(scan_asm(bad)[0]) == 1


def _built_asm():
    if not os.path.isdir(OBJ):
        return []
    return sorted(os.path.join(OBJ, f) for f in os.listdir(OBJ) if f.endswith("-hip-amdgcn-amd-amdhsa-gfx950.s"))


@pytest.mark.skipif(not os.path.exists(LIB), reason="library not built")
def test_built_library_has_no_undefined_store_address():
    files = _built_asm()
    assert len(files) >= 20, "no gfx950 assembly next to the objects: build with the Makefile (-save-temps=obj)"
    lib_t = os.path.getmtime(LIB)
    stale = [os.path.basename(f) for f in files if os.path.getmtime(f) > lib_t + 1]
    assert not stale, f"assembly newer than the library (rebuild it): {stale[:3]}"
    from concurrent.futures import ProcessPoolExecutor
    total, hits = 0, []
    with ProcessPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        for f, (h, n) in zip(files, ex.map(_scan_file, files)):
            total += n
            hits += [(os.path.basename(f), *x) for x in h]
    assert total > 1000, "parsed almost no stores"
    assert not hits, hits[:5]


def _scan_file(path):
    with open(path) as fh:
        return scan_asm(fh.read().splitlines())
