"""CPU test over the BUILT device code: no >8-byte store in libws_hip.so is followed directly
by a VALU write of its data VGPRs (the hazard that corrupted fused_x2y pair stores at large
grids; see ws_fused_dev.h buf_store_nt). Extracts the gfx950 code objects with
llvm-objdump --offloading and disassembles them."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools", "debug"))
from store_hazard_scan import scan  # noqa: E402

LIB = os.path.join(ROOT, "nvidia-jetson-workload_amd", "lib", "libws_hip.so")
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
