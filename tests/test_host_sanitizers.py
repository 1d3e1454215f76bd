"""ASan + UBSan over the library's host code (SURVEY §5's sanitizer build; GPU sanitizers are
not used): tools/sanitize/host_sanitize.sh rebuilds ws_runtime.cpp, ws_initial_conditions.cpp
and ws_comm.cpp with host-side -fsanitize=address,undefined (no recovery), links them with the
normal device objects, and runs tools/sanitize/abi_host_check.c -- the slab partition, the halo
exchange plan over many shapes, argument validation and the no-device error paths of the C
ABI (the no-device paths where no GPU is visible)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJ = os.path.join(ROOT, "nvidia-jetson-workload_amd", "csrc", "_obj")


@pytest.mark.skipif(not (shutil.which("/opt/rocm/bin/hipcc") and os.path.isdir(OBJ)),
                    reason="needs hipcc and the library's built objects")
def test_host_code_under_asan_and_ubsan(tmp_path):
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "sanitize", "host_sanitize.sh")],
                       env=dict(os.environ, OUT=str(tmp_path)), capture_output=True, text=True, timeout=900)
    assert r.returncode == 0 and "host sanitizer check ok" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]
