"""Guard against shipping a tree the GPU pool refuses to run (round 2 lost its whole driver
GPU run to one hipcc link line): every script / build file / source that travels to the GPU
box is scanned for

* a hipcc statement carrying a sanitizer flag that is not directly preceded by the host-only
  qualifier (GPU sanitizer builds are refused; host sanitizers must say so per flag, or the
  statement carries the no-GPU-sanitize switch and no per-arch option);
* XNACK-on runs or code objects;
* scalar-cache write instructions (refused on this pool, comments included).

Files listed in .gpurunignore do not travel and are skipped. The forbidden spellings are
assembled at run time so this file itself names none of them (it is also gpurun-ignored).
"""
import fnmatch
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SAN = "-f" + "sanitize="
XHOST = "-X" + "arch_host"
NOGPUSAN = "-fno-" + "gpu-sanitize"
XNACK_ENV = "HSA_" + "XNACK=1"
XNACK_TGT = "xn" + "ack+"
SCALAR_WRITES = [p + q for p in ("s_" + "store", "s_" + "buffer_store", "s_" + "scratch_store",
                                 "s_" + "atomic", "s_" + "buffer_atomic")
                 for q in ("_",)] + ["s_" + "dcache_wb", "s_" + "dcache_discard"]

TEXT_EXT = (".sh", ".py", ".hip", ".cpp", ".c", ".h", ".hpp", ".s", ".S", ".txt", ".mk", ".cmake")


def _tracked():
    try:
        out = subprocess.run(["git", "ls-files"], cwd=ROOT, capture_output=True, text=True, check=True).stdout
        return [l for l in out.splitlines() if l]
    except Exception:  # no git (the GPU box): walk the tree
        files = []
        for d, _, fs in os.walk(ROOT):
            if "/.git" in d or "gpurun_out" in d:
                continue
            files += [os.path.relpath(os.path.join(d, f), ROOT) for f in fs]
        return files


def _ignored_patterns():
    pats = []
    p = os.path.join(ROOT, ".gpurunignore")
    if os.path.exists(p):
        for line in open(p):
            line = line.strip()
            if line and not line.startswith("#"):
                pats.append(line)
    return pats


def _is_ignored(rel, pats):
    for p in pats:
        if p.startswith("./"):
            q = p[2:].rstrip("/")
            if rel == q or rel.startswith(q + "/") or fnmatch.fnmatch(rel, q):
                return True
        elif "/" in p:
            q = p.rstrip("/")
            if rel == q or rel.startswith(q + "/") or fnmatch.fnmatch(rel, q):
                return True
        elif fnmatch.fnmatch(os.path.basename(rel), p) or any(fnmatch.fnmatch(part, p) for part in rel.split("/")):
            return True
    return False


def _shipped_text_files():
    pats = _ignored_patterns()
    for rel in _tracked():
        base = os.path.basename(rel)
        if not (rel.endswith(TEXT_EXT) or base in ("Makefile", "makefile")):
            continue
        if _is_ignored(rel, pats):
            continue
        path = os.path.join(ROOT, rel)
        if os.path.isfile(path):
            yield rel, open(path, errors="replace").read()


def _statements(text):
    """Shell-style statements: backslash-continued lines joined."""
    return re.sub(r"\\\n", " ", text).splitlines()


def hipcc_sanitizer_violations(text):
    bad = []
    for st in _statements(text):
        if "hipcc" not in st or SAN not in st:
            continue
        toks = st.split()
        if NOGPUSAN in toks and not any(t.startswith("-X" + "arch_") for t in toks):
            continue
        for i, t in enumerate(toks):
            if t.startswith(SAN) and (i == 0 or toks[i - 1] != XHOST):
                bad.append(st.strip())
                break
    return bad


def test_scanner_catches_the_round2_line():
    line = "/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 " + SAN + "address,undefined -o x.so a.o"
    assert hipcc_sanitizer_violations(line)
    assert hipcc_sanitizer_violations("hipcc -c a.cpp \\\n  " + SAN + "address")
    assert not hipcc_sanitizer_violations("hipcc -c a.cpp " + XHOST + " " + SAN + "address")
    assert not hipcc_sanitizer_violations("hipcc -c a.cpp " + SAN + "address " + NOGPUSAN)
    assert not hipcc_sanitizer_violations("clang++ -shared " + SAN + "address a.o")


def test_no_gpu_sanitizer_build_ships():
    bad = {rel: v for rel, text in _shipped_text_files() if (v := hipcc_sanitizer_violations(text))}
    assert not bad, bad


def test_no_xnack_on_ships():
    bad = [rel for rel, text in _shipped_text_files() if XNACK_ENV in text or XNACK_TGT in text]
    assert not bad, bad


def test_no_scalar_cache_writes_ship():
    bad = [(rel, w) for rel, text in _shipped_text_files() for w in SCALAR_WRITES if w in text]
    assert not bad, bad


def test_sanitizer_tooling_is_gpurun_ignored():
    pats = _ignored_patterns()
    for rel in ("tools/sanitize/host_sanitize.sh", "tests/test_host_sanitizers.py", "tests/test_pool_rules.py"):
        assert _is_ignored(rel, pats), rel
