#!/usr/bin/env python3
"""Build the REFERENCE weather-sim CPU solver into oracle/_ref/ (test infrastructure).

Recipe (SURVEY.md §8(c) "Verified oracle recipe"):

* Sources are read from /root/reference/src/weather-sim/cpp (read-only) and copied into a
  scratch directory under /tmp -- never into this repository.
* The reference does not compile as shipped. We apply only the
  mechanical compile fixes below, each asserted to match exactly once. None changes
  arithmetic:
    1. weather_sim.hpp:397 declares `index_t height_` next to `ScalarField2D height_`
       (:404). Rename the grid-dimension member to `height_dim_` (and its uses in
       weather_sim.hpp:285 and weather_grid.cpp ctors / diagnostics / swap).
    2. initial_conditions.hpp uses std::map (:62) without `#include <map>`.
    3. weather_simulation.cpp:315-317 (RK2, PE branch) uses `current_temp`,
       `tendency_temp`, `current_pressure`, `tendency_pressure` out of scope; re-declare
       them in that block exactly as :264-270 does.
    fp64 variant only:
    4. weather_sim.hpp:24 `using scalar_t = float;` -> `double`.
    5. initial_conditions.cpp:227-228 `std::max(r, 1.0e-6f)` is ambiguous for double;
       use `std::max<scalar_t>`.
* Only weather_grid.cpp, weather_simulation.cpp and initial_conditions.cpp are compiled
  (the hot path and its input generator). gpu_adaptability.cpp is NOT compiled and no
  stub is written for it: its entry points are reached only when compute_backend is
  CUDA/Hybrid/Adaptive (weather_simulation.cpp:492,564,570); the driver uses the CPU
  backend, so those calls are never made and stay unresolved, lazily bound.
* Flags follow the reference's Release build (build.sh:40): -O3 -fopenmp -std=c++17,
  no -march=native, no fast-math.

Outputs: oracle/_ref/ws_ref_f32, oracle/_ref/ws_ref_f64 (git-ignored; they travel to the
GPU box with the snapshot, where /root/reference does not exist).
"""
import os
import shutil
import subprocess
import sys
import tempfile

REF = "/root/reference/src/weather-sim/cpp"
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(os.path.dirname(HERE), "_ref")

COMMON_PATCHES = [
    ("include/weather_sim/weather_sim.hpp",
     "    index_t height_;      // Grid height", "    index_t height_dim_;  // Grid height"),
    ("include/weather_sim/weather_sim.hpp",
     "index_t getHeight() const { return height_; }", "index_t getHeight() const { return height_dim_; }"),
    ("src/weather_grid.cpp", "      height_(height), ", "      height_dim_(height), "),
    ("src/weather_grid.cpp", "      height_(config.grid_height),", "      height_dim_(config.grid_height),"),
    ("src/weather_grid.cpp", "for (index_t y = 0; y < height_; ++y) {", "for (index_t y = 0; y < height_dim_; ++y) {"),
    ("src/weather_grid.cpp", "std::min(height_ - 1, y + 1)", "std::min(height_dim_ - 1, y + 1)"),
    ("src/weather_grid.cpp", "height_ != other.height_", "height_dim_ != other.height_dim_"),
    ("include/weather_sim/initial_conditions.hpp", "#include <functional>\n", "#include <functional>\n#include <map>\n"),
    ("src/weather_simulation.cpp",
     "        auto& next_temp = next_grid_->getTemperatureField();\n"
     "        auto& next_pressure = next_grid_->getPressureField();\n"
     "        \n"
     "        for (index_t i = 0; i < current_temp.data.size(); ++i) {\n"
     "            next_temp.data[i] = current_temp.data[i] + dt_ * tendency_temp.data[i];",
     "        auto& next_temp = next_grid_->getTemperatureField();\n"
     "        auto& next_pressure = next_grid_->getPressureField();\n"
     "        auto& current_temp = current_grid_->getTemperatureField();\n"
     "        auto& tendency_temp = tendency_grid_->getTemperatureField();\n"
     "        auto& current_pressure = current_grid_->getPressureField();\n"
     "        auto& tendency_pressure = tendency_grid_->getPressureField();\n"
     "        \n"
     "        for (index_t i = 0; i < current_temp.data.size(); ++i) {\n"
     "            next_temp.data[i] = current_temp.data[i] + dt_ * tendency_temp.data[i];"),
]
# multi-occurrence patches: (file, old, new, expected count)
MULTI = [
    ("src/weather_grid.cpp", "for (index_t y = 0; y < height_; ++y) {", 2),
    ("src/weather_grid.cpp", "std::min(height_ - 1, y + 1)", 2),
]
FP64_PATCHES = [
    ("include/weather_sim/weather_sim.hpp", "using scalar_t = float;", "using scalar_t = double;"),
    ("src/initial_conditions.cpp", "std::max(r, 1.0e-6f)", "std::max<scalar_t>(r, 1.0e-6f)"),
]
MULTI_FP64 = {("src/initial_conditions.cpp", "std::max(r, 1.0e-6f)"): 2}


def apply(root, patches, multi):
    for rel, old, new in patches:
        p = os.path.join(root, rel)
        s = open(p).read()
        want = multi.get((rel, old), 1)
        got = s.count(old)
        if got != want:
            raise SystemExit(f"patch mismatch in {rel}: {old!r} found {got}x, expected {want}")
        open(p, "w").write(s.replace(old, new))


def build(variant):
    if not os.path.isdir(REF):
        raise SystemExit(f"{REF} not present: the reference build runs only in the survey container")
    os.makedirs(OUT, exist_ok=True)
    with tempfile.TemporaryDirectory(prefix="ws_ref_", dir="/tmp") as tmp:
        for d in ("include", "src"):
            shutil.copytree(os.path.join(REF, d), os.path.join(tmp, d))
        multi = {(f, o): n for f, o, n in MULTI}
        apply(tmp, COMMON_PATCHES, multi)
        if variant == "f64":
            apply(tmp, FP64_PATCHES, MULTI_FP64)
        lib = os.path.join(OUT, f"libws_ref_{variant}.so")
        exe = os.path.join(OUT, f"ws_ref_{variant}")
        flags = ["g++", "-std=c++17", "-O3", "-DNDEBUG", "-fopenmp", "-w", "-I", os.path.join(tmp, "include")]
        # the reference TUs as a shared library: undefined (never-called) gpu_adaptability
        # functions stay lazily-bound PLT entries
        subprocess.check_call(flags + ["-shared", "-fPIC",
                               os.path.join(tmp, "src", "weather_grid.cpp"),
                               os.path.join(tmp, "src", "weather_simulation.cpp"),
                               os.path.join(tmp, "src", "initial_conditions.cpp"),
                               "-o", lib, "-Wl,-z,lazy"])
        subprocess.check_call(flags + [os.path.join(HERE, "ref_driver.cpp"), "-o", exe,
                               "-L", OUT, f"-lws_ref_{variant}", "-Wl,-rpath,$ORIGIN",
                               "-Wl,--allow-shlib-undefined", "-Wl,-z,lazy"])
        return exe


if __name__ == "__main__":
    variants = sys.argv[1:] or ["f32", "f64"]
    for v in variants:
        print(build(v))
