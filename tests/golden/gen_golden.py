#!/usr/bin/env python3
"""Generate golden fixtures from the REFERENCE solver (run only in the survey container).

The reference binaries are built by oracle/ref/build_ref.py from /root/reference sources
(compile-fixed in /tmp, never copied here). This script drives them through their public
C++ API (WeatherSimulation / WeatherGrid / InitialCondition, exactly what pyweather_sim
binds: python_bindings.cpp:240-353) and stores inputs and outputs as data:

  tests/golden/ref_small_f32.npz, ref_small_f64.npz
      48x32 (non-square) cases: every IC's initial fields (IC parity) and the state after
      1 / 10 / 50 steps for each (model, method, IC) case (stepping parity), incl. the
      vorticity diagnostic, plus API-behaviour cases (max_time cap, run_until step count,
      p/T/q alternation, PE T/P drift, stale grid handle, set_dt).
  tests/golden/ref_large.json
      SHA-256 digests + L2 norms of the reference outputs for full-size configs
      (C1 256^2 dam-break 1000 steps; C2-shape 4096^2 fp64 RK4; C3 2048^2 Barotropic;
      C4 per-level 1024^2 PE levels), used by the GPU parity tests at full size.

  --long: only the long-horizon pin of the benched workload (C2 jet_stream 4096^2 fp64 RK4,
      LONG_STEPS steps), merged into ref_large.json.

Usage: python tests/golden/gen_golden.py [--skip-large | --long]
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF = os.path.join(ROOT, "oracle", "_ref")
OUT = os.path.dirname(os.path.abspath(__file__))
FIELDS = ("u", "v", "h", "p", "t", "q", "vort")

# enum values (weather_sim.hpp:30-56)
SWE, BARO, PE, GCM = 0, 1, 2, 3
EULER, RK2, RK4, AB, SEMI = 0, 1, 2, 3, 4

SW, SH = 48, 32  # small non-square grid


def read_snap(path):
    b = open(path, "rb").read()
    hdr = np.frombuffer(b[:16], np.int32)
    assert hdr[0] == 0x57534731
    W, H, sz = int(hdr[1]), int(hdr[2]), int(hdr[3])
    step = int(np.frombuffer(b[16:20], np.int32)[0])
    t = float(np.frombuffer(b[20:28], np.float64)[0])
    dt = np.float32 if sz == 4 else np.float64
    arr = np.frombuffer(b[28:], dt).reshape(7, H, W)
    return {"step": step, "time": t, **{f: arr[i].copy() for i, f in enumerate(FIELDS)}}


def run_spec(variant, lines, tmp):
    spec = os.path.join(tmp, "spec.txt")
    with open(spec, "w") as f:
        f.write("\n".join(lines) + "\n")
    r = subprocess.run([os.path.join(REF, f"ws_ref_{variant}"), spec], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(r.stderr)
    return r.stdout


def cfg_lines(W, H, model=SWE, method=RK4, dt=None, dx=None, dy=None, g=None, f=None, max_time=None):
    L = [f"cfg width {W}", f"cfg height {H}", f"cfg model {model}", f"cfg method {method}"]
    for k, v in (("dt", dt), ("dx", dx), ("dy", dy), ("gravity", g), ("coriolis_f", f), ("max_time", max_time)):
        if v is not None:
            L.append(f"cfg {k} {v!r}")
    return L


def dam_break(W, H, width_cells, dtype):
    """Smooth dam-break height: h = 10 + 0.5*(1 - tanh((x - W/2)/w))."""
    x = np.arange(W, dtype=np.float64)
    row = 10.0 + 0.5 * (1.0 - np.tanh((x - W / 2) / width_cells))
    return np.broadcast_to(row, (H, W)).astype(dtype)


# IC name -> constructor args (the Python wrapper's defaults, weather_simulation.py:388-447)
ICS = {
    "uniform": [], "zonal_flow": [], "vortex": [], "jet_stream": [], "breaking_wave": [],
    "front": [], "mountain": [], "random": ["42", "1.0"],
    "atmospheric_profile": ["standard"], "atmospheric_profile_tropical": ["tropical"],
    "atmospheric_profile_polar": ["polar"],
    "jet_stream_custom": ["0.3", "0.07", "13.5", "9.75"],
    "vortex_custom": ["0.4", "0.6", "0.2", "5.0", "11.0"],
}


def ic_line(name):
    base = name.replace("_tropical", "").replace("_polar", "").replace("_custom", "")
    return f"ic {base} " + " ".join(ICS[name])


def small_cases(variant, tmp):
    dtype = np.float32 if variant == "f32" else np.float64
    data, meta = {}, {}

    def put(case, snapname, snap):
        for k in FIELDS:
            data[f"{case}/{snapname}/{k}"] = snap[k]
        meta.setdefault(case, {})[snapname] = {"step": snap["step"], "time": snap["time"]}

    # 1) IC parity: every IC on a standalone-equivalent fresh grid (initialize() applies it)
    for name in ICS:
        lines = cfg_lines(SW, SH) + ["create", ic_line(name), "initialize", f"snap {tmp}/s.bin"]
        run_spec(variant, lines, tmp)
        put(f"ic/{name}", "s0", read_snap(f"{tmp}/s.bin"))
    # IC at a second (odd) size, exercising the (W-1)/(H-1) normalisations
    for name in ("zonal_flow", "vortex", "jet_stream", "breaking_wave", "mountain", "atmospheric_profile", "front"):
        lines = cfg_lines(37, 53) + ["create", ic_line(name), "initialize", f"snap {tmp}/s.bin"]
        run_spec(variant, lines, tmp)
        put(f"ic37x53/{name}", "s0", read_snap(f"{tmp}/s.bin"))

    # 2) stepping parity: (model, method, IC, extra cfg)
    cases = []
    for ic in ("jet_stream", "zonal_flow", "breaking_wave", "mountain", "dam_break"):
        for method in (EULER, RK2, RK4):
            cases.append((SWE, method, ic, {}))
    cases += [
        (BARO, RK4, "zonal_flow", {}), (BARO, EULER, "breaking_wave", {}),
        (PE, EULER, "jet_stream", {}), (PE, RK2, "front", {}), (PE, RK4, "atmospheric_profile", {}),
        (GCM, RK4, "mountain", {}), (SWE, AB, "breaking_wave", {}), (SWE, SEMI, "jet_stream", {}),
        (SWE, RK4, "breaking_wave", {"dx": 0.75, "dy": 1.3, "f": 1.0e-2, "g": 9.5, "dt": 0.005}),
        (SWE, EULER, "mountain", {"dx": 2.0, "dy": 0.5, "f": 0.5}),
        (SWE, RK2, "vortex_custom", {"dx": 3.0, "dy": 3.0}),
    ]
    for model, method, ic, kw in cases:
        case = f"step/m{model}_i{method}_{ic}" + ("".join(f"_{k}{v}" for k, v in sorted(kw.items())))
        meta.setdefault(case, {})["cfg"] = dict(width=SW, height=SH, model=model, method=method, **kw)
        lines = cfg_lines(SW, SH, model, method, **kw) + ["create"]
        if ic == "dam_break":
            dam_break(SW, SH, 4.0, dtype).tofile(f"{tmp}/h.bin")
            lines += ["initialize", f"setfield h {tmp}/h.bin"]
        else:
            lines += [ic_line(ic), "initialize"]
        lines += [f"snap {tmp}/s0.bin", "step 1", f"snap {tmp}/s1.bin", "run 9", f"snap {tmp}/s10.bin",
                  "run 40", f"snap {tmp}/s50.bin"]
        run_spec(variant, lines, tmp)
        for s in ("s0", "s1", "s10", "s50"):
            put(case, s, read_snap(f"{tmp}/{s}.bin"))

    # 3) API-behaviour cases
    # max_time cap: run(2000) with default max_time=10, dt=0.01 stops after 1000 steps
    lines = cfg_lines(16, 12, SWE, EULER) + ["create", ic_line("jet_stream"), "initialize", "run 2000",
                                             f"snap {tmp}/a.bin"]
    run_spec(variant, lines, tmp)
    put("api/max_time_cap", "end", read_snap(f"{tmp}/a.bin"))
    # run_until(0.5) at dt=0.1 -> int(0.5/0.1)+1 steps; then run_until(0.55) -> 0 steps
    lines = cfg_lines(16, 12, SWE, RK2, dt=0.1) + ["create", ic_line("zonal_flow"), "initialize", "run_until 0.5",
                                                   f"snap {tmp}/a.bin", "run_until 0.55", f"snap {tmp}/b.bin",
                                                   "run_until 1.25", f"snap {tmp}/c.bin"]
    run_spec(variant, lines, tmp)
    put("api/run_until", "a", read_snap(f"{tmp}/a.bin"))
    put("api/run_until", "b", read_snap(f"{tmp}/b.bin"))
    put("api/run_until", "c", read_snap(f"{tmp}/c.bin"))
    # p/T/q alternation for SWE; T/P drift + q alternation for PE (IC sets p,T,q)
    for model in (SWE, PE):
        lines = cfg_lines(16, 12, model, EULER) + ["create", "ic uniform 1.0 0.5 10.0 1000.0 300.0 0.25", "initialize",
                                                   "step 1", f"snap {tmp}/a.bin", "step 1", f"snap {tmp}/b.bin",
                                                   "step 1", f"snap {tmp}/c.bin"]
        run_spec(variant, lines, tmp)
        for s in "abc":
            put(f"api/alternation_m{model}", s, read_snap(f"{tmp}/{s}.bin"))
    # stale handle: grid held before a step shows the previous state afterwards
    lines = cfg_lines(16, 12, SWE, RK4) + ["create", ic_line("breaking_wave"), "initialize", "step 2", "hold",
                                           f"snap {tmp}/a.bin", "step 1", f"snap_held {tmp}/b.bin",
                                           f"snap {tmp}/c.bin", "step 1", f"snap_held {tmp}/d.bin"]
    run_spec(variant, lines, tmp)
    for s in "abcd":
        put("api/stale_handle", s, read_snap(f"{tmp}/{s}.bin"))
    # set_dt mid-run
    lines = cfg_lines(16, 12, SWE, RK4) + ["create", ic_line("jet_stream"), "initialize", "step 3", "set_dt 0.02",
                                           "step 4", f"snap {tmp}/a.bin"]
    run_spec(variant, lines, tmp)
    put("api/set_dt", "a", read_snap(f"{tmp}/a.bin"))
    # re-initialize after stepping (current grid reset + IC again; next grid keeps old data)
    lines = cfg_lines(16, 12, SWE, EULER) + ["create", "ic uniform 1.0 0.5 10.0 1000.0 300.0 0.25", "initialize",
                                             "step 3", "initialize", "step 1", f"snap {tmp}/a.bin",
                                             "step 1", f"snap {tmp}/b.bin"]
    run_spec(variant, lines, tmp)
    put("api/reinit", "a", read_snap(f"{tmp}/a.bin"))
    put("api/reinit", "b", read_snap(f"{tmp}/b.bin"))
    return data, meta


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def large_cases(tmp):
    out = {}

    def record(name, variant, lines, fields=("u", "v", "h", "vort")):
        run_spec(variant, lines, tmp)
        s = read_snap(f"{tmp}/L.bin")
        out[name] = {"variant": variant, "step": s["step"], "time": s["time"],
                     "sha256": {k: digest(s[k]) for k in fields},
                     "l2": {k: float(np.linalg.norm(s[k].astype(np.float64))) for k in fields},
                     "spec": [l for l in lines if not l.startswith(("snap", "setfield"))]}
        print(name, out[name]["step"], out[name]["time"], flush=True)

    # C1: 256^2 smooth dam-break, CPU config, Euler and RK4, 1000 steps (max_time lifted)
    for method in (EULER, RK4):
        dam_break(256, 256, 8.0, np.float32).tofile(f"{tmp}/h.bin")
        lines = cfg_lines(256, 256, SWE, method, max_time=1e30) + ["create", "initialize",
                                                                  f"setfield h {tmp}/h.bin", "run 1000",
                                                                  f"snap {tmp}/L.bin"]
        record(f"C1_dam_break_256_i{method}_f32", "f32", lines)
    # C2 shape: 4096^2 fp64, smooth dam-break (width 128) and jet_stream, RK4 and Euler, 5 steps
    dam_break(4096, 4096, 128.0, np.float64).tofile(f"{tmp}/h64.bin")
    for method in (RK4, EULER):
        lines = cfg_lines(4096, 4096, SWE, method, max_time=1e30) + ["create", "initialize",
                                                                    f"setfield h {tmp}/h64.bin", "run 5",
                                                                    f"snap {tmp}/L.bin"]
        record(f"C2_dam_break_4096_i{method}_f64", "f64", lines)
    lines = cfg_lines(4096, 4096, SWE, RK4, max_time=1e30) + ["create", ic_line("jet_stream"), "initialize",
                                                             "run 5", f"snap {tmp}/L.bin"]
    record("C2_jet_stream_4096_i2_f64", "f64", lines)
    # C3: 2048^2 fp32 Barotropic (RK4 -> RK2), zonal_flow, 20 steps
    lines = cfg_lines(2048, 2048, BARO, RK4, max_time=1e30) + ["create", ic_line("zonal_flow"), "initialize",
                                                              "run 20", f"snap {tmp}/L.bin"]
    record("C3_zonal_flow_2048_baro_f32", "f32", lines)
    # C4: PE 1024^2, per-level jet_stream strength 10*(1+k/32); levels 0, 7, 31 (10 steps)
    for k in (0, 7, 31):
        strength = 10.0 * (1.0 + k / 32.0)
        lines = cfg_lines(1024, 1024, PE, RK4, max_time=1e30) + [
            "create", f"ic jet_stream 0.5 0.1 {strength!r} 10.0", "initialize", "run 10", f"snap {tmp}/L.bin"]
        record(f"C4_pe_1024_level{k}_f32", "f32", lines, fields=("u", "v", "h", "p", "t", "vort"))
    return out


LONG_STEPS = 240  # 40 six-step slab blocks, 120 two-step launches


def long_case(tmp):
    """The benched workload (bench.py c2: jet_stream, RK4, fp64) after LONG_STEPS steps."""
    out = {}
    lines = cfg_lines(4096, 4096, SWE, RK4, max_time=1e30) + ["create", ic_line("jet_stream"), "initialize",
                                                             f"run {LONG_STEPS}", f"snap {tmp}/L.bin"]
    run_spec("f64", lines, tmp)
    s = read_snap(f"{tmp}/L.bin")
    name = f"C2_jet_stream_4096_i2_f64_{LONG_STEPS}"
    fields = ("u", "v", "h", "vort")
    out[name] = {"variant": "f64", "step": s["step"], "time": s["time"],
                 "sha256": {k: digest(s[k]) for k in fields},
                 "l2": {k: float(np.linalg.norm(s[k].astype(np.float64))) for k in fields},
                 "spec": [l for l in lines if not l.startswith(("snap", "setfield"))]}
    print(name, out[name]["step"], out[name]["time"], flush=True)
    return out


def main():
    skip_large = "--skip-large" in sys.argv
    if "--long" in sys.argv:
        path = os.path.join(OUT, "ref_large.json")
        with open(path) as f:
            large = json.load(f)
        with tempfile.TemporaryDirectory(prefix="ws_gold_", dir="/tmp") as tmp:
            large.update(long_case(tmp))
        with open(path, "w") as f:
            json.dump(large, f, indent=1, sort_keys=True)
        return
    with tempfile.TemporaryDirectory(prefix="ws_gold_", dir="/tmp") as tmp:
        for variant in ("f32", "f64"):
            data, meta = small_cases(variant, tmp)
            data["__meta__"] = np.frombuffer(json.dumps(meta).encode(), np.uint8)
            np.savez_compressed(os.path.join(OUT, f"ref_small_{variant}.npz"), **data)
            print(variant, len(data), "arrays")
        if not skip_large:
            large = large_cases(tmp)
            with open(os.path.join(OUT, "ref_large.json"), "w") as f:
                json.dump(large, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
