#!/usr/bin/env python3
"""Benchmark: cell-updates/s of the weather-sim time step on MI355X (BASELINE.json metric).

Default workload (BASELINE configs[1], "C2"): Shallow Water 4096 x 4096, fp64, RK4 (the
reference's default integrator, weather_sim.hpp:159), jet_stream initial condition,
inputs resident in HBM. One "step" = one full time step of the whole grid, all N ranks.

  python bench.py [--gpus N --steps K --warmup W] [--config c2|c3|c4|c5] [--method rk4|rk2|euler]

N > 1 (one process per GPU: launched by torch.distributed.run, or -- with no launcher --
bench.py starts torch.distributed.run with N ranks itself; a WORLD_SIZE other than --gpus is
an error, exit status 2): the same global grid is
y-slab decomposed over the ranks (strong scaling) and halo rows move over RCCL inside
libws_hip.so. Timing: barrier + torch.cuda.synchronize() on both sides of exactly K steps,
max over ranks. value = W*H*L*K / that time (whole job).

The JSON line also carries:
  roofline     dominant stage kernel: algorithmic bytes per launch / mean launch time
               (HIP events on the kernel's stream inside the timed region) vs 8 TB/s;
               traffic from profiles/traffic_<config>.json (rocprofv3 PMC) when present.
  cpu_baseline the reference CPU solver (oracle/_ref, compiled from /root/reference
               sources) or, if absent, the C oracle port, timed on host cores on a bounded
               sample of the same workload (rank 0, N = 1 only).
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "nvidia-jetson-workload_amd"))
sys.path.insert(0, ROOT)

METRIC = "cell-updates/sec + achieved HBM GB/s, SWE 4096^2 at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
SIMDS = 1024           # 256 CUs x 4 SIMDs
CLOCK_HZ = 2.4e9       # max engine clock (MI355X_MICROARCH.md)
# issue cycles of one wave64 VALU instruction on a SIMD-32 at saturation: 2 (32 lanes per cycle,
# MI355X_MICROARCH.md). Measured on this chip for fp64 too (tools/issue_probe.hip,
# profiles/r04_issue_probe.txt): independent v_fma_f64 streams cost 5.2 / 3.5 / 3.0 / 2.4 SIMD
# cycles per instruction at 1 / 2 / 3 / 4 waves per SIMD, DPP moves 4.4 / 3.2 / 2.8 / 2.6 -- fp64
# is not half rate here, and the fused kernels' limit is issue latency at their occupancy.
VALU_CYC = 2
# ... and the cycles a wave64 instruction of the fused march's mix (16 fp64 : 9 DPP) costs at the
# occupancy it runs with (waves per SIMD -> SIMD cycles per instruction, the same probe): the
# issue rate a latency-bound kernel can actually reach, so valu_frac_at_occupancy is the upper end
# of the VALU utilisation range [valu_frac, valu_frac_at_occupancy]
MIX_CYC_AT_WAVES = {1: 5.16, 2: 3.33, 3: 2.80, 4: 2.54}
RAMP_S = 0.4           # untimed sustained load before the timed steps (DVFS clock ramp)

CONFIGS = {
    # BASELINE configs[0]: the reference's CPU configuration (its example / test size), a smooth
    # dam-break (h = 10 + 0.5 (1 - tanh((x - W/2) / 8)), u = v = 0; tests/golden/gen_golden.py C1),
    # measured here on the GPU beside the reference CPU solver on the same workload
    "c1": dict(W=256, H=256, L=1, model=0, fp64=False, ic="dam_break", dam_width=8.0, cpu_steps_cap=1000,
               workload="C1: Shallow Water 256x256 smooth dam-break fp32 (the reference's CPU configuration)"),
    "c2": dict(W=4096, H=4096, L=1, model=0, fp64=True, ic="jet_stream",
               workload="C2: Shallow Water 4096x4096 fp64, 1 level"),
    "c3": dict(W=2048, H=2048, L=1, model=1, fp64=False, ic="zonal_flow",
               workload="C3: Barotropic (reference semantics: SWE tendencies, RK4->RK2) 2048x2048 fp32"),
    "c4": dict(W=1024, H=1024, L=32, model=2, fp64=False, ic="jet_stream",
               workload="C4: Primitive Equations (reference semantics) 1024x1024x32 levels fp32"),
    "c5": dict(W=16384, H=16384, L=1, model=0, fp64=True, ic="jet_stream",
               workload="C5: Shallow Water 16384x16384 fp64"),
    # one rank's share of C2 at 2 / 4 / 8 GPUs (measurement aid for the strong-scaling budget)
    "c2_slab2": dict(W=4096, H=2048, L=1, model=0, fp64=True, ic="jet_stream",
                     workload="C2 slab of 2: Shallow Water 4096x2048 fp64"),
    "c2_slab4": dict(W=4096, H=1024, L=1, model=0, fp64=True, ic="jet_stream",
                     workload="C2 slab of 4: Shallow Water 4096x1024 fp64"),
    "c2_slab8": dict(W=4096, H=512, L=1, model=0, fp64=True, ic="jet_stream",
                     workload="C2 slab of 8: Shallow Water 4096x512 fp64"),
    # C3 as BASELINE describes it ("Jacobian + Laplacian"): the physics-mode barotropic
    # vorticity model (no reference semantics, see weather_sim/physics.py)
    "c3p": dict(W=2048, H=2048, L=1, model=1, fp64=False, ic="rossby",
                workload="C3 physics mode: barotropic vorticity (Arakawa Jacobian + Laplacian, hipFFT Poisson) "
                         "2048x2048 fp32"),
    # C4 as BASELINE describes it ("3D stencil, vertical columns in LDS"): the physics-mode
    # layered primitive-equation model (no reference semantics)
    "c4p": dict(W=1024, H=1024, L=32, model=2, fp64=False, ic="layers",
                workload="C4 physics mode: layered primitive equations (isopycnal, Montgomery-potential column "
                         "scan in LDS) 1024x1024x32 fp32"),
}
METHODS = {"euler": 0, "rk2": 1, "rk4": 2}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def bootstrap_uid(dist, rank, make_uid, nbytes=128):
    """Rank 0 creates the RCCL unique id; every rank receives it over the (gloo) host group."""
    import torch
    uid = torch.zeros(nbytes, dtype=torch.uint8)
    if rank == 0:
        raw = make_uid()
        assert len(raw) == nbytes
        uid = torch.tensor(list(raw), dtype=torch.uint8)
    dist.broadcast(uid, 0)
    return bytes(uid.tolist())


def max_over_ranks(dist, seconds):
    """The contract's job time: the slowest rank's."""
    import torch
    t = torch.tensor([seconds], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t[0])


def host_cores():
    """Cores this process may run on: its CPU affinity set, capped by a cgroup CPU quota
    (cpu.max) when one is set -- on the GPU pool the affinity shows the whole machine while
    the quota gives the box's share. Returns (cores, how it was determined)."""
    aff = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            q = max(1, int(int(quota) // int(period)))
            if q < aff:
                return q, f"cgroup cpu.max quota {quota}/{period} (affinity {aff} CPUs)"
    except (OSError, ValueError):
        pass
    return aff, f"sched_getaffinity: {aff} CPUs"


def dam_break_height(W, H, width_cells, dtype):
    """C1's smooth dam-break height, exactly as tests/golden/gen_golden.py builds it."""
    import numpy as np
    x = np.arange(W, dtype=np.float64)
    row = 10.0 + 0.5 * (1.0 - np.tanh((x - W / 2) / width_cells))
    return np.broadcast_to(row, (H, W)).astype(dtype)


def cpu_baseline(conf, method, budget_s=20.0):
    """Time the reference CPU solver (or the oracle port) on a bounded sample, with one
    OpenMP thread per host core this process may use (host_cores)."""
    threads, how = host_cores()
    env = dict(os.environ, OMP_NUM_THREADS=str(threads))
    variant = "f64" if conf["fp64"] else "f32"
    ref = os.path.join(ROOT, "oracle", "_ref", f"ws_ref_{variant}")
    W, H = conf["W"], conf["H"] * conf["L"]  # levels stacked (the reference is 2-D only)
    if conf["H"] * conf["W"] * conf["L"] > 4096 * 4096 * 2:
        W, H = 4096, 4096  # C5 does not fit host memory in the reference layout: same per-cell work
    # pilot: 1 step to size the sample to ~budget_s
    def run_ref(steps):
        tmpfiles = []
        if conf["ic"] == "dam_break":  # a height field, loaded into the reference grid
            import numpy as np
            with tempfile.NamedTemporaryFile("wb", suffix=".bin", delete=False) as hf:
                dam_break_height(W, H, conf["dam_width"], np.float64 if conf["fp64"] else np.float32).tofile(hf)
            tmpfiles.append(hf.name)
            ic_lines = ["initialize", f"setfield h {hf.name}"]
        else:
            ic_lines = [f"ic {conf['ic']}", "initialize"]
        spec = "\n".join([f"cfg width {W}", f"cfg height {H}", f"cfg model {conf['model']}",
                          f"cfg method {method}", "cfg max_time 1e30", "create", *ic_lines,
                          "time_run 1", f"time_run {steps}"]) + "\n"
        with tempfile.NamedTemporaryFile("w", suffix=".txt", delete=False) as f:
            f.write(spec)
        tmpfiles.append(f.name)
        try:
            out = subprocess.run([ref, f.name], env=env, capture_output=True, text=True, timeout=600).stdout
        finally:
            for t in tmpfiles:
                os.unlink(t)
        secs = [float(l.split()[2]) for l in out.splitlines() if l.startswith("TIME_RUN")]
        return secs[-1]

    if os.path.exists(ref):
        pilot = run_ref(1)
        steps = max(1, min(conf.get("cpu_steps_cap", 200), int(budget_s / max(pilot, 1e-6))))
        secs = run_ref(steps)
        kind = "reference"
        what = f"reference weather_simulation.cpp (oracle/_ref/ws_ref_{variant}, -O3 -fopenmp)"
    else:
        from oracle.ws_oracle import OracleSim
        import numpy as np
        sim = OracleSim(W, H, conf["model"], method, max_time=1e30, precision=variant)
        sim.initialize()
        t0 = time.perf_counter()
        sim.step()
        pilot = time.perf_counter() - t0
        steps = max(1, min(200, int(budget_s / max(pilot, 1e-6))))
        t0 = time.perf_counter()
        sim.run(steps)
        secs = time.perf_counter() - t0
        kind = "port"
        what = "C oracle port (oracle/ws_oracle.c, -O3 -fopenmp)"
    return {"value": W * H * steps / secs, "unit": "cell-updates/s", "cores": threads, "kind": kind,
            "sample": f"{what}: {W}x{H}, {steps} steps after 1 warm-up step, {secs:.2f} s wall, "
                      f"OMP_NUM_THREADS={threads} ({how})"}


SLAB_GOLDEN = os.path.join(ROOT, "tests", "golden", "ref_slab_digests.json")
FAST_TOL = 1e-10  # north_star: fields within 1e-10 relative L2 of the reference (fp64)


def load_slab_golden():
    """Reference per-slab digests (tests/golden/gen_slab_digests.py): C2 jet_stream RK4 fp64."""
    if not os.path.exists(SLAB_GOLDEN):
        return None
    with open(SLAB_GOLDEN) as f:
        return json.load(f)


def slab_sha256(fields):
    import hashlib
    import numpy as np
    return {k: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest() for k, a in fields.items()}


def verdict_over_ranks(dist, ok):
    """Every rank learns whether all ranks passed (MIN over a gloo group; world 1: itself)."""
    if dist is None or not dist.is_initialized():
        return bool(ok)
    import torch
    t = torch.tensor([1 if ok else 0], dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t[0])


def clock_ramp(run_chunk, dist=None, enabled=True):
    """Untimed sustained load for RAMP_S seconds before the timed steps (the chip raises its
    clocks over tens of milliseconds of load). Returns the steps run. With more than one rank
    the stop decision is collective (a MIN over the gloo group after every chunk): each chunk
    of a slab decomposition is a collective run(), so every rank must run the same number."""
    steps, t_ramp = 0, time.perf_counter()
    multi = dist is not None and dist.is_initialized() and dist.get_world_size() > 1
    while enabled:
        go = time.perf_counter() - t_ramp < RAMP_S
        if multi:
            go = verdict_over_ranks(dist, go)
        if not go:
            break
        steps += run_chunk()
    return steps


def sum_over_ranks(dist, values):
    if dist is None or not dist.is_initialized():
        return list(values)
    import torch
    t = torch.tensor(list(values), dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.tolist()


def check_slab_parity(dist, rank, world, row0, rows, exact_fields, fast_fields, golden):
    """The self-check of a (multi-GPU) run against the reference, before the timed region.

    exact_fields: this rank's owned rows of u, v, h, vorticity after golden["steps"] steps in
    exact numerics -- their SHA-256 must equal the reference's for this rank of this world
    size (bit-for-bit, every rank). fast_fields (or None): the same run in the fp64 default
    fast numerics -- relative L2 against the exact (= reference) fields over the whole grid
    (sums over ranks) must be <= FAST_TOL. Returns (verdict "ok" | "fail", detail dict); every
    rank returns the same verdict."""
    import numpy as np
    want = golden["slabs"].get(str(world))
    detail = {"case": golden["case"], "steps": golden["steps"], "ranks_checked": world}
    if want is None:
        detail["error"] = f"no reference digests for {world} ranks"
        return "fail", detail
    mine = want[rank]
    ok = mine["row0"] == row0 and mine["rows"] == rows
    got = slab_sha256(exact_fields)
    bad = sorted(k for k in golden["fields"] if got.get(k) != mine["sha256"][k])
    ok = ok and not bad
    exact_ok = verdict_over_ranks(dist, ok)
    detail["exact"] = "bitwise == reference" if exact_ok else "MISMATCH"
    if not ok:
        detail["rank_mismatch"] = {"rank": rank, "fields": bad, "row0": row0, "rows": rows}
    fast_ok = True
    if fast_fields is not None:
        sums = []
        for k in ("u", "v", "h"):
            e = exact_fields[k].astype(np.float64)
            d = fast_fields[k].astype(np.float64) - e
            sums += [float(np.sum(d * d)), float(np.sum(e * e))]
        tot = sum_over_ranks(dist, sums)
        rel = {k: (tot[2 * i] ** 0.5) / max(tot[2 * i + 1] ** 0.5, 1e-300) for i, k in enumerate(("u", "v", "h"))}
        detail["fast_rel_l2"] = rel
        detail["fast_tol"] = FAST_TOL
        fast_ok = all(np.isfinite(v) and v <= FAST_TOL for v in rel.values())
    return ("ok" if exact_ok and fast_ok else "fail"), detail


def slab_fields(sim):
    g = sim.get_current_grid()
    u, v = g.get_velocity_field()
    return {"u": u, "v": v, "h": g.get_height_field(), "vort": g.get_vorticity_field()}


def self_check(sim, ic, dist, rank, world, golden):
    """Run the golden case on this simulation (exact, then the default numerics) and check it."""
    default = sim.get_numerics()
    sim.set_numerics("exact")
    sim.set_initial_condition(ic)
    sim.initialize()
    assert sim.run(golden["steps"]) == golden["steps"]
    exact = slab_fields(sim)
    fast = None
    if default != "exact":
        sim.set_numerics(default)
        sim.initialize()
        assert sim.run(golden["steps"]) == golden["steps"]
        fast = slab_fields(sim)
    row0 = getattr(sim, "row0", 0) or 0
    rows = exact["u"].shape[0]
    return check_slab_parity(dist, rank, world, row0, rows, exact, fast, golden)


def bvort_words_per_cell(method, W, H):
    """Algorithmic traffic of one barotropic step in words per cell: per RK stage an R2C
    (read W*H reals, write (W/2+1)*H complex), the column pass (read + write the spectrum;
    the hipFFT path's separate spectral scale moves the same bytes), a C2R (read the
    spectrum, write W*H reals) and the stage stencil (read zeta_s, psi, zeta_0 [+ acc],
    write zeta_out [+ acc])."""
    spec = 2.0 * (W // 2 + 1) * H / (W * H)  # complex spectrum, in real words per cell
    fft = (1 + spec) + 2 * spec + (spec + 1)
    stencil = {0: [4], 1: [4, 4], 2: [5, 6, 6, 5]}[method]
    return sum(fft + s for s in stencil)


def bench_bvort(args, conf, method, world, rank=0, local=0, dist=None):
    """Physics-mode barotropic (config c3p): one GPU; `--slabs N` N slabs of the ring
    decomposition on this GPU (one process: block transposes and halos by device copies);
    world > 1 one rank per GPU (ws_bvort_create_slab: RCCL block all-to-all + ring halos;
    strong scaling of the global grid)."""
    import numpy as np
    import torch
    import weather_sim as ws
    from oracle import bvort_oracle as bo

    W, H = conf["W"], conf["H"]
    cfg = ws.SimulationConfig()
    cfg.grid_width, cfg.grid_height = W, H
    cfg.integration_method = method
    cfg.double_precision = conf["fp64"]
    # beta small enough that the gravest Rossby mode (omega ~ beta W / 2 pi) stays inside
    # RK4's stability region at this dt
    cfg.dt, cfg.beta, cfg.viscosity = 0.05, 1e-3, 0.01
    cfg.device_id = local
    if world > 1:
        m = ws.BarotropicVorticityModel(cfg, slab=(rank, world, bootstrap_uid(dist, rank, ws.new_comm_id)))
        parallelism = f"y-slabs over {world} GPUs (RCCL block transposes + ring halos)"
    elif args.slabs > 1:
        m = ws.BarotropicVorticityModel(cfg, devices=[local] * args.slabs)
        parallelism = f"{args.slabs} y-slabs on one GPU (one process, device-copy transposes and halos)"
    else:
        m = ws.BarotropicVorticityModel(cfg)
        parallelism = "single GPU"
    z0 = bo.rossby_mode(W, H, 1.0, 1.0, 5, 3, amp=1e-2) + bo.rossby_mode(W, H, 1.0, 1.0, 2, 7, amp=5e-3)
    m.set_vorticity(z0[m.row0:m.row0 + m.rows])  # a rank's slab: its own rows
    if args.warmup > 0:
        m.run(args.warmup)
    clock_ramp(lambda: m.run(2) or 2, dist if world > 1 else None, args.warmup > 0)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    m.run(args.steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed = max_over_ranks(dist, elapsed)
    dev_ms, launches = m.last_run_stats()
    if not np.isfinite(m.get_vorticity_field()).all():
        raise SystemExit("c3p: vorticity is not finite after the timed run")
    if rank != 0:
        return
    w = 8 if conf["fp64"] else 4
    step_bytes = bvort_words_per_cell(method, W, H) * w * W * m.rows  # this rank's (or the whole) grid
    step_ms = dev_ms / args.steps
    achieved = step_bytes / (step_ms * 1e-3) / 1e9
    result = {
        "metric": METRIC, "value": W * H * args.steps / elapsed, "unit": "cell-updates/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
        "dtype": "f64" if conf["fp64"] else "f32",
        "data": "synthetic (two Rossby modes), inputs resident in HBM",
        "config": {"workload": conf["workload"] + f", {args.method.upper()}", "grid": [W, H], "levels": 1,
                   "integrator": args.method, "parallelism": parallelism},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS,
                     "traffic": _step_traffic(args, launches / args.steps) if parallelism == "single GPU" else None,
                     "kernel": "whole step (LDS-FFT Poisson: bv_rowfft_fwd + bv_colsolve + bv_rowfft_inv, then bv_stage_kernel)",
                     "bytes_per_launch": step_bytes, "mean_launch_ms": step_ms,
                     "note": "device time of the run (hipEvents on the model's stream) per step; "
                             "bytes = bvort_words_per_cell x cells"},
        "launches_per_step": launches / args.steps,
    }
    if not args.no_cpu_baseline and world == 1:
        # the NumPy oracle (a port: no reference exists for this model), bounded sample
        z = z0.astype(np.float64)
        t0 = time.perf_counter()
        n = 0
        while time.perf_counter() - t0 < 15.0 and n < 50:
            z = bo.step(z, cfg.dt, 1.0, 1.0, cfg.beta, cfg.viscosity, method)
            n += 1
        secs = time.perf_counter() - t0
        result["cpu_baseline"] = {"value": W * H * n / secs, "unit": "cell-updates/s", "cores": 1, "kind": "port",
                                  "sample": f"oracle/bvort_oracle.py (NumPy, fp64): {W}x{H}, {n} steps, {secs:.2f} s"}
    print(json.dumps(result), flush=True)


def _step_traffic(args, stage_launches_per_step):
    """HBM bytes per physics-mode step from rocprofv3 PMC (profiles/traffic_<config>_<method>.json):
    "step" = the bytes of every kernel of a step (tools/traffic_step.py), or "kind0" = bytes
    per stage-kernel dispatch (tools/traffic.py) x stage launches per step; None when no PMC
    summary for this config is committed."""
    tfile = os.path.join(ROOT, "profiles", f"traffic_{args.config}_{args.method}.json")
    if not os.path.exists(tfile):
        return None
    with open(tfile) as f:
        t = json.load(f)
    if "step" in t:
        return t["step"]
    return None if t.get("kind0") is None else t["kind0"] * stage_launches_per_step


def lpe_words_per_cell(method):
    """Algorithmic traffic of one layered-PE step in words per cell and level: per stage
    the stage input u, v, h, h again for the column scan, the step's base u, v, h, the RK4
    accumulator (read from stage 2 on, written up to stage 3) and the stage output."""
    stages = {0: [(0, 0)], 1: [(0, 0), (0, 0)], 2: [(0, 3), (3, 3), (3, 3), (3, 0)]}[method]
    return sum(3 + 1 + 3 + acc_r + acc_w + 3 for acc_r, acc_w in stages)


def bench_lpe(args, conf, method, world, rank=0, local=0, dist=None):
    """Physics-mode layered primitive equations (config c4p): one GPU; `--slabs N` N slabs of
    the ring decomposition on this GPU (one process, the pull transport); world > 1 one rank
    per GPU (ws_lpe_create_slab, RCCL halos; strong scaling of the global grid)."""
    import numpy as np
    import torch
    import weather_sim as ws
    from oracle import layered_pe_oracle as lp

    W, H, L = conf["W"], conf["H"], conf["L"]
    cfg = ws.SimulationConfig()
    cfg.grid_width, cfg.grid_height, cfg.num_levels = W, H, L
    cfg.integration_method = method
    cfg.double_precision = conf["fp64"]
    cfg.dx = cfg.dy = 1000.0
    cfg.dt, cfg.gravity, cfg.coriolis_f = 5.0, 9.81, 1e-4
    cfg.device_id = local
    gp = 0.02
    if world > 1:
        m = ws.LayeredPrimitiveEquationsModel(cfg, reduced_gravity=gp,
                                              slab=(rank, world, bootstrap_uid(dist, rank, ws.new_comm_id)))
        parallelism = f"y-slabs over {world} GPUs (RCCL ring halos)"
    elif args.slabs > 1:
        m = ws.LayeredPrimitiveEquationsModel(cfg, reduced_gravity=gp, devices=[local] * args.slabs)
        parallelism = f"{args.slabs} y-slabs on one GPU (one process, halo pull kernels)"
    else:
        m = ws.LayeredPrimitiveEquationsModel(cfg, reduced_gravity=gp)
        parallelism = "single GPU"

    def initial(Wi, Hi):
        u, v, h = lp.rest_state(L, Hi, Wi, [40.0 + 2.0 * k for k in range(L)])
        x = np.arange(Wi)[None, :]
        y = np.arange(Hi)[:, None]
        for k in range(L):
            h[k] += 0.5 * np.cos(2 * np.pi * (3 * x / Wi + 2 * y / Hi) + 0.1 * k)
        return u, v, h

    s0 = initial(W, H)
    m.set_state(*(a[:, m.row0:m.row0 + m.rows] for a in s0))  # a rank's slab: its own rows
    if args.warmup > 0:
        m.run(args.warmup)
    clock_ramp(lambda: m.run(2) or 2, dist if world > 1 else None, args.warmup > 0)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    m.run(args.steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed = max_over_ranks(dist, elapsed)
    dev_ms, launches = m.last_run_stats()
    if not np.isfinite(m.get_field("h")).all():
        raise SystemExit("c4p: state is not finite after the timed run")
    if rank != 0:
        return
    w = 8 if conf["fp64"] else 4
    cells = W * H * L
    step_bytes = lpe_words_per_cell(method) * w * m.rows * W * L  # this rank's (or the whole) grid
    step_ms = dev_ms / args.steps
    achieved = step_bytes / (step_ms * 1e-3) / 1e9
    result = {
        "metric": METRIC, "value": cells * args.steps / elapsed, "unit": "cell-updates/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
        "dtype": "f64" if conf["fp64"] else "f32",
        "data": "synthetic (stacked layers with an interface wave), inputs resident in HBM",
        "config": {"workload": conf["workload"] + f", {args.method.upper()}", "grid": [W, H], "levels": L,
                   "integrator": args.method, "parallelism": parallelism},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS,
                     "traffic": _step_traffic(args, launches / args.steps) if parallelism == "single GPU" else None,
                     "kernel": "lpe_stage_kernel (whole step)",
                     "bytes_per_launch": step_bytes, "mean_launch_ms": step_ms,
                     "note": "device time of the run (hipEvents on the model's stream) per step; "
                             "bytes = lpe_words_per_cell x cells x levels"},
        "launches_per_step": launches / args.steps,
    }
    if not args.no_cpu_baseline and world == 1:
        # the NumPy oracle (a port: no reference exists for this model) on a 256 x 256 x L
        # sample of the same per-cell work, bounded
        Ws = Hs = 256
        s = initial(Ws, Hs)
        t0 = time.perf_counter()
        n = 0
        while time.perf_counter() - t0 < 15.0 and n < 50:
            s = lp.step(s, cfg.dt, cfg.dx, cfg.dy, cfg.gravity, gp, cfg.coriolis_f, method)
            n += 1
        secs = time.perf_counter() - t0
        result["cpu_baseline"] = {"value": Ws * Hs * L * n / secs, "unit": "cell-updates/s", "cores": 1,
                                  "kind": "port",
                                  "sample": f"oracle/layered_pe_oracle.py (NumPy, fp64): {Ws}x{Hs}x{L}, {n} steps, "
                                            f"{secs:.2f} s"}
    print(json.dumps(result), flush=True)


def launcher_command(n, argv, port):
    """The torch.distributed.run command bench.py starts for `--gpus n` without a launcher:
    one process per GPU of this node, rendezvous on 127.0.0.1."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(n, argv, runner=subprocess.call):
    """Run bench.py under torch.distributed.run with n ranks as a child process (no GPU has
    been touched in this process: a launcher must not be exec'd from a GPU process) and return
    its exit status."""
    cmd = launcher_command(n, argv, free_port())
    log(f"--gpus {n} without a launcher: starting {n} ranks: {' '.join(cmd)}")
    return runner(cmd)


def rank_count_check(gpus, env):
    """(world size, error or None): the ranks of this launch must be exactly --gpus -- a
    "multi-GPU" number must never silently come from fewer (or more) ranks."""
    try:
        world = int(env.get("WORLD_SIZE", "1"))
    except ValueError:
        return 1, f"WORLD_SIZE={env.get('WORLD_SIZE')!r} is not an integer"
    if world != gpus:
        return world, (f"--gpus {gpus} but this launch has WORLD_SIZE={world} ranks; launch with "
                       f"--nproc-per-node {gpus}, or run without a launcher to let bench.py start them")
    return world, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--method", default="rk4", choices=sorted(METHODS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--slabs", type=int, default=1, help="c3p / c4p: N y-slabs of the ring decomposition on this "
                                                          "GPU (one process; measures the decomposition's cost)")
    ap.add_argument("--no-check", action="store_true", help="skip the parity self-check (profiling runs)")
    ap.add_argument("--pin", default=None, help="kernel:steps_per_launch:seg_rows:align (profiling runs pin "
                                                "the variant a bench run chose)")
    args = ap.parse_args()

    # --gpus N > 1 without a launcher: start N ranks ourselves -- torch.distributed.run as a
    # fresh child process, before anything here touches the GPU -- and exit with its status
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args.gpus, sys.argv[1:]))
    world, why = rank_count_check(args.gpus, os.environ)
    if why:
        log(f"error: {why}")
        sys.exit(2)

    os.environ.setdefault("WS_QUIET", "1")
    import torch  # plumbing: contract timing (barrier + torch.cuda.synchronize); loaded before libws_hip
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("gloo")  # bootstrap (RCCL unique id) + host-side max over ranks

    import weather_sim as ws

    conf = CONFIGS[args.config]
    method = METHODS[args.method]
    if args.config == "c3p":
        return bench_bvort(args, conf, method, world, rank, local, dist)
    if args.config == "c4p":
        return bench_lpe(args, conf, method, world, rank, local, dist)
    cfg = ws.SimulationConfig()
    cfg.grid_width, cfg.grid_height, cfg.num_levels = conf["W"], conf["H"], conf["L"]
    cfg.model = conf["model"]
    cfg.integration_method = method
    cfg.double_precision = conf["fp64"]
    cfg.device_id = local
    cfg.max_time = 1e30  # run() would otherwise stop at t >= 10 (1000 steps of dt = 0.01)

    if world > 1:  # one rank of the decomposition over processes (weather_sim.SlabSimulation)
        uid = bootstrap_uid(dist, rank, ws.new_comm_id)
        sim = ws.SlabSimulation(cfg, rank, world, uid)
    else:
        sim = ws.WeatherSimulation(cfg)

    if args.pin:
        k, tb, seg, al = args.pin.split(":")
        sim.pin_variant(kernel=k, steps_per_launch=int(tb), seg_rows=int(seg) or None, align=bool(int(al)))
    ic = {"jet_stream": ws.JetStreamInitialCondition, "zonal_flow": ws.ZonalFlowInitialCondition,
          "dam_break": lambda: None}[conf["ic"]]()  # C1: no IC object (the reset state + the h field)
    # parity self-check before the timed region: the reference's per-slab digests of the C2
    # jet_stream RK4 fp64 case (bitwise, exact numerics) and the default numerics within the
    # north_star tolerance; a failure is reported and the run exits non-zero
    parity, parity_detail = None, {"note": "self-check covers the c2 rk4 workload"}
    golden = load_slab_golden()
    if args.config == "c2" and args.method == "rk4" and golden is not None and not args.no_check:
        parity, parity_detail = self_check(sim, ic, dist if world > 1 else None, rank, world, golden)
        if rank == 0:
            log(f"parity self-check: {parity} {json.dumps(parity_detail)}")
    if ic is not None:
        sim.set_initial_condition(ic)
    sim.initialize()  # on a slab, the IC is evaluated in global coordinates for the owned rows
    if conf["ic"] == "dam_break":  # C1: the reference driver's `initialize` + `setfield h` (gen_golden.py)
        import numpy as np
        hfull = dam_break_height(conf["W"], conf["H"], conf["dam_width"], np.float64 if conf["fp64"] else np.float32)
        sim.get_current_grid().set_height_field(np.ascontiguousarray(hfull[sim.row0:sim.row0 + sim.rows]))

    def barrier():
        if world > 1:
            dist.barrier()

    if args.warmup > 0:
        sim.run(args.warmup)
    # clock ramp (untimed): the chip raises its clocks over tens of milliseconds of sustained
    # load, and W short warm-up steps from idle leave the timed steps on the ramp (measured:
    # C2 0.243 ms per two-step launch warm vs 0.277 when the timed run starts cold). Keep the
    # GPU busy for >= RAMP_S seconds of untimed steps first; reported as ramp_steps.
    # (chunks of >= 16 blocks: the slab auto schedule's first such run holds its trial)
    chunk = max(96, 16 * sim.slab_schedule()[0])
    ramp_steps = clock_ramp(lambda: sim.run(chunk), dist if world > 1 else None, args.warmup > 0)
    sim.set_kernel_timing(True, reserve=4 * args.steps + 16)  # events created outside the timed region
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    taken = sim.run(args.steps)
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    assert taken == args.steps, (taken, args.steps)
    if world > 1:
        elapsed = max_over_ranks(dist, elapsed)

    cells = conf["W"] * conf["H"] * conf["L"]
    value = cells * args.steps / elapsed
    # CFL of the final state by the device max-reduction (outside the timed region; a
    # collective over the ranks of a slab decomposition, so every rank calls it)
    sim.get_cfl()  # first call: HIP loads the reduction kernels' code lazily
    cfl, cfl_ms = sim.get_cfl(with_time=True)
    stats = sim.kernel_timing()
    variant, seg_rows, out_cols = sim.fused_variant()
    tb = sim.steps_per_launch()
    block, overlap = sim.slab_schedule()
    dev_ms, launches = sim.last_run_stats()
    # dominant kernel = largest total device time
    kind, (n, tot_ms, bpl) = max(stats.items(), key=lambda kv: kv[1][1])
    step_bytes = sum(b for (_, _, b) in stats.values()) / tb  # one launch per kind covers tb steps
    # PMC of the same variant (tools/profile_round.sh -> profiles/traffic_<config>_<method>.json):
    # HBM bytes and VALU wave-instructions per launch -- used only when the profiled variant
    # (kernel, steps per launch) is the one this run's autotuner chose
    traffic, valu_insts, traffic_variant, f64_frac = None, None, None, None
    tfile = os.path.join(ROOT, "profiles", f"traffic_{args.config}_{args.method}.json")
    if os.path.exists(tfile) and world == 1:
        with open(tfile) as f:
            tj = json.load(f)
        traffic_variant = tj.get("variant")
        if traffic_variant is None or traffic_variant == {"kernel": variant.replace("fused_", ""), "tb": tb}:
            traffic, valu_insts = tj.get(f"kind{kind}"), tj.get("valu_insts")
            f64_frac = tj.get("valu_f64_frac")
    launch_s = tot_ms / n * 1e-3
    # algorithmic bytes of one launch: y_n read + y_(n+k) written once (6 words per cell; the k
    # steps in between never leave the chip) -- the launch's compulsory HBM traffic
    compulsory = bpl / tb if variant != "stage_kernels" else bpl
    valu_frac = valu_insts * VALU_CYC / (SIMDS * CLOCK_HZ * launch_s) if valu_insts else None
    waves = sim.kernel_occupancy()
    occ_cyc = MIX_CYC_AT_WAVES.get(min(waves, 4)) if waves > 0 else None
    valu_frac_occ = valu_insts * occ_cyc / (SIMDS * CLOCK_HZ * launch_s) if valu_insts and occ_cyc else None
    dram_frac = traffic / launch_s / 1e9 / HBM_PEAK_GBS if traffic else None
    binding = None
    if valu_frac is not None and dram_frac is not None:
        hi = valu_frac_occ if valu_frac_occ is not None else valu_frac
        # VALU utilisation is known only within [valu_frac, valu_frac_occ]: a DRAM fraction
        # inside that range names no binding resource
        binding = "hbm" if dram_frac > hi else "valu" if valu_frac > dram_frac else None
    achieved = compulsory / launch_s / 1e9
    result = {
        "metric": METRIC,
        "value": value,
        "unit": "cell-updates/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ramp_steps": ramp_steps,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64" if conf["fp64"] else "f32",
        "data": "synthetic (reference jet_stream/zonal_flow initial condition), inputs resident in HBM",
        "config": {"workload": conf["workload"] + f", {args.method.upper()}", "grid": [conf["W"], conf["H"]],
                   "levels": conf["L"], "integrator": args.method,
                   "parallelism": f"y-slab x{world}" if world > 1 else "single GPU",
                   **({"slab_schedule": {"steps_per_exchange": block,
                                         "overlap": ["stream-ordered", "edge bands + exchange on a second stream"][overlap],
                                         "measured_exchange_us": sim.slab_exchange_us(),
                                         "choice": "auto: the first run of >= 16 blocks times the last three blocks of alternating "
                                                   "four-block segments of each schedule, best of two, and keeps the faster (ws_schedule.cpp run_steps)"
                                                   if os.environ.get("WS_SLAB_OVERLAP") is None else
                                                   "fixed by WS_SLAB_OVERLAP"}}
                      if world > 1 else {})},
        "roofline": {"bound": binding or "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS,
                     "traffic": traffic,
                     "traffic_variant": traffic_variant,
                     "kernel": variant if variant != "stage_kernels" else f"stage{kind}",
                     "seg_rows": seg_rows, "strip_out_cols": out_cols, "steps_per_launch": tb,
                     "bytes_per_launch": compulsory, "mean_launch_ms": tot_ms / n,
                     "byte_model": (f"algorithmic bytes per launch = 6 words per cell (read u, v, h of y_n + write "
                                    f"u, v, h of y_(n+{tb}): the {tb} step(s) in between stay on chip) x {cells} "
                                    f"cells ({'f64' if conf['fp64'] else 'f32'}); achieved = those bytes / the "
                                    f"kernel's mean launch time (HIP events on its stream); traffic = rocprofv3 PMC "
                                    f"HBM bytes per launch (2 x FETCH_SIZE + WRITE_SIZE, "
                                    f"profiles/traffic_{args.config}_{args.method}.json), dram_gbs = traffic / the "
                                    f"same launch time"
                                    if variant != "stage_kernels" else "SURVEY 8(d) stage-kernel words per launch"),
                     "dram_gbs": traffic / launch_s / 1e9 if traffic else None,
                     "dram_frac": dram_frac,
                     "valu_insts_per_launch": valu_insts,
                     "valu_f64_frac": f64_frac,
                     "valu_frac": valu_frac,
                     "waves_per_simd": waves,
                     "valu_frac_at_occupancy": valu_frac_occ,
                     "valu_model": f"SQ_INSTS_VALU per launch (PMC) x {VALU_CYC} issue cycles per wave64 "
                                   f"instruction on SIMD-32 (fp64 included: measured, tools/issue_probe.hip) / "
                                   f"({SIMDS} SIMDs x {CLOCK_HZ / 1e9:.1f} GHz x mean launch time); "
                                   f"valu_frac_at_occupancy: the same at the kernel mix's measured issue cycles for "
                                   f"its waves per SIMD ({MIX_CYC_AT_WAVES}, profiles/r04_issue_probe.txt); "
                                   f"valu_f64_frac = the fp64 share (PMC SQ_INSTS_VALU_{{ADD,MUL,FMA,TRANS}}_F64)",
                     "binding": binding,
                     "binding_note": (None if valu_frac is None or dram_frac is None else
                                      "DRAM utilisation lies inside the VALU range [valu_frac, "
                                      "valu_frac_at_occupancy]: no single binding resource" if binding is None else
                                      f"{binding} is the larger measured utilisation; below 0.7 neither HBM nor "
                                      f"VALU issue saturates (latency / occupancy bound)"
                                      if max(valu_frac_occ or valu_frac, dram_frac) < 0.7 else f"{binding}-bound"),
                     "one_step_equivalent_gbs": bpl / launch_s / 1e9,
                     "one_step_equivalent_note": "6 words per cell-update x cell-updates per launch / launch time: "
                                                 "the HBM rate a one-step-per-launch kernel would need for this "
                                                 "cell-update rate (can exceed the peak with two steps per launch)"},
        "achieved_hbm_gbs_step": step_bytes / (dev_ms / args.steps * 1e-3) / 1e9 if dev_ms > 0 else None,
        "cfl": {"value": cfl, "reduction_ms": cfl_ms,
                "gbs": 3 * (8 if conf["fp64"] else 4) * cells / world / (cfl_ms * 1e-3) / 1e9 if cfl_ms > 0 else None,
                "note": "max((|u|+sqrt(gh))dt/dx, (|v|+sqrt(gh))dt/dy) of the final state; device DPP max-reduction "
                        "reading u, v, h once (gbs = 3 words per local cell / reduction time)"},
        "kernel_stats": {f"stage{k}": {"launches": v[0], "mean_ms": v[1] / v[0], "bytes": v[2],
                                       "gbs": v[2] / (v[1] / v[0] * 1e-3) / 1e9} for k, v in stats.items()},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            result["cpu_baseline"] = cpu_baseline(conf, method)
        except Exception as e:  # the GPU number stands on its own
            log(f"cpu baseline failed: {e!r}")
            result["cpu_baseline"] = None
    result["parity"] = parity
    result["parity_detail"] = parity_detail
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if parity == "fail":
        sys.exit(3)


if __name__ == "__main__":
    main()
