"""bench.py's launch contract on CPU: `--gpus N` without a launcher starts N ranks itself
(torch.distributed.run as a child process, before any GPU call), and a launch whose rank
count differs from --gpus exits non-zero instead of quietly measuring fewer GPUs."""
import os
import subprocess
import sys

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_launcher_command():
    cmd = bench.launcher_command(8, ["--gpus", "8", "--steps", "5"], 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29555" in cmd
    i = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[i + 1:] == ["--gpus", "8", "--steps", "5"]


def test_self_launch_runs_child_and_returns_status():
    seen = []

    def runner(cmd):
        seen.append(cmd)
        return 7

    assert bench.self_launch(4, ["--gpus", "4"], runner=runner) == 7
    assert len(seen) == 1 and "--nproc-per-node=4" in seen[0]
    port = int(next(a for a in seen[0] if a.startswith("--master-port=")).split("=")[1])
    assert 0 < port < 65536


def test_rank_count_check():
    assert bench.rank_count_check(1, {}) == (1, None)
    assert bench.rank_count_check(4, {"WORLD_SIZE": "4"}) == (4, None)
    world, why = bench.rank_count_check(8, {"WORLD_SIZE": "1"})
    assert world == 1 and "--gpus 8" in why
    assert bench.rank_count_check(1, {"WORLD_SIZE": "2"})[1] is not None
    assert bench.rank_count_check(2, {"WORLD_SIZE": "x"})[1] is not None


def _run(args, env_extra, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env, capture_output=True,
                          text=True, timeout=timeout)


def test_rank_count_mismatch_exits_nonzero():
    p = _run(["--gpus", "2", "--steps", "1"], {"WORLD_SIZE": "1"})
    assert p.returncode == 2, p.stderr
    assert "WORLD_SIZE=1" in p.stderr and not p.stdout


def test_self_launch_end_to_end_reaches_the_ranks():
    """No launcher: bench.py starts torch.distributed.run with 2 ranks. On this GPU-less
    container the ranks then fail at the device step, so the whole launch must fail -- but
    only after the ranks started with WORLD_SIZE=2 (they passed the rank-count check)."""
    p = _run(["--gpus", "2", "--steps", "1", "--warmup", "0", "--no-cpu-baseline"], {})
    assert "starting 2 ranks" in p.stderr
    assert p.returncode != 0
    assert "error: --gpus" not in p.stderr  # the ranks saw WORLD_SIZE == --gpus
    assert not p.stdout.strip()  # no JSON line from a failed multi-GPU launch
