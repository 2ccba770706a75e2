"""CPU: bench.py's multi-rank launcher (VERDICT r02 "Next round" 1).

`python bench.py --gpus N` with no WORLD_SIZE in the environment must start the N ranks itself (a child
torch.distributed.run, before any GPU call) and pass rank 0's single JSON line through; a WORLD_SIZE that
differs from --gpus must fail. `--stub-gpu` replaces the GPU work with a gloo all-gather of each rank's
RANK / WORLD_SIZE / LOCAL_RANK, so this runs here.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")
_RANK_ENV = ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")


def _env(**extra):
    env = {k: v for k, v in os.environ.items() if k not in _RANK_ENV}
    env.update(extra)
    return env


def test_gpus2_launches_two_ranks_and_prints_one_line():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--stub-gpu"], env=_env(), cwd=ROOT,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [x for x in r.stdout.splitlines() if x.strip()]
    assert len(lines) == 1, r.stdout  # the ranks' fd-1 banners went to stderr
    assert "stand-in banner" in r.stderr
    j = json.loads(lines[0])
    assert j["n_gpus"] == 2 and j["stub"] is True
    # every rank ran with RANK / WORLD_SIZE / LOCAL_RANK set by the launcher
    assert sorted(tuple(x) for x in j["ranks"]) == [(0, 2, 0), (1, 2, 1)]
    # the per-rank diagnostics of the real line (stand-in values): kernel time and placement of every rank
    assert j["roofline"]["per_rank_avg_kernel_us"] == [40.0, 41.0]
    assert j["per_rank_device"] == [0, 1] and j["per_rank_torch_device"] == [0, 1]
    assert j["per_rank_local_rank"] == [0, 1] and j["placement_ok"] is True


def test_gpus1_runs_in_process():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--stub-gpu"], env=_env(), cwd=ROOT,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    j = json.loads(r.stdout.strip())  # exactly one line: the banner printed on fd 1 went to stderr
    assert j["n_gpus"] == 1 and j["ranks"] == [[0, 1, 0]]
    assert j["roofline"]["per_rank_avg_kernel_us"] == [40.0] and j["per_rank_device"] == [0]


def test_world_size_must_equal_gpus():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--stub-gpu"],
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"), cwd=ROOT,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=120)
    assert r.returncode != 0 and r.stdout.strip() == ""
    assert "WORLD_SIZE=2 but --gpus 1" in r.stderr


def _run_failing(mode, timeout_s):
    import time

    t0 = time.monotonic()
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--stub-gpu", "--stub-fail-rank", "1",
                        "--stub-fail-mode", mode, "--dist-timeout", str(timeout_s)], env=_env(), cwd=ROOT,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=240)
    return r, time.monotonic() - t0


def test_a_failing_rank_fails_the_run_promptly():
    """A rank that raises ends the whole run with a non-zero exit and no JSON line: torch.distributed.run stops the
    other rank, which would otherwise wait in its collective (the driver's 8-GPU run must not hang on one rank)."""
    r, took = _run_failing("raise", 30)
    assert r.returncode != 0 and r.stdout.strip() == "", (r.returncode, r.stdout)
    assert "this rank fails" in r.stderr
    assert took < 120, took


def test_a_stalled_rank_times_out_the_run():
    """A rank that stalls (sleeps far past the process-group timeout before its collective): the other rank's
    collective raises after --dist-timeout seconds, its non-zero exit stops the group, and the launcher returns
    non-zero with no JSON line, in about that long rather than the library's default of 10-30 minutes."""
    r, took = _run_failing("stall", 8)
    assert r.returncode != 0 and r.stdout.strip() == "", (r.returncode, r.stdout)
    assert took < 120, took
