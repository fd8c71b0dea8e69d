"""bench.py --gpus N spawns its own N worker processes (RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_* set, before any GPU or thesia import) -- the launcher plumbing and the gloo
reductions (barrier, max time, per-rank report), on CPU via --selftest."""
import argparse
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env,
                          capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("n", [2, 3])
def test_launcher_spawns_n_workers(n):
    r = _run("--gpus", str(n), "--selftest")
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1  # one JSON line, rank 0's
    d = lines[0]
    assert d["n_ranks"] == n and d["n_gpus"] == n
    assert d["per_rank_frames"] == [1000 * (k + 1) for k in range(n)]
    assert len(set(d["pids"])) == n and os.getpid() not in d["pids"]
    # max over ranks: the slowest rank sleeps 50 ms x n
    assert d["ms_per_step"] >= 50.0 * n
    assert abs(d["value"] - sum(d["per_rank_frames"]) / (d["ms_per_step"] * 1e-3)) < 1e-6 * d["value"]


def test_single_process_without_launcher():
    r = _run("--selftest")
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["n_ranks"] == 1 and d["per_rank_frames"] == [1000]


def test_failing_worker_fails_the_launch():
    r = _run("--gpus", "2", "--selftest", "--selftest-fail-rank", "1")
    assert r.returncode != 0


def test_profile_records_behind_the_bench_line():
    """The default bench line's `roofline.traffic` and `roofline_valu_issue` come from the PMC
    record of exactly its workload (profiles/pmc_traffic.json: every launch parameter equal) and
    say so (`traffic_source` / `valu_insts_source`: stored, not measured in this run); any other
    workload (fewer tracks, another n_mels, another kernel) gets none. The issue roofline is the
    kernel's VALU wave-instructions over the kernel time against 256 CUs x 4 SIMDs x 2.4 GHz / 2."""
    sys.path.insert(0, ROOT)
    import bench
    saved, sys.argv = sys.argv, ["bench.py"]
    try:
        args = bench.parse()
    finally:
        sys.argv = saved
    rec = bench.profile_record(bench.workload_params(args, 5))
    assert rec is not None and rec["hbm_bytes_per_launch"] > 12.96e9  # >= the algorithmic bytes
    src = bench.provenance(rec)
    assert src["measured_in_this_run"] is False and src["profile"].startswith("profiles/r05_close")
    ic = bench.issue_ceiling(rec, 4.0)
    assert ic["bound"] == "valu-issue" and ic["peak"] == 1228.8
    assert abs(ic["achieved"] - ic["valu_insts_per_launch"] / 4e-3 / 1e9) < 1e-9 * ic["achieved"]
    assert abs(ic["frac"] - ic["achieved"] / ic["peak"]) < 1e-12
    assert ic["valu_insts_source"]["measured_in_this_run"] is False
    for change in ({"tracks": 100}, {"n_mels": 64}, {"seconds": 10.0}):
        other = argparse.Namespace(**dict(vars(args), **change))
        assert bench.profile_record(bench.workload_params(other, 5)) is None
    assert bench.profile_record(bench.workload_params(args, 3)) is None
    assert bench.issue_ceiling(None, 4.0) is None
