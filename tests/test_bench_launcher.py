"""bench.py --gpus N without an external launcher starts N ranks itself
(a child torch.distributed.run, one process per GPU), relays rank 0's line
and propagates a failing rank's exit status.  CPU only: the ranks stop at the
launcher self-test hook, before anything touches a device."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(n, extra_env):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.update({"KZGX_BENCH_LAUNCH_SELFTEST": "1"}, **extra_env)
    return subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--steps", "2"], env=env,
                          capture_output=True, text=True, timeout=240)


def test_launch_command():
    sys.path.insert(0, ROOT)
    import bench
    cmd = bench.rank_launch_cmd(4, ["--gpus", "4", "--workload", "cfg5"], 29512)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29512" in cmd
    assert cmd[-5:] == [BENCH, "--gpus", "4", "--workload", "cfg5"]


def test_two_ranks_start_and_rank0_reports():
    r = _run(2, {})
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert lines == [{"selftest": True, "world": 2, "rank": 0, "gpus": 2}]


def test_failing_rank_fails_the_run():
    r = _run(2, {"KZGX_BENCH_FAIL_RANK": "1"})
    assert r.returncode != 0


def test_world_must_match_gpus():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", KZGX_BENCH_LAUNCH_SELFTEST="1")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4"], env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=2 but --gpus 4" in r.stderr


def test_rank_records_reach_rank0():
    """every rank's provenance record (rank, device, elapsed, its own fields)
    and the backend in use appear on rank 0's line (a SCALE run
    must show what ran); gloo on the CPU here, RCCL on the GPU node"""
    r = _run(3, {"KZGX_BENCH_LAUNCH_SELFTEST": "dist"})
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1
    ranks = lines[0]["ranks"]
    assert [x["rank"] for x in ranks] == [0, 1, 2]
    assert [x["batch"] for x in ranks] == [7, 8, 9]
    assert all(x["elapsed_s"] >= 0 for x in ranks)
    assert lines[0]["dist"]["backend"] == "gloo" and lines[0]["dist"]["world_size"] == 3
