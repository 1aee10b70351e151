"""bench.py's own contract on the GPU: the single-GPU JSON line, and the multi-rank line of a
2-rank run (torch.distributed.run, both ranks on this box's GPU over gloo), for both partitions."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(args, nproc=1, port=29641):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    if nproc == 1:
        cmd = [sys.executable, "bench.py"] + args
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--backend", "gloo"] + args
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


def test_single_gpu_line():
    r = run(["--res", "64", "--steps", "3", "--warmup", "1", "--cpu-seconds", "1"])
    assert r["metric"] == "optimizer iterations/sec (fwd+adjoint), 64³ voxels × 64 angles"
    assert r["n_gpus"] == 1 and r["steps"] == 3 and r["value"] > 0
    assert r["cpu_baseline"]["kind"] == "port" and r["cpu_baseline"]["host"]["threads"] >= 1
    # the baseline runs on the affinity's CPUs, the OMP share timed beside it
    assert r["cpu_baseline"]["host"]["threads"] == len(os.sched_getaffinity(0)) == r["cpu_baseline"]["cores"]
    if r["cpu_baseline"]["host"]["omp_threads"] != r["cpu_baseline"]["host"]["threads"]:
        assert r["cpu_baseline"]["at_omp_num_threads"]["value"] > 0
    # the median of the timed steps beside the mean, and the dense-gradient adjoint
    steps = r["ms_per_step_min_max"]
    assert steps[0] <= r["ms_per_step_median"] <= steps[1]
    assert abs(r["value_median"] * r["ms_per_step_median"] - 1e3) < 1e-6 * r["value_median"] * r["ms_per_step_median"]
    assert r["dense_gradient"]["adj_ms"] > 0 and r["dense_gradient"]["ms_per_step_model"] > 0
    # counter summaries are committed for the BASELINE sizes only (profiles/r03/roofline_config<K>.json)
    assert set(r["roofline"]) >= {"bound", "achieved", "peak", "unit", "frac", "traffic"}
    assert r["roofline"]["frac"] is None and r["roofline"]["fwd_call_ms"] > 0


@pytest.mark.parametrize("shard,port", [("slab", 29651), ("angle", 29653)])
def test_two_rank_line(shard, port):
    r = run(["--res", "64", "--steps", "3", "--warmup", "1", "--shard", shard], nproc=2, port=port)
    assert r["n_gpus"] == 2 and r["value"] > 0 and r["cpu_baseline"] is None
    assert ("z-slab" if shard == "slab" else "angle-shard") in r["config"]["parallelism"]


def test_gpus_flag_launches_ranks():
    """`bench.py --gpus 2` with no torch.distributed environment starts both ranks itself (both on
    this box's one GPU over gloo) and prints rank 0's line with the world it measured."""
    r = run(["--gpus", "2", "--backend", "gloo", "--res", "64", "--steps", "2", "--warmup", "1",
             "--shard", "angle"])
    assert r["n_gpus"] == 2 and r["world_size"] == 2 and r["backend"] == "gloo" and r["value"] > 0
    assert "angle-shard x2" in r["config"]["parallelism"]
