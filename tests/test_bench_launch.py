"""bench.py --gpus N on the CPU: without a torch.distributed environment the parent starts N ranks
itself (a child torch.distributed.run) and passes rank 0's line through; each rank checks that the
world it joined has --gpus ranks.  --launch-check stops after one all-reduce, so no GPU is needed."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, "bench.py"] + args, cwd=ROOT, env=env, capture_output=True, text=True,
                          timeout=240)


def line(out):
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert out.returncode == 0 and len(lines) == 1, (out.stdout, out.stderr[-2000:])
    return json.loads(lines[0])


def test_gpus_two_spawns_two_ranks():
    r = line(run(["--gpus", "2", "--backend", "gloo", "--launch-check"]))
    assert r["n_gpus"] == 2 and r["allreduce_ranks"] == 2 and r["backend"] == "gloo"


def test_gpus_one_stays_in_process():
    out = run(["--gpus", "1", "--launch-check"])
    r = line(out)
    assert r["n_gpus"] == 1 and r["backend"] is None
    assert "launching" not in out.stderr


def test_gpus_must_match_world_size():
    out = run(["--gpus", "4", "--launch-check"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert out.returncode != 0 and "--gpus 4 but WORLD_SIZE 2" in out.stderr
