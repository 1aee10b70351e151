"""The record writer's closed-form brick count (sc_brick_count, drtvam_amd/csrc/tvam_bricks.h)
against the bin fill's walk (sc_walk_bricks) on random segments, host-compiled
(tools/brick_count_check.hip: grids that are and are not brick multiples, axis-parallel and
near-axis directions, origins on voxel faces).  The GPU side of the same check: the fill kernel
counts disagreeing slots, bin_stats()["count_mismatch"] (tests/test_gpu_bin_chunks.py)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"), reason="no hipcc")
def test_closed_form_brick_count_matches_walk(tmp_path):
    env = dict(os.environ, TMPDIR=str(tmp_path))
    r = subprocess.run([os.path.join(ROOT, "tools", "brick_count_check.sh"), "100000"], capture_output=True, text=True,
                       env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout
