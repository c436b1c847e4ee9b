"""bench.py's N > 1 path on the one-GPU box.

  * ``python bench.py --gpus 2`` with one visible GPU exits 2 without a bench line;
  * ``--gpus 2 --one-device-rehearsal`` launches two ranks through torch.distributed.run
    (this script's own launcher), both on cuda:0 over gloo, and runs the whole N > 1 bench —
    sharded-panel search, timed steps, max-over-ranks timing, the 2-rank training leg with
    the panel sharded 2-way and the bucketed gradient all-reduce — at a small size.  The
    numbers are not a measurement; the test checks the line's world size and shape.
"""

import json
import os
import subprocess
import sys
from pathlib import Path

import pytest
import torch

pytestmark = pytest.mark.gpu
REPO = Path(__file__).resolve().parents[1]


def _env():
    return {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}


@pytest.mark.timeout(200)
def test_bench_more_gpus_than_visible_fails_loudly():
    n = torch.cuda.device_count()
    r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", str(n + 1), "--steps", "1"],
                       capture_output=True, text=True, timeout=180, env=_env(), cwd=str(REPO))
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert f"needs {n + 1} visible GPUs, found {n}" in r.stderr
    assert '"n_gpus"' not in r.stdout


@pytest.mark.timeout(400)
def test_bench_two_rank_rehearsal_on_one_gpu():
    cmd = [sys.executable, "-u", str(REPO / "bench.py"), "--gpus", "2", "--one-device-rehearsal",
           "--n-ref", "20000", "--batch", "4", "--layers", "2", "--steps", "2", "--warmup", "1",
           "--f32-leg", "0", "--c2-n", "0", "--train-steps", "1", "--cpu-baseline", "0"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=380, env=_env(), cwd=str(REPO))
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    lines = [json.loads(s) for s in r.stdout.splitlines() if s.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    line = lines[0]
    assert line["n_gpus"] == 2
    assert line["distributed"] == {"backend": "gloo", "world_size": 2, "rehearsal_one_device": True}
    assert line["config"]["global_batch"] == 8
    assert "panel sharded 2-way" in line["config"]["parallelism"]
    assert line["masked_snvs_per_step_per_gpu"] > 0 and line["value"] > 0
    assert line["train"]["n_gpus"] == 2 and line["train"]["panel"] == "sharded 2-way"
    assert line["cpu_baseline"] is None
