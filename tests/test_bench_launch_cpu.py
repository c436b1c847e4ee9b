"""bench.py's multi-GPU launch logic, on the CPU:

  * ``--gpus N`` (N > 1) started directly checks that N devices are visible BEFORE any GPU
    call and otherwise exits with status 2 and no bench line (here: no GPU at all);
  * with N devices it starts ``torch.distributed.run --nproc-per-node N`` on itself as a
    child process (not an exec) with the same arguments and returns the child's status;
  * a rank started by a launcher refuses a WORLD_SIZE different from --gpus.
"""

import json
import os
import subprocess
import sys
from pathlib import Path

import pytest
import torch

REPO = Path(__file__).resolve().parents[1]


def _bench():
    import bench
    return bench


def test_launch_command_starts_n_ranks_of_this_script():
    b = _bench()
    argv = ["--gpus", "8", "--steps", "3", "--warmup", "1"]
    args = b.parse(argv)
    cmd = b.launch_command(args, argv, 29511)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29511"
    assert Path(cmd[cmd.index("--master-port") + 2]) == REPO / "bench.py"
    assert cmd[-len(argv):] == argv


def test_launch_ranks_spawns_child_with_enough_devices(monkeypatch):
    b = _bench()
    calls = []
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    monkeypatch.setattr(subprocess, "call", lambda cmd, env=None: calls.append((cmd, env)) or 7)
    argv = ["--gpus", "4", "--steps", "2"]
    assert b.launch_ranks(b.parse(argv), argv) == 7
    (cmd, env), = calls
    assert "--nproc-per-node=4" in cmd and cmd[-2:] == ["--steps", "2"]
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    assert "WORLD_SIZE" not in env or env["WORLD_SIZE"] == os.environ.get("WORLD_SIZE")


def test_launch_ranks_refuses_missing_devices(monkeypatch):
    b = _bench()
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    monkeypatch.setattr(subprocess, "call", lambda *a, **k: pytest.fail("must not launch"))
    with pytest.raises(SystemExit) as e:
        b.launch_ranks(b.parse(["--gpus", "2"]), ["--gpus", "2"])
    assert e.value.code == 2


def test_rank_refuses_world_size_mismatch(monkeypatch):
    b = _bench()
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("LOCAL_RANK", "0")
    with pytest.raises(SystemExit) as e:
        b.setup_dist(b.parse(["--gpus", "4"]))
    assert e.value.code == 2


def test_bench_gpus2_without_devices_fails_loudly():
    """The real entry point, as the driver would start it, on a box with fewer GPUs than asked."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=str(REPO))
    assert r.returncode == 2, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    assert "needs 2 visible GPUs" in r.stderr
    for line in r.stdout.splitlines():
        with pytest.raises(json.JSONDecodeError):
            json.loads(line)
