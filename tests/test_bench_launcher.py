"""bench.py's N-GPU launcher (VERDICT r3 Next #1): ``--gpus N`` without a WORLD_SIZE launches N ranks
through torch.distributed.run (fresh processes, no exec, nothing touches the GPU first); under an
external launcher a WORLD_SIZE that disagrees with --gpus is refused instead of silently reporting
a different world."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


@pytest.fixture()
def bench(monkeypatch):
    import importlib
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    return importlib.import_module("bench")


def test_world_size_mismatch_exits_nonzero():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode == 2, (p.returncode, p.stderr[-500:])
    assert "WORLD_SIZE=2" in p.stderr and "--gpus 4" in p.stderr


def test_launcher_spawns_n_ranks(bench, monkeypatch):
    calls = []
    monkeypatch.setattr(bench.subprocess, "call", lambda cmd: calls.append(cmd) or 7)
    rc = bench._launch_ranks(["--gpus", "3", "--steps", "2", "--warmup", "1"])
    assert rc == 7 and len(calls) == 1  # the children's status is the parent's exit status
    cmd = calls[0]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=3" in cmd and "--nnodes=1" in cmd and "--master-addr=127.0.0.1" in cmd
    assert any(c.startswith("--master-port=") for c in cmd)
    assert cmd[-6:] == ["--gpus", "3", "--steps", "2", "--warmup", "1"]
    assert cmd[-7].endswith("bench.py")


def test_launcher_runs_in_process_when_it_is_a_rank_or_one_gpu(bench, monkeypatch):
    monkeypatch.setattr(bench.subprocess, "call", lambda cmd: pytest.fail("must not spawn"))
    assert bench._launch_ranks(["--gpus", "1"]) is None
    assert bench._launch_ranks([]) is None
    monkeypatch.setenv("WORLD_SIZE", "4")
    assert bench._launch_ranks(["--gpus", "4"]) is None
    assert bench._launch_ranks(["--gpus", "2"]) == 2
