"""bench.py's driver contract, checked without a GPU: `--gpus N` (N > 1) outside torchrun
relaunches the script under torch.distributed.run with N ranks on 127.0.0.1 before anything
touches the GPU, and a rank whose WORLD_SIZE disagrees with --gpus refuses to run."""
import os
import sys

import pytest

import bench


def test_multi_gpu_relaunches_under_torchrun(monkeypatch):
    calls = []
    monkeypatch.setattr(bench.subprocess, "call", lambda cmd, env=None: calls.append((cmd, env)) or 0)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "3", "--warmup", "1"])
    assert bench.main() == 0
    (cmd, env), = calls
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "4"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index(os.path.abspath(bench.__file__)) + 1:] == ["--gpus", "4", "--steps", "3", "--warmup", "1"]
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    assert "torch" not in sys.modules or not _cuda_initialised()


def _cuda_initialised():
    import torch
    return torch.cuda.is_initialized()


def test_world_size_must_match_gpus(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4"])
    with pytest.raises(SystemExit):
        bench.main()


def test_single_gpu_does_not_relaunch(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench, "relaunch", lambda args: pytest.fail("relaunched at --gpus 1"))
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    import torch
    if torch.cuda.is_available():
        pytest.skip("would run the benchmark")
    with pytest.raises(Exception):  # no GPU here: fails at the first device call, not at relaunch
        bench.main()
