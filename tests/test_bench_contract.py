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
    assert "--standalone" in cmd and cmd[cmd.index("--local-addr") + 1] == "127.0.0.1"  # torchrun binds the port
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


# ---- profiles/traffic.json: the counter bytes the bench line's roofline.traffic comes from -------
# Read bytes are measured from request counts by size (tools/pmc_traffic.py, method_version 2).
# A kernel that streams its input once cannot read less than that input: a figure below it means
# the counters were mis-read or mis-scaled (round 4 halved them for kernels missing from a hand-kept
# list).  Floors, in bytes per record of the entry's `records`, per kernel whose reads are known:
TRAFFIC_FLOORS = {
    "possible_fraud": {"k_c1_scatter": 16},             # key + ts
    "possible_fraud_sparse_keys": {"k_c1_scatter": 16},
    "hopping_double": {"k_c1v_scatter": 24},            # key + ts + amount (per record of the leg)
    "repartition_sum": {"k_shuf_write1": 24,            # region + ts + amount
                        "k_shuf_count1": 8},            # ts (+ the two validity bitmaps)
}


def _traffic():
    import json
    with open(os.path.join(os.path.dirname(bench.__file__), "profiles", "traffic.json")) as f:
        return json.load(f)


def test_traffic_entries_read_at_least_their_streamed_input():
    t = _traffic()
    checked = 0
    for cfg, floors in TRAFFIC_FLOORS.items():
        rec = t.get(cfg)
        if not rec or rec.get("method_version", 1) < 2:
            continue
        for k, per_record in floors.items():
            pk = rec["per_kernel"].get(k)
            if pk is None:
                continue
            floor = 0.97 * per_record * rec["records"]
            assert pk["read_bytes_per_step"] >= floor, (cfg, k, pk["read_bytes_per_step"], floor)
            checked += 1
    assert checked >= 1, "no method_version-2 entry to check"


def test_bench_uses_only_measured_traffic_entries():
    """bench.load_traffic ignores entries from before the size-classed read counters."""
    import json
    import tempfile
    with tempfile.NamedTemporaryFile("w", suffix=".json", delete=False) as f:
        json.dump({"x": {"records": 10, "hbm_bytes_per_step": 5.0},
                   "y": {"records": 10, "hbm_bytes_per_step": 7.0, "method_version": 2}}, f)
    assert bench.load_traffic(f.name, "x", 10) is None
    assert bench.load_traffic(f.name, "y", 10) == 7.0
    assert bench.load_traffic(f.name, "y", 11) is None
    os.unlink(f.name)


# ---- the bench line's per-phase figures: bytes a phase really moves, never above peak -----------
# partition_ms was credited with 40 B/record (scatter + refine) while its events
# bracket check + chunks + refine only, so the line showed 10 TB/s against an 8 TB/s peak.

def _check_per_kernel(per_kernel, n, pipeline=None):
    tot = 0.0
    for k, v in per_kernel.items():
        gbs = v["bytes_per_record"] * n / (v["ms"] / 1000.0) / 1e9
        assert abs(gbs - v["GB/s"]) <= 1e-6 * gbs, (k, gbs, v)
        assert v["GB/s"] <= bench.HBM_PEAK_GBS, (k, v)
        tot += v["bytes_per_record"]
    if pipeline is not None:
        assert abs(tot - pipeline) < 1e-9, (tot, pipeline)


def test_c2_phase_bytes_replayed_on_the_r05_line():
    """Replay the committed round-5 default line's phase times through today's byte map."""
    import json
    path = os.path.join(os.path.dirname(bench.__file__), "profiles", "r05", "final2", "bench.jsonl")
    d = json.loads(open(path).readline())
    n, groups = d["config"]["records_per_gpu"], d["config"]["groups_per_gpu"]
    phase = {k: v["ms"] for k, v in d["roofline"]["push"]["per_kernel"].items()}
    for wide in (False, True):
        own = bench.c2_phase_bytes(True, wide, False, groups, n)
        pk = bench.per_phase_block(phase, own, n)
        assert set(pk) == set(phase)
        _check_per_kernel(pk, n, sum(own.values()))
    own = bench.c2_phase_bytes(True, False, False, groups, n)
    assert own["stream_time_ms"] == 24 and own["partition_ms"] == 16  # scatter 16 in + 8 out; refine 8 + 8
    assert abs(own["apply_ms"] - (8 + 32.0 * groups / n)) < 1e-12


def test_value_phase_bytes():
    own = bench.value_phase_bytes(False)
    assert own["stream_time_ms"] == 40.125 and own["partition_ms"] == 32 and own["apply_ms"] == 16
    assert bench.value_phase_bytes(True)["stream_time_ms"] == 48


def test_committed_r06_lines_per_phase_below_peak():
    """Every bench line committed this round under profiles/r06/: per-phase GB/s at or below peak,
    and on the C2 line the phases' bytes sum to pipeline_bytes_per_record."""
    import glob
    import json
    root = os.path.join(os.path.dirname(bench.__file__), "profiles", "r06")
    seen = 0
    for path in glob.glob(os.path.join(root, "**", "*.jsonl"), recursive=True):
        for ln in open(path):
            if not ln.startswith("{"):
                continue
            d = json.loads(ln)
            roof = d.get("roofline") or {}
            n = (d.get("config") or {}).get("records_per_gpu")
            if not n:
                continue
            pk = (roof.get("push") or {}).get("per_kernel")
            if pk:
                _check_per_kernel(pk, n, roof.get("pipeline_bytes_per_record"))
                seen += 1
            if roof.get("per_kernel"):  # C3: per step of n records
                _check_per_kernel(roof["per_kernel"], n)
                seen += 1
    if seen == 0:
        pytest.skip("no round-6 bench lines committed yet")
