"""bench.py contract and its multi-rank self-check, rehearsed on the CPU.

The driver runs ``bench.py`` under ``torch.distributed.run`` on 1/2/4/8
GPUs.  A single-GPU lease cannot exercise RCCL, so the multi-rank path is
rehearsed here with gloo ranks on the torch backend: every decomposition
(optimiser choice, explicit 2x2x1 / 2x2x2 grids, blocked and single-step
passes) must end with the serial run's field energy -- the checksum the JSON
carries.  Also checks the metric label and the RCCL argument construction.
"""

import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIZE = ["40", "36", "44"]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(nproc, extra, steps=9, warmup=3):
    args = ["bench.py", "--backend", "torch", "--size"] + SIZE + ["--steps", str(steps), "--warmup", str(warmup),
                                                                 "--gpus", str(nproc), "--timeout", "120"] + extra
    env = dict(os.environ, FDTD_BENCH_COMM="gloo", OMP_NUM_THREADS="1")
    if nproc == 1:
        cmd = [sys.executable] + args
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
               "--master-addr", "127.0.0.1", "--master-port", str(_port())] + args
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.fixture(scope="module")
def serial():
    return _run(1, [])


def test_serial_record(serial):
    assert serial["metric"] == "Mcells/sec (whole node), 3D vacuum 40x36x44 grid at 1/2/4/8 MI355X"
    assert serial["n_gpus"] == 1 and serial["steps"] == 9 and serial["warmup"] == 3
    ck = serial["checksum"]
    # random-init fields, bounded evolution (PEC walls zeroed)
    assert ck["energy0"] > 0 and 0.5 < ck["energy"] / ck["energy0"] < 3.0
    assert serial["config"]["time_block"] == 5


def test_metric_label():
    sys.path.insert(0, ROOT)
    import bench
    assert bench.metric_name((1024, 1024, 1024)) == "Mcells/sec (whole node), 3D vacuum 1024^3 grid at 1/2/4/8 MI355X"
    assert bench.metric_name((2048, 1024, 1024)).startswith("Mcells/sec (whole node), 3D vacuum 2048x1024x1024 grid")


@pytest.mark.parametrize("nproc,extra,topo", [
    (2, [], "2x1x1"),
    (4, ["--topology", "2x2x1"], "2x2x1"),
    (8, ["--topology", "2x2x2"], "2x2x2"),
    (4, ["--topology", "xyz", "--time-block", "1", "--buffer-size", "1"], None),
])
def test_decomposed_equals_serial(serial, nproc, extra, topo):
    out = _run(nproc, extra)
    if topo is not None:
        assert out["config"]["parallelism"].startswith("domain-decomposition %s" % topo)
    assert out["n_gpus"] == nproc
    assert out["checksum"]["energy0"] == pytest.approx(serial["checksum"]["energy0"], rel=1e-12)
    assert out["checksum"]["energy"] == pytest.approx(serial["checksum"]["energy"], rel=1e-9)
    assert out["config"]["halo_bytes_per_step"] > 0
    assert out["config"]["halo_ms_per_pass_max"] >= out["config"]["halo_ms_per_pass_mean"] > 0


def test_nccl_p2p_ops_built_as_one_group(monkeypatch):
    """The RCCL branch of DistComm.post: every send and receive of one
    exchange goes into ONE batch_isend_irecv call with the right peers / tags
    (mocked: no second device here)."""
    import torch
    import torch.distributed as dist
    from fdtd3d_amd.parallel import comm as C

    made, batches = [], []

    class FakeOp:
        def __init__(self, op, tensor, peer, group, tag):
            made.append((op, tensor, peer, group, tag))

    monkeypatch.setattr(dist, "P2POp", FakeOp)
    monkeypatch.setattr(dist, "batch_isend_irecv", lambda ops: batches.append(list(ops)) or ["w"] * len(ops))
    dc = C.DistComm.__new__(C.DistComm)
    dc.group, dc.backend = "G", "nccl"
    a, b = torch.zeros(3), torch.zeros(4)
    works = dc.post([C.P2P(True, a, 3, 305), C.P2P(False, b, 5, 321)])
    assert len(batches) == 1 and len(batches[0]) == 2 and works == ["w", "w"]
    assert made[0] == (dist.isend, a, 3, "G", 305)
    assert made[1] == (dist.irecv, b, 5, "G", 321)


def test_nccl_init_kwargs_have_timeout_and_priority():
    import datetime
    from fdtd3d_amd.parallel import comm as C
    kw = C.nccl_init_kwargs(None, 42)
    assert kw["timeout"] == datetime.timedelta(seconds=42)
    assert kw["pg_options"].is_high_priority_stream
    assert "device_id" not in kw
