"""bench.py's multi-rank path (--gpus N under torch.distributed.run) on one MI355X.

The driver runs `torch.distributed.run --nproc-per-node N bench.py --gpus N` on an 8-GPU
node with backend nccl (RCCL).  That branch -- process group, rank 0 generating the
dataset, replicate_dataset to the other ranks, each rank fitting its own 128 learners,
barrier + max-over-ranks timing, one JSON line from rank 0 -- is rehearsed here with two
ranks sharing cuda:0 over gloo (bench.py --backend gloo: the same code with host-staged
collectives), so a crash there shows up before the driver's scaling run
(ml/regression/BaggingRegressor.scala:158-191: learners fitted independently over one
persisted dataset).
"""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_two_ranks_gloo_one_gpu():
    rows = 2_000_000
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo", "--rows", str(rows),
           "--steps", "1", "--warmup", "1", "--sampler-partitions", "128"]
    env = dict(os.environ)
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-4000:]  # one JSON line, from rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["backend"] == "gloo"
    assert out["config"]["learners_total"] == 256 and out["config"]["rows"] == rows
    assert out["value"] > 0 and out["ms_per_step"] > 0
    rep = out["replication"]
    assert rep is not None and rep["seconds"] > 0 and rep["bytes"] >= rows * 100
    assert 0 < out["value_incl_replication"] <= out["value"]
    assert out["roofline"]["frac"] > 0
    assert "cpu_baseline" not in out  # rank 0 at N = 1 only
