"""bench.py's multi-rank code end to end on a one-GPU box (rehearsal, not a
perf number): the torch.distributed.run relaunch, the gloo barrier, the
max-over-ranks reduce, the rank != 0 exit and the one JSON line, with the
candidates exchanged host-staged (two ranks cannot share a GPU over RCCL);
and --single-process with a repeated GPU id (kp_create_multi, in-process
exchange). The line must carry the oracle's round / pass / placement counts.
The 8-GPU RCCL form itself runs only on the driver's 8-GPU node."""
import json
import os
import socket
import subprocess
import sys

import pytest

from kplace import _abi, synth

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
J, N = 20_000, 2_000


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "2",
           "--warmup", "1", "--jobs", str(J), "--nodes", str(N), "--place-steps", "1",
           "--no-cpu-baseline", "--no-stream", "--no-config4", "--master-port", str(_port())] + extra
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 only
    return json.loads(lines[0])


@pytest.fixture(scope="module")
def want(oracle):
    w = synth.config3(J, N)
    p = _abi.default_params(**synth.CONFIG_PARAMS[3])
    return oracle.place(oracle.SnapshotBuf.from_workload(w), p, nthreads=8)


@pytest.mark.parametrize("extra", [["--exchange", "host"], ["--single-process", "--gpu-ids", "0,0"]])
def test_bench_multi_rank_rehearsal(want, extra):
    b = _run(extra)
    assert b["n_gpus"] == 2 and b["steps"] == 2 and b["ms_per_step"] > 0 and b["value"] > 0
    assert "REHEARSAL" in b["data"]
    c = b["config"]
    assert (c["rounds"], c["passes"], c["placed_jobs"]) == (want["rounds"], want["passes"], want["placed"])
    assert b["latency_ms"] > 0
