"""bench.py's multi-rank code end to end on a one-GPU box (rehearsal, not a
perf number): the torch.distributed.run relaunch, the gloo barrier, the
max-over-ranks reduce, the rank != 0 exit and the one JSON line, with the
candidates exchanged host-staged (two ranks cannot share a GPU over RCCL);
and --single-process with a repeated GPU id (kp_create_multi, in-process
exchange). The line must carry the oracle's round / pass / placement counts,
the phase split of the config #3 solve (candidate phase / exchange /
passes), the per-rank score-matrix leg, and the config #4 leg run sharded
over the same ranks (solve + kp_preempt) with the counts of the oracle's
full-size config #4 digests (tests/golden/large_digests.json) and its own
phase split. The 8-GPU RCCL form itself runs only on the driver's 8-GPU
node."""
import json
import os
import socket
import subprocess
import sys

import pytest

from kplace import _abi, synth

GOLD = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                                   "large_digests.json")))

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
J, N = 20_000, 2_000


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(extra, config4=False):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "2",
           "--warmup", "1", "--jobs", str(J), "--nodes", str(N), "--place-steps", "1",
           "--no-cpu-baseline", "--no-stream", "--master-port", str(_port()), "--score-steps", "1",
           "--c4-steps", "1"] + ([] if config4 else ["--no-config4"]) + extra
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


@pytest.mark.parametrize("extra,config4", [(["--exchange", "host"], True),
                                           (["--single-process", "--gpu-ids", "0,0"], False)])
def test_bench_multi_rank_rehearsal(want, extra, config4):
    b = _run(extra, config4)
    assert b["n_gpus"] == 2 and b["steps"] == 2 and b["ms_per_step"] > 0 and b["value"] > 0
    assert "REHEARSAL" in b["data"]
    c = b["config"]
    assert (c["rounds"], c["passes"], c["placed_jobs"]) == (want["rounds"], want["passes"], want["placed"])
    assert b["latency_ms"] > 0
    ph = b["phases"]
    # one process per rank reports every rank, --single-process every shard
    # (kp_last_timing_shards)
    assert ph["rounds"] == want["rounds"] and len(ph["per_rank"]) == 2
    assert ph["cand_ms"] > 0 and ph["xchg_ms"] > 0 and ph["pass_ms"] > 0
    for r in ph["per_rank"]:  # the phases of one rank sum to at most its solve
        assert r["cand_ms"] + r["xchg_ms"] + r["pass_ms"] <= r["solve_ms"] * 1.001
    if "--single-process" not in extra:  # one-GPU contexts per rank, each its row block
        sm = b["score_matrix"]
        assert sm["n_gpus"] == 2 and sum(sm["rows_per_rank"]) == J and sm["achieved"] > 0
    if config4:
        c4, g4 = b["config4"], GOLD["config4"]
        assert c4["n_gpus"] == 2 and c4["solve_ms"] > 0 and c4["preempt_ms"] > 0
        assert (c4["rounds"], c4["passes"], c4["placed_jobs"]) == \
            (g4["counts"]["rounds"], g4["counts"]["passes"], g4["counts"]["placed"])
        assert (c4["preemptors"], c4["nominated"]) == \
            (g4["preempt_counts"]["preemptors"], g4["preempt_counts"]["nominated"])
        ph4 = c4["phases"]
        assert ph4["rounds"] == g4["counts"]["rounds"] and ph4["xchg_ms"] > 0 and ph4["preempt_ms"] > 0
