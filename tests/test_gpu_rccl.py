"""The RCCL exchange executed on a one-GPU box (verdict r05 item 1).

Every multi-rank test elsewhere exchanges candidates host-staged or
in-process, because two ranks cannot share one GPU over RCCL. Here the
library's test knob KP_RCCL_SOLO=1 (honoured only under KP_DEBUG_KNOBS=1,
which tests/conftest.py sets) makes a ONE-rank context run the multi-rank
solve over a real one-rank RCCL communicator:

  - kp_create(world_size=1, nccl_id=...) -> ncclCommInitRank(comm, 1, id, 0);
  - kp_create_multi([0])                 -> ncclCommInitAll(comms, 1, {0});

and then, every round, the same stream order each rank of an N-GPU job runs:
k_pack -> ncclAllGather -> k_unpack, the replicated passes on the unpacked
union, and after the solve kp_preempt's one all-gather of the nominations.
Results must equal the oracle's bit for bit, and kp_timing.rccl_calls proves
the RCCL branch ran (one ncclAllGather per round, +1 per kp_preempt).
Reference anchor: one manager process drives the placement
(cmd/manager/main.go:157-200).
"""
import os

import numpy as np
import pytest

from kplace import _abi, synth
from kplace.engine import Placer, unique_id

pytestmark = pytest.mark.gpu

NTH = min(16, os.cpu_count() or 1)
_CACHE = {}


def _assert_same(g, o, ctx):
    for k in ("node", "score", "status", "used"):
        assert np.array_equal(g[k], o[k]), f"{ctx}: {k} differs from the oracle"
    for k in ("rounds", "passes", "placed", "unplaced", "units", "pairs"):
        assert g[k] == o[k], f"{ctx} {k}: gpu={g[k]} cpu={o[k]}"


def _config3_full(oracle):
    if "c3" not in _CACHE:
        w = synth.config3()
        p = _abi.default_params(**synth.CONFIG_PARAMS[3])
        _CACHE["c3"] = (w, p, oracle.place(oracle.SnapshotBuf.from_workload(w), p, nthreads=NTH))
    return _CACHE["c3"]


def _config4_small(oracle):
    if "c4" not in _CACHE:
        w = synth.config4(20_000, 2_000)
        m = w.meta
        p = _abi.default_params(**synth.CONFIG_PARAMS[4])
        o = oracle.preempt(oracle.SnapshotBuf.from_workload(w), p, m["run_node"], m["run_req"],
                           m["run_prio"], nthreads=NTH)
        _CACHE["c4"] = (w, p, o)
    return _CACHE["c4"]


@pytest.fixture
def solo(monkeypatch):
    monkeypatch.setenv("KP_RCCL_SOLO", "1")  # read at context creation


def _rank_placer():
    return Placer(device=0, world_size=1, rank=0, nccl_id=unique_id())


def _exchanges_ran(tm, rounds):
    # one all-gather per round, plus the final round that finds no active unit
    assert rounds <= tm["rccl_calls"] <= rounds + 1, (tm["rccl_calls"], rounds)


def test_rccl_rank_config3_full(oracle, solo):
    """kp_create + ncclCommInitRank(1 rank): the full 100k x 10k config #3,
    the one-shot kp_place and the staged solve, each round exchanged over
    ncclAllGather; the phase split sees the exchange."""
    w, p, o = _config3_full(oracle)
    with _rank_placer() as pl:
        g = pl.place(w, p)
        _assert_same(g, o, "config3 full, RCCL rank")
        _exchanges_ran(pl.timing(), g["rounds"])
        pl.reset_nodes()
        pl.set_profiling(2)
        st = pl.solve(p)
        tm = pl.timing()
        g2 = pl.fetch()
    _assert_same(g2, o, "config3 full, RCCL rank, staged")
    assert st["rounds"] == o["rounds"]
    _exchanges_ran(tm, st["rounds"])
    assert tm["xchg_ms"] > 0 and tm["cand_ms"] > 0 and tm["pass_ms"] > 0
    assert tm["cand_ms"] + tm["xchg_ms"] + tm["pass_ms"] <= tm["solve_ms"] * 1.001


def test_rccl_rank_config4_preempt(oracle, solo):
    """Config #4's shape (20k x 2k, 30 % occupancy) over the one-rank
    communicator: the solve and kp_preempt's all-gather of the nominations;
    placement and every nomination equal the oracle's."""
    w, p, (o, opr) = _config4_small(oracle)
    m = w.meta
    with _rank_placer() as pl:
        pl.load_nodes(w.cap, w.used, w.topo)
        pl.load_running(m["run_node"], m["run_req"], m["run_prio"])
        pl.load_jobs(w.req, w.prio, w.gang_id, w.gang_size)
        st = pl.solve(p)
        n_solve = pl.timing()["rccl_calls"]
        g = pl.fetch()
        pr = pl.preempt()
        n_all = pl.timing()["rccl_calls"]
    _assert_same(g, o, "config4 20k, RCCL rank")
    for k in ("node", "victims", "cost"):
        assert np.array_equal(pr[k], opr[k]), f"config4 20k, RCCL rank: preempt {k}"
    for k in ("preemptors", "nominated", "pairs"):
        assert pr[k] == opr[k], (k, pr[k], opr[k])
    assert opr["preemptors"] > 0
    _exchanges_ran({"rccl_calls": n_solve}, st["rounds"])
    assert n_all == n_solve + 1  # kp_preempt: one all-gather


def test_rccl_multi_one_gpu_config3_full(oracle, solo):
    """kp_create_multi([0]) + ncclCommInitAll(1 GPU): the single-process form
    the manager uses, its worker thread and its RCCL
    exchange, on the full config #3; per-shard timing from
    kp_last_timing_shards."""
    w, p, o = _config3_full(oracle)
    with Placer(gpu_ids=[0]) as pl:
        g = pl.place(w, p)
        shards = pl.timing_shards()
    _assert_same(g, o, "config3 full, kp_create_multi([0]) over RCCL")
    assert len(shards) == 1
    _exchanges_ran(shards[0], g["rounds"])


def test_rccl_multi_one_gpu_config4_preempt(oracle, solo):
    w, p, (o, opr) = _config4_small(oracle)
    m = w.meta
    with Placer(gpu_ids=[0]) as pl:
        pl.load_nodes(w.cap, w.used, w.topo)
        pl.load_running(m["run_node"], m["run_req"], m["run_prio"])
        pl.load_jobs(w.req, w.prio, w.gang_id, w.gang_size)
        pl.solve(p)
        g = pl.fetch()
        pr = pl.preempt()
        assert pl.timing()["rccl_calls"] > 1
    _assert_same(g, o, "config4 20k, kp_create_multi([0]) over RCCL")
    for k in ("node", "victims", "cost"):
        assert np.array_equal(pr[k], opr[k]), f"preempt {k}"


def test_no_rccl_without_the_knob(oracle):
    """Without KP_RCCL_SOLO a one-rank context ignores the id: the one-GPU
    solve, no communicator, no all-gather."""
    w = synth.config3(6_000, 512)
    p = _abi.default_params(**synth.CONFIG_PARAMS[3])
    with _rank_placer() as pl:
        g = pl.place(w, p)
        assert pl.timing()["rccl_calls"] == 0
    o = oracle.place(oracle.SnapshotBuf.from_workload(w), p, nthreads=NTH)
    _assert_same(g, o, "one rank, no knob")


def test_multi_timing_is_max_over_shards(oracle):
    """kp_last_timing on a kp_create_multi context: every time field is the
    slowest shard's, the byte counts the sum; kp_last_timing_shards returns
    one entry per shard."""
    w = synth.config3(20_000, 2_000)
    p = _abi.default_params(**synth.CONFIG_PARAMS[3])
    with Placer(gpu_ids=[0, 0, 0]) as pl:
        pl.load_nodes(w.cap, w.used, w.topo)
        pl.load_jobs(w.req, w.prio, w.gang_id, w.gang_size)
        pl.set_profiling(2)
        pl.solve(p)
        sh = pl.timing_shards()
        tm = pl.timing()
    assert len(sh) == 3
    for k in ("solve_ms", "score_ms", "cand_ms", "xchg_ms", "pass_ms"):
        assert tm[k] == max(s[k] for s in sh), k
    for k in ("score_bytes", "score_launches"):
        assert tm[k] == sum(s[k] for s in sh), k
    assert all(s["xchg_ms"] > 0 and s["rccl_calls"] == 0 for s in sh)  # in-process exchange
