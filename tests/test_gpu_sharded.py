"""The sharded solve at BASELINE config #3's full size, and
the failure paths of the multi-GPU contexts.

BASELINE configs[2] is "100k jobs x 10k nodes ... job rows sharded across
1/2/4/8 GPUs". On a one-GPU box the shards share the GPU: kp_create_multi
with a repeated id runs the sharded code (k_pack / exchange / k_unpack, the
per-rank slot bound, the replicated passes) with an in-process host
all-gather in place of ncclAllGather. Every shard count must reproduce the
oracle's placement bit for bit, with the oracle's round and pass counts.
Reference anchor: one manager process drives the placement
(cmd/manager/main.go:157-200).
"""
import os

import numpy as np
import pytest

from kplace import _abi, synth
from kplace.engine import KPlaceError, Placer

pytestmark = pytest.mark.gpu

NTH = min(16, os.cpu_count() or 1)
_CACHE = {}


def _config3_full(oracle):
    if "c3" not in _CACHE:
        w = synth.config3()
        p = _abi.default_params(**synth.CONFIG_PARAMS[3])
        _CACHE["c3"] = (w, p, oracle.place(oracle.SnapshotBuf.from_workload(w), p, nthreads=NTH))
    return _CACHE["c3"]


def _assert_same(g, o, ctx):
    for k in ("node", "score", "status", "used"):
        assert np.array_equal(g[k], o[k]), f"{ctx}: {k} differs from the oracle"
    for k in ("rounds", "passes", "placed", "unplaced", "units", "pairs"):
        assert g[k] == o[k], f"{ctx} {k}: gpu={g[k]} cpu={o[k]}"


@pytest.mark.parametrize("shards", [2, 4, 8])
def test_config3_full_sharded_in_process(oracle, shards):
    """kp_create_multi([0] * G): G row shards of the 26,525 units, one worker
    thread each, candidates exchanged once per round."""
    w, p, o = _config3_full(oracle)
    with Placer(gpu_ids=[0] * shards) as pl:
        g = pl.place(w, p)
        pl.reset_nodes()  # the staged form on the resident snapshot: same result
        st = pl.solve(p)
        g2 = pl.fetch()
    _assert_same(g, o, f"config3 full, {shards} shards")
    _assert_same(g2, o, f"config3 full, {shards} shards, staged")
    assert st["rounds"] == o["rounds"] and st["passes"] == o["passes"]


@pytest.mark.parametrize("follow", ["0", "1"])
def test_config3_full_sharded_pass_follow(oracle, monkeypatch, follow):
    """The sharded solve with host-followed passes off (every round enqueues
    max_passes) and at M = 1 (each shard's host waits for every pass flag
    before enqueueing the next pass): 4 worker threads, each following its own
    replicated passes after the round's exchange; same placement and counts."""
    monkeypatch.setenv("KP_PASS_FOLLOW", follow)
    w, p, o = _config3_full(oracle)
    with Placer(gpu_ids=[0] * 4) as pl:
        g = pl.place(w, p)
    _assert_same(g, o, f"config3 full, 4 shards, follow {follow}")


def test_create_multi_distinct_ids_beyond_the_box():
    """Distinct GPU ids take the RCCL form (ncclCommInitAll). On a box with
    fewer GPUs than ids the context must fail cleanly with KP_ENODEV, not
    hang in communicator setup."""
    import torch
    ndev = torch.cuda.device_count()
    ids = list(range(ndev + 1))
    with pytest.raises(KPlaceError) as e:
        Placer(gpu_ids=ids)
    assert e.value.code == _abi.KP_ENODEV
    with pytest.raises(KPlaceError) as e:
        Placer(gpu_ids=[0, -1])
    assert e.value.code == _abi.KP_ENODEV


@pytest.mark.parametrize("ids,fail_rank", [([0, 0], 1), ([0, 0], 0), ([0, 0, 0], 2)])
def test_create_multi_shard_failure_releases_peers(oracle, monkeypatch, ids, fail_rank):
    """One shard fails before its first exchange (KP_TEST_FAIL_SOLVE): its
    peers, waiting for that exchange, must return at once; the call reports
    the failing shard's own error (not a peer's), and the context stays
    usable: the next solve is bit-exact."""
    monkeypatch.setenv("KP_TEST_FAIL_SOLVE", str(fail_rank))
    w = synth.config3(6_000, 512)
    p = _abi.default_params(**synth.CONFIG_PARAMS[3])
    with Placer(gpu_ids=ids) as pl:
        monkeypatch.delenv("KP_TEST_FAIL_SOLVE")  # read at creation only
        pl.load_nodes(w.cap, w.used, w.topo)
        pl.load_jobs(w.req, w.prio, w.gang_id, w.gang_size)
        with pytest.raises(KPlaceError) as e:
            pl.solve(p)
        assert e.value.code == _abi.KP_ENOMEM
        assert f"shard {fail_rank}:" in e.value.detail and "KP_TEST_FAIL_SOLVE" in e.value.detail
        pl.reset_nodes()
        pl.solve(p)
        g = pl.fetch()
    o = oracle.place(oracle.SnapshotBuf.from_workload(w), p, nthreads=NTH)
    _assert_same(g, o, f"after an injected failure of shard {fail_rank}")


# ---------------------------------------------------------------------------
# BASELINE config #4 sharded: placement + preemption over row shards
# ---------------------------------------------------------------------------
def _config4(oracle, J=None, N=None):
    key = ("c4", J, N)
    if key not in _CACHE:
        w = synth.config4(J, N) if J else synth.config4()
        m = w.meta
        p = _abi.default_params(**synth.CONFIG_PARAMS[4])
        o = None
        if J:
            o = oracle.preempt(oracle.SnapshotBuf.from_workload(w), p, m["run_node"], m["run_req"],
                               m["run_prio"], nthreads=NTH)
        _CACHE[key] = (w, p, o)
    return _CACHE[key]


def _solve_preempt(pl, w, p):
    m = w.meta
    pl.load_nodes(w.cap, w.used, w.topo)
    pl.load_running(m["run_node"], m["run_req"], m["run_prio"])
    pl.load_jobs(w.req, w.prio, w.gang_id, w.gang_size)
    st = pl.solve(p)
    return st, pl.fetch(), pl.preempt()


@pytest.mark.parametrize("shards", [2, 4])
def test_config4_sharded_parity(oracle, shards):
    """kp_create_multi([0] * G) on config #4's shape (20k x 2k, 30 % occupancy):
    the candidate phase row-sharded with one exchange per round, and the
    preemption scoring row-sharded too (shard r scores preemptors
    [P r / G, P (r + 1) / G), one all-gather of the nominations). Placement,
    counts and every nomination equal the oracle's."""
    w, p, (o, opr) = _config4(oracle, 20_000, 2_000)
    with Placer(gpu_ids=[0] * shards) as pl:
        st, g, pr = _solve_preempt(pl, w, p)
    _assert_same(g, o, f"config4 20k, {shards} shards")
    for k in ("node", "victims", "cost"):
        assert np.array_equal(pr[k], opr[k]), f"config4 20k, {shards} shards: preempt {k}"
    for k in ("preemptors", "nominated", "pairs"):
        assert pr[k] == opr[k], (k, pr[k], opr[k])
    assert opr["nominated"] > 0


@pytest.mark.parametrize("shards", [2, 4])
def test_config4_full_size_sharded_digests(shards):
    """Config #4 at BASELINE size (200k x 20k) over 2 and 4 in-process shards:
    the same digests as the one-GPU run (tests/golden/large_digests.json)."""
    import hashlib
    import json

    gold = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                                       "large_digests.json")))["config4"]

    def digest(a):
        a = np.ascontiguousarray(a)
        return hashlib.sha256(a.astype(a.dtype.newbyteorder("<")).tobytes()).hexdigest()

    w = synth.config4()
    p = _abi.default_params(**synth.CONFIG_PARAMS[4])
    with Placer(gpu_ids=[0] * shards) as pl:
        st, g, pr = _solve_preempt(pl, w, p)
    assert {k: digest(g[k]) for k in ("node", "score", "status", "used")} == gold["place"]
    assert {k: digest(pr[k]) for k in ("node", "victims", "cost")} == gold["preempt"]
    assert {k: int(g[k]) for k in gold["counts"]} == gold["counts"]
    assert {k: int(pr[k]) for k in gold["preempt_counts"]} == gold["preempt_counts"]
