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
