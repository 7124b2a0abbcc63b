"""BASELINE configs #3 (runner), #4 and #5 at their stated sizes on the GPU.

Parity: against SHA-256 digests of the CPU oracle's outputs on the same
seeded snapshots, computed in the build container by
tests/golden/make_large.py (config #4 placement + preemption; the first 3
micro-batches of config #5), plus size-independent properties over the whole
run: capacity, all-or-nothing, usage == the replayed sum of placements minus
completions, nominees are NO_FIT singletons with a non-empty victim set.
"""
import hashlib
import json
import os
import time

import numpy as np
import pytest

from kplace import _abi, binder, metrics, packer, runner, synth
from kplace.engine import Placer

pytestmark = pytest.mark.gpu

GOLD = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                                   "large_digests.json")))


def digest(a) -> str:
    a = np.ascontiguousarray(a)
    return hashlib.sha256(a.astype(a.dtype.newbyteorder("<")).tobytes()).hexdigest()


def test_score_dev_full_size_config3():
    """kp_score_dev over the WHOLE config #3 queue (100k x 10k, the bench's
    score_matrix leg) into caller device buffers: the score matrix and the
    feasibility bitmask equal the oracle's (kpo_score) SHA-256 digests; the
    padding columns are infeasible; the score-only and mask-only kernel
    instances write the same bytes."""
    from kplace.devmem import DeviceBuffer
    w = synth.config3()
    g3 = GOLD["config3_score"]
    assert {k: digest(v) for k, v in dict(req=w.req, cap=w.cap, used=w.used).items()} == g3["inputs"]
    p = _abi.default_params(**synth.CONFIG_PARAMS[3])
    J, N = w.J, w.N
    Ns = (N + 63) // 64 * 64
    words, uw = Ns // 64, (N + 63) // 64
    chunk = 5_000
    with DeviceBuffer(J * Ns * 4) as sc, DeviceBuffer(J * words * 8) as mk, \
            DeviceBuffer(J * Ns * 4, fill=0) as sc2, DeviceBuffer(J * words * 8, fill=0) as mk2:
        with Placer(device=0) as pl:
            pl.load_nodes(w.cap, w.used, w.topo)
            pl.load_jobs(w.req, w.prio, w.gang_id, w.gang_size)
            pl.set_profiling(True)
            pl.score_dev(p, 0, J, sc.ptr, mk.ptr)
            t = pl.timing()
            pl.score_dev(p, 0, J, sc2.ptr, None)
            pl.score_dev(p, 0, J, None, mk2.ptr)
        print(f"kp_score_dev full config #3: {t['score_ms']:.3f} ms, {t['score_launches']} launch(es)")
        hs, hm = hashlib.sha256(), hashlib.sha256()
        feasible = 0
        for lo in range(0, J, chunk):
            n = min(chunk, J - lo)
            a = sc.to_numpy(np.int32, (n, Ns), offset=lo * Ns * 4)
            assert (a[:, N:] == -1).all()
            assert np.array_equal(a, sc2.to_numpy(np.int32, (n, Ns), offset=lo * Ns * 4))
            m = mk.to_numpy(np.uint64, (n, words), offset=lo * words * 8)
            assert np.array_equal(m, mk2.to_numpy(np.uint64, (n, words), offset=lo * words * 8))
            hs.update(np.ascontiguousarray(a[:, :N]).astype("<i4").tobytes())
            hm.update(np.ascontiguousarray(m[:, :uw]).astype("<u8").tobytes())
            feasible += int((a[:, :N] >= 0).sum())
    assert feasible == g3["feasible_pairs"]
    assert hs.hexdigest() == g3["score"] and hm.hexdigest() == g3["mask"]


def test_config4_full_size_parity_and_properties():
    w = synth.config4()
    m = w.meta
    g4 = GOLD["config4"]
    ins = dict(req=w.req, cap=w.cap, used=w.used, prio=w.prio, run_node=m["run_node"],
               run_req=m["run_req"], run_prio=m["run_prio"])
    assert {k: digest(v) for k, v in ins.items()} == g4["inputs"], "config #4 generator changed"
    util = w.used.sum(1) / w.cap.sum(1)
    assert (util >= 0.30).all(), util  # >= 0.30 in every dim
    p = _abi.default_params(**synth.CONFIG_PARAMS[4])
    with Placer(device=0) as pl:
        pl.load_nodes(w.cap, w.used, w.topo)
        pl.load_running(m["run_node"], m["run_req"], m["run_prio"])
        pl.load_jobs(w.req, w.prio, w.gang_id, w.gang_size)
        t = time.perf_counter()
        st = pl.solve(p)
        g = pl.fetch()
        pr = pl.preempt()
        dt = time.perf_counter() - t
    print(f"config4 GPU solve+fetch+preempt {dt * 1e3:.1f} ms, {st}")
    assert {k: digest(g[k]) for k in ("node", "score", "status", "used")} == g4["place"]
    assert {k: digest(pr[k]) for k in ("node", "victims", "cost")} == g4["preempt"]
    assert {k: int(g[k]) for k in g4["counts"]} == g4["counts"]
    assert {k: int(pr[k]) for k in g4["preempt_counts"]} == g4["preempt_counts"]
    # properties
    placed = g["node"] >= 0
    used = w.used.copy()
    np.add.at(used.T, g["node"][placed], w.req[:, placed].T)
    assert np.array_equal(used, g["used"]) and (g["used"] <= w.cap).all()
    nom = pr["node"] >= 0
    assert (g["status"][nom] == _abi.KP_JOB_NO_FIT).all() and (pr["victims"][nom] >= 1).all()
    assert ((g["status"] == _abi.KP_JOB_PLACED) == placed).all()


def test_config5_full_trace_parity_and_properties():
    """The whole 1M-job trace in 5k micro-batches against 50k nodes; the first
    3 batches bit-exact against the oracle's digests, every batch checked for
    capacity and usage == replayed placements - completions."""
    total, N, B = 1_000_000, 50_000, 5_000
    cap, topo, req, prio = synth.config5_trace(total, N)
    g5 = GOLD["config5"]
    assert {"cap": digest(cap), "req": digest(req), "prio": digest(prio)} == g5["inputs"]
    p = _abi.default_params(**synth.CONFIG_PARAMS[5])
    used_h = np.zeros_like(cap)
    run_node = np.zeros(0, np.int32)
    run_job = np.zeros(0, np.int64)
    lat = []
    placed_total = 0
    with Placer(device=0) as pl:
        pl.load_nodes(cap, None, topo)
        for b in range(total // B):
            lo, hi = b * B, (b + 1) * B
            rq = np.ascontiguousarray(req[:, lo:hi])
            t = time.perf_counter()
            pl.load_jobs(rq, prio[lo:hi])
            st = pl.solve(p)
            g = pl.fetch()
            lat.append(time.perf_counter() - t)
            ok = g["node"] >= 0
            placed_total += int(ok.sum())
            np.add.at(used_h.T, g["node"][ok], rq[:, ok].T)
            assert np.array_equal(g["used"], used_h), f"batch {b}: usage drifted"
            assert (g["used"] <= cap).all(), f"batch {b}: capacity exceeded"
            assert ((g["status"] == _abi.KP_JOB_PLACED) == ok).all()
            if b < len(g5["batches"]):
                want = g5["batches"][b]
                assert {k: digest(g[k]) for k in ("node", "score", "status", "used")} == \
                    {k: want[k] for k in ("node", "score", "status", "used")}, f"batch {b}"
                assert {k: int(st[k]) for k in want["counts"]} == want["counts"], f"batch {b}"
            run_node = np.concatenate([run_node, g["node"][ok]])
            run_job = np.concatenate([run_job, lo + np.nonzero(ok)[0]])
            done = synth.config5_completions(b, run_job)
            if done.any():
                pl.apply_delta(run_node[done], -req[:, run_job[done]])
                np.subtract.at(used_h.T, run_node[done], req[:, run_job[done]].T)
            run_node, run_job = run_node[~done], run_job[~done]
        assert np.array_equal(pl.fetch()["used"], used_h)
    ms = np.array(lat) * 1e3
    print(f"config5: {placed_total} placed, per-batch p50 {np.percentile(ms, 50):.2f} ms "
          f"p99 {np.percentile(ms, 99):.2f} ms (load+solve+fetch incl. used)")


def test_config3_runner_gpu():
    """The host path at config #3 scale: 26,525 LLMService CRs (every 5th with
    CacheStrategy shared and a coordinator) + 10k Node reports through
    packer -> kp_place (GPU) -> binder, one batch, latency in the metrics
    histogram; the placement equals a direct kp_place of the packed snapshot."""
    w = synth.config3()
    crs, nodes, pods = synth.workload_objects(w, shared_every=5)
    written = {}
    m = metrics.PlacementMetrics()
    p = _abi.default_params(**synth.CONFIG_PARAMS[3])
    with Placer(device=0) as pl:
        r = runner.BatchRunner(pl, lambda: crs, lambda: nodes,
                               lambda k, st: written.__setitem__(k, st), p, metrics=m,
                               pod_nodes=lambda: pods)
        r.reconcile(("default", "llm-0"))
        s = r.run_batch()
        pk = packer.pack(crs, nodes, pod_nodes=pods)
        direct = pl.place(pk.workload, p)
    assert s["crs"] == len(crs) == 26_525 and s["invalid_crs"] == 0
    assert len(written) == len(crs)
    assert m.batch_latency._sum.get() > 0  # one observation, the batch's wall time
    assert s["placed"] == direct["placed"]
    n_true = sum(v["conditions"][0]["status"] == "True" for v in written.values())
    conds = binder.conditions(pk, direct, now="t")
    assert n_true == sum(c["status"] == "True" for c in conds.values())
    aff = pk.workload.affinity
    placed = direct["node"] >= 0
    hit = (pk.workload.topo[direct["node"][placed & (aff >= 0)]] == aff[placed & (aff >= 0)]).mean()
    print(f"runner batch {s['seconds'] * 1e3:.1f} ms, placed {s['placed']}, "
          f"shared replicas in the coordinator's domain {hit:.2f}")
