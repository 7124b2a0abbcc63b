"""GPU parity of the incremental candidate phase (kp_incr.hip).

A measured alternative (KP_INCR=1; off by default): rounds
after the first re-score only the nodes the previous round changed,
against per-unit top-KL lists with a bound; rows the lists cannot answer are
rescanned in full. Bar: bit-exact node / score / status / usage and equal
round / pass counts against the oracle (which scans every node every round),
for every mix of incremental rows, rescanned rows and full-scan rounds.
"""
import numpy as np
import pytest

from kplace import _abi, synth
from kplace.engine import Placer

from test_gpu_parity import NTH, _assert_same, _snap, few_class_workload

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _incr_on(monkeypatch):
    monkeypatch.setenv("KP_INCR", "1")  # a measured alternative, off by default


def _place(w, p):
    with Placer(device=0) as pl:
        g = pl.place(w, p)
        t = pl.timing()
        g2 = pl.place(w, p)  # the lists are rebuilt by the next solve's first round
    return g, g2, t


INCR_CASES = [  # (D, score_mode, tie_mode, n_cand, N, classes, seed)
    (4, 0, 1, 16, 3000, 5, 1), (4, 1, 1, 16, 2000, 3, 2), (1, 0, 0, 1, 700, 3, 3),
    (2, 1, 0, 4, 1025, 2, 4), (3, 0, 1, 32, 2100, 9, 5), (4, 0, 0, 8, 640, 4, 6),
    (8, 1, 1, 16, 1500, 6, 7), (4, 1, 0, 5, 4100, 1, 8),
]


@pytest.mark.parametrize("case", range(len(INCR_CASES)))
def test_incr_parity(oracle, case):
    """Incremental rounds on few-class snapshots: dims 1..8, both score modes
    (LeastAllocated scores fall where usage grows, MostAllocated ones rise),
    both tie modes, K in {1..32} (K = 32: the list holds exactly K, so any
    changed entry forces a rescan), gangs, affinity."""
    D, mode, tie, K, N, classes, seed = INCR_CASES[case]
    w = few_class_workload(700 + seed, J=3000, N=N, D=D, classes=classes)
    p = _abi.default_params(score_mode=mode, tie_mode=tie, n_cand=K, gpu_dim=D - 1,
                            w_dim=[(3 * d + 1) % 7 for d in range(8)], util_scale=[100, 7, 1024][case % 3])
    g, g2, t = _place(w, p)
    o = oracle.place(_snap(oracle, w), p, nthreads=NTH)
    assert t["fused"] == 1
    # rounds after the first (+ the trailing empty round the host enqueues)
    assert t["incr_rounds"] >= o["rounds"] - 1, t
    _assert_same(g, o, f"incr case {case}")
    _assert_same(g2, o, f"incr case {case}, second solve")


@pytest.mark.parametrize("div", ["1", "1000000"])
def test_incr_rescan_thresholds(oracle, monkeypatch, div):
    """KP_INCR_CTHR_DIV: 1 = never a full rescan round (every changed-node
    count is re-scored incrementally, up to N); 1,000,000 = rounds with more
    than 64 changed nodes rescan every row, the others update incrementally."""
    monkeypatch.setenv("KP_INCR_CTHR_DIV", div)
    w = synth.config3(20_000, 2_000)
    p = _abi.default_params(**synth.CONFIG_PARAMS[3])
    g, g2, t = _place(w, p)
    o = oracle.place(_snap(oracle, w), p, nthreads=NTH)
    _assert_same(g, o, f"cthr div {div}")
    _assert_same(g2, o, f"cthr div {div}, second solve")


def test_incr_off_equals_on(oracle, monkeypatch):
    """KP_INCR=0 (every round a full scan) and the default give the same
    placement as the oracle on config #4's shape (singletons, 4 shapes,
    priority tiers, 30 % occupancy), reduced to 20k x 2k."""
    w = synth.config4(20_000, 2_000)
    p = _abi.default_params(**synth.CONFIG_PARAMS[4])
    g, _, t = _place(w, p)
    monkeypatch.setenv("KP_INCR", "0")
    g0, _, t0 = _place(w, p)
    o = oracle.place(_snap(oracle, w), p, nthreads=NTH)
    assert t0["incr_rounds"] == 0 and t["incr_rounds"] >= o["rounds"] - 1
    _assert_same(g, o, "config4 20k incremental")
    _assert_same(g0, o, "config4 20k full scans")


def test_incr_streaming_batches(oracle):
    """Config #5's shape: consecutive solves against a resident table with
    completions applied between them; every batch's first round is a full
    scan, the lists never leak across solves."""
    cap, topo, req, prio = synth.config5_trace(20_000, 3_000)
    p = _abi.default_params(**synth.CONFIG_PARAMS[5])
    B = 2_000
    used = np.zeros_like(cap)
    with Placer(device=0) as pl:
        pl.load_nodes(cap, None, topo)
        run_node, run_job = np.zeros(0, np.int32), np.zeros(0, np.int64)
        for b in range(4):
            lo, hi = b * B, (b + 1) * B
            rq = np.ascontiguousarray(req[:, lo:hi])
            pl.load_jobs(rq, prio[lo:hi])
            pl.solve(p)
            g = pl.fetch(want_used=True)
            o = oracle.place(oracle.SnapshotBuf(rq, cap, used, prio[lo:hi], topo=topo), p, nthreads=NTH)
            for k in ("node", "score", "status"):
                assert np.array_equal(g[k], o[k]), f"batch {b} {k}"
            assert np.array_equal(g["used"], o["used"]), f"batch {b} used"
            used = o["used"].copy()
            ok = g["node"] >= 0
            run_node = np.concatenate([run_node, g["node"][ok]])
            run_job = np.concatenate([run_job, lo + np.nonzero(ok)[0]])
            done = synth.config5_completions(b, run_job)
            if done.any():
                dn = np.ascontiguousarray(run_node[done])
                dd = np.ascontiguousarray(-req[:, run_job[done]])
                pl.apply_delta(dn, dd)
                np.add.at(used.T, dn, dd.T)
            run_node, run_job = run_node[~done], run_job[~done]


def test_incr_many_changed_nodes(oracle, monkeypatch):
    """More changed nodes per round than one re-scoring sweep (64) and more
    re-scored keys above the bound than the per-wave buffer holds: rows fall
    back to the rescan list inside an incremental round."""
    monkeypatch.setenv("KP_INCR_CTHR_DIV", "1")
    w = few_class_workload(991, J=6000, N=3000, D=4, classes=2, used_frac=0.1, affinity=False)
    p = _abi.default_params(n_cand=32, score_mode=0)
    g, g2, t = _place(w, p)
    o = oracle.place(_snap(oracle, w), p, nthreads=NTH)
    _assert_same(g, o, "many changed nodes")
    _assert_same(g2, o, "many changed nodes, second solve")
