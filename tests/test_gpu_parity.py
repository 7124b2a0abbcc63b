"""GPU parity: libkplace.so (HIP, gfx950) against the CPU oracle.

Bar: bit-exact (integer path) — node_of_job, score_of_job, status_of_job,
used_out and the round/pass counts must equal the oracle's on the same
seeded snapshot. At BASELINE sizes the oracle still finishes (OpenMP), and
size-independent properties (capacity, gang all-or-nothing, determinism) are
checked on top.
"""
import os

import numpy as np
import pytest

from kplace import _abi, synth
from kplace.engine import KPlaceError, Placer

pytestmark = pytest.mark.gpu

NTH = min(16, os.cpu_count() or 1)


def _snap(ob, w):
    return ob.SnapshotBuf.from_workload(w)


def _assert_same(g, o, ctx=""):
    for k in ("node", "score", "status"):
        bad = np.nonzero(g[k] != o[k])[0]
        assert bad.size == 0, f"{ctx} {k} differs at {bad[:10]}: gpu={g[k][bad[:10]]} cpu={o[k][bad[:10]]}"
    assert np.array_equal(g["used"], o["used"]), f"{ctx} used_out differs"
    for k in ("rounds", "passes", "placed", "unplaced", "units", "pairs"):
        assert g[k] == o[k], f"{ctx} {k}: gpu={g[k]} cpu={o[k]}"


def random_workload(seed, J, N, D=4, gangs=True, used_frac=0.3, zero_dims=True, max_gang=8,
                    prio_levels=4):
    rng = np.random.default_rng(seed)
    cap = rng.integers(0, 64, size=(D, N)).astype(np.int64) * rng.choice([1, 7, 1000], size=(D, 1))
    if zero_dims:
        cap[:, rng.random(N) < 0.1] = 0          # dead nodes
        cap[rng.integers(0, D), rng.random(N) < 0.2] = 0
    used = (cap * rng.random((D, N)) * used_frac).astype(np.int64)
    sizes = []
    tot = 0
    while tot < J:
        s = int(rng.integers(1, max_gang + 1)) if gangs and rng.random() < 0.4 else 1
        s = min(s, J - tot)
        sizes.append(s)
        tot += s
    sizes = np.array(sizes)
    ncr = len(sizes)
    req_cr = (rng.integers(0, 16, size=(D, ncr)) * rng.choice([1, 7, 1000], size=(D, 1))).astype(np.int64)
    req_cr[:, rng.random(ncr) < 0.05] = 0         # zero-request jobs
    prio_cr = rng.integers(0, prio_levels, size=ncr).astype(np.int32)
    cr = np.repeat(np.arange(ncr), sizes)
    gid = np.where(np.repeat(sizes, sizes) > 1, cr, -1).astype(np.int32) if gangs else np.full(J, -1, np.int32)
    return synth.Workload(J, N, D, np.ascontiguousarray(req_cr[:, cr]), cap, used,
                          prio_cr[cr], gid, np.repeat(sizes, sizes).astype(np.int32),
                          (np.arange(N) // 5).astype(np.int32), name=f"rand{seed}")


# ---------------------------------------------------------------------------
# filter + score matrix (kp_score) — the materialised outputs
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("scale", [100, 1024, 7])
def test_score_matrix_parity(oracle, placer, mode, scale):
    w = random_workload(11 + mode + scale, J=300, N=333, gangs=False)
    p = _abi.default_params(score_mode=mode, util_scale=scale)
    placer.load_nodes(w.cap, w.used, w.topo)
    placer.load_jobs(w.req)
    sc, mk = placer.score(p, 0, w.J)
    osc, omk = oracle.score(oracle.SnapshotBuf(w.req, w.cap, w.used, topo=w.topo), p, 0, w.J)
    assert np.array_equal(sc, osc)
    assert np.array_equal(mk, omk)
    assert np.array_equal(sc >= 0, np.unpackbits(mk.view(np.uint8), axis=1, bitorder="little")[:, :w.N] == 1)


def wide_workload(seed, J, N, D=4, top=32):
    """Caps and requests across the 32-bit range (top = log2 bound): per dim
    some waves hold only caps < 2^24 (full-rate 24-bit multiply), some caps up
    to 2^top (quarter-rate path), some tiny caps <= S (the R-hi term); gangs of
    up to 8 members so member-count products exceed 2^32 when top = 32."""
    rng = np.random.default_rng(seed)
    hi = np.int64(1) << np.int64(top)
    cap = np.empty((D, N), np.int64)
    for d in range(D):
        kind = rng.integers(0, 3, size=N)
        cap[d] = np.where(kind == 0, rng.integers(0, 100, size=N),
                          np.where(kind == 1, rng.integers(1 << 20, 1 << 24, size=N),
                                   rng.integers(1 << 24, hi, size=N)))
        cap[d, :N // 3] = rng.integers(1 << 10, 1 << 23, size=N // 3)  # whole fast-24 waves
    used = (cap * rng.random((D, N)) * 0.4).astype(np.int64)
    w = random_workload(seed, J, N, D=D)
    scale = rng.choice([1, 1 << 8, 1 << 16, 1 << 22], size=(D, 1))
    req = np.minimum(w.req * scale, hi - 1)
    # identical requests within a gang (random_workload's CR structure)
    return synth.Workload(J, N, D, np.ascontiguousarray(req), cap, used, w.prio, w.gang_id,
                          w.gang_size, w.topo, name=f"wide{seed}")


@pytest.mark.parametrize("top", [31, 32])
@pytest.mark.parametrize("mode", [0, 1])
def test_score_matrix_wide_32bit(oracle, placer, top, mode):
    w = wide_workload(40 + top + mode, J=200, N=1500, top=top)
    p = _abi.default_params(score_mode=mode)
    placer.load_nodes(w.cap, w.used, w.topo)
    placer.load_jobs(w.req)
    sc, mk = placer.score(p, 0, w.J)
    osc, omk = oracle.score(oracle.SnapshotBuf(w.req, w.cap, w.used, topo=w.topo), p, 0, w.J)
    assert np.array_equal(sc, osc) and np.array_equal(mk, omk)


@pytest.mark.parametrize("seed", range(4))
def test_place_wide_32bit_parity(oracle, placer, seed):
    # full placements on the 32-bit score / plan paths with wide values
    w = wide_workload(seed, J=1500, N=400, top=31 + seed % 2)
    assert int(w.cap.max()) < (1 << 32) and int(w.req.max()) < (1 << 32)
    p = _abi.default_params(score_mode=seed % 2, util_scale=[100, 1024, 7, 100][seed])
    g, o = _place_both(oracle, placer, w, p)
    _assert_same(g, o, f"wide seed {seed}")


@pytest.mark.parametrize("D", [1, 2, 3, 5, 8])
def test_score_matrix_dims(oracle, placer, D):
    w = random_workload(100 + D, J=130, N=200, D=D, gangs=False)
    p = _abi.default_params(gpu_dim=D - 1, w_dim=[(3 * d + 1) % 7 for d in range(8)])
    placer.load_nodes(w.cap, w.used, w.topo)
    placer.load_jobs(w.req)
    sc, mk = placer.score(p, 5, 120)
    osc, omk = oracle.score(oracle.SnapshotBuf(w.req, w.cap, w.used, topo=w.topo), p, 5, 120)
    assert np.array_equal(sc, osc) and np.array_equal(mk, omk)


def test_score_matrix_large_values(oracle, placer):
    # caps beyond 2^32 exercise the 64-bit reciprocal path
    rng = np.random.default_rng(5)
    D, N, J = 4, 257, 64
    cap = rng.integers(1, 1 << 50, size=(D, N), dtype=np.int64)
    used = (cap // rng.integers(2, 9, size=(D, N))).astype(np.int64)
    req = rng.integers(0, 1 << 48, size=(D, J), dtype=np.int64)
    p = _abi.default_params(util_scale=1024)
    placer.load_nodes(cap, used)
    placer.load_jobs(req)
    sc, mk = placer.score(p, 0, J)
    osc, omk = oracle.score(oracle.SnapshotBuf(req, cap, used), p, 0, J)
    assert np.array_equal(sc, osc) and np.array_equal(mk, omk)


# ---------------------------------------------------------------------------
# full placement (kp_place)
# ---------------------------------------------------------------------------
def _place_both(oracle, placer, w, p):
    g = placer.place(w, p)
    o = oracle.place(_snap(oracle, w), p, nthreads=NTH)
    return g, o


@pytest.mark.parametrize("seed", range(6))
def test_place_random_parity(oracle, placer, seed):
    w = random_workload(seed, J=700 + 37 * seed, N=90 + 11 * seed)
    p = _abi.default_params(tie_mode=seed % 2, score_mode=(seed // 2) % 2,
                            n_cand=[16, 4, 32, 1, 8, 16][seed], max_passes=[16, 3, 64, 1, 8, 16][seed])
    g, o = _place_both(oracle, placer, w, p)
    _assert_same(g, o, f"seed {seed}")


@pytest.mark.parametrize("spread", [3, 1 << 30])
def test_place_priority_range_parity(oracle, placer, spread):
    """Unit rank order (prio desc, leader asc) by the host's counting sort
    (priorities within a small range) and by its comparison-sort fallback."""
    w = random_workload(77, J=1200, N=150)
    rng = np.random.default_rng(5)
    cr = np.cumsum(np.r_[1, (w.gang_id[1:] != w.gang_id[:-1]) | (w.gang_id[1:] < 0)]) - 1
    pcr = rng.integers(-spread, spread + 1, size=int(cr.max()) + 1).astype(np.int32)
    w = synth.Workload(w.J, w.N, w.D, w.req, w.cap, w.used, pcr[cr], w.gang_id, w.gang_size,
                       w.topo, name=f"prio{spread}")
    p = _abi.default_params()
    g, o = _place_both(oracle, placer, w, p)
    _assert_same(g, o, f"priority spread {spread}")


def test_place_config2_parity(oracle, placer):
    w = synth.config2(10_000, 1_000)
    p = _abi.default_params(**synth.CONFIG_PARAMS[2])
    g, o = _place_both(oracle, placer, w, p)
    _assert_same(g, o, "config2")


def test_place_config3_small_parity(oracle, placer):
    w = synth.config3(20_000, 2_000)
    p = _abi.default_params(**synth.CONFIG_PARAMS[3])
    g, o = _place_both(oracle, placer, w, p)
    _assert_same(g, o, "config3 20k")


@pytest.mark.parametrize("knob,n_cand,tie", [
    (("KP_SELECT_LDS_CAP", "33"), 16, 1),   # threshold select, threshold-raise path
    (("KP_SELECT_LDS_CAP", "33"), 32, 0),
    (("KP_SELECT_GENERIC", "1"), 16, 1),    # generic per-lane top-K select
    (("KP_SELECT_GENERIC", "1"), 5, 0),
])
def test_select_paths_parity(oracle, monkeypatch, knob, n_cand, tie):
    """Every top-K select form gives the oracle's candidates (checked through
    the whole placement, which depends on every candidate list)."""
    monkeypatch.setenv(*knob)
    w = synth.config3(6_000, 600)
    p = _abi.default_params(**synth.CONFIG_PARAMS[3], n_cand=n_cand, tie_mode=tie)
    with Placer(device=0) as pl:
        g = pl.place(w, p)
    o = oracle.place(_snap(oracle, w), p, nthreads=NTH)
    _assert_same(g, o, f"{knob} K={n_cand}")


@pytest.mark.parametrize("knobs", [
    (("KP_SCORE_WG_TARGET", "64"),),                                 # 128 rows per workgroup
    (("KP_SCORE_WG_TARGET", "1000000"), ("KP_SCORE_MIN_RPB", "1")),  # one row per workgroup
    (("KP_SCORE_NPL", "4"),),                                        # 4 nodes per lane
    (("KP_SCORE_NPL", "4"), ("KP_SCORE_MIN_RPB", "3")),              # ragged last row block
])
def test_score_geometry_parity(oracle, monkeypatch, knobs):
    """Every filter+score launch geometry (rows per workgroup, nodes per lane)
    gives the oracle's placement; N = 1,500 leaves a partial node tile."""
    for k, v in knobs:
        monkeypatch.setenv(k, v)
    w = synth.config3(7_000, 1_500)
    p = _abi.default_params(**synth.CONFIG_PARAMS[3])
    with Placer(device=0) as pl:
        g = pl.place(w, p)
    o = oracle.place(_snap(oracle, w), p, nthreads=NTH)
    _assert_same(g, o, f"score geometry {knobs}")


@pytest.mark.parametrize("cmax", ["0", "3000"])
def test_active_compaction_paths_parity(oracle, monkeypatch, cmax):
    """The multi-workgroup form of the active-unit compaction (chunk counts +
    chunk scatter; every round, or only the large early rounds) gives the
    same placement as the one-workgroup kernel and the oracle."""
    monkeypatch.setenv("KP_COMPACT_MAX", cmax)
    w = synth.config3(20_000, 1_000)
    p = _abi.default_params(**synth.CONFIG_PARAMS[3])
    with Placer(device=0) as pl:
        g = pl.place(w, p)
    o = oracle.place(_snap(oracle, w), p, nthreads=NTH)
    _assert_same(g, o, f"KP_COMPACT_MAX={cmax}")


@pytest.mark.parametrize("cmax", ["0"])
def test_preempt_compaction_paths_parity(oracle, monkeypatch, cmax):
    """kp_preempt's preemptor list (and every round's active units) through
    the multi-workgroup compaction (2 chunks of 16,384 flags) equals the
    oracle's nominations (config #4's shape, 1/10 size)."""
    monkeypatch.setenv("KP_COMPACT_MAX", cmax)
    w = synth.config4(20_000, 2_000)
    p = _abi.default_params(**synth.CONFIG_PARAMS[4])
    m = w.meta
    with Placer(device=0) as pl:
        g, gp, o, op = _preempt_both(oracle, pl, w, p, m["run_node"], m["run_req"], m["run_prio"])
    _assert_same(g, o, f"config4 KP_COMPACT_MAX={cmax}")
    _assert_same_pre(gp, op, f"config4 KP_COMPACT_MAX={cmax}")


@pytest.mark.parametrize("knobs", [
    (("KP_CSR_SORT", "1"),),            # every round's bidder index by the radix sort
    (("KP_CSR_BM_MAX", "40000"),),      # large early rounds sort, later rounds count
    (("KP_KEYS_MERGE", "0"), ("KP_ROUND_BEGIN", "0")),  # k_csr_keys, k_round_start + k_compact launches
    (("KP_ACC_WAVES", "0"),),           # one accept wave per listed node
    (("KP_ACC_WAVES", "64"),),          # accept grid-stride over many nodes per wave
    (("KP_ACC_LIST", "0"),),            # accept walks every node once entries >= nodes
])
def test_csr_build_paths_parity(oracle, monkeypatch, knobs):
    """The node -> bidder index is the same whether built by counting (slot
    bitmap + row ranks, the default) or by the radix sort, also when a solve
    switches between them from round to round."""
    for k, v in knobs:
        monkeypatch.setenv(k, v)
    w = synth.config3(20_000, 2_000)
    p = _abi.default_params(**synth.CONFIG_PARAMS[3])
    with Placer(device=0) as pl:
        g = pl.place(w, p)
        g2 = pl.place(w, p)  # the bitmap is all-zero again after a solve
    o = oracle.place(_snap(oracle, w), p, nthreads=NTH)
    _assert_same(g, o, f"csr {knobs}")
    _assert_same(g2, o, f"csr {knobs} second solve")


@pytest.mark.parametrize("M", ["0", "1", "2", "3", "15", "16"])
@pytest.mark.parametrize("cfg", [(3, 20_000, 2_000, 16), (4, 8_000, 1_500, 16), (2, 6_000, 600, 3)])
def test_pass_follow_parity(oracle, monkeypatch, M, cfg):
    """Host-followed passes (KP_PASS_FOLLOW = M): pass p is enqueued only once
    pass p - M's flag, stored by k_accept into coherent host memory, shows
    proposals. M = 0 and M >= max_passes enqueue every pass; M = 1 waits for
    each pass before the next. Same placement, rounds and passes as the oracle,
    a second solve too (the flags are tagged with the round serial, so stale
    flags of the previous solve never end a round)."""
    monkeypatch.setenv("KP_PASS_FOLLOW", M)
    no, J, N, max_passes = cfg
    w = synth.config(no, J, N)
    p = _abi.default_params(**{**synth.CONFIG_PARAMS[no], "max_passes": max_passes})
    with Placer(device=0) as pl:
        g = pl.place(w, p)
        g2 = pl.place(w, p)
    o = oracle.place(_snap(oracle, w), p, nthreads=NTH)
    _assert_same(g, o, f"pass follow M {M} cfg {cfg}")  # incl. rounds and passes
    _assert_same(g2, o, f"pass follow M {M} cfg {cfg}, second solve")


@pytest.mark.parametrize("seed", range(4))
def test_accept_long_row_form_parity(oracle, monkeypatch, seed):
    """k_accept's long-row form (KP_ACC_BIG flagged windows per load round
    trip; chosen when A*K >= KP_ACC_BIG_RATIO * N) forced on every round
    (ratio 1) of random gang snapshots and of config #4's shape, both N32 and
    64-bit first-fit sums (caps >= 2^26 in seed 3)."""
    monkeypatch.setenv("KP_ACC_BIG_RATIO", "1")
    if seed == 2:
        w = synth.config4(20_000, 2_000)
        p = _abi.default_params(**synth.CONFIG_PARAMS[4])
    else:
        w = random_workload(500 + seed, J=4000, N=300, max_gang=8)
        if seed == 3:
            w = synth.Workload(w.J, w.N, w.D, w.req * (1 << 22), w.cap * (1 << 22), w.used * (1 << 22),
                               w.prio, w.gang_id, w.gang_size, w.topo, name="rand_big_caps")
        p = _abi.default_params(score_mode=seed % 2, n_cand=[16, 8, 16, 32][seed])
    with Placer(device=0) as pl:
        g = pl.place(w, p)
        g2 = pl.place(w, p)
    o = oracle.place(_snap(oracle, w), p, nthreads=NTH)
    _assert_same(g, o, f"accept long-row form seed {seed}")
    _assert_same(g2, o, f"accept long-row form seed {seed}, second solve")


@pytest.mark.parametrize("win", ["1", "2", "8"])
@pytest.mark.parametrize("case", ["config4", "gangs", "big_caps"])
def test_long_row_bid_minima_parity(oracle, monkeypatch, win, case):
    """Per-pass window bid minima of long bidder rows (plan atomicMax, tagged
    with the pass) forced on rows of >= KP_BMIN_WIN windows — with 1 every
    row, so windows that straddle a long and a short row, gang bids (members
    x request) and 64-bit requests all meet accept's skip test. Same
    placement as the oracle, a second solve too (stale tags of the previous
    round or solve never skip a window)."""
    monkeypatch.setenv("KP_BMIN_WIN", win)
    if case == "config4":
        w = synth.config4(20_000, 2_000)
        p = _abi.default_params(**synth.CONFIG_PARAMS[4])
    else:
        w = random_workload(700 + int(win), J=4000, N=300, max_gang=8)
        if case == "big_caps":
            w = synth.Workload(w.J, w.N, w.D, w.req * (1 << 22), w.cap * (1 << 22), w.used * (1 << 22),
                               w.prio, w.gang_id, w.gang_size, w.topo, name="rand_big_caps")
        p = _abi.default_params(score_mode=int(win) % 2, n_cand=16)
    with Placer(device=0) as pl:
        g = pl.place(w, p)
        g2 = pl.place(w, p)
    o = oracle.place(_snap(oracle, w), p, nthreads=NTH)
    _assert_same(g, o, f"bid minima win {win} {case}")
    _assert_same(g2, o, f"bid minima win {win} {case}, second solve")


def test_csr_scan_many_nodes(oracle):
    """More than one 65,536-node tile in the node scan of the counting-mode
    bidder index (running carry between tiles)."""
    w = synth.config3(3_000, 70_000)
    p = _abi.default_params(**synth.CONFIG_PARAMS[3])
    with Placer(device=0) as pl:
        g = pl.place(w, p)
    o = oracle.place(_snap(oracle, w), p, nthreads=NTH)
    _assert_same(g, o, "csr scan 70k nodes")


def few_class_workload(seed, J, N, D=4, classes=5, used_frac=0.5, affinity=True):
    """Nodes of a few capacity classes (with cap-0 dims inside a class) and
    random usage: the fused filter + score + top-K path's layout."""
    rng = np.random.default_rng(seed)
    shapes = rng.integers(1, 64, size=(classes, D)) * rng.choice([1, 7, 1000], size=(1, D))
    shapes[rng.random((classes, D)) < 0.1] = 0
    cap = np.ascontiguousarray(shapes[rng.integers(0, classes, size=N)].T.astype(np.int64))
    used = (cap * rng.random((D, N)) * used_frac).astype(np.int64)
    b = random_workload(seed, J, N, D=D)
    aff = np.full(J, -1, np.int32)
    if affinity:
        for j in range(J):
            same = j > 0 and b.gang_id[j] >= 0 and b.gang_id[j] == b.gang_id[j - 1]
            aff[j] = aff[j - 1] if same else (rng.integers(0, N // 5) if rng.random() < 0.3 else -1)
    return synth.Workload(J, N, D, b.req, cap, used, b.prio, b.gang_id, b.gang_size, b.topo,
                          name=f"fc{seed}", affinity=aff)


FUSED_CASES = [  # (D, score_mode, tie_mode, n_cand, N, classes)
    (4, 0, 1, 16, 3000, 5), (1, 1, 0, 1, 700, 3), (2, 0, 0, 4, 1025, 2),
    (3, 1, 1, 32, 2100, 9), (5, 0, 1, 8, 640, 4), (8, 1, 0, 16, 1500, 6),
    (4, 1, 1, 5, 4100, 1), (4, 0, 0, 16, 130, 3),
]


@pytest.mark.parametrize("crec", ["1", "0"])
@pytest.mark.parametrize("case", range(len(FUSED_CASES)))
def test_fused_topk_parity(oracle, monkeypatch, case, crec):
    """The fused filter + score + top-K candidate phase (no score matrix) is
    bit-exact with the oracle: dims 1..8, both score modes and tie modes,
    K in {1..32}, partial tiles, cap-0 dims inside classes, affinity; with the
    per-solve row-record table (k_unit_rec) and with the records computed
    inside the kernel (KP_FZ_CREC=0)."""
    monkeypatch.setenv("KP_FZ_CREC", crec)
    D, mode, tie, K, N, classes = FUSED_CASES[case]
    w = few_class_workload(500 + case, J=2500, N=N, D=D, classes=classes)
    p = _abi.default_params(score_mode=mode, tie_mode=tie, n_cand=K, gpu_dim=D - 1,
                            w_dim=[(3 * d + 1) % 7 for d in range(8)], util_scale=[100, 7, 1024][case % 3])
    with Placer(device=0) as pl:
        g = pl.place(w, p)
        assert pl.timing()["fused"] == 1
    o = oracle.place(_snap(oracle, w), p, nthreads=NTH)
    _assert_same(g, o, f"fused case {case}")


@pytest.mark.parametrize("knobs", [
    (("KP_FUSED", "0"),),           # materialised score matrix + select
    (("KP_FZ_WG_TARGET", "64"),),   # 128 rows per fused workgroup
    (("KP_FZ_WG_TARGET", "1000000"),),  # 8 rows (one chunk) per fused workgroup
    (("KP_FZ_H16", "0"),),          # 32-bit LDS scores (single buffer, two barriers)
    (("KP_FZ_CREC", "0"),),         # row records computed inside the kernel (no per-solve table)
    (("KP_FZ_CREC", "0"), ("KP_FZ_H16", "0")),
])
def test_fused_knobs_parity(oracle, monkeypatch, knobs):
    for k, v in knobs:
        monkeypatch.setenv(k, v)
    w = synth.config3(8_000, 1_300)
    p = _abi.default_params(**synth.CONFIG_PARAMS[3])
    with Placer(device=0) as pl:
        g = pl.place(w, p)
        assert pl.timing()["fused"] == (0 if knobs[0] == ("KP_FUSED", "0") else 1)
    o = oracle.place(_snap(oracle, w), p, nthreads=NTH)
    _assert_same(g, o, f"fused knobs {knobs}")


@pytest.mark.parametrize("w,mode", [(1000, 0), (1000, 1), (40, 0)])
def test_fused_wide_scores(oracle, w, mode):
    """Scores above 2^16 take the fused kernel's 32-bit LDS form (w = 1000:
    scores up to ~4e5, 13 tie-key bits in the 32-bit keys); w = 40 the 16-bit
    form with scores up to ~1.6e4."""
    wl = few_class_workload(900 + w + mode, J=2000, N=1500, D=4, classes=4)
    p = _abi.default_params(score_mode=mode, w_dim=[w] * 8, w_gpu_fit=3 * w, w_affinity=w)
    with Placer(device=0) as pl:
        g = pl.place(wl, p)
        assert pl.timing()["fused"] == 1
    o = oracle.place(_snap(oracle, wl), p, nthreads=NTH)
    _assert_same(g, o, f"wide scores w={w}")


def test_fused_many_tiles_parity(oracle):
    """More than 64 tiles per row (70k nodes): the merge holds two lists per
    lane."""
    w = few_class_workload(77, J=1200, N=70_000, D=4, classes=3, affinity=False)
    p = _abi.default_params(n_cand=8)
    with Placer(device=0) as pl:
        g = pl.place(w, p)
        assert pl.timing()["fused"] == 1
    o = oracle.place(_snap(oracle, w), p, nthreads=NTH)
    _assert_same(g, o, "many tiles")


@pytest.mark.parametrize("mpm", [512 * 900, 640 * 3000])
def test_materialised_chunked_parity(oracle, monkeypatch, mpm):
    """The materialised candidate phase with a score matrix chunked into
    several row blocks per round (the exact-count round path)."""
    monkeypatch.setenv("KP_FUSED", "0")
    w = synth.config3(9_000, 640)
    p = _abi.default_params(**synth.CONFIG_PARAMS[3])
    with Placer(device=0, max_pairs_matrix=mpm) as pl:
        g = pl.place(w, p)
        assert pl.timing()["fused"] == 0
    o = oracle.place(_snap(oracle, w), p, nthreads=NTH)
    _assert_same(g, o, f"chunked mpm={mpm}")


@pytest.mark.parametrize("tie", [0, 1])
def test_fused_all_equal_nodes(oracle, tie):
    """Identical empty nodes: every column of a tile ties on score and only
    the tie keys separate them (tie_mode 0: the tile-relative position bits
    of the select phase; tie_mode 1: the top bits of the rotated key)."""
    N, J = 3000, 400
    cap = np.tile(np.array([[64000], [262144], [8], [1 << 20]], np.int64), (1, N))
    w = synth.Workload(J, N, 4, np.tile(np.array([[1000], [4096], [1], [1 << 16]], np.int64), (1, J)),
                       cap, np.zeros_like(cap), np.zeros(J, np.int32), np.full(J, -1, np.int32),
                       np.ones(J, np.int32), (np.arange(N) // 8).astype(np.int32), name="equal")
    p = _abi.default_params(tie_mode=tie)
    with Placer(device=0) as pl:
        g = pl.place(w, p)
        assert pl.timing()["fused"] == 1
    o = oracle.place(_snap(oracle, w), p, nthreads=NTH)
    _assert_same(g, o, f"all equal tie {tie}")


def test_fused_falls_back_on_many_classes(oracle, placer):
    """Hundreds of capacity classes make the class-aligned layout too sparse:
    the solve uses the materialised path, with the same result."""
    w = random_workload(77, J=900, N=700)
    p = _abi.default_params()
    g, o = _place_both(oracle, placer, w, p)
    assert placer.timing()["fused"] == 0
    _assert_same(g, o, "many classes")


def test_place_wide_rows_parity(oracle, placer):
    """Rows above 16384 nodes take the 1024-thread select form."""
    w = synth.config2(3_000, 20_000)
    w.used = (w.cap * (np.arange(w.N) % 7) // 9).astype(np.int64)  # uneven usage
    p = _abi.default_params(**synth.CONFIG_PARAMS[2])
    g, o = _place_both(oracle, placer, w, p)
    _assert_same(g, o, "wide rows")


def test_place_config3_full_parity_and_properties(oracle, placer):
    """BASELINE config #3 at full size: bit-exact + size-independent checks."""
    w = synth.config3()
    p = _abi.default_params(**synth.CONFIG_PARAMS[3])
    g, o = _place_both(oracle, placer, w, p)
    _assert_same(g, o, "config3 full")
    _check_properties(w, g)
    g2 = placer.place(w, p)  # idempotent per snapshot (leader fail-over safety)
    assert np.array_equal(g2["node"], g["node"]) and np.array_equal(g2["score"], g["score"])


def _check_properties(w, g):
    node = g["node"]
    placed = node >= 0
    used = w.used.copy()
    np.add.at(used.T, node[placed], w.req[:, placed].T)
    assert np.array_equal(used, g["used"]), "used_out != used + sum of placed requests"
    assert (g["used"] <= w.cap).all(), "capacity exceeded"
    # gangs: all members placed or none
    gid = w.gang_id
    for g_ in np.unique(gid[gid >= 0])[:2000]:
        m = placed[gid == g_]
        assert m.all() or not m.any(), f"gang {g_} partially placed"
    assert ((g["status"] == 0) == placed).all()


def test_place_edge_cases(oracle, placer):
    p = _abi.default_params()
    # exact fit: 4 jobs of 2 GPUs on one 8-GPU node, equal scores everywhere
    cap = np.array([[8], [8], [8], [8]], np.int64)
    req = np.full((4, 4), 2, np.int64)
    w = synth.Workload(4, 1, 4, req, cap, np.zeros_like(cap), np.zeros(4, np.int32),
                       np.full(4, -1, np.int32), np.ones(4, np.int32), np.zeros(1, np.int32))
    g, o = _place_both(oracle, placer, w, p)
    _assert_same(g, o, "exact fit")
    assert (g["node"] == 0).all()
    # gang larger than the cluster -> NO_FIT, nothing placed
    req = np.full((4, 3), 5, np.int64)
    w = synth.Workload(3, 1, 4, req, cap, np.zeros_like(cap), np.zeros(3, np.int32),
                       np.zeros(3, np.int32), np.full(3, 3, np.int32), np.zeros(1, np.int32))
    g, o = _place_both(oracle, placer, w, p)
    _assert_same(g, o, "gang overflow")
    assert (g["node"] == -1).all() and (g["status"] == _abi.KP_JOB_NO_FIT).all()
    # many identical nodes, lowest-index tie-break
    cap = np.full((4, 100), 10, np.int64)
    req = np.ones((4, 50), np.int64)
    w = synth.Workload(50, 100, 4, req, cap, np.zeros_like(cap), np.zeros(50, np.int32),
                       np.full(50, -1, np.int32), np.ones(50, np.int32), np.zeros(100, np.int32))
    for tie in (0, 1):
        g, o = _place_both(oracle, placer, w, _abi.default_params(tie_mode=tie))
        _assert_same(g, o, f"ties {tie}")


def test_place_round_limit(oracle, placer):
    w = synth.config3(5_000, 300)
    p = _abi.default_params(**synth.CONFIG_PARAMS[3], max_rounds=2)
    g, o = _place_both(oracle, placer, w, p)
    _assert_same(g, o, "round limit")
    assert g["rounds"] == 2 and (g["status"] == _abi.KP_JOB_ROUND_LIMIT).any()


def test_place_empty_and_zero_nodes(oracle, placer):
    p = _abi.default_params()
    cap = np.full((4, 3), 10, np.int64)
    w = synth.Workload(0, 3, 4, np.zeros((4, 0), np.int64), cap, np.zeros_like(cap),
                       np.zeros(0, np.int32), np.zeros(0, np.int32), np.zeros(0, np.int32),
                       np.zeros(3, np.int32))
    g, o = _place_both(oracle, placer, w, p)
    assert g["placed"] == 0 and g["rounds"] == 0 and o["rounds"] == 0
    w = synth.Workload(5, 0, 4, np.ones((4, 5), np.int64), np.zeros((4, 0), np.int64),
                       np.zeros((4, 0), np.int64), np.zeros(5, np.int32), np.full(5, -1, np.int32),
                       np.ones(5, np.int32), np.zeros(0, np.int32))
    g, o = _place_both(oracle, placer, w, p)
    _assert_same(g, o, "N=0")
    assert (g["node"] == -1).all()


def test_invalid_inputs_rejected(placer):
    p = _abi.default_params()
    cap = np.full((4, 2), 10, np.int64)
    used = cap + 1  # used > cap
    with pytest.raises(KPlaceError) as e:
        placer.load_nodes(cap, used)
    assert e.value.code == _abi.KP_EINVAL
    placer.load_nodes(cap)
    with pytest.raises(KPlaceError):
        placer.load_jobs(-np.ones((4, 2), np.int64))
    # gang members with different requests
    req = np.array([[1, 2]] * 4, np.int64)
    with pytest.raises(KPlaceError):
        placer.load_jobs(req, gang_id=np.array([7, 7], np.int32))
    # a gang id reappearing in a later run: small ids (seen-table check) and
    # ids far above the unit count (sorted check)
    req3 = np.ones((4, 3), np.int64)
    for gid in (5, 2_000_000_000):
        with pytest.raises(KPlaceError) as e:
            placer.load_jobs(req3, gang_id=np.array([gid, -1, gid], np.int32))
        assert e.value.code == _abi.KP_EINVAL
    placer.load_jobs(np.ones((4, 2), np.int64))
    bad = _abi.default_params(n_cand=0)
    with pytest.raises(KPlaceError):
        placer.solve(bad)
    placer.solve(p)


def test_streaming_apply_delta(oracle, placer):
    """config #5 shape in miniature: micro-batches against a resident table."""
    w = synth.config2(3_000, 400)
    p = _abi.default_params(**synth.CONFIG_PARAMS[2])
    placer.load_nodes(w.cap, w.used, w.topo)
    used = w.used.copy()
    rng = np.random.default_rng(3)
    for b in range(3):
        lo, hi = b * 1000, (b + 1) * 1000
        req = np.ascontiguousarray(w.req[:, lo:hi])
        placer.load_jobs(req, w.prio[lo:hi])
        placer.solve(p)
        g = placer.fetch()
        o = oracle.place(oracle.SnapshotBuf(req, w.cap, used, w.prio[lo:hi], topo=w.topo), p, NTH)
        _assert_same(g, o, f"batch {b}")
        used = g["used"].copy()
        # 20% of the placed jobs complete: negative deltas
        done = np.nonzero(g["node"] >= 0)[0]
        done = done[rng.random(done.size) < 0.2]
        placer.apply_delta(g["node"][done], -req[:, done])
        np.subtract.at(used.T, g["node"][done], req[:, done].T)


# ---------------------------------------------------------------------------
# preemption candidates (kp_load_running + kp_preempt)
# ---------------------------------------------------------------------------
def _preempt_both(oracle, placer, w, p, rn, rq, rp):
    placer.load_nodes(w.cap, w.used, w.topo)
    placer.load_running(rn, rq, rp)
    placer.load_jobs(w.req, w.prio, w.gang_id, w.gang_size)
    placer.solve(p)
    g = placer.fetch()
    gp = placer.preempt()
    o, op = oracle.preempt(_snap(oracle, w), p, rn, rq, rp, nthreads=NTH)
    return g, gp, o, op


def _assert_same_pre(gp, op, ctx=""):
    for k in ("node", "victims", "cost"):
        bad = np.nonzero(gp[k] != op[k])[0]
        assert bad.size == 0, f"{ctx} preempt {k} differs at {bad[:10]}: gpu={gp[k][bad[:10]]} cpu={op[k][bad[:10]]}"
    for k in ("preemptors", "nominated", "pairs"):
        assert gp[k] == op[k], f"{ctx} {k}: gpu={gp[k]} cpu={op[k]}"


@pytest.mark.parametrize("seed", range(4))
def test_preempt_random_parity(oracle, placer, seed):
    from test_oracle import rand_running
    w = random_workload(300 + seed, J=900, N=70 + 13 * seed, used_frac=0.9)
    rn, rq, rp = rand_running(seed, w, per_node=1 + seed)
    p = _abi.default_params(tie_mode=seed % 2, score_mode=(seed // 2) % 2)
    g, gp, o, op = _preempt_both(oracle, placer, w, p, rn, rq, rp)
    _assert_same(g, o, f"seed {seed}")
    _assert_same_pre(gp, op, f"seed {seed}")


def test_preempt_config4_parity(oracle, placer):
    """BASELINE config #4 shape at 1/10 size: priority tiers, running jobs
    filling every dim to >= 30%, preemption candidates for every NO_FIT job."""
    w = synth.config4(20_000, 2_000)
    p = _abi.default_params(**synth.CONFIG_PARAMS[4])
    m = w.meta
    g, gp, o, op = _preempt_both(oracle, placer, w, p, m["run_node"], m["run_req"], m["run_prio"])
    _assert_same(g, o, "config4")
    _assert_same_pre(gp, op, "config4")
    # properties: nominees are NO_FIT singletons; a victim set is non-empty
    nom = gp["node"] >= 0
    assert (g["status"][nom] == _abi.KP_JOB_NO_FIT).all()
    assert (gp["victims"][nom] >= 1).all()


@pytest.mark.parametrize("per_node", [6, 12, 30])
def test_preempt_long_victim_lists(oracle, placer, per_node):
    """Up to 2 x per_node running jobs per node: nodes with more than the 16
    that the tiled preemption kernel holds in registers take its per-row
    walk over global memory, next to nodes with short lists."""
    from test_oracle import rand_running
    w = random_workload(777 + per_node, J=1500, N=150, used_frac=0.95)
    rn, rq, rp = rand_running(per_node, w, per_node=2 * per_node)
    p = _abi.default_params(score_mode=per_node % 2)
    g, gp, o, op = _preempt_both(oracle, placer, w, p, rn, rq, rp)
    _assert_same(g, o, f"long victim lists {per_node}")
    _assert_same_pre(gp, op, f"long victim lists {per_node}")
    assert np.bincount(rn, minlength=w.N).max() > (16 if per_node >= 12 else 8)


def test_preempt_wide_priorities(oracle, placer):
    """Priority sums that do not fit the tiled kernel's packed 32-bit cost
    field (|sum| >= 2^31 on some node) take the per-row kernel; negative
    priorities included."""
    from test_oracle import rand_running
    w = random_workload(4242, J=1200, N=110, used_frac=0.9)
    rn, rq, rp = rand_running(11, w, per_node=6)
    rp = ((rp.astype(np.int64) - 2) * (1 << 29)).astype(np.int32)
    prio = ((w.prio.astype(np.int64) - 2) * (1 << 29) + 7).astype(np.int32)
    w = synth.Workload(w.J, w.N, w.D, w.req, w.cap, w.used, prio, w.gang_id, w.gang_size, w.topo,
                       name="wideprio")
    p = _abi.default_params()
    g, gp, o, op = _preempt_both(oracle, placer, w, p, rn, rq, rp)
    _assert_same(g, o, "wide priorities")
    _assert_same_pre(gp, op, "wide priorities")


def test_preempt_kernel_forms_agree(oracle, monkeypatch):
    """KP_PREEMPT32=0 (the per-row 64-bit kernel on a 32-bit table) gives the
    same nominations as the default register-resident 32-bit kernel."""
    w = synth.config4(20_000, 2_000)
    p = _abi.default_params(**synth.CONFIG_PARAMS[4])
    m = w.meta
    out = []
    for v in ("1", "0"):
        monkeypatch.setenv("KP_PREEMPT32", v)
        with Placer(device=0) as pl:
            _, gp, _, op = _preempt_both(oracle, pl, w, p, m["run_node"], m["run_req"], m["run_prio"])
        _assert_same_pre(gp, op, f"KP_PREEMPT32={v}")
        out.append(gp)
    for k in ("node", "victims", "cost"):
        assert np.array_equal(out[0][k], out[1][k])


def test_preempt_requires_solve_and_valid_pool(placer):
    cap = np.full((4, 3), 10, np.int64)
    used = np.full((4, 3), 5, np.int64)
    placer.load_nodes(cap, used)
    with pytest.raises(KPlaceError) as e:
        placer.load_running(np.array([0], np.int32), np.full((4, 1), 6, np.int64),
                            np.array([0], np.int32))   # 6 > used 5
    assert e.value.code == _abi.KP_EINVAL
    placer.load_running(np.array([0, 2], np.int32), np.full((4, 2), 5, np.int64),
                        np.array([0, 1], np.int32))
    placer.load_jobs(np.full((4, 2), 7, np.int64), np.array([3, 0], np.int32))
    placer.solve(_abi.default_params())
    pr = placer.preempt()
    assert pr["node"].tolist() == [0, -1] and pr["victims"].tolist() == [1, 0]


# ---------------------------------------------------------------------------
# streaming churn (config #5 shape): micro-batches against a resident table
# ---------------------------------------------------------------------------
def test_streaming_config5_trace_parity(oracle, placer):
    """BASELINE config #5 in miniature: a trace replayed in micro-batches; after
    each batch a deterministic 20% of the running jobs complete (negative
    kp_apply_delta). The oracle replays the same trace with its own usage."""
    total, N, B = 12_000, 3_000, 1_000
    cap, topo, req, prio = synth.config5_trace(total, N)
    p = _abi.default_params(**synth.CONFIG_PARAMS[5])
    placer.load_nodes(cap, None, topo)
    used_o = np.zeros_like(cap)
    run_node = np.zeros(0, np.int32)
    run_job = np.zeros(0, np.int64)
    for b in range(total // B):
        lo, hi = b * B, (b + 1) * B
        rq = np.ascontiguousarray(req[:, lo:hi])
        placer.load_jobs(rq, prio[lo:hi])
        placer.solve(p)
        g = placer.fetch()
        o = oracle.place(oracle.SnapshotBuf(rq, cap, used_o, prio[lo:hi], topo=topo), p, NTH)
        _assert_same(g, o, f"batch {b}")
        used_o = o["used"].copy()
        ok = g["node"] >= 0
        run_node = np.concatenate([run_node, g["node"][ok]])
        run_job = np.concatenate([run_job, lo + np.nonzero(ok)[0]])
        done = synth.config5_completions(b, run_job)
        placer.apply_delta(run_node[done], -req[:, run_job[done]])
        np.subtract.at(used_o.T, run_node[done], req[:, run_job[done]].T)
        run_node, run_job = run_node[~done], run_job[~done]
    assert np.array_equal(placer.fetch()["used"], used_o)


def test_apply_delta_all_or_nothing(placer):
    cap = np.full((4, 4), 10, np.int64)
    used = np.full((4, 4), 3, np.int64)
    placer.load_nodes(cap, used)
    placer.load_jobs(np.ones((4, 1), np.int64))
    placer.solve(_abi.default_params())
    before = placer.fetch()["used"]
    # node 1 would go to -1 in dim 0: rejected, nothing applied
    with pytest.raises(KPlaceError) as e:
        placer.apply_delta(np.array([0, 1, 1], np.int32),
                           np.array([[-1, -2, -2], [0, 0, 0], [0, 0, 0], [1, 1, 1]], np.int64))
    assert e.value.code == _abi.KP_EINVAL
    assert np.array_equal(placer.fetch()["used"], before)
    with pytest.raises(KPlaceError):
        placer.apply_delta(np.array([4], np.int32), np.zeros((4, 1), np.int64))  # bad node
    placer.apply_delta(np.array([2, 2], np.int32), np.full((4, 2), 3, np.int64))
    after = placer.fetch()["used"]
    assert (after[:, 2] == before[:, 2] + 6).all()


def test_place_widest_rows_parity(oracle, placer):
    """Rows of 50k nodes (config #5's table) take the 768-thread select form."""
    w = synth.config2(1_500, 50_000)
    w.used = (w.cap * (np.arange(w.N) % 5) // 7).astype(np.int64)
    p = _abi.default_params(**synth.CONFIG_PARAMS[3])
    g, o = _place_both(oracle, placer, w, p)
    _assert_same(g, o, "widest rows")


def test_config1_runner_gpu(oracle, placer):
    """BASELINE config #1: the reference's sample CRs + synthetic CRs and Node
    reports through packer -> kp_place (GPU) -> status writer; every CR's
    Placed condition equals the oracle-backed run of the same batch."""
    from test_host import OraclePlacer, run_config1
    _, _, got, s_gpu, _ = run_config1(placer)
    _, _, want, s_cpu, _ = run_config1(OraclePlacer(oracle))
    strip = lambda d: {k: [{kk: vv for kk, vv in c.items() if kk != "lastUpdateTime"}
                           for c in v["conditions"]] for k, v in d.items()}
    assert strip(got) == strip(want)
    assert (s_gpu["placed"], s_gpu["rounds"]) == (s_cpu["placed"], s_cpu["rounds"])


# ---------------------------------------------------------------------------
# exact utilisation at the boundaries: every division form of
# k_score32 (E / C / W waves, mixed waves) and of the 64-bit path
# ---------------------------------------------------------------------------
def boundary_nodes(rng, N, top):
    """Caps across the division modes; usage so that x = used + q hits
    {cap, cap - 1, 1, 0, random} for the probe requests."""
    kinds = rng.integers(0, 5, size=N)
    cap = np.where(kinds == 0, rng.integers(0, 4096, size=N),
                   np.where(kinds == 1, rng.integers(4096, 1 << 24, size=N),
                            np.where(kinds == 2, rng.integers(1 << 24, 1 << top, size=N),
                                     np.where(kinds == 3, (1 << rng.integers(1, top, size=N)) - 1,
                                              1 << rng.integers(0, top - 1, size=N)))))
    cap[: N // 2] = rng.integers(1, 1 << 24, size=N // 2)  # whole fast waves too
    return cap.astype(np.int64)


@pytest.mark.parametrize("top,mode,scale", [(31, 0, 100), (32, 1, 100), (32, 0, 1024),
                                            (25, 1, 7), (50, 0, 1024), (56, 1, 100)])
def test_score_matrix_boundaries(oracle, placer, top, mode, scale):
    rng = np.random.default_rng(top * 10 + mode)
    D, N = 2, 1400
    cap = np.stack([boundary_nodes(rng, N, min(top, 56)) for _ in range(D)])
    # probe q = 1 on every node; usage cap - 1, cap - 2, 0, random: x = cap,
    # cap - 1, 1 and random after the request
    pick = rng.integers(0, 4, size=(D, N))
    used = np.where(pick == 0, cap - 1, np.where(pick == 1, cap - 2, np.where(
        pick == 2, 0, (cap * rng.random((D, N))).astype(np.int64))))
    used = np.clip(used, 0, cap)
    req = np.ones((D, 3), np.int64)
    req[:, 1] = 0
    req[:, 2] = 2
    p = _abi.default_params(score_mode=mode, util_scale=scale, gpu_dim=-1, w_dim=(3, 5))
    placer.load_nodes(cap, used)
    placer.load_jobs(req)
    sc, mk = placer.score(p, 0, 3)
    osc, omk = oracle.score(oracle.SnapshotBuf(req, cap, used), p, 0, 3)
    bad = np.argwhere(sc != osc)
    assert bad.size == 0, f"first mismatches {bad[:5].tolist()}: gpu {sc[tuple(bad[0])]} cpu {osc[tuple(bad[0])]}"
    assert np.array_equal(mk, omk)


def test_full_node_scores_S_gpu(oracle, placer):
    a = synth.SHAPES[0].reshape(4, 1)
    placer.load_nodes(np.repeat(a, 70, axis=1))
    placer.load_jobs(np.repeat(a, 2, axis=1))
    sc, _ = placer.score(_abi.default_params(w_dim=(1, 1, 4, 2), w_gpu_fit=0), 0, 2)
    assert (sc == 800).all()


def affinity_workload(seed, J, N):
    w = random_workload(seed, J, N)
    rng = np.random.default_rng(seed + 99)
    aff = rng.integers(-1, N // 5 + 1, size=w.J).astype(np.int32)
    for g in np.unique(w.gang_id[w.gang_id >= 0]):
        aff[w.gang_id == g] = aff[w.gang_id == g][0]
    w.affinity = aff
    return w


@pytest.mark.parametrize("seed", range(4))
def test_place_affinity_parity(oracle, placer, seed):
    """CacheStrategy=shared: the affinity bonus on the job's domain."""
    w = affinity_workload(500 + seed, J=900, N=120 + 7 * seed)
    p = _abi.default_params(w_affinity=[512, 37, 4096, 0][seed], score_mode=seed % 2,
                            tie_mode=(seed // 2) % 2)
    g, o = _place_both(oracle, placer, w, p)
    _assert_same(g, o, f"affinity seed {seed}")
    if p.w_affinity:
        ok = (g["node"] >= 0) & (w.affinity >= 0)
        assert (w.topo[g["node"][ok]] == w.affinity[ok]).mean() > 0.2


def test_place_affinity_wide_parity(oracle, placer):
    # 64-bit path (caps >= 2^32) with affinity
    w = affinity_workload(600, J=500, N=90)
    w.cap = w.cap * (1 << 30)
    w.used = w.used * (1 << 30)
    w.req = w.req * (1 << 29)
    p = _abi.default_params(w_affinity=700)
    g, o = _place_both(oracle, placer, w, p)
    _assert_same(g, o, "affinity wide")


# ---------------------------------------------------------------------------
# the C-ABI contract for the Go host (include/kplace.h): atomic kp_place,
# per-context error text, failed loads leave no snapshot
# ---------------------------------------------------------------------------
def test_place_is_atomic_across_threads(oracle):
    """Two OS threads call kp_place on ONE context with different snapshots;
    every result equals the oracle's for its own snapshot (no interleaving of
    one thread's load with the other's solve)."""
    import threading
    ws = [synth.config3(3_000, 300), synth.config2(2_000, 250)]
    ps = [_abi.default_params(**synth.CONFIG_PARAMS[3]), _abi.default_params(**synth.CONFIG_PARAMS[2])]
    want = [oracle.place(_snap(oracle, w), p, nthreads=NTH) for w, p in zip(ws, ps)]
    errors = []
    with Placer(device=0) as pl:
        def run(i):
            try:
                for _ in range(6):
                    g = pl.place(ws[i], ps[i])
                    for k in ("node", "score", "status", "used"):
                        if not np.array_equal(g[k], want[i][k]):
                            errors.append((i, k))
            except Exception as e:  # noqa: BLE001
                errors.append((i, repr(e)))
        ts = [threading.Thread(target=run, args=(i,)) for i in (0, 1)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
    assert not errors, errors


def test_last_error_is_per_context_and_failed_load_unloads(placer):
    cap = np.full((4, 3), 10, np.int64)
    with pytest.raises(KPlaceError) as e:
        placer.load_nodes(cap, cap + 1)
    assert e.value.code == _abi.KP_EINVAL and "used" in e.value.detail
    assert "used" in placer.last_error()
    placer.load_nodes(cap)
    placer.load_jobs(np.ones((4, 2), np.int64))
    placer.solve(_abi.default_params())
    assert placer.last_error() == ""
    with pytest.raises(KPlaceError):  # a failed job load after a good one ...
        placer.load_jobs(-np.ones((4, 5), np.int64))
    with pytest.raises(KPlaceError) as e:  # ... leaves no queue to solve or fetch
        placer.solve(_abi.default_params())
    assert e.value.code == _abi.KP_ESTATE
    with pytest.raises(KPlaceError) as e:
        placer.fetch()
    assert e.value.code == _abi.KP_ESTATE
    with pytest.raises(KPlaceError):  # a failed node load drops the node table
        placer.load_nodes(cap, -cap)
    with pytest.raises(KPlaceError) as e:
        placer.load_jobs(np.ones((4, 2), np.int64))
    assert e.value.code == _abi.KP_ESTATE


# ---------------------------------------------------------------------------
# kp_create_multi: one context, one worker thread per shard (here several
# shards on the one GPU of the box, exchanging in process; distinct GPUs use
# RCCL) — bit-exact with the oracle and with the single-GPU context
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("ids,cfg", [([0, 0], (3, 8_000, 640)), ([0, 0, 0], (2, 3_000, 300)),
                                     ([0, 0], (3, 1, 64)), ([0], (3, 4_000, 400))])
def test_create_multi_parity(oracle, ids, cfg):
    no, J, N = cfg
    w = synth.config(no, J, N)
    p = _abi.default_params(**synth.CONFIG_PARAMS[no])
    with Placer(gpu_ids=ids) as pl:
        g = pl.place(w, p)
        g2 = pl.place(w, p)
    o = oracle.place(_snap(oracle, w), p, nthreads=NTH)
    _assert_same(g, o, f"multi {ids}")
    _assert_same(g2, o, f"multi {ids} again")


def test_create_multi_streaming(oracle):
    cap, topo, req, prio = synth.config5_trace(4_000, 1_000)
    p = _abi.default_params(**synth.CONFIG_PARAMS[5])
    used_o = np.zeros_like(cap)
    with Placer(gpu_ids=[0, 0]) as pl:
        pl.load_nodes(cap, None, topo)
        for b in range(4):
            lo, hi = b * 1000, (b + 1) * 1000
            rq = np.ascontiguousarray(req[:, lo:hi])
            pl.load_jobs(rq, prio[lo:hi])
            pl.solve(p)
            g = pl.fetch()
            o = oracle.place(oracle.SnapshotBuf(rq, cap, used_o, prio[lo:hi], topo=topo), p, NTH)
            _assert_same(g, o, f"multi batch {b}")
            used_o = o["used"].copy()
            done = np.nonzero(g["node"] >= 0)[0][::3]
            pl.apply_delta(g["node"][done], -rq[:, done])
            np.subtract.at(used_o.T, g["node"][done], rq[:, done].T)


@pytest.mark.parametrize("tie", [0, 1])
@pytest.mark.parametrize("bits,K", [(1, 16), (1, 32), (3, 32), (5, 32), (8, 8)])
def test_fused_key_collisions(oracle, monkeypatch, tie, bits, K):
    """Fewer tie bits in the select phase's 32-bit keys (KP_FZ_TIE_BITS, a
    test knob) make keys collide: more survivors than one per lane (two-per-
    lane rank, up to 128) and more than 128 (exact 64-bit bisection). The
    lists stay exact."""
    monkeypatch.setenv("KP_FZ_TIE_BITS", str(bits))
    w = few_class_workload(1300 + 7 * bits + K + tie, J=1500, N=2600, D=3, classes=2)
    p = _abi.default_params(tie_mode=tie, n_cand=K)
    with Placer(device=0) as pl:
        g = pl.place(w, p)
        assert pl.timing()["fused"] == 1
    o = oracle.place(_snap(oracle, w), p, nthreads=NTH)
    _assert_same(g, o, f"collisions tie={tie} bits={bits} K={K}")


@pytest.mark.parametrize("tie", [0, 1])
@pytest.mark.parametrize("K", [4, 16, 32])
def test_fused_bisection_all_ties(oracle, monkeypatch, tie, K):
    """Every column of every tile ties on score (identical empty nodes, one
    request shape) and the select keys keep one tie bit (KP_FZ_TIE_BITS=1):
    about half of each tile's 1,024 columns reach T, far past the 128
    survivor slots, so every row takes the exact 64-bit bisection, which
    must re-read all 16 columns of each lane (4-column groups L + 64k)."""
    monkeypatch.setenv("KP_FZ_TIE_BITS", "1")
    N, J = 3000, 700
    cap = np.ascontiguousarray(np.tile(np.array([[64000], [524288], [8], [8 * 294912]], np.int64), (1, N)))
    req = np.ascontiguousarray(np.tile(np.array([[1000], [1024], [1], [16384]], np.int64), (1, J)))
    w = synth.Workload(J, N, 4, req, cap, np.zeros_like(cap), np.zeros(J, np.int32),
                       np.full(J, -1, np.int32), np.ones(J, np.int32),
                       (np.arange(N) // 32).astype(np.int32), name="ties")
    p = _abi.default_params(tie_mode=tie, n_cand=K, w_spread=0)
    with Placer(device=0) as pl:
        g = pl.place(w, p)
        assert pl.timing()["fused"] == 1
    o = oracle.place(_snap(oracle, w), p, nthreads=NTH)
    _assert_same(g, o, f"all ties tie={tie} K={K}")


# ---------------------------------------------------------------------------
# the product is the default path: knobs need the gate, fixtures hold on the GPU
# ---------------------------------------------------------------------------
def test_knobs_ignored_without_debug_gate(oracle, monkeypatch):
    """A manager process's inherited environment cannot switch kernels or key
    encodings: without KP_DEBUG_KNOBS=1, KP_FUSED=0 and KP_FZ_TIE_BITS=1 are
    ignored at kp_create, so the solve runs the fused candidate phase with the
    full tie-key width and returns the oracle's placement."""
    monkeypatch.delenv("KP_DEBUG_KNOBS", raising=False)
    monkeypatch.setenv("KP_FUSED", "0")
    monkeypatch.setenv("KP_FZ_TIE_BITS", "1")
    monkeypatch.setenv("KP_ACC_BIG_RATIO", "1")
    w = synth.config3(8_000, 800)
    p = _abi.default_params(**synth.CONFIG_PARAMS[3])
    with Placer(device=0) as pl:
        pl.set_profiling(True)
        g = pl.place(w, p)
        assert pl.timing()["fused"] == 1, "KP_FUSED=0 honoured without the KP_DEBUG_KNOBS gate"
    _assert_same(g, oracle.place(_snap(oracle, w), p, nthreads=NTH), "knobs without the gate")


GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.parametrize("name", sorted(f for f in os.listdir(GOLDEN) if f.startswith("place_")
                                        and f.endswith(".npz")))
def test_golden_fixture_gpu(name):
    """Every committed golden vector (tests/golden/make_golden.py) fed straight
    to libkplace: node / score / status / usage and the round and pass counts
    equal the stored outputs (no oracle in the loop)."""
    z = np.load(os.path.join(GOLDEN, name), allow_pickle=False)
    pd = {k[2:]: z[k] for k in z.files if k.startswith("p_")}
    p = _abi.default_params(**{k: (tuple(int(x) for x in v) if v.ndim else int(v))
                               for k, v in pd.items()})
    w = synth.Workload(int(z["req"].shape[1]), int(z["cap"].shape[1]), int(z["req"].shape[0]),
                       z["req"], z["cap"], z["used"], z["prio"], z["gang_id"], z["gang_size"],
                       z["topo"], affinity=z["affinity"] if "affinity" in z.files else None)
    with Placer(device=0) as pl:
        g = pl.place(w, p)
    for k in ("node", "score", "status", "used"):
        assert np.array_equal(g[k], z["out_" + k]), f"{name}: {k}"
    assert g["rounds"] == int(z["out_rounds"]) and g["passes"] == int(z["out_passes"]), name


# ---------------------------------------------------------------------------
# k_score32's class form (few capacity vectors) and kp_score_dev
# ---------------------------------------------------------------------------
def class_form_workload(seed, J, N, D=4, classes=3, wide=False):
    """Node tables of `classes` capacity vectors (incl. a class with cap-0 dims)
    in shuffled node order, usage anywhere in [0, cap], random requests:
    k_score32's class form on every wave."""
    rng = np.random.default_rng(seed)
    top = (1 << 31) if wide else 64
    shapes = rng.integers(1, top, size=(classes, D)).astype(np.int64)
    shapes[0, D - 1] = 0  # a class with a cap-0 dim
    cls = rng.integers(0, classes, size=N)
    cap = np.ascontiguousarray(shapes[cls].T)
    used = (cap * rng.random((D, N))).astype(np.int64)
    full = rng.random(N) < 0.05
    used[:, full] = cap[:, full]
    req = (rng.integers(0, max(2, top // 4), size=(D, J))).astype(np.int64)
    req[:, rng.random(J) < 0.05] = 0
    topo = (np.arange(N) // 7).astype(np.int32)
    aff = np.where(rng.random(J) < 0.3, rng.integers(0, N // 7 + 1, size=J), -1).astype(np.int32)
    return synth.Workload(J, N, D, np.ascontiguousarray(req), cap, used,
                          np.zeros(J, np.int32), np.full(J, -1, np.int32), np.ones(J, np.int32),
                          topo, name=f"fewcls{seed}", affinity=aff)


@pytest.mark.parametrize("classes,mode,scale,wide", [(1, 0, 100, False), (3, 1, 100, False),
                                                     (8, 0, 1024, False), (5, 1, 7, True),
                                                     (9, 0, 100, False)])
def test_score_matrix_class_form(oracle, monkeypatch, classes, mode, scale, wide):
    """kp_score through the class form (<= 8 capacity classes; 9 takes the
    per-wave form) equals the oracle's kpo_score, and the per-wave form
    (KP_SCORE_CLASSES=0) agrees; timing reports which form ran."""
    w = class_form_workload(classes * 7 + mode, J=257, N=1111, classes=classes, wide=wide)
    p = _abi.default_params(score_mode=mode, util_scale=scale)
    osc, omk = oracle.score(oracle.SnapshotBuf(w.req, w.cap, w.used, topo=w.topo,
                                               affinity=w.affinity), p, 0, w.J)
    for knob in ("1", "0"):
        monkeypatch.setenv("KP_SCORE_CLASSES", knob)
        with Placer(device=0) as pl:
            pl.load_nodes(w.cap, w.used, w.topo)
            pl.load_jobs(w.req, affinity=w.affinity)
            sc, mk = pl.score(p, 0, w.J)
        assert np.array_equal(sc, osc), f"classes {classes} knob {knob}"
        assert np.array_equal(mk, omk), f"classes {classes} knob {knob}"


@pytest.mark.parametrize("cfg", [(2, 3_000, 1_000), (3, 4_000, 1_500), (4, 3_000, 2_000),
                                 (3, 2_000, 3_001)])
@pytest.mark.parametrize("outputs", ["both", "score", "mask"])
def test_score_dev_parity(oracle, cfg, outputs):
    """kp_score_dev into caller device buffers (padded rows of round_up(N, 64)):
    the first N columns equal the oracle's matrix and mask, padding columns are
    infeasible / zero bits; either output alone (the kernel's score-only and
    mask-only instances) writes the same values and leaves the other buffer
    untouched; profiling reports the class form and algorithmic bytes."""
    from kplace.devmem import DeviceBuffer
    no, J, N = cfg
    w = synth.config(no, J, N)
    p = _abi.default_params(**synth.CONFIG_PARAMS[no])
    Ns = (N + 63) // 64 * 64
    lo, hi = 17, J - 5
    with DeviceBuffer((hi - lo) * Ns * 4, fill=0x5A) as sc, \
            DeviceBuffer((hi - lo) * (Ns // 64) * 8, fill=0x5A) as mk:
        with Placer(device=0) as pl:
            pl.load_nodes(w.cap, w.used, w.topo)
            pl.load_jobs(w.req, w.prio, w.gang_id, w.gang_size)
            pl.set_profiling(True)
            pl.score_dev(p, lo, hi, sc.ptr if outputs != "mask" else None,
                         mk.ptr if outputs != "score" else None)
            t = pl.timing()
        g = sc.to_numpy(np.int32, (hi - lo, Ns))
        gm = mk.to_numpy(np.uint64, (hi - lo, Ns // 64))
    osc, omk = oracle.score(_snap(oracle, w), p, lo, hi)
    if outputs == "mask":
        assert (g.view(np.uint32) == 0x5A5A5A5A).all()
    else:
        assert np.array_equal(g[:, :N], osc) and (g[:, N:] == -1).all()
    if outputs == "score":
        assert (gm == 0x5A5A5A5A5A5A5A5A).all()
    else:
        assert np.array_equal(gm[:, :omk.shape[1]], omk)
    assert t["score_form"] == 1 and t["score_classes"] >= 1 and t["score_launches"] == 1
    assert t["score_bytes"] > (hi - lo) * (Ns * 4 if outputs != "mask" else Ns // 8)
    assert t["score_ms"] > 0
