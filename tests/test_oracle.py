"""CPU tests of the oracle (test infrastructure) against hand-derived known
answers, an independent pure-Python restatement (tests/spec_py.py) and the
committed golden fixtures (tests/golden/). Parity of the placement with the
reference itself is "unpinned" (the reference has no placement code,
SURVEY.md §0); these tests pin the oracle to the written spec.
"""
import glob
import os

import numpy as np
import pytest

import spec_py
from kplace import _abi, synth

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def W(req, cap, used=None, prio=None, gang_id=None, topo=None):
    req = np.array(req, np.int64)
    cap = np.array(cap, np.int64)
    D, J = req.shape
    N = cap.shape[1]
    used = np.zeros_like(cap) if used is None else np.array(used, np.int64)
    prio = np.zeros(J, np.int32) if prio is None else np.array(prio, np.int32)
    gid = np.full(J, -1, np.int32) if gang_id is None else np.array(gang_id, np.int32)
    gsz = np.ones(J, np.int32)
    for g in set(gid.tolist()) - {-1}:
        gsz[gid == g] = (gid == g).sum()
    topo = np.arange(N, dtype=np.int32) if topo is None else np.array(topo, np.int32)
    return synth.Workload(J, N, D, req, cap, used, prio, gid, gsz, topo)


def P(**kw):
    base = dict(w_dim=(1,) * 8, gpu_dim=-1, w_gpu_fit=0, w_spread=0, tie_mode=0)
    base.update(kw)
    return _abi.default_params(**base)


def run(oracle, w, p, threads=1):
    r = oracle.place(oracle.SnapshotBuf.from_workload(w), p, nthreads=threads)
    assert not isinstance(r, int), f"oracle error {r}"
    return r


# ---------------------------------------------------------------------------
# known answers, derived by hand from DESIGN.md §2
# ---------------------------------------------------------------------------
def test_kat_priority_and_capacity(oracle):
    # one node (cpu 10, mem 10); job1 (prio 1) outranks job0 (prio 0)
    w = W([[6, 6], [1, 1]], [[10], [10]], prio=[0, 1])
    r = run(oracle, w, P())
    # util = ((used+q) * floor(100*2^32/10)) >> 32 -> cpu 60, mem 10
    assert r["node"].tolist() == [-1, 0]
    assert r["score"].tolist() == [-1, 70]
    assert r["status"].tolist() == [_abi.KP_JOB_NO_FIT, _abi.KP_JOB_PLACED]
    assert r["used"].tolist() == [[6], [1]]
    assert r["rounds"] == 2 and r["passes"] == 1


def test_kat_first_fit_not_prefix(oracle):
    # A(6) accepted, B(6) rejected, C(3) still accepted in the same pass
    w = W([[6, 6, 3]], [[10]])
    r = run(oracle, w, P(max_passes=1, max_rounds=1))
    assert r["node"].tolist() == [0, -1, 0]
    assert r["status"].tolist() == [0, _abi.KP_JOB_ROUND_LIMIT, 0]


def test_kat_gang_split_across_nodes(oracle):
    # gang of two 6-GPU replicas, two 8-GPU nodes: util 6*12.5 = 75 each
    w = W([[6, 6]], [[8, 8]], gang_id=[3, 3])
    r = run(oracle, w, P(gpu_dim=0))
    assert r["node"].tolist() == [0, 1]
    assert r["score"].tolist() == [75, 75]
    assert r["rounds"] == 1 and r["passes"] == 1


def test_kat_gang_all_or_nothing(oracle):
    # 3 x 5 GPUs cannot fit two 8-GPU nodes: nothing placed
    w = W([[5, 5, 5]], [[8, 8]], gang_id=[0, 0, 0])
    r = run(oracle, w, P(gpu_dim=0))
    assert r["node"].tolist() == [-1, -1, -1]
    assert r["status"].tolist() == [_abi.KP_JOB_NO_FIT] * 3
    assert r["used"].tolist() == [[0, 0]]


def test_kat_gpu_fit_bonus(oracle):
    # n0: 4 of 8 GPUs used, n1: 2 used; job needs 4 -> n0 is an exact fill
    w = W([[4]], [[8, 8]], used=[[4, 2]])
    r = run(oracle, w, P(gpu_dim=0, w_gpu_fit=1024))
    assert r["node"].tolist() == [0] and r["score"].tolist() == [100 + 1024]
    r = run(oracle, w, P(gpu_dim=0, w_gpu_fit=1024, score_mode=1))  # LeastAllocated
    assert r["node"].tolist() == [0] and r["score"].tolist() == [0 + 1024]
    r = run(oracle, w, P(gpu_dim=0, w_gpu_fit=0, score_mode=1))
    assert r["node"].tolist() == [1] and r["score"].tolist() == [100 - 75]


def test_kat_spread_penalty(oracle):
    # 2-member gang, 3 empty identical nodes; n0,n1 share topo domain 0.
    # Without spread both members pack onto n0 (bin-pack favours fuller);
    # with a large spread penalty the second member leaves domain 0.
    w = W([[1, 1]], [[4, 4, 4]], gang_id=[9, 9], topo=[0, 0, 1])
    r = run(oracle, w, P(gpu_dim=0))
    assert r["node"].tolist() == [0, 0]
    r = run(oracle, w, P(gpu_dim=0, w_spread=100))
    assert r["node"].tolist() == [0, 2]


def test_kat_rotated_tie_break(oracle):
    N, seed = 37, 0x1234
    w = W([[1]], [[5] * N])
    r = run(oracle, w, P(tie_mode=1, tie_seed=seed))
    salt = spec_py.fmix32(0 ^ seed)
    want = min(range(N), key=lambda n: (n * spec_py.TIE_MUL + salt) & spec_py.MASK32)
    assert r["node"].tolist() == [want]
    assert run(oracle, w, P(tie_mode=0))["node"].tolist() == [0]


def test_kat_zero_capacity_dims(oracle):
    # a node with cap 0 in a dim only takes jobs that request 0 there
    w = W([[1, 1], [0, 1]], [[4, 4], [0, 4]])
    r = run(oracle, w, P())
    assert r["node"][1] == 1 and r["node"][0] in (0, 1)


@pytest.mark.parametrize("bad", [
    "used_gt_cap", "neg_req", "gang_mixed_req", "gang_reused", "gang_size", "n_cand",
    "scale", "passes", "gpu_dim", "weight", "topo",
])
def test_validation(oracle, bad):
    req = [[1, 1, 1], [1, 1, 1]]
    cap = [[4, 4], [4, 4]]
    kw = {}
    p = P()
    if bad == "used_gt_cap":
        kw["used"] = [[5, 0], [0, 0]]
    elif bad == "neg_req":
        req = [[1, -1, 1], [1, 1, 1]]
    elif bad == "gang_mixed_req":
        req = [[1, 2, 1], [1, 1, 1]]
        kw["gang_id"] = [0, 0, -1]
    elif bad == "gang_reused":
        kw["gang_id"] = [0, 1, 0]
    elif bad == "topo":
        kw["topo"] = [0, -1]
    elif bad == "n_cand":
        p = P(n_cand=0)
    elif bad == "scale":
        p = P(util_scale=0)
    elif bad == "passes":
        p = P(max_passes=65)
    elif bad == "gpu_dim":
        p = P(gpu_dim=2)
    elif bad == "weight":
        p = P(w_dim=(70000,) + (1,) * 7)
    w = W(req, cap, **kw)
    if bad == "gang_size":
        w.gang_size[:] = 2
    r = oracle.place(oracle.SnapshotBuf.from_workload(w), p)
    assert r == _abi.KP_EINVAL


# ---------------------------------------------------------------------------
# two independent restatements agree
# ---------------------------------------------------------------------------
def rand_w(seed, J, N, D=3):
    rng = np.random.default_rng(seed)
    cap = rng.integers(0, 12, size=(D, N)).astype(np.int64)
    used = (cap * rng.random((D, N)) * 0.4).astype(np.int64)
    sizes, tot = [], 0
    while tot < J:
        s = min(int(rng.integers(1, 5)) if rng.random() < 0.4 else 1, J - tot)
        sizes.append(s)
        tot += s
    sizes = np.array(sizes)
    reqc = rng.integers(0, 5, size=(D, len(sizes))).astype(np.int64)
    prc = rng.integers(0, 3, size=len(sizes)).astype(np.int32)
    cr = np.repeat(np.arange(len(sizes)), sizes)
    gid = np.where(np.repeat(sizes, sizes) > 1, cr, -1).astype(np.int32)
    affc = rng.integers(-1, N // 3 + 1, size=len(sizes)).astype(np.int32)  # -1 = none
    return synth.Workload(J, N, D, np.ascontiguousarray(reqc[:, cr]), cap, used, prc[cr], gid,
                          np.repeat(sizes, sizes).astype(np.int32),
                          (np.arange(N) // 3).astype(np.int32), affinity=affc[cr])


@pytest.mark.parametrize("seed", range(12))
def test_oracle_matches_python_spec(oracle, seed):
    w = rand_w(seed, J=40 + 7 * seed, N=6 + seed)
    p = P(w_dim=(1, 3, 2) + (1,) * 5, gpu_dim=seed % 3 - 1, w_gpu_fit=50 * (seed % 2),
          w_spread=7 * (seed % 3), tie_mode=seed % 2, score_mode=(seed // 2) % 2,
          n_cand=1 + seed % 5, max_passes=1 + seed % 4, util_scale=[100, 16, 1024][seed % 3],
          w_affinity=[0, 3, 40][seed % 3])
    r = run(oracle, w, p, threads=2)
    s = spec_py.place(w.req, w.cap, w.used, w.prio, w.gang_id, w.topo, _abi.params_dict(p),
                      affinity=w.affinity)
    assert r["node"].tolist() == s["node"]
    assert r["score"].tolist() == s["score"]
    assert r["status"].tolist() == s["status"]
    assert r["used"].tolist() == s["used"]
    assert (r["rounds"], r["passes"]) == (s["rounds"], s["passes"])


def test_oracle_thread_count_invariant(oracle):
    w = synth.config3(4000, 400)
    p = _abi.default_params(**synth.CONFIG_PARAMS[3])
    a = run(oracle, w, p, threads=1)
    b = run(oracle, w, p, threads=8)
    for k in ("node", "score", "status", "used"):
        assert np.array_equal(a[k], b[k])


def test_score_matrix_matches_python(oracle):
    w = rand_w(77, J=30, N=70, D=4)
    p = P(w_dim=(2, 1, 3, 1) + (1,) * 4, gpu_dim=2, w_gpu_fit=9, score_mode=1, util_scale=50)
    sc, mk = oracle.score(oracle.SnapshotBuf(w.req, w.cap, w.used), p, 0, w.J)
    pd = _abi.params_dict(p)
    for j in range(w.J):
        for n in range(w.N):
            one = spec_py.place(w.req[:, j:j + 1], w.cap[:, n:n + 1], w.used[:, n:n + 1],
                                None, None, None, dict(pd, max_rounds=1, max_passes=1, n_cand=1,
                                                       w_affinity=0))
            want = one["score"][0]
            assert sc[j, n] == want, (j, n)
            assert bool((int(mk[j, n // 64]) >> (n % 64)) & 1) == (want >= 0)


# ---------------------------------------------------------------------------
# committed golden fixtures (tests/golden/make_golden.py)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "place_*.npz"))))
def test_golden_fixture(oracle, path):
    z = np.load(path, allow_pickle=False)
    pd = {k[2:]: z[k] for k in z.files if k.startswith("p_")}
    p = _abi.default_params(**{k: (tuple(int(x) for x in v) if v.ndim else int(v))
                               for k, v in pd.items()})
    w = synth.Workload(int(z["req"].shape[1]), int(z["cap"].shape[1]), int(z["req"].shape[0]),
                       z["req"], z["cap"], z["used"], z["prio"], z["gang_id"], z["gang_size"],
                       z["topo"], affinity=z["affinity"] if "affinity" in z.files else None)
    r = run(oracle, w, p, threads=4)
    for k in ("node", "score", "status", "used"):
        assert np.array_equal(r[k], z["out_" + k]), k
    assert r["rounds"] == int(z["out_rounds"]) and r["passes"] == int(z["out_passes"])


def test_golden_present():
    assert len(glob.glob(os.path.join(GOLDEN, "place_*.npz"))) >= 4


# ---------------------------------------------------------------------------
# preemption candidates
# ---------------------------------------------------------------------------
def run_pre(oracle, w, p, rn, rq, rp, threads=1):
    out = oracle.preempt(oracle.SnapshotBuf.from_workload(w), p, rn, rq, rp, nthreads=threads)
    assert not isinstance(out, int), f"oracle error {out}"
    return out


def test_kat_preempt_fewest_then_cheapest(oracle):
    # n0 (cap 8, full): running prio 0 (4) and prio 2 (4); n1 (cap 8, full):
    # running prio 1 (8). A prio-2 job needing 4 fits nowhere; evicting the
    # prio-0 job on n0 (cost 0) beats evicting the prio-1 job on n1 (cost 1).
    w = W([[4]], [[8, 8]], used=[[8, 8]], prio=[2])
    r, pr = run_pre(oracle, w, P(), [0, 0, 1], [[4, 4, 8]], [0, 2, 1])
    assert r["status"].tolist() == [_abi.KP_JOB_NO_FIT]
    assert pr["node"].tolist() == [0] and pr["victims"].tolist() == [1]
    assert pr["cost"].tolist() == [0]
    assert (pr["preemptors"], pr["nominated"]) == (1, 1)


def test_kat_preempt_reprieve(oracle):
    # two prio-0 jobs of 2 on a full 4-node: the first (lower index) is spared,
    # the second is evicted; a prio-0 preemptor may evict nobody.
    w = W([[2, 2]], [[4]], used=[[4]], prio=[1, 0])
    r, pr = run_pre(oracle, w, P(), [0, 0], [[2, 2]], [0, 0])
    assert pr["node"].tolist() == [0, -1]
    assert pr["victims"].tolist() == [1, 0]
    assert (pr["preemptors"], pr["nominated"]) == (2, 1)


def test_preempt_validation(oracle):
    w = W([[4]], [[8]], used=[[3]], prio=[1])
    assert oracle.preempt(oracle.SnapshotBuf.from_workload(w), P(), [0], [[4]], [0]) == \
        _abi.KP_EINVAL  # running usage 4 > used 3
    assert oracle.preempt(oracle.SnapshotBuf.from_workload(w), P(), [1], [[1]], [0]) == \
        _abi.KP_EINVAL  # node out of range


def rand_running(seed, w, per_node=3):
    rng = np.random.default_rng(seed)
    rn, rq, rp = [], [], []
    used = w.used.copy()
    for n in range(w.N):
        for _ in range(int(rng.integers(0, per_node + 1))):
            q = (used[:, n] * rng.random(w.D) * 0.6).astype(np.int64)
            rn.append(n)
            rq.append(q)
            rp.append(int(rng.integers(0, 4)))
            used[:, n] -= q
    rq = np.array(rq, np.int64).T.reshape(w.D, len(rn))
    return np.array(rn, np.int32), np.ascontiguousarray(rq), np.array(rp, np.int32)


@pytest.mark.parametrize("seed", range(6))
def test_preempt_matches_python_spec(oracle, seed):
    w = rand_w(200 + seed, J=50 + 9 * seed, N=8 + seed)
    w.used = (w.cap * 0.7).astype(np.int64)
    rn, rq, rp = rand_running(seed, w)
    p = P(w_dim=(1, 3, 2) + (1,) * 5, tie_mode=seed % 2, n_cand=1 + seed % 4)
    r, pr = run_pre(oracle, w, p, rn, rq, rp, threads=2)
    single = [True] * w.J
    for g in set(w.gang_id.tolist()) - {-1}:
        idx = np.nonzero(w.gang_id == g)[0]
        if idx.size > 1:
            for j in idx:
                single[j] = False
    n, v, c = spec_py.preempt(w.req, w.cap, r["used"], w.prio, r["status"], single, rn, rq, rp)
    assert pr["node"].tolist() == n
    assert pr["victims"].tolist() == v
    assert pr["cost"].tolist() == c
    assert pr["preemptors"] == sum(1 for j in range(w.J) if r["status"][j] == 1 and single[j])


def test_config4_generator_occupancy():
    w = synth.config4(4000, 400)
    util = w.used.sum(1) / w.cap.sum(1)
    assert (util >= 0.30).all(), util  # Sum(used)/Sum(cap) >= 0.30 per dim
    rn, rq, rp = w.meta["run_node"], w.meta["run_req"], w.meta["run_prio"]
    back = np.zeros_like(w.used)
    np.add.at(back.T, rn, rq.T)
    assert np.array_equal(back, w.used)  # the victim pool is exactly the usage
    assert rp.min() >= 0 and rp.max() <= 3
