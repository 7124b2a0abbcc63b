"""CPU checks of the exact utilisation arithmetic.

1. The oracle: a full node scores S in every dim (the r01 reciprocal form gave
   99 for x = cap = 128000 at S = 100), LeastAllocated follows kube-scheduler's
   leastRequestedScore, boundaries x in {0, 1, cap-1, cap} across cap ranges
   up to 2^56, all against Python big-integer arithmetic.
2. The GPU kernels' 32-bit division (kp_device.hpp div_prep / div_floor32 and
   the 24-bit fast path of k_score32), emulated instruction for instruction in
   numpy (v_mul_u32_u24 = low 32 bits of a 24 x 24-bit product), over caps
   of every mode and the boundary x values: exhaustive for cap < 5000.
"""
import numpy as np
import pytest

from kplace import _abi, synth

M32 = np.uint64(0xFFFFFFFF)
M24 = np.uint64(0xFFFFFF)
E_FLAG, W_FLAG = 0x100, 0x200


def div_prep(c: int, S: int):
    """Restatement of kp_device.hpp div_prep (per node and dim)."""
    if c == 0:
        return 0, 1 | E_FLAG
    fl = c.bit_length() - 1
    if c < (1 << 12):
        kE = 2 * fl + 2
        top = S << kE
        RE = top // c + 1
        if top + c < (1 << 32) and RE < (1 << 24):
            return RE, kE | E_FLAG
    kC = fl + 1
    if c < (1 << 24) and (S << kC) < (1 << 32):
        return (S << kC) // c, kC
    return (S << 32) // c, 32 | W_FLAG


def mul24(a, b):
    return ((a & M24) * (b & M24)) & M32


def fast_path(x, c, R, K, S, use_check):
    """k_score32's non-W form: t = mul24(x, R) >> k (+ remainder check)."""
    k = (K & np.uint64(63))
    t = mul24(x, R) >> k
    cc = np.where(c == 0, np.uint64(1), c)
    if not use_check:
        return t, None
    r = (mul24(x, np.uint64(S)) - mul24(t, cc)) & M32
    up = r >= cc
    t = t + up.astype(np.uint64)
    r = np.where(up, (r - cc) & M32, r)
    return t, r != 0


def generic_path(x, c, R, K, S):
    """div_floor32: 64-bit products, any mode."""
    k = (K & np.uint64(63))
    t = (x * R) >> k
    cc = np.where(c == 0, np.uint64(1), c)
    r = x * np.uint64(S) - t * cc
    up = r >= cc
    t = t + up.astype(np.uint64)
    r = np.where(up, r - cc, r)
    return t, r != 0


def cap_samples(rng):
    caps = list(range(0, 5000))
    for b in range(12, 32):
        caps += [(1 << b) - 1, 1 << b, (1 << b) + 1]
    caps += rng.integers(1 << 12, 1 << 24, 3000).tolist()
    caps += rng.integers(1 << 24, 1 << 32, 3000).tolist()
    caps += [128000, 192000, 64000, 96000, 1048576, 2097152, 524288, 786432, 8 * 294912,
             4 * 196608, (1 << 32) - 1]
    return sorted(set(caps))


@pytest.mark.parametrize("S", [1, 7, 100, 128, 1000, 1024])
def test_kernel_division_emulated(S):
    rng = np.random.default_rng(S)
    caps = cap_samples(rng)
    RK = [div_prep(c, S) for c in caps]
    c = np.array(caps, np.uint64)
    R = np.array([r for r, _ in RK], np.uint64)
    K = np.array([k for _, k in RK], np.uint64)
    isE = (K & np.uint64(E_FLAG)) != 0
    isW = (K & np.uint64(W_FLAG)) != 0
    # operand bounds the fast path relies on (C and E modes)
    fast = ~isW
    assert (R[fast] < (1 << 24)).all() and (c[fast] < (1 << 24)).all()
    assert ((K[fast] & np.uint64(63)) <= 24).all()
    xs = [np.zeros_like(c), np.minimum(c, 1), np.where(c > 0, c - 1, 0), c,
          (c.astype(np.float64) * rng.random(c.size)).astype(np.uint64),
          (c.astype(np.float64) * rng.random(c.size)).astype(np.uint64)]
    for x in xs:
        want_f = np.array([(int(a) * S) // int(b) if b else 0 for a, b in zip(x, c)], np.uint64)
        want_c = np.array([-((-int(a) * S) // int(b)) if b else 0 for a, b in zip(x, c)], np.uint64)
        # generic form: every mode
        t, nz = generic_path(x, c, R, K, S)
        assert np.array_equal(t, want_f)
        assert np.array_equal(t + nz.astype(np.uint64), want_c)
        # fast form with the remainder check: C and E lanes (mixed waves)
        t, nz = fast_path(x[fast], c[fast], R[fast], K[fast], S, True)
        assert np.array_equal(t, want_f[fast])
        assert np.array_equal(t + nz.astype(np.uint64), want_c[fast])
        # fast form without the check: exact on E lanes (all-E waves)
        t, _ = fast_path(x[isE], c[isE], R[isE], K[isE], S, False)
        assert np.array_equal(t, want_f[isE])
        # the 32-bit product of the fast form never wraps on feasible pairs
        assert (x[fast] * R[fast] < (1 << 32)).all()


def test_modes_cover_the_config_shapes():
    # every cap of the synthetic node shapes takes the full-rate path
    for cap in synth.SHAPES.reshape(-1):
        R, K = div_prep(int(cap), 100)
        assert not (K & W_FLAG), cap
    assert div_prep(8, 100)[1] & E_FLAG  # GPU counts: no remainder check


# ---------------------------------------------------------------------------
# oracle
# ---------------------------------------------------------------------------
def P(**kw):
    base = dict(w_dim=(1,) * 8, gpu_dim=-1, w_gpu_fit=0, w_spread=0, tie_mode=0)
    base.update(kw)
    return _abi.default_params(**base)


def one_node_score(oracle, q, cap, used, p):
    q = np.array(q, np.int64).reshape(-1, 1)
    cap = np.array(cap, np.int64).reshape(-1, 1)
    used = np.array(used, np.int64).reshape(-1, 1)
    sc, _ = oracle.score(oracle.SnapshotBuf(q, cap, used), p, 0, 1)
    return int(sc[0, 0])


def test_full_node_scores_S(oracle):
    # a completely full A-shape node scored 99 in cpu / gpu_mem
    a = synth.SHAPES[0]
    for d in range(4):
        w = [0] * 8
        w[d] = 1
        s = one_node_score(oracle, a.tolist(), a.tolist(), [0] * 4, P(w_dim=w))
        assert s == 100, (d, s)
    s = one_node_score(oracle, a.tolist(), a.tolist(), [0] * 4, P(w_dim=(1, 1, 4, 2)))
    assert s == 800


@pytest.mark.parametrize("most", [True, False])
def test_oracle_boundaries_exact(oracle, most):
    rng = np.random.default_rng(7 + most)
    caps = [1, 2, 3, 7, 100, 101, 4095, 4096, (1 << 24) - 1, 1 << 24, (1 << 31) + 5,
            (1 << 32) - 1, 1 << 32, (1 << 32) + 1, 3 ** 30, (1 << 50) + 12345, 1 << 56]
    caps += rng.integers(1, 1 << 56, 20, dtype=np.int64).tolist()
    for S in (1, 100, 1023, 1024):
        p = P(util_scale=S, score_mode=0 if most else 1)
        for c in caps:
            for x in {0, 1, c - 1, c, c // 3}:
                if x < 0 or x > c:
                    continue
                got = one_node_score(oracle, [x], [c], [0], p)
                want = (x * S) // c if most else ((c - x) * S) // c
                assert got == want, (S, c, x, got, want)


def test_oracle_least_allocated_kube_formula(oracle):
    # leastRequestedScore = (cap - req) * 100 / cap, per dim, integer division
    p = P(score_mode=1, w_dim=(1, 1))
    assert one_node_score(oracle, [3, 1], [8, 3], [0, 0], p) == (5 * 100) // 8 + (2 * 100) // 3


def test_oracle_affinity_bonus(oracle):
    # two identical empty nodes in domains 0 and 1; the job prefers domain 1
    w = synth.Workload(1, 2, 1, np.array([[2]], np.int64), np.array([[8, 8]], np.int64),
                       np.zeros((1, 2), np.int64), np.zeros(1, np.int32), np.full(1, -1, np.int32),
                       np.ones(1, np.int32), np.array([0, 1], np.int32),
                       affinity=np.array([1], np.int32))
    r = oracle.place(oracle.SnapshotBuf.from_workload(w), P(w_affinity=40), nthreads=1)
    assert r["node"].tolist() == [1] and r["score"].tolist() == [25 + 40]
    r = oracle.place(oracle.SnapshotBuf.from_workload(w), P(w_affinity=0), nthreads=1)
    assert r["node"].tolist() == [0] and r["score"].tolist() == [25]
    # gang members must agree on the affinity domain
    w2 = synth.Workload(2, 2, 1, np.array([[2, 2]], np.int64), w.cap, w.used,
                        np.zeros(2, np.int32), np.array([5, 5], np.int32), np.full(2, 2, np.int32),
                        w.topo, affinity=np.array([1, 0], np.int32))
    assert oracle.place(oracle.SnapshotBuf.from_workload(w2), P(), 1) == _abi.KP_EINVAL
