"""Thin Python handle over libkplace.so (the product is the C-ABI library).

Every method maps 1:1 onto an entry point of include/kplace.h, with the same
argument meaning and error behaviour: a negative return code raises
KPlaceError carrying the code and kp_strerror(). There is no fallback: if the
shared library or a gfx950 device is missing, construction fails.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _abi

_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        _lib = _abi.load_library()
    return _lib


class KPlaceError(RuntimeError):
    def __init__(self, code: int, where: str, detail: str = ""):
        self.code = code
        self.detail = detail
        msg = lib().kp_strerror(code).decode(errors="replace")
        super().__init__(f"{where}: kplace error {code} ({msg})" + (f": {detail}" if detail else ""))


def _check(rc: int, where: str, h=None) -> None:
    if rc != _abi.KP_OK:
        detail = ""
        if h is not None and h.value:
            detail = last_error(h)
        raise KPlaceError(rc, where, detail)


def last_error(h) -> str:
    """kp_last_error_r: the context's last error text, copied under its lock
    (safe while other threads call into the same context)."""
    buf = C.create_string_buffer(512)
    lib().kp_last_error_r(h, buf, len(buf))
    return buf.value.decode(errors="replace")


def _ptr(a, t):
    return None if a is None else a.ctypes.data_as(C.POINTER(t))


def _c(a, dt):
    return None if a is None else np.ascontiguousarray(a, dtype=dt)


def default_params_lib() -> _abi.Params:
    p = _abi.Params()
    lib().kp_params_default(C.byref(p))
    return p


def unique_id() -> bytes:
    buf = C.create_string_buffer(128)
    _check(lib().kp_dist_unique_id(buf), "kp_dist_unique_id")
    return buf.raw


class Placer:
    """One kp_ctx: a GPU (one rank of a multi-process job) and its resident
    node table."""

    def __init__(self, device: int = 0, world_size: int = 1, rank: int = 0,
                 nccl_id: bytes | None = None, max_pairs_matrix: int = 0,
                 allgather=None, gpu_ids=None):
        """`allgather` (multi-process without RCCL): a callable taking this
        rank's bytes and returning every rank's bytes concatenated in rank
        order (kp_set_allgather). `gpu_ids` (a list): one context over
        several GPUs of this process (kp_create_multi); device / world_size /
        rank / nccl_id are then unused."""
        cfg = _abi.Config()
        cfg.device = device
        cfg.world_size = world_size
        cfg.rank = rank
        self._id = None
        if nccl_id is not None:
            self._id = C.create_string_buffer(nccl_id, 128)
            cfg.nccl_id = C.cast(self._id, C.c_void_p)
        cfg.max_pairs_matrix = max_pairs_matrix
        h = C.c_void_p()
        if gpu_ids is not None:
            ids = np.ascontiguousarray(gpu_ids, dtype=np.int32)
            _check(lib().kp_create_multi(C.byref(h), _ptr(ids, C.c_int32), ids.size,
                                         C.byref(cfg)), "kp_create_multi")
        else:
            _check(lib().kp_create(C.byref(h), C.byref(cfg)), "kp_create")
        self._h = h
        self.J = self.N = self.D = 0
        self._cb = None
        if allgather is not None:
            def _cb(user, send, nbytes, recv):
                try:
                    out = allgather(C.string_at(send, nbytes))
                    if len(out) != nbytes * world_size:
                        return 1
                    C.memmove(recv, out, len(out))
                    return 0
                except Exception:  # never unwind through the C frames
                    return 1
            self._cb = _abi.ALLGATHER_FN(_cb)
            _check(lib().kp_set_allgather(self._h, self._cb, None), "kp_set_allgather", self._h)

    def last_error(self) -> str:
        """kp_last_error: detail of the last failed call on this context."""
        return last_error(self._h)

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().kp_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ---- staged interface -------------------------------------------------
    def load_nodes(self, cap, used=None, topo=None) -> None:
        cap = _c(cap, np.int64)
        D, N = cap.shape
        used = _c(used, np.int64)
        topo = _c(topo, np.int32)
        _check(lib().kp_load_nodes(self._h, N, D, _ptr(cap, C.c_int64), _ptr(used, C.c_int64),
                                   _ptr(topo, C.c_int32)), "kp_load_nodes", self._h)
        self.N, self.D = N, D

    def load_jobs(self, req, prio=None, gang_id=None, gang_size=None, affinity=None) -> None:
        req = _c(req, np.int64)
        J = req.shape[1]
        prio, gang_id, gang_size = _c(prio, np.int32), _c(gang_id, np.int32), _c(gang_size, np.int32)
        affinity = _c(affinity, np.int32)
        _check(lib().kp_load_jobs(self._h, J, _ptr(req, C.c_int64), _ptr(prio, C.c_int32),
                                  _ptr(gang_id, C.c_int32), _ptr(gang_size, C.c_int32),
                                  _ptr(affinity, C.c_int32)),
               "kp_load_jobs", self._h)
        self.J = J

    def solve(self, params: _abi.Params) -> dict:
        r = _abi.Result()
        _check(lib().kp_solve(self._h, C.byref(params), C.byref(r)), "kp_solve", self._h)
        return dict(rounds=r.rounds, passes=r.passes, placed=r.placed_jobs,
                    unplaced=r.unplaced_jobs, units=r.units, pairs=r.pairs_scored)

    def fetch(self, want_used: bool = True) -> dict:
        node = np.empty(self.J, np.int32)
        score = np.empty(self.J, np.int32)
        status = np.empty(self.J, np.int32)
        used = np.empty((self.D, self.N), np.int64) if want_used else None
        r = _abi.Result(_ptr(node, C.c_int32), _ptr(score, C.c_int32), _ptr(status, C.c_int32),
                        _ptr(used, C.c_int64))
        _check(lib().kp_fetch(self._h, C.byref(r)), "kp_fetch", self._h)
        return dict(node=node, score=score, status=status, used=used, rounds=r.rounds,
                    passes=r.passes, placed=r.placed_jobs, unplaced=r.unplaced_jobs,
                    units=r.units, pairs=r.pairs_scored)

    def apply_delta(self, node_idx, delta) -> None:
        node_idx = _c(node_idx, np.int32)
        delta = _c(delta, np.int64)
        K = node_idx.shape[0]
        _check(lib().kp_apply_delta(self._h, _ptr(node_idx, C.c_int32), _ptr(delta, C.c_int64), K),
               "kp_apply_delta", self._h)

    def load_running(self, node, req, prio) -> None:
        """kp_load_running: the victim pool (running jobs) of the resident
        node table, req [D, R]."""
        node, req, prio = _c(node, np.int32), _c(req, np.int64), _c(prio, np.int32)
        R = node.shape[0]
        _check(lib().kp_load_running(self._h, R, _ptr(node, C.c_int32), _ptr(req, C.c_int64),
                                     _ptr(prio, C.c_int32)), "kp_load_running", self._h)

    def preempt(self) -> dict:
        """kp_preempt after a solve: per-job nominated node / victims / cost."""
        node = np.empty(self.J, np.int32)
        vict = np.empty(self.J, np.int32)
        cost = np.empty(self.J, np.int64)
        r = _abi.Preemption(_ptr(node, C.c_int32), _ptr(vict, C.c_int32), _ptr(cost, C.c_int64))
        _check(lib().kp_preempt(self._h, C.byref(r)), "kp_preempt", self._h)
        return dict(node=node, victims=vict, cost=cost, preemptors=r.preemptors,
                    nominated=r.nominated, pairs=r.pairs_scored)

    def reset_nodes(self) -> None:
        _check(lib().kp_reset_nodes(self._h), "kp_reset_nodes", self._h)

    def score(self, params: _abi.Params, lo: int, hi: int):
        rows = hi - lo
        sc = np.empty((rows, self.N), np.int32)
        mk = np.empty((rows, (self.N + 63) // 64), np.uint64)
        _check(lib().kp_score(self._h, C.byref(params), lo, hi, _ptr(sc, C.c_int32),
                              _ptr(mk, C.c_uint64)), "kp_score", self._h)
        return sc, mk

    def score_dev(self, params: _abi.Params, lo: int, hi: int, score_ptr: int | None,
                  mask_ptr: int | None) -> None:
        """kp_score_dev: the filter + score pass into caller-owned device memory
        (raw device addresses, e.g. torch.Tensor.data_ptr(); rows of
        Ns = round_up(N, 64) int32 scores and Ns / 64 uint64 mask words)."""
        _check(lib().kp_score_dev(self._h, C.byref(params), lo, hi, C.c_void_p(score_ptr or None),
                                  C.c_void_p(mask_ptr or None)), "kp_score_dev", self._h)

    def set_profiling(self, on) -> None:
        """False/0 off, True/1 filter+score events, 2 also the per-round phase split."""
        level = int(on) if not isinstance(on, bool) else (1 if on else 0)
        _check(lib().kp_set_profiling(self._h, level), "kp_set_profiling", self._h)

    def timing(self) -> dict:
        t = _abi.Timing()
        _check(lib().kp_last_timing(self._h, C.byref(t)), "kp_last_timing", self._h)
        return {k: getattr(t, k) for k, _ in _abi.Timing._fields_}

    def timing_shards(self) -> list:
        """kp_last_timing_shards: one timing dict per shard (kp_create_multi),
        a single one for a one-GPU / one-rank context."""
        n = lib().kp_last_timing_shards(self._h, None, 0)
        _check(min(n, 0), "kp_last_timing_shards", self._h)
        ts = (_abi.Timing * n)()
        got = lib().kp_last_timing_shards(self._h, ts, n)
        _check(min(got, 0), "kp_last_timing_shards", self._h)
        return [{k: getattr(t, k) for k, _ in _abi.Timing._fields_} for t in ts]

    # ---- one-shot ----------------------------------------------------------
    def place(self, w, params: _abi.Params) -> dict:
        """kp_place on a synth.Workload-like object (req/cap/used/prio/gang_id/
        gang_size/topo attributes)."""
        req, cap = _c(w.req, np.int64), _c(w.cap, np.int64)
        D, J = req.shape
        N = cap.shape[1]
        used, prio = _c(w.used, np.int64), _c(w.prio, np.int32)
        gid, gsz, topo = _c(w.gang_id, np.int32), _c(w.gang_size, np.int32), _c(w.topo, np.int32)
        aff = _c(getattr(w, "affinity", None), np.int32)
        snap = _abi.Snapshot(J, N, D, _ptr(req, C.c_int64), _ptr(cap, C.c_int64),
                             _ptr(used, C.c_int64), _ptr(prio, C.c_int32), _ptr(gid, C.c_int32),
                             _ptr(gsz, C.c_int32), _ptr(topo, C.c_int32), _ptr(aff, C.c_int32))
        node = np.empty(J, np.int32)
        score = np.empty(J, np.int32)
        status = np.empty(J, np.int32)
        used_out = np.empty((D, N), np.int64)
        r = _abi.Result(_ptr(node, C.c_int32), _ptr(score, C.c_int32), _ptr(status, C.c_int32),
                        _ptr(used_out, C.c_int64))
        _check(lib().kp_place(self._h, C.byref(snap), C.byref(params), C.byref(r)), "kp_place", self._h)
        self.J, self.N, self.D = J, N, D
        return dict(node=node, score=score, status=status, used=used_out, rounds=r.rounds,
                    passes=r.passes, placed=r.placed_jobs, unplaced=r.unplaced_jobs,
                    units=r.units, pairs=r.pairs_scored)
