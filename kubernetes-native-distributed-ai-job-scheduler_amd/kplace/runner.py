"""Batched Reconcile runner.

The reference reconciles one CR at a time (LLMServiceReconciler.Reconcile,
internal/controller/llmservice_controller.go:66-174, default one worker) and
leaves each pod to kube-scheduler. Here Reconcile keeps its contract — a key in,
(Result, error) out, never mutating cached objects — but only marks the queue
dirty; `run_batch` (one goroutine in the Go host, debounced) lists every
pending CR and node, packs them, runs ONE kp_place over the whole queue and
writes every CR's Placed condition through the status writer. A placement is
a pure function of the snapshot, so a new leader after fail-over recomputes
the same assignment (controller-runtime leader election,
cmd/manager/main.go:162-163).
"""
from __future__ import annotations

import logging
import threading
import time
from dataclasses import dataclass

from . import binder, packer

log = logging.getLogger("kplace.runner")


@dataclass
class Result:
    """ctrl.Result: Requeue / RequeueAfter (seconds)."""
    requeue: bool = False
    requeue_after: float = 0.0


class BatchRunner:
    def __init__(self, placer, list_crs, list_nodes, write_status, params, node_usage=None,
                 running=None, metrics=None, debounce_s: float = 0.02, pod_nodes=None,
                 retry_s: float = 1.0):
        """placer: a kplace.engine.Placer (anything with .place(w, p), and
        .load_running/.preempt for nominations); list_crs / list_nodes:
        informer-cache listers; write_status(key, status): the status
        subresource update; node_usage(): {node: {dim: used}}; running():
        (node_idx, req [D,R], prio) victim pool or None; pod_nodes():
        {(namespace, pod): node} for CacheStrategy=shared."""
        self.placer, self.list_crs, self.list_nodes = placer, list_crs, list_nodes
        self.write_status, self.params = write_status, params
        self.node_usage, self.running, self.metrics = node_usage, running, metrics
        self.debounce_s, self.pod_nodes, self.retry_s = debounce_s, pod_nodes, retry_s
        self.failures = 0
        self._dirty = threading.Event()
        self._lock = threading.Lock()
        self.last = None

    # controller-runtime Reconcile contract: mark dirty, return Result{}
    def reconcile(self, key) -> tuple[Result, Exception | None]:
        self._dirty.set()
        return Result(), None

    def run_batch(self) -> dict:
        """Snapshot -> one batched placement -> statuses. Returns a summary."""
        with self._lock:
            self._dirty.clear()
            crs = list(self.list_crs())
            nodes = list(self.list_nodes())
            pk = packer.pack(crs, nodes, self.node_usage() if self.node_usage else None,
                             self.pod_nodes() if self.pod_nodes else None)
            t = time.perf_counter()
            res = self.placer.place(pk.workload, self.params)
            pre = None
            if self.running is not None and hasattr(self.placer, "preempt"):
                pool = self.running()
                if pool is not None:
                    self.placer.load_running(*pool)
                    pre = self.placer.preempt()
            dt = time.perf_counter() - t
            if self.metrics is not None:
                self.metrics.record(dt, res)
            conds = binder.conditions(pk, res, pre)
            by_key = {((c.get("metadata", {}) or {}).get("namespace", "default"),
                       c["metadata"]["name"]): c for c in crs}
            for key, cond in conds.items():
                self.write_status(key, binder.status_with_condition(by_key[key], cond))
            self.last = {"crs": len(crs), "jobs": pk.workload.J, "nodes": len(nodes),
                         "placed": res["placed"], "rounds": res["rounds"], "seconds": dt,
                         "invalid_crs": len(pk.invalid), "bad_nodes": len(pk.bad_nodes)}
            return self.last

    def serve(self, stop: threading.Event, timeout: float = 0.5) -> None:
        """The batch goroutine: wait for a dirty mark, debounce, run a batch.
        A failed batch (engine error, lister error) is logged and retried
        after `retry_s` — like a Reconcile error's rate-limited requeue — and
        never ends the loop."""
        while not stop.is_set():
            if self._dirty.wait(timeout):
                time.sleep(self.debounce_s)
                try:
                    self.run_batch()
                    self.failures = 0
                except Exception:  # noqa: BLE001 -- the loop must survive any batch
                    self.failures += 1
                    log.exception("placement batch failed (%d in a row); retrying",
                                  self.failures)
                    self._dirty.set()
                    stop.wait(self.retry_s)
