"""Placement metrics, in the style of the reference's
pkg/metrics/metrics.go:120-169 (Prometheus collectors on one registry, helper
recorders): batch latency histogram (DefBuckets, as ReconcileDuration), pairs
scored, jobs by outcome, rounds per batch."""
from __future__ import annotations

from prometheus_client import CollectorRegistry, Counter, Histogram

# prometheus.DefBuckets (pkg/metrics/metrics.go:143)
DEF_BUCKETS = (0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1.0, 2.5, 5.0, 10.0)


class PlacementMetrics:
    def __init__(self, registry: CollectorRegistry | None = None):
        self.registry = registry or CollectorRegistry()
        self.batch_latency = Histogram(
            "kubeinfer_placement_batch_latency_seconds",
            "Wall time of one batched placement (snapshot in host memory to assignment in host "
            "memory)", buckets=DEF_BUCKETS, registry=self.registry)
        self.pairs_scored = Counter(
            "kubeinfer_placement_pairs_scored_total", "Job-node pairs scored",
            registry=self.registry)
        self.assigned = Counter(
            "kubeinfer_placement_jobs_total", "Pending replicas by placement outcome",
            ["result"], registry=self.registry)
        self.rounds = Histogram(
            "kubeinfer_placement_rounds", "Auction rounds per batch",
            buckets=(1, 2, 4, 8, 16, 32, 64, 128, 256), registry=self.registry)

    def record(self, seconds: float, result: dict) -> None:
        self.batch_latency.observe(seconds)
        self.pairs_scored.inc(int(result.get("pairs", 0)))
        self.rounds.observe(int(result.get("rounds", 0)))
        placed = int(result.get("placed", 0))
        self.assigned.labels("placed").inc(placed)
        self.assigned.labels("unplaced").inc(int(result.get("unplaced", 0)))
