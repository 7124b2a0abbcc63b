#!/usr/bin/env python3
"""bench.py — full-queue placement on MI355X (BASELINE.json config #3).

A "step" is one full placement of the pending queue (100k jobs x 10k nodes,
gangs of {1,2,4,8}, 8-GPU xGMI-island nodes) with the snapshot already
resident in HBM: kp_reset_nodes (device copy of the loaded usage) + kp_solve
(every filter+score pass, top-K select, acceptance pass and commit, plus the
RCCL candidate exchange when N>1). `value` = J*N job-node pairs resolved per
second of whole-job wall time (max over ranks); the total problem is fixed as
N grows (strong scaling). Synthetic data (splitmix64 generator).

Multi-GPU: one process per GPU (torch.distributed.run); the control plane
(barrier, unique-id broadcast, max-reduce of times) runs on gloo, the data
path's candidate exchange on RCCL inside libkplace.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "kubernetes-native-distributed-ai-job-scheduler_amd")
sys.path.insert(0, PKG)

import numpy as np  # noqa: E402

from kplace import _abi, synth  # noqa: E402
from kplace.engine import Placer, unique_id  # noqa: E402

METRIC = "job-node pairs scored/sec + full-queue placement latency (100k jobs × 10k nodes)"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def cpu_baseline(args):
    """Timed CPU restatement (oracle/, test infrastructure) on a bounded
    sample of the same workload family: config #3 shrunk by `cpu_shrink` in
    both jobs and nodes (1/shrink^2 of the pairs), full placement."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_bind as ob
    J, N = args.jobs // args.cpu_shrink, args.nodes // args.cpu_shrink
    w = synth.config3(J, N)
    p = _abi.default_params(**synth.CONFIG_PARAMS[3])
    threads = min(16, os.cpu_count() or 1)
    sb = ob.SnapshotBuf.from_workload(w)
    t = time.perf_counter()
    r = ob.place(sb, p, nthreads=threads)
    dt = time.perf_counter() - t
    return {"value": J * N / dt, "unit": "pairs/s", "cores": threads, "kind": "port",
            "sample": f"oracle/kp_oracle.c full placement of config3 {J}x{N} "
                      f"(1/{args.cpu_shrink**2} of the pairs), {r['rounds']} rounds, "
                      f"{dt*1e3:.0f} ms, OpenMP {threads} threads"}


def streaming(args):
    """BASELINE config #5: a 1M-job trace replayed in micro-batches against a
    50k-node resident table; after each batch a deterministic 20% of the
    running jobs complete (negative kp_apply_delta). Per-batch latency =
    apply the previous completions + load the batch + solve + fetch, host
    wall clock (the latency-bound small-batch path)."""
    cap, topo, req, prio = synth.config5_trace(args.stream_jobs, args.stream_nodes)
    p = _abi.default_params(**synth.CONFIG_PARAMS[5])
    B = args.stream_batch
    lat = []
    placed = 0
    with Placer(device=int(os.environ.get("LOCAL_RANK", "0"))) as pl:
        pl.load_nodes(cap, None, topo)
        run_node = np.zeros(0, np.int32)
        run_job = np.zeros(0, np.int64)
        pend_n, pend_d = None, None
        for b in range(args.stream_jobs // B):
            lo, hi = b * B, (b + 1) * B
            rq = np.ascontiguousarray(req[:, lo:hi])
            t = time.perf_counter()
            if pend_n is not None and pend_n.size:
                pl.apply_delta(pend_n, pend_d)
            pl.load_jobs(rq, prio[lo:hi])
            pl.solve(p)
            g = pl.fetch(want_used=False)
            lat.append(time.perf_counter() - t)
            ok = g["node"] >= 0
            placed += int(ok.sum())
            run_node = np.concatenate([run_node, g["node"][ok]])
            run_job = np.concatenate([run_job, lo + np.nonzero(ok)[0]])
            done = synth.config5_completions(b, run_job)
            pend_n = np.ascontiguousarray(run_node[done])
            pend_d = np.ascontiguousarray(-req[:, run_job[done]])
            run_node, run_job = run_node[~done], run_job[~done]
    lat_ms = np.array(lat) * 1e3
    return {"config": f"#5 streaming: {args.stream_jobs} jobs in {B}-job micro-batches vs "
                      f"{args.stream_nodes} nodes, 20% completions per batch",
            "batches": len(lat), "p50_ms": float(np.percentile(lat_ms, 50)),
            "p99_ms": float(np.percentile(lat_ms, 99)), "max_ms": float(lat_ms.max()),
            "jobs_per_s": args.stream_jobs / float(np.sum(lat)), "placed_jobs": placed}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--jobs", type=int, default=100_000)
    ap.add_argument("--nodes", type=int, default=10_000)
    ap.add_argument("--cpu-shrink", type=int, default=4)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--out", default=None, help="also write the JSON line here")
    ap.add_argument("--stream-jobs", type=int, default=1_000_000)
    ap.add_argument("--stream-batch", type=int, default=5_000)
    ap.add_argument("--stream-nodes", type=int, default=50_000)
    ap.add_argument("--no-stream", action="store_true")
    ap.add_argument("--no-kernel-events", action="store_true",
                    help="time the steps without per-launch HIP events (no roofline)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)

    nid = None
    if world > 1:
        obj = [unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        nid = obj[0]

    w = synth.config3(args.jobs, args.nodes)
    p = _abi.default_params(**synth.CONFIG_PARAMS[3])
    pl = Placer(device=local, world_size=world, rank=rank, nccl_id=nid)
    pl.load_nodes(w.cap, w.used, w.topo)
    pl.load_jobs(w.req, w.prio, w.gang_id, w.gang_size)

    def barrier():
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        pl.reset_nodes()
        pl.solve(p)
    pl.set_profiling(not args.no_kernel_events)
    barrier()
    t0 = time.perf_counter()
    score_ms = score_b = select_ms = 0.0
    launches = 0
    st = None
    for _ in range(args.steps):
        pl.reset_nodes()
        st = pl.solve(p)  # synchronous: returns after the device finished
        tm = pl.timing()
        score_ms += tm["score_ms"]
        score_b += tm["score_bytes"]
        select_ms += tm["select_ms"]
        launches += tm["score_launches"]
    barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        import torch
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ms = dt * 1e3 / args.steps
    if rank != 0:
        dist.barrier()
        return
    pairs = float(args.jobs) * args.nodes
    achieved = (score_b / 1e9) / (score_ms / 1e3) if score_ms > 0 else 0.0
    traffic, traffic_src = None, None
    pmc = os.path.join(REPO, "profiles", "r01_pmc.json")
    if os.path.exists(pmc):  # HBM-side bytes per launch from rocprofv3 PMC passes
        with open(pmc) as f:
            k = [v for n, v in json.load(f)["kernels"].items() if n.startswith("k_score")]
        if k:
            traffic = k[0]["traffic_bytes_per_launch"]
            traffic_src = "profiles/r01_pmc.json (FETCH_SIZE x2 + WRITE_SIZE, tools/gpu_evidence.sh)"
    out = {
        "metric": METRIC,
        "value": pairs / (ms / 1e3),
        "unit": "pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic (splitmix64 config #3 generator, SURVEY.md §8d)",
        "config": {"workload": "config3: 100k jobs x 10k nodes x 4 dims, gangs {1,2,4,8}, "
                               "A/B 8-GPU nodes, bin-pack + spread + GPU-fit",
                   "jobs": args.jobs, "nodes": args.nodes, "dims": 4,
                   "units": st["units"], "rounds": st["rounds"], "passes": st["passes"],
                   "placed_jobs": st["placed"], "pairs_scored": st["pairs"],
                   "parallelism": f"job-row shards x{world}"},
        "latency_ms": ms,
        "roofline": {"bound": "hbm", "kernel": "k_score (filter+score, materialised matrix)",
                     "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_unit": "bytes per launch", "traffic_source": traffic_src,
                     "algorithmic_bytes_per_launch": score_b / max(launches, 1),
                     "frac_of_achievable_6290": achieved / 6290.0,
                     "launches_per_step": launches / args.steps,
                     "avg_launch_ms": score_ms / max(launches, 1)},
    }
    if not args.no_cpu_baseline and world == 1:
        out["cpu_baseline"] = cpu_baseline(args)
    if not args.no_stream and world == 1:
        out["streaming"] = streaming(args)
    line = json.dumps(out)
    print(line, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")
    if dist is not None:
        dist.barrier()


if __name__ == "__main__":
    main()
