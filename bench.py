#!/usr/bin/env python3
"""bench.py — full-queue placement on MI355X (BASELINE.json config #3).

A "step" is one full placement of the pending queue (100k jobs x 10k nodes,
gangs of {1,2,4,8}, 8-GPU xGMI-island nodes) with the snapshot already
resident in HBM: kp_reset_nodes (device copy of the loaded usage) + kp_solve
(every filter+score pass, top-K select, acceptance pass and commit, plus the
candidate exchange when N>1). `value` = J*N job-node pairs resolved per second
of whole-job wall time (max over ranks); the total problem is fixed as N grows
(strong scaling). Synthetic data (splitmix64 generator).

Beside the step (same run, outside the timed steps):
  latency_ms      kp_place from host arrays: validate + upload the snapshot,
                  solve, download the assignment (the headline "full-queue
                  placement latency"; the reference's analogue is
                  the reconcile histogram around Reconcile,
                  internal/controller/llmservice_controller.go:70-73);
  phases          one extra solve with per-round phase events: candidate
                  phase / candidate exchange / passes (max over ranks);
  score_matrix    the materialised int32 score matrix + feasibility bitmask
                  of the whole queue (kp_score_dev; on N GPUs each rank its
                  row block) against the HBM roofline;
  config2         BASELINE config #2 (10k x 1k bin-pack, 1 GPU): device solve,
                  pairs/s, host->host latency, the oracle on the same snapshot;
  config4         BASELINE config #4 (200k x 20k, running jobs filling every
                  dim to >= 30% of its capacity): solve + kp_preempt on the
                  same N GPUs (row-sharded, collective), with its phase split
                  and, at N = 1, the oracle timed beside it on a stated sample;
  streaming       BASELINE config #5 (1M-job trace, 5k micro-batches, 50k nodes),
                  with the oracle timed beside it on the first batches (N = 1);
  cpu_baseline    the CPU restatement (oracle/, test infrastructure) on the SAME
                  full config #3, on 1 thread and on every host core given to
                  this job.

Multi-GPU: one process per GPU (torch.distributed.run); the control plane
(barrier, unique-id broadcast, max-reduce of times) runs on gloo, the data
path's candidate exchange on RCCL inside libkplace. `--gpus N` without a
launcher re-launches itself under torch.distributed.run (before anything
touches a GPU); `--single-process` drives the N GPUs from this one process
instead (kp_create_multi: one worker thread per GPU inside the library).
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import re
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "kubernetes-native-distributed-ai-job-scheduler_amd")
sys.path.insert(0, PKG)

import numpy as np  # noqa: E402

from kplace import _abi, synth  # noqa: E402

METRIC = "job-node pairs scored/sec + full-queue placement latency (100k jobs × 10k nodes)"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
# VALU peak for 32-bit integer ops: 256 CUs x 4 SIMDs x 32 lanes/cycle (a wave64
# VALU op issues over 2 cycles on a SIMD-32, MI355X_MICROARCH.md) x 2.4 GHz
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12
# measured: independent v_add_u32 / compare-select / sub-min chains on every
# SIMD issue ~56 T lane-ops/s (tools/valu_peak.hip, profiles/r05_valu_peak.txt:
# 32 lanes per clock at the ~1.7 GHz the chip holds under that load)
VALU_ACHIEVABLE_TOPS = 56.4


def newest(kind: str) -> list:
    """profiles/rNN_<kind>.json, newest round first (the evidence the line cites)."""
    d = os.path.join(REPO, "profiles")
    names = [n for n in os.listdir(d) if re.fullmatch(r"r\d\d_" + kind + r"\.json", n)] if os.path.isdir(d) else []
    return sorted(names, reverse=True)


def progress(msg: str) -> None:
    """A progress line on stderr (long legs; the JSON line stays on stdout)."""
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def host_cores() -> int:
    """Cores this job may use: the box's share (OMP_NUM_THREADS is set to it
    on the GPU pool; os.cpu_count() there shows the whole machine)."""
    n = os.environ.get("OMP_NUM_THREADS")
    return max(1, int(n)) if n and n.isdigit() else (os.cpu_count() or 1)


def cpu_baseline(args, w, p):
    """The CPU restatement (oracle/kp_oracle.c, OpenMP candidate phase) on the
    same full config #3, single-threaded and on every host core."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_bind as ob
    sb = ob.SnapshotBuf.from_workload(w)
    pairs = float(w.J) * w.N
    out = {}
    for label, threads in (("all_cores", host_cores()), ("single", 1)):
        if label == "single" and args.cpu_single_sample < 1.0:
            # bounded sample: the first rounds of the same solve
            continue
        progress(f"cpu baseline: oracle on {threads} thread(s)")
        t = time.perf_counter()
        r = ob.place(sb, p, nthreads=threads)
        dt = time.perf_counter() - t
        out[label] = {"pairs_per_s": pairs / dt, "seconds": dt, "threads": threads,
                      "rounds": r["rounds"], "placed_jobs": r["placed"]}
    allc = out["all_cores"]
    return {"value": allc["pairs_per_s"], "unit": "pairs/s", "cores": allc["threads"],
            "kind": "port", "cpu_model": cpu_model(), "os_cpu_count": os.cpu_count(),
            "sample": f"oracle/kp_oracle.c full placement of the same config3 {w.J}x{w.N} "
                      f"snapshot ({allc['rounds']} rounds), OpenMP over the host cores; "
                      f"'single' = 1 thread",
            **out}


def streaming(args, make_placer):
    """BASELINE config #5: a 1M-job trace replayed in micro-batches against a
    50k-node resident table; after each batch a deterministic 20% of the
    running jobs complete (negative kp_apply_delta). Per-batch latency =
    apply the previous completions + load the batch + solve + fetch, host
    wall clock (the latency-bound small-batch path)."""
    cap, topo, req, prio = synth.config5_trace(args.stream_jobs, args.stream_nodes)
    p = _abi.default_params(**synth.CONFIG_PARAMS[5])
    B = args.stream_batch
    lat, parts = [], {"apply": 0.0, "load": 0.0, "solve": 0.0, "fetch": 0.0}
    placed = rounds = 0
    with make_placer() as pl:
        pl.load_nodes(cap, None, topo)
        run_node = np.zeros(0, np.int32)
        run_job = np.zeros(0, np.int64)
        pend_n, pend_d = None, None
        for b in range(args.stream_jobs // B):
            if b % 50 == 0:
                progress(f"streaming batch {b}")
            lo, hi = b * B, (b + 1) * B
            rq = np.ascontiguousarray(req[:, lo:hi])
            t0 = time.perf_counter()
            if pend_n is not None and pend_n.size:
                pl.apply_delta(pend_n, pend_d)
            t1 = time.perf_counter()
            pl.load_jobs(rq, prio[lo:hi])
            t2 = time.perf_counter()
            st = pl.solve(p)
            t3 = time.perf_counter()
            g = pl.fetch(want_used=False)
            t4 = time.perf_counter()
            lat.append(t4 - t0)
            for k, a, z in (("apply", t0, t1), ("load", t1, t2), ("solve", t2, t3), ("fetch", t3, t4)):
                parts[k] += z - a
            rounds += st["rounds"]
            ok = g["node"] >= 0
            placed += int(ok.sum())
            run_node = np.concatenate([run_node, g["node"][ok]])
            run_job = np.concatenate([run_job, lo + np.nonzero(ok)[0]])
            done = synth.config5_completions(b, run_job)
            pend_n = np.ascontiguousarray(run_node[done])
            pend_d = np.ascontiguousarray(-req[:, run_job[done]])
            run_node, run_job = run_node[~done], run_job[~done]
    lat_ms = np.array(lat) * 1e3
    n = len(lat)
    cpu = None if args.no_cpu_baseline else streaming_cpu(args, cap, topo, req, prio, p)
    return {"cpu_baseline": cpu,
            "config": f"#5 streaming: {args.stream_jobs} jobs in {B}-job micro-batches vs "
                      f"{args.stream_nodes} nodes, 20% completions per batch",
            "batches": n, "p50_ms": float(np.percentile(lat_ms, 50)),
            "p99_ms": float(np.percentile(lat_ms, 99)), "max_ms": float(lat_ms.max()),
            "jobs_per_s": args.stream_jobs / float(np.sum(lat)), "placed_jobs": placed,
            "mean_rounds": rounds / max(n, 1),
            "mean_ms": {k: v * 1e3 / max(n, 1) for k, v in parts.items()}}


def streaming_cpu(args, cap, topo, req, prio, p):
    """The oracle beside the config #5 leg (bounded sample): the first
    `--cpu-stream-batches` micro-batches replayed exactly as the GPU leg does
    (per batch: a full placement of the batch against the resident usage,
    then the 20% completions), on every host core and, for batch 0 only, on 1
    thread. Per-batch wall time of the oracle call."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_bind as ob
    B, nb = args.stream_batch, args.cpu_stream_batches
    out = {}
    for label, threads, batches in (("all_cores", host_cores(), nb), ("single", 1, 1)):
        progress(f"cpu baseline (config #5): oracle, {threads} thread(s), {batches} batch(es)")
        used = np.zeros_like(cap)
        run_node, run_job = np.zeros(0, np.int32), np.zeros(0, np.int64)
        per = []
        for b in range(batches):
            lo, hi = b * B, (b + 1) * B
            rq = np.ascontiguousarray(req[:, lo:hi])
            t = time.perf_counter()
            o = ob.place(ob.SnapshotBuf(rq, cap, used, prio[lo:hi], topo=topo), p, nthreads=threads)
            per.append(time.perf_counter() - t)
            used = o["used"].copy()
            ok = o["node"] >= 0
            run_node = np.concatenate([run_node, o["node"][ok]])
            run_job = np.concatenate([run_job, lo + np.nonzero(ok)[0]])
            done = synth.config5_completions(b, run_job)
            np.subtract.at(used.T, run_node[done], req[:, run_job[done]].T)
            run_node, run_job = run_node[~done], run_job[~done]
        out[label] = {"threads": threads, "batches": batches,
                      "batch_ms": [1e3 * x for x in per], "jobs_per_s": B * batches / sum(per)}
    return {"value": out["all_cores"]["jobs_per_s"], "unit": "jobs/s", "cores": host_cores(),
            "kind": "port", "cpu_model": cpu_model(),
            "sample": f"oracle/kp_oracle.c on the first {nb} {B}-job micro-batches of the same "
                      f"trace (batch 0 only on 1 thread); GPU leg: all batches", **out}


def config4_cpu(args, w, p, post=None):
    """The oracle beside the config #4 leg (bounded samples; the full 200k x 20k
    solve + preemption takes the oracle ~25 min on 6 cores), on every host
    core and on 1 thread, as scored job-node pairs per second:
      solve    the first `--cpu-c4-jobs` pending jobs of the same snapshot
               (same nodes, running jobs and usage), the first
               `--cpu-c4-rounds` rounds of their solve;
      preempt  (`post`: the GPU leg's final solve, node usage and status)
               the first `--cpu-c4-preemptors` of the GPU leg's actual
               preemptors (NO_FIT singletons) against the full node pool at
               the GPU solve's post-solve usage, with the same running jobs:
               kpo_preempt (its solve of these rows is one round in which
               every row is NO_FIT) minus kpo_place of the same snapshot =
               the preemption scoring alone."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_bind as ob
    Js = min(args.cpu_c4_jobs, w.J)
    m = w.meta
    sb = ob.SnapshotBuf(np.ascontiguousarray(w.req[:, :Js]), w.cap, w.used, w.prio[:Js],
                        topo=w.topo)
    p = _abi.default_params(**{**synth.CONFIG_PARAMS[4], "max_rounds": args.cpu_c4_rounds})
    out = {}
    for label, threads in (("all_cores", host_cores()), ("single", 1)):
        progress(f"cpu baseline (config #4): oracle on {threads} thread(s), {Js} jobs")
        t = time.perf_counter()
        r = ob.place(sb, p, nthreads=threads)
        dt = time.perf_counter() - t
        out[label] = {"threads": threads, "seconds": dt, "rounds": r["rounds"],
                      "placed_jobs": r["placed"], "pairs_per_s": float(r["pairs"]) / dt}
    pre = None
    if post is not None:
        pj = np.flatnonzero((post["status"] == _abi.KP_JOB_NO_FIT) & (w.gang_size == 1))
        pj = pj[:args.cpu_c4_preemptors]
        sp = ob.SnapshotBuf(np.ascontiguousarray(w.req[:, pj]), w.cap, post["used"], w.prio[pj],
                            topo=w.topo)
        p1 = _abi.default_params(**synth.CONFIG_PARAMS[4])
        pre = {"sample": f"the first {pj.size} of the GPU leg's {post['preemptors']} preemptors "
                         f"(NO_FIT singletons, job order) against all {w.N} nodes at the GPU "
                         f"solve's post-solve usage, {m['run_node'].size} running jobs"}
        for label, threads in (("all_cores", host_cores()), ("single", 1)):
            progress(f"cpu baseline (config #4 preemption): oracle on {threads} thread(s), "
                     f"{pj.size} preemptors")
            t = time.perf_counter()
            r = ob.place(sp, p1, nthreads=threads)
            t_place = time.perf_counter() - t
            t = time.perf_counter()
            r2, pr = ob.preempt(sp, p1, m["run_node"], m["run_req"], m["run_prio"], nthreads=threads)
            t_all = time.perf_counter() - t
            dt = max(t_all - t_place, 1e-9)
            pre[label] = {"threads": threads, "seconds": dt, "preemptors": pr["preemptors"],
                          "nominated": pr["nominated"], "placed_in_sample": r2["placed"],
                          "pairs_per_s": float(pr["pairs"]) / dt}
        pre["value"] = pre["all_cores"]["pairs_per_s"]
    return {"value": out["all_cores"]["pairs_per_s"], "unit": "pairs/s", "cores": host_cores(),
            "kind": "port", "cpu_model": cpu_model(),
            "sample": f"oracle/kp_oracle.c: the first {args.cpu_c4_rounds} rounds of the solve of "
                      f"the first {Js} of the {w.J} pending jobs against the same {w.N}-node "
                      f"snapshot and running jobs; pairs = scored job-node pairs of the solve; "
                      f"preemption: see preempt.sample", **out, "preempt": pre}


def config2(args, make_placer):
    """BASELINE config #2 (10k jobs x 1k nodes x 4 dims, bin-pack score only,
    singletons, empty cluster, 1 GPU): device solve on the resident snapshot
    (kp_reset_nodes + kp_solve, the headline's step), host->host kp_place
    latency, and the oracle beside it on the SAME full snapshot (1 thread and
    every host core; small enough to run whole)."""
    w = synth.config2(args.c2_jobs, args.c2_nodes)
    p = _abi.default_params(**synth.CONFIG_PARAMS[2])
    with make_placer() as pl:
        pl.load_nodes(w.cap, w.used, w.topo)
        pl.load_jobs(w.req, w.prio, w.gang_id, w.gang_size)
        for _ in range(3):  # warmup
            pl.reset_nodes()
            pl.solve(p)
        t = time.perf_counter()
        for _ in range(args.c2_steps):
            pl.reset_nodes()
            st = pl.solve(p)
        s_ms = 1e3 * (time.perf_counter() - t) / args.c2_steps
        lat = []
        for _ in range(args.c2_steps):
            t = time.perf_counter()
            g = pl.place(w, p)
            lat.append(time.perf_counter() - t)
    cpu = None
    if not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(REPO, "tests"))
        import oracle_bind as ob
        sb = ob.SnapshotBuf.from_workload(w)
        cpu = {"unit": "pairs/s", "kind": "port", "cpu_model": cpu_model(), "cores": host_cores(),
               "sample": f"oracle/kp_oracle.c full placement of the same config2 {w.J}x{w.N} "
                         f"snapshot (the whole workload, not a sample)"}
        for label, threads in (("all_cores", host_cores()), ("single", 1)):
            progress(f"cpu baseline (config #2): oracle on {threads} thread(s)")
            t = time.perf_counter()
            o = ob.place(sb, p, nthreads=threads)
            dt = time.perf_counter() - t
            cpu[label] = {"threads": threads, "ms": 1e3 * dt, "pairs_per_s": float(w.J) * w.N / dt,
                          "rounds": o["rounds"], "placed_jobs": o["placed"]}
        cpu["value"] = cpu["all_cores"]["pairs_per_s"]
        cpu["same_placement"] = bool(np.array_equal(o["node"], g["node"]))
    return {"config": f"#2 bin-pack: {w.J} jobs x {w.N} nodes x 4 dims, singletons, empty cluster, "
                      f"w_dim (1,1,1,1), no GPU-fit / spread",
            "solve_ms": s_ms, "pairs_per_s": float(w.J) * w.N / (s_ms / 1e3),
            "pairs_scored_per_s": float(st["pairs"]) / (s_ms / 1e3),
            "latency_ms": 1e3 * float(np.median(lat)),
            "latency_def": f"kp_place host->host, median of {len(lat)}",
            "rounds": st["rounds"], "passes": st["passes"], "placed_jobs": st["placed"],
            "steps": args.c2_steps, "cpu_baseline": cpu}


def phase_split(pl, p, sync=lambda x: x, gather=lambda d: [d]) -> dict:
    """One extra solve (after the timed steps, from the same reset snapshot)
    with the per-round phase events on (kp_set_profiling level 2): candidate
    phase (round start + filter/score/top-K + merge), candidate exchange
    (pack + all-gather + unpack; multi-rank only), passes (bidder index +
    plan/accept + commit), summed over the rounds. Per rank; `value` fields
    are the max over ranks."""
    pl.reset_nodes()
    pl.set_profiling(2)
    st = pl.solve(p)
    shards = pl.timing_shards()  # one per kp_create_multi shard, else this rank's
    pl.set_profiling(False)
    mine = [{"solve_ms": tm["solve_ms"], "cand_ms": tm["cand_ms"], "xchg_ms": tm["xchg_ms"],
             "pass_ms": tm["pass_ms"], "rccl_calls": tm["rccl_calls"], "rounds": st["rounds"]}
            for tm in shards]
    ranks = [r for rk in gather(mine) for r in rk]
    out = {k: max(r[k] for r in ranks) for k in ("solve_ms", "cand_ms", "xchg_ms", "pass_ms")}
    out.update(rounds=st["rounds"], per_rank=ranks, rccl_calls=ranks[0]["rccl_calls"],
               note="device time from HIP events at each round's phase boundaries (their own "
                    "records add a few us per round); max over ranks (or kp_create_multi shards); "
                    "rccl_calls = ncclAllGather calls of the solve (one per round over RCCL)")
    return out


def config4(args, make_placer, n_gpus=1, barrier=lambda: None, max_over_ranks=lambda x: x,
            gather=lambda d: [d]):
    """BASELINE config #4: 200k pending x 20k nodes pre-filled with running
    jobs (priorities 0-3) to 30% GPU occupancy; one step = reset the resident
    usage + solve + preemption nominations for every NO_FIT singleton. On N
    GPUs every rank runs the same calls (the solve and kp_preempt are
    collective: row shards of the candidate phase and of the preemptors, one
    all-gather per round / per preempt call); times are the max over ranks."""
    w = synth.config4(args.c4_jobs, args.c4_nodes)
    p = _abi.default_params(**synth.CONFIG_PARAMS[4])
    m = w.meta
    with make_placer() as pl:
        pl.load_nodes(w.cap, w.used, w.topo)
        pl.load_running(m["run_node"], m["run_req"], m["run_prio"])
        pl.load_jobs(w.req, w.prio, w.gang_id, w.gang_size)
        sol, pre = [], []
        post = None
        for it in range(args.c4_steps + 1):
            progress(f"config #4 step {it}")
            pl.reset_nodes()
            barrier()
            t0 = time.perf_counter()
            st = pl.solve(p)
            t1 = time.perf_counter()
            barrier()
            t1b = time.perf_counter()
            pr = pl.preempt()
            t2 = time.perf_counter()
            if it:  # first iteration: warmup
                sol.append(max_over_ranks(t1 - t0))
                pre.append(max_over_ranks(t2 - t1b))
        if n_gpus == 1 and not args.no_cpu_baseline:  # the CPU preemption sample's rows + usage
            g = pl.fetch()
            post = {"status": g["status"], "used": g["used"], "preemptors": pr["preemptors"]}
        phases = None
        if not args.no_phases:
            progress("config #4 phase split")
            phases = phase_split(pl, p, gather=gather)
            pl.reset_nodes()
            phases["preempt_ms"] = 1e3 * float(np.mean(pre))
    s_ms, p_ms = 1e3 * float(np.mean(sol)), 1e3 * float(np.mean(pre))
    util = w.used.sum(1) / w.cap.sum(1)
    cpu = None if args.no_cpu_baseline or n_gpus > 1 else config4_cpu(args, w, p, post)
    return {"config": f"#4 preemption: {w.J} pending x {w.N} nodes, {m['run_node'].size} running "
                      f"jobs; occupancy per dim (cpu, mem, gpu, gpu_mem) "
                      f"{', '.join(f'{x:.3f}' for x in util)} (every dim >= 0.30)",
            "n_gpus": n_gpus,
            "solve_ms": s_ms, "preempt_ms": p_ms,
            "pairs_per_s": float(w.J) * w.N / ((s_ms + p_ms) / 1e3),
            "pairs_scored_per_s": (float(st["pairs"]) + float(pr["pairs"])) / ((s_ms + p_ms) / 1e3),
            "cpu_baseline": cpu,
            "rounds": st["rounds"], "passes": st["passes"], "placed_jobs": st["placed"],
            "preemptors": pr["preemptors"], "nominated": pr["nominated"],
            "preempt_pairs": pr["pairs"], "preempt_pairs_per_s": float(pr["pairs"]) / (p_ms / 1e3),
            "steps": args.c4_steps, "phases": phases}


def score_matrix(args, make_placer, w, p, rank=0, world=1, gather=lambda d: [d]):
    """The materialised filter + score outputs north_star names (int32 score
    matrix + feasibility bitmask) for the WHOLE config #3 queue, written into
    HBM by kp_score_dev (k_score32c, the capacity-class form): HIP-event kernel
    time and algorithmic bytes (outputs once + requests + node planes) from
    kp_last_timing, against the HBM peak. On N GPUs (one process per GPU) each
    rank scores its contiguous block of rows on its own GPU (a one-GPU
    context: no exchange is needed); aggregate = all ranks' bytes / the
    slowest rank's kernel time."""
    from kplace.devmem import DeviceBuffer  # libkplace's own HIP runtime (not torch's)
    Ns = (w.N + 63) // 64 * 64
    lo, hi = w.J * rank // world, w.J * (rank + 1) // world
    sc = DeviceBuffer((hi - lo) * Ns * 4)
    mk = DeviceBuffer((hi - lo) * (Ns // 64) * 8)
    ms, by, ln, tm = 0.0, 0, 0, None
    with make_placer() as pl:
        pl.load_nodes(w.cap, w.used, w.topo)
        pl.load_jobs(w.req, w.prio, w.gang_id, w.gang_size)
        pl.set_profiling(True)
        for it in range(args.score_steps + 1):
            pl.score_dev(p, lo, hi, sc.ptr, mk.ptr)
            tm = pl.timing()
            if it:  # first call: warmup
                ms += tm["score_ms"]
                by += tm["score_bytes"]
                ln += tm["score_launches"]
    sc.close()
    mk.close()
    ranks = gather({"ms": ms, "bytes": by, "launches": ln, "rows": hi - lo})
    ms = max(r["ms"] for r in ranks)
    by = sum(r["bytes"] for r in ranks)
    ln = ranks[0]["launches"]
    gbs = (by / 1e9) / (ms / 1e3) if ms > 0 else 0.0
    pairs = float(w.J) * w.N * args.score_steps
    kname = "k_score32c" if tm["score_form"] == 1 else "k_score32"
    traffic, traffic_src = None, None
    for pmc in newest("pmc"):  # HBM-side bytes per launch (rocprofv3 PMC), newest first
        path = os.path.join(REPO, "profiles", pmc)
        if os.path.exists(path):
            with open(path) as f:
                k = [v for n, v in json.load(f)["kernels"].items() if n.startswith(kname + "<") or n == kname]
            if k and world == 1:
                traffic = k[0]["traffic_bytes_per_launch"] * (ln / max(args.score_steps, 1))
                traffic_src = f"profiles/{pmc} (FETCH_SIZE x2 + WRITE_SIZE per launch x launches per call)"
                break
    return {"kernel": "k_score32c (capacity-class form)" if tm["score_form"] == 1 else "k_score32",
            "traffic": traffic, "traffic_source": traffic_src,
            "entry": "kp_score_dev", "rows": w.J, "nodes": w.N, "row_stride": Ns, "n_gpus": world,
            "rows_per_rank": [r["rows"] for r in ranks],
            "capacity_classes": tm["score_classes"], "calls": args.score_steps,
            "launches_per_call": ln / max(args.score_steps, 1),
            "bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS * world, "unit": "GB/s",
            "frac": gbs / (HBM_PEAK_GBS * world), "bytes_per_call": by / max(args.score_steps, 1),
            "ms_per_call": ms / max(args.score_steps, 1), "pairs_per_s": pairs / (ms / 1e3) if ms else 0.0,
            "algorithmic_bytes": "rows x Ns x 4 (scores) + rows x Ns / 8 (mask) + rows x (8D + 4) "
                                 "(requests) + (2D + 4) x 4 x Ns (node planes)"}


def relaunch_distributed(args) -> int:
    """`--gpus N` without a launcher: run this script under
    torch.distributed.run as N ranks (a child process; this process never
    touches a GPU) and return its exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           "--master-port", str(args.master_port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--jobs", type=int, default=100_000)
    ap.add_argument("--nodes", type=int, default=10_000)
    ap.add_argument("--single-process", action="store_true",
                    help="drive --gpus N GPUs from this process (kp_create_multi)")
    ap.add_argument("--master-port", type=int, default=29533)
    ap.add_argument("--exchange", choices=("rccl", "host"), default="rccl",
                    help="candidate exchange of a multi-rank run: RCCL (one GPU per rank), or "
                         "host-staged over the gloo group (rehearsal of the multi-rank code on a "
                         "box with fewer GPUs than ranks: rank r uses GPU r mod count; not a "
                         "perf number)")
    ap.add_argument("--gpu-ids", default=None,
                    help="--single-process: comma-separated GPU ids (a repeated id runs the "
                         "in-process exchange; rehearsal only)")
    ap.add_argument("--place-steps", type=int, default=5, help="kp_place (host->host) repetitions")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-single-sample", type=float, default=1.0,
                    help="<1: skip the single-thread oracle run")
    ap.add_argument("--out", default=None, help="also write the JSON line here")
    ap.add_argument("--stream-jobs", type=int, default=1_000_000)
    ap.add_argument("--stream-batch", type=int, default=5_000)
    ap.add_argument("--stream-nodes", type=int, default=50_000)
    ap.add_argument("--no-stream", action="store_true")
    ap.add_argument("--c4-jobs", type=int, default=200_000)
    ap.add_argument("--c4-nodes", type=int, default=20_000)
    ap.add_argument("--c4-steps", type=int, default=3)
    ap.add_argument("--no-config4", action="store_true")
    ap.add_argument("--no-score-matrix", action="store_true")
    ap.add_argument("--score-steps", type=int, default=3, help="kp_score_dev calls of the score-matrix leg")
    ap.add_argument("--cpu-c4-jobs", type=int, default=25_000,
                    help="config #4 CPU baseline sample: the first N pending jobs")
    ap.add_argument("--cpu-c4-rounds", type=int, default=3,
                    help="config #4 CPU baseline sample: rounds of their solve")
    ap.add_argument("--cpu-c4-preemptors", type=int, default=10_000,
                    help="config #4 CPU preemption sample: the first N of the GPU leg's preemptors")
    ap.add_argument("--c2-jobs", type=int, default=10_000)
    ap.add_argument("--c2-nodes", type=int, default=1_000)
    ap.add_argument("--c2-steps", type=int, default=20)
    ap.add_argument("--no-config2", action="store_true")
    ap.add_argument("--cpu-stream-batches", type=int, default=8,
                    help="config #5 CPU baseline sample: the first N micro-batches")
    ap.add_argument("--no-phases", action="store_true",
                    help="skip the extra solve with per-round phase events (profiling runs that count "
                         "kernel launches per solve)")
    ap.add_argument("--no-kernel-events", action="store_true",
                    help="time the steps without per-launch HIP events (no roofline)")
    args = ap.parse_args()

    env_world = os.environ.get("WORLD_SIZE")
    if args.gpus > 1 and env_world is None and not args.single_process:
        sys.exit(relaunch_distributed(args))
    world = int(env_world or "1")
    if not args.single_process and world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} ranks; one rank per GPU")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    from kplace.engine import Placer, unique_id  # noqa: E402  (loads libkplace.so)

    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)

    def fresh_id():
        """A new RCCL unique id for every multi-rank context (an id
        bootstraps one communicator), broadcast from rank 0 over gloo."""
        if world == 1 or args.exchange != "rccl":
            return None
        obj = [unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        return obj[0]

    def gather(d: dict) -> list:
        """Every rank's dict, rank order (rank 0 reports them)."""
        if dist is None:
            return [d]
        out = [None] * world
        dist.all_gather_object(out, d)
        return out

    rehearsal = False
    if args.single_process:
        ids = [int(x) for x in args.gpu_ids.split(",")] if args.gpu_ids else list(range(args.gpus))
        if len(ids) != args.gpus:
            sys.exit(f"bench.py: --gpus {args.gpus} but --gpu-ids names {len(ids)} GPUs")
        rehearsal = len(set(ids)) < len(ids)
        make_placer = lambda: Placer(gpu_ids=ids)  # noqa: E731
        make_local = None  # kp_score_dev needs a one-GPU context
        parallelism = f"job-row shards x{args.gpus} (one process, kp_create_multi)"
        n_gpus = args.gpus
    elif world > 1 and args.exchange == "host":
        import torch

        def allgather(data: bytes) -> bytes:  # host-staged exchange over the gloo group
            t = torch.frombuffer(bytearray(data), dtype=torch.uint8)
            bufs = [torch.empty_like(t) for _ in range(world)]
            dist.all_gather(bufs, t)
            return b"".join(b.numpy().tobytes() for b in bufs)

        dev = local % max(1, torch.cuda.device_count())
        rehearsal = True
        make_placer = lambda: Placer(device=dev, world_size=world, rank=rank,  # noqa: E731
                                     allgather=allgather)
        make_local = lambda: Placer(device=dev)  # noqa: E731
        parallelism = f"job-row shards x{world} (host-staged exchange)"
        n_gpus = world
    else:
        make_placer = lambda: Placer(device=local, world_size=world, rank=rank,  # noqa: E731
                                     nccl_id=fresh_id())
        make_local = lambda: Placer(device=local)  # noqa: E731  (a one-GPU context on this rank's GPU)
        parallelism = f"job-row shards x{world}"
        n_gpus = world

    w = synth.config3(args.jobs, args.nodes)
    p = _abi.default_params(**synth.CONFIG_PARAMS[3])
    pl = make_placer()
    pl.load_nodes(w.cap, w.used, w.topo)
    pl.load_jobs(w.req, w.prio, w.gang_id, w.gang_size)

    def barrier():
        if dist is not None:
            dist.barrier()

    def max_over_ranks(x: float) -> float:
        if dist is None:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    for _ in range(args.warmup):
        pl.reset_nodes()
        pl.solve(p)
    pl.set_profiling(not args.no_kernel_events)
    barrier()
    t0 = time.perf_counter()
    score_ms = score_b = 0.0
    launches = 0
    st = None
    for _ in range(args.steps):
        pl.reset_nodes()
        st = pl.solve(p)  # synchronous: returns after the device finished
        tm = pl.timing()
        score_ms += tm["score_ms"]
        score_b += tm["score_bytes"]
        launches += tm["score_launches"]
    barrier()
    dt = max_over_ranks(time.perf_counter() - t0)
    ms = dt * 1e3 / args.steps
    pl.set_profiling(False)
    # where a solve's time goes (outside the timed steps): candidate phase /
    # exchange / passes, max over ranks
    progress("phase split")
    phases = None if args.no_phases else phase_split(pl, p, gather=gather)

    # full-queue placement latency: snapshot in host memory -> assignment in
    # host memory (kp_place: validate + H2D + solve + D2H), outside the steps
    lat = []
    for _ in range(args.place_steps):
        barrier()
        t = time.perf_counter()
        pl.place(w, p)
        lat.append(max_over_ranks(time.perf_counter() - t))
    pl.close()
    latency_ms = 1e3 * float(np.median(lat)) if lat else None

    # the other legs: every rank runs the collective ones (config #4 solve +
    # kp_preempt on N GPUs); the streaming leg (latency-bound 5k-job batches)
    # and the CPU baselines run at N = 1 only
    legs = {}
    if not args.no_score_matrix and (n_gpus == 1 or make_local is not None):
        progress("score matrix leg")
        legs["score_matrix"] = score_matrix(args, make_local if n_gpus > 1 else make_placer, w, p,
                                            rank=rank, world=world, gather=gather)
    if not args.no_config2 and n_gpus == 1:
        progress("config #2 leg")
        legs["config2"] = config2(args, make_placer)
    if not args.no_config4:
        progress("config #4 leg")
        legs["config4"] = config4(args, make_placer, n_gpus, barrier, max_over_ranks, gather)
    if not args.no_stream and n_gpus == 1:
        progress("config #5 streaming leg")
        legs["streaming"] = streaming(args, make_placer)
    if not args.no_cpu_baseline and n_gpus == 1:
        progress("cpu baseline leg")
        legs["cpu_baseline"] = cpu_baseline(args, w, p)
    if rank != 0:
        dist.barrier()
        return
    pairs = float(args.jobs) * args.nodes
    achieved = (score_b / 1e9) / (score_ms / 1e3) if score_ms > 0 else 0.0
    fused = bool(tm["fused"])
    kname = "k_score_topk" if fused else "k_score32"
    traffic, traffic_src, valu = None, None, None
    for pmc in newest("pmc"):  # HBM-side bytes per launch (rocprofv3 PMC), newest first
        path = os.path.join(REPO, "profiles", pmc)
        if os.path.exists(path):
            with open(path) as f:
                k = [v for n, v in json.load(f)["kernels"].items() if n.startswith(kname)]
            if k:
                traffic = k[0]["traffic_bytes_per_launch"]
                traffic_src = f"profiles/{pmc} (FETCH_SIZE x2 + WRITE_SIZE, tools/gpu_evidence.sh)"
                break
    if fused:
        # SURVEY §8(d) honesty clause: the fused kernel never writes the
        # matrix, so its HBM fraction is on compulsory bytes only; it is
        # judged on pairs/s and on the VALU roofline (lane-ops per pair from
        # the SQ_INSTS_VALU counter of the same solve, profiles/r0N_valu.json)
        opp, vsrc = None, None
        for vj in newest("valu"):  # newest evidence first
            path = os.path.join(REPO, "profiles", vj)
            if os.path.exists(path):
                with open(path) as f:
                    opp = json.load(f)["kernels"].get(kname, {}).get("valu_lane_ops_per_pair")
                if opp:
                    vsrc = vj
                    break
        score_s = score_ms / 1e3 / max(args.steps, 1)  # per solve
        kpairs = st["pairs"] / score_s if score_s > 0 else 0.0
        valu = {"bound": "valu", "kernel": kname, "unit": "Tops/s (int32 lane-ops)",
                "peak": VALU_PEAK_TOPS, "pairs_per_s_kernel": kpairs,
                "lane_ops_per_pair": opp,
                "lane_ops_source": f"profiles/{vsrc} (SQ_INSTS_VALU x 64 / pairs, tools/gpu_evidence.sh)"}
        if opp:
            valu["achieved"] = kpairs * opp / 1e12
            valu["frac"] = valu["achieved"] / VALU_PEAK_TOPS
            valu["achievable"] = VALU_ACHIEVABLE_TOPS
            valu["frac_of_achievable"] = valu["achieved"] / VALU_ACHIEVABLE_TOPS
            valu["achievable_source"] = "tools/valu_peak.hip (profiles/r05_valu_peak.txt)"
    out = {
        "metric": METRIC,
        "value": pairs / (ms / 1e3),
        "unit": "pairs/s",
        "n_gpus": n_gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic (splitmix64 config #3 generator, SURVEY.md §8d)" +
                (" [REHEARSAL: several ranks share one GPU; not a perf number]" if rehearsal else ""),
        "config": {"workload": "config3: 100k jobs x 10k nodes x 4 dims, gangs {1,2,4,8}, "
                               "A/B 8-GPU nodes, bin-pack + spread + GPU-fit",
                   "jobs": args.jobs, "nodes": args.nodes, "dims": 4,
                   "units": st["units"], "rounds": st["rounds"], "passes": st["passes"],
                   "placed_jobs": st["placed"], "pairs_scored": st["pairs"],
                   "parallelism": parallelism},
        "solve_ms": ms,
        "latency_ms": latency_ms,
        "latency_def": "kp_place host->host (validate, H2D, solve, D2H), median of "
                       f"{len(lat)}",
        "pairs_scored_per_s": st["pairs"] / (ms / 1e3),
        "roofline": {"bound": "hbm",
                     "kernel": ("k_score_topk (fused filter+score+top-K, no matrix: compulsory "
                                "bytes only, see valu)") if fused else
                               "k_score32 (filter+score, materialised matrix)",
                     "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_unit": "bytes per launch", "traffic_source": traffic_src,
                     "algorithmic_bytes_per_launch": score_b / max(launches, 1),
                     "frac_of_achievable_6290": achieved / 6290.0,
                     "launches_per_step": launches / args.steps,
                     "avg_launch_ms": score_ms / max(launches, 1),
                     "valu": valu},
        "phases": phases,
    }
    out.update(legs)
    line = json.dumps(out)
    print(line, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")
    if dist is not None:
        dist.barrier()


if __name__ == "__main__":
    main()
