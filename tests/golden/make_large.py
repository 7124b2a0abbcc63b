#!/usr/bin/env python3
"""Golden digests for the BASELINE configs at their stated sizes, from the CPU
oracle (test infrastructure), so that the GPU box only runs the GPU side:

  config4   200k pending x 20k nodes, 30% GPU occupancy of running jobs:
            placement + preemption nominations (kpo_preempt);
  config5   the first 3 micro-batches (5k jobs each) of the 1M-job trace
            against the 50k-node table, with the 20% completions between them;
  config3_score  the materialised filter + score outputs (kpo_score) of the
            whole config #3 queue, 100k x 10k: the int32 score matrix (N
            columns per row) and the feasibility bitmask (ceil(N/64) words per
            row), row after row, as two SHA-256 digests.

Each entry holds SHA-256 digests of the int arrays (little-endian bytes) plus
the scalar counters; the inputs' digests pin the generator. Run from the repo
root: python tests/golden/make_large.py [entry ...]  (minutes on 8 cores; named
entries are recomputed, the others kept).
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "kubernetes-native-distributed-ai-job-scheduler_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

import oracle_bind as ob  # noqa: E402
from kplace import _abi, synth  # noqa: E402


def digest(a) -> str:
    a = np.ascontiguousarray(a)
    return hashlib.sha256(a.astype(a.dtype.newbyteorder("<")).tobytes()).hexdigest()


def config4_entry(threads):
    w = synth.config4()
    p = _abi.default_params(**synth.CONFIG_PARAMS[4])
    m = w.meta
    t = time.time()
    r, pr = ob.preempt(ob.SnapshotBuf.from_workload(w), p, m["run_node"], m["run_req"],
                       m["run_prio"], nthreads=threads)
    print(f"config4 oracle {time.time() - t:.1f}s rounds {r['rounds']} placed {r['placed']} "
          f"preemptors {pr['preemptors']} nominated {pr['nominated']}", flush=True)
    return {
        "inputs": {k: digest(v) for k, v in dict(req=w.req, cap=w.cap, used=w.used, prio=w.prio,
                                                  run_node=m["run_node"], run_req=m["run_req"],
                                                  run_prio=m["run_prio"]).items()},
        "place": {k: digest(r[k]) for k in ("node", "score", "status", "used")},
        "preempt": {k: digest(pr[k]) for k in ("node", "victims", "cost")},
        "counts": {k: int(r[k]) for k in ("rounds", "passes", "placed", "unplaced", "units", "pairs")},
        "preempt_counts": {k: int(pr[k]) for k in ("preemptors", "nominated", "pairs")},
    }


def config5_entry(threads, batches=3, total=1_000_000, N=50_000, B=5_000):
    cap, topo, req, prio = synth.config5_trace(total, N)
    p = _abi.default_params(**synth.CONFIG_PARAMS[5])
    used = np.zeros_like(cap)
    run_node = np.zeros(0, np.int32)
    run_job = np.zeros(0, np.int64)
    out = {"inputs": {"cap": digest(cap), "req": digest(req), "prio": digest(prio)}, "batches": []}
    for b in range(batches):
        lo, hi = b * B, (b + 1) * B
        rq = np.ascontiguousarray(req[:, lo:hi])
        t = time.time()
        o = ob.place(ob.SnapshotBuf(rq, cap, used, prio[lo:hi], topo=topo), p, threads)
        print(f"config5 batch {b} oracle {time.time() - t:.1f}s rounds {o['rounds']} "
              f"placed {o['placed']}", flush=True)
        out["batches"].append({
            **{k: digest(o[k]) for k in ("node", "score", "status", "used")},
            "counts": {k: int(o[k]) for k in ("rounds", "passes", "placed", "pairs")}})
        used = o["used"].copy()
        ok = o["node"] >= 0
        run_node = np.concatenate([run_node, o["node"][ok]])
        run_job = np.concatenate([run_job, lo + np.nonzero(ok)[0]])
        done = synth.config5_completions(b, run_job)
        np.subtract.at(used.T, run_node[done], req[:, run_job[done]].T)
        run_node, run_job = run_node[~done], run_job[~done]
    return out


def config3_score_entry(threads, chunk=4_000):
    w = synth.config3()
    p = _abi.default_params(**synth.CONFIG_PARAMS[3])
    sb = ob.SnapshotBuf.from_workload(w)
    hs, hm = hashlib.sha256(), hashlib.sha256()
    feasible = 0
    t = time.time()
    for lo in range(0, w.J, chunk):
        sc, mk = ob.score(sb, p, lo, min(w.J, lo + chunk))
        hs.update(sc.astype("<i4").tobytes())
        hm.update(mk.astype("<u8").tobytes())
        feasible += int((sc >= 0).sum())
    print(f"config3_score oracle {time.time() - t:.1f}s, {feasible} feasible pairs", flush=True)
    return {"inputs": {"req": digest(w.req), "cap": digest(w.cap), "used": digest(w.used)},
            "rows": w.J, "nodes": w.N, "score": hs.hexdigest(), "mask": hm.hexdigest(),
            "feasible_pairs": feasible}


ENTRIES = {"config5": config5_entry, "config4": config4_entry, "config3_score": config3_score_entry}


def main():
    threads = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
    ob.build()
    path = os.path.join(HERE, "large_digests.json")
    res = json.load(open(path)) if os.path.exists(path) else {}
    res["generator"] = "tests/golden/make_large.py"
    for name in sys.argv[1:] or list(ENTRIES):
        res[name] = ENTRIES[name](threads)
    with open(path, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print("wrote large_digests.json")


if __name__ == "__main__":
    main()
