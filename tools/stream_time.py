"""Config #5 streaming timing for A/B runs (KPLACE_LIB selects the library
build): the first BATCHES (default 60) micro-batches of the bench's replay
(apply completions, load, solve, fetch), p50 / p99 per-batch latency."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "kubernetes-native-distributed-ai-job-scheduler_amd"))
from kplace import _abi, synth  # noqa: E402
from kplace.engine import Placer  # noqa: E402

nb = int(os.environ.get("BATCHES", "60"))
B, total, N = 5_000, 1_000_000, 50_000
cap, topo, req, prio = synth.config5_trace(total, N)
p = _abi.default_params(**synth.CONFIG_PARAMS[5])
lat, sol = [], []
with Placer(device=0) as pl:
    pl.load_nodes(cap, None, topo)
    run_node, run_job = np.zeros(0, np.int32), np.zeros(0, np.int64)
    pend_n = pend_d = None
    for b in range(nb):
        lo, hi = b * B, (b + 1) * B
        rq = np.ascontiguousarray(req[:, lo:hi])
        t0 = time.perf_counter()
        if pend_n is not None and pend_n.size:
            pl.apply_delta(pend_n, pend_d)
        pl.load_jobs(rq, prio[lo:hi])
        t1 = time.perf_counter()
        st = pl.solve(p)
        t2 = time.perf_counter()
        g = pl.fetch(want_used=False)
        lat.append(time.perf_counter() - t0)
        sol.append(t2 - t1)
        ok = g["node"] >= 0
        run_node = np.concatenate([run_node, g["node"][ok]])
        run_job = np.concatenate([run_job, lo + np.nonzero(ok)[0]])
        done = synth.config5_completions(b, run_job)
        pend_n = np.ascontiguousarray(run_node[done])
        pend_d = np.ascontiguousarray(-req[:, run_job[done]])
        run_node, run_job = run_node[~done], run_job[~done]
lat_ms, sol_ms = 1e3 * np.array(lat[1:]), 1e3 * np.array(sol[1:])
print(f"{os.path.basename(os.environ.get('KPLACE_LIB', 'libkplace.so'))} stream {nb} batches: p50 "
      f"{np.percentile(lat_ms, 50):.2f} p99 {np.percentile(lat_ms, 99):.2f} ms, solve p50 "
      f"{np.percentile(sol_ms, 50):.2f} ms", flush=True)
