"""Host->host placement latency split on config #3: kp_place as one call vs
the staged calls (load_nodes / load_jobs / solve / fetch), medians of 5."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "kubernetes-native-distributed-ai-job-scheduler_amd"))
import numpy as np  # noqa: E402

from kplace import _abi, synth  # noqa: E402
from kplace.engine import Placer  # noqa: E402

w = synth.config3()
p = _abi.default_params(**synth.CONFIG_PARAMS[3])
T = {k: [] for k in ("place", "load_nodes", "load_jobs", "solve", "fetch")}
with Placer(device=0) as pl:
    pl.place(w, p)
    for _ in range(6):
        t = time.perf_counter()
        pl.place(w, p)
        T["place"].append(time.perf_counter() - t)
        t0 = time.perf_counter()
        pl.load_nodes(w.cap, w.used, w.topo)
        t1 = time.perf_counter()
        pl.load_jobs(w.req, w.prio, w.gang_id, w.gang_size)
        t2 = time.perf_counter()
        pl.solve(p)
        t3 = time.perf_counter()
        pl.fetch()
        t4 = time.perf_counter()
        for k, a, b in (("load_nodes", t0, t1), ("load_jobs", t1, t2), ("solve", t2, t3), ("fetch", t3, t4)):
            T[k].append(b - a)
for k, v in T.items():
    print(f"{k:10s} median {1e3 * np.median(v[1:]):7.3f} ms")
