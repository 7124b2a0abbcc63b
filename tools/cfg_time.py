"""Config #3 solve timing with parameter overrides, for A/B runs of library
builds (KPLACE_LIB) on non-default parameters:
    python tools/cfg_time.py tie_mode=0 n_cand=32"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "kubernetes-native-distributed-ai-job-scheduler_amd"))
from kplace import _abi, synth  # noqa: E402
from kplace.engine import Placer  # noqa: E402

over = {k: int(v) for k, v in (a.split("=") for a in sys.argv[1:])}
w = synth.config3()
p = _abi.default_params(**{**synth.CONFIG_PARAMS[3], **over})
with Placer(device=0) as pl:
    pl.load_nodes(w.cap, w.used, w.topo)
    pl.load_jobs(w.req, w.prio, w.gang_id, w.gang_size)
    ts = []
    for it in range(int(os.environ.get("SOLVES", "6"))):
        pl.reset_nodes()
        t = time.perf_counter()
        st = pl.solve(p)
        ts.append(time.perf_counter() - t)
    print(f"{os.path.basename(os.environ.get('KPLACE_LIB', 'libkplace.so'))} {over} solve ms "
          f"{1e3 * np.median(ts[1:]):.2f} rounds {st['rounds']} passes {st['passes']} "
          f"placed {st['placed']} fused {pl.timing()['fused']}", flush=True)
