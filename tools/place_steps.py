"""kp_place (host arrays -> host arrays) on config #3: one warm-up call, then
timed calls, for the HIP runtime trace of tools/gpu_evidence.sh (every device
allocation must happen in the warm-up, none inside the timed calls)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "kubernetes-native-distributed-ai-job-scheduler_amd"))
from kplace import _abi, synth  # noqa: E402
from kplace.engine import Placer  # noqa: E402

w = synth.config3()
p = _abi.default_params(**synth.CONFIG_PARAMS[3])
with Placer(device=0) as pl:
    pl.place(w, p)
    for i in range(3):
        t = time.perf_counter()
        pl.place(w, p)
        print(f"place {i}: {1e3 * (time.perf_counter() - t):.2f} ms", flush=True)
