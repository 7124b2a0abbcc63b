"""bench.py's launcher contract (CPU: nothing here touches a GPU)."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_refuses_fewer_ranks_than_gpus():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "one rank per GPU" in r.stderr


def test_bench_parses():
    import ast
    ast.parse(open(os.path.join(REPO, "bench.py")).read())


def test_config4_cpu_baseline_samples(oracle):
    """bench.py's config #4 CPU legs on a small snapshot (the GPU leg's
    post-solve state stood in by the oracle's own): the solve sample and the
    preemption sample, which must score actual preemptors (NO_FIT singletons)."""
    import argparse

    import numpy as np

    sys.path.insert(0, REPO)
    import bench
    from kplace import _abi, synth

    w = synth.config4(4_000, 400)
    p = _abi.default_params(**synth.CONFIG_PARAMS[4])
    m = w.meta
    o, opr = oracle.preempt(oracle.SnapshotBuf.from_workload(w), p, m["run_node"], m["run_req"],
                            m["run_prio"], nthreads=2)
    post = {"status": o["status"], "used": o["used"], "preemptors": opr["preemptors"]}
    args = argparse.Namespace(cpu_c4_jobs=1_000, cpu_c4_rounds=2, cpu_c4_preemptors=300)
    cpu = bench.config4_cpu(args, w, p, post)
    assert cpu["all_cores"]["pairs_per_s"] > 0 and cpu["single"]["rounds"] <= 2
    pre = cpu["preempt"]
    n = min(300, opr["preemptors"])
    assert n > 0
    for k in ("all_cores", "single"):
        assert pre[k]["preemptors"] == n and pre[k]["placed_in_sample"] == 0
        assert pre[k]["pairs_per_s"] > 0
    assert np.isfinite(pre["value"])
