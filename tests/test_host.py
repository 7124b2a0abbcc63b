"""Host side above the C-ABI (CPU): snapshot packer, bind-result writer,
batched Reconcile runner and placement metrics, on BASELINE
config #1 — the reference's own sample CRs (tests/golden/sample_crs.json,
from config/samples/*.yaml) plus synthetic CRs and Node reports. The
placement itself comes from the CPU oracle here (test infrastructure); the
GPU run of the same batch is tests/test_gpu_parity.py::test_config1_runner_gpu.
"""
import copy
import json
import os

import numpy as np
import pytest

from kplace import _abi, binder, metrics, packer, runner, synth

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "sample_crs.json")


def samples():
    return json.load(open(GOLDEN))


def test_sample_crs_pack_like_the_golden_rows():
    for cr in samples():
        rows = packer.job_rows(cr["spec_in"])
        assert rows == cr["expect_rows"], cr["name"]
        d = packer.defaulted_spec(cr["spec_in"])
        for k, v in cr["spec_defaulted"].items():
            assert d[k] == v, (cr["name"], k)


@pytest.mark.parametrize("q,milli", [("500m", 500), ("128", 128000), ("1.5", 1500), ("2k", 2000000)])
def test_cpu_quantities(q, milli):
    assert packer.cpu_milli(q) == milli


@pytest.mark.parametrize("q,mib", [("1Ti", 1048576), ("512Gi", 524288), ("1024Mi", 1024),
                                   ("1073741824", 1024), ("1.5Gi", 1536), ("2G", 1907)])
def test_memory_quantities(q, mib):
    assert packer.mem_mib(q) == mib


@pytest.mark.parametrize("spec", [
    {"replicas": 1},                                        # model required
    {"model": "m", "replicas": 0},                          # Minimum=1
    {"model": "m", "gpuPerReplica": -1},                    # Minimum=0
    {"model": "m", "cacheStrategy": "private"},             # Enum none;shared
    {"model": "m", "gpuMemory": "24G"},                     # Pattern ^\d+(Gi|Mi)$
    {"model": "m", "replicas": 65},                         # gang limit
])
def test_crd_validation(spec):
    with pytest.raises(packer.PackError):
        packer.job_rows(spec)


def test_pack_config1_shapes():
    crs, nodes = synth.config1_objects([c["spec_in"] for c in samples()])
    pk = packer.pack(crs, nodes)
    w = pk.workload
    assert w.N == 64 and len(pk.cr_keys) == 3 + 100
    assert w.J == sum(int(c["spec"].get("replicas", 1)) for c in crs)
    # one CR = one gang of identical replicas, contiguous rows
    for i in range(len(crs)):
        idx = np.nonzero(pk.job_cr == i)[0]
        assert (np.diff(idx) == 1).all() and (w.gang_size[idx] == idx.size).all()
        assert (w.req[:, idx] == w.req[:, idx[:1]]).all()
    assert w.topo.max() == 1  # two xGMI islands of 32 nodes
    assert (w.cap[2] % 4 == 0).all() and (w.cap[3] == w.cap[2] * 294912 // 8).sum() > 0


class OraclePlacer:
    """Test double with the Placer.place signature, backed by the CPU oracle."""

    def __init__(self, oracle):
        self.ob = oracle

    def place(self, w, p):
        return self.ob.place(self.ob.SnapshotBuf.from_workload(w), p, nthreads=4)


def run_config1(placer, reg=None):
    crs, nodes = synth.config1_objects([c["spec_in"] for c in samples()])
    cache = copy.deepcopy(crs)
    written = {}
    m = metrics.PlacementMetrics(reg)
    r = runner.BatchRunner(placer, lambda: crs, lambda: nodes,
                           lambda key, st: written.__setitem__(key, st),
                           _abi.default_params(**synth.CONFIG_PARAMS[1]), metrics=m)
    res, err = r.reconcile(("default", "llm-0"))
    assert err is None and not res.requeue
    summary = r.run_batch()
    assert crs == cache, "cached objects must not be mutated"
    return crs, nodes, written, summary, m


def test_config1_batch_runner_with_oracle(oracle):
    crs, nodes, written, summary, m = run_config1(OraclePlacer(oracle))
    assert len(written) == len(crs)
    placed = 0
    for cr in crs:
        key = ("default", cr["metadata"]["name"])
        conds = written[key]["conditions"]
        assert [c["type"] for c in conds] == ["Placed"]
        c = conds[0]
        if c["status"] == "True":
            placed += 1
            reps = int(cr["spec"].get("replicas", 1))
            assert c["message"].count("->") == reps
        else:
            assert c["reason"] in ("NoFit", "RoundLimit")
    assert placed >= 40 and summary["placed"] > 0  # the cluster is ~2x oversubscribed in GPUs
    assert m.assigned.labels("placed")._value.get() == summary["placed"]
    # deterministic: the same snapshot gives the same statuses (fail-over safety)
    _, _, written2, _, _ = run_config1(OraclePlacer(oracle))
    strip = lambda d: {k: [{kk: vv for kk, vv in c.items() if kk != "lastUpdateTime"}
                           for c in v["conditions"]] for k, v in d.items()}
    assert strip(written) == strip(written2)


def test_status_writer_replaces_only_its_condition():
    cr = {"metadata": {"name": "x"}, "status": {"availableReplicas": 2, "conditions": [
        {"type": "Ready", "status": "True"}, {"type": "Placed", "status": "False"}]}}
    before = copy.deepcopy(cr)
    st = binder.status_with_condition(cr, {"type": "Placed", "status": "True"})
    assert cr == before
    assert st["availableReplicas"] == 2
    assert [c["type"] for c in st["conditions"]] == ["Ready", "Placed"]
    assert st["conditions"][1]["status"] == "True"


# ---------------------------------------------------------------------------
# invalid objects, failing batches, CacheStrategy shared, scale
# ---------------------------------------------------------------------------
def _nodes(n=4):
    return [{"metadata": {"name": f"n{i}", "labels": {"kubeinfer.ai/gpu-memory": "288Gi",
                                                      "kubeinfer.ai/xgmi-island": f"isl-{i // 2}"}},
             "status": {"allocatable": {"cpu": "128", "memory": "1Ti", "amd.com/gpu": "8"}}}
            for i in range(n)]


def test_bad_cr_and_bad_node_do_not_abort_the_batch(oracle):
    crs = [{"metadata": {"name": "good-a"}, "spec": {"model": "m", "replicas": 2, "gpuPerReplica": 1}},
           {"metadata": {"name": "too-big"}, "spec": {"model": "m", "replicas": 65}},
           {"metadata": {"name": "bad-mem"}, "spec": {"model": "m", "gpuMemory": "24G"}},
           {"metadata": {"name": "good-b"}, "spec": {"model": "m", "gpuPerReplica": 2}}]
    nodes = _nodes() + [{"metadata": {"name": "broken"},
                         "status": {"allocatable": {"cpu": "lots"}}}]
    written = {}
    r = runner.BatchRunner(OraclePlacer(oracle), lambda: crs, lambda: nodes,
                           lambda k, st: written.__setitem__(k, st), _abi.default_params())
    s = r.run_batch()
    assert s["invalid_crs"] == 2 and s["bad_nodes"] == 1 and s["nodes"] == 5
    cond = {k[1]: v["conditions"][0] for k, v in written.items()}
    assert cond["good-a"]["status"] == "True" and cond["good-b"]["status"] == "True"
    assert cond["too-big"]["reason"] == "Invalid" and "gang limit" in cond["too-big"]["message"]
    assert cond["bad-mem"]["reason"] == "Invalid"
    assert "broken" not in cond["good-a"]["message"]


def test_serve_survives_a_failing_batch(oracle):
    import threading

    class Flaky(OraclePlacer):
        calls = 0

        def place(self, w, p):
            Flaky.calls += 1
            if Flaky.calls == 1:
                raise RuntimeError("transient engine failure")
            return super().place(w, p)

    crs = [{"metadata": {"name": "a"}, "spec": {"model": "m"}}]
    written = {}
    r = runner.BatchRunner(Flaky(oracle), lambda: crs, lambda: _nodes(),
                           lambda k, st: written.__setitem__(k, st), _abi.default_params(),
                           debounce_s=0.0, retry_s=0.01)
    stop = threading.Event()
    t = threading.Thread(target=r.serve, args=(stop, 0.01))
    t.start()
    r.reconcile(("default", "a"))
    for _ in range(500):
        if written:
            break
        stop.wait(0.01)
    stop.set()
    t.join(5)
    assert Flaky.calls >= 2 and written[("default", "a")]["conditions"][0]["status"] == "True"


def test_cache_shared_affinity_packing():
    cache = [c for c in samples() if c["spec_in"].get("cacheStrategy") == "shared"][0]
    crs = [{"metadata": {"name": "test-cache-llm", "namespace": "default"},
            "spec": cache["spec_in"], "status": {"cacheCoordinator": "test-cache-llm-0"}},
           {"metadata": {"name": "same-model", "namespace": "default"},
            "spec": dict(cache["spec_in"], replicas=1)},                   # no coordinator yet
           {"metadata": {"name": "plain", "namespace": "default"},
            "spec": {"model": cache["spec_in"]["model"]}}]                 # cacheStrategy none
    pk = packer.pack(crs, _nodes(), pod_nodes={("default", "test-cache-llm-0"): "n3"})
    w = pk.workload
    dom = int(w.topo[pk.node_names.index("n3")])
    assert w.affinity.tolist() == [dom] * 3 + [dom] + [-1]
    # without the pod map the coordinator's domain is unknown
    assert (packer.pack(crs, _nodes()).workload.affinity == -1).all()


def test_cache_shared_sample_places_in_coordinator_domain(oracle):
    cache = [c for c in samples() if c["spec_in"].get("cacheStrategy") == "shared"][0]
    crs = [{"metadata": {"name": "test-cache-llm", "namespace": "default"},
            "spec": cache["spec_in"], "status": {"cacheCoordinator": "coord"}}]
    pk = packer.pack(crs, _nodes(8), pod_nodes={("default", "coord"): "n5"})
    res = OraclePlacer(oracle).place(pk.workload, _abi.default_params(**synth.CONFIG_PARAMS[1]))
    doms = {int(pk.workload.topo[n]) for n in res["node"]}
    assert doms == {int(pk.workload.topo[5])}


def _naive_conditions(packed, result):
    out = {}
    for i, key in enumerate(packed.cr_keys):
        jobs = [j for j in range(len(packed.job_cr)) if packed.job_cr[j] == i]
        out[key] = bool(jobs) and all(result["node"][j] >= 0 for j in jobs)
    return out


def test_binder_grouping_matches_naive_and_scales():
    import time
    w = synth.config3(3_000, 200)
    crs, nodes, pods = synth.workload_objects(w, shared_every=7)
    pk = packer.pack(crs, nodes, pod_nodes=pods)
    rng = np.random.default_rng(0)
    res = {"node": np.where(rng.random(pk.workload.J) < 0.7,
                            rng.integers(0, pk.workload.N, pk.workload.J), -1).astype(np.int32),
           "status": np.zeros(pk.workload.J, np.int32)}
    got = binder.conditions(pk, res, now="t")
    naive = _naive_conditions(pk, res)
    assert {k: v["status"] == "True" for k, v in got.items()} == naive
    # config #3 scale: 26k CRs / 100k jobs in well under a second of grouping
    w = synth.config3()
    crs, nodes, _ = synth.workload_objects(w)
    t = time.perf_counter()
    pk = packer.pack(crs, nodes)
    res = {"node": np.zeros(pk.workload.J, np.int32), "status": np.zeros(pk.workload.J, np.int32)}
    conds = binder.conditions(pk, res, now="t")
    assert len(conds) == len(crs) == 26_525
    assert time.perf_counter() - t < 30
