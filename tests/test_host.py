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
    assert placed > 50 and summary["placed"] > 0
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
