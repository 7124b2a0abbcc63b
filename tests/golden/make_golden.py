#!/usr/bin/env python3
"""Regenerates the committed golden fixtures.

1. place_*.npz — seeded snapshots + the oracle's outputs (regression vectors
   for the oracle and the GPU path; they pin both to the spec as it stands,
   not to the reference, which has no placement code).
2. sample_crs.json — the reference's own sample LLMService CRs
   (config/samples/*.yaml in Moore-Z/Kubernetes-Native-Distributed-AI-Job-Scheduler)
   reduced to their spec fields, with the CRD defaults applied
   (api/v1/llmservice_types.go:29-51) and the packed job rows the snapshot
   packer must produce. Generated only where /root/reference exists; the
   committed JSON is data (inputs + expected outputs), not reference source.

Run from the repo root: python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "kubernetes-native-distributed-ai-job-scheduler_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

import oracle_bind as ob  # noqa: E402
from kplace import _abi, synth  # noqa: E402
from test_gpu_parity import random_workload  # noqa: E402


def save(name, w, p):
    r = ob.place(ob.SnapshotBuf.from_workload(w), p, nthreads=4)
    assert not isinstance(r, int), r
    pd = _abi.params_dict(p)
    arrs = dict(req=w.req, cap=w.cap, used=w.used, prio=w.prio, gang_id=w.gang_id,
                gang_size=w.gang_size, topo=w.topo,
                **({} if w.affinity is None else {"affinity": w.affinity}),
                out_node=r["node"], out_score=r["score"], out_status=r["status"],
                out_used=r["used"], out_rounds=np.int64(r["rounds"]),
                out_passes=np.int64(r["passes"]))
    for k, v in pd.items():
        arrs["p_" + k] = np.array(v, dtype=np.int64)
    np.savez_compressed(os.path.join(HERE, f"place_{name}.npz"), **arrs)
    print(name, "rounds", r["rounds"], "passes", r["passes"], "placed", r["placed"])


def sample_crs():
    import yaml
    src = "/root/reference/config/samples"
    if not os.path.isdir(src):
        print("reference not present: sample_crs.json left as committed")
        return
    crs = []
    for fn in sorted(os.listdir(src)):
        if not fn.endswith(".yaml") or fn == "kustomization.yaml":
            continue
        with open(os.path.join(src, fn)) as f:
            for doc in yaml.safe_load_all(f):
                if not doc or doc.get("kind") != "LLMService":
                    continue
                spec = doc.get("spec", {})
                crs.append({"file": fn, "name": doc["metadata"]["name"], "spec": spec})
    # CRD defaults (api/v1/llmservice_types.go:29-51, CRD yaml:39-71)
    out = []
    for cr in crs:
        s = dict(cr["spec"])
        s.setdefault("replicas", 1)
        s.setdefault("gpuPerReplica", 0)
        s.setdefault("cacheStrategy", "none")
        s.setdefault("image", "vllm/vllm-openai:latest")
        gm = s.get("gpuMemory", "")
        mib = 0 if gm == "" else int(gm[:-2]) * (1024 if gm.endswith("Gi") else 1)
        out.append({"name": cr["name"], "file": cr["file"], "spec_in": cr["spec"],
                    "spec_defaulted": s,
                    # one job row per replica (desiredDeployment: Replicas identical
                    # pods, llmservice_controller.go:183,203); the CR has no cpu/mem
                    # fields and the pod template sets no resources (:217-289)
                    "expect_rows": [{"cpu_milli": 0, "mem_MiB": 0, "gpu": s["gpuPerReplica"],
                                     "gpu_mem_MiB": mib}
                                    for _ in range(s["replicas"])]})
    with open(os.path.join(HERE, "sample_crs.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("sample_crs.json:", len(out), "CRs")


def main():
    ob.build()
    save("rand0", random_workload(1000, J=600, N=80), _abi.default_params())
    save("rand1_least_idx", random_workload(1001, J=500, N=120),
         _abi.default_params(score_mode=1, tie_mode=0, n_cand=4, max_passes=3))
    save("rand2_k1", random_workload(1002, J=400, N=64, gangs=False),
         _abi.default_params(n_cand=1, max_passes=1, util_scale=1024))
    save("config2_small", synth.config2(2000, 200), _abi.default_params(**synth.CONFIG_PARAMS[2]))
    save("config3_small", synth.config3(2000, 160), _abi.default_params(**synth.CONFIG_PARAMS[3]))
    w = random_workload(1003, J=500, N=96)
    rng = np.random.default_rng(1003)
    gid = w.gang_id
    aff = rng.integers(-1, 96 // 5, size=w.J).astype(np.int32)
    for g in np.unique(gid[gid >= 0]):  # one domain per gang
        aff[gid == g] = aff[gid == g][0]
    w.affinity = aff
    save("rand3_affinity", w, _abi.default_params(w_affinity=300))
    save("rand4_least_scale", random_workload(1004, J=400, N=77),
         _abi.default_params(score_mode=1, util_scale=1023))
    sample_crs()


if __name__ == "__main__":
    main()
