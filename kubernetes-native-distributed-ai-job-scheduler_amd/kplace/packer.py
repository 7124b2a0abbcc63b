"""Snapshot packer: LLMService CRs + Node reports -> the C-ABI SoA of
include/kplace.h (what `pkg/placement/pack.go` does in the
Go host).

Job side (api/v1/llmservice_types.go:25-52, CRD
config/crd/bases/ai.ruijie.io_llmservices.yaml:39-71): CRD defaults are
applied (replicas 1, gpuPerReplica 0, cacheStrategy none, image
vllm/vllm-openai:latest) and validated (model required, replicas >= 1,
gpuPerReplica >= 0, cacheStrategy in {none, shared}, gpuMemory matching
^\\d+(Gi|Mi)$ — parsed by the library's kp_parse_gpu_memory). One CR becomes
Spec.Replicas identical job rows (desiredDeployment builds Replicas identical
pods, internal/controller/llmservice_controller.go:183,203) forming one
all-or-nothing gang; cpu/mem requests are 0 because the CR has no such fields
and the pod template sets no resources (:217-289). The CRD has no priority
field: priority defaults to 0 and may be set by the host through the
annotation `kubeinfer.ai/priority` (an extension of this build).

Node side: corev1.Node objects (the synthetic "agent node reports" of config
#1): status.allocatable cpu / memory / amd.com/gpu (Kubernetes quantities),
the per-GPU memory from the label `kubeinfer.ai/gpu-memory` (e.g. "288Gi"),
the topology domain (xGMI island / rack) from `kubeinfer.ai/xgmi-island`
(falling back to topology.kubernetes.io/rack, then to the node itself), and
the current usage from an optional `used` mapping (node name -> per-dim
amounts) that the host sums from bound pods.
"""
from __future__ import annotations

import ctypes as C
import re
from dataclasses import dataclass, field

import numpy as np

from . import engine, synth

DIMS = ("cpu_milli", "mem_MiB", "gpu", "gpu_mem_MiB")
GPU_RESOURCE = "amd.com/gpu"
LABEL_GPU_MEMORY = "kubeinfer.ai/gpu-memory"
LABEL_ISLAND = "kubeinfer.ai/xgmi-island"
LABEL_RACK = "topology.kubernetes.io/rack"
ANNOT_PRIORITY = "kubeinfer.ai/priority"

CRD_DEFAULTS = {"replicas": 1, "gpuPerReplica": 0, "cacheStrategy": "none",
                "image": "vllm/vllm-openai:latest"}


class PackError(ValueError):
    """A CR or Node that the CRD / quantity rules reject (the apiserver would
    have rejected the CR; the packer refuses it instead of guessing)."""


def parse_gpu_memory(s: str) -> int:
    """LLMServiceSpec.GPUMemory -> MiB through the library (kp_parse_gpu_memory,
    CRD pattern ^\\d+(Gi|Mi)$). "" -> 0."""
    v = C.c_int64(0)
    if engine.lib().kp_parse_gpu_memory(s.encode(), C.byref(v)) != 0:
        raise PackError(f"gpuMemory {s!r} does not match ^\\d+(Gi|Mi)$")
    return v.value


_QTY = re.compile(r"^([0-9]+)(\.[0-9]+)?(m|k|M|G|T|P|E|Ki|Mi|Gi|Ti|Pi|Ei)?$")
_BIN = {"Ki": 2 ** 10, "Mi": 2 ** 20, "Gi": 2 ** 30, "Ti": 2 ** 40, "Pi": 2 ** 50, "Ei": 2 ** 60}
_DEC = {"k": 10 ** 3, "M": 10 ** 6, "G": 10 ** 9, "T": 10 ** 12, "P": 10 ** 15, "E": 10 ** 18}


def _quantity_scaled(s: str, unit_num: int, unit_den: int) -> int:
    """Kubernetes quantity -> floor(value * unit_num / unit_den), exact
    (integer arithmetic; decimal fractions allowed)."""
    m = _QTY.match(str(s).strip())
    if not m:
        raise PackError(f"bad quantity {s!r}")
    whole, frac, suf = m.group(1), m.group(2) or "", m.group(3) or ""
    num = int(whole + frac[1:]) if frac else int(whole)
    den = 10 ** (len(frac) - 1) if frac else 1
    if suf == "m":
        den *= 1000
    elif suf in _BIN:
        num *= _BIN[suf]
    elif suf in _DEC:
        num *= _DEC[suf]
    return (num * unit_num) // (den * unit_den)


def cpu_milli(q) -> int:
    return _quantity_scaled(q, 1000, 1)


def mem_mib(q) -> int:
    return _quantity_scaled(q, 1, 2 ** 20)


def defaulted_spec(spec: dict) -> dict:
    """CRD defaulting + validation of one LLMServiceSpec (returns a copy)."""
    s = dict(CRD_DEFAULTS)
    s.update({k: v for k, v in spec.items() if v is not None})
    if not s.get("model"):
        raise PackError("spec.model is required")
    if int(s["replicas"]) < 1:
        raise PackError("spec.replicas must be >= 1")
    if int(s["replicas"]) > 64:  # KP_MAX_GANG: one CR is one all-or-nothing gang
        raise PackError("spec.replicas above the gang limit (64)")
    if int(s["gpuPerReplica"]) < 0:
        raise PackError("spec.gpuPerReplica must be >= 0")
    if s["cacheStrategy"] not in ("none", "shared"):
        raise PackError("spec.cacheStrategy must be none or shared")
    s["gpuMemoryMiB"] = parse_gpu_memory(s.get("gpuMemory", "") or "")
    return s


def job_rows(spec: dict) -> list[dict]:
    """The job rows of one (defaulted) CR: Replicas identical replicas."""
    s = defaulted_spec(spec)
    row = {"cpu_milli": 0, "mem_MiB": 0, "gpu": int(s["gpuPerReplica"]),
           "gpu_mem_MiB": int(s["gpuMemoryMiB"])}
    return [dict(row) for _ in range(int(s["replicas"]))]


@dataclass
class Packed:
    """A packed snapshot plus the maps back to the API objects."""
    workload: synth.Workload
    cr_keys: list                 # [(namespace, name)] per CR, CR index order
    job_cr: np.ndarray            # [J] CR index of each job row
    job_replica: np.ndarray       # [J] replica ordinal within its CR
    node_names: list              # [N]
    domains: list = field(default_factory=list)  # topology domain names, index order


def _meta(o):
    return o.get("metadata", {}) or {}


def pack(crs: list[dict], nodes: list[dict], used: dict | None = None) -> Packed:
    """CRs (LLMService objects as dicts, in the order the batch runner lists
    them) and Node objects -> one kp_snapshot-shaped Workload."""
    rows, job_cr, job_rep, prio, keys = [], [], [], [], []
    for i, cr in enumerate(crs):
        md = _meta(cr)
        keys.append((md.get("namespace", "default"), md["name"]))
        p = int((md.get("annotations") or {}).get(ANNOT_PRIORITY, 0))
        rs = job_rows(cr.get("spec", {}))
        for r_i, r in enumerate(rs):
            rows.append([r[d] for d in DIMS])
            job_cr.append(i)
            job_rep.append(r_i)
            prio.append(p)
    J, N, D = len(rows), len(nodes), len(DIMS)
    req = np.ascontiguousarray(np.array(rows, np.int64).reshape(J, D).T)
    job_cr = np.array(job_cr, np.int32)
    gsz = np.bincount(job_cr, minlength=len(crs)).astype(np.int32)[job_cr] if J else \
        np.zeros(0, np.int32)
    cap = np.zeros((D, N), np.int64)
    usedv = np.zeros((D, N), np.int64)
    names, dom_of = [], []
    for n, node in enumerate(nodes):
        md = _meta(node)
        names.append(md["name"])
        alloc = (node.get("status", {}) or {}).get("allocatable", {}) or {}
        labels = md.get("labels", {}) or {}
        gpus = int(alloc.get(GPU_RESOURCE, 0))
        per_gpu = parse_gpu_memory(labels.get(LABEL_GPU_MEMORY, "") or "") if gpus else 0
        cap[:, n] = [cpu_milli(alloc.get("cpu", 0)), mem_mib(alloc.get("memory", 0)), gpus,
                     gpus * per_gpu]
        dom_of.append(labels.get(LABEL_ISLAND) or labels.get(LABEL_RACK) or "node/" + md["name"])
        if used and md["name"] in used:
            usedv[:, n] = [int(used[md["name"]].get(d, 0)) for d in DIMS]
    if (usedv > cap).any() or (usedv < 0).any():
        raise PackError("node usage outside [0, allocatable]")
    domains = sorted(set(dom_of))
    index = {d: i for i, d in enumerate(domains)}
    topo = np.array([index[d] for d in dom_of], np.int32)
    w = synth.Workload(J, N, D, req, cap, usedv, np.array(prio, np.int32), job_cr.copy(), gsz,
                       topo, name="packed")
    return Packed(w, keys, job_cr, np.array(job_rep, np.int32), names, domains)
