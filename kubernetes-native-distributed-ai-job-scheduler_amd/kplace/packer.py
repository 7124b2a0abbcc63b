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

CacheStrategy "shared" (api/v1/llmservice_types.go:42-44): the CR's replicas
prefer the topology domain of the node that runs its cache coordinator pod
(Status.CacheCoordinator, :60; the agent's lease holder,
cmd/agent/main.go:175-201), so that followers pull the model from a peer on
the same xGMI island / rack; a shared CR without a coordinator yet prefers
the domain of another shared CR of the same model that has one ("prefer nodes
that already hold the cache", docs/PROJECT_ROADMAP.md:173-174). The host
passes the pod -> node map (`pod_nodes`, from its pod informer); the result is
the snapshot's per-job `affinity` (kp_snapshot.affinity).

Invalid objects never abort a batch: a CR the CRD rules reject is left out of
the snapshot and reported in Packed.invalid (the runner writes it a
Placed=False / Invalid condition), as the reference reconciles one CR at a
time and a bad CR fails only its own Reconcile; a Node with an unparsable
quantity is left out (Packed.bad_nodes) and receives no placement.

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
    if int(s["gpuPerReplica"]) > (1 << 31) - 1:
        raise PackError("spec.gpuPerReplica out of int32 range")
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
    cr_keys: list                 # [(namespace, name)] per packed CR, CR index order
    job_cr: np.ndarray            # [J] CR index of each job row
    job_replica: np.ndarray       # [J] replica ordinal within its CR
    node_names: list              # [N]
    domains: list = field(default_factory=list)  # topology domain names, index order
    invalid: dict = field(default_factory=dict)  # (namespace, name) -> reason, not packed
    bad_nodes: dict = field(default_factory=dict)  # node name -> reason, not packed


def _meta(o):
    return o.get("metadata", {}) or {}


def _cr_key(cr) -> tuple:
    md = _meta(cr)
    return (md.get("namespace", "default"), md.get("name", ""))


def pack(crs: list[dict], nodes: list[dict], used: dict | None = None,
         pod_nodes: dict | None = None) -> Packed:
    """CRs (LLMService objects as dicts, in the order the batch runner lists
    them) and Node objects -> one kp_snapshot-shaped Workload. `used`: node
    name -> per-dim usage; `pod_nodes`: (namespace, pod) -> node name, for the
    CacheStrategy "shared" affinity."""
    # ---- nodes ----------------------------------------------------------
    D = len(DIMS)
    caps, useds, names, dom_of, bad_nodes = [], [], [], [], {}
    for node in nodes:
        md = _meta(node)
        name = md.get("name", "")
        alloc = (node.get("status", {}) or {}).get("allocatable", {}) or {}
        labels = md.get("labels", {}) or {}
        try:
            gpus = int(alloc.get(GPU_RESOURCE, 0))
            per_gpu = parse_gpu_memory(labels.get(LABEL_GPU_MEMORY, "") or "") if gpus else 0
            cap = [cpu_milli(alloc.get("cpu", 0)), mem_mib(alloc.get("memory", 0)), gpus,
                   gpus * per_gpu]
            u = [int((used or {}).get(name, {}).get(d, 0)) for d in DIMS]
            if gpus < 0 or any(x < 0 or x > synth_max for x in cap) or \
                    any(x < 0 or x > c for x, c in zip(u, cap)):
                raise PackError("allocatable / usage out of range")
        except (PackError, ValueError, TypeError) as e:
            bad_nodes[name] = str(e)
            continue
        caps.append(cap)
        useds.append(u)
        names.append(name)
        dom_of.append(labels.get(LABEL_ISLAND) or labels.get(LABEL_RACK) or "node/" + name)
    N = len(names)
    cap = np.ascontiguousarray(np.array(caps, np.int64).reshape(N, D).T)
    usedv = np.ascontiguousarray(np.array(useds, np.int64).reshape(N, D).T)
    domains = sorted(set(dom_of))
    index = {d: i for i, d in enumerate(domains)}
    topo = np.array([index[d] for d in dom_of], np.int32)
    node_index = {n: i for i, n in enumerate(names)}

    # ---- CRs -------------------------------------------------------------
    def coordinator_domain(cr) -> int:
        coord = ((cr.get("status", {}) or {}).get("cacheCoordinator") or "")
        if not coord or not pod_nodes:
            return -1
        node = pod_nodes.get((_cr_key(cr)[0], coord))
        return int(topo[node_index[node]]) if node in node_index else -1

    good, invalid = [], {}
    for cr in crs:
        key = _cr_key(cr)
        try:
            if not key[1]:
                raise PackError("metadata.name is required")
            s = defaulted_spec(cr.get("spec", {}) or {})
            p = int((_meta(cr).get("annotations") or {}).get(ANNOT_PRIORITY, 0))
        except (PackError, ValueError, TypeError) as e:
            invalid[key] = str(e)
            continue
        good.append((cr, key, s, p))
    # a shared model's cache domain: its own coordinator, else another shared
    # CR of the same model that has one
    model_dom = {}
    for cr, key, s, p in good:
        if s["cacheStrategy"] == "shared":
            d = coordinator_domain(cr)
            if d >= 0:
                model_dom.setdefault(s["model"], d)
    rows, job_cr, job_rep, prio, aff, keys = [], [], [], [], [], []
    for i, (cr, key, s, p) in enumerate(good):
        keys.append(key)
        a = -1
        if s["cacheStrategy"] == "shared":
            a = coordinator_domain(cr)
            if a < 0:
                a = model_dom.get(s["model"], -1)
        row = [0, 0, int(s["gpuPerReplica"]), int(s["gpuMemoryMiB"])]
        reps = int(s["replicas"])
        rows.extend([row] * reps)
        job_cr.extend([i] * reps)
        job_rep.extend(range(reps))
        prio.extend([p] * reps)
        aff.extend([a] * reps)
    J = len(rows)
    req = np.ascontiguousarray(np.array(rows, np.int64).reshape(J, D).T)
    job_cr = np.array(job_cr, np.int32)
    gsz = np.bincount(job_cr, minlength=len(keys)).astype(np.int32)[job_cr] if J else \
        np.zeros(0, np.int32)
    w = synth.Workload(J, N, D, req, cap, usedv, np.array(prio, np.int32), job_cr.copy(), gsz,
                       topo, name="packed", affinity=np.array(aff, np.int32))
    return Packed(w, keys, job_cr, np.array(job_rep, np.int32), names, domains, invalid,
                  bad_nodes)


synth_max = 1 << 56  # KP_MAX_VALUE: include/kplace.h
