"""Synthetic clusters and pending queues for BASELINE.json configs #2-#5.

Generator contract: splitmix64 with
seed = 0x6B706C6163650000 + config_no; every draw is lo + (x mod (hi-lo+1))
on uint64. Draw k of stream s is splitmix64 output number (s << 40) + k + 1
of that seed, so the whole snapshot is generated with vectorised numpy and is
identical for any consumer (library, oracle, tests, bench).

Node shapes (x mod 4, or x mod 2 = A/B only for config #3):
  A 128000 mCPU, 1 TiB, 8 GPU, 8x288 GiB; B 192000, 2 TiB, 8, 8x288 GiB;
  C 64000, 512 GiB, 0, 0;               D 96000, 768 GiB, 4, 4x192 GiB.
topo_domain = n // 32 (xGMI island / rack).
Job (= one replica of an LLMService CR; a CR's replicas = one gang):
  gpu in {0:40%, 1:30%, 2:15%, 4:10%, 8:5%}; cpu_milli = 1000*[1,32];
  mem_MiB = 1024*[1,128]; gpu_mem_MiB = gpu*1024*[16,288]; prio in [0,3].
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

GAMMA = np.uint64(0x9E3779B97F4A7C15)
M1 = np.uint64(0xBF58476D1CE4E5B9)
M2 = np.uint64(0x94D049BB133111EB)
SEED_BASE = 0x6B706C6163650000

SHAPES = np.array([
    [128000, 1048576, 8, 8 * 294912],   # A
    [192000, 2097152, 8, 8 * 294912],   # B
    [64000, 524288, 0, 0],              # C
    [96000, 786432, 4, 4 * 196608],     # D
], dtype=np.int64)

D = 4  # cpu_milli, mem_MiB, gpu_count, gpu_mem_MiB


def splitmix64(seed: int, stream: int, idx: np.ndarray) -> np.ndarray:
    """splitmix64 output number (stream << 40) + idx + 1 of `seed`."""
    with np.errstate(over="ignore"):
        k = (np.uint64(stream) << np.uint64(40)) + idx.astype(np.uint64) + np.uint64(1)
        z = np.uint64(seed) + k * GAMMA
        z = (z ^ (z >> np.uint64(30))) * M1
        z = (z ^ (z >> np.uint64(27))) * M2
        return z ^ (z >> np.uint64(31))


def draw(x: np.ndarray, lo: int, hi: int) -> np.ndarray:
    return (np.uint64(lo) + x % np.uint64(hi - lo + 1)).astype(np.int64)


@dataclass
class Workload:
    """One snapshot in the C-ABI's SoA layout (include/kplace.h)."""
    J: int
    N: int
    D: int
    req: np.ndarray          # int64 [D, J]
    cap: np.ndarray          # int64 [D, N]
    used: np.ndarray         # int64 [D, N]
    prio: np.ndarray         # int32 [J]
    gang_id: np.ndarray      # int32 [J]
    gang_size: np.ndarray    # int32 [J]
    topo: np.ndarray         # int32 [N]
    name: str = ""
    meta: dict = field(default_factory=dict)
    affinity: np.ndarray | None = None  # int32 [J] preferred topo domain, -1 = none

    def arrays(self):
        return dict(req=self.req, cap=self.cap, used=self.used, prio=self.prio,
                    gang_id=self.gang_id, gang_size=self.gang_size, topo=self.topo,
                    affinity=self.affinity)


def make_nodes(seed: int, N: int, ab_only: bool) -> tuple[np.ndarray, np.ndarray]:
    x = splitmix64(seed, 0, np.arange(N, dtype=np.uint64))
    shape = (x % np.uint64(2 if ab_only else 4)).astype(np.int64)
    cap = SHAPES[shape].T.copy()            # [D, N]
    topo = (np.arange(N, dtype=np.int64) // 32).astype(np.int32)
    return np.ascontiguousarray(cap), topo


def make_crs(seed: int, n_cr: int, gangs: bool):
    """Per-CR draws: (size, gpu, cpu, mem, gpu_mem, prio)."""
    base = np.arange(n_cr, dtype=np.uint64) * np.uint64(8)
    r = [splitmix64(seed, 1, base + np.uint64(k)) for k in range(6)]
    size = np.array([1, 2, 4, 8], np.int64)[(r[0] % np.uint64(4)).astype(np.int64)] if gangs \
        else np.ones(n_cr, np.int64)
    pct = (r[1] % np.uint64(100)).astype(np.int64)
    gpu = np.select([pct < 40, pct < 70, pct < 85, pct < 95], [0, 1, 2, 4], 8).astype(np.int64)
    cpu = 1000 * draw(r[2], 1, 32)
    mem = 1024 * draw(r[3], 1, 128)
    gmem = gpu * 1024 * draw(r[4], 16, 288)
    prio = draw(r[5], 0, 3).astype(np.int32)
    return size, np.stack([cpu, mem, gpu, gmem]), prio


def expand_crs(J: int, size, req_cr, prio_cr, gangs: bool):
    ends = np.cumsum(size)
    n_cr = int(np.searchsorted(ends, J, side="left")) + 1
    size = size[:n_cr].copy()
    size[-1] -= int(ends[n_cr - 1]) - J          # truncate the last gang to fit J
    cr_of_job = np.repeat(np.arange(n_cr), size)
    req = np.ascontiguousarray(req_cr[:, cr_of_job])
    prio = prio_cr[cr_of_job].astype(np.int32)
    if gangs:
        gang_id = cr_of_job.astype(np.int32)
        gang_size = size[cr_of_job].astype(np.int32)
    else:
        gang_id = np.full(J, -1, np.int32)
        gang_size = np.ones(J, np.int32)
    return req, prio, gang_id, gang_size


def config2(J: int = 10_000, N: int = 1_000) -> Workload:
    """#2: J x N x 4, used = 0, singletons, bin-pack score only."""
    seed = SEED_BASE + 2
    cap, topo = make_nodes(seed, N, ab_only=False)
    size, req_cr, prio_cr = make_crs(seed, J, gangs=False)
    req, prio, gid, gsz = expand_crs(J, size, req_cr, prio_cr, gangs=False)
    return Workload(J, N, D, req, cap, np.zeros_like(cap), prio, gid, gsz, topo,
                    name=f"config2_{J}x{N}")


def config3(J: int = 100_000, N: int = 10_000) -> Workload:
    """#3: A/B nodes (8-GPU xGMI islands), gangs of {1,2,4,8} replicas."""
    seed = SEED_BASE + 3
    cap, topo = make_nodes(seed, N, ab_only=True)
    size, req_cr, prio_cr = make_crs(seed, J, gangs=True)
    req, prio, gid, gsz = expand_crs(J, size, req_cr, prio_cr, gangs=True)
    return Workload(J, N, D, req, cap, np.zeros_like(cap), prio, gid, gsz, topo,
                    name=f"config3_{J}x{N}")


def prefill_running(seed: int, cap: np.ndarray, occupancy: float, probes: int = 64):
    """Pre-place synthetic running jobs (the victim pool of config #4) until
    Sum(used)/Sum(cap) >= `occupancy` in EVERY dim.

    Running job k draws its request and priority like a pending job (seed +
    0x1000, so the draws are independent of the queue) and a start node
    x mod N (stream 2); it goes to the first node of start, start+1, ...
    (at most `probes`) where it fits, or is dropped. Phase 1 places the draws
    as drawn until both GPU dims (count, memory) reach `occupancy`; GPU memory
    is the later one (a job asks 16-288 GiB per GPU of a node's 288), so the
    GPU count ends near 0.53 at occupancy 0.30. Phase 2 continues the same
    stream with the GPU fields of each draw zeroed (GPU-less jobs, e.g. the
    CPU side of a serving stack) until CPU and memory reach `occupancy` too.
    Returns (used [D, N], node [R], req [D, R], prio [R])."""
    D_, N = cap.shape
    used = np.zeros_like(cap)
    tot = cap.sum(1).astype(np.float64)
    sums = np.zeros(D_, np.float64)
    rs = seed + 0x1000
    nodes, reqs, prios = [], [], []
    gpu_dims = [d for d in (2, 3) if d < D_]
    phase = 1
    k = 0
    batch = 4096
    done = False
    while not done and k < 40 * N:
        _, rq, pr = make_crs(rs, k + batch, gangs=False)
        starts = (splitmix64(rs, 2, np.arange(k, k + batch, dtype=np.uint64))
                  % np.uint64(N)).astype(np.int64)
        for i in range(batch):
            if phase == 1 and all(sums[d] >= occupancy * tot[d] for d in gpu_dims):
                phase = 2
            if phase == 2 and bool(np.all(sums >= occupancy * tot)):
                done = True
                break
            q = rq[:, k + i].copy()
            if phase == 2:
                q[gpu_dims] = 0
            cand = (starts[i] + np.arange(probes)) % N
            fits = np.all(used[:, cand] + q[:, None] <= cap[:, cand], axis=0)
            hit = np.flatnonzero(fits)
            if hit.size:
                n = int(cand[hit[0]])
                used[:, n] += q
                sums += q
                nodes.append(n)
                reqs.append(q)
                prios.append(int(pr[k + i]))
        k += batch
    req = np.ascontiguousarray(np.array(reqs, np.int64).T.reshape(D_, len(reqs)))
    return used, np.array(nodes, np.int32), req, np.array(prios, np.int32)


def config4(J: int = 200_000, N: int = 20_000, occupancy: float = 0.30) -> Workload:
    """#4: priority tiers 0-3 against a cluster pre-filled with running jobs
    (priorities 0-3; the victim pool for preemption scoring, w.meta['run_*'])
    until every dim is at least `occupancy` used (prefill_running). Singletons
    (one pod each), shapes A-D."""
    seed = SEED_BASE + 4
    cap, topo = make_nodes(seed, N, ab_only=False)
    size, req_cr, prio_cr = make_crs(seed, J, gangs=False)
    req, prio, gid, gsz = expand_crs(J, size, req_cr, prio_cr, gangs=False)
    used, rnode, rreq, rprio = prefill_running(seed, cap, occupancy)
    return Workload(J, N, D, req, cap, used, prio, gid, gsz, topo, name=f"config4_{J}x{N}",
                    meta=dict(run_node=rnode, run_req=rreq, run_prio=rprio))


def config5_trace(total: int = 1_000_000, N: int = 50_000):
    """#5: the streaming trace — a 1M-job queue (singletons, prio 0-3) and a
    50k-node cluster. Returns (cap, topo, req [D, total], prio [total])."""
    seed = SEED_BASE + 5
    cap, topo = make_nodes(seed, N, ab_only=False)
    size, req_cr, prio_cr = make_crs(seed, total, gangs=False)
    req, prio, _, _ = expand_crs(total, size, req_cr, prio_cr, gangs=False)
    return cap, topo, req, prio


def config5_completions(batch_no: int, running_jobs: np.ndarray) -> np.ndarray:
    """Deterministic 20% of the running (previously placed) trace jobs that
    complete after micro-batch `batch_no`: splitmix64(seed, 3 + batch, job)
    mod 5 == 0. Returns a boolean mask over `running_jobs` (trace indices)."""
    x = splitmix64(SEED_BASE + 5, 3 + batch_no, running_jobs.astype(np.uint64))
    return (x % np.uint64(5)) == np.uint64(0)


def config1_objects(sample_specs: list[dict], K: int = 100, N: int = 64):
    """#1: the reference's sample CRs (config/samples, as committed in
    tests/golden/sample_crs.json) plus K synthetic LLMService CRs
    (replicas in [1,8], gpuPerReplica in {0,1,2,4,8}, gpuMemory "<n>Gi") and N
    synthetic corev1.Node reports (shapes A-D, topology label = n // 32), as
    API-object dicts for the snapshot packer (kplace/packer.py)."""
    seed = SEED_BASE + 1
    crs = []
    for i, spec in enumerate(sample_specs):
        crs.append({"metadata": {"name": f"sample-{i}", "namespace": "default"},
                    "spec": dict(spec)})
    r = [splitmix64(seed, 1, np.arange(K, dtype=np.uint64) * np.uint64(4) + np.uint64(k))
         for k in range(4)]
    reps = draw(r[0], 1, 8)
    gpu = np.array([0, 1, 2, 4, 8], np.int64)[(r[1] % np.uint64(5)).astype(np.int64)]
    gmem = draw(r[2], 2, 48) * np.maximum(gpu, 1)
    prio = draw(r[3], 0, 3)
    for k in range(K):
        crs.append({"metadata": {"name": f"llm-{k}", "namespace": "default",
                                 "annotations": {"kubeinfer.ai/priority": str(int(prio[k]))}},
                    "spec": {"model": f"org/model-{k % 7}", "replicas": int(reps[k]),
                             "gpuPerReplica": int(gpu[k]), "gpuMemory": f"{int(gmem[k])}Gi"}})
    x = splitmix64(seed, 0, np.arange(N, dtype=np.uint64))
    shape = (x % np.uint64(4)).astype(np.int64)
    nodes = []
    for n in range(N):
        cpu, mem, g, gm = (int(v) for v in SHAPES[shape[n]])
        labels = {"kubeinfer.ai/xgmi-island": f"island-{n // 32}"}
        if g:
            labels["kubeinfer.ai/gpu-memory"] = f"{gm // g // 1024}Gi"
        nodes.append({"metadata": {"name": f"node-{n:03d}", "labels": labels},
                      "status": {"allocatable": {"cpu": str(cpu // 1000), "memory": f"{mem}Mi",
                                                 "amd.com/gpu": str(g)}}})
    return crs, nodes


def workload_objects(w: Workload, shared_every: int = 0):
    """A workload as API objects for the host path (packer -> kp_place ->
    binder): one LLMService CR per gang (replicas = gang size, gpuPerReplica
    and gpuMemory from the job's request, priority annotation) and one Node
    per node (allocatable cpu / memory / amd.com/gpu, per-GPU memory label,
    xGMI island label = topo domain). The CRD has no cpu/mem fields, so the
    packed queue carries gpu and gpu memory only. Every `shared_every`-th CR
    uses CacheStrategy shared with a coordinator pod on node (CR index mod
    N); returns (crs, nodes, pod_nodes)."""
    J, N = w.J, w.N
    starts = np.flatnonzero(np.r_[True, (w.gang_id[1:] != w.gang_id[:-1]) | (w.gang_id[1:] < 0)])
    sizes = np.diff(np.r_[starts, J])
    crs, pod_nodes = [], {}
    for i, (j, sz) in enumerate(zip(starts.tolist(), sizes.tolist())):
        spec = {"model": f"org/model-{i % 13}", "replicas": int(sz),
                "gpuPerReplica": int(w.req[2, j]), "gpuMemory": f"{int(w.req[3, j])}Mi"}
        cr = {"metadata": {"name": f"llm-{i}", "namespace": "default",
                           "annotations": {"kubeinfer.ai/priority": str(int(w.prio[j]))}},
              "spec": spec}
        if shared_every and i % shared_every == 0:
            spec["cacheStrategy"] = "shared"
            cr["status"] = {"cacheCoordinator": f"llm-{i}-coord"}
            pod_nodes[("default", f"llm-{i}-coord")] = f"node-{i % N:05d}"
        crs.append(cr)
    nodes = []
    for n in range(N):
        g = int(w.cap[2, n])
        labels = {"kubeinfer.ai/xgmi-island": f"island-{int(w.topo[n]):05d}"}
        if g:
            labels["kubeinfer.ai/gpu-memory"] = f"{int(w.cap[3, n]) // g}Mi"
        nodes.append({"metadata": {"name": f"node-{n:05d}", "labels": labels},
                      "status": {"allocatable": {"cpu": f"{int(w.cap[0, n])}m",
                                                 "memory": f"{int(w.cap[1, n])}Mi",
                                                 "amd.com/gpu": str(g)}}})
    return crs, nodes, pod_nodes


# scoring knobs per config
CONFIG_PARAMS = {
    2: dict(w_dim=(1, 1, 1, 1), w_gpu_fit=0, w_spread=0),
    3: dict(w_dim=(1, 1, 4, 2), w_gpu_fit=1024, w_spread=256),
    1: dict(w_dim=(1, 1, 4, 2), w_gpu_fit=1024, w_spread=256),
    4: dict(w_dim=(1, 1, 4, 2), w_gpu_fit=1024, w_spread=0),
    # streaming: 32 candidates per unit (13 vs 22 rounds per 5k batch in steady state)
    5: dict(w_dim=(1, 1, 4, 2), w_gpu_fit=1024, w_spread=0, n_cand=32),
}


def config(no: int, J: int | None = None, N: int | None = None) -> Workload:
    if no == 2:
        return config2(J or 10_000, N or 1_000)
    if no == 3:
        return config3(J or 100_000, N or 10_000)
    if no == 4:
        return config4(J or 200_000, N or 20_000)
    raise ValueError(f"config #{no} generator not implemented")
