"""world_size 2 (gloo, CPU) test of the multi-GPU protocol:
units are sharded by rank position; each rank runs the candidate phase
(the J x N part) for its shard only, candidates are all-gathered, and every
rank runs the same acceptance passes on the union. The result must equal the
single-process placement bit for bit on every rank. libkplace runs the same
protocol over RCCL (kp_api.cpp exchange_candidates); this test pins the
protocol itself with the CPU oracle as the per-rank compute."""
import ctypes as C
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, cfg, out_q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.join(os.path.dirname(here),
                                    "kubernetes-native-distributed-ai-job-scheduler_amd"))
    import torch
    import oracle_bind as ob
    from kplace import _abi, synth
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    no, J, N = cfg
    w = synth.config(no, J, N)
    p = _abi.default_params(**synth.CONFIG_PARAMS[no])
    L = ob.lib()
    sb = ob.SnapshotBuf.from_workload(w)
    st = C.c_void_p()
    assert L.kpo_state_new(C.byref(sb.snap), C.byref(p), C.byref(st)) == 0
    U, K = L.kpo_state_units(st), p.n_cand
    lo, hi = U * rank // world, U * (rank + 1) // world
    sizes = [U * (r + 1) // world - U * r // world for r in range(world)]
    maxs = max(sizes)
    while L.kpo_state_active(st) > 0:
        local = np.full((maxs, K), -1, np.int32)
        L.kpo_round_candidates(st, lo, hi, local.ctypes.data_as(C.POINTER(C.c_int32)), 2)
        bufs = [torch.empty((maxs, K), dtype=torch.int32) for _ in range(world)]
        dist.all_gather(bufs, torch.from_numpy(local))
        cand = np.concatenate([b.numpy()[:sizes[r]] for r, b in enumerate(bufs)])
        cand = np.ascontiguousarray(cand.reshape(-1))
        L.kpo_round_run(st, cand.ctypes.data_as(C.POINTER(C.c_int32)))
    rb = ob.ResultBuf(w.J, w.D, w.N)
    L.kpo_state_result(st, C.byref(rb.res))
    L.kpo_state_free(st)
    got = rb.as_dict()
    # every rank must hold the identical assignment
    t = torch.from_numpy(got["node"].astype(np.int64))
    all_nodes = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(all_nodes, t)
    same = all(torch.equal(all_nodes[0], x) for x in all_nodes)
    if rank == 0:
        ref = ob.place(sb, p, nthreads=2)
        ok = same and all(np.array_equal(got[k], ref[k]) for k in ("node", "score", "status", "used"))
        out_q.put((ok, got["rounds"], ref["rounds"], got["passes"], ref["passes"]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("cfg", [(2, 3000, 300), (3, 4000, 256)])
def test_sharded_protocol_matches_single_process(oracle, cfg):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, cfg, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = q.get(timeout=300)
    for pr in procs:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    ok, r1, r0, p1, p0 = res
    assert ok, "sharded placement differs from the single-process one"
    assert (r1, p1) == (r0, p0)
