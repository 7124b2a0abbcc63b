"""Per-round shape of a solve, from the CPU oracle's stepwise interface
(analysis tool, not product code): active slots A, bidder entries A*K, distinct
candidate nodes (the bid-node bound), the longest bidder row, unit sizes and the
passes the round ran. Sizes the one-workgroup LDS round kernel.

  python tools/round_shape.py [config_no] [J] [N]     (MAXR=r: the first r rounds only)
"""
import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tests"))
import oracle_bind as ob  # noqa: E402
from kplace import _abi, synth  # noqa: E402


def main():
    no = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    J = int(sys.argv[2]) if len(sys.argv) > 2 else None
    N = int(sys.argv[3]) if len(sys.argv) > 3 else None
    w = synth.config(no, J, N)
    p = _abi.default_params(**synth.CONFIG_PARAMS[no])
    L = ob.lib()
    sb = ob.SnapshotBuf.from_workload(w)
    st = C.c_void_p()
    assert L.kpo_state_new(C.byref(sb.snap), C.byref(p), C.byref(st)) == 0
    U, K = L.kpo_state_units(st), p.n_cand
    sizes = np.array([L.kpo_state_unit_size(st, u) for u in range(U)], np.int32)
    cand = np.full((U, K), -1, np.int32)
    r = 0
    print("round      A    A*K  nodes  maxrow  size>1  passes")
    tot_p = 0
    maxr = int(os.environ.get("MAXR", "0"))
    while L.kpo_state_active(st) > 0 and not (maxr and r >= maxr):
        cand[:] = -1
        L.kpo_round_candidates(st, 0, U, cand.ctypes.data_as(C.POINTER(C.c_int32)), os.cpu_count())
        act = cand[:, 0] >= 0
        A = int(act.sum())
        c = cand[act]
        valid = c[c >= 0]
        nodes, counts = np.unique(valid, return_counts=True)
        res = ob.ResultBuf(w.J, w.D, w.N)
        L.kpo_state_result(st, C.byref(res.res))
        p0 = res.res.passes
        L.kpo_round_run(st, cand.reshape(-1).ctypes.data_as(C.POINTER(C.c_int32)))
        L.kpo_state_result(st, C.byref(res.res))
        passes = res.res.passes - p0
        tot_p += passes
        print(f"{r:5d} {A:6d} {valid.size:6d} {nodes.size:6d} {counts.max() if counts.size else 0:7d} "
              f"{int((sizes[act] > 1).sum()):7d} {passes:7d}")
        r += 1
    print(f"rounds {r} passes {tot_p}")
    L.kpo_state_free(st)


if __name__ == "__main__":
    main()
