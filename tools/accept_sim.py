"""Offline model of k_accept's memory round trips per pass (analysis tool, not
product code). Replays the oracle's proposals (KPO_DUMP, oracle/kp_oracle.c)
over the GPU's bidder index layout (rows of (slot, candidate) entries in node
order, slots in rank order, 64-entry windows) and counts, per node with bids,
the dependent load levels its wave walks: the node record, the node's flag +
usage, the window flags + minima of each 64-window chunk, and one level per
batch of flagged windows that pass the window-minimum test. The per-pass
critical path is the node with the most levels.

  make -C oracle analysis
  KPO_LIB=$PWD/oracle/libkp_oracle_analysis.so KPO_DUMP=/tmp/c3.dump python tools/round_shape.py 3 > /dev/null
  python tools/accept_sim.py /tmp/c3.dump 3
  TAIL=1 ...: per pass, the node with the most decided windows (the tail of the
  launch): its bidder entries, windows, flagged windows, windows that pass the
  window-minimum test (decided), windows with a bidder that fits, accepted bids
"""
import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tests"))
import oracle_bind as ob  # noqa: E402
from kplace import _abi, synth  # noqa: E402


def read_dump(path):
    a = np.fromfile(path, dtype=np.int32)
    i, rounds = 0, []
    while i < a.size:
        tag = a[i]
        if tag == -1:
            r, U, K = a[i + 1], a[i + 2], a[i + 3]
            cand = a[i + 4:i + 4 + U * K].reshape(U, K)
            i += 4 + U * K
            rounds.append({"round": int(r), "cand": cand, "passes": []})
        else:
            assert tag == -2
            npr = a[i + 2]
            props = a[i + 4:i + 4 + 4 * npr].reshape(npr, 4)
            i += 4 + 4 * npr
            rounds[-1]["passes"].append(props)
    return rounds


def main():
    path, no = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 3
    batch = int(os.environ.get("BATCH", "2"))
    w = synth.config(no)
    p = _abi.default_params(**synth.CONFIG_PARAMS[no])
    L = ob.lib()
    sb = ob.SnapshotBuf.from_workload(w)
    st = C.c_void_p()
    assert L.kpo_state_new(C.byref(sb.snap), C.byref(p), C.byref(st)) == 0
    U = L.kpo_state_units(st)
    lead = np.array([L.kpo_state_unit_leader(st, u) for u in range(U)], np.int64)
    L.kpo_state_free(st)
    q = w.req[:, lead]  # [D, U]
    D = q.shape[0]
    used = w.used.copy()
    rounds = read_dump(path)
    MODES = ("cur", "bidmin", "wg", "wg8", "wg16")
    tot = {k: 0 for k in MODES}
    per_round = []
    for rd in rounds:
        cand = rd["cand"]
        K = cand.shape[1]
        act = np.nonzero(cand[:, 0] >= 0)[0]  # slots in rank order
        ent_slot = np.repeat(act, K)
        ent_node = cand[act].reshape(-1)
        ok = ent_node >= 0
        ent_slot, ent_node = ent_slot[ok], ent_node[ok]
        order = np.lexsort((ent_slot, ent_node))  # rows in node order, slots in rank order
        ent_slot, ent_node = ent_slot[order], ent_node[order]
        P = ent_node.size
        nodes, starts, counts = np.unique(ent_node, return_index=True, return_counts=True)
        nwin = (P + 63) // 64
        pad = nwin * 64 - P
        qe = q[:, ent_slot]
        winmin = np.pad(qe, ((0, 0), (0, pad)), constant_values=np.iinfo(np.int64).max)
        winmin = winmin.reshape(D, nwin, 64).min(axis=2)
        key = ent_node.astype(np.int64) * (U + 1) + ent_slot
        rsum = {k: 0 for k in MODES}
        for props in rd["passes"]:
            # entry of every proposal; window flags of this pass
            pk = props[:, 1].astype(np.int64) * (U + 1) + props[:, 0]
            e = np.searchsorted(key, pk)
            assert np.array_equal(key[e], pk)
            m = np.zeros(P, np.int64)
            m[e] = props[:, 2]
            flag = np.zeros(nwin, bool)
            flag[e // 64] = True
            need = qe * m  # [D, P]
            bidmin = np.where(m > 0, need, np.iinfo(np.int64).max)
            bidmin = np.pad(bidmin, ((0, 0), (0, pad)), constant_values=np.iinfo(np.int64).max)
            bidmin = bidmin.reshape(D, nwin, 64).min(axis=2)
            worst = {k: 0 for k in MODES}
            bid_nodes = np.unique(props[:, 1])
            if os.environ.get("TAIL"):
                tail = None
                for n in bid_nodes:
                    i = np.searchsorted(nodes, n)
                    e0, e1 = starts[i], starts[i] + counts[i]
                    rem = w.cap[:, n] - used[:, n]
                    dec = fitw = acc = nfl = 0
                    for x in range(e0 // 64, (e1 - 1) // 64 + 1):
                        if not flag[x]:
                            continue
                        nfl += 1
                        if not (winmin[:, x] <= rem).all():
                            continue
                        dec += 1
                        lo, hi = max(x * 64, e0), min(x * 64 + 64, e1)
                        any_fit = False
                        for ee in range(lo, hi):
                            if m[ee] and (need[:, ee] <= rem).all():
                                rem = rem - need[:, ee]
                                acc += 1
                                any_fit = True
                        fitw += any_fit
                    if tail is None or dec > tail[4]:
                        tail = (n, e1 - e0, (e1 - 1) // 64 - e0 // 64 + 1, nfl, dec, fitw, acc)
                print(f"  pass: node {tail[0]} entries {tail[1]} windows {tail[2]} flagged {tail[3]} "
                      f"decided {tail[4]} with-fit {tail[5]} accepted {tail[6]}", flush=True)
            for n in bid_nodes:
                i = np.searchsorted(nodes, n)
                e0, e1 = starts[i], starts[i] + counts[i]
                w0, w1 = e0 // 64, (e1 - 1) // 64
                for mode in MODES:
                    rem = w.cap[:, n] - used[:, n]
                    lv = 2  # node record; node flag + usage
                    # wg8 / wg16: a workgroup per node loads the first chunk's window
                    # flags with the node flag, then up to 8 / 16 windows per level
                    merged = mode in ("wg8", "wg16")
                    if w0 == w1:
                        lv += 1
                    else:
                        mins = bidmin if mode == "bidmin" else winmin
                        wb = w0
                        while wb <= w1:
                            if not (merged and wb == w0):
                                lv += 1  # chunk flags + minima
                            ws = [x for x in range(wb, min(wb + 64, w1 + 1)) if flag[x]]
                            pending = list(ws)
                            while True:
                                pending = [x for x in pending if (mins[:, x] <= rem).all()]
                                if not pending:
                                    break
                                bm = {"wg": 1 << 30, "wg8": 8, "wg16": 16}.get(mode, batch)
                                take = pending[:bm]
                                lv += 1
                                for x in take:
                                    lo, hi = max(x * 64, e0), min(x * 64 + 64, e1)
                                    for ee in range(lo, hi):
                                        if m[ee] and (need[:, ee] <= rem).all():
                                            rem = rem - need[:, ee]
                                pending = pending[len(take):]
                            wb += 64
                    worst[mode] = max(worst[mode], lv)
            for k in worst:
                rsum[k] += worst[k]
            # commit (all-or-nothing per unit)
            bad = np.zeros(U, bool)
            bad[props[props[:, 3] == 0, 0]] = True
            good = ~bad[props[:, 0]]
            for u, n, c, _ in props[good]:
                used[:, n] += c * q[:, u]
        per_round.append((rd["round"], len(rd["passes"]), rsum))
        for k in tot:
            tot[k] += rsum[k]
        print(f"round {rd['round']:3d} passes {len(rd['passes']):2d} levels/pass: "
              + " ".join(f"{k} {rsum[k] / max(1, len(rd['passes'])):.1f}" for k in rsum), flush=True)
    npass = sum(x[1] for x in per_round)
    print("total passes", npass, "mean critical-path levels per pass:",
          {k: round(v / npass, 2) for k, v in tot.items()})


if __name__ == "__main__":
    main()
