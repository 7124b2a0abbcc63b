"""Second, independent CPU restatement of the placement spec
in plain Python, for small cases only. Test infrastructure: it cross-checks
the C oracle (oracle/kp_oracle.c) so that neither restatement is trusted
alone. Written from the spec text, not from the C code: it keeps whole
candidate lists sorted with Python's sort and recomputes scores from scratch.
"""
from __future__ import annotations

MASK32 = 0xFFFFFFFF
TIE_MUL = 0x9E3779B1


def fmix32(h):
    h &= MASK32
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & MASK32
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & MASK32
    h ^= h >> 16
    return h


def util(x, c, S, most):
    """One dimension's utilisation score, kube-scheduler's integer formulas:
    mostRequestedScore floor(x*S/c), leastRequestedScore floor((c-x)*S/c)."""
    return (x * S) // c if most else ((c - x) * S) // c


def place(req, cap, used, prio, gang_id, topo, p, affinity=None):
    """req[d][j], cap[d][n], used[d][n] as nested lists / numpy; p = dict of
    kp_params fields; affinity[j] = preferred topo domain or -1. Returns
    dict(node, score, status, used, rounds, passes)."""
    D = len(cap)
    N = len(cap[0]) if D else 0
    J = len(req[0]) if D else 0
    cap = [[int(x) for x in row] for row in cap]
    used = [[int(x) for x in row] for row in used]
    req = [[int(x) for x in row] for row in req]
    topo = [int(t) for t in topo] if topo is not None else list(range(N))
    S = p["util_scale"]
    w = p["w_dim"]
    most = p["score_mode"] == 0
    aff_j = [int(a) for a in affinity] if affinity is not None else [-1] * J

    # §2.2 units
    units = []  # (leader, size, prio)
    j = 0
    while j < J:
        g = gang_id[j] if gang_id is not None else -1
        e = j + 1
        if g >= 0:
            while e < J and gang_id[e] == g:
                e += 1
        units.append((j, e - j, int(prio[j]) if prio is not None else 0, aff_j[j]))
        j = e
    units.sort(key=lambda u: (-u[2], u[0]))
    U = len(units)
    salt = [fmix32(u[0] ^ p["tie_seed"]) for u in units]
    status = ["A"] * U
    job_node = [-1] * J
    job_score = [-1] * J

    def S_(u, q, n, bu):
        s = 0
        for d in range(D):
            if q[d] > cap[d][n] - bu[d]:
                return -1
            if cap[d][n] > 0:
                s += w[d] * util(bu[d] + q[d], cap[d][n], S, most)
        g = p["gpu_dim"]
        if g >= 0 and q[g] > 0 and cap[g][n] - bu[g] - q[g] == 0:
            s += p["w_gpu_fit"]
        a = units[u][3]
        if a >= 0 and topo[n] == a:
            s += p.get("w_affinity", 0)
        return s

    # canonical position: rank in the order (cap vector, node index)
    order = sorted(range(N), key=lambda n: (tuple(cap[d][n] for d in range(D)), n))
    pos = [0] * N
    for i, n in enumerate(order):
        pos[n] = i

    def tie(u, n):
        return pos[n] if p["tie_mode"] == 0 else (pos[n] * TIE_MUL + salt[u]) & MASK32

    def q_of(u):
        return [req[d][units[u][0]] for d in range(D)]

    rounds = passes = 0
    K = p["n_cand"]
    while any(s == "A" for s in status):
        if p["max_rounds"] and rounds >= p["max_rounds"]:
            break
        # §2.4 candidates against round-start usage
        cands = {}
        for u in range(U):
            if status[u] != "A":
                continue
            q = q_of(u)
            scored = [(S_(u, q, n, [used[d][n] for d in range(D)]), n) for n in range(N)]
            scored = [(s, n) for s, n in scored if s >= 0]
            scored.sort(key=lambda t: (-t[0], tie(u, t[1])))
            cands[u] = [n for _, n in scored[:K]]
            if not cands[u]:
                status[u] = "F"
        open_ = {u for u in cands if cands[u]}
        for ps in range(p["max_passes"]):
            props = []
            for u in sorted(open_):
                q = q_of(u)
                cl = cands[u]
                planned = [0] * len(cl)
                ok = True
                for _m in range(units[u][1]):
                    best = None
                    for c, n in enumerate(cl):
                        bu = [used[d][n] + planned[c] * q[d] for d in range(D)]
                        s = S_(u, q, n, bu)
                        if s < 0:
                            continue
                        dom = sum(planned[c2] for c2 in range(len(cl)) if topo[cl[c2]] == topo[n])
                        v = s - p["w_spread"] * dom
                        if best is None or v > best[0]:
                            best = (v, c)
                    if best is None:
                        ok = False
                        break
                    planned[best[1]] += 1
                if not ok:
                    open_.discard(u)
                    if ps == 0:
                        status[u] = "F"
                    continue
                off = 0
                for c, n in enumerate(cl):
                    if planned[c]:
                        props.append((n, u, planned[c], off,
                                      S_(u, q, n, [used[d][n] for d in range(D)])))
                        off += planned[c]
            if not props:
                break
            passes += 1
            props.sort(key=lambda t: (t[0], t[1], t[3]))
            okp = {}
            rem = {}
            for (n, u, cnt, off, sc) in props:
                if n not in rem:
                    rem[n] = [cap[d][n] - used[d][n] for d in range(D)]
                q = q_of(u)
                fits = all(cnt * q[d] <= rem[n][d] for d in range(D))
                okp[(n, u, off)] = fits
                if fits:
                    for d in range(D):
                        rem[n][d] -= cnt * q[d]
            bad = {u for (n, u, off), f in okp.items() if not f}
            for (n, u, cnt, off, sc) in props:
                if u in bad:
                    continue
                q = q_of(u)
                for d in range(D):
                    used[d][n] += cnt * q[d]
                for m in range(cnt):
                    job_node[units[u][0] + off + m] = n
                    job_score[units[u][0] + off + m] = sc
                status[u] = "P"
                open_.discard(u)
        rounds += 1
    code = {"P": 0, "F": 1, "A": 2}
    out_status = [0] * J
    for u, (ld, sz, _, _a) in enumerate(units):
        for m in range(sz):
            out_status[ld + m] = code[status[u]]
            if status[u] != "P":
                job_node[ld + m] = -1
                job_score[ld + m] = -1
    return dict(node=job_node, score=job_score, status=out_status, used=used,
                rounds=rounds, passes=passes)


def preempt(req, cap, used_after, prio, status, singleton, run_node, run_req, run_prio):
    """Preemption candidates, restated from the spec text:
    for each NO_FIT singleton job, every node's evictable running jobs
    (priority below the job's) in (priority desc, index asc) reprieve order;
    best node by (victims, sum of victim priorities, node index).
    Returns (node, victims, cost) lists over jobs."""
    D = len(cap)
    N = len(cap[0]) if D else 0
    J = len(prio)
    R = len(run_node)
    by_node = {n: [] for n in range(N)}
    for r in range(R):
        by_node[int(run_node[r])].append(r)
    for n in by_node:
        by_node[n].sort(key=lambda r: (-int(run_prio[r]), r))
    out_n, out_v, out_c = [-1] * J, [0] * J, [0] * J
    for j in range(J):
        if int(status[j]) != 1 or not singleton[j]:   # KP_JOB_NO_FIT, gang size 1
            continue
        p = int(prio[j])
        q = [int(req[d][j]) for d in range(D)]
        best = None
        for n in range(N):
            V = [r for r in by_node[n] if int(run_prio[r]) < p]
            avail = [int(cap[d][n]) - int(used_after[d][n]) + sum(int(run_req[d][r]) for r in V)
                     for d in range(D)]
            if any(q[d] > avail[d] for d in range(D)):
                continue
            cnt = cost = 0
            for r in V:
                rq = [int(run_req[d][r]) for d in range(D)]
                if all(q[d] <= avail[d] - rq[d] for d in range(D)):
                    avail = [avail[d] - rq[d] for d in range(D)]
                else:
                    cnt += 1
                    cost += int(run_prio[r])
            if best is None or (cnt, cost, n) < best:
                best = (cnt, cost, n)
        if best is not None:
            out_n[j], out_v[j], out_c[j] = best[2], best[0], best[1]
    return out_n, out_v, out_c
