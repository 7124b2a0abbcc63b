"""Bind-result writer: a placement -> one
LLMServiceCondition per CR, written through the status subresource without any
API type change (api/v1/llmservice_types.go:55-61,92-98; the reference's
status write is `r.Status().Update`, internal/controller/llmservice_controller.go:164).

Condition `Placed`: Status "True" when every replica of the CR got a node
(Reason "BatchPlaced", Message "replica 0 -> node-a, replica 1 -> node-b, ..."),
"False" otherwise (Reason "NoFit" / "RoundLimit" from the job status, plus the
preemption nomination when kp_preempt produced one). Objects from the informer
cache are never mutated: the writer returns new status dicts.
"""
from __future__ import annotations

import copy
import datetime as _dt

import numpy as np

from . import _abi

COND_TYPE = "Placed"


def _now() -> str:
    return _dt.datetime.now(_dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


def conditions(packed, result: dict, preemption: dict | None = None, now: str | None = None):
    """{(namespace, name): condition dict} for every CR of the packed batch,
    plus a Placed=False / Invalid condition for every CR the packer rejected.
    Jobs are grouped by CR once (their rows are contiguous per CR), so the
    writer is O(J + CRs), not O(J x CRs)."""
    now = now or _now()
    node = np.asarray(result["node"])
    status = np.asarray(result["status"])
    n_cr = len(packed.cr_keys)
    job_cr = np.asarray(packed.job_cr)
    counts = np.bincount(job_cr, minlength=n_cr) if job_cr.size else np.zeros(n_cr, np.int64)
    order = np.argsort(job_cr, kind="stable")
    starts = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.int64)
    ok = node[order] >= 0
    # per CR: every replica placed (empty CRs: not placed)
    all_ok = np.zeros(n_cr, bool)
    nz = counts > 0
    if ok.size:
        all_ok[nz] = np.logical_and.reduceat(ok, starts[nz])
    names = packed.node_names
    out = {}
    for i, key in enumerate(packed.cr_keys):
        jobs = order[starts[i]:starts[i] + counts[i]]
        if all_ok[i]:
            msg = ", ".join(f"replica {int(packed.job_replica[j])} -> {names[node[j]]}"
                            for j in jobs)
            out[key] = {"type": COND_TYPE, "status": "True", "reason": "BatchPlaced",
                        "message": msg, "lastUpdateTime": now}
            continue
        st = int(status[jobs[0]]) if jobs.size else _abi.KP_JOB_NO_FIT
        reason = "RoundLimit" if st == _abi.KP_JOB_ROUND_LIMIT else "NoFit"
        msg = f"{jobs.size} replica(s) unplaced"
        if preemption is not None and jobs.size and preemption["node"][jobs[0]] >= 0:
            j = jobs[0]
            msg += (f"; nominated {names[preemption['node'][j]]} "
                    f"(evicts {int(preemption['victims'][j])}, priority cost "
                    f"{int(preemption['cost'][j])})")
        out[key] = {"type": COND_TYPE, "status": "False", "reason": reason, "message": msg,
                    "lastUpdateTime": now}
    for key, why in getattr(packed, "invalid", {}).items():
        out[key] = {"type": COND_TYPE, "status": "False", "reason": "Invalid",
                    "message": why, "lastUpdateTime": now}
    return out


def status_with_condition(cr: dict, cond: dict) -> dict:
    """New LLMServiceStatus for `cr` with its Placed condition replaced (the
    cached object is left untouched; AvailableReplicas is kept)."""
    st = copy.deepcopy(cr.get("status", {}) or {})
    st.setdefault("availableReplicas", 0)
    conds = [c for c in st.get("conditions", []) or [] if c.get("type") != COND_TYPE]
    conds.append(dict(cond))
    st["conditions"] = conds
    return st
