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

from . import _abi

COND_TYPE = "Placed"


def _now() -> str:
    return _dt.datetime.now(_dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


def conditions(packed, result: dict, preemption: dict | None = None, now: str | None = None):
    """{(namespace, name): condition dict} for every CR of the packed batch."""
    now = now or _now()
    node, status = result["node"], result["status"]
    out = {}
    for i, key in enumerate(packed.cr_keys):
        jobs = [j for j in range(len(packed.job_cr)) if packed.job_cr[j] == i]
        if jobs and all(node[j] >= 0 for j in jobs):
            msg = ", ".join(f"replica {int(packed.job_replica[j])} -> {packed.node_names[node[j]]}"
                            for j in jobs)
            out[key] = {"type": COND_TYPE, "status": "True", "reason": "BatchPlaced",
                        "message": msg, "lastUpdateTime": now}
            continue
        st = int(status[jobs[0]]) if jobs else _abi.KP_JOB_NO_FIT
        reason = "RoundLimit" if st == _abi.KP_JOB_ROUND_LIMIT else "NoFit"
        msg = f"{len(jobs)} replica(s) unplaced"
        if preemption is not None and jobs and preemption["node"][jobs[0]] >= 0:
            j = jobs[0]
            msg += (f"; nominated {packed.node_names[preemption['node'][j]]} "
                    f"(evicts {int(preemption['victims'][j])}, priority cost "
                    f"{int(preemption['cost'][j])})")
        out[key] = {"type": COND_TYPE, "status": "False", "reason": reason, "message": msg,
                    "lastUpdateTime": now}
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
