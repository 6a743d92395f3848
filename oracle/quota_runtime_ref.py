"""ElasticQuota runtime (RefreshRuntime) restated at object level — TEST INFRASTRUCTURE ONLY.

Follows the reference (paths under pkg/scheduler/plugins/elasticquota/core/):

* request aggregation, bottom-up: ``recursiveUpdateGroupTreeWithDeltaRequest``
  (group_quota_manager.go:184-226): a quota's ChildRequest is its own pods' request plus its
  children's *limited* requests; a quota that does not allow lending requests at least its Min
  (:201-213); the limited request is min(Request, Max) on the keys of Max
  (quota_info.go:217-228, ``getLimitRequestNoLock``).
* runtime, top-down: ``refreshRuntimeNoLock`` (group_quota_manager.go:266-326) hands each
  parent's runtime to its children's calculator; the root's children share
  ``totalResourceExceptSystemAndDefaultUsed``.  Per resource dimension, ``redistribution`` /
  ``iterationForRedistribution`` (runtime_quota_calculator.go:111-168) give every child
  max(min, guarantee) (or its request when it may lend and asks for less) and then share the
  rest by sharedWeight, ``int64(float64(w)*float64(total)/float64(Σw) + 0.5)``, until no
  child asks for more.
* the dimensions of every calculator are the union of all quotas' Max keys
  (``updateResourceKeyNoLock``, group_quota_manager.go:565-583); missing values are 0.

Not modelled: the scale-min-quota manager (``scaleMinQuotaEnabled``; AutoScaleMin = Min here).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional


@dataclass
class Quota:
    name: str
    parent: Optional[str]  # None = child of the root quota
    max: Dict[str, int]
    min: Dict[str, int] = field(default_factory=dict)
    shared_weight: Optional[Dict[str, int]] = None  # default: Max (AnnotationSharedWeight absent)
    guaranteed: Dict[str, int] = field(default_factory=dict)
    self_request: Dict[str, int] = field(default_factory=dict)  # Σ requests of pods in this quota
    allow_lent: bool = True


def _limit_request(request: Dict[str, int], mx: Dict[str, int]) -> Dict[str, int]:
    out = dict(request)
    for r, q in request.items():
        if r in mx and q > mx[r]:
            out[r] = mx[r]
    return out


def aggregate_requests(quotas: List[Quota]) -> Dict[str, Dict[str, int]]:
    """Request (after the allow-lent rule) of every quota, children before parents."""
    by = {q.name: q for q in quotas}
    children: Dict[Optional[str], List[str]] = {}
    for q in quotas:
        children.setdefault(q.parent, []).append(q.name)
    request: Dict[str, Dict[str, int]] = {}

    def visit(name: str) -> Dict[str, int]:
        q = by[name]
        child = {r: max(v, 0) for r, v in q.self_request.items()}
        for c in children.get(name, []):
            for r, v in _limit_request(visit(c), by[c].max).items():
                child[r] = child.get(r, 0) + v
        real = dict(child)
        if not q.allow_lent:
            for r, m in q.min.items():
                if r not in real or m > real[r]:
                    real[r] = m
        request[name] = real
        return real

    for root_child in children.get(None, []):
        visit(root_child)
    return request


def redistribution(total: int, nodes: List[dict]) -> None:
    """runtime_quota_calculator.go:111-143 on one dimension; nodes get 'runtime'."""
    to_partition = total
    total_sw = 0
    adjust = []
    for n in nodes:
        mn = n["min"]
        if n["guarantee"] > mn:
            mn = n["guarantee"]
        if n["request"] > mn:
            adjust.append(n)
            total_sw += n["sw"]
            n["runtime"] = mn
        else:
            n["runtime"] = n["request"] if n["allow_lent"] else mn
        to_partition -= n["runtime"]
    if to_partition > 0:
        _iterate(to_partition, total_sw, adjust)


def _iterate(total: int, total_sw: int, nodes: List[dict]) -> None:
    """runtime_quota_calculator.go:145-168"""
    while True:
        if total_sw <= 0:
            return
        adjust = []
        to_partition, adjust_sw = 0, 0
        for n in nodes:
            delta = int(float(n["sw"]) * float(total) / float(total_sw) + 0.5)
            n["runtime"] += delta
            if n["runtime"] < n["request"]:
                adjust.append(n)
                adjust_sw += n["sw"]
            else:
                to_partition += n["runtime"] - n["request"]
                n["runtime"] = n["request"]
        if not (to_partition > 0 and adjust):
            return
        total, total_sw, nodes = to_partition, adjust_sw, adjust


def refresh_runtime(quotas: List[Quota], cluster_total: Dict[str, int]) -> Dict[str, Dict[str, int]]:
    """Runtime of every quota on every resource key (the union of all Max keys)."""
    keys = set()
    for q in quotas:
        keys.update(q.max.keys())
    request = aggregate_requests(quotas)
    by = {q.name: q for q in quotas}
    children: Dict[Optional[str], List[str]] = {}
    for q in quotas:
        children.setdefault(q.parent, []).append(q.name)
    runtime: Dict[str, Dict[str, int]] = {q.name: {} for q in quotas}

    def level(parent: Optional[str], total: Dict[str, int]) -> None:
        kids = children.get(parent, [])
        if not kids:
            return
        for r in keys:
            nodes = []
            for c in kids:
                q = by[c]
                sw = (q.shared_weight if q.shared_weight is not None else q.max).get(r, 0)
                nodes.append({"name": c, "sw": sw, "request": _limit_request(request[c], q.max).get(r, 0),
                              "min": q.min.get(r, 0), "guarantee": q.guaranteed.get(r, 0),
                              "allow_lent": q.allow_lent, "runtime": 0})
            redistribution(total.get(r, 0), nodes)
            for n in nodes:
                runtime[n["name"]][r] = n["runtime"]
        for c in kids:
            level(c, runtime[c])

    level(None, cluster_total)
    return runtime
