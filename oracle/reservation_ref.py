"""Reservation plugin restated at object level — TEST INFRASTRUCTURE ONLY.

Resources are dicts {name: int64} with cpu in milli-cores (Quantity.MilliValue) and everything
else in Value() units, as the reduced form uses.  Paths below are under
pkg/scheduler/plugins/reservation/ unless stated.

* restore (BeforePreFilter, transformer.go:41-235): per node, available reservations whose
  owners match the pod (and are schedulable, not allocate-once-and-used) are "matched": their
  reserve pod is removed from NodeInfo (restoreMatchedReservation :241-264).  Other reservations
  that already have assigned pods are "unmatched": the reserve pod's request is replaced by what
  is left of it, max(allocatable - allocated, 0) (restoreUnmatchedReservations :266-292,
  updateNodeInfoRequested :294-307).  podRequested is NodeInfo.Requested after the unmatched
  step; rAllocated = Σ matched Allocated.
* fits_node (plugin.go:445-496) and filter_with_reservations (plugin.go:377-440).
* nominate (nominator.go:134-192): reservations passing FilterReservation (plugin.go:503-530); the
  lowest non-zero order label wins (scoring.go:162-181), else the best ScoreReservation.
* score_reservation (scoring.go:183-203): MostAllocated over the non-zero allocatable resources.
* node scores (scoring.go:42-131): the node with the lowest order label scores 1000
  (mostPreferredScore), a node with a nominated reservation its ScoreReservation, others 0; then
  DefaultNormalizeScore(100) (frameworkext/normalize_score.go:24-52).

Canonical choices where the reference iterates Go maps or sorts unstably: reservations in list
order, nodes in list order, ties to the earlier entry.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional

DEFAULT_MILLI_CPU = 100            # schedutil.DefaultMilliCPURequest
DEFAULT_MEMORY = 200 * 1024 * 1024  # schedutil.DefaultMemoryRequest

ALIGNED, DEFAULT, RESTRICTED = "Aligned", "Default", "Restricted"


@dataclass
class Reservation:
    name: str
    allocatable: Dict[str, int]                 # ReservationRequests(r)
    allocated: Dict[str, int] = field(default_factory=dict)
    reserve_request: Optional[Dict[str, int]] = None  # reserve pod request in NodeInfo (default: allocatable)
    resource_names: Optional[List[str]] = None  # default: keys of allocatable (Restricted may narrow)
    policy: str = DEFAULT
    order: int = 0                              # label reservation-order (0 = none / invalid)
    owner_match: bool = True                    # MatchReservationOwners(pod, r.OwnerMatchers)
    available: bool = True
    unschedulable: bool = False
    allocate_once: bool = False
    assigned: int = 0

    def names(self):
        return list(self.resource_names) if self.resource_names is not None else list(self.allocatable)

    def rreq(self):
        return dict(self.reserve_request) if self.reserve_request is not None else dict(self.allocatable)


def _nonzero(req: Dict[str, int]):
    """schedutil.GetNonzeroRequests of one container's requests."""
    return (req["cpu"] if "cpu" in req else DEFAULT_MILLI_CPU,
            req["memory"] if "memory" in req else DEFAULT_MEMORY)


def _sub_nonneg(a: Dict[str, int], b: Dict[str, int]):
    """quotav1.SubtractWithNonNegativeResult"""
    out = {k: max(v - b.get(k, 0), 0) for k, v in a.items()}
    for k in b:
        out.setdefault(k, 0)
    return out


@dataclass
class NodeState:
    allocatable: Dict[str, int]
    allowed_pods: int
    requested: Dict[str, int]
    nonzero: Dict[str, int]   # {"cpu":, "memory":}
    pods: int


def eligible(r: Reservation) -> bool:
    return r.available and not (r.allocate_once and r.assigned > 0)


def restore(node: NodeState, reservations: List[Reservation], is_reserve_pod=False, has_affinity=False):
    """returns (effective NodeState, podRequested, rAllocated, matched) or None when skipped"""
    matched, unmatched = [], []
    for r in reservations:
        if not eligible(r):
            continue
        if not is_reserve_pod and not r.unschedulable and r.owner_match:
            matched.append(r)
        elif r.assigned > 0:
            unmatched.append(r)
    if not matched and not unmatched:
        return None
    if has_affinity and not matched:
        return None
    req = dict(node.requested)
    nz = dict(node.nonzero)
    pods = node.pods
    for r in unmatched:
        rq = r.rreq()
        for k, v in rq.items():
            req[k] = req.get(k, 0) - v
        c, m = _nonzero(rq)
        nz["cpu"] -= c
        nz["memory"] -= m
        rem = _sub_nonneg(r.allocatable, r.allocated)
        if any(v != 0 for v in rem.values()):
            for k, v in rem.items():
                req[k] = req.get(k, 0) + v
            c, m = _nonzero(rem)
            nz["cpu"] += c
            nz["memory"] += m
    pod_requested = dict(req)
    r_alloc: Dict[str, int] = {}
    for r in matched:
        rq = r.rreq()
        for k, v in rq.items():
            req[k] = req.get(k, 0) - v
        c, m = _nonzero(rq)
        nz["cpu"] -= c
        nz["memory"] -= m
        pods -= 1
        for k, v in r.allocated.items():
            r_alloc[k] = r_alloc.get(k, 0) + v
    eff = NodeState(node.allocatable, node.allowed_pods, req, nz, pods)
    return eff, pod_requested, r_alloc, matched


def fits_node(pod_req, node_alloc, allowed, pods_eff, n_matched, pod_requested, r_alloc, r: Optional[Reservation]):
    """plugin.go:445-496; returns the insufficient resource names"""
    out = []
    if pods_eff - n_matched + 1 > allowed:
        out.append("pods")
    scalars = [k for k in pod_req if k not in ("cpu", "memory", "ephemeral-storage")]
    if pod_req.get("cpu", 0) == 0 and pod_req.get("memory", 0) == 0 and pod_req.get("ephemeral-storage", 0) == 0 \
            and not scalars:
        return out
    rrem = {k: v - (r.allocated.get(k, 0)) for k, v in r.allocatable.items()} if r is not None else {}
    if r is not None:
        for k, v in r.allocated.items():
            rrem.setdefault(k, -v)
    for k in ["cpu", "memory", "ephemeral-storage"] + scalars:
        if pod_req.get(k, 0) > node_alloc.get(k, 0) - (pod_requested.get(k, 0) - rrem.get(k, 0) - r_alloc.get(k, 0)):
            out.append(k)
    return out


def restricted_fits(pod_req, r: Reservation):
    names = r.names()
    allocated = {k: v for k, v in r.allocated.items() if k in names}
    rrem = _sub_nonneg(r.allocatable, allocated)
    req = {k: v for k, v in pod_req.items() if k in names}
    bad = [k for k, v in rrem.items() if k in req and req[k] > v]
    return not bad, bad


def filter_with_reservations(pod_req, node_alloc, allowed, pods_eff, n_matched, pod_requested, r_alloc, rlist,
                             required):
    """plugin.go:377-440 -> (ok, reasons); n_matched = len(nodeRState.matched) of the node"""
    by_node, by_res = set(), set()
    for r in rlist:
        if not set(r.names()) & set(pod_req):
            continue
        ins = fits_node(pod_req, node_alloc, allowed, pods_eff, n_matched, pod_requested, r_alloc, r)
        if r.policy in (DEFAULT, ALIGNED):
            if not ins:
                return True, []
            by_node.update(ins)
        elif r.policy == RESTRICTED:
            ok, bad = restricted_fits(pod_req, r)
            if ok and not ins:
                return True, []
            by_node.update(ins)
            by_res.update(bad)
    if required:
        reasons = [f"Insufficient {x} by node" for x in sorted(by_node)] + \
                  [f"Insufficient {x} by reservation" for x in sorted(by_res)]
        return False, reasons or ["no reservations meet the requirement"]
    return True, []


def score_reservation(pod_req, r: Reservation, allocated=None):
    allocated = r.allocated if allocated is None else allocated
    requested = dict(pod_req)
    for k, v in allocated.items():
        requested[k] = requested.get(k, 0) + v
    resources = {k: v for k, v in r.allocatable.items() if v != 0}
    w = len(resources)
    if w <= 0:
        return 0
    s = 0
    for k, cap in resources.items():
        req = requested.get(k, 0)
        if req <= cap:
            # MilliValue() on both sides: cpu already milli, other resources x1000 (same floor)
            s += 100 * req // cap
    return s // w


def most_preferred_by_order(rs: List[Reservation]):
    best, order = None, None
    for r in rs:
        if r.order != 0 and (order is None or r.order < order):
            best, order = r, r.order
    return best, order


def nominate(pod_req, node_alloc, allowed, pods_eff, pod_requested, r_alloc, matched):
    cands = []
    for r in matched:
        if r.allocate_once and r.assigned > 0:
            continue
        ok, _ = filter_with_reservations(pod_req, node_alloc, allowed, pods_eff, len(matched), pod_requested, r_alloc,
                                         [r], True)
        if ok:
            cands.append(r)
    if not cands:
        return None
    by_order, _ = most_preferred_by_order(cands)
    if by_order is not None:
        return by_order
    best, bs = None, -1
    for r in cands:
        s = score_reservation(pod_req, r)
        if s > bs:
            best, bs = r, s
    return best


def default_normalize(scores: List[int], max_priority: int = 100) -> List[int]:
    m = max(scores) if scores else 0
    if m == 0:
        return list(scores)
    return [max_priority * s // m for s in scores]
