"""TEST INFRASTRUCTURE (oracle): a direct restatement of the upstream TaintToleration and NodeAffinity plugins on
taint / toleration / label objects, with no dictionaries and no bit masks.  Only tests/ use it, as the checker of
koordinator_amd/static_plugins.py (the host compiler) and of the C oracle's bit-mask evaluation
(oracle/koord_oracle.c static_filter / static_raw / static_normalize).

Upstream is kube-scheduler v1.24.15 (k8s.io/kubernetes, go.mod:276 of the reference), not on disk: parity unpinned.
Restated from its published source:
  plugins/tainttoleration/taint_toleration.go
    Filter   -- v1helper.FindMatchingUntoleratedTaint(node.Spec.Taints, pod.Spec.Tolerations,
                effect NoSchedule or NoExecute) found -> UnschedulableAndUnresolvable
    PreScore -- getAllTolerationPreferNoSchedule: tolerations with an empty effect or PreferNoSchedule
    Score    -- countIntolerableTaintsPreferNoSchedule: PreferNoSchedule taints none of those tolerates
    NormalizeScore -- helper.DefaultNormalizeScore(framework.MaxNodeScore, true, scores)
  plugins/nodeports/node_ports.go
    Filter   -- fitsPorts: HostPortInfo.CheckConflict(ip, protocol, port) for every wanted port (same protocol and
                port, and equal host IPs or either 0.0.0.0; ports <= 0 never conflict)
  plugins/nodeaffinity/node_affinity.go
    Filter   -- nodeaffinity.GetRequiredNodeAffinity(pod).Match(node): pod.Spec.NodeSelector AND (OR over the
                required NodeSelectorTerms; a term with no requirements matches nothing)
    Score    -- sum of the weights of the preferred terms that match (weight-0 terms dropped)
    NormalizeScore -- helper.DefaultNormalizeScore(framework.MaxNodeScore, false, scores)
DefaultNormalizeScore is also the reference's frameworkext/normalize_score.go:24-52.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

from koordinator_amd.static_plugins import (NO_EXECUTE, NO_SCHEDULE, PREFER_NO_SCHEDULE, NodeSpec, PodAffinitySpec,
                                            Requirement, requirement_matches)


def taint_filter(pod: PodAffinitySpec, node: NodeSpec) -> bool:
    for t in node.taints:
        if t.effect not in (NO_SCHEDULE, NO_EXECUTE):
            continue
        if not any(x.tolerates(t) for x in pod.tolerations):
            return False
    return True


def taint_raw(pod: PodAffinitySpec, node: NodeSpec) -> int:
    tols = [x for x in pod.tolerations if x.effect in ("", PREFER_NO_SCHEDULE)]
    return sum(1 for t in node.taints if t.effect == PREFER_NO_SCHEDULE and not any(x.tolerates(t) for x in tols))


def _term_match(reqs: List[Requirement], node: NodeSpec) -> bool:
    return bool(reqs) and all(requirement_matches(r, node) for r in reqs)


def affinity_filter(pod: PodAffinitySpec, node: NodeSpec) -> bool:
    if not all(node.labels.get(k) == v and k in node.labels for k, v in pod.node_selector.items()):
        return False
    if pod.required is None:
        return True
    return any(_term_match(list(t.requirements), node) for t in pod.required)


def affinity_raw(pod: PodAffinitySpec, node: NodeSpec) -> int:
    return sum(w for w, t in pod.preferred if w != 0 and _term_match(list(t.requirements), node))


def default_normalize(scores: Sequence[int], reverse: bool) -> List[int]:
    mx = max(scores, default=0)
    if mx == 0:
        return [100 if reverse else s for s in scores]
    out = []
    for s in scores:
        v = 100 * s // mx
        out.append(100 - v if reverse else v)
    return out


def ports_filter(pod: PodAffinitySpec, node: NodeSpec) -> bool:
    """upstream plugins/nodeports/node_ports.go fitsPorts: no wanted port conflicts with NodeInfo.UsedPorts"""
    return not any(w.conflicts(u) for w in pod.host_ports for u in node.used_ports)


def evaluate(pod: PodAffinitySpec, nodes: Sequence[NodeSpec], feasible_other: Sequence[bool]) -> Tuple[
        List[bool], List[int], List[int]]:
    """Per node: feasible (the other plugins' verdict AND both Filters) and the two normalized scores
    (0 on infeasible nodes)."""
    feas = [bool(f) and taint_filter(pod, n) and affinity_filter(pod, n) and ports_filter(pod, n)
            for f, n in zip(feasible_other, nodes)]
    idx = [i for i, f in enumerate(feas) if f]
    tn = default_normalize([taint_raw(pod, nodes[i]) for i in idx], True)
    an = default_normalize([affinity_raw(pod, nodes[i]) for i in idx], False)
    ts = [0] * len(nodes)
    as_ = [0] * len(nodes)
    for k, i in enumerate(idx):
        ts[i] = tn[k]
        as_[i] = an[k]
    return feas, ts, as_
