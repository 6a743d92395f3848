"""TEST INFRASTRUCTURE ONLY -- restatement of the upstream PodTopologySpread and InterPodAffinity plugins
(kube-scheduler v1.24.15 plugins/podtopologyspread, plugins/interpodaffinity) on pod / node objects, for one pod at a
time.  The upstream sources are not on disk (koordinator vendors kube-scheduler as a go.mod dependency,
k8s.io/kubernetes v1.24.15): parity is unpinned against reference fixtures; this file restates their published
algorithm in the plugins' own terms -- topology pairs, TpPairToMatchNum / critical paths, affinityCounts /
antiAffinityCounts / existingAntiAffinityCounts, topologyScore maps -- and the tests check the host compiler +
C oracle (counters and query terms) and the device against it.

It does not use koordinator_amd's matching code: label selectors, namespaces and the system default constraints are
restated here.  Objects: koordinator_amd.topology_plugins.TopoPod / SpreadConstraint / AffinityTerm / LabelSelector
(plain records); nodes are label dicts (the hostname label implied by the node index).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence, Tuple

HOSTNAME = "kubernetes.io/hostname"
MAX_NODE_SCORE = 100
MAX_INT32 = 2147483647


def _labels(node_labels: Dict[str, str], i: int) -> Dict[str, str]:
    d = dict(node_labels)
    d.setdefault(HOSTNAME, f"node-{i}")
    return d


def _selector_matches(sel, labels: Dict[str, str]) -> bool:
    """metav1.LabelSelectorAsSelector(sel).Matches(labels): nil selects nothing, {} everything"""
    if sel is None:
        return False
    for k, v in sel.match_labels:
        if k not in labels or labels[k] != v:
            return False
    for k, op, vals in sel.match_expressions:
        if op == "In" and not (k in labels and labels[k] in vals):
            return False
        if op == "NotIn" and (k in labels and labels[k] in vals):
            return False
        if op == "Exists" and k not in labels:
            return False
        if op == "DoesNotExist" and k in labels:
            return False
    return True


def _term_matches(term, owner, pod, ns_labels) -> bool:
    """framework.AffinityTerm.Matches(pod, nsLabels): Namespaces.Has(pod.Namespace) || NamespaceSelector.Matches(the
    pod namespace's labels), then the term's selector; Namespaces = getNamespacesFromPodAffinityTerm (the owner's
    namespace when the term lists none and has no namespaceSelector); a nil namespaceSelector selects nothing"""
    nss = term.namespaces if (term.namespaces or term.namespace_selector is not None) else (owner.namespace,)
    ns_ok = pod.namespace in nss or _selector_matches(term.namespace_selector, ns_labels.get(pod.namespace, {}))
    return ns_ok and _selector_matches(term.selector, pod.labels)


def _node_affinity_match(pod, i: int, node_aff) -> bool:
    """nodeaffinity.GetRequiredNodeAffinity(pod).Match(node i) through the test's hook (a callable on the node index)"""
    return node_aff is None or bool(node_aff(i))


def _constraints(pod, want: str):
    """filterTopologySpreadConstraints / buildDefaultConstraints (systemDefaulted: hostname 3, zone 5)"""
    if pod.spread:
        return [c for c in pod.spread if c.when_unsatisfiable == want]
    if want == "DoNotSchedule" or pod.default_selector is None:
        return []
    sel = pod.default_selector
    if not sel.match_labels and not sel.match_expressions:
        return []

    class C:  # a system default constraint
        pass

    out = []
    for key, skew in ((HOSTNAME, 3), ("topology.kubernetes.io/zone", 5)):
        c = C()
        c.max_skew, c.topology_key, c.when_unsatisfiable, c.selector = skew, key, "ScheduleAnyway", sel
        out.append(c)
    return out


def _count_match(pods_on_node, sel, ns) -> int:
    """countPodsMatchSelector: terminating pods and other namespaces skipped"""
    return sum(1 for p in pods_on_node if not p.terminating and p.namespace == ns and _selector_matches(sel, p.labels))


def evaluate(pod, nodes: Sequence[Dict[str, str]], existing: Sequence[Tuple[int, object]], feasible_other: Sequence[bool],
             spread_weight: int = 2, affinity_weight: int = 1, hard_weight: int = 1, node_aff=None, ns_labels=None):
    """One pod against the cluster: returns (pts_fail[n], ipa_fail[n] in {None, "affinity", "anti", "existing"},
    pts_norm[n], ipa_norm[n], totals_add[n]) where the scores are over the nodes feasible for every Filter
    (feasible_other and both plugins' Filters); node_aff(i) -> bool is the pod's required node affinity on node i."""
    N = len(nodes)
    nsl = ns_labels or {}
    labels = [_labels(nodes[i], i) for i in range(N)]
    on_node: List[List[object]] = [[] for _ in range(N)]
    for nd, p in existing:
        on_node[nd].append(p)

    # ---- PodTopologySpread PreFilter (calPreFilterState) + Filter ----
    hard = _constraints(pod, "DoNotSchedule")
    pair_match: Dict[Tuple[str, str], int] = {}
    crit: Dict[str, int] = {c.topology_key: MAX_INT32 for c in hard}
    if hard:
        for i in range(N):
            if not _node_affinity_match(pod, i, node_aff):
                continue
            if not all(c.topology_key in labels[i] for c in hard):
                continue
            for c in hard:
                pair = (c.topology_key, labels[i][c.topology_key])
                pair_match[pair] = pair_match.get(pair, 0) + _count_match(on_node[i], c.selector, pod.namespace)
        for (k, v), cnt in pair_match.items():
            if k in crit:
                crit[k] = min(crit[k], cnt)
    pts_fail = [False] * N
    for i in range(N):
        for c in hard:
            if c.topology_key not in labels[i]:
                pts_fail[i] = True
                break
            self_match = 1 if _selector_matches(c.selector, pod.labels) else 0
            match = pair_match.get((c.topology_key, labels[i][c.topology_key]), 0)
            if match + self_match - crit[c.topology_key] > c.max_skew:
                pts_fail[i] = True
                break

    # ---- InterPodAffinity PreFilter + Filter ----
    aff_counts: Dict[Tuple[str, str], int] = {}
    anti_counts: Dict[Tuple[str, str], int] = {}
    exist_anti: Dict[Tuple[str, str], int] = {}
    for i in range(N):
        for ep in on_node[i]:
            # getExistingAntiAffinityCounts: the placed pods' required anti-affinity terms that match the pod
            for t in ep.anti_required:
                if _term_matches(t, ep, pod, nsl) and t.topology_key in labels[i]:
                    pr = (t.topology_key, labels[i][t.topology_key])
                    exist_anti[pr] = exist_anti.get(pr, 0) + 1
            # getIncomingAffinityAntiAffinityCounts
            if pod.affinity_required and all(_term_matches(t, pod, ep, nsl) for t in pod.affinity_required):
                for t in pod.affinity_required:
                    if t.topology_key in labels[i]:
                        pr = (t.topology_key, labels[i][t.topology_key])
                        aff_counts[pr] = aff_counts.get(pr, 0) + 1
            for t in pod.anti_required:
                if _term_matches(t, pod, ep, nsl) and t.topology_key in labels[i]:
                    pr = (t.topology_key, labels[i][t.topology_key])
                    anti_counts[pr] = anti_counts.get(pr, 0) + 1
    aff_counts = {k: v for k, v in aff_counts.items() if v != 0}
    self_all = bool(pod.affinity_required) and all(_term_matches(t, pod, pod, nsl) for t in pod.affinity_required)
    ipa_fail: List[Optional[str]] = [None] * N
    for i in range(N):
        ok = True
        exist = True
        for t in pod.affinity_required:
            if t.topology_key in labels[i]:
                if aff_counts.get((t.topology_key, labels[i][t.topology_key]), 0) <= 0:
                    exist = False
            else:
                ok = False
                break
        if ok and not exist:
            ok = len(aff_counts) == 0 and self_all
        if not ok:
            ipa_fail[i] = "affinity"
            continue
        if anti_counts and any(t.topology_key in labels[i] and
                               anti_counts.get((t.topology_key, labels[i][t.topology_key]), 0) > 0
                               for t in pod.anti_required):
            ipa_fail[i] = "anti"
            continue
        if exist_anti and any(exist_anti.get((k, v), 0) > 0 for k, v in labels[i].items()):
            ipa_fail[i] = "existing"
    feasible = [bool(feasible_other[i]) and not pts_fail[i] and ipa_fail[i] is None for i in range(N)]
    fidx = [i for i in range(N) if feasible[i]]

    # ---- PodTopologySpread PreScore / Score / NormalizeScore ----
    soft = _constraints(pod, "ScheduleAnyway")
    pts_norm = [0] * N
    if soft:
        require_all = bool(pod.spread)
        ignored = set()
        pair_counts: Dict[Tuple[str, str], int] = {}
        topo_size = [0] * len(soft)
        for i in fidx:
            if require_all and not all(c.topology_key in labels[i] for c in soft):
                ignored.add(i)
                continue
            for k, c in enumerate(soft):
                if c.topology_key == HOSTNAME:
                    continue
                pair = (c.topology_key, labels[i].get(c.topology_key, ""))
                if pair not in pair_counts:
                    pair_counts[pair] = 0
                    topo_size[k] += 1
        weights = []
        for k, c in enumerate(soft):
            sz = topo_size[k]
            if c.topology_key == HOSTNAME:
                sz = len(fidx) - len(ignored)
            weights.append(math.log(float(sz + 2)))
        for i in range(N):
            if not _node_affinity_match(pod, i, node_aff):
                continue
            if require_all and not all(c.topology_key in labels[i] for c in soft):
                continue
            for c in soft:
                pair = (c.topology_key, labels[i].get(c.topology_key, ""))
                if pair in pair_counts:
                    pair_counts[pair] += _count_match(on_node[i], c.selector, pod.namespace)
        raw = {}
        for i in fidx:
            if i in ignored:
                raw[i] = 0
                continue
            score = 0.0
            for k, c in enumerate(soft):
                if c.topology_key in labels[i]:
                    if c.topology_key == HOSTNAME:
                        cnt = _count_match(on_node[i], c.selector, pod.namespace)
                    else:
                        cnt = pair_counts[(c.topology_key, labels[i][c.topology_key])]
                    score += float(cnt) * weights[k] + float(c.max_skew - 1)
            raw[i] = int(_go_round(score))
        mn, mx = None, 0
        for i in fidx:
            if i in ignored:
                continue
            mn = raw[i] if mn is None or raw[i] < mn else mn
            mx = max(mx, raw[i])
        for i in fidx:
            if i in ignored:
                pts_norm[i] = 0
            elif mx == 0:
                pts_norm[i] = MAX_NODE_SCORE
            else:
                pts_norm[i] = MAX_NODE_SCORE * (mx + mn - raw[i]) // mx
    else:
        for i in fidx:
            pts_norm[i] = MAX_NODE_SCORE

    # ---- InterPodAffinity PreScore / Score / NormalizeScore ----
    topo_score: Dict[str, Dict[str, int]] = {}

    def process(term, weight, check_pod, owner, node_i, mult):
        if _term_matches(term, owner, check_pod, nsl) and term.topology_key in labels[node_i]:
            m = topo_score.setdefault(term.topology_key, {})
            v = labels[node_i][term.topology_key]
            m[v] = m.get(v, 0) + weight * mult

    for i in range(N):
        for ep in on_node[i]:
            for w, t in pod.affinity_preferred:
                process(t, w, ep, pod, i, 1)
            for w, t in pod.anti_preferred:
                process(t, w, ep, pod, i, -1)
            if hard_weight > 0:
                for t in ep.affinity_required:
                    process(t, hard_weight, pod, ep, i, 1)
            for w, t in ep.affinity_preferred:
                process(t, w, pod, ep, i, 1)
            for w, t in ep.anti_preferred:
                process(t, w, pod, ep, i, -1)
    ipa_raw = {}
    for i in fidx:
        s = 0
        for k, m in topo_score.items():
            if k in labels[i]:
                s += m.get(labels[i][k], 0)
        ipa_raw[i] = s
    ipa_norm = [0] * N
    if topo_score:
        mx = max([0] + [ipa_raw[i] for i in fidx])
        mn = min([0] + [ipa_raw[i] for i in fidx])
        diff = mx - mn
        for i in fidx:
            ipa_norm[i] = int(float(MAX_NODE_SCORE) * (float(ipa_raw[i] - mn) / float(diff))) if diff > 0 else 0
    add = [pts_norm[i] * spread_weight + ipa_norm[i] * affinity_weight if feasible[i] else None for i in range(N)]
    return pts_fail, ipa_fail, pts_norm, ipa_norm, add


def _go_round(x: float) -> float:
    """math.Round: half away from zero"""
    a = abs(x)
    r = math.floor(a)
    if a - r >= 0.5:  # exact: a - floor(a) is representable
        r += 1
    return r if x >= 0 else -r
