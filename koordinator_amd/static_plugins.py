"""Host side of the upstream TaintToleration and NodeAffinity plugins (kube-scheduler v1.24.15
``plugins/tainttoleration``, ``plugins/nodeaffinity``; the v1beta2 default profile enables both with weight 1).

The string matching -- tolerations against taints, label selector requirements against node labels -- runs here,
once per distinct taint and once per distinct requirement, and reaches the device as 64-bit masks over two
dictionaries (``include/koordgpu.h`` ``ks_static_plugin_args``):

* taint dictionary: the distinct (key, value, effect) taints of the nodes; a node carries ``taints_hard`` (effects
  NoSchedule / NoExecute) and ``taints_soft`` (PreferNoSchedule); a pod carries ``tolerated`` = the taints some of
  its tolerations tolerate (``Toleration.ToleratesTaint``).
* label dictionary: the distinct node selector requirements of the pods (``nodeSelector`` entries become
  ``key In [value]``, ``matchFields`` on ``metadata.name`` are requirements on the node name); a node carries
  ``labels`` = the requirements it satisfies; a pod carries its required terms (the nodeSelector requirements ANDed
  into each) and preferred terms as requirement masks.  An empty term matches nothing (``KS_LABEL_NEVER``).

This is what the Go cgo shim does at informer time ("Taints and node affinity").  The per-(pod, node)
Filter and Score then run on the device (``ks_device.h`` ``stat_eval``).  ``oracle/static_plugins_ref.py`` restates
the plugins directly on these objects; the tests check that both agree.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import abi
from .cluster import NodeTable, PodTable

NO_SCHEDULE = "NoSchedule"
PREFER_NO_SCHEDULE = "PreferNoSchedule"
NO_EXECUTE = "NoExecute"
EFFECTS = (NO_SCHEDULE, PREFER_NO_SCHEDULE, NO_EXECUTE)
OPERATORS = ("In", "NotIn", "Exists", "DoesNotExist", "Gt", "Lt")
FIELD_NAME = "metadata.name"


class StaticPluginError(ValueError):
    """A cluster the dictionaries cannot represent (the shim keeps the reference path for it)."""


@dataclass(frozen=True)
class Taint:
    key: str
    value: str = ""
    effect: str = NO_SCHEDULE


@dataclass(frozen=True)
class Toleration:
    key: str = ""
    operator: str = "Equal"  # "Equal" (or "") / "Exists"
    value: str = ""
    effect: str = ""         # "" = every effect

    def tolerates(self, t: Taint) -> bool:
        """core/v1 Toleration.ToleratesTaint (k8s.io/api/core/v1/toleration.go)."""
        if self.effect and self.effect != t.effect:
            return False
        if self.key and self.key != t.key:
            return False
        if self.operator in ("", "Equal"):
            return self.value == t.value
        if self.operator == "Exists":
            return True
        return False


@dataclass(frozen=True)
class Requirement:
    """One NodeSelectorRequirement (matchExpressions) or, with field=True, a matchFields requirement."""
    key: str
    operator: str
    values: Tuple[str, ...] = ()
    field: bool = False


@dataclass
class Term:
    """NodeSelectorTerm: every requirement must hold; a term without requirements matches nothing."""
    requirements: List[Requirement] = field(default_factory=list)


@dataclass(frozen=True)
class HostPort:
    """A container port with a host port (framework.HostPortInfo entry); sanitized like HostPortInfo.sanitize:
    empty host IP -> 0.0.0.0, empty protocol -> TCP."""
    port: int
    protocol: str = "TCP"
    host_ip: str = "0.0.0.0"

    def sanitized(self) -> "HostPort":
        return HostPort(self.port, self.protocol or "TCP", self.host_ip or "0.0.0.0")

    def conflicts(self, other: "HostPort") -> bool:
        """HostPortInfo.CheckConflict for one used entry: same protocol and port, and equal IPs or either 0.0.0.0"""
        a, b = self.sanitized(), other.sanitized()
        if a.port <= 0 or b.port <= 0 or a.protocol != b.protocol or a.port != b.port:
            return False
        return a.host_ip == b.host_ip or a.host_ip == "0.0.0.0" or b.host_ip == "0.0.0.0"


@dataclass
class PodAffinitySpec:
    tolerations: List[Toleration] = field(default_factory=list)
    node_selector: Dict[str, str] = field(default_factory=dict)
    required: Optional[List[Term]] = None             # requiredDuringSchedulingIgnoredDuringExecution terms
    preferred: List[Tuple[int, Term]] = field(default_factory=list)  # (weight, preference)
    host_ports: List[HostPort] = field(default_factory=list)          # NodePorts: the containers' host ports


@dataclass
class NodeSpec:
    name: str
    labels: Dict[str, str] = field(default_factory=dict)
    taints: List[Taint] = field(default_factory=list)
    used_ports: List[HostPort] = field(default_factory=list)         # NodeInfo.UsedPorts of the running pods


def _parse_int(v: str) -> Optional[int]:
    """strconv.ParseInt(v, 10, 64)"""
    try:
        if not v or v.strip() != v or "_" in v:
            return None
        x = int(v, 10)
    except ValueError:
        return None
    return x if -(1 << 63) <= x < (1 << 63) else None


def validate_requirement(r: Requirement) -> None:
    if r.field:
        if r.key != FIELD_NAME or r.operator not in ("In", "NotIn") or len(r.values) != 1:
            # nodeaffinity v1.24: matchFields support metadata.name with In / NotIn and exactly one value
            raise StaticPluginError(f"unsupported matchFields requirement {r}")
        return
    if r.operator not in OPERATORS:
        raise StaticPluginError(f"unsupported operator {r.operator}")
    if r.operator in ("In", "NotIn") and not r.values:
        raise StaticPluginError(f"{r.operator} needs values: {r}")
    if r.operator in ("Exists", "DoesNotExist") and r.values:
        raise StaticPluginError(f"{r.operator} takes no values: {r}")
    if r.operator in ("Gt", "Lt") and (len(r.values) != 1 or _parse_int(r.values[0]) is None):
        raise StaticPluginError(f"{r.operator} needs one integer value: {r}")


def requirement_matches(r: Requirement, node: NodeSpec) -> bool:
    """labels.Requirement.Matches (apimachinery labels/selector.go) / the metadata.name field selector."""
    if r.field:
        hit = node.name in r.values
        return hit if r.operator == "In" else not hit
    has = r.key in node.labels
    v = node.labels.get(r.key, "")
    if r.operator == "In":
        return has and v in r.values
    if r.operator == "NotIn":
        return not has or v not in r.values
    if r.operator == "Exists":
        return has
    if r.operator == "DoesNotExist":
        return not has
    if not has:
        return False
    x = _parse_int(v)
    if x is None:
        return False
    y = _parse_int(r.values[0])
    return x > y if r.operator == "Gt" else x < y


def _term_reqs(pod: PodAffinitySpec, term: Optional[Term]) -> List[Requirement]:
    sel = [Requirement(k, "In", (v,)) for k, v in sorted(pod.node_selector.items())]
    return sel + (list(term.requirements) if term is not None else [])


@dataclass
class Dictionaries:
    taints: List[Taint]
    requirements: List[Requirement]
    ports: List[HostPort] = field(default_factory=list)


def build_dictionaries(nodes: Sequence[NodeSpec], pods: Sequence[PodAffinitySpec]) -> Dictionaries:
    taints: Dict[Taint, int] = {}
    for nd in nodes:
        for t in nd.taints:
            if t.effect not in EFFECTS:
                raise StaticPluginError(f"node {nd.name}: taint effect {t.effect}")
            taints.setdefault(t, len(taints))
    if len(taints) > 64:
        raise StaticPluginError(f"{len(taints)} distinct taints (the device dictionary holds 64)")
    reqs: Dict[Requirement, int] = {}
    for p in pods:
        lists: List[List[Requirement]] = []
        if p.required is not None:
            lists += [_term_reqs(p, t) for t in p.required]
        elif p.node_selector:
            lists.append(_term_reqs(p, None))
        lists += [list(t.requirements) for w, t in p.preferred if w != 0]  # (nodeSelector is not part of these)
        for rl in lists:
            for r in rl:
                validate_requirement(r)
                reqs.setdefault(r, len(reqs))
    if len(reqs) > 63:
        raise StaticPluginError(f"{len(reqs)} distinct node selector requirements (the device dictionary holds 63)")
    ports: Dict[HostPort, int] = {}
    for hp in [h for nd in nodes for h in nd.used_ports] + [h for p in pods for h in p.host_ports]:
        hp = hp.sanitized()
        if hp.port > 0:
            ports.setdefault(hp, len(ports))
    if len(ports) > 64:
        raise StaticPluginError(f"{len(ports)} distinct host ports (the device dictionary holds 64)")
    return Dictionaries(list(taints), list(reqs), list(ports))


def _lookup(index: Dict, item, what: str) -> int:
    """The dictionary bit of `item`; an item the prebuilt dictionaries do not hold (the informer path keeps them across
    cycles) means they must be rebuilt, which the shim handles like every other StaticPluginError (reference path)."""
    k = index.get(item)
    if k is None:
        raise StaticPluginError(f"{what} {item} not in dictionary: rebuild the dictionaries")
    return k


def _mask(reqs: List[Requirement], index: Dict[Requirement, int]) -> int:
    m = 0
    for r in reqs:
        m |= 1 << _lookup(index, r, "node selector requirement")
    return m


def compile_cluster(nodes: Sequence[NodeSpec], pods: Sequence[PodAffinitySpec], node_table: NodeTable,
                    pod_table: PodTable, dicts: Optional[Dictionaries] = None) -> Dictionaries:
    """Fill node_table.{taints_hard, taints_soft, labels} and pod_table.{tolerated, affinity_*} from the specs."""
    if len(nodes) != node_table.n or len(pods) != pod_table.n:
        raise ValueError("spec / table length mismatch")
    if dicts is not None:
        # the pods' requirements are validated here too (build_dictionaries does it for new dictionaries)
        for p in pods:
            for rl in ([_term_reqs(p, t) for t in p.required] if p.required is not None else
                       ([_term_reqs(p, None)] if p.node_selector else [])) + [list(t.requirements) for w, t in p.preferred if w != 0]:
                for r in rl:
                    validate_requirement(r)
    d = dicts or build_dictionaries(nodes, pods)
    tindex = {t: i for i, t in enumerate(d.taints)}
    rindex = {r: i for i, r in enumerate(d.requirements)}
    hard = np.zeros(len(nodes), np.uint64)
    soft = np.zeros(len(nodes), np.uint64)
    labels = np.zeros(len(nodes), np.uint64)
    for i, nd in enumerate(nodes):
        h = s = 0
        for t in nd.taints:
            b = 1 << _lookup(tindex, t, "taint")
            if t.effect == PREFER_NO_SCHEDULE:
                s |= b
            else:
                h |= b
        lab = 0
        for r, k in rindex.items():
            if requirement_matches(r, nd):
                lab |= 1 << k
        hard[i], soft[i], labels[i] = h, s, lab
    node_table.taints_hard = hard
    node_table.taints_soft = soft
    node_table.labels = labels
    pindex = {hp: i for i, hp in enumerate(d.ports)}
    used = np.zeros(len(nodes), np.uint64)
    for i, nd in enumerate(nodes):
        m = 0
        for hp in nd.used_ports:
            hp = hp.sanitized()
            if hp.port > 0:
                m |= 1 << _lookup(pindex, hp, "host port")
        used[i] = m
    node_table.host_ports = used
    T = abi.KS_AFFINITY_TERMS
    tol = np.zeros(len(pods), np.uint64)
    nreq = np.zeros(len(pods), np.int32)
    req = np.zeros((T, len(pods)), np.uint64)
    pref = np.zeros((T, len(pods)), np.uint64)
    wt = np.zeros((T, len(pods)), np.int32)
    never = abi.KS_LABEL_NEVER
    for i, p in enumerate(pods):
        m = 0
        for k, t in enumerate(d.taints):
            if any(x.tolerates(t) for x in p.tolerations):
                m |= 1 << k
        tol[i] = m
        if p.required is not None:
            terms = list(p.required)
            if len(terms) > T:
                raise StaticPluginError(f"pod {i}: {len(terms)} required terms (the device evaluates {T})")
            if not terms:
                # NodeSelector with no terms matches nothing
                nreq[i] = 1
                req[0, i] = never
            else:
                nreq[i] = len(terms)
                for k, t in enumerate(terms):
                    req[k, i] = _mask(_term_reqs(p, t), rindex) if t.requirements else never
        elif p.node_selector:
            nreq[i] = 1
            req[0, i] = _mask(_term_reqs(p, None), rindex)
        prefs = [(w, t) for w, t in p.preferred if w != 0]
        if len(prefs) > T:
            raise StaticPluginError(f"pod {i}: {len(prefs)} preferred terms (the device evaluates {T})")
        for k, (w, t) in enumerate(prefs):
            if not 1 <= w <= 100:
                raise StaticPluginError(f"pod {i}: preferred weight {w} outside [1, 100]")
            # upstream component-helpers nodeaffinity.NewPreferredSchedulingTerms (k8s v1.24.15, not on disk) skips a term
            # with weight 0 or an empty preference (isEmptyNodeSelectorTerm: no matchExpressions and no matchFields);
            # an empty term compiled to KS_LABEL_NEVER never matches, so it adds 0 like a skipped one
            pref[k, i] = _mask(list(t.requirements), rindex) if t.requirements else never
            wt[k, i] = w
    want = np.zeros(len(pods), np.uint64)
    conf = np.zeros(len(pods), np.uint64)
    for i, p in enumerate(pods):
        w = c = 0
        for hp in p.host_ports:
            hp = hp.sanitized()
            if hp.port <= 0:
                continue
            w |= 1 << _lookup(pindex, hp, "host port")
            for k, q in enumerate(d.ports):
                if hp.conflicts(q):
                    c |= 1 << k
        want[i], conf[i] = w, c
    pod_table.host_ports = want
    pod_table.host_ports_conflict = conf
    pod_table.tolerated = tol
    pod_table.affinity_required_n = nreq
    pod_table.affinity_required = req
    pod_table.affinity_preferred = pref
    pod_table.affinity_weight = wt
    return d
