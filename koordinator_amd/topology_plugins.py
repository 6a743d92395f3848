"""Host side of the upstream PodTopologySpread and InterPodAffinity plugins (kube-scheduler v1.24.15
``plugins/podtopologyspread``, ``plugins/interpodaffinity``; the v1beta2 default profile enables both, weights 2 and
1, and appends them to every koord-scheduler profile through ``defaultprofile.AppendDefaultPlugins``).

Both plugins count *pods* per topology domain.  The label selector work -- which pods match which selector or affinity
term -- runs here, once per distinct selector / term, and reaches the device as (``include/koordgpu.h``
``ks_topology_args``):

* properties (<= KS_TOPO_MAX_PROPS): predicates on pods.  ``sel``: in namespace ns, not terminating, matching a spread
  constraint's selector (``countPodsMatchSelector``); ``term``: matching an affinity term (its namespaces and
  selector, ``AffinityTerm.Matches``); ``all``: matching every required affinity term of one pod
  (``podMatchesAllAffinityTerms``); ``carry``: carrying one required anti-affinity term, or hard / preferred
  (anti-)affinity terms identical up to their weights, with the summed score weight.  Every node holds, per property,
  the number of its pods that have it (``ks_node_cols.topo_count``, updated by every Reserve); every pod lists the
  properties it has (``ks_pod_cols.topo_props``, a CSR list).
* topology keys: key 0 is the hostname (every node is its own domain); every other label key a constraint or a term
  names is a key k >= 1 whose value index per node is ``ks_node_cols.topo_domain`` (-1 when the label is absent).
* per pod <= KS_TOPO_MAX_TERMS query terms (``ks_pod_cols.topo_terms``, a CSR list): what PreFilter / Filter / PreScore /
  Score of the two plugins ask of the counters -- spread constraints (hard and soft, the system default constraints
  included), required affinity / anti-affinity, the existing pods' anti-affinity terms that match the pod, and the score
  terms (the pod's preferred terms, the existing pods' hard and preferred terms that match it, with their weights).

A pod with no query term scores the constant 100 (PodTopologySpread's NormalizeScore with no constraint) and 0
(InterPodAffinity) everywhere and never fails their Filters; the others are *topology pods* (KS_TOPO_DYN) and the
device schedules each of them as the first pod of its pass.

``oracle/topology_ref.py`` restates both plugins directly on these objects; the tests check that both agree.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import abi
from .static_plugins import PodAffinitySpec, StaticPluginError

HOSTNAME = "kubernetes.io/hostname"
ZONE = "topology.kubernetes.io/zone"
DO_NOT_SCHEDULE = "DoNotSchedule"
SCHEDULE_ANYWAY = "ScheduleAnyway"
SELECTOR_OPS = ("In", "NotIn", "Exists", "DoesNotExist")


@dataclass(frozen=True)
class LabelSelector:
    """metav1.LabelSelector: matchLabels AND matchExpressions (In / NotIn / Exists / DoesNotExist)."""
    match_labels: Tuple[Tuple[str, str], ...] = ()
    match_expressions: Tuple[Tuple[str, str, Tuple[str, ...]], ...] = ()


@dataclass(frozen=True)
class SpreadConstraint:
    max_skew: int
    topology_key: str
    when_unsatisfiable: str = DO_NOT_SCHEDULE
    selector: Optional[LabelSelector] = None  # nil: matches nothing (LabelSelectorAsSelector(nil) = labels.Nothing())


@dataclass(frozen=True)
class AffinityTerm:
    """PodAffinityTerm: the pods of `namespaces` and of the namespaces `namespace_selector` selects (by the namespaces'
    labels) whose labels `selector` selects; neither given = the owning pod's namespace (getNamespacesFromPodAffinityTerm).
    A nil selector selects nothing, an empty one everything."""
    topology_key: str
    selector: Optional[LabelSelector] = None
    namespaces: Tuple[str, ...] = ()
    namespace_selector: Optional[LabelSelector] = None


@dataclass
class TopoPod:
    """The parts of a pod the two plugins read."""
    namespace: str = "default"
    labels: Dict[str, str] = field(default_factory=dict)
    terminating: bool = False  # DeletionTimestamp != nil (countPodsMatchSelector skips it)
    spread: List[SpreadConstraint] = field(default_factory=list)
    # the selector helper.DefaultSelector builds from the services / RCs / RSs / StatefulSets selecting the pod
    # (None = none: no system default constraints)
    default_selector: Optional[LabelSelector] = None
    affinity_required: List[AffinityTerm] = field(default_factory=list)
    affinity_preferred: List[Tuple[int, AffinityTerm]] = field(default_factory=list)
    anti_required: List[AffinityTerm] = field(default_factory=list)
    anti_preferred: List[Tuple[int, AffinityTerm]] = field(default_factory=list)
    node_affinity: Optional[PodAffinitySpec] = None  # nodeSelector / required node affinity (spreading eligibility)


# v1.24 podtopologyspread systemDefaultConstraints (plugins/podtopologyspread/plugin.go)
SYSTEM_DEFAULT_CONSTRAINTS = ((HOSTNAME, 3), (ZONE, 5))


def selector_matches(sel: Optional[LabelSelector], labels: Dict[str, str]) -> bool:
    """labels.Selector.Matches of LabelSelectorAsSelector(sel); nil matches nothing, an empty selector everything"""
    if sel is None:
        return False
    for k, v in sel.match_labels:
        if labels.get(k) != v:
            return False
    for k, op, vals in sel.match_expressions:
        has = k in labels
        if op == "In":
            if not has or labels[k] not in vals:
                return False
        elif op == "NotIn":
            if has and labels[k] in vals:
                return False
        elif op == "Exists":
            if not has:
                return False
        elif op == "DoesNotExist":
            if has:
                return False
        else:
            raise StaticPluginError(f"label selector operator {op!r}")
    return True


def term_namespaces(term: AffinityTerm, owner: TopoPod,
                    namespace_labels: Optional[Dict[str, Dict[str, str]]] = None) -> Tuple[str, ...]:
    """The namespaces whose pods the term can match: getNamespacesFromPodAffinityTerm (the term's namespaces, or the
    owner's when it lists none and has no namespaceSelector) plus the namespaces its namespaceSelector selects
    (AffinityTerm.Matches' NamespaceSelector.Matches(nsLabels) / mergeAffinityTermNamespacesIfNotEmpty), resolved over
    the namespace labels the shim's namespace lister holds"""
    if not term.namespaces and term.namespace_selector is None:
        return (owner.namespace,)
    out = set(term.namespaces)
    for ns, lab in (namespace_labels or {}).items():
        if selector_matches(term.namespace_selector, lab):
            out.add(ns)
    return tuple(sorted(out))


def term_matches(term: AffinityTerm, owner: TopoPod, pod: TopoPod,
                 namespace_labels: Optional[Dict[str, Dict[str, str]]] = None) -> bool:
    """AffinityTerm.Matches (framework/types.go): the pod's namespace among the term's and its labels selected"""
    return pod.namespace in term_namespaces(term, owner, namespace_labels) and selector_matches(term.selector, pod.labels)


def spread_constraints(pod: TopoPod, hard: bool) -> List[SpreadConstraint]:
    """filterTopologySpreadConstraints + the system defaults (buildDefaultConstraints) when the pod has none"""
    want = DO_NOT_SCHEDULE if hard else SCHEDULE_ANYWAY
    if pod.spread:
        return [c for c in pod.spread if c.when_unsatisfiable == want]
    if hard or pod.default_selector is None:
        return []
    sel = pod.default_selector
    if not sel.match_labels and not sel.match_expressions:
        return []  # an empty DefaultSelector: no default constraints
    return [SpreadConstraint(skew, key, SCHEDULE_ANYWAY, sel) for key, skew in SYSTEM_DEFAULT_CONSTRAINTS]


# ---- compilation to properties, counters and query terms ----

KIND = {"spread_hard": 1, "spread_soft": 2, "affinity": 3, "anti": 4, "existing_anti": 5, "score": 6}


@dataclass
class Compiled:
    props: List[tuple]                 # property identities, index = property
    keys: List[str]                    # topology keys, index = key (0 = the hostname)
    values: List[List[str]]            # per key >= 1: its label values, index = value index
    node_domain: np.ndarray            # [len(keys) - 1][n] int32 value index of key k + 1, -1 = absent
    node_count: np.ndarray             # [P][n] int32 pods with property p on node n
    pod_props: List[List[int]]         # per pending pod: its properties
    pod_terms: List[List[int]]         # per pending pod: its packed query terms
    pod_flags: np.ndarray              # [p] uint32 KS_TOPO_*

    @property
    def ndomains(self) -> int:
        return max([1] + [len(v) for v in self.values])

    def values_of(self, key: str) -> List[str]:
        return self.values[self.keys.index(key) - 1] if key in self.keys[1:] else []

    @property
    def zones(self) -> List[str]:
        return self.values_of(ZONE)


def _prop_has(prop: tuple, pod: TopoPod, hard_weight: int = 1, nsl=None) -> bool:
    kind = prop[0]
    if kind == "sel":  # countPodsMatchSelector: not terminating, same namespace, selector
        _, ns, sel = prop
        return not pod.terminating and pod.namespace == ns and selector_matches(sel, pod.labels)
    if kind == "term":
        _, nss, sel = prop
        return pod.namespace in nss and selector_matches(sel, pod.labels)
    if kind == "all":
        return all(pod.namespace in nss and selector_matches(sel, pod.labels) for nss, sel in prop[1])
    if kind == "carry":
        return prop in _carried(pod, hard_weight, nsl)
    raise AssertionError(prop)


def _carried(pod: TopoPod, hard_weight: int = 1, nsl=None) -> set:
    """The carry properties of a pod: its required anti-affinity terms, and per distinct (namespaces, selector,
    topologyKey) its hard / preferred (anti-)affinity terms' summed score weight (hard affinity terms weigh
    HardPodAffinityWeight, anti-affinity ones count negative).  processExistingPod adds every term's weight on its own;
    the sum per identical term is that total with one property bit per pod."""
    out = set()
    for t in pod.anti_required:
        out.add(("carry", "anti", term_namespaces(t, pod, nsl), t.selector, t.topology_key, 0))
    w_of: Dict[tuple, int] = {}
    order: List[tuple] = []

    def add(t: AffinityTerm, w: int):
        k = (term_namespaces(t, pod, nsl), t.selector, t.topology_key)
        if k not in w_of:
            w_of[k] = 0
            order.append(k)
        w_of[k] += w

    if hard_weight > 0:
        for t in pod.affinity_required:
            add(t, hard_weight)
    for w, t in pod.affinity_preferred:
        add(t, w)
    for w, t in pod.anti_preferred:
        add(t, -w)
    for k in order:
        if w_of[k] != 0:
            out.add(("carry", "score") + k + (w_of[k],))
    return out


def pack_term(kind: int, prop: int, key: int, param: int, flags: int = 0) -> int:
    """ks_pod_cols.topo_terms word: kind (bits 0-3), flags (4-7: KS_TOPO_T_*), topology key (8-15: 0 hostname, k >= 1
    ks_node_cols.topo_domain key k), property (16-31), param (32-63, int32: maxSkew or the score weight)"""
    assert 0 <= kind < 16 and 0 <= flags < 16 and 0 <= key < abi.KS_TOPO_MAX_KEYS and 0 <= prop < abi.KS_TOPO_MAX_PROPS
    return kind | (flags << 4) | (key << 8) | (prop << 16) | ((param & 0xFFFFFFFF) << 32)


def unpack_term(w: int) -> Tuple[int, int, int, int, int]:
    """(kind, prop, key, param, flags) of a packed term"""
    w = int(w)
    p = (w >> 32) & 0xFFFFFFFF
    return w & 0xF, (w >> 16) & 0xFFFF, (w >> 8) & 0xFF, p - (1 << 32) if p >= 1 << 31 else p, (w >> 4) & 0xF


def compile_topology(node_labels: Sequence[Dict[str, str]], existing: Sequence[Tuple[int, TopoPod]],
                     pending: Sequence[TopoPod], hard_weight: int = 1,
                     namespace_labels: Optional[Dict[str, Dict[str, str]]] = None) -> Compiled:
    """The properties, node counters and per-pod query terms of a cluster: node labels (every node has its hostname),
    the running pods as (node row, pod), the pending pods in queue order, the namespaces' labels (namespaceSelector).
    Topology keys: the hostname is key 0; every other key a constraint or an affinity term names gets an index in
    order of first use, its values a value index in node order.  Raises StaticPluginError for what the device does not model (too many keys / properties / terms)."""
    nsl = namespace_labels
    n = len(node_labels)
    keys: List[str] = [HOSTNAME]

    def key_index(k: str) -> int:
        if k not in keys:
            keys.append(k)
            if len(keys) > abi.KS_TOPO_MAX_KEYS:
                raise StaticPluginError(f"{len(keys)} topology keys (the device holds {abi.KS_TOPO_MAX_KEYS})")
        return keys.index(k)

    everyone = [p for _, p in existing] + list(pending)
    carried_all = set()
    for p in everyone:
        carried_all |= _carried(p, hard_weight, nsl)
    carried_sorted = sorted(carried_all, key=repr)
    props: List[tuple] = []
    prop_of: Dict[tuple, int] = {}

    def prop_index(pr: tuple) -> int:
        if pr not in prop_of:
            prop_of[pr] = len(props)
            props.append(pr)
            if len(props) > abi.KS_TOPO_MAX_PROPS:
                raise StaticPluginError(f"{len(props)} topology properties (the device holds {abi.KS_TOPO_MAX_PROPS})")
        return prop_of[pr]

    terms_per_pod: List[List[int]] = []
    flags = np.zeros(len(pending), np.uint32)
    for i, pod in enumerate(pending):
        terms: List[int] = []
        seen = set()
        for c in pod.spread:
            if (c.topology_key, c.when_unsatisfiable) in seen:
                # ValidateTopologySpreadConstraints: a duplicate {topologyKey, whenUnsatisfiable} pair is invalid
                raise StaticPluginError(f"pod {i}: duplicate spread constraint {c.topology_key}/{c.when_unsatisfiable}")
            seen.add((c.topology_key, c.when_unsatisfiable))
        hard = spread_constraints(pod, True)
        soft = spread_constraints(pod, False)
        for c in hard:
            pi = prop_index(("sel", pod.namespace, c.selector))
            self_match = abi.KS_TOPO_T_SELF if selector_matches(c.selector, pod.labels) else 0
            terms.append(pack_term(KIND["spread_hard"], pi, key_index(c.topology_key), c.max_skew, self_match))
        if soft and pod.spread:
            flags[i] |= abi.KS_TOPO_SOFT_ALL_KEYS  # requireAllTopologies: the pod's own constraints
        for c in soft:
            pi = prop_index(("sel", pod.namespace, c.selector))
            terms.append(pack_term(KIND["spread_soft"], pi, key_index(c.topology_key), c.max_skew))
        if pod.affinity_required:
            pi = prop_index(("all", tuple((term_namespaces(t, pod, nsl), t.selector) for t in pod.affinity_required)))
            for t in pod.affinity_required:
                terms.append(pack_term(KIND["affinity"], pi, key_index(t.topology_key), 0))
            if all(term_matches(t, pod, pod, nsl) for t in pod.affinity_required):
                flags[i] |= abi.KS_TOPO_SELF_AFFINITY
        for t in pod.anti_required:
            pi = prop_index(("term", term_namespaces(t, pod, nsl), t.selector))
            terms.append(pack_term(KIND["anti"], pi, key_index(t.topology_key), 0))
        for cp in carried_sorted:
            _, kind, nss, sel, key, w = cp
            if not (pod.namespace in nss and selector_matches(sel, pod.labels)):
                continue
            if kind == "anti":
                terms.append(pack_term(KIND["existing_anti"], prop_index(cp), key_index(key), 0))
            else:
                terms.append(pack_term(KIND["score"], prop_index(cp), key_index(key), w))
        for w, t in pod.affinity_preferred:
            terms.append(pack_term(KIND["score"], prop_index(("term", term_namespaces(t, pod, nsl), t.selector)),
                                   key_index(t.topology_key), w))
        for w, t in pod.anti_preferred:
            terms.append(pack_term(KIND["score"], prop_index(("term", term_namespaces(t, pod, nsl), t.selector)),
                                   key_index(t.topology_key), -w))
        if len(terms) > abi.KS_TOPO_MAX_TERMS:
            raise StaticPluginError(f"pod {i}: {len(terms)} topology terms (the device holds {abi.KS_TOPO_MAX_TERMS})")
        if terms:
            flags[i] |= abi.KS_TOPO_DYN
        terms_per_pod.append(terms)
    # every key's values in node order
    values: List[List[str]] = [[] for _ in keys[1:]]
    node_domain = np.full((len(keys) - 1, n), -1, np.int32)
    for k, key in enumerate(keys[1:]):
        idx: Dict[str, int] = {}
        for i, lab in enumerate(node_labels):
            if key in lab:
                v = lab[key]
                if v not in idx:
                    idx[v] = len(values[k])
                    values[k].append(v)
                node_domain[k, i] = idx[v]
    P = len(props)
    node_count = np.zeros((P, n), np.int32)
    for nd, pod in existing:
        for pi in _props_of(pod, props, hard_weight, nsl):
            node_count[pi, nd] += 1
    pod_props = [_props_of(pod, props, hard_weight, nsl) for pod in pending]
    return Compiled(props, keys, values, node_domain, node_count, pod_props, terms_per_pod, flags)


def _props_of(pod: TopoPod, props: List[tuple], hard_weight: int, nsl) -> List[int]:
    carried = _carried(pod, hard_weight, nsl)
    out = []
    for pi, pr in enumerate(props):
        if pr[0] == "carry":
            if pr in carried:
                out.append(pi)
        elif _prop_has(pr, pod, hard_weight, nsl):
            out.append(pi)
    return out


def install(c: Compiled, node_table, pod_table) -> None:
    """Write the compiled columns into the tables (ks_node_cols.topo_*, ks_pod_cols.topo_*)."""
    node_table.topo_domain = c.node_domain.copy()
    node_table.topo_count = c.node_count.copy()
    node_table.topo_ndomains = c.ndomains
    pod_table.topo_flags[:] = c.pod_flags
    pod_table.set_topo(c.pod_props, c.pod_terms)
