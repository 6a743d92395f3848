"""Upstream PodTopologySpread and InterPodAffinity (kube-scheduler v1.24.15 plugins/podtopologyspread,
plugins/interpodaffinity; not on disk -- a go.mod dependency of the reference -- so parity is unpinned against
reference fixtures).  CPU only:
  * hand-worked cases of the host compiler (koordinator_amd/topology_plugins.py: properties, counters, query terms,
    system default constraints, refusals);
  * the C oracle's evaluation of the compiled form against oracle/topology_ref.py, which restates both plugins on the
    pod objects (topology pairs, critical paths, affinity / anti-affinity counts, topologyScore maps): per-node Filter
    verdicts, normalized scores and totals, alone, with node affinity, and next to NodeResourcesFit;
  * whole queues: ko_schedule against a sequential loop over the restatement (each placed pod joins the running pods
    of its node), and the counters ks_read_nodes reports after it."""
import copy

import numpy as np
import pytest

from koordinator_amd import abi, synth
from koordinator_amd.config import SchedulerProfile
from koordinator_amd.static_plugins import StaticPluginError
from koordinator_amd.topology_plugins import (DO_NOT_SCHEDULE, HOSTNAME, KIND, SCHEDULE_ANYWAY, ZONE, AffinityTerm,
                                              LabelSelector, SpreadConstraint, TopoPod, compile_topology, install,
                                              unpack_term)
from oracle import topology_ref as ref
from oracle.oracle import Oracle

IPA_BITS = {"affinity": abi.KS_R_POD_AFFINITY, "anti": abi.KS_R_POD_ANTI_AFFINITY,
            "existing": abi.KS_R_EXISTING_ANTI_AFFINITY}


def _profile(fit=False, static=False):
    kw = dict(topology=True, topology_spread_weight=2, inter_pod_affinity_weight=1, loadaware=None)
    if not fit:
        kw["fit"] = None
    if static:
        kw.update(node_affinity=True, node_affinity_weight=1)
    return SchedulerProfile(**kw)


def _workload(n_nodes, n_pods, seed, static=False, **kw):
    w = synth.c1(n_nodes=n_nodes, n_pods=n_pods)
    if static:
        w = synth.with_static_plugins(w, seed=seed + 100)
    return synth.with_topology(w, seed=seed, **kw)


def _node_aff(w, i):
    if not hasattr(w, "specs"):
        return None
    from oracle import static_plugins_ref as sref
    nspec, pspec = w.specs
    return lambda n: sref.affinity_filter(pspec[i], nspec[n])


def _check_eval(w, profile, pods, base_profile=None, other_fn=None):
    node_labels, existing, pending = w.topo
    orc = Oracle(profile.to_ks_config(), w.nodes.copy())
    base = Oracle(base_profile.to_ks_config(), w.nodes.copy()) if base_profile else None
    try:
        for i in pods:
            one = w.pods.rows([i])
            r, s, t = orc.eval_pod(one)
            other = [True] * w.nodes.n if other_fn is None else [other_fn(i, n) for n in range(w.nodes.n)]
            bt = None
            if base is not None:
                rb, sb, bt = base.eval_pod(one)
                other = list(rb == 0)
            pf, ipf, pn, inn, add = ref.evaluate(pending[i], node_labels, existing, other, node_aff=_node_aff(w, i),
                                                 ns_labels=synth.TOPO_NAMESPACE_LABELS)
            for n in range(w.nodes.n):
                assert bool(r[n] & abi.KS_R_TOPOLOGY_SPREAD) == pf[n], f"pod {i} node {n}: spread filter"
                want = IPA_BITS.get(ipf[n], 0)
                got = int(r[n]) & (abi.KS_R_POD_AFFINITY | abi.KS_R_POD_ANTI_AFFINITY | abi.KS_R_EXISTING_ANTI_AFFINITY)
                assert got == want, f"pod {i} node {n}: inter-pod affinity filter {got:#x} vs {ipf[n]}"
            assert list(s[:, abi.KS_SCORE_TOPOLOGY_SPREAD]) == pn, f"pod {i}: spread scores"
            assert list(s[:, abi.KS_SCORE_POD_AFFINITY]) == inn, f"pod {i}: inter-pod affinity scores"
            if base is None and other_fn is None:
                assert list(t) == [a if a is not None else -1 for a in add], f"pod {i}: totals"
    finally:
        orc.close()
        if base is not None:
            base.close()


def test_compile_hand_cases():
    sel_a = LabelSelector((("app", "a"),))
    nodes = [{ZONE: "z1"}, {ZONE: "z1"}, {ZONE: "z2"}, {}]
    existing = [(0, TopoPod(labels={"app": "a"})), (0, TopoPod(labels={"app": "a"}, terminating=True)),
                (2, TopoPod(labels={"app": "a"}, anti_required=[AffinityTerm(HOSTNAME, sel_a)]))]
    pending = [
        TopoPod(labels={"app": "a"}, spread=[SpreadConstraint(1, ZONE, DO_NOT_SCHEDULE, sel_a)]),
        TopoPod(labels={"app": "b"}),                                        # nothing: not a topology pod
        TopoPod(labels={"app": "b"}, default_selector=sel_a),                # system defaults: two soft terms
        TopoPod(labels={"app": "a"}),                                        # matches the running anti term
        TopoPod(namespace="x", labels={"app": "a"}),                         # other namespace: does not
    ]
    c = compile_topology(nodes, existing, pending)
    assert c.keys[0] == HOSTNAME and list(c.node_domain[c.keys.index(ZONE) - 1]) == [0, 0, 1, -1]
    kinds = [[unpack_term(w)[0] for w in c.pod_terms[i]] for i in range(len(pending))]
    # (pod 0 is app=a in namespace default too: the running pod's anti-affinity term applies to it)
    assert kinds[0] == [KIND["spread_hard"], KIND["existing_anti"]] and kinds[1] == [] and kinds[2] == [KIND["spread_soft"]] * 2
    assert kinds[3] == [KIND["existing_anti"]] and kinds[4] == []
    assert [bool(f & abi.KS_TOPO_DYN) for f in c.pod_flags] == [True, False, True, True, False]
    # the selector property of pod 0 counts app=a pods of namespace default that are not terminating
    k0, p0, key0, param0, fl0 = unpack_term(c.pod_terms[0][0])
    assert list(c.node_count[p0, :4]) == [1, 0, 1, 0]
    assert fl0 & abi.KS_TOPO_T_SELF and param0 == 1 and c.keys[key0] == ZONE
    # the carried anti-affinity term: one pod on node 2; pod 3 and pod 0 (app=a, default) have it as a property
    pa = unpack_term(c.pod_terms[3][0])[1]
    assert list(c.node_count[pa, :4]) == [0, 0, 1, 0]
    assert pa not in c.pod_props[3]  # pod 3 does not carry the term itself
    # any other node label is a topology key of its own
    c2 = compile_topology(nodes + [{"rack": "r1"}], [], [TopoPod(spread=[SpreadConstraint(1, "rack", DO_NOT_SCHEDULE, sel_a)])])
    assert c2.keys == [HOSTNAME, "rack"] and list(c2.node_domain[0]) == [-1, -1, -1, -1, 0]
    many = [TopoPod(labels={"app": "x"}, anti_preferred=[(1 + k, AffinityTerm(HOSTNAME, LabelSelector((("app", str(k)),))))
                                                         for k in range(abi.KS_TOPO_MAX_TERMS + 1)])]
    with pytest.raises(StaticPluginError):
        compile_topology(nodes, [], many)


def test_compile_duplicate_scored_terms():
    """a running pod carrying the same scored term twice (a required affinity term and the same term preferred with
    weight 1; one preferred term listed twice) counts it with the summed weight: one carry property of weight 2 / 2w"""
    sel_a = LabelSelector((("app", "a"),))
    t = AffinityTerm(HOSTNAME, sel_a)
    nodes = [{ZONE: "z1"}, {ZONE: "z1"}]
    existing = [(0, TopoPod(labels={"app": "b"}, affinity_required=[t], affinity_preferred=[(1, t)])),
                (1, TopoPod(labels={"app": "b"}, affinity_preferred=[(7, t), (7, t)]))]
    pending = [TopoPod(labels={"app": "a"})]
    c = compile_topology(nodes, existing, pending)
    params = sorted(unpack_term(w)[3] for w in c.pod_terms[0] if unpack_term(w)[0] == KIND["score"])
    assert params == [2, 14]
    _, _, _, inn, _ = ref.evaluate(pending[0], nodes, existing, [True, True])
    w = synth.c1(n_nodes=2, n_pods=1)
    install(c, w.nodes, w.pods)
    orc = Oracle(_profile().to_ks_config(), w.nodes.copy())
    _, s, _ = orc.eval_pod(w.pods.rows([0]))
    orc.close()
    assert list(s[:, abi.KS_SCORE_POD_AFFINITY]) == inn == [14, 100]


def test_hand_worked_spread_and_affinity():
    """two zones; app=a pods: z1 holds 2 (nodes 0, 1), z2 holds 0; a DoNotSchedule zone constraint with maxSkew 1
    rejects z1 (2 + 1 - 0 > 1); a required anti-affinity to app=a per hostname rejects nodes 0 and 1; a required
    affinity to app=a per zone admits z1 only"""
    sel_a = LabelSelector((("app", "a"),))
    nodes = [{ZONE: "z1"}, {ZONE: "z1"}, {ZONE: "z2"}, {ZONE: "z2"}]
    existing = [(0, TopoPod(labels={"app": "a"})), (1, TopoPod(labels={"app": "a"}))]
    pending = [TopoPod(labels={"app": "a"}, spread=[SpreadConstraint(1, ZONE, DO_NOT_SCHEDULE, sel_a)]),
               TopoPod(labels={"app": "b"}, anti_required=[AffinityTerm(HOSTNAME, sel_a)]),
               TopoPod(labels={"app": "b"}, affinity_required=[AffinityTerm(ZONE, sel_a)]),
               TopoPod(labels={"app": "b"}, affinity_preferred=[(50, AffinityTerm(HOSTNAME, sel_a))])]
    w = synth.c1(n_nodes=4, n_pods=len(pending))
    install(compile_topology(nodes, existing, pending), w.nodes, w.pods)
    orc = Oracle(_profile().to_ks_config(), w.nodes.copy())
    r, s, t = orc.eval_pod(w.pods.rows([0]))
    assert list(r) == [abi.KS_R_TOPOLOGY_SPREAD] * 2 + [0, 0]
    r, s, t = orc.eval_pod(w.pods.rows([1]))
    assert list(r) == [abi.KS_R_POD_ANTI_AFFINITY] * 2 + [0, 0]
    r, s, t = orc.eval_pod(w.pods.rows([2]))
    assert list(r) == [0, 0] + [abi.KS_R_POD_AFFINITY] * 2
    r, s, t = orc.eval_pod(w.pods.rows([3]))
    # preferred affinity raw 50 / 50 / 0 / 0 -> 100 / 100 / 0 / 0; no spread constraint: 100 everywhere
    assert list(s[:, abi.KS_SCORE_POD_AFFINITY]) == [100, 100, 0, 0]
    assert list(s[:, abi.KS_SCORE_TOPOLOGY_SPREAD]) == [100] * 4
    assert list(t) == [300, 300, 200, 200]
    orc.close()


@pytest.mark.parametrize("seed", [1, 2])
def test_oracle_against_restatement(seed):
    w = _workload(120, 150, seed)
    _check_eval(w, _profile(), range(150))


def test_oracle_against_restatement_node_affinity():
    """the pods' required node affinity decides which nodes count for spreading; NodeAffinity's Filter runs too"""
    w = _workload(100, 120, 3, static=True)
    _check_eval(w, _profile(static=True), range(120), other_fn=lambda i, n: _node_aff(w, i)(n))


def test_oracle_against_restatement_with_fit():
    """next to NodeResourcesFit: the normalizations run over the nodes every Filter leaves"""
    w = _workload(90, 100, 4, per_node=(2, 9))
    _check_eval(w, _profile(fit=True), range(100), base_profile=SchedulerProfile(loadaware=None))


def test_schedule_against_restatement():
    """ko_schedule with only the two plugins against a sequential loop over the restatement: max total, lowest
    index; the placed pod joins its node's running pods (and its carried terms count from then on)"""
    w = _workload(12, 160, 5, per_node=(0, 2), spread_frac=0.35, anti_frac=0.15)
    node_labels, existing, pending = w.topo
    existing = list(existing)
    orc = Oracle(_profile().to_ks_config(), w.nodes.copy())
    got = orc.schedule(w.pods)
    st = orc.read_nodes()
    orc.close()
    for i, p in enumerate(pending):
        _, _, _, _, add = ref.evaluate(p, node_labels, existing, [True] * len(node_labels),
                                       ns_labels=synth.TOPO_NAMESPACE_LABELS)
        totals = [a if a is not None else -1 for a in add]
        best = max(totals)
        want = totals.index(best) if best >= 0 else -1
        assert int(got["node"][i]) == want, f"pod {i}"
        if want >= 0:
            assert int(got["score"][i]) == best, f"pod {i}: score"
            existing.append((want, p))
        else:
            assert int(got["status"][i]) == abi.KS_S_UNSCHEDULABLE
    # the counters after the queue are the compiled counters of the final pod set
    c = compile_topology(node_labels, existing, pending, namespace_labels=synth.TOPO_NAMESPACE_LABELS)
    assert np.array_equal(st.topo_count, c.node_count)
    assert (got["status"] == abi.KS_S_UNSCHEDULABLE).sum() > 0


def test_namespace_selector_cases():
    """namespaceSelector: the term reaches the selected namespaces' pods (with or without listed namespaces); a nil
    selector next to listed namespaces adds none; neither = the owner's namespace"""
    from koordinator_amd.topology_plugins import term_namespaces
    nsl = {"default": {"team": "a"}, "other": {"team": "b"}, "x": {}}
    owner = TopoPod(namespace="default")
    team_b = LabelSelector(match_expressions=(("team", "In", ("b",)),))
    assert term_namespaces(AffinityTerm(HOSTNAME), owner, nsl) == ("default",)
    assert term_namespaces(AffinityTerm(HOSTNAME, namespace_selector=LabelSelector()), owner, nsl) == ("default", "other", "x")
    assert term_namespaces(AffinityTerm(HOSTNAME, namespace_selector=team_b), owner, nsl) == ("other",)
    assert term_namespaces(AffinityTerm(HOSTNAME, namespaces=("x",), namespace_selector=team_b), owner, nsl) == ("other", "x")
    assert term_namespaces(AffinityTerm(HOSTNAME, namespaces=("x",)), owner, nsl) == ("x",)
    # through the oracle: anti-affinity to app=a of team b's namespaces rejects only the node holding other/app=a
    sel_a = LabelSelector((("app", "a"),))
    nodes = [{ZONE: "z1"}, {ZONE: "z1"}, {ZONE: "z2"}]
    existing = [(0, TopoPod(namespace="default", labels={"app": "a"})), (1, TopoPod(namespace="other", labels={"app": "a"}))]
    pending = [TopoPod(labels={"app": "b"}, anti_required=[AffinityTerm(HOSTNAME, sel_a, namespace_selector=team_b)])]
    w = synth.c1(n_nodes=3, n_pods=1)
    install(compile_topology(nodes, existing, pending, namespace_labels=nsl), w.nodes, w.pods)
    orc = Oracle(_profile().to_ks_config(), w.nodes.copy())
    r, _, _ = orc.eval_pod(w.pods.rows([0]))
    orc.close()
    assert list(r) == [0, abi.KS_R_POD_ANTI_AFFINITY, 0]
    pf, ipf, _, _, _ = ref.evaluate(pending[0], nodes, existing, [True] * 3, ns_labels=nsl)
    assert ipf == [None, "anti", None]


EDGE_SHAPES = [
    ("no zone labels", dict(unzoned_frac=1.0)),
    ("one zone", dict(n_zones=1, unzoned_frac=0.0)),
    ("64 zones", dict(n_zones=64, unzoned_frac=0.02)),
    ("200 zones", dict(n_zones=200, unzoned_frac=0.02)),
    ("empty cluster", dict(per_node=(0, 0))),
    ("anti-affinity heavy", dict(anti_frac=0.6, per_node=(0, 1))),
    ("system defaults only", dict(default_frac=1.0, spread_frac=0.0, anti_frac=0.0, affinity_frac=0.0, pref_frac=0.0)),
]


@pytest.mark.parametrize("label,kw", EDGE_SHAPES)
def test_oracle_against_restatement_edge_shapes(label, kw):
    """the C oracle on the compiled form against the object-level restatement on the domain's edge shapes (the same
    shapes tests/test_gpu_topology.py::test_edge_shapes runs on the device)"""
    w = _workload(60, 24, 70 + len(label), **kw)
    _check_eval(w, _profile(), range(w.pods.n))


BREADTH = dict(n_apps=240, extra_keys={"topology.kubernetes.io/region": 3, "example.com/rack": 40}, breadth_frac=0.3,
               dup_frac=0.1)


def test_breadth_compiles_wide():
    """>= 200 distinct selectors, two keys besides the hostname and the zone, pods with more than 8 terms"""
    w = _workload(300, 400, 91, **BREADTH)
    node_labels, existing, pending = w.topo
    c = compile_topology(node_labels, existing, pending, namespace_labels=synth.TOPO_NAMESPACE_LABELS)
    assert len(c.keys) == 4
    assert len({p[2] for p in c.props if p[0] == "sel"} | {p[2] for p in c.props if p[0] == "term"}) >= 200
    assert max(len(t) for t in c.pod_terms) > 8


@pytest.mark.parametrize("seed", [92, 93])
def test_oracle_against_restatement_breadth(seed):
    w = _workload(80, 90, seed, **BREADTH)
    _check_eval(w, _profile(), range(w.pods.n))


def test_schedule_against_restatement_breadth():
    w = _workload(16, 120, 94, per_node=(0, 2), **BREADTH)
    node_labels, existing, pending = w.topo
    existing = list(existing)
    orc = Oracle(_profile().to_ks_config(), w.nodes.copy())
    got = orc.schedule(w.pods)
    st = orc.read_nodes()
    orc.close()
    for i, p in enumerate(pending):
        _, _, _, _, add = ref.evaluate(p, node_labels, existing, [True] * len(node_labels),
                                       ns_labels=synth.TOPO_NAMESPACE_LABELS)
        totals = [a if a is not None else -1 for a in add]
        best = max(totals)
        want = totals.index(best) if best >= 0 else -1
        assert int(got["node"][i]) == want, f"pod {i}"
        if want >= 0:
            existing.append((want, p))
    c = compile_topology(node_labels, existing, pending, namespace_labels=synth.TOPO_NAMESPACE_LABELS)
    assert np.array_equal(st.topo_count, c.node_count)
