"""Upstream TaintToleration and NodeAffinity (kube-scheduler v1.24.15 plugins/tainttoleration, plugins/nodeaffinity;
not on disk, so parity is unpinned against reference fixtures).  CPU only:
  * hand-worked matching cases (Toleration.ToleratesTaint, labels.Requirement.Matches, empty terms);
  * the host compiler (koordinator_amd/static_plugins.py: dictionaries + bit masks) with the C oracle's bit-mask
    evaluation against oracle/static_plugins_ref.py, which restates both plugins on the taint / label objects --
    per-node Filter verdicts and normalized scores, alone and next to NodeResourcesFit (normalization over the
    nodes the other Filters leave);
  * refusals the device dictionaries imply."""
import numpy as np
import pytest

from koordinator_amd import abi, synth
from koordinator_amd.cluster import NodeTable, PodTable
from koordinator_amd.config import SchedulerProfile
from koordinator_amd.static_plugins import (FIELD_NAME, NO_EXECUTE, NO_SCHEDULE, PREFER_NO_SCHEDULE, NodeSpec,
                                            PodAffinitySpec, Requirement, StaticPluginError, Taint, Term, Toleration,
                                            compile_cluster, requirement_matches)
from oracle import static_plugins_ref as ref
from oracle.oracle import Oracle


def test_toleration_cases():
    t_ns = Taint("dedicated", "infra", NO_SCHEDULE)
    t_pns = Taint("dedicated", "infra", PREFER_NO_SCHEDULE)
    assert Toleration("", "Exists").tolerates(t_ns) and Toleration("", "Exists").tolerates(t_pns)
    assert Toleration("dedicated", "Exists", "", NO_SCHEDULE).tolerates(t_ns)
    assert not Toleration("dedicated", "Exists", "", NO_SCHEDULE).tolerates(t_pns)  # effect mismatch
    assert Toleration("dedicated", "Equal", "infra").tolerates(t_pns)                # empty effect: every effect
    assert Toleration("dedicated", "", "infra").tolerates(t_ns)                       # "" operator = Equal
    assert not Toleration("dedicated", "Equal", "db").tolerates(t_ns)
    assert not Toleration("other", "Exists").tolerates(t_ns)
    assert not Toleration("dedicated", "Bogus", "infra").tolerates(t_ns)


def test_requirement_cases():
    n = NodeSpec("n1", {"zone": "a", "rack": "12", "bad": "x1"})
    assert requirement_matches(Requirement("zone", "In", ("a", "b")), n)
    assert not requirement_matches(Requirement("zone", "In", ("b",)), n)
    assert requirement_matches(Requirement("missing", "NotIn", ("a",)), n)  # NotIn holds when the key is absent
    assert not requirement_matches(Requirement("zone", "NotIn", ("a",)), n)
    assert requirement_matches(Requirement("zone", "Exists"), n)
    assert requirement_matches(Requirement("missing", "DoesNotExist"), n)
    assert requirement_matches(Requirement("rack", "Gt", ("11",)), n)
    assert not requirement_matches(Requirement("rack", "Gt", ("12",)), n)
    assert requirement_matches(Requirement("rack", "Lt", ("13",)), n)
    assert not requirement_matches(Requirement("bad", "Gt", ("0",)), n)      # label not an integer
    assert not requirement_matches(Requirement("missing", "Lt", ("5",)), n)  # Gt / Lt need the key
    assert requirement_matches(Requirement(FIELD_NAME, "In", ("n1",), field=True), n)
    assert requirement_matches(Requirement(FIELD_NAME, "NotIn", ("n2",), field=True), n)


def _profile(fit=False):
    p = SchedulerProfile(fit=None, loadaware=None, taint_toleration=True, node_affinity=True,
                         taint_toleration_weight=2, node_affinity_weight=3, node_ports=True)
    if fit:
        p = SchedulerProfile(loadaware=None, taint_toleration=True, node_affinity=True,
                             taint_toleration_weight=2, node_affinity_weight=3, node_ports=True)
    return p


def _compare(w, fit: bool, pods=range(60)):
    nspec, pspec = w.specs
    cfg = _profile(fit).to_ks_config()
    orc = Oracle(cfg, w.nodes.copy())
    base = None
    if fit:
        bcfg = SchedulerProfile(loadaware=None).to_ks_config()
        base = Oracle(bcfg, w.nodes.copy())
    for i in pods:
        one = w.pods.rows([i])
        r, s, t = orc.eval_pod(one)
        other = [True] * len(nspec)
        if base is not None:
            rb, sb, tb = base.eval_pod(one)
            other = list(rb == 0)
        feas, ts, as_ = ref.evaluate(pspec[i], nspec, other)
        assert list(r == 0) == feas, f"pod {i}: feasibility"
        for n in range(len(nspec)):
            if base is None:
                assert bool(r[n] & abi.KS_R_TAINT) == (not ref.taint_filter(pspec[i], nspec[n]))
                assert bool(r[n] & abi.KS_R_NODE_AFFINITY) == (not ref.affinity_filter(pspec[i], nspec[n]))
                assert bool(r[n] & abi.KS_R_NODE_PORTS) == (not ref.ports_filter(pspec[i], nspec[n]))
        assert list(s[:, abi.KS_SCORE_TAINT]) == ts, f"pod {i}: TaintToleration scores"
        assert list(s[:, abi.KS_SCORE_NODE_AFFINITY]) == as_, f"pod {i}: NodeAffinity scores"
        if base is None:
            want_t = [2 * a + 3 * b if f else -1 for a, b, f in zip(ts, as_, feas)]
            assert list(t) == want_t, f"pod {i}: totals"
    orc.close()
    if base is not None:
        base.close()


@pytest.mark.parametrize("fit", [False, True])
def test_oracle_against_restatement(fit):
    w = synth.with_static_plugins(synth.c1(n_nodes=300, n_pods=120), seed=11)
    _compare(w, fit)


def test_empty_terms_and_selector():
    nodes = [NodeSpec("a", {"zone": "z1"}), NodeSpec("b", {"zone": "z2"}, [Taint("t", "", PREFER_NO_SCHEDULE)])]
    pods = [PodAffinitySpec(required=[]),                                   # no terms: nothing matches
            PodAffinitySpec(required=[Term([])]),                           # an empty term matches nothing
            PodAffinitySpec(node_selector={"zone": "z2"}),
            PodAffinitySpec(node_selector={"zone": "z2"}, required=[Term([Requirement("zone", "In", ("z1",))])]),
            PodAffinitySpec(preferred=[(10, Term([])), (5, Term([Requirement("zone", "In", ("z1",))]))])]
    nt = synth.make_nodes(2, np.random.Generator(np.random.PCG64(1)))
    pt = synth.make_pods(len(pods), np.random.Generator(np.random.PCG64(2)))
    compile_cluster(nodes, pods, nt, pt)
    orc = Oracle(_profile().to_ks_config(), nt)
    want_feas = [[False, False], [False, False], [False, True], [False, False], [True, True]]
    for i in range(len(pods)):
        r, s, t = orc.eval_pod(pt.rows([i]))
        assert list(r == 0) == want_feas[i], i
        feas, ts, as_ = ref.evaluate(pods[i], nodes, [True, True])
        assert feas == want_feas[i]
        assert list(s[:, abi.KS_SCORE_TAINT]) == ts and list(s[:, abi.KS_SCORE_NODE_AFFINITY]) == as_
    # pod 4: affinity raw 5 / 0 -> 100 / 0; taint raw 0 / 1 -> reverse 100 / 0
    r, s, t = orc.eval_pod(pt.rows([4]))
    assert list(s[:, abi.KS_SCORE_NODE_AFFINITY]) == [100, 0] and list(s[:, abi.KS_SCORE_TAINT]) == [100, 0]
    orc.close()


def test_host_port_cases():
    from koordinator_amd.static_plugins import HostPort
    any80 = HostPort(80, "", "")
    assert any80.conflicts(HostPort(80, "TCP", "10.0.0.1")) and HostPort(80, "TCP", "10.0.0.1").conflicts(any80)
    assert not HostPort(80, "TCP", "10.0.0.1").conflicts(HostPort(80, "TCP", "10.0.0.2"))
    assert not HostPort(80, "UDP").conflicts(HostPort(80, "TCP"))
    assert not HostPort(0).conflicts(HostPort(0))  # no host port: never a conflict
    nodes = [NodeSpec("a", used_ports=[HostPort(80, "TCP", "10.0.0.1")]), NodeSpec("b")]
    pods = [PodAffinitySpec(host_ports=[HostPort(80, "TCP", "10.0.0.2")]), PodAffinitySpec(host_ports=[any80])]
    nt = synth.make_nodes(2, np.random.Generator(np.random.PCG64(1)))
    pt = synth.make_pods(2, np.random.Generator(np.random.PCG64(2)))
    compile_cluster(nodes, pods, nt, pt)
    cfg = SchedulerProfile(fit=None, loadaware=None, node_ports=True).to_ks_config()
    orc = Oracle(cfg, nt)
    r, _, _ = orc.eval_pod(pt.rows([0]))
    assert list(r) == [0, 0]
    r, _, _ = orc.eval_pod(pt.rows([1]))
    assert list(r) == [abi.KS_R_NODE_PORTS, 0]
    # schedule both: pod 0 takes 10.0.0.2:80 on node a (lowest index on a tie), pod 1 (0.0.0.0:80) then fits b only
    res = orc.schedule(pt)
    assert list(res["node"]) == [0, 1]
    st = orc.read_nodes()
    assert int(st.host_ports[0]) == int(nt.host_ports[0]) | int(pt.host_ports[0])
    orc.close()


def test_refusals():
    nodes = [NodeSpec(f"n{i}", {}, [Taint(f"k{i}", "", NO_EXECUTE)]) for i in range(65)]
    with pytest.raises(StaticPluginError):
        compile_cluster(nodes, [], NodeTable(65), PodTable(0))
    pods = [PodAffinitySpec(required=[Term([Requirement("z", "In", (str(i),))]) for i in range(5)])]
    with pytest.raises(StaticPluginError):
        compile_cluster([NodeSpec("a")], pods, NodeTable(1), PodTable(1))
    with pytest.raises(StaticPluginError):
        compile_cluster([NodeSpec("a")], [PodAffinitySpec(required=[Term([Requirement("z", "Gt", ("x",))])])],
                        NodeTable(1), PodTable(1))


def test_schedule_against_restatement():
    # whole queues, one pod at a time: the C oracle (bit masks, ko_schedule) against a sequential loop over the
    # restatement on raw objects -- Filter, normalized Scores, selectHost (max total, lowest index), and NodePorts'
    # Reserve (the placed pod's host ports join the node's UsedPorts) -- with only these plugins enabled
    import copy
    w = synth.with_static_plugins(synth.c1(n_nodes=40, n_pods=160), seed=13)
    nspec, pspec = copy.deepcopy(w.specs[0]), w.specs[1]
    cfg = _profile().to_ks_config()  # taint x2, affinity x3, ports
    orc = Oracle(cfg, w.nodes.copy())
    got = orc.schedule(w.pods)
    orc.close()
    for i, p in enumerate(pspec):
        feas, ts, as_ = ref.evaluate(p, nspec, [True] * len(nspec))
        totals = [2 * a + 3 * b if f else -1 for a, b, f in zip(ts, as_, feas)]
        best = max(totals)
        want = totals.index(best) if best >= 0 else -1
        assert int(got["node"][i]) == want, f"pod {i}"
        if want >= 0:
            assert int(got["score"][i]) == best
            nspec[want].used_ports = list(nspec[want].used_ports) + [h.sanitized() for h in p.host_ports if h.port > 0]
        else:
            assert int(got["status"][i]) == abi.KS_S_UNSCHEDULABLE


def test_prebuilt_dictionaries_refuse_unknown_items():
    """The informer path keeps the dictionaries across cycles: a requirement, host port or taint that arrives later is
    refused with StaticPluginError (the shim falls back to the reference path and rebuilds), never a bare KeyError;
    the new pods' requirements are validated on that path too."""
    from koordinator_amd.static_plugins import HostPort, build_dictionaries

    nodes = [NodeSpec("a", {"zone": "z1"}, [Taint("t", "", NO_SCHEDULE)], used_ports=[HostPort(80)])]
    pods = [PodAffinitySpec(node_selector={"zone": "z1"}, host_ports=[HostPort(80)])]
    d = build_dictionaries(nodes, pods)
    compile_cluster(nodes, pods, NodeTable(1), PodTable(1), dicts=d)  # the same items: fine
    later = [PodAffinitySpec(node_selector={"zone": "z2"})]
    with pytest.raises(StaticPluginError):
        compile_cluster(nodes, later, NodeTable(1), PodTable(1), dicts=d)
    with pytest.raises(StaticPluginError):
        compile_cluster(nodes, [PodAffinitySpec(host_ports=[HostPort(8080)])], NodeTable(1), PodTable(1), dicts=d)
    tainted = [NodeSpec("a", {"zone": "z1"}, [Taint("new", "", NO_EXECUTE)])]
    with pytest.raises(StaticPluginError):
        compile_cluster(tainted, pods, NodeTable(1), PodTable(1), dicts=d)
    bad = [PodAffinitySpec(required=[Term([Requirement("zone", "Gt", ("x",))])])]
    with pytest.raises(StaticPluginError):
        compile_cluster(nodes, bad, NodeTable(1), PodTable(1), dicts=d)


def test_matching_rules_against_independent_restatement():
    """The host compiler's matching rules (Toleration.tolerates, requirement_matches, HostPort.conflicts) against
    oracle/static_plugins_ref.py's own restatement of ToleratesTaint, labels.Requirement.Matches and
    HostPortInfo.CheckConflict on random objects (including Gt / Lt on non-numeric and signed values)."""
    from koordinator_amd.static_plugins import HostPort

    rng = np.random.Generator(np.random.PCG64(77))
    vals = ["", "a", "b", "10", "-3", "+7", "007", "1_000", " 5", "x1"]
    keys = ["k", "zone", "n"]
    for _ in range(3000):
        labels = {k: str(rng.choice(vals)) for k in keys if rng.random() < 0.6}
        node = NodeSpec(str(rng.choice(["n1", "n2"])), labels)
        op = str(rng.choice(["In", "NotIn", "Exists", "DoesNotExist", "Gt", "Lt"]))
        if op in ("Exists", "DoesNotExist"):
            r = Requirement(str(rng.choice(keys)), op, ())
        elif op in ("Gt", "Lt"):
            r = Requirement(str(rng.choice(keys)), op, (str(rng.choice(["5", "-1", "0", "12"])),))
        elif rng.random() < 0.2:
            r = Requirement(FIELD_NAME, op, (str(rng.choice(["n1", "n2"])),), field=True)
        else:
            r = Requirement(str(rng.choice(keys)), op, tuple(sorted({str(v) for v in rng.choice(vals, 2)})))
        assert requirement_matches(r, node) == ref.node_requirement_matches(r, node), (r, labels)
        t = Taint(str(rng.choice(["", "k"])), str(rng.choice(["", "v"])),
                  str(rng.choice([NO_SCHEDULE, NO_EXECUTE, PREFER_NO_SCHEDULE])))
        tol = Toleration(str(rng.choice(["", "k", "x"])), str(rng.choice(["", "Equal", "Exists", "Bogus"])),
                         str(rng.choice(["", "v"])), str(rng.choice(["", NO_SCHEDULE, PREFER_NO_SCHEDULE])))
        assert tol.tolerates(t) == ref.tolerates_taint(tol, t), (tol, t)
        a = HostPort(int(rng.choice([0, 80, 81])), str(rng.choice(["", "TCP", "UDP"])), str(rng.choice(["", "0.0.0.0", "10.0.0.1", "10.0.0.2"])))
        b = HostPort(int(rng.choice([0, 80, 81])), str(rng.choice(["", "TCP", "UDP"])), str(rng.choice(["", "0.0.0.0", "10.0.0.1", "10.0.0.2"])))
        assert a.conflicts(b) == ref.check_conflict(ref.host_port_info([b]), a.host_ip, a.protocol, a.port), (a, b)
