"""GPU parity of upstream PodTopologySpread and InterPodAffinity (ks_topo.h / ks_topo.hip: a topology pod is scheduled
alone by the topology step -- eval_debug_kernel, topo_filter_kernel, topo_norm_kernel, a one-pod commit -- and the
regular passes end before it; every Reserve counts the pod's properties on its node) with the CPU oracle, which the
CPU tests (tests/test_topology.py) check against the object-level restatement oracle/topology_ref.py.  Parity of the
upstream plugins themselves is unpinned (kube-scheduler v1.24.15 is not on disk).  Per-node reasons / scores /
totals through ks_eval_pod; whole queues through the pass loop -- with only the two plugins, C2-shaped under the
v1beta2 default plugin set (ElasticQuota, BalancedAllocation, TaintToleration, NodeAffinity, NodePorts), with
Reservation, with NUMA + DeviceShare (C3); the counters read back; ks_assume / ks_unreserve; the refusals."""
import numpy as np
import pytest

from helpers import assert_same_results, assert_same_state
from koordinator_amd import abi, synth
from koordinator_amd.config import SchedulerProfile

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def runtime():
    from koordinator_amd import runtime as rt

    rt.lib()  # the in-tree HIP library; no fallback
    return rt


def run(runtime, oracle_lib, w, label):
    cfg = w.cfg
    ev = runtime.Evaluator(cfg, w.nodes.copy(), **w.tables())
    orc = oracle_lib.Oracle(cfg, w.nodes.copy(), nthreads=8, **w.tables())
    try:
        got = ev.schedule(w.pods)
        st = ev.stats()
        want = orc.schedule(w.pods)
        assert_same_results(got, want, label)
        assert_same_state(ev.read_nodes(), orc.read_nodes(), label)
        for k in ("reservation", "gpu_minors", "rdma_minors"):
            assert np.array_equal(got[k], want[k]), f"{label}: {k}"
        if w.quotas is not None:
            assert np.array_equal(ev.read_quota_used(), orc.read_quota_used()), f"{label}: quota used"
    finally:
        ev.close()
        orc.close()
    return got, st


def topo_only(n_nodes, n_pods, seed, **kw):
    w = synth.c1(n_nodes=n_nodes, n_pods=n_pods)
    w = synth.with_topology(w, seed=seed, **kw)
    return w


def test_eval_pod(runtime, oracle_lib):
    w = synth.with_topology(synth.with_static_plugins(synth.c1(n_nodes=700, n_pods=160), seed=31), seed=32)
    cfg = w.cfg
    ev = runtime.Evaluator(cfg, w.nodes.copy())
    orc = oracle_lib.Oracle(cfg, w.nodes.copy())
    seen = 0
    try:
        for i in range(w.pods.n):
            one = w.pods.rows([i])
            r_g, s_g, t_g = ev.eval_pod(one)
            r_o, s_o, t_o = orc.eval_pod(one)
            assert np.array_equal(r_g, r_o), f"pod {i}: reasons at nodes {np.nonzero(r_g != r_o)[0][:5]}"
            assert np.array_equal(s_g, s_o), f"pod {i}: scores at {np.argwhere(s_g != s_o)[:5].tolist()}"
            assert np.array_equal(t_g, t_o), f"pod {i}: totals"
            seen |= int(np.bitwise_or.reduce(r_g))
    finally:
        ev.close()
        orc.close()
    for bit in (abi.KS_R_TOPOLOGY_SPREAD, abi.KS_R_POD_AFFINITY, abi.KS_R_POD_ANTI_AFFINITY,
                abi.KS_R_EXISTING_ANTI_AFFINITY):
        assert seen & bit, hex(bit)


def test_topology_only_queue(runtime, oracle_lib):
    """the two plugins alone (Fit + LoadAware off): tight hostname / zone skews and anti-affinity decide placements"""
    w = topo_only(60, 500, 41, per_node=(0, 2), spread_frac=0.35, anti_frac=0.15)
    w.profile.fit = None
    w.profile.loadaware = None
    got, st = run(runtime, oracle_lib, w, "topology-only")
    assert (got["status"] == abi.KS_S_UNSCHEDULABLE).sum() > 0


@pytest.mark.parametrize("seed", [42, 43])
def test_with_fit_loadaware(runtime, oracle_lib, seed):
    w = topo_only(800, 2000, seed)
    run(runtime, oracle_lib, w, f"fit+la+topology seed {seed}")


def test_c2_default_with_topology(runtime, oracle_lib):
    """C2 under the v1beta2 default plugin set with the two plugins as well (weights 2 / 1)"""
    w = synth.with_topology(synth.c2_default(n_nodes=1500, n_pods=3000), seed=44)
    got, st = run(runtime, oracle_lib, w, "c2-default+topology")
    assert (got["status"] == abi.KS_S_SCHEDULED).sum() > 1000


def test_reservation_with_topology(runtime, oracle_lib):
    w = synth.with_topology(synth.c4(n_nodes=1000, n_reservations=2500, n_pods=2000), seed=45)
    run(runtime, oracle_lib, w, "c4+topology")


def test_c3_with_topology(runtime, oracle_lib):
    """NUMA + DeviceShare (C3) with the two plugins: cpuset / device Reserves of topology pods in the one-pod commit"""
    w = synth.with_topology(synth.c3(n_nodes=800, n_pods=1600), seed=46)
    run(runtime, oracle_lib, w, "c3+topology")


def test_c3_topology_queue_head_on_poisoned_lists(runtime, oracle_lib, monkeypatch):
    """A new context whose queue starts with more topology pods than one pass's topology steps take (C3: reserve_pre_kernel
    runs ahead of every regular pass's commit): the regular pass that meets a topology pod at the cursor has no candidate
    lists (its sweep and select return at once), and the Reserve pre-pass must not read the lists' memory as nodes.
    KS_TEST_POISON_LISTS=1 makes ks_create fill the lists with large words instead of zeros, so the condition is forced
    rather than left to the allocator; the pre-pass stops where the commit stops (topo_pass_pods) and drops any list
    entry outside the cluster."""
    monkeypatch.setenv("KS_TEST_POISON_LISTS", "1")
    w = synth.with_topology(synth.c3(n_nodes=800, n_pods=1600), seed=46)
    dyn = (w.pods.topo_flags & abi.KS_TOPO_DYN) != 0
    assert dyn[:9].all()  # the queue's head: more topology pods in a row than the 8 topology steps of a pass
    run(runtime, oracle_lib, w, "c3+topology, poisoned lists")


def test_assume_unreserve_counters(runtime, oracle_lib):
    w = topo_only(300, 200, 47)
    ev = runtime.Evaluator(w.cfg, w.nodes.copy())
    orc = oracle_lib.Oracle(w.cfg, w.nodes.copy())
    try:
        held = []
        for i in range(120):
            pod = w.pods.rows([i])
            rg, _, tg = ev.eval_pod(pod)
            ro, _, to = orc.eval_pod(pod)
            assert np.array_equal(rg, ro) and np.array_equal(tg, to), f"pod {i}: eval"
            if tg.max() < 0:
                continue
            node = int(np.argmax(tg))
            a, _, _ = ev.assume(pod, node)
            b, _, _ = orc.assume(pod, node)
            assert a[0]["status"] == b[0]["status"]
            held.append((i, a))
        assert_same_state(ev.read_nodes(), orc.read_nodes(), "assumed")
        for i, a in held[::2]:
            pod = w.pods.rows([i])
            ev.unreserve(pod, a)
            orc.unreserve(pod, a)
        assert_same_state(ev.read_nodes(), orc.read_nodes(), "half unreserved")
        rest = w.pods.rows(list(range(120, 200)))
        assert_same_results(ev.schedule(rest), orc.schedule(rest), "after unreserve")
        assert_same_state(ev.read_nodes(), orc.read_nodes(), "after the queue")
    finally:
        ev.close()
        orc.close()


def test_checkpoint_restores_counters(runtime, oracle_lib):
    w = topo_only(400, 600, 48)
    ev = runtime.Evaluator(w.cfg, w.nodes.copy())
    try:
        ev.checkpoint()
        first = ev.schedule(w.pods)
        c1 = ev.read_nodes().topo_count.copy()
        ev.restore()
        assert np.array_equal(ev.read_nodes().topo_count, w.nodes.topo_count)
        second = ev.schedule(w.pods)
        assert_same_results(second, first, "after restore")
        assert np.array_equal(ev.read_nodes().topo_count, c1)
    finally:
        ev.close()


def test_refusals(runtime):
    w = topo_only(64, 8, 49)
    ev = runtime.Evaluator(w.cfg, w.nodes.copy())
    try:
        for mutate in (lambda t: t.__setitem__(0, np.uint64(7)),                   # kind 7: no such term
                       lambda t: t.__setitem__(0, t[0] | np.uint64(0xFFFF << 16)),  # property 65535: not loaded
                       lambda t: t.__setitem__(0, t[0] | np.uint64(0xF0 << 8))):    # key 240: not loaded
            bad = w.pods.rows([0])
            assert len(bad.topo_terms) > 0
            mutate(bad.topo_terms)
            with pytest.raises(runtime.KsError) as e:
                ev.schedule(bad)
            assert e.value.rc == abi.KS_EINVAL
        many = w.pods.rows([0])
        many.set_topo([[]], [[int(many.topo_terms[0])] * (abi.KS_TOPO_MAX_TERMS + 1)])
        with pytest.raises(runtime.KsError) as e:
            ev.schedule(many)
        assert e.value.rc == abi.KS_EINVAL
    finally:
        ev.close()


def test_graph_and_direct_launches_agree(runtime, oracle_lib):
    """the topology path's iterations run as one HIP graph per 4 iterations; with per-kernel profiling events on they
    are launched one by one -- both give the oracle's schedule, and the step runs several topology steps per pass"""
    w = synth.with_topology(synth.c2_default(n_nodes=600, n_pods=900), seed=50)
    orc = oracle_lib.Oracle(w.cfg, w.nodes.copy(), nthreads=8, **w.tables())
    want = orc.schedule(w.pods)
    orc.close()
    for prof in (False, True):
        ev = runtime.Evaluator(w.cfg, w.nodes.copy(), **w.tables())
        try:
            ev.set_profile(prof)
            got = ev.schedule(w.pods)
            assert_same_results(got, want, f"profile={prof}")
            st = ev.stats()
            assert st["passes"] > 0.8 * w.pods.n  # (every topology pod is a one-pod commit)
        finally:
            ev.close()



@pytest.mark.parametrize("label,kw", [
    ("no zone labels", dict(unzoned_frac=1.0)),
    ("one zone", dict(n_zones=1, unzoned_frac=0.0)),
    ("64 zones", dict(n_zones=64, unzoned_frac=0.02)),
    ("1000 zones", dict(n_zones=1000, unzoned_frac=0.02)),
    ("empty cluster", dict(per_node=(0, 0))),
    ("anti-affinity heavy", dict(anti_frac=0.6, per_node=(0, 1))),
    ("system defaults only", dict(default_frac=1.0, spread_frac=0.0, anti_frac=0.0, affinity_frac=0.0, pref_frac=0.0)),
    ("hard spread heavy", dict(spread_frac=0.9, default_frac=0.0)),
])
def test_edge_shapes(runtime, oracle_lib, label, kw):
    """the domain's edge shapes: nodes without the zonal key (every zonal constraint fails / is ignored), a single
    domain, 64 and 1000 values of a key (a wave's nodes in many domains), no placed pods, saturating anti-affinity, only the system default constraints, mostly
    DoNotSchedule constraints -- placements, counters and node state equal the oracle's"""
    w = topo_only(300, 400, 60 + len(label), **kw)
    got, st = run(runtime, oracle_lib, w, label)
    assert got["status"].shape[0] == 400


# breadth: 240 apps (one selector each), region and rack keys besides the hostname and the zone, pods with many terms
# over every key, pods carrying one scored term twice
BREADTH = dict(n_apps=240, extra_keys={"topology.kubernetes.io/region": 3, "example.com/rack": 40}, breadth_frac=0.3,
               dup_frac=0.1)


def test_breadth_eval_pod(runtime, oracle_lib):
    w = topo_only(900, 200, 71, **BREADTH)
    c = w.topo_compiled
    assert len(c.keys) == 4 and len(c.props) > 200 and max(len(t) for t in c.pod_terms) > 8
    ev = runtime.Evaluator(w.cfg, w.nodes.copy())
    orc = oracle_lib.Oracle(w.cfg, w.nodes.copy())
    try:
        for i in range(w.pods.n):
            one = w.pods.rows([i])
            r_g, s_g, t_g = ev.eval_pod(one)
            r_o, s_o, t_o = orc.eval_pod(one)
            assert np.array_equal(r_g, r_o), f"pod {i}: reasons at nodes {np.nonzero(r_g != r_o)[0][:5]}"
            assert np.array_equal(s_g, s_o), f"pod {i}: scores at {np.argwhere(s_g != s_o)[:5].tolist()}"
            assert np.array_equal(t_g, t_o), f"pod {i}: totals"
    finally:
        ev.close()
        orc.close()


@pytest.mark.parametrize("seed", [72, 73])
def test_breadth_queue(runtime, oracle_lib, seed):
    w = topo_only(1200, 2500, seed, **BREADTH)
    got, _ = run(runtime, oracle_lib, w, f"breadth seed {seed}")
    assert (got["status"] == abi.KS_S_SCHEDULED).sum() > 500


def test_breadth_c2_default(runtime, oracle_lib):
    """the complete v1beta2 default profile (C2 shape) at breadth"""
    w = synth.with_topology(synth.c2_default(n_nodes=1500, n_pods=3000), seed=74, **BREADTH)
    run(runtime, oracle_lib, w, "c2-default breadth")


@pytest.mark.parametrize("nranks,vshards", [(2, 1), (2, 2)])
def test_sharded_topology(runtime, oracle_lib, nranks, vshards):
    """node sharding with topology pods: every rank runs the topology steps over the whole (replicated) node table, the
    regular passes are sharded and merged (the loopback transport of tests/test_gpu_shard_loopback.py)"""
    w = synth.with_topology(synth.c2_default(n_nodes=1000, n_pods=1500), seed=75, **BREADTH)
    cfg = w.cfg
    tables = w.tables()
    evs = [runtime.Evaluator(cfg, w.nodes.copy(), **{k: v.copy() for k, v in tables.items()}) for _ in range(nranks)]
    try:
        runtime.shard_loopback(evs, vshards)
        outs = runtime.run_ranks(lambda ev: {"got": ev.schedule(w.pods), "state": ev.read_nodes()}, evs)
    finally:
        for ev in evs:
            ev.close()
    orc = oracle_lib.Oracle(cfg, w.nodes.copy(), nthreads=8, **tables)
    want = orc.schedule(w.pods)
    try:
        for r, o in enumerate(outs):
            assert_same_results(o["got"], want, f"rank {r}")
            assert_same_state(o["state"], orc.read_nodes(), f"rank {r}")
    finally:
        orc.close()
