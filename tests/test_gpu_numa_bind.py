"""GPU parity for required CPU bind policies -- a pod's requiredCPUBindPolicy or a node's CPU bind label -- on nodes
with a NUMA topology policy: the Filter runs the policy conflict and SMT alignment checks but no trial
Allocate (nodenumaresource/plugin.go:303-327), FilterByNUMANode trims each NUMA node's available cpu to the CPUs the
policy keeps there (trimNUMANodeResources, resource_manager.go:144-167) for the hints and for the allocation,
splitQuantity splits a required FullPCPUs request in whole cores (:285-300), and allocateCPUSet takes, per allocated
NUMA node, min(the filtered CPUs there, its whole CPUs) and must satisfy the policy (:314-401).  The device keeps per
NUMA node the whole free cores and the cores with a free CPU (numa_free_word); the oracle runs allocateCPUSet for
real.  Against the reference's TestResourceManagerAllocate cases on a SingleNUMANode node and against the oracle on
C3-shaped queues with half the nodes under a NUMA policy (placements, scores, statuses, minors, cpusets, CPU state,
NUMA-node state, node columns), single-pod Filter / Score, and the per-pod framework mode with Unreserve."""
import numpy as np
import pytest

from assume_util import assert_states_equal, state
from cpuset_util import allocate_cases, policy_bind_cluster
from helpers import assert_same_results, assert_same_state
from koordinator_amd import abi, synth
from koordinator_amd.cluster import mask_cpus

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def runtime():
    from koordinator_amd import runtime as rt

    rt.lib()
    return rt


@pytest.mark.parametrize("case", allocate_cases(), ids=[c[0] for c in allocate_cases()])
def test_reference_allocate_cases_on_policy_node(runtime, oracle_lib, case):
    _, bind, allocated, want = case
    cfg, nodes, st, pod, nn = policy_bind_cluster((2, 1, 26, 2), allocated=allocated, bind=bind, required=True)
    ev = runtime.Evaluator(cfg, nodes.copy(), cpu_state=st.copy(), numa_nodes=nn.copy())
    orc = oracle_lib.Oracle(cfg, nodes.copy(), cpu_state=st.copy(), numa_nodes=nn.copy())
    try:
        r = ev.schedule(pod)
        w = orc.schedule(pod)
        assert r["status"][0] == w["status"][0]
        assert np.array_equal(ev.eval_pod(pod)[0], orc.eval_pod(pod)[0])
        if want is None:
            assert r["status"][0] == abi.KS_S_UNSCHEDULABLE
        else:
            assert r["status"][0] == abi.KS_S_SCHEDULED
            assert mask_cpus(ev.fetch_cpusets(1)[0]) == want
            assert np.array_equal(ev.fetch_numa_alloc(1), orc.fetch_numa_alloc(1))
    finally:
        ev.close()
        orc.close()


@pytest.mark.parametrize("alloc,cpu,mem", [([], 16000, 0), ([], 16000, 1 << 30), ([0], 14000, 0), ([0, 9], 12000, 0)])
def test_full_pcpus_split_in_whole_cores(runtime, oracle_lib, alloc, cpu, mem):
    """the hand-worked BestEffort cases of tests/test_cpu_bind_policy.py through HIP"""
    cfg, nodes, st, pod, nn = policy_bind_cluster((2, 1, 4, 2), allocated=alloc, bind=abi.KS_CPU_BIND_FULL_PCPUS,
                                                  required=True, cpu_milli=cpu, policy=abi.KS_NUMA_POLICY_BEST_EFFORT)
    pod.req_memory[:] = mem
    ev = runtime.Evaluator(cfg, nodes.copy(), cpu_state=st.copy(), numa_nodes=nn.copy())
    orc = oracle_lib.Oracle(cfg, nodes.copy(), cpu_state=st.copy(), numa_nodes=nn.copy())
    try:
        r, w = ev.schedule(pod), orc.schedule(pod)
        assert_same_results(r, w, f"split {alloc} {cpu}")
        assert np.array_equal(ev.fetch_cpusets(1), orc.fetch_cpusets(1))
    finally:
        ev.close()
        orc.close()


def check(runtime, oracle_lib, w, label):
    ev = runtime.Evaluator(w.cfg, w.nodes.copy(), **w.tables())
    orc = oracle_lib.Oracle(w.cfg, w.nodes.copy(), nthreads=8, **w.tables())
    try:
        got = ev.schedule(w.pods)
        want = orc.schedule(w.pods)
        assert_same_results(got, want, label)
        for k in ("gpu_minors", "rdma_minors"):
            assert np.array_equal(got[k], want[k]), f"{label}: {k} differ"
        cs_g, cs_o = ev.fetch_cpusets(w.pods.n), orc.fetch_cpusets(w.pods.n)
        bad = np.nonzero((cs_g != cs_o).any(axis=1))[0]
        assert bad.size == 0, (f"{label}: cpusets differ for pods {bad[:8]}: "
                               f"{[mask_cpus(cs_g[i]) for i in bad[:2]]} vs {[mask_cpus(cs_o[i]) for i in bad[:2]]}")
        for a, b in zip(ev.read_cpu_state(), orc.read_cpu_state()):
            assert np.array_equal(a, b), f"{label}: CPU state differs"
        for a, b in zip(ev.read_numa_nodes(), orc.read_numa_nodes()):
            assert np.array_equal(a, b), f"{label}: NUMA-node state differs"
        assert_same_state(ev.read_nodes(), orc.read_nodes(), label)
        stats = ev.stats()
    finally:
        ev.close()
        orc.close()
    return got, stats


def policy_bind_stats(w, got):
    """(required or label-bound pods placed on NUMA-policy nodes, passes)"""
    pol = (w.nodes.numa_flags >> abi.KS_NUMA_POLICY_SHIFT) & 3
    lab = (w.nodes.numa_flags >> abi.KS_NUMA_CPU_BIND_SHIFT) & 3
    ok = got["status"] == abi.KS_S_SCHEDULED
    nd = np.maximum(got["node"], 0)
    req = (w.pods.cpu_bind & abi.KS_CPU_BIND_REQUIRED) != 0
    plain = (w.pods.flags & abi.KS_POD_CPU_BIND) == 0
    return int((ok & (pol[nd] > 0) & (req | ((lab[nd] > 0) & plain))).sum())


@pytest.mark.parametrize("seed,policy", [(91, abi.KS_NUMA_POLICY_SINGLE_NUMA_NODE), (92, abi.KS_NUMA_POLICY_BEST_EFFORT),
                                         (93, abi.KS_NUMA_POLICY_RESTRICTED)])
def test_c3_required_policies_on_policy_nodes(runtime, oracle_lib, seed, policy):
    w = synth.c3_bind(seed=seed, n_nodes=1500, n_pods=3000, label_frac=0.4, required_frac=0.5, policy_frac=0.5,
                      policy=policy)
    got, stats = check(runtime, oracle_lib, w, f"c3-bind-policy{policy}")
    assert policy_bind_stats(w, got) > 200, policy_bind_stats(w, got)


def test_c3_required_policies_5k(runtime, oracle_lib):
    """SURVEY C3 at full size with labels on 40 % of the nodes and required policies on half the cpuset pods"""
    w = synth.c3_bind(seed=94, n_nodes=5000, n_pods=10000, label_frac=0.4, required_frac=0.5, policy_frac=0.5)
    got, stats = check(runtime, oracle_lib, w, "c3-bind-policy-5k")
    assert policy_bind_stats(w, got) > 800


def test_c3_required_policies_tight(runtime, oracle_lib):
    """few nodes: whole cores run out on the NUMA nodes, trims leave no hint, passes are cut on dirty policy slots"""
    w = synth.c3_bind(seed=95, n_nodes=80, n_pods=1500, label_frac=0.6, required_frac=0.6, policy_frac=0.8)
    got, stats = check(runtime, oracle_lib, w, "c3-bind-policy-tight")
    assert (got["status"] != abi.KS_S_SCHEDULED).sum() > 100 and stats["cut_passes"] > 0


def test_c3_required_policies_eval_pod(runtime, oracle_lib):
    w = synth.c3_bind(seed=96, n_nodes=400, n_pods=400, label_frac=0.5, required_frac=0.6, policy_frac=0.6)
    bind = (w.pods.flags & abi.KS_POD_CPU_BIND) != 0
    req = (w.pods.cpu_bind & abi.KS_CPU_BIND_REQUIRED) != 0
    whole = (w.pods.req_milli_cpu % 1000 == 0) & ~bind
    idx = np.concatenate([np.nonzero(req)[0][:25], np.nonzero(bind & ~req)[0][:10], np.nonzero(whole)[0][:25]])
    ev = runtime.Evaluator(w.cfg, w.nodes.copy(), **w.tables())
    orc = oracle_lib.Oracle(w.cfg, w.nodes.copy(), **w.tables())
    try:
        for i in idx:
            one = w.pods.rows([int(i)])
            r_g, s_g, t_g = ev.eval_pod(one)
            r_o, s_o, t_o = orc.eval_pod(one)
            assert np.array_equal(r_g, r_o), f"pod {i}: reasons at nodes {np.nonzero(r_g != r_o)[0][:5]}"
            assert np.array_equal(s_g, s_o), f"pod {i}: scores"
            assert np.array_equal(t_g, t_o), f"pod {i}: totals"
    finally:
        ev.close()
        orc.close()


def test_c3_required_policies_assume_unreserve(runtime, oracle_lib):
    """per-pod mode: ks_assume on policy nodes with required / label-bound pods, ks_unreserve gives the CPUs and the
    NUMA nodes' core counts back, a later queue schedules as on the oracle"""
    w = synth.c3_bind(seed=97, n_nodes=200, n_pods=300, label_frac=0.6, required_frac=0.6, policy_frac=0.7)
    ev = runtime.Evaluator(w.cfg, w.nodes.copy(), **w.tables())
    orc = oracle_lib.Oracle(w.cfg, w.nodes.copy(), **w.tables())
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
            a, csa, naa = ev.assume(pod, node)
            b, csb, nab = orc.assume(pod, node)
            assert a[0]["status"] == b[0]["status"], f"pod {i}"
            assert np.array_equal(csa, csb), f"pod {i}: cpuset {mask_cpus(csa)} vs {mask_cpus(csb)}"
            assert np.array_equal(naa, nab), f"pod {i}: NUMA allocation"
            if a[0]["status"] == abi.KS_S_SCHEDULED:
                held.append((i, a, csa, naa))
        assert len(held) > 60
        assert_states_equal(state(ev, w), state(orc, w), "assumed")
        for i, a, cs, na in held[::2]:
            pod = w.pods.rows([i])
            ev.unreserve(pod, a, cs, na)
            orc.unreserve(pod, a, cs, na)
        assert_states_equal(state(ev, w), state(orc, w), "half unreserved")
        rest = w.pods.rows(list(range(120, 300)))
        got, want = ev.schedule(rest), orc.schedule(rest)
        assert_same_results(got, want, "after unreserve")
        assert np.array_equal(ev.fetch_cpusets(rest.n), orc.fetch_cpusets(rest.n))
    finally:
        ev.close()
        orc.close()
