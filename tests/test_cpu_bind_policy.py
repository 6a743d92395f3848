"""NodeNUMAResource node CPU bind policies (the node-cpu-bind-policy label) and required pod CPU bind policies on
the CPU oracle: the reference's Filter cases (plugin_test.go:592-760) and required-policy allocations
(resource_manager_test.go:95-330) as known answers, then the semantics the device path relies on (Reserve of a
pod cpu-bind only through the node's policy, count form of the trial Allocate)."""
import numpy as np
import pytest

from cpuset_util import allocate_cases, bind_policy_cluster, filter_cases, policy_bind_cluster
from koordinator_amd import abi, synth
from koordinator_amd.cluster import mask_cpus
from oracle.oracle import Oracle


@pytest.mark.parametrize("case", filter_cases(), ids=[c[0] for c in filter_cases()])
def test_reference_filter_cases(case):
    _, label, bind, required, cpu, want = case
    cfg, nodes, st, pod = bind_policy_cluster((2, 1, 4, 2), label=label, cpu_milli=cpu, bind=bind, required=required)
    o = Oracle(cfg, nodes, cpu_state=st)
    assert int(o.eval_pod(pod)[0][0]) == want
    o.close()


@pytest.mark.parametrize("case", allocate_cases(), ids=[c[0] for c in allocate_cases()])
def test_reference_allocate_cases(case):
    _, bind, allocated, want = case
    cfg, nodes, st, pod = bind_policy_cluster((2, 1, 26, 2), allocated=allocated, bind=bind, required=True)
    o = Oracle(cfg, nodes, cpu_state=st)
    r = o.schedule(pod)
    if want is None:
        # the Filter's trial Allocate fails: "not enough cpus available to satisfy request"
        assert r["status"][0] == abi.KS_S_UNSCHEDULABLE
        assert int(o.eval_pod(pod)[0][0]) == abi.KS_R_NUMA_CPUSET
    else:
        assert r["status"][0] == abi.KS_S_SCHEDULED
        assert mask_cpus(o.fetch_cpusets(1)[0]) == want
    o.close()


@pytest.mark.parametrize("case", allocate_cases(), ids=[c[0] for c in allocate_cases()])
def test_reference_allocate_cases_on_numa_policy_node(case):
    """the same TestResourceManagerAllocate cases (their hint is NUMA node 0) on a SingleNUMANode node: the topology
    manager admits NUMA node 0 (trimNUMANodeResources leaves node 1, whose CPUs are all allocated, no cpu), the NUMA
    allocation is 4 CPUs there and allocateCPUSet takes the reference's CPUs; where the reference's Allocate fails, the
    trimmed hints already leave nothing to admit"""
    _, bind, allocated, want = case
    cfg, nodes, st, pod, nn = policy_bind_cluster((2, 1, 26, 2), allocated=allocated, bind=bind, required=True)
    o = Oracle(cfg, nodes, cpu_state=st, numa_nodes=nn)
    r = o.schedule(pod)
    if want is None:
        assert r["status"][0] == abi.KS_S_UNSCHEDULABLE
    else:
        assert r["status"][0] == abi.KS_S_SCHEDULED
        assert mask_cpus(o.fetch_cpusets(1)[0]) == want
        na = o.fetch_numa_alloc(1)[0]
        assert na[0][0] == 4000 and na[1][0] == 0  # NUMANodeResources: cpu 4 on NUMA node 0
    o.close()


def test_required_full_pcpus_split_over_two_numa_nodes():
    """BestEffort node, 16 CPUs required FullPCPUs (no memory request: the cpu hints alone) on 2 x (4 cores x 2
    threads): neither NUMA node alone has 16 CPUs, the {0, 1} hint splits in whole cores (splitQuantity :290-296:
    8 + 8).  With CPU 0 taken and 14 CPUs: NUMA node 0 keeps 3 whole cores (trimNUMANodeResources: 7000 -> 6000),
    the split gives 3 cores there and 4 on node 1, and allocateCPUSet takes cores 1-3 and 4-7.  (With a memory request
    the memory list's single-NUMA hints narrow the merged affinity to {0}, whose allocation then fails: the
    reference's merge prefers the narrower non-preferred hint.)"""
    cfg, nodes, st, pod, nn = policy_bind_cluster((2, 1, 4, 2), allocated=[], bind=abi.KS_CPU_BIND_FULL_PCPUS,
                                                  required=True, cpu_milli=16000,
                                                  policy=abi.KS_NUMA_POLICY_BEST_EFFORT)
    pod.req_memory[:] = 0
    o = Oracle(cfg, nodes, cpu_state=st, numa_nodes=nn)
    r = o.schedule(pod)
    assert r["status"][0] == abi.KS_S_SCHEDULED and len(mask_cpus(o.fetch_cpusets(1)[0])) == 16
    o.close()
    pod.req_memory[:] = 1 << 30
    o = Oracle(cfg, nodes, cpu_state=st, numa_nodes=nn)
    assert o.schedule(pod)["status"][0] != abi.KS_S_SCHEDULED
    o.close()
    cfg, nodes, st, pod, nn = policy_bind_cluster((2, 1, 4, 2), allocated=[0], bind=abi.KS_CPU_BIND_FULL_PCPUS,
                                                  required=True, cpu_milli=14000,
                                                  policy=abi.KS_NUMA_POLICY_BEST_EFFORT)
    pod.req_memory[:] = 0
    o = Oracle(cfg, nodes, cpu_state=st, numa_nodes=nn)
    r = o.schedule(pod)
    # 14 CPUs = 7 cores: NUMA 0 keeps cores 1-3 (6 CPUs), NUMA 1 all 4 cores (8): split 3 + 4 cores ... 6 + 8 = 14
    assert r["status"][0] == abi.KS_S_SCHEDULED
    got = mask_cpus(o.fetch_cpusets(1)[0])
    assert len(got) == 14 and 0 not in got and 1 not in got
    o.close()


def test_label_makes_plain_pod_cpu_bind():
    """a whole-CPU pod without a cpuset request on a FullPCPUsOnly node gets whole cores, counted in the node's cpuset
    CPUs; the same pod on an unlabelled node gets none"""
    for label, want in ((abi.KS_NODE_CPU_BIND_FULL_PCPUS_ONLY, 4), (0, 0)):
        cfg, nodes, st, pod = bind_policy_cluster((2, 1, 4, 2), allocated=[1], label=label, cpu_milli=4000)
        o = Oracle(cfg, nodes, cpu_state=st)
        r = o.schedule(pod)
        assert r["status"][0] == abi.KS_S_SCHEDULED
        got = mask_cpus(o.fetch_cpusets(1)[0])
        assert len(got) == want
        if want:
            assert 0 not in got and 1 not in got  # core 0 is not whole
        o.close()


def test_spread_label_takes_one_cpu_per_core():
    cfg, nodes, st, pod = bind_policy_cluster((2, 1, 4, 2), allocated=[0], label=abi.KS_NODE_CPU_BIND_SPREAD_BY_PCPUS,
                                              cpu_milli=3000, bind=abi.KS_CPU_BIND_FULL_PCPUS)
    o = Oracle(cfg, nodes, cpu_state=st)
    r = o.schedule(pod)
    assert r["status"][0] == abi.KS_S_SCHEDULED
    got = mask_cpus(o.fetch_cpusets(1)[0])
    assert len({c // 2 for c in got}) == 3  # three distinct cores (CPU ids are core-major)
    o.close()


def test_trial_allocate_is_a_core_count():
    """the device path's count form of the required trial Allocate: FullPCPUs fits iff whole cores x CPUsPerCore >=
    needed, SpreadByPCPUs iff cores with an available CPU >= needed (random allocations, 2-thread cores)"""
    rng = np.random.default_rng(5)
    for _ in range(150):
        taken = sorted(rng.choice(16, int(rng.integers(0, 16)), replace=False).tolist())
        bind = int(rng.choice([abi.KS_CPU_BIND_FULL_PCPUS, abi.KS_CPU_BIND_SPREAD_BY_PCPUS]))
        need = int(rng.integers(1, 9)) * (2 if bind == abi.KS_CPU_BIND_FULL_PCPUS else 1)
        cfg, nodes, st, pod = bind_policy_cluster((2, 1, 4, 2), allocated=taken, cpu_milli=need * 1000, bind=bind,
                                                  required=True)
        nodes.alloc_milli_cpu[:] = 64000  # the Fit plugin never decides
        free = [c for c in range(16) if c not in taken]
        full = sum(1 for k in range(8) if 2 * k in free and 2 * k + 1 in free)
        anyc = len({c // 2 for c in free})
        fits = (full * 2 >= need) if bind == abi.KS_CPU_BIND_FULL_PCPUS else (anyc >= need)
        o = Oracle(cfg, nodes, cpu_state=st)
        assert (int(o.eval_pod(pod)[0][0]) == 0) == fits, (taken, bind, need)
        o.close()


def test_c3_bind_oracle_runs():
    w = synth.c3_bind(n_nodes=150, n_pods=400)
    o = Oracle(w.cfg, w.nodes.copy(), **w.tables())
    r = o.schedule(w.pods)
    lab = (w.nodes.numa_flags >> abi.KS_NUMA_CPU_BIND_SHIFT) & 3
    ok = r["status"] == abi.KS_S_SCHEDULED
    cs = o.fetch_cpusets(w.pods.n)
    plain = (w.pods.flags & abi.KS_POD_CPU_BIND) == 0
    on_lab = ok & plain & (lab[np.maximum(r["node"], 0)] > 0)
    assert on_lab.sum() > 20
    for i in np.nonzero(on_lab)[0]:
        assert len(mask_cpus(cs[i])) == w.pods.req_milli_cpu[i] // 1000
    o.close()
