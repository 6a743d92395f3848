"""NodeNUMAResource node CPU bind policies (the node-cpu-bind-policy label) and required pod CPU bind policies on
the CPU oracle: the reference's Filter cases (plugin_test.go:592-760) and required-policy allocations
(resource_manager_test.go:95-330) as known answers, then the semantics the device path relies on (Reserve of a
pod cpu-bind only through the node's policy, count form of the trial Allocate)."""
import numpy as np
import pytest

from cpuset_util import allocate_cases, bind_policy_cluster, filter_cases
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
