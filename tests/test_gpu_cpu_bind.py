"""GPU parity for node CPU bind policies (the node-cpu-bind-policy label: a whole-CPU pod becomes cpu-bind, a
fractional one fails ErrInvalidRequestedCPUs) and required pod CPU bind policies (the Filter's policy conflict,
SMT alignment and trial Allocate, the allocation's required filter), against the CPU oracle: the reference's
Filter and Allocate cases, whole C3-shaped queues (placements, statuses, scores, minors, per-pod cpusets, CPU
state, node columns), single-pod Filter/Score parity, and the per-pod framework mode with Unreserve."""
import numpy as np
import pytest

from assume_util import assert_states_equal, state
from cpuset_util import allocate_cases, bind_policy_cluster, filter_cases
from helpers import assert_same_results, assert_same_state
from koordinator_amd import abi, synth
from koordinator_amd.cluster import mask_cpus

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def runtime():
    from koordinator_amd import runtime as rt

    rt.lib()
    return rt


@pytest.mark.parametrize("case", filter_cases(), ids=[c[0] for c in filter_cases()])
def test_reference_filter_cases(runtime, case):
    _, label, bind, required, cpu, want = case
    cfg, nodes, st, pod = bind_policy_cluster((2, 1, 4, 2), label=label, cpu_milli=cpu, bind=bind, required=required)
    ev = runtime.Evaluator(cfg, nodes, cpu_state=st)
    # (preferred FullPCPUs requests in split cores included)
    assert int(ev.eval_pod(pod)[0][0]) == want
    ev.close()


@pytest.mark.parametrize("case", allocate_cases(), ids=[c[0] for c in allocate_cases()])
def test_reference_allocate_cases(runtime, case):
    _, bind, allocated, want = case
    cfg, nodes, st, pod = bind_policy_cluster((2, 1, 26, 2), allocated=allocated, bind=bind, required=True)
    ev = runtime.Evaluator(cfg, nodes, cpu_state=st)
    r = ev.schedule(pod)
    if want is None:
        assert r["status"][0] == abi.KS_S_UNSCHEDULABLE
        assert int(ev.eval_pod(pod)[0][0]) == abi.KS_R_NUMA_CPUSET
    else:
        assert r["status"][0] == abi.KS_S_SCHEDULED
        assert mask_cpus(ev.fetch_cpusets(1)[0]) == want
    ev.close()


def check(runtime, oracle_lib, w, label):
    ev = runtime.Evaluator(w.cfg, w.nodes.copy(), **w.tables())
    got = ev.schedule(w.pods)
    orc = oracle_lib.Oracle(w.cfg, w.nodes.copy(), nthreads=8, **w.tables())
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
    assert_same_state(ev.read_nodes(), orc.read_nodes(), label)
    stats = ev.stats()
    ev.close()
    orc.close()
    return got, stats


def bind_stats(w, got):
    lab = (w.nodes.numa_flags >> abi.KS_NUMA_CPU_BIND_SHIFT) & 3
    ok = got["status"] == abi.KS_S_SCHEDULED
    plain = (w.pods.flags & abi.KS_POD_CPU_BIND) == 0
    req = (w.pods.cpu_bind & abi.KS_CPU_BIND_REQUIRED) != 0
    on_lab = ok & (lab[np.maximum(got["node"], 0)] > 0)
    return int((on_lab & plain).sum()), int((ok & req).sum())


@pytest.mark.parametrize("label_frac,required_frac", [(0.4, 0.4), (0.6, 0.0), (0.0, 0.8)],
                         ids=["labels+required", "labels", "required"])
def test_c3_bind_queue(runtime, oracle_lib, label_frac, required_frac):
    w = synth.c3_bind(seed=81, n_nodes=2000, n_pods=4000, label_frac=label_frac, required_frac=required_frac)
    got, stats = check(runtime, oracle_lib, w, f"c3-bind-{label_frac}-{required_frac}")
    plain_on_lab, req = bind_stats(w, got)
    if label_frac:
        assert plain_on_lab > 300, plain_on_lab
    if required_frac:
        assert req > 100, req


def test_c3_bind_tight_nodes(runtime, oracle_lib):
    """few nodes, many pods: whole cores run out, required pods fail the trial Allocate, passes are cut"""
    w = synth.c3_bind(seed=82, n_nodes=60, n_pods=1500, label_frac=0.6, required_frac=0.6)
    got, stats = check(runtime, oracle_lib, w, "c3-bind-tight")
    assert (got["status"] != abi.KS_S_SCHEDULED).sum() > 100


def test_c3_bind_eval_pod_parity(runtime, oracle_lib):
    w = synth.c3_bind(seed=83, n_nodes=400, n_pods=400)
    bind = (w.pods.flags & abi.KS_POD_CPU_BIND) != 0
    req = (w.pods.cpu_bind & abi.KS_CPU_BIND_REQUIRED) != 0
    whole = (w.pods.req_milli_cpu % 1000 == 0) & ~bind
    idx = np.concatenate([np.nonzero(req)[0][:20], np.nonzero(bind & ~req)[0][:15], np.nonzero(whole)[0][:20],
                          np.nonzero(~bind & ~whole)[0][:10]])
    ev = runtime.Evaluator(w.cfg, w.nodes.copy(), **w.tables())
    orc = oracle_lib.Oracle(w.cfg, w.nodes.copy(), **w.tables())
    for i in idx:
        one = w.pods.rows([int(i)])
        r_g, s_g, t_g = ev.eval_pod(one)
        r_o, s_o, t_o = orc.eval_pod(one)
        assert np.array_equal(r_g, r_o), f"pod {i}: reasons {np.nonzero(r_g != r_o)[0][:5]}"
        assert np.array_equal(s_g, s_o), f"pod {i}: scores"
        assert np.array_equal(t_g, t_o), f"pod {i}: totals"
    ev.close()
    orc.close()


def test_c3_bind_assume_unreserve(runtime, oracle_lib):
    """per-pod mode on labelled nodes: ks_assume takes the node's policy, ks_unreserve gives the CPUs (and the core
    counts) back, and a later queue schedules as on the oracle"""
    w = synth.c3_bind(seed=84, n_nodes=200, n_pods=300, label_frac=0.7, required_frac=0.5)
    ev = runtime.Evaluator(w.cfg, w.nodes.copy(), **w.tables())
    orc = oracle_lib.Oracle(w.cfg, w.nodes.copy(), **w.tables())
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
    ev.close()
    orc.close()
