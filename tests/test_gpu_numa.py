"""GPU parity for NodeNUMAResource (SURVEY a21-a23 on topology-policy-None nodes; cpuset pods in test_gpu_cpuset.py):
the golden tables through the HIP library, and whole-queue scheduling vs the oracle with
amplified CPUs and cpuset-held CPUs on the nodes, alone and with Fit + LoadAware + Reservation."""
import numpy as np
import pytest

from helpers import assert_same_results, assert_same_state
from koordinator_amd import abi, synth
from koordinator_amd.config import CPU, MEMORY, NodeNUMAResourceArgs
from numa_util import G, nodes_of, numa_only, pod_of

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def runtime():
    from koordinator_amd import runtime as rt

    rt.lib()
    return rt


@pytest.mark.parametrize("c", G["filter"], ids=[c["name"] for c in G["filter"]])
def test_golden_filter(runtime, c):
    ev = runtime.Evaluator(numa_only(), nodes_of([c["node"]]))
    reasons, _, _ = ev.eval_pod(pod_of(c["pod"]))
    assert (reasons[0] == 0) == c["want_ok"]
    if not c["want_ok"]:
        assert reasons[0] == abi.KS_R_NUMA_AMPLIFIED_CPU
    ev.close()


@pytest.mark.parametrize("c", G["score"], ids=[c["name"] for c in G["score"]])
def test_golden_score(runtime, c):
    ev = runtime.Evaluator(numa_only(c["strategy"]), nodes_of(c["nodes"]))
    _, scores, total = ev.eval_pod(pod_of(c["pod"]))
    assert scores[:, abi.KS_SCORE_NUMA].tolist() == c["want"]
    assert total.tolist() == c["want"]
    ev.close()


def numa_nodes(n, rng, base=None):
    nodes = base if base is not None else synth.make_nodes(n, rng)
    nodes.numa_cpu_amplification[:] = rng.choice(np.array([0.0, 1.0, 1.25, 1.5, 2.0, 3.0]), n)
    amp = nodes.numa_cpu_amplification > 1
    # allocatable advertised amplified (the NodeResource controller), cpuset pods hold some CPUs
    nodes.alloc_milli_cpu[amp] = np.ceil(nodes.alloc_milli_cpu[amp] * nodes.numa_cpu_amplification[amp]).astype(np.int64)
    nodes.numa_cpuset_cpus[:] = np.where(rng.random(n) < 0.5, rng.integers(0, 24, n), 0)
    nodes.numa_flags[:] = np.where(rng.random(n) < 0.02, abi.KS_NUMA_INVALID_RATIO, 0)
    return nodes


def prof_with_numa(p, strategy="LeastAllocated", weight=1):
    p.numa = NodeNUMAResourceArgs(strategy=strategy, resources={CPU: 1, MEMORY: 1})
    p.numa_weight = weight
    return p


def check(runtime, oracle_lib, p, nodes, pods, rs=None, label=""):
    cfg = p.to_ks_config()
    ev = runtime.Evaluator(cfg, nodes.copy(), reservations=rs.copy() if rs is not None else None)
    got = ev.schedule(pods)
    orc = oracle_lib.Oracle(cfg, nodes.copy(), nthreads=8, reservations=rs.copy() if rs is not None else None)
    want = orc.schedule(pods)
    assert_same_results(got, want, label)
    assert np.array_equal(got["reservation"], want["reservation"]), label
    assert_same_state(ev.read_nodes(), orc.read_nodes(), label)
    ev.close()
    orc.close()
    return got


def test_eval_debug_with_numa(runtime, oracle_lib):
    rng = np.random.Generator(np.random.PCG64(31))
    nodes = numa_nodes(600, rng)
    pods = synth.make_pods(40, rng)
    pods.req_milli_cpu[::7] = 0
    for p in (prof_with_numa(synth.koord_profile()), prof_with_numa(synth.koord_profile(), "MostAllocated", 2)):
        cfg = p.to_ks_config()
        ev = runtime.Evaluator(cfg, nodes)
        orc = oracle_lib.Oracle(cfg, nodes)
        for i in range(pods.n):
            one = pods.rows([i])
            r_g, s_g, t_g = ev.eval_pod(one)
            r_o, s_o, t_o = orc.eval_pod(one)
            assert np.array_equal(r_g, r_o), f"pod {i}: reasons"
            assert np.array_equal(s_g, s_o), f"pod {i}: scores"
            assert np.array_equal(t_g, t_o), f"pod {i}: totals"
        ev.close()
        orc.close()


@pytest.mark.parametrize("strategy,batch", [("LeastAllocated", 64), ("MostAllocated", 64), ("LeastAllocated", 1)])
def test_schedule_with_numa(runtime, oracle_lib, strategy, batch):
    rng = np.random.Generator(np.random.PCG64(33))
    nodes = numa_nodes(1500, rng)
    pods = synth.make_pods(2000, rng)
    got = check(runtime, oracle_lib, prof_with_numa(synth.koord_profile(batch_pods=batch), strategy), nodes, pods,
                label=f"numa-{strategy}-{batch}")
    assert (got["status"] == 0).sum() > 1000


def test_schedule_numa_with_reservations(runtime, oracle_lib):
    rng = np.random.Generator(np.random.PCG64(34))
    w = synth.c4(n_nodes=1500, n_reservations=3500, n_pods=1500)
    numa_nodes(w.nodes.n, rng, base=w.nodes)
    got = check(runtime, oracle_lib, prof_with_numa(w.profile), w.nodes, w.pods, w.reservations, "numa+rsv")
    assert (got["reservation"] >= 0).sum() > 100


def test_cpu_bind_pod_needs_policy(runtime):
    """KS_POD_CPU_BIND without a bind policy in ks_pod_cols.cpu_bind is an invalid argument"""
    rng = np.random.Generator(np.random.PCG64(35))
    nodes = numa_nodes(64, rng)
    pods = synth.make_pods(4, rng)
    pods.flags[1] |= abi.KS_POD_CPU_BIND
    pods.req_milli_cpu[1] = 4000
    ev = runtime.Evaluator(prof_with_numa(synth.koord_profile()).to_ks_config(), nodes)
    with pytest.raises(runtime.KsError) as ei:
        ev.schedule(pods)
    assert ei.value.rc == abi.KS_EINVAL
    ev.close()
