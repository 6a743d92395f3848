"""GPU parity for NUMA topology policies (SURVEY a24 hints, a25 topology manager): the reference's
TestNUMANodeScore table through the HIP library, and whole-queue scheduling against the oracle on clusters
where half of the nodes carry a best-effort / restricted / single-numa-node policy: placements, scores,
filter reasons, per-plugin scores, Requested and the NUMA nodes' allocatedResources after every commit."""
import numpy as np
import pytest

from helpers import assert_same_results, assert_same_state
from koordinator_amd import abi, synth
from koordinator_amd.config import CPU, MEMORY, NodeNUMAResourceArgs
from numa_policy_util import G, distribute_case, numa_profile, score_case

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def runtime():
    from koordinator_amd import runtime as rt

    rt.lib()
    return rt


@pytest.mark.parametrize("c", G["score"], ids=[c["name"] for c in G["score"]])
def test_numa_node_score_golden(runtime, c):
    nodes, nn, pod = score_case(c)
    ev = runtime.Evaluator(numa_profile(), nodes, numa_nodes=nn)
    reasons, scores, _ = ev.eval_pod(pod)
    assert reasons.tolist() == [0] * nodes.n
    assert scores[:, abi.KS_SCORE_NUMA].tolist() == c["want"]
    ev.close()


@pytest.mark.parametrize("c", [c for c in G["distribute"] if c["end_to_end"]],
                         ids=[c["name"] for c in G["distribute"] if c["end_to_end"]])
def test_distribute_golden(runtime, c):
    nodes, nn, pod = distribute_case(c)
    ev = runtime.Evaluator(numa_profile(), nodes, numa_nodes=nn)
    r = ev.schedule(pod)
    if not c["want_ok"]:
        assert r["status"][0] == abi.KS_S_UNSCHEDULABLE
        return
    used_cpu, _ = ev.read_numa_nodes()
    assert (used_cpu[0, :2] - np.asarray(c["used_cpu_milli"])).tolist() == c["want_cpu_milli"]
    ev.close()


def policy_cluster(seed, n_nodes, n_pods, numa_strategy="LeastAllocated", strategy="LeastAllocated"):
    rng = np.random.Generator(np.random.PCG64(seed))
    nodes = synth.make_nodes(n_nodes, rng)
    ratio = rng.choice(np.array([0.0, 1.0, 1.5]), n_nodes)
    cores = nodes.alloc_milli_cpu // 1000
    amp = ratio > 1
    nodes.numa_cpu_amplification[:] = ratio
    nodes.alloc_milli_cpu[amp] = np.ceil(nodes.alloc_milli_cpu[amp] * ratio[amp]).astype(np.int64)
    nn = synth.make_numa_nodes(nodes, rng, cores=cores)
    nn.cpuset_cpus[:, :] = np.where(nn.used_present == 1, rng.integers(0, 4, nn.cpuset_cpus.shape), 0)
    pods = synth.make_pods(n_pods, rng)
    p = synth.koord_profile()
    p.numa = NodeNUMAResourceArgs(strategy=strategy, resources={CPU: 1, MEMORY: 1}, numa_scoring_strategy=numa_strategy)
    return p.to_ks_config(), nodes, nn, pods


def run_pair(runtime, oracle_lib, cfg, nodes, nn, pods, label):
    ev = runtime.Evaluator(cfg, nodes.copy(), numa_nodes=nn.copy())
    got = ev.schedule(pods)
    orc = oracle_lib.Oracle(cfg, nodes.copy(), nthreads=8, numa_nodes=nn.copy())
    want = orc.schedule(pods)
    assert_same_results(got, want, label)
    assert_same_state(ev.read_nodes(), orc.read_nodes(), label)
    for a, b in zip(ev.read_numa_nodes(), orc.read_numa_nodes()):
        assert np.array_equal(a, b), f"{label}: NUMA used differs"
    ev.close()
    orc.close()
    return got


@pytest.mark.parametrize("seed,numa_strategy,strategy", [(61, "LeastAllocated", "LeastAllocated"),
                                                         (62, "MostAllocated", "LeastAllocated"),
                                                         (63, "LeastAllocated", "MostAllocated")])
def test_schedule_numa_policies(runtime, oracle_lib, seed, numa_strategy, strategy):
    cfg, nodes, nn, pods = policy_cluster(seed, 800, 1500, numa_strategy, strategy)
    got = run_pair(runtime, oracle_lib, cfg, nodes, nn, pods, f"numa-policy-{seed}")
    assert (got["status"] == 0).sum() > 1000


def test_schedule_numa_policies_tight(runtime, oracle_lib):
    """few nodes: NUMA allocations fill up, single-numa-node and restricted nodes start refusing pods"""
    cfg, nodes, nn, pods = policy_cluster(64, 60, 1200)
    got = run_pair(runtime, oracle_lib, cfg, nodes, nn, pods, "numa-policy-tight")
    assert (got["status"] != 0).sum() > 0


def test_eval_debug_numa_policies(runtime, oracle_lib):
    cfg, nodes, nn, pods = policy_cluster(65, 500, 40)
    ev = runtime.Evaluator(cfg, nodes, numa_nodes=nn)
    orc = oracle_lib.Oracle(cfg, nodes, numa_nodes=nn)
    for i in range(pods.n):
        one = pods.rows([i])
        r_g, s_g, t_g = ev.eval_pod(one)
        r_o, s_o, t_o = orc.eval_pod(one)
        assert np.array_equal(r_g, r_o), f"pod {i}: reasons"
        assert np.array_equal(s_g, s_o), f"pod {i}: scores"
        assert np.array_equal(t_g, t_o), f"pod {i}: totals"
    ev.close()
    orc.close()


def test_numa_policy_checkpoint_restore(runtime):
    cfg, nodes, nn, pods = policy_cluster(66, 200, 600)
    ev = runtime.Evaluator(cfg, nodes, numa_nodes=nn)
    ev.stage(pods)
    ev.checkpoint()
    outs = []
    for _ in range(2):
        ev.restore()
        ev.schedule_staged()
        outs.append((ev.fetch(), ev.read_numa_nodes()[0]))
    for k in ("node", "status", "score"):
        assert np.array_equal(outs[0][0][k], outs[1][0][k])
    assert np.array_equal(outs[0][1], outs[1][1])
    ev.close()
