"""NUMA topology policies (SURVEY a24 hints / a25 topology manager) on the CPU oracle, pinned by the
reference's TestNUMANodeScore and TestAllocateDistributeEvenly tables."""
import numpy as np
import pytest

from koordinator_amd import abi
from numa_policy_util import G, distribute_case, numa_profile, score_case
from oracle.oracle import Oracle


@pytest.mark.parametrize("c", G["score"], ids=[c["name"] for c in G["score"]])
def test_numa_node_score_golden(c):
    nodes, nn, pod = score_case(c)
    o = Oracle(numa_profile(), nodes, numa_nodes=nn)
    reasons, scores, _ = o.eval_pod(pod)
    assert reasons.tolist() == [0] * nodes.n
    assert scores[:, abi.KS_SCORE_NUMA].tolist() == c["want"]


@pytest.mark.parametrize("c", [c for c in G["distribute"] if c["end_to_end"]],
                         ids=[c["name"] for c in G["distribute"] if c["end_to_end"]])
def test_distribute_evenly_golden(c):
    nodes, nn, pod = distribute_case(c)
    o = Oracle(numa_profile(), nodes, numa_nodes=nn)
    r = o.schedule(pod)
    if not c["want_ok"]:
        assert r["status"][0] == abi.KS_S_UNSCHEDULABLE
        reasons, _, _ = o.eval_pod(pod)
        assert reasons[0] & (abi.KS_R_NUMA_AFFINITY | abi.KS_R_NUMA_INSUFFICIENT)
        return
    assert r["status"][0] == abi.KS_S_SCHEDULED
    used_cpu, _ = o.read_numa_nodes()
    assert (used_cpu[0, :2] - np.asarray(c["used_cpu_milli"])).tolist() == c["want_cpu_milli"]


def test_single_numa_rejects_pod_wider_than_a_numa_node():
    c = dict(G["score"][0])
    c["pod"] = {"cpu": 60, "memory_gi": 40}  # > 52 CPUs of one NUMA node, < 104 of the machine
    nodes, nn, pod = score_case(c)
    o = Oracle(numa_profile(), nodes, numa_nodes=nn)
    reasons, _, _ = o.eval_pod(pod)
    assert reasons[0] == abi.KS_R_NUMA_AFFINITY
    assert reasons[1] == 0  # node 2 has one 64-CPU NUMA node


def test_missing_numa_resources():
    c = dict(G["score"][0])
    nodes, nn, pod = score_case(c)
    nn.count[1] = 0
    o = Oracle(numa_profile(), nodes, numa_nodes=nn)
    reasons, _, _ = o.eval_pod(pod)
    assert reasons[1] == abi.KS_R_NUMA_MISSING


def test_oracle_random_policy_cluster_runs():
    from koordinator_amd import synth
    from koordinator_amd.config import CPU, MEMORY, NodeNUMAResourceArgs

    rng = np.random.Generator(np.random.PCG64(7))
    nodes = synth.make_nodes(200, rng)
    nn = synth.make_numa_nodes(nodes, rng)
    pods = synth.make_pods(400, rng)
    p = synth.koord_profile()
    p.numa = NodeNUMAResourceArgs(resources={CPU: 1, MEMORY: 1})
    o = Oracle(p.to_ks_config(), nodes, nthreads=4, numa_nodes=nn)
    r = o.schedule(pods)
    assert (r["status"] == 0).sum() > 300
    used, _ = o.read_numa_nodes()
    assert (used > nn.used_cpu).any()
