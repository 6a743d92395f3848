"""NodeNUMAResource (non-cpuset pods on topology-policy-None nodes): the C oracle
against the reference's TestFilterWithAmplifiedCPUs / TestScoreWithAmplifiedCPUs tables."""
import pytest

from koordinator_amd import abi
from numa_util import G, nodes_of, numa_only, pod_of
from oracle.oracle import Oracle


@pytest.mark.parametrize("c", G["filter"], ids=[c["name"] for c in G["filter"]])
def test_filter_amplified_cpus(c):
    o = Oracle(numa_only(), nodes_of([c["node"]]))
    reasons, _, _ = o.eval_pod(pod_of(c["pod"]))
    assert (reasons[0] == 0) == c["want_ok"]
    if not c["want_ok"]:
        assert reasons[0] == abi.KS_R_NUMA_AMPLIFIED_CPU


@pytest.mark.parametrize("c", G["score"], ids=[c["name"] for c in G["score"]])
def test_score_amplified_cpus(c):
    o = Oracle(numa_only(c["strategy"]), nodes_of(c["nodes"]))
    reasons, scores, total = o.eval_pod(pod_of(c["pod"]))
    assert scores[:, abi.KS_SCORE_NUMA].tolist() == c["want"]
    assert total.tolist() == c["want"]


def test_invalid_ratio_rejects_cpu_pods_only():
    spec = dict(G["filter"][2]["node"])
    nodes = nodes_of([spec])
    nodes.numa_flags[:] = abi.KS_NUMA_INVALID_RATIO
    o = Oracle(numa_only(), nodes)
    r, _, _ = o.eval_pod(pod_of({"cpu": 1000, "memory": 0}))
    assert r[0] == abi.KS_R_NUMA_INVALID_RATIO
    r, _, _ = o.eval_pod(pod_of({"cpu": 0, "memory": 1 << 30}))
    assert r[0] == 0
