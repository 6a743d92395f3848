"""Upstream NodeResourcesBalancedAllocation (kube-scheduler v1.24.15 noderesources/balanced_allocation.go, the v1beta2
default profile's plugin; not on disk, so parity is unpinned against reference fixtures): the C oracle against a
Python restatement of balancedResourceScorer (useRequested = true) and hand-worked cases.  CPU only."""
import numpy as np
import pytest

from koordinator_amd import abi, synth
from koordinator_amd.config import CPU, MEMORY, NodeResourcesBalancedAllocationArgs, SchedulerProfile
from numa_util import nodes_of, pod_of
from oracle.oracle import Oracle

GI = 1 << 30


def balanced_ref(alloc, requested, pod, resources=(CPU, MEMORY)):
    """balancedResourceScorer over (Requested + pod request) / Allocatable; Python floats are IEEE f64 like Go's"""
    fr = []
    for r in resources:
        if alloc[r] == 0:
            continue
        f = float(requested[r] + pod[r]) / float(alloc[r])
        fr.append(1.0 if f > 1 else f)
    std = abs((fr[0] - fr[1]) / 2) if len(fr) == 2 else 0.0
    return int((1 - std) * 100)


def bal_only(resources=(CPU, MEMORY)):
    return SchedulerProfile(fit=None, loadaware=None,
                            balanced=NodeResourcesBalancedAllocationArgs(resources={r: 1 for r in resources})).to_ks_config()


def node(acpu, amem, rcpu, rmem):
    return dict(alloc_milli_cpu=acpu, alloc_memory=amem, req_milli_cpu=rcpu, req_memory=rmem, ratio=0.0, cpuset_cpus=0)


CASES = [
    # (node, pod, want): fractions 0.5 / 0.375 -> std 0.0625 -> int64(93.75) = 93
    (node(4000, 8 * GI, 1000, 2 * GI), {"cpu": 1000, "memory": 1 * GI}, 93),
    # balanced: 0.5 / 0.5 -> 100
    (node(4000, 8 * GI, 1000, 2 * GI), {"cpu": 1000, "memory": 2 * GI}, 100),
    # over-committed cpu is capped at 1: 1 / 0.25 -> std 0.375 -> 62
    (node(4000, 8 * GI, 4000, 1 * GI), {"cpu": 500, "memory": 1 * GI}, 62),
    # zero cpu allocatable: one fraction -> std 0 -> 100
    (node(0, 8 * GI, 0, 7 * GI), {"cpu": 0, "memory": 1 * GI}, 100),
    # the pod asks for nothing: the node's own balance, 0.75 / 0.125 -> std 0.3125 -> 68
    (node(8000, 16 * GI, 6000, 2 * GI), {"cpu": 0, "memory": 0}, 68),
    # thirds: 1/3 and 2/3 are inexact in f64; std = |1/3 - 2/3| / 2 -> (1 - 0.1666..) * 100 = 83.33 -> 83
    (node(3000, 3 * GI, 0, 1 * GI), {"cpu": 1000, "memory": 1 * GI}, 83),
]


@pytest.mark.parametrize("i", range(len(CASES)))
def test_balanced_cases(i):
    n, p, want = CASES[i]
    alloc = {CPU: n["alloc_milli_cpu"], MEMORY: n["alloc_memory"]}
    req = {CPU: n["req_milli_cpu"], MEMORY: n["req_memory"]}
    assert balanced_ref(alloc, req, {CPU: p["cpu"], MEMORY: p["memory"]}) == want
    o = Oracle(bal_only(), nodes_of([n]))
    r, s, t = o.eval_pod(pod_of(p))
    assert r[0] == 0 and s[0, abi.KS_SCORE_BALANCED] == want and t[0] == want


def test_single_resource_lists():
    n, p, _ = CASES[0]
    for res in ((CPU,), (MEMORY,)):
        o = Oracle(bal_only(res), nodes_of([n]))
        _, s, _ = o.eval_pod(pod_of(p))
        assert s[0, abi.KS_SCORE_BALANCED] == 100  # one fraction: std 0


def test_oracle_matches_restatement_on_random_nodes():
    rng = np.random.default_rng(3)
    nodes = synth.make_nodes(400, rng)
    pods = synth.make_pods(30, rng)
    o = Oracle(SchedulerProfile(balanced=NodeResourcesBalancedAllocationArgs(), balanced_weight=2).to_ks_config(), nodes)
    for i in range(pods.n):
        r, s, _ = o.eval_pod(pods.rows([i]))
        for n in range(nodes.n):
            if r[n]:
                assert s[n, abi.KS_SCORE_BALANCED] == 0
                continue
            want = balanced_ref({CPU: int(nodes.alloc_milli_cpu[n]), MEMORY: int(nodes.alloc_memory[n])},
                                {CPU: int(nodes.req_milli_cpu[n]), MEMORY: int(nodes.req_memory[n])},
                                {CPU: int(pods.req_milli_cpu[i]), MEMORY: int(pods.req_memory[i])})
            assert s[n, abi.KS_SCORE_BALANCED] == want, (i, n)


def test_unsupported_resources_refused():
    from koordinator_amd.config import ValidationError

    with pytest.raises(ValidationError):
        SchedulerProfile(balanced=NodeResourcesBalancedAllocationArgs(resources={"ephemeral-storage": 1})).to_ks_config()
