"""The ElasticQuota PostFilter restated in the CPU oracle (ko_preempt), checked on hand-worked cases.

Reference: pkg/scheduler/plugins/elasticquota/plugin.go:263-321 (AddPod / RemovePod / PostFilter), preempt.go
(SelectVictimsOnNode :113-217, filterPodsWithPDBViolation :223-265, canPreempt :283-294, PodEligibleToPreemptOthers
:60-97) and upstream kube-scheduler v1.24 framework/preemption (Preempt, DryRunPreemption, pickOneNodeForPreemption),
which is not on disk: the expected values below follow those functions step by step (comments give the steps).  The
quota arithmetic of AddPod / RemovePod is pinned by the reference's own TestPlugin_AddPod / TestPlugin_RemovePod
(plugin_test.go:950-1051: used 10 + request 1 = 11, 10 - 1 = 9 per dimension), reproduced through a dry run in
test_add_remove_tables.
"""
import numpy as np
import pytest

from helpers import profile
from koordinator_amd import abi
from koordinator_amd.cluster import NodePodTable, NodeTable, PodTable, QuotaTable

GI = 1 << 30
CPU, MEM = 0, 1


def cluster(n_nodes, alloc_cpu=4000, alloc_mem=16 * GI, allowed=110):
    t = NodeTable(n_nodes)
    t.alloc_milli_cpu[:] = alloc_cpu
    t.alloc_memory[:] = alloc_mem
    t.alloc_ephemeral[:] = 100 * GI
    t.allowed_pods[:] = allowed
    return t


def running(nodes, specs, npdb=0, allowed=()):
    """specs: (node, priority, start, cpu, quota[, flags[, pdb]]); memory 1 GiB each.  Sets NodeInfo.Requested."""
    t = NodePodTable(len(specs), npdb)
    for i, s in enumerate(specs):
        node, prio, start, cpu, quota = s[:5]
        t.node[i], t.priority[i], t.start_time[i], t.quota[i] = node, prio, start, quota
        t.flags[i] = s[5] if len(s) > 5 else abi.KS_NPOD_IN_QUOTA
        t.pdb[i] = s[6] if len(s) > 6 else -1
        t.req[0, i], t.req[1, i] = cpu, GI
        t.quota_req[CPU, i], t.quota_req[MEM, i] = cpu, GI
    t.pdb_allowed[:] = list(allowed) if allowed else 0
    nodes.req_milli_cpu[:] = np.bincount(t.node, weights=t.req[0], minlength=nodes.n).astype(np.int64)
    nodes.req_memory[:] = np.bincount(t.node, weights=t.req[1], minlength=nodes.n).astype(np.int64)
    nodes.pod_count[:] = np.bincount(t.node, minlength=nodes.n).astype(np.int32)
    return t


def quotas(t, nq=2, limit_cpu=1 << 40):
    q = QuotaTable(nq)
    q.limit_mask[:] = (1 << CPU) | (1 << MEM)
    q.limit[CPU] = limit_cpu
    q.limit[MEM] = 1 << 50
    inq = (t.flags & abi.KS_NPOD_IN_QUOTA) != 0
    for d in (CPU, MEM):
        q.used[d] = np.bincount(t.quota[inq], weights=t.quota_req[d][inq].astype(np.float64), minlength=nq).astype(np.int64)
    return q


def preemptor(cpu, quota=0, mem=GI):
    p = PodTable(1)
    p.req_milli_cpu[0], p.req_memory[0] = cpu, mem
    p.nonzero_milli_cpu[0], p.nonzero_memory[0] = cpu, mem
    p.flags[0] = abi.KS_POD_PROD
    p.quota[0] = quota
    p.quota_req[CPU, 0], p.quota_req[MEM, 0] = cpu, mem
    p.quota_mask[0] = (1 << CPU) | (1 << MEM)
    return p


def run(nodes, t, q, pod, prio, **kw):
    from oracle.oracle import Oracle

    o = Oracle(profile(quota=True).to_ks_config(), nodes.copy(), q.copy())
    try:
        o.load_node_pods(t)
        return o.preempt(pod, prio, node_status=True, **kw)
    finally:
        o.close()


# node 0 full (4 x 1000m): p0, p1 preemptible (priority 100, quota 0), p2 higher priority, p3 another quota
BASE = [(0, 100, 1, 1000, 0), (0, 100, 2, 1000, 0), (0, 5000, 3, 1000, 0), (0, 100, 4, 1000, 1)]


def test_both_victims_needed():
    # remove p0, p1 (canPreempt) -> 2000m free >= 1500m; reprieve p0 (earlier start first): 1000m free < 1500m -> victim;
    # p1 likewise -> victims [p0, p1]
    nodes = cluster(1)
    t = running(nodes, BASE)
    r = run(nodes, t, quotas(t), preemptor(1500), 1000)
    assert r["status"] == abi.KS_P_NOMINATED and r["node"] == 0
    assert list(r["victims"]) == [0, 1] and r["num_pdb_violations"] == 0 and r["candidates"] == 1


def test_more_important_pod_is_reprieved():
    # 500m: p0 reprieved (1000m free), p1 not (0m free) -> victims [p1]
    nodes = cluster(1)
    t = running(nodes, BASE)
    r = run(nodes, t, quotas(t), preemptor(500), 1000)
    assert list(r["victims"]) == [1]


def test_quota_branch_makes_victims():
    # quota 0 used 3000m (p0, p1, p2), limit 2000m: after the removal used = 1000m; reprieve p0: fits, used 2000m,
    # 2000 + 500 > 2000 -> removed again, a victim; p1 the same -> victims [p0, p1]
    nodes = cluster(1)
    t = running(nodes, BASE)
    r = run(nodes, t, quotas(t, limit_cpu=2000), preemptor(500), 1000)
    assert r["status"] == abi.KS_P_NOMINATED and list(r["victims"]) == [0, 1]


def test_fit_and_quota_failure_is_an_error():
    # 1500m with limit 2000m: reprieve p0 fails the fit (removed, victim), then 1000 + 1500 > 2000 removes it a second
    # time: NodeInfo.RemovePod errors -> the node's dry run is an Error, no candidate -> Error status
    nodes = cluster(1)
    t = running(nodes, BASE)
    r = run(nodes, t, quotas(t, limit_cpu=2000), preemptor(1500), 1000)
    assert r["status"] == abi.KS_P_ERROR and r["node_status"][0] == abi.KS_PN_ERROR


def test_pdb_violating_victims_are_reprieved_first():
    # p1 in a budget with DisruptionsAllowed 0 -> violating; violating first: p1 reprieved (1000m free >= 500m), then p0
    # -> victims [p0], no violation counted (p1 fit)
    nodes = cluster(1)
    specs = [BASE[0], (0, 100, 2, 1000, 0, abi.KS_NPOD_IN_QUOTA, 0), BASE[2], BASE[3]]
    t = running(nodes, specs, npdb=1, allowed=[0])
    r = run(nodes, t, quotas(t), preemptor(500), 1000)
    assert list(r["victims"]) == [0] and r["num_pdb_violations"] == 0
    # 1500m: the violating p1 does not fit back -> a victim with a violation
    r = run(nodes, t, quotas(t), preemptor(1500), 1000)
    assert list(r["victims"]) == [1, 0] and r["num_pdb_violations"] == 1


def test_pdb_budget_shared_in_sorted_order():
    # budget 0 allows 1: of p0, p1 (both in it) the first in MoreImportantPod order keeps the budget, the second violates
    nodes = cluster(1)
    specs = [(0, 100, 2, 1000, 0, abi.KS_NPOD_IN_QUOTA, 0), (0, 100, 1, 1000, 0, abi.KS_NPOD_IN_QUOTA, 0), BASE[2], BASE[3]]
    t = running(nodes, specs, npdb=1, allowed=[1])
    # sorted: row 1 (start 1), row 0 (start 2); row 0 violates -> reprieved first at 500m
    r = run(nodes, t, quotas(t), preemptor(500), 1000)
    assert list(r["victims"]) == [1]


def test_pod_matching_two_budgets():
    # filterPodsWithPDBViolation (preempt.go:232-257) loops over every PDB: each match decrements that budget, and the pod
    # violates if any goes below 0.  Budget 0 allows 1 (p0, p1), budget 1 allows 0 (p1 only).
    nodes = cluster(1)
    specs = [(0, 100, 1, 1000, 0, abi.KS_NPOD_IN_QUOTA, 0), (0, 100, 2, 1000, 0, abi.KS_NPOD_IN_QUOTA, 0), BASE[2], BASE[3]]
    t = running(nodes, specs, npdb=2, allowed=[1, 0])
    t.pdb_more[0, 1] = 1
    # sorted p0 (start 1), p1: budget 0 -> 0 after p0, -1 after p1; budget 1 -> -1 after p1.  Only p1 violates.  At 1500m
    # p1 is reprieved first and does not fit (1000m free): a victim with a violation; then p0 likewise.
    r = run(nodes, t, quotas(t), preemptor(1500), 1000)
    assert list(r["victims"]) == [1, 0] and r["num_pdb_violations"] == 1
    # p1 in budget 0's DisruptedPods (the shim drops budget 0 for it) but matching budget 1 (allowed 0): still violating
    t.pdb[1], t.pdb_more[0, 1] = 1, -1
    r = run(nodes, t, quotas(t), preemptor(1500), 1000)
    assert list(r["victims"]) == [1, 0] and r["num_pdb_violations"] == 1
    # budget 1 allows 1: nobody violates; sorted order p0 then p1, both victims, no violation
    t.pdb_allowed[1] = 1
    r = run(nodes, t, quotas(t), preemptor(1500), 1000)
    assert list(r["victims"]) == [0, 1] and r["num_pdb_violations"] == 0


def test_non_preemptible_and_other_quota_are_not_victims():
    nodes = cluster(1)
    specs = [(0, 100, 1, 1000, 0, abi.KS_NPOD_IN_QUOTA | abi.KS_NPOD_NONPREEMPTIBLE), (0, 100, 2, 1000, 1),
             (0, 5000, 3, 1000, 0), (0, 5000, 4, 1000, 0)]
    t = running(nodes, specs)
    r = run(nodes, t, quotas(t), preemptor(500), 1000)
    assert r["status"] == abi.KS_P_NO_CANDIDATE and r["node_status"][0] == abi.KS_PN_NO_VICTIMS


def test_filter_failing_without_victims():
    # the pod does not fit even with every potential victim gone (2000m free < 2500m)
    nodes = cluster(1)
    t = running(nodes, BASE)
    r = run(nodes, t, quotas(t), preemptor(2500), 1000)
    assert r["status"] == abi.KS_P_NO_CANDIDATE and r["node_status"][0] == abi.KS_PN_FILTER


def test_pick_one_node_order():
    from koordinator_amd import abi as A

    # node 0: one victim in a violated budget; node 1: two victims without violations -> node 1 (fewer violations)
    nodes = cluster(2)
    specs = [(0, 100, 1, 4000, 0, A.KS_NPOD_IN_QUOTA, 0), (1, 100, 2, 2000, 0), (1, 100, 3, 2000, 0)]
    t = running(nodes, specs, npdb=1, allowed=[0])
    r = run(nodes, t, quotas(t), preemptor(3000), 1000)
    assert r["node"] == 1 and r["candidates"] == 2 and list(r["victims"]) == [1, 2]
    # lower priority of the first victim: node 1 (victim priority 100) over node 0 (victim priority 500)
    specs = [(0, 500, 1, 4000, 0), (1, 100, 2, 4000, 0)]
    t = running(nodes, specs)
    r = run(nodes, t, quotas(t), preemptor(3000), 1000)
    assert r["node"] == 1
    # equal first priority, smaller sum (one victim instead of two) -> node 1
    specs = [(0, 100, 1, 2000, 0), (0, 100, 2, 2000, 0), (1, 100, 3, 4000, 0)]
    t = running(nodes, specs)
    r = run(nodes, t, quotas(t), preemptor(3000), 1000)
    assert r["node"] == 1
    # everything equal but the victims' start times: the later earliest start wins (node 0, start 9)
    specs = [(0, 100, 9, 4000, 0), (1, 100, 3, 4000, 0)]
    t = running(nodes, specs)
    r = run(nodes, t, quotas(t), preemptor(3000), 1000)
    assert r["node"] == 0
    # a full tie: the lowest node row
    specs = [(0, 100, 5, 4000, 0), (1, 100, 5, 4000, 0)]
    t = running(nodes, specs)
    r = run(nodes, t, quotas(t), preemptor(3000), 1000)
    assert r["node"] == 0


def test_eligibility_and_unresolvable_nodes():
    nodes = cluster(2)
    specs = BASE + [(1, 100, 5, 4000, 0, abi.KS_NPOD_IN_QUOTA | abi.KS_NPOD_TERMINATING)]
    t = running(nodes, specs)
    q = quotas(t)
    assert run(nodes, t, q, preemptor(500), 1000, flags=abi.KS_PREEMPT_NEVER)["status"] == abi.KS_P_NOT_ELIGIBLE
    # a terminating lower-priority pod of the same quota on the nominated node
    assert run(nodes, t, q, preemptor(500), 1000, nominated_node=1)["status"] == abi.KS_P_NOT_ELIGIBLE
    # ... unless the nominated node's status was UnschedulableAndUnresolvable: then only node 0 is a potential node
    r = run(nodes, t, q, preemptor(500), 1000, nominated_node=1, unresolvable=np.array([0, 1], np.uint8))
    assert r["status"] == abi.KS_P_NOMINATED and r["node"] == 0 and r["potential_nodes"] == 1
    assert r["node_status"][1] == abi.KS_PN_UNRESOLVABLE


def test_add_remove_tables():
    # TestPlugin_RemovePod: used 10 -> RemovePod of a request-1 pod -> 9; TestPlugin_AddPod: 10 + 1 -> 11 (per dimension).
    # One dry run observes both: quota used 10 cores (the victim's 1 core included), limit 9 + 2 cores for a 2-core pod:
    # with the victim removed used is 9 (9 + 2 <= 11 passes the quota), re-added it is 10 (10 + 2 > 11: a victim).
    nodes = cluster(1, alloc_cpu=64000)
    t = running(nodes, [(0, 100, 1, 1000, 0), (0, 5000, 2, 9000, 0)])
    q = quotas(t, limit_cpu=11000)
    assert q.used[CPU, 0] == 10000
    r = run(nodes, t, q, preemptor(2000), 1000)
    assert r["status"] == abi.KS_P_NOMINATED and list(r["victims"]) == [0]
    q.limit[CPU, 0] = 12000  # 10 + 2 <= 12: the re-added pod stays, no victim -> "expected at least one victim" (Error)
    r = run(nodes, t, q, preemptor(2000), 1000)
    assert r["status"] == abi.KS_P_ERROR
