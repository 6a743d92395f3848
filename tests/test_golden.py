"""Golden vectors from the reference's own test tables (tests/golden/*.json).

Three layers are pinned against the SAME expected values:
  1. oracle/loadaware_ref.py      object-level restatement of the plugin
  2. koordinator_amd.ingest + oracle/koord_oracle.c   host reduction -> SoA -> C oracle
  3. (tests/test_gpu_golden.py)   host reduction -> SoA -> libkoordgpu.so on the GPU
"""
import json
import os

import numpy as np
import pytest

from koordinator_amd import abi, ingest
from koordinator_amd.cluster import NodeTable, PodTable, QuotaTable
from koordinator_amd.config import SchedulerProfile
from oracle import loadaware_ref as ref

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


FILTER = load("loadaware_filter.json")["cases"]
SCORE = load("loadaware_score.json")["cases"]
EST = load("loadaware_estimator.json")
QUOTA = load("elasticquota_prefilter.json")


def reason_of(bits: int) -> tuple:
    if bits == 0:
        return ("Success", "")
    res = "cpu" if bits & abi.KS_R_LA_CPU else "memory"
    if bits & abi.KS_R_LA_AGGREGATED:
        return ("Unschedulable", f"node(s) {res} aggregated usage exceed threshold")
    return ("Unschedulable", f"node(s) {res} usage exceed threshold")


def want_of(case) -> tuple:
    w = case["want"]
    return (w["status"], w.get("reason", ""))


def filter_lister(case):
    return ingest.lister_from(case.get("listerPods") or [])


def score_lister(case):
    pods = list(case.get("listerPods") or [])
    if case.get("pod"):
        pods.append(case["pod"])
    pods += [a["pod"] for a in case.get("assignedPods") or []]
    return ingest.lister_from(pods)


def build_one(case, lister, enable_filter=True, enable_score=True):
    """ingest one golden case into a 1-node / 1-pod ks_* problem (LoadAware only)."""
    la = ingest.args_from_json(case.get("args") or {})
    prof = SchedulerProfile(fit=None, loadaware=la)
    cfg = prof.to_ks_config()
    cfg.loadaware.enable_filter = 1 if enable_filter else 0
    cfg.loadaware.enable_score = 1 if enable_score else 0
    nodes = NodeTable(1)
    ingest.node_to_columns(nodes, 0, la, case["node"], case.get("nodeMetric"), lister,
                           case.get("assignedPods") or [], now=0)
    nodes.allowed_pods[:] = 110
    pods = ingest.pods_to_table([case.get("pod")])
    return cfg, nodes, pods


# ------------------------------------------------------------- layer 1: object-level restatement

@pytest.mark.parametrize("case", FILTER, ids=[c["name"] for c in FILTER])
def test_ref_filter(case):
    got = ref.filter_node(case.get("args") or {}, case["node"], case.get("nodeMetric"),
                          ingest.lister_from(case.get("listerPods") or []), case.get("pod"), now=0)
    assert got == want_of(case)


@pytest.mark.parametrize("case", SCORE, ids=[c["name"] for c in SCORE])
def test_ref_score(case):
    got = ref.score_node(case.get("args") or {}, case["node"], case.get("nodeMetric"), score_lister(case),
                         case.get("assignedPods") or [], case.get("pod"), now=0)
    assert got == case["want"]["score"]


@pytest.mark.parametrize("case", EST["pods"], ids=[c["name"] for c in EST["pods"]])
def test_ref_estimate_pod(case):
    args = ref.set_defaults({"estimatedScalingFactors": case.get("scalingFactors")})
    assert ref.estimate_pod(args, case["pod"]) == case["want"]


@pytest.mark.parametrize("case", EST["nodes"], ids=[c["name"] for c in EST["nodes"]])
def test_ref_estimate_node(case):
    got = ref.estimate_node(case["node"])
    assert got == {k: ref.quantity(v) for k, v in case["want"].items()}


# ------------------------------------------------------------- layer 2: ingest -> SoA -> C oracle

@pytest.mark.parametrize("case", FILTER, ids=[c["name"] for c in FILTER])
def test_oracle_soa_filter(case, oracle_lib):
    cfg, nodes, pods = build_one(case, filter_lister(case))
    o = oracle_lib.Oracle(cfg, nodes)
    reasons, _, _ = o.eval_pod(pods)
    assert reason_of(int(reasons[0])) == want_of(case)


@pytest.mark.parametrize("case", SCORE, ids=[c["name"] for c in SCORE])
def test_oracle_soa_score(case, oracle_lib):
    cfg, nodes, pods = build_one(case, score_lister(case), enable_filter=False)
    o = oracle_lib.Oracle(cfg, nodes)
    reasons, scores, total = o.eval_pod(pods)
    assert reasons[0] == 0
    assert scores[0, abi.KS_SCORE_LOADAWARE] == case["want"]["score"]
    assert total[0] == case["want"]["score"]


@pytest.mark.parametrize("case", EST["pods"], ids=[c["name"] for c in EST["pods"]])
def test_oracle_estimated_used(case, oracle_lib):
    L = oracle_lib.lib()
    sf = {"cpu": 85, "memory": 70}
    sf.update(case.get("scalingFactors") or {})
    t = ingest.pods_to_table([case["pod"]])
    cpu = L.ko_estimated_used(int(t.la_req_cpu[0]), int(t.la_lim_cpu[0]), sf["cpu"], int(t.la_dflt_cpu[0]))
    mem = L.ko_estimated_used(int(t.la_req_memory[0]), int(t.la_lim_memory[0]), sf["memory"], int(t.la_dflt_memory[0]))
    assert {"cpu": cpu, "memory": mem} == case["want"]


def quota_problem(dims_limit, dims_used, pod_req, parent=None, check_parent=False):
    """1 always-feasible node, 1 pod, ElasticQuota rows; dims: 0 cpu, 1 memory, 2 gpu."""
    idx = {"cpu": 0, "memory": 1, "gpu": 2}
    prof = SchedulerProfile(fit=None, loadaware=None)
    from koordinator_amd.config import ElasticQuotaArgs
    prof.quota = ElasticQuotaArgs(enable_check_parent_quota=check_parent)
    cfg = prof.to_ks_config()
    nodes = NodeTable(1)
    nodes.allowed_pods[:] = 110
    rows = [(dims_limit, dims_used)] + ([parent] if parent else [])
    q = QuotaTable(len(rows))
    for r, (lim, used) in enumerate(rows):
        for k, v in lim.items():
            q.limit_mask[r] |= 1 << idx[k]
            q.limit[idx[k], r] = v
        for k, v in used.items():
            q.used[idx[k], r] = v
    if parent:
        q.parent[0] = 1
    pods = PodTable(1)
    pods.quota[0] = 0
    for k, v in pod_req.items():
        pods.quota_mask[0] |= 1 << idx[k]
        pods.quota_req[idx[k], 0] = v
    return cfg, nodes, q, pods


@pytest.mark.parametrize("case", QUOTA["admission"], ids=[c["name"] for c in QUOTA["admission"]])
def test_oracle_quota_admission(case, oracle_lib):
    cfg, nodes, q, pods = quota_problem(case["limit"], case["used"], case["pod"])
    r = oracle_lib.Oracle(cfg, nodes, q).schedule(pods)
    want = abi.KS_S_QUOTA if case["want"] == "Unschedulable" else abi.KS_S_SCHEDULED
    assert r["status"][0] == want


@pytest.mark.parametrize("case", QUOTA["parent"], ids=[c["name"] for c in QUOTA["parent"]])
def test_oracle_quota_parent(case, oracle_lib):
    cfg, nodes, q, pods = quota_problem(case["child"]["limit"], case["child"]["used"], case["pod"],
                                        parent=(case["parent"]["limit"], case["parent"]["used"]), check_parent=True)
    r = oracle_lib.Oracle(cfg, nodes, q).schedule(pods)
    assert r["status"][0] == abi.KS_S_QUOTA | abi.KS_S_QUOTA_PARENT


@pytest.mark.parametrize("case", QUOTA["reserve"], ids=[c["name"] for c in QUOTA["reserve"]])
def test_oracle_quota_reserve(case, oracle_lib):
    cfg, nodes, q, pods = quota_problem({}, case["used"], case["pod"])
    o = oracle_lib.Oracle(cfg, nodes, q)
    r = o.schedule(pods)
    assert r["status"][0] == 0
    used = o.read_quota_used()[0]
    assert [used[0], used[1], used[2]] == [case["want_used"]["cpu"], case["want_used"]["memory"], case["want_used"]["gpu"]]


# ------------------------------------------------------------- worked example from SURVEY §8(c)

def test_score_load_node_worked_example(oracle_lib):
    """alloc 96 CPU / 512Gi, usage 32 CPU / 10Gi, pod 16 CPU / 32Gi -> (52+93)/2 = 72 (load_aware_test.go:1068)."""
    L = oracle_lib.lib()
    est_cpu = L.ko_estimated_used(16000, 16000, 85, 250)
    est_mem = L.ko_estimated_used(32 << 30, 32 << 30, 70, 200 << 20)
    assert (est_cpu, est_mem) == (13600, 24051816858)
    cpu = L.ko_least_requested_score(est_cpu + 32000, 96000)
    mem = L.ko_least_requested_score(est_mem + (10 << 30), 512 << 30)
    assert (cpu, mem, (cpu + mem) // 2) == (52, 93, 72)
