"""Golden vectors through the HIP library (layer 3): ingest -> SoA -> libkoordgpu.so."""
import pytest

from koordinator_amd import abi
from test_golden import (EST, FILTER, QUOTA, SCORE, build_one, filter_lister, quota_problem, reason_of, score_lister,
                         want_of)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rt():
    from koordinator_amd import runtime

    runtime.lib()
    return runtime


@pytest.mark.parametrize("case", FILTER, ids=[c["name"] for c in FILTER])
def test_gpu_filter(case, rt):
    cfg, nodes, pods = build_one(case, filter_lister(case))
    ev = rt.Evaluator(cfg, nodes)
    reasons, _, _ = ev.eval_pod(pods)
    assert reason_of(int(reasons[0])) == want_of(case)


@pytest.mark.parametrize("case", SCORE, ids=[c["name"] for c in SCORE])
def test_gpu_score(case, rt):
    cfg, nodes, pods = build_one(case, score_lister(case), enable_filter=False)
    ev = rt.Evaluator(cfg, nodes)
    reasons, scores, total = ev.eval_pod(pods)
    assert reasons[0] == 0
    assert scores[0, abi.KS_SCORE_LOADAWARE] == case["want"]["score"]
    # and through the full schedule path (sweep -> select -> commit)
    r = ev.schedule(pods)
    assert r["node"][0] == 0 and r["score"][0] == case["want"]["score"]


@pytest.mark.parametrize("case", QUOTA["admission"], ids=[c["name"] for c in QUOTA["admission"]])
def test_gpu_quota_admission(case, rt):
    cfg, nodes, q, pods = quota_problem(case["limit"], case["used"], case["pod"])
    r = rt.Evaluator(cfg, nodes, q).schedule(pods)
    assert r["status"][0] == (abi.KS_S_QUOTA if case["want"] == "Unschedulable" else abi.KS_S_SCHEDULED)


@pytest.mark.parametrize("case", QUOTA["parent"], ids=[c["name"] for c in QUOTA["parent"]])
def test_gpu_quota_parent(case, rt):
    cfg, nodes, q, pods = quota_problem(case["child"]["limit"], case["child"]["used"], case["pod"],
                                        parent=(case["parent"]["limit"], case["parent"]["used"]), check_parent=True)
    r = rt.Evaluator(cfg, nodes, q).schedule(pods)
    assert r["status"][0] == abi.KS_S_QUOTA | abi.KS_S_QUOTA_PARENT


@pytest.mark.parametrize("case", QUOTA["reserve"], ids=[c["name"] for c in QUOTA["reserve"]])
def test_gpu_quota_reserve(case, rt):
    cfg, nodes, q, pods = quota_problem({}, case["used"], case["pod"])
    ev = rt.Evaluator(cfg, nodes, q)
    assert ev.schedule(pods)["status"][0] == 0
    used = ev.read_quota_used()[0]
    assert [used[0], used[1], used[2]] == [case["want_used"]["cpu"], case["want_used"]["memory"], case["want_used"]["gpu"]]


@pytest.mark.parametrize("case", EST["pods"], ids=[c["name"] for c in EST["pods"]])
def test_gpu_estimate_pod_via_commit(case, rt):
    """EstimatePod runs on the device (prep_pods_kernel); a commit adds it to the node term."""
    from koordinator_amd import ingest
    from koordinator_amd.cluster import NodeTable
    from koordinator_amd.config import LoadAwareSchedulingArgs, SchedulerProfile

    # the reference test builds the estimator directly (no args validation), e.g. scaling 110
    cfg = SchedulerProfile(fit=None, loadaware=LoadAwareSchedulingArgs()).to_ks_config()
    sf = {"cpu": 85, "memory": 70}
    sf.update(case.get("scalingFactors") or {})
    cfg.loadaware.scaling_cpu, cfg.loadaware.scaling_memory = sf["cpu"], sf["memory"]
    nodes = NodeTable(1)
    nodes.allowed_pods[:] = 110
    nodes.la_flags[:] = abi.KS_LA_HAS_METRIC
    pods = ingest.pods_to_table([case["pod"]])
    ev = rt.Evaluator(cfg, nodes)
    assert ev.schedule(pods)["node"][0] == 0
    st = ev.read_nodes()
    assert {"cpu": int(st.la_term_milli_cpu[0]), "memory": int(st.la_term_memory[0])} == case["want"]
