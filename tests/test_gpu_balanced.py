"""GPU parity of upstream NodeResourcesBalancedAllocation (the v1beta2 default profile's plugin, kernel
balanced_score in ks_device.h) with the CPU oracle: per-node scores through ks_eval_pod, and whole queues through
the sweep / select / commit path, where the plugin makes keys non-monotone (a commit can raise a node's balance):
alone with Fit + LoadAware, with ElasticQuota, with Reservation, with NUMA + DeviceShare, and pipelined."""
import numpy as np
import pytest

from helpers import assert_same_results, assert_same_state, nested_quotas, profile, stress_nodes, stress_pods
from koordinator_amd import abi, synth
from koordinator_amd.config import NodeResourcesBalancedAllocationArgs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def runtime():
    from koordinator_amd import runtime as rt

    rt.lib()  # the in-tree HIP library; no fallback
    return rt


def run(runtime, oracle_lib, cfg, nodes, pods, label, pipeline=None, **tables):
    ev = runtime.Evaluator(cfg, nodes.copy(), **{k: v.copy() for k, v in tables.items()})
    if pipeline is not None:
        ev.set_pipeline(pipeline)
    got = ev.schedule(pods)
    st = ev.stats()
    orc = oracle_lib.Oracle(cfg, nodes.copy(), nthreads=8, **{k: v.copy() for k, v in tables.items()})
    want = orc.schedule(pods)
    assert_same_results(got, want, label)
    assert_same_state(ev.read_nodes(), orc.read_nodes(), label)
    if "quotas" in tables:
        assert np.array_equal(ev.read_quota_used(), orc.read_quota_used()), f"{label}: quota used"
    if "reservations" in tables:
        assert np.array_equal(got["reservation"], want["reservation"]), f"{label}: nominated reservations"
    ev.close()
    orc.close()
    return got, st


def with_balanced(w, weight=1):
    w.profile.balanced = NodeResourcesBalancedAllocationArgs()
    w.profile.balanced_weight = weight
    return w


def test_eval_pod_scores(runtime, oracle_lib):
    rng = np.random.Generator(np.random.PCG64(41))
    nodes = stress_nodes(700, rng)
    pods = stress_pods(48, rng)
    for prof in (profile(balanced=1), profile(strategy="MostAllocated", balanced=3, la_weight=2)):
        cfg = prof.to_ks_config()
        ev = runtime.Evaluator(cfg, nodes)
        orc = oracle_lib.Oracle(cfg, nodes)
        for i in range(pods.n):
            one = pods.rows([i])
            r_g, s_g, t_g = ev.eval_pod(one)
            r_o, s_o, t_o = orc.eval_pod(one)
            assert np.array_equal(r_g, r_o), f"pod {i}: reasons"
            assert np.array_equal(s_g[:, abi.KS_SCORE_BALANCED], s_o[:, abi.KS_SCORE_BALANCED]), f"pod {i}: balanced"
            assert np.array_equal(s_g, s_o) and np.array_equal(t_g, t_o), f"pod {i}: scores / totals"
        ev.close()
        orc.close()


@pytest.mark.parametrize("cand", [2, 32])
def test_schedule_fit_loadaware_balanced(runtime, oracle_lib, cand):
    rng = np.random.Generator(np.random.PCG64(42 + cand))
    nodes = stress_nodes(1200, rng)
    pods = stress_pods(1500, rng)
    _, st = run(runtime, oracle_lib, profile(balanced=1, candidates=cand).to_ks_config(), nodes, pods, f"bal-k{cand}")
    assert st["passes"] >= 1500 // 64


def test_c2_prefix_with_quotas(runtime, oracle_lib):
    w = with_balanced(synth.c2(n_pods=2500))
    got, _ = run(runtime, oracle_lib, w.cfg, w.nodes, w.pods, "c2-bal", quotas=w.quotas)
    assert ((got["status"] & abi.KS_S_QUOTA) != 0).sum() > 0


def test_quota_chain(runtime, oracle_lib):
    rng = np.random.Generator(np.random.PCG64(43))
    nodes = stress_nodes(900, rng, tight=True)
    pods = stress_pods(800, rng, n_quotas=16)
    quotas = nested_quotas(pods, rng, 16)
    run(runtime, oracle_lib, profile(quota=True, check_parent=True, balanced=2).to_ks_config(), nodes, pods,
        "bal-quota-chain", quotas=quotas)


def test_reservations(runtime, oracle_lib):
    w = with_balanced(synth.c4(n_nodes=1500, n_reservations=3500, n_pods=800))
    got, _ = run(runtime, oracle_lib, w.cfg, w.nodes, w.pods, "c4-bal", reservations=w.reservations)
    assert (got["reservation"] >= 0).sum() > 0


def test_numa_and_devices(runtime, oracle_lib):
    w = with_balanced(synth.c3(seed=44, n_nodes=300, n_pods=500))
    ev = runtime.Evaluator(w.cfg, w.nodes.copy(), **w.tables())
    got = ev.schedule(w.pods)
    orc = oracle_lib.Oracle(w.cfg, w.nodes.copy(), nthreads=8, **w.tables())
    want = orc.schedule(w.pods)
    assert_same_results(got, want, "c3-bal")
    for k in ("gpu_minors", "rdma_minors"):
        assert np.array_equal(got[k], want[k]), k
    assert np.array_equal(ev.fetch_cpusets(w.pods.n), orc.fetch_cpusets(w.pods.n))
    assert_same_state(ev.read_nodes(), orc.read_nodes(), "c3-bal")
    ev.close()
    orc.close()


def test_pipelined_not_patched(runtime, oracle_lib):
    rng = np.random.Generator(np.random.PCG64(45))
    nodes = stress_nodes(1000, rng)
    pods = stress_pods(700, rng)
    _, st = run(runtime, oracle_lib, profile(balanced=1, candidates=4).to_ks_config(), nodes, pods, "bal-pipe",
                pipeline=2)
    assert st["pipelined"] == 1  # not monotone: the select follows the re-sweep
