"""GPU parity: libkoordgpu.so (HIP, gfx950) vs the CPU oracle, bit-exact.

Placements, per-pod statuses, chosen-node scores, per-node filter reasons and
per-plugin scores, and the node / quota state after every commit must be
identical to oracle/koord_oracle.c (the reduced-form restatement of the
reference, itself pinned by tests/golden/).
"""
import numpy as np
import pytest

from helpers import (assert_same_results, assert_same_state, homogeneous_pods, nested_quotas, profile,
                     stress_nodes, stress_pods)
from koordinator_amd import abi, synth
from koordinator_amd.cluster import PodTable

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def runtime():
    from koordinator_amd import runtime as rt

    rt.lib()  # must load the in-tree HIP library; no fallback
    return rt


def run_both(runtime, oracle_lib, prof, nodes, pods, quotas=None, nthreads=4):
    cfg = prof.to_ks_config()
    ev = runtime.Evaluator(cfg, nodes.copy(), quotas.copy() if quotas is not None else None)
    got = ev.schedule(pods)
    orc = oracle_lib.Oracle(cfg, nodes.copy(), quotas.copy() if quotas is not None else None, nthreads=nthreads)
    want = orc.schedule(pods)
    return ev, orc, got, want


def check_run(runtime, oracle_lib, prof, nodes, pods, quotas=None, label=""):
    ev, orc, got, want = run_both(runtime, oracle_lib, prof, nodes, pods, quotas)
    assert_same_results(got, want, label)
    assert_same_state(ev.read_nodes(), orc.read_nodes(), label)
    if quotas is not None:
        assert np.array_equal(ev.read_quota_used(), orc.read_quota_used()), f"{label}: quota used differs"
    st = ev.stats()
    ev.close()
    orc.close()
    return got, st


def test_eval_debug_matches_oracle(runtime, oracle_lib):
    rng = np.random.Generator(np.random.PCG64(7))
    nodes = stress_nodes(777, rng)
    pods = stress_pods(64, rng)
    for prof in (profile(), profile(strategy="MostAllocated", prod_usage=True, eph_weight=2, fit_weight=3, la_weight=2),
                 profile(filter_expired=False)):
        cfg = prof.to_ks_config()
        ev = runtime.Evaluator(cfg, nodes)
        orc = oracle_lib.Oracle(cfg, nodes)
        for i in range(pods.n):
            one = pods.rows([i])
            r_g, s_g, t_g = ev.eval_pod(one)
            r_o, s_o, t_o = orc.eval_pod(one)
            assert np.array_equal(r_g, r_o), f"pod {i}: filter reasons differ at nodes {np.nonzero(r_g != r_o)[0][:10]}"
            assert np.array_equal(s_g, s_o), f"pod {i}: plugin scores differ at nodes {np.nonzero((s_g != s_o).any(1))[0][:10]}"
            assert np.array_equal(t_g, t_o), f"pod {i}: totals differ"
        ev.close()
        orc.close()


def test_c1_schedule_matches_oracle(runtime, oracle_lib):
    w = synth.c1()
    got, st = check_run(runtime, oracle_lib, w.profile, w.nodes, w.pods, None, "C1")
    assert (got["status"] == 0).sum() > 900
    assert st["passes"] >= 1000 // 64


def test_c2_quota_schedule_matches_oracle(runtime, oracle_lib):
    w = synth.c2(n_pods=3000)
    got, _ = check_run(runtime, oracle_lib, w.profile, w.nodes, w.pods, w.quotas, "C2-3k")
    rejected = (got["status"] & abi.KS_S_QUOTA) != 0
    assert 0 < rejected.sum() < len(rejected)


def test_c2_full_queue_matches_oracle(runtime, oracle_lib):
    """The headline workload exactly as bench.py runs it: all 10k pods of C2 onto its 5k nodes with the 32 quotas."""
    w = synth.c2()
    cfg = w.profile.to_ks_config()
    ev = runtime.Evaluator(cfg, w.nodes.copy(), w.quotas.copy())
    got = ev.schedule(w.pods)
    orc = oracle_lib.Oracle(cfg, w.nodes.copy(), w.quotas.copy(), nthreads=16)
    want = orc.schedule(w.pods)
    assert_same_results(got, want, "C2-10k")
    assert_same_state(ev.read_nodes(), orc.read_nodes(), "C2-10k")
    assert np.array_equal(ev.read_quota_used(), orc.read_quota_used()), "C2-10k: quota used differs"
    assert (got["status"] == 0).sum() > 8000
    ev.close()
    orc.close()


@pytest.mark.parametrize("batch,cand", [(1, 1), (7, 2), (64, 1), (64, 64), (33, 5)])
def test_batch_and_candidate_sizes(runtime, oracle_lib, batch, cand):
    rng = np.random.Generator(np.random.PCG64(100 + batch * 3 + cand))
    nodes = stress_nodes(1000, rng)
    pods = stress_pods(400, rng)
    check_run(runtime, oracle_lib, profile(batch_pods=batch, candidates=cand), nodes, pods, None, f"b{batch}k{cand}")


def test_homogeneous_pods_force_cuts_and_rescans(runtime, oracle_lib):
    rng = np.random.Generator(np.random.PCG64(11))
    nodes = synth.make_nodes(300, rng)
    pods = homogeneous_pods(2000)
    _, st = check_run(runtime, oracle_lib, profile(candidates=2), nodes, pods, None, "homogeneous")
    assert st["rescans"] > 0


def test_most_allocated_non_monotone(runtime, oracle_lib):
    rng = np.random.Generator(np.random.PCG64(12))
    nodes = stress_nodes(640, rng)
    pods = stress_pods(500, rng)
    check_run(runtime, oracle_lib, profile(strategy="MostAllocated", candidates=4), nodes, pods, None, "most")


def test_stress_filters_and_quota_chain(runtime, oracle_lib):
    rng = np.random.Generator(np.random.PCG64(13))
    nodes = stress_nodes(1500, rng, tight=True)
    pods = stress_pods(1200, rng, n_quotas=24)
    quotas = nested_quotas(pods, rng, 24)
    for prof in (profile(quota=True, prod_usage=True), profile(quota=True, check_parent=True, candidates=3)):
        check_run(runtime, oracle_lib, prof, nodes, pods, quotas, "stress")


@pytest.mark.parametrize("batch", [64, 33, 8])
def test_quota_admission_edges(runtime, oracle_lib, batch):
    """ElasticQuota admission inside a pass (flat quotas): few quotas whose limits are crossed inside a pass, tight
    non-preemptible mins, pods that pass the quota but fit no node (their requests never reach used), negative and
    out-of-mask request words, pods without a quota."""
    rng = np.random.Generator(np.random.PCG64(31 + batch))
    nodes = stress_nodes(700, rng)
    pods = stress_pods(1500, rng, n_quotas=3)
    pods.req_milli_cpu[::11] = 10 ** 9  # admitted or not, never placed
    pods.quota_req[0][::11] = pods.req_milli_cpu[::11] // 1000
    pods.quota_req[5][::13] = -7  # a request word outside every quota's mask / a negative one
    pods.quota_mask[::13] |= np.uint32(1 << 5)
    pods.flags[rng.random(pods.n) < 0.3] |= abi.KS_POD_NONPREEMPTIBLE
    quotas = synth.make_quotas(pods, 3, rng, admit_frac=0.35)
    quotas.limit_mask[:] |= np.uint32(1 << 5)
    quotas.limit[5][:] = 1 << 40
    quotas.min_mask[:] = quotas.limit_mask
    quotas.min[:, :] = quotas.limit // 3
    got, _ = check_run(runtime, oracle_lib, profile(quota=True, batch_pods=batch), nodes, pods, quotas, f"cert-b{batch}")
    st = got["status"]
    assert ((st & abi.KS_S_QUOTA) != 0).sum() > 100
    assert (st == abi.KS_S_QUOTA_NONPREEMPTIBLE).sum() > 0
    assert (st == 0).sum() > 100


def test_unschedulable_and_tiny_clusters(runtime, oracle_lib):
    rng = np.random.Generator(np.random.PCG64(14))
    for n in (1, 63, 64, 65, 130):
        nodes = synth.make_nodes(n, rng)
        pods = stress_pods(150, rng)
        pods.req_milli_cpu[::7] = 10 ** 9  # never fits
        check_run(runtime, oracle_lib, profile(), nodes, pods, None, f"n={n}")


def test_zero_pods_and_zero_nodes(runtime, oracle_lib):
    rng = np.random.Generator(np.random.PCG64(15))
    nodes = synth.make_nodes(10, rng)
    ev = runtime.Evaluator(profile().to_ks_config(), nodes)
    r = ev.schedule(PodTable(0))
    assert len(r["node"]) == 0
    empty = synth.make_nodes(0, rng)
    ev2 = runtime.Evaluator(profile().to_ks_config(), empty)
    r2 = ev2.schedule(stress_pods(5, rng))
    assert (r2["node"] == -1).all() and (r2["status"] == abi.KS_S_UNSCHEDULABLE).all()


def test_update_nodes_then_schedule(runtime, oracle_lib):
    rng = np.random.Generator(np.random.PCG64(16))
    nodes = stress_nodes(900, rng)
    pods = stress_pods(300, rng)
    cfg = profile().to_ks_config()
    ev = runtime.Evaluator(cfg, nodes)
    idx = rng.choice(900, 120, replace=False).astype(np.int32)
    newer = stress_nodes(120, rng)
    ev.update_nodes(idx, newer)
    merged = nodes.copy()
    for k, v in newer.columns().items():
        getattr(merged, k)[idx] = v
    merged.alloc_scalar[:, idx] = newer.alloc_scalar
    merged.req_scalar[:, idx] = newer.req_scalar
    got = ev.schedule(pods)
    orc = oracle_lib.Oracle(cfg, merged)
    assert_same_results(got, orc.schedule(pods), "update")
    assert_same_state(ev.read_nodes(), orc.read_nodes(), "update")


def test_checkpoint_restore_repeatable(runtime, oracle_lib):
    w = synth.c2(n_nodes=2000, n_pods=1500)
    ev = runtime.Evaluator(w.cfg, w.nodes, w.quotas)
    ev.stage(w.pods)
    ev.checkpoint()
    ev.schedule_staged()
    a = ev.fetch()
    ev.restore()
    ev.schedule_staged()
    b = ev.fetch()
    assert_same_results(a, b, "restore")


def test_large_cluster_properties(runtime, oracle_lib):
    """100k nodes (the C5 shape): exact vs oracle on a short pod prefix, plus invariants."""
    w = synth.c5(n_pods=400)
    got, _ = check_run(runtime, oracle_lib, w.profile, w.nodes, w.pods, None, "C5-prefix")
    ok = got["status"] == 0
    assert ok.all()
    assert (got["node"][ok] >= 0).all() and (got["node"][ok] < w.nodes.n).all()
