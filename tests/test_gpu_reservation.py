"""GPU parity for the Reservation plugin: libkoordgpu.so vs the CPU oracle.

The oracle (oracle/koord_oracle.c) restates the reference per pod and per node — BeforePreFilter
restore, Filter, PreScore nomination and preferred node, Score + DefaultNormalizeScore, Reserve into
the nominated reservation — and is itself checked against the object-level restatement
(tests/test_reservation_oracle.py) and the reference's reservation test tables
(tests/golden/reservation.json).  Everything here must match bit for bit: placements, statuses,
chosen-node scores, nominated reservations, per-node reasons and per-plugin scores, node state and
the reservation cache (Allocated, assigned pods) after every commit.
"""
import numpy as np
import pytest

from helpers import assert_same_results, assert_same_state
from koordinator_amd import abi, synth
from koordinator_amd.cluster import NodeTable, PodTable, ReservationTable
from koordinator_amd.config import CPU, MEMORY, NodeResourcesFitArgs, SchedulerProfile

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def runtime():
    from koordinator_amd import runtime as rt

    rt.lib()
    return rt


def workload(seed, n=700, r=1800, p=500, n_classes=8, tight=False, order_frac=0.05):
    rng = np.random.Generator(np.random.PCG64(seed))
    nodes = synth.make_nodes(n, rng)
    for col in ("req_milli_cpu", "req_memory", "nonzero_milli_cpu", "nonzero_memory"):
        setattr(nodes, col, getattr(nodes, col) // 2)
    if tight:
        nodes.allowed_pods[:] = rng.integers(3, 12, n)
        nodes.pod_count[:] = 0
    rs = synth.make_reservations(nodes, r, rng, n_classes=n_classes, order_frac=order_frac, assigned_frac=0.35)
    # Restricted reservations narrowed to cpu, a few with an extended resource, odd sizes
    narrow = (rs.policy == abi.KS_RSV_POLICY_RESTRICTED) & (rng.random(r) < 0.3)
    rs.key_mask[narrow] = 0b1
    rs.allocatable[1][narrow] = 0
    rs.allocated[1][narrow] = 0
    pods = synth.make_pods(p, rng)
    synth.reservation_pods(pods, rng, n_classes=n_classes, class_frac=0.75, affinity_frac=0.15)
    big = rng.random(p) < 0.1
    pods.req_milli_cpu[big] *= 4
    pods.nonzero_milli_cpu[big] *= 4
    return nodes, rs, pods


def prof(**kw):
    fit_res = kw.pop("fit_res", {CPU: 1, MEMORY: 1, synth.BATCH_CPU: 1, synth.BATCH_MEMORY: 1})
    strategy = kw.pop("strategy", "LeastAllocated")
    return SchedulerProfile(fit=NodeResourcesFitArgs(strategy=strategy, resources=fit_res), reservation_weight=5000,
                            **kw)


def run(runtime, oracle_lib, p, nodes, rs, pods, nthreads=8):
    cfg = p.to_ks_config()
    ev = runtime.Evaluator(cfg, nodes.copy(), reservations=rs.copy())
    got = ev.schedule(pods)
    orc = oracle_lib.Oracle(cfg, nodes.copy(), nthreads=nthreads, reservations=rs.copy())
    want = orc.schedule(pods)
    return ev, orc, got, want


def check(runtime, oracle_lib, p, nodes, rs, pods, label):
    ev, orc, got, want = run(runtime, oracle_lib, p, nodes, rs, pods)
    assert_same_results(got, want, label)
    assert np.array_equal(got["reservation"], want["reservation"]), f"{label}: nominated reservations differ"
    assert_same_state(ev.read_nodes(), orc.read_nodes(), label)
    ga, gs = ev.read_reservations()
    oa, os_ = orc.read_reservations()
    assert np.array_equal(ga, oa), f"{label}: reservation Allocated differs"
    assert np.array_equal(gs, os_), f"{label}: reservation assigned counts differ"
    assert (got["reservation"] >= 0).any(), f"{label}: no pod went into a reservation"
    st = ev.stats()
    ev.close()
    orc.close()
    return got, st


def test_eval_debug_matches_oracle(runtime, oracle_lib):
    nodes, rs, pods = workload(11, n=500, r=1300, p=48)
    for p in (prof(), prof(strategy="MostAllocated", fit_weight=2, loadaware_weight=3)):
        cfg = p.to_ks_config()
        ev = runtime.Evaluator(cfg, nodes, reservations=rs)
        orc = oracle_lib.Oracle(cfg, nodes, reservations=rs)
        for i in range(pods.n):
            one = pods.rows([i])
            r_g, s_g, t_g = ev.eval_pod(one)
            r_o, s_o, t_o = orc.eval_pod(one)
            assert np.array_equal(r_g, r_o), f"pod {i}: reasons differ"
            assert np.array_equal(s_g, s_o), f"pod {i}: per-plugin scores differ"
            assert np.array_equal(t_g, t_o), f"pod {i}: totals differ"
        ev.close()
        orc.close()


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_schedule_matches_oracle(runtime, oracle_lib, seed):
    nodes, rs, pods = workload(seed)
    check(runtime, oracle_lib, prof(), nodes, rs, pods, f"seed{seed}")


@pytest.mark.parametrize("batch,cand", [(1, 1), (64, 1), (17, 3), (64, 64)])
def test_batch_and_candidates(runtime, oracle_lib, batch, cand):
    nodes, rs, pods = workload(5, n=400, r=1200, p=300)
    check(runtime, oracle_lib, prof(batch_pods=batch, candidates=cand), nodes, rs, pods, f"b{batch}k{cand}")


def test_tight_nodes_most_allocated(runtime, oracle_lib):
    nodes, rs, pods = workload(8, n=300, r=900, p=400, tight=True)
    check(runtime, oracle_lib, prof(strategy="MostAllocated"), nodes, rs, pods, "tight-most")


def test_ordered_reservations_drive_placement(runtime, oracle_lib):
    nodes, rs, pods = workload(9, n=400, r=1000, p=300, order_frac=0.3)
    got, _ = check(runtime, oracle_lib, prof(), nodes, rs, pods, "ordered")
    assert (got["score"] >= 500000).sum() > 0


def test_few_classes_many_commits_per_reservation(runtime, oracle_lib):
    # two classes: pods pile into the same reservations (Allocated / AllocateOnce updates inside a pass)
    nodes, rs, pods = workload(12, n=200, r=500, p=600, n_classes=2, order_frac=0.0)
    check(runtime, oracle_lib, prof(), nodes, rs, pods, "two-classes")


def test_checkpoint_restore_and_update_nodes(runtime, oracle_lib):
    nodes, rs, pods = workload(13, n=300, r=800, p=200)
    cfg = prof().to_ks_config()
    ev = runtime.Evaluator(cfg, nodes.copy(), reservations=rs.copy())
    base = ev.read_nodes()
    want_nodes = nodes
    assert np.array_equal(base.req_milli_cpu, want_nodes.req_milli_cpu)  # read back is the reference's NodeInfo
    assert np.array_equal(base.nonzero_memory, want_nodes.nonzero_memory)
    ev.checkpoint()
    a = ev.schedule(pods)
    ev.restore()
    b = ev.schedule(pods)
    assert np.array_equal(a["node"], b["node"]) and np.array_equal(a["reservation"], b["reservation"])
    ev.restore()
    # informer delta on some nodes, then schedule: same as the oracle on the updated snapshot
    upd = nodes.copy()
    idx = np.array([3, 50, 120, 299], np.int32)
    upd.req_milli_cpu[idx] += 1000
    upd.nonzero_milli_cpu[idx] += 1000
    ev.update_nodes(idx, upd.rows(idx))
    got = ev.schedule(pods)
    orc = oracle_lib.Oracle(cfg, upd.copy(), reservations=rs.copy())
    want = orc.schedule(pods)
    assert_same_results(got, want, "update")
    assert np.array_equal(got["reservation"], want["reservation"])
    ev.close()
    orc.close()


def test_affinity_without_reservations_unschedulable(runtime, oracle_lib):
    nodes = synth.make_nodes(100, np.random.Generator(np.random.PCG64(3)))
    pods = synth.make_pods(20, np.random.Generator(np.random.PCG64(4)))
    pods.rsv_class[:] = 0
    pods.flags[::2] |= abi.KS_POD_RSV_AFFINITY
    cfg = prof().to_ks_config()
    ev = runtime.Evaluator(cfg, nodes)
    got = ev.schedule(pods)
    orc = oracle_lib.Oracle(cfg, nodes)
    want = orc.schedule(pods)
    assert_same_results(got, want, "no-rsv")
    assert (got["status"][::2] == abi.KS_S_UNSCHEDULABLE).all()


def test_score_with_order_cluster(runtime):
    """TestScoreWithOrder (reservation/scoring_test.go:255) as a 4-node cluster on the GPU."""
    GI = 1 << 30
    nodes = NodeTable(4)
    nodes.alloc_milli_cpu[:] = 32000
    nodes.alloc_memory[:] = 64 * GI
    nodes.allowed_pods[:] = 110
    nodes.req_milli_cpu[:] = 4000
    nodes.req_memory[:] = 8 * GI
    nodes.nonzero_milli_cpu[:] = 4000
    nodes.nonzero_memory[:] = 8 * GI
    nodes.pod_count[:] = 1
    rs = ReservationTable(4)
    rs.node[:] = [0, 1, 2, 3]
    rs.owner_classes[:] = 1
    rs.key_mask[:] = 3
    rs.allocatable[0] = 4000
    rs.allocatable[1] = 8 * GI
    rs.order[3] = 123456
    pod = PodTable(1)
    pod.req_milli_cpu[:] = 4000
    pod.req_memory[:] = 8 * GI
    pod.nonzero_milli_cpu[:] = 4000
    pod.nonzero_memory[:] = 8 * GI
    pod.rsv_class[:] = 0
    p = SchedulerProfile(fit=NodeResourcesFitArgs(resources={CPU: 1, MEMORY: 1}), loadaware=None, reservation_weight=5000)
    ev = runtime.Evaluator(p.to_ks_config(), nodes, reservations=rs)
    reasons, scores, _ = ev.eval_pod(pod)
    assert reasons.tolist() == [0, 0, 0, 0]
    assert scores[:, abi.KS_SCORE_RESERVATION].tolist() == [10, 10, 10, 100]
    res = ev.schedule(pod)
    assert res["node"][0] == 3 and res["reservation"][0] == 3
    ev.close()


def test_virtual_shards_match(runtime, oracle_lib):
    nodes, rs, pods = workload(21, n=900, r=2000, p=300)
    cfg = prof().to_ks_config()
    ev = runtime.Evaluator(cfg, nodes.copy(), reservations=rs.copy())
    ev.shard(1, 0, None, virtual_shards=3)
    got = ev.schedule(pods)
    orc = oracle_lib.Oracle(cfg, nodes.copy(), nthreads=8, reservations=rs.copy())
    want = orc.schedule(pods)
    assert_same_results(got, want, "vshards")
    assert np.array_equal(got["reservation"], want["reservation"])
    ev.close()
    orc.close()


def test_c4_sample_matches_oracle(runtime, oracle_lib):
    """The C4 benchmark cluster (20k nodes, 50k reservations) on its first 5000 pods."""
    w = synth.c4(n_pods=5000)
    got, st = check(runtime, oracle_lib, w.profile, w.nodes, w.reservations, w.pods, "c4")
    print("c4 sample stats", {k: st[k] for k in ("passes", "cut_passes", "rescans", "total_ms")})


def test_unmatched_pods_fast_path_and_raised_nodes(runtime, oracle_lib):
    """Pods of class -1 (no reservation matches them) take the monotone fast path in the Reservation kernels; a commit
    that lowers a node's restored Requested turns it off for the rest of the pass.  Here it happens on purpose: cpu-only
    reservations with one assigned pod and 500m left, filled by 500m / 1 MiB pods of their class -- the remainder's
    default non-zero memory (200 MiB) leaves the restore while the pod adds 1 MiB, so the node's NonZeroRequested memory
    drops and its Fit score rises for the class -1 pods after it."""
    rng = np.random.Generator(np.random.PCG64(404))
    n, r, p = 400, 600, 900
    nodes = synth.make_nodes(n, rng)
    rs = ReservationTable(r)
    rs.node[:] = rng.integers(0, n, r)
    rs.owner_classes[:] = np.uint64(1) << rng.integers(0, 4, r).astype(np.uint64)
    rs.key_mask[:] = 0b1
    rs.allocatable[0] = 1000
    rs.allocated[0] = 500
    rs.assigned[:] = 1
    nodes.req_milli_cpu[:] += np.bincount(rs.node, weights=np.full(r, 1500.0), minlength=n).astype(np.int64)
    nodes.nonzero_milli_cpu[:] += np.bincount(rs.node, weights=np.full(r, 1500.0), minlength=n).astype(np.int64)
    nodes.nonzero_memory[:] += np.bincount(rs.node, weights=np.full(r, float(2 * synth.DEFAULT_MEMORY_NZ)), minlength=n).astype(np.int64)
    nodes.pod_count[:] += np.bincount(rs.node, weights=np.full(r, 2.0), minlength=n).astype(np.int32)
    pods = synth.make_pods(p, rng)
    matched = rng.random(p) < 0.4
    pods.rsv_class[:] = np.where(matched, rng.integers(0, 4, p), -1)
    pods.req_milli_cpu[matched] = 500
    pods.nonzero_milli_cpu[matched] = 500
    pods.req_memory[matched] = synth.MI
    pods.nonzero_memory[matched] = synth.MI
    got, st = check(runtime, oracle_lib, prof(), nodes, rs, pods, "class -1 fast path")
    assert st["diag"][7] > 0, "no class -1 pod took the fast path"
