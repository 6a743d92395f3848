"""GPU parity of the ElasticQuota PostFilter (ks_preempt, koordinator_amd/csrc/ks_preempt.h) against the CPU oracle
(ko_preempt, a literal restatement of preempt.go's SelectVictimsOnNode and upstream's candidate selection, pinned by
tests/test_preempt.py): status, nominated node, victims in order, PDB violations, candidate and potential-node counts
and every node's dry-run outcome must be identical."""
import numpy as np
import pytest

import test_preempt as hand
from helpers import profile
from koordinator_amd import abi, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def runtime():
    from koordinator_amd import runtime as rt

    rt.lib()
    return rt


KEYS = ("status", "node", "num_pdb_violations", "candidates", "potential_nodes")


def compare(runtime, oracle_lib, cfg, nodes, quotas, t, pods, prios, label, **kw):
    ev = runtime.Evaluator(cfg, nodes.copy(), quotas.copy())
    orc = oracle_lib.Oracle(cfg, nodes.copy(), quotas.copy())
    try:
        ev.load_node_pods(t)
        orc.load_node_pods(t)
        outs = []
        for i in range(pods.n):
            extra = {k: (v[i] if isinstance(v, list) else v) for k, v in kw.items()}
            g = ev.preempt(pods.rows([i]), int(prios[i]), node_status=True, **extra)
            w = orc.preempt(pods.rows([i]), int(prios[i]), node_status=True, **extra)
            for k in KEYS:
                assert g[k] == w[k], f"{label} pod {i}: {k} {g[k]} (GPU) vs {w[k]} (oracle)"
            assert np.array_equal(g["victims"], w["victims"]), f"{label} pod {i}: victims {g['victims']} vs {w['victims']}"
            assert np.array_equal(g["node_status"], w["node_status"]), f"{label} pod {i}: node statuses differ"
            outs.append(g)
        return outs
    finally:
        ev.close()
        orc.close()


def test_hand_cases_through_hip(runtime, oracle_lib):
    cfg = profile(quota=True).to_ks_config()
    cases = [(hand.BASE, 1500, 1 << 40), (hand.BASE, 500, 1 << 40), (hand.BASE, 500, 2000), (hand.BASE, 1500, 2000),
             (hand.BASE, 2500, 1 << 40)]
    for specs, cpu, lim in cases:
        nodes = hand.cluster(1)
        t = hand.running(nodes, specs)
        p = hand.preemptor(cpu)
        compare(runtime, oracle_lib, cfg, nodes, hand.quotas(t, limit_cpu=lim), t, p, [1000], f"hand {cpu}/{lim}")


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_c2_shaped_cluster(runtime, oracle_lib, seed):
    w = synth.c2_preempt(seed=seed, n_nodes=2000, n_preemptors=24)
    outs = compare(runtime, oracle_lib, w.cfg, w.nodes, w.quotas, w.node_pods, w.preemptors, w.priority, f"c2p{seed}")
    st = [o["status"] for o in outs]
    assert st.count(abi.KS_P_NOMINATED) >= 8, st  # the workload exercises real preemptions
    assert sum(len(o["victims"]) for o in outs) > 0


def test_unresolvable_masks_and_nominated_nodes(runtime, oracle_lib):
    w = synth.c2_preempt(seed=7, n_nodes=1500, n_preemptors=16)
    rng = np.random.Generator(np.random.PCG64(7))
    masks = [(rng.random(w.nodes.n) < f).astype(np.uint8) for f in np.linspace(0.0, 0.97, w.preemptors.n)]
    nominated = [int(x) for x in rng.integers(-1, w.nodes.n, w.preemptors.n)]
    compare(runtime, oracle_lib, w.cfg, w.nodes, w.quotas, w.node_pods, w.preemptors, w.priority, "masks",
            unresolvable=masks, nominated_node=nominated)


@pytest.mark.parametrize("per_node,allowed", [((60, 120), 130), ((150, 250), 256)])
def test_large_nodes(runtime, oracle_lib, per_node, allowed):
    # 2 and 4 positions per lane of the dry run (nodes with up to 128 / 256 pods)
    rng = np.random.Generator(np.random.PCG64(per_node[1]))
    nodes = synth.make_nodes(300, rng)
    nodes.allowed_pods[:] = allowed
    t, used = synth.make_node_pods(nodes, rng, 8, per_node=per_node, n_pdb=6, pdb_frac=0.4)
    nodes.alloc_milli_cpu[:] = np.maximum(nodes.req_milli_cpu + rng.integers(0, 3000, nodes.n), 1000)
    q = synth.QuotaTable(8)
    q.limit_mask[:] = 0xF
    q.used[:] = used
    q.limit[:] = (used * 1.01).astype(np.int64)
    pods = synth.make_pods(12, rng, 8)
    prio = rng.choice(np.array([1000, 5000, 9000], np.int32), 12)
    compare(runtime, oracle_lib, profile(quota=True).to_ks_config(), nodes, q, t, pods, prio, f"large{per_node}")


def test_pdb_heavy(runtime, oracle_lib):
    rng = np.random.Generator(np.random.PCG64(31))
    nodes = synth.make_nodes(800, rng)
    # every running pod in an exhausted budget: every victim violates (the budgets shared by several victims of a
    # node, decremented in the sorted order, are covered by test_large_nodes)
    t, used = synth.make_node_pods(nodes, rng, 4, per_node=(10, 50), n_pdb=5, pdb_frac=1.0)
    t.pdb_allowed[:] = 0
    nodes.alloc_milli_cpu[:] = np.maximum(nodes.req_milli_cpu + rng.integers(0, 2000, nodes.n), 1000)
    q = synth.QuotaTable(4)
    q.limit_mask[:] = 0xF
    q.used[:] = used
    q.limit[:] = used * 2
    pods = synth.make_pods(16, rng, 4)
    prio = np.full(16, 9000, np.int32)
    outs = compare(runtime, oracle_lib, profile(quota=True).to_ks_config(), nodes, q, t, pods, prio, "pdb")
    assert any(o["num_pdb_violations"] > 0 for o in outs)


def test_edge_inputs(runtime, oracle_lib):
    """No running pod anywhere; every node unresolvable; one running pod that is not preemptible; a node holding
    the dry run's maximum of 256 pods."""
    w = synth.c2_preempt(seed=11, n_nodes=300, n_preemptors=4)
    empty = w.node_pods.rows(np.arange(0))
    compare(runtime, oracle_lib, w.cfg, w.nodes, w.quotas, empty, w.preemptors, w.priority, "no running pods")
    compare(runtime, oracle_lib, w.cfg, w.nodes, w.quotas, w.node_pods, w.preemptors, w.priority, "all unresolvable",
            unresolvable=np.ones(w.nodes.n, np.uint8))
    one = w.node_pods.rows(np.arange(1))
    one.flags[:] |= abi.KS_NPOD_NONPREEMPTIBLE
    compare(runtime, oracle_lib, w.cfg, w.nodes, w.quotas, one, w.preemptors, w.priority, "one non-preemptible pod")
    rng = np.random.Generator(np.random.PCG64(12))
    nodes = synth.make_nodes(40, rng)
    nodes.allowed_pods[:] = 300
    t, used = synth.make_node_pods(nodes, rng, 8, per_node=(256, 256), n_pdb=4, pdb_frac=0.3)
    nodes.alloc_milli_cpu[:] = np.maximum(nodes.req_milli_cpu + rng.integers(0, 2000, nodes.n), 1000)
    q = synth.QuotaTable(8)
    q.limit_mask[:] = 0xF
    q.used[:] = used
    q.limit[:] = (used * 1.02).astype(np.int64)
    pods = synth.make_pods(6, rng, 8)
    compare(runtime, oracle_lib, profile(quota=True).to_ks_config(), nodes, q, t, pods,
            np.full(6, 9000, np.int32), "256 pods per node")


def test_overlapping_budgets(runtime, oracle_lib):
    """Pods matching 2-4 PodDisruptionBudgets (filterPodsWithPDBViolation decrements every matching budget, preempt.go
    :232-257): the hand-worked case, then random nodes of 10-250 pods with tight budgets."""
    cfg = profile(quota=True).to_ks_config()
    nodes = hand.cluster(1)
    specs = [(0, 100, 1, 1000, 0, abi.KS_NPOD_IN_QUOTA, 0), (0, 100, 2, 1000, 0, abi.KS_NPOD_IN_QUOTA, 0),
             hand.BASE[2], hand.BASE[3]]
    t = hand.running(nodes, specs, npdb=2, allowed=[1, 0])
    t.pdb_more[0, 1] = 1
    outs = compare(runtime, oracle_lib, cfg, nodes, hand.quotas(t), t, hand.preemptor(1500), [1000], "two budgets")
    assert list(outs[0]["victims"]) == [1, 0] and outs[0]["num_pdb_violations"] == 1
    viol = 0
    for seed, per_node in ((41, (10, 60)), (42, (100, 250))):
        rng = np.random.Generator(np.random.PCG64(seed))
        nodes = synth.make_nodes(400, rng)
        nodes.allowed_pods[:] = 256
        t, used = synth.make_node_pods(nodes, rng, 4, per_node=per_node, n_pdb=9, pdb_frac=0.7, multi_pdb_frac=0.5)
        t.pdb_allowed[:] = rng.integers(0, 3, 9)
        assert (t.pdb_more[2] >= 0).any()
        nodes.alloc_milli_cpu[:] = np.maximum(nodes.req_milli_cpu + rng.integers(0, 1000, nodes.n), 1000)
        q = synth.QuotaTable(4)
        q.limit_mask[:] = 0xF
        q.used[:] = used
        q.limit[:] = used * 2
        pods = synth.make_pods(10, rng, 4)
        pods.req_milli_cpu[:] = np.maximum(pods.req_milli_cpu, 4000)
        outs = compare(runtime, oracle_lib, cfg, nodes, q, t, pods, np.full(10, 9000, np.int32), f"multi-pdb {seed}")
        viol += sum(o["num_pdb_violations"] for o in outs)
    assert viol > 0  # (seed 42's 100-250-pod nodes: every chosen node has violating victims)


def test_reloaded_nodes_drop_the_node_pod_table(runtime):
    """ks_load_nodes invalidates the node-pod table (its rows and scratch belong to the old nodes): ks_preempt refuses
    with KS_ESTATE until ks_load_node_pods runs again, then works at the new node count."""
    w = synth.c2_preempt(seed=5, n_nodes=200, n_preemptors=2)
    ev = runtime.Evaluator(w.cfg, w.nodes.copy(), w.quotas.copy())
    try:
        ev.load_node_pods(w.node_pods)
        ev.preempt(w.preemptors.rows([0]), int(w.priority[0]))
        big = synth.c2_preempt(seed=6, n_nodes=900, n_preemptors=2)
        ev.load_nodes(big.nodes.copy())
        with pytest.raises(runtime.KsError) as e:
            ev.preempt(big.preemptors.rows([0]), int(big.priority[0]))
        assert e.value.rc == abi.KS_ESTATE
        ev.load_node_pods(big.node_pods)
        r = ev.preempt(big.preemptors.rows([0]), int(big.priority[0]), node_status=True)
        assert len(r["node_status"]) == 900
    finally:
        ev.close()
