"""GPU: the informer-delta entry points (ks_update_devices / _cpu_state / _quotas / _reservation_usage) leave
the context exactly as the CPU oracle loaded with the merged tables -- same placements, scores, minors, CPUs and
state after scheduling a queue -- on C3 (devices, CPU state, SingleNUMANode nodes), C2 (quotas) and C4
(reservation usage).  The HIP context gets the old tables plus the delta; the oracle gets the new tables whole."""
import numpy as np
import pytest

from assume_util import assert_states_equal, state
from koordinator_amd import abi, synth
from koordinator_amd.cluster import CpuState, DeviceTable, QuotaTable

pytestmark = pytest.mark.gpu


def oracle_on(oracle_lib, w, nodes=None):
    return oracle_lib.Oracle(w.cfg, (nodes if nodes is not None else w.nodes).copy(), nthreads=8, **w.tables())


@pytest.fixture(scope="module")
def runtime():
    from koordinator_amd import runtime as rt

    rt.lib()
    return rt


def dev_rows(t: DeviceTable, idx) -> DeviceTable:
    r = DeviceTable(len(idx))
    r.flags = t.flags[idx].copy()
    for k in vars(t):
        v = getattr(t, k)
        if isinstance(v, np.ndarray) and v.ndim == 2:
            setattr(r, k, v[:, idx].copy())
    return r


def cpu_rows(t: CpuState, idx) -> CpuState:
    r = CpuState(len(idx), t.topologies)
    for k in ("topology", "allocated", "excl_pcpu", "excl_numa", "reserved"):
        setattr(r, k, getattr(t, k)[idx].copy())
    return r


def quota_rows(t: QuotaTable, idx) -> QuotaTable:
    r = QuotaTable(len(idx))
    for k in ("parent", "limit_mask", "min_mask"):
        setattr(r, k, getattr(t, k)[idx].copy())
    for k in ("limit", "used", "min", "nonpreemptible_used"):
        setattr(r, k, getattr(t, k)[:, idx].copy())
    return r


def check_same(runtime, a, b, w, label):
    """a: the HIP context after the deltas; b: the oracle on the merged tables."""
    ra, rb = a.schedule(w.pods), b.schedule(w.pods)
    for k in ("node", "status", "score", "reservation", "gpu_minors", "rdma_minors"):
        assert np.array_equal(ra[k], rb[k]), f"{label}: {k}"
    if w.cpus is not None:
        assert np.array_equal(a.fetch_cpusets(w.pods.n), b.fetch_cpusets(w.pods.n)), label
    assert_states_equal(state(a, w), state(b, w), label)


def test_update_devices_and_cpu_state(runtime, oracle_lib):
    w = synth.c3(seed=91, n_nodes=400, n_pods=500)
    w2 = synth.c3(seed=91, n_nodes=400, n_pods=500)  # same nodes; devices / CPU state re-drawn below
    rng = np.random.default_rng(5)
    idx = np.sort(rng.choice(400, 60, replace=False)).astype(np.int32)
    # new device usage and CPU allocations for the chosen nodes (a later snapshot of the same machines)
    dv = w.devices.copy()
    for k in range(abi.KS_MAX_GPUS):
        dv.used_core[k, idx] = np.where(dv.total_core[k, idx] > 0, rng.choice([0, 25, 50, 100], idx.size), 0)
        dv.used_ratio[k, idx] = dv.used_core[k, idx]
        dv.used_memory[k, idx] = dv.used_core[k, idx] * dv.total_memory[k, idx] // 100
    cs = w.cpus.copy()
    for i in idx:
        if cs.topology[i] >= 0:
            cs.allocated[i] = 0
            cs.excl_pcpu[i] = 0
            cs.excl_numa[i] = 0
    a = runtime.Evaluator(w.cfg, w.nodes.copy(), **w.tables())
    a.update_devices(idx, dev_rows(dv, idx))
    a.update_cpu_state(idx, cpu_rows(cs, idx))
    w2.devices, w2.cpus = dv, cs
    # the node table's cpuset counts follow the CPU state (numa_cpuset_cpus), as the host would resend them
    b = oracle_on(oracle_lib, w2, w.nodes)
    w.devices, w.cpus = dv, cs
    check_same(runtime, a, b, w, "devices + cpu")
    a.close()
    b.close()


def test_update_quotas(runtime, oracle_lib):
    w = synth.c2(n_nodes=500, n_pods=800, n_quotas=16)
    q2 = w.quotas.copy()
    idx = np.array([1, 4, 7, 11], np.int32)
    q2.limit[:, idx] = q2.limit[:, idx] // 2
    q2.used[:, idx] = q2.used[:, idx] + 1000
    a = runtime.Evaluator(w.cfg, w.nodes.copy(), **w.tables())
    a.update_quotas(idx, quota_rows(q2, idx))
    w.quotas = q2
    b = oracle_on(oracle_lib, w)
    check_same(runtime, a, b, w, "quotas")
    a.close()
    b.close()


def test_update_reservation_usage(runtime, oracle_lib):
    w = synth.c4(n_nodes=800, n_reservations=2000, n_pods=600)
    rs2 = w.reservations.copy()
    rng = np.random.default_rng(9)
    rows = np.sort(rng.choice(2000, 150, replace=False)).astype(np.int32)
    rs2.allocated[:, rows] = rs2.allocatable[:, rows] * rng.integers(0, 3, rows.size) // 4
    rs2.assigned[rows] = rng.integers(0, 3, rows.size)
    a = runtime.Evaluator(w.cfg, w.nodes.copy(), **w.tables())
    a.update_reservation_usage(rows, rs2.allocated[:, rows], rs2.assigned[rows])
    w.reservations = rs2
    b = oracle_on(oracle_lib, w)
    check_same(runtime, a, b, w, "reservation usage")
    a.close()
    b.close()


def rsv_rows(t, idx):
    from koordinator_amd.cluster import ReservationTable

    idx = np.asarray(idx)
    r = ReservationTable(idx.size)
    for k in ("node", "owner_classes", "flags", "policy", "order", "key_mask", "assigned"):
        setattr(r, k, getattr(t, k)[idx].copy())
    for k in ("allocatable", "allocated"):
        setattr(r, k, getattr(t, k)[:, idx].copy())
    return r


def test_add_delete_reservations(runtime, oracle_lib):
    """ks_add_reservations / ks_delete_reservations between two scheduled queues: the second queue's results and
    the final state equal the oracle loaded from scratch with the state after the first queue (node columns,
    reservation Allocated / assigned) and the merged reservation set."""
    w = synth.c4(n_nodes=800, n_reservations=2400, n_pods=700)
    rs = w.reservations
    first, later = np.arange(1800), np.arange(1800, 2400)
    rng = np.random.default_rng(12)
    dead = np.sort(rng.choice(1800, 150, replace=False))
    q1, q2 = w.pods.rows(range(250)), w.pods.rows(range(250, 700))
    ev = runtime.Evaluator(w.cfg, w.nodes.copy(), reservations=rsv_rows(rs, first))
    orc1 = oracle_lib.Oracle(w.cfg, w.nodes.copy(), nthreads=8, reservations=rsv_rows(rs, first))
    g1, o1 = ev.schedule(q1), orc1.schedule(q1)
    assert np.array_equal(g1["reservation"], o1["reservation"]) and np.array_equal(g1["node"], o1["node"])
    # the oracle's state after queue 1 as a fresh snapshot
    st = orc1.read_nodes()
    nodes2 = w.nodes.copy()
    for k, v in st.as_dict().items():
        setattr(nodes2, k, v.copy())
    allocd, assigned = orc1.read_reservations()
    orc1.close()
    rs1 = rsv_rows(rs, first)
    rs1.allocated = np.ascontiguousarray(allocd.T, np.int64)
    rs1.assigned = assigned.copy()
    # the deltas on the GPU context
    assert ev.add_reservations(rsv_rows(rs, later)) == 1800
    ev.delete_reservations(dead)
    live = np.setdiff1d(np.arange(2400), dead)  # caller rows of the merged table, in the oracle's row order
    merged = rsv_rows(rs, np.arange(2400))
    merged.allocated[:, :1800] = rs1.allocated
    merged.assigned[:1800] = rs1.assigned
    merged = rsv_rows(merged, live)
    orc2 = oracle_lib.Oracle(w.cfg, nodes2, nthreads=8, reservations=merged)
    g2, o2 = ev.schedule(q2), orc2.schedule(q2)
    for k in ("node", "status", "score"):
        assert np.array_equal(g2[k], o2[k]), k
    want_rsv = np.where(o2["reservation"] >= 0, live[np.maximum(o2["reservation"], 0)], -1)
    assert np.array_equal(g2["reservation"], want_rsv)
    assert (g2["reservation"] >= 1800).any(), "no pod went into an added reservation"
    assert not np.isin(g2["reservation"], dead).any()
    assert_states_equal({k: v for k, v in ev.read_nodes().as_dict().items()},
                        {k: v for k, v in orc2.read_nodes().as_dict().items()}, "nodes after deltas")
    ga, gs = ev.read_reservations()
    oa, os_ = orc2.read_reservations()
    assert np.array_equal(ga[live], oa) and np.array_equal(gs[live], os_)
    assert not ga[dead].any() and not gs[dead].any()
    ev.close()
    orc2.close()


def numa_rows(t, idx):
    from koordinator_amd.cluster import NumaNodes

    r = NumaNodes(len(idx))
    for k in ("count", "alloc_cpu", "alloc_memory", "used_cpu", "used_memory", "used_present", "cpuset_cpus"):
        setattr(r, k, getattr(t, k)[idx].copy())
    return r


def test_update_numa_nodes(runtime, oracle_lib):
    """ks_update_numa_nodes (NodeAllocation allocatedResources changed on some NUMA-policy nodes) == the oracle
    loaded with the merged NUMA-node table"""
    w = synth.c3(seed=93, n_nodes=400, n_pods=500)
    pol = np.nonzero(((w.nodes.numa_flags >> abi.KS_NUMA_POLICY_SHIFT) & 3) != 0)[0]
    rng = np.random.default_rng(14)
    idx = np.sort(rng.choice(pol, 60, replace=False)).astype(np.int32)
    nn = w.numa_nodes.copy()
    for i in idx:
        for k in range(nn.count[i]):
            nn.used_cpu[i, k] = nn.alloc_cpu[i, k] * rng.integers(0, 4) // 8
            nn.used_memory[i, k] = nn.alloc_memory[i, k] * rng.integers(0, 4) // 8
            nn.used_present[i, k] = 1 if (nn.used_cpu[i, k] or nn.used_memory[i, k] or rng.random() < 0.3) else 0
    a = runtime.Evaluator(w.cfg, w.nodes.copy(), **w.tables())
    a.update_numa_nodes(idx, numa_rows(nn, idx))
    w.numa_nodes = nn
    b = oracle_on(oracle_lib, w)
    check_same(runtime, a, b, w, "numa nodes")
    a.close()
    b.close()
