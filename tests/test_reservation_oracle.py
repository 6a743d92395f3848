"""The C oracle's Reservation path (oracle/koord_oracle.c) against the object-level restatement
(oracle/reservation_ref.py, itself pinned by the reference's reservation tests) on small random
clusters: placements, scores, nominated reservations and the reservation cache after Reserve."""
import numpy as np
import pytest

from koordinator_amd import abi
from koordinator_amd.cluster import NodeTable, PodTable, ReservationTable
from koordinator_amd.config import CPU, MEMORY, NodeResourcesFitArgs, SchedulerProfile
from oracle import reservation_ref as R
from oracle.oracle import Oracle

GI = 1 << 30
W_RES = 5000
POLICIES = {abi.KS_RSV_POLICY_DEFAULT: R.DEFAULT, abi.KS_RSV_POLICY_ALIGNED: R.ALIGNED,
            abi.KS_RSV_POLICY_RESTRICTED: R.RESTRICTED}


def make_case(seed, n=6, nr=12, p=40):
    rng = np.random.default_rng(seed)
    nodes = NodeTable(n)
    nodes.alloc_milli_cpu[:] = rng.choice([8000, 16000, 32000], n)
    nodes.alloc_memory[:] = rng.choice([16, 32, 64], n) * GI
    nodes.allowed_pods[:] = rng.choice([5, 8, 110], n)
    rs = ReservationTable(nr)
    rs.node[:] = rng.integers(0, n, nr)
    rs.owner_classes[:] = [np.uint64(rng.integers(0, 16)) for _ in range(nr)]
    rs.flags[:] = rng.choice([0, 0, 0, abi.KS_RSV_UNSCHEDULABLE, abi.KS_RSV_ALLOCATE_ONCE], nr)
    rs.policy[:] = rng.choice([0, 1, 2], nr)
    rs.order[:] = np.where(rng.random(nr) < 0.25, rng.integers(1, 5, nr), 0)
    rs.key_mask[:] = rng.choice([1, 3, 3, 3], nr)
    rs.allocatable[0] = rng.choice([1000, 2000, 4000], nr)
    rs.allocatable[1] = np.where(rs.key_mask & 2, rng.choice([1, 2, 4], nr) * GI, 0)
    rs.assigned[:] = np.where(rng.random(nr) < 0.3, rng.integers(1, 3, nr), 0)
    rs.allocated[0] = np.where(rs.assigned > 0, rs.allocatable[0] * rng.choice([0, 1, 2, 4], nr) // 4, 0)
    rs.allocated[1] = np.where(rs.assigned > 0, rs.allocatable[1] * rng.choice([0, 1, 4], nr) // 4, 0)
    # NodeInfo holds the reserve pods plus the pods assigned to them, and some other pods
    base_cpu = rng.integers(0, 4, n) * 1000
    base_mem = rng.integers(0, 8, n) * GI
    nodes.req_milli_cpu[:] = base_cpu
    nodes.req_memory[:] = base_mem
    nodes.nonzero_milli_cpu[:] = base_cpu
    nodes.nonzero_memory[:] = base_mem
    nodes.pod_count[:] = rng.integers(0, 3, n)
    for r in range(nr):
        k = rs.node[r]
        nodes.req_milli_cpu[k] += rs.allocatable[0, r] + rs.allocated[0, r]
        nodes.req_memory[k] += rs.allocatable[1, r] + rs.allocated[1, r]
        nodes.nonzero_milli_cpu[k] += rs.allocatable[0, r] + rs.allocated[0, r]
        nodes.nonzero_memory[k] += (rs.allocatable[1, r] if rs.key_mask[r] & 2 else 200 << 20) + rs.allocated[1, r]
        nodes.pod_count[k] += 1 + rs.assigned[r]
    pods = PodTable(p)
    pods.req_milli_cpu[:] = rng.choice([0, 250, 500, 1000, 2000, 3000], p)
    pods.req_memory[:] = rng.choice([0, 256 << 20, GI, 2 * GI], p)
    pods.nonzero_milli_cpu[:] = np.where(pods.req_milli_cpu > 0, pods.req_milli_cpu, 100)
    pods.nonzero_memory[:] = np.where(pods.req_memory > 0, pods.req_memory, 200 << 20)
    pods.rsv_class[:] = np.where(rng.random(p) < 0.8, rng.integers(0, 16, p), -1)
    pods.flags[:] = np.where(rng.random(p) < 0.2, abi.KS_POD_RSV_AFFINITY, 0)
    return nodes, rs, pods


def py_schedule(nodes, rs, pods):
    """one pod at a time with reservation_ref; NodeResourcesFit LeastAllocated cpu/memory w=1"""
    n = nodes.n
    req = {"cpu": nodes.req_milli_cpu.copy(), "memory": nodes.req_memory.copy()}
    nz = {"cpu": nodes.nonzero_milli_cpu.copy(), "memory": nodes.nonzero_memory.copy()}
    podc = nodes.pod_count.astype(np.int64).copy()
    alloc = {"cpu": nodes.alloc_milli_cpu, "memory": nodes.alloc_memory}
    names = ["cpu", "memory"]
    allocated = [{names[d]: int(rs.allocated[d, r]) for d in range(2) if rs.key_mask[r] >> d & 1} for r in range(rs.r)]
    assigned = [int(a) for a in rs.assigned]
    out = []
    for i in range(pods.n):
        pod_req = {k: int(v) for k, v in (("cpu", pods.req_milli_cpu[i]), ("memory", pods.req_memory[i])) if v}
        cls = int(pods.rsv_class[i])
        aff = bool(pods.flags[i] & abi.KS_POD_RSV_AFFINITY)
        feas, fit, noms, orders = {}, {}, {}, {}
        for k in range(n):
            rows = [r for r in range(rs.r) if rs.node[r] == k]
            objs = []
            for r in rows:
                objs.append(R.Reservation(
                    name=str(r), allocatable={names[d]: int(rs.allocatable[d, r]) for d in range(2) if rs.key_mask[r] >> d & 1},
                    allocated=dict(allocated[r]), policy=POLICIES[int(rs.policy[r])], order=int(rs.order[r]),
                    owner_match=cls >= 0 and bool((int(rs.owner_classes[r]) >> cls) & 1),
                    unschedulable=bool(rs.flags[r] & abi.KS_RSV_UNSCHEDULABLE),
                    allocate_once=bool(rs.flags[r] & abi.KS_RSV_ALLOCATE_ONCE), assigned=assigned[r]))
            node = R.NodeState({"cpu": int(alloc["cpu"][k]), "memory": int(alloc["memory"][k])},
                               int(nodes.allowed_pods[k]), {"cpu": int(req["cpu"][k]), "memory": int(req["memory"][k])},
                               {"cpu": int(nz["cpu"][k]), "memory": int(nz["memory"][k])}, int(podc[k]))
            res = R.restore(node, objs, False, aff)
            eff, matched = (res[0], res[3]) if res else (node, [])
            ok = eff.pods + 1 <= eff.allowed_pods
            if pod_req:
                ok &= pod_req.get("cpu", 0) <= eff.allocatable["cpu"] - eff.requested.get("cpu", 0)
                ok &= pod_req.get("memory", 0) <= eff.allocatable["memory"] - eff.requested.get("memory", 0)
            if aff:
                if not matched:
                    ok = False
                else:
                    ok &= R.filter_with_reservations(pod_req, eff.allocatable, eff.allowed_pods, eff.pods, len(matched),
                                                     res[1], res[2], matched, True)[0]
            if not ok:
                continue
            feas[k] = True
            s = 0
            for d, pnz in (("cpu", pods.nonzero_milli_cpu[i]), ("memory", pods.nonzero_memory[i])):
                cap, rq = int(eff.allocatable[d]), int(eff.nonzero[d] + pnz)
                s += 0 if rq > cap else (cap - rq) * 100 // cap
            fit[k] = s // 2
            if matched:
                noms[k] = R.nominate(pod_req, eff.allocatable, eff.allowed_pods, eff.pods, res[1], res[2], matched)
                _, o = R.most_preferred_by_order(matched)
                orders[k] = o or 0
        if not feas:
            out.append((-1, 0, -1))
            continue
        ks = sorted(feas)
        pref = None
        for k in ks:
            if orders.get(k, 0) and (pref is None or orders[k] < orders[pref]):
                pref = k
        raw = [1000 if k == pref else (R.score_reservation(pod_req, noms[k]) if noms.get(k) else 0) for k in ks]
        norm = R.default_normalize(raw)
        tot = [fit[k] + W_RES * s for k, s in zip(ks, norm)]
        best = max(range(len(ks)), key=lambda j: (tot[j], -ks[j]))
        k = ks[best]
        nom = noms.get(k)
        rid = int(nom.name) if nom else -1
        out.append((k, tot[best], rid))
        if rid >= 0:
            for d in range(2):
                if rs.key_mask[rid] >> d & 1 and names[d] in pod_req:
                    allocated[rid][names[d]] = allocated[rid].get(names[d], 0) + pod_req[names[d]]
            assigned[rid] += 1
        req["cpu"][k] += pods.req_milli_cpu[i]
        req["memory"][k] += pods.req_memory[i]
        nz["cpu"][k] += pods.nonzero_milli_cpu[i]
        nz["memory"][k] += pods.nonzero_memory[i]
        podc[k] += 1
    return out, allocated, assigned


def profile():
    return SchedulerProfile(fit=NodeResourcesFitArgs(resources={CPU: 1, MEMORY: 1}), loadaware=None,
                            reservation_weight=W_RES).to_ks_config()


@pytest.mark.parametrize("seed", range(12))
def test_c_oracle_matches_object_level(seed):
    nodes, rs, pods = make_case(seed)
    o = Oracle(profile(), nodes, reservations=rs)
    got = o.schedule(pods)
    want, allocated, assigned = py_schedule(nodes, rs, pods)
    assert [tuple(x) for x in zip(got["node"].tolist(), got["score"].tolist(), got["reservation"].tolist())] == want
    g_alloc, g_assigned = o.read_reservations()
    assert g_assigned.tolist() == assigned
    for r in range(rs.r):
        for d, name in enumerate(("cpu", "memory")):
            assert g_alloc[r, d] == allocated[r].get(name, rs.allocated[d, r] if not (rs.key_mask[r] >> d & 1) else 0)


def test_score_with_order_cluster():
    """TestScoreWithOrder (scoring_test.go:255) as a 4-node cluster through the C oracle."""
    nodes = NodeTable(4)
    nodes.alloc_milli_cpu[:] = 32000
    nodes.alloc_memory[:] = 64 * GI
    nodes.allowed_pods[:] = 110
    rs = ReservationTable(4)
    rs.node[:] = [0, 1, 2, 3]
    rs.owner_classes[:] = 1
    rs.key_mask[:] = 3
    rs.allocatable[0] = 4000
    rs.allocatable[1] = 8 * GI
    rs.order[3] = 123456
    nodes.req_milli_cpu[:] = 4000
    nodes.req_memory[:] = 8 * GI
    nodes.nonzero_milli_cpu[:] = 4000
    nodes.nonzero_memory[:] = 8 * GI
    nodes.pod_count[:] = 1
    pod = PodTable(1)
    pod.req_milli_cpu[:] = 4000
    pod.req_memory[:] = 8 * GI
    pod.nonzero_milli_cpu[:] = 4000
    pod.nonzero_memory[:] = 8 * GI
    pod.rsv_class[:] = 0
    o = Oracle(profile(), nodes, reservations=rs)
    reasons, scores, total = o.eval_pod(pod)
    assert reasons.tolist() == [0, 0, 0, 0]
    assert scores[:, abi.KS_SCORE_RESERVATION].tolist() == [10, 10, 10, 100]
    res = o.schedule(pod)
    assert res["node"][0] == 3 and res["reservation"][0] == 3


def test_device_pods_never_nominated_into_device_less_reservations():
    """DeviceShare's FilterReservation (deviceshare/plugin.go:322-358) fails for a reservation whose reserve pod holds
    no device when the pod has device requests, so NominateReservation (nominator.go:163-168) skips it and Reserve
    (reservation/plugin.go:546-560) assumes the pod into none; with DeviceShare off the same pods go into them."""
    from koordinator_amd import synth

    w = synth.c3_rsv(seed=91, n_nodes=150, n_pods=400, policy_frac=0.3)
    dev = (w.pods.gpu_core + w.pods.gpu_memory + w.pods.gpu_memory_ratio + w.pods.rdma) > 0
    orc = Oracle(w.cfg, w.nodes.copy(), **w.tables())
    got = orc.schedule(w.pods)
    orc.close()
    placed = got["status"] == abi.KS_S_SCHEDULED
    assert (placed & dev & (w.pods.rsv_class >= 0)).sum() > 20
    assert not (dev & (got["reservation"] >= 0)).any()
    assert ((~dev) & (got["reservation"] >= 0)).sum() > 20
    w.profile.deviceshare = None
    orc = Oracle(w.cfg, w.nodes.copy(), **w.tables())
    got2 = orc.schedule(w.pods)
    orc.close()
    assert (dev & (got2["reservation"] >= 0)).sum() > 10


def test_device_pods_into_device_holding_reservations():
    """Reservations holding GPUs / RDMA (deviceshare/reservation.go): device pods are nominated only into them, and each
    assigned pod's allocation on the reservation's minors joins its allocated (never outside its minors)."""
    from koordinator_amd import synth

    w = synth.c3_rsv(seed=92, n_nodes=200, n_pods=800, policy_frac=0.3, dev_rsv_frac=0.7)
    rs = w.reservations
    held = (rs.dev_allocatable != 0).any(axis=1)
    dev = (w.pods.gpu_core + w.pods.gpu_memory + w.pods.gpu_memory_ratio + w.pods.rdma) > 0
    orc = Oracle(w.cfg, w.nodes.copy(), **w.tables())
    got = orc.schedule(w.pods)
    dald = orc.read_reservation_devices()
    orc.close()
    into = got["reservation"]
    di = dev & (into >= 0)
    assert di.sum() > 10
    assert held[into[di]].all()
    grown = dald != rs.dev_allocated
    assert grown.any()
    assert not (grown & (rs.dev_allocatable == 0)).any()
    assert (dald >= rs.dev_allocated).all()
