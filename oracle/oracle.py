"""ctypes wrapper of oracle/libkoord_oracle.so — TEST INFRASTRUCTURE ONLY.

Used by tests/ (parity checker), __graft_entry__.smoke() and bench.py's
cpu_baseline leg.  Consumes the same SoA tables as the HIP library
(koordinator_amd.cluster), so both sides see byte-identical inputs.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from koordinator_amd import abi
from koordinator_amd.cluster import (CpuState, DeviceTable, NodePodTable, NumaNodes, NodeState, NodeTable, PodTable,
                                     QuotaTable, ReservationTable)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libkoord_oracle.so")


def build(force: bool = False) -> str:
    srcs = [os.path.join(HERE, f) for f in ("koord_oracle.c", "cpu_accumulator.c", "cpu_accumulator.h")]
    if force or not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < max(os.path.getmtime(f) for f in srcs):
        subprocess.check_call(["make", "-s", "-C", HERE])
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.ko_create.restype = C.c_void_p
        L.ko_create.argtypes = [C.POINTER(abi.KsConfig), C.POINTER(abi.KsNodeCols), C.c_int64, C.c_int]
        L.ko_destroy.argtypes = [C.c_void_p]
        L.ko_load_quotas.argtypes = [C.c_void_p, C.POINTER(abi.KsQuotaCols), C.c_int32]
        L.ko_load_reservations.argtypes = [C.c_void_p, C.POINTER(abi.KsReservationCols), C.c_int32]
        L.ko_read_reservations.argtypes = [C.c_void_p, abi.P64, abi.P32]
        L.ko_read_reservation_devices.argtypes = [C.c_void_p, abi.P64]
        L.ko_load_devices.argtypes = [C.c_void_p, C.POINTER(abi.KsDeviceCols)]
        L.ko_read_devices.argtypes = [C.c_void_p, abi.P64, abi.P64, abi.P64]
        L.ko_read_devices_rdma.argtypes = [C.c_void_p, abi.P64]
        L.ko_load_cpu_state.argtypes = [C.c_void_p, C.POINTER(abi.KsCpuTopology), C.c_int32, C.POINTER(abi.KsCpuStateCols)]
        L.ko_read_cpu_state.argtypes = [C.c_void_p, abi.PU64, abi.PU64, abi.PU64]
        L.ko_fetch_cpusets.argtypes = [C.c_void_p, abi.PU64, C.c_int32]
        L.ko_fetch_numa_alloc.argtypes = [C.c_void_p, abi.P64, C.c_int32]
        L.ko_load_numa_nodes.argtypes = [C.c_void_p, C.POINTER(abi.KsNumaNodeCols)]
        L.ko_read_numa_nodes.argtypes = [C.c_void_p, abi.P64, abi.P64]
        L.ko_schedule.argtypes = [C.c_void_p, C.POINTER(abi.KsPodCols), C.c_int32, C.POINTER(abi.KsResult)]
        L.ko_eval_pod.argtypes = [C.c_void_p, C.POINTER(abi.KsPodCols), abi.PU32, abi.P64, abi.P64]
        L.ko_assume.argtypes = [C.c_void_p, C.POINTER(abi.KsPodCols), C.c_int32, C.POINTER(abi.KsResult), abi.P64]
        L.ko_unreserve.argtypes = [C.c_void_p, C.POINTER(abi.KsPodCols), C.POINTER(abi.KsResult), abi.PU64, abi.P64]
        L.ko_read_nodes.argtypes = [C.c_void_p, C.POINTER(abi.KsNodeState)]
        L.ko_read_quota_used.argtypes = [C.c_void_p, abi.P64]
        L.ko_load_node_pods.argtypes = [C.c_void_p, C.POINTER(abi.KsNodePodCols), C.c_int64, abi.P32, C.c_int32]
        L.ko_preempt.argtypes = [C.c_void_p, C.POINTER(abi.KsPodCols), C.c_int32, C.c_uint32, C.c_int32,
                                 C.POINTER(C.c_uint8), C.POINTER(abi.KsPreemptResult), abi.P32, C.c_int32,
                                 C.POINTER(C.c_uint8)]
        L.ko_least_requested_score.restype = C.c_int64
        L.ko_least_requested_score.argtypes = [C.c_int64, C.c_int64]
        L.ko_most_requested_score.restype = C.c_int64
        L.ko_most_requested_score.argtypes = [C.c_int64, C.c_int64]
        L.ko_estimated_used.restype = C.c_int64
        L.ko_estimated_used.argtypes = [C.c_int64, C.c_int64, C.c_int64, C.c_int64]
        L.ko_take_cpus.restype = C.c_int
        L.ko_take_cpus.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int,
                                   C.c_int, C.c_void_p]
        L.ko_spread_order.restype = C.c_int
        L.ko_spread_order.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
        L.ko_topo_finish.argtypes = [C.c_void_p]
        L.ko_topology_merge.restype = C.c_int
        L.ko_topology_merge.argtypes = [C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                        C.POINTER(C.c_uint32), C.POINTER(C.c_int)]
        L.ko_dev_hints.argtypes = [C.c_void_p, C.POINTER(abi.KsPodCols), C.c_int64, C.POINTER(C.c_int),
                                   C.POINTER(C.c_int), C.c_void_p, C.c_void_p]
        _lib = L
    return _lib


KO_MAX_CPUS = 256
EXCL = {"None": 0, "PCPULevel": 1, "NUMANodeLevel": 2}
BIND = {"FullPCPUs": 1, "SpreadByPCPUs": 2}
STRATEGY = {"Most": 0, "Least": 1}


class KoTopo(C.Structure):
    _fields_ = [("ncpus", C.c_int), ("core", C.c_int * KO_MAX_CPUS), ("node", C.c_int * KO_MAX_CPUS),
                ("socket", C.c_int * KO_MAX_CPUS), ("num_cores", C.c_int), ("num_nodes", C.c_int),
                ("num_sockets", C.c_int)]


def topo_from_ids(core, node, socket) -> KoTopo:
    t = KoTopo()
    t.ncpus = len(core)
    for i in range(len(core)):
        t.core[i], t.node[i], t.socket[i] = int(core[i]), int(node[i]), int(socket[i])
    lib().ko_topo_finish(C.byref(t))
    return t


def take_cpus(t: KoTopo, avail, needed: int, bind: str, excl: str = "None", strategy: str = "Most",
              max_ref: int = 1, refcount=None, alloc_excl=None):
    """takeCPUs on the oracle; returns the sorted CPU list or None on error."""
    n = t.ncpus
    av = np.zeros(KO_MAX_CPUS, np.uint8)
    av[:n] = np.asarray(avail, np.uint8)[:n]
    rc = np.zeros(KO_MAX_CPUS, np.int32)
    if refcount is not None:
        rc[:n] = refcount
    ex = np.full(KO_MAX_CPUS, -1, np.int8)
    if alloc_excl is not None:
        ex[:n] = alloc_excl
    out = np.zeros(KO_MAX_CPUS, np.uint8)
    rv = lib().ko_take_cpus(C.byref(t), max_ref, av.ctypes.data, rc.ctypes.data, ex.ctypes.data, needed,
                            BIND[bind], EXCL[excl], STRATEGY[strategy], out.ctypes.data)
    return None if rv != 0 else [int(c) for c in np.nonzero(out[:n])[0]]


def spread_order(t: KoTopo, strategy: str = "Most"):
    out = np.zeros(KO_MAX_CPUS, np.int32)
    k = lib().ko_spread_order(C.byref(t), STRATEGY[strategy], out.ctypes.data)
    return [int(x) for x in out[:k]]


POLICY = {"best-effort": abi.KS_NUMA_POLICY_BEST_EFFORT, "restricted": abi.KS_NUMA_POLICY_RESTRICTED,
          "single-numa-node": abi.KS_NUMA_POLICY_SINGLE_NUMA_NODE}


def topology_merge(policy: str, numa_nodes: int, lists):
    """The topology manager's Merge (koord_oracle.c ko_merge_hints) over hint lists after
    filterProvidersHints; a hint is (mask, preferred, score), mask 0 = nil.  Returns (admit, mask, preferred)."""
    lens = np.array([len(l) for l in lists] or [0], np.int32)
    flat = [h for l in lists for h in l] or [(0, 0, 0)]
    masks = np.array([h[0] for h in flat], np.uint32)
    prefs = np.array([int(h[1]) for h in flat], np.int32)
    scores = np.array([h[2] for h in flat], np.int64)
    aff = C.c_uint32()
    pref = C.c_int()
    admit = lib().ko_topology_merge(POLICY[policy], numa_nodes, len(lists), lens.ctypes.data, masks.ctypes.data,
                                    prefs.ctypes.data, scores.ctypes.data, C.byref(aff), C.byref(pref))
    return admit, aff.value, bool(pref.value)


class Oracle:
    """Sequential one-pod-at-a-time scheduler on the CPU (reduced form)."""

    def __init__(self, cfg: abi.KsConfig, nodes: NodeTable, quotas: QuotaTable | None = None, nthreads: int = 1,
                 reservations: ReservationTable | None = None, devices: DeviceTable | None = None,
                 cpu_state: CpuState | None = None, numa_nodes: NumaNodes | None = None):
        self.L = lib()
        self.cfg = cfg
        self.n = nodes.n
        self.nprops = int(np.asarray(nodes.topo_count).shape[0])
        self._cols = nodes.ks()
        self.h = self.L.ko_create(C.byref(cfg), C.byref(self._cols), nodes.n, int(nthreads))
        self.nq = 0
        if quotas is not None:
            self._q = quotas.ks()
            self.L.ko_load_quotas(self.h, C.byref(self._q), quotas.q)
            self.nq = quotas.q
        self.nr = 0
        if reservations is not None:
            self._r = reservations.ks()
            if self.L.ko_load_reservations(self.h, C.byref(self._r), reservations.r) != 0:
                raise ValueError("reservation row references an unknown node")
            self.nr = reservations.r
        if devices is not None:
            self._d = devices.ks()
            self.L.ko_load_devices(self.h, C.byref(self._d))
        if cpu_state is not None:
            self._cs = cpu_state.ks()
            self._ct = cpu_state.topo_array()
            self.L.ko_load_cpu_state(self.h, self._ct, len(cpu_state.topologies), C.byref(self._cs))
        if numa_nodes is not None:
            self._nn = numa_nodes.ks()
            self.L.ko_load_numa_nodes(self.h, C.byref(self._nn))

    def close(self):
        if self.h:
            self.L.ko_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def schedule(self, pods: PodTable):
        out = (abi.KsResult * max(pods.n, 1))()
        cols = pods.ks()
        self.L.ko_schedule(self.h, C.byref(cols), pods.n, out)
        arr = np.frombuffer(out, dtype=np.dtype(abi.RESULT_DTYPE_FIELDS), count=pods.n)
        return {"node": arr["node"].copy(), "status": arr["status"].copy(), "score": arr["score"].copy(),
                "reservation": arr["reservation"].copy(), "gpu_minors": arr["gpu_minors"].copy(),
                "rdma_minors": arr["rdma_minors"].copy()}

    def schedule_raw(self, pods: PodTable) -> np.ndarray:
        out = (abi.KsResult * max(pods.n, 1))()
        cols = pods.ks()
        self.L.ko_schedule(self.h, C.byref(cols), pods.n, out)
        return np.frombuffer(out, dtype=np.dtype(abi.RESULT_DTYPE_FIELDS), count=pods.n).copy()

    def assume(self, pod: PodTable, node: int):
        """ko_assume: (result record, cpuset words, NUMA allocation [KS_MAX_NUMA][2])"""
        r = (abi.KsResult * 1)()
        na = np.zeros((abi.KS_MAX_NUMA, 2), np.int64)
        cols = pod.ks()
        if self.L.ko_assume(self.h, C.byref(cols), int(node), r, na.ctypes.data_as(abi.P64)) != 0:
            raise ValueError("ko_assume failed")
        rec = np.frombuffer(r, dtype=np.dtype(abi.RESULT_DTYPE_FIELDS), count=1).copy()
        return rec, self.fetch_cpusets(1)[0].copy(), na

    def unreserve(self, pod: PodTable, r, cpuset=None, numa_alloc=None):
        rec = np.ascontiguousarray(r, np.dtype(abi.RESULT_DTYPE_FIELDS)).reshape(1)
        cols = pod.ks()
        cs = None if cpuset is None else np.ascontiguousarray(cpuset, np.uint64)
        na = None if numa_alloc is None else np.ascontiguousarray(numa_alloc, np.int64)
        if self.L.ko_unreserve(self.h, C.byref(cols), rec.ctypes.data_as(C.POINTER(abi.KsResult)),
                               cs.ctypes.data_as(abi.PU64) if cs is not None else None,
                               na.ctypes.data_as(abi.P64) if na is not None else None) != 0:
            raise ValueError("ko_unreserve failed")

    def eval_pod(self, pod: PodTable):
        reasons = np.zeros(self.n, np.uint32)
        scores = np.zeros(self.n * abi.KS_NUM_SCORE_PLUGINS, np.int64)
        total = np.zeros(self.n, np.int64)
        cols = pod.ks()
        self.L.ko_eval_pod(self.h, C.byref(cols), reasons.ctypes.data_as(abi.PU32),
                           scores.ctypes.data_as(abi.P64), total.ctypes.data_as(abi.P64))
        return reasons, scores.reshape(self.n, abi.KS_NUM_SCORE_PLUGINS), total

    def dev_hints(self, pod: PodTable, node: int):
        """DeviceShare's topology hints for pod 0 on `node`: (lists, [(mask, preferred)]); lists 0 = none."""
        cols = pod.ks()
        lists, nh = C.c_int(), C.c_int()
        masks = np.zeros(16, np.uint32)
        prefs = np.zeros(16, np.int32)
        self.L.ko_dev_hints(self.h, C.byref(cols), node, C.byref(lists), C.byref(nh), masks.ctypes.data,
                            prefs.ctypes.data)
        return lists.value, [(int(masks[i]), bool(prefs[i])) for i in range(nh.value)]

    def read_nodes(self) -> NodeState:
        st = NodeState(self.n, getattr(self, 'nprops', 0))
        s = st.ks()
        self.L.ko_read_nodes(self.h, C.byref(s))
        return st

    def read_reservations(self):
        allocated = np.zeros(max(self.nr, 1) * abi.KS_RSV_DIMS, np.int64)
        assigned = np.zeros(max(self.nr, 1), np.int32)
        self.L.ko_read_reservations(self.h, allocated.ctypes.data_as(abi.P64), assigned.ctypes.data_as(abi.P32))
        return allocated[: self.nr * abi.KS_RSV_DIMS].reshape(self.nr, abi.KS_RSV_DIMS), assigned[: self.nr]

    def read_reservation_devices(self):
        out = np.zeros(max(self.nr, 1) * abi.KS_DEV_WORDS, np.int64)
        self.L.ko_read_reservation_devices(self.h, out.ctypes.data_as(abi.P64))
        return out[: self.nr * abi.KS_DEV_WORDS].reshape(self.nr, abi.KS_DEV_WORDS)

    def read_devices(self):
        G = abi.KS_MAX_GPUS
        out = [np.zeros(G * max(self.n, 1), np.int64) for _ in range(3)]
        self.L.ko_read_devices(self.h, *[o.ctypes.data_as(abi.P64) for o in out])
        R = abi.KS_MAX_RDMA
        r = np.zeros(R * max(self.n, 1), np.int64)
        self.L.ko_read_devices_rdma(self.h, r.ctypes.data_as(abi.P64))
        return tuple(o[: G * self.n].reshape(G, self.n) for o in out) + (r[: R * self.n].reshape(R, self.n),)

    def read_numa_nodes(self):
        K = abi.KS_MAX_NUMA
        out = [np.zeros((max(self.n, 1), K), np.int64) for _ in range(2)]
        self.L.ko_read_numa_nodes(self.h, *[o.ctypes.data_as(abi.P64) for o in out])
        return tuple(o[: self.n] for o in out)

    def read_cpu_state(self):
        W = abi.KS_CPU_WORDS
        out = [np.zeros((max(self.n, 1), W), np.uint64) for _ in range(3)]
        self.L.ko_read_cpu_state(self.h, *[o.ctypes.data_as(abi.PU64) for o in out])
        return tuple(o[: self.n] for o in out)

    def fetch_cpusets(self, p: int) -> np.ndarray:
        if not self.h:
            raise ValueError("oracle closed")
        out = np.zeros((max(p, 1), abi.KS_CPU_WORDS), np.uint64)
        if self.L.ko_fetch_cpusets(self.h, out.ctypes.data_as(abi.PU64), p) != 0:
            raise ValueError("no cpusets for that many pods")
        return out[:p]

    def fetch_numa_alloc(self, p: int) -> np.ndarray:
        """each pod's NUMA-node allocation [p][KS_MAX_NUMA][2] (cpu milli, memory) of the last schedule"""
        if not self.h:
            raise ValueError("oracle closed")
        out = np.zeros((max(p, 1), abi.KS_MAX_NUMA, 2), np.int64)
        if self.L.ko_fetch_numa_alloc(self.h, out.ctypes.data_as(abi.P64), p) != 0:
            raise ValueError("no NUMA allocations for that many pods")
        return out[:p]

    def load_node_pods(self, t: NodePodTable):
        cols = t.ks()
        if self.L.ko_load_node_pods(self.h, C.byref(cols), t.m, t.pdb_allowed.ctypes.data_as(abi.P32),
                                    len(t.pdb_allowed)) != 0:
            raise ValueError("ko_load_node_pods: a row references a node outside the table")
        self.npods = t.m

    def preempt(self, pod: PodTable, priority: int, flags: int = 0, nominated_node: int = -1, unresolvable=None,
                node_status: bool = False) -> dict:
        out = abi.KsPreemptResult()
        cap = max(getattr(self, "npods", 0), 1)
        vic = np.zeros(cap, np.int32)
        ns = np.zeros(max(self.n, 1), np.uint8) if node_status else None
        ur = None if unresolvable is None else np.ascontiguousarray(unresolvable, np.uint8)
        cols = pod.ks()
        if self.L.ko_preempt(self.h, C.byref(cols), int(priority), int(flags), int(nominated_node),
                             ur.ctypes.data_as(C.POINTER(C.c_uint8)) if ur is not None else None, C.byref(out),
                             vic.ctypes.data_as(abi.P32), cap,
                             ns.ctypes.data_as(C.POINTER(C.c_uint8)) if ns is not None else None) != 0:
            raise ValueError("ko_preempt: no node-pod table, ElasticQuota off or the pod has no quota")
        r = {"status": out.status, "node": out.node, "victims": vic[: out.num_victims].copy(),
             "num_pdb_violations": out.num_pdb_violations, "candidates": out.candidates,
             "potential_nodes": out.potential_nodes}
        if ns is not None:
            r["node_status"] = ns[: self.n].copy()
        return r

    def read_quota_used(self) -> np.ndarray:
        used = np.zeros(max(self.nq, 1) * abi.KS_QUOTA_DIMS, np.int64)
        self.L.ko_read_quota_used(self.h, used.ctypes.data_as(abi.P64))
        return used[: self.nq * abi.KS_QUOTA_DIMS].reshape(self.nq, abi.KS_QUOTA_DIMS)
