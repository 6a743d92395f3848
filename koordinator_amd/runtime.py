"""ctypes binding of libkoordgpu.so — the product path.

``Evaluator`` owns one ``ks_ctx`` (one scheduler profile on one GPU).  There
is no CPU fallback: if the in-tree HIP library is missing or no GPU is visible
the constructor raises.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from typing import Optional

import numpy as np

from . import abi
from .cluster import (CpuState, DeviceTable, NodePodTable, NumaNodes, NodeState, NodeTable, PodTable, QuotaTable,
                      QuotaTree, ReservationTable)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("KS_LIB_PATH") or os.path.join(HERE, "libkoordgpu.so")
CSRC = os.path.join(HERE, "csrc")

RESULT_DTYPE = np.dtype(abi.RESULT_DTYPE_FIELDS)


class KsError(RuntimeError):
    def __init__(self, rc: int, msg: str):
        super().__init__(f"ks error {rc}: {msg}")
        self.rc = rc


def build(force: bool = False) -> str:
    """Compile libkoordgpu.so for gfx950 in-tree (hipcc; the kernel variants are separate objects, built in
    parallel)."""
    jobs = max(1, min(16, os.cpu_count() or 1))
    args = ["make", "-s", f"-j{jobs}", "-C", CSRC]
    if force:
        args.append("-B")
    subprocess.check_call(args)
    return LIB_PATH


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise FileNotFoundError(f"{LIB_PATH} is not built; run koordinator_amd.runtime.build() (hipcc, gfx950)")
    L = C.CDLL(LIB_PATH)
    vp = C.c_void_p
    L.ks_create.argtypes = [C.POINTER(abi.KsConfig), C.POINTER(vp)]
    L.ks_destroy.argtypes = [vp]
    L.ks_destroy.restype = None
    L.ks_last_error.argtypes = [vp]
    L.ks_last_error.restype = C.c_char_p
    L.ks_load_nodes.argtypes = [vp, C.POINTER(abi.KsNodeCols), C.c_int64]
    L.ks_update_nodes.argtypes = [vp, abi.P32, C.POINTER(abi.KsNodeCols), C.c_int64]
    L.ks_load_quotas.argtypes = [vp, C.POINTER(abi.KsQuotaCols), C.c_int32]
    L.ks_load_reservations.argtypes = [vp, C.POINTER(abi.KsReservationCols), C.c_int32]
    L.ks_read_reservations.argtypes = [vp, abi.P64, abi.P32]
    L.ks_read_reservation_devices.argtypes = [vp, abi.P64]
    L.ks_load_devices.argtypes = [vp, C.POINTER(abi.KsDeviceCols), C.c_int64]
    L.ks_read_devices.argtypes = [vp, abi.P64, abi.P64, abi.P64]
    L.ks_read_devices_rdma.argtypes = [vp, abi.P64]
    L.ks_load_cpu_state.argtypes = [vp, C.POINTER(abi.KsCpuTopology), C.c_int32, C.POINTER(abi.KsCpuStateCols)]
    L.ks_read_cpu_state.argtypes = [vp, abi.PU64, abi.PU64, abi.PU64]
    L.ks_fetch_cpusets.argtypes = [vp, abi.PU64, C.c_int32]
    L.ks_load_numa_nodes.argtypes = [vp, C.POINTER(abi.KsNumaNodeCols)]
    L.ks_read_numa_nodes.argtypes = [vp, abi.P64, abi.P64]
    L.ks_refresh_quota_runtime.argtypes = [vp, C.POINTER(abi.KsQuotaTree), C.c_int32, abi.P64, abi.PU32]
    L.ks_schedule.argtypes = [vp, C.POINTER(abi.KsPodCols), C.c_int32, C.POINTER(abi.KsResult)]
    L.ks_stage_pods.argtypes = [vp, C.POINTER(abi.KsPodCols), C.c_int32]
    L.ks_schedule_staged.argtypes = [vp]
    L.ks_fetch_results.argtypes = [vp, C.POINTER(abi.KsResult), C.c_int32]
    L.ks_checkpoint.argtypes = [vp]
    L.ks_restore.argtypes = [vp]
    L.ks_eval_pod_debug.argtypes = [vp, C.POINTER(abi.KsPodCols), abi.PU32, abi.P64, abi.P64]
    L.ks_eval_pod.argtypes = [vp, C.POINTER(abi.KsPodCols), abi.PU32, abi.P64, abi.P64]
    L.ks_assume.argtypes = [vp, C.POINTER(abi.KsPodCols), C.c_int32, C.POINTER(abi.KsResult), abi.PU64, abi.P64]
    L.ks_unreserve.argtypes = [vp, C.POINTER(abi.KsPodCols), C.POINTER(abi.KsResult), abi.PU64, abi.P64]
    L.ks_fetch_numa_alloc.argtypes = [vp, abi.P64, C.c_int32]
    L.ks_update_devices.argtypes = [vp, abi.P32, C.POINTER(abi.KsDeviceCols), C.c_int64]
    L.ks_update_cpu_state.argtypes = [vp, abi.P32, C.POINTER(abi.KsCpuStateCols), C.c_int64]
    L.ks_update_quotas.argtypes = [vp, abi.P32, C.POINTER(abi.KsQuotaCols), C.c_int32]
    L.ks_update_reservation_usage.argtypes = [vp, abi.P32, C.POINTER(abi.P64), abi.P32, C.c_int32]
    L.ks_update_numa_nodes.argtypes = [vp, abi.P32, C.POINTER(abi.KsNumaNodeCols), C.c_int64]
    L.ks_add_reservations.argtypes = [vp, C.POINTER(abi.KsReservationCols), C.c_int32, abi.P32]
    L.ks_delete_reservations.argtypes = [vp, abi.P32, C.c_int32]
    L.ks_read_nodes.argtypes = [vp, C.POINTER(abi.KsNodeState)]
    L.ks_read_quota_used.argtypes = [vp, abi.P64]
    L.ks_get_stats.argtypes = [vp, C.POINTER(abi.KsStats)]
    L.ks_set_profile.argtypes = [vp, C.c_int32]
    L.ks_set_pipeline.argtypes = [vp, C.c_int32]
    L.ks_shard_unique_id.argtypes = [C.POINTER(C.c_uint8)]
    L.ks_shard_init.argtypes = [vp, C.c_int32, C.c_int32, C.POINTER(C.c_uint8), C.c_int32]
    L.ks_shard_init_loopback.argtypes = [C.POINTER(vp), C.c_int32, C.c_int32]
    L.ks_abi_layout.argtypes = [abi.P64, C.c_int32]
    L.ks_load_node_pods.argtypes = [vp, C.POINTER(abi.KsNodePodCols), C.c_int64, abi.P32, C.c_int32]
    L.ks_preempt.argtypes = [vp, C.POINTER(abi.KsPodCols), C.c_int32, C.c_uint32, C.c_int32, C.POINTER(C.c_uint8),
                             C.POINTER(abi.KsPreemptResult), abi.P32, C.c_int32, C.POINTER(C.c_uint8)]
    for name in abi.EXPORTED_SYMBOLS:
        if name not in ("ks_destroy", "ks_last_error"):
            getattr(L, name).restype = C.c_int
    check_layout(L)
    _lib = L
    return L


def expected_layout() -> list:
    """ks_abi_layout's words as this binding's ctypes mirrors of include/koordgpu.h lay them out"""
    return [abi.KS_ABI_VERSION, abi.KS_NUM_SCORE_PLUGINS] + [C.sizeof(t) for t in (
        abi.KsConfig, abi.KsNodeCols, abi.KsPodCols, abi.KsQuotaCols, abi.KsQuotaTree, abi.KsReservationCols,
        abi.KsDeviceCols, abi.KsCpuTopology, abi.KsCpuStateCols, abi.KsNumaNodeCols, abi.KsResult, abi.KsNodeState,
        abi.KsStats, abi.KsNodePodCols, abi.KsPreemptResult)]


def check_layout(L) -> None:
    """Refuse a library compiled from another header than this binding mirrors (a stale libkoordgpu.so would write
    score rows or results past the buffers this module allocates)."""
    want = expected_layout()
    got = (C.c_int64 * len(want))()
    n = L.ks_abi_layout(got, len(want))
    if n != len(want) or list(got) != want:
        raise ImportError(f"{LIB_PATH} was built from another include/koordgpu.h (library layout {list(got)[:n]}, "
                          f"binding {want}); rebuild it with koordinator_amd.runtime.build()")


def shard_unique_id() -> bytes:
    """RCCL unique id for ks_shard_init (call on rank 0, broadcast the bytes to the other ranks)."""
    L = lib()
    buf = (C.c_uint8 * abi.KS_SHARD_ID_BYTES)()
    rc = L.ks_shard_unique_id(buf)
    if rc != abi.KS_OK:
        raise KsError(rc, "ncclGetUniqueId failed")
    return bytes(buf)


def shard_loopback(evaluators, virtual_shards: int = 1):
    """Test transport (ks_shard_init_loopback): the evaluators (same node table, batch and candidates) become ranks
    0..n-1 of one node-sharded group whose candidate exchange is device copies between them instead of RCCL.  Each
    rank's schedule* must then run concurrently on its own thread (run_ranks)."""
    L = lib()
    hs = (C.c_void_p * len(evaluators))(*[ev.h.value for ev in evaluators])
    rc = L.ks_shard_init_loopback(hs, len(evaluators), virtual_shards)
    if rc != abi.KS_OK:
        msgs = [L.ks_last_error(ev.h).decode() for ev in evaluators]
        raise KsError(rc, "ks_shard_init_loopback: " + "; ".join(m for m in msgs if m))


def run_ranks(fn, evaluators):
    """fn(evaluator) on every rank concurrently, one host thread each (ctypes releases the GIL inside the library);
    returns the per-rank results and re-raises the first rank's exception."""
    import threading

    out = [None] * len(evaluators)
    err = [None] * len(evaluators)

    def body(i):
        try:
            out[i] = fn(evaluators[i])
        except BaseException as e:  # noqa: BLE001 - re-raised below
            err[i] = e

    ts = [threading.Thread(target=body, args=(i,)) for i in range(len(evaluators))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for e in err:
        if e is not None:
            raise e
    return out


class Evaluator:
    """One scheduler profile's device-resident node snapshot + the sweep/commit pipeline."""

    def __init__(self, cfg: abi.KsConfig, nodes: Optional[NodeTable] = None, quotas: Optional[QuotaTable] = None,
                 reservations: Optional[ReservationTable] = None, devices: Optional[DeviceTable] = None,
                 cpu_state: Optional[CpuState] = None, numa_nodes: Optional[NumaNodes] = None):
        self.L = lib()
        self.cfg = cfg
        h = C.c_void_p()
        rc = self.L.ks_create(C.byref(cfg), C.byref(h))
        if rc != abi.KS_OK:
            raise KsError(rc, self.L.ks_last_error(None).decode())
        self.h = h
        self.n = 0
        self.nq = 0
        self.nr = 0
        self.np_staged = 0
        if nodes is not None:
            self.load_nodes(nodes)
        if quotas is not None:
            self.load_quotas(quotas)
        if reservations is not None:
            self.load_reservations(reservations)
        if devices is not None:
            self.load_devices(devices)
        if cpu_state is not None:
            self.load_cpu_state(cpu_state)
        if numa_nodes is not None:
            self.load_numa_nodes(numa_nodes)

    def _chk(self, rc: int):
        if rc != abi.KS_OK:
            raise KsError(rc, self.L.ks_last_error(self.h).decode())

    def close(self):
        if getattr(self, "h", None):
            self.L.ks_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def load_nodes(self, nodes: NodeTable):
        cols = nodes.ks()
        self._chk(self.L.ks_load_nodes(self.h, C.byref(cols), nodes.n))
        self.n = nodes.n
        self.nprops = int(np.asarray(nodes.topo_count).shape[0])

    def update_nodes(self, idx, rows: NodeTable):
        idx = np.ascontiguousarray(idx, np.int32)
        cols = rows.ks()
        self._chk(self.L.ks_update_nodes(self.h, idx.ctypes.data_as(abi.P32), C.byref(cols), rows.n))

    def load_quotas(self, quotas: QuotaTable):
        cols = quotas.ks()
        self._chk(self.L.ks_load_quotas(self.h, C.byref(cols), quotas.q))
        self.nq = quotas.q

    def load_reservations(self, rs: ReservationTable):
        cols = rs.ks()
        self._chk(self.L.ks_load_reservations(self.h, C.byref(cols), rs.r))
        self.nr = rs.r

    def add_reservations(self, rs: ReservationTable) -> int:
        """informer add: rs's rows become caller rows first .. first + rs.r - 1; returns first"""
        cols = rs.ks()
        first = np.zeros(1, np.int32)
        self._chk(self.L.ks_add_reservations(self.h, C.byref(cols), rs.r, first.ctypes.data_as(abi.P32)))
        self.nr = int(first[0]) + rs.r
        return int(first[0])

    def update_numa_nodes(self, idx, rows):
        """informer delta: node idx[i]'s NUMA-node table from row i of rows (a NumaNodeTable of len(idx) nodes)"""
        idx = np.ascontiguousarray(idx, np.int32)
        cols = rows.ks()
        self._chk(self.L.ks_update_numa_nodes(self.h, idx.ctypes.data_as(abi.P32), C.byref(cols), idx.size))

    def delete_reservations(self, rows):
        """informer delete of caller rows (their numbers are not reused)"""
        rows = np.ascontiguousarray(rows, np.int32)
        self._chk(self.L.ks_delete_reservations(self.h, rows.ctypes.data_as(abi.P32), rows.size))

    def load_devices(self, dev: DeviceTable):
        cols = dev.ks()
        self._chk(self.L.ks_load_devices(self.h, C.byref(cols), dev.n))

    def load_cpu_state(self, st: CpuState):
        """CPU topologies + per-node allocation for cpuset (KS_POD_CPU_BIND) pods."""
        cols = st.ks()
        topos = st.topo_array()
        self._chk(self.L.ks_load_cpu_state(self.h, topos, len(st.topologies), C.byref(cols)))

    def load_numa_nodes(self, nn: NumaNodes):
        """NUMA node resources of the nodes with a NUMA topology policy."""
        cols = nn.ks()
        self._chk(self.L.ks_load_numa_nodes(self.h, C.byref(cols)))

    def read_numa_nodes(self):
        """(used_cpu, used_memory), each [n][KS_MAX_NUMA]"""
        K = abi.KS_MAX_NUMA
        out = [np.zeros((max(self.n, 1), K), np.int64) for _ in range(2)]
        self._chk(self.L.ks_read_numa_nodes(self.h, *[o.ctypes.data_as(abi.P64) for o in out]))
        return tuple(o[: self.n] for o in out)

    def read_cpu_state(self):
        """(allocated, excl_pcpu, excl_numa), each [n][KS_CPU_WORDS] uint64"""
        W = abi.KS_CPU_WORDS
        out = [np.zeros((max(self.n, 1), W), np.uint64) for _ in range(3)]
        self._chk(self.L.ks_read_cpu_state(self.h, *[o.ctypes.data_as(abi.PU64) for o in out]))
        return tuple(o[: self.n] for o in out)

    def fetch_cpusets(self, p: int) -> np.ndarray:
        """[p][KS_CPU_WORDS] uint64: the CPUs each pod of the last schedule call was allocated."""
        out = np.zeros((max(p, 1), abi.KS_CPU_WORDS), np.uint64)
        self._chk(self.L.ks_fetch_cpusets(self.h, out.ctypes.data_as(abi.PU64), p))
        return out[:p]

    def read_devices(self):
        """(used_core, used_memory, used_ratio) [KS_MAX_GPUS][n], used_rdma [KS_MAX_RDMA][n]"""
        G = abi.KS_MAX_GPUS
        out = [np.zeros(G * max(self.n, 1), np.int64) for _ in range(3)]
        self._chk(self.L.ks_read_devices(self.h, *[o.ctypes.data_as(abi.P64) for o in out]))
        R = abi.KS_MAX_RDMA
        r = np.zeros(R * max(self.n, 1), np.int64)
        self._chk(self.L.ks_read_devices_rdma(self.h, r.ctypes.data_as(abi.P64)))
        return tuple(o[: G * self.n].reshape(G, self.n) for o in out) + (r[: R * self.n].reshape(R, self.n),)

    def read_reservations(self):
        """(allocated [r][KS_RSV_DIMS], assigned [r]) after commits"""
        allocated = np.zeros(max(self.nr, 1) * abi.KS_RSV_DIMS, np.int64)
        assigned = np.zeros(max(self.nr, 1), np.int32)
        self._chk(self.L.ks_read_reservations(self.h, allocated.ctypes.data_as(abi.P64),
                                              assigned.ctypes.data_as(abi.P32)))
        return allocated[: self.nr * abi.KS_RSV_DIMS].reshape(self.nr, abi.KS_RSV_DIMS), assigned[: self.nr]

    def read_reservation_devices(self):
        """the assigned pods' device allocations on each reservation's minors [r][KS_DEV_WORDS] after commits"""
        out = np.zeros(max(self.nr, 1) * abi.KS_DEV_WORDS, np.int64)
        self._chk(self.L.ks_read_reservation_devices(self.h, out.ctypes.data_as(abi.P64)))
        return out[: self.nr * abi.KS_DEV_WORDS].reshape(self.nr, abi.KS_DEV_WORDS)

    def shard(self, nranks: int = 1, rank: int = 0, unique_id: Optional[bytes] = None, virtual_shards: int = 1):
        """Node sharding: this rank sweeps its chunk range; candidates are exchanged by RCCL allgather."""
        uid = None
        if unique_id is not None:
            uid = (C.c_uint8 * abi.KS_SHARD_ID_BYTES).from_buffer_copy(unique_id)
        self._chk(self.L.ks_shard_init(self.h, nranks, rank, uid, virtual_shards))

    def refresh_quota_runtime(self, tree: QuotaTree):
        """RefreshRuntime for every quota (on the device); installs it as the admission limit of the
        loaded quota table when the row counts agree.  Returns (runtime [dim][quota], mask)."""
        rt = np.zeros((max(tree.q, 1), abi.KS_QUOTA_DIMS), np.int64)
        mask = np.zeros(max(tree.q, 1), np.uint32)
        cols = tree.ks()
        self._chk(self.L.ks_refresh_quota_runtime(self.h, C.byref(cols), tree.q, rt.ctypes.data_as(abi.P64),
                                                  mask.ctypes.data_as(abi.PU32)))
        return rt[: tree.q].T.copy(), mask[: tree.q]

    def schedule(self, pods: PodTable) -> dict:
        out = np.zeros(max(pods.n, 1), RESULT_DTYPE)
        cols = pods.ks()
        self._chk(self.L.ks_schedule(self.h, C.byref(cols), pods.n, out.ctypes.data_as(C.POINTER(abi.KsResult))))
        out = out[: pods.n]
        return {"node": out["node"].copy(), "status": out["status"].copy(), "score": out["score"].copy(),
                "reservation": out["reservation"].copy(), "gpu_minors": out["gpu_minors"].copy(),
                "rdma_minors": out["rdma_minors"].copy()}

    def stage(self, pods: PodTable):
        cols = pods.ks()
        self._chk(self.L.ks_stage_pods(self.h, C.byref(cols), pods.n))
        self.np_staged = pods.n

    def schedule_staged(self):
        self._chk(self.L.ks_schedule_staged(self.h))

    def fetch(self) -> dict:
        out = np.zeros(max(self.np_staged, 1), RESULT_DTYPE)
        self._chk(self.L.ks_fetch_results(self.h, out.ctypes.data_as(C.POINTER(abi.KsResult)), self.np_staged))
        out = out[: self.np_staged]
        return {"node": out["node"].copy(), "status": out["status"].copy(), "score": out["score"].copy(),
                "reservation": out["reservation"].copy(), "gpu_minors": out["gpu_minors"].copy(),
                "rdma_minors": out["rdma_minors"].copy()}

    def checkpoint(self):
        self._chk(self.L.ks_checkpoint(self.h))

    def restore(self):
        self._chk(self.L.ks_restore(self.h))

    def eval_pod(self, pod: PodTable):
        reasons = np.zeros(max(self.n, 1), np.uint32)
        scores = np.zeros(max(self.n, 1) * abi.KS_NUM_SCORE_PLUGINS, np.int64)
        total = np.zeros(max(self.n, 1), np.int64)
        cols = pod.ks()
        self._chk(self.L.ks_eval_pod(self.h, C.byref(cols), reasons.ctypes.data_as(abi.PU32),
                                     scores.ctypes.data_as(abi.P64), total.ctypes.data_as(abi.P64)))
        n = self.n
        return reasons[:n], scores[: n * abi.KS_NUM_SCORE_PLUGINS].reshape(n, abi.KS_NUM_SCORE_PLUGINS), total[:n]

    def assume(self, pod: PodTable, node: int):
        """Reserve of pod 0 on `node` (the framework's choice): (result record, cpuset words, NUMA allocation
        [KS_MAX_NUMA][2])."""
        r = np.zeros(1, RESULT_DTYPE)
        cs = np.zeros(abi.KS_CPU_WORDS, np.uint64)
        na = np.zeros((abi.KS_MAX_NUMA, 2), np.int64)
        cols = pod.ks()
        self._chk(self.L.ks_assume(self.h, C.byref(cols), int(node), r.ctypes.data_as(C.POINTER(abi.KsResult)),
                                   cs.ctypes.data_as(abi.PU64), na.ctypes.data_as(abi.P64)))
        return r, cs, na

    def unreserve(self, pod: PodTable, r, cpuset=None, numa_alloc=None):
        """Unreserve of pod 0 placed as the result record r says (a 1-element RESULT_DTYPE array)."""
        r = np.ascontiguousarray(r, RESULT_DTYPE).reshape(1)
        cols = pod.ks()
        cs = None if cpuset is None else np.ascontiguousarray(cpuset, np.uint64)
        na = None if numa_alloc is None else np.ascontiguousarray(numa_alloc, np.int64)
        self._chk(self.L.ks_unreserve(self.h, C.byref(cols), r.ctypes.data_as(C.POINTER(abi.KsResult)),
                                      cs.ctypes.data_as(abi.PU64) if cs is not None else None,
                                      na.ctypes.data_as(abi.P64) if na is not None else None))

    def update_devices(self, idx, rows: DeviceTable):
        """informer delta: node idx[i]'s devices from row i of rows"""
        idx = np.ascontiguousarray(idx, np.int32)
        cols = rows.ks()
        self._chk(self.L.ks_update_devices(self.h, idx.ctypes.data_as(abi.P32), C.byref(cols), rows.n))

    def update_cpu_state(self, idx, rows: CpuState):
        """informer delta: node idx[i]'s CPU state from row i (topology indices into the loaded table)"""
        idx = np.ascontiguousarray(idx, np.int32)
        cols = rows.ks()
        self._chk(self.L.ks_update_cpu_state(self.h, idx.ctypes.data_as(abi.P32), C.byref(cols), rows.n))

    def update_quotas(self, idx, rows: QuotaTable):
        """informer delta: quota idx[i]'s limits / usage from row i"""
        idx = np.ascontiguousarray(idx, np.int32)
        cols = rows.ks()
        self._chk(self.L.ks_update_quotas(self.h, idx.ctypes.data_as(abi.P32), C.byref(cols), rows.q))

    def update_reservation_usage(self, rows, allocated, assigned):
        """informer delta: allocated [KS_RSV_DIMS][m] and assigned [m] of reservation rows `rows`"""
        rows = np.ascontiguousarray(rows, np.int32)
        allocated = np.ascontiguousarray(allocated, np.int64)
        assigned = np.ascontiguousarray(assigned, np.int32)
        ptrs = (abi.P64 * abi.KS_RSV_DIMS)(*[allocated[d].ctypes.data_as(abi.P64) for d in range(abi.KS_RSV_DIMS)])
        self._chk(self.L.ks_update_reservation_usage(self.h, rows.ctypes.data_as(abi.P32), ptrs,
                                                     assigned.ctypes.data_as(abi.P32), len(rows)))

    def fetch_numa_alloc(self, p: int) -> np.ndarray:
        out = np.zeros((max(p, 1), abi.KS_MAX_NUMA, 2), np.int64)
        self._chk(self.L.ks_fetch_numa_alloc(self.h, out.ctypes.data_as(abi.P64), p))
        return out[:p]

    def schedule_raw(self, pods: PodTable) -> np.ndarray:
        """ks_schedule's result records (RESULT_DTYPE), for ks_unreserve"""
        out = np.zeros(max(pods.n, 1), RESULT_DTYPE)
        cols = pods.ks()
        self._chk(self.L.ks_schedule(self.h, C.byref(cols), pods.n, out.ctypes.data_as(C.POINTER(abi.KsResult))))
        return out[: pods.n]

    def load_node_pods(self, t: NodePodTable):
        """NodeInfo.Pods of every node + the PDBs' DisruptionsAllowed, the victims pool of preempt()"""
        cols = t.ks()
        self._chk(self.L.ks_load_node_pods(self.h, C.byref(cols), t.m, t.pdb_allowed.ctypes.data_as(abi.P32),
                                           len(t.pdb_allowed)))
        self.npods = t.m

    def preempt(self, pod: PodTable, priority: int, flags: int = 0, nominated_node: int = -1, unresolvable=None,
                node_status: bool = False) -> dict:
        """ElasticQuota PostFilter of pod 0 (ks_preempt): {status, node, victims (node-pod table rows, Victims.Pods
        order), num_pdb_violations, candidates, potential_nodes[, node_status]}"""
        out = abi.KsPreemptResult()
        cap = max(getattr(self, "npods", 0), 1)
        vic = np.zeros(cap, np.int32)
        ns = np.zeros(max(self.n, 1), np.uint8) if node_status else None
        ur = None if unresolvable is None else np.ascontiguousarray(unresolvable, np.uint8)
        cols = pod if isinstance(pod, abi.KsPodCols) else pod.ks()  # (a prebuilt pointer struct: no per-call rebuild)
        self._chk(self.L.ks_preempt(self.h, C.byref(cols), int(priority), int(flags), int(nominated_node),
                                    ur.ctypes.data_as(C.POINTER(C.c_uint8)) if ur is not None else None, C.byref(out),
                                    vic.ctypes.data_as(abi.P32), cap,
                                    ns.ctypes.data_as(C.POINTER(C.c_uint8)) if ns is not None else None))
        r = {"status": out.status, "node": out.node, "victims": vic[: out.num_victims].copy(),
             "num_pdb_violations": out.num_pdb_violations, "candidates": out.candidates,
             "potential_nodes": out.potential_nodes}
        if ns is not None:
            r["node_status"] = ns[: self.n].copy()
        return r

    def read_nodes(self) -> NodeState:
        st = NodeState(self.n, getattr(self, 'nprops', 0))
        s = st.ks()
        self._chk(self.L.ks_read_nodes(self.h, C.byref(s)))
        return st

    def read_quota_used(self) -> np.ndarray:
        used = np.zeros(max(self.nq, 1) * abi.KS_QUOTA_DIMS, np.int64)
        self._chk(self.L.ks_read_quota_used(self.h, used.ctypes.data_as(abi.P64)))
        return used[: self.nq * abi.KS_QUOTA_DIMS].reshape(self.nq, abi.KS_QUOTA_DIMS)

    def set_profile(self, on: bool):
        self._chk(self.L.ks_set_profile(self.h, 1 if on else 0))

    def set_pipeline(self, mode: int):
        """0 off, 1 automatic (large clusters), 2 always: overlap each pass's sweep with the previous commit
        (results are identical either way)."""
        self._chk(self.L.ks_set_pipeline(self.h, int(mode)))

    def stats(self) -> dict:
        s = abi.KsStats()
        self._chk(self.L.ks_get_stats(self.h, C.byref(s)))
        out = {k: getattr(s, k) for k, _ in abi.KsStats._fields_}
        out["diag"] = list(s.diag)
        return out
