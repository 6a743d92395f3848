"""Structure-of-arrays tables for the C ABI (host side).

``NodeTable`` / ``PodTable`` / ``QuotaTable`` own numpy columns laid out exactly
as ``ks_node_cols`` / ``ks_pod_cols`` / ``ks_quota_cols`` expect and build the
ctypes pointer structs on demand.  This is the Python stand-in for what the Go
cgo shim does at informer time: NodeInfo fields come from the
scheduler cache snapshot, the ``la_*`` block from the LoadAware reduction in
:mod:`.ingest`.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, Optional

import numpy as np

from . import abi

NODE_I64 = [
    "alloc_milli_cpu", "alloc_memory", "alloc_ephemeral",
    "req_milli_cpu", "req_memory", "req_ephemeral",
    "nonzero_milli_cpu", "nonzero_memory",
    "la_alloc_milli_cpu", "la_alloc_memory",
    "la_term_milli_cpu", "la_term_memory", "la_prod_term_milli_cpu", "la_prod_term_memory",
    "la_total_milli_cpu", "la_total_milli_memory",
    "la_usage_milli_cpu", "la_usage_milli_memory",
    "la_prod_usage_milli_cpu", "la_prod_usage_milli_memory",
]
NODE_I32 = ["allowed_pods", "pod_count", "la_thr_cpu", "la_thr_memory", "la_prod_thr_cpu", "la_prod_thr_memory",
            "numa_cpuset_cpus"]
NODE_U32 = ["la_flags", "numa_flags"]
# TaintToleration / NodeAffinity dictionary bits (static_plugins.compile_cluster)
NODE_U64 = ["taints_hard", "taints_soft", "labels", "host_ports"]

POD_I64 = [
    "req_milli_cpu", "req_memory", "req_ephemeral",
    "nonzero_milli_cpu", "nonzero_memory",
    "la_req_cpu", "la_lim_cpu", "la_dflt_cpu", "la_req_memory", "la_lim_memory", "la_dflt_memory",
    "gpu_core", "gpu_memory", "gpu_memory_ratio", "rdma",
]
POD_I32 = ["quota", "rsv_class", "affinity_required_n"]
POD_U32 = ["flags", "quota_mask", "cpu_bind"]
POD_U8 = ["joint"]
POD_U64 = ["tolerated", "host_ports", "host_ports_conflict"]

STATE_I64 = [
    "req_milli_cpu", "req_memory", "req_ephemeral", "nonzero_milli_cpu", "nonzero_memory",
    "la_term_milli_cpu", "la_term_memory", "la_prod_term_milli_cpu", "la_prod_term_memory",
]

MAX_QUANTITY = 1 << 56  # ks ABI supported range


def _p64(a: np.ndarray):
    return a.ctypes.data_as(abi.P64)


def _p32(a: np.ndarray):
    return a.ctypes.data_as(abi.P32)


def _pu32(a: np.ndarray):
    return a.ctypes.data_as(abi.PU32)


class _Table:
    I64: list = []
    I32: list = []
    U32: list = []
    U8: list = []
    U64: list = []
    N_SCALAR_ARRAYS: tuple = ()

    def __init__(self, n: int):
        self.n = int(n)
        for name in self.I64:
            setattr(self, name, np.zeros(self.n, np.int64))
        for name in self.I32:
            setattr(self, name, np.zeros(self.n, np.int32))
        for name in self.U32:
            setattr(self, name, np.zeros(self.n, np.uint32))
        for name in self.U8:
            setattr(self, name, np.zeros(self.n, np.uint8))
        for name in self.U64:
            setattr(self, name, np.zeros(self.n, np.uint64))

    def columns(self) -> Dict[str, np.ndarray]:
        return {k: getattr(self, k) for k in self.I64 + self.I32 + self.U32 + self.U8 + self.U64}

    def _fix(self):
        for name in self.I64:
            a = getattr(self, name)
            if a.dtype != np.int64 or not a.flags.c_contiguous:
                setattr(self, name, np.ascontiguousarray(a, np.int64))
        for name in self.I32:
            a = getattr(self, name)
            if a.dtype != np.int32 or not a.flags.c_contiguous:
                setattr(self, name, np.ascontiguousarray(a, np.int32))
        for name in self.U32:
            a = getattr(self, name)
            if a.dtype != np.uint32 or not a.flags.c_contiguous:
                setattr(self, name, np.ascontiguousarray(a, np.uint32))
        for name in self.U8:
            a = getattr(self, name)
            if a.dtype != np.uint8 or not a.flags.c_contiguous:
                setattr(self, name, np.ascontiguousarray(a, np.uint8))
        for name in self.U64:
            a = getattr(self, name)
            if a.dtype != np.uint64 or not a.flags.c_contiguous:
                setattr(self, name, np.ascontiguousarray(a, np.uint64))


class NodeTable(_Table):
    I64 = NODE_I64
    I32 = NODE_I32
    U32 = NODE_U32
    U64 = NODE_U64

    def __init__(self, n: int):
        super().__init__(n)
        self.alloc_scalar = np.zeros((abi.KS_MAX_SCALARS, self.n), np.int64)
        self.req_scalar = np.zeros((abi.KS_MAX_SCALARS, self.n), np.int64)
        self.numa_cpu_amplification = np.zeros(self.n, np.float64)  # <= 1: not amplified
        # PodTopologySpread / InterPodAffinity (topology_plugins.compile_topology): per key (besides the hostname) the
        # node's value index (-1 = absent), per property the node's pods having it; values of every key < topo_ndomains
        self.topo_domain = np.full((0, self.n), -1, np.int32)
        self.topo_count = np.zeros((0, self.n), np.int32)
        self.topo_ndomains = 1

    def copy(self) -> "NodeTable":
        t = NodeTable(self.n)
        for k, v in self.columns().items():
            setattr(t, k, v.copy())
        t.alloc_scalar = self.alloc_scalar.copy()
        t.req_scalar = self.req_scalar.copy()
        t.numa_cpu_amplification = self.numa_cpu_amplification.copy()
        t.topo_domain = self.topo_domain.copy()
        t.topo_count = self.topo_count.copy()
        t.topo_ndomains = self.topo_ndomains
        return t

    def rows(self, idx) -> "NodeTable":
        idx = np.asarray(idx)
        t = NodeTable(len(idx))
        for k, v in self.columns().items():
            setattr(t, k, np.ascontiguousarray(v[idx]))
        t.alloc_scalar = np.ascontiguousarray(self.alloc_scalar[:, idx])
        t.req_scalar = np.ascontiguousarray(self.req_scalar[:, idx])
        t.numa_cpu_amplification = np.ascontiguousarray(self.numa_cpu_amplification[idx])
        t.topo_domain = np.ascontiguousarray(self.topo_domain[:, idx])
        t.topo_count = np.ascontiguousarray(self.topo_count[:, idx])
        t.topo_ndomains = self.topo_ndomains
        return t

    def check_range(self) -> None:
        for name in NODE_I64:
            a = getattr(self, name)
            if a.size and (a.min() < 0 or a.max() >= MAX_QUANTITY):
                raise ValueError(f"{name} outside [0, 2^56)")

    def ks(self) -> abi.KsNodeCols:
        self._fix()
        self.alloc_scalar = np.ascontiguousarray(self.alloc_scalar, np.int64)
        self.req_scalar = np.ascontiguousarray(self.req_scalar, np.int64)
        c = abi.KsNodeCols()
        for name in NODE_I64:
            setattr(c, name, _p64(getattr(self, name)))
        for name in NODE_I32:
            setattr(c, name, _p32(getattr(self, name)))
        c.la_flags = _pu32(self.la_flags)
        c.numa_flags = _pu32(self.numa_flags)
        for name in NODE_U64:
            setattr(c, name, getattr(self, name).ctypes.data_as(C.POINTER(C.c_uint64)))
        self.numa_cpu_amplification = np.ascontiguousarray(self.numa_cpu_amplification, np.float64)
        c.numa_cpu_amplification = self.numa_cpu_amplification.ctypes.data_as(C.POINTER(C.c_double))
        for k in range(abi.KS_MAX_SCALARS):
            c.alloc_scalar[k] = _p64(self.alloc_scalar[k])
            c.req_scalar[k] = _p64(self.req_scalar[k])
        self.topo_domain = _rows2d(self.topo_domain, self.n)
        self.topo_count = _rows2d(self.topo_count, self.n)
        c.topo_nkeys = self.topo_domain.shape[0]
        c.topo_ndomains = int(self.topo_ndomains)
        c.topo_nprops = self.topo_count.shape[0]
        c.topo_domain = _p32(self.topo_domain) if self.topo_domain.size else None
        c.topo_count = _p32(self.topo_count) if self.topo_count.size else None
        c._keep = self  # keep arrays alive with the struct
        return c


def _rows2d(a, n: int) -> np.ndarray:
    """[rows][n] int32, C-contiguous (a per-key / per-property block of node columns)"""
    a = np.ascontiguousarray(a, np.int32)
    if a.ndim != 2:
        a = a.reshape(-1, n) if n else np.zeros((0, 0), np.int32)
    return a


def _csr_rows(beg: np.ndarray, vals: np.ndarray, idx: np.ndarray):
    """rows idx of a CSR list: (new beg, new values)"""
    idx = np.asarray(idx, np.int64)
    beg = np.asarray(beg, np.int64)
    cnt = beg[idx + 1] - beg[idx]
    nb = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int64)
    if nb[-1] == 0:
        return nb.astype(np.int32), vals[:0].copy()
    pos = np.repeat(beg[idx] - nb[:-1], cnt) + np.arange(nb[-1])
    return nb.astype(np.int32), np.ascontiguousarray(vals[pos])


class PodTable(_Table):
    I64 = POD_I64
    I32 = POD_I32
    U32 = POD_U32
    U8 = POD_U8
    U64 = POD_U64

    def __init__(self, n: int):
        super().__init__(n)
        self.quota[:] = -1
        self.rsv_class[:] = -1
        self.req_scalar = np.zeros((abi.KS_MAX_SCALARS, self.n), np.int64)
        self.quota_req = np.zeros((abi.KS_QUOTA_DIMS, self.n), np.int64)
        # NodeAffinity terms over the label dictionary (static_plugins.compile_cluster)
        self.affinity_required = np.zeros((abi.KS_AFFINITY_TERMS, self.n), np.uint64)
        self.affinity_preferred = np.zeros((abi.KS_AFFINITY_TERMS, self.n), np.uint64)
        self.affinity_weight = np.zeros((abi.KS_AFFINITY_TERMS, self.n), np.int32)
        # PodTopologySpread / InterPodAffinity (topology_plugins.compile_topology): flags, and the CSR lists of the
        # pods' properties and query terms (pod i: [beg[i], beg[i + 1]))
        self.topo_flags = np.zeros(self.n, np.uint32)
        self.topo_prop_beg = np.zeros(self.n + 1, np.int32)
        self.topo_props = np.zeros(0, np.int32)
        self.topo_term_beg = np.zeros(self.n + 1, np.int32)
        self.topo_terms = np.zeros(0, np.uint64)

    def set_topo(self, props, terms) -> None:
        """The CSR lists from one list per pod (property indices; packed query terms)."""
        assert len(props) == self.n and len(terms) == self.n
        self.topo_prop_beg = np.concatenate([[0], np.cumsum([len(x) for x in props])]).astype(np.int32)
        self.topo_props = np.array([v for x in props for v in x], np.int32)
        self.topo_term_beg = np.concatenate([[0], np.cumsum([len(x) for x in terms])]).astype(np.int32)
        self.topo_terms = np.array([v for x in terms for v in x], np.uint64)

    def topo_lists(self, i: int):
        """pod i's (properties, query terms)"""
        return (self.topo_props[self.topo_prop_beg[i]:self.topo_prop_beg[i + 1]].tolist(),
                self.topo_terms[self.topo_term_beg[i]:self.topo_term_beg[i + 1]].tolist())

    def rows(self, idx) -> "PodTable":
        idx = np.asarray(idx)
        t = PodTable(len(idx))
        for k, v in self.columns().items():
            setattr(t, k, np.ascontiguousarray(v[idx]))
        t.req_scalar = np.ascontiguousarray(self.req_scalar[:, idx])
        t.quota_req = np.ascontiguousarray(self.quota_req[:, idx])
        for k in ("affinity_required", "affinity_preferred", "affinity_weight"):
            setattr(t, k, np.ascontiguousarray(getattr(self, k)[:, idx]))
        t.topo_flags = np.ascontiguousarray(self.topo_flags[idx])
        t.topo_prop_beg, t.topo_props = _csr_rows(self.topo_prop_beg, self.topo_props, idx)
        t.topo_term_beg, t.topo_terms = _csr_rows(self.topo_term_beg, self.topo_terms, idx)
        return t

    def ks(self) -> abi.KsPodCols:  # noqa: C901
        self._fix()
        self.req_scalar = np.ascontiguousarray(self.req_scalar, np.int64)
        self.quota_req = np.ascontiguousarray(self.quota_req, np.int64)
        c = abi.KsPodCols()
        for name in POD_I64:
            setattr(c, name, _p64(getattr(self, name)))
        c.quota = _p32(self.quota)
        c.rsv_class = _p32(self.rsv_class)
        c.flags = _pu32(self.flags)
        c.quota_mask = _pu32(self.quota_mask)
        c.cpu_bind = _pu32(self.cpu_bind)
        c.joint = self.joint.ctypes.data_as(C.POINTER(C.c_uint8))
        for k in range(abi.KS_MAX_SCALARS):
            c.req_scalar[k] = _p64(self.req_scalar[k])
        for d in range(abi.KS_QUOTA_DIMS):
            c.quota_req[d] = _p64(self.quota_req[d])
        for name in POD_U64:
            setattr(c, name, getattr(self, name).ctypes.data_as(C.POINTER(C.c_uint64)))
        c.affinity_required_n = _p32(self.affinity_required_n)
        self.affinity_required = np.ascontiguousarray(self.affinity_required, np.uint64)
        self.affinity_preferred = np.ascontiguousarray(self.affinity_preferred, np.uint64)
        self.affinity_weight = np.ascontiguousarray(self.affinity_weight, np.int32)
        for t in range(abi.KS_AFFINITY_TERMS):
            c.affinity_required[t] = self.affinity_required[t].ctypes.data_as(C.POINTER(C.c_uint64))
            c.affinity_preferred[t] = self.affinity_preferred[t].ctypes.data_as(C.POINTER(C.c_uint64))
            c.affinity_weight[t] = _p32(self.affinity_weight[t])
        self.topo_flags = np.ascontiguousarray(self.topo_flags, np.uint32)
        self.topo_prop_beg = np.ascontiguousarray(self.topo_prop_beg, np.int32)
        self.topo_term_beg = np.ascontiguousarray(self.topo_term_beg, np.int32)
        # (never a NULL list pointer: an empty list is one unused word)
        self._props_buf = np.ascontiguousarray(self.topo_props if len(self.topo_props) else np.zeros(1), np.int32)
        self._terms_buf = np.ascontiguousarray(self.topo_terms if len(self.topo_terms) else np.zeros(1), np.uint64)
        c.topo_flags = _pu32(self.topo_flags)
        c.topo_prop_beg = _p32(self.topo_prop_beg)
        c.topo_props = _p32(self._props_buf)
        c.topo_term_beg = _p32(self.topo_term_beg)
        c.topo_terms = self._terms_buf.ctypes.data_as(C.POINTER(C.c_uint64))
        c._keep = self
        return c


class QuotaTable:
    def __init__(self, q: int):
        self.q = int(q)
        self.parent = np.full(self.q, -1, np.int32)
        self.limit_mask = np.zeros(self.q, np.uint32)
        self.min_mask = np.zeros(self.q, np.uint32)
        self.limit = np.zeros((abi.KS_QUOTA_DIMS, self.q), np.int64)
        self.used = np.zeros((abi.KS_QUOTA_DIMS, self.q), np.int64)
        self.min = np.zeros((abi.KS_QUOTA_DIMS, self.q), np.int64)
        self.nonpreemptible_used = np.zeros((abi.KS_QUOTA_DIMS, self.q), np.int64)

    def copy(self) -> "QuotaTable":
        t = QuotaTable(self.q)
        for k in ("parent", "limit_mask", "min_mask", "limit", "used", "min", "nonpreemptible_used"):
            setattr(t, k, getattr(self, k).copy())
        return t

    def ks(self) -> abi.KsQuotaCols:
        c = abi.KsQuotaCols()
        self.parent = np.ascontiguousarray(self.parent, np.int32)
        c.parent = _p32(self.parent)
        c.limit_mask = _pu32(self.limit_mask)
        c.min_mask = _pu32(self.min_mask)
        for name in ("limit", "used", "min", "nonpreemptible_used"):
            arr = np.ascontiguousarray(getattr(self, name), np.int64)
            setattr(self, name, arr)
            field = getattr(c, name)
            for d in range(abi.KS_QUOTA_DIMS):
                field[d] = _p64(arr[d])
        c._keep = self
        return c


class QuotaTree:
    """ElasticQuota tree for ks_refresh_quota_runtime (one row per quota; values [dim][quota]).

    Mirrors the QuotaInfo fields RefreshRuntime reads (pkg/scheduler/plugins/elasticquota/core/
    quota_info.go CalculateInfo: Max, Min/AutoScaleMin, SharedWeight, Guaranteed, the quota's own
    pods' Request) plus AllowLentResource and the tree's total resource."""

    def __init__(self, q: int):
        self.q = int(q)
        self.parent = np.full(self.q, -1, np.int32)
        self.allow_lent = np.ones(self.q, np.uint8)
        self.max_mask = np.zeros(self.q, np.uint32)
        D = abi.KS_QUOTA_DIMS
        self.max = np.zeros((D, self.q), np.int64)
        self.min = np.zeros((D, self.q), np.int64)
        self.shared_weight: Optional[np.ndarray] = None  # None = Max
        self.guaranteed = np.zeros((D, self.q), np.int64)
        self.self_request = np.zeros((D, self.q), np.int64)
        self.cluster_total = np.zeros(D, np.int64)

    def ks(self) -> abi.KsQuotaTree:
        c = abi.KsQuotaTree()
        self.parent = np.ascontiguousarray(self.parent, np.int32)
        self.allow_lent = np.ascontiguousarray(self.allow_lent, np.uint8)
        self.max_mask = np.ascontiguousarray(self.max_mask, np.uint32)
        c.parent = _p32(self.parent)
        c.allow_lent = self.allow_lent.ctypes.data_as(C.POINTER(C.c_uint8))
        c.max_mask = _pu32(self.max_mask)
        for name in ("max", "min", "guaranteed", "self_request", "shared_weight"):
            arr = getattr(self, name)
            if arr is None:
                continue
            arr = np.ascontiguousarray(arr, np.int64)
            setattr(self, name, arr)
            field = getattr(c, name)
            for d in range(abi.KS_QUOTA_DIMS):
                field[d] = _p64(arr[d])
        for d in range(abi.KS_QUOTA_DIMS):
            c.cluster_total[d] = int(self.cluster_total[d])
        c._keep = self
        return c


DEV_I64 = ("total_core", "total_memory", "total_ratio", "used_core", "used_memory", "used_ratio")
DEV_RDMA = ("total_rdma", "used_rdma")
DEV_TOPO = (("gpu_pcie", abi.KS_MAX_GPUS), ("rdma_pcie", abi.KS_MAX_RDMA), ("pcie_numa", abi.KS_MAX_PCIE),
            ("pcie_socket", abi.KS_MAX_PCIE))


class DeviceTable:
    """Devices per node (ks_device_cols): [minor][node] arrays of total / used gpu-core, gpu-memory,
    gpu-memory-ratio and koordinator.sh/rdma (deviceshare nodeDeviceCache deviceTotal / deviceUsed), and the
    device topology: each minor's PCIe switch (dense per node in (socket, NUMA node, pcieID) order,
    KS_PCIE_NONE = no topology) and each switch's NUMA node and socket (newNUMATopology)."""

    def __init__(self, n: int):
        self.n = int(n)
        G = abi.KS_MAX_GPUS
        self.flags = np.zeros(self.n, np.uint32)
        for name in DEV_I64:
            setattr(self, name, np.zeros((G, self.n), np.int64))
        for name in DEV_RDMA:
            setattr(self, name, np.zeros((abi.KS_MAX_RDMA, self.n), np.int64))
        for name, k in DEV_TOPO:
            setattr(self, name, np.full((k, self.n), abi.KS_PCIE_NONE if name.endswith("pcie") else 0, np.uint8))

    def copy(self) -> "DeviceTable":
        t = DeviceTable(self.n)
        for k in ("flags",) + DEV_I64 + DEV_RDMA + tuple(x for x, _ in DEV_TOPO):
            setattr(t, k, getattr(self, k).copy())
        return t

    def ks(self) -> abi.KsDeviceCols:
        c = abi.KsDeviceCols()
        self.flags = np.ascontiguousarray(self.flags, np.uint32)
        c.flags = _pu32(self.flags)
        for name in DEV_I64 + DEV_RDMA:
            arr = np.ascontiguousarray(getattr(self, name), np.int64)
            setattr(self, name, arr)
            field = getattr(c, name)
            for k in range(arr.shape[0]):
                field[k] = _p64(arr[k])
        for name, kk in DEV_TOPO:
            arr = np.ascontiguousarray(getattr(self, name), np.uint8)
            setattr(self, name, arr)
            field = getattr(c, name)
            for k in range(kk):
                field[k] = arr[k].ctypes.data_as(C.POINTER(C.c_uint8))
        c._keep = self
        return c


def cpu_topology(core, numa_node, socket) -> abi.KsCpuTopology:
    """ks_cpu_topology from per-CPU ids (CPU c = index c)."""
    t = abi.KsCpuTopology()
    t.ncpus = len(core)
    for i in range(len(core)):
        t.core[i], t.numa_node[i], t.socket[i] = int(core[i]), int(numa_node[i]), int(socket[i])
    return t


def regular_topology(sockets: int, nodes_per_socket: int, cores_per_node: int, cpus_per_core: int) -> abi.KsCpuTopology:
    """CPU ids in (socket, node, core, thread) order, like buildCPUTopologyForTest
    (nodenumaresource/cpu_accumulator_test.go:30-57)."""
    core, node, sock = [], [], []
    cid = nid = 0
    for s in range(sockets):
        for _ in range(nodes_per_socket):
            for _ in range(cores_per_node):
                for _ in range(cpus_per_core):
                    core.append(cid)
                    node.append(nid)
                    sock.append(s)
                cid += 1
            nid += 1
    return cpu_topology(core, node, sock)


def cpu_mask(cpus) -> np.ndarray:
    """CPU list -> KS_CPU_WORDS uint64 words."""
    m = np.zeros(abi.KS_CPU_WORDS, np.uint64)
    for c in cpus:
        m[c >> 6] |= np.uint64(1) << np.uint64(c & 63)
    return m


def mask_cpus(m) -> list:
    out = []
    for w in range(abi.KS_CPU_WORDS):
        v = int(m[w])
        for b in range(64):
            if (v >> b) & 1:
                out.append(w * 64 + b)
    return out


class CpuState:
    """ks_cpu_state_cols + the topology table: per node a topology index (-1 = none) and CPU sets
    [node][KS_CPU_WORDS] (allocated, allocated with PCPULevel / NUMANodeLevel exclusivity, reserved)."""

    def __init__(self, n: int, topologies=()):
        self.n = int(n)
        self.topologies = list(topologies)
        self.topology = np.full(self.n, -1, np.int32)
        W = abi.KS_CPU_WORDS
        for k in ("allocated", "excl_pcpu", "excl_numa", "reserved"):
            setattr(self, k, np.zeros((self.n, W), np.uint64))

    def copy(self) -> "CpuState":
        t = CpuState(self.n, self.topologies)
        for k in ("topology", "allocated", "excl_pcpu", "excl_numa", "reserved"):
            setattr(t, k, getattr(self, k).copy())
        return t

    def topo_array(self):
        arr = (abi.KsCpuTopology * max(len(self.topologies), 1))()
        for i, t in enumerate(self.topologies):
            arr[i] = t
        return arr

    def ks(self) -> abi.KsCpuStateCols:
        c = abi.KsCpuStateCols()
        self.topology = np.ascontiguousarray(self.topology, np.int32)
        c.topology = _p32(self.topology)
        for k in ("allocated", "excl_pcpu", "excl_numa", "reserved"):
            arr = np.ascontiguousarray(getattr(self, k), np.uint64)
            setattr(self, k, arr)
            setattr(c, k, arr.ctypes.data_as(abi.PU64))
        c._keep = self
        return c


class NumaNodes:
    """ks_numa_node_cols: per node the NUMA nodes of a node with a NUMA topology policy, [node][k] arrays
    (NUMANodeResources cpu milli / memory, allocatedResources used cpu / memory + presence, cpuset CPUs)."""

    def __init__(self, n: int):
        self.n = int(n)
        K = abi.KS_MAX_NUMA
        self.count = np.zeros(self.n, np.int32)
        for k in ("alloc_cpu", "alloc_memory", "used_cpu", "used_memory"):
            setattr(self, k, np.zeros((self.n, K), np.int64))
        self.used_present = np.zeros((self.n, K), np.uint8)
        self.cpuset_cpus = np.zeros((self.n, K), np.int32)

    def copy(self) -> "NumaNodes":
        t = NumaNodes(self.n)
        for k in ("count", "alloc_cpu", "alloc_memory", "used_cpu", "used_memory", "used_present", "cpuset_cpus"):
            setattr(t, k, getattr(self, k).copy())
        return t

    def ks(self) -> abi.KsNumaNodeCols:
        c = abi.KsNumaNodeCols()
        self.count = np.ascontiguousarray(self.count, np.int32)
        c.count = _p32(self.count)
        for k in ("alloc_cpu", "alloc_memory", "used_cpu", "used_memory"):
            arr = np.ascontiguousarray(getattr(self, k), np.int64)
            setattr(self, k, arr)
            setattr(c, k, _p64(arr))
        self.used_present = np.ascontiguousarray(self.used_present, np.uint8)
        c.used_present = self.used_present.ctypes.data_as(C.POINTER(C.c_uint8))
        self.cpuset_cpus = np.ascontiguousarray(self.cpuset_cpus, np.int32)
        c.cpuset_cpus = _p32(self.cpuset_cpus)
        c._keep = self
        return c


class ReservationTable:
    """Available reservations (ks_reservation_cols): one row per ReservationInfo
    (pkg/scheduler/frameworkext/reservation_info.go:37-115); resources [dim][row] with dims
    cpu (milli), memory, ephemeral-storage, scalar[k].  DeviceShare (deviceshare/reservation.go): dev_allocatable /
    dev_allocated [row][KS_DEV_WORDS] (abi.dev_word) are the reserve pod's device allocation and its assigned pods'
    allocations on those minors; None = no reservation holds a device."""

    def __init__(self, r: int):
        self.r = int(r)
        self.dev_allocatable = None
        self.dev_allocated = None
        D = abi.KS_RSV_DIMS
        self.node = np.zeros(self.r, np.int32)
        self.owner_classes = np.zeros(self.r, np.uint64)
        self.flags = np.zeros(self.r, np.uint32)
        self.policy = np.zeros(self.r, np.uint32)
        self.order = np.zeros(self.r, np.int64)
        self.key_mask = np.zeros(self.r, np.uint32)
        self.allocatable = np.zeros((D, self.r), np.int64)
        self.allocated = np.zeros((D, self.r), np.int64)
        self.assigned = np.zeros(self.r, np.int32)

    def copy(self) -> "ReservationTable":
        t = ReservationTable(self.r)
        for k in ("node", "owner_classes", "flags", "policy", "order", "key_mask", "allocatable", "allocated",
                  "assigned"):
            setattr(t, k, getattr(self, k).copy())
        for k in ("dev_allocatable", "dev_allocated"):
            v = getattr(self, k)
            setattr(t, k, None if v is None else v.copy())
        return t

    def hold_devices(self) -> "ReservationTable":
        """allocate the device columns (zeros)"""
        if self.dev_allocatable is None:
            self.dev_allocatable = np.zeros((self.r, abi.KS_DEV_WORDS), np.int64)
            self.dev_allocated = np.zeros((self.r, abi.KS_DEV_WORDS), np.int64)
        return self

    def ks(self) -> abi.KsReservationCols:
        c = abi.KsReservationCols()
        for name, dt in (("node", np.int32), ("owner_classes", np.uint64), ("flags", np.uint32),
                         ("policy", np.uint32), ("order", np.int64), ("key_mask", np.uint32),
                         ("assigned", np.int32), ("allocatable", np.int64), ("allocated", np.int64)):
            setattr(self, name, np.ascontiguousarray(getattr(self, name), dt))
        c.node = _p32(self.node)
        c.owner_classes = self.owner_classes.ctypes.data_as(C.POINTER(C.c_uint64))
        c.flags = _pu32(self.flags)
        c.policy = _pu32(self.policy)
        c.order = _p64(self.order)
        c.key_mask = _pu32(self.key_mask)
        c.assigned = _p32(self.assigned)
        for d in range(abi.KS_RSV_DIMS):
            c.allocatable[d] = _p64(self.allocatable[d])
            c.allocated[d] = _p64(self.allocated[d])
        if self.dev_allocatable is not None:
            self.dev_allocatable = np.ascontiguousarray(self.dev_allocatable, np.int64).reshape(self.r, abi.KS_DEV_WORDS)
            self.dev_allocated = np.ascontiguousarray(self.dev_allocated, np.int64).reshape(self.r, abi.KS_DEV_WORDS)
            c.dev_allocatable = _p64(self.dev_allocatable)
            c.dev_allocated = _p64(self.dev_allocated)
        c._keep = self
        return c


class NodePodTable:
    """NodeInfo.Pods of every node for the preemption dry runs (ks_node_pod_cols): one row per running pod with its
    node, priority, start time, KS_NPOD_* flags, quota row, PodDisruptionBudget index, its part of NodeInfo.Requested
    ([dim][row]: cpu, memory, ephemeral-storage, scalar[k]) and its quota request (PodRequestsAndLimits,
    [dim][row]); plus the PodDisruptionBudgets' DisruptionsAllowed."""

    def __init__(self, m: int, npdb: int = 0):
        self.m = int(m)
        self.node = np.zeros(self.m, np.int32)
        self.priority = np.zeros(self.m, np.int32)
        self.start_time = np.zeros(self.m, np.int64)
        self.flags = np.full(self.m, abi.KS_NPOD_IN_QUOTA, np.uint32)
        self.quota = np.full(self.m, -1, np.int32)
        self.pdb = np.full(self.m, -1, np.int32)
        # further PodDisruptionBudgets the pod matches ([k][row], -1 = none; ks_node_pod_cols.pdb_more)
        self.pdb_more = np.full((abi.KS_NPOD_MORE_PDBS, self.m), -1, np.int32)
        self.req = np.zeros((abi.KS_RSV_DIMS, self.m), np.int64)
        self.quota_req = np.zeros((abi.KS_QUOTA_DIMS, self.m), np.int64)
        self.pdb_allowed = np.zeros(int(npdb), np.int32)

    def copy(self) -> "NodePodTable":
        t = NodePodTable(self.m, len(self.pdb_allowed))
        for k in ("node", "priority", "start_time", "flags", "quota", "pdb", "pdb_more", "req", "quota_req", "pdb_allowed"):
            setattr(t, k, getattr(self, k).copy())
        return t

    def rows(self, idx) -> "NodePodTable":
        idx = np.asarray(idx)
        t = NodePodTable(len(idx), len(self.pdb_allowed))
        for k in ("node", "priority", "start_time", "flags", "quota", "pdb"):
            setattr(t, k, getattr(self, k)[idx].copy())
        t.req = self.req[:, idx].copy()
        t.quota_req = self.quota_req[:, idx].copy()
        t.pdb_more = self.pdb_more[:, idx].copy()
        t.pdb_allowed = self.pdb_allowed.copy()
        return t

    def ks(self) -> abi.KsNodePodCols:
        c = abi.KsNodePodCols()
        for name, dt in (("node", np.int32), ("priority", np.int32), ("start_time", np.int64), ("flags", np.uint32),
                         ("quota", np.int32), ("pdb", np.int32), ("pdb_more", np.int32), ("req", np.int64),
                         ("quota_req", np.int64), ("pdb_allowed", np.int32)):
            setattr(self, name, np.ascontiguousarray(getattr(self, name), dt))
        c.node = _p32(self.node)
        c.priority = _p32(self.priority)
        c.start_time = _p64(self.start_time)
        c.flags = _pu32(self.flags)
        c.quota = _p32(self.quota)
        c.pdb = _p32(self.pdb)
        c.req_milli_cpu = _p64(self.req[0])
        c.req_memory = _p64(self.req[1])
        c.req_ephemeral = _p64(self.req[2])
        for k in range(abi.KS_MAX_SCALARS):
            c.req_scalar[k] = _p64(self.req[3 + k])
        for d in range(abi.KS_QUOTA_DIMS):
            c.quota_req[d] = _p64(self.quota_req[d])
        for k in range(abi.KS_NPOD_MORE_PDBS):
            c.pdb_more[k] = _p32(self.pdb_more[k])
        c._keep = self
        return c


class NodeState:
    """Host buffers for ks_read_nodes / ko_read_nodes."""

    def __init__(self, n: int, nprops: int = 0):
        self.n = n
        for name in STATE_I64:
            setattr(self, name, np.zeros(n, np.int64))
        self.pod_count = np.zeros(n, np.int32)
        self.req_scalar = np.zeros((abi.KS_MAX_SCALARS, n), np.int64)
        self.host_ports = np.zeros(n, np.uint64)
        self.topo_count = np.zeros((nprops, n), np.int32)

    def ks(self) -> abi.KsNodeState:
        s = abi.KsNodeState()
        for name in STATE_I64:
            setattr(s, name, _p64(getattr(self, name)))
        s.pod_count = _p32(self.pod_count)
        s.host_ports = self.host_ports.ctypes.data_as(C.POINTER(C.c_uint64))
        for k in range(abi.KS_MAX_SCALARS):
            s.req_scalar[k] = _p64(self.req_scalar[k])
        s.topo_count = _p32(self.topo_count) if self.topo_count.size else None
        s._keep = self
        return s

    def as_dict(self) -> Dict[str, np.ndarray]:
        d = {k: getattr(self, k) for k in STATE_I64}
        d["pod_count"] = self.pod_count
        d["req_scalar"] = self.req_scalar
        d["host_ports"] = self.host_ports
        d["topo_count"] = self.topo_count
        return d


def results_to_numpy(res) -> Dict[str, np.ndarray]:
    arr = np.ctypeslib.as_array(res)
    return {
        "node": np.array([r.node for r in res], np.int32) if arr.dtype.names is None else arr["node"].copy(),
        "status": np.array([r.status for r in res], np.uint32) if arr.dtype.names is None else arr["status"].copy(),
        "score": np.array([r.score for r in res], np.int64) if arr.dtype.names is None else arr["score"].copy(),
        "reservation": np.array([r.reservation for r in res], np.int32) if arr.dtype.names is None
        else arr["reservation"].copy(),
    }
