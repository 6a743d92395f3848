"""Synthetic clusters for the benchmark configurations.

All generators are deterministic (numpy PCG64, seed 20261015 by default) and
emit the structure-of-arrays tables the C ABI consumes, i.e. what the Go host
would produce from a scheduler-cache snapshot plus NodeMetric objects:

* C1  500 nodes, 1k pods, NodeResourcesFit + LoadAwareScheduling
* C2  5k nodes, 10k pods, + ElasticQuota admission (32 leaf quotas under root,
      limits sized so roughly a tenth of the pods are rejected)
* C3  5k nodes with 8 (or 4) 80 GiB GPUs and 4 RDMA devices on 4 PCIe switches / 2 NUMA nodes each
      (make_devices, the device_allocator_test.go layout) and cpu amplification ratios with cpuset-held
      CPUs (NodeNUMAResource); 10k pods, 40 % requesting GPUs (whole devices 1/2/4, half a GPU by ratio,
      or a gpu-memory amount; half of the whole-GPU pods with rdma 1 and joint [gpu, rdma] allocation,
      half of those SamePCIe), a few RDMA-only pods, and cpuset (LSR) pods; Fit + LoadAware +
      NodeNUMAResource + DeviceShare.  Half of the nodes carry the SingleNUMANode topology policy with two
      NUMA nodes (policy_numa_nodes): NodeNUMAResource and DeviceShare are both hint providers there, and
      cpuset pods take their CPUs per allocated NUMA node
* C4  20k nodes with 50k reservations (make_reservations), 10k pods of which 60 % belong to one
      of 16 reservation owner classes, NodeResourcesFit + LoadAwareScheduling + Reservation (weight 5000)
* C5  100k nodes, C1 pod distribution (the multi-GPU sharding config)

Node model: allocatable cpu ∈ {32,48,64,96} cores, memory ∈ {128,256,384,512}
GiB, ephemeral 1 TiB, 110 pods; already-running pods give requested ≈ U(0,0.5)
of allocatable; NodeMetric usage cpu ~ U(0,0.75)·alloc, memory ~ U(0,0.95)·alloc,
reported at the frozen "now" (so nothing is expired and no assigned pod is
counted twice); batch-cpu / batch-memory allocatable (koordlet batch resource)
= 40 % of allocatable.

Pod model: 70 % default-priority pods (Burstable → koord-prod by QoS, priority_utils.go:26-47)
and 20 % explicit koord-prod pods requesting cpu ∈ {250m..8000m step 250m} and
memory ∈ {256Mi..16Gi step 256Mi}, 30 % of them with limit = 1.5 × request;
10 % koord-batch pods requesting the same shapes as kubernetes.io/batch-cpu
(milli-cores as a plain integer) and kubernetes.io/batch-memory.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import abi
from .cluster import CpuState, DeviceTable, NodeTable, PodTable, QuotaTable, ReservationTable, cpu_mask, regular_topology
from .config import BATCH_CPU, BATCH_MEMORY, CPU, MEMORY, ElasticQuotaArgs, NodeResourcesFitArgs, SchedulerProfile

SEED = 20261015
GI = 1 << 30
MI = 1 << 20
DEFAULT_MILLI_CPU_LA = 250  # loadaware estimator DefaultMilliCPURequest
DEFAULT_MEMORY_LA = 200 * MI
DEFAULT_MILLI_CPU_NZ = 100  # upstream schedutil.DefaultMilliCPURequest (non-zero request)
DEFAULT_MEMORY_NZ = 200 * MI

SLOT_BATCH_CPU = 0
SLOT_BATCH_MEMORY = 1

QDIM_CPU, QDIM_MEMORY, QDIM_BATCH_CPU, QDIM_BATCH_MEMORY = 0, 1, 2, 3


@dataclass
class Workload:
    name: str
    profile: SchedulerProfile
    nodes: NodeTable
    pods: PodTable
    quotas: Optional[QuotaTable]
    reservations: Optional[ReservationTable] = None
    devices: Optional["DeviceTable"] = None
    cpus: Optional[CpuState] = None
    numa_nodes: Optional["NumaNodes"] = None

    @property
    def cfg(self) -> abi.KsConfig:
        return self.profile.to_ks_config()

    def tables(self, copy: bool = True) -> dict:
        """The non-node tables as the keyword arguments of runtime.Evaluator / the oracle (copies by default:
        both consume and mutate what they are given)."""
        out = {}
        for k, v in (("quotas", self.quotas), ("reservations", self.reservations), ("devices", self.devices),
                     ("cpu_state", self.cpus), ("numa_nodes", self.numa_nodes)):
            if v is not None:
                out[k] = v.copy() if copy else v
        return out


def koord_profile(with_quota: bool = False, batch_pods: int = 0, candidates: int = 0,
                  with_reservation: bool = False) -> SchedulerProfile:
    """NodeResourcesFit (LeastAllocated cpu/memory/batch-cpu/batch-memory, weight 1 each:
    config/manager/scheduler-config.yaml:17-31) + LoadAwareScheduling defaults (+ Reservation, weight
    5000 in the same profile)."""
    fit = NodeResourcesFitArgs(resources={CPU: 1, MEMORY: 1, BATCH_CPU: 1, BATCH_MEMORY: 1})
    return SchedulerProfile(fit=fit, quota=ElasticQuotaArgs() if with_quota else None,
                            reservation_weight=5000 if with_reservation else None,
                            batch_pods=batch_pods, candidates=candidates)


def make_nodes(n: int, rng: np.random.Generator, thresholds=(65, 95)) -> NodeTable:
    t = NodeTable(n)
    cores = rng.choice(np.array([32, 48, 64, 96], np.int64), n)
    mem_gi = rng.choice(np.array([128, 256, 384, 512], np.int64), n)
    t.alloc_milli_cpu[:] = cores * 1000
    t.alloc_memory[:] = mem_gi * GI
    t.alloc_ephemeral[:] = 1024 * GI
    t.allowed_pods[:] = 110
    t.pod_count[:] = rng.integers(0, 60, n)
    frac_c = rng.uniform(0.0, 0.5, n)
    frac_m = rng.uniform(0.0, 0.5, n)
    t.req_milli_cpu[:] = (t.alloc_milli_cpu * frac_c).astype(np.int64)
    t.req_memory[:] = (t.alloc_memory * frac_m).astype(np.int64) // MI * MI
    t.req_ephemeral[:] = rng.integers(0, 64, n) * GI
    t.nonzero_milli_cpu[:] = t.req_milli_cpu + t.pod_count * 0  # every running pod declared requests
    t.nonzero_memory[:] = t.req_memory
    # koordlet batch resources (kubernetes.io/batch-cpu in milli-cores, batch-memory in bytes)
    t.alloc_scalar[SLOT_BATCH_CPU] = t.alloc_milli_cpu * 4 // 10
    t.alloc_scalar[SLOT_BATCH_MEMORY] = t.alloc_memory * 4 // 10
    t.req_scalar[SLOT_BATCH_CPU] = (t.alloc_scalar[SLOT_BATCH_CPU] * rng.uniform(0, 0.3, n)).astype(np.int64)
    t.req_scalar[SLOT_BATCH_MEMORY] = (t.alloc_scalar[SLOT_BATCH_MEMORY] * rng.uniform(0, 0.3, n)).astype(np.int64)
    # NodeMetric: usage, frozen now, nothing expired, no assigned-not-reported pods
    use_c = (t.alloc_milli_cpu * rng.uniform(0.0, 0.75, n)).astype(np.int64)
    use_m = (t.alloc_memory * rng.uniform(0.0, 0.95, n)).astype(np.int64)
    prod_share = rng.uniform(0.3, 0.9, n)
    t.la_flags[:] = (abi.KS_LA_HAS_METRIC | abi.KS_LA_HAS_STATUS_METRIC | abi.KS_LA_FILTER_USAGE_PRESENT
                     | abi.KS_LA_NODE_THR_NONEMPTY | abi.KS_LA_HAS_PODS_METRIC)
    t.la_alloc_milli_cpu[:] = t.alloc_milli_cpu
    t.la_alloc_memory[:] = t.alloc_memory
    t.la_term_milli_cpu[:] = use_c
    t.la_term_memory[:] = use_m
    t.la_prod_term_milli_cpu[:] = (use_c * prod_share).astype(np.int64)
    t.la_prod_term_memory[:] = (use_m * prod_share).astype(np.int64)
    t.la_thr_cpu[:] = thresholds[0]
    t.la_thr_memory[:] = thresholds[1]
    t.la_total_milli_cpu[:] = t.alloc_milli_cpu
    t.la_total_milli_memory[:] = t.alloc_memory * 1000
    t.la_usage_milli_cpu[:] = use_c
    t.la_usage_milli_memory[:] = use_m * 1000
    t.la_prod_usage_milli_cpu[:] = t.la_prod_term_milli_cpu
    t.la_prod_usage_milli_memory[:] = t.la_prod_term_memory * 1000
    return t


def make_pods(p: int, rng: np.random.Generator, n_quotas: int = 0) -> PodTable:
    t = PodTable(p)
    cpu = rng.integers(1, 33, p) * 250
    mem = rng.integers(1, 65, p) * 256 * MI
    has_lim = rng.random(p) < 0.3
    lim_cpu = np.where(has_lim, cpu * 3 // 2, 0)
    lim_mem = np.where(has_lim, mem * 3 // 2, 0)
    kind = rng.choice(np.array([0, 1, 2]), p, p=[0.7, 0.2, 0.1])  # 0 default, 1 explicit prod, 2 batch
    batch = kind == 2
    t.flags[:] = np.where(batch, 0, abi.KS_POD_PROD).astype(np.uint32)
    t.flags[batch] |= abi.KS_POD_SCALAR_KEYS
    t.req_milli_cpu[:] = np.where(batch, 0, cpu)
    t.req_memory[:] = np.where(batch, 0, mem)
    t.req_scalar[SLOT_BATCH_CPU] = np.where(batch, cpu, 0)
    t.req_scalar[SLOT_BATCH_MEMORY] = np.where(batch, mem, 0)
    t.nonzero_milli_cpu[:] = np.where(batch, DEFAULT_MILLI_CPU_NZ, cpu)
    t.nonzero_memory[:] = np.where(batch, DEFAULT_MEMORY_NZ, mem)
    # EstimatePod: translated resource (batch pods -> batch-cpu / batch-memory) request/limit
    t.la_req_cpu[:] = cpu
    t.la_lim_cpu[:] = lim_cpu
    t.la_req_memory[:] = mem
    t.la_lim_memory[:] = lim_mem
    t.la_dflt_cpu[:] = DEFAULT_MILLI_CPU_LA
    t.la_dflt_memory[:] = DEFAULT_MEMORY_LA
    if n_quotas:
        t.quota[:] = rng.integers(0, n_quotas, p)
        t.quota_req[QDIM_CPU] = t.req_milli_cpu
        t.quota_req[QDIM_MEMORY] = t.req_memory
        t.quota_req[QDIM_BATCH_CPU] = t.req_scalar[SLOT_BATCH_CPU]
        t.quota_req[QDIM_BATCH_MEMORY] = t.req_scalar[SLOT_BATCH_MEMORY]
        t.quota_mask[:] = np.where(batch, (1 << QDIM_BATCH_CPU) | (1 << QDIM_BATCH_MEMORY),
                                   (1 << QDIM_CPU) | (1 << QDIM_MEMORY)).astype(np.uint32)
    return t


def make_quotas(pods: PodTable, n_quotas: int, rng: np.random.Generator, admit_frac: float = 0.9) -> QuotaTable:
    """Leaf quotas directly under root whose runtime limits admit ~admit_frac of demand."""
    q = QuotaTable(n_quotas)
    q.limit_mask[:] = (1 << QDIM_CPU) | (1 << QDIM_MEMORY) | (1 << QDIM_BATCH_CPU) | (1 << QDIM_BATCH_MEMORY)
    for d in (QDIM_CPU, QDIM_MEMORY, QDIM_BATCH_CPU, QDIM_BATCH_MEMORY):
        has = pods.quota >= 0
        demand = np.bincount(pods.quota[has], weights=pods.quota_req[d][has].astype(np.float64), minlength=n_quotas)
        q.limit[d] = (demand * admit_frac * rng.uniform(0.95, 1.05, n_quotas)).astype(np.int64)
    q.min_mask[:] = q.limit_mask
    q.min[:] = q.limit // 2
    return q


def make_reservations(nodes: NodeTable, r: int, rng: np.random.Generator, n_classes: int = 16,
                      order_frac: float = 0.03, assigned_frac: float = 0.25) -> ReservationTable:
    """Available reservations spread uniformly over the nodes (~r/n per node).  Each reserves
    cpu ∈ {2,4,8} cores with 2 or 4 GiB memory per core (keys cpu + memory), belongs to one owner
    class (10 % to two), 5 % are unschedulable, 20 % AllocateOnce, policies Default 60 % / Aligned
    25 % / Restricted 15 %, a few carry a reservation-order label, and a quarter already hold 1-3
    assigned pods using part of them.  The reserve pods and the assigned pods are added to the
    nodes' NodeInfo (requested, non-zero requested, pod count) as the scheduler cache holds them."""
    t = ReservationTable(r)
    t.node[:] = rng.integers(0, nodes.n, r)
    cls = rng.integers(0, n_classes, r).astype(np.uint64)
    two = rng.random(r) < 0.1
    cls2 = rng.integers(0, n_classes, r).astype(np.uint64)
    t.owner_classes[:] = (np.uint64(1) << cls) | np.where(two, np.uint64(1) << cls2, np.uint64(0))
    u = rng.random(r)
    t.flags[:] = np.where(u < 0.05, abi.KS_RSV_UNSCHEDULABLE, np.where(u < 0.25, abi.KS_RSV_ALLOCATE_ONCE, 0))
    t.policy[:] = rng.choice(np.array([abi.KS_RSV_POLICY_DEFAULT, abi.KS_RSV_POLICY_ALIGNED,
                                       abi.KS_RSV_POLICY_RESTRICTED], np.uint32), r, p=[0.6, 0.25, 0.15])
    t.order[:] = np.where(rng.random(r) < order_frac, rng.integers(1, 1000, r), 0)
    t.key_mask[:] = 0b11
    cores = rng.choice(np.array([2, 4, 8], np.int64), r)
    t.allocatable[0] = cores * 1000
    t.allocatable[1] = cores * rng.choice(np.array([2, 4], np.int64), r) * GI
    has = rng.random(r) < assigned_frac
    t.assigned[:] = np.where(has, rng.integers(1, 4, r), 0)
    frac = rng.choice(np.array([1, 2, 3, 4], np.int64), r)
    t.allocated[0] = np.where(has, t.allocatable[0] * frac // 4, 0)
    t.allocated[1] = np.where(has, t.allocatable[1] * frac // 4 // MI * MI, 0)
    add_cpu = t.allocatable[0] + t.allocated[0]
    add_mem = t.allocatable[1] + t.allocated[1]
    nodes.req_milli_cpu[:] += np.bincount(t.node, weights=add_cpu, minlength=nodes.n).astype(np.int64)
    nodes.req_memory[:] += np.bincount(t.node, weights=add_mem.astype(np.float64), minlength=nodes.n).astype(np.int64)
    nodes.nonzero_milli_cpu[:] += np.bincount(t.node, weights=add_cpu, minlength=nodes.n).astype(np.int64)
    nodes.nonzero_memory[:] += np.bincount(t.node, weights=add_mem.astype(np.float64), minlength=nodes.n).astype(np.int64)
    nodes.pod_count[:] += np.bincount(t.node, weights=1 + t.assigned, minlength=nodes.n).astype(np.int32)
    return t


def reservation_pods(pods: PodTable, rng: np.random.Generator, n_classes: int = 16, class_frac: float = 0.6,
                     affinity_frac: float = 0.05) -> PodTable:
    """Give pods an owner class (matching reservations of that class) and, for a few, a required
    reservation affinity."""
    p = pods.n
    classed = rng.random(p) < class_frac
    pods.rsv_class[:] = np.where(classed, rng.integers(0, n_classes, p), -1)
    aff = classed & (rng.random(p) < affinity_frac)
    pods.flags[aff] |= abi.KS_POD_RSV_AFFINITY
    return pods


def make_devices(nodes: NodeTable, rng: np.random.Generator, gpu_frac: float = 0.9, rdma: bool = False) -> "DeviceTable":
    """GPU devices (DeviceShare): 90 % of the nodes carry 8 (or 4) GPUs of 80 GiB (gpu-core 100,
    gpu-memory-ratio 100 each), some already partly used by running GPU pods; the rest have no
    device information.  A few nodes carry an unhealthy minor (zero totals)."""
    from .cluster import DeviceTable
    n = nodes.n
    d = DeviceTable(n)
    has = rng.random(n) < gpu_frac
    d.flags[:] = np.where(has, abi.KS_DEV_PRESENT, 0)
    count = np.where(rng.random(n) < 0.75, 8, 4)
    for k in range(abi.KS_MAX_GPUS):
        on = has & (k < count) & (rng.random(n) > 0.01)
        d.total_core[k] = np.where(on, 100, 0)
        d.total_ratio[k] = np.where(on, 100, 0)
        d.total_memory[k] = np.where(on, 80 * GI, 0)
        used = on & (rng.random(n) < 0.3)
        part = rng.choice(np.array([25, 50, 100], np.int64), n)
        d.used_core[k] = np.where(used, part, 0)
        d.used_ratio[k] = np.where(used, part, 0)
        d.used_memory[k] = np.where(used, part * 80 * GI // 100, 0)
    if rdma:
        # the layout of deviceshare/device_allocator_test.go:49-57: GPU k on PCIe switch k // 2, RDMA minor
        # j = 1..4 on switch j - 1, switches 0-1 on socket 0 / NUMA node 0 and 2-3 on socket 1 / node 1;
        # koordinator.sh/rdma 100 per RDMA device, some partly used
        for k in range(abi.KS_MAX_GPUS):
            d.gpu_pcie[k] = np.where(d.total_ratio[k] > 0, k // 2, abi.KS_PCIE_NONE)
        for j in range(1, 5):
            on = has & (rng.random(n) > 0.02)
            d.total_rdma[j] = np.where(on, 100, 0)
            d.used_rdma[j] = np.where(on & (rng.random(n) < 0.3), rng.choice(np.array([1, 50, 100], np.int64), n), 0)
            d.rdma_pcie[j] = j - 1
        for p in range(4):
            d.pcie_numa[p] = p // 2
            d.pcie_socket[p] = p // 2
    return d


def rdma_pods(pods: PodTable, rng: np.random.Generator, joint_frac: float = 0.5, rdma_only: float = 0.03,
              joint_no_rdma: float = 0.0) -> PodTable:
    """Half of the whole-GPU pods also ask for koordinator.sh/rdma 1 with joint [gpu, rdma] allocation (half of
    those with RequiredScope SamePCIe, SURVEY C3's "GPU+RDMA joint SamePCIe" pods); a few pods ask for RDMA
    only (1, 50 or 100 = one whole device).  joint_no_rdma: that fraction of the joint pods keeps the joint spec
    without the RDMA request (jointAllocate then takes RDMA devices with a nil request)."""
    p = pods.n
    whole = (pods.gpu_core >= 100) & (pods.gpu_core % 100 == 0)
    j = whole & (rng.random(p) < joint_frac)
    same = rng.random(p) < 0.5
    pods.rdma[:] = np.where(j, 1, 0)
    pods.joint[:] = np.where(j, np.where(same, abi.KS_JOINT_GPU_RDMA_SAME_PCIE, abi.KS_JOINT_GPU_RDMA), 0)
    only = (pods.gpu_core + pods.gpu_memory + pods.gpu_memory_ratio == 0) & (rng.random(p) < rdma_only)
    pods.rdma[:] = np.where(only, rng.choice(np.array([1, 50, 100], np.int64), p), pods.rdma)
    if joint_no_rdma:
        pods.rdma[:] = np.where(j & (rng.random(p) < joint_no_rdma), 0, pods.rdma)
    return pods


def gpu_pods(pods: PodTable, rng: np.random.Generator, frac: float = 0.4) -> PodTable:
    """40 % of the pods request GPUs: whole devices (nvidia.com/gpu 1, 2, 4 -> core = ratio = 100 x n),
    half a GPU by ratio, or a memory amount (gpu-memory, ratio derived per node)."""
    p = pods.n
    g = rng.random(p) < frac
    kind = rng.choice(np.array([0, 1, 2, 3, 4]), p, p=[0.35, 0.2, 0.1, 0.2, 0.15])
    whole = np.array([100, 200, 400, 50, 0])[kind]
    pods.gpu_core[:] = np.where(g & (kind < 4), whole, 0)
    pods.gpu_memory_ratio[:] = np.where(g & (kind < 4), whole, 0)
    pods.gpu_memory[:] = np.where(g & (kind == 4), rng.choice(np.array([10, 20, 40], np.int64), p) * GI, 0)
    pods.flags[:] |= np.where(g & (kind < 4), abi.KS_POD_GPU_CORE, 0).astype(np.uint32)
    pods.flags[:] |= np.where(g & (kind == 4), abi.KS_POD_GPU_MEMORY, 0).astype(np.uint32)
    return pods


# node CPU topologies by core count: (sockets, NUMA nodes per socket, cores per NUMA node, threads per core)
CPU_TOPOLOGIES = {32: (2, 1, 8, 2), 48: (2, 1, 12, 2), 64: (2, 2, 8, 2), 96: (2, 2, 12, 2)}
# the two-NUMA-node layout of the same core counts (one NUMA node per socket), for nodes with a NUMA policy
CPU_TOPOLOGIES_2NUMA = {32: (2, 1, 8, 2), 48: (2, 1, 12, 2), 64: (2, 1, 16, 2), 96: (2, 1, 24, 2)}


def make_cpu_state(nodes: NodeTable, rng: np.random.Generator, cores=None, no_topology: float = 0.05,
                   max_alloc: float = 0.3, label_frac: float = 0.2, two_numa=None) -> CpuState:
    """NodeResourceTopology-derived CPU state: a regular topology per node (by its core count), a
    fragmented set of already-allocated CPUs (exclusive policy None / PCPULevel / NUMANodeLevel), kubelet
    reserved CPUs 0-1 on a third of the nodes, and numa-allocate-strategy labels on some nodes.  Node
    Requested cpu and numa_cpuset_cpus are raised to include the allocated cpusets.  Nodes in two_numa
    (a mask) get the one-NUMA-node-per-socket layout."""
    n = nodes.n
    cores = np.asarray(cores if cores is not None else nodes.alloc_milli_cpu // 1000)
    keys = sorted(CPU_TOPOLOGIES)
    st = CpuState(n, [regular_topology(*CPU_TOPOLOGIES[k]) for k in keys] +
                  [regular_topology(*CPU_TOPOLOGIES_2NUMA[k]) for k in keys])
    two = np.zeros(n, bool) if two_numa is None else np.asarray(two_numa, bool)
    W = abi.KS_CPU_WORDS
    for i in range(n):
        c = int(cores[i])
        if c not in CPU_TOPOLOGIES or rng.random() < no_topology:
            continue
        st.topology[i] = keys.index(c) + (len(keys) if two[i] else 0)
        resv = [0, 1] if rng.random() < 0.33 else []
        free = np.array([x for x in range(c) if x not in resv])
        k = int(rng.integers(0, int(max_alloc * c) + 1))
        taken = rng.choice(free, k, replace=False) if k else np.zeros(0, np.int64)
        pol = rng.choice(np.array([0, 1, 2]), len(taken), p=[0.6, 0.3, 0.1])
        st.allocated[i] = cpu_mask(taken)
        st.excl_pcpu[i] = cpu_mask(taken[pol == 1])
        st.excl_numa[i] = cpu_mask(taken[pol == 2])
        st.reserved[i] = cpu_mask(resv)
        nodes.numa_cpuset_cpus[i] = len(taken)
        nodes.req_milli_cpu[i] += len(taken) * 1000
        nodes.nonzero_milli_cpu[i] += len(taken) * 1000
    lab = rng.random(n) < label_frac
    nodes.numa_flags[:] |= np.where(lab, np.where(rng.random(n) < 0.5, abi.KS_NUMA_ALLOC_MOST, abi.KS_NUMA_ALLOC_LEAST),
                                    0).astype(np.uint32)
    assert st.allocated.shape == (n, W)
    return st


def cpuset_pods(pods: PodTable, rng: np.random.Generator, frac: float = 0.4, exclude=None) -> PodTable:
    """LSR/LSE prod pods with a preferred cpuset: 4-16 CPUs (FullPCPUs requests in whole 2-thread cores),
    70 % FullPCPUs / 30 % SpreadByPCPUs, exclusive policy None / PCPULevel / NUMANodeLevel."""
    p = pods.n
    sel = rng.random(p) < frac
    if exclude is not None:
        sel &= ~np.asarray(exclude)
    full = rng.random(p) < 0.7
    k = np.where(full, 2 * rng.integers(2, 9, p), rng.integers(4, 17, p))
    excl = rng.choice(np.array([0, 1, 2]), p, p=[0.6, 0.25, 0.15])
    bind = np.where(full, abi.KS_CPU_BIND_FULL_PCPUS, abi.KS_CPU_BIND_SPREAD_BY_PCPUS) | (excl << abi.KS_CPU_EXCL_SHIFT)
    cpu = k * 1000
    pods.cpu_bind[:] = np.where(sel, bind, 0).astype(np.uint32)
    pods.flags[:] = np.where(sel, (pods.flags & ~np.uint32(abi.KS_POD_SCALAR_KEYS)) | abi.KS_POD_PROD | abi.KS_POD_CPU_BIND,
                             pods.flags).astype(np.uint32)
    mem = np.where(pods.req_memory > 0, pods.req_memory, pods.req_scalar[SLOT_BATCH_MEMORY])
    pods.req_milli_cpu[:] = np.where(sel, cpu, pods.req_milli_cpu)
    pods.req_memory[:] = np.where(sel, mem, pods.req_memory)
    pods.nonzero_milli_cpu[:] = np.where(sel, cpu, pods.nonzero_milli_cpu)
    pods.nonzero_memory[:] = np.where(sel, mem, pods.nonzero_memory)
    pods.la_req_cpu[:] = np.where(sel, cpu, pods.la_req_cpu)
    pods.la_lim_cpu[:] = np.where(sel, 0, pods.la_lim_cpu)
    for slot in (SLOT_BATCH_CPU, SLOT_BATCH_MEMORY):
        pods.req_scalar[slot] = np.where(sel, 0, pods.req_scalar[slot])
    return pods


def cpu_bind_policies(nodes: NodeTable, pods: PodTable, rng: np.random.Generator, label_frac: float = 0.4,
                      required_frac: float = 0.4, whole_frac: float = 0.5, odd_frac: float = 0.1) -> None:
    """Node CPU bind policies (the node-cpu-bind-policy label, FullPCPUsOnly / SpreadByPCPUs in equal parts) on
    label_frac of the nodes; a required bind policy on required_frac of the cpuset pods (some required FullPCPUs
    requests an odd number of CPUs: the SMT alignment check); whole-CPU requests for whole_frac of the other pods
    (cpu-bind on a labelled node, requestCPUBind util.go:105-122; the rest fail ErrInvalidRequestedCPUs there)."""
    n, p = nodes.n, pods.n
    lab = np.where(rng.random(n) < label_frac, rng.integers(1, 3, n), 0).astype(np.uint32)
    nodes.numa_flags[:] = (nodes.numa_flags & ~np.uint32(3 << abi.KS_NUMA_CPU_BIND_SHIFT)) | (lab << abi.KS_NUMA_CPU_BIND_SHIFT)
    bind = (pods.flags & abi.KS_POD_CPU_BIND) != 0
    req = bind & (rng.random(p) < required_frac)
    pods.cpu_bind[:] = np.where(req, pods.cpu_bind | abi.KS_CPU_BIND_REQUIRED, pods.cpu_bind).astype(np.uint32)
    odd = req & ((pods.cpu_bind & abi.KS_CPU_BIND_POLICY_MASK) == abi.KS_CPU_BIND_FULL_PCPUS) & (rng.random(p) < odd_frac)
    for col in ("req_milli_cpu", "nonzero_milli_cpu", "la_req_cpu"):
        v = getattr(pods, col)
        v[:] = np.where(odd, v + 1000, v)
    whole = ~bind & (pods.req_milli_cpu > 0) & (rng.random(p) < whole_frac)
    cpu = np.clip((pods.req_milli_cpu + 999) // 1000, 1, 24) * 1000
    for col in ("req_milli_cpu", "nonzero_milli_cpu"):
        v = getattr(pods, col)
        v[:] = np.where(whole, cpu, v)


def make_numa_nodes(nodes: NodeTable, rng: np.random.Generator, policy_frac: float = 0.5, cores=None):
    """NUMA topology policies on a fraction of the nodes (best-effort / restricted / single-numa-node in equal
    parts), 1, 2 or 4 NUMA nodes splitting the node's CPUs and memory, and earlier pods' NUMA allocations
    (allocatedResources) on some NUMA nodes.  Returns the NumaNodes table; policies go into numa_flags."""
    from .cluster import NumaNodes
    n = nodes.n
    cores = np.asarray(cores if cores is not None else nodes.alloc_milli_cpu // 1000)
    nn = NumaNodes(n)
    pol = np.where(rng.random(n) < policy_frac, rng.integers(1, 4, n), 0).astype(np.uint32)
    nodes.numa_flags[:] = (nodes.numa_flags & ~np.uint32(3 << abi.KS_NUMA_POLICY_SHIFT)) | (pol << abi.KS_NUMA_POLICY_SHIFT)
    cnt = rng.choice(np.array([1, 2, 4]), n, p=[0.2, 0.6, 0.2])
    for i in range(n):
        if pol[i] == 0:
            continue
        k = int(cnt[i])
        nn.count[i] = k
        nn.alloc_cpu[i, :k] = int(cores[i]) * 1000 // k
        nn.alloc_memory[i, :k] = int(nodes.alloc_memory[i]) // k
        for j in range(k):
            if rng.random() < 0.5:
                f = rng.random() * 0.6
                nn.used_cpu[i, j] = int(nn.alloc_cpu[i, j] * f) // 1000 * 1000
                nn.used_memory[i, j] = int(nn.alloc_memory[i, j] * f) // MI * MI
                nn.used_present[i, j] = 1
    return nn


def policy_numa_nodes(nodes: NodeTable, cpus: CpuState, policy_mask, rng: np.random.Generator, cores,
                      policy: int = abi.KS_NUMA_POLICY_SINGLE_NUMA_NODE) -> "NumaNodes":
    """NodeResourceTopology zones of the policy nodes, consistent with their CPU state: two NUMA nodes (the
    one-NUMA-node-per-socket CPU topology) splitting cpu and memory, the allocated cpuset CPUs counted per NUMA
    node (cpuset_cpus, and in allocatedResources cpu), plus earlier non-cpuset pods' NUMA allocations."""
    from .cluster import NumaNodes
    n = nodes.n
    nn = NumaNodes(n)
    pol = np.where(policy_mask, policy, 0).astype(np.uint32)
    nodes.numa_flags[:] = (nodes.numa_flags & ~np.uint32(3 << abi.KS_NUMA_POLICY_SHIFT)) | (pol << abi.KS_NUMA_POLICY_SHIFT)
    W = abi.KS_CPU_WORDS
    for i in np.flatnonzero(policy_mask):
        c = int(cores[i])
        nn.count[i] = 2
        nn.alloc_cpu[i, :2] = c * 1000 // 2
        nn.alloc_memory[i, :2] = int(nodes.alloc_memory[i]) // 2
        if cpus.topology[i] >= 0:
            bits = np.unpackbits(cpus.allocated[i].view(np.uint8), bitorder="little")[: W * 64]
            held = np.flatnonzero(bits)
            for k in range(2):
                nn.cpuset_cpus[i, k] = int(np.count_nonzero(held // (c // 2) == k))
        for k in range(2):
            extra = 0
            if rng.random() < 0.5:
                f = rng.random() * 0.4
                extra = int(nn.alloc_cpu[i, k] * f) // 1000 * 1000
                nn.used_memory[i, k] = int(nn.alloc_memory[i, k] * f) // MI * MI
            nn.used_cpu[i, k] = int(nn.cpuset_cpus[i, k]) * 1000 + extra
            nn.used_present[i, k] = 1 if (nn.used_cpu[i, k] or nn.used_memory[i, k]) else 0
    return nn


def c1(seed: int = SEED, n_nodes: int = 500, n_pods: int = 1000, **kw) -> Workload:
    rng = np.random.Generator(np.random.PCG64(seed))
    nodes = make_nodes(n_nodes, rng)
    pods = make_pods(n_pods, rng)
    return Workload("C1", koord_profile(**kw), nodes, pods, None)


def c2(seed: int = SEED, n_nodes: int = 5000, n_pods: int = 10000, n_quotas: int = 32, **kw) -> Workload:
    rng = np.random.Generator(np.random.PCG64(seed))
    nodes = make_nodes(n_nodes, rng)
    pods = make_pods(n_pods, rng, n_quotas)
    quotas = make_quotas(pods, n_quotas, rng)
    return Workload("C2", koord_profile(with_quota=True, **kw), nodes, pods, quotas)


def c3(seed: int = SEED, n_nodes: int = 5000, n_pods: int = 10_000, policy_frac: float = 0.5,
       policy: int = abi.KS_NUMA_POLICY_SINGLE_NUMA_NODE, **kw) -> Workload:
    from .config import GPU_MEMORY_RATIO, DeviceShareArgs, NodeNUMAResourceArgs
    rng = np.random.Generator(np.random.PCG64(seed))
    nodes = make_nodes(n_nodes, rng)
    ratio = rng.choice(np.array([0.0, 1.0, 1.5, 2.0]), n_nodes)
    amp = ratio > 1
    cores = nodes.alloc_milli_cpu // 1000
    nodes.numa_cpu_amplification[:] = ratio
    nodes.alloc_milli_cpu[amp] = np.ceil(nodes.alloc_milli_cpu[amp] * ratio[amp]).astype(np.int64)
    pmask = rng.random(n_nodes) < policy_frac
    cpus = make_cpu_state(nodes, rng, cores=cores, two_numa=pmask)
    devs = make_devices(nodes, rng, rdma=True)
    numa = policy_numa_nodes(nodes, cpus, pmask, rng, cores, policy) if policy_frac > 0 else None
    pods = rdma_pods(gpu_pods(make_pods(n_pods, rng), rng), rng)
    pods = cpuset_pods(pods, rng, 0.4 / 0.6, exclude=pods.gpu_memory_ratio + pods.gpu_memory > 0)
    prof = koord_profile(**kw)
    prof.numa = NodeNUMAResourceArgs()
    prof.deviceshare = DeviceShareArgs()  # v1beta2 defaults: gpu-memory-ratio, rdma, fpga weight 1
    return Workload("C3", prof, nodes, pods, None, None, devs, cpus, numa)


def device_reservations(w: Workload, rng: np.random.Generator, frac: float = 0.4) -> Workload:
    """Reservations holding devices (deviceshare/reservation.go): frac of the reservations on nodes with device
    information and no NUMA topology policy reserve one or two GPUs (a whole or half instance each) and, on half of
    them, an RDMA device share; the reserve pod's allocation counts in the node's device used (nodeDeviceCache), and a
    reservation with assigned pods has them use part of its first minor (counted in used a second time, as the
    cache holds both the reserve pod and the assigned pods)."""
    rs, dv = w.reservations, w.devices
    rs.hold_devices()
    pol = (w.nodes.numa_flags >> abi.KS_NUMA_POLICY_SHIFT) & 3
    G = abi.KS_MAX_GPUS
    for r in range(rs.r):
        n = int(rs.node[r])
        if not (dv.flags[n] & abi.KS_DEV_PRESENT) or pol[n] != 0 or rng.random() >= frac:
            continue
        minors = [k for k in range(G) if dv.total_ratio[k, n] > 0]
        if not minors:
            continue
        pick = rng.choice(minors, min(len(minors), int(rng.integers(1, 3))), replace=False)
        for i, k in enumerate(sorted(int(x) for x in pick)):
            part = int(rng.choice([50, 100]))
            mem = part * int(dv.total_memory[k, n]) // 100
            for q, v in ((0, part), (1, mem), (2, part)):
                rs.dev_allocatable[r, abi.dev_word("gpu", k, q)] = v
            dv.used_core[k, n] += part
            dv.used_memory[k, n] += mem
            dv.used_ratio[k, n] += part
            if i == 0 and rs.assigned[r] > 0:
                use = part // 2
                for q, v in ((0, use), (1, use * int(dv.total_memory[k, n]) // 100), (2, use)):
                    rs.dev_allocated[r, abi.dev_word("gpu", k, q)] = v
                dv.used_core[k, n] += use
                dv.used_memory[k, n] += use * int(dv.total_memory[k, n]) // 100
                dv.used_ratio[k, n] += use
        rm = [j for j in range(abi.KS_MAX_RDMA) if dv.total_rdma[j, n] > 0]
        if rm and rng.random() < 0.5:
            j = int(rng.choice(rm))
            rs.dev_allocatable[r, abi.dev_word("rdma", j)] = 50
            dv.used_rdma[j, n] += 50
    return w


def c3_rsv(seed: int = SEED, n_nodes: int = 5000, n_pods: int = 10_000, rsv_per_node: float = 2.5,
           policy_frac: float = 0.5, policy: int = abi.KS_NUMA_POLICY_SINGLE_NUMA_NODE, dev_rsv_frac: float = 0.0,
           **kw) -> Workload:
    """The shipped koord-scheduler profile's plugin set (config/manager/scheduler-config.yaml:58-96: Reservation +
    NodeNUMAResource + DeviceShare next to Fit + LoadAware): C3's nodes (NUMA topology policies, cpuset pods, GPU /
    RDMA devices) with C4's reservations (~2.5 per node, 16 owner classes; their reserve pods in NodeInfo) and 60 % of
    the pods in an owner class.  Reservations hold no cpuset; with dev_rsv_frac > 0 that fraction of the
    reservations on non-policy device nodes holds GPUs / RDMA (device_reservations, deviceshare/reservation.go)."""
    w = c3(seed=seed, n_nodes=n_nodes, n_pods=n_pods, policy_frac=policy_frac, policy=policy, **kw)
    rng = np.random.Generator(np.random.PCG64(seed + 3))
    for col in ("req_milli_cpu", "req_memory", "nonzero_milli_cpu", "nonzero_memory"):
        setattr(w.nodes, col, getattr(w.nodes, col) // 2)
    w.reservations = make_reservations(w.nodes, int(n_nodes * rsv_per_node), rng)
    reservation_pods(w.pods, rng)
    w.profile.reservation_weight = 5000
    w.name = "C3-rsv"
    if dev_rsv_frac > 0:
        device_reservations(w, rng, dev_rsv_frac)
    return w


def c3_bind(seed: int = SEED, n_nodes: int = 2000, n_pods: int = 4000, label_frac: float = 0.4,
            required_frac: float = 0.4, policy_frac: float = 0.0, **kw) -> Workload:
    """C3 with node CPU bind policies and required pod bind policies (cpu_bind_policies); without NUMA topology
    policies by default, with policy_frac > 0 the labels and required policies meet NUMA-policy nodes too"""
    w = c3(seed=seed, n_nodes=n_nodes, n_pods=n_pods, policy_frac=policy_frac, **kw)
    rng = np.random.Generator(np.random.PCG64(seed + 1))
    cpu_bind_policies(w.nodes, w.pods, rng, label_frac, required_frac)
    w.name = "C3-bind"
    return w


def c4(seed: int = SEED, n_nodes: int = 20_000, n_reservations: int = 50_000, n_pods: int = 10_000, **kw) -> Workload:
    rng = np.random.Generator(np.random.PCG64(seed))
    nodes = make_nodes(n_nodes, rng)
    # other running pods use up to a quarter of the node; the reservations come on top
    for col in ("req_milli_cpu", "req_memory", "nonzero_milli_cpu", "nonzero_memory"):
        setattr(nodes, col, getattr(nodes, col) // 2)
    rs = make_reservations(nodes, n_reservations, rng)
    pods = reservation_pods(make_pods(n_pods, rng), rng)
    return Workload("C4", koord_profile(with_reservation=True, **kw), nodes, pods, None, rs)


def c5(seed: int = SEED, n_nodes: int = 100_000, n_pods: int = 1_000_000, **kw) -> Workload:
    rng = np.random.Generator(np.random.PCG64(seed))
    nodes = make_nodes(n_nodes, rng)
    pods = make_pods(n_pods, rng)
    return Workload("C5", koord_profile(**kw), nodes, pods, None)


def static_specs(n_nodes: int, n_pods: int, rng: np.random.Generator):
    """Node labels / taints and pod tolerations / node selectors / node affinity for the upstream TaintToleration and
    NodeAffinity plugins (static_plugins): 4 zones, 3 instance types, integer rack labels (Gt / Lt), GPU labels;
    NoSchedule / NoExecute / PreferNoSchedule taints on part of the nodes; pods with Equal / Exists / wildcard
    tolerations, nodeSelectors, required terms (In, NotIn, Gt, matchFields) and weighted preferred terms."""
    from .static_plugins import (NO_EXECUTE, NO_SCHEDULE, PREFER_NO_SCHEDULE, FIELD_NAME, HostPort, NodeSpec,
                                 PodAffinitySpec, Requirement, Taint, Term, Toleration)
    zones = ["zone-a", "zone-b", "zone-c", "zone-d"]
    types = ["m.large", "m.xlarge", "c.2xlarge"]
    nodes = []
    for i in range(n_nodes):
        lab = {"topology.kubernetes.io/zone": zones[rng.integers(0, 4)],
               "node.kubernetes.io/instance-type": types[rng.integers(0, 3)],
               "rack": str(int(rng.integers(0, 20)))}
        if rng.random() < 0.1:
            lab["accelerator"] = "mi355x"
        taints = []
        u = rng.random()
        if u < 0.08:
            taints.append(Taint("dedicated", "infra", NO_SCHEDULE))
        elif u < 0.12:
            taints.append(Taint("maintenance", "", NO_EXECUTE))
        if rng.random() < 0.25:
            taints.append(Taint("spot", "true", PREFER_NO_SCHEDULE))
        if rng.random() < 0.15:
            taints.append(Taint("noisy", "", PREFER_NO_SCHEDULE))
        used = []
        if rng.random() < 0.2:
            used.append(HostPort(80, "TCP", rng.choice(["0.0.0.0", "10.0.0.1", "10.0.0.2"])))
        if rng.random() < 0.1:
            used.append(HostPort(443))
        nodes.append(NodeSpec(f"node-{i}", lab, taints, used))
    pods = []
    for i in range(n_pods):
        tol = []
        if rng.random() < 0.3:
            tol.append(Toleration("dedicated", "Equal", "infra", NO_SCHEDULE))
        if rng.random() < 0.05:
            tol.append(Toleration("", "Exists"))  # tolerates everything
        if rng.random() < 0.4:
            tol.append(Toleration("spot", "Equal", "true", rng.choice(["", PREFER_NO_SCHEDULE])))
        if rng.random() < 0.1:
            tol.append(Toleration("noisy", "Exists", "", PREFER_NO_SCHEDULE))
        sel = {}
        if rng.random() < 0.15:
            sel["topology.kubernetes.io/zone"] = zones[rng.integers(0, 4)]
        req = None
        u = rng.random()
        if u < 0.15:
            z = tuple(sorted(rng.choice(zones, 2, replace=False)))
            req = [Term([Requirement("topology.kubernetes.io/zone", "In", z)]),
                   Term([Requirement("rack", "Gt", (str(int(rng.integers(8, 16))),))])]
        elif u < 0.2:
            req = [Term([Requirement("node.kubernetes.io/instance-type", "NotIn", (types[rng.integers(0, 3)],)),
                         Requirement("accelerator", "DoesNotExist")])]
        elif u < 0.21:
            req = [Term([Requirement(FIELD_NAME, "NotIn", (f"node-{int(rng.integers(0, min(n_nodes, 8)))}",), field=True)])]
        pref = []
        if rng.random() < 0.4:
            pref.append((int(rng.integers(1, 101)), Term([Requirement("topology.kubernetes.io/zone", "In",
                                                                      (zones[rng.integers(0, 4)],))])))
            if rng.random() < 0.5:
                pref.append((int(rng.integers(1, 101)), Term([Requirement("rack", "Lt", ("5",))])))
            if rng.random() < 0.3:
                pref.append((int(rng.integers(1, 101)), Term([Requirement("accelerator", "Exists")])))
        ports = []
        u = rng.random()
        if u < 0.1:
            ports.append(HostPort(80, "", ""))  # sanitized to TCP on 0.0.0.0
        elif u < 0.15:
            ports.append(HostPort(80, "TCP", rng.choice(["10.0.0.1", "10.0.0.3"])))
        elif u < 0.18:
            ports += [HostPort(443), HostPort(9100, "UDP")]
        pods.append(PodAffinitySpec(tol, sel, req, pref, ports))
    return nodes, pods


def with_static_plugins(w: Workload, seed: int = SEED + 7, weight_taint: int = 1, weight_affinity: int = 1) -> Workload:
    """The workload with upstream TaintToleration, NodeAffinity and NodePorts switched on and random specs compiled
    in."""
    from .static_plugins import compile_cluster
    rng = np.random.Generator(np.random.PCG64(seed))
    nspec, pspec = static_specs(w.nodes.n, w.pods.n, rng)
    compile_cluster(nspec, pspec, w.nodes, w.pods)
    w.profile.taint_toleration = True
    w.profile.taint_toleration_weight = weight_taint
    w.profile.node_affinity = True
    w.profile.node_affinity_weight = weight_affinity
    w.profile.node_ports = True
    w.specs = (nspec, pspec)
    return w


def topology_specs(n_nodes: int, n_pods: int, rng: np.random.Generator, per_node=(0, 6), n_zones: int = 8,
                   unzoned_frac: float = 0.1, spread_frac: float = 0.2, default_frac: float = 0.25,
                   anti_frac: float = 0.08, affinity_frac: float = 0.06, pref_frac: float = 0.12,
                   n_apps: int = 4, extra_keys=None, breadth_frac: float = 0.0, dup_frac: float = 0.0):
    """Zone labels (n_zones zones, unzoned_frac of the nodes without one), running pods (per_node) and pending pods
    for the upstream PodTopologySpread / InterPodAffinity plugins (topology_plugins): four apps in namespace
    "default" plus app-A pods in namespace "other"; pending pods with their own spread constraints (hostname / zone,
    DoNotSchedule / ScheduleAnyway, skews 1-3), the system default constraints (an owner selector), a required
    anti-affinity to app A per hostname, a required affinity to app D per zone, preferred (anti-)affinity terms;
    running pods that carry the same terms, a few terminating.  Returns (node_labels, existing, pending).

    Breadth (off by default): n_apps apps (one selector each), extra_keys {label key: values} further topology keys on
    the nodes (a node misses each with probability unzoned_frac), breadth_frac of the pending pods with many terms over
    every key (a spread constraint per key, anti-affinity / affinity / preferred terms on random keys and apps), and
    dup_frac of the pods (running and pending) carrying one scored term twice (a required affinity term and the same
    term preferred with weight 1, or one preferred term listed twice)."""
    from .topology_plugins import (HOSTNAME, SCHEDULE_ANYWAY, DO_NOT_SCHEDULE, ZONE, AffinityTerm, LabelSelector,
                                   SpreadConstraint, TopoPod)
    apps = ["A", "B", "C", "D"] + [f"app{k}" for k in range(4, n_apps)]
    sel = {a: LabelSelector((("app", a),)) for a in apps}
    anti_a = AffinityTerm(HOSTNAME, sel["A"])
    aff_d = AffinityTerm(ZONE, sel["D"])
    # (namespaceSelector {} = every namespace: app-C pods of "other" count too)
    pref_c = (20, AffinityTerm(HOSTNAME, sel["C"], namespace_selector=LabelSelector()))
    pref_b = (30, AffinityTerm(ZONE, sel["B"]))
    node_labels = []
    for i in range(n_nodes):
        lab = {}
        if rng.random() >= unzoned_frac:
            lab[ZONE] = f"zone-{int(rng.integers(0, n_zones))}"
        for key, nv in (extra_keys or {}).items():
            if rng.random() >= unzoned_frac:
                lab[key] = f"{key}-{int(rng.integers(0, nv))}"
        node_labels.append(lab)
    all_keys = [HOSTNAME, ZONE] + list(extra_keys or {})

    def rkey():
        return all_keys[int(rng.integers(0, len(all_keys)))]

    def rsel():
        return sel[apps[int(rng.integers(0, len(apps)))]]

    def dup(p):
        if rng.random() < 0.5:
            t = AffinityTerm(rkey(), rsel())
            p.affinity_required = p.affinity_required + [t]
            p.affinity_preferred = p.affinity_preferred + [(1, t)]
        else:
            t = (int(rng.integers(1, 50)), AffinityTerm(rkey(), rsel()))
            p.affinity_preferred = p.affinity_preferred + [t, t]

    def app_pod(ns="default"):
        a = apps[int(rng.integers(0, len(apps)))]
        return TopoPod(namespace=ns, labels={"app": a, "tier": str(rng.choice(["web", "batch"]))})

    existing = []
    for i in range(n_nodes):
        for _ in range(int(rng.integers(per_node[0], per_node[1] + 1))):
            p = app_pod("other" if rng.random() < 0.1 else "default")
            p.terminating = rng.random() < 0.03
            u = rng.random()
            if u < 0.05 and p.namespace == "default":
                p.anti_required = [anti_a]
            elif u < 0.1 and p.namespace == "default":
                p.affinity_required = [aff_d]
            elif u < 0.16 and p.namespace == "default":
                p.affinity_preferred = [pref_c]
            elif u < 0.2 and p.namespace == "default":
                p.anti_preferred = [pref_b]
            if dup_frac and p.namespace == "default" and rng.random() < dup_frac:
                dup(p)
            existing.append((i, p))
    pending = []
    for i in range(n_pods):
        p = app_pod("other" if rng.random() < 0.05 else "default")
        u = rng.random()
        own = LabelSelector((("app", p.labels["app"]),))
        if u < spread_frac:
            # (the API rejects two constraints with the same topologyKey and whenUnsatisfiable)
            for key in ([HOSTNAME, ZONE] if rng.random() < 0.4 else [[HOSTNAME, ZONE][int(rng.integers(0, 2))]]):
                when = DO_NOT_SCHEDULE if rng.random() < 0.5 else SCHEDULE_ANYWAY
                s = own if rng.random() < 0.9 else sel[apps[int(rng.integers(0, 4))]]
                p.spread.append(SpreadConstraint(int(rng.integers(1, 4)), key, when, s))
        elif u < spread_frac + default_frac:
            p.default_selector = own
        u = rng.random()
        if p.namespace == "default":
            if u < anti_frac:
                p.anti_required = [anti_a]
            elif u < anti_frac + affinity_frac:
                p.affinity_required = [aff_d]
            elif u < anti_frac + affinity_frac + pref_frac and not p.spread:
                if rng.random() < 0.5:
                    p.affinity_preferred = [pref_c]
                else:
                    p.anti_preferred = [pref_b]
        if breadth_frac and rng.random() < breadth_frac:
            # many terms over every key: a spread constraint per key (no soft duplicates: one per key), required
            # anti-affinity / affinity and preferred terms on random keys and apps
            p.default_selector = None
            p.spread = [SpreadConstraint(int(rng.integers(1, 5)), k,
                                         DO_NOT_SCHEDULE if rng.random() < 0.3 else SCHEDULE_ANYWAY, rsel())
                        for k in all_keys if rng.random() < 0.7]
            p.anti_required = p.anti_required + [AffinityTerm(rkey(), rsel()) for _ in range(int(rng.integers(0, 3)))]
            if rng.random() < 0.3:
                p.affinity_required = [AffinityTerm(rkey(), LabelSelector((("tier", "web"),)))]
            p.affinity_preferred = p.affinity_preferred + [(int(rng.integers(1, 100)), AffinityTerm(rkey(), rsel()))
                                                           for _ in range(int(rng.integers(0, 4)))]
            p.anti_preferred = p.anti_preferred + [(int(rng.integers(1, 100)), AffinityTerm(rkey(), rsel()))
                                                   for _ in range(int(rng.integers(0, 3)))]
        if dup_frac and p.namespace == "default" and rng.random() < dup_frac:
            dup(p)
        pending.append(p)
    return node_labels, existing, pending


# the namespaces' labels (the shim's namespace lister) for namespaceSelector terms
TOPO_NAMESPACE_LABELS = {"default": {"team": "a"}, "other": {"team": "b"}}


def with_topology(w: Workload, seed: int = SEED + 8, spread_weight: int = 2, affinity_weight: int = 1,
                  **kw) -> Workload:
    """The workload with upstream PodTopologySpread and InterPodAffinity switched on and topology_specs compiled into
    the node counters and pod query terms (topology_plugins.compile_topology); w.topo keeps the objects."""
    from .topology_plugins import compile_topology, install
    rng = np.random.Generator(np.random.PCG64(seed))
    node_labels, existing, pending = topology_specs(w.nodes.n, w.pods.n, rng, **kw)
    c = compile_topology(node_labels, existing, pending, namespace_labels=TOPO_NAMESPACE_LABELS)
    install(c, w.nodes, w.pods)
    w.topo_compiled = c
    w.profile.topology = True
    w.profile.topology_spread_weight = spread_weight
    w.profile.inter_pod_affinity_weight = affinity_weight
    w.topo = (node_labels, existing, pending)
    return w


def c3_full(seed: int = SEED, n_nodes: int = 5000, n_pods: int = 10_000, n_quotas: int = 32, **kw) -> Workload:
    """C3 (NUMA topology policies, cpuset pods, GPU / RDMA devices) under the rest of the shipped profile as well:
    ElasticQuota (32 leaf quotas) and the v1beta2 default plugins TaintToleration, NodeAffinity and NodePorts -- the
    combination whose commit kernel holds the NUMA slot cache, the device slot cache, the dictionary-plugin words and the
    quota rows in one workgroup's LDS."""
    w = c3(seed=seed, n_nodes=n_nodes, n_pods=n_pods, **kw)
    rng = np.random.Generator(np.random.PCG64(seed + 5))
    p = w.pods
    batch = (p.flags & abi.KS_POD_PROD) == 0
    p.quota[:] = rng.integers(0, n_quotas, p.n)
    p.quota_req[QDIM_CPU] = p.req_milli_cpu
    p.quota_req[QDIM_MEMORY] = p.req_memory
    p.quota_req[QDIM_BATCH_CPU] = p.req_scalar[SLOT_BATCH_CPU]
    p.quota_req[QDIM_BATCH_MEMORY] = p.req_scalar[SLOT_BATCH_MEMORY]
    p.quota_mask[:] = np.where(batch, (1 << QDIM_BATCH_CPU) | (1 << QDIM_BATCH_MEMORY),
                               (1 << QDIM_CPU) | (1 << QDIM_MEMORY)).astype(np.uint32)
    w.quotas = make_quotas(p, n_quotas, rng)
    w.profile.quota = ElasticQuotaArgs()
    w = with_static_plugins(w, seed=seed + 6)
    w.name = "C3-full"
    return w


def c2_default(seed: int = SEED, n_nodes: int = 5000, n_pods: int = 10000, **kw) -> Workload:
    """C2 under the v1beta2 default profile's upstream plugins as well: NodeResourcesBalancedAllocation,
    TaintToleration and NodeAffinity (weight 1 each) and NodePorts next to Fit + LoadAware + ElasticQuota."""
    from .config import NodeResourcesBalancedAllocationArgs
    w = c2(seed=seed, n_nodes=n_nodes, n_pods=n_pods, **kw)
    w.profile.balanced = NodeResourcesBalancedAllocationArgs()
    w = with_static_plugins(w)
    w.name = "C2-static"
    return w


# ---- preemption (ks_preempt) ----

PRIORITIES = np.array([0, 100, 1000, 3000, 5000, 8000], np.int32)


def make_node_pods(nodes: NodeTable, rng: np.random.Generator, n_quotas: int, per_node=(4, 40), n_pdb: int = 12,
                   pdb_frac: float = 0.15, nonpreemptible_frac: float = 0.08, terminating_frac: float = 0.02,
                   out_of_quota_frac: float = 0.03, multi_pdb_frac: float = 0.0):
    """Running pods on every node (make_pods' request distribution), with priorities, distinct start times, quotas,
    PDBs and flags.  The nodes' NodeInfo columns (Requested, NonZeroRequested, pod count) are set to the sums over their
    pods, so the table is the NodeInfo.Pods the columns were built from.  Returns (NodePodTable, per-quota used [dim][q])
    -- the quotas' used of their in-quota pods (QuotaInfo.CalculateInfo.Used)."""
    from .cluster import NodePodTable

    counts = rng.integers(per_node[0], per_node[1] + 1, nodes.n)
    counts = np.minimum(counts, nodes.allowed_pods - 1)
    m = int(counts.sum())
    src = make_pods(m, rng, n_quotas)
    t = NodePodTable(m, n_pdb)
    t.node[:] = np.repeat(np.arange(nodes.n, dtype=np.int32), counts)
    t.priority[:] = rng.choice(PRIORITIES, m)
    t.start_time[:] = rng.permutation(m).astype(np.int64) * 1_000_000 + 1_700_000_000_000_000_000
    fl = np.full(m, abi.KS_NPOD_IN_QUOTA, np.uint32)
    fl[rng.random(m) < nonpreemptible_frac] |= abi.KS_NPOD_NONPREEMPTIBLE
    fl[rng.random(m) < terminating_frac] |= abi.KS_NPOD_TERMINATING
    fl[rng.random(m) < out_of_quota_frac] &= ~np.uint32(abi.KS_NPOD_IN_QUOTA)
    t.flags[:] = fl
    t.quota[:] = src.quota if n_quotas else -1
    t.pdb[:] = np.where(rng.random(m) < pdb_frac, rng.integers(0, max(n_pdb, 1), m), -1) if n_pdb else -1
    t.pdb_allowed[:] = rng.integers(0, 4, n_pdb)
    if multi_pdb_frac > 0 and n_pdb > 1:
        # pods matching several budgets (filterPodsWithPDBViolation decrements each): up to 1 + KS_NPOD_MORE_PDBS distinct
        for i in np.nonzero((t.pdb >= 0) & (rng.random(m) < multi_pdb_frac))[0]:
            k = int(rng.integers(1, min(n_pdb, 1 + abi.KS_NPOD_MORE_PDBS)))
            extra = rng.permutation(np.setdiff1d(np.arange(n_pdb), [t.pdb[i]]))[:k]
            t.pdb_more[:k, i] = extra
    t.req[0] = src.req_milli_cpu
    t.req[1] = src.req_memory
    t.req[2] = 0
    t.req[3 + SLOT_BATCH_CPU] = src.req_scalar[SLOT_BATCH_CPU]
    t.req[3 + SLOT_BATCH_MEMORY] = src.req_scalar[SLOT_BATCH_MEMORY]
    t.quota_req[:] = src.quota_req
    # NodeInfo = the sum over the node's pods
    nodes.req_milli_cpu[:] = np.bincount(t.node, weights=t.req[0], minlength=nodes.n).astype(np.int64)
    nodes.req_memory[:] = np.bincount(t.node, weights=t.req[1], minlength=nodes.n).astype(np.int64)
    nodes.req_ephemeral[:] = 0
    for k in (SLOT_BATCH_CPU, SLOT_BATCH_MEMORY):
        nodes.req_scalar[k] = np.bincount(t.node, weights=t.req[3 + k], minlength=nodes.n).astype(np.int64)
    nodes.nonzero_milli_cpu[:] = np.bincount(t.node, weights=src.nonzero_milli_cpu, minlength=nodes.n).astype(np.int64)
    nodes.nonzero_memory[:] = np.bincount(t.node, weights=src.nonzero_memory, minlength=nodes.n).astype(np.int64)
    nodes.pod_count[:] = counts.astype(np.int32)
    used = np.zeros((abi.KS_QUOTA_DIMS, max(n_quotas, 1)), np.int64)
    inq = ((t.flags & abi.KS_NPOD_IN_QUOTA) != 0) & (t.quota >= 0)
    for d in range(abi.KS_QUOTA_DIMS):
        used[d] = np.bincount(t.quota[inq], weights=t.quota_req[d][inq].astype(np.float64),
                              minlength=max(n_quotas, 1)).astype(np.int64)
    return t, used[:, :n_quotas]


@dataclass
class PreemptWorkload:
    name: str
    profile: SchedulerProfile
    nodes: NodeTable
    quotas: QuotaTable
    node_pods: "NodePodTable"
    preemptors: PodTable
    priority: np.ndarray  # [preemptors.n]

    @property
    def cfg(self) -> abi.KsConfig:
        return self.profile.to_ks_config()


def c2_preempt(seed: int = SEED, n_nodes: int = 5000, n_preemptors: int = 64, n_quotas: int = 32, per_node=(4, 40),
               headroom=(0.97, 1.03), tight_nodes: float = 0.6, **kw) -> PreemptWorkload:
    """C2's cluster and profile (Fit + LoadAware + ElasticQuota) with NodeInfo.Pods on every node and quotas at their
    runtime limits, so a new pod is rejected by the quota PreFilter (and every node's status is Unschedulable) or
    finds no room: the ElasticQuota PostFilter then looks for same-quota lower-priority victims on every node."""
    rng = np.random.Generator(np.random.PCG64(seed))
    nodes = make_nodes(n_nodes, rng)
    t, used = make_node_pods(nodes, rng, n_quotas, per_node=per_node)
    # a share of the nodes filled up (Requested close to Allocatable): preemption must free room there
    tight = rng.random(n_nodes) < tight_nodes
    nodes.alloc_milli_cpu[tight] = np.maximum(nodes.req_milli_cpu[tight] + rng.integers(0, 4000, int(tight.sum())) // 250 * 250,
                                              1000)
    q = QuotaTable(n_quotas)
    q.limit_mask[:] = (1 << QDIM_CPU) | (1 << QDIM_MEMORY) | (1 << QDIM_BATCH_CPU) | (1 << QDIM_BATCH_MEMORY)
    q.used[:] = used
    q.limit[:] = (used * rng.uniform(headroom[0], headroom[1], (abi.KS_QUOTA_DIMS, n_quotas))).astype(np.int64)
    q.min_mask[:] = q.limit_mask
    q.min[:] = q.limit // 2
    pre = make_pods(n_preemptors, rng, n_quotas)
    prio = rng.choice(np.array([1000, 3000, 5000, 9000], np.int32), n_preemptors)
    return PreemptWorkload("C2-preempt", koord_profile(with_quota=True, **kw), nodes, q, t, pre, prio)
