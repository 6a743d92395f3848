"""ctypes mirror of include/koordgpu.h (the C ABI of libkoordgpu.so).

Plain data layout only — every struct here is field-for-field identical to the
header, so the same SoA buffers can be handed to the HIP library and to the CPU
oracle.  Keep in sync with include/koordgpu.h (tests/test_abi.py checks sizes).
"""
from __future__ import annotations

import ctypes as C

KS_ABI_VERSION = 10
KS_MAX_SCALARS = 4
KS_QUOTA_DIMS = 8
KS_MAX_GPUS = 8
KS_MAX_RDMA = 8
KS_MAX_PCIE = 8
KS_DEV_WORDS = 3 * 8 + 8  # ks_reservation_cols.dev_*: GPU minor k core / memory / ratio at k, 8 + k, 16 + k; RDMA j at 24 + j


def dev_word(kind: str, minor: int, q: int = 0) -> int:
    """word of the KS_DEV_WORDS layout: kind "gpu" (q = 0 core, 1 memory, 2 ratio) or "rdma" """
    return q * KS_MAX_GPUS + minor if kind == "gpu" else 3 * KS_MAX_GPUS + minor
KS_PCIE_NONE = 0xFF
KS_JOINT_NONE = 0
KS_POD_UNMODELLED = 0x100
KS_DEV_UNMODELLED = 0x2
KS_NUMA_MAX_REF_COUNT = 0x200
KS_JOINT_GPU_RDMA = 1
KS_JOINT_GPU_RDMA_SAME_PCIE = 2
KS_MAX_CPUS = 256
KS_CPU_WORDS = 4
KS_MAX_NUMA = 8
KS_RSV_DIMS = 3 + KS_MAX_SCALARS
KS_RSV_CLASSES = 64

KS_OK = 0
KS_EINVAL = -1
KS_EHIP = -2
KS_ESTATE = -3
KS_EUNSUPPORTED = -4
KS_ENOMEM = -5

KS_LEAST_ALLOCATED = 0
KS_MOST_ALLOCATED = 1

KS_LA_HAS_METRIC = 0x01
KS_LA_EXPIRED = 0x02
KS_LA_HAS_STATUS_METRIC = 0x04
KS_LA_FILTER_USAGE_PRESENT = 0x08
KS_LA_AGGREGATED_FILTER = 0x10
KS_LA_NODE_THR_NONEMPTY = 0x20
KS_LA_PROD_THR_NONEMPTY = 0x40
KS_LA_HAS_PODS_METRIC = 0x80

KS_POD_PROD = 0x01
KS_POD_DAEMONSET = 0x02
KS_POD_NONPREEMPTIBLE = 0x04
KS_POD_SCALAR_KEYS = 0x08
KS_POD_RSV_AFFINITY = 0x10
KS_POD_CPU_BIND = 0x20
KS_POD_GPU_CORE = 0x40
KS_POD_GPU_MEMORY = 0x80
KS_DEV_PRESENT = 0x1

KS_NUMA_INVALID_RATIO = 0x1
KS_NUMA_CPU_BIND_POLICY = 0x2
KS_NUMA_TOPOLOGY_POLICY = 0x4
KS_NUMA_ALLOC_LEAST = 0x8
KS_NUMA_ALLOC_MOST = 0x10
KS_NUMA_POLICY_SHIFT = 5
KS_NUMA_POLICY_NONE = 0
KS_NUMA_POLICY_BEST_EFFORT = 1
KS_NUMA_POLICY_RESTRICTED = 2
KS_NUMA_POLICY_SINGLE_NUMA_NODE = 3
KS_NUMA_CPU_BIND_SHIFT = 7
KS_NODE_CPU_BIND_NONE = 0
KS_NODE_CPU_BIND_FULL_PCPUS_ONLY = 1
KS_NODE_CPU_BIND_SPREAD_BY_PCPUS = 2

KS_CPU_BIND_FULL_PCPUS = 1
KS_CPU_BIND_SPREAD_BY_PCPUS = 2
KS_CPU_BIND_POLICY_MASK = 0x3
KS_CPU_BIND_REQUIRED = 0x10
KS_CPU_EXCL_SHIFT = 2
KS_CPU_EXCL_NONE = 0
KS_CPU_EXCL_PCPU_LEVEL = 1
KS_CPU_EXCL_NUMA_NODE_LEVEL = 2

KS_R_FIT_PODS = 0x001
KS_R_FIT_CPU = 0x002
KS_R_FIT_MEMORY = 0x004
KS_R_FIT_EPHEMERAL = 0x008
KS_R_FIT_SCALAR = 0x010
KS_R_LA_CPU = 0x020
KS_R_LA_MEMORY = 0x040
KS_R_LA_AGGREGATED = 0x080
KS_R_LA_PROD = 0x100
KS_R_RSV_AFFINITY = 0x200
KS_R_RSV_NO_FIT = 0x400
KS_R_NUMA_AMPLIFIED_CPU = 0x800
KS_R_NUMA_INVALID_RATIO = 0x1000
KS_R_DEV_INSUFFICIENT = 0x2000
KS_R_DEV_NO_GPU = 0x4000
KS_R_DEV_NO_RDMA = 0x80000
KS_R_DEV_JOINT = 0x100000
KS_R_NUMA_INVALID_TOPOLOGY = 0x8000
KS_R_NUMA_AFFINITY = 0x10000
KS_R_NUMA_INSUFFICIENT = 0x20000
KS_R_NUMA_MISSING = 0x40000
KS_R_NUMA_CPUSET = 0x200000
KS_R_NUMA_INVALID_CPUS = 0x400000
KS_R_NUMA_BIND_CONFLICT = 0x800000
KS_R_NUMA_SMT = 0x1000000
KS_R_TAINT = 0x2000000
KS_R_NODE_AFFINITY = 0x4000000
KS_R_NODE_PORTS = 0x8000000
KS_R_TOPOLOGY_SPREAD = 0x10000000
KS_R_POD_AFFINITY = 0x20000000
KS_R_POD_ANTI_AFFINITY = 0x40000000
KS_R_EXISTING_ANTI_AFFINITY = 0x80000000

KS_S_SCHEDULED = 0x0
KS_S_QUOTA = 0x1
KS_S_QUOTA_NONPREEMPTIBLE = 0x2
KS_S_QUOTA_PARENT = 0x4
KS_S_UNSCHEDULABLE = 0x8
KS_S_RESERVE_FAILED = 0x10

KS_SCORE_FIT = 0
KS_SCORE_LOADAWARE = 1
KS_SCORE_RESERVATION = 2
KS_SCORE_NUMA = 3
KS_SCORE_DEVICESHARE = 4
KS_SCORE_BALANCED = 5
KS_SCORE_TAINT = 6
KS_SCORE_NODE_AFFINITY = 7
KS_SCORE_TOPOLOGY_SPREAD = 8
KS_SCORE_POD_AFFINITY = 9
KS_NUM_SCORE_PLUGINS = 10
KS_AFFINITY_TERMS = 4
KS_LABEL_NEVER = 1 << 63
KS_BAL_CPU = 0x1
KS_BAL_MEMORY = 0x2
KS_TOPO_MAX_KEYS = 256
KS_TOPO_MAX_PROPS = 65536
KS_TOPO_MAX_TERMS = 64
KS_TOPO_DYN = 0x1
KS_TOPO_SELF_AFFINITY = 0x2
KS_TOPO_SOFT_ALL_KEYS = 0x4
KS_TOPO_K_SPREAD_HARD = 1
KS_TOPO_K_SPREAD_SOFT = 2
KS_TOPO_K_AFFINITY = 3
KS_TOPO_K_ANTI = 4
KS_TOPO_K_EXISTING_ANTI = 5
KS_TOPO_K_SCORE = 6
KS_TOPO_T_SELF = 0x1

KS_RSV_UNSCHEDULABLE = 0x1
KS_RSV_ALLOCATE_ONCE = 0x2
KS_RSV_POLICY_DEFAULT = 0
KS_RSV_POLICY_ALIGNED = 1
KS_RSV_POLICY_RESTRICTED = 2

P64 = C.POINTER(C.c_int64)
P32 = C.POINTER(C.c_int32)
PU32 = C.POINTER(C.c_uint32)


class KsFitArgs(C.Structure):
    _fields_ = [
        ("enable_filter", C.c_int32),
        ("enable_score", C.c_int32),
        ("strategy", C.c_int32),
        ("_pad0", C.c_int32),
        ("weight_cpu", C.c_int64),
        ("weight_memory", C.c_int64),
        ("weight_ephemeral", C.c_int64),
        ("weight_scalar", C.c_int64 * KS_MAX_SCALARS),
        ("plugin_weight", C.c_int64),
    ]


class KsLoadAwareArgs(C.Structure):
    _fields_ = [
        ("enable_filter", C.c_int32),
        ("enable_score", C.c_int32),
        ("filter_expired_node_metrics", C.c_int32),
        ("score_according_prod_usage", C.c_int32),
        ("weight_cpu", C.c_int64),
        ("weight_memory", C.c_int64),
        ("scaling_cpu", C.c_int64),
        ("scaling_memory", C.c_int64),
        ("plugin_weight", C.c_int64),
    ]


class KsQuotaArgs(C.Structure):
    _fields_ = [("enable", C.c_int32), ("enable_check_parent_quota", C.c_int32)]


class KsReservationArgs(C.Structure):
    _fields_ = [("enable", C.c_int32), ("_pad0", C.c_int32), ("plugin_weight", C.c_int64)]


class KsNumaArgs(C.Structure):
    _fields_ = [("enable", C.c_int32), ("strategy", C.c_int32), ("weight_cpu", C.c_int64),
                ("weight_memory", C.c_int64), ("plugin_weight", C.c_int64), ("numa_scoring_strategy", C.c_int32),
                ("_pad0", C.c_int32)]


class KsDeviceShareArgs(C.Structure):
    _fields_ = [("enable", C.c_int32), ("strategy", C.c_int32), ("weight_gpu_core", C.c_int64),
                ("weight_gpu_memory", C.c_int64), ("weight_gpu_memory_ratio", C.c_int64), ("plugin_weight", C.c_int64),
                ("weight_rdma", C.c_int64)]


class KsBalancedArgs(C.Structure):
    _fields_ = [("enable", C.c_int32), ("resources", C.c_int32), ("plugin_weight", C.c_int64)]


class KsStaticPluginArgs(C.Structure):
    _fields_ = [("enable_filter", C.c_int32), ("enable_score", C.c_int32), ("plugin_weight", C.c_int64)]


class KsTopologyArgs(C.Structure):
    _fields_ = [("enable", C.c_int32), ("_pad0", C.c_int32), ("spread_weight", C.c_int64),
                ("affinity_weight", C.c_int64)]


class KsConfig(C.Structure):
    _fields_ = [
        ("abi_version", C.c_int32),
        ("device", C.c_int32),
        ("fit", KsFitArgs),
        ("loadaware", KsLoadAwareArgs),
        ("quota", KsQuotaArgs),
        ("batch_pods", C.c_int32),
        ("candidates", C.c_int32),
        ("profile", C.c_int32),
        ("_pad1", C.c_int32),
        ("reservation", KsReservationArgs),
        ("numa", KsNumaArgs),
        ("deviceshare", KsDeviceShareArgs),
        ("balanced", KsBalancedArgs),
        ("taint", KsStaticPluginArgs),
        ("affinity", KsStaticPluginArgs),
        ("nodeports", KsStaticPluginArgs),
        ("topology", KsTopologyArgs),
    ]


NODE_COLS = [
    ("alloc_milli_cpu", P64),
    ("alloc_memory", P64),
    ("alloc_ephemeral", P64),
    ("allowed_pods", P32),
    ("req_milli_cpu", P64),
    ("req_memory", P64),
    ("req_ephemeral", P64),
    ("pod_count", P32),
    ("nonzero_milli_cpu", P64),
    ("nonzero_memory", P64),
    ("alloc_scalar", P64 * KS_MAX_SCALARS),
    ("req_scalar", P64 * KS_MAX_SCALARS),
    ("la_flags", PU32),
    ("la_alloc_milli_cpu", P64),
    ("la_alloc_memory", P64),
    ("la_term_milli_cpu", P64),
    ("la_term_memory", P64),
    ("la_prod_term_milli_cpu", P64),
    ("la_prod_term_memory", P64),
    ("la_thr_cpu", P32),
    ("la_thr_memory", P32),
    ("la_prod_thr_cpu", P32),
    ("la_prod_thr_memory", P32),
    ("la_total_milli_cpu", P64),
    ("la_total_milli_memory", P64),
    ("la_usage_milli_cpu", P64),
    ("la_usage_milli_memory", P64),
    ("la_prod_usage_milli_cpu", P64),
    ("la_prod_usage_milli_memory", P64),
    ("numa_cpu_amplification", C.POINTER(C.c_double)),
    ("numa_cpuset_cpus", P32),
    ("numa_flags", PU32),
    ("taints_hard", C.POINTER(C.c_uint64)),
    ("taints_soft", C.POINTER(C.c_uint64)),
    ("labels", C.POINTER(C.c_uint64)),
    ("host_ports", C.POINTER(C.c_uint64)),
    ("topo_nkeys", C.c_int32),
    ("topo_ndomains", C.c_int32),
    ("topo_nprops", C.c_int32),
    ("_topo_pad", C.c_int32),
    ("topo_domain", P32),
    ("topo_count", P32),
]


class KsNodeCols(C.Structure):
    _fields_ = NODE_COLS


POD_COLS = [
    ("req_milli_cpu", P64),
    ("req_memory", P64),
    ("req_ephemeral", P64),
    ("req_scalar", P64 * KS_MAX_SCALARS),
    ("nonzero_milli_cpu", P64),
    ("nonzero_memory", P64),
    ("flags", PU32),
    ("la_req_cpu", P64),
    ("la_lim_cpu", P64),
    ("la_dflt_cpu", P64),
    ("la_req_memory", P64),
    ("la_lim_memory", P64),
    ("la_dflt_memory", P64),
    ("quota", P32),
    ("quota_mask", PU32),
    ("quota_req", P64 * KS_QUOTA_DIMS),
    ("rsv_class", P32),
    ("gpu_core", P64),
    ("gpu_memory", P64),
    ("gpu_memory_ratio", P64),
    ("cpu_bind", PU32),
    ("rdma", P64),
    ("joint", C.POINTER(C.c_uint8)),
    ("tolerated", C.POINTER(C.c_uint64)),
    ("affinity_required_n", P32),
    ("affinity_required", C.POINTER(C.c_uint64) * KS_AFFINITY_TERMS),
    ("affinity_preferred", C.POINTER(C.c_uint64) * KS_AFFINITY_TERMS),
    ("affinity_weight", P32 * KS_AFFINITY_TERMS),
    ("host_ports", C.POINTER(C.c_uint64)),
    ("host_ports_conflict", C.POINTER(C.c_uint64)),
    ("topo_flags", PU32),
    ("topo_prop_beg", P32),
    ("topo_props", P32),
    ("topo_term_beg", P32),
    ("topo_terms", C.POINTER(C.c_uint64)),
]


class KsPodCols(C.Structure):
    _fields_ = POD_COLS


QUOTA_COLS = [
    ("parent", P32),
    ("limit_mask", PU32),
    ("limit", P64 * KS_QUOTA_DIMS),
    ("used", P64 * KS_QUOTA_DIMS),
    ("min_mask", PU32),
    ("min", P64 * KS_QUOTA_DIMS),
    ("nonpreemptible_used", P64 * KS_QUOTA_DIMS),
]


class KsQuotaCols(C.Structure):
    _fields_ = QUOTA_COLS


class KsQuotaTree(C.Structure):
    _fields_ = [
        ("parent", P32),
        ("allow_lent", C.POINTER(C.c_uint8)),
        ("max_mask", PU32),
        ("max", P64 * KS_QUOTA_DIMS),
        ("min", P64 * KS_QUOTA_DIMS),
        ("shared_weight", P64 * KS_QUOTA_DIMS),
        ("guaranteed", P64 * KS_QUOTA_DIMS),
        ("self_request", P64 * KS_QUOTA_DIMS),
        ("cluster_total", C.c_int64 * KS_QUOTA_DIMS),
    ]


class KsReservationCols(C.Structure):
    _fields_ = [
        ("node", P32),
        ("owner_classes", C.POINTER(C.c_uint64)),
        ("flags", PU32),
        ("policy", PU32),
        ("order", P64),
        ("key_mask", PU32),
        ("allocatable", P64 * KS_RSV_DIMS),
        ("allocated", P64 * KS_RSV_DIMS),
        ("assigned", P32),
        ("reserve_nonzero_milli_cpu", P64),
        ("reserve_nonzero_memory", P64),
        ("dev_allocatable", P64),
        ("dev_allocated", P64),
    ]


class KsDeviceCols(C.Structure):
    _fields_ = [
        ("flags", PU32),
        ("total_core", P64 * KS_MAX_GPUS),
        ("total_memory", P64 * KS_MAX_GPUS),
        ("total_ratio", P64 * KS_MAX_GPUS),
        ("used_core", P64 * KS_MAX_GPUS),
        ("used_memory", P64 * KS_MAX_GPUS),
        ("used_ratio", P64 * KS_MAX_GPUS),
        ("total_rdma", P64 * KS_MAX_RDMA),
        ("used_rdma", P64 * KS_MAX_RDMA),
        ("gpu_pcie", C.POINTER(C.c_uint8) * KS_MAX_GPUS),
        ("rdma_pcie", C.POINTER(C.c_uint8) * KS_MAX_RDMA),
        ("pcie_numa", C.POINTER(C.c_uint8) * KS_MAX_PCIE),
        ("pcie_socket", C.POINTER(C.c_uint8) * KS_MAX_PCIE),
    ]


class KsCpuTopology(C.Structure):
    _fields_ = [("ncpus", C.c_int32), ("core", C.c_int32 * KS_MAX_CPUS), ("numa_node", C.c_int32 * KS_MAX_CPUS),
                ("socket", C.c_int32 * KS_MAX_CPUS)]


PU64 = C.POINTER(C.c_uint64)


class KsCpuStateCols(C.Structure):
    _fields_ = [("topology", P32), ("allocated", PU64), ("excl_pcpu", PU64), ("excl_numa", PU64),
                ("reserved", PU64)]


class KsNumaNodeCols(C.Structure):
    _fields_ = [("count", P32), ("alloc_cpu", P64), ("alloc_memory", P64), ("used_cpu", P64), ("used_memory", P64),
                ("used_present", C.POINTER(C.c_uint8)), ("cpuset_cpus", P32)]


class KsResult(C.Structure):
    _fields_ = [("node", C.c_int32), ("status", C.c_uint32), ("score", C.c_int64), ("reservation", C.c_int32),
                ("gpu_minors", C.c_uint32), ("rdma_minors", C.c_uint32), ("_pad0", C.c_int32)]


RESULT_DTYPE_FIELDS = [("node", "<i4"), ("status", "<u4"), ("score", "<i8"), ("reservation", "<i4"),
                       ("gpu_minors", "<u4"), ("rdma_minors", "<u4"), ("_pad0", "<i4")]


NODE_STATE_COLS = [
    ("req_milli_cpu", P64),
    ("req_memory", P64),
    ("req_ephemeral", P64),
    ("pod_count", P32),
    ("nonzero_milli_cpu", P64),
    ("nonzero_memory", P64),
    ("req_scalar", P64 * KS_MAX_SCALARS),
    ("la_term_milli_cpu", P64),
    ("la_term_memory", P64),
    ("la_prod_term_milli_cpu", P64),
    ("la_prod_term_memory", P64),
    ("host_ports", C.POINTER(C.c_uint64)),
    ("topo_count", P32),
]


class KsNodeState(C.Structure):
    _fields_ = NODE_STATE_COLS


class KsStats(C.Structure):
    _fields_ = [
        ("passes", C.c_int64),
        ("cut_passes", C.c_int64),
        ("rescans", C.c_int64),
        ("sweep_ms", C.c_double),
        ("select_ms", C.c_double),
        ("commit_ms", C.c_double),
        ("total_ms", C.c_double),
        ("sweep_launches", C.c_int64),
        ("sweep_bytes", C.c_int64),
        ("slot_misses", C.c_int64),
        ("diag", C.c_int64 * 8),
        ("bubble_passes", C.c_int64),
        ("fixup_ms", C.c_double),
        ("pipelined", C.c_int64),
        ("pre_reserves", C.c_int64),
        ("commit_lds_bytes", C.c_int64),
        ("commit_helpers", C.c_int64),
    ]


# every symbol include/koordgpu.h declares (checked by tests/test_abi.py)
EXPORTED_SYMBOLS = [
    "ks_abi_layout",
    "ks_create",
    "ks_destroy",
    "ks_last_error",
    "ks_load_nodes",
    "ks_update_nodes",
    "ks_load_quotas",
    "ks_load_devices",
    "ks_read_devices",
    "ks_read_devices_rdma",
    "ks_load_cpu_state",
    "ks_read_cpu_state",
    "ks_fetch_cpusets",
    "ks_load_numa_nodes",
    "ks_read_numa_nodes",
    "ks_load_reservations",
    "ks_read_reservations",
    "ks_read_reservation_devices",
    "ks_refresh_quota_runtime",
    "ks_schedule",
    "ks_stage_pods",
    "ks_schedule_staged",
    "ks_fetch_results",
    "ks_checkpoint",
    "ks_restore",
    "ks_eval_pod_debug",
    "ks_eval_pod",
    "ks_assume",
    "ks_unreserve",
    "ks_fetch_numa_alloc",
    "ks_update_devices",
    "ks_update_cpu_state",
    "ks_update_quotas",
    "ks_update_reservation_usage",
    "ks_add_reservations",
    "ks_update_numa_nodes",
    "ks_delete_reservations",
    "ks_read_nodes",
    "ks_read_quota_used",
    "ks_get_stats",
    "ks_set_profile",
    "ks_set_pipeline",
    "ks_shard_unique_id",
    "ks_shard_init",
    "ks_shard_init_loopback",
    "ks_load_node_pods",
    "ks_preempt",
]
KS_SHARD_ID_BYTES = 128

# ---- preemption (ElasticQuota PostFilter) ----
KS_NPOD_NONPREEMPTIBLE = 0x1
KS_NPOD_IN_QUOTA = 0x2
KS_NPOD_TERMINATING = 0x4
KS_P_NOMINATED = 0
KS_P_NOT_ELIGIBLE = 1
KS_P_NO_CANDIDATE = 2
KS_P_ERROR = 3
KS_PN_CANDIDATE = 0
KS_PN_UNRESOLVABLE = 1
KS_PN_NO_VICTIMS = 2
KS_PN_FILTER = 3
KS_PN_ERROR = 4
KS_PREEMPT_NEVER = 0x1
KS_NPOD_MORE_PDBS = 3


class KsNodePodCols(C.Structure):
    _fields_ = [
        ("node", P32),
        ("priority", P32),
        ("start_time", P64),
        ("flags", PU32),
        ("quota", P32),
        ("pdb", P32),
        ("req_milli_cpu", P64),
        ("req_memory", P64),
        ("req_ephemeral", P64),
        ("req_scalar", P64 * KS_MAX_SCALARS),
        ("quota_req", P64 * KS_QUOTA_DIMS),
        ("pdb_more", P32 * KS_NPOD_MORE_PDBS),
    ]


class KsPreemptResult(C.Structure):
    _fields_ = [
        ("node", C.c_int32),
        ("status", C.c_uint32),
        ("num_victims", C.c_int32),
        ("num_pdb_violations", C.c_int32),
        ("candidates", C.c_int32),
        ("potential_nodes", C.c_int32),
    ]
KS_ABI_LAYOUT_WORDS = 17
