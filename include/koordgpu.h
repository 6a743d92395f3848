/*
 * koordgpu.h — C ABI of the MI355X scheduling evaluator (libkoordgpu.so).
 *
 * This is the drop-in boundary for koord-scheduler's per-pod Filter/Score
 * sweep.  A Go cgo shim or any C/C++ host calls it.
 * Plain C types only: caller-owned flat arrays, int status codes, no torch or
 * HIP types in any signature.
 *
 * What each entry point replaces in the reference (xulinfei1996/koordinator,
 * paths relative to its root; "upstream" = k8s.io/kubernetes v1.24.15):
 *
 *   ks_create          plugin construction through PluginFactoryProxy
 *                      (pkg/scheduler/frameworkext/framework_extender_factory.go:209-221)
 *                      for LoadAwareScheduling (pkg/scheduler/plugins/loadaware/load_aware.go:76-110),
 *                      NodeResourcesFit (upstream noderesources/fit.go NewFit) and
 *                      ElasticQuota (pkg/scheduler/plugins/elasticquota/plugin.go:102);
 *                      args mirror pkg/scheduler/apis/config/types.go:30-62.
 *   ks_load_nodes      scheduler cache snapshot (upstream Cache.UpdateSnapshot) + the
 *   ks_update_nodes    LoadAware NodeMetric lister / podAssignCache state
 *                      (load_aware.go:133,278; pod_assign_cache.go:53-117).
 *   ks_load_quotas     GroupQuotaManager QuotaInfo used/runtime
 *                      (pkg/scheduler/plugins/elasticquota/core/group_quota_manager.go:259-326).
 *   ks_schedule        the per-pod cycle (upstream schedule_one.go schedulePod:
 *                      PreFilter -> findNodesThatPassFilters -> prioritizeNodes -> selectHost)
 *                      followed by Reserve (framework_extender.go:457; load_aware.go:260;
 *                      elasticquota/plugin.go:323), for a batch of pods in queue order,
 *                      with exact one-pod-at-a-time semantics.
 *   ks_eval_pod        one pod's Filter + Score over every node without Reserve
 *   ks_assume          Reserve of one pod on the node the framework chose; ks_unreserve its Unreserve
 *                      (framework_extender.go:204 RunFilterPluginsWithNominatedPods,
 *                      :237 RunScorePlugins) — the parity/debug entry point.
 *
 * Semantics pinned by this ABI: percentageOfNodesToScore=100 (every node is
 * evaluated), and selectHost ties are broken by the LOWEST node index (the
 * reference picks uniformly at random among ties).
 *
 * Quantities are int64 after the host's resource.Quantity conversion exactly as
 * the reference does it: cpu -> MilliValue(), everything else -> Value()
 * (pkg/scheduler/plugins/loadaware/helper.go:146-151).  Values must be in
 * [0, 2^56); larger values are rejected with KS_EINVAL.
 */
#ifndef KOORDGPU_H
#define KOORDGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KS_ABI_VERSION 10

#define KS_MAX_SCALARS 4 /* scalar (extended) resource slots, e.g. kubernetes.io/batch-cpu */
#define KS_QUOTA_DIMS 8  /* resource dimensions tracked by ElasticQuota admission */
#define KS_SHARD_ID_BYTES 128 /* opaque RCCL unique id (ks_shard_unique_id) */
#define KS_RSV_DIMS (3 + KS_MAX_SCALARS) /* reservation resources: cpu, memory, ephemeral-storage, scalar[k] */
#define KS_RSV_CLASSES 64 /* pod match classes (ks_reservation_cols.owner_classes bits) */
#define KS_MAX_GPUS 8     /* GPU minors per node (ks_device_cols); minor = slot index */
#define KS_MAX_RDMA 8     /* RDMA minors per node (ks_device_cols); minor = slot index */
#define KS_MAX_PCIE 8     /* PCIe switches per node (ks_device_cols.pcie_*) */
#define KS_PCIE_NONE 0xFFu /* device without topology (DeviceInfo.Topology == nil) */
/* device words of one reservation's device resources (ks_reservation_cols.dev_*): GPU minor k's gpu-core at k,
 * gpu-memory at KS_MAX_GPUS + k, gpu-memory-ratio at 2 * KS_MAX_GPUS + k; RDMA minor j's koordinator.sh/rdma at
 * 3 * KS_MAX_GPUS + j */
#define KS_DEV_WORDS (3 * KS_MAX_GPUS + KS_MAX_RDMA)
#define KS_MAX_CPUS 256   /* logical CPUs per node topology (ks_cpu_topology); CPU ids 0..ncpus-1 */
#define KS_CPU_WORDS 4    /* uint64 words of a CPU set (bit c = CPU c) */
#define KS_MAX_NUMA 8     /* NUMA nodes per node (ks_numa_node_cols); the device evaluates up to 4 */

/* ---- status codes ---- */
#define KS_OK 0
#define KS_EINVAL (-1)       /* bad argument / value out of supported range   */
#define KS_EHIP (-2)         /* HIP runtime error                               */
#define KS_ESTATE (-3)       /* call out of order (e.g. schedule before load)   */
#define KS_EUNSUPPORTED (-4) /* configuration not supported by this build       */
#define KS_ENOMEM (-5)

/* ---- NodeResourcesFit scoring strategy (pkg/scheduler/apis/config/types.go:84-92) ---- */
#define KS_LEAST_ALLOCATED 0
#define KS_MOST_ALLOCATED 1

/* ---- per-node LoadAware flags (ks_node_cols.la_flags) ----
 * Resolved by the host from the NodeMetric object, node annotations and the
 * plugin args, exactly at the points the reference reads them. */
#define KS_LA_HAS_METRIC 0x01u          /* nodeMetricLister.Get found it (load_aware.go:133,278)          */
#define KS_LA_EXPIRED 0x02u             /* isNodeMetricExpired(nm, NodeMetricExpirationSeconds) (helper.go:36) */
#define KS_LA_HAS_STATUS_METRIC 0x04u   /* nm.Status.NodeMetric != nil (load_aware.go:174)                */
#define KS_LA_FILTER_USAGE_PRESENT 0x08u /* filter profile's nodeUsage != nil (load_aware.go:195-208)     */
#define KS_LA_AGGREGATED_FILTER 0x10u   /* filter profile uses AggregatedUsage (reason string variant)    */
#define KS_LA_NODE_THR_NONEMPTY 0x20u   /* len(usageThresholds) > 0 (load_aware.go:159)                   */
#define KS_LA_PROD_THR_NONEMPTY 0x40u   /* len(ProdUsageThresholds) > 0 (load_aware.go:148)               */
#define KS_LA_HAS_PODS_METRIC 0x80u     /* len(nm.Status.PodsMetric) > 0 (load_aware.go:227)              */

/* ---- per-pod flags (ks_pod_cols.flags) ---- */
#define KS_POD_PROD 0x01u            /* GetPodPriorityClassWithDefault == koord-prod (apis/extension/priority_utils.go:26) */
#define KS_POD_DAEMONSET 0x02u       /* isDaemonSetPod(ownerRefs) (loadaware/helper.go:188)          */
#define KS_POD_NONPREEMPTIBLE 0x04u  /* extension.IsPodNonPreemptible (elasticquota/plugin.go:236)   */
#define KS_POD_SCALAR_KEYS 0x08u     /* podRequest.ScalarResources has at least one key (upstream fitsRequest) */
#define KS_POD_RSV_AFFINITY 0x10u    /* GetRequiredReservationAffinity != nil (reservation/transformer.go:51, stateData.hasAffinity) */
#define KS_POD_CPU_BIND 0x20u        /* NodeNUMAResource preFilterState.requestCPUBind (nodenumaresource/plugin.go:236-262):
                                        a preferred FullPCPUs / SpreadByPCPUs policy of an LSE/LSR prod pod with a whole-CPU
                                        request; policy and exclusive policy in ks_pod_cols.cpu_bind, KS_CPU_BIND_REQUIRED
                                        when the policy is resourceSpec.requiredCPUBindPolicy */
#define KS_POD_GPU_CORE 0x40u        /* DeviceShare: the converted GPU request has a gpu-core key (deviceshare/utils.go:96-146) */
#define KS_POD_UNMODELLED 0x100u     /* set by the shim for a pod with anything the library does not model: FPGA requests,
                                        DeviceShare allocate hints (VF selectors, RequestsAsCount, exclusive policies), a
                                        reserve pod as the scheduling subject; every pod entry point refuses it with
                                        KS_EUNSUPPORTED (the pod keeps the reference path) */
#define KS_POD_GPU_MEMORY 0x80u      /* DeviceShare: gpu-memory given (ratio derived per node, devicehandler_gpu.go:71-89);
                                        otherwise gpu-memory-ratio given (memory derived) */

/* ---- per-node NodeNUMAResource flags (ks_node_cols.numa_flags) ---- */
#define KS_NUMA_INVALID_RATIO 0x1u   /* GetNodeResourceAmplificationRatio returned an error (plugin.go:348-351)   */
#define KS_NUMA_CPU_BIND_POLICY 0x2u /* a node CPU bind policy the caller cannot encode in bits 7-8: unsupported    */
#define KS_NUMA_TOPOLOGY_POLICY 0x4u /* NUMA topology policy != None (getNUMATopologyPolicy): unsupported         */
#define KS_NUMA_ALLOC_LEAST 0x8u     /* label numa-allocate-strategy = LeastAllocated (GetNUMAAllocateStrategy, util.go:30-36) */
#define KS_NUMA_ALLOC_MOST 0x10u     /* label numa-allocate-strategy = MostAllocated                                */
#define KS_NUMA_POLICY_SHIFT 5       /* bits 5-6: NUMA topology policy (getNUMATopologyPolicy, util.go:52-58)          */
#define KS_NUMA_POLICY_NONE 0u
#define KS_NUMA_POLICY_BEST_EFFORT 1u
#define KS_NUMA_POLICY_RESTRICTED 2u
#define KS_NUMA_POLICY_SINGLE_NUMA_NODE 3u
#define KS_NUMA_CPU_BIND_SHIFT 7     /* bits 7-8: node CPU bind policy, extension.GetNodeCPUBindPolicy (apis/extension/
                                        numa_aware.go:314-325: the node-cpu-bind-policy label, or a static kubelet CPU
                                        manager with full-pcpus-only = FullPCPUsOnly).  Not combined with a NUMA policy. */
#define KS_NUMA_MAX_REF_COUNT 0x200u /* the node shares CPUs (NodeAllocation maxRefCount > 1, node_allocation.go:133-149):
                                        refused with KS_EUNSUPPORTED */
#define KS_NODE_CPU_BIND_NONE 0u
#define KS_NODE_CPU_BIND_FULL_PCPUS_ONLY 1u
#define KS_NODE_CPU_BIND_SPREAD_BY_PCPUS 2u

/* ---- pod cpuset request (ks_pod_cols.cpu_bind, with KS_POD_CPU_BIND) ---- */
#define KS_CPU_BIND_FULL_PCPUS 1u       /* schedulingconfig.CPUBindPolicyFullPCPUs     */
#define KS_CPU_BIND_SPREAD_BY_PCPUS 2u  /* schedulingconfig.CPUBindPolicySpreadByPCPUs */
#define KS_CPU_BIND_POLICY_MASK 0x3u
#define KS_CPU_BIND_REQUIRED 0x10u      /* the policy is required (resourceSpec.requiredCPUBindPolicy, PreFilter
                                           plugin.go:245-250): Filter checks it on every node (plugin.go:303-327) and
                                           allocateCPUSet keeps only CPUs that satisfy it (resource_manager.go:322-330) */
#define KS_CPU_EXCL_SHIFT 2             /* bits 2-3: preferredCPUExclusivePolicy */
#define KS_CPU_EXCL_NONE 0u
#define KS_CPU_EXCL_PCPU_LEVEL 1u
#define KS_CPU_EXCL_NUMA_NODE_LEVEL 2u

/* ---- per-node filter reason bits (ks_eval_pod_debug) ---- */
#define KS_R_FIT_PODS 0x001u      /* "Too many pods"                                    */
#define KS_R_FIT_CPU 0x002u       /* "Insufficient cpu"                                 */
#define KS_R_FIT_MEMORY 0x004u    /* "Insufficient memory"                              */
#define KS_R_FIT_EPHEMERAL 0x008u /* "Insufficient ephemeral-storage"                   */
#define KS_R_FIT_SCALAR 0x010u    /* "Insufficient <scalar>"                            */
#define KS_R_LA_CPU 0x020u        /* ErrReasonUsageExceedThreshold cpu (load_aware.go:45) */
#define KS_R_LA_MEMORY 0x040u     /* ErrReasonUsageExceedThreshold memory               */
#define KS_R_LA_AGGREGATED 0x080u /* the failure used ErrReasonAggregatedUsageExceedThreshold */
#define KS_R_LA_PROD 0x100u       /* the failure came from filterProdUsage              */
#define KS_R_RSV_AFFINITY 0x200u  /* ErrReasonReservationAffinity: no matched reservation (reservation/plugin.go:236,343) */
#define KS_R_RSV_NO_FIT 0x400u    /* filterWithReservations: no matched reservation satisfies the pod (plugin.go:425-437) */
#define KS_R_NUMA_AMPLIFIED_CPU 0x800u  /* ErrInsufficientAmplifiedCPU (nodenumaresource/plugin.go:369-371)       */
#define KS_R_NUMA_INVALID_RATIO 0x1000u /* ErrInvalidCPUAmplificationRatio (plugin.go:348-351)                    */
#define KS_R_DEV_INSUFFICIENT 0x2000u   /* DeviceShare "Insufficient gpu devices" (device_allocator.go:453-456)  */
#define KS_R_DEV_NO_GPU 0x4000u         /* DeviceShare: node has no (healthy) GPU (devicehandler_gpu.go:41-50)  */
#define KS_R_NUMA_INVALID_TOPOLOGY 0x8000u /* ErrInvalidCPUTopology: cpu-bind pod on a node without a valid CPU topology (plugin.go:296-301) */
#define KS_R_NUMA_AFFINITY 0x10000u    /* topology manager Admit: "node(s) NUMA Topology affinity error" (topologymanager/manager.go:64-66) */
#define KS_R_NUMA_INSUFFICIENT 0x20000u /* NUMA Allocate: "Insufficient NUMA <resource>" (resource_manager.go:269-276) */
#define KS_R_NUMA_MISSING 0x40000u     /* "node(s) missing NUMA resources" (topology_hint.go:33-36) */
#define KS_R_DEV_NO_RDMA 0x80000u      /* DeviceShare: "Insufficient rdma devices", no RDMA device on the node
                                          (DefaultDeviceHandler, devicehandler_default.go:45-48) */
#define KS_R_DEV_JOINT 0x100000u       /* DeviceShare joint allocation: "node(s) Joint-Allocate rules not met" or
                                          "Device Joint-Allocate rules violation" (device_allocator.go:252,280) */
#define KS_R_NUMA_CPUSET 0x200000u     /* NUMA Allocate of a cpu-bind pod on a NUMA-policy node: "not enough cpus available
                                          to satisfy request" (allocateCPUSet, resource_manager.go:333-335,366-368); on a
                                          node without NUMA policy the trial Allocate of a required CPU bind policy
                                          (plugin.go:318-327) */
#define KS_R_NUMA_INVALID_CPUS 0x400000u  /* ErrInvalidRequestedCPUs: a node CPU bind policy and a request that is not
                                             whole CPUs (requestCPUBind, util.go:105-122) */
#define KS_R_NUMA_BIND_CONFLICT 0x800000u /* ErrCPUBindPolicyConflict: the pod's required policy differs from the
                                             node's (plugin.go:310-312) */
#define KS_R_NUMA_SMT 0x1000000u          /* ErrSMTAlignmentError: required FullPCPUs and numCPUsNeeded not a multiple
                                             of the node's CPUsPerCore (plugin.go:314-317) */
#define KS_R_TAINT 0x2000000u             /* upstream TaintToleration Filter: "node(s) had untolerated taint" (a NoSchedule /
                                             NoExecute taint no toleration of the pod tolerates) */
#define KS_R_NODE_AFFINITY 0x4000000u     /* upstream NodeAffinity Filter: "node(s) didn't match Pod's node affinity/selector" */
#define KS_R_NODE_PORTS 0x8000000u        /* upstream NodePorts Filter: "node(s) didn't have free ports for the requested pod ports" */
/* upstream PodTopologySpread Filter (ABI 8): "node(s) didn't match pod topology spread constraints" (ErrReasonConstraintsNotMatch)
 * or its "(missing required label)" variant (ErrReasonNodeLabelNotMatch) */
#define KS_R_TOPOLOGY_SPREAD 0x10000000u
/* upstream InterPodAffinity Filter (ABI 8), the first failing check of the three in the plugin's order: */
#define KS_R_POD_AFFINITY 0x20000000u          /* "node(s) didn't match pod affinity rules" */
#define KS_R_POD_ANTI_AFFINITY 0x40000000u     /* "node(s) didn't match pod anti-affinity rules" */
#define KS_R_EXISTING_ANTI_AFFINITY 0x80000000u /* "node(s) didn't satisfy existing pods anti-affinity rules" */

/* ---- per-pod result status (ks_result.status) ---- */
#define KS_S_SCHEDULED 0x0u
#define KS_S_QUOTA 0x1u                /* ElasticQuota PreFilter: "Insufficient quotas"            */
#define KS_S_QUOTA_NONPREEMPTIBLE 0x2u /* ElasticQuota PreFilter: "Insufficient non-preemptible quotas" */
#define KS_S_QUOTA_PARENT 0x4u         /* checkQuotaRecursive rejected at a parent                 */
#define KS_S_UNSCHEDULABLE 0x8u        /* no node passed Filter                                    */
#define KS_S_RESERVE_FAILED 0x10u      /* a Reserve plugin failed on the selected node and every plugin unreserved
                                          (NodeNUMAResource Allocate: "not enough cpus available", resource_manager.go:333-335);
                                          node = the selected node, nothing is applied */

/* score plugin slots for ks_eval_pod_debug's per-plugin score matrix */
#define KS_SCORE_FIT 0
#define KS_SCORE_LOADAWARE 1
#define KS_SCORE_RESERVATION 2 /* after DefaultNormalizeScore (reservation/scoring.go:126-131) */
#define KS_SCORE_NUMA 3        /* NodeNUMAResource scoreWithAmplifiedCPUs (nodenumaresource/scoring.go:98-114) */
#define KS_SCORE_DEVICESHARE 4 /* after DefaultNormalizeScore (deviceshare/scoring.go:95-97) */
#define KS_SCORE_BALANCED 5    /* upstream NodeResourcesBalancedAllocation (balanced_allocation.go, v1.24) */
#define KS_SCORE_TAINT 6       /* upstream TaintToleration after DefaultNormalizeScore(100, reverse) (v1.24) */
#define KS_SCORE_NODE_AFFINITY 7 /* upstream NodeAffinity after DefaultNormalizeScore(100) (v1.24) */
#define KS_SCORE_TOPOLOGY_SPREAD 8 /* upstream PodTopologySpread after its NormalizeScore (v1.24, ABI 8) */
#define KS_SCORE_POD_AFFINITY 9    /* upstream InterPodAffinity after its NormalizeScore (v1.24, ABI 8) */
#define KS_NUM_SCORE_PLUGINS 10

/* ---- per-node DeviceShare flags (ks_device_cols.flags) ---- */
#define KS_DEV_PRESENT 0x1u /* nodeDeviceCache.getNodeDevice != nil (deviceshare/plugin.go:286-289) */
#define KS_DEV_UNMODELLED 0x2u /* set by the shim for device state the library does not model on the node (FPGA or
                                  VF-allocated devices): ks_load_devices / ks_update_devices refuse it.  Device-holding
                                  reservations are modelled (ks_reservation_cols.dev_*); preemptible device capacity
                                  (device_cache.go:314) exists only inside a preemption dry run, which ks_preempt refuses
                                  with DeviceShare */

/* ---- reservation flags (ks_reservation_cols.flags) ---- */
#define KS_RSV_UNSCHEDULABLE 0x1u /* ReservationInfo.IsUnschedulable (transformer.go:113)              */
#define KS_RSV_ALLOCATE_ONCE 0x2u /* IsAllocateOnce (transformer.go:109, plugin.go:523)                */
#define KS_RSV_POLICY_DEFAULT 0u    /* ReservationAllocatePolicy (ks_reservation_cols.policy) */
#define KS_RSV_POLICY_ALIGNED 1u
#define KS_RSV_POLICY_RESTRICTED 2u

/* NodeResourcesFitArgs.scoringStrategy (upstream apis/config/types.go; the profile in
 * config/manager/scheduler-config.yaml:17-31). A weight of 0 means "not listed". */
typedef struct ks_fit_args {
  int32_t enable_filter;
  int32_t enable_score;
  int32_t strategy; /* KS_LEAST_ALLOCATED | KS_MOST_ALLOCATED */
  int32_t _pad0;
  int64_t weight_cpu;
  int64_t weight_memory;
  int64_t weight_ephemeral;
  int64_t weight_scalar[KS_MAX_SCALARS];
  int64_t plugin_weight; /* profile score weight */
} ks_fit_args;

/* LoadAwareSchedulingArgs (pkg/scheduler/apis/config/types.go:30-62) after
 * SetDefaults_LoadAwareSchedulingArgs (v1beta2/defaults.go:77-100).  Per-node
 * thresholds (custom-usage-thresholds annotation, aggregated profile) are
 * resolved by the host into ks_node_cols; only the pod-independent knobs that
 * the sweep needs live here.  Only cpu and memory may carry weights. */
typedef struct ks_loadaware_args {
  int32_t enable_filter;
  int32_t enable_score;
  int32_t filter_expired_node_metrics; /* FilterExpiredNodeMetrics (load_aware.go:141) */
  int32_t score_according_prod_usage;  /* ScoreAccordingProdUsage (load_aware.go:294)  */
  int64_t weight_cpu;                  /* ResourceWeights[cpu]; 0 = not listed          */
  int64_t weight_memory;
  int64_t scaling_cpu;                 /* EstimatedScalingFactors                        */
  int64_t scaling_memory;
  int64_t plugin_weight;
} ks_loadaware_args;

/* ElasticQuotaArgs (pkg/scheduler/apis/config/types.go) */
typedef struct ks_quota_args {
  int32_t enable;
  int32_t enable_check_parent_quota; /* EnableCheckParentQuota (plugin.go:250) */
} ks_quota_args;

/* Reservation plugin (pkg/scheduler/plugins/reservation): profile score weight
 * (config/manager/scheduler-config.yaml: 5000).  The device ranks nodes by the exact
 * lexicographic order the normalized score induces, which requires
 * plugin_weight > 100 * (fit.plugin_weight + loadaware.plugin_weight);
 * other weights are rejected with KS_EUNSUPPORTED. */
typedef struct ks_reservation_args {
  int32_t enable;
  int32_t _pad0;
  int64_t plugin_weight;
} ks_reservation_args;

/* NodeNUMAResourceArgs.ScoringStrategy (pkg/scheduler/apis/config/types.go; defaults
 * v1beta2/defaults.go:107-136: LeastAllocated, cpu 1, memory 1).  Node CPU bind policies
 * (numa_flags bits 7-8), NUMA topology policies (bits 5-6, with ks_load_numa_nodes) and cpuset pods
 * (KS_POD_CPU_BIND, preferred or KS_CPU_BIND_REQUIRED) are supported on nodes whose CPU topology and
 * allocation state were given to ks_load_cpu_state; a CPU bind policy together with a NUMA policy is not. */
typedef struct ks_numa_args {
  int32_t enable;
  int32_t strategy; /* KS_LEAST_ALLOCATED | KS_MOST_ALLOCATED */
  int64_t weight_cpu;
  int64_t weight_memory;
  int64_t plugin_weight;
  /* NUMAScoringStrategy.Type: the default NUMA allocate strategy of the CPU accumulator
   * (GetDefaultNUMAAllocateStrategy, util.go:22-28): KS_MOST_ALLOCATED -> NUMAMostAllocated, else NUMALeastAllocated */
  int32_t numa_scoring_strategy;
  int32_t _pad0;
} ks_numa_args;

/* DeviceShareArgs.ScoringStrategy (defaults v1beta2/defaults.go:187-207: LeastAllocated,
 * gpu-memory-ratio 1, rdma 1).  GPU and RDMA devices with joint [gpu, rdma] allocation; no allocate
 * hints, FPGAs, NUMA affinity, VFs or device-holding reservations. */
typedef struct ks_deviceshare_args {
  int32_t enable;
  int32_t strategy; /* KS_LEAST_ALLOCATED | KS_MOST_ALLOCATED */
  int64_t weight_gpu_core;
  int64_t weight_gpu_memory;
  int64_t weight_gpu_memory_ratio;
  int64_t plugin_weight;
  int64_t weight_rdma; /* koordinator.sh/rdma (default 1): scores RDMA minors and the RDMA part of scoreNode */
} ks_deviceshare_args;

/* Upstream NodeResourcesBalancedAllocation (kube-scheduler v1.24.15 noderesources/balanced_allocation.go, enabled with
 * weight 1 by the v1beta2 default profile): score = int64((1 - std) * 100) over the fractions
 * (Requested + pod request) / Allocatable, each capped at 1, of the listed resources with Allocatable != 0; std is
 * |f_cpu - f_memory| / 2 for two fractions and 0 for fewer (balancedResourceScorer, useRequested = true).  The
 * resource set is cpu and/or memory (NodeResourcesBalancedAllocationArgs.Resources; the v1beta2 default is both);
 * other resources are refused.  Pod overhead is not modelled (the host folds it into the request vector). */
#define KS_BAL_CPU 0x1
#define KS_BAL_MEMORY 0x2
typedef struct ks_balanced_args {
  int32_t enable;
  int32_t resources; /* KS_BAL_* bits */
  int64_t plugin_weight;
} ks_balanced_args;

/* Upstream TaintToleration and NodeAffinity (kube-scheduler v1.24.15 plugins/tainttoleration, plugins/nodeaffinity;
 * both enabled with weight 1 by the v1beta2 default profile).  The label and taint matching runs on the host once per
 * distinct taint / label requirement and reaches the device as bit masks over two per-context dictionaries
 * (INTEGRATION.md "Taints and node affinity"):
 *   taint dictionary   <= 64 distinct node taints (key, value, effect); ks_node_cols.taints_hard / taints_soft carry
 *                      the node's NoSchedule|NoExecute / PreferNoSchedule taints, ks_pod_cols.tolerated the taints
 *                      some toleration of the pod tolerates (Toleration.ToleratesTaint);
 *   label dictionary   <= 63 distinct node selector requirements (key, operator, values) of the pending pods
 *                      (nodeSelector entries become key In [value]); ks_node_cols.labels bit i = requirement i
 *                      matches the node's labels (or metadata.name for matchFields); bit 63 (KS_LABEL_NEVER) is
 *                      never set on a node and stands for an empty NodeSelectorTerm, which matches nothing.
 * TaintToleration Filter: no NoSchedule/NoExecute taint untolerated; Score: the number of PreferNoSchedule taints
 * untolerated, DefaultNormalizeScore(100, reverse = true) over the feasible nodes.  NodeAffinity Filter: the pod's
 * required terms (nodeSelector requirements ANDed into every term) -- one term whose requirement bits are all set on
 * the node; Score: sum of the weights of the preferred terms whose bits are all set, DefaultNormalizeScore(100). */
#define KS_AFFINITY_TERMS 4
#define KS_LABEL_NEVER (1ull << 63)
typedef struct ks_static_plugin_args {
  int32_t enable_filter;
  int32_t enable_score;
  int64_t plugin_weight;
} ks_static_plugin_args;

/* Upstream PodTopologySpread and InterPodAffinity (kube-scheduler v1.24.15 plugins/podtopologyspread,
 * plugins/interpodaffinity; the v1beta2 default profile enables both, weights 2 and 1, with the system default
 * spreading constraints and hardPodAffinityWeight 1).  Both count pods per topology domain.  The label selector
 * matching runs on the host once per distinct selector / affinity term (koordinator_amd/topology_plugins.py,
 * INTEGRATION.md "Pod topology spread and inter-pod affinity") and reaches the device as:
 *   properties   ks_node_cols.topo_nprops (<= KS_TOPO_MAX_PROPS) predicates on pods (matches a spread constraint's
 *                selector in a namespace, matches an affinity term, matches all required affinity terms of a pod,
 *                carries an anti-affinity term or weighted affinity terms); ks_node_cols.topo_count[p * n + i] = node
 *                i's pods with property p (every Reserve adds the pod's property list, ks_pod_cols.topo_props,
 *                ks_unreserve removes it, ks_read_nodes reads the counters back);
 *   domains      key 0 is the hostname (every node its own domain); keys 1..topo_nkeys (<= KS_TOPO_MAX_KEYS - 1) are
 *                any other node labels: ks_node_cols.topo_domain[(k - 1) * n + i] = node i's value index of key k,
 *                0..topo_ndomains-1, -1 = label absent;
 *   query terms  <= KS_TOPO_MAX_TERMS per pod (ks_pod_cols.topo_terms, packed words, see KS_TOPO_K_*): what the two
 *                plugins' PreFilter / Filter / PreScore / Score ask of the counters for that pod.
 * A pod without query terms (KS_TOPO_DYN clear) never fails their Filters and scores 100 (PodTopologySpread's
 * NormalizeScore with no constraint) and 0 everywhere; a pod with them is scheduled alone against the counters of
 * every pod placed before it, on every rank over the whole (replicated) node table under
 * ks_shard_init.  Not with ks_preempt. */
#define KS_TOPO_MAX_KEYS 256      /* topology keys, the hostname included */
#define KS_TOPO_MAX_PROPS 65536   /* properties per context */
#define KS_TOPO_MAX_TERMS 64      /* query terms per pod */
/* ks_pod_cols.topo_flags */
#define KS_TOPO_DYN 0x1u           /* the pod has query terms */
#define KS_TOPO_SELF_AFFINITY 0x2u /* podMatchesAllAffinityTerms(pod's own required affinity terms, pod) */
#define KS_TOPO_SOFT_ALL_KEYS 0x4u /* PreScore requireAllTopologies: the soft constraints are the pod's own (not the
                                      system defaults), so nodes without every soft key are ignored */
/* topo_terms word: kind (bits 0-3), flags (4-7), key (8-15: 0 hostname, k >= 1 topo_domain key k), property
 * (16-31), param (32-63, int32: maxSkew, or the score weight with its sign) */
#define KS_TOPO_K_SPREAD_HARD 1    /* DoNotSchedule constraint: skew = domain matches + self - min over domains */
#define KS_TOPO_K_SPREAD_SOFT 2    /* ScheduleAnyway constraint (the pod's own or a system default) */
#define KS_TOPO_K_AFFINITY 3       /* required affinity term (property: pods matching all of the pod's terms) */
#define KS_TOPO_K_ANTI 4           /* required anti-affinity term */
#define KS_TOPO_K_EXISTING_ANTI 5  /* a placed pod's required anti-affinity term that matches the pod */
#define KS_TOPO_K_SCORE 6          /* weighted score term: weight x matching pods in the node's domain */
#define KS_TOPO_T_SELF 0x1u        /* spread: the constraint's selector matches the pod itself */
typedef struct ks_topology_args {
  int32_t enable;
  int32_t _pad0;
  int64_t spread_weight;   /* PodTopologySpread profile weight (v1beta2 default 2) */
  int64_t affinity_weight; /* InterPodAffinity profile weight (default 1) */
} ks_topology_args;

typedef struct ks_config {
  int32_t abi_version; /* = KS_ABI_VERSION */
  int32_t device;      /* HIP device ordinal */
  ks_fit_args fit;
  ks_loadaware_args loadaware;
  ks_quota_args quota;
  int32_t batch_pods;  /* pods evaluated per sweep pass (0 = default 64, max 64) */
  int32_t candidates;  /* candidate node chunks kept per pod per pass (0 = default 32, max 64) */
  int32_t profile;     /* 1 = bracket every kernel with HIP events (ks_get_stats) */
  int32_t _pad1;
  ks_reservation_args reservation;
  ks_numa_args numa;
  ks_deviceshare_args deviceshare;
  ks_balanced_args balanced; /* ABI 5 */
  ks_static_plugin_args taint;    /* ABI 6: upstream TaintToleration */
  ks_static_plugin_args affinity; /* ABI 6: upstream NodeAffinity */
  ks_static_plugin_args nodeports; /* ABI 6: upstream NodePorts (Filter only: enable_score / plugin_weight unused) */
  ks_topology_args topology;       /* ABI 8: upstream PodTopologySpread + InterPodAffinity */
} ks_config;

/* Node snapshot, structure-of-arrays, one entry per node.  NodeInfo fields are
 * upstream framework.NodeInfo (Allocatable/Requested/NonZeroRequested/Pods).
 * The LoadAware block is the host-side reduction of NodeMetric + podAssignCache
 * documented in DESIGN.md §2 (reference: load_aware.go:123-376, helper.go:36-186). */
typedef struct ks_node_cols {
  const int64_t *alloc_milli_cpu;
  const int64_t *alloc_memory;
  const int64_t *alloc_ephemeral;
  const int32_t *allowed_pods;
  const int64_t *req_milli_cpu;   /* NodeInfo.Requested */
  const int64_t *req_memory;
  const int64_t *req_ephemeral;
  const int32_t *pod_count;       /* len(NodeInfo.Pods) */
  const int64_t *nonzero_milli_cpu; /* NodeInfo.NonZeroRequested */
  const int64_t *nonzero_memory;
  const int64_t *alloc_scalar[KS_MAX_SCALARS]; /* NULL = slot unused (treated as 0) */
  const int64_t *req_scalar[KS_MAX_SCALARS];
  /* LoadAwareScheduling */
  const uint32_t *la_flags;        /* KS_LA_* */
  const int64_t *la_alloc_milli_cpu; /* EstimateNode() allocatable (estimator/default_estimator.go:110-129) */
  const int64_t *la_alloc_memory;
  const int64_t *la_term_milli_cpu;  /* Σ assigned-estimated + node usage (load_aware.go:294-325), all pods */
  const int64_t *la_term_memory;
  const int64_t *la_prod_term_milli_cpu; /* same with filterProdPod=true (prod pod, ScoreAccordingProdUsage) */
  const int64_t *la_prod_term_memory;
  const int32_t *la_thr_cpu;          /* filter usage thresholds, 0 = skip (load_aware.go:185-187) */
  const int32_t *la_thr_memory;
  const int32_t *la_prod_thr_cpu;     /* prod usage thresholds, 0 = skip */
  const int32_t *la_prod_thr_memory;
  const int64_t *la_total_milli_cpu;  /* EstimateNode allocatable .MilliValue() (load_aware.go:214) */
  const int64_t *la_total_milli_memory;
  const int64_t *la_usage_milli_cpu;  /* filter profile usage .MilliValue() (node or aggregated) */
  const int64_t *la_usage_milli_memory;
  const int64_t *la_prod_usage_milli_cpu; /* Σ prod pod usages .MilliValue() (load_aware.go:231-248) */
  const int64_t *la_prod_usage_milli_memory;
  /* NodeNUMAResource */
  const double *numa_cpu_amplification; /* node annotation cpu amplification ratio; NULL / <= 1 = none */
  const int32_t *numa_cpuset_cpus;      /* CPUs allocated to cpuset pods: GetAvailableCPUs' allocated.Size() */
  const uint32_t *numa_flags;           /* KS_NUMA_* */
  /* TaintToleration / NodeAffinity (ABI 6; NULL = 0): bits over the context's taint / label dictionaries, see
   * ks_static_plugin_args.  Static per node: changed only through ks_load_nodes / ks_update_nodes. */
  const uint64_t *taints_hard;  /* taints with effect NoSchedule or NoExecute */
  const uint64_t *taints_soft;  /* taints with effect PreferNoSchedule */
  const uint64_t *labels;       /* node selector requirements the node matches (bit 63 must be 0) */
  /* NodePorts (ABI 6; NULL = 0): host-port dictionary bits in use on the node (NodeInfo.UsedPorts); every Reserve
   * adds the pod's bits while ks_config.nodeports is on (read back with ks_read_nodes) */
  const uint64_t *host_ports;
  /* PodTopologySpread / InterPodAffinity (ABI 9; NULL = -1 / 0), see ks_topology_args.  The three sizes are fixed by
   * ks_load_nodes; ks_update_nodes rows carry the same. */
  int32_t topo_nkeys;            /* topology keys besides the hostname (keys 1..topo_nkeys) */
  int32_t topo_ndomains;         /* value indices of every key are below this (>= 1 with keys) */
  int32_t topo_nprops;           /* properties */
  int32_t _topo_pad;
  const int32_t *topo_domain;    /* [topo_nkeys][n]: key k's value index on node i at (k - 1) * n + i, -1 = absent */
  const int32_t *topo_count;     /* [topo_nprops][n]: the node's pods with property p at p * n + i */
} ks_node_cols;

/* Pending pods, queue order, structure-of-arrays. */
typedef struct ks_pod_cols {
  const int64_t *req_milli_cpu;  /* upstream computePodResourceRequest (Fit PreFilter) */
  const int64_t *req_memory;
  const int64_t *req_ephemeral;
  const int64_t *req_scalar[KS_MAX_SCALARS]; /* NULL = 0 */
  const int64_t *nonzero_milli_cpu; /* non-zero request (100m / 200Mi defaults) for Fit score + NonZeroRequested */
  const int64_t *nonzero_memory;
  const uint32_t *flags;          /* KS_POD_* */
  /* EstimatePod inputs (estimator/default_estimator.go:57-108): request/limit of the
   * priority-translated resource name (resource.go:53-58), plus the value used when
   * the quantity is zero (250 / 209715200 / 0). */
  const int64_t *la_req_cpu;
  const int64_t *la_lim_cpu;
  const int64_t *la_dflt_cpu;
  const int64_t *la_req_memory;
  const int64_t *la_lim_memory;
  const int64_t *la_dflt_memory;
  /* ElasticQuota */
  const int32_t *quota;           /* quota row, -1 = no quota (plugin.go:211-215) */
  const uint32_t *quota_mask;     /* bit d: dimension d present in PodRequestsAndLimits keys */
  const int64_t *quota_req[KS_QUOTA_DIMS];
  /* Reservation: the pod's match class (-1 = matches no reservation; NULL = all -1).  Pods
   * whose MatchReservationOwners / reservation-affinity outcome is identical for every
   * reservation share a class (matchReservation, transformer.go:349-373); reserve pods
   * themselves are not scheduled through this entry point. */
  const int32_t *rsv_class;
  /* DeviceShare: the pod's converted GPU request (GetPodDeviceRequests, utils.go:232-252; nvidia.com/gpu
   * and koordinator.sh/gpu converted to core + ratio by the host); NULL = no GPU request */
  const int64_t *gpu_core;
  const int64_t *gpu_memory;
  const int64_t *gpu_memory_ratio;
  /* NodeNUMAResource cpuset request with KS_POD_CPU_BIND: KS_CPU_BIND_* | exclusive policy << KS_CPU_EXCL_SHIFT
   * (preferredCPUBindPolicy after the args default, preferredCPUExclusivePolicy); numCPUsNeeded =
   * req_milli_cpu / 1000 (a multiple of 1000).  NULL = none */
  const uint32_t *cpu_bind;
  /* DeviceShare RDMA request koordinator.sh/rdma (DefaultDeviceHandler, devicehandler_default.go:44-93: a value
   * > 100 and divisible by 100 asks for value/100 devices); NULL = none */
  const int64_t *rdma;
  /* DeviceShare joint allocation (apiext.DeviceJointAllocate, device_allocator.go:188-339): KS_JOINT_*; the
   * only supported DeviceTypes list is [gpu, rdma]; NULL = none */
  const uint8_t *joint;
  /* TaintToleration / NodeAffinity (ABI 6; NULL = none): see ks_static_plugin_args */
  const uint64_t *tolerated;                              /* dictionary taints some toleration tolerates */
  const int32_t *affinity_required_n;                     /* required terms (0 = no nodeSelector / required affinity) */
  const uint64_t *affinity_required[KS_AFFINITY_TERMS];   /* term t: the requirement bits it needs */
  const uint64_t *affinity_preferred[KS_AFFINITY_TERMS];  /* preferred term t: the requirement bits it needs */
  const int32_t *affinity_weight[KS_AFFINITY_TERMS];      /* preferred term t's weight, 1..100 (0 = unused) */
  /* NodePorts (ABI 6; NULL = none): the pod's host ports as dictionary bits (the entries it uses) and the entries
   * any of them conflicts with (HostPortInfo.CheckConflict: same protocol and port, equal host IPs or either
   * 0.0.0.0) */
  const uint64_t *host_ports;
  const uint64_t *host_ports_conflict;
  /* PodTopologySpread / InterPodAffinity (ABI 9; NULL = none), see ks_topology_args.  Two CSR lists over the pods of
   * the call: pod i's entries are [beg[i], beg[i + 1]) */
  const uint32_t *topo_flags;     /* KS_TOPO_DYN | KS_TOPO_SELF_AFFINITY | KS_TOPO_SOFT_ALL_KEYS */
  const int32_t *topo_prop_beg;   /* [p + 1] */
  const int32_t *topo_props;      /* the pod's properties (counted where it is placed; each at most once) */
  const int32_t *topo_term_beg;   /* [p + 1] (at most KS_TOPO_MAX_TERMS per pod) */
  const uint64_t *topo_terms;     /* the pod's query terms */
} ks_pod_cols;

#define KS_JOINT_NONE 0u
#define KS_JOINT_GPU_RDMA 1u           /* DeviceTypes [gpu, rdma], no RequiredScope (best effort) */
#define KS_JOINT_GPU_RDMA_SAME_PCIE 2u /* DeviceTypes [gpu, rdma], RequiredScope SamePCIe */

/* ElasticQuota table: QuotaInfo.CalculateInfo per quota (core/quota_info.go). */
typedef struct ks_quota_cols {
  const int32_t *parent;          /* parent row, -1 = child of root (plugin_helper.go:292) */
  const uint32_t *limit_mask;     /* keys of getQuotaInfoUsedLimit (Runtime, or Max if !EnableRuntimeQuota) */
  const int64_t *limit[KS_QUOTA_DIMS];
  const int64_t *used[KS_QUOTA_DIMS];
  const uint32_t *min_mask;       /* keys of CalculateInfo.Min */
  const int64_t *min[KS_QUOTA_DIMS];
  const int64_t *nonpreemptible_used[KS_QUOTA_DIMS];
} ks_quota_cols;

/* ElasticQuota tree for RefreshRuntime (pkg/scheduler/plugins/elasticquota/core/group_quota_manager.go:259-326):
 * one row per quota of the tree (the system / default quotas excluded, as the reference does),
 * values per resource dimension (cpu -> MilliValue, others -> Value). */
typedef struct ks_quota_tree {
  const int32_t *parent;          /* parent row, -1 = child of the root quota */
  const uint8_t *allow_lent;      /* AllowLentResource (quota label allow-lent-resource, default true) */
  const uint32_t *max_mask;       /* keys of CalculateInfo.Max */
  const int64_t *max[KS_QUOTA_DIMS];
  const int64_t *min[KS_QUOTA_DIMS];           /* Min (= AutoScaleMin; scale-min-quota not modelled) */
  const int64_t *shared_weight[KS_QUOTA_DIMS]; /* NULL = Max (annotation shared-weight absent) */
  const int64_t *guaranteed[KS_QUOTA_DIMS];    /* NULL = 0 (feature ElasticQuotaGuaranteeUsage off) */
  const int64_t *self_request[KS_QUOTA_DIMS];  /* Σ PodRequestsAndLimits of the quota's own pods */
  int64_t cluster_total[KS_QUOTA_DIMS];        /* totalResourceExceptSystemAndDefaultUsed */
} ks_quota_tree;

/* Available reservations (reservationCache.forEachAvailableReservationOnNode,
 * reservation/cache.go:256-291), one row per reservation; rows of the same node are visited
 * in table order (the canonical order for the reference's map iteration).  ReservationInfo
 * fields: frameworkext/reservation_info.go:37-115.  The reserve pod in NodeInfo requests
 * exactly `allocatable` (reservationutil.NewReservePod). */
typedef struct ks_reservation_cols {
  const int32_t *node;            /* Status.NodeName as node row */
  const uint64_t *owner_classes;  /* bit c: pods of class c match (owners + reservation affinity) */
  const uint32_t *flags;          /* KS_RSV_* */
  const uint32_t *policy;         /* KS_RSV_POLICY_* (GetAllocatePolicy) */
  const int64_t *order;           /* label reservation-order parsed (scoring.go:162-181); 0 = none */
  const uint32_t *key_mask;       /* bit d: dimension d is a key of Allocatable (= ResourceNames) */
  const int64_t *allocatable[KS_RSV_DIMS];
  const int64_t *allocated[KS_RSV_DIMS];  /* NULL = 0 */
  const int32_t *assigned;        /* len(AssignedPods); NULL = 0 */
  const int64_t *reserve_nonzero_milli_cpu; /* reserve pod's NonZeroRequested; NULL = from allocatable */
  const int64_t *reserve_nonzero_memory;
  /* DeviceShare (deviceshare/reservation.go:118-171): [r * KS_DEV_WORDS + w] the reserve pod's device allocation
   * (nodeDeviceCache.getUsed of the reserve pod: the reservation's allocatable per minor; a minor with a non-zero word
   * is one of its minors) and the allocations of its assigned pods on those minors (appendAllocatedByHints).  NULL =
   * no reservation holds a device / nothing allocated.  The node's device used (ks_device_cols.used_*) counts both, as
   * nodeDeviceCache does.  Reservations holding devices on a node with a NUMA topology policy are not supported. */
  const int64_t *dev_allocatable;
  const int64_t *dev_allocated;
} ks_reservation_cols;

/* Node GPU devices (nodeDeviceCache, deviceshare/device_cache.go): per minor k the device total and
 * the used amount (deviceTotal / deviceUsed) of gpu-core, gpu-memory, gpu-memory-ratio.  A minor
 * whose totals are all zero is absent / unhealthy. */
typedef struct ks_device_cols {
  const uint32_t *flags; /* KS_DEV_* */
  const int64_t *total_core[KS_MAX_GPUS];
  const int64_t *total_memory[KS_MAX_GPUS];
  const int64_t *total_ratio[KS_MAX_GPUS];
  const int64_t *used_core[KS_MAX_GPUS];   /* NULL = 0 */
  const int64_t *used_memory[KS_MAX_GPUS];
  const int64_t *used_ratio[KS_MAX_GPUS];
  /* RDMA minors: koordinator.sh/rdma total and used (a minor with total 0 is absent); NULL = 0 */
  const int64_t *total_rdma[KS_MAX_RDMA];
  const int64_t *used_rdma[KS_MAX_RDMA];
  /* device topology (newNUMATopology, numa_topology.go:46-96): per node the PCIe switches are numbered
   * 0..KS_MAX_PCIE-1 in ascending (socketID, nodeID, pcieID) order (the order newDeviceTopologyGuide sorts
   * them into, numa_topology.go:141-151); gpu_pcie / rdma_pcie give each minor's switch (KS_PCIE_NONE: no
   * topology), pcie_numa / pcie_socket each switch's NUMA node and socket.  NULL = no topology */
  const uint8_t *gpu_pcie[KS_MAX_GPUS];
  const uint8_t *rdma_pcie[KS_MAX_RDMA];
  const uint8_t *pcie_numa[KS_MAX_PCIE];
  const uint8_t *pcie_socket[KS_MAX_PCIE];
} ks_device_cols;

/* A node CPU topology (CPUTopology, nodenumaresource/cpu_topology.go:27-33, built from the
 * NodeResourceTopology): CPU c has core / NUMA node / socket ids (ids < KS_MAX_CPUS, at most 8 CPUs
 * per core).  Nodes refer to a topology by index, so identical machines share one entry. */
typedef struct ks_cpu_topology {
  int32_t ncpus;
  int32_t core[KS_MAX_CPUS];
  int32_t numa_node[KS_MAX_CPUS];
  int32_t socket[KS_MAX_CPUS];
} ks_cpu_topology;

/* Per-node CPU allocation state (NodeAllocation, node_allocation.go:37-177) as CPU sets of
 * KS_CPU_WORDS words per node ([node*KS_CPU_WORDS + w]).  maxRefCount is 1 (every allocated CPU is
 * unavailable).  The cpuset millicores of ks_node_cols.numa_cpuset_cpus must match |allocated|. */
typedef struct ks_cpu_state_cols {
  const int32_t *topology;      /* index into the topology table, -1 = no valid topology */
  const uint64_t *allocated;    /* allocatedCPUs */
  const uint64_t *excl_pcpu;    /* allocated with CPUExclusivePolicy PCPULevel; NULL = none */
  const uint64_t *excl_numa;    /* allocated with CPUExclusivePolicy NUMANodeLevel; NULL = none */
  const uint64_t *reserved;     /* kubelet reserved CPUs (TopologyOptions.ReservedCPUs); NULL = none */
} ks_cpu_state_cols;

/* NUMA node resources of the nodes with a NUMA topology policy (TopologyOptions.NUMANodeResources and
 * NodeAllocation.allocatedResources, node_allocation.go:37-177), [node*KS_MAX_NUMA + k] for NUMA node k
 * (ids 0..count-1).  The cpu amplification ratio of the node (ks_node_cols.numa_cpu_amplification)
 * amplifies alloc_cpu and the cpuset part of used_cpu as amplifyNUMANodeResources /
 * getAvailableNUMANodeResources do. */
typedef struct ks_numa_node_cols {
  const int32_t *count;         /* [node] NUMA nodes with resources (0 = none) */
  const int64_t *alloc_cpu;     /* milli-CPU, before amplification */
  const int64_t *alloc_memory;
  const int64_t *used_cpu;      /* NULL = 0 */
  const int64_t *used_memory;   /* NULL = 0 */
  const uint8_t *used_present;  /* an allocatedResources entry exists for the NUMA node; NULL = used != 0 */
  const int32_t *cpuset_cpus;   /* allocated cpuset CPUs on the NUMA node; NULL = 0 */
} ks_numa_node_cols;

typedef struct ks_result {
  int32_t node;    /* chosen node index, -1 if not scheduled */
  uint32_t status; /* KS_S_* */
  int64_t score;   /* total weighted score of the chosen node */
  int32_t reservation; /* reservation row the pod was assumed into (Reserve, plugin.go:532-570), -1 = none */
  uint32_t gpu_minors; /* DeviceShare Reserve: bit k = GPU minor k allocated (plugin.go:377-430) */
  uint32_t rdma_minors; /* DeviceShare Reserve: bit k = RDMA minor k allocated */
  int32_t _pad0;
} ks_result;

/* Mutable node state after commits (read back for parity). */
typedef struct ks_node_state {
  int64_t *req_milli_cpu;
  int64_t *req_memory;
  int64_t *req_ephemeral;
  int32_t *pod_count;
  int64_t *nonzero_milli_cpu;
  int64_t *nonzero_memory;
  int64_t *req_scalar[KS_MAX_SCALARS]; /* NULL = skip */
  int64_t *la_term_milli_cpu;
  int64_t *la_term_memory;
  int64_t *la_prod_term_milli_cpu;
  int64_t *la_prod_term_memory;
  uint64_t *host_ports;  /* ABI 6: NodePorts dictionary bits in use (NULL = skip) */
  int32_t *topo_count;  /* ABI 9: [topo_nprops][n] the pods with each topology property (NULL = skip) */
} ks_node_state;

typedef struct ks_stats {
  int64_t passes;          /* sweep passes executed by the last ks_schedule* call */
  int64_t cut_passes;      /* passes ended early because a pod's candidates were exhausted */
  int64_t rescans;         /* dirty-chunk rescans done by the commit kernel */
  double sweep_ms;         /* summed HIP-event time of the sweep kernels */
  double select_ms;        /* summed HIP-event time of the candidate-selection kernels */
  double commit_ms;        /* summed HIP-event time of the commit kernels */
  double total_ms;         /* wall time of the last call on the device stream */
  int64_t sweep_launches;
  int64_t sweep_bytes;     /* algorithmic bytes one sweep launch reads/writes */
  int64_t slot_misses;     /* commits whose node row was not prefetched (one extra HBM round trip) */
  int64_t diag[8];         /* diagnostic build only (KS_COMMIT_STAMPS): commit-phase cycle sums */
  int64_t bubble_passes;   /* pipelined passes whose commit did nothing (the pass before was cut) */
  double fixup_ms;         /* summed HIP-event time of the pipelined dirty-chunk re-sweeps */
  int64_t pipelined;       /* 1 = the last call overlapped each pass's sweep with the previous commit; 2 = its
                              select too, the lists patched after the commit (monotone plugin sets) */
  int64_t pre_reserves;    /* Reserves whose NodeNUMAResource / DeviceShare allocation was computed ahead of the commit
                              (the pod's node ranked in its snapshot top) */
  int64_t commit_lds_bytes; /* the commit kernel's LDS image for this context (of the CU's 160 KB) */
  int64_t commit_helpers;   /* 1 = the NUMA-policy + DeviceShare commit ran its helper waves (their region fit the LDS
                               next to the slot caches; 0 = wave 0 computed the device hints itself) */
} ks_stats;

/* ---- preemption: the ElasticQuota PostFilter ----
 * NodeInfo.Pods of every node, the victims pool of the dry runs (one row per running pod; rows of a node in any
 * order).  The host resolves each pod's quota (getPodAssociateQuotaName, elasticquota/plugin_helper.go:41-61) to a
 * quota row of ks_load_quotas and its PodDisruptionBudget (filterPodsWithPDBViolation's namespace + selector match,
 * preempt.go:222-265) to indices of ks_load_node_pods' pdb_allowed: every PDB whose namespace and selector match and whose
 * DisruptedPods does not list the pod, in any order (`pdb`, then `pdb_more[k]`; -1 = none; an index listed twice for
 * one pod is KS_EINVAL).  The shim keeps the reference PostFilter when some pod matches more than 1 + KS_NPOD_MORE_PDBS
 * budgets. */
#define KS_NPOD_MORE_PDBS 3
#define KS_NPOD_NONPREEMPTIBLE 0x1u /* extension.IsPodNonPreemptible: never a victim (preempt.go:284-287) */
#define KS_NPOD_IN_QUOTA 0x2u       /* quotaInfo.IsPodExist (the pod is in its quota's PodCache): the dry run's
                                       quota used follows its removal / re-add (elasticquota/plugin.go:263-301) */
#define KS_NPOD_TERMINATING 0x4u    /* DeletionTimestamp != nil (PodEligibleToPreemptOthers, preempt.go:80-90) */
typedef struct ks_node_pod_cols {
  const int32_t *node;         /* node row (NodeInfo) */
  const int32_t *priority;     /* corev1helpers.PodPriority */
  const int64_t *start_time;   /* util.GetPodStartTime, any monotone unit (e.g. unix ns) */
  const uint32_t *flags;       /* KS_NPOD_*; NULL = KS_NPOD_IN_QUOTA */
  const int32_t *quota;        /* quota row, -1 = none (never a victim: the preemptor has a quota) */
  const int32_t *pdb;          /* PodDisruptionBudget index, -1 = none; NULL = none */
  /* the pod's part of NodeInfo.Requested (upstream computePodResourceRequest), removed / re-added by the dry run */
  const int64_t *req_milli_cpu;
  const int64_t *req_memory;
  const int64_t *req_ephemeral;
  const int64_t *req_scalar[KS_MAX_SCALARS]; /* NULL = 0 */
  const int64_t *quota_req[KS_QUOTA_DIMS];   /* core.PodRequestsAndLimits requests per quota dimension; NULL = 0 */
  const int32_t *pdb_more[KS_NPOD_MORE_PDBS]; /* further matching PDB indices of the pod, -1 = none; NULL = none */
} ks_node_pod_cols;

/* ks_preempt result (upstream preemption.Evaluator.Preempt, k8s v1.24 framework/preemption/preemption.go, driven by the
 * ElasticQuota plugin's SelectVictimsOnNode / PodEligibleToPreemptOthers / GetOffsetAndNumCandidates) */
#define KS_P_NOMINATED 0    /* Success: PostFilterResult.NominatedNodeName = node; delete the victims */
#define KS_P_NOT_ELIGIBLE 1 /* Unschedulable: PodEligibleToPreemptOthers refused (PreemptNever, or a terminating
                               lower-priority pod of the same quota on the nominated node) */
#define KS_P_NO_CANDIDATE 2 /* Unschedulable: no node where preemption helps (FitError) */
#define KS_P_ERROR 3        /* Error: no candidate and some node's dry run failed with an error (KS_PN_ERROR) */
typedef struct ks_preempt_result {
  int32_t node;               /* nominated node row, -1 = none */
  uint32_t status;            /* KS_P_* */
  int32_t num_victims;        /* len(Victims.Pods) of the chosen node */
  int32_t num_pdb_violations; /* Victims.NumPDBViolations */
  int32_t candidates;         /* nodes whose dry run found victims (len(candidates)) */
  int32_t potential_nodes;    /* nodesWherePreemptionMightHelp */
} ks_preempt_result;
/* per-node dry-run outcome (ks_preempt node_status) */
#define KS_PN_CANDIDATE 0   /* victims found: a candidate */
#define KS_PN_UNRESOLVABLE 1 /* the node's filter status was UnschedulableAndUnresolvable: not a potential node */
#define KS_PN_NO_VICTIMS 2  /* "No victims found on node" (UnschedulableAndUnresolvable) */
#define KS_PN_FILTER 3      /* the filters fail with every potential victim removed */
#define KS_PN_ERROR 4       /* Error: a victim removed twice (reprievePod's quota branch after a failed fit, preempt.go:192-199
                               after :180-186) or every potential victim reprieved ("expected at least one victim pod") */

typedef struct ks_ctx ks_ctx;

/* The layout this library was compiled with, for a binding to refuse a library built from another header (a stale
 * .so whose score-matrix width or struct sizes differ writes past the caller's buffers): out[0] = KS_ABI_VERSION,
 * out[1] = KS_NUM_SCORE_PLUGINS, then sizeof ks_config, ks_node_cols, ks_pod_cols, ks_quota_cols, ks_quota_tree,
 * ks_reservation_cols, ks_device_cols, ks_cpu_topology, ks_cpu_state_cols, ks_numa_node_cols, ks_result,
 * ks_node_state, ks_stats, ks_node_pod_cols, ks_preempt_result (KS_ABI_LAYOUT_WORDS words; n < that fills the first n).  Returns KS_ABI_LAYOUT_WORDS. */
#define KS_ABI_LAYOUT_WORDS 17
int ks_abi_layout(int64_t *out, int32_t n);

/* Returns KS_OK and *out on success.  On failure *out is NULL and
 * ks_last_error(NULL) describes the problem. */
int ks_create(const ks_config *cfg, ks_ctx **out);
void ks_destroy(ks_ctx *ctx);
const char *ks_last_error(const ks_ctx *ctx);

int ks_load_nodes(ks_ctx *ctx, const ks_node_cols *nodes, int64_t n);
/* Informer deltas: rows[i] replaces node idx[i]; arrays in `rows` have length m. */
int ks_update_nodes(ks_ctx *ctx, const int32_t *idx, const ks_node_cols *rows, int64_t m);
int ks_load_quotas(ks_ctx *ctx, const ks_quota_cols *quotas, int32_t q);

/* ---- informer deltas for the other tables (f1): rows replaced in place on the device, the rest of each table
 * untouched; idx / rows are distinct.  A batch of deltas is applied at a ks_schedule boundary (the snapshot
 * semantics); ks_checkpoint after them if the bench restores. ---- */
/* deviceshare nodeDeviceCache.updateNodeDevice (device_cache.go:489-527): rows[i] is node idx[i]'s devices;
 * KS_ESTATE for a node that holds a ks_assume'd device pod (see ks_assume) */
int ks_update_devices(ks_ctx *ctx, const int32_t *idx, const ks_device_cols *rows, int64_t m);
/* NodeResourceTopology / NodeAllocation changes (nodenumaresource topology_eventhandler.go, resource_manager.go
 * Update / Release): node idx[i]'s CPU state from row i, topology indices into the table of the last
 * ks_load_cpu_state */
int ks_update_cpu_state(ks_ctx *ctx, const int32_t *idx, const ks_cpu_state_cols *rows, int64_t m);
/* GroupQuotaManager OnQuotaUpdate / pod events (elasticquota/core/group_quota_manager.go:736-870): quota idx[i]'s
 * limit, min, used, non-preemptible used and masks from row i (the parents stay; a tree change is ks_load_quotas) */
int ks_update_quotas(ks_ctx *ctx, const int32_t *idx, const ks_quota_cols *rows, int32_t m);
/* reservation cache updates of loaded reservations (reservation/cache.go:104-216): the allocated amounts
 * (allocated[d][i], d < KS_RSV_DIMS as in ks_reservation_cols) and assigned-pod counts of the caller rows rows[i]; the
 * nodes' reservation restore and owner classes follow.  Adding or removing a reservation is ks_load_reservations. */
int ks_update_reservation_usage(ks_ctx *ctx, const int32_t *rows, const int64_t *const *allocated,
                                const int32_t *assigned, int32_t m);

/* GPU devices of the loaded nodes (deviceshare nodeDeviceCache, device_cache.go:44-160); call after
 * ks_load_nodes.  Reserve (plugin.go:377-430 -> updateCacheUsed) adds each allocation to used. */
int ks_load_devices(ks_ctx *ctx, const ks_device_cols *dev, int64_t n);
/* used amounts after commits, [k*n + node] for minor k; NULL = skip */
int ks_read_devices(ks_ctx *ctx, int64_t *used_core, int64_t *used_memory, int64_t *used_ratio);
/* RDMA used amounts after commits, [k*n + node] for minor k */
int ks_read_devices_rdma(ks_ctx *ctx, int64_t *used_rdma);

/* CPU topologies and per-node CPU allocation state for cpuset pods (NodeNUMAResource
 * resourceManager / NodeAllocation, resource_manager.go:58-401); call after ks_load_nodes.  Reserve of
 * a KS_POD_CPU_BIND pod allocates its CPUs with the CPU accumulator (takeCPUs, cpu_accumulator.go:86-232)
 * and adds them to the node's allocation (NodeAllocation.addPodAllocation, node_allocation.go:75-100). */
int ks_load_cpu_state(ks_ctx *ctx, const ks_cpu_topology *topologies, int32_t ntopo, const ks_cpu_state_cols *state);
/* NUMA node resources of the nodes with a NUMA topology policy (policy in ks_node_cols.numa_flags); call
 * after ks_load_nodes.  Pods on such nodes go through the hint providers, the topology manager merge
 * and the NUMA allocation; Reserve adds the allocation to used. */
int ks_load_numa_nodes(ks_ctx *ctx, const ks_numa_node_cols *numa);
/* used amounts after commits, [node*KS_MAX_NUMA + k]; NULL = skip */
/* informer delta for the NUMA-node table (NodeResourceTopology / NodeAllocation changes, topology_eventhandler.go,
 * node_allocation.go): row i of rows ([i*KS_MAX_NUMA + k]) replaces node idx[i]'s NUMA-node resources, allocated
 * resources and cpuset CPUs; the available CPUs per NUMA node follow from the loaded CPU state.  KS_ESTATE when no
 * NUMA-node table is loaded; ks_checkpoint again afterwards if the caller restores. */
int ks_update_numa_nodes(ks_ctx *ctx, const int32_t *idx, const ks_numa_node_cols *rows, int64_t m);
int ks_read_numa_nodes(ks_ctx *ctx, int64_t *used_cpu, int64_t *used_memory);
/* CPU sets after commits, [node*KS_CPU_WORDS + w]; NULL = skip */
int ks_read_cpu_state(ks_ctx *ctx, uint64_t *allocated, uint64_t *excl_pcpu, uint64_t *excl_numa);
/* The CPUs allocated to each pod of the last ks_schedule / ks_schedule_staged call ([pod*KS_CPU_WORDS + w],
 * zero for pods without a cpuset), the PodAllocation.CPUSet written by PreBind */
int ks_fetch_cpusets(ks_ctx *ctx, uint64_t *out, int32_t p);

/* Reservation cache snapshot (reservation/cache.go:104-291) for the Reservation plugin's
 * BeforePreFilter restore (transformer.go:41-307), Filter (plugin.go:311-496), PreScore
 * nomination (scoring.go:42-101, nominator.go:134-192), Score/NormalizeScore (scoring.go:103-203)
 * and Reserve (plugin.go:532-570 -> cache.go:171-192 -> reservation_info.go:379-388).
 * Node columns stay the reference's NodeInfo (reserve pods included); call after ks_load_nodes. */
int ks_load_reservations(ks_ctx *ctx, const ks_reservation_cols *rsv, int32_t r);
/* Reservation informer events between cycles (reservationCache updateReservation / deleteReservation,
 * reservation/cache.go:104-216).  ks_add_reservations appends r rows; they get the caller rows *first_row ..
 * *first_row + r - 1 (ks_result.reservation, ks_read_reservations, ks_update_reservation_usage use them).
 * ks_delete_reservations removes caller rows; their numbers are not reused and read back as zeros.  Both keep the
 * Allocated / assigned state of the other rows (commits included) and re-derive the node columns' reservation
 * base restore; ks_checkpoint again afterwards if the caller restores. */
int ks_add_reservations(ks_ctx *ctx, const ks_reservation_cols *rsv, int32_t r, int32_t *first_row);
int ks_delete_reservations(ks_ctx *ctx, const int32_t *rows, int32_t m);
/* Allocated (r*KS_RSV_DIMS, row-major) and len(AssignedPods) after commits; NULL = skip. */
int ks_read_reservations(ks_ctx *ctx, int64_t *allocated, int32_t *assigned);
/* The assigned pods' device allocations on each reservation's minors after commits ([r*KS_DEV_WORDS + w], the
 * layout of ks_reservation_cols.dev_allocated; zeros without device-holding reservations) */
int ks_read_reservation_devices(ks_ctx *ctx, int64_t *dev_allocated);

/* RefreshRuntime for every quota of the tree at once, on the device
 * (replaces GroupQuotaManager.RefreshRuntime, group_quota_manager.go:259-326, with the request
 * aggregation of recursiveUpdateGroupTreeWithDeltaRequest :184-226 and the water-filling of
 * runtime_quota_calculator.go:111-168).  runtime[i*KS_QUOTA_DIMS+d] and runtime_mask[i] (the
 * calculators' resource keys = union of all Max keys) are written when non-NULL.  When quotas
 * with the same row count are loaded, the runtime also becomes their admission limit
 * (ElasticQuota PreFilter with EnableRuntimeQuota, plugin.go:221-223 / plugin_helper.go:314-319). */
int ks_refresh_quota_runtime(ks_ctx *ctx, const ks_quota_tree *tree, int32_t q, int64_t *runtime,
                             uint32_t *runtime_mask);

/* Schedule `p` pods in order with commits; out[i] for pod i. Host buffers. */
int ks_schedule(ks_ctx *ctx, const ks_pod_cols *pods, int32_t p, ks_result *out);

/* Device-resident variant: stage pods once (host buffers copied to HBM), then
 * schedule the staged batch; results stay in HBM until ks_fetch_results.  Every
 * ks_schedule_staged call starts from the staged columns (the pods' PreFilter work — request
 * vectors, EstimatePod, flags — runs on the device as part of the call), so a staged queue can be
 * scheduled repeatedly (e.g. after ks_restore). */
int ks_stage_pods(ks_ctx *ctx, const ks_pod_cols *pods, int32_t p);
int ks_schedule_staged(ks_ctx *ctx);
int ks_fetch_results(ks_ctx *ctx, ks_result *out, int32_t p);

/* Snapshot save/restore of the mutable node + quota state (for repeatable benches). */
int ks_checkpoint(ks_ctx *ctx);
int ks_restore(ks_ctx *ctx);

/* ---- per-pod framework mode (INTEGRATION.md "per-pod drop-in"): the Go framework keeps its own
 * scheduleOne and calls the plugins' PreFilter/Filter/Score through ks_eval_pod, selects the node, then reports
 * Reserve (ks_assume) and, when Reserve of another plugin, Permit or Bind fails, Unreserve (ks_unreserve). ---- */

/* Evaluate pod 0 of `pod` against every node without Reserve (PreFilter + Filter + Score +
 * NormalizeScore of every enabled plugin; upstream findNodesThatPassFilters + prioritizeNodes).
 * reasons[n] gets KS_R_* bits (0 = feasible); scores[n*KS_NUM_SCORE_PLUGINS+k]
 * the un-weighted plugin-k score (0 for infeasible nodes); total[n] the weighted
 * sum (-1 for infeasible). Any output pointer may be NULL.  Writes only into the caller's buffers; its
 * device scratch lives with the context (no per-call allocation). */
int ks_eval_pod(ks_ctx *ctx, const ks_pod_cols *pod, uint32_t *reasons, int64_t *scores, int64_t *total);
/* the same entry under its round-1 name */
int ks_eval_pod_debug(ks_ctx *ctx, const ks_pod_cols *pod, uint32_t *reasons, int64_t *scores,
                      int64_t *total);

/* Reserve of pod 0 of `pod` on `node`, which the framework chose: every enabled plugin's Reserve
 * (load_aware.go:260; elasticquota/plugin.go:323-335; reservation/plugin.go:532-570 with NominateReservation on
 * the node; deviceshare/plugin.go:377-430; nodenumaresource/plugin.go:375-419) plus the scheduler cache's
 * AssumePod (NodeInfo.AddPod).  No Filter and no quota admission run.  out: status KS_S_SCHEDULED or
 * KS_S_RESERVE_FAILED (NodeNUMAResource could not allocate the cpuset; nothing changed), the reservation row
 * and the GPU / RDMA minors; score is 0.  cpuset (optional): the pod's CPUs [KS_CPU_WORDS]; numa_alloc
 * (optional): its NUMA-node allocation [KS_MAX_NUMA][2] (cpu milli, memory) on a NUMA-policy node.  Keep them
 * for ks_unreserve.  The assume reuses the batch's cpuset / NUMA buffers: ks_fetch_cpusets and ks_fetch_numa_alloc
 * return KS_ESTATE until the next ks_schedule*.  A node holding an assumed device pod refuses ks_update_devices
 * (KS_ESTATE) until the pod is ks_unreserve'd, because Unreserve derives the per-instance request from the node's
 * device totals (devicehandler_gpu.go:40-98), which must be the ones Reserve saw. */
int ks_assume(ks_ctx *ctx, const ks_pod_cols *pod, int32_t node, ks_result *out, uint64_t *cpuset,
              int64_t *numa_alloc);

/* Unreserve of every plugin (load_aware.go:265; elasticquota/plugin.go:339; reservation/plugin.go:572;
 * deviceshare/plugin.go:432; nodenumaresource/plugin.go:421 -> NodeAllocation.release node_allocation.go:105-131)
 * plus the cache's ForgetPod, for pod 0 of `pod` placed as `r` says (a ks_assume or ks_schedule result with
 * status KS_S_SCHEDULED) with the CPUs `cpuset` and NUMA allocation `numa_alloc` it got (either may be NULL
 * when the pod has none). */
int ks_unreserve(ks_ctx *ctx, const ks_pod_cols *pod, const ks_result *r, const uint64_t *cpuset,
                 const int64_t *numa_alloc);

/* The NUMA-node allocation [p][KS_MAX_NUMA][2] of the last ks_schedule* call's first p pods (zeros off
 * NUMA-policy nodes). */
int ks_fetch_numa_alloc(ks_ctx *ctx, int64_t *out, int32_t p);

int ks_read_nodes(ks_ctx *ctx, ks_node_state *out);
int ks_read_quota_used(ks_ctx *ctx, int64_t *used /* q*KS_QUOTA_DIMS, row-major */);
int ks_get_stats(const ks_ctx *ctx, ks_stats *out);
/* Turn the per-kernel HIP-event bracketing (ks_config.profile) on or off for later calls: the events
 * add dispatch gaps between the pass kernels, so throughput is timed with them off and the kernel split
 * from separate profiled calls. */
int ks_set_profile(ks_ctx *ctx, int32_t on);
/* Pipelined passes: each pass's sweep runs on a second stream while the previous pass
 * commits, then the chunks that commit wrote are re-swept, so results are identical either way.
 * mode 0 = off, 1 = automatic (clusters of at least 32,768 nodes; env KS_PIPE_MIN_NODES), 2 = always
 * (plugin sets without DeviceShare / NodeNUMAResource only). */
int ks_set_pipeline(ks_ctx *ctx, int32_t mode);

/* Node sharding over GPUs (one process per GPU).  The node table stays replicated
 * (every rank applies the same commits); shard s = rank * virtual_shards + v sweeps and selects
 * over its contiguous node-chunk range, the per-shard top-K candidate lists are exchanged with
 * one RCCL allgather per pass, and a merge kernel rebuilds exactly the list a single sweep would
 * give, so placements are identical for any shard count.  Replaces the reference's single-process
 * Parallelizer over nodes (pkg/util/parallelize/parallelism.go:29-49 / upstream
 * findNodesThatPassFilters + prioritizeNodes).  ks_shard_unique_id is called on rank 0 and the
 * bytes broadcast by the host; virtual_shards > 1 splits one GPU's range into several shards
 * (exercises the merge on one GPU). */
/* ---- preemption (ElasticQuota PostFilter, pkg/scheduler/plugins/elasticquota/plugin.go:302-321, preempt.go) ---- */
/* NodeInfo.Pods of every loaded node (replaces the table; m rows) and the PodDisruptionBudgets' DisruptionsAllowed
 * (npdb entries).  Call after ks_load_nodes; refresh at a ks_schedule boundary from the informer's pod events
 * (including the pods ks_schedule placed). */
int ks_load_node_pods(ks_ctx *ctx, const ks_node_pod_cols *pods, int64_t m, const int32_t *pdb_allowed, int32_t npdb);
/* PostFilter of pod 0 of `pod` (priority `priority`, flags KS_PREEMPT_*, nominated node row or -1) after a failed
 * scheduling cycle: unresolvable[n] != 0 for the nodes whose filter status was UnschedulableAndUnresolvable (NULL =
 * none, e.g. an ElasticQuota PreFilter rejection, which gives every node Unschedulable).  Every node's dry run
 * (SelectVictimsOnNode: the same-quota lower-priority preemptible pods removed, the Filter plugins, the PDB split, the
 * reprieve loop with the quota check) runs on the device; the candidate is chosen as pickOneNodeForPreemption does,
 * remaining ties to the lowest node row.  victims[0..min(cap, num_victims)) get the chosen node's victims as rows of
 * the ks_load_node_pods table, in Victims.Pods order; node_status[n] (optional) the KS_PN_* of every node.  Nothing
 * is changed: the caller deletes the victims (prepareCandidate) and refreshes the tables.  Supported with Fit,
 * LoadAware, ElasticQuota (required; the pod needs a quota row), BalancedAllocation, TaintToleration and NodeAffinity;
 * Reservation, NodeNUMAResource, DeviceShare and NodePorts (filters that read other pods of the node) give
 * KS_EUNSUPPORTED.  ks_get_stats afterwards: sweep_bytes = the dry-run launch's algorithmic bytes and, with
 * ks_set_profile on, sweep_ms / select_ms / total_ms = the dry-run kernel, the selection kernel, both. */
#define KS_PREEMPT_NEVER 0x1u /* pod.Spec.PreemptionPolicy == Never */
int ks_preempt(ks_ctx *ctx, const ks_pod_cols *pod, int32_t priority, uint32_t flags, int32_t nominated_node,
               const uint8_t *unresolvable, ks_preempt_result *out, int32_t *victims, int32_t victims_cap,
               uint8_t *node_status);

int ks_shard_unique_id(uint8_t *out /* KS_SHARD_ID_BYTES */);
/* Node sharding over nranks processes (one per GPU): this rank sweeps its chunk range as virtual_shards
 * shards; the per-shard candidates are exchanged by one ncclAllGather per pass and the normalization maxima by one
 * ncclAllReduce(max), on an RCCL communicator made from rank 0's ks_shard_unique_id.  nranks == 1 with a unique id
 * makes a one-rank communicator, so the RCCL exchange calls run on a single GPU (with virtual_shards > 1); nranks == 1
 * without one shards virtually with no exchange. */
int ks_shard_init(ks_ctx *ctx, int32_t nranks, int32_t rank, const uint8_t *unique_id, int32_t virtual_shards);
/* Test transport for the nranks > 1 path without RCCL: ctxs[0..nranks) (contexts of this process, each loaded with the
 * same node table, batch and candidate count) become ranks 0..nranks-1 of one sharded group whose candidate allgather
 * and normalization-max all-reduce are device copies between the contexts' buffers, ordered by host barriers and HIP
 * events.  Every rank's ks_schedule* must then be called concurrently, each from its own host thread (a rank waits at
 * most 120 s for its peers, then fails with KS_EHIP).  Everything else -- rank chunk ranges, the rank-offset gather
 * slots, merge_kernel, the replicated commits -- is the RCCL path's code.  ks_shard_init or ks_destroy leaves the
 * group. */
int ks_shard_init_loopback(ks_ctx *const *ctxs, int32_t nranks, int32_t virtual_shards);

#ifdef __cplusplus
}
#endif
#endif /* KOORDGPU_H */
