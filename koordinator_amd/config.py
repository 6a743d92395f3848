"""Plugin args mirrors with the reference's defaults and validation.

Each dataclass mirrors one args type of the reference so a host that already
holds a KubeSchedulerConfiguration profile can fill them field for field:

* ``LoadAwareSchedulingArgs``  pkg/scheduler/apis/config/types.go:30-62,
  defaults v1beta2/defaults.go:33-48,77-100, validation
  validation/validation_pluginargs.go:31-96.
* ``NodeResourcesFitArgs``     upstream k8s v1.24 NodeResourcesFitArgs
  (scoringStrategy), as configured by config/manager/scheduler-config.yaml:17-31.
* ``ElasticQuotaArgs``         pkg/scheduler/apis/config/types.go (EnableRuntimeQuota
  default true, EnableCheckParentQuota default false: v1beta2/defaults.go:70-71).

``SchedulerProfile.to_ks_config()`` lowers them to the C ABI ``ks_config``.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, Optional

from . import abi

CPU = "cpu"
MEMORY = "memory"
EPHEMERAL = "ephemeral-storage"
BATCH_CPU = "kubernetes.io/batch-cpu"
BATCH_MEMORY = "kubernetes.io/batch-memory"
GPU_CORE = "koordinator.sh/gpu-core"
GPU_MEMORY = "koordinator.sh/gpu-memory"
GPU_MEMORY_RATIO = "koordinator.sh/gpu-memory-ratio"
RDMA = "koordinator.sh/rdma"
FPGA = "koordinator.sh/fpga"

DEFAULT_NODE_METRIC_EXPIRATION_SECONDS = 180
DEFAULT_RESOURCE_WEIGHTS = {CPU: 1, MEMORY: 1}
DEFAULT_USAGE_THRESHOLDS = {CPU: 65, MEMORY: 95}
DEFAULT_ESTIMATED_SCALING_FACTORS = {CPU: 85, MEMORY: 70}


class ValidationError(ValueError):
    pass


@dataclass
class LoadAwareSchedulingArgs:
    filter_expired_node_metrics: Optional[bool] = None
    node_metric_expiration_seconds: Optional[int] = None
    resource_weights: Dict[str, int] = field(default_factory=dict)
    usage_thresholds: Dict[str, int] = field(default_factory=dict)
    prod_usage_thresholds: Dict[str, int] = field(default_factory=dict)
    score_according_prod_usage: bool = False
    estimator: str = ""
    estimated_scaling_factors: Optional[Dict[str, int]] = None
    # Aggregated (types.go:64-78): usage thresholds + aggregation type/duration
    aggregated_usage_thresholds: Dict[str, int] = field(default_factory=dict)
    aggregated_usage_type: str = ""
    aggregated_usage_duration_s: int = 0
    aggregated_score_type: str = ""
    aggregated_score_duration_s: int = 0

    def set_defaults(self) -> "LoadAwareSchedulingArgs":
        """SetDefaults_LoadAwareSchedulingArgs (v1beta2/defaults.go:77-100)."""
        if self.filter_expired_node_metrics is None:
            self.filter_expired_node_metrics = True
        if self.node_metric_expiration_seconds is None:
            self.node_metric_expiration_seconds = DEFAULT_NODE_METRIC_EXPIRATION_SECONDS
        if not self.resource_weights:
            self.resource_weights = dict(DEFAULT_RESOURCE_WEIGHTS)
        if not self.usage_thresholds:
            self.usage_thresholds = dict(DEFAULT_USAGE_THRESHOLDS)
        if self.estimated_scaling_factors is None:
            self.estimated_scaling_factors = dict(DEFAULT_ESTIMATED_SCALING_FACTORS)
        else:
            for k, v in DEFAULT_ESTIMATED_SCALING_FACTORS.items():
                self.estimated_scaling_factors.setdefault(k, v)
        return self

    def validate(self) -> None:
        """ValidateLoadAwareSchedulingArgs (validation_pluginargs.go:31-96)."""
        if self.node_metric_expiration_seconds is not None and self.node_metric_expiration_seconds <= 0:
            raise ValidationError("nodeMetricExpiredSeconds should be a positive value")
        for r, w in self.resource_weights.items():
            if w <= 0 or w > 100:
                raise ValidationError(f"resource Weight of {r} should be in (0, 100], got {w}")
        for r, t in self.usage_thresholds.items():
            if t < 0 or t > 100:
                raise ValidationError(f"resource Threshold of {r} should be in [0, 100], got {t}")
        for r, t in (self.estimated_scaling_factors or {}).items():
            if t <= 0 or t > 100:
                raise ValidationError(f"estimated resource Threshold of {r} should be in (0, 100], got {t}")
        for r in self.resource_weights:
            if r not in (self.estimated_scaling_factors or {}):
                raise ValidationError(f"estimatedScalingFactors: {r} not found")

    def filter_with_aggregation(self) -> bool:
        """helper.go:92-94"""
        return bool(self.aggregated_usage_thresholds) and self.aggregated_usage_type != ""

    def score_with_aggregation(self) -> bool:
        """helper.go:96-98"""
        return self.aggregated_score_type != ""


@dataclass
class NodeResourcesFitArgs:
    strategy: str = "LeastAllocated"
    # scoringStrategy.resources; the koord-scheduler profile lists cpu, memory,
    # batch-cpu and batch-memory with weight 1 (scheduler-config.yaml:21-31)
    resources: Dict[str, int] = field(default_factory=lambda: {CPU: 1, MEMORY: 1})


@dataclass
class NodeNUMAResourceArgs:
    """NodeNUMAResourceArgs.ScoringStrategy after v1beta2 defaults (defaults.go:107-136)."""
    strategy: str = "LeastAllocated"
    resources: Dict[str, int] = field(default_factory=lambda: {CPU: 1, MEMORY: 1})
    # NUMAScoringStrategy.Type: the CPU accumulator's default NUMA allocate strategy
    # (GetDefaultNUMAAllocateStrategy, nodenumaresource/util.go:22-28)
    numa_scoring_strategy: str = "LeastAllocated"


@dataclass
class DeviceShareArgs:
    """DeviceShareArgs.ScoringStrategy after v1beta2 defaults (defaults.go:187-207): LeastAllocated,
    gpu-memory-ratio, rdma and fpga weight 1."""
    strategy: str = "LeastAllocated"
    resources: Dict[str, int] = field(default_factory=lambda: {GPU_MEMORY_RATIO: 1, RDMA: 1, FPGA: 1})


@dataclass
class NodeResourcesBalancedAllocationArgs:
    """Upstream NodeResourcesBalancedAllocationArgs (kube-scheduler v1.24 config/v1beta2 defaults: cpu and memory,
    weight 1; the weights do not enter balancedResourceScorer, only the resource set does)."""
    resources: Dict[str, int] = field(default_factory=lambda: {CPU: 1, MEMORY: 1})


@dataclass
class ElasticQuotaArgs:
    enable_runtime_quota: bool = True
    enable_check_parent_quota: bool = False


@dataclass
class SchedulerProfile:
    """One koord-scheduler profile restricted to the plugins the evaluator runs."""

    fit: Optional[NodeResourcesFitArgs] = field(default_factory=NodeResourcesFitArgs)
    fit_weight: int = 1
    loadaware: Optional[LoadAwareSchedulingArgs] = field(default_factory=LoadAwareSchedulingArgs)
    loadaware_weight: int = 1
    quota: Optional[ElasticQuotaArgs] = None
    reservation_weight: Optional[int] = None  # Reservation plugin score weight (koord profile: 5000); None = off
    numa: Optional[NodeNUMAResourceArgs] = None
    numa_weight: int = 1
    deviceshare: Optional[DeviceShareArgs] = None
    deviceshare_weight: int = 1
    balanced: Optional[NodeResourcesBalancedAllocationArgs] = None  # upstream default plugin; None = disabled
    balanced_weight: int = 1
    # upstream TaintToleration / NodeAffinity (v1beta2 default profile: both on, weight 1); the host compiles taints,
    # tolerations, node labels and node selectors into dictionary bits (static_plugins.compile_cluster)
    taint_toleration: bool = False
    taint_toleration_weight: int = 1
    node_affinity: bool = False
    node_affinity_weight: int = 1
    node_ports: bool = False  # upstream NodePorts (Filter only); host ports as dictionary bits (static_plugins)
    # upstream PodTopologySpread / InterPodAffinity (v1beta2 default profile: weights 2 and 1); the host compiles
    # selectors and affinity terms into per-node counters and per-pod query terms (topology_plugins.compile_topology)
    topology: bool = False
    topology_spread_weight: int = 2
    inter_pod_affinity_weight: int = 1
    scalar_slots: tuple = (BATCH_CPU, BATCH_MEMORY)  # scalar resource name per ks slot
    batch_pods: int = 0
    candidates: int = 0
    device: int = 0

    def __post_init__(self):
        if self.loadaware is not None:
            self.loadaware.set_defaults()
            self.loadaware.validate()

    def to_ks_config(self) -> abi.KsConfig:
        c = abi.KsConfig()
        c.abi_version = abi.KS_ABI_VERSION
        c.device = self.device
        c.batch_pods = self.batch_pods
        c.candidates = self.candidates
        if self.fit is not None:
            c.fit.enable_filter = 1
            c.fit.enable_score = 1 if self.fit_weight else 0
            strat = self.fit.strategy
            if strat == "LeastAllocated":
                c.fit.strategy = abi.KS_LEAST_ALLOCATED
            elif strat == "MostAllocated":
                c.fit.strategy = abi.KS_MOST_ALLOCATED
            else:
                raise ValidationError(f"unsupported NodeResourcesFit scoring strategy {strat}")
            for name, w in self.fit.resources.items():
                if name == CPU:
                    c.fit.weight_cpu = w
                elif name == MEMORY:
                    c.fit.weight_memory = w
                elif name == EPHEMERAL:
                    c.fit.weight_ephemeral = w
                elif name in self.scalar_slots:
                    c.fit.weight_scalar[self.scalar_slots.index(name)] = w
                else:
                    raise ValidationError(f"resource {name} has no scalar slot")
            c.fit.plugin_weight = self.fit_weight
        if self.loadaware is not None:
            la = self.loadaware
            c.loadaware.enable_filter = 1
            c.loadaware.enable_score = 1 if self.loadaware_weight else 0
            c.loadaware.filter_expired_node_metrics = 1 if la.filter_expired_node_metrics else 0
            c.loadaware.score_according_prod_usage = 1 if la.score_according_prod_usage else 0
            for name, w in la.resource_weights.items():
                if name not in (CPU, MEMORY):
                    raise ValidationError(f"LoadAware weight on {name} is not supported (cpu/memory only)")
            c.loadaware.weight_cpu = la.resource_weights.get(CPU, 0)
            c.loadaware.weight_memory = la.resource_weights.get(MEMORY, 0)
            c.loadaware.scaling_cpu = la.estimated_scaling_factors.get(CPU, 0)
            c.loadaware.scaling_memory = la.estimated_scaling_factors.get(MEMORY, 0)
            c.loadaware.plugin_weight = self.loadaware_weight
        if self.numa is not None:
            c.numa.enable = 1
            c.numa.strategy = abi.KS_MOST_ALLOCATED if self.numa.strategy == "MostAllocated" else abi.KS_LEAST_ALLOCATED
            for name, w in self.numa.resources.items():
                if name not in (CPU, MEMORY):
                    raise ValidationError(f"NodeNUMAResource weight on {name} is not supported (cpu/memory only)")
            c.numa.weight_cpu = self.numa.resources.get(CPU, 0)
            c.numa.weight_memory = self.numa.resources.get(MEMORY, 0)
            c.numa.plugin_weight = self.numa_weight
            c.numa.numa_scoring_strategy = (abi.KS_MOST_ALLOCATED if self.numa.numa_scoring_strategy == "MostAllocated"
                                            else abi.KS_LEAST_ALLOCATED)
        if self.deviceshare is not None:
            d = self.deviceshare
            c.deviceshare.enable = 1
            c.deviceshare.strategy = abi.KS_MOST_ALLOCATED if d.strategy == "MostAllocated" else abi.KS_LEAST_ALLOCATED
            for name in d.resources:
                if name not in (GPU_CORE, GPU_MEMORY, GPU_MEMORY_RATIO, RDMA, FPGA):
                    raise ValidationError(f"DeviceShare weight on {name} is not supported")
            c.deviceshare.weight_gpu_core = d.resources.get(GPU_CORE, 0)
            c.deviceshare.weight_gpu_memory = d.resources.get(GPU_MEMORY, 0)
            c.deviceshare.weight_gpu_memory_ratio = d.resources.get(GPU_MEMORY_RATIO, 0)
            c.deviceshare.weight_rdma = d.resources.get(RDMA, 0)
            c.deviceshare.plugin_weight = self.deviceshare_weight
        if self.balanced is not None:
            c.balanced.enable = 1
            for name in self.balanced.resources:
                if name == CPU:
                    c.balanced.resources |= abi.KS_BAL_CPU
                elif name == MEMORY:
                    c.balanced.resources |= abi.KS_BAL_MEMORY
                else:
                    raise ValidationError(f"NodeResourcesBalancedAllocation on {name} is not supported (cpu/memory only)")
            c.balanced.plugin_weight = self.balanced_weight
        if self.taint_toleration:
            c.taint.enable_filter = 1
            c.taint.enable_score = 1 if self.taint_toleration_weight else 0
            c.taint.plugin_weight = self.taint_toleration_weight
        if self.node_affinity:
            c.affinity.enable_filter = 1
            c.affinity.enable_score = 1 if self.node_affinity_weight else 0
            c.affinity.plugin_weight = self.node_affinity_weight
        if self.node_ports:
            c.nodeports.enable_filter = 1
        if self.topology:
            c.topology.enable = 1
            c.topology.spread_weight = self.topology_spread_weight
            c.topology.affinity_weight = self.inter_pod_affinity_weight
        if self.reservation_weight is not None:
            c.reservation.enable = 1
            c.reservation.plugin_weight = int(self.reservation_weight)
        if self.quota is not None:
            c.quota.enable = 1
            c.quota.enable_check_parent_quota = 1 if self.quota.enable_check_parent_quota else 0
        return c
