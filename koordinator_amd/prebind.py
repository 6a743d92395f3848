"""PreBind write-back: the annotations koord-scheduler's PreBind writes, materialised from what
ks_schedule / ks_assume return (ks_result.node / reservation / gpu_minors / rdma_minors, ks_fetch_cpusets,
ks_fetch_numa_alloc).  The Go shim writes the same strings with the reference's own helpers; this module is the
host-side mirror the tests and the Python callers use.

* NodeNUMAResource PreBind (``nodenumaresource/plugin.go:439-478``): ``scheduling.koordinator.sh/resource-status``
  = ``json.Marshal(ResourceStatus)`` (``apis/extension/numa_aware.go:71-82``, ``SetResourceStatus`` :232-248):
  ``cpuset`` (Linux CPU list, omitted when empty) and ``numaNodeResources`` (per allocated NUMA node, omitted when
  none).
* DeviceShare PreBind (``deviceshare/plugin.go:490-503``): ``scheduling.koordinator.sh/device-allocated`` =
  ``json.Marshal(DeviceAllocations)`` (``apis/extension/device_share.go:151-165``), one entry per allocated minor
  holding the per-instance request (``devicehandler_gpu.go:56-63``: gpu-core and gpu-memory-ratio DecimalSI,
  gpu-memory BinarySI; ``devicehandler_default.go:58``: rdma DecimalSI).
* Reservation PreBind: ``scheduling.koordinator.sh/reservation-allocated`` = ``{"name": .., "uid": ..}``.
* NodeNUMAResource PreBind of a cpu-bind pod also writes ``scheduling.koordinator.sh/resource-spec`` back when the
  pod did not state the policy the scheduler enforced (``appendResourceSpecIfMissed``, ``plugin.go:552-578``).

Go's ``encoding/json`` sorts map keys and writes no spaces; Kubernetes ``resource.Quantity`` marshals as its
canonical string (``Quantity.String``), restated in ``quantity_string``.
"""
from __future__ import annotations

import json
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

ANNOTATION_RESOURCE_STATUS = "scheduling.koordinator.sh/resource-status"
ANNOTATION_DEVICE_ALLOCATED = "scheduling.koordinator.sh/device-allocated"
ANNOTATION_RESERVATION_ALLOCATED = "scheduling.koordinator.sh/reservation-allocated"
ANNOTATION_RESOURCE_SPEC = "scheduling.koordinator.sh/resource-spec"

CPU_BIND_POLICY_DEFAULT = "Default"
CPU_BIND_POLICY_FULL_PCPUS = "FullPCPUs"
CPU_BIND_POLICY_SPREAD_BY_PCPUS = "SpreadByPCPUs"
NODE_CPU_BIND_POLICY_FULL_PCPUS_ONLY = "FullPCPUsOnly"
NODE_CPU_BIND_POLICY_SPREAD_BY_PCPUS = "SpreadByPCPUs"

RESOURCE_GPU_CORE = "koordinator.sh/gpu-core"
RESOURCE_GPU_MEMORY = "koordinator.sh/gpu-memory"
RESOURCE_GPU_MEMORY_RATIO = "koordinator.sh/gpu-memory-ratio"
RESOURCE_RDMA = "koordinator.sh/rdma"

_DEC_SUFFIX = {-3: "m", 0: "", 3: "k", 6: "M", 9: "G", 12: "T", 15: "P", 18: "E"}
_BIN_SUFFIX = ["", "Ki", "Mi", "Gi", "Ti", "Pi", "Ei"]


def quantity_string(value: int, fmt: str = "DecimalSI", milli: bool = False) -> str:
    """Canonical ``resource.Quantity`` string of an integer amount (``value`` in units, or in thousandths with
    ``milli``), as ``Quantity.String`` / ``CanonicalizeBytes`` print it (k8s.io/apimachinery
    pkg/api/resource/quantity.go): DecimalSI picks the largest power-of-1000 exponent (from m up to E) that leaves
    an integral mantissa; BinarySI uses the largest power of 1024 that divides the value exactly, and prints as
    DecimalSI when |value| < 1024 or the value is not a whole number of units."""
    v = int(value)
    if fmt == "BinarySI" and not (milli and v % 1000):
        units = v // 1000 if milli else v
        if abs(units) >= 1024:
            e = 0
            while e < len(_BIN_SUFFIX) - 1 and units % 1024 == 0 and units != 0:
                units //= 1024
                e += 1
            return f"{units}{_BIN_SUFFIX[e]}"
    if fmt not in ("DecimalSI", "BinarySI"):
        raise ValueError(f"unsupported quantity format {fmt!r}")
    # DecimalSI: mantissa * 10^exp with exp a multiple of 3, as large as keeps the mantissa integral
    mant, exp = (v, -3) if milli else (v, 0)
    if mant == 0:
        return "0"
    while exp < 18 and mant % 1000 == 0:
        mant //= 1000
        exp += 3
    return f"{mant}{_DEC_SUFFIX[exp]}"


def cpuset_string(cpus: Iterable[int]) -> str:
    """``cpuset.CPUSet.String``: sorted CPU ids as a Linux list, runs of consecutive ids as ``a-b``."""
    ids = sorted(set(int(c) for c in cpus))
    out: List[str] = []
    i = 0
    while i < len(ids):
        j = i
        while j + 1 < len(ids) and ids[j + 1] == ids[j] + 1:
            j += 1
        out.append(str(ids[i]) if i == j else f"{ids[i]}-{ids[j]}")
        i = j + 1
    return ",".join(out)


def _marshal(obj) -> str:
    return json.dumps(obj, separators=(",", ":"), sort_keys=True)


def resource_status(cpus: Sequence[int] = (), numa_nodes: Sequence[Tuple[int, int, int]] = ()) -> str:
    """resource-status annotation.  ``cpus``: the pod's CPU ids (``ks_fetch_cpusets``); ``numa_nodes``: per
    allocated NUMA node ``(node, cpu_milli, memory_bytes)`` (``ks_fetch_numa_alloc``; zero amounts are left out of
    the resource list, a node with neither is skipped).  Field order is the struct's (cpuset, numaNodeResources)."""
    st: Dict[str, object] = {}
    cs = cpuset_string(cpus)
    if cs:
        st["cpuset"] = cs
    res = []
    for node, cpu_milli, mem in numa_nodes:
        rl = {}
        if cpu_milli:
            rl["cpu"] = quantity_string(cpu_milli, "DecimalSI", milli=True)
        if mem:
            rl["memory"] = quantity_string(mem, "BinarySI")
        if rl:
            res.append({"node": int(node), "resources": dict(sorted(rl.items()))})
    if res:
        st["numaNodeResources"] = res
    # struct fields keep declaration order (json.Marshal of a struct); only the maps inside are sorted
    return json.dumps(st, separators=(",", ":"))


def _minors(mask: int) -> List[int]:
    return [k for k in range(32) if (int(mask) >> k) & 1]


def device_allocated(gpu_minors: int = 0, gpu_core: Optional[int] = None, gpu_memory: int = 0,
                     gpu_memory_ratio: int = 0, rdma_minors: int = 0, rdma: int = 0, *,
                     gpu_memory_format: str = "BinarySI", gpu_order: Optional[Sequence[int]] = None,
                     rdma_order: Optional[Sequence[int]] = None) -> str:
    """device-allocated annotation from the ``ks_result`` minor masks and the pod's per-instance request
    (``CalcDesiredRequestsAndCount``, ``devicehandler_gpu.go:40-64`` / ``devicehandler_default.go:58``).

    * Several GPUs (memory ratio > 100 and a multiple of 100): the per-instance list is rebuilt with all three
      names, so gpu-core is present (``gpuCore.Value()/desiredCount``, 0 when the pod asked for none), gpu-memory
      BinarySI and the ratio DecimalSI.
    * One GPU: the pod's own request list after ``fillGPUTotalMem``: gpu-core only when the pod asked for it
      (``gpu_core`` None otherwise), gpu-memory in the pod's own Quantity format when the pod gave bytes
      (``gpu_memory_format``; BinarySI when it was derived from the ratio by ``memoryRatioToBytes``).
    * Entries follow the allocation order, ``sortDeviceResourcesByMinor`` (``device_allocator.go:415-433``:
      preferred first, then device score descending, then minor).  ``gpu_order`` / ``rdma_order`` give it when the
      caller has it; without them minors ascend, which is the reference's order whenever the allocated devices
      scored alike (e.g. all free) and otherwise differs only in the order of the list's entries.
    """
    def ordered(mask: int, order: Optional[Sequence[int]]) -> List[int]:
        ms = _minors(mask)
        if order is None:
            return ms
        o = [int(m) for m in order]
        if sorted(o) != ms:
            raise ValueError(f"allocation order {o} does not list the minors of mask {mask:#x}")
        return o

    alloc: Dict[str, list] = {}
    if gpu_minors:
        multi = bin(int(gpu_minors)).count("1") > 1  # one instance per minor: desiredCount > 1
        rl = {RESOURCE_GPU_MEMORY: quantity_string(gpu_memory, "BinarySI" if multi else gpu_memory_format),
              RESOURCE_GPU_MEMORY_RATIO: quantity_string(gpu_memory_ratio, "DecimalSI")}
        if gpu_core is not None or multi:
            rl[RESOURCE_GPU_CORE] = quantity_string(gpu_core or 0, "DecimalSI")
        alloc["gpu"] = [{"minor": m, "resources": rl} for m in ordered(gpu_minors, gpu_order)]
    if rdma_minors:
        # (a joint [gpu, rdma] pod without an RDMA request gets RDMA devices with a nil request list: null)
        alloc["rdma"] = [{"minor": m, "resources": {RESOURCE_RDMA: quantity_string(rdma, "DecimalSI")} if rdma else None}
                         for m in ordered(rdma_minors, rdma_order)]
    return _marshal(alloc)


def reservation_allocated(name: str, uid: str) -> str:
    """reservation-allocated annotation (``apiext.ReservationAllocated``: name, uid in declaration order)."""
    return json.dumps({"name": name, "uid": uid}, separators=(",", ":"))


def cpu_bind_policy(state_required: str, state_preferred: str, node_policy: str = "") -> Tuple[str, bool]:
    """``getCPUBindPolicy`` (``nodenumaresource/util.go:85-103``): the pod's required policy wins; otherwise the
    node's CPU bind policy label (``FullPCPUsOnly`` / ``SpreadByPCPUs``; a static kubelet CPU manager with
    ``full-pcpus-only`` is the caller's ``FullPCPUsOnly``) makes the policy required; otherwise the PreFilter's
    preferred policy (the plugin default already filled in for ``Default``), not required."""
    if state_required:
        return state_required, True
    if node_policy == NODE_CPU_BIND_POLICY_SPREAD_BY_PCPUS:
        return CPU_BIND_POLICY_SPREAD_BY_PCPUS, True
    if node_policy == NODE_CPU_BIND_POLICY_FULL_PCPUS_ONLY:
        return CPU_BIND_POLICY_FULL_PCPUS, True
    return state_preferred, False


def resource_spec_json(spec: Dict[str, str]) -> str:
    """``json.Marshal(ResourceSpec)`` (``apis/extension/numa_aware.go:60-68``): the struct's field order, empty
    fields omitted."""
    out = {}
    for k in ("requiredCPUBindPolicy", "preferredCPUBindPolicy", "preferredCPUExclusivePolicy"):
        if spec.get(k):
            out[k] = spec[k]
    return json.dumps(out, separators=(",", ":"))


def resource_spec_writeback(existing: Optional[Dict[str, str]], state_required: str, state_preferred: str,
                            node_policy: str = "") -> Optional[Dict[str, str]]:
    """``appendResourceSpecIfMissed`` (``nodenumaresource/plugin.go:552-578``), run by PreBind for every pod that
    requests CPU binding on the chosen node (``requestCPUBind``).  ``existing`` is the pod's own resource-spec
    annotation (parsed; None when absent); ``state_required`` / ``state_preferred`` are the PreFilter state's
    policies (``plugin.go:238-261``: ``Default`` replaced by the plugin's DefaultCPUBindPolicy).  Returns the spec
    to write back, or None when the reference leaves the annotation alone."""
    policy, required = cpu_bind_policy(state_required, state_preferred, node_policy)
    spec = dict(existing or {})
    write = False
    if required and spec.get("requiredCPUBindPolicy", "") in ("", CPU_BIND_POLICY_DEFAULT):
        spec["requiredCPUBindPolicy"] = policy
        write = True
    if spec.get("preferredCPUBindPolicy", "") == CPU_BIND_POLICY_DEFAULT:
        spec["preferredCPUBindPolicy"] = policy
        write = True
    if not spec.get("requiredCPUBindPolicy") and not spec.get("preferredCPUBindPolicy") and policy:
        spec["preferredCPUBindPolicy"] = policy
        write = True
    return spec if write else None


def prebind_annotations(result, cpus: Sequence[int] = (), numa_nodes: Sequence[Tuple[int, int, int]] = (),
                        gpu_request: Optional[Tuple[Optional[int], int, int]] = None, rdma_request: int = 0,
                        reservation: Optional[Tuple[str, str]] = None,
                        cpu_bind: Optional[Tuple[Optional[Dict[str, str]], str, str, str]] = None) -> Dict[str, str]:
    """Every PreBind annotation of one scheduled pod: ``result`` is its ``ks_result`` row (a mapping or numpy
    record with ``gpu_minors`` / ``rdma_minors``); ``gpu_request`` = (core or None, memory bytes, ratio) per
    instance; ``reservation`` = (name, uid) of ``result.reservation``'s row when it is >= 0; ``cpu_bind`` =
    (the pod's resource-spec annotation parsed or None, PreFilter required policy, PreFilter preferred policy, the
    chosen node's CPU bind policy) for a pod that requests CPU binding there (``requestCPUBind``, which a cpuset in
    ``cpus`` implies) — NodeNUMAResource PreBind then also writes the resource-spec annotation back when
    ``appendResourceSpecIfMissed`` does (``plugin.go:460-464``)."""
    out: Dict[str, str] = {}
    if cpu_bind is not None:
        spec = resource_spec_writeback(*cpu_bind)
        if spec is not None:
            out[ANNOTATION_RESOURCE_SPEC] = resource_spec_json(spec)
    if len(cpus) or len(numa_nodes):
        out[ANNOTATION_RESOURCE_STATUS] = resource_status(cpus, numa_nodes)
    gm, rm = int(result["gpu_minors"]), int(result["rdma_minors"])
    if gm or rm:
        core, mem, ratio = gpu_request if gpu_request is not None else (None, 0, 0)
        out[ANNOTATION_DEVICE_ALLOCATED] = device_allocated(gm, core, mem, ratio, rm, rdma_request)
    if reservation is not None:
        out[ANNOTATION_RESERVATION_ALLOCATED] = reservation_allocated(*reservation)
    return out
