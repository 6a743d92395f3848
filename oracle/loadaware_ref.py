"""Pure-Python restatement of the LoadAwareScheduling plugin at object level.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Small cases only: this is
the reference's per-call logic on one node, used to check the golden vectors in
tests/golden/ and the host-side reduction in koordinator_amd/ingest.py.

Restated from (paths relative to the reference root):
  Filter                      pkg/scheduler/plugins/loadaware/load_aware.go:123-254
  Score                       load_aware.go:269-397
  helpers                     loadaware/helper.go:36-196
  EstimatePod / EstimateNode  loadaware/estimator/default_estimator.go:57-129
  priority class              apis/extension/priority_utils.go:26-47, priority.go:71-100,
                              qos_utils.go:30-84
  resource name translation   apis/extension/resource.go:40-58
  custom thresholds           apis/extension/load_aware.go:51-62
  raw allocatable             apis/extension/node_resource_amplification.go:113-125
Upstream pieces restated from k8s v1.24 (not on disk, documented semantics):
  resource.Quantity Value()/MilliValue() round up; PodRequestsAndLimits = sum(containers)
  max'd with each init container, plus overhead; kube QoS (v1qos.GetPodQOS).
"""
from __future__ import annotations

import math
from fractions import Fraction
from typing import Dict, Optional

CPU, MEMORY = "cpu", "memory"
BATCH_CPU, BATCH_MEMORY = "kubernetes.io/batch-cpu", "kubernetes.io/batch-memory"
MID_CPU, MID_MEMORY = "kubernetes.io/mid-cpu", "kubernetes.io/mid-memory"
DEFAULT_MILLI_CPU_REQUEST = 250
DEFAULT_MEMORY_REQUEST = 200 * 1024 * 1024
DEFAULT_REPORT_INTERVAL_NS = 60 * 10**9

_BIN = {"Ki": 2**10, "Mi": 2**20, "Gi": 2**30, "Ti": 2**40, "Pi": 2**50, "Ei": 2**60}
_DEC = {"n": Fraction(1, 10**9), "u": Fraction(1, 10**6), "m": Fraction(1, 1000), "": 1, "k": 10**3,
        "M": 10**6, "G": 10**9, "T": 10**12, "P": 10**15, "E": 10**18}


def quantity(s) -> Fraction:
    """resource.MustParse subset: decimal numbers with binary/decimal SI suffixes or e-notation."""
    if isinstance(s, (int, Fraction)):
        return Fraction(s)
    s = str(s).strip()
    for suf in sorted(_BIN, key=len, reverse=True):
        if s.endswith(suf):
            return Fraction(s[: -len(suf)]) * _BIN[suf]
    if "e" in s or "E" in s:
        m, e = s.replace("E", "e").split("e")
        return Fraction(m) * Fraction(10) ** int(e)
    if s and s[-1] in _DEC and not s[-1].isdigit():
        return Fraction(s[:-1]) * _DEC[s[-1]]
    return Fraction(s)


def value(q: Fraction) -> int:
    return math.ceil(q)


def milli_value(q: Fraction) -> int:
    return math.ceil(q * 1000)


def resource_value(name: str, q: Fraction) -> int:
    """getResourceValue (helper.go:146-151)."""
    return milli_value(q) if name == CPU else value(q)


def rl(d: Optional[dict]) -> Dict[str, Fraction]:
    return {k: quantity(v) for k, v in (d or {}).items()}


# ---------------------------------------------------------------- pods

def pod_requests_and_limits(pod: dict):
    """upstream pkg/api/v1/resource PodRequestsAndLimits."""
    reqs: Dict[str, Fraction] = {}
    lims: Dict[str, Fraction] = {}
    for c in pod.get("containers", []):
        for k, v in rl(c.get("requests")).items():
            reqs[k] = reqs.get(k, 0) + v
        for k, v in rl(c.get("limits")).items():
            lims[k] = lims.get(k, 0) + v
    for c in pod.get("initContainers", []):
        for k, v in rl(c.get("requests")).items():
            if v > reqs.get(k, 0):
                reqs[k] = v
        for k, v in rl(c.get("limits")).items():
            if v > lims.get(k, 0):
                lims[k] = v
    for k, v in rl(pod.get("overhead")).items():
        reqs[k] = reqs.get(k, 0) + v
        if k in lims:
            lims[k] = lims[k] + v
    return reqs, lims


def kube_qos(pod: dict) -> str:
    """upstream v1qos.GetPodQOS (cpu and memory only)."""
    requests: Dict[str, Fraction] = {}
    limits: Dict[str, Fraction] = {}
    guaranteed = True
    for c in pod.get("containers", []) + pod.get("initContainers", []):
        r, lm = rl(c.get("requests")), rl(c.get("limits"))
        for k in (CPU, MEMORY):
            if k in r and r[k] != 0:
                requests[k] = requests.get(k, 0) + r[k]
            if k in lm and lm[k] != 0:
                limits[k] = limits.get(k, 0) + lm[k]
        if not all(k in lm and lm[k] != 0 for k in (CPU, MEMORY)):
            guaranteed = False
    if not requests and not limits:
        return "BestEffort"
    if guaranteed:
        for k in (CPU, MEMORY):
            if requests.get(k, limits.get(k)) != limits.get(k):
                guaranteed = False
    return "Guaranteed" if guaranteed else "Burstable"


def priority_class(pod: Optional[dict]) -> str:
    """GetPodPriorityClassWithDefault (priority_utils.go:26-47)."""
    if pod is None:
        return ""
    lab = (pod.get("labels") or {}).get("koordinator.sh/priority-class")
    if lab in ("koord-prod", "koord-mid", "koord-batch", "koord-free"):
        return lab
    p = pod.get("priority")
    if p is not None:
        if 9000 <= p <= 9999:
            return "koord-prod"
        if 7000 <= p <= 7999:
            return "koord-mid"
        if 5000 <= p <= 5999:
            return "koord-batch"
        if 3000 <= p <= 3999:
            return "koord-free"
    qos = (pod.get("labels") or {}).get("koordinator.sh/qosClass")
    if qos is None:
        qos = {"Guaranteed": "LSR", "Burstable": "LS", "BestEffort": "BE"}[kube_qos(pod)]
    if qos in ("SYSTEM", "LSE", "LSR", "LS"):
        return "koord-prod"
    if qos == "BE":
        return "koord-batch"
    return ""


def translate(priority: str, name: str) -> str:
    """TranslateResourceNameByPriorityClass (resource.go:53-58)."""
    if priority in ("koord-prod", ""):
        return name
    table = {"koord-batch": {CPU: BATCH_CPU, MEMORY: BATCH_MEMORY}, "koord-mid": {CPU: MID_CPU, MEMORY: MID_MEMORY}}
    return table.get(priority, {}).get(name, "")


def estimated_used_by_resource(reqs, lims, name: str, scaling: int) -> int:
    """default_estimator.go:73-108."""
    limit_q = lims.get(name, Fraction(0))
    request_q = reqs.get(name, Fraction(0))
    if limit_q > request_q:
        scaling = 100
        q = limit_q
    else:
        q = request_q
    if q == 0:
        if name in (CPU, BATCH_CPU):
            return DEFAULT_MILLI_CPU_REQUEST
        if name in (MEMORY, BATCH_MEMORY):
            return DEFAULT_MEMORY_REQUEST
        return 0
    if name == CPU:
        est = int(round_half_away(float(milli_value(q)) * float(scaling) / 100))
        lim = milli_value(limit_q)
    else:
        est = int(round_half_away(float(value(q)) * float(scaling) / 100))
        lim = value(limit_q)
    if lim > 0 and est > lim:
        est = lim
    return est


def round_half_away(x: float) -> float:
    """Go math.Round."""
    return math.floor(x + 0.5) if x >= 0 else -math.floor(-x + 0.5)


def estimate_pod(args: dict, pod: dict) -> Dict[str, int]:
    reqs, lims = pod_requests_and_limits(pod)
    pc = priority_class(pod)
    return {r: estimated_used_by_resource(reqs, lims, translate(pc, r), args["estimatedScalingFactors"].get(r, 0))
            for r in args["resourceWeights"]}


def estimate_node(node: dict) -> Dict[str, Fraction]:
    """EstimateNode (default_estimator.go:110-129)."""
    alloc = rl(node.get("allocatable"))
    raw = rl(node.get("rawAllocatable")) if node.get("rawAllocatable") else {}
    if not raw or raw == alloc:
        return alloc
    out = dict(alloc)
    out.update(raw)
    return out


# ---------------------------------------------------------------- args

def set_defaults(a: dict) -> dict:
    """SetDefaults_LoadAwareSchedulingArgs (v1beta2/defaults.go:77-100)."""
    a = dict(a)
    if a.get("filterExpiredNodeMetrics") is None:
        a["filterExpiredNodeMetrics"] = True
    if a.get("nodeMetricExpirationSeconds") is None:
        a["nodeMetricExpirationSeconds"] = 180
    if not a.get("resourceWeights"):
        a["resourceWeights"] = {CPU: 1, MEMORY: 1}
    if not a.get("usageThresholds"):
        a["usageThresholds"] = {CPU: 65, MEMORY: 95}
    sf = a.get("estimatedScalingFactors")
    if sf is None:
        a["estimatedScalingFactors"] = {CPU: 85, MEMORY: 70}
    else:
        sf = dict(sf)
        sf.setdefault(CPU, 85)
        sf.setdefault(MEMORY, 70)
        a["estimatedScalingFactors"] = sf
    a.setdefault("prodUsageThresholds", {})
    a.setdefault("scoreAccordingProdUsage", False)
    a.setdefault("aggregated", None)
    return a


def filter_profile(node: dict, a: dict):
    """generateUsageThresholdsFilterProfile (helper.go:102-140)."""
    agg_args = a.get("aggregated") or {}
    filter_agg = bool(agg_args.get("usageThresholds")) and agg_args.get("usageAggregationType", "") != ""
    custom = node.get("customUsageThresholds")
    if custom is None:
        prof = {"usageThresholds": a["usageThresholds"], "prodUsageThresholds": a["prodUsageThresholds"], "aggregatedUsage": None}
        if filter_agg:
            prof["aggregatedUsage"] = {"usageThresholds": agg_args["usageThresholds"],
                                       "usageAggregationType": agg_args["usageAggregationType"],
                                       "usageAggregatedDurationS": agg_args.get("usageAggregatedDurationS", 0)}
        return prof
    prof = {"usageThresholds": custom.get("usageThresholds") or a["usageThresholds"],
            "prodUsageThresholds": custom.get("prodUsageThresholds") or a["prodUsageThresholds"],
            "aggregatedUsage": custom.get("aggregatedUsage")}
    au = prof["aggregatedUsage"]
    if au is not None and (not au.get("usageThresholds") or au.get("usageAggregationType", "") == ""):
        prof["aggregatedUsage"] = None
    if prof["aggregatedUsage"] is None and filter_agg:
        prof["aggregatedUsage"] = {"usageThresholds": agg_args["usageThresholds"],
                                   "usageAggregationType": agg_args["usageAggregationType"],
                                   "usageAggregatedDurationS": agg_args.get("usageAggregatedDurationS", 0)}
    return prof


# ---------------------------------------------------------------- NodeMetric helpers

def is_expired(nm: Optional[dict], exp_s: int, now: int) -> bool:
    """isNodeMetricExpired (helper.go:36-41)."""
    return nm is None or nm.get("updateTime") is None or (exp_s > 0 and now - nm["updateTime"] >= exp_s * 10**9)


def target_aggregated_usage(nm: dict, duration_s: int, agg_type: str) -> Optional[Dict[str, Fraction]]:
    """getTargetAggregatedUsage (helper.go:58-90)."""
    info = nm.get("nodeMetric")
    if info is None or not info.get("aggregatedNodeUsages"):
        return None
    entries = info["aggregatedNodeUsages"]
    if not duration_s:
        max_d, max_i = 0, 0
        for i, e in enumerate(entries):
            if e["durationS"] > max_d:
                max_d, max_i = e["durationS"], i
        u = rl(entries[max_i]["usage"].get(agg_type))
        return u if u else None
    for e in entries:
        if e["durationS"] == duration_s:
            u = rl(e["usage"].get(agg_type))
            if u:
                return u
    return None


def pod_metric_map(nm: dict, lister: dict, filter_prod: bool) -> Dict[str, Dict[str, Fraction]]:
    """buildPodMetricMap (helper.go:153-170); lister maps 'ns/name' -> pod dict."""
    out = {}
    for pm in nm.get("podsMetric") or []:
        key = f"{pm['namespace']}/{pm['name']}"
        pod = lister.get(key)
        if pod is None:
            continue
        if filter_prod and priority_class(pod) != "koord-prod":
            continue
        out[key] = rl(pm.get("usage"))
    return out


def sum_pod_usages(pod_metrics, estimated: set):
    """sumPodUsages (helper.go:172-186)."""
    if not pod_metrics:
        return None, None
    usages: Dict[str, Fraction] = {}
    est: Dict[str, Fraction] = {}
    for name, u in pod_metrics.items():
        target = est if name in estimated else usages
        for k, v in u.items():
            target[k] = target.get(k, 0) + v
    return usages, est


# ---------------------------------------------------------------- plugin

def filter_node(args: dict, node: dict, nm: Optional[dict], lister: dict, pod: Optional[dict], now: int = 0):
    """Filter (load_aware.go:123-254). Returns ("Success", "") or ("Unschedulable", reason)."""
    a = set_defaults(args)
    pod = pod or {}
    if "DaemonSet" in (pod.get("ownerKinds") or []):
        return "Success", ""
    if nm is None:
        return "Success", ""
    if a["filterExpiredNodeMetrics"] and a["nodeMetricExpirationSeconds"] is not None and \
            is_expired(nm, a["nodeMetricExpirationSeconds"], now):
        return "Success", ""
    prof = filter_profile(node, a)
    total_alloc = estimate_node(node)
    if prof["prodUsageThresholds"] and priority_class(pod) == "koord-prod":
        if not nm.get("podsMetric"):
            return "Success", ""
        prod_usage, _ = sum_pod_usages(pod_metric_map(nm, lister, True), set())
        prod_usage = prod_usage or {}
        for r in sorted(prof["prodUsageThresholds"], key=_res_order):
            thr = prof["prodUsageThresholds"][r]
            if thr == 0:
                continue
            total = total_alloc.get(r, Fraction(0))
            if total == 0:
                continue
            used = prod_usage.get(r, Fraction(0))
            usage = int(round_half_away(float(milli_value(used)) / float(milli_value(total)) * 100))
            if usage >= thr:
                return "Unschedulable", f"node(s) {r} usage exceed threshold"
        return "Success", ""
    agg = prof["aggregatedUsage"]
    thresholds = agg["usageThresholds"] if agg is not None else prof["usageThresholds"]
    if not thresholds:
        return "Success", ""
    if nm.get("nodeMetric") is None:
        return "Success", ""
    for r in sorted(thresholds, key=_res_order):
        thr = thresholds[r]
        if thr == 0:
            continue
        total = total_alloc.get(r, Fraction(0))
        if total == 0:
            continue
        if agg is not None:
            usage_map = target_aggregated_usage(nm, agg.get("usageAggregatedDurationS", 0), agg["usageAggregationType"])
        else:
            usage_map = rl(nm["nodeMetric"].get("nodeUsage"))
        if usage_map is None:
            continue
        used = usage_map.get(r, Fraction(0))
        usage = int(round_half_away(float(milli_value(used)) / float(milli_value(total)) * 100))
        if usage >= thr:
            if agg is not None:
                return "Unschedulable", f"node(s) {r} aggregated usage exceed threshold"
            return "Unschedulable", f"node(s) {r} usage exceed threshold"
    return "Success", ""


def _res_order(r: str):
    # the reference iterates a Go map (random order); cpu is checked first here and in the kernels
    return (0 if r == CPU else 1 if r == MEMORY else 2, r)


def score_node(args: dict, node: dict, nm: Optional[dict], lister: dict, assigned: list,
               pod: Optional[dict], now: int = 0) -> int:
    """Score (load_aware.go:269-335) + estimatedAssignedPodUsed (:337-376) + scorer (:378-397)."""
    a = set_defaults(args)
    if nm is None:
        return 0
    if a["nodeMetricExpirationSeconds"] is not None and is_expired(nm, a["nodeMetricExpirationSeconds"], now):
        return 0
    pod = pod or {}
    prod_pod = priority_class(pod) == "koord-prod" and a["scoreAccordingProdUsage"]
    metrics = pod_metric_map(nm, lister, prod_pod)
    estimated = dict(estimate_pod(a, pod))
    agg_args = a.get("aggregated") or {}
    score_agg = agg_args.get("scoreAggregationType", "") != ""
    # estimatedAssignedPodUsed
    upd = nm.get("updateTime")
    interval = nm.get("reportIntervalSeconds")
    interval_ns = DEFAULT_REPORT_INTERVAL_NS if interval is None else interval * 10**9
    assigned_used: Dict[str, int] = {}
    estimated_pods = set()
    for item in assigned:
        ap = item["pod"]
        if prod_pod and priority_class(ap) != "koord-prod":
            continue
        name = f"{ap.get('namespace', '')}/{ap.get('name', '')}"
        pod_usage = metrics.get(name, {})
        ts = item["timestamp"]
        missed = upd is None or ts > upd
        in_interval = upd is not None and ts < upd and (upd - ts) < interval_ns
        agg_missing = score_agg and target_aggregated_usage(nm, agg_args.get("scoreAggregatedDurationS", 0),
                                                             agg_args["scoreAggregationType"]) is None
        if not pod_usage or missed or in_interval or agg_missing:
            est = estimate_pod(a, ap)
            for r, v in est.items():
                if r in pod_usage:
                    u = resource_value(r, pod_usage[r])
                    if u > v:
                        v = u
                assigned_used[r] = assigned_used.get(r, 0) + v
            estimated_pods.add(name)
    for r, v in assigned_used.items():
        estimated[r] = estimated.get(r, 0) + v
    actual, est_actual = sum_pod_usages(metrics, estimated_pods)
    if prod_pod:
        for r, q in (actual or {}).items():
            estimated[r] = estimated.get(r, 0) + resource_value(r, q)
    elif nm.get("nodeMetric") is not None:
        if score_agg:
            usage = target_aggregated_usage(nm, agg_args.get("scoreAggregatedDurationS", 0), agg_args["scoreAggregationType"])
        else:
            usage = rl(nm["nodeMetric"].get("nodeUsage"))
        if usage is not None:
            for r, q in usage.items():
                e = (est_actual or {}).get(r, Fraction(0))
                if e != 0 and q >= e:
                    q = q - e
                estimated[r] = estimated.get(r, 0) + resource_value(r, q)
    alloc = estimate_node(node)
    node_score = weight_sum = 0
    for r, w in a["resourceWeights"].items():
        node_score += least_requested_score(estimated.get(r, 0), resource_value(r, alloc.get(r, Fraction(0)))) * w
        weight_sum += w
    return node_score // weight_sum


def least_requested_score(requested: int, capacity: int) -> int:
    if capacity == 0 or requested > capacity:
        return 0
    return ((capacity - requested) * 100) // capacity
