"""Host-side ingestion: Kubernetes-shaped objects -> the ks_* structure-of-arrays.

This is what the Go cgo shim does at informer time, written
here in Python so the product path can be exercised end-to-end from the
reference's own test tables (tests/golden/).  It reduces, per node, the
LoadAware state that the reference recomputes inside every Filter/Score call
(NodeMetric lister lookups, assign-cache scan, pod-metric sums) into a handful
of int64 columns, and per pod the request/limit inputs of EstimatePod:

  la_flags / thresholds / usages   Filter inputs (load_aware.go:123-254, helper.go:36-140)
  la_alloc_*                       EstimateNode (estimator/default_estimator.go:110-129)
  la_term_*                        Score's node term for non-prod pods: assigned-not-reported
                                   pods' estimates + node usage minus their actual usage
                                   (load_aware.go:294-325, :337-376)
  la_prod_term_*                   the same with filterProdPod=true (ScoreAccordingProdUsage)

Objects are plain dicts in the JSON layout of tests/golden/*.json.  Times are
integer nanoseconds; ``now`` is the scheduling-cycle time the host freezes.
"""
from __future__ import annotations

import math
from fractions import Fraction
from typing import Dict, List, Optional, Tuple

import numpy as np

from . import abi
from .cluster import NodeTable, PodTable
from .config import BATCH_CPU, BATCH_MEMORY, CPU, MEMORY, LoadAwareSchedulingArgs

MID_CPU, MID_MEMORY = "kubernetes.io/mid-cpu", "kubernetes.io/mid-memory"
LA_DEFAULT_MILLI_CPU = 250
LA_DEFAULT_MEMORY = 200 * 1024 * 1024
NZ_DEFAULT_MILLI_CPU = 100
NZ_DEFAULT_MEMORY = 200 * 1024 * 1024
REPORT_INTERVAL_NS = 60 * 10**9

_SUFFIX = [("Ki", 2**10), ("Mi", 2**20), ("Gi", 2**30), ("Ti", 2**40), ("Pi", 2**50), ("Ei", 2**60),
           ("n", Fraction(1, 10**9)), ("u", Fraction(1, 10**6)), ("m", Fraction(1, 1000)),
           ("k", 10**3), ("M", 10**6), ("G", 10**9), ("T", 10**12), ("P", 10**15), ("E", 10**18)]


def parse_quantity(s) -> Fraction:
    """resource.Quantity parse (canonical suffix forms)."""
    if isinstance(s, (int, Fraction)):
        return Fraction(s)
    s = str(s).strip()
    for suf, mul in _SUFFIX:
        if s.endswith(suf) and s[: -len(suf)].replace(".", "", 1).lstrip("+-").isdigit():
            return Fraction(s[: -len(suf)]) * mul
    if "e" in s.lower():
        mant, exp = s.lower().split("e")
        return Fraction(mant) * Fraction(10) ** int(exp)
    return Fraction(s)


def q_value(q: Fraction) -> int:
    return math.ceil(q)


def q_milli(q: Fraction) -> int:
    return math.ceil(q * 1000)


def res_value(name: str, q: Fraction) -> int:
    return q_milli(q) if name == CPU else q_value(q)


def _rl(d) -> Dict[str, Fraction]:
    return {k: parse_quantity(v) for k, v in (d or {}).items()}


def go_round(x: float) -> int:
    return int(math.floor(x + 0.5)) if x >= 0 else -int(math.floor(-x + 0.5))


# ------------------------------------------------------------------ pods

def requests_and_limits(pod: dict) -> Tuple[Dict[str, Fraction], Dict[str, Fraction]]:
    req: Dict[str, Fraction] = {}
    lim: Dict[str, Fraction] = {}
    for c in pod.get("containers", []):
        for k, v in _rl(c.get("requests")).items():
            req[k] = req.get(k, 0) + v
        for k, v in _rl(c.get("limits")).items():
            lim[k] = lim.get(k, 0) + v
    for c in pod.get("initContainers", []):
        for k, v in _rl(c.get("requests")).items():
            req[k] = max(req.get(k, Fraction(0)), v)
        for k, v in _rl(c.get("limits")).items():
            lim[k] = max(lim.get(k, Fraction(0)), v)
    for k, v in _rl(pod.get("overhead")).items():
        req[k] = req.get(k, 0) + v
        if k in lim:
            lim[k] += v
    return req, lim


def _kube_qos(pod: dict) -> str:
    req: Dict[str, Fraction] = {}
    lim: Dict[str, Fraction] = {}
    full_limits = True
    for c in pod.get("containers", []) + pod.get("initContainers", []):
        r, lm = _rl(c.get("requests")), _rl(c.get("limits"))
        for k in (CPU, MEMORY):
            if r.get(k, 0) != 0:
                req[k] = req.get(k, 0) + r[k]
            if lm.get(k, 0) != 0:
                lim[k] = lim.get(k, 0) + lm[k]
        full_limits &= all(lm.get(k, 0) != 0 for k in (CPU, MEMORY))
    if not req and not lim:
        return "BestEffort"
    if full_limits and all(req.get(k, lim.get(k)) == lim.get(k) for k in (CPU, MEMORY)):
        return "Guaranteed"
    return "Burstable"


def priority_class(pod: Optional[dict]) -> str:
    """GetPodPriorityClassWithDefault (apis/extension/priority_utils.go:26-47)."""
    if pod is None:
        return ""
    label = (pod.get("labels") or {}).get("koordinator.sh/priority-class")
    if label in ("koord-prod", "koord-mid", "koord-batch", "koord-free"):
        return label
    p = pod.get("priority")
    if p is not None:
        for lo, hi, name in ((9000, 9999, "koord-prod"), (7000, 7999, "koord-mid"), (5000, 5999, "koord-batch"),
                             (3000, 3999, "koord-free")):
            if lo <= p <= hi:
                return name
    qos = (pod.get("labels") or {}).get("koordinator.sh/qosClass")
    if qos is None:
        qos = {"Guaranteed": "LSR", "Burstable": "LS", "BestEffort": "BE"}[_kube_qos(pod)]
    return "koord-prod" if qos in ("SYSTEM", "LSE", "LSR", "LS") else ("koord-batch" if qos == "BE" else "")


def _translate(pc: str, name: str) -> str:
    if pc in ("koord-prod", ""):
        return name
    return {"koord-batch": {CPU: BATCH_CPU, MEMORY: BATCH_MEMORY},
            "koord-mid": {CPU: MID_CPU, MEMORY: MID_MEMORY}}.get(pc, {}).get(name, "")


def _la_inputs(pod: dict, name: str) -> Tuple[int, int, int]:
    """(request, limit, zero-default) of the priority-translated resource, in the units
    estimatedUsedByResource uses (MilliValue for "cpu", Value otherwise)."""
    req, lim = requests_and_limits(pod)
    real = _translate(priority_class(pod), name)
    conv = q_milli if real == CPU else q_value
    r = req.get(real, Fraction(0))
    lm = lim.get(real, Fraction(0))
    dflt = LA_DEFAULT_MILLI_CPU if real in (CPU, BATCH_CPU) else LA_DEFAULT_MEMORY if real in (MEMORY, BATCH_MEMORY) else 0
    # the device compares the converted ints; identical to Quantity.Cmp unless the two
    # quantities differ below the conversion unit (sub-milli cpu / sub-byte memory)
    return conv(r), conv(lm), dflt


def estimate_pod(pod: dict, scaling: Dict[str, int]) -> Dict[str, int]:
    """EstimatePod on the host (used for assigned pods in the node-term reduction)."""
    out = {}
    for name in (CPU, MEMORY):
        r, lm, dflt = _la_inputs(pod, name)
        sf = scaling.get(name, 0)
        if lm > r:
            sf, q = 100, lm
        else:
            q = r
        if q == 0:
            out[name] = dflt
            continue
        est = go_round(float(q) * float(sf) / 100)
        if lm > 0 and est > lm:
            est = lm
        out[name] = est
    return out


def pods_to_table(pods: List[Optional[dict]], scalar_slots=(BATCH_CPU, BATCH_MEMORY)) -> PodTable:
    t = PodTable(len(pods))
    for i, pod in enumerate(pods):
        pod = pod or {}
        req, _ = requests_and_limits(pod)
        t.req_milli_cpu[i] = q_milli(req.get(CPU, Fraction(0)))
        t.req_memory[i] = q_value(req.get(MEMORY, Fraction(0)))
        t.req_ephemeral[i] = q_value(req.get("ephemeral-storage", Fraction(0)))
        flags = 0
        scal = [k for k in req if "/" in k and k not in (CPU, MEMORY)]
        for k in scal:
            if k in scalar_slots:
                t.req_scalar[scalar_slots.index(k), i] = q_value(req[k])
        if scal:
            flags |= abi.KS_POD_SCALAR_KEYS
        nz_cpu = nz_mem = 0
        for c in pod.get("containers", []):
            r = _rl(c.get("requests"))
            nz_cpu += q_milli(r[CPU]) if CPU in r else NZ_DEFAULT_MILLI_CPU
            nz_mem += q_value(r[MEMORY]) if MEMORY in r else NZ_DEFAULT_MEMORY
        t.nonzero_milli_cpu[i] = nz_cpu
        t.nonzero_memory[i] = nz_mem
        if priority_class(pod) == "koord-prod":
            flags |= abi.KS_POD_PROD
        if "DaemonSet" in (pod.get("ownerKinds") or []):
            flags |= abi.KS_POD_DAEMONSET
        t.flags[i] = flags
        t.la_req_cpu[i], t.la_lim_cpu[i], t.la_dflt_cpu[i] = _la_inputs(pod, CPU)
        t.la_req_memory[i], t.la_lim_memory[i], t.la_dflt_memory[i] = _la_inputs(pod, MEMORY)
    return t


# ------------------------------------------------------------------ nodes

def _expired(nm: Optional[dict], exp_s: Optional[int], now: int) -> bool:
    return nm is None or nm.get("updateTime") is None or (exp_s is not None and exp_s > 0 and
                                                          now - nm["updateTime"] >= exp_s * 10**9)


def _agg_usage(nm: dict, duration_s: int, typ: str) -> Optional[Dict[str, Fraction]]:
    info = nm.get("nodeMetric")
    if info is None or not info.get("aggregatedNodeUsages"):
        return None
    entries = info["aggregatedNodeUsages"]
    if not duration_s:
        best, idx = 0, 0
        for i, e in enumerate(entries):
            if e["durationS"] > best:
                best, idx = e["durationS"], i
        u = _rl(entries[idx]["usage"].get(typ))
        return u or None
    for e in entries:
        if e["durationS"] == duration_s:
            u = _rl(e["usage"].get(typ))
            if u:
                return u
    return None


def _pod_metrics(nm: dict, lister: Dict[str, dict], prod_only: bool) -> Dict[str, Dict[str, Fraction]]:
    out = {}
    for pm in nm.get("podsMetric") or []:
        key = f"{pm['namespace']}/{pm['name']}"
        pod = lister.get(key)
        if pod is None or (prod_only and priority_class(pod) != "koord-prod"):
            continue
        out[key] = _rl(pm.get("usage"))
    return out


def _node_term(la: LoadAwareSchedulingArgs, nm: dict, lister, assigned: list, prod: bool) -> Dict[str, int]:
    """Σ assigned-not-reported estimates + usage term of Score for one pod class."""
    metrics = _pod_metrics(nm, lister, prod)
    upd = nm.get("updateTime")
    iv = nm.get("reportIntervalSeconds")
    interval = REPORT_INTERVAL_NS if iv is None else iv * 10**9
    score_agg = la.score_with_aggregation()
    agg_missing = score_agg and _agg_usage(nm, la.aggregated_score_duration_s, la.aggregated_score_type) is None
    term = {CPU: 0, MEMORY: 0}
    estimated = set()
    for item in assigned:
        ap = item["pod"]
        if prod and priority_class(ap) != "koord-prod":
            continue
        name = f"{ap.get('namespace', '')}/{ap.get('name', '')}"
        usage = metrics.get(name, {})
        ts = item["timestamp"]
        if (not usage or upd is None or ts > upd or (ts < upd and upd - ts < interval) or agg_missing):
            for r, v in estimate_pod(ap, la.estimated_scaling_factors).items():
                if r in usage:
                    v = max(v, res_value(r, usage[r]))
                term[r] += v
            estimated.add(name)
    actual: Dict[str, Fraction] = {}
    est_actual: Dict[str, Fraction] = {}
    for name, u in metrics.items():
        tgt = est_actual if name in estimated else actual
        for k, v in u.items():
            tgt[k] = tgt.get(k, 0) + v
    if prod:
        for r in term:
            if r in actual:
                term[r] += res_value(r, actual[r])
    elif nm.get("nodeMetric") is not None:
        usage = _agg_usage(nm, la.aggregated_score_duration_s, la.aggregated_score_type) if score_agg \
            else _rl(nm["nodeMetric"].get("nodeUsage"))
        if usage is not None:
            for r in term:
                if r not in usage:
                    continue
                q = usage[r]
                e = est_actual.get(r, Fraction(0))
                if e != 0 and q >= e:
                    q = q - e
                term[r] += res_value(r, q)
    return term


def node_to_columns(t: NodeTable, i: int, la: LoadAwareSchedulingArgs, node: dict, nm: Optional[dict],
                    lister: Dict[str, dict], assigned: list, now: int,
                    scalar_slots=(BATCH_CPU, BATCH_MEMORY)) -> None:
    """Fill row i of `t` from one node (+ its NodeMetric and assign-cache entries)."""
    alloc = _rl(node.get("allocatable"))
    t.alloc_milli_cpu[i] = q_milli(alloc.get(CPU, Fraction(0)))
    t.alloc_memory[i] = q_value(alloc.get(MEMORY, Fraction(0)))
    t.alloc_ephemeral[i] = q_value(alloc.get("ephemeral-storage", Fraction(0)))
    t.allowed_pods[i] = q_value(alloc.get("pods", Fraction(110)))
    for k, name in enumerate(scalar_slots):
        t.alloc_scalar[k, i] = q_value(alloc.get(name, Fraction(0)))
    req = _rl(node.get("requested"))
    t.req_milli_cpu[i] = q_milli(req.get(CPU, Fraction(0)))
    t.req_memory[i] = q_value(req.get(MEMORY, Fraction(0)))
    t.nonzero_milli_cpu[i] = t.req_milli_cpu[i]
    t.nonzero_memory[i] = t.req_memory[i]
    t.pod_count[i] = int(node.get("podCount", 0))
    # EstimateNode: raw-allocatable annotation overrides (default_estimator.go:110-129)
    est_alloc = dict(alloc)
    raw = _rl(node.get("rawAllocatable")) if node.get("rawAllocatable") else {}
    if raw and raw != alloc:
        est_alloc.update(raw)
    t.la_alloc_milli_cpu[i] = q_milli(est_alloc.get(CPU, Fraction(0)))
    t.la_alloc_memory[i] = q_value(est_alloc.get(MEMORY, Fraction(0)))
    t.la_total_milli_cpu[i] = q_milli(est_alloc.get(CPU, Fraction(0)))
    t.la_total_milli_memory[i] = q_milli(est_alloc.get(MEMORY, Fraction(0)))
    flags = 0
    if nm is not None:
        flags |= abi.KS_LA_HAS_METRIC
        if _expired(nm, la.node_metric_expiration_seconds, now):
            flags |= abi.KS_LA_EXPIRED
        if nm.get("nodeMetric") is not None:
            flags |= abi.KS_LA_HAS_STATUS_METRIC
        if nm.get("podsMetric"):
            flags |= abi.KS_LA_HAS_PODS_METRIC
        # filter profile (helper.go:102-140)
        custom = node.get("customUsageThresholds")
        agg_default = None
        if la.filter_with_aggregation():
            agg_default = {"usageThresholds": la.aggregated_usage_thresholds, "usageAggregationType": la.aggregated_usage_type,
                           "usageAggregatedDurationS": la.aggregated_usage_duration_s}
        if custom is None:
            usage_thr, prod_thr, agg = la.usage_thresholds, la.prod_usage_thresholds, agg_default
        else:
            usage_thr = custom.get("usageThresholds") or la.usage_thresholds
            prod_thr = custom.get("prodUsageThresholds") or la.prod_usage_thresholds
            agg = custom.get("aggregatedUsage")
            if agg is not None and (not agg.get("usageThresholds") or not agg.get("usageAggregationType")):
                agg = None
            if agg is None:
                agg = agg_default
        thr = agg["usageThresholds"] if agg is not None else usage_thr
        if thr:
            flags |= abi.KS_LA_NODE_THR_NONEMPTY
        if prod_thr:
            flags |= abi.KS_LA_PROD_THR_NONEMPTY
        t.la_thr_cpu[i] = thr.get(CPU, 0)
        t.la_thr_memory[i] = thr.get(MEMORY, 0)
        t.la_prod_thr_cpu[i] = prod_thr.get(CPU, 0)
        t.la_prod_thr_memory[i] = prod_thr.get(MEMORY, 0)
        usage = None
        if nm.get("nodeMetric") is not None:
            if agg is not None:
                flags |= abi.KS_LA_AGGREGATED_FILTER
                usage = _agg_usage(nm, agg.get("usageAggregatedDurationS", 0), agg["usageAggregationType"])
            else:
                usage = _rl(nm["nodeMetric"].get("nodeUsage"))
        if usage is not None:
            flags |= abi.KS_LA_FILTER_USAGE_PRESENT
            t.la_usage_milli_cpu[i] = q_milli(usage.get(CPU, Fraction(0)))
            t.la_usage_milli_memory[i] = q_milli(usage.get(MEMORY, Fraction(0)))
        prod_usage: Dict[str, Fraction] = {}
        for u in _pod_metrics(nm, lister, True).values():
            for k, v in u.items():
                prod_usage[k] = prod_usage.get(k, 0) + v
        t.la_prod_usage_milli_cpu[i] = q_milli(prod_usage.get(CPU, Fraction(0)))
        t.la_prod_usage_milli_memory[i] = q_milli(prod_usage.get(MEMORY, Fraction(0)))
        all_term = _node_term(la, nm, lister, assigned, prod=False)
        prod_term = _node_term(la, nm, lister, assigned, prod=True)
        t.la_term_milli_cpu[i], t.la_term_memory[i] = all_term[CPU], all_term[MEMORY]
        t.la_prod_term_milli_cpu[i], t.la_prod_term_memory[i] = prod_term[CPU], prod_term[MEMORY]
    t.la_flags[i] = flags


def args_from_json(a: dict) -> LoadAwareSchedulingArgs:
    agg = a.get("aggregated") or {}
    la = LoadAwareSchedulingArgs(
        filter_expired_node_metrics=a.get("filterExpiredNodeMetrics"),
        node_metric_expiration_seconds=a.get("nodeMetricExpirationSeconds"),
        resource_weights=dict(a.get("resourceWeights") or {}),
        usage_thresholds=dict(a.get("usageThresholds") or {}),
        prod_usage_thresholds=dict(a.get("prodUsageThresholds") or {}),
        score_according_prod_usage=bool(a.get("scoreAccordingProdUsage", False)),
        estimated_scaling_factors=dict(a["estimatedScalingFactors"]) if a.get("estimatedScalingFactors") else None,
        aggregated_usage_thresholds=dict(agg.get("usageThresholds") or {}),
        aggregated_usage_type=agg.get("usageAggregationType", ""),
        aggregated_usage_duration_s=agg.get("usageAggregatedDurationS", 0),
        aggregated_score_type=agg.get("scoreAggregationType", ""),
        aggregated_score_duration_s=agg.get("scoreAggregatedDurationS", 0),
    )
    return la.set_defaults()


def lister_from(pods: List[dict]) -> Dict[str, dict]:
    return {f"{p.get('namespace', '')}/{p.get('name', '')}": p for p in pods}
