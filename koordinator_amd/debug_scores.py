"""The --debug-scores top-N table (frameworkext/debug.go:61-108), fed by the device's Score results.

koord-scheduler's framework extender logs this table after RunScorePlugins (framework_extender.go:254-257) when
`--debug-scores` / `-s` is above 0 (debug.go:36-48).  Each row is a feasible node; its cells are the plugins' weighted,
normalized scores, as RunScorePlugins returns them (v1.24 framework: NormalizeScore, then score x weight).  The device
returns the same numbers through `ks_eval_pod` (un-weighted per-plugin scores, which `plugin_scores` multiplies by the
profile's weights), so the host renders the table without re-running any plugin.

Parity: the markdown layout is pinned by the reference's TestDebugScores (debug_test.go:91-176, the golden in
tests/test_debug_scores.py).  Order of equal totals is not pinned: debug.go sorts with Go's unstable sort.Slice; here
equal totals keep node order (a stable sort).
"""
from __future__ import annotations

import numpy as np

from . import abi

# (plugin name, score column of ks_eval_pod, enabled(cfg), weight(cfg))
SCORE_PLUGINS = [
    ("NodeResourcesFit", abi.KS_SCORE_FIT, lambda c: c.fit.enable_score, lambda c: c.fit.plugin_weight),
    ("LoadAwareScheduling", abi.KS_SCORE_LOADAWARE, lambda c: c.loadaware.enable_score,
     lambda c: c.loadaware.plugin_weight),
    ("Reservation", abi.KS_SCORE_RESERVATION, lambda c: c.reservation.enable, lambda c: c.reservation.plugin_weight),
    ("NodeNUMAResource", abi.KS_SCORE_NUMA, lambda c: c.numa.enable, lambda c: c.numa.plugin_weight),
    ("DeviceShare", abi.KS_SCORE_DEVICESHARE, lambda c: c.deviceshare.enable, lambda c: c.deviceshare.plugin_weight),
    ("NodeResourcesBalancedAllocation", abi.KS_SCORE_BALANCED, lambda c: c.balanced.enable,
     lambda c: c.balanced.plugin_weight),
    ("TaintToleration", abi.KS_SCORE_TAINT, lambda c: c.taint.enable_score, lambda c: c.taint.plugin_weight),
    ("NodeAffinity", abi.KS_SCORE_NODE_AFFINITY, lambda c: c.affinity.enable_score, lambda c: c.affinity.plugin_weight),
    ("PodTopologySpread", abi.KS_SCORE_TOPOLOGY_SPREAD, lambda c: c.topology.enable, lambda c: c.topology.spread_weight),
    ("InterPodAffinity", abi.KS_SCORE_POD_AFFINITY, lambda c: c.topology.enable, lambda c: c.topology.affinity_weight),
]


def plugin_scores(cfg, reasons, scores):
    """RunScorePlugins' result over the feasible nodes: (feasible node indices in node order, {plugin: weighted scores
    aligned with them}) from ks_eval_pod's reasons [n] and un-weighted scores [n, KS_NUM_SCORE_PLUGINS]."""
    feas = np.flatnonzero(np.asarray(reasons) == 0)
    scores = np.asarray(scores, np.int64)
    out = {}
    for name, col, enabled, weight in SCORE_PLUGINS:
        if enabled(cfg):
            out[name] = [int(v) * int(weight(cfg)) for v in scores[feas, col]]
    return feas, out


def debug_scores(top_n: int, pod_ref: str, plugin_to_node_scores: dict, node_names) -> str:
    """debugScores (debug.go:61-108) rendered as go-pretty's RenderMarkdown: rows are the first top_n nodes by total
    score (descending), columns `#`, `Pod` (klog.KObj: namespace/name), `Node`, `Score` and the plugins in name order;
    numeric columns right-aligned."""
    names = sorted(plugin_to_node_scores)
    total = [sum(plugin_to_node_scores[p][i] for p in names) for i in range(len(node_names))]
    order = sorted(range(len(node_names)), key=lambda i: -total[i])

    def row(cells):
        return "| " + " | ".join(str(c).replace("|", "\\|") for c in cells) + " |"

    lines = [row(["#", "Pod", "Node", "Score"] + names),
             "|" + "|".join([" --- "] * 3 + [" ---:"] * (1 + len(names))) + "|"]
    for rank, i in enumerate(order[:max(top_n, 0)]):
        lines.append(row([rank, pod_ref, node_names[i], total[i]] + [plugin_to_node_scores[p][i] for p in names]))
    return "\n".join(lines)


def eval_debug_table(ev, cfg, pod, node_names, top_n: int, pod_ref: str):
    """The table the extender logs for pod 0 of `pod` against the evaluator's current state, or None where it logs
    nothing: top_n <= 0 (debug.go hook), or fewer than two feasible nodes (the v1.24 scheduler skips scoring for one
    feasible node and fails the pod for none)."""
    if top_n <= 0:
        return None
    reasons, scores, _ = ev.eval_pod(pod)
    feas, per_plugin = plugin_scores(cfg, reasons, scores)
    if len(feas) < 2:
        return None
    return debug_scores(top_n, pod_ref, per_plugin, [node_names[i] for i in feas])
