"""Transcribe the topology manager's merge tables into tests/golden/topology_merge.json.

Source (read as text, never executed): pkg/scheduler/frameworkext/topologymanager/policy_test.go
(commonPolicyMergeTestCases :59-380, bestEffortPolicy.mergeTestCases :344-645, singleNumaNodePolicy.mergeTestCases
:649-934) and the per-policy harnesses policy_best_effort_test.go:53-61 (NUMA nodes 0-3),
policy_restricted_test.go:71-79 (0-3, the best-effort cases too: restrictedPolicy embeds bestEffortPolicy),
policy_single_numa_node_test.go:159-167 (0-1).  Each case is stored as its hint providers: null = the
provider returns a nil map, {} = an empty map, else resource -> hint list (null = nil list); a hint is
[mask bits, preferred, score] with mask bits null for a nil NUMANodeAffinity.  Resources keep their source
order (the reference iterates a Go map there).  Usage: python make_topology_merge_golden.py /path/to/reference
"""
import json
import os
import re
import sys


def block(s, i):
    """s[i] == '{': return the index after the matching '}'."""
    depth = 0
    for j in range(i, len(s)):
        if s[j] == "{":
            depth += 1
        elif s[j] == "}":
            depth -= 1
            if depth == 0:
                return j + 1
    raise ValueError("unbalanced")


def items(body):
    """split a composite-literal body into its top-level elements"""
    out, depth, start = [], 0, 0
    for j, ch in enumerate(body):
        if ch in "{(":
            depth += 1
        elif ch in "})":
            depth -= 1
        elif ch == "," and depth == 0:
            if body[start:j].strip():
                out.append(body[start:j].strip())
            start = j + 1
    if body[start:].strip():
        out.append(body[start:].strip())
    return out


def mask_of(expr, numa_nodes):
    expr = expr.strip()
    if expr == "nil":
        return None
    m = re.fullmatch(r"NewTestBitMask\((.*)\)", expr)
    if m.group(1).strip() == "numaNodes...":
        return list(numa_nodes)
    return [int(x) for x in m.group(1).split(",") if x.strip()]


def hint(lit, numa_nodes):
    body = lit.strip()
    if body.startswith("{"):
        body = body[1:-1]
    fields = dict((k.strip(), v.strip()) for k, v in (x.split(":", 1) for x in items(body)))
    return [mask_of(fields.get("NUMANodeAffinity", "nil"), numa_nodes), fields.get("Preferred", "false") == "true",
            int(fields.get("Score", "0"))]


def provider(lit, numa_nodes):
    inner = lit[lit.index("{") + 1: lit.rindex("}")].strip()
    if inner in ("", "nil") or inner.startswith("nil"):
        return None
    body = inner[inner.index("{") + 1: inner.rindex("}")]
    res = {}
    for kv in items(body):
        k, v = kv.split(":", 1)
        v = v.strip()
        if v == "nil":
            res[k.strip().strip('"')] = None
        else:
            res[k.strip().strip('"')] = [hint(h, numa_nodes) for h in items(v[1:-1])]
    return res


def cases(src, func_pat, numa_nodes):
    m = re.search(func_pat, src)
    start = src.index("return []policyMergeTestCase{", m.end()) + len("return []policyMergeTestCase")
    body = src[start + 1: block(src, start) - 1]
    out = []
    for c in items(body):
        name = re.search(r'name:\s*"([^"]*)"', c).group(1)
        i = c.index("hp:")
        j = c.index("{", i)
        hp_body = c[j + 1: block(c, j) - 1]
        provs = [provider(p, numa_nodes) for p in items(hp_body)]
        k = c.index("expected:")
        e = c.index("{", k)
        exp = hint(c[e: block(c, e)], numa_nodes)
        out.append({"name": name, "providers": provs, "expected": exp})
    return out


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    src = open(os.path.join(ref, "pkg/scheduler/frameworkext/topologymanager/policy_test.go")).read()
    common = r"func commonPolicyMergeTestCases\(numaNodes \[\]int\)"
    be = r"func \(p \*bestEffortPolicy\) mergeTestCases\(numaNodes \[\]int\)"
    sn = r"func \(p \*singleNumaNodePolicy\) mergeTestCases\(numaNodes \[\]int\)"
    quad, pair = [0, 1, 2, 3], [0, 1]
    out = {"source": "pkg/scheduler/frameworkext/topologymanager/policy_test.go (policy merge tables) with the "
                     "harnesses of policy_best_effort_test.go:53, policy_restricted_test.go:71, "
                     "policy_single_numa_node_test.go:159",
           "suites": [
               {"policy": "best-effort", "numa_nodes": quad, "cases": cases(src, common, quad) + cases(src, be, quad)},
               {"policy": "restricted", "numa_nodes": quad, "cases": cases(src, common, quad) + cases(src, be, quad)},
               {"policy": "single-numa-node", "numa_nodes": pair, "cases": cases(src, common, pair) + cases(src, sn, pair)},
           ]}
    here = os.path.dirname(os.path.abspath(__file__))
    with open(os.path.join(here, "topology_merge.json"), "w") as f:
        json.dump(out, f, indent=1)
    print({s["policy"]: len(s["cases"]) for s in out["suites"]})


if __name__ == "__main__":
    main()
