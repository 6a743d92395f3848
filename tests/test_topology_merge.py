"""The topology manager's Merge (oracle/koord_oracle.c ko_merge_hints) against the reference's own merge tables
(pkg/scheduler/frameworkext/topologymanager/policy_test.go, transcribed by tests/golden/make_topology_merge_golden.py
into tests/golden/topology_merge.json), for the best-effort, restricted and single-numa-node policies."""
import json
import os

import pytest

from oracle.oracle import topology_merge

G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "topology_merge.json")))


def bits(b):
    return 0 if b is None else sum(1 << i for i in b)


def provider_lists(providers):
    """filterProvidersHints (policy.go:96-127): a nil / empty provider map -> one preferred any-numa hint; a nil
    resource list -> the same; an empty list -> one non-preferred any-numa hint; else the list itself."""
    out = []
    for prov in providers:
        if not prov:
            out.append([(0, True, 0)])
            continue
        for hints in prov.values():
            if hints is None:
                out.append([(0, True, 0)])
            elif not hints:
                out.append([(0, False, 0)])
            else:
                out.append([(bits(m), p, s) for m, p, s in hints])
    return out


CASES = [(s["policy"], s["numa_nodes"], c) for s in G["suites"] for c in s["cases"]]


@pytest.mark.parametrize("policy,numa_nodes,case", CASES, ids=[f"{p}:{c['name']}" for p, _, c in CASES])
def test_merge_matches_reference_table(policy, numa_nodes, case):
    admit, mask, pref = topology_merge(policy, len(numa_nodes), provider_lists(case["providers"]))
    want_mask, want_pref, _ = case["expected"]
    assert (mask, pref) == (bits(want_mask), want_pref), case["name"]
    # canAdmitPodResult: best-effort admits everything, restricted / single-numa-node only preferred hints
    assert admit == (True if policy == "best-effort" else want_pref)
