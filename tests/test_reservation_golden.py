"""Reservation plugin: the object-level restatement (oracle/reservation_ref.py)
against the reference's own test tables (tests/golden/reservation.json)."""
import json
import os

import pytest

from oracle import reservation_ref as R

G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reservation.json")))["cases"]


def res_of(d):
    return R.Reservation(name=d["name"], allocatable=d["allocatable"], allocated=d.get("allocated", {}),
                         policy=d.get("policy", R.DEFAULT), order=d.get("order", 0),
                         owner_match=d.get("owner_match", True), assigned=d.get("assigned", 0),
                         resource_names=d.get("resource_names"))


@pytest.mark.parametrize("c", G["score"], ids=[c["name"] for c in G["score"]])
def test_score(c):
    matched = [res_of(x) for x in c["matched"]]
    if c.get("reserve_pod") or not matched:
        score, nom = 0, None
    else:
        nom = R.nominate(c["pod_req"], c["allocatable"], c["allowed_pods"], c["pods_eff"], c["pod_requested"],
                         c["r_allocated"], matched)
        score = R.score_reservation(c["pod_req"], nom) if nom is not None else 0
    assert score == c["want_score"]
    if "want_nominated" in c:
        assert nom is not None and nom.name == c["want_nominated"]


def test_score_with_order_and_normalize():
    c = G["score_order"][0]
    raws, orders = [], []
    for n in c["nodes"]:
        matched = [res_of(x) for x in n["matched"]]
        _, order = R.most_preferred_by_order(matched)
        orders.append(order)
        nom = R.nominate(c["pod_req"], {}, 0, 0, {}, {}, matched)
        raws.append(R.score_reservation(c["pod_req"], nom) if nom else 0)
    pref = min((o, i) for i, o in enumerate(orders) if o)[1]
    assert c["nodes"][pref]["name"] == c["want_preferred"]
    raws[pref] = 1000
    assert raws == c["want_raw"]
    assert R.default_normalize(raws) == c["want_normalized"]


@pytest.mark.parametrize("c", G["filter"], ids=[c["name"] for c in G["filter"]])
def test_filter_with_reservations(c):
    matched = [res_of(x) for x in c["matched"]]
    ok, reasons = R.filter_with_reservations(c["pod_req"], c["allocatable"], c["allowed_pods"], c["pods_eff"],
                                             len(matched), c["pod_requested"], c["r_allocated"], matched,
                                             c["has_affinity"])
    assert ok == c["want_ok"]
    if "want_reasons" in c:
        assert reasons == c["want_reasons"]


def test_restore():
    c = G["restore"][0]
    n = c["node"]
    node = R.NodeState(n["allocatable"], n["allowed_pods"], n["requested"], n["nonzero"], n["pods"])
    eff, pod_requested, r_alloc, matched = R.restore(node, [res_of(x) for x in c["reservations"]])
    w = c["want"]
    assert eff.requested == w["requested"] and eff.nonzero == w["nonzero"] and eff.pods == w["pods"]
    assert pod_requested == w["pod_requested"] and r_alloc == w["r_allocated"]
    assert [r.name for r in matched] == w["matched"]
