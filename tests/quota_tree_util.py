"""Shared helpers: golden/random ElasticQuota trees as oracle objects and as QuotaTree tables."""
import json
import os

import numpy as np

from koordinator_amd import abi
from koordinator_amd.cluster import QuotaTree
from oracle.quota_runtime_ref import Quota

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
DIMS = ["cpu", "memory", "ephemeral-storage", "kubernetes.io/batch-cpu", "kubernetes.io/batch-memory", "nvidia.com/gpu",
        "d6", "d7"]


def golden_cases():
    with open(os.path.join(GOLDEN, "elasticquota_runtime.json")) as f:
        return json.load(f)["cases"]


def quotas_of(case):
    return [Quota(name=x["name"], parent=x["parent"], max=x["max"], min=x.get("min", {}),
                  shared_weight=x.get("shared_weight"), guaranteed=x.get("guaranteed", {}),
                  self_request=x.get("self_request", {}), allow_lent=x["allow_lent"]) for x in case["quotas"]]


def tree_of(quotas, cluster_total):
    """Oracle quota objects -> QuotaTree (row i = quotas[i])."""
    idx = {q.name: i for i, q in enumerate(quotas)}
    t = QuotaTree(len(quotas))
    sw = np.zeros((abi.KS_QUOTA_DIMS, t.q), np.int64)
    any_sw = False
    for i, q in enumerate(quotas):
        t.parent[i] = -1 if q.parent is None else idx[q.parent]
        t.allow_lent[i] = 1 if q.allow_lent else 0
        for r, v in q.max.items():
            d = DIMS.index(r)
            t.max[d, i] = v
            t.max_mask[i] |= 1 << d
        for r, v in q.min.items():
            t.min[DIMS.index(r), i] = v
        for r, v in q.guaranteed.items():
            t.guaranteed[DIMS.index(r), i] = v
        for r, v in q.self_request.items():
            t.self_request[DIMS.index(r), i] = v
        src = q.shared_weight if q.shared_weight is not None else q.max
        any_sw |= q.shared_weight is not None
        for r, v in src.items():
            sw[DIMS.index(r), i] = v
    t.shared_weight = sw if any_sw else None
    for r, v in cluster_total.items():
        t.cluster_total[DIMS.index(r)] = v
    return t


def random_quotas(rng, n, dims=("cpu", "memory", "ephemeral-storage"), depth=4):
    quotas = []
    for i in range(n):
        parent = None
        if i > 0 and rng.random() < 0.7:
            cand = [q for q in quotas if q.name.count("/") < depth - 1]
            if cand:
                parent = cand[int(rng.integers(len(cand)))].name
        name = f"{parent}/q{i}" if parent else f"q{i}"
        mx = {r: int(rng.integers(0, 200_000)) for r in dims if rng.random() < 0.9}
        mn = {r: int(rng.integers(0, v + 1)) for r, v in mx.items() if rng.random() < 0.8}
        sw = {r: int(rng.integers(0, 100)) for r in dims} if rng.random() < 0.5 else None
        req = {r: int(rng.integers(0, 150_000)) for r in dims if rng.random() < 0.6}
        gu = {r: int(rng.integers(0, 50_000)) for r in dims if rng.random() < 0.1}
        quotas.append(Quota(name=name, parent=parent, max=mx, min=mn, shared_weight=sw, guaranteed=gu,
                            self_request=req, allow_lent=bool(rng.random() < 0.7)))
    total = {r: int(rng.integers(0, 1_000_000)) for r in dims}
    return quotas, total


def runtime_matrix(quotas, rt):
    """oracle runtime dict -> [dim][quota] int64 over the union of Max keys (0 elsewhere)."""
    keys = set()
    for q in quotas:
        keys.update(q.max)
    out = np.zeros((abi.KS_QUOTA_DIMS, len(quotas)), np.int64)
    for i, q in enumerate(quotas):
        for r in keys:
            out[DIMS.index(r), i] = rt[q.name].get(r, 0)
    mask = 0
    for r in keys:
        mask |= 1 << DIMS.index(r)
    return out, mask
