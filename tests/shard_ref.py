"""Numpy restatement of the per-pod candidate selection and of the shard merge — TEST INFRASTRUCTURE.

select_chunks mirrors koordgpu.hip select_kernel (every chunk above the K-th chunk score, plus the
first equal-score chunks in chunk order); merge_lists mirrors merge_kernel.  Used by the CPU gloo
test to check that merging per-shard lists reproduces a single select over every chunk.
"""
import numpy as np


def shard_ranges(nchunks, nshards):
    b = [nchunks * s // nshards for s in range(nshards + 1)]
    return [(b[s], b[s + 1]) for s in range(nshards)]


def select_chunks(h, K, c0=0):
    """h: chunk scores (0 = no feasible node) of chunks c0.. ; returns (chunk ids, total, exhaustive)."""
    h = np.asarray(h, np.int64)
    total = int((h > 0).sum())
    if total <= K:
        ids = np.nonzero(h > 0)[0]
        return list(ids + c0), total, True
    t = np.sort(h[h > 0])[::-1][K - 1]
    need_eq = K - int((h > t).sum())
    out, eq = [], 0
    for i, v in enumerate(h):
        if v > t:
            out.append(i + c0)
        elif v == t and v > 0:
            if eq < need_eq:
                out.append(i + c0)
            eq += 1
    return out, total, False


def merge_lists(lists, totals, h_of, K):
    """lists: per-shard chunk-id lists in shard order; h_of: chunk id -> score."""
    total = sum(totals)
    union = [c for lst in lists for c in lst]
    if total <= K:
        return union, True
    hs = np.array([h_of[c] for c in union], np.int64)
    t = np.sort(hs)[::-1][K - 1]
    need_eq = K - int((hs > t).sum())
    out, eq = [], 0
    for c, v in zip(union, hs):
        if v > t:
            out.append(c)
        elif v == t:
            if eq < need_eq:
                out.append(c)
            eq += 1
    return out, False
