// ks_numa.h — NodeNUMAResource on nodes with a NUMA topology policy (SURVEY a24 hints, a25 topology manager).
//
// Per (pod, node): the NUMA plugin's hints (generateResourceHints, resource_manager.go:459-593: per NUMA-node
// mask in IterateBitMasks order, a hint per requested resource when the mask's total and free amounts
// cover the request; preferred = the narrowest mask size that could hold it; hint score = the
// NUMAScoringStrategy scorer over the mask), the topology manager merge (topologymanager/policy.go:96-187,
// cpu then memory list, first list outermost) with the best-effort / restricted / single-numa-node policy,
// the NUMA allocation of the merged hint (tryBestToDistributeEvenly, resource_manager.go:221-283, including
// its slice-position comparator) and the node score over the allocated NUMA nodes
// (calculateAllocatableAndRequested, scoring.go:116-163).  Up to kNumaDev NUMA nodes per node: at most 15
// masks and 225 hint permutations per lane.  The oracle (oracle/koord_oracle.c numa_policy_eval) restates
// the same code independently with per-NUMA arrays.
#pragma once

#include "ks_device.h"

namespace ks {

constexpr int kNumaDev = 4;  // NUMA nodes per node the device evaluates
constexpr int kNumaMasks = (1 << kNumaDev) - 1;

struct DevNuma {
  const int32_t* count;  // [npad] NUMA nodes with resources
  const int64_t* total;  // [2][kNumaDev][npad] amplified NUMANodeResources (cpu milli, memory)
  int64_t* used;         // [2][kNumaDev][npad] allocatedResources (raw; mutable)
  const int64_t* off;    // [kNumaDev][npad] cpuset amplification of the allocated cpu: Amplify(cs) - cs
  uint32_t* present;     // [npad] bit k: an allocatedResources entry exists (mutable)
  const uint32_t* flags; // [npad] ks_node_cols.numa_flags (policy in bits 5-6)
  int64_t npad;
};

// node view: HBM columns or the commit kernel's LDS copy (tot/use[r*kNumaDev+k], off[k])
struct NumaGView {
  const DevNuma& d;
  int64_t n;
  __device__ __forceinline__ int policy() const { return (int)((gld(d.flags + n) >> KS_NUMA_POLICY_SHIFT) & 3u); }
  __device__ __forceinline__ int count() const { return gld(d.count + n); }
  __device__ __forceinline__ uint32_t present() const { return gld(d.present + n); }
  __device__ __forceinline__ int64_t total(int r, int k) const { return gld(d.total + ((int64_t)r * kNumaDev + k) * d.npad + n); }
  __device__ __forceinline__ int64_t used(int r, int k) const { return gld(d.used + ((int64_t)r * kNumaDev + k) * d.npad + n); }
  __device__ __forceinline__ int64_t off(int k) const { return gld(d.off + (int64_t)k * d.npad + n); }
};

struct NumaLView {
  const int64_t* w;  // [2*kNumaDev total | 2*kNumaDev used | kNumaDev off | meta]
  __device__ __forceinline__ int policy() const { return (int)(w[5 * kNumaDev] & 3); }
  __device__ __forceinline__ int count() const { return (int)((w[5 * kNumaDev] >> 8) & 0xFF); }
  __device__ __forceinline__ uint32_t present() const { return (uint32_t)(w[5 * kNumaDev] >> 32); }
  __device__ __forceinline__ int64_t total(int r, int k) const { return w[r * kNumaDev + k]; }
  __device__ __forceinline__ int64_t used(int r, int k) const { return w[2 * kNumaDev + r * kNumaDev + k]; }
  __device__ __forceinline__ int64_t off(int k) const { return w[4 * kNumaDev + k]; }
};
constexpr int kNumaSlotWords = 5 * kNumaDev + 1;

struct NumaPolOut {
  uint32_t reasons;
  int32_t score;
  int64_t alloc[2][kNumaDev];  // the pod's NUMA allocation (cpu milli, memory)
};

// resourceAllocationScorer.score over cpu / memory with the plugin weights (scoring.go:206-242)
__device__ __forceinline__ int32_t numa_res_score(const Cfg& c, bool most, int64_t rq_cpu, int64_t rq_mem,
                                                  int64_t al_cpu, int64_t al_mem, const PodRec& p) {
  int32_t ns = 0, ws = 0;
  if (c.nw_cpu && al_cpu != 0) {
    const int64_t rq = rq_cpu + p.cpu;
    ns += (most ? pct_floor_i64(rq > al_cpu ? al_cpu : rq, al_cpu) : (rq > al_cpu ? 0 : pct_floor_i64(al_cpu - rq, al_cpu))) * c.nw_cpu;
    ws += c.nw_cpu;
  }
  if (c.nw_mem && al_mem != 0) {
    const int64_t rq = rq_mem + p.mem;
    ns += (most ? pct_floor_i64(rq > al_mem ? al_mem : rq, al_mem) : (rq > al_mem ? 0 : pct_floor_i64(al_mem - rq, al_mem))) * c.nw_mem;
    ws += c.nw_mem;
  }
  return ws ? small_div(ns, ws) : 0;
}

// IterateBitMasks order for K NUMA nodes: size 1..K, lexicographic index lists (bitmask.go:206-222)
__device__ __forceinline__ int numa_masks(int K, uint32_t* m) {
  int n = 0;
  for (int size = 1; size <= K; ++size) {
    for (int i0 = 0; i0 < K; ++i0) {
      if (size == 1) { m[n++] = 1u << i0; continue; }
      for (int i1 = i0 + 1; i1 < K; ++i1) {
        if (size == 2) { m[n++] = (1u << i0) | (1u << i1); continue; }
        for (int i2 = i1 + 1; i2 < K; ++i2) {
          if (size == 3) { m[n++] = (1u << i0) | (1u << i1) | (1u << i2); continue; }
          for (int i3 = i2 + 1; i3 < K; ++i3) m[n++] = (1u << i0) | (1u << i1) | (1u << i2) | (1u << i3);
        }
      }
    }
  }
  return n;
}

__device__ __forceinline__ bool numa_narrower(uint32_t a, uint32_t b) {
  const int ca = __builtin_popcount(a), cb = __builtin_popcount(b);
  return ca == cb ? a < b : ca < cb;
}

// Filter (FilterByNUMANode -> Admit -> Allocate) and Score of one (pod, node) with a NUMA policy.
// plain_*: nodeInfo.Requested / Allocatable for the score when the allocation holds no NUMA node.
template <typename V>
__device__ __forceinline__ NumaPolOut numa_policy_eval(const Cfg& c, const PodRec& p, const V& v, int64_t plain_req_cpu,
                                                       int64_t plain_req_mem, int64_t plain_alloc_cpu,
                                                       int64_t plain_alloc_mem) {
  NumaPolOut o;
  o.reasons = 0;
  o.score = 0;
#pragma unroll
  for (int k = 0; k < kNumaDev; ++k) o.alloc[0][k] = o.alloc[1][k] = 0;
  const int K = v.count();
  if (K == 0) {
    o.reasons = KS_R_NUMA_MISSING;
    return o;
  }
  const int pol = v.policy();
  const uint32_t pres = v.present();
  int64_t tot[2][kNumaDev], use[2][kNumaDev], av[2][kNumaDev];
#pragma unroll
  for (int k = 0; k < kNumaDev; ++k) {
    const bool in = k < K, pr = in && ((pres >> k) & 1u);
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      tot[r][k] = in ? v.total(r, k) : 0;
      use[r][k] = pr ? v.used(r, k) + (r == 0 ? v.off(k) : 0) : 0;
      const int64_t a = tot[r][k] - use[r][k];
      av[r][k] = a < 0 ? 0 : a;
    }
  }
  const int64_t req[2] = {p.cpu, p.mem};
  const bool want[2] = {p.cpu != 0, p.mem != 0};
  uint32_t masks[kNumaMasks];
  const int nm = numa_masks(K, masks);
  uint32_t lack[2] = {0u, 0u};
#pragma unroll
  for (int k = 0; k < kNumaDev; ++k)
#pragma unroll
    for (int r = 0; r < 2; ++r)
      if (k < K && av[r][k] == 0) lack[r] |= 1u << k;
  // hints: bit i of hset[r] = mask i is a hint of resource r; one score per mask
  uint32_t hset[2] = {0u, 0u};
  int min_size[2] = {K, K};
  int32_t hsc[kNumaMasks];
  const bool nmost = c.numa_sc_most != 0;
  for (int i = 0; i < nm; ++i) {
    int64_t ts[2] = {0, 0}, fs[2] = {0, 0};
#pragma unroll
    for (int k = 0; k < kNumaDev; ++k)
      if ((masks[i] >> k) & 1u)
#pragma unroll
        for (int r = 0; r < 2; ++r) {
          ts[r] += tot[r][k];
          fs[r] += av[r][k];
        }
    hsc[i] = numa_res_score(c, nmost, ts[0] - fs[0], ts[1] - fs[1], ts[0], ts[1], p);
    const int cnt = __builtin_popcount(masks[i]);
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      if (!want[r] || ts[r] < req[r] || (masks[i] & lack[r])) continue;
      min_size[r] = cnt < min_size[r] ? cnt : min_size[r];
      if (fs[r] >= req[r]) hset[r] |= 1u << i;
    }
  }
  // filterProvidersHints: the lists (cpu, then memory) — a hint entry is (mask index, or -1 = nil)
  int nl = 0;
  int lres[2];
#pragma unroll
  for (int r = 0; r < 2; ++r)
    if (want[r]) lres[nl++] = r;
  const bool single = pol == KS_NUMA_POLICY_SINGLE_NUMA_NODE;
  auto pref_of = [&](int r, int i) { return __builtin_popcount(masks[i]) == min_size[r]; };
  // list l: entries = hint masks of lres[l] (filtered for single-numa-node), or one nil non-preferred
  // entry when the resource has no hint (single-numa-node drops it: the list becomes empty)
  uint32_t lset[2] = {0u, 0u};
  bool lnil[2] = {false, false};
  for (int l = 0; l < nl; ++l) {
    const int r = lres[l];
    if (hset[r] == 0) {
      lnil[l] = !single;  // {nil, false}: kept by best-effort / restricted, dropped by single-numa-node
    } else {
      uint32_t s = hset[r];
      if (single) {
        uint32_t f = 0;
        for (int i = 0; i < nm; ++i)
          if (((s >> i) & 1u) && __builtin_popcount(masks[i]) == 1 && pref_of(r, i)) f |= 1u << i;
        s = f;
      }
      lset[l] = s;
    }
  }
  const uint32_t dflt = (1u << K) - 1u;
  uint32_t best_mask = dflt;
  bool best_pref = false;
  int32_t best_score = 0;
  if (nl == 0) {
    best_pref = true;  // no NUMA resource requested: one preferred any-numa hint
  } else {
    bool empty = false;
    for (int l = 0; l < nl; ++l) empty |= (lset[l] == 0 && !lnil[l]);
    if (!empty) {
      // entries of list l: -1 (nil) or the mask indices of lset[l] in order
      const int n0 = lnil[0] ? 1 : __builtin_popcount(lset[0]);
      const int n1 = nl > 1 ? (lnil[1] ? 1 : __builtin_popcount(lset[1])) : 1;
      int e0 = -1;
      uint32_t rest0 = lset[0];
      for (int a = 0; a < n0; ++a) {
        if (!lnil[0]) {
          e0 = __builtin_ctz(rest0);
          rest0 &= rest0 - 1;
        }
        uint32_t rest1 = nl > 1 ? lset[1] : 0u;
        for (int b = 0; b < n1; ++b) {
          int e1 = -2;  // -2: no second list
          if (nl > 1) {
            if (lnil[1]) e1 = -1;
            else {
              e1 = __builtin_ctz(rest1);
              rest1 &= rest1 - 1;
            }
          }
          // mergePermutation
          uint32_t merged = dflt, first = 0;
          bool pref = true, have = false;
          const int es[2] = {e0, e1};
          for (int l = 0; l < nl; ++l) {
            const int e = es[l];
            const bool hp = e >= 0 ? pref_of(lres[l], e) : false;  // nil entries here are {nil, false}
            if (e >= 0) {
              const uint32_t m = masks[e];
              if (!have) first = m;
              else if (m != first) pref = false;
              have = true;
              merged &= m;
            }
            if (!hp) pref = false;
          }
          if (merged == 0) continue;
          int32_t msc = 0;
          for (int l = 0; l < nl; ++l)
            if (es[l] >= 0 && masks[es[l]] == merged && hsc[es[l]] > msc) msc = hsc[es[l]];
          if (pref && !best_pref) {
            best_mask = merged; best_pref = true; best_score = msc;
          } else if (!pref && best_pref) {
          } else if (!numa_narrower(merged, best_mask)) {
            if (__builtin_popcount(merged) == __builtin_popcount(best_mask) && msc > best_score) {
              best_mask = merged; best_pref = pref; best_score = msc;
            }
          } else {
            best_mask = merged; best_pref = pref; best_score = msc;
          }
        }
      }
    }
  }
  uint32_t affinity = best_mask;
  bool admit = true;
  if (single) {
    if (affinity == dflt) affinity = 0u;
    admit = best_pref;
  } else if (pol == KS_NUMA_POLICY_RESTRICTED) {
    admit = best_pref;
  }
  if (!admit) {
    o.reasons = KS_R_NUMA_AFFINITY;
    return o;
  }
  if (affinity) {
    int bits[kNumaDev], nb = 0;
#pragma unroll
    for (int k = 0; k < kNumaDev; ++k)
      if ((affinity >> k) & 1u) bits[nb++] = k;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      if (!want[r]) continue;
      int ord[kNumaDev];
#pragma unroll
      for (int i = 0; i < kNumaDev; ++i) ord[i] = i < nb ? bits[i] : 0;
      // sort.Slice insertion sort with less(i, j) comparing totalAvailable by slice position
      for (int i = 1; i < nb; ++i)
        for (int j = i; j > 0; --j) {
          const int64_t aj = j < K ? av[r][j] : 0, ai = (j - 1) < K ? av[r][j - 1] : 0;
          if (!(aj < ai)) break;
          const int t = ord[j];
          ord[j] = ord[j - 1];
          ord[j - 1] = t;
        }
      int64_t q = req[r];
      for (int i = 0; i < nb; ++i) {
        const int64_t split = q / (nb - i);
        const int64_t a = av[r][ord[i]];
        const int64_t got = a > split ? split : a;
        o.alloc[r][ord[i]] = got;
        q -= got;
      }
      if (q != 0) {
        o.reasons = KS_R_NUMA_INSUFFICIENT;
        return o;
      }
    }
  }
  int64_t trq[2] = {0, 0}, tal[2] = {0, 0};
  bool any = false;
#pragma unroll
  for (int k = 0; k < kNumaDev; ++k) {
    if (o.alloc[0][k] == 0 && o.alloc[1][k] == 0) continue;
    any = true;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      tal[r] += tot[r][k];
      trq[r] += use[r][k];
    }
  }
  if (!any) {
    trq[0] = plain_req_cpu;
    trq[1] = plain_req_mem;
    tal[0] = plain_alloc_cpu;
    tal[1] = plain_alloc_mem;
  }
  o.score = numa_res_score(c, c.numa_most != 0, trq[0], trq[1], tal[0], tal[1], p);
  return o;
}

// Replace the policy-None NodeNUMAResource result of eval with the policy path's (the amplified-CPU
// filter and a cpu-bind topology failure come first, plugin.go:275-338).
template <bool DEBUG>
__device__ __forceinline__ void numa_policy_apply(const Cfg& c, const PodRec& p, EvalOut& o, uint32_t numa_rs,
                                                  const NumaPolOut& pr) {
  if (p.flags & kPodReqZero) return;
  if (numa_rs == 0) o.reasons |= DEBUG ? pr.reasons : (pr.reasons ? KS_R_FIT_PODS : 0u);
  o.total += (pr.score - o.numa) * c.numa_pw;
  o.numa = pr.score;
}

// The policy path for one lane after eval_full: view_fn() gives the node's NUMA view.
template <int NSC, bool DEBUG, int FEAT, typename VF>
__device__ __forceinline__ void numa_policy_fix(const Cfg& c, const PodRec& p, const NodeReg<NSC>& r, EvalOut& o,
                                                VF&& view_fn) {
  if (!(FEAT & 8) || !c.numa || !c.numa_pol || (p.flags & kPodReqZero)) return;
  const auto v = view_fn();
  if (v.policy() == 0) return;
  const NumaPolOut pr = numa_policy_eval(c, p, v, r.t_ncpu.c - r.free_cpu, r.t_nmem.c - r.free_mem, r.t_ncpu.c, r.t_nmem.c);
  numa_policy_apply<DEBUG>(c, p, o, o.numa_rs, pr);
}

}  // namespace ks
