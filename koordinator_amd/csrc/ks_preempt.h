// ks_preempt.h — the ElasticQuota PostFilter's preemption dry runs on the device.
//
// pkg/scheduler/plugins/elasticquota/plugin.go:302-321 hands the unschedulable pod to upstream's
// preemption.Evaluator.Preempt with the plugin as its Interface: every node whose filter status was not
// UnschedulableAndUnresolvable gets a dry run -- SelectVictimsOnNode (preempt.go:113-217) on a copy of its NodeInfo and of
// the ElasticQuota PostFilterState -- and pickOneNodeForPreemption chooses among the nodes that found victims.  One
// dry run touches one node's pods only, so the sweep is a wave per node:
//
//   preempt_dry_run_kernel  lane l holds the node's pods b + 64 s + l (slot s < S, S <= 4: nodes of up to 256 pods),
//                           host-sorted by util.MoreImportantPod.  canPreempt (:283-294) is per lane; removing every
//                           potential victim is a wave sum (NodeInfo.Requested and the pod count go down, the quota used
//                           goes down clamped at 0 -- SubtractWithNonNegativeResult of non-negative amounts, so the
//                           order does not matter); the Filter plugins run once on that; the PDB split
//                           (filterPodsWithPDBViolation :223-265) ranks, per budget, its members among the potential
//                           victims with ballots (a pod may match several budgets); the reprieve loop (:172-216) is wave-uniform over the victims in
//                           order, each step reading the pod's 15 request words from the lane that holds it.
//   preempt_select_kernel   one workgroup: PodEligibleToPreemptOthers (:60-97) on the nominated node, the candidate
//                           counts, the lexicographic minimum of pickOneNodeForPreemption's keys (fewest PDB violations,
//                           lowest first-victim priority, lowest priority sum, fewest victims, latest earliest start of
//                           the highest-priority victims, then the lowest node row), and the chosen node's victims.
#pragma once

#include "ks_device.h"
#include "ks_rsv.h"

namespace ks {

__device__ __forceinline__ int64_t pre_sum_i64(int64_t v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ int64_t pre_lane_i64(int64_t v, int l) { return (int64_t)readlane64((uint64_t)v, l); }

constexpr int kPreemptMaxSlots = 4;               // positions per lane
constexpr int kPreemptPdbs = 1 + KS_NPOD_MORE_PDBS;  // PodDisruptionBudgets one pod may match
constexpr int kPreemptMaxPods = 64 * kPreemptMaxSlots;  // pods per node the dry run holds

// NodeInfo.Pods of every node, positions in (node, MoreImportantPod, caller row) order (ks_load_node_pods)
struct DevNodePods {
  const int64_t* beg;   // [n + 1]
  const int32_t* prio;
  const int64_t* start;
  const uint32_t* flags;
  const int32_t* quota;
  const int32_t* pdb;   // [kPreemptPdbs][m], -1 = none
  const int32_t* row;   // caller row
  const int64_t* req;   // [kRsvDims][m]: cpu, memory, ephemeral, scalar[k] (NodeInfo.Requested share)
  const int64_t* qreq;  // [KS_QUOTA_DIMS][m]
  const int32_t* pdb_allowed;
  int64_t m;
  int32_t npdb;
};

// one node's dry-run outcome: pickOneNodeForPreemption's keys
struct PreemptCand {
  int32_t status, nviol, hprio, nvict;
  int64_t sum, earliest;
};

struct PreemptOut {
  int32_t node;
  uint32_t status;
  int32_t nvict, nviol, candidates, potential;
};

struct PreemptArgs {
  const DevNodes* dn;
  DevNodePods t;
  DevQuotas q;
  DevPodQuota pq;  // the preemptor's quota request (column 0)
  Cfg c;
  const PodRec* pod;
  const PodStat* pst;
  int32_t prio;
  uint32_t pflags;  // KS_PREEMPT_*
  int32_t nominated;
  const uint8_t* unresolvable;  // [n] or null
  int64_t n;
  PreemptCand* cand;  // [n]
  int32_t* vrank;     // [m]: the position's index in its node's victims, -1 (written by the dry run)
  uint8_t* status;    // [n] KS_PN_*
  PreemptOut* out;
  int32_t* victims;   // [kPreemptMaxPods]: the chosen node's victims as caller rows
};

// upstream fitsRequest (noderesources/fit.go) on the dry run's Requested / pod count (free = Allocatable - Requested)
__device__ __forceinline__ bool dry_fit(const Cfg& c, const PodRec& p, const int64_t* free, int64_t pods, int64_t allowed) {
  if (!c.fit_filter) return true;
  if (pods + 1 > allowed) return false;
  if (p.flags & kPodAllZero) return true;
  if (p.cpu > free[0] || p.mem > free[1] || p.eph > free[2]) return false;
#pragma unroll
  for (int k = 0; k < KS_MAX_SCALARS; ++k)
    if (p.sc[k] != 0 && p.sc[k] > free[3 + k]) return false;
  return true;
}

template <int S>
__global__ __launch_bounds__(256) void preempt_dry_run_kernel(PreemptArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t n = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (n >= a.n) return;
  PreemptCand out{KS_PN_UNRESOLVABLE, 0, 0, 0, 0, 0};
  auto finish = [&]() {
    if (lane == 0) {
      a.cand[n] = out;
      a.status[n] = (uint8_t)out.status;
    }
  };
  const int64_t b = a.t.beg[n], cnt = a.t.beg[n + 1] - b;
  for (int64_t i = lane; i < cnt; i += 64) a.vrank[b + i] = -1;  // (the victims' ranks are written after these)
  if (a.unresolvable && a.unresolvable[n]) {  // nodesWherePreemptionMightHelp
    finish();
    return;
  }
  const PodRec p = load_pod_uniform(a.pod);
  const int32_t Q = p.quota;
  // ---- the node's pods, canPreempt (preempt.go:283-294) ----
  bool canp[S], inq[S];
  int32_t pdbv[S][kPreemptPdbs], prv[S];
  int64_t stv[S], rq[S][kRsvDims], qq[S][KS_QUOTA_DIMS];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int64_t i = 64 * s + lane;
    const bool ok = i < cnt;
    const int64_t pos = b + (ok ? i : 0);
    const uint32_t f = ok ? gld(a.t.flags + pos) : KS_NPOD_NONPREEMPTIBLE;
    prv[s] = ok ? gld(a.t.prio + pos) : 0;
    stv[s] = ok ? gld(a.t.start + pos) : 0;
#pragma unroll
    for (int k = 0; k < kPreemptPdbs; ++k) pdbv[s][k] = ok ? gld(a.t.pdb + (int64_t)k * a.t.m + pos) : -1;
    const int32_t vq = ok ? gld(a.t.quota + pos) : -1;
    canp[s] = ok && !(f & KS_NPOD_NONPREEMPTIBLE) && a.prio > prv[s] && vq == Q;
    inq[s] = (f & KS_NPOD_IN_QUOTA) != 0;
#pragma unroll
    for (int d = 0; d < kRsvDims; ++d) rq[s][d] = canp[s] ? gld(a.t.req + (int64_t)d * a.t.m + pos) : 0;
#pragma unroll
    for (int d = 0; d < KS_QUOTA_DIMS; ++d) qq[s][d] = (canp[s] && inq[s]) ? gld(a.t.qreq + (int64_t)d * a.t.m + pos) : 0;
  }
  // ---- remove every potential victim: NodeInfo.RemovePod + ElasticQuota RemovePod (plugin.go:283-299) ----
  int32_t nv = 0;
  int64_t dreq[kRsvDims], dq[KS_QUOTA_DIMS];
#pragma unroll
  for (int d = 0; d < kRsvDims; ++d) {
    int64_t v = 0;
#pragma unroll
    for (int s = 0; s < S; ++s) v += rq[s][d];
    dreq[d] = pre_sum_i64(v);
  }
#pragma unroll
  for (int d = 0; d < KS_QUOTA_DIMS; ++d) {
    int64_t v = 0;
#pragma unroll
    for (int s = 0; s < S; ++s) v += qq[s][d];
    dq[d] = pre_sum_i64(v);
  }
  uint64_t pm[S];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    pm[s] = __ballot(canp[s]);
    nv += __popcll(pm[s]);
  }
  if (nv == 0) {
    out.status = KS_PN_NO_VICTIMS;
    finish();
    return;
  }
  const DevNodes& d = *a.dn;
  const int64_t alloc[kRsvDims] = {gld(d.alloc_cpu + n), gld(d.alloc_mem + n), gld(d.alloc_eph + n), gld(d.alloc_sc[0] + n),
                                   gld(d.alloc_sc[1] + n), gld(d.alloc_sc[2] + n), gld(d.alloc_sc[3] + n)};
  const int64_t reqn[kRsvDims] = {gld(d.req_cpu + n), gld(d.req_mem + n), gld(d.req_eph + n), gld(d.req_sc[0] + n),
                                  gld(d.req_sc[1] + n), gld(d.req_sc[2] + n), gld(d.req_sc[3] + n)};
  int64_t free[kRsvDims];
#pragma unroll
  for (int k = 0; k < kRsvDims; ++k) free[k] = alloc[k] - (reqn[k] - dreq[k]);
  int64_t pods = (int64_t)gld(d.pod_count + n) - nv;
  const int64_t allowed = gld(d.allowed_pods + n);
  int64_t used[KS_QUOTA_DIMS], limit[KS_QUOTA_DIMS], preq[KS_QUOTA_DIMS];
  const uint32_t lmask = gld(a.q.limit_mask + Q), pmask = gld(a.pq.mask);
#pragma unroll
  for (int k = 0; k < KS_QUOTA_DIMS; ++k) {
    const int64_t u = gld(a.q.used + (int64_t)Q * KS_QUOTA_DIMS + k) - dq[k];
    used[k] = u > 0 ? u : 0;
    limit[k] = gld(a.q.limit + (int64_t)Q * KS_QUOTA_DIMS + k);
    preq[k] = gld(a.pq.req[k]);
  }
  // ---- RunFilterPluginsWithNominatedPods with every potential victim gone (no nominated pods) ----
  bool static_ok = true;
  if (a.c.la_filter && !(p.flags & KS_POD_DAEMONSET))
    static_ok = !(gld(d.la_bits + n) & ((p.flags & KS_POD_PROD) ? kLaFailProd : kLaFailNonProd));
  if (a.c.stat) {
    EvalOut so{};
    stat_eval(a.c, *a.pst, gld(d.taints_hard + n), 0ull, gld(d.labels + n), 0ull, so);
    static_ok = static_ok && so.reasons == 0;
  }
  if (!static_ok || !dry_fit(a.c, p, free, pods, allowed)) {
    out.status = KS_PN_FILTER;
    finish();
    return;
  }
  // ---- filterPodsWithPDBViolation (preempt.go:222-265): each potential victim, in the sorted order, decrements every
  // budget it matches; it violates when one of them goes below 0.  Wave-uniform over the distinct budgets the node's
  // potential victims match: one ballot per (slot, list entry) gives a budget's members, and a member's rank among
  // them (the decrements before its own) is the popcount of the members at earlier positions. ----
  uint64_t vm[S], pend[S][kPreemptPdbs];
  bool viol[S];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    viol[s] = false;
#pragma unroll
    for (int k = 0; k < kPreemptPdbs; ++k) pend[s][k] = __ballot(canp[s] && pdbv[s][k] >= 0 && pdbv[s][k] < a.t.npdb);
  }
  const uint64_t lt_mask = (1ull << lane) - 1ull;
  for (;;) {
    int32_t j = -1;  // the next budget (wave-uniform)
#pragma unroll
    for (int s = 0; s < S; ++s)
#pragma unroll
      for (int k = 0; k < kPreemptPdbs; ++k)
        if (j < 0 && pend[s][k]) j = __builtin_amdgcn_readlane(pdbv[s][k], (int)__builtin_ctzll(pend[s][k]));
    if (j < 0) break;
    const int32_t allowed = gld(a.t.pdb_allowed + j);
    int32_t before = 0;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      uint64_t mem = 0;
#pragma unroll
      for (int k = 0; k < kPreemptPdbs; ++k) {
        const uint64_t mk = __ballot(canp[s] && pdbv[s][k] == j);
        mem |= mk;
        pend[s][k] &= ~mk;
      }
      if (((mem >> lane) & 1ull) && before + __popcll(mem & lt_mask) + 1 > allowed) viol[s] = true;
      before += __popcll(mem);
    }
  }
#pragma unroll
  for (int s = 0; s < S; ++s) vm[s] = __ballot(viol[s]);
  // ---- reprievePod (preempt.go:172-216): the violating victims first, then the others, each in the sorted order ----
  int32_t nvict = 0, nviol = 0, maxp = 0;
  int64_t sum = 0, earliest = 0;
  bool err = false;
  for (int pass = 0; pass < 2 && !err; ++pass) {
#pragma unroll
    for (int s = 0; s < S; ++s) {
      uint64_t m = pass == 0 ? (pm[s] & vm[s]) : (pm[s] & ~vm[s]);
      while (m && !err) {
        const int k = __builtin_ctzll(m);
        m &= m - 1;
        int64_t r[kRsvDims], qv[KS_QUOTA_DIMS];
#pragma unroll
        for (int dd = 0; dd < kRsvDims; ++dd) r[dd] = pre_lane_i64(rq[s][dd], k);
#pragma unroll
        for (int dd = 0; dd < KS_QUOTA_DIMS; ++dd) qv[dd] = pre_lane_i64(qq[s][dd], k);
        const int32_t pr = __builtin_amdgcn_readlane(prv[s], k);
        const int64_t st = pre_lane_i64(stv[s], k);
        // addPod: NodeInfo.AddPodInfo + ElasticQuota AddPod (used += the pod's request when it is in the quota)
#pragma unroll
        for (int dd = 0; dd < kRsvDims; ++dd) free[dd] -= r[dd];
        ++pods;
#pragma unroll
        for (int dd = 0; dd < KS_QUOTA_DIMS; ++dd) used[dd] += qv[dd];
        const bool fits = static_ok && dry_fit(a.c, p, free, pods, allowed);
        bool victim = false;
        if (!fits) {  // removePod again; the pod is a victim
#pragma unroll
          for (int dd = 0; dd < kRsvDims; ++dd) free[dd] += r[dd];
          --pods;
#pragma unroll
          for (int dd = 0; dd < KS_QUOTA_DIMS; ++dd) used[dd] = used[dd] - qv[dd] > 0 ? used[dd] - qv[dd] : 0;
          victim = true;
        }
        // quotav1.LessThanOrEqual(Mask(Add(used, podReq), names(podReq)), usedLimit)
        bool exceed = false;
#pragma unroll
        for (int dd = 0; dd < KS_QUOTA_DIMS; ++dd)
          exceed |= ((lmask & pmask) >> dd & 1u) && used[dd] + preq[dd] > limit[dd];
        if (exceed) {
          if (!fits) {  // the pod is no longer on the node: NodeInfo.RemovePod fails
            err = true;
            break;
          }
#pragma unroll
          for (int dd = 0; dd < kRsvDims; ++dd) free[dd] += r[dd];
          --pods;
#pragma unroll
          for (int dd = 0; dd < KS_QUOTA_DIMS; ++dd) used[dd] = used[dd] - qv[dd] > 0 ? used[dd] - qv[dd] : 0;
          victim = true;
        }
        if (pass == 0 && !fits) ++nviol;
        if (victim) {
          if (lane == 0) a.vrank[b + 64 * s + k] = nvict;
          // util.GetEarliestPodStartTime over the victims in order; Pods[0] is pickOneNodeForPreemption's "highest"
          if (nvict == 0) {
            out.hprio = pr;
            maxp = pr;
            earliest = st;
          } else if (pr == maxp) {
            earliest = st < earliest ? st : earliest;
          } else if (pr > maxp) {
            maxp = pr;
            earliest = st;
          }
          sum += (int64_t)pr + 2147483648ll;
          ++nvict;
        }
      }
    }
  }
  out.nviol = nviol;
  out.nvict = nvict;
  out.sum = sum;
  out.earliest = earliest;
  // DryRunPreemption: success without a victim is an error too ("expected at least one victim pod on node")
  out.status = (err || nvict == 0) ? KS_PN_ERROR : KS_PN_CANDIDATE;
  finish();
}

// pickOneNodeForPreemption's order: fewer PDB violations, lower first-victim priority, lower sum of priorities, fewer
// victims, later earliest start, lower node row (the reference iterates a map there)
__device__ __forceinline__ bool preempt_better(const PreemptCand& x, int64_t xn, const PreemptCand& y, int64_t yn) {
  if (xn < 0) return false;
  if (yn < 0) return true;
  if (x.nviol != y.nviol) return x.nviol < y.nviol;
  if (x.hprio != y.hprio) return x.hprio < y.hprio;
  if (x.sum != y.sum) return x.sum < y.sum;
  if (x.nvict != y.nvict) return x.nvict < y.nvict;
  if (x.earliest != y.earliest) return x.earliest > y.earliest;
  return xn < yn;
}

constexpr int kPreemptSelThreads = 1024;

__global__ __launch_bounds__(kPreemptSelThreads) void preempt_select_kernel(PreemptArgs a) {
  __shared__ PreemptCand sc[kPreemptSelThreads];
  __shared__ int64_t sn[kPreemptSelThreads];
  __shared__ int32_t scnt[3][kPreemptSelThreads / 64];
  __shared__ int32_t s_blocked;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid == 0) s_blocked = (a.pflags & KS_PREEMPT_NEVER) ? 1 : 0;
  __syncthreads();
  // PodEligibleToPreemptOthers: a terminating lower-priority pod of the same quota on the nominated node (unless the
  // nominated node's status was UnschedulableAndUnresolvable)
  const int32_t Q = a.pod->quota;
  if (a.nominated >= 0 && a.nominated < a.n && !(a.unresolvable && a.unresolvable[a.nominated])) {
    for (int64_t pos = a.t.beg[a.nominated] + tid; pos < a.t.beg[a.nominated + 1]; pos += kPreemptSelThreads)
      if ((a.t.flags[pos] & KS_NPOD_TERMINATING) && a.t.quota[pos] == Q && a.t.prio[pos] < a.prio)
        atomicOr(&s_blocked, 1);
  }
  __syncthreads();
  if (s_blocked) {
    for (int64_t i = tid; i < a.n; i += kPreemptSelThreads) a.status[i] = KS_PN_UNRESOLVABLE;
    if (tid == 0) *a.out = PreemptOut{-1, KS_P_NOT_ELIGIBLE, 0, 0, 0, 0};
    return;
  }
  PreemptCand best{};
  int64_t bn = -1;
  int32_t pot = 0, cands = 0, errs = 0;
  // kSelPro candidates per thread in flight at once (one HBM round trip for 8k nodes, not one per 1,024); the order
  // of the comparisons does not matter (preempt_better is a total order).  (Fusing this selection into the dry-run
  // launch behind a last-workgroup ticket measured slower: each workgroup's device-scope release fence writes back its
  // XCD's L2, 64 -> 79 us per call.)
  constexpr int kSelPro = 8;
  for (int64_t i0 = tid; i0 < a.n; i0 += (int64_t)kPreemptSelThreads * kSelPro) {
    PreemptCand cb[kSelPro];
#pragma unroll
    for (int u = 0; u < kSelPro; ++u) {
      const int64_t i = i0 + (int64_t)u * kPreemptSelThreads;
      if (i < a.n) cb[u] = a.cand[i];
    }
#pragma unroll
    for (int u = 0; u < kSelPro; ++u) {
      const int64_t i = i0 + (int64_t)u * kPreemptSelThreads;
      if (i >= a.n) continue;
      const PreemptCand& c = cb[u];
      pot += c.status != KS_PN_UNRESOLVABLE;
      errs += c.status == KS_PN_ERROR;
      if (c.status != KS_PN_CANDIDATE) continue;
      ++cands;
      if (preempt_better(c, i, best, bn)) {
        best = c;
        bn = i;
      }
    }
  }
  pot = wave_sum_i32(pot);
  cands = wave_sum_i32(cands);
  errs = wave_sum_i32(errs);
  if (lane == 0) {
    scnt[0][wv] = pot;
    scnt[1][wv] = cands;
    scnt[2][wv] = errs;
  }
  sc[tid] = best;
  sn[tid] = bn;
  __syncthreads();
  for (int w = kPreemptSelThreads / 2; w > 0; w >>= 1) {
    if (tid < w && preempt_better(sc[tid + w], sn[tid + w], sc[tid], sn[tid])) {
      sc[tid] = sc[tid + w];
      sn[tid] = sn[tid + w];
    }
    __syncthreads();
  }
  const int64_t node = sn[0];
  if (tid == 0) {
    int32_t p = 0, c = 0, e = 0;
    for (int w = 0; w < kPreemptSelThreads / 64; ++w) {
      p += scnt[0][w];
      c += scnt[1][w];
      e += scnt[2][w];
    }
    PreemptOut o{-1, (uint32_t)(c ? KS_P_NOMINATED : (e ? KS_P_ERROR : KS_P_NO_CANDIDATE)), 0, 0, c, p};
    if (node >= 0) {
      o.node = (int32_t)node;
      o.nvict = sc[0].nvict;
      o.nviol = sc[0].nviol;
    }
    *a.out = o;
  }
  if (node >= 0)
    for (int64_t pos = a.t.beg[node] + tid; pos < a.t.beg[node + 1]; pos += kPreemptSelThreads) {
      const int32_t r = a.vrank[pos];
      if (r >= 0) a.victims[r] = a.t.row[pos];
    }
}

}  // namespace ks
