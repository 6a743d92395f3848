// ks_topo.h — upstream PodTopologySpread and InterPodAffinity (kube-scheduler v1.24.15 plugins/podtopologyspread,
// plugins/interpodaffinity) on the device: the node counters and pod query terms of include/koordgpu.h
// ks_topology_args (compiled on the host by koordinator_amd/topology_plugins.py), the kernels that schedule a
// topology pod (KS_TOPO_DYN) alone against them, and the commit kernels' hooks.
//
// A topology pod's Filter needs per-domain sums over every eligible node (PreFilter) and its Score a normalization
// over every feasible node, so it cannot share a pass with other pods: the pass loop runs, before each regular pass,
// a topology step that acts only when the pod at the cursor is one --
//   eval_debug_kernel   every other plugin's Filter / Score on every node (ks_debug.hip, the ks_eval_pod path)
//   topo_filter_kernel  PreFilter domain sums (one workgroup, LDS) + both plugins' Filters, OR-ed into the reasons
//   topo_norm_kernel    the other plugins' normalizations, PodTopologySpread PreScore / Score / NormalizeScore and
//                       InterPodAffinity Score / NormalizeScore over the feasible nodes, the best node (max total,
//                       lowest index) as a one-candidate set
//   commit_kernel       (CommitArgs.topo = 2) admission + every Reserve on that node, the counters of the pod's
//                       properties
// -- and every regular pass ends before its first topology pod (CommitArgs.topo = 1).
#pragma once

#include <hip/hip_runtime.h>

#include <climits>

#include "ks_device.h"

namespace ks {

// internal pod flag (PodRec.flags): the pod has topology query terms (KS_TOPO_DYN)
constexpr uint32_t kPodTopoDyn = 0x4000u;

// Per pending pod, queue order (staged with the pod columns): the query terms and properties.
struct __attribute__((aligned(16))) TopoRec {
  uint64_t term[KS_TOPO_TERMS];
  uint32_t props, flags;
  int32_t nterms, _pad;
};
static_assert(sizeof(TopoRec) == 80, "TopoRec layout");

// Node side: zonal domain, per-property counters ([p][npad]), the topologyNormalizingWeight table
// lw[s] = log(s + 2) for s in [0, nlw) (computed by the host's libm, the oracle's log)
struct DevTopo {
  int32_t* zone;
  int32_t* count;
  int64_t npad;
  const double* lw;
  int32_t nlw;
};

// The topology step's reductions (HBM, one per context).  Every field is back at its initial value after each step
// (topo_norm_kernel's last workgroup resets it; topo_install writes the initial image).
struct TopoScratch {
  long long zsum[KS_TOPO_TERMS][KS_TOPO_ZONES];  // per term: the zone's counted pods over the term's eligible nodes (0)
  unsigned long long zpres[KS_TOPO_TERMS];        // hard spread: zones with an eligible node (0)
  int hmin[KS_TOPO_TERMS];                        // hard spread, hostname: min count over the eligible nodes (INT_MAX)
  int any_all;                                    // InterPodAffinity: affinityCounts is not empty (0)
  unsigned long long hsize, zones;                // feasible non-ignored nodes, their zones (0)
  int empty;                                      // a feasible non-ignored node without the zone label (0)
  int dev_max, taint_max, aff_max;                // DeviceShare / TaintToleration / NodeAffinity raw maxima (0)
  long long imin, imax;                           // InterPodAffinity raw extrema, from 0 (0)
  long long smin, smax;                           // PodTopologySpread raw extrema over the non-ignored nodes (LLONG_MAX, 0)
  unsigned long long rsv_pref, rsv_max;           // Reservation preferred-node key, raw max (0)
  unsigned long long best;                        // selectHost key (total + 1) << 32 | ~node (0)
  unsigned int done;                              // topo_norm_kernel workgroups finished (0)
  long long best_total;                           // the chosen node's total (the pod's result score)
  long long best_node;                            // ... the node (-1 = none feasible)
  // the step's pod, written by topo_sums_kernel (the first kernel of a step) from *cursor: the later kernels read it
  // with one load instead of the cursor -> record chain (-1 = the cursor's pod is not a topology pod)
  int32_t cur_pi, _pad1[3];
  TopoRec cur_rec;
};

__device__ __forceinline__ int tp_kind(uint64_t w) { return (int)(w & 0xFF); }
__device__ __forceinline__ int tp_prop(uint64_t w) { return (int)((w >> 8) & 0xFF); }
__device__ __forceinline__ int tp_key(uint64_t w) { return (int)((w >> 16) & 0xFF); }
__device__ __forceinline__ uint32_t tp_flags(uint64_t w) { return (uint32_t)((w >> 24) & 0xFF); }
__device__ __forceinline__ int32_t tp_param(uint64_t w) { return (int32_t)(uint32_t)(w >> 32); }

// nodeaffinity.GetRequiredNodeAffinity(pod).Match(node) over the label dictionary (NodeAffinity's Filter test)
__device__ __forceinline__ bool tp_node_aff(const PodStat* s, uint64_t labels) {
  if (!s || s->nreq <= 0) return true;
  bool ok = false;
  for (int t = 0; t < KS_AFFINITY_TERMS; ++t) ok |= t < s->nreq && (labels & s->req[t]) == s->req[t];
  return ok;
}

// ---- commit kernel hooks (ks_pass.h commit_kernel, ks_mono.h commit_mono_kernel) ----

// The pods the pass commits: mode 1 ends it before its first topology pod (0: the kernel returns, the topology step
// of the next iteration takes that pod), mode 2 (the topology step's commit) is the pod at the cursor if it is one,
// else nothing; mode 3 (ks_assume) and 0 leave np.  Wave-uniform (every wave computes the same ballot).
template <typename A>
__device__ __forceinline__ int32_t topo_pass_pods(const A& a, int32_t cursor0, int32_t np) {
  if (a.topo == 0 || a.topo == 3) return np;
  const int lane = threadIdx.x & 63;
  const uint32_t f = lane < np ? a.topo_rec[cursor0 + lane].flags : 0u;
  const uint64_t dyn = __ballot((f & KS_TOPO_DYN) != 0u);
  if (a.topo == 2) return (dyn & 1ull) ? 1 : 0;
  return dyn ? (int32_t)(__ffsll((long long)dyn) - 1) : np;
}

// Write-back of one result: the counters of the placed pod's properties (NodeInfo.AddPod), its score (the topology
// step's total; a pod without query terms gets PodTopologySpread's constant 100 x weight on every node)
template <typename A>
__device__ __forceinline__ void topo_writeback(const A& a, int32_t pod, ks_result& r) {
  if (a.topo == 0 || r.status != KS_S_SCHEDULED || r.node < 0) return;
  const TopoRec& t = a.topo_rec[pod];
  if (a.topo == 2) r.score = *a.topo_best;
  else if (a.topo == 1 && !(t.flags & KS_TOPO_DYN)) r.score += a.topo_const;
  uint32_t m = t.props;
  while (m) {
    const int q = __ffs((int)m) - 1;
    m &= m - 1u;
    atomicAdd(a.topo_count + (int64_t)q * a.topo_npad + r.node, 1);
  }
}

// ---- topology step kernels (ks_topo.hip) ----

struct TopoKArgs {
  DevTopo t;
  const uint64_t* labels;  // DevNodes.labels (required node affinity of the spread constraints)
  const PodStat* stat;     // the stage's PodStat records (NULL = no node affinity)
  const TopoRec* trec;     // the stage's TopoRec records
  const int32_t* cursor;   // the pod at *cursor, only if it is a topology pod; NULL = pod 0, always (ks_eval_pod)
  int32_t total_pods;
  int64_t n;
  uint32_t* reasons;       // [n] every plugin's KS_R_* (eval_debug_kernel's), topology bits OR-ed in
  int64_t* scores;         // [n][KS_NUM_SCORE_PLUGINS] (ks_eval_pod; NULL in the batch step: not written)
  int64_t* total;          // [n] weighted total, -1 = infeasible
  const int32_t* rraw;     // Reservation raw score, order rank (eval_debug_kernel's)
  const int32_t* rhi;
  const int32_t* draw;     // DeviceShare raw
  const int32_t* traw;     // TaintToleration raw
  const int32_t* araw;     // NodeAffinity raw
  long long* sraw;         // [n] PodTopologySpread raw score (topo_pts_kernel)
  long long* iraw;         // [n] InterPodAffinity raw score (eval_debug_kernel)
  int32_t dev_on, taint_on, aff_on, rsv_on;
  int64_t dev_w, taint_w, aff_w, rsv_w, spread_w, ipa_w;
  TopoScratch* scr;
  // the batch step's one-candidate set of the chosen node (commit_kernel's lists, pod 0 of a one-pod pass); NULL in
  // ks_eval_pod
  uint32_t* cand_chunk;
  uint2* cand_t;
  int32_t* cand_count;
  uint64_t *cand_bound, *cand_top, *cand_second;
};

// the pod of the step (-1 = nothing to do: the cursor's pod is not a topology pod); rec = its record
__device__ __forceinline__ int32_t topo_pod(const TopoKArgs& a, TopoRec& rec) {
  int32_t pi = 0;
  if (a.cursor) {
    pi = *a.cursor;
    if (pi >= a.total_pods) return -1;
  }
  rec = a.trec[pi];
  if (a.cursor && !(rec.flags & KS_TOPO_DYN)) return -1;
  return pi;
}

// the step's pod as topo_sums_kernel left it (every later kernel of the step)
__device__ __forceinline__ int32_t topo_cur(const TopoKArgs& a, TopoRec& rec) {
  rec = a.scr->cur_rec;
  return a.scr->cur_pi;
}

// the node counts for the term (hard spread: required node affinity + every hard key; soft spread: required node
// affinity + every soft key when requireAllTopologies; InterPodAffinity: every node)
__device__ __forceinline__ bool tp_eligible(uint64_t w, uint32_t pflags, bool aff, bool zone_ok) {
  const int k = tp_kind(w);
  if (k == KS_TOPO_K_SPREAD_HARD) return aff && (!(tp_flags(w) & KS_TOPO_T_ELIG_ZONE) || zone_ok);
  if (k == KS_TOPO_K_SPREAD_SOFT)
    return aff && (!((pflags & KS_TOPO_SOFT_ALL_KEYS) && (tp_flags(w) & KS_TOPO_T_ELIG_ZONE)) || zone_ok);
  return true;
}

__device__ __forceinline__ long long wave_max_i64(long long v) {
  return (long long)(wave_max_u64((uint64_t)v ^ (1ull << 63)) ^ (1ull << 63));
}
__device__ __forceinline__ long long wave_min_i64(long long v) {
  return (long long)(~wave_max_u64(~((uint64_t)v ^ (1ull << 63))) ^ (1ull << 63));
}

__device__ __forceinline__ uint64_t wave_or_u64(uint64_t v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const uint32_t lo = __shfl_xor((int)(uint32_t)v, off, 64), hi = __shfl_xor((int)(uint32_t)(v >> 32), off, 64);
    v |= ((uint64_t)hi << 32) | lo;
  }
  return v;
}

// The block's LDS copy of the step's domain sums (TopoLds) and the hard spread constraints' minimum match count per
// term (TpKeyToCriticalPaths[key][0].MatchNum; MaxInt32 when no domain is eligible), from what topo_sums_kernel left
// in the scratch: one load per thread, the minima by LDS atomics.  Every thread of the block calls it.
struct TopoLds {
  long long zsum[KS_TOPO_TERMS][KS_TOPO_ZONES];
  unsigned long long zpres[KS_TOPO_TERMS];
  long long mins[KS_TOPO_TERMS];
  int any_all;  // affinityCounts is not empty
};
__device__ __forceinline__ void topo_stage(const TopoKArgs& a, const TopoRec& tr, TopoLds& l) {
  const int tid = threadIdx.x;
  if (tid < KS_TOPO_TERMS) {
    l.zpres[tid] = a.scr->zpres[tid];
    l.mins[tid] = a.scr->hmin[tid];
  }
  if (tid == 0) l.any_all = a.scr->any_all;
  for (int k = tid; k < KS_TOPO_TERMS * KS_TOPO_ZONES; k += blockDim.x) (&l.zsum[0][0])[k] = (&a.scr->zsum[0][0])[k];
  __syncthreads();
  uint32_t zkey = 0;  // terms with the zonal key (a register mask: no dynamic index into the record)
#pragma unroll
  for (int t = 0; t < KS_TOPO_TERMS; ++t) zkey |= (tp_key(tr.term[t]) == 1 ? 1u : 0u) << t;
  for (int k = tid; k < KS_TOPO_TERMS * KS_TOPO_ZONES; k += blockDim.x) {
    const int t = k / KS_TOPO_ZONES, z = k - t * KS_TOPO_ZONES;
    if (((zkey >> t) & 1u) && ((l.zpres[t] >> z) & 1ull)) atomicMin(&l.mins[t], l.zsum[t][z]);
  }
  __syncthreads();
}

// topo_eval_node's node inputs, loaded as soon as the step's pod record is known (with the stage's loads, ahead of
// the plugin evaluation): the zone, the labels, the hostname-keyed terms' counts
struct TopoPre {
  int32_t z;
  uint64_t lab;
  int32_t cnt[KS_TOPO_TERMS];
};
__device__ __forceinline__ TopoPre topo_pre(const TopoKArgs& a, const TopoRec& tr, int64_t i, bool valid) {
  TopoPre p;
  const int64_t n = valid ? i : 0;
  p.z = valid ? a.t.zone[n] : -1;
  p.lab = a.labels ? a.labels[n] : 0ull;
  const bool dyn = (tr.flags & KS_TOPO_DYN) != 0;
#pragma unroll
  for (int t = 0; t < KS_TOPO_TERMS; ++t) {
    const uint64_t w = tr.term[t];
    p.cnt[t] = (dyn && w && tp_key(w) == 0) ? a.t.count[(int64_t)tp_prop(w) * a.t.npad + n] : 0;
  }
  return p;
}
// ... and the evaluation's results for the node (registers, not re-read from the buffers just written)
struct TopoNodeIn {
  uint32_t base;  // every other plugin's reasons
  int32_t dr, trw, arw, rhi;
};

// eval_debug_kernel's topology part for node i (every lane of the wave calls it, converged; valid = a node of the
// cluster): both plugins' Filters OR-ed into the node's reasons (total -1 and the score row zeroed when they fail),
// InterPodAffinity's raw score, and the node's part of the normalizations' reductions (one global atomic per wave)
__device__ __forceinline__ void topo_eval_node(const TopoKArgs& a, const TopoRec& tr, int32_t pi, int64_t i, bool valid,
                                               const TopoLds& l, const TopoPre& pre, const TopoNodeIn& in) {
  const bool dyn = (tr.flags & KS_TOPO_DYN) != 0;
  bool soft_zone = false, need_aff = false;
#pragma unroll
  for (int t = 0; t < KS_TOPO_TERMS; ++t) {
    const int k = tp_kind(tr.term[t]);
    soft_zone |= k == KS_TOPO_K_SPREAD_SOFT && (tp_flags(tr.term[t]) & KS_TOPO_T_ELIG_ZONE);
    need_aff |= k == KS_TOPO_K_SPREAD_HARD;
  }
  const bool soft_all = (tr.flags & KS_TOPO_SOFT_ALL_KEYS) != 0;
  bool feas = false, counted = false;
  int32_t z = -1;
  long long ir = 0;
  int32_t dr = 0, trw = 0, arw = 0;
  uint64_t pref = 0;
  if (valid) {
    const uint32_t base = in.base;
    z = pre.z;
    const bool has_zone = z >= 0;
    uint32_t r = 0;
    if (dyn) {
      auto domain = [&](int t) -> long long {
        const uint64_t w = tr.term[t];
        return tp_key(w) == 1 ? l.zsum[t][z] : (long long)pre.cnt[t];
      };
      const bool aff = need_aff ? tp_node_aff(a.stat ? a.stat + pi : nullptr, pre.lab) : true;
      // PodTopologySpread Filter: the first hard constraint that fails
    #pragma unroll
  for (int t = 0; t < KS_TOPO_TERMS; ++t) {
        const uint64_t w = tr.term[t];
        if (tp_kind(w) != KS_TOPO_K_SPREAD_HARD) continue;
        if (tp_key(w) == 1 && !has_zone) {  // ErrReasonNodeLabelNotMatch
          r = KS_R_TOPOLOGY_SPREAD;
          break;
        }
        long long match;
        if (tp_key(w) == 1) match = ((l.zpres[t] >> z) & 1ull) ? l.zsum[t][z] : 0;
        else match = tp_eligible(w, tr.flags, aff, has_zone) ? (long long)pre.cnt[t] : 0;
        const long long self = (tp_flags(w) & KS_TOPO_T_SELF) ? 1 : 0;
        if (match + self - l.mins[t] > (long long)tp_param(w)) {  // ErrReasonConstraintsNotMatch
          r = KS_R_TOPOLOGY_SPREAD;
          break;
        }
      }
      // InterPodAffinity Filter: affinity, anti-affinity, existing pods' anti-affinity -- the first that fails
      bool aff_terms = false, missing = false, exist = true;
    #pragma unroll
  for (int t = 0; t < KS_TOPO_TERMS; ++t) {
        if (tp_kind(tr.term[t]) != KS_TOPO_K_AFFINITY) continue;
        aff_terms = true;
        if (tp_key(tr.term[t]) == 1 && !has_zone) missing = true;
        else if (domain(t) <= 0) exist = false;
      }
      uint32_t ipa = 0;
      if (aff_terms && (missing || (!exist && !(l.any_all == 0 && (tr.flags & KS_TOPO_SELF_AFFINITY))))) {
        ipa = KS_R_POD_AFFINITY;
      } else {
#pragma unroll
        for (int t = 0; t < KS_TOPO_TERMS; ++t) {
          if (ipa) break;
          const uint64_t w = tr.term[t];
          if (tp_kind(w) == KS_TOPO_K_ANTI && (tp_key(w) == 0 || has_zone) && domain(t) > 0) ipa = KS_R_POD_ANTI_AFFINITY;
        }
#pragma unroll
        for (int t = 0; t < KS_TOPO_TERMS; ++t) {
          if (ipa) break;
          const uint64_t w = tr.term[t];
          if (tp_kind(w) == KS_TOPO_K_EXISTING_ANTI && (tp_key(w) == 0 || has_zone) && domain(t) > 0)
            ipa = KS_R_EXISTING_ANTI_AFFINITY;
        }
      }
      r |= ipa;
      if (r) {
        a.reasons[i] = base | r;
        a.total[i] = -1;
        if (a.scores)
          for (int k = 0; k < KS_NUM_SCORE_PLUGINS; ++k) a.scores[i * KS_NUM_SCORE_PLUGINS + k] = 0;
      }
      // InterPodAffinity Score: weight x matching pods in the node's domain, per score term
    #pragma unroll
  for (int t = 0; t < KS_TOPO_TERMS; ++t) {
        const uint64_t w = tr.term[t];
        if (tp_kind(w) == KS_TOPO_K_SCORE && (tp_key(w) == 0 || has_zone)) ir += (long long)tp_param(w) * domain(t);
      }
    }
    feas = (base | r) == 0;
    counted = feas && !(soft_all && soft_zone && !has_zone);  // initPreScoreState: not an ignored node
    if (feas) {
      a.iraw[i] = ir;
      dr = in.dr;
      trw = in.trw;
      arw = in.arw;
      if (a.rsv_on && in.rhi > 0) pref = ((uint64_t)in.rhi << 32) | (0xFFFFFFFFull - (uint64_t)i);
    }
  }
  // the wave's part of every reduction, then one atomic per quantity
  const int lane = threadIdx.x & 63;
  const uint64_t cnt = __ballot(counted);
  const uint64_t zbits = wave_or_u64(counted && z >= 0 ? (1ull << z) : 0ull);
  const bool emp = __ballot(counted && z < 0) != 0;
  const long long imn = wave_min_i64(feas ? ir : 0), imx = wave_max_i64(feas ? ir : 0);
  const uint32_t dmx = wave_max_u32((uint32_t)dr), tmx = wave_max_u32((uint32_t)trw), amx = wave_max_u32((uint32_t)arw);
  const uint64_t pmx = wave_max_u64(pref);
  if (lane == 0) {
    TopoScratch* s = a.scr;
    if (cnt) atomicAdd(&s->hsize, (unsigned long long)__popcll(cnt));
    if (zbits) atomicOr(&s->zones, zbits);
    if (emp) atomicOr(&s->empty, 1);
    if (imn < 0) atomicMin(&s->imin, imn);
    if (imx > 0) atomicMax(&s->imax, imx);
    if (dmx) atomicMax(&s->dev_max, (int)dmx);
    if (tmx) atomicMax(&s->taint_max, (int)tmx);
    if (amx) atomicMax(&s->aff_max, (int)amx);
    if (pmx) atomicMax(&s->rsv_pref, (unsigned long long)pmx);
  }
}

// The lean one-pod commit of a topology pod for the plugin sets whose Reserve is NodeInfo.AddPod + the LoadAware
// assign cache + ElasticQuota (kernel variants 0 and 4 without DeviceShare, Reservation, NodeNUMAResource)
struct TopoCommitArgs {
  DevNodes d;
  DevQuotas q;
  DevPodQuota pq;
  const PodRec* pods;
  const PodStat* pstat;
  const TopoRec* trec;
  int32_t* cursor;
  int32_t total_pods;
  int32_t quota_enable, quota_parent, ports;
  ks_result* results;
  unsigned long long* counters;
  int32_t* topo_count;
  int64_t topo_npad;
  const TopoScratch* scr;
};

hipError_t launch_topo_sums(hipStream_t s, const TopoKArgs& a);
hipError_t launch_topo_pts(hipStream_t s, const TopoKArgs& a);
// c != NULL: the last workgroup commits the pod (the lean commit); NULL: it leaves the one-candidate set
hipError_t launch_topo_norm(hipStream_t s, const TopoKArgs& a, const TopoCommitArgs* c = nullptr);
TopoScratch topo_scratch_init();

}  // namespace ks
