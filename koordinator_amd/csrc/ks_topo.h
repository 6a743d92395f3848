// ks_topo.h — upstream PodTopologySpread and InterPodAffinity (kube-scheduler v1.24.15 plugins/podtopologyspread,
// plugins/interpodaffinity) on the device: the node counters and pod query terms of include/koordgpu.h
// ks_topology_args (compiled on the host by koordinator_amd/topology_plugins.py), the kernels that schedule a
// topology pod (KS_TOPO_DYN) alone against them, and the commit kernels' hooks.
//
// A topology pod's Filter needs per-domain sums over every eligible node (PreFilter) and its Score a normalization
// over every feasible node, so it cannot share a pass with other pods: the pass loop runs, before each regular pass,
// a topology step that acts only when the pod at the cursor is one --
//   topo_sums_kernel    PreFilter: per query term the domain sums over its eligible nodes
//   eval_debug_kernel   every other plugin's Filter / Score on every node (ks_debug.hip, the ks_eval_pod path) with
//                       both plugins' Filters and InterPodAffinity's raw score folded in (topo_eval_node)
//   topo_pts_kernel     PodTopologySpread PreScore / Score
//   topo_norm_kernel    every NormalizeScore, the weighted totals, the best node (max total, lowest index)
//   commit_kernel       (CommitArgs.topo = 2) admission + every Reserve on that node, the counters of the pod's
//                       properties (or the lean commit in topo_norm_kernel's last workgroup)
// -- and every regular pass ends before its first topology pod (CommitArgs.topo = 1).
//
// Sizes are the context's (ks_node_cols.topo_nkeys / topo_ndomains / topo_nprops): a query term names one of up to 256
// topology keys (key 0 the hostname, whose domain is the node itself; key k >= 1 a node label whose value index is
// DevTopo.dom) and one of up to 65,536 properties; a pod has up to KS_TOPO_MAX_TERMS terms and any number of
// properties (CSR lists staged with the pod columns).  The per-domain sums of a step live in HBM ([term][domain],
// DevTopo.zsum), reduced by wave-segmented atomics: one atomic per distinct domain of a wave.
#pragma once

#include <hip/hip_runtime.h>

#include <climits>

#include "ks_device.h"

namespace ks {

// internal pod flag (PodRec.flags): the pod has topology query terms (KS_TOPO_DYN)
constexpr uint32_t kPodTopoDyn = 0x4000u;
constexpr int kTopoTerms = KS_TOPO_MAX_TERMS;
constexpr int kTopoInline = 8;  // the step pod's first terms, held in (wave-uniform) registers by every step kernel

// Per pending pod, queue order (staged with the pod columns): its query terms and properties in the stage's lists
struct __attribute__((aligned(16))) TopoRec {
  int32_t tbeg, nterms;  // [tbeg, tbeg + nterms) of the stage's term list
  int32_t pbeg, nprops;  // [pbeg, pbeg + nprops) of the stage's property list
  uint32_t flags;        // KS_TOPO_*
  int32_t _pad[3];
};
static_assert(sizeof(TopoRec) == 32, "TopoRec layout");

// Node side and the step's per-domain scratch.  lw[s] = log(s + 2) for s in [0, nlw) (the host's libm, the oracle's log).
struct DevTopo {
  int32_t* dom;       // [nkeys][npad]: value index of key k + 1 (-1 = absent)
  int32_t* count;     // [nprops][npad]: pods with property p
  int64_t npad;
  int32_t nkeys, ndom;
  const double* lw;
  int32_t nlw;
  int32_t nw;         // 32-bit words of a domain bit set: (ndom + 31) / 32
  long long* zsum;    // [kTopoTerms][ndom]: per term the domain's counted pods over the term's eligible nodes (0)
  uint32_t* zpres;    // [kTopoTerms][nw]: hard spread: domains with an eligible node (0)
  uint32_t* zsize;    // [kTopoTerms][nw]: soft spread: domains of the counted nodes (initPreScoreState's topoSize) (0)
};

// The topology step's reductions (HBM, one per context).  Every field is back at its initial value after each step
// (topo_norm_kernel resets it; topo_install writes the initial image).
struct TopoScratch {
  int hmin[kTopoTerms];                           // hard spread, hostname: min count over the eligible nodes (INT_MAX)
  int tempty[kTopoTerms];                         // soft spread: a counted node without the key (the value "") (0)
  int any_all;                                    // InterPodAffinity: affinityCounts is not empty (0)
  int _pad0;
  unsigned long long hsize;                       // feasible non-ignored nodes (0)
  int dev_max, taint_max, aff_max, _pad1;         // DeviceShare / TaintToleration / NodeAffinity raw maxima (0)
  long long imin, imax;                           // InterPodAffinity raw extrema, from 0 (0)
  long long smin, smax;                           // PodTopologySpread raw extrema over the non-ignored nodes (LLONG_MAX, 0)
  unsigned long long rsv_pref, rsv_max;           // Reservation preferred-node key, raw max (0)
  unsigned long long best;                        // selectHost key (total + 1) << 32 | ~node (0)
  unsigned int done, _pad2;                       // topo_norm_kernel workgroups finished (0)
  long long best_total;                           // the chosen node's total (the pod's result score)
  long long best_node;                            // ... the node (-1 = none feasible)
  // the step's pod, written by topo_sums_kernel (the first kernel of a step) from *cursor: the later kernels read it
  // with one load instead of the cursor -> record chain (-1 = the cursor's pod is not a topology pod)
  int32_t cur_pi, _pad3[3];
  TopoRec cur_rec;
  uint64_t cur_terms[kTopoInline];  // ... and its first terms
};

// The step pod's first kTopoInline terms (registers); later ones are read from the stage's list
struct TopoTerms {
  uint64_t w[kTopoInline];
};

__device__ __forceinline__ int tp_kind(uint64_t w) { return (int)(w & 0xF); }
__device__ __forceinline__ uint32_t tp_flags(uint64_t w) { return (uint32_t)((w >> 4) & 0xF); }
__device__ __forceinline__ int tp_key(uint64_t w) { return (int)((w >> 8) & 0xFF); }
__device__ __forceinline__ int tp_prop(uint64_t w) { return (int)((w >> 16) & 0xFFFF); }
__device__ __forceinline__ int32_t tp_param(uint64_t w) { return (int32_t)(uint32_t)(w >> 32); }

// A node's value indices of keys 1..kTopoPreKeys, loaded with the node's other inputs before the step's pod record
// arrives (a kernel would otherwise wait for the record, then for the term, then for the domain)
constexpr int kTopoPreKeys = 4;
struct TopoNodeDom {
  int32_t d[kTopoPreKeys];
  int64_t n;
};
__device__ __forceinline__ TopoNodeDom topo_node_dom(const DevTopo& t, int64_t n) {
  TopoNodeDom nd;
#pragma unroll
  for (int k = 0; k < kTopoPreKeys; ++k) nd.d[k] = k < t.nkeys ? t.dom[(int64_t)k * t.npad + n] : -1;
  nd.n = n;
  return nd;
}
// the node's value index of key k >= 1 (-1 = the label is absent); k is wave-uniform
__device__ __forceinline__ int32_t tp_dom(const DevTopo& t, const TopoNodeDom& nd, int k) {
  if (k <= kTopoPreKeys) return k == 1 ? nd.d[0] : k == 2 ? nd.d[1] : k == 3 ? nd.d[2] : nd.d[3];
  return t.dom[(int64_t)(k - 1) * t.npad + nd.n];
}
__device__ __forceinline__ int32_t tp_count(const DevTopo& t, uint64_t w, int64_t n) {
  return t.count[(int64_t)tp_prop(w) * t.npad + n];
}

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

// NodeInfo.AddPod / RemovePod for the two plugins: the counters of the pod's properties on node n (delta +1 / -1)
__device__ __forceinline__ void topo_count_pod(int32_t* count, int64_t npad, const int32_t* props, const TopoRec& t,
                                               int64_t n, int32_t delta) {
  for (int32_t k = 0; k < t.nprops; ++k) atomicAdd(count + (int64_t)props[t.pbeg + k] * npad + n, delta);
}

// Write-back of one result: the counters of the placed pod's properties (NodeInfo.AddPod), its score (the topology
// step's total; a pod without query terms gets PodTopologySpread's constant 100 x weight on every node)
template <typename A>
__device__ __forceinline__ void topo_writeback(const A& a, int32_t pod, ks_result& r) {
  if (a.topo == 0 || r.status != KS_S_SCHEDULED || r.node < 0) return;
  const TopoRec& t = a.topo_rec[pod];
  if (a.topo == 2) r.score = *a.topo_best;
  else if (a.topo == 1 && !(t.flags & KS_TOPO_DYN)) r.score += a.topo_const;
  topo_count_pod(a.topo_count, a.topo_npad, a.topo_props, t, r.node, 1);
}

// ---- topology step kernels (ks_topo.hip) ----

struct TopoKArgs {
  DevTopo t;
  const uint64_t* labels;  // DevNodes.labels (required node affinity of the spread constraints)
  const PodStat* stat;     // the stage's PodStat records (NULL = no node affinity)
  const TopoRec* trec;     // the stage's TopoRec records
  const uint64_t* terms;   // the stage's query-term list
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

// the step pod's term t (wave-uniform scalar load)
__device__ __forceinline__ uint64_t topo_term(const TopoKArgs& a, const TopoRec& tr, int t) { return a.terms[tr.tbeg + t]; }

__device__ __forceinline__ TopoTerms topo_terms_of(const TopoKArgs& a, const TopoRec& tr) {
  TopoTerms tt;
#pragma unroll
  for (int t = 0; t < kTopoInline; ++t) tt.w[t] = t < tr.nterms ? a.terms[tr.tbeg + t] : 0ull;
  return tt;
}
__device__ __forceinline__ TopoTerms topo_terms_cur(const TopoKArgs& a) {
  TopoTerms tt;
#pragma unroll
  for (int t = 0; t < kTopoInline; ++t) tt.w[t] = a.scr->cur_terms[t];
  return tt;
}

// f(t, w) over the step pod's terms in order (the first kTopoInline from registers: unrolled, no dynamic index);
// f returns false to stop
template <typename F>
__device__ __forceinline__ void topo_each(const TopoKArgs& a, const TopoRec& tr, const TopoTerms& tt, F f) {
#pragma unroll
  for (int t = 0; t < kTopoInline; ++t)
    if (t < tr.nterms && !f(t, tt.w[t])) return;
  for (int t = kTopoInline; t < tr.nterms; ++t)
    if (!f(t, topo_term(a, tr, t))) return;
}

// nodeLabelsMatchSpreadConstraints over the pod's hard and soft constraints: node n has every key they name
struct TopoKeysOk {
  bool hard, soft;
};
__device__ __forceinline__ TopoKeysOk topo_keys_ok(const TopoKArgs& a, const TopoRec& tr, const TopoTerms& tt,
                                                   const TopoNodeDom& nd) {
  TopoKeysOk k{true, true};
  topo_each(a, tr, tt, [&](int, uint64_t w) {
    const int kd = tp_kind(w);
    if ((kd == KS_TOPO_K_SPREAD_HARD || kd == KS_TOPO_K_SPREAD_SOFT) && tp_key(w) != 0) {
      const bool has = tp_dom(a.t, nd, tp_key(w)) >= 0;
      if (kd == KS_TOPO_K_SPREAD_HARD) k.hard = k.hard && has;
      else k.soft = k.soft && has;
    }
    return true;
  });
  return k;
}

// the node counts for term w (hard spread: required node affinity + every hard key; soft spread: required node
// affinity + every soft key when requireAllTopologies; InterPodAffinity: every node)
__device__ __forceinline__ bool tp_eligible(uint64_t w, uint32_t pflags, bool aff, bool hard_keys, bool soft_keys) {
  const int k = tp_kind(w);
  if (k == KS_TOPO_K_SPREAD_HARD) return aff && hard_keys;
  if (k == KS_TOPO_K_SPREAD_SOFT) return aff && (!(pflags & KS_TOPO_SOFT_ALL_KEYS) || soft_keys);
  return true;
}

__device__ __forceinline__ long long wave_max_i64(long long v) {
  return (long long)(wave_max_u64((uint64_t)v ^ (1ull << 63)) ^ (1ull << 63));
}
__device__ __forceinline__ long long wave_min_i64(long long v) {
  return (long long)(~wave_max_u64(~((uint64_t)v ^ (1ull << 63))) ^ (1ull << 63));
}
__device__ __forceinline__ long long wave_sum_i64(long long v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const uint32_t lo = __shfl_xor((int)(uint32_t)v, off, 64), hi = __shfl_xor((int)(uint32_t)((uint64_t)v >> 32), off, 64);
    v += (long long)(((uint64_t)hi << 32) | lo);
  }
  return v;
}

// Wave-segmented reduction into HBM (every lane calls it, converged): lanes with `on` add `v` (a node's pod count,
// >= 0) to sum[z] and set bit z of bits (either may be NULL); one atomic per distinct z of the wave
__device__ __forceinline__ void topo_seg_add(long long* sum, uint32_t* bits, bool on, int32_t z, int32_t v) {
  uint64_t act = __ballot(on);
  while (act) {
    const int l = __ffsll((long long)act) - 1;
    const int32_t z0 = __builtin_amdgcn_readlane(z, l);
    const bool mine = on && z == z0;
    const uint64_t m = __ballot(mine);
    const uint32_t s = sum ? wave_sum_u32(mine ? (uint32_t)v : 0u) : 0u;
    if ((threadIdx.x & 63) == l) {
      if (sum && s) atomicAdd((unsigned long long*)(sum + z0), (unsigned long long)s);
      if (bits) atomicOr(bits + (z0 >> 5), 1u << (z0 & 31));
    }
    act &= ~m;
  }
}

// Wave-level domain bit set (bits: a [nw] word array; every lane calls it, converged): one 64-bit OR per wave when
// every domain index fits a word pair, else one atomic per distinct domain of the wave
__device__ __forceinline__ void topo_bits_or(uint32_t* bits, int32_t ndom, bool on, int32_t z) {
  if (ndom <= 64) {
    const uint64_t o = wave_or_u64(on ? (1ull << z) : 0ull);
    if ((threadIdx.x & 63) == 0) {
      if ((uint32_t)o) atomicOr(bits, (uint32_t)o);
      if (o >> 32) atomicOr(bits + 1, (uint32_t)(o >> 32));
    }
  } else {
    topo_seg_add(nullptr, bits, on, z, 0);
  }
}

// The block's LDS copy of the hard spread constraints' minimum match count per term (TpKeyToCriticalPaths[key][0]
// .MatchNum; MaxInt32 when no domain is eligible) and affinityCounts' emptiness, from what topo_sums_kernel left in
// the scratch.  Every thread of the block calls it.
struct TopoLds {
  long long mins[kTopoTerms];
  int any_all;
};
__device__ __forceinline__ void topo_stage(const TopoKArgs& a, const TopoRec& tr, const TopoTerms& tt, TopoLds& l) {
  const int tid = threadIdx.x;
  if (tid < kTopoTerms) l.mins[tid] = a.scr->hmin[tid];
  if (tid == 0) l.any_all = a.scr->any_all;
  __syncthreads();
  topo_each(a, tr, tt, [&](int t, uint64_t w) {
    if (tp_kind(w) != KS_TOPO_K_SPREAD_HARD || tp_key(w) == 0) return true;  // (wave-uniform)
    long long m = LLONG_MAX;
    for (int z = tid; z < a.t.ndom; z += blockDim.x)
      if ((a.t.zpres[(int64_t)t * a.t.nw + (z >> 5)] >> (z & 31)) & 1u) {
        const long long v = a.t.zsum[(int64_t)t * a.t.ndom + z];
        m = v < m ? v : m;
      }
    m = wave_min_i64(m);
    if ((tid & 63) == 0 && m != LLONG_MAX) atomicMin(&l.mins[t], m);
    return true;
  });
  __syncthreads();
}

// topo_eval_node's results of the other plugins for the node (registers, not re-read from the buffers just written)
struct TopoNodeIn {
  uint32_t base;  // every other plugin's reasons
  int32_t dr, trw, arw, rhi;
};

// eval_debug_kernel's topology part for node i (every lane of the wave calls it, converged; valid = a node of the
// cluster): both plugins' Filters OR-ed into the node's reasons (total -1 and the score row zeroed when they fail),
// InterPodAffinity's raw score, the counted nodes' domains of the soft constraints (topology sizes), and the node's part
// of the normalizations' reductions (one global atomic per wave)
__device__ __forceinline__ void topo_eval_node(const TopoKArgs& a, const TopoRec& tr, const TopoTerms& tt,
                                               const TopoNodeDom& nd, int32_t pi, int64_t i, bool valid,
                                               const TopoLds& l, const TopoNodeIn& in) {
  const bool dyn = (tr.flags & KS_TOPO_DYN) != 0;
  const bool soft_all = (tr.flags & KS_TOPO_SOFT_ALL_KEYS) != 0;
  const int64_t n = valid ? i : 0;
  bool feas = false, counted = false;
  long long ir = 0;
  int32_t dr = 0, trw = 0, arw = 0;
  uint64_t pref = 0;
  TopoKeysOk keys{true, true};
  if (dyn) keys = topo_keys_ok(a, tr, tt, nd);
  if (valid) {
    const uint32_t base = in.base;
    uint32_t r = 0;
    if (dyn) {
      // the term's count in the node's domain (the node has the key's label)
      auto domain = [&](int t, uint64_t w) -> long long {
        if (tp_key(w) == 0) return (long long)tp_count(a.t, w, n);
        return a.t.zsum[(int64_t)t * a.t.ndom + tp_dom(a.t, nd, tp_key(w))];
      };
      auto has_key = [&](uint64_t w) { return tp_key(w) == 0 || tp_dom(a.t, nd, tp_key(w)) >= 0; };
      // PodTopologySpread Filter: the first hard constraint that fails
      bool aff = true, aff_done = false;
      topo_each(a, tr, tt, [&](int t, uint64_t w) {
        if (tp_kind(w) != KS_TOPO_K_SPREAD_HARD) return true;
        const int32_t z = tp_key(w) == 0 ? 0 : tp_dom(a.t, nd, tp_key(w));
        if (z < 0) {  // ErrReasonNodeLabelNotMatch
          r = KS_R_TOPOLOGY_SPREAD;
          return false;
        }
        long long match;
        if (tp_key(w) != 0) {
          match = ((a.t.zpres[(int64_t)t * a.t.nw + (z >> 5)] >> (z & 31)) & 1u) ? a.t.zsum[(int64_t)t * a.t.ndom + z] : 0;
        } else {
          if (!aff_done) {
            aff = tp_node_aff(a.stat ? a.stat + pi : nullptr, a.labels ? a.labels[n] : 0ull);
            aff_done = true;
          }
          match = (aff && keys.hard) ? (long long)tp_count(a.t, w, n) : 0;
        }
        const long long self = (tp_flags(w) & KS_TOPO_T_SELF) ? 1 : 0;
        if (match + self - l.mins[t] > (long long)tp_param(w)) {  // ErrReasonConstraintsNotMatch
          r = KS_R_TOPOLOGY_SPREAD;
          return false;
        }
        return true;
      });
      // InterPodAffinity Filter: affinity, anti-affinity, existing pods' anti-affinity -- the first that fails
      bool aff_terms = false, missing = false, exist = true;
      topo_each(a, tr, tt, [&](int t, uint64_t w) {
        if (tp_kind(w) != KS_TOPO_K_AFFINITY) return true;
        aff_terms = true;
        if (!has_key(w)) missing = true;
        else if (domain(t, w) <= 0) exist = false;
        return true;
      });
      uint32_t ipa = 0;
      if (aff_terms && (missing || (!exist && !(l.any_all == 0 && (tr.flags & KS_TOPO_SELF_AFFINITY))))) {
        ipa = KS_R_POD_AFFINITY;
      } else {
        topo_each(a, tr, tt, [&](int t, uint64_t w) {
          if (tp_kind(w) == KS_TOPO_K_ANTI && has_key(w) && domain(t, w) > 0) ipa = KS_R_POD_ANTI_AFFINITY;
          return ipa == 0;
        });
        if (!ipa)
          topo_each(a, tr, tt, [&](int t, uint64_t w) {
            if (tp_kind(w) == KS_TOPO_K_EXISTING_ANTI && has_key(w) && domain(t, w) > 0) ipa = KS_R_EXISTING_ANTI_AFFINITY;
            return ipa == 0;
          });
      }
      r |= ipa;
      if (r) {
        a.reasons[i] = base | r;
        a.total[i] = -1;
        if (a.scores)
          for (int k = 0; k < KS_NUM_SCORE_PLUGINS; ++k) a.scores[i * KS_NUM_SCORE_PLUGINS + k] = 0;
      }
      // InterPodAffinity Score: weight x matching pods in the node's domain, per score term
      if ((base | r) == 0)
        topo_each(a, tr, tt, [&](int t, uint64_t w) {
          if (tp_kind(w) == KS_TOPO_K_SCORE && has_key(w)) ir += (long long)tp_param(w) * domain(t, w);
          return true;
        });
    }
    feas = (base | r) == 0;
    // initPreScoreState: a node without every soft key is ignored under requireAllTopologies
    counted = feas && !(dyn && soft_all && !keys.soft);
    if (feas) {
      a.iraw[i] = ir;
      dr = in.dr;
      trw = in.trw;
      arw = in.arw;
      if (a.rsv_on && in.rhi > 0) pref = ((uint64_t)in.rhi << 32) | (0xFFFFFFFFull - (uint64_t)i);
    }
  }
  // topology sizes of the soft constraints over the counted nodes: per term the domains (a node without the key: "")
  if (dyn)
    topo_each(a, tr, tt, [&](int t, uint64_t w) {
      if (tp_kind(w) != KS_TOPO_K_SPREAD_SOFT || tp_key(w) == 0) return true;  // (wave-uniform)
      const int32_t z = counted ? tp_dom(a.t, nd, tp_key(w)) : -1;
      topo_bits_or(a.t.zsize + (int64_t)t * a.t.nw, a.t.ndom, counted && z >= 0, z);
      if (__ballot(counted && z < 0) && (threadIdx.x & 63) == 0) atomicOr(&a.scr->tempty[t], 1);
      return true;
    });
  // the wave's part of every other reduction, then one atomic per quantity
  const int lane = threadIdx.x & 63;
  const uint64_t cnt = __ballot(counted);
  const long long imn = wave_min_i64(feas ? ir : 0), imx = wave_max_i64(feas ? ir : 0);
  const uint32_t dmx = wave_max_u32((uint32_t)dr), tmx = wave_max_u32((uint32_t)trw), amx = wave_max_u32((uint32_t)arw);
  const uint64_t pmx = wave_max_u64(pref);
  if (lane == 0) {
    TopoScratch* s = a.scr;
    if (cnt) atomicAdd(&s->hsize, (unsigned long long)__popcll(cnt));
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
  const int32_t* props;  // the stage's property list
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
