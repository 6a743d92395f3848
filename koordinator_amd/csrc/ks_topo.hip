// ks_topo.hip — the topology step's kernels (ks_topo.h): one workgroup each; the pod's domain sums and
// normalization extrema live in LDS, the per-node work is a strided loop over the node columns (a few int32 words per
// node and term: HBM traffic of a few hundred KB per topology pod at 5k nodes).
//
// Upstream kube-scheduler v1.24.15 (not on disk: parity unpinned, restated on objects by oracle/topology_ref.py and on
// the compiled form by oracle/koord_oracle.c tp_*):
//   podtopologyspread/filtering.go  calPreFilterState (TpPairToMatchNum over the nodes passing the pod's required node
//                                   affinity and holding every constraint key; critical paths = the per-key minimum),
//                                   Filter (missing key; matchNum + selfMatchNum - minMatchNum > maxSkew)
//   podtopologyspread/scoring.go    initPreScoreState (ignored nodes, topoSize), PreScore's pair counts, Score
//                                   (scoreForCount = cnt * log(size + 2) + maxSkew - 1, math.Round), NormalizeScore
//   interpodaffinity/filtering.go   affinityCounts / antiAffinityCounts / existingAntiAffinityCounts, satisfyPodAffinity
//                                   (with the first-pod-of-a-series rule), satisfyPodAntiAffinity,
//                                   satisfyExistingPodsAntiAffinity -- the first failing one
//   interpodaffinity/scoring.go     processExistingPod's topologyScore, Score, NormalizeScore (min / max from 0)
// Every f64 operation is Go's, in Go's order (-ffp-contract=off).
#include "ks_topo.h"

namespace ks {

constexpr int kTopoThreads = 1024;

// the pod of the step: -1 = nothing to do
__device__ __forceinline__ int32_t topo_pod(const TopoKArgs& a, TopoRec& tr) {
  int32_t pi = 0;
  if (a.cursor) {
    pi = *a.cursor;
    if (pi >= a.total_pods) return -1;
  }
  tr = a.trec[pi];
  if (a.cursor && !(tr.flags & KS_TOPO_DYN)) return -1;
  return pi;
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

__global__ __launch_bounds__(kTopoThreads) void topo_filter_kernel(TopoKArgs a) {
  __shared__ long long zsum[KS_TOPO_TERMS][KS_TOPO_ZONES];
  __shared__ unsigned long long zpres[KS_TOPO_TERMS];
  __shared__ int hmin[KS_TOPO_TERMS];
  __shared__ long long mins[KS_TOPO_TERMS];
  __shared__ int any_all;
  TopoRec tr;
  const int32_t pi = topo_pod(a, tr);
  if (pi < 0 || !(tr.flags & KS_TOPO_DYN)) return;
  const int tid = threadIdx.x;
  for (int i = tid; i < KS_TOPO_TERMS * KS_TOPO_ZONES; i += kTopoThreads) (&zsum[0][0])[i] = 0;
  if (tid < KS_TOPO_TERMS) {
    zpres[tid] = 0;
    hmin[tid] = 0x7FFFFFFF;  // newCriticalPaths: MatchNum math.MaxInt32
  }
  if (tid == 0) any_all = 0;
  __syncthreads();
  const PodStat* ps = a.stat ? a.stat + pi : nullptr;
  bool aff_host = false, need_aff = false;
  for (int t = 0; t < KS_TOPO_TERMS; ++t) {
    aff_host |= tp_kind(tr.term[t]) == KS_TOPO_K_AFFINITY && tp_key(tr.term[t]) == 0;
    need_aff |= tp_kind(tr.term[t]) == KS_TOPO_K_SPREAD_HARD || tp_kind(tr.term[t]) == KS_TOPO_K_SPREAD_SOFT;
  }
  // ---- PreFilter: the domain sums ----
  for (int64_t n = tid; n < a.n; n += kTopoThreads) {
    const int32_t z = a.t.zone[n];
    const bool aff = need_aff ? tp_node_aff(ps, a.labels ? a.labels[n] : 0ull) : true;
    for (int t = 0; t < KS_TOPO_TERMS; ++t) {
      const uint64_t w = tr.term[t];
      if (!w || !tp_eligible(w, tr.flags, aff, z >= 0)) continue;
      const int32_t cnt = a.t.count[(int64_t)tp_prop(w) * a.t.npad + n];
      if (tp_key(w) == 1) {
        if (z >= 0) {
          if (cnt) atomicAdd((unsigned long long*)&zsum[t][z], (unsigned long long)(long long)cnt);
          atomicOr(&zpres[t], 1ull << z);
        }
      } else if (tp_kind(w) == KS_TOPO_K_SPREAD_HARD) {
        atomicMin(&hmin[t], cnt);
      }
      if (tp_kind(w) == KS_TOPO_K_AFFINITY && cnt > 0 && (aff_host || z >= 0)) any_all = 1;
    }
  }
  __syncthreads();
  if (tid < KS_TOPO_TERMS) {
    long long m = hmin[tid];
    if (tp_key(tr.term[tid]) == 1)
      for (int z = 0; z < KS_TOPO_ZONES; ++z)
        if (((zpres[tid] >> z) & 1ull) && zsum[tid][z] < m) m = zsum[tid][z];
    mins[tid] = m;
  }
  __syncthreads();
  // ---- Filters ----
  for (int64_t n = tid; n < a.n; n += kTopoThreads) {
    const int32_t z = a.t.zone[n];
    const bool has_zone = z >= 0;
    uint32_t r = 0;
    bool aff = true;
    if (need_aff) aff = tp_node_aff(ps, a.labels ? a.labels[n] : 0ull);
    for (int t = 0; t < KS_TOPO_TERMS; ++t) {
      const uint64_t w = tr.term[t];
      if (tp_kind(w) != KS_TOPO_K_SPREAD_HARD) continue;
      if (tp_key(w) == 1 && !has_zone) {  // ErrReasonNodeLabelNotMatch
        r = KS_R_TOPOLOGY_SPREAD;
        break;
      }
      long long match;
      if (tp_key(w) == 1) match = ((zpres[t] >> z) & 1ull) ? zsum[t][z] : 0;
      else match = tp_eligible(w, tr.flags, aff, has_zone) ? a.t.count[(int64_t)tp_prop(w) * a.t.npad + n] : 0;
      const long long self = (tp_flags(w) & KS_TOPO_T_SELF) ? 1 : 0;
      if (match + self - mins[t] > (long long)tp_param(w)) {  // ErrReasonConstraintsNotMatch
        r = KS_R_TOPOLOGY_SPREAD;
        break;
      }
    }
    auto domain = [&](int t) -> long long {
      const uint64_t w = tr.term[t];
      return tp_key(w) == 1 ? zsum[t][z] : (long long)a.t.count[(int64_t)tp_prop(w) * a.t.npad + n];
    };
    bool aff_terms = false, missing = false, exist = true;
    for (int t = 0; t < KS_TOPO_TERMS; ++t) {
      if (tp_kind(tr.term[t]) != KS_TOPO_K_AFFINITY) continue;
      aff_terms = true;
      if (tp_key(tr.term[t]) == 1 && !has_zone) missing = true;
      else if (domain(t) <= 0) exist = false;
    }
    uint32_t ipa = 0;
    if (aff_terms && (missing || (!exist && !(any_all == 0 && (tr.flags & KS_TOPO_SELF_AFFINITY))))) {
      ipa = KS_R_POD_AFFINITY;
    } else {
      for (int t = 0; t < KS_TOPO_TERMS && !ipa; ++t) {
        const uint64_t w = tr.term[t];
        if (tp_kind(w) == KS_TOPO_K_ANTI && (tp_key(w) == 0 || has_zone) && domain(t) > 0) ipa = KS_R_POD_ANTI_AFFINITY;
      }
      for (int t = 0; t < KS_TOPO_TERMS && !ipa; ++t) {
        const uint64_t w = tr.term[t];
        if (tp_kind(w) == KS_TOPO_K_EXISTING_ANTI && (tp_key(w) == 0 || has_zone) && domain(t) > 0)
          ipa = KS_R_EXISTING_ANTI_AFFINITY;
      }
    }
    r |= ipa;
    if (r) {
      a.reasons[n] |= r;
      a.total[n] = -1;
      for (int k = 0; k < KS_NUM_SCORE_PLUGINS; ++k) a.scores[n * KS_NUM_SCORE_PLUGINS + k] = 0;
    }
  }
  // the sums for topo_norm_kernel
  for (int i = tid; i < KS_TOPO_TERMS * KS_TOPO_ZONES; i += kTopoThreads) (&a.scr->zsum[0][0])[i] = (&zsum[0][0])[i];
  if (tid < KS_TOPO_TERMS) a.scr->zpres[tid] = zpres[tid];
}

// DefaultNormalizeScore(100, reverse) of one raw column over the feasible nodes (DeviceShare, TaintToleration,
// NodeAffinity: normalize_score.go:24-52), weighted into total
__device__ void norm_default(const TopoKArgs& a, const int32_t* raw, int slot, int64_t w, bool reverse, int* smax) {
  if (threadIdx.x == 0) *smax = 0;
  __syncthreads();
  for (int64_t i = threadIdx.x; i < a.n; i += kTopoThreads)
    if (!a.reasons[i]) atomicMax(smax, raw[i]);
  __syncthreads();
  const int64_t mx = *smax;
  for (int64_t i = threadIdx.x; i < a.n; i += kTopoThreads) {
    if (a.reasons[i]) continue;
    int64_t sc;
    if (mx == 0) sc = reverse ? 100 : raw[i];
    else sc = reverse ? 100 - 100 * (int64_t)raw[i] / mx : 100 * (int64_t)raw[i] / mx;
    a.scores[i * KS_NUM_SCORE_PLUGINS + slot] = sc;
    a.total[i] += sc * w;
  }
  __syncthreads();
}

__global__ __launch_bounds__(kTopoThreads) void topo_norm_kernel(TopoKArgs a) {
  __shared__ long long zsum[KS_TOPO_TERMS][KS_TOPO_ZONES];
  __shared__ int smax32;
  __shared__ unsigned long long s_pref, s_max, s_zones, s_best;
  __shared__ long long s_hsize, s_smin, s_smax, s_imin, s_imax;
  __shared__ int s_empty;
  TopoRec tr;
  const int32_t pi = topo_pod(a, tr);
  if (pi < 0) return;
  const int tid = threadIdx.x;
  if (a.norm_others) {
    if (a.dev_on) norm_default(a, a.draw, KS_SCORE_DEVICESHARE, a.dev_w, false, &smax32);
    if (a.taint_on) norm_default(a, a.traw, KS_SCORE_TAINT, a.taint_w, true, &smax32);
    if (a.aff_on) norm_default(a, a.araw, KS_SCORE_NODE_AFFINITY, a.aff_w, false, &smax32);
    if (a.rsv_on) {
      // Reservation: the preferred node by order (scoring.go:87-96), Score, DefaultNormalizeScore
      if (tid == 0) {
        s_pref = 0;
        s_max = 0;
      }
      __syncthreads();
      for (int64_t i = tid; i < a.n; i += kTopoThreads)
        if (!a.reasons[i] && a.rhi[i] > 0)
          atomicMax(&s_pref, ((unsigned long long)a.rhi[i] << 32) | (0xFFFFFFFFull - (unsigned long long)i));
      __syncthreads();
      const int64_t pref = s_pref ? (int64_t)(0xFFFFFFFFull - (s_pref & 0xFFFFFFFFull)) : -1;
      for (int64_t i = tid; i < a.n; i += kTopoThreads)
        if (!a.reasons[i]) atomicMax(&s_max, (unsigned long long)(i == pref ? 1000 : a.rraw[i]));
      __syncthreads();
      const int64_t mx = (int64_t)s_max;
      for (int64_t i = tid; i < a.n; i += kTopoThreads) {
        if (a.reasons[i]) continue;
        const int64_t rs = i == pref ? 1000 : a.rraw[i];
        const int64_t sc = mx == 0 ? rs : 100 * rs / mx;
        a.scores[i * KS_NUM_SCORE_PLUGINS + KS_SCORE_RESERVATION] = sc;
        a.total[i] += sc * a.rsv_w;
      }
      __syncthreads();
    }
  }
  if (!(tr.flags & KS_TOPO_DYN)) {
    // no constraint: PodTopologySpread's NormalizeScore gives 100 everywhere (maxScore 0), InterPodAffinity 0
    for (int64_t n = tid; n < a.n; n += kTopoThreads) {
      if (a.reasons[n]) continue;
      a.scores[n * KS_NUM_SCORE_PLUGINS + KS_SCORE_TOPOLOGY_SPREAD] = 100;
      a.scores[n * KS_NUM_SCORE_PLUGINS + KS_SCORE_POD_AFFINITY] = 0;
      a.total[n] += 100 * a.spread_w;
    }
  } else {
    for (int i = tid; i < KS_TOPO_TERMS * KS_TOPO_ZONES; i += kTopoThreads) (&zsum[0][0])[i] = (&a.scr->zsum[0][0])[i];
    bool soft_zone = false;
    for (int t = 0; t < KS_TOPO_TERMS; ++t)
      soft_zone |= tp_kind(tr.term[t]) == KS_TOPO_K_SPREAD_SOFT && (tp_flags(tr.term[t]) & KS_TOPO_T_ELIG_ZONE);
    const bool soft_all = (tr.flags & KS_TOPO_SOFT_ALL_KEYS) != 0;
    if (tid == 0) {
      s_hsize = 0;
      s_zones = 0;
      s_empty = 0;
      s_smin = 0x7FFFFFFFFFFFFFFFll;
      s_smax = 0;
      s_imin = 0;
      s_imax = 0;
    }
    __syncthreads();
    // initPreScoreState: ignored nodes, topology sizes over the feasible nodes
    for (int64_t n = tid; n < a.n; n += kTopoThreads) {
      if (a.reasons[n]) continue;
      const int32_t z = a.t.zone[n];
      if (soft_all && soft_zone && z < 0) continue;
      atomicAdd((unsigned long long*)&s_hsize, 1ull);
      if (z >= 0) atomicOr(&s_zones, 1ull << z);
      else s_empty = 1;  // the pair (zone, "") of a node without the label
    }
    __syncthreads();
    const int64_t hsz = s_hsize, zsz = __popcll(s_zones) + s_empty;
    const double hw = a.t.lw[hsz < a.t.nlw ? hsz : a.t.nlw - 1], zw = a.t.lw[zsz < a.t.nlw ? zsz : a.t.nlw - 1];
    auto raws = [&](int64_t n, bool& ignored, long long& sr, long long& ir) {
      const int32_t z = a.t.zone[n];
      const bool has_zone = z >= 0;
      ignored = soft_all && soft_zone && !has_zone;
      double score = 0.0;
      ir = 0;
      for (int t = 0; t < KS_TOPO_TERMS; ++t) {
        const uint64_t w = tr.term[t];
        const int k = tp_kind(w);
        if (k != KS_TOPO_K_SPREAD_SOFT && k != KS_TOPO_K_SCORE) continue;
        if (tp_key(w) == 1 && !has_zone) continue;
        const long long cnt = tp_key(w) == 1 ? zsum[t][z] : (long long)a.t.count[(int64_t)tp_prop(w) * a.t.npad + n];
        if (k == KS_TOPO_K_SPREAD_SOFT) {
          if (!ignored) score = __dadd_rn(score, __dadd_rn(__dmul_rn((double)cnt, tp_key(w) == 1 ? zw : hw),
                                                           (double)(tp_param(w) - 1)));
        } else {
          ir += (long long)tp_param(w) * cnt;
        }
      }
      sr = ignored ? 0 : (long long)::round(score);
    };
    for (int64_t n = tid; n < a.n; n += kTopoThreads) {
      if (a.reasons[n]) continue;
      bool ig;
      long long sr, ir;
      raws(n, ig, sr, ir);
      if (!ig) {
        atomicMin(&s_smin, sr);
        atomicMax(&s_smax, sr);
      }
      atomicMin(&s_imin, ir);
      atomicMax(&s_imax, ir);
    }
    __syncthreads();
    const long long smin = s_smin, smx = s_smax, imin = s_imin, imax = s_imax;
    for (int64_t n = tid; n < a.n; n += kTopoThreads) {
      if (a.reasons[n]) continue;
      bool ig;
      long long sr, ir;
      raws(n, ig, sr, ir);
      long long sn;
      if (ig) sn = 0;
      else if (smx == 0) sn = 100;
      else sn = 100 * (smx + smin - sr) / smx;
      const long long diff = imax - imin;
      long long in = 0;
      if (diff > 0) in = (long long)__dmul_rn(100.0, __ddiv_rn((double)(ir - imin), (double)diff));
      a.scores[n * KS_NUM_SCORE_PLUGINS + KS_SCORE_TOPOLOGY_SPREAD] = sn;
      a.scores[n * KS_NUM_SCORE_PLUGINS + KS_SCORE_POD_AFFINITY] = in;
      a.total[n] += sn * a.spread_w + in * a.ipa_w;
    }
  }
  if (!a.cursor) return;
  // ---- selectHost: max total, lowest index; the one-candidate set for the commit ----
  __syncthreads();
  if (tid == 0) s_best = 0;
  __syncthreads();
  for (int64_t n = tid; n < a.n; n += kTopoThreads) {
    const int64_t t = a.total[n];
    if (t >= 0) atomicMax(&s_best, ((unsigned long long)(t + 1) << 32) | (0xFFFFFFFFull - (unsigned long long)n));
  }
  __syncthreads();
  if (tid == 0) {
    const unsigned long long b = s_best;
    if (b) {
      const int64_t node = (int64_t)(0xFFFFFFFFull - (b & 0xFFFFFFFFull));
      a.cand_chunk[0] = (uint32_t)(node >> 6);
      a.cand_t[0] = make_uint2((1u << 6) | (uint32_t)(63 - (node & 63)), 0u);  // an untouched node, key taken as is
      a.cand_count[0] = 1;
      a.scr->best_total = (int64_t)(b >> 32) - 1;
    } else {
      a.cand_count[0] = 0;  // no feasible node: the commit reports it unschedulable
      a.scr->best_total = 0;
    }
    a.cand_bound[0] = 0;
    a.cand_top[0] = 0;
    a.cand_second[0] = 0;
  }
}

hipError_t launch_topo_filter(hipStream_t s, const TopoKArgs& a) {
  hipLaunchKernelGGL(topo_filter_kernel, dim3(1), dim3(kTopoThreads), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_topo_norm(hipStream_t s, const TopoKArgs& a) {
  hipLaunchKernelGGL(topo_norm_kernel, dim3(1), dim3(kTopoThreads), 0, s, a);
  return hipGetLastError();
}

}  // namespace ks
