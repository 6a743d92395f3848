// ks_topo.hip — the topology step's kernels (ks_topo.h).  One thread per node, 256-thread workgroups over the
// cluster; each wave pre-reduces (per quantity, or per distinct domain of its nodes) and issues one global atomic each,
// so a reduction over 5k nodes is ~80 atomics per address rather than 5k.  The step's sequence:
//   topo_sums_kernel   PreFilter: per term the domain sums, domains present, hostname minimum (eligible nodes only)
//   eval_debug_kernel  every plugin's Filter / Score + topo_eval_node: both plugins' Filters, InterPodAffinity's raw
//                      score, the other plugins' normalization maxima (ks_debug.hip)
//   topo_pts_kernel    PodTopologySpread PreScore / Score: the topology sizes' weights (per soft constraint, from the
//                      counted nodes' domains eval_debug_kernel marked), raw scores, their extrema;
//                      the Reservation raw maximum (needs the preferred node)
//   topo_norm_kernel   every NormalizeScore + weighted totals + selectHost; the per-domain scratch zeroed by every
//                      workgroup's slice; the last workgroup writes the one-candidate set (or commits) and puts the
//                      scratch back to its initial image
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
// Every f64 operation is Go's, in Go's order (-ffp-contract=off, explicit _rn intrinsics).
#include <climits>
#include <cstring>

#include "ks_pass.h"  // (quota_admit)
#include "ks_topo.h"

namespace ks {

constexpr int kTopoThreads = 256;

TopoScratch topo_scratch_init() {
  TopoScratch s;
  std::memset(&s, 0, sizeof(s));
  for (int t = 0; t < kTopoTerms; ++t) s.hmin[t] = INT_MAX;  // newCriticalPaths: MatchNum math.MaxInt32
  s.smin = LLONG_MAX;
  s.cur_pi = -1;
  return s;
}

// LDS slots of a workgroup's domain sums ([term][domain], u32: a workgroup's nodes' counts): when the step's terms x
// domains fit, each workgroup sums in LDS and issues one global atomic per non-zero slot; else one per distinct domain
// of each wave (topo_seg_add)
constexpr int kTopoLdsSums = 4096;

__global__ __launch_bounds__(kTopoThreads) void topo_sums_kernel(TopoKArgs a) {
  __shared__ uint32_t zl[kTopoLdsSums];
  const int tid = threadIdx.x;
  const int64_t n = (int64_t)blockIdx.x * kTopoThreads + tid;
  const bool in = n < a.n;
  const int64_t n0 = in ? n : 0;
  const uint64_t lab = a.labels ? a.labels[n0] : 0ull;  // (the node's loads issued with the cursor -> record chain)
  const TopoNodeDom nd = topo_node_dom(a.t, n0);
  TopoRec tr;
  const int32_t pi = topo_pod(a, tr);
  const TopoTerms tt = pi >= 0 ? topo_terms_of(a, tr) : TopoTerms{};
  if (blockIdx.x == 0 && tid < 64) {
    if (tid == 0) {
      a.scr->cur_pi = pi;
      a.scr->cur_rec = tr;
    }
    if (tid < kTopoInline) a.scr->cur_terms[tid] = (pi >= 0 && tid < tr.nterms) ? a.terms[tr.tbeg + tid] : 0ull;
  }
  if (pi < 0 || !(tr.flags & KS_TOPO_DYN)) return;  // (grid-uniform)
  // the first terms' counts and domains, loaded together
  int32_t c8[kTopoInline], z8[kTopoInline];
#pragma unroll
  for (int t = 0; t < kTopoInline; ++t) {
    const uint64_t w = tt.w[t];
    c8[t] = t < tr.nterms ? tp_count(a.t, w, n0) : 0;
    z8[t] = (t < tr.nterms && tp_key(w) != 0) ? tp_dom(a.t, nd, tp_key(w)) : 0;
  }
  const int32_t nslot = tr.nterms * a.t.ndom;
  const bool lds = nslot <= kTopoLdsSums;  // (grid-uniform)
  if (lds)
    for (int k = tid; k < nslot; k += kTopoThreads) zl[k] = 0u;
  bool need_aff = false;
  topo_each(a, tr, tt, [&](int, uint64_t w) {
    const int k = tp_kind(w);
    need_aff |= k == KS_TOPO_K_SPREAD_HARD || k == KS_TOPO_K_SPREAD_SOFT;
    return true;
  });
  const bool aff = need_aff ? tp_node_aff(a.stat ? a.stat + pi : nullptr, lab) : true;
  const TopoKeysOk keys = topo_keys_ok(a, tr, tt, nd);
  TopoScratch* s = a.scr;
  bool aav = false;
  __syncthreads();
  auto term = [&](int t, uint64_t w, int32_t c, int32_t zn) {  // (wave-uniform)
    const bool el = in && tp_eligible(w, tr.flags, aff, keys.hard, keys.soft);
    const int32_t cnt = el ? c : 0;
    int32_t z = 0;
    if (tp_key(w) != 0) {
      z = in ? zn : -1;
      // the domain's sum, and for a hard constraint the domains with an eligible node (TpPairToMatchNum's keys)
      const bool on = el && z >= 0;
      if (lds) {
        if (on && cnt) atomicAdd(&zl[t * a.t.ndom + z], (uint32_t)cnt);
      } else {
        topo_seg_add(a.t.zsum + (int64_t)t * a.t.ndom, nullptr, on, z, cnt);
      }
      if (tp_kind(w) == KS_TOPO_K_SPREAD_HARD) topo_bits_or(a.t.zpres + (int64_t)t * a.t.nw, a.t.ndom, on, z);
    } else if (tp_kind(w) == KS_TOPO_K_SPREAD_HARD) {
      const uint32_t m = ~wave_max_u32(~(uint32_t)(el ? cnt : INT_MAX));  // (counts are >= 0)
      if ((tid & 63) == 0 && m != (uint32_t)INT_MAX) atomicMin(&s->hmin[t], (int)m);
    }
    // affinityCounts: a pod matching every required term counts on each term's (key, value) the node has
    if (tp_kind(w) == KS_TOPO_K_AFFINITY) aav |= el && cnt > 0 && z >= 0;
  };
#pragma unroll
  for (int t = 0; t < kTopoInline; ++t)
    if (t < tr.nterms) term(t, tt.w[t], c8[t], z8[t]);
  for (int t = kTopoInline; t < tr.nterms; ++t) {
    const uint64_t w = topo_term(a, tr, t);
    term(t, w, tp_count(a.t, w, n0), tp_key(w) != 0 ? tp_dom(a.t, nd, tp_key(w)) : 0);
  }
  if (__ballot(aav) && (tid & 63) == 0) atomicOr(&s->any_all, 1);
  if (lds) {  // the workgroup's sums: [term][domain] is zsum's layout
    __syncthreads();
    for (int k = tid; k < nslot; k += kTopoThreads)
      if (zl[k]) atomicAdd((unsigned long long*)(a.t.zsum + k), (unsigned long long)zl[k]);
  }
}

// topologyNormalizingWeight(size) = log(size + 2), from the host's table
__device__ __forceinline__ double topo_weight(const DevTopo& t, unsigned long long size) {
  return t.lw[size < (unsigned long long)t.nlw ? size : (unsigned long long)t.nlw - 1];
}

// Issue the node's loads with the step's pod record, then wait once (a kernel of the step otherwise waits for the record,
// branches, and only then loads its node)
#define KS_TOPO_ISSUED(...) asm volatile("" ::__VA_ARGS__)

__global__ __launch_bounds__(kTopoThreads) void topo_pts_kernel(TopoKArgs a) {
  __shared__ double tw[kTopoTerms];
  __shared__ unsigned int tsz[kTopoTerms];
  const int tid = threadIdx.x;
  const int64_t i = (int64_t)blockIdx.x * kTopoThreads + tid;
  const bool in = i < a.n;
  const TopoScratch* s = a.scr;
  const uint32_t rs = in ? a.reasons[i] : 1u;
  const int32_t rr = (in && a.rsv_on) ? a.rraw[i] : 0;
  const unsigned long long hs = s->hsize, rp = s->rsv_pref;
  const TopoNodeDom nd = topo_node_dom(a.t, in ? i : 0);
  TopoRec tr;
  const int32_t pi = topo_cur(a, tr);
  const TopoTerms tt = topo_terms_cur(a);
  KS_TOPO_ISSUED("v"(rs), "v"(rr));
  if (pi < 0) return;  // (grid-uniform)
  const bool dyn = (tr.flags & KS_TOPO_DYN) != 0;
  const bool soft_all = (tr.flags & KS_TOPO_SOFT_ALL_KEYS) != 0;
  // initPreScoreState's sizes per soft constraint: the hostname's the non-ignored feasible nodes, another key's their
  // distinct values (a node without the label counts as the value "")
  if (dyn) {
    if (tid < kTopoTerms) tsz[tid] = 0u;
    __syncthreads();
    topo_each(a, tr, tt, [&](int t, uint64_t w) {
      if (tp_kind(w) != KS_TOPO_K_SPREAD_SOFT || tp_key(w) == 0) return true;
      unsigned int c = 0;
      for (int k = tid; k < a.t.nw; k += kTopoThreads) c += (unsigned int)__popc(a.t.zsize[(int64_t)t * a.t.nw + k]);
      c = wave_sum_u32(c);
      if (c && (tid & 63) == 0) atomicAdd(&tsz[t], c);
      return true;
    });
    __syncthreads();
    if (tid < tr.nterms) {
      const uint64_t w = topo_term(a, tr, tid);
      tw[tid] = topo_weight(a.t, tp_key(w) == 0 ? hs : (unsigned long long)tsz[tid] + (s->tempty[tid] ? 1ull : 0ull));
    }
    __syncthreads();
  }
  const int64_t pref = rp ? (int64_t)(0xFFFFFFFFull - (rp & 0xFFFFFFFFull)) : -1;
  bool counted = false;
  long long sr = 0;
  uint64_t rmx = 0;
  if (in && rs == 0) {
    if (a.rsv_on) rmx = i == pref ? 1000ull : (uint64_t)(uint32_t)rr;
    if (dyn) {
      // PodTopologySpread's raw score (PreScore's pair counts, Score's scoreForCount summed in term order in Go's f64
      // order, math.Round); an ignored node (requireAllTopologies, a soft key missing) scores 0 and is not counted
      const bool ignored = soft_all && !topo_keys_ok(a, tr, tt, nd).soft;
      double score = 0.0;
      topo_each(a, tr, tt, [&](int t, uint64_t w) {
        if (tp_kind(w) != KS_TOPO_K_SPREAD_SOFT) return true;  // (wave-uniform)
        long long cnt;
        if (tp_key(w) == 0) {
          cnt = (long long)tp_count(a.t, w, i);
        } else {
          const int32_t z = tp_dom(a.t, nd, tp_key(w));
          if (z < 0) return true;  // (a node without the key adds nothing)
          cnt = a.t.zsum[(int64_t)t * a.t.ndom + z];
        }
        score = __dadd_rn(score, __dadd_rn(__dmul_rn((double)cnt, tw[t]), (double)(tp_param(w) - 1)));
        return true;
      });
      counted = !ignored;
      sr = ignored ? 0 : (long long)::round(score);
      a.sraw[i] = sr;
    }
  }
  const long long smn = wave_min_i64(counted ? sr : LLONG_MAX), smx = wave_max_i64(counted ? sr : 0);
  const uint64_t rm = wave_max_u64(rmx);
  if ((tid & 63) == 0) {
    TopoScratch* w = a.scr;
    if (smn != LLONG_MAX) atomicMin(&w->smin, smn);
    if (smx > 0) atomicMax(&w->smax, smx);
    if (rm) atomicMax(&w->rsv_max, (unsigned long long)rm);
  }
}

// One wave (lane = quota dimension): ElasticQuota PreFilter (quota_admit), then on the step's chosen node the Reserve of
// the plugin sets without DeviceShare / Reservation / NodeNUMAResource -- NodeInfo.AddPod (Requested, NonZeroRequested,
// pod count, UsedPorts), podAssignCache.assign (the LoadAware estimate terms, prod too for a prod pod), the quota chain's
// used (non-preemptible used) and the pod's topology properties -- the same column updates the commit kernel's slot rows
// write back (ks_unreserve's inverse), then the cursor.  p / pmask / qreq: pod c's records, loaded ahead by the caller.
__device__ __forceinline__ void topo_commit_one(const TopoCommitArgs& a, int lane, int32_t c, const TopoRec& tr,
                                                const PodRec& p, uint32_t pmask, int64_t qreq, int64_t n, long long total) {
  uint32_t st = 0;
  if (a.quota_enable && p.quota >= 0)
    st = quota_admit(a.q.parent, a.q.limit_mask, a.q.min_mask, a.q.limit, a.q.used, a.q.min, a.q.npused,
                     a.quota_parent != 0, p.quota, p.flags, pmask, qreq);
  ks_result r{-1, st, 0, -1, 0, 0, 0};
  if (!st && n < 0) r.status = KS_S_UNSCHEDULABLE;
  if (!st && n >= 0) {
    r = ks_result{(int32_t)n, KS_S_SCHEDULED, total, -1, 0, 0, 0};
    if (a.quota_enable && p.quota >= 0 && lane < KS_QUOTA_DIMS && ((pmask >> lane) & 1u))
      for (int32_t cur = p.quota; cur >= 0; cur = a.q.parent[cur]) {
        a.q.used[(size_t)cur * KS_QUOTA_DIMS + lane] += qreq;
        if (p.flags & KS_POD_NONPREEMPTIBLE) a.q.npused[(size_t)cur * KS_QUOTA_DIMS + lane] += qreq;
      }
    if (lane == 0) {
      const DevNodes& d = a.d;
      d.req_cpu[n] += p.cpu;
      d.req_mem[n] += p.mem;
      d.req_eph[n] += p.eph;
      for (int k = 0; k < KS_MAX_SCALARS; ++k) d.req_sc[k][n] += p.sc[k];
      d.nz_cpu[n] += p.nzcpu;
      d.nz_mem[n] += p.nzmem;
      d.pod_count[n] += 1;
      d.la_term_cpu[n] += p.est_cpu;
      d.la_term_mem[n] += p.est_mem;
      if (p.flags & KS_POD_PROD) {
        d.la_pterm_cpu[n] += p.est_cpu;
        d.la_pterm_mem[n] += p.est_mem;
      }
      if (a.ports & 1) d.host_ports[n] |= a.pstat[c].pwant;
    }
    // the pod's properties (lanes over its list)
    for (int32_t k = lane; k < tr.nprops; k += 64) atomicAdd(a.topo_count + (int64_t)a.props[tr.pbeg + k] * a.topo_npad + n, 1);
  }
  if (lane == 0) {
    a.results[c] = r;
    *a.cursor = c + 1;
    atomicAdd(&a.counters[0], 1ull);
  }
}

// The last-workgroup hand-off below relies on gfx9's vmcnt covering non-returning atomics (each wave waits for its own
// atomics before the workgroup's arrival) and on agent-scope atomics being performed at the memory side across XCDs,
// so that the arrival ticket needs no L2 write-back fence.  Another ISA needs a release / acquire
// ticket instead.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "topo_norm_kernel's fence-free arrival ticket is written for gfx950"
#endif

// lean != 0: the last workgroup also commits the pod (topo_commit_one, the plugin sets whose Reserve is AddPod + the
// assign cache + quota); else it leaves the one-candidate set and the chosen node for the general commit kernel
__global__ __launch_bounds__(kTopoThreads) void topo_norm_kernel(TopoKArgs a, TopoCommitArgs ca, int32_t lean) {
  __shared__ bool last;
  const int tid = threadIdx.x;
  const int64_t i = (int64_t)blockIdx.x * kTopoThreads + tid;
  const bool in = i < a.n;
  TopoScratch* s = a.scr;
  // the node's inputs and the reductions' results, issued with the step's pod record
  const uint32_t rs = in ? a.reasons[i] : 1u;
  const int64_t tot0 = in ? a.total[i] : 0;
  const int32_t dr = (in && a.dev_on) ? a.draw[i] : 0, tr_ = (in && a.taint_on) ? a.traw[i] : 0,
                ar = (in && a.aff_on) ? a.araw[i] : 0, rr = (in && a.rsv_on) ? a.rraw[i] : 0;
  const long long sri = in ? a.sraw[i] : 0, iri = in ? a.iraw[i] : 0;
  const int64_t dmx = s->dev_max, tmx = s->taint_max, amx = s->aff_max;
  const int64_t rmx = (int64_t)s->rsv_max;
  const unsigned long long rp = s->rsv_pref;
  const long long smin = s->smin, smax = s->smax, imin = s->imin, imax = s->imax;
  TopoRec tr;
  const int32_t pi = topo_cur(a, tr);
  const TopoTerms tt = topo_terms_cur(a);
  KS_TOPO_ISSUED("v"(rs), "v"(tot0), "v"(dr), "v"(tr_), "v"(ar), "v"(rr), "v"(sri), "v"(iri));
  if (pi < 0) return;
  // the commit's pod records (wave 0 of every workgroup: the last one to finish uses them)
  PodRec p{};
  uint32_t pmask = 0;
  int64_t qreq = 0;
  if (lean && tid < 64) {
    p = ca.pods[pi];
    pmask = ca.pq.mask[pi];
    qreq = tid < KS_QUOTA_DIMS ? ca.pq.req[tid][pi] : 0;
  }
  const bool dyn = (tr.flags & KS_TOPO_DYN) != 0;
  const bool soft_all = (tr.flags & KS_TOPO_SOFT_ALL_KEYS) != 0;
  const int64_t pref = rp ? (int64_t)(0xFFFFFFFFull - (rp & 0xFFFFFFFFull)) : -1;
  uint64_t key = 0;
  if (in && rs == 0) {
    int64_t* sc = a.scores ? a.scores + i * KS_NUM_SCORE_PLUGINS : nullptr;  // (NULL: the batch step)
    int64_t tot = tot0;
    // DefaultNormalizeScore (normalize_score.go:24-52): DeviceShare, TaintToleration (reverse), NodeAffinity
    if (a.dev_on) {
      const int64_t v = dmx == 0 ? dr : 100 * (int64_t)dr / dmx;
      if (sc) sc[KS_SCORE_DEVICESHARE] = v;
      tot += v * a.dev_w;
    }
    if (a.taint_on) {
      const int64_t v = tmx == 0 ? 100 : 100 - 100 * (int64_t)tr_ / tmx;
      if (sc) sc[KS_SCORE_TAINT] = v;
      tot += v * a.taint_w;
    }
    if (a.aff_on) {
      const int64_t v = amx == 0 ? ar : 100 * (int64_t)ar / amx;
      if (sc) sc[KS_SCORE_NODE_AFFINITY] = v;
      tot += v * a.aff_w;
    }
    // Reservation: the preferred node scores mostPreferredScore (scoring.go:87-122), DefaultNormalizeScore
    if (a.rsv_on) {
      const int64_t r = i == pref ? 1000 : rr, v = rmx == 0 ? r : 100 * r / rmx;
      if (sc) sc[KS_SCORE_RESERVATION] = v;
      tot += v * a.rsv_w;
    }
    long long pts = 100, ipa = 0;  // no constraint: NormalizeScore's maxScore == 0 gives MaxNodeScore
    if (dyn) {
      const bool ig = soft_all && !topo_keys_ok(a, tr, tt, topo_node_dom(a.t, i)).soft;
      if (ig) pts = 0;
      else if (smax != 0) pts = 100 * (smax + smin - sri) / smax;
      const long long diff = imax - imin;
      if (diff > 0) ipa = (long long)__dmul_rn(100.0, __ddiv_rn((double)(iri - imin), (double)diff));
    }
    if (sc) {
      sc[KS_SCORE_TOPOLOGY_SPREAD] = pts;
      sc[KS_SCORE_POD_AFFINITY] = ipa;
    }
    tot += pts * a.spread_w + ipa * a.ipa_w;
    a.total[i] = tot;
    key = ((uint64_t)(tot + 1) << 32) | (0xFFFFFFFFull - (uint64_t)i);  // selectHost: max total, lowest index
  }
  const uint64_t km = wave_max_u64(key);
  if ((tid & 63) == 0 && km) atomicMax(&s->best, (unsigned long long)km);
  // the step's per-domain scratch back to zero (read by no kernel after topo_pts_kernel): every workgroup a slice
  if (dyn) {
    const int64_t stride = (int64_t)gridDim.x * kTopoThreads;
    const int64_t g = (int64_t)blockIdx.x * kTopoThreads + tid;
    topo_each(a, tr, tt, [&](int t, uint64_t w) {
      if (tp_key(w) == 0) return true;
      for (int64_t z = g; z < a.t.ndom; z += stride) a.t.zsum[(int64_t)t * a.t.ndom + z] = 0;
      for (int64_t k = g; k < a.t.nw; k += stride) {
        a.t.zpres[(int64_t)t * a.t.nw + k] = 0u;
        a.t.zsize[(int64_t)t * a.t.nw + k] = 0u;
      }
      return true;
    });
  }
  // the last workgroup: the commit or the one-candidate set, then the scratch back to its initial image.  The only
  // value handed between workgroups is `best`, an agent-scope atomic performed at the memory side: each wave waits
  // for its own atomic to complete before the workgroup's arrival (no L2 write-back fence: the scores and totals are
  // read only after the kernel), and the last workgroup reads it with an agent-scope load.  This relies on gfx9's
  // counters: vmcnt also covers the non-returning atomicMax (gfx10+ split the store counter off), so other targets
  // must not build it (the error below) and need a release / acquire pair on `done` instead.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "topo_norm_kernel's fence-free hand-over is written for gfx950's vmcnt semantics"
#endif
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) last = __hip_atomic_fetch_add(&s->done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  const unsigned long long b = __hip_atomic_load(&s->best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const long long best_total = b ? (long long)(b >> 32) - 1 : 0;
  const long long best_node = b ? (long long)(0xFFFFFFFFull - (b & 0xFFFFFFFFull)) : -1;
  if (lean) {
    if (tid < 64) topo_commit_one(ca, tid, pi, tr, p, pmask, qreq, best_node, best_total);
  } else if (tid == 0) {
    if (a.cand_chunk) {
      if (b) {
        a.cand_chunk[0] = (uint32_t)(best_node >> 6);
        a.cand_t[0] = make_uint2((1u << 6) | (uint32_t)(63 - (best_node & 63)), 0u);  // an untouched node, key as is
        a.cand_count[0] = 1;
      } else {
        a.cand_count[0] = 0;  // no feasible node: the commit reports the pod unschedulable
      }
      a.cand_bound[0] = 0;
      a.cand_top[0] = 0;
      a.cand_second[0] = 0;
    }
    s->best_total = best_total;
    s->best_node = best_node;
  }
  if (tid < kTopoTerms) {
    s->hmin[tid] = INT_MAX;
    s->tempty[tid] = 0;
  }
  if (tid == 0) {
    s->any_all = 0;
    s->hsize = 0;
    s->dev_max = s->taint_max = s->aff_max = 0;
    s->imin = s->imax = 0;
    s->smin = LLONG_MAX;
    s->smax = 0;
    s->rsv_pref = s->rsv_max = 0;
    s->best = 0;
    s->done = 0;
  }
}

static unsigned topo_blocks(const TopoKArgs& a) { return (unsigned)std::max<int64_t>(1, (a.n + kTopoThreads - 1) / kTopoThreads); }

hipError_t launch_topo_sums(hipStream_t s, const TopoKArgs& a) {
  hipLaunchKernelGGL(topo_sums_kernel, dim3(topo_blocks(a)), dim3(kTopoThreads), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_topo_pts(hipStream_t s, const TopoKArgs& a) {
  hipLaunchKernelGGL(topo_pts_kernel, dim3(topo_blocks(a)), dim3(kTopoThreads), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_topo_norm(hipStream_t s, const TopoKArgs& a, const TopoCommitArgs* c) {
  hipLaunchKernelGGL(topo_norm_kernel, dim3(topo_blocks(a)), dim3(kTopoThreads), 0, s, a, c ? *c : TopoCommitArgs{},
                     (int32_t)(c != nullptr));
  return hipGetLastError();
}

}  // namespace ks
