// ks_mono.h — the commit kernel for monotone plugin sets without Reservation, NodeNUMAResource or DeviceShare:
// NodeResourcesFit (LeastAllocated) + LoadAwareScheduling [+ ElasticQuota admission], SURVEY C1 / C2 / C5.
//
// Same contract as commit_kernel (ks_pass.h): one wave walks the pass's pods in queue order and applies every
// Reserve, so placements are those of scheduling one pod at a time.  What the plugin set lets it
// drop is most of the per-pod latency:
//  * every pod's snapshot-best ("top") node gets its slot row built in the prologue by all four waves, so the
//    fast path (top still untouched: commits only lower keys, it wins) reserves into a ready LDS row;
//  * a row is 54 words (f64 score terms, int64 headrooms / capacities, counts), built and reserved with one
//    word group per lane, and read lane = slot by the touched-slot evaluation through eval_pod_node (the one
//    Filter / Score implementation the sweep also runs);
//  * a slow pod's likely winner (its best untouched candidate) has its raw row put in flight from HBM as soon
//    as the candidates are resolved, before the touched-slot evaluation and rescans it overlaps;
//  * the loop state is a handful of lane-held words (no plugin switches: there is nothing to switch).
#pragma once

#include "ks_pass.h"

namespace ks {

// score terms and headrooms of a mono row
enum MonoTerm : int { MT_CPU = 0, MT_MEM = 1, MT_EPH = 2, MT_SC = 3, MT_LCPU = 7, MT_LMEM = 8, MT_PLCPU = 9, MT_PLMEM = 10, MT_N = 11 };
enum MonoFree : int { MF_CPU = 0, MF_MEM = 1, MF_EPH = 2, MF_SC = 3, MF_N = 7 };

struct __attribute__((aligned(16))) MonoRow {
  double hd[MT_N];     // 100 x headroom (f64 score path), 0 when the capacity is 0
  double r[MT_N];      // 1 / capacity, 0 when the capacity is 0
  int64_t fr[MF_N];    // Allocatable - Requested (Fit Filter)
  int64_t c[MT_N];     // capacity (int64 score path, write-back)
  int64_t h[MT_N];     // headroom, offset by kNoCap when the capacity is 0 (term_requested)
  uint32_t la_bits;
  int32_t fit_ws, allowed, pod_count;
  int64_t _pad;
};
// 432 B = 27 x 16 B (an odd number of 16 B units): lane = slot reads of one field are spread over the banks
static_assert(sizeof(MonoRow) == 432, "MonoRow layout");

constexpr int kMonoRows = 2 * kMaxBatch;  // rows 0..63: the top node of pod p (row p, for the first pod with
                                          // that top); rows 64..127: nodes first touched by slow pods

template <int NSC>
__device__ __forceinline__ void mono_to_reg(const MonoRow& m, NodeReg<NSC>& r) {
  auto term = [&](int t) { return Term{m.c[t], m.h[t], m.hd[t], m.r[t]}; };
  r.free_cpu = m.fr[MF_CPU];
  r.free_mem = m.fr[MF_MEM];
  r.free_eph = m.fr[MF_EPH];
  r.t_cpu = term(MT_CPU);
  r.t_mem = term(MT_MEM);
  r.t_eph = term(MT_EPH);
#pragma unroll
  for (int k = 0; k < NSC; ++k) {
    r.free_sc[k] = m.fr[MF_SC + k];
    r.t_sc[k] = term(MT_SC + k);
  }
  r.t_lcpu = term(MT_LCPU);
  r.t_lmem = term(MT_LMEM);
  r.t_plcpu = term(MT_PLCPU);
  r.t_plmem = term(MT_PLMEM);
  r.la_bits = m.la_bits;
  r.fit_ws = m.fit_ws;
  r.allowed = m.allowed;
  r.pod_count = m.pod_count;
  r.pods_full = (int64_t)m.pod_count + 1 > (int64_t)m.allowed;
  r.valid = 1;
  r.rsv_cls = 0;
  r.numa_A = 0;
  r.numa_off = 0;
  r.numa_ratio = 0.0;
  r.cpu_free = -1;
  r.cpu_cores = 0;
}

// Lane roles for building / reserving a row: lanes 0..10 own score term t = lane, lanes 11..17 headroom
// f = lane - 11, lane 18 the counts.  cap / req are raw row fields (RF_*), pw / pw100 PodRec words.
struct MonoRole {
  int32_t cap, req, pw, pw100;
  bool prod_only;
};

__device__ __forceinline__ MonoRole mono_role(int lane) {
  MonoRole o{0, 0, 0, 0, false};
  if (lane < MT_N) {
    const int t = lane;
    if (t == MT_CPU) o = MonoRole{RF_ALLOC_CPU, RF_NZ_CPU, 3, 12, false};
    else if (t == MT_MEM) o = MonoRole{RF_ALLOC_MEM, RF_NZ_MEM, 4, 13, false};
    else if (t == MT_EPH) o = MonoRole{RF_ALLOC_EPH, RF_REQ_EPH, 2, 14, false};
    else if (t < MT_LCPU) o = MonoRole{RF_ALLOC_SC + (t - MT_SC), RF_REQ_SC + (t - MT_SC), 7 + (t - MT_SC), 17 + (t - MT_SC), false};
    else if (t == MT_LCPU) o = MonoRole{RF_LA_ALLOC_CPU, RF_TERM_CPU, 5, 15, false};
    else if (t == MT_LMEM) o = MonoRole{RF_LA_ALLOC_MEM, RF_TERM_MEM, 6, 16, false};
    else if (t == MT_PLCPU) o = MonoRole{RF_LA_ALLOC_CPU, RF_PTERM_CPU, 5, 15, true};
    else o = MonoRole{RF_LA_ALLOC_MEM, RF_PTERM_MEM, 6, 16, true};
  } else if (lane < MT_N + MF_N) {
    const int f = lane - MT_N;
    if (f == MF_CPU) o = MonoRole{RF_ALLOC_CPU, RF_REQ_CPU, 0, 0, false};
    else if (f == MF_MEM) o = MonoRole{RF_ALLOC_MEM, RF_REQ_MEM, 1, 0, false};
    else if (f == MF_EPH) o = MonoRole{RF_ALLOC_EPH, RF_REQ_EPH, 2, 0, false};
    else o = MonoRole{RF_ALLOC_SC + (f - MF_SC), RF_REQ_SC + (f - MF_SC), 7 + (f - MF_SC), 0, false};
  }
  return o;
}

// make_node of a raw row (raw[RF_*]) into m, by lane role (lanes 0..18 of a wave, or one role per thread)
__device__ __forceinline__ void mono_build(const Cfg& cfg, MonoRow& m, const int64_t* raw, int role, const MonoRole& ro) {
  if (role < MT_N) {
    const int64_t cap = raw[ro.cap], req = raw[ro.req];
    m.c[role] = cap;
    m.h[role] = cap - req + (cap != 0 ? 0 : kNoCap);
    m.hd[role] = cap != 0 ? (double)(cap - req) * 100.0 : 0.0;
    m.r[role] = cap != 0 ? 1.0 / (double)cap : 0.0;
  } else if (role < MT_N + MF_N) {
    m.fr[role - MT_N] = raw[ro.cap] - raw[ro.req];
  } else if (role == MT_N + MF_N) {
    m.la_bits = (uint32_t)raw[RF_LA_BITS];
    m.allowed = (int32_t)raw[RF_ALLOWED];
    m.pod_count = (int32_t)raw[RF_POD_COUNT];
    m.fit_ws = (raw[RF_ALLOC_CPU] != 0 ? cfg.fw_cpu : 0) + (raw[RF_ALLOC_MEM] != 0 ? cfg.fw_mem : 0) +
               (raw[RF_ALLOC_EPH] != 0 ? cfg.fw_eph : 0);
  }
}

// reserve_row (NodeInfo.AddPod + podAssignCache.assign) of the pod whose PodRec words are podw, by lane role
__device__ __forceinline__ void mono_reserve(MonoRow& m, const int64_t* podw, bool prod, int role, const MonoRole& ro) {
  if (role < MT_N) {
    if (!ro.prod_only || prod) {
      m.h[role] -= podw[ro.pw];
      m.hd[role] -= __longlong_as_double(podw[ro.pw100]);
    }
  } else if (role < MT_N + MF_N) {
    m.fr[role - MT_N] -= podw[ro.pw];
  } else if (role == MT_N + MF_N) {
    m.pod_count += 1;
  }
}

struct MonoLayout {
  size_t rows, pods, res, pqreq, cand_t, cand_chunk, tops, raw1, quota, touched, total;
};

__host__ __device__ inline MonoLayout mono_layout(int32_t k, int64_t nchunks, bool qc, int32_t qrows = kQuotaLdsRows) {
  MonoLayout L;
  size_t o = 0;
  L.rows = o;
  o += (size_t)kMonoRows * sizeof(MonoRow);
  L.pods = o;
  o += (size_t)kMaxBatch * sizeof(PodRec);
  L.res = o;
  o += align16((size_t)kMaxBatch * sizeof(ks_result));
  L.pqreq = o;
  o += (size_t)kMaxBatch * KS_QUOTA_DIMS * 8;
  L.cand_t = o;
  o += (size_t)kMaxBatch * k * sizeof(uint2);
  L.cand_chunk = o;
  o += align16((size_t)kMaxBatch * k * 4);
  L.tops = o;
  o += (size_t)kMaxBatch * 8 + 32 * 4;  // per pod: top node, owner pod (the first pod with that top); field widths
  L.raw1 = o;
  o += 32 * 8;  // one raw row being turned into a slot row
  L.quota = o;
  if (qc) o += align16(quota_lds_bytes(qrows));
  L.touched = o;
  o += (size_t)nchunks * 8;
  L.total = o;
  return L;
}

// rescan_untouched for the mono kernel: the node-column pointers are re-read per rescan through an opaque
// pointer, so the compiler cannot hoist ~40 of them into SGPRs for the whole loop (rescans are rare)
template <int NSC>
__device__ __forceinline__ uint64_t mono_rescan(const DevNodes* dnp, const Cfg& cfg, const PodRec& pod, int64_t chunk,
                                             uint64_t touched_mask, int64_t n) {
  const int lane = threadIdx.x & 63;
  const int64_t node = chunk * 64 + lane;
  asm volatile("" : "+s"(dnp));
  const DevNodes d = *dnp;
  NodeReg<NSC> r;
  load_node<NSC>(cfg, d, node, node < n, r);
  const EvalOut o = eval_pod_node<NSC, false>(cfg, pod, r);
  const bool skip = o.reasons || ((touched_mask >> lane) & 1ull);
  return wave_max_u64(skip ? 0ull : gkey(o.total, node));
}

template <int NSC, bool QC>
__global__ __launch_bounds__(commit_threads(0)) void commit_mono_kernel(CommitArgs a) {
  constexpr int NT = commit_threads(0);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const int32_t K = a.k;
  const MonoLayout lay = mono_layout(K, a.nchunks, QC, a.q.q);
  MonoRow* rows = reinterpret_cast<MonoRow*>(smem_raw + lay.rows);
  PodRec* spods = reinterpret_cast<PodRec*>(smem_raw + lay.pods);
  ks_result* sres = reinterpret_cast<ks_result*>(smem_raw + lay.res);
  int64_t* pqreq = reinterpret_cast<int64_t*>(smem_raw + lay.pqreq);
  uint2* cand_t = reinterpret_cast<uint2*>(smem_raw + lay.cand_t);
  uint32_t* cand_chunk = reinterpret_cast<uint32_t*>(smem_raw + lay.cand_chunk);
  int32_t* top_node = reinterpret_cast<int32_t*>(smem_raw + lay.tops);
  int32_t* top_owner = top_node + kMaxBatch;
  int64_t* raw1 = reinterpret_cast<int64_t*>(smem_raw + lay.raw1);
  QuotaRowsLds qview = quota_lds(smem_raw + lay.quota, a.q.q);
  QuotaRowsLds* qlds = &qview;
  unsigned long long* touched = reinterpret_cast<unsigned long long*>(smem_raw + lay.touched);
  // prologue staging of the top nodes' raw rows ([64][32] words) in the dynamic-row half of `rows`
  int64_t* rawtop = reinterpret_cast<int64_t*>(rows + kMaxBatch);
  static_assert((size_t)kMaxBatch * 32 * 8 <= (size_t)kMaxBatch * sizeof(MonoRow), "rawtop staging");
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int32_t cursor0 = __builtin_amdgcn_readfirstlane(*a.cursor);
  if (cursor0 >= a.total_pods) {
    if (threadIdx.x == 0) pipe_next(a, cursor0);  // the queue is done: so are the speculative sweeps after it
    return;
  }
  if (pipe_bubble(a, cursor0)) return;
  const int32_t np = topo_pass_pods(a, cursor0, min(a.batch, a.total_pods - cursor0));
  if (np == 0) return;  // a topology pod at the cursor: the next topology step takes it
  const Cfg cfg = a.c;
#if defined(KS_COMMIT_SEG) && !defined(KS_COMMIT_CAT)
#define KS_COMMIT_CAT
#endif
#ifdef KS_COMMIT_CAT
  // diagnostic builds.  KS_COMMIT_CAT: whole-iteration cycles per pod category in diag[0..4] (0 quota-rejected,
  // 1 fast, 2 slow onto a new slot, 3 slow onto a touched slot, 4 unschedulable), counts of 2 / 3 in diag[5..6].
  // KS_COMMIT_SEG: the fast pods' iteration split in diag[0..3] (admission + fast check, slot assignment,
  // row reserve, result + quota), the other pods' cycles in diag[4].
  uint64_t ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t tcat = 0, tseg[4] = {0, 0, 0, 0};
  int32_t cat = 0;
#define KS_MCAT(c) cat = (c)
#ifdef KS_COMMIT_SEG
#define KS_MSEG(i) tseg[i] = __builtin_amdgcn_s_memtime()
#else
#define KS_MSEG(i) \
  do {             \
  } while (0)
#endif
#else
#define KS_MSEG(i) \
  do {             \
  } while (0)
#define KS_MCAT(c) \
  do {             \
  } while (0)
#endif

  // ---- prologue: the pass into LDS (all four waves, independent loads in one burst) ----
  lds_copy<NT>(cand_chunk, a.cand_chunk, np * K, tid);
  lds_copy<NT>(cand_t, a.cand_t, np * K, tid);
  for (int32_t i = tid; i < np * KS_QUOTA_DIMS; i += NT) {
    const int32_t p = i / KS_QUOTA_DIMS, dd = i - p * KS_QUOTA_DIMS;
    pqreq[i] = a.pq.req[dd][cursor0 + p];
  }
  {
    const int64_t* src = reinterpret_cast<const int64_t*>(a.pods + cursor0);
    int64_t* dst = reinterpret_cast<int64_t*>(spods);
    const int32_t words = np * (int32_t)(sizeof(PodRec) / 8);
    lds_copy<NT>(dst, src, words, tid);
  }
  for (int64_t c = tid; c < a.nchunks; c += NT) touched[c] = 0ull;
  if (QC) {
    for (int32_t r = tid; r < a.q.q; r += NT) {
      qlds->parent[r] = a.q.parent[r];
      qlds->limit_mask[r] = a.q.limit_mask[r];
      qlds->min_mask[r] = a.q.min_mask[r];
    }
    for (int32_t i = tid; i < a.q.q * KS_QUOTA_DIMS; i += NT) {
      qlds->limit[i] = a.q.limit[i];
      qlds->used[i] = a.q.used[i];
      qlds->min[i] = a.q.min[i];
      qlds->npused[i] = a.q.npused[i];
    }
  }
  // raw rows of every pod's top node (a node shared by several pods is loaded once per pod: no dependency on
  // the owner computation, which runs while these loads are in flight)
  lds_rawtop<NT>(rawtop, a.cand_top, a.rowcols, np, tid);
  if (tid < kMaxBatch) {
    const uint64_t t = tid < np ? a.cand_top[tid] : 0ull;
    top_node[tid] = t ? (int32_t)gkey_node(t) : -1;
  }
  __syncthreads();
  constexpr int kRoles = MT_N + MF_N + 1;
  // every top row (role per thread); wave 0 also finds each pod's owner: the first pod of the pass with the same
  // top node, whose row the slot of that node uses
  for (int32_t i = tid; i < np * kRoles; i += NT) {
    const int32_t p = i / kRoles, role = i - p * kRoles;
    if (top_node[p] >= 0) mono_build(cfg, rows[p], rawtop + p * 32, role, mono_role(role));
  }
  // and the previous pod with the same top node (my_prev; -1: none), which bounds a run of fast pods
  int32_t my_prev = -1;
  if (tid < 64) {
    const int32_t tn = top_node[lane];
    int32_t own = -1;
    for (int32_t q = 0; q < np; ++q) {
      const int32_t v = __builtin_amdgcn_readlane(tn, q);
      own = (own < 0 && v == tn) ? q : own;
      my_prev = (q < lane && v == tn) ? q : my_prev;
    }
    top_owner[lane] = own;
  }
  // wave 1 stages pod p's small per-pod values and the row-field columns in LDS (raw1 / the res area are free until
  // the loop): wave 0 reads them from there, so no global load is outstanding when its loop starts (the loop
  // header's wait state would otherwise merge them with the speculative row loads in flight across iterations
  // and wait for everything at every iteration's top)
  int64_t* stage = reinterpret_cast<int64_t*>(sres);  // bound [64], top [64], count / quota mask [64] x i32
  static_assert(sizeof(ks_result) * kMaxBatch >= 64 * 8 * 3, "per-pod staging");
  if (tid >= 64 && tid < 128 && lane < np) {
    stage[lane] = (int64_t)a.cand_bound[lane];
    stage[64 + lane] = (int64_t)a.cand_top[lane];
    int32_t* st32 = reinterpret_cast<int32_t*>(stage + 128);
    st32[lane] = a.cand_count[lane];
    st32[64 + lane] = (int32_t)a.pq.mask[cursor0 + lane];
  }
  if (tid >= 128 && tid < 128 + RF_N) {
    raw1[lane] = (int64_t)(uintptr_t)a.rowcols[lane].p;
    reinterpret_cast<int32_t*>(top_node + 2 * kMaxBatch)[lane] = a.rowcols[lane].width;
  }
  __syncthreads();
  if (tid >= 64) return;  // the other waves are done; wave 0 runs the sequential loop alone
  int32_t my_cnt = 0, my_quota = -1, my_tn = -1, my_own = 0;
  uint32_t my_flags = 0, my_pmask = 0;
  uint64_t my_bound = 0, my_top = 0;
  if (lane < np) {
    my_bound = (uint64_t)stage[lane];
    my_top = (uint64_t)stage[64 + lane];
    const int32_t* st32 = reinterpret_cast<const int32_t*>(stage + 128);
    my_cnt = st32[lane];
    my_pmask = (uint32_t)st32[64 + lane];
    my_quota = spods[lane].quota;
    my_flags = spods[lane].flags;
    my_tn = top_node[lane];
    my_own = top_owner[lane];
  }
  const void* my_col = nullptr;
  int32_t my_w = 8;
  if (lane < RF_N) {
    my_col = (const void*)(uintptr_t)raw1[lane];
    my_w = reinterpret_cast<const int32_t*>(top_node + 2 * kMaxBatch)[lane];
  }
  const MonoRole ro = mono_role(lane);
  const int32_t Kc = K;

  int32_t snode = -1, srow = -1;  // lane s: node and row of slot s
  int32_t nslots = 0, ndyn = 0;
  int32_t processed = np;
  uint32_t rescans = 0, misses = 0, fast = 0;
  FieldLd spec_val{0u, 0u, false};  // raw row field `lane` of spec_node, in flight from HBM (combined at its use)
  int32_t spec_node = -1;
#ifdef KS_COMMIT_CAT
  tcat = __builtin_amdgcn_s_memtime();
#endif

  for (int32_t j = 0; j < np; ++j) {
    KS_MCAT(0);
    if (!QC && !cfg.quota_enable) {
      // ---- a run of fast pods, committed together ----
      // Pods j, j+1, .. whose snapshot-best (top) nodes are untouched and distinct from each other's are all
      // fast one after the other: each commit touches only its own top, so the next pod's top is still
      // untouched and still wins.  Lane p tests pod p; the run ends at the first pod that fails (it takes the
      // per-pod path below).  Their slots, touched bits, results and Reserves are independent of each other.
      bool ok = false;
      if (lane >= j && lane < np && my_top != 0ull && my_prev < j)
        ok = !((touched[my_tn >> 6] >> (my_tn & 63)) & 1ull);
      const uint64_t bad = ~__ballot(ok) & (~0ull << j);
      const int32_t end = min(np, bad ? (int32_t)__ffsll((long long)bad) - 1 : 64);
      const int32_t R = end - j;
      if (R > 1) {
        const bool in_run = lane >= j && lane < end;
        if (in_run) {
          atomicOr(&touched[my_tn >> 6], 1ull << (my_tn & 63));
          sres[lane] = ks_result{my_tn, KS_S_SCHEDULED, gkey_score(my_top), -1, 0, 0, 0};
        }
        // slot nslots + k <- pod j + k (its top node and that node's prebuilt row)
        const int32_t src = lane - nslots + j;
        const int32_t tn_s = __shfl(my_tn, src & 63, 64), own_s = __shfl(my_own, src & 63, 64);
        if (lane >= nslots && lane < nslots + R) {
          snode = tn_s;
          srow = own_s;
        }
        // Reserve: (pod, role) items, one per lane
        // (the shuffles run with every lane active; only the store is predicated)
        for (int32_t i0 = 0; i0 < R * kRoles; i0 += 64) {
          const int32_t i = i0 + lane;
          const int32_t k = min(i / kRoles, R - 1), role = i - k * kRoles;
          const int32_t pj = j + k;
          const int32_t ri = __shfl(my_own, pj, 64);
          const uint32_t pf = (uint32_t)__shfl((int32_t)my_flags, pj, 64);
          if (i < R * kRoles)
            mono_reserve(rows[ri], reinterpret_cast<const int64_t*>(&spods[pj]), (pf & KS_POD_PROD) != 0, role,
                         mono_role(role));
        }
        nslots += R;
        fast += (uint32_t)R;
        j = end - 1;
#ifdef KS_COMMIT_CAT
        {
          const uint64_t t_ = __builtin_amdgcn_s_memtime();
          ph[1] += t_ - tcat;
          tcat = t_;
        }
#endif
        continue;
      }
    }
    // ---- ElasticQuota admission (lane d = dimension d) and the fast check, their LDS reads issued together ----
    const uint64_t top = readlane64(my_top, j);
    const int32_t tn = top ? (int32_t)gkey_node(top) : 0;
    const uint64_t tw = touched[tn >> 6];
    uint32_t st = 0;
    const int32_t qrow = __builtin_amdgcn_readlane(my_quota, j);
    const uint32_t pflags = __builtin_amdgcn_readlane(my_flags, j);
    if (cfg.quota_enable && qrow >= 0) {
      const uint32_t pmask = __builtin_amdgcn_readlane(my_pmask, j);
      const int64_t req = pqreq[j * KS_QUOTA_DIMS + (lane & (KS_QUOTA_DIMS - 1))];
      st = QC ? quota_admit(qlds->parent, qlds->limit_mask, qlds->min_mask, qlds->limit, qlds->used, qlds->min,
                            qlds->npused, cfg.quota_parent, qrow, pflags, pmask, req)
              : quota_admit(a.q.parent, a.q.limit_mask, a.q.min_mask, a.q.limit, a.q.used, a.q.min, a.q.npused,
                            cfg.quota_parent, qrow, pflags, pmask, req);
    }
    if (st) {
      if (lane == 0) sres[j] = ks_result{-1, st, 0, -1, 0, 0, 0};
      goto next_pod;
    }
    {
      uint64_t best;
      if (top && !((tw >> (tn & 63)) & 1ull)) {
        best = top;  // the snapshot-best node is untouched: commits only lower keys, so it wins
        ++fast;
        KS_MCAT(1);
      } else {
        KS_MCAT(2);
        const Cands cj = resolve_cands(cand_chunk, cand_t, touched, j, Kc, __builtin_amdgcn_readlane(my_cnt, j));
        // the likely winner's raw row in flight from HBM (unless it has a prebuilt top row) while the touched
        // slots are evaluated
        if (cj.umax) {
          const int32_t un = (int32_t)gkey_node(cj.umax);
          if (un != spec_node && !__ballot(lane < np && my_tn == un)) {
            spec_node = un;
            if (lane < RF_N) spec_val = field_issue(my_col, my_w, un);
          }
        }
        PodRec pod = spods[j];
        pod.flags = pflags;
        uint64_t key_mod = 0;
        if (lane < nslots) {
          NodeReg<NSC> r;
          mono_to_reg<NSC>(rows[srow], r);
          const EvalOut o = eval_pod_node<NSC, false>(cfg, pod, r);
          if (o.reasons == 0) key_mod = gkey(o.total, snode);
        }
        best = umax64(cj.umax, wave_max_u64(key_mod));
        uint64_t need = __ballot(!cj.exact && cj.valid && cj.ub > best);
        while (need) {
          const uint64_t kmax = wave_max_u64(((need >> lane) & 1ull) ? cj.ub : 0ull);
          const int sel = __ffsll((long long)__ballot(((need >> lane) & 1ull) && cj.ub == kmax)) - 1;
          const int64_t c = (int64_t)(uint32_t)__shfl((int)cj.chunk, sel, 64);
          const uint64_t v = mono_rescan<NSC>(a.dn, cfg, pod, c, touched[c], a.n);
          ++rescans;
          best = umax64(best, v);
          need &= ~(1ull << sel);
          need &= __ballot(cj.ub > best);
        }
        if (best < readlane64(my_bound, j)) {
          processed = j;  // an untouched chunk outside the list may hold a better node: re-sweep from j
          break;
        }
      }
      KS_MSEG(0);
      if (best == 0) {
        KS_MCAT(4);
        if (lane == 0) sres[j] = ks_result{-1, KS_S_UNSCHEDULABLE, 0, -1, 0, 0, 0};
        goto next_pod;
      }
      const int32_t node = (int32_t)gkey_node(best);
      const int64_t* podw = reinterpret_cast<const int64_t*>(&spods[j]);
      int32_t s = __ffsll((long long)__ballot(snode == node)) - 1;
      int32_t ri;
      if (s >= 0) {
        KS_MCAT(3);
        ri = __builtin_amdgcn_readlane(srow, s);
      } else {
        // a new slot: the prebuilt row of a pod's top node (untouched until now, so still the snapshot), or a
        // row built from the node's raw fields
        s = nslots++;
        if (lane == 0) atomicOr(&touched[node >> 6], 1ull << (node & 63));
        const uint64_t own = __ballot(lane < np && my_tn == node && my_own == lane);
        if (own) {
          ri = __ffsll((long long)own) - 1;
        } else {
          ri = kMaxBatch + ndyn++;
          int64_t v = 0;
          if (node != spec_node) {
            ++misses;
            if (lane < RF_N) v = load_field(my_col, my_w, node);
          } else {
            v = field_value(spec_val);
          }
          if (lane < RF_N) raw1[lane] = v;
          if (lane < kRoles) mono_build(cfg, rows[ri], raw1, lane, ro);
        }
        if (lane == s) {
          snode = node;
          srow = ri;
        }
      }
      KS_MSEG(1);
      if (lane < kRoles) mono_reserve(rows[ri], podw, (pflags & KS_POD_PROD) != 0, lane, ro);
      KS_MSEG(2);
      if (lane == 0) sres[j] = ks_result{node, KS_S_SCHEDULED, gkey_score(best), -1, 0, 0, 0};
      if (cfg.quota_enable && qrow >= 0) {
        const uint32_t pmask = __builtin_amdgcn_readlane(my_pmask, j);
        if (lane < KS_QUOTA_DIMS && ((pmask >> lane) & 1u)) {
          // updatePodUsedNoLock -> updateGroupDeltaUsedNoLock (group_quota_manager.go:620-655)
          const int64_t qreq = pqreq[j * KS_QUOTA_DIMS + lane];
          const bool np_ = (pflags & KS_POD_NONPREEMPTIBLE) != 0;
          if (QC) {
            for (int32_t cur = qrow; cur >= 0;) {
              const int32_t up = qlds->parent[cur];
              atomicAdd((unsigned long long*)&qlds->used[(size_t)cur * KS_QUOTA_DIMS + lane], (unsigned long long)qreq);
              if (np_) atomicAdd((unsigned long long*)&qlds->npused[(size_t)cur * KS_QUOTA_DIMS + lane], (unsigned long long)qreq);
              cur = up;
            }
          } else {
            for (int32_t cur = qrow; cur >= 0; cur = a.q.parent[cur]) {
              a.q.used[(size_t)cur * KS_QUOTA_DIMS + lane] += qreq;
              if (np_) a.q.npused[(size_t)cur * KS_QUOTA_DIMS + lane] += qreq;
            }
          }
        }
      }
    }
  next_pod:;
#ifdef KS_COMMIT_CAT
    {
      const uint64_t t_ = __builtin_amdgcn_s_memtime();
#ifdef KS_COMMIT_SEG
      if (cat == 1) {
        ph[0] += tseg[0] - tcat;
        ph[1] += tseg[1] - tseg[0];
        ph[2] += tseg[2] - tseg[1];
        ph[3] += t_ - tseg[2];
      } else {
        ph[4] += t_ - tcat;
      }
#else
      ph[cat] += t_ - tcat;
      if (cat == 2) ph[5] += 1;
      if (cat == 3) ph[6] += 1;
#endif
      tcat = t_;
    }
#endif
  }
  // ---- write back: results, touched rows, quota usage ----
  if (lane < processed) {
    ks_result r = sres[lane];
    topo_writeback(a, cursor0 + lane, r);
    a.results[cursor0 + lane] = r;
  }
  if (lane < nslots) {
    const DevNodes d = *a.dn;
    const MonoRow& m = rows[srow];
    const int64_t node = snode;
    auto requested = [&](int t) { return m.c[t] - m.h[t] + (m.c[t] != 0 ? 0 : kNoCap); };
    gst(d.req_cpu + node, m.c[MT_CPU] - m.fr[MF_CPU]);
    gst(d.req_mem + node, m.c[MT_MEM] - m.fr[MF_MEM]);
    gst(d.req_eph + node, m.c[MT_EPH] - m.fr[MF_EPH]);
    gst(d.nz_cpu + node, requested(MT_CPU));
    gst(d.nz_mem + node, requested(MT_MEM));
#pragma unroll
    for (int k = 0; k < KS_MAX_SCALARS; ++k) gst(d.req_sc[k] + node, m.c[MT_SC + k] - m.fr[MF_SC + k]);
    gst(d.pod_count + node, m.pod_count);
    gst(d.la_term_cpu + node, requested(MT_LCPU));
    gst(d.la_term_mem + node, requested(MT_LMEM));
    gst(d.la_pterm_cpu + node, requested(MT_PLCPU));
    gst(d.la_pterm_mem + node, requested(MT_PLMEM));
  }
  if (QC) {
    for (int32_t i = lane; i < a.q.q * KS_QUOTA_DIMS; i += 64) {
      a.q.used[i] = qlds->used[i];
      a.q.npused[i] = qlds->npused[i];
    }
  }
  pipe_carry(a, nslots, snode);
  if (a.top_reset) a.top_reset[lane] = 0ull;
  if (lane == 0) {
    *a.cursor = cursor0 + processed;
    pipe_next(a, cursor0 + processed);
    atomicAdd(&a.counters[0], 1ull);
    if (processed < np) atomicAdd(&a.counters[1], 1ull);
    atomicAdd(&a.counters[2], (unsigned long long)rescans);
    atomicAdd(&a.counters[3], (unsigned long long)misses);
    atomicAdd(&a.counters[15], (unsigned long long)fast);  // ks_stats.diag[7]: monotone fast picks
#ifdef KS_COMMIT_CAT
    for (int i = 0; i < 7; ++i) atomicAdd(&a.counters[8 + i], (unsigned long long)ph[i]);
#endif
  }
#undef KS_MCAT
#undef KS_MSEG
}

}  // namespace ks
