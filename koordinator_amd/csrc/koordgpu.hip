// koordgpu.hip — MI355X (gfx950) scheduling evaluator behind the C ABI in include/koordgpu.h.
//
// Pipeline for ks_schedule (one "pass" = up to 64 queued pods):
//
//   sweep_kernel    streams the node SoA once per pod group, evaluates Filter+Score for every
//                   (pod, node) with the reference's int64 formulas, and reduces each 64-node
//                   chunk to its best (score, lowest index) per pod          -> chunk maxima
//   select_kernel   per pod: the K best chunks (exact top-K by key)          -> candidate lists
//   commit_kernel   ONE wave walks the pass's pods in queue order: quota admission, pick the best
//                   candidate whose chunk no earlier pod of the pass touched, re-scan touched
//                   chunks exactly, Reserve (NodeInfo/assign-cache/quota updates)  -> results
//
// Exactness: a pod's best node is max(best untouched node, best touched node).  Untouched nodes
// keep their snapshot score, so chunk maxima of untouched chunks are exact; touched chunks are
// re-scanned with the current state.  When every candidate chunk of a pod is touched and their
// re-scanned best is below the K-th snapshot key, an untouched chunk outside the list could win:
// the pass is cut there and the next pass re-sweeps from that pod.  Results are therefore
// identical to scheduling one pod at a time (oracle/koord_oracle.c).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include <rccl/rccl.h>

#include "ks_pass.h"
#include "ks_mono.h"
#include "ks_debug.h"
#include "ks_topo.h"
#include "ks_preempt.h"

using namespace ks;

// Launch-shape overrides for tuning runs (tools/sweep_shape.sh); unset = the built-in heuristic.
// A malformed or out-of-range value is reported on stderr and ignored (the default is used).
static int64_t env_i64(const char* name, int64_t dflt, int64_t lo, int64_t hi) {
  const char* v = std::getenv(name);
  if (!v || !*v) return dflt;
  char* end = nullptr;
  const long long x = std::strtoll(v, &end, 10);
  if (*end != '\0' || x < lo || x > hi) {
    fprintf(stderr, "libkoordgpu: ignoring %s=%s (expected an integer in [%lld, %lld])\n", name, v, (long long)lo,
            (long long)hi);
    return dflt;
  }
  return (int64_t)x;
}

// the candidate lists' initial fill byte (KS_TEST_POISON_LISTS=1: large words, for tests; else zeros)
static int list_fill() { return env_i64("KS_TEST_POISON_LISTS", 0, 0, 1) ? 0x3F : 0; }

// ------------------------------------------------------------------------------------------
// prep kernels
// ------------------------------------------------------------------------------------------

// usage := int64(math.Round(float64(used.MilliValue()) / float64(total.MilliValue()) * 100))
// (load_aware.go:214,248); threshold 0 and zero total are skipped (:185-192)
__device__ __forceinline__ bool usage_exceeds(int64_t used, int64_t total, int32_t thr) {
  if (thr == 0 || total == 0) return false;
  const int64_t usage = (int64_t)::round((double)used / (double)total * 100.0);
  return usage >= thr;
}

// Per-node LoadAware filter/score flags; pod-dependent only through prod / daemonset.
__global__ void prep_nodes_kernel(DevNodes d, int64_t n, int32_t filter_expired) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t f = d.la_flags[i];
  uint32_t bits = 0;
  if (!(f & KS_LA_HAS_METRIC) || (f & KS_LA_EXPIRED)) bits |= kLaZeroScore;  // load_aware.go:278-289
  const bool pass_all = !(f & KS_LA_HAS_METRIC) || (filter_expired && (f & KS_LA_EXPIRED));
  uint32_t r_np = 0, r_p = 0;
  if (!pass_all) {
    // filterNodeUsage (load_aware.go:173-224)
    if ((f & KS_LA_NODE_THR_NONEMPTY) && (f & KS_LA_HAS_STATUS_METRIC) && (f & KS_LA_FILTER_USAGE_PRESENT)) {
      const uint32_t agg = (f & KS_LA_AGGREGATED_FILTER) ? KS_R_LA_AGGREGATED : 0u;
      if (usage_exceeds(d.la_usage_cpu[i], d.la_total_cpu[i], d.la_thr_cpu[i]))
        r_np = KS_R_LA_CPU | agg;
      else if (usage_exceeds(d.la_usage_mem[i], d.la_total_mem[i], d.la_thr_mem[i]))
        r_np = KS_R_LA_MEMORY | agg;
    }
    if (f & KS_LA_PROD_THR_NONEMPTY) {
      // filterProdUsage (load_aware.go:226-254)
      if (f & KS_LA_HAS_PODS_METRIC) {
        if (usage_exceeds(d.la_pusage_cpu[i], d.la_total_cpu[i], d.la_pthr_cpu[i]))
          r_p = KS_R_LA_CPU | KS_R_LA_PROD;
        else if (usage_exceeds(d.la_pusage_mem[i], d.la_total_mem[i], d.la_pthr_mem[i]))
          r_p = KS_R_LA_MEMORY | KS_R_LA_PROD;
      }
    } else {
      r_p = r_np;  // prod pods fall back to the node-usage path (load_aware.go:148-168)
    }
  }
  if (r_np) bits |= kLaFailNonProd | (r_np << kLaReasonNonProdShift);
  if (r_p) bits |= kLaFailProd | (r_p << kLaReasonProdShift);
  // NodeNUMAResource: Amplify(allocated, ratio) = int64(math.Ceil(float64(allocated) * ratio)), ratio > 1
  // (apis/extension/node_resource_amplification.go:170-175)
  const double ratio = d.numa_ratio[i];
  const int64_t A = (int64_t)d.numa_cpus[i] * 1000;
  const bool amp = ratio > 1.0;
  d.numa_amilli[i] = A;
  d.numa_off[i] = amp ? (int64_t)::ceil((double)A * ratio) - A : 0;
  if (amp) bits |= kNumaAmp;
  if ((d.numa_flags[i] >> KS_NUMA_POLICY_SHIFT) & 3u) bits |= kNumaPolNode;
  if (d.numa_flags[i] & KS_NUMA_INVALID_RATIO) bits |= kNumaInvalid;
  // a score-term capacity outside the f64 path's range (ks_device.h term_least): the node scores in int64
  bool big = d.alloc_cpu[i] >= kBigCap || d.alloc_mem[i] >= kBigCap || d.alloc_eph[i] >= kBigCap ||
             d.la_alloc_cpu[i] >= kBigCap || d.la_alloc_mem[i] >= kBigCap;
  for (int k = 0; k < KS_MAX_SCALARS; ++k) big |= d.alloc_sc[k][i] >= kBigCap;
  if (big) bits |= kNodeBigCap;
  d.la_bits[i] = bits;
}

struct DevPodCols {
  int64_t *cpu, *mem, *eph, *nzcpu, *nzmem;
  int64_t *sc[KS_MAX_SCALARS];
  uint32_t *flags;
  int32_t *quota;
  int64_t *la_req_cpu, *la_lim_cpu, *la_dflt_cpu, *la_req_mem, *la_lim_mem, *la_dflt_mem;
  int32_t *rsv_class;
  int64_t *gpu_core, *gpu_mem, *gpu_ratio, *rdma;
  uint32_t* cpu_bind;
  uint8_t* joint;
  uint8_t* stat_dyn;  // per pod: 1 = a TaintToleration / NodeAffinity raw score can differ between nodes (host-built)
  const TopoRec* topo;  // PodTopologySpread / InterPodAffinity records (NULL = off)
};

// estimatedUsedByResource (estimator/default_estimator.go:73-108)
__device__ __forceinline__ int64_t estimated_used(int64_t req, int64_t lim, int64_t sf, int64_t dflt) {
  int64_t q;
  if (lim > req) {
    sf = 100;
    q = lim;
  } else {
    q = req;
  }
  if (q == 0) return dflt;
  int64_t est = (int64_t)::round((double)q * (double)sf / 100.0);
  if (lim > 0 && est > lim) est = lim;
  return est;
}

__global__ void prep_pods_kernel(DevPodCols s, PodRec* out, int32_t np, int64_t sf_cpu, int64_t sf_mem, int32_t dev_on) {
  const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= np) return;
  PodRec r;
  r.cpu = s.cpu[i];
  r.mem = s.mem[i];
  r.eph = s.eph[i];
  r.nzcpu = s.nzcpu[i];
  r.nzmem = s.nzmem[i];
  r.est_cpu = estimated_used(s.la_req_cpu[i], s.la_lim_cpu[i], sf_cpu, s.la_dflt_cpu[i]);
  r.est_mem = estimated_used(s.la_req_mem[i], s.la_lim_mem[i], sf_mem, s.la_dflt_mem[i]);
  for (int k = 0; k < KS_MAX_SCALARS; ++k) r.sc[k] = s.sc[k][i];
  uint32_t fl = s.flags[i] & 0xffu;
  if (r.cpu == 0 && r.mem == 0 && r.eph == 0 && !(fl & KS_POD_SCALAR_KEYS)) fl |= kPodAllZero;
  r.flags = fl;
  r.quota = s.quota[i];
  // 100 x the score-term requests as f64 (exact below kBigReq; a larger request sends the pod's terms to the
  // int64 path, ks_device.h term_least)
  r.h_nzcpu = (double)r.nzcpu * 100.0;
  r.h_nzmem = (double)r.nzmem * 100.0;
  r.h_eph = (double)r.eph * 100.0;
  r.h_est_cpu = (double)r.est_cpu * 100.0;
  r.h_est_mem = (double)r.est_mem * 100.0;
  bool big = false;
  for (int k = 0; k < KS_MAX_SCALARS; ++k) {
    r.h_sc[k] = (double)r.sc[k] * 100.0;
    big |= r.sc[k] >= kBigReq || r.sc[k] < 0;
  }
  const int64_t tw[7] = {r.cpu, r.mem, r.eph, r.nzcpu, r.nzmem, r.est_cpu, r.est_mem};
  for (int k = 0; k < 7; ++k) big |= tw[k] >= kBigReq || tw[k] < 0;
  if (big) fl |= kPodBigReq;
  r.flags = fl;
  r.rsv_class = s.rsv_class[i];
  uint32_t keys = 0;
  const int64_t dims[3] = {r.cpu, r.mem, r.eph};
  for (int d = 0; d < 3; ++d) keys |= dims[d] != 0 ? (1u << d) : 0u;
  for (int k = 0; k < KS_MAX_SCALARS; ++k) keys |= r.sc[k] != 0 ? (1u << (3 + k)) : 0u;
  r.rsv_keys = keys;
  if (keys == 0) r.flags |= kPodReqZero;
  r.h_cpu = (double)r.cpu * 100.0;
  r.h_mem = (double)r.mem * 100.0;
  r.gpu_core = s.gpu_core[i];
  r.gpu_mem = s.gpu_mem[i];
  r.gpu_ratio = s.gpu_ratio[i];
  if (r.gpu_core != 0 || r.gpu_mem != 0 || r.gpu_ratio != 0) r.flags |= kPodHasGpu | kPodGpuReq;
  r.rdma = s.rdma ? s.rdma[i] : 0;
  r.joint = s.joint ? s.joint[i] : 0u;
  r._pad0 = 0;
  if (r.rdma > 0) r.flags |= kPodHasGpu;
  if (dev_on && (r.flags & kPodHasGpu)) r.flags |= kPodDevNoNom;
  // a normalized score that can differ between nodes: DeviceShare (device requests), TaintToleration / NodeAffinity
  if ((r.flags & kPodHasGpu) || s.stat_dyn[i]) r.flags |= kPodNormDyn;
  if (s.topo && (s.topo[i].flags & KS_TOPO_DYN)) r.flags |= kPodTopoDyn;
  r.cpu_bind = (r.flags & KS_POD_CPU_BIND) ? ((s.cpu_bind[i] & 0x1Fu) | ((uint32_t)(r.cpu / 1000) << 8)) : 0u;
  out[i] = r;
}

// ------------------------------------------------------------------------------------------
// select: top-K chunks per pod (by chunk best)
// ------------------------------------------------------------------------------------------

struct SelectArgs {
  const uint2* __restrict__ in;  // sweep output
  const int32_t* __restrict__ cursor;
  uint32_t* cand_chunk;          // [64][K]
  uint2* cand_t;                 // [64][K] {best, runner-up} local keys
  uint64_t* cand_bound;          // [64]
  uint64_t* cand_top;            // [64] the pod's snapshot-best key over every chunk
  uint64_t* cand_second;         // [64] the pod's second-best key (its best node other than the top's)
  int32_t* cand_count;           // [64]
  int32_t* cand_total;           // [64] feasible chunks in this range (before the top-K cut)
  int64_t nchunks;               // row stride of the sweep output
  int64_t c0, c1;                // chunk range selected over
  int32_t total_pods, batch, k;
  // Pipelined passes: block 0 writes the first pod of the NEXT pass's speculative sweep.  *cursor is
  // this pass's first pod, *real_cursor where the previous commit left the queue: this pass commits iff they are
  // equal, and then the next pass starts after its pods; otherwise (a bubble) the next pass starts at the cursor.
  int32_t* next_base;            // NULL = not pipelined
  const int32_t* real_cursor;
  const PodRec* pods;            // a topology pod at the cursor: nothing to select (ks_topo.h)
};


// One workgroup of four waves per pod.  The pod's column of chunk keys (the sweep output is chunk-major: its
// coalesced side is the sweep's stores, and the 16 pods sharing a 128 B line are 16 workgroups of this launch, served by
// L2) is staged in LDS once as a row: every thread
// issues up to kSelUnroll independent loads before the first wait, so at C5 (1,563 chunks) the row arrives
// in about one HBM round trip instead of one per 64 chunks (one wave walking the row was latency-bound:
// 18.8 us per launch).  All four waves build an LDS histogram of the chunk scores; wave 0 finds the K-th
// largest score from it (binary search over the LDS copy when the score range exceeds the histogram) and
// writes the candidate list in chunk order.
constexpr int kSelHistBins = 1024;
constexpr int kSelThreads = 256;
constexpr int kSelUnroll = 8;
constexpr size_t kSelScratch = 128;  // cross-wave partials after the histogram
constexpr int kSelBlocks = 2 * kMaxBatch;  // (select_kernel: pods 16x..16x+15 on the blocks of XCD x < 4)
__host__ __device__ inline size_t select_smem(int64_t nc) { return (size_t)nc * sizeof(uint2) + kSelHistBins * 4 + kSelScratch; }

__global__ __launch_bounds__(kSelThreads) void select_kernel(SelectArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint2 srow[];  // [nchunks]
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = tid >> 6;
  const int32_t cursor = __builtin_amdgcn_readfirstlane(*a.cursor);
  if (a.next_base && blockIdx.x == 0 && tid == 0) {
    const int32_t rc = *a.real_cursor;
    *a.next_base = (cursor == rc && cursor < a.total_pods) ? cursor + min(a.batch, a.total_pods - cursor) : rc;
  }
  if (cursor < a.total_pods && (__builtin_amdgcn_readfirstlane(a.pods[cursor].flags) & kPodTopoDyn)) return;
  if (cursor >= a.total_pods) return;
  const int32_t np = min(a.batch, a.total_pods - cursor);
  // XCD-aware pod placement (blocks are dealt round-robin over the 8 XCDs): the 16 pods whose words share a 128-B line
  // of a chunk row run on one XCD, so each line is fetched into one L2 once, not by every XCD (kSelBlocks blocks, those
  // of XCDs 4-7 idle)
  const int32_t xcd = (int32_t)(blockIdx.x & 7u);
  if (xcd >= kMaxBatch / 16) return;
  const int32_t p = xcd * 16 + (int32_t)(blockIdx.x >> 3);
  if (p >= np) return;
  const int32_t K = a.k;
  const int64_t nc = a.c1 - a.c0;  // LDS row index e <-> chunk c0 + e
  const uint2* in = a.in + (size_t)a.c0 * kMaxBatch + p;  // chunk-major sweep output: the pod's column, stride 64
  uint32_t* hist = reinterpret_cast<uint32_t*>(srow + nc);
  uint64_t* xw = reinterpret_cast<uint64_t*>(hist + kSelHistBins);  // [0..3] top, [4..7] cnt | hmax << 32, [8] t | need_eq << 32
  int32_t cnt = 0;
  uint32_t hmax = 0;
  uint64_t top = 0;
  for (int i = tid; i < kSelHistBins; i += kSelThreads) hist[i] = 0u;
  for (int64_t e0 = tid; e0 < nc; e0 += (int64_t)kSelThreads * kSelUnroll) {
    uint2 v[kSelUnroll];
#pragma unroll
    for (int u = 0; u < kSelUnroll; ++u) {
      const int64_t e = e0 + (int64_t)u * kSelThreads;
      v[u] = e < nc ? in[(size_t)e * kMaxBatch] : make_uint2(0u, 0u);
    }
#pragma unroll
    for (int u = 0; u < kSelUnroll; ++u) {
      const int64_t e = e0 + (int64_t)u * kSelThreads;
      if (e < nc) {
        srow[e] = v[u];
        const uint32_t h = v[u].x >> 6;
        cnt += h != 0;
        hmax = h > hmax ? h : hmax;
        top = umax64(top, local_gkey(v[u].x, a.c0 + e));
      }
    }
  }
  cnt = wave_sum_i32(cnt);
  hmax = wave_max_u32(hmax);
  top = wave_max_u64(top);
  if (lane == 0) {
    xw[wv] = top;
    xw[4 + wv] = (uint64_t)(uint32_t)cnt | ((uint64_t)hmax << 32);
  }
  __syncthreads();
  cnt = 0;
  hmax = 0;
  top = 0;
#pragma unroll
  for (int w = 0; w < kSelThreads / 64; ++w) {
    top = umax64(top, xw[w]);
    cnt += (int32_t)(uint32_t)xw[4 + w];
    const uint32_t hm = (uint32_t)(xw[4 + w] >> 32);
    hmax = hm > hmax ? hm : hmax;
  }
  uint32_t t = 1;  // admit h >= t
  int32_t need_eq = 0x7fffffff;
  const bool exhaustive = cnt <= K;
  const bool use_hist = !exhaustive && hmax < kSelHistBins;
  if (use_hist) {
    // histogram of chunk scores (LDS atomics from all four waves)
    for (int64_t e = tid; e < nc; e += kSelThreads) {
      const uint32_t h = srow[e].x >> 6;
      if (h) atomicAdd(&hist[h], 1u);
    }
    __syncthreads();
  }
  if (wv != 0) return;  // waves 1-3 are done
  if (!exhaustive) {
    if (use_hist) {
      // the largest t with count(h >= t) >= K by a suffix scan over the bins (lane l owns bins [l*B, l*B+B))
      constexpr int B = kSelHistBins / 64;
      uint32_t mine[B];
      uint32_t part = 0;
#pragma unroll
      for (int i = 0; i < B; ++i) {
        mine[i] = hist[lane * B + i];
        part += mine[i];
      }
      // inclusive suffix sum of the per-lane partials: count of h in bins >= lane*B
      uint32_t suf = part;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const uint32_t v = __shfl_down(suf, off, 64);
        suf += (lane + off < 64) ? v : 0u;
      }
      // the lane holding t: suf(lane) >= K and suf(lane+1) < K
      const uint32_t suf_next = suf - part;
      const bool here = suf >= (uint32_t)K && suf_next < (uint32_t)K;
      uint32_t tl = 0, gtl = 0;
      if (here) {
        uint32_t acc = suf_next;
        for (int i = B - 1; i >= 0; --i) {
          if (acc + mine[i] >= (uint32_t)K) {
            tl = (uint32_t)(lane * B + i);
            gtl = acc;  // count of h > t
            break;
          }
          acc += mine[i];
        }
      }
      const uint64_t hb = __ballot(here);
      const int src = __ffsll((long long)hb) - 1;
      t = (uint32_t)__shfl((int)tl, src, 64);
      need_eq = K - (int32_t)__shfl((int)gtl, src, 64);
    } else {
      uint32_t lo = 1, hi = hmax;  // largest t with count(h >= t) >= K
      while (lo < hi) {
        const uint32_t mid = lo + (hi - lo + 1) / 2;
        int32_t c = 0;
        for (int64_t e = lane; e < nc; e += 64) c += (srow[e].x >> 6) >= mid;
        c = wave_sum_i32(c);
        if (c >= K) lo = mid;
        else hi = mid - 1;
      }
      t = lo;
      int32_t gt = 0;
      for (int64_t e = lane; e < nc; e += 64) gt += (srow[e].x >> 6) > t;
      gt = wave_sum_i32(gt);
      need_eq = K - gt;
    }
  }
  // every h > t, plus the first need_eq entries (chunk order) with h == t; on the way, the second-best key over
  // every chunk (the top's chunk contributes its runner-up): the commit prefetches that node's row too
  int32_t base = 0, eq_taken = 0;
  uint64_t bound = 0, second = 0;
  const int64_t etop = top ? gkey_node(top) / 64 - a.c0 : -1;
  const uint64_t lanemask_lt = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
  for (int64_t e0 = 0; e0 < nc; e0 += 64) {
    const int64_t e = e0 + lane;
    const uint2 loc = e < nc ? srow[e] : make_uint2(0u, 0u);
    second = umax64(second, local_gkey(e == etop ? loc.y : loc.x, a.c0 + e));
    const uint32_t h = loc.x >> 6;
    const bool is_gt = h > t;
    const bool is_eq = (h == t) && h != 0;
    const uint64_t beq = __ballot(is_eq);
    const int32_t eq_rank = eq_taken + __popcll(beq & lanemask_lt);
    const bool take_eq = is_eq && eq_rank < need_eq;
    const bool take = is_gt || take_eq;
    const uint64_t btake = __ballot(take);
    if (take) {
      const int32_t pos = base + __popcll(btake & lanemask_lt);
      a.cand_chunk[p * K + pos] = (uint32_t)(a.c0 + e);
      a.cand_t[p * K + pos] = loc;
      if (take_eq && eq_rank == need_eq - 1) bound = local_gkey(loc.x, a.c0 + e);
    }
    base += __popcll(btake);
    eq_taken += __popcll(beq);
  }
  bound = wave_max_u64(bound);  // only one lane holds a non-zero bound
  second = wave_max_u64(second);
  if (lane == 0) {
    a.cand_count[p] = base;
    a.cand_total[p] = cnt;
    a.cand_bound[p] = exhaustive ? 0ull : bound;
    a.cand_top[p] = top;
    a.cand_second[p] = second;
  }
}


// ------------------------------------------------------------------------------------------
// merge: per-shard candidate lists -> the list a single select over every chunk would produce
// ------------------------------------------------------------------------------------------
//
// Shards own contiguous chunk ranges in shard order, so concatenating the shard lists keeps
// global chunk order.  A shard's list holds every chunk above its own K-th score t_s <= t (the
// global K-th score) and its first equal-score chunks, so the union holds every chunk above t and
// the first need_eq = K - #(h > t) chunks equal to t in global chunk order: the same selection
// rule applied to the union reproduces the single-GPU list, bound and top exactly.

struct MergeArgs {
  const unsigned char* __restrict__ gather;  // [nslots] CandSlot blocks
  const int32_t* __restrict__ cursor;
  uint32_t* cand_chunk;
  uint2* cand_t;
  uint64_t* cand_bound;
  uint64_t* cand_top;
  uint64_t* cand_second;
  int32_t* cand_count;
  int32_t nslots, total_pods, batch, k;
};

__global__ __launch_bounds__(64) void merge_kernel(MergeArgs a) {
  const int lane = threadIdx.x;
  const int32_t cursor = __builtin_amdgcn_readfirstlane(*a.cursor);
  if (cursor >= a.total_pods) return;
  const int32_t np = min(a.batch, a.total_pods - cursor);
  const int32_t p = blockIdx.x;
  if (p >= np) return;
  const int32_t K = a.k;
  const CandSlot L = cand_slot_layout(K);
  int32_t total = 0;
  uint64_t top = 0;
  for (int32_t s = 0; s < a.nslots; ++s) {
    const unsigned char* b = a.gather + (size_t)s * L.bytes;
    total += reinterpret_cast<const int32_t*>(b + L.total)[p];
    top = umax64(top, reinterpret_cast<const uint64_t*>(b + L.top)[p]);
  }
  // the union, in shard order, walked 64 entries at a time
  auto entry = [&](int32_t s, int32_t i, uint32_t& chunk, uint2& t) {
    const unsigned char* b = a.gather + (size_t)s * L.bytes;
    chunk = reinterpret_cast<const uint32_t*>(b + L.chunk)[p * K + i];
    t = reinterpret_cast<const uint2*>(b + L.t)[p * K + i];
  };
  uint32_t t_thr = 1;
  int32_t need_eq = 0x7fffffff;
  const bool exhaustive = total <= K;
  if (!exhaustive) {
    uint32_t hmax = 0;
    for (int32_t s = 0; s < a.nslots; ++s) {
      const int32_t cnt = reinterpret_cast<const int32_t*>(a.gather + (size_t)s * L.bytes + L.count)[p];
      for (int32_t i = lane; i < cnt; i += 64) {
        uint32_t c;
        uint2 t;
        entry(s, i, c, t);
        hmax = umax32(hmax, t.x >> 6);
      }
    }
    hmax = wave_max_u32(hmax);
    auto count_ge = [&](uint32_t x, bool strict) {
      int32_t n = 0;
      for (int32_t s = 0; s < a.nslots; ++s) {
        const int32_t cnt = reinterpret_cast<const int32_t*>(a.gather + (size_t)s * L.bytes + L.count)[p];
        for (int32_t i = lane; i < cnt; i += 64) {
          uint32_t c;
          uint2 t;
          entry(s, i, c, t);
          const uint32_t h = t.x >> 6;
          n += strict ? (h > x) : (h >= x);
        }
      }
      return wave_sum_i32(n);
    };
    uint32_t lo = 1, hi = hmax;  // largest t with count(h >= t) >= K
    while (lo < hi) {
      const uint32_t mid = lo + (hi - lo + 1) / 2;
      if (count_ge(mid, false) >= K) lo = mid;
      else hi = mid - 1;
    }
    t_thr = lo;
    need_eq = K - count_ge(t_thr, true);
  }
  int32_t base = 0, eq_taken = 0;
  uint64_t bound = 0, second = 0;
  const int64_t ctop = top ? gkey_node(top) / 64 : -1;  // the second-best key over the union (as select_kernel)
  const uint64_t lanemask_lt = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
  for (int32_t s = 0; s < a.nslots; ++s) {
    const int32_t cnt = reinterpret_cast<const int32_t*>(a.gather + (size_t)s * L.bytes + L.count)[p];
    for (int32_t i0 = 0; i0 < cnt; i0 += 64) {
      const int32_t i = i0 + lane;
      uint32_t c = 0;
      uint2 t = make_uint2(0u, 0u);
      if (i < cnt) entry(s, i, c, t);
      if (i < cnt) second = umax64(second, local_gkey((int64_t)c == ctop ? t.y : t.x, c));
      const uint32_t h = t.x >> 6;
      const bool is_gt = h > t_thr;
      const bool is_eq = (h == t_thr) && h != 0;
      const uint64_t beq = __ballot(is_eq);
      const int32_t eq_rank = eq_taken + __popcll(beq & lanemask_lt);
      const bool take_eq = is_eq && eq_rank < need_eq;
      const bool take = is_gt || take_eq;
      const uint64_t btake = __ballot(take);
      if (take) {
        const int32_t pos = base + __popcll(btake & lanemask_lt);
        a.cand_chunk[p * K + pos] = c;
        a.cand_t[p * K + pos] = t;
        if (take_eq && eq_rank == need_eq - 1) bound = local_gkey(t.x, c);
      }
      base += __popcll(btake);
      eq_taken += __popcll(beq);
    }
  }
  bound = wave_max_u64(bound);
  second = wave_max_u64(second);
  if (lane == 0) {
    a.cand_count[p] = base;
    a.cand_bound[p] = exhaustive ? 0ull : bound;
    a.cand_top[p] = top;
    a.cand_second[p] = second;
  }
}

// ------------------------------------------------------------------------------------------
// ElasticQuota RefreshRuntime for the whole tree (group_quota_manager.go:259-326)
// ------------------------------------------------------------------------------------------
//
// One wave per resource dimension.  Per-quota state lives in LDS ([dims][n] int64 x3).  The host
// lays the tree out breadth-first (children of one parent contiguous) with depth levels and
// sibling groups, so the wave can (1) aggregate requests bottom-up a level at a time
// (recursiveUpdateGroupTreeWithDeltaRequest :184-226: ChildRequest = own pods + children's limited
// requests; a non-lending quota asks for at least Min; limited = min(Request, Max) on Max's keys,
// quota_info.go:217-228) and (2) run redistribution / iterationForRedistribution
// (runtime_quota_calculator.go:111-168) for each sibling group top-down, lanes over siblings.
// The float64 share int64(float64(w)*float64(total)/float64(Σw) + 0.5) is computed with IEEE
// double ops in Go's order (-ffp-contract=off).

struct QrtArgs {
  int32_t n, ngroups, nlevels, dim0, ndims;
  uint32_t keys;                  // union of all Max keys (the calculators' resource keys)
  const int32_t* __restrict__ order;      // breadth-first quota order
  const int32_t* __restrict__ level_off;  // [nlevels+1] ranges of `order` by depth (depth 1 first)
  const int32_t* __restrict__ grp_parent; // [ngroups] parent quota of sibling group g (-1 = root)
  const int32_t* __restrict__ grp_off;    // [ngroups+1] ranges of `order` holding group g
  const int32_t* __restrict__ parent;
  const uint8_t* __restrict__ allow;
  const uint32_t* __restrict__ maxmask;
  const int64_t* __restrict__ mx;         // [n][KS_QUOTA_DIMS]
  const int64_t* __restrict__ mn;
  const int64_t* __restrict__ sw;
  const int64_t* __restrict__ guar;
  const int64_t* __restrict__ selfreq;
  const int64_t* __restrict__ total;      // [KS_QUOTA_DIMS]
  int64_t* __restrict__ runtime;          // [n][KS_QUOTA_DIMS]
};

__device__ __forceinline__ int64_t wave_sum_i64(int64_t v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__global__ __launch_bounds__(512) void quota_runtime_kernel(QrtArgs a) {
  extern __shared__ __attribute__((aligned(16))) int64_t qlds[];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int d = a.dim0 + w;
  if (w >= a.ndims || d >= KS_QUOTA_DIMS) return;
  const int32_t n = a.n;
  int64_t* creq = qlds + (size_t)w * 3 * n;  // ChildRequest, then the limited request
  int64_t* rt = creq + n;                    // runtime
  int64_t* lreq = rt + n;                    // limited request
  const bool key = (a.keys >> d) & 1u;
  for (int32_t q = lane; q < n; q += 64) {
    const int64_t s = a.selfreq[(size_t)q * KS_QUOTA_DIMS + d];
    creq[q] = s > 0 ? s : 0;
    rt[q] = 0;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  // (1) requests, deepest level first
  for (int32_t l = a.nlevels - 1; l >= 0; --l) {
    for (int32_t i = a.level_off[l] + lane; i < a.level_off[l + 1]; i += 64) {
      const int32_t q = a.order[i];
      const size_t o = (size_t)q * KS_QUOTA_DIMS + d;
      int64_t req = creq[q];
      if (!a.allow[q] && a.mn[o] > req) req = a.mn[o];
      if (((a.maxmask[q] >> d) & 1u) && req > a.mx[o]) req = a.mx[o];
      lreq[q] = req;
      const int32_t p = a.parent[q];
      if (p >= 0) atomicAdd((unsigned long long*)&creq[p], (unsigned long long)req);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  // (2) runtime, sibling groups in breadth-first order (a parent's runtime precedes its children)
  for (int32_t g = 0; g < a.ngroups && key; ++g) {
    const int32_t p = a.grp_parent[g];
    int64_t tot = p < 0 ? a.total[d] : rt[p];
    const int32_t b0 = a.grp_off[g], b1 = a.grp_off[g + 1];
    int64_t used = 0, tsw = 0;
    for (int32_t i = b0 + lane; i < b1; i += 64) {
      const int32_t c = a.order[i];
      const size_t o = (size_t)c * KS_QUOTA_DIMS + d;
      int64_t m = a.mn[o];
      if (a.guar[o] > m) m = a.guar[o];
      const int64_t r = lreq[c];
      int64_t v;
      if (r > m) {
        v = m;
        tsw += a.sw[o];
        creq[c] = 1;  // reused: "still adjusting"
      } else {
        v = a.allow[c] ? r : m;
        creq[c] = 0;
      }
      rt[c] = v;
      used += v;
    }
    used = wave_sum_i64(used);
    tsw = wave_sum_i64(tsw);
    int64_t part = tot - used;
    if (part > 0) {
      while (tsw > 0) {
        int64_t npart = 0, nsw = 0, nadj = 0;
        for (int32_t i = b0 + lane; i < b1; i += 64) {
          const int32_t c = a.order[i];
          if (!creq[c]) continue;
          const size_t o = (size_t)c * KS_QUOTA_DIMS + d;
          const int64_t wgt = a.sw[o];
          const int64_t delta = (int64_t)((double)wgt * (double)part / (double)tsw + 0.5);
          int64_t v = rt[c] + delta;
          const int64_t r = lreq[c];
          if (v < r) {
            nsw += wgt;
            nadj += 1;
          } else {
            npart += v - r;
            v = r;
            creq[c] = 0;
          }
          rt[c] = v;
        }
        npart = wave_sum_i64(npart);
        nsw = wave_sum_i64(nsw);
        nadj = wave_sum_i64(nadj);
        if (!(npart > 0 && nadj > 0)) break;
        part = npart;
        tsw = nsw;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  for (int32_t q = lane; q < n; q += 64) a.runtime[(size_t)q * KS_QUOTA_DIMS + d] = key ? rt[q] : 0;
}

// DeviceShare NormalizeScore (DefaultNormalizeScore(100), scoring.go:95-97) for the debug path (one block)
__global__ __launch_bounds__(1024) void dev_normalize_debug_kernel(int64_t n, const uint32_t* reasons,
                                                                   const int32_t* draw, int64_t* scores,
                                                                   int64_t* total, int64_t w) {
  __shared__ int32_t s_max;
  if (threadIdx.x == 0) s_max = 0;
  __syncthreads();
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x)
    if (!reasons[i]) atomicMax(&s_max, draw[i]);
  __syncthreads();
  const int64_t mx = s_max;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    if (reasons[i]) continue;
    const int64_t sc = mx == 0 ? draw[i] : 100 * (int64_t)draw[i] / mx;
    scores[i * KS_NUM_SCORE_PLUGINS + KS_SCORE_DEVICESHARE] = sc;
    total[i] += sc * w;
  }
}

// TaintToleration (reverse) / NodeAffinity NormalizeScore = DefaultNormalizeScore(100, reverse) over the feasible
// nodes for the debug path (one block); slot = KS_SCORE_TAINT or KS_SCORE_NODE_AFFINITY
__global__ __launch_bounds__(1024) void stat_normalize_debug_kernel(int64_t n, const uint32_t* reasons,
                                                                    const int32_t* raw, int64_t* scores,
                                                                    int64_t* total, int64_t w, int32_t slot,
                                                                    int32_t reverse) {
  __shared__ int32_t s_max;
  if (threadIdx.x == 0) s_max = 0;
  __syncthreads();
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x)
    if (!reasons[i]) atomicMax(&s_max, raw[i]);
  __syncthreads();
  const int64_t mx = s_max;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    if (reasons[i]) continue;
    int64_t sc;
    if (mx == 0) sc = reverse ? 100 : raw[i];
    else sc = reverse ? 100 - 100 * (int64_t)raw[i] / mx : 100 * (int64_t)raw[i] / mx;
    scores[i * KS_NUM_SCORE_PLUGINS + slot] = sc;
    total[i] += sc * w;
  }
}

// Reservation PreScore preferred node (scoring.go:87-96), Score (:103-122) and DefaultNormalizeScore
// (normalize_score.go:24-52) over the feasible nodes for the debug path (one block).
__global__ __launch_bounds__(1024) void rsv_normalize_debug_kernel(int64_t n, const uint32_t* reasons,
                                                                   const int32_t* raw, const int32_t* hiord,
                                                                   int64_t* scores, int64_t* total, int64_t w) {
  __shared__ unsigned long long s_pref, s_max;
  if (threadIdx.x == 0) {
    s_pref = 0;
    s_max = 0;
  }
  __syncthreads();
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    if (reasons[i]) continue;
    if (hiord[i] > 0)  // larger hiord = smaller order label; ties to the lowest index
      atomicMax(&s_pref, ((unsigned long long)hiord[i] << 32) | (0xFFFFFFFFull - (unsigned long long)i));
  }
  __syncthreads();
  const bool has_pref = s_pref != 0;
  const int64_t pref = has_pref ? (int64_t)(0xFFFFFFFFull - (s_pref & 0xFFFFFFFFull)) : -1;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    if (reasons[i]) continue;
    atomicMax(&s_max, (unsigned long long)(i == pref ? 1000 : raw[i]));
  }
  __syncthreads();
  const int64_t mx = (int64_t)s_max;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    if (reasons[i]) continue;
    const int64_t rs = i == pref ? 1000 : raw[i];
    const int64_t sc = mx == 0 ? rs : 100 * rs / mx;
    scores[i * KS_NUM_SCORE_PLUGINS + KS_SCORE_RESERVATION] = sc;
    total[i] += sc * w;
  }
}

// Base restore of the reservation table (ks_rsv.h): add (sign = +1) or remove (-1) every eligible
// reservation's unmatched replacement (transformer.go:266-307) on the node columns; with classes != 0
// also (re)compute the node's matchable owner-class union.  idx = NULL: nodes [0, count).
// ------------------------------------------------------------------------------------------
// NodeNUMAResource cpusets: the CPU ids of every cpu-bind Reserve, per node in placement order
// ------------------------------------------------------------------------------------------
//
// One thread per node.  The block stages the (pod, node) list through LDS; a thread runs takeCPUs
// (ks_cpuset.h) for each of its node's entries in list order and adds the CPUs to the node's
// allocation (NodeAllocation.addPodAllocation, node_allocation.go:75-100: allocated, exclusive policy).
constexpr int kCpusetStage = 1024;

__global__ __launch_bounds__(256) void cpuset_kernel(DevCpu cpu, const int2* list, const int32_t* count_p,
                                                     const uint32_t* split, const PodRec* pods, CpuSet* out,
                                                     const uint32_t* numa_flags, uint32_t* cores, int32_t default_most,
                                                     int32_t* numa_free, int64_t numa_npad, int64_t n) {
  __shared__ int2 stage[kCpusetStage];
  const int64_t node = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int32_t count = *count_p;
  uint64_t keys[KS_MAX_CPUS];
  bool any = false;
  for (int32_t base = 0; base < count; base += kCpusetStage) {
    const int32_t m = min(kCpusetStage, count - base);
    for (int32_t i = threadIdx.x; i < m; i += blockDim.x) stage[i] = list[base + i];
    __syncthreads();
    for (int32_t i = 0; i < m && node < n; ++i) {
      if (stage[i].y != (int32_t)node) continue;
      const int32_t pod = stage[i].x;
      const int32_t tid = cpu.topo_id[node];
      if (tid < 0) continue;  // unreachable: the Filter rejects nodes without a topology
      const CpuTopo& t = cpu.topo[tid];
      const uint32_t nf = numa_flags[node], label = (nf >> KS_NUMA_CPU_BIND_SHIFT) & 3u;
      // getCPUBindPolicy (util.go:85-103): the pod's required policy, else the node's (required), else the pod's
      // preferred one; a pod that is cpu-bind only through the node's policy has no exclusive policy
      uint32_t cb = pods[pod].cpu_bind;
      if (cb == 0) cb = label | KS_CPU_BIND_REQUIRED | ((uint32_t)(pods[pod].cpu / 1000) << 8);
      else if (label && !(cb & KS_CPU_BIND_REQUIRED)) cb = (cb & ~KS_CPU_BIND_POLICY_MASK) | label | KS_CPU_BIND_REQUIRED;
      const int pol = (int)(cb & KS_CPU_BIND_POLICY_MASK);
      any = true;
      const CpuSet alloc = cpu.allocated[node], xp = cpu.excl_pcpu[node], xn = cpu.excl_numa[node];
      CpuSet avail = cs_andnot(cs_andnot(t.all, alloc), cpu.reserved[node]);
      if (cb & KS_CPU_BIND_REQUIRED) avail = filter_required(t, avail, pol);  // (resource_manager.go:322-330)
      CpuSet exc_cores = cs_zero();
      uint64_t exc_nodes = 0;
      for (int w = 0; w < kCpuW; ++w) {
        for (uint64_t b = xp.w[w]; b; b &= b - 1) cs_add(exc_cores, t.core_of[w * 64 + __builtin_ctzll(b)]);
        for (uint64_t b = xn.w[w]; b; b &= b - 1) exc_nodes |= 1ull << t.node_of[w * 64 + __builtin_ctzll(b)];
      }
      const int32_t excl = (int32_t)((cb >> KS_CPU_EXCL_SHIFT) & 3u);
      const bool most = (nf & KS_NUMA_ALLOC_MOST) ? true : ((nf & KS_NUMA_ALLOC_LEAST) ? false : default_most != 0);
      // allocateCPUSet (resource_manager.go:314-401): with a NUMA allocation one takeCPUs per allocated NUMA node over
      // its available CPUs, each against the allocation before this pod; else one over the whole node
      const uint32_t sp = split[pod];
      CpuSet res = cs_zero();
      for (int k = 0; k < (sp ? kNumaDev : 1); ++k) {
        const int32_t need = sp ? (int32_t)((sp >> (8 * k)) & 0xFFu) : (int32_t)(cb >> 8);
        if (sp && need == 0) continue;
        CpuAcc a;
        a.t = &t;
        a.al = sp ? cs_and(avail, t.node_mask[k]) : avail;
        a.res = cs_zero();
        a.exc_cores = exc_cores;
        a.exc_nodes = exc_nodes;
        a.excl = excl;
        a.most = most;
        a.needed = need;
        if (take_cpus(a, pol, keys)) res = cs_or(res, a.res);  // (count checked)
      }
      cpu.allocated[node] = cs_or(alloc, res);
      if (excl == KS_CPU_EXCL_PCPU_LEVEL) cpu.excl_pcpu[node] = cs_or(xp, res);
      if (excl == KS_CPU_EXCL_NUMA_NODE_LEVEL) cpu.excl_numa[node] = cs_or(xn, res);
      out[pod] = res;
    }
    __syncthreads();
  }
  if (any && node < n) {
    const CpuTopo& t = cpu.topo[cpu.topo_id[node]];
    const CpuSet av = cs_andnot(cs_andnot(t.all, cpu.allocated[node]), cpu.reserved[node]);
    cores[node] = cores_word(t, av, (numa_flags[node] >> KS_NUMA_CPU_BIND_SHIFT) & 3u);
    // the NUMA nodes' words too: the commit kept their CPU counts, the core counts follow the CPU ids chosen here
    if (numa_free)
      for (int k = 0; k < kNumaDev; ++k) numa_free[(int64_t)k * numa_npad + node] = numa_free_word(t, av, k);
  }
}

// CoresWord of every node (idx = NULL) or of idx[0..count): the node's CPU bind label, and its core counts when the
// CPU state is loaded and the node has a topology.
__global__ void cores_kernel(DevCpu cpu, int32_t loaded, const uint32_t* numa_flags, uint32_t* cores, const int32_t* idx,
                             int64_t count) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= count) return;
  const int64_t i = idx ? idx[t] : t;
  const uint32_t label = (numa_flags[i] >> KS_NUMA_CPU_BIND_SHIFT) & 3u;
  const int32_t tid = loaded ? cpu.topo_id[i] : -1;
  if (tid < 0) {
    cores[i] = label << kCoresLabelShift;
    return;
  }
  const CpuTopo& tp = cpu.topo[tid];
  cores[i] = cores_word(tp, cs_andnot(cs_andnot(tp.all, cpu.allocated[i]), cpu.reserved[i]), label);
}

// CPUs of each NUMA node available to cpuset pods (topology CPUs of the node - allocated - reserved) and its core
// counts (numa_free_word), for the NUMA policy path's allocateCPUSet check and a required CPU bind policy's trim;
// NUMA node k = the topology's k-th NUMA id (ids are 0..n-1, ks_load_cpu_state).
__global__ void numa_free_kernel(DevCpu cpu, DevNuma nv, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t tid = cpu.topo_id[i];
  for (int k = 0; k < kNumaDev; ++k) {
    int32_t f = 0;
    if (tid >= 0) {
      const CpuTopo& t = cpu.topo[tid];
      f = numa_free_word(t, cs_andnot(cs_andnot(t.all, cpu.allocated[i]), cpu.reserved[i]), k);
    }
    nv.free[(int64_t)k * nv.npad + i] = f;
  }
}

__global__ void rsv_base_kernel(DevNodes d, DevRsv rv, const int32_t* idx, int64_t count, int64_t sign, int32_t classes) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= count) return;
  const int64_t n = idx ? idx[t] : t;
  const int64_t b = rv.beg[n], e = rv.beg[n + 1];
  int64_t dq[kRsvDims] = {0, 0, 0, 0, 0, 0, 0}, dz[2] = {0, 0};
  uint64_t cls = 0;
  for (int64_t i = b; i < e; ++i) {
    const uint32_t meta = rv.meta[i];
    const int32_t a = rv.assigned[i];
    const bool ao = (meta & KS_RSV_ALLOCATE_ONCE) != 0;
    if (!(ao && a > 0) && !(meta & KS_RSV_UNSCHEDULABLE)) cls |= rv.cls[i];
    if (ao || a <= 0) continue;  // not eligible, or no assigned pods: not restored as unmatched
    int64_t rem[kRsvDims];
    bool nzr = false;
    for (int dd = 0; dd < kRsvDims; ++dd) {
      const int64_t v = rv.alloc[dd * rv.nr + i] - rv.allocd[dd * rv.nr + i];
      rem[dd] = v > 0 ? v : 0;
      nzr |= rem[dd] != 0;
    }
    for (int dd = 0; dd < kRsvDims; ++dd) dq[dd] += (nzr ? rem[dd] : 0) - rv.alloc[dd * rv.nr + i];
    const uint32_t keys = rsv_keys(meta);
    dz[0] += (nzr ? ((keys & 1u) ? rem[0] : kDefaultMilliCPU) : 0) - rv.rnz[i];
    dz[1] += (nzr ? ((keys & 2u) ? rem[1] : kDefaultMemory) : 0) - rv.rnz[rv.nr + i];
  }
  d.req_cpu[n] += sign * dq[0];
  d.req_mem[n] += sign * dq[1];
  d.req_eph[n] += sign * dq[2];
  for (int k = 0; k < KS_MAX_SCALARS; ++k) d.req_sc[k][n] += sign * dq[3 + k];
  d.nz_cpu[n] += sign * dz[0];
  d.nz_mem[n] += sign * dz[1];
  if (classes) d.rsv_cls[n] = cls;
}

// scatter m staged rows into the node columns (informer deltas)
__global__ void scatter_rows_kernel(void* const* dst_cols, const void* const* src_cols, const int32_t* widths,
                                    int32_t ncols, const int32_t* idx, int64_t m) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const int64_t to = idx[i];
  for (int32_t k = 0; k < ncols; ++k) {
    if (widths[k] == 8)
      ((int64_t*)dst_cols[k])[to] = ((const int64_t*)src_cols[k])[i];
    else
      ((int32_t*)dst_cols[k])[to] = ((const int32_t*)src_cols[k])[i];
  }
}

// ==========================================================================================
// host side
// ==========================================================================================

namespace {

thread_local std::string g_create_error;

struct Col {
  void** dev;       // address of the DevNodes pointer field
  int32_t width;    // bytes per element
  bool mutable_;    // changed by commits (checkpointed)
};

}  // namespace

constexpr int kPipeEvents = 4;  // ring of cross-stream events of the pipelined passes

struct PodStage {
  void* blob = nullptr;
  int32_t cap = 0;
  PodRec* recs = nullptr;       // [cap] built by prep_pods_kernel
  PodStat* stat = nullptr;      // [cap] TaintToleration / NodeAffinity inputs (host-built at staging)
  ks_result* results = nullptr; // [cap]
  DevPodCols cols{};            // the caller's columns in HBM
  DevPodQuota pq{};             // quota request columns (read by the commit kernel)
  std::vector<PodStat> h_stat;  // host staging of stat (kept until the async copy has run: the stream syncs
  std::vector<uint8_t> h_dyn;   // before the next stage_cols)
  // small batches (ks_eval_pod, ks_assume, ks_preempt, short queues): the column region [cols.cpu, end) packed on the
  // host in its device layout and sent with one copy instead of ~35 (each a HIP API round trip)
  void* h_pack = nullptr;       // pinned, kPackPods pods
  size_t pack_bytes = 0;
  size_t col8 = 0, col4 = 0;    // device column strides of this stage
  // PodTopologySpread / InterPodAffinity (ks_topo.h): per pod its TopoRec, and the stage's query-term and property
  // lists the records point into; ndyn = topology pods of the stage
  TopoRec* topo = nullptr;
  uint64_t* topo_terms = nullptr;
  int32_t* topo_props = nullptr;
  int32_t topo_cap = 0;
  int64_t topo_tcap = 0, topo_pcap = 0;
  int32_t ndyn = 0;
  std::vector<TopoRec> h_topo;
};
constexpr int32_t kPackPods = 64;

// Test transport for nranks > 1 without RCCL (ks_shard_init_loopback): the ranks are contexts of one process, each
// driven by its own host thread.  An exchange is two host barriers and device copies: every rank records an event
// behind its block, waits at the first barrier until every rank has, then pulls the peers' blocks into its own buffer
// behind their events and records a second event; past the second barrier it waits for the peers' second events, so
// no rank overwrites its block (the next pass's select) before every peer has copied it.  Each wait is enqueued after
// the record it waits on (the barriers order them), so the streams cannot deadlock.
struct LoopGroup {
  int32_t n = 0;
  std::vector<ks_ctx*> ranks;  // rank r's context (nullptr once destroyed)
  std::mutex mu;
  std::condition_variable cv;
  int32_t arrived = 0;
  int64_t gen = 0;
  bool broken = false;  // a rank failed or timed out: every later barrier fails at once
  int32_t refs = 0;
};

struct ks_ctx {
  ks_config cfg{};
  Cfg kc{};
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  // nodes
  int64_t n = 0, npad = 0, nchunks = 0;
  int nsc = 0;
  DevNodes d{};
  std::vector<Col> cols;
  void* node_blob = nullptr;
  void* ckpt_blob = nullptr;
  size_t mut_bytes = 0;
  // quotas
  DevQuotas q{};
  void* quota_blob = nullptr;
  int64_t* quota_used_ckpt = nullptr;
  int64_t* quota_npused_ckpt = nullptr;
  // pods
  int32_t np = 0;
  PodStage st{};   // staged pods of ks_stage_pods / ks_schedule
  PodStage est{};  // single-pod evaluation (ks_eval_pod)
  PodStage ast{};  // per-pod framework mode (ks_assume / ks_unreserve)
  int64_t* numa_alloc = nullptr;  // [cpuset_cap][2][kNumaDev] NUMA-policy allocation per pod of the last call
  void* evbuf = nullptr;          // ks_eval_pod scratch, kept across calls
  size_t evbuf_bytes = 0;
  void* ures = nullptr;           // ks_unreserve scratch: node index, the pod's cpuset and NUMA allocation
  void* rdscratch = nullptr;      // ks_read_nodes: the NodeInfo view of the reservation-restored columns
  std::vector<int32_t> h_rsv_gi;  // caller reservation row -> CSR position
  // pass scratch
  uint2* sweep_out = nullptr;
  uint32_t* cand_chunk = nullptr;
  uint2* cand_t = nullptr;
  uint64_t* cand_bound = nullptr;
  uint64_t* cand_top = nullptr;
  uint64_t* cand_second = nullptr;
  PreRsv* pre_rsv = nullptr;       // [kMaxBatch][kPreRsvM] reserve_pre_kernel's records (NUMA / device variants)
  int32_t* cand_total = nullptr;
  // node sharding: shard s = rank * vshards + v owns chunks [s*nchunks/S, (s+1)*nchunks/S)
  int32_t nranks = 1, rank = 0, vshards = 1;
  ncclComm_t comm = nullptr;
  struct LoopGroup* loop = nullptr;  // test transport (ks_shard_init_loopback) in place of comm
  hipEvent_t lev[2][2] = {};         // loopback: [parity][0 = block ready, 1 = peers' blocks pulled]
  int64_t loop_seq = 0;              // loopback exchanges so far (every rank makes the same sequence)
  unsigned long long* loop_scratch = nullptr;  // loopback all-reduce: the peers' blocks [nranks][kNormRows * kMaxBatch]
  unsigned char* gather = nullptr;  // [nranks * vshards] CandSlot blocks
  size_t gather_bytes = 0;
  int32_t* cand_count = nullptr;
  int32_t* cursor = nullptr;
  unsigned long long* counters = nullptr;
  int32_t batch = 64, k = 32;
  RowCol* rowcols = nullptr;  // [RF_N] device column of each slot-row field
  DevNodes* dnodes = nullptr;  // device copy of d (the hot kernels read column pointers from it)
  // reservations (ks_rsv.h)
  void* rsv_blob = nullptr;
  DevRsv rv{};               // host copy of the device table
  DevRsv* drv = nullptr;     // device copy (kernels read it through a pointer)
  bool rsv_based = false;    // node columns hold the base restore of rv
  int64_t* rsv_allocd_ckpt = nullptr;
  int32_t* rsv_assigned_ckpt = nullptr;
  int32_t rsv_ndist = 0;     // distinct order labels
  int32_t rsv_nrows = 0;     // caller rows (deleted ones included)
  int32_t rsv_live = 0;      // rows of the device table (the caller rows not deleted)
  std::vector<int32_t> rsv_perm;  // CSR position -> caller row
  // host mirror of the caller rows, for ks_add_reservations / ks_delete_reservations (allocated / assigned are
  // refreshed from the device before each change)
  struct RsvMirror {
    std::vector<int32_t> node, assigned;
    std::vector<uint64_t> cls;
    std::vector<uint32_t> flags, policy, key_mask;
    std::vector<int64_t> order, rnz_cpu, rnz_mem;
    std::vector<int64_t> alloc[kRsvDims], allocd[kRsvDims];
    std::vector<int64_t> dal, dald;  // [row * KS_DEV_WORDS + w]
    std::vector<uint8_t> live;
  } rmir;
  // DeviceShare GPUs (ks_dev.h)
  void* dev_blob = nullptr;
  DevDev dv{};
  DevDev* ddv = nullptr;
  bool dev_loaded = false;
  int64_t* dev_used_ckpt = nullptr;
  unsigned long long* dev_M = nullptr;  // [3][64] per pass: normalization maxima (ks_pass.h SweepArgs.dev_M)
  uint64_t soft_union = 0;  // TaintToleration: OR of every node's PreferNoSchedule taint bits (kPodNormDyn at staging)
  unsigned long long* dcache = nullptr;  // [64][npad] DeviceShare phase-0 results (SweepArgs.dcache)
  int64_t dcache_words = 0;
  // NodeNUMAResource cpusets (ks_cpuset.h)
  void* cpu_blob = nullptr;
  DevCpu cpu{};
  bool cpu_loaded = false;
  std::vector<int32_t> cpu_cpc;          // CPUsPerCore of each loaded topology
  CpuSet* cpu_ckpt = nullptr;            // allocated / excl_pcpu / excl_numa at ks_checkpoint
  int2* cpuset_list = nullptr;           // [pod_cap] (pod, node) of every cpu-bind Reserve
  int32_t* cpuset_n = nullptr;
  CpuSet* cpuset_out = nullptr;          // [pod_cap] CPUs allocated per pod of the last schedule
  int32_t cpuset_cap = 0;
  // NUMA topology policies (ks_numa.h)
  void* numa_blob = nullptr;
  DevNuma nv{};
  DevNuma* dnv = nullptr;    // device copy (always allocated: kernels take its address)
  char* numa_ckpt = nullptr;       // checkpoint copy of the mutable NUMA block (numa_mut_bytes)
  int64_t numa_policy_nodes = 0;  // nodes with a NUMA topology policy
  bool cpu_bind_labels = false;   // a node CPU bind policy was loaded (sticky)
  bool cpu_bind_required = false;    // the current operation's pods include a required CPU bind policy
  bool val_bind_required = false;    // ... set by the last successful validate_pods
  bool staged_bind_required = false; // ... of the staged batch (ks_stage_pods)
  bool cpusets_clobbered = false;    // ks_assume reused the batch's cpuset / NUMA buffers since the last schedule
  // nodes with device pods placed by ks_assume and not yet ks_unreserve'd: their Unreserve re-derives the
  // per-instance request from the node's device totals, so ks_update_devices must not change those meanwhile
  std::vector<int32_t> h_dev_assumed, h_dev_assumed_ckpt;
  std::vector<int8_t> h_numa_k;    // per node: NUMA node count of a policy node (0 = no policy / none)
  std::vector<uint16_t> h_dev_ids; // per node: NUMA ids of the device topology (DeviceShare hints)
  std::vector<uint8_t> h_pol;      // per node: a NUMA topology policy (numa_flags)
  std::vector<uint8_t> h_dev_held; // per node: a reservation on it holds devices (kDevRsvHeld)
  bool dev_held_any = false;       // ... on some node (the pass kernels' FEAT bit 16)
  int64_t* rsv_dald_ckpt = nullptr;  // checkpoint of the reservations' device allocated
  std::vector<int8_t> h_cpu_nn;    // per node: NUMA nodes of its CPU topology (0 = none, -1 = ids not 0..n-1)
  std::vector<CpuTopo> h_topos;    // the loaded CPU topologies (ks_update_cpu_state refers to them)
  std::vector<int8_t> h_topo_dense;
  std::vector<int32_t> h_rsv_node; // CSR position -> node
  void* dscratch = nullptr;        // delta uploads (ks_update_*): indices + row words
  size_t dscratch_bytes = 0;
  uint32_t* cpuset_split = nullptr;  // [cpuset_cap] per pod (CommitArgs.cpuset_split)
  // pipelined passes: sweep + select on sstream while the commit runs on stream
  hipStream_t sstream = nullptr;   // shared by the process's contexts on this device (ensure_pipe), never destroyed
  hipStream_t cstream = nullptr;   // the pipelined commits: the CU the sweep stream leaves out (or `stream`)
  int32_t* pipe = nullptr;          // [0..1] speculative first pod per pass parity, [4..68] commit carry list
  unsigned long long* pipe_top = nullptr;  // patched passes: [2][64] each pod's top after the list re-evaluation
  hipEvent_t pev_sel[kPipeEvents] = {};
  hipEvent_t pev_com[kPipeEvents] = {};
  int64_t pipe_k = 0;               // pass index within the current ks_schedule* call
  int32_t pipe_mode = -1;           // ks_set_pipeline (-1: KS_PIPE, default automatic)
  // preemption (ks_load_node_pods / ks_preempt, ks_preempt.h)
  void* npod_blob = nullptr;       // the node-pod table (positions sorted per node) + per-call scratch
  DevNodePods npt{};
  int32_t npod_slots = 0;          // positions per lane of the dry run (max pods on a node / 64, rounded up)
  PreemptCand* pre_cand = nullptr; // [n]
  int32_t* pre_vrank = nullptr;    // [m]
  uint8_t* pre_status = nullptr;   // [n]
  PreemptOut* pre_out = nullptr;
  int32_t* pre_victims = nullptr;  // [kPreemptMaxPods]
  // PodTopologySpread / InterPodAffinity (ks_topo.h): node columns in the node blob (counters mutable, zone
  // read-only), the normalizing-weight table, the topology step's scratch and one-candidate set
  int32_t topo_nkeys = 0, topo_ndom = 1, topo_nprops = 0;
  std::vector<int32_t*> topo_dom_v;    // [nkeys] column bases (contiguous, stride npad): key k + 1's value index
  std::vector<int32_t*> topo_count_v;  // [nprops] (contiguous, stride npad, mutable): pods with property p
  int32_t* topo_dom = nullptr;         // topo_dom_v[0]
  int32_t* topo_count = nullptr;       // topo_count_v[0]
  long long* topo_zsum = nullptr;      // the step's per-domain scratch (ks_topo.h DevTopo)
  uint32_t *topo_zpres = nullptr, *topo_zsize = nullptr;
  void* topo_blob = nullptr;
  double* topo_lw = nullptr;
  int32_t topo_nlw = 0;
  TopoScratch* topo_scr = nullptr;
  long long *topo_sraw = nullptr, *topo_iraw = nullptr;  // [npad] per-node raw scores of the step
  int32_t topo_k = 1;  // topology steps per regular pass (queues of mostly topology pods run several in a row)
  uint32_t* topo_cchunk = nullptr;
  uint2* topo_ct = nullptr;
  int32_t* topo_ccount = nullptr;
  uint64_t *topo_cbound = nullptr, *topo_ctop = nullptr, *topo_csecond = nullptr;
  // stats
  ks_stats stats{};
  std::vector<hipEvent_t> ev_pool;
};

#define KS_FAIL(ctx, code, ...)                                        \
  do {                                                                 \
    char buf_[512];                                                    \
    snprintf(buf_, sizeof(buf_), __VA_ARGS__);                         \
    (ctx)->err = buf_;                                                 \
    return (code);                                                     \
  } while (0)

#define HIPCHK(ctx, expr)                                                                    \
  do {                                                                                       \
    hipError_t e_ = (expr);                                                                  \
    if (e_ != hipSuccess) KS_FAIL(ctx, KS_EHIP, "%s failed: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

static int dev_alloc(ks_ctx* ctx, void** p, size_t bytes) {
  if (bytes == 0) bytes = 16;
  hipError_t e = hipMalloc(p, bytes);
  if (e != hipSuccess) KS_FAIL(ctx, KS_ENOMEM, "hipMalloc(%zu) failed: %s", bytes, hipGetErrorString(e));
  return KS_OK;
}

static void dev_free(void*& p) {
  if (p) (void)hipFree(p);
  p = nullptr;
}

// Leave the loopback group (ks_shard_init_loopback): the group is freed with its last member.
static void loop_leave(ks_ctx* ctx) {
  if (ctx->loop) {
    LoopGroup* g = ctx->loop;
    bool last = false;
    {
      std::lock_guard<std::mutex> lk(g->mu);
      if ((size_t)ctx->rank < g->ranks.size() && g->ranks[(size_t)ctx->rank] == ctx) g->ranks[(size_t)ctx->rank] = nullptr;
      g->broken = true;  // a group with a missing rank cannot exchange any more
      g->cv.notify_all();
      last = --g->refs == 0;
    }
    if (last) delete g;
    ctx->loop = nullptr;
  }
  for (auto& pr : ctx->lev)
    for (hipEvent_t& e : pr) {
      if (e) (void)hipEventDestroy(e);
      e = nullptr;
    }
  void* p = ctx->loop_scratch;
  dev_free(p);
  ctx->loop_scratch = nullptr;
}

static Cfg make_cfg(const ks_config& c, int nsc) {
  Cfg k{};
  k.cpuset = c.numa.enable ? 1 : 0;  // cpu-bind pods: topology check, amplified request, Reserve counts
  k.fit_filter = c.fit.enable_filter;
  k.fit_score = c.fit.enable_score;
  k.fit_most = c.fit.strategy == KS_MOST_ALLOCATED;
  k.nsc = nsc;
  k.fw_cpu = (int32_t)c.fit.weight_cpu;
  k.fw_mem = (int32_t)c.fit.weight_memory;
  k.fw_eph = (int32_t)c.fit.weight_ephemeral;
  for (int i = 0; i < KS_MAX_SCALARS; ++i) k.fw_sc[i] = (int32_t)c.fit.weight_scalar[i];
  k.fit_pw = (int32_t)c.fit.plugin_weight;
  k.la_filter = c.loadaware.enable_filter;
  k.la_score = c.loadaware.enable_score;
  k.la_filter_expired = c.loadaware.filter_expired_node_metrics;
  k.la_prod_usage = c.loadaware.score_according_prod_usage;
  k.lw_cpu = (int32_t)c.loadaware.weight_cpu;
  k.lw_mem = (int32_t)c.loadaware.weight_memory;
  k.la_pw = (int32_t)c.loadaware.plugin_weight;
  k.quota_enable = c.quota.enable;
  k.quota_parent = c.quota.enable_check_parent_quota;
  // LeastAllocated Fit + LoadAware: a commit only raises requested/estimated usage, so a node's
  // key can only drop and its Filter can only start failing.
  k.monotone = c.fit.strategy == KS_LEAST_ALLOCATED || !c.fit.enable_score;
  k.numa = c.numa.enable ? 1 : 0;
  k.numa_most = c.numa.strategy == KS_MOST_ALLOCATED;
  k.numa_sc_most = c.numa.numa_scoring_strategy == KS_MOST_ALLOCATED;  // hint scores (NUMAScoringStrategy)
  k.nw_cpu = (int32_t)c.numa.weight_cpu;
  k.nw_mem = (int32_t)c.numa.weight_memory;
  k.numa_pw = c.numa.enable ? (int32_t)c.numa.plugin_weight : 0;
  if (k.numa && k.numa_most) k.monotone = 0;
  k.dev = c.deviceshare.enable ? 1 : 0;
  k.dev_most = c.deviceshare.strategy == KS_MOST_ALLOCATED;
  k.dw_core = (int32_t)c.deviceshare.weight_gpu_core;
  k.dw_mem = (int32_t)c.deviceshare.weight_gpu_memory;
  k.dw_ratio = (int32_t)c.deviceshare.weight_gpu_memory_ratio;
  k.dw_rdma = (int32_t)c.deviceshare.weight_rdma;
  k.dev_pw = c.deviceshare.enable ? (int32_t)c.deviceshare.plugin_weight : 0;
  k.monotone_nd = k.monotone;
  if (k.dev) k.monotone = 0;  // a commit changes the pod's DeviceShare normalization max
  k.rsv = c.reservation.enable ? 1 : 0;
  // upstream NodeResourcesBalancedAllocation: a commit can move a node's fractions closer together, i.e. raise its
  // score, so keys are not monotone with it
  k.bal = c.balanced.enable ? (c.balanced.resources & (KS_BAL_CPU | KS_BAL_MEMORY)) : 0;
  k.bal_pw = c.balanced.enable ? (int32_t)c.balanced.plugin_weight : 0;
  if (k.bal) {
    k.monotone = 0;
    k.monotone_nd = 0;
  }
  // upstream TaintToleration / NodeAffinity: static per (pod, node), but normalized over the feasible nodes, so a
  // commit that makes the max-holding node infeasible changes the pod's scores elsewhere (monotone_nd covers the
  // pods whose raw scores are 0 everywhere, kPodNormDyn)
  k.taint = c.taint.enable_filter ? 1 : 0;
  k.taint |= c.taint.enable_score ? 2 : 0;
  k.taint_pw = c.taint.enable_score ? (int32_t)c.taint.plugin_weight : 0;
  k.aff = c.affinity.enable_filter ? 1 : 0;
  k.aff |= c.affinity.enable_score ? 2 : 0;
  k.aff_pw = c.affinity.enable_score ? (int32_t)c.affinity.plugin_weight : 0;
  k.ports = c.nodeports.enable_filter ? 1 : 0;
  k.stat = (k.taint | k.aff | k.ports) ? 1 : 0;
  if ((k.taint | k.aff) & 2) k.monotone = 0;
  k.rsv_F = (int32_t)(100 * ((c.fit.enable_score ? c.fit.plugin_weight : 0) +
                             (c.loadaware.enable_score ? c.loadaware.plugin_weight : 0) + k.numa_pw + k.dev_pw +
                             k.bal_pw + k.taint_pw + k.aff_pw) + 1);
  // a pod that matches no reservation sees every node through the base restore only (ks_rsv.h): a commit there lowers
  // the node's key unless it lowers the restored Requested (a reservation whose remainder shrank to zero), which the
  // commit kernel detects per pass
  k.monotone_rsv = (k.rsv && !k.dev && !k.stat && !k.numa && !k.bal) ? k.monotone_nd : 0;
  // a commit into a reservation can raise that node's Reservation score for later pods
  if (k.rsv) k.monotone = 0;
  if (k.rsv) k.monotone_nd = 0;
  return k;
}

// C-ABI entry points: declared extern "C" in include/koordgpu.h, so these definitions have C linkage.

const char* ks_last_error(const ks_ctx* ctx) { return ctx ? ctx->err.c_str() : g_create_error.c_str(); }

int ks_abi_layout(int64_t* out, int32_t n) {
  const int64_t v[KS_ABI_LAYOUT_WORDS] = {
      KS_ABI_VERSION, KS_NUM_SCORE_PLUGINS, sizeof(ks_config), sizeof(ks_node_cols), sizeof(ks_pod_cols),
      sizeof(ks_quota_cols), sizeof(ks_quota_tree), sizeof(ks_reservation_cols), sizeof(ks_device_cols),
      sizeof(ks_cpu_topology), sizeof(ks_cpu_state_cols), sizeof(ks_numa_node_cols), sizeof(ks_result),
      sizeof(ks_node_state), sizeof(ks_stats), sizeof(ks_node_pod_cols), sizeof(ks_preempt_result)};
  for (int32_t i = 0; out && i < n && i < KS_ABI_LAYOUT_WORDS; ++i) out[i] = v[i];
  return KS_ABI_LAYOUT_WORDS;
}

int ks_create(const ks_config* cfg, ks_ctx** out) {
  if (out) *out = nullptr;
  if (!cfg || !out) {
    g_create_error = "ks_create: null argument";
    return KS_EINVAL;
  }
  if (cfg->abi_version != KS_ABI_VERSION) {
    g_create_error = "ks_create: ABI version mismatch";
    return KS_EINVAL;
  }
  const ks_loadaware_args& la = cfg->loadaware;
  if (la.weight_cpu < 0 || la.weight_cpu > 100 || la.weight_memory < 0 || la.weight_memory > 100 ||
      (la.enable_score && la.weight_cpu + la.weight_memory == 0)) {
    g_create_error = "ks_create: LoadAware resource weights must be in [1,100] (validation_pluginargs.go:60-70)";
    return KS_EINVAL;
  }
  {
    // upstream ValidateNodeResourcesFitArgs: every listed resource weight in [1, 100] (0 = not listed)
    const ks_fit_args& fa = cfg->fit;
    bool ok = fa.weight_cpu >= 0 && fa.weight_cpu <= 100 && fa.weight_memory >= 0 && fa.weight_memory <= 100 &&
              fa.weight_ephemeral >= 0 && fa.weight_ephemeral <= 100;
    for (int k = 0; k < KS_MAX_SCALARS; ++k) ok = ok && fa.weight_scalar[k] >= 0 && fa.weight_scalar[k] <= 100;
    if (!ok) {
      g_create_error = "ks_create: NodeResourcesFit resource weights must be in [1,100] (upstream ValidateNodeResourcesFitArgs)";
      return KS_EINVAL;
    }
  }
  const int64_t max_total = 100 * (std::max<int64_t>(cfg->fit.plugin_weight, 0) +
                                   std::max<int64_t>(cfg->loadaware.plugin_weight, 0));
  if (cfg->fit.plugin_weight < 0 || cfg->loadaware.plugin_weight < 0 || max_total >= (1 << 25)) {
    g_create_error = "ks_create: plugin weights out of supported range";
    return KS_EINVAL;
  }
  if (cfg->numa.enable) {
    const ks_numa_args& na = cfg->numa;
    if (na.weight_cpu < 0 || na.weight_cpu > 100 || na.weight_memory < 0 || na.weight_memory > 100 ||
        na.plugin_weight < 0 || na.plugin_weight > 1000 || (na.strategy != KS_LEAST_ALLOCATED && na.strategy != KS_MOST_ALLOCATED)) {
      g_create_error = "ks_create: NodeNUMAResource args out of range";
      return KS_EINVAL;
    }
  }
  if (cfg->deviceshare.enable) {
    const ks_deviceshare_args& da = cfg->deviceshare;
    if (da.weight_gpu_core < 0 || da.weight_gpu_core > 100 || da.weight_gpu_memory < 0 || da.weight_gpu_memory > 100 ||
        da.weight_gpu_memory_ratio < 0 || da.weight_gpu_memory_ratio > 100 || da.plugin_weight < 0 ||
        da.weight_rdma < 0 || da.weight_rdma > 100 ||
        da.plugin_weight > 1000 || (da.strategy != KS_LEAST_ALLOCATED && da.strategy != KS_MOST_ALLOCATED)) {
      g_create_error = "ks_create: DeviceShare args out of range";
      return KS_EINVAL;
    }
  }
  if (cfg->balanced.enable) {
    const ks_balanced_args& ba = cfg->balanced;
    if (ba.plugin_weight < 0 || ba.plugin_weight > 1000) {
      g_create_error = "ks_create: NodeResourcesBalancedAllocation plugin weight out of range";
      return KS_EINVAL;
    }
    if (ba.resources == 0 || (ba.resources & ~(KS_BAL_CPU | KS_BAL_MEMORY)) != 0) {
      g_create_error = "ks_create: NodeResourcesBalancedAllocation resources other than cpu / memory are not supported";
      return KS_EUNSUPPORTED;
    }
  }
  for (const ks_static_plugin_args* sp : {&cfg->taint, &cfg->affinity}) {
    if (sp->enable_score && (sp->plugin_weight < 0 || sp->plugin_weight > 1000)) {
      g_create_error = "ks_create: TaintToleration / NodeAffinity plugin weight out of range";
      return KS_EINVAL;
    }
  }
  if (cfg->reservation.enable) {
    const int64_t fitla = 100 * ((cfg->fit.enable_score ? cfg->fit.plugin_weight : 0) +
                                 (cfg->loadaware.enable_score ? cfg->loadaware.plugin_weight : 0) +
                                 (cfg->numa.enable ? cfg->numa.plugin_weight : 0) +
                                 (cfg->deviceshare.enable ? cfg->deviceshare.plugin_weight : 0) +
                                 (cfg->balanced.enable ? cfg->balanced.plugin_weight : 0) +
                                 (cfg->taint.enable_score ? cfg->taint.plugin_weight : 0) +
                                 (cfg->affinity.enable_score ? cfg->affinity.plugin_weight : 0));
    if (cfg->reservation.plugin_weight <= fitla || cfg->reservation.plugin_weight > ((int64_t)1 << 40) ||
        (fitla + 1) * (kRsvOrderBase + 1) >= (1 << 26)) {
      g_create_error = "ks_create: Reservation plugin weight must exceed 100 x (Fit + LoadAware weights) (ks_rsv.h ranking)";
      return KS_EUNSUPPORTED;
    }
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    g_create_error = "ks_create: no HIP device available";
    return KS_EHIP;
  }
  if (cfg->device < 0 || cfg->device >= ndev) {
    g_create_error = "ks_create: device ordinal out of range";
    return KS_EINVAL;
  }
  ks_ctx* ctx = new ks_ctx();
  ctx->cfg = *cfg;
  ctx->device = cfg->device;
  ctx->batch = cfg->batch_pods > 0 ? std::min(cfg->batch_pods, kMaxBatch) : 64;
  ctx->k = cfg->candidates > 0 ? std::min(cfg->candidates, kMaxCand) : 32;
  if (hipSetDevice(ctx->device) != hipSuccess || hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
    g_create_error = "ks_create: cannot create HIP stream";
    delete ctx;
    return KS_EHIP;
  }
  void* p = nullptr;
  // two sets of candidate lists (CandSet): pipelined passes select pass k+1 while pass k commits
  size_t cand_bytes = (size_t)2 * kMaxBatch * kMaxCand;
  if (dev_alloc(ctx, &p, cand_bytes * 4) != KS_OK) goto fail;
  ctx->cand_chunk = (uint32_t*)p;
  if (dev_alloc(ctx, &p, cand_bytes * 8) != KS_OK) goto fail;
  ctx->cand_t = (uint2*)p;
  if (dev_alloc(ctx, &p, 2 * kMaxBatch * 8) != KS_OK) goto fail;
  ctx->cand_bound = (uint64_t*)p;
  if (dev_alloc(ctx, &p, 2 * kMaxBatch * 8) != KS_OK) goto fail;
  ctx->cand_top = (uint64_t*)p;
  if (dev_alloc(ctx, &p, 2 * kMaxBatch * 8) != KS_OK) goto fail;
  ctx->cand_second = (uint64_t*)p;
  if (dev_alloc(ctx, &p, (size_t)kMaxBatch * kPreRsvM * sizeof(PreRsv)) != KS_OK) goto fail;
  ctx->pre_rsv = (PreRsv*)p;
  if (dev_alloc(ctx, &p, 2 * kMaxBatch * 4) != KS_OK) goto fail;
  ctx->cand_total = (int32_t*)p;
  if (dev_alloc(ctx, &p, 2 * kMaxBatch * 4) != KS_OK) goto fail;
  ctx->cand_count = (int32_t*)p;
  if (dev_alloc(ctx, &p, 64) != KS_OK) goto fail;
  ctx->cursor = (int32_t*)p;
  if (dev_alloc(ctx, &p, 256) != KS_OK) goto fail;
  ctx->counters = (unsigned long long*)p;
  if (dev_alloc(ctx, &p, kNormRows * kMaxBatch * 8) != KS_OK) goto fail;
  ctx->dev_M = (unsigned long long*)p;
  // empty candidate lists until a select writes them: a kernel that reads a list the pass did not write sees no node
  // rather than whatever the allocation held.  KS_TEST_POISON_LISTS=1 (tests only) fills them with large words
  // instead, so a test can check that no kernel reads a list its pass did not write as nodes
  if (hipMemsetAsync(ctx->cand_count, list_fill(), 2 * kMaxBatch * 4, ctx->stream) != hipSuccess ||
      hipMemsetAsync(ctx->cand_chunk, list_fill(), cand_bytes * 4, ctx->stream) != hipSuccess ||
      hipMemsetAsync(ctx->cand_t, list_fill(), cand_bytes * 8, ctx->stream) != hipSuccess ||
      hipStreamSynchronize(ctx->stream) != hipSuccess) {
    g_create_error = "ks_create: cannot clear the candidate lists";
    ks_destroy(ctx);
    return KS_EHIP;
  }
  *out = ctx;
  return KS_OK;
fail:
  g_create_error = ctx->err;
  ks_destroy(ctx);
  return KS_ENOMEM;
}

void ks_destroy(ks_ctx* ctx) {
  if (!ctx) return;
  // This context's work only: its own stream, and on the process-wide pipeline streams (shared with other contexts,
  // ensure_pipe) the last records of its own events -- each pipelined pass ends its sweep-stream work with a
  // pev_sel record and its commit-stream work with a pev_com record.  Synchronizing the shared streams instead would
  // also wait for every other context's in-flight passes.
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  for (int i = 0; i < kPipeEvents; ++i) {
    if (ctx->pev_sel[i]) (void)hipEventSynchronize(ctx->pev_sel[i]);
    if (ctx->pev_com[i]) (void)hipEventSynchronize(ctx->pev_com[i]);
  }
  for (auto& pr : ctx->lev)
    for (hipEvent_t e : pr)
      if (e) (void)hipEventSynchronize(e);
  dev_free(ctx->node_blob);
  dev_free(ctx->ckpt_blob);
  dev_free(ctx->quota_blob);
  void* p;
  dev_free(ctx->st.blob);
  dev_free(ctx->est.blob);
  dev_free(ctx->ast.blob);
  for (PodStage* ps : {&ctx->st, &ctx->est, &ctx->ast})
    if (ps->h_pack) (void)hipHostFree(ps->h_pack);
  dev_free(ctx->evbuf);
  dev_free(ctx->ures);
  dev_free(ctx->rdscratch);
  dev_free(ctx->dscratch);
  p = ctx->sweep_out; dev_free(p);
  p = ctx->cand_chunk; dev_free(p);
  p = ctx->cand_t; dev_free(p);
  p = ctx->cand_bound; dev_free(p);
  p = ctx->cand_top; dev_free(p);
  p = ctx->cand_second; dev_free(p);
  p = ctx->cand_total; dev_free(p);
  p = ctx->gather; dev_free(p);
  if (ctx->comm) (void)ncclCommDestroy(ctx->comm);
  loop_leave(ctx);
  p = ctx->cand_count; dev_free(p);
  p = ctx->cursor; dev_free(p);
  p = ctx->counters; dev_free(p);
  p = ctx->rowcols; dev_free(p);
  p = ctx->dnodes; dev_free(p);
  p = ctx->drv; dev_free(p);
  dev_free(ctx->rsv_blob);
  p = ctx->ddv; dev_free(p);
  dev_free(ctx->dev_blob);
  p = ctx->dev_M; dev_free(p);
  p = ctx->dcache; dev_free(p);
  dev_free(ctx->cpu_blob);
  p = ctx->cpuset_list; dev_free(p);
  dev_free(ctx->numa_blob);
  p = ctx->dnv; dev_free(p);
  p = ctx->pipe; dev_free(p);
  p = ctx->pipe_top; dev_free(p);
  dev_free(ctx->npod_blob);
  dev_free(ctx->topo_blob);
  for (PodStage* ps : {&ctx->st, &ctx->est, &ctx->ast}) {
    void* t = ps->topo;
    dev_free(t);
    t = ps->topo_terms;
    dev_free(t);
    t = ps->topo_props;
    dev_free(t);
  }
  for (int i = 0; i < kPipeEvents; ++i) {
    if (ctx->pev_sel[i]) (void)hipEventDestroy(ctx->pev_sel[i]);
    if (ctx->pev_com[i]) (void)hipEventDestroy(ctx->pev_com[i]);
  }
  for (hipEvent_t e : ctx->ev_pool) (void)hipEventDestroy(e);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

static void build_col_table(ks_ctx* ctx) {
  DevNodes& d = ctx->d;
  ctx->cols.clear();
  auto add = [&](void* field, int w, bool mut) { ctx->cols.push_back(Col{(void**)field, w, mut}); };
  // mutable columns first (contiguous -> one checkpoint copy)
  add(&d.req_cpu, 8, true);
  add(&d.req_mem, 8, true);
  add(&d.req_eph, 8, true);
  add(&d.nz_cpu, 8, true);
  add(&d.nz_mem, 8, true);
  for (int k = 0; k < KS_MAX_SCALARS; ++k) add(&d.req_sc[k], 8, true);
  add(&d.la_term_cpu, 8, true);
  add(&d.la_term_mem, 8, true);
  add(&d.la_pterm_cpu, 8, true);
  add(&d.la_pterm_mem, 8, true);
  add(&d.rsv_cls, 8, true);
  add(&d.numa_amilli, 8, true);
  add(&d.numa_off, 8, true);
  add(&d.pod_count, 4, true);
  add(&d.numa_cpus, 4, true);
  add(&d.cpu_free, 4, true);
  add(&d.cpu_cores, 4, true);
  add(&d.host_ports, 8, true);
  ctx->topo_count_v.assign((size_t)(ctx->cfg.topology.enable ? ctx->topo_nprops : 0), nullptr);
  ctx->topo_dom_v.assign((size_t)(ctx->cfg.topology.enable ? ctx->topo_nkeys : 0), nullptr);
  for (int32_t*& c : ctx->topo_count_v) add(&c, 4, true);
  // read-only columns
  add(&d.alloc_cpu, 8, false);
  add(&d.alloc_mem, 8, false);
  add(&d.alloc_eph, 8, false);
  for (int k = 0; k < KS_MAX_SCALARS; ++k) add(&d.alloc_sc[k], 8, false);
  add(&d.la_alloc_cpu, 8, false);
  add(&d.la_alloc_mem, 8, false);
  add(&d.la_total_cpu, 8, false);
  add(&d.la_total_mem, 8, false);
  add(&d.la_usage_cpu, 8, false);
  add(&d.la_usage_mem, 8, false);
  add(&d.la_pusage_cpu, 8, false);
  add(&d.la_pusage_mem, 8, false);
  add(&d.allowed_pods, 4, false);
  add(&d.la_flags, 4, false);
  add(&d.la_thr_cpu, 4, false);
  add(&d.la_thr_mem, 4, false);
  add(&d.la_pthr_cpu, 4, false);
  add(&d.la_pthr_mem, 4, false);
  add(&d.la_bits, 4, false);
  add(&d.numa_ratio, 8, false);
  add(&d.numa_flags, 4, false);
  add(&d.taints_hard, 8, false);
  add(&d.taints_soft, 8, false);
  add(&d.labels, 8, false);
  for (int32_t*& c : ctx->topo_dom_v) add(&c, 4, false);
}

// host source pointers in the same order as build_col_table (NULL = zeros); n = the rows of c
static std::vector<const void*> host_cols(const ks_ctx* ctx, const ks_node_cols* c, int64_t n) {
  std::vector<const void*> v;
  v.push_back(c->req_milli_cpu);
  v.push_back(c->req_memory);
  v.push_back(c->req_ephemeral);
  v.push_back(c->nonzero_milli_cpu);
  v.push_back(c->nonzero_memory);
  for (int k = 0; k < KS_MAX_SCALARS; ++k) v.push_back(c->req_scalar[k]);
  v.push_back(c->la_term_milli_cpu);
  v.push_back(c->la_term_memory);
  v.push_back(c->la_prod_term_milli_cpu);
  v.push_back(c->la_prod_term_memory);
  v.push_back(nullptr);  // rsv_cls: derived from the reservation table
  v.push_back(nullptr);  // numa_amilli: derived on device
  v.push_back(nullptr);  // numa_off: derived on device
  v.push_back(c->pod_count);
  v.push_back(c->numa_cpuset_cpus);
  v.push_back(nullptr);  // cpu_free: ks_load_cpu_state (-1 = no CPU topology)
  v.push_back(nullptr);  // cpu_cores: cores_refresh
  v.push_back(c->host_ports);
  for (size_t q = 0; q < ctx->topo_count_v.size(); ++q) v.push_back(c->topo_count ? c->topo_count + (int64_t)q * n : nullptr);
  v.push_back(c->alloc_milli_cpu);
  v.push_back(c->alloc_memory);
  v.push_back(c->alloc_ephemeral);
  for (int k = 0; k < KS_MAX_SCALARS; ++k) v.push_back(c->alloc_scalar[k]);
  v.push_back(c->la_alloc_milli_cpu);
  v.push_back(c->la_alloc_memory);
  v.push_back(c->la_total_milli_cpu);
  v.push_back(c->la_total_milli_memory);
  v.push_back(c->la_usage_milli_cpu);
  v.push_back(c->la_usage_milli_memory);
  v.push_back(c->la_prod_usage_milli_cpu);
  v.push_back(c->la_prod_usage_milli_memory);
  v.push_back(c->allowed_pods);
  v.push_back(c->la_flags);
  v.push_back(c->la_thr_cpu);
  v.push_back(c->la_thr_memory);
  v.push_back(c->la_prod_thr_cpu);
  v.push_back(c->la_prod_thr_memory);
  v.push_back(nullptr);  // la_bits: derived on device
  v.push_back(c->numa_cpu_amplification);
  v.push_back(c->numa_flags);
  v.push_back(c->taints_hard);
  v.push_back(c->taints_soft);
  v.push_back(c->labels);
  // (NULL: -1, set after the copy)
  for (size_t k = 0; k < ctx->topo_dom_v.size(); ++k) v.push_back(c->topo_domain ? c->topo_domain + (int64_t)k * n : nullptr);
  return v;
}

static int check_range64(ks_ctx* ctx, const int64_t* p, int64_t n, const char* what) {
  if (!p) return KS_OK;
  const int64_t lim = (int64_t)1 << 56;
  for (int64_t i = 0; i < n; ++i)
    if (p[i] < 0 || p[i] >= lim) KS_FAIL(ctx, KS_EINVAL, "%s[%lld]=%lld outside [0, 2^56)", what, (long long)i, (long long)p[i]);
  return KS_OK;
}

static int validate_nodes(ks_ctx* ctx, const ks_node_cols* c, int64_t n) {
  if (ctx->cfg.topology.enable) {
    if (c->topo_nkeys < 0 || c->topo_nkeys > KS_TOPO_MAX_KEYS - 1 || c->topo_nprops < 0 ||
        c->topo_nprops > KS_TOPO_MAX_PROPS || c->topo_ndomains < 1 || c->topo_ndomains > (1 << 30))
      KS_FAIL(ctx, KS_EINVAL, "topology sizes: %d keys (max %d), %d domains, %d properties (max %d)", c->topo_nkeys,
              KS_TOPO_MAX_KEYS - 1, c->topo_ndomains, c->topo_nprops, KS_TOPO_MAX_PROPS);
    const int64_t nk = c->topo_nkeys, np = c->topo_nprops;
    for (int64_t i = 0; c->topo_domain && i < nk * n; ++i)
      if (c->topo_domain[i] < -1 || c->topo_domain[i] >= c->topo_ndomains)
        KS_FAIL(ctx, KS_EINVAL, "topo_domain[%lld]=%d outside [-1, %d)", (long long)i, c->topo_domain[i], c->topo_ndomains);
    for (int64_t i = 0; c->topo_count && i < np * n; ++i)
      if (c->topo_count[i] < 0) KS_FAIL(ctx, KS_EINVAL, "topo_count[%lld] < 0", (long long)i);
  }
  if (!c->alloc_milli_cpu || !c->alloc_memory || !c->allowed_pods || !c->req_milli_cpu || !c->req_memory ||
      !c->pod_count || !c->nonzero_milli_cpu || !c->nonzero_memory || !c->la_flags)
    KS_FAIL(ctx, KS_EINVAL, "ks_node_cols: required column missing");
  for (int64_t i = 0; c->labels && i < n; ++i)
    if (c->labels[i] & KS_LABEL_NEVER) KS_FAIL(ctx, KS_EINVAL, "node %lld: labels bit 63 (KS_LABEL_NEVER) set", (long long)i);
  const int64_t* cols64[] = {c->alloc_milli_cpu, c->alloc_memory, c->alloc_ephemeral, c->req_milli_cpu, c->req_memory,
                             c->req_ephemeral, c->nonzero_milli_cpu, c->nonzero_memory, c->la_alloc_milli_cpu,
                             c->la_alloc_memory, c->la_term_milli_cpu, c->la_term_memory, c->la_prod_term_milli_cpu,
                             c->la_prod_term_memory};
  for (const int64_t* col : cols64)
    if (check_range64(ctx, col, n, "node quantity") != KS_OK) return KS_EINVAL;
  for (int k = 0; k < KS_MAX_SCALARS; ++k) {
    if (check_range64(ctx, c->alloc_scalar[k], n, "alloc_scalar") != KS_OK) return KS_EINVAL;
    if (check_range64(ctx, c->req_scalar[k], n, "req_scalar") != KS_OK) return KS_EINVAL;
  }
  if (ctx->cfg.numa.enable) {
    for (int64_t i = 0; c->numa_flags && i < n; ++i)
    {
      const uint32_t f = c->numa_flags[i], label = (f >> KS_NUMA_CPU_BIND_SHIFT) & 3u;
      if (f & KS_NUMA_MAX_REF_COUNT)
        KS_FAIL(ctx, KS_EUNSUPPORTED, "node %lld: CPU sharing with maxRefCount > 1 (node_allocation.go:133-149) is not modelled", (long long)i);
      if (f & (KS_NUMA_CPU_BIND_POLICY | KS_NUMA_TOPOLOGY_POLICY))
        KS_FAIL(ctx, KS_EUNSUPPORTED, "node %lld: numa_flags 0x%x: encode the CPU bind / NUMA topology policy in its bits", (long long)i, f);
      if (label == 3u || (f >> (KS_NUMA_CPU_BIND_SHIFT + 2)))
        KS_FAIL(ctx, KS_EINVAL, "node %lld: numa_flags 0x%x invalid", (long long)i, f);
    }
    for (int64_t i = 0; c->numa_cpuset_cpus && i < n; ++i)
      if (c->numa_cpuset_cpus[i] < 0 || c->numa_cpuset_cpus[i] > (1 << 20))
        KS_FAIL(ctx, KS_EINVAL, "node %lld: numa_cpuset_cpus out of range", (long long)i);
    for (int64_t i = 0; c->numa_cpu_amplification && i < n; ++i)
      if (!(c->numa_cpu_amplification[i] <= 1024.0))  // also rejects NaN
        KS_FAIL(ctx, KS_EINVAL, "node %lld: cpu amplification ratio out of range", (long long)i);
  }
  return KS_OK;
}

// Device table of the slot-row fields' columns (RowField order), read by the commit kernel.
static int upload_rowcols(ks_ctx* ctx) {
  const DevNodes& d = ctx->d;
  RowCol h[RF_N] = {};
  auto set = [&](int f, const void* p, int w) { h[f].p = p; h[f].width = w; };
  set(RF_REQ_CPU, d.req_cpu, 8);
  set(RF_REQ_MEM, d.req_mem, 8);
  set(RF_REQ_EPH, d.req_eph, 8);
  set(RF_NZ_CPU, d.nz_cpu, 8);
  set(RF_NZ_MEM, d.nz_mem, 8);
  for (int k = 0; k < 4; ++k) set(RF_REQ_SC + k, d.req_sc[k], 8);
  set(RF_TERM_CPU, d.la_term_cpu, 8);
  set(RF_TERM_MEM, d.la_term_mem, 8);
  set(RF_PTERM_CPU, d.la_pterm_cpu, 8);
  set(RF_PTERM_MEM, d.la_pterm_mem, 8);
  set(RF_POD_COUNT, d.pod_count, 4);
  set(RF_ALLOC_CPU, d.alloc_cpu, 8);
  set(RF_ALLOC_MEM, d.alloc_mem, 8);
  set(RF_ALLOC_EPH, d.alloc_eph, 8);
  for (int k = 0; k < 4; ++k) set(RF_ALLOC_SC + k, d.alloc_sc[k], 8);
  set(RF_LA_ALLOC_CPU, d.la_alloc_cpu, 8);
  set(RF_LA_ALLOC_MEM, d.la_alloc_mem, 8);
  set(RF_ALLOWED, d.allowed_pods, 4);
  set(RF_LA_BITS, d.la_bits, 4);
  set(RF_RSV_CLS, d.rsv_cls, 8);
  set(RF_RSV_BEG, ctx->rv.beg ? (const void*)ctx->rv.beg : (const void*)d.la_bits, 4);
  set(RF_RSV_END, ctx->rv.beg ? (const void*)(ctx->rv.beg + 1) : (const void*)d.la_bits, 4);
  set(RF_NUMA_A, d.numa_amilli, 8);
  set(RF_NUMA_OFF, d.numa_off, 8);
  set(RF_NUMA_RATIO, d.numa_ratio, 8);
  set(RF_CPU_FREE, d.cpu_free, 4);
  if (!ctx->rowcols) {
    void* p = nullptr;
    if (dev_alloc(ctx, &p, sizeof(h)) != KS_OK) return KS_ENOMEM;
    ctx->rowcols = (RowCol*)p;
  }
  if (!ctx->dnodes) {
    void* p = nullptr;
    if (dev_alloc(ctx, &p, sizeof(DevNodes)) != KS_OK) return KS_ENOMEM;
    ctx->dnodes = (DevNodes*)p;
  }
  if (!ctx->dnv) {
    void* p = nullptr;
    if (dev_alloc(ctx, &p, sizeof(DevNuma)) != KS_OK) return KS_ENOMEM;
    HIPCHK(ctx, hipMemsetAsync(p, 0, sizeof(DevNuma), ctx->stream));
    ctx->dnv = (DevNuma*)p;
  }
  HIPCHK(ctx, hipMemcpyAsync(ctx->rowcols, h, sizeof(h), hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(ctx, hipMemcpyAsync(ctx->dnodes, &ctx->d, sizeof(DevNodes), hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  return KS_OK;
}

static int upload_prep_nodes(ks_ctx* ctx) {
  const int threads = 256;
  const int blocks = (int)((ctx->n + threads - 1) / threads);
  if (blocks > 0)
    hipLaunchKernelGGL(prep_nodes_kernel, dim3(blocks), dim3(threads), 0, ctx->stream, ctx->d, ctx->n,
                       ctx->cfg.loadaware.filter_expired_node_metrics);
  HIPCHK(ctx, hipGetLastError());
  return KS_OK;
}

// CoresWord of every node (ks_device.h) after a load or delta of the node rows or the CPU state; the schedule
// passes keep it current themselves (cpuset_kernel), as does ks_unreserve.
// the NUMA-node words cpuset_kernel refreshes (DevNuma.free), or none without a NUMA-node table
static int32_t* numa_words(const ks_ctx* ctx) { return (ctx->numa_blob && ctx->kc.numa_pol) ? ctx->nv.free : nullptr; }

static int cores_refresh(ks_ctx* ctx) {
  if (!ctx->cfg.numa.enable || ctx->n == 0) return KS_OK;
  hipLaunchKernelGGL(cores_kernel, dim3((unsigned)((ctx->n + 255) / 256)), dim3(256), 0, ctx->stream, ctx->cpu,
                     (int32_t)ctx->cpu_loaded, (const uint32_t*)ctx->d.numa_flags, ctx->d.cpu_cores, (const int32_t*)nullptr,
                     ctx->n);
  HIPCHK(ctx, hipGetLastError());
  return KS_OK;
}

// Cfg.cores: the per-node core counts take part in the Filter once a node CPU bind policy or a required pod policy
// has been seen; the passes then choose CPU ids after every commit (cpuset_kernel) so that the counts stay exact.
static void cores_mode(ks_ctx* ctx) {
  ctx->kc.cores = (ctx->cfg.numa.enable && (ctx->cpu_bind_labels || ctx->cpu_bind_required)) ? 1 : 0;
}

static int rsv_install(ks_ctx* ctx, const ks_reservation_cols* rc, int32_t nr, const int32_t* caller = nullptr,
                       int32_t ncaller = -1);
static int dev_install(ks_ctx* ctx, const ks_device_cols* dc);
static int numa_install(ks_ctx* ctx, const ks_numa_node_cols* nc, const uint32_t* flags_h, const double* ratio_h);
static int check_dev_numa(ks_ctx* ctx);
static int numa_refresh_free(ks_ctx* ctx);

// PodTopologySpread / InterPodAffinity: the topologyNormalizingWeight table log(s + 2) for every topology size a
// pod can see (s <= nodes; the host's libm, as the oracle), the topology step's scratch and one-candidate set
static int topo_install(ks_ctx* ctx) {
  dev_free(ctx->topo_blob);
  // sizes a pod can see: the hostname's up to n nodes, another key's up to ndom values + ""
  const int32_t nlw = (int32_t)std::max<int64_t>(ctx->n, ctx->topo_ndom + 1) + 2;
  const size_t b_lw = ((size_t)nlw * 8 + 255) / 256 * 256;
  const size_t b_scr = (sizeof(TopoScratch) + 255) / 256 * 256;
  const size_t b_cand = (size_t)kMaxBatch * kMaxCand * (4 + 8) + (size_t)kMaxBatch * (4 + 8 * 3);
  const size_t b_raw = (size_t)ctx->npad * 8 * 2;
  const size_t nw = ((size_t)ctx->topo_ndom + 31) / 32;
  const size_t b_zsum = (size_t)kTopoTerms * (size_t)ctx->topo_ndom * 8, b_bits = (size_t)kTopoTerms * nw * 4;
  const size_t tot = b_lw + b_scr + b_cand + b_raw + b_zsum + 2 * b_bits;
  if (dev_alloc(ctx, &ctx->topo_blob, tot) != KS_OK) return KS_ENOMEM;
  char* b = (char*)ctx->topo_blob;
  HIPCHK(ctx, hipMemsetAsync(b, 0, tot, ctx->stream));
  ctx->topo_sraw = (long long*)(b + b_lw + b_scr + b_cand);
  ctx->topo_iraw = ctx->topo_sraw + ctx->npad;
  ctx->topo_zsum = (long long*)(b + b_lw + b_scr + b_cand + b_raw);
  ctx->topo_zpres = (uint32_t*)(b + b_lw + b_scr + b_cand + b_raw + b_zsum);
  ctx->topo_zsize = (uint32_t*)(b + b_lw + b_scr + b_cand + b_raw + b_zsum + b_bits);
  ctx->topo_lw = (double*)b;
  ctx->topo_nlw = nlw;
  ctx->topo_scr = (TopoScratch*)(b + b_lw);
  char* c = b + b_lw + b_scr;
  ctx->topo_ct = (uint2*)c;
  c += (size_t)kMaxBatch * kMaxCand * 8;
  ctx->topo_cbound = (uint64_t*)c;
  c += kMaxBatch * 8;
  ctx->topo_ctop = (uint64_t*)c;
  c += kMaxBatch * 8;
  ctx->topo_csecond = (uint64_t*)c;
  c += kMaxBatch * 8;
  ctx->topo_cchunk = (uint32_t*)c;
  c += (size_t)kMaxBatch * kMaxCand * 4;
  ctx->topo_ccount = (int32_t*)c;
  std::vector<double> lw((size_t)nlw);
  for (int32_t i = 0; i < nlw; ++i) lw[(size_t)i] = log((double)(i + 2));
  HIPCHK(ctx, hipMemcpyAsync(ctx->topo_lw, lw.data(), (size_t)nlw * 8, hipMemcpyHostToDevice, ctx->stream));
  const TopoScratch init = topo_scratch_init();
  HIPCHK(ctx, hipMemcpyAsync(ctx->topo_scr, &init, sizeof(init), hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));  // (pageable source)
  return KS_OK;
}

static DevTopo dev_topo(const ks_ctx* ctx) {
  DevTopo t;
  t.dom = ctx->topo_dom;
  t.count = ctx->topo_count;
  t.npad = ctx->npad;
  t.nkeys = ctx->topo_nkeys;
  t.ndom = ctx->topo_ndom;
  t.lw = ctx->topo_lw;
  t.nlw = ctx->topo_nlw;
  t.nw = (ctx->topo_ndom + 31) / 32;
  t.zsum = ctx->topo_zsum;
  t.zpres = ctx->topo_zpres;
  t.zsize = ctx->topo_zsize;
  return t;
}

int ks_load_nodes(ks_ctx* ctx, const ks_node_cols* nodes, int64_t n) {
  if (!ctx || !nodes || n < 0 || n >= ((int64_t)1 << 31)) return ctx ? (ctx->err = "ks_load_nodes: bad args", KS_EINVAL) : KS_EINVAL;
  if (int rc = validate_nodes(ctx, nodes, n); rc != KS_OK) return rc;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  ctx->h_dev_assumed.clear();
  dev_free(ctx->node_blob);
  dev_free(ctx->ckpt_blob);
  void* p = ctx->sweep_out;
  dev_free(p);
  ctx->sweep_out = nullptr;
  ctx->rsv_based = false;  // fresh columns (a loaded reservation table is dropped: reload it)
  ctx->rsv_nrows = 0;
  ctx->rsv_live = 0;
  ctx->rmir = ks_ctx::RsvMirror{};
  // the node-pod table (ks_load_node_pods) is indexed by the old node rows and its per-call scratch is sized to the
  // old node count: drop it, so ks_preempt returns KS_ESTATE until it is reloaded for these nodes
  dev_free(ctx->npod_blob);
  ctx->npt = DevNodePods{};
  ctx->pre_cand = nullptr;
  ctx->pre_vrank = nullptr;
  ctx->pre_status = nullptr;
  ctx->pre_out = nullptr;
  ctx->pre_victims = nullptr;
  ctx->n = n;
  ctx->nchunks = (n + 63) / 64;
  if (ctx->nchunks == 0) ctx->nchunks = 1;
  ctx->npad = ctx->nchunks * 64;
  int nsc = 0;
  for (int k = 0; k < KS_MAX_SCALARS; ++k) {
    bool used = ctx->cfg.fit.weight_scalar[k] != 0;
    for (int64_t i = 0; !used && nodes->alloc_scalar[k] && i < n; ++i) used = nodes->alloc_scalar[k][i] != 0;
    for (int64_t i = 0; !used && nodes->req_scalar[k] && i < n; ++i) used = nodes->req_scalar[k][i] != 0;
    if (used) nsc = k + 1;
  }
  ctx->nsc = nsc <= 0 ? 0 : (nsc <= 2 ? 2 : 4);
  ctx->kc = make_cfg(ctx->cfg, ctx->nsc);
  ctx->soft_union = 0;
  for (int64_t i = 0; nodes->taints_soft && i < n; ++i) ctx->soft_union |= nodes->taints_soft[i];
  ctx->topo_nkeys = ctx->cfg.topology.enable ? nodes->topo_nkeys : 0;
  ctx->topo_ndom = ctx->cfg.topology.enable ? nodes->topo_ndomains : 1;
  ctx->topo_nprops = ctx->cfg.topology.enable ? nodes->topo_nprops : 0;
  build_col_table(ctx);
  size_t total = 0, mut = 0;
  for (const Col& c : ctx->cols) {
    total += (size_t)ctx->npad * c.width;
    if (c.mutable_) mut += (size_t)ctx->npad * c.width;
  }
  ctx->mut_bytes = mut;
  if (dev_alloc(ctx, &ctx->node_blob, total) != KS_OK) return KS_ENOMEM;
  HIPCHK(ctx, hipMemsetAsync(ctx->node_blob, 0, total, ctx->stream));
  char* base = (char*)ctx->node_blob;
  std::vector<const void*> src = host_cols(ctx, nodes, n);
  for (size_t i = 0; i < ctx->cols.size(); ++i) {
    *ctx->cols[i].dev = base;
    if (src[i] && n > 0)
      HIPCHK(ctx, hipMemcpyAsync(base, src[i], (size_t)n * ctx->cols[i].width, hipMemcpyHostToDevice, ctx->stream));
    base += (size_t)ctx->npad * ctx->cols[i].width;
  }
  HIPCHK(ctx, hipMemsetAsync(ctx->d.cpu_free, 0xFF, (size_t)ctx->npad * 4, ctx->stream));  // no CPU topology yet
  if (ctx->cfg.topology.enable) {
    ctx->topo_dom = ctx->topo_dom_v.empty() ? nullptr : ctx->topo_dom_v[0];
    ctx->topo_count = ctx->topo_count_v.empty() ? nullptr : ctx->topo_count_v[0];
    if (!nodes->topo_domain && ctx->topo_dom)
      HIPCHK(ctx, hipMemsetAsync(ctx->topo_dom, 0xFF, (size_t)ctx->npad * 4 * ctx->topo_nkeys, ctx->stream));
    if (topo_install(ctx) != KS_OK) return KS_ENOMEM;
  }
  ctx->cpu_loaded = false;
  // two sweep outputs: patched pipelined passes sweep pass k+1 while pass k's re-sweep still reads pass k's
  if (dev_alloc(ctx, &p, (size_t)2 * ctx->nchunks * 64 * 8) != KS_OK) return KS_ENOMEM;
  ctx->sweep_out = (uint2*)p;
  if (upload_rowcols(ctx) != KS_OK) return KS_ENOMEM;
  if (upload_prep_nodes(ctx) != KS_OK) return KS_EHIP;
  if (ctx->cfg.reservation.enable && rsv_install(ctx, nullptr, 0) != KS_OK) return KS_EHIP;
  if (ctx->cfg.deviceshare.enable && dev_install(ctx, nullptr) != KS_OK) return KS_EHIP;
  // NUMA topology policies: an empty NUMA-node table until ks_load_numa_nodes
  ctx->numa_policy_nodes = 0;
  ctx->cpu_bind_labels = false;
  ctx->h_pol.assign((size_t)n, 0);
  for (int64_t i = 0; ctx->cfg.numa.enable && nodes->numa_flags && i < n; ++i) {
    ctx->h_pol[(size_t)i] = ((nodes->numa_flags[i] >> KS_NUMA_POLICY_SHIFT) & 3u) != 0;
    ctx->numa_policy_nodes += ((nodes->numa_flags[i] >> KS_NUMA_POLICY_SHIFT) & 3u) != 0;
    ctx->cpu_bind_labels |= ((nodes->numa_flags[i] >> KS_NUMA_CPU_BIND_SHIFT) & 3u) != 0;
  }
  cores_mode(ctx);
  if (cores_refresh(ctx) != KS_OK) return KS_EHIP;
  dev_free(ctx->numa_blob);
  if (ctx->numa_policy_nodes > 0) {
    if (numa_install(ctx, nullptr, nullptr, nullptr) != KS_OK) return KS_EHIP;
    ctx->kc.numa_pol = 1;
    ctx->kc.monotone = 0;  // a Reserve can move a node's best NUMA hint: keys are not monotone
    ctx->kc.monotone_nd = 0;
  }
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  return KS_OK;
}

// kDevRsvHeld into the device table's node flags from h_dev_held (after a reservation or a device install)
__global__ void dev_held_kernel(uint32_t* flags, const uint8_t* held, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  flags[i] = (flags[i] & ~kDevRsvHeld) | (held[i] ? kDevRsvHeld : 0u);
}

static int dev_apply_held(ks_ctx* ctx) {
  ctx->dev_held_any = false;
  if (!ctx->dev_blob || ctx->n == 0) return KS_OK;
  if (ctx->h_dev_held.size() != (size_t)ctx->n) ctx->h_dev_held.assign((size_t)ctx->n, 0);
  for (uint8_t h : ctx->h_dev_held) ctx->dev_held_any = ctx->dev_held_any || h != 0;
  void* p = nullptr;
  if (dev_alloc(ctx, &p, (size_t)ctx->n) != KS_OK) return KS_ENOMEM;
  HIPCHK(ctx, hipMemcpyAsync(p, ctx->h_dev_held.data(), (size_t)ctx->n, hipMemcpyHostToDevice, ctx->stream));
  hipLaunchKernelGGL(dev_held_kernel, dim3((unsigned)((ctx->n + 255) / 256)), dim3(256), 0, ctx->stream,
                     const_cast<uint32_t*>(ctx->dv.flags), (const uint8_t*)p, ctx->n);
  HIPCHK(ctx, hipGetLastError());
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  dev_free(p);
  return KS_OK;
}

static int rsv_launch_base(ks_ctx* ctx, const int32_t* didx, int64_t count, int64_t sign, int32_t classes) {
  if (count <= 0) return KS_OK;
  hipLaunchKernelGGL(rsv_base_kernel, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, ctx->stream, ctx->d, ctx->rv,
                     didx, count, sign, classes);
  HIPCHK(ctx, hipGetLastError());
  return KS_OK;
}

// Upload the reservation table (CSR by node), add its base restore to the node columns.
// rc holds the device table's rows; caller[r] is row r's caller row (NULL: r itself) of ncaller caller rows.
static int rsv_install(ks_ctx* ctx, const ks_reservation_cols* rc, int32_t nr, const int32_t* caller,
                       int32_t ncaller) {
  constexpr int D = kRsvDims;
  if (ncaller < 0) ncaller = nr;
  auto crow = [&](int32_t r) { return caller ? caller[r] : r; };
  if (nr > 0 && (!rc || !rc->node || !rc->owner_classes || !rc->key_mask))
    KS_FAIL(ctx, KS_EINVAL, "ks_reservation_cols: node, owner_classes and key_mask are required");
  for (int32_t r = 0; r < nr; ++r) {
    if (rc->node[r] < 0 || rc->node[r] >= ctx->n) KS_FAIL(ctx, KS_EINVAL, "reservation %d: node %d out of range", r, rc->node[r]);
    if (rc->assigned && rc->assigned[r] < 0) KS_FAIL(ctx, KS_EINVAL, "reservation %d: negative assigned count", r);
    if (rc->key_mask[r] >> D) KS_FAIL(ctx, KS_EINVAL, "reservation %d: key_mask has bits beyond KS_RSV_DIMS", r);
  }
  for (int d = 0; d < D; ++d) {
    if (check_range64(ctx, rc ? rc->allocatable[d] : nullptr, nr, "reservation allocatable") != KS_OK) return KS_EINVAL;
    if (check_range64(ctx, rc ? rc->allocated[d] : nullptr, nr, "reservation allocated") != KS_OK) return KS_EINVAL;
  }
  if (nr > 0) {
    if (check_range64(ctx, rc->reserve_nonzero_milli_cpu, nr, "reserve_nonzero_milli_cpu") != KS_OK) return KS_EINVAL;
    if (check_range64(ctx, rc->reserve_nonzero_memory, nr, "reserve_nonzero_memory") != KS_OK) return KS_EINVAL;
  }
  // DeviceShare reservations (deviceshare/reservation.go): a reservation holding devices on a NUMA-policy node is
  // refused (the topology hints would run tryAllocateFromReservation per NUMA mask)
  std::vector<uint8_t> held((size_t)ctx->n, 0);
  const bool devr = rc && rc->dev_allocatable;
  if (devr) {
    if (check_range64(ctx, rc->dev_allocatable, (int64_t)nr * KS_DEV_WORDS, "reservation dev_allocatable") != KS_OK ||
        check_range64(ctx, rc->dev_allocated, (int64_t)nr * KS_DEV_WORDS, "reservation dev_allocated") != KS_OK)
      return KS_EINVAL;
    if (!ctx->cfg.deviceshare.enable) KS_FAIL(ctx, KS_ESTATE, "reservations hold devices but DeviceShare is not enabled");
    for (int32_t r = 0; r < nr; ++r) {
      bool h = false;
      for (int w = 0; w < KS_DEV_WORDS; ++w) h |= rc->dev_allocatable[(size_t)r * KS_DEV_WORDS + w] != 0;
      if (!h) continue;
      if ((size_t)rc->node[r] < ctx->h_pol.size() && ctx->h_pol[(size_t)rc->node[r]])
        KS_FAIL(ctx, KS_EUNSUPPORTED, "reservation %d holds devices on node %d, which has a NUMA topology policy", r,
                rc->node[r]);
      held[(size_t)rc->node[r]] = 1;
    }
  }
  // order labels -> composite ranks (smaller label = larger hi)
  std::vector<int64_t> ords;
  for (int32_t r = 0; r < nr; ++r)
    if (rc->order && rc->order[r] != 0) ords.push_back(rc->order[r]);
  std::sort(ords.begin(), ords.end());
  ords.erase(std::unique(ords.begin(), ords.end()), ords.end());
  const int64_t ndist = (int64_t)ords.size();
  if ((int64_t)(kRsvOrderBase + ndist + 1) * ctx->kc.rsv_F >= ((int64_t)1 << 26))
    KS_FAIL(ctx, KS_EUNSUPPORTED, "too many distinct reservation order labels (%lld) for the key width", (long long)ndist);
  // remove the previous table's base restore
  if (ctx->rsv_based) {
    if (rsv_launch_base(ctx, nullptr, ctx->n, -1, 0) != KS_OK) return KS_EHIP;
    ctx->rsv_based = false;
  }
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  std::vector<int32_t> perm(nr);
  for (int32_t r = 0; r < nr; ++r) perm[r] = r;
  std::stable_sort(perm.begin(), perm.end(), [&](int32_t x, int32_t y) { return rc->node[x] < rc->node[y]; });
  const size_t m = (size_t)(nr > 0 ? nr : 1);
  auto al16 = [](size_t x) { return (x + 15) / 16 * 16; };
  const size_t o_beg = 0, o_cls = al16((size_t)(ctx->npad + 1) * 4), o_meta = o_cls + al16(m * 8),
               o_ohi = o_meta + al16(m * 4), o_alloc = o_ohi + al16(m * 4), o_allocd = o_alloc + al16(D * m * 8),
               o_asg = o_allocd + al16(D * m * 8), o_rnz = o_asg + al16(m * 4), o_row = o_rnz + al16(2 * m * 8),
               o_ck_allocd = o_row + al16(m * 4), o_ck_asg = o_ck_allocd + al16(D * m * 8),
               o_dal = o_ck_asg + al16(m * 4), o_dald = o_dal + al16((size_t)kDevQW * m * 8),
               o_ck_dald = o_dald + al16((size_t)kDevQW * m * 8), o_dmask = o_ck_dald + al16((size_t)kDevQW * m * 8),
               bytes = o_dmask + al16(m * 4);
  std::vector<char> h(bytes, 0);
  int32_t* beg = (int32_t*)(h.data() + o_beg);
  uint64_t* cls = (uint64_t*)(h.data() + o_cls);
  uint32_t* meta = (uint32_t*)(h.data() + o_meta);
  int32_t* ohi = (int32_t*)(h.data() + o_ohi);
  int64_t* alloc = (int64_t*)(h.data() + o_alloc);
  int64_t* allocd = (int64_t*)(h.data() + o_allocd);
  int32_t* asg = (int32_t*)(h.data() + o_asg);
  int64_t* rnz = (int64_t*)(h.data() + o_rnz);
  int32_t* rowid = (int32_t*)(h.data() + o_row);
  int64_t* dal = (int64_t*)(h.data() + o_dal);
  int64_t* dald = (int64_t*)(h.data() + o_dald);
  uint32_t* dmask = (uint32_t*)(h.data() + o_dmask);
  for (int32_t i = 0; i < nr; ++i) beg[rc->node[perm[i]] + 1]++;
  for (int64_t n = 0; n < ctx->npad; ++n) beg[n + 1] += beg[n];
  ctx->h_rsv_gi.assign((size_t)ncaller, -1);
  ctx->h_rsv_node.assign((size_t)nr, -1);
  for (int32_t i = 0; i < nr; ++i) {
    const int32_t r = perm[i];
    rowid[i] = crow(r);
    ctx->h_rsv_gi[(size_t)crow(r)] = i;
    ctx->h_rsv_node[(size_t)i] = rc->node[r];
    cls[i] = rc->owner_classes[r];
    const uint32_t flags = rc->flags ? rc->flags[r] & 0xfu : 0u;
    const uint32_t pol = rc->policy ? std::min<uint32_t>(rc->policy[r], 0xfu) : 0u;
    int32_t nd = 0;
    for (int d = 0; d < D; ++d)
      if ((rc->allocatable[d] && rc->allocatable[d][r]) || (rc->allocated[d] && rc->allocated[d][r])) nd = d + 1;
    meta[i] = flags | (pol << 4) | (rc->key_mask[r] << 8) | ((uint32_t)nd << 16);
    if (devr) {
      bool h = false;
      for (int w = 0; w < kDevQW; ++w) {
        dal[(size_t)w * m + i] = rc->dev_allocatable[(size_t)r * KS_DEV_WORDS + w];
        dald[(size_t)w * m + i] = rc->dev_allocated ? rc->dev_allocated[(size_t)r * KS_DEV_WORDS + w] : 0;
        h |= dal[(size_t)w * m + i] != 0;
        dmask[i] |= dal[(size_t)w * m + i] != 0 ? (1u << w) : 0u;
      }
      if (h) meta[i] |= kRsvMetaDev;
    }
    const int64_t o = rc->order ? rc->order[r] : 0;
    if (o != 0) {
      const int64_t rank = std::lower_bound(ords.begin(), ords.end(), o) - ords.begin();
      ohi[i] = (int32_t)(kRsvOrderBase + (ndist - 1 - rank));
    }
    for (int d = 0; d < D; ++d) {
      alloc[(size_t)d * m + i] = rc->allocatable[d] ? rc->allocatable[d][r] : 0;
      allocd[(size_t)d * m + i] = rc->allocated[d] ? rc->allocated[d][r] : 0;
    }
    asg[i] = rc->assigned ? rc->assigned[r] : 0;
    // reserve pod's NonZeroRequested (one container with the allocatable as requests by default)
    const uint32_t keys = rc->key_mask[r];
    rnz[i] = rc->reserve_nonzero_milli_cpu ? rc->reserve_nonzero_milli_cpu[r]
                                           : ((keys & 1u) ? alloc[i] : kDefaultMilliCPU);
    rnz[m + i] = rc->reserve_nonzero_memory ? rc->reserve_nonzero_memory[r]
                                            : ((keys & 2u) ? alloc[m + i] : kDefaultMemory);
  }
  dev_free(ctx->rsv_blob);
  if (dev_alloc(ctx, &ctx->rsv_blob, bytes) != KS_OK) return KS_ENOMEM;
  HIPCHK(ctx, hipMemcpyAsync(ctx->rsv_blob, h.data(), bytes, hipMemcpyHostToDevice, ctx->stream));
  char* b = (char*)ctx->rsv_blob;
  DevRsv& rv = ctx->rv;
  rv.beg = (const int32_t*)(b + o_beg);
  rv.cls = (const uint64_t*)(b + o_cls);
  rv.meta = (const uint32_t*)(b + o_meta);
  rv.ohi = (const int32_t*)(b + o_ohi);
  rv.alloc = (const int64_t*)(b + o_alloc);
  rv.allocd = (int64_t*)(b + o_allocd);
  rv.assigned = (int32_t*)(b + o_asg);
  rv.rnz = (const int64_t*)(b + o_rnz);
  rv.rowid = (const int32_t*)(b + o_row);
  rv.dal = (const int64_t*)(b + o_dal);
  rv.dald = (int64_t*)(b + o_dald);
  rv.dmask = (const uint32_t*)(b + o_dmask);
  ctx->rsv_dald_ckpt = (int64_t*)(b + o_ck_dald);
  rv.ncls = ctx->d.rsv_cls;
  rv.nr = (int64_t)m;  // row stride of the [dim][row] tables
  rv.w100 = 100 * ctx->cfg.reservation.plugin_weight;
  ctx->rsv_allocd_ckpt = (int64_t*)(b + o_ck_allocd);
  ctx->rsv_assigned_ckpt = (int32_t*)(b + o_ck_asg);
  ctx->rsv_ndist = (int32_t)ndist;
  ctx->rsv_nrows = ncaller;
  ctx->rsv_live = nr;
  for (int32_t i = 0; i < nr; ++i) perm[i] = crow(perm[i]);
  ctx->rsv_perm = perm;
  if (!ctx->drv) {
    void* p = nullptr;
    if (dev_alloc(ctx, &p, sizeof(DevRsv)) != KS_OK) return KS_ENOMEM;
    ctx->drv = (DevRsv*)p;
  }
  HIPCHK(ctx, hipMemcpyAsync(ctx->drv, &ctx->rv, sizeof(DevRsv), hipMemcpyHostToDevice, ctx->stream));
  if (upload_rowcols(ctx) != KS_OK) return KS_ENOMEM;  // row fields RF_RSV_BEG / RF_RSV_END
  if (rsv_launch_base(ctx, nullptr, ctx->n, +1, 1) != KS_OK) return KS_EHIP;
  ctx->rsv_based = true;
  ctx->h_dev_held = held;
  if (dev_apply_held(ctx) != KS_OK) return KS_EHIP;
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  return KS_OK;
}

// Upload the device table (kDevTW words of totals + topology, kDevQW words of used, flags per node; ks_dev.h);
// dc == NULL: no device info.
// The device table words of `rows` rows of dc: flags[r], total[w * np + r], used[w * np + r] and the NUMA ids of
// the device topology (dev_hints) per row; np = the column stride.
static int dev_encode(ks_ctx* ctx, const ks_device_cols* dc, int64_t rows, size_t np, uint32_t* flags, int64_t* total,
                      int64_t* used, uint16_t* ids_out) {
  if (dc) {
    for (int k = 0; k < kGpus; ++k) {
      const int64_t* cols[6] = {dc->total_core[k], dc->total_memory[k], dc->total_ratio[k],
                                dc->used_core[k], dc->used_memory[k], dc->used_ratio[k]};
      for (int c = 0; c < 6; ++c)
        if (check_range64(ctx, cols[c], rows, "device quantity") != KS_OK) return KS_EINVAL;
      for (int64_t n = 0; n < rows; ++n)
        for (int q = 0; q < 3; ++q) {
          total[((size_t)q * kGpus + k) * np + n] = cols[q] ? cols[q][n] : 0;
          used[((size_t)q * kGpus + k) * np + n] = cols[3 + q] ? cols[3 + q][n] : 0;
        }
    }
    for (int j = 0; j < kRdma; ++j) {
      if (check_range64(ctx, dc->total_rdma[j], rows, "rdma quantity") != KS_OK ||
          check_range64(ctx, dc->used_rdma[j], rows, "rdma quantity") != KS_OK)
        return KS_EINVAL;
      for (int64_t n = 0; n < rows; ++n) {
        total[((size_t)kDevRdmaW + j) * np + n] = dc->total_rdma[j] ? dc->total_rdma[j][n] : 0;
        used[((size_t)kDevRdmaW + j) * np + n] = dc->used_rdma[j] ? dc->used_rdma[j][n] : 0;
      }
    }
    // topology: 4-bit switch per minor, NUMA node / socket per switch; switches numbered in (socket, node) order
    for (int64_t n = 0; n < rows; ++n) {
      uint64_t topo = 0, meta = 0;
      uint32_t used_sw = 0;
      auto sw = [&](const uint8_t* col, int k, int shift) -> int {
        const uint32_t p = col ? col[n] : KS_PCIE_NONE;
        if (p != KS_PCIE_NONE && p >= (uint32_t)kPcie) return -1;
        topo |= (uint64_t)(p == KS_PCIE_NONE ? 0xFu : p) << (shift + 4 * k);
        if (p != KS_PCIE_NONE) used_sw |= 1u << p;
        return 0;
      };
      for (int k = 0; k < kGpus; ++k)
        if (sw(dc->gpu_pcie[k], k, 0)) KS_FAIL(ctx, KS_EINVAL, "node %lld: gpu %d PCIe switch >= %d", (long long)n, k, kPcie);
      for (int j = 0; j < kRdma; ++j)
        if (sw(dc->rdma_pcie[j], j, 32)) KS_FAIL(ctx, KS_EINVAL, "node %lld: rdma %d PCIe switch >= %d", (long long)n, j, kPcie);
      int last = -1;
      for (int p = 0; p < kPcie; ++p) {
        const uint32_t nu = dc->pcie_numa[p] ? dc->pcie_numa[p][n] : 0, so = dc->pcie_socket[p] ? dc->pcie_socket[p][n] : 0;
        if (nu > 15 || so > 15) KS_FAIL(ctx, KS_EINVAL, "node %lld: PCIe switch %d NUMA node / socket > 15", (long long)n, p);
        meta |= (uint64_t)(nu | (so << 4)) << (8 * p);
        if (!((used_sw >> p) & 1u)) continue;
        // the device walks switches in index order: it must be (socket, node) order (newDeviceTopologyGuide)
        if (last >= 0) {
          const uint32_t lnu = (uint32_t)(meta >> (8 * last)) & 0xFu, lso = (uint32_t)(meta >> (8 * last + 4)) & 0xFu;
          if (so < lso || (so == lso && nu < lnu))
            KS_FAIL(ctx, KS_EINVAL, "node %lld: PCIe switches not numbered in (socket, NUMA node) order", (long long)n);
        }
        last = p;
      }
      total[(size_t)kDevTopoW * np + n] = (int64_t)topo;
      total[(size_t)kDevMetaW * np + n] = (int64_t)meta;
    }
    for (int64_t n = 0; n < rows; ++n) {
      flags[n] = dc->flags ? dc->flags[n] : 0;
      if (flags[n] & KS_DEV_UNMODELLED)
        KS_FAIL(ctx, KS_EUNSUPPORTED, "node row %lld: preemptible device capacity or device-holding reservations "
                                      "(device_cache.go:314, deviceshare/reservation.go) are not modelled", (long long)n);
      if (flags[n] & ~(uint32_t)KS_DEV_PRESENT) KS_FAIL(ctx, KS_EINVAL, "node row %lld: device flags 0x%x", (long long)n, flags[n]);
    }
  }
  // NUMA nodes of the device topology per node, as dev_hints (ks_numa.h) derives them
  for (int64_t n = 0; n < rows; ++n) ids_out[n] = 0;
  for (int64_t n = 0; dc && n < rows; ++n) {
    const uint64_t topo = (uint64_t)total[(size_t)kDevTopoW * np + n], meta = (uint64_t)total[(size_t)kDevMetaW * np + n];
    uint32_t ids = 0;
    for (int k = 0; k < kGpus; ++k) {
      const uint32_t pc = (uint32_t)(topo >> (4 * k)) & 0xFu;
      bool ex = false;
      for (int q = 0; q < 3; ++q) ex |= total[((size_t)q * kGpus + k) * np + n] != 0;
      if (ex && pc < 8u) ids |= 1u << ((uint32_t)(meta >> (8 * pc)) & 0xFu);
    }
    for (int j = 0; j < kRdma; ++j) {
      const uint32_t pc = (uint32_t)(topo >> (32 + 4 * j)) & 0xFu;
      if (total[((size_t)kDevRdmaW + j) * np + n] != 0 && pc < 8u) ids |= 1u << ((uint32_t)(meta >> (8 * pc)) & 0xFu);
    }
    ids_out[n] = (uint16_t)ids;
  }
  return KS_OK;
}

static int dev_install(ks_ctx* ctx, const ks_device_cols* dc) {
  const size_t np = (size_t)ctx->npad, tw = (size_t)kDevTW * np, uw = (size_t)kDevQW * np;
  const size_t o_flags = 0, o_total = (np * 4 + 15) / 16 * 16, o_used = o_total + tw * 8, o_ck = o_used + uw * 8,
               bytes = o_ck + uw * 8;
  std::vector<char> h(bytes, 0);
  uint32_t* flags = (uint32_t*)(h.data() + o_flags);
  int64_t* total = (int64_t*)(h.data() + o_total);
  int64_t* used = (int64_t*)(h.data() + o_used);
  ctx->h_dev_ids.assign((size_t)ctx->n, 0);
  if (int rc = dev_encode(ctx, dc, ctx->n, np, flags, total, used, ctx->h_dev_ids.data()); rc != KS_OK) return rc;
  dev_free(ctx->dev_blob);
  if (dev_alloc(ctx, &ctx->dev_blob, bytes) != KS_OK) return KS_ENOMEM;
  HIPCHK(ctx, hipMemcpyAsync(ctx->dev_blob, h.data(), bytes, hipMemcpyHostToDevice, ctx->stream));
  char* b = (char*)ctx->dev_blob;
  ctx->dv.flags = (const uint32_t*)(b + o_flags);
  ctx->dv.total = (const int64_t*)(b + o_total);
  ctx->dv.used = (int64_t*)(b + o_used);
  ctx->dv.npad = (int64_t)np;
  ctx->dev_used_ckpt = (int64_t*)(b + o_ck);
  if (!ctx->ddv) {
    void* p = nullptr;
    if (dev_alloc(ctx, &p, sizeof(DevDev)) != KS_OK) return KS_ENOMEM;
    ctx->ddv = (DevDev*)p;
  }
  HIPCHK(ctx, hipMemcpyAsync(ctx->ddv, &ctx->dv, sizeof(DevDev), hipMemcpyHostToDevice, ctx->stream));
  ctx->dev_loaded = dc != nullptr;
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  if (dev_apply_held(ctx) != KS_OK) return KS_EHIP;
  return check_dev_numa(ctx);
}

int ks_load_devices(ks_ctx* ctx, const ks_device_cols* dev, int64_t n) {
  if (!ctx || !dev) return ctx ? (ctx->err = "ks_load_devices: bad args", KS_EINVAL) : KS_EINVAL;
  if (!ctx->node_blob) KS_FAIL(ctx, KS_ESTATE, "ks_load_devices before ks_load_nodes");
  if (n != ctx->n) KS_FAIL(ctx, KS_EINVAL, "ks_load_devices: %lld rows for %lld nodes", (long long)n, (long long)ctx->n);
  if (!ctx->cfg.deviceshare.enable) KS_FAIL(ctx, KS_ESTATE, "ks_load_devices: the DeviceShare plugin is not enabled");
  HIPCHK(ctx, hipSetDevice(ctx->device));
  ctx->h_dev_assumed.clear();  // a full reload carries its own usage
  return dev_install(ctx, dev);
}

static int read_dev_used(ks_ctx* ctx, std::vector<int64_t>& u) {
  u.resize((size_t)kDevQW * (size_t)ctx->npad);
  HIPCHK(ctx, hipMemcpyAsync(u.data(), ctx->dv.used, u.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  return KS_OK;
}

int ks_read_devices(ks_ctx* ctx, int64_t* used_core, int64_t* used_memory, int64_t* used_ratio) {
  if (!ctx) return KS_EINVAL;
  if (!ctx->dev_blob) return KS_OK;
  const size_t np = (size_t)ctx->npad, n = (size_t)ctx->n;
  std::vector<int64_t> u;
  if (read_dev_used(ctx, u) != KS_OK) return KS_EHIP;
  int64_t* outs[3] = {used_core, used_memory, used_ratio};
  for (int q = 0; q < 3; ++q)
    if (outs[q])
      for (int k = 0; k < kGpus; ++k) memcpy(outs[q] + (size_t)k * n, u.data() + ((size_t)q * kGpus + k) * np, n * 8);
  return KS_OK;
}

int ks_read_devices_rdma(ks_ctx* ctx, int64_t* used_rdma) {
  if (!ctx || !used_rdma) return KS_EINVAL;
  if (!ctx->dev_blob) return KS_OK;
  const size_t np = (size_t)ctx->npad, n = (size_t)ctx->n;
  std::vector<int64_t> u;
  if (read_dev_used(ctx, u) != KS_OK) return KS_EHIP;
  for (int j = 0; j < kRdma; ++j) memcpy(used_rdma + (size_t)j * n, u.data() + ((size_t)kDevRdmaW + j) * np, n * 8);
  return KS_OK;
}

// Dense form of one ks_cpu_topology (ids in ascending order -> indices); checks the shape assumptions.
static int build_cpu_topo(ks_ctx* ctx, const ks_cpu_topology& in, int32_t ti, CpuTopo& t) {
  memset(&t, 0, sizeof(t));
  const int nc = in.ncpus;
  if (nc <= 0 || nc > KS_MAX_CPUS) KS_FAIL(ctx, KS_EINVAL, "cpu topology %d: ncpus %d outside (0, %d]", ti, nc, KS_MAX_CPUS);
  std::vector<int32_t> cores(in.core, in.core + nc), nodes(in.numa_node, in.numa_node + nc), socks(in.socket, in.socket + nc);
  for (int c = 0; c < nc; ++c)
    if (in.core[c] < 0 || in.numa_node[c] < 0 || in.socket[c] < 0)
      KS_FAIL(ctx, KS_EINVAL, "cpu topology %d: negative id for CPU %d", ti, c);
  auto uniq = [](std::vector<int32_t>& v) { std::sort(v.begin(), v.end()); v.erase(std::unique(v.begin(), v.end()), v.end()); };
  uniq(cores);
  uniq(nodes);
  uniq(socks);
  if ((int)nodes.size() > kMaxNumaNodes || (int)socks.size() > kMaxNumaNodes)
    KS_FAIL(ctx, KS_EUNSUPPORTED, "cpu topology %d: more than %d NUMA nodes or sockets", ti, kMaxNumaNodes);
  if (socks.size() > 12)
    KS_FAIL(ctx, KS_EUNSUPPORTED, "cpu topology %d: more than 12 sockets (Go's sort order is only stable up to 12)", ti);
  auto idx = [](const std::vector<int32_t>& v, int32_t x) { return (int)(std::lower_bound(v.begin(), v.end(), x) - v.begin()); };
  std::vector<int> core_n(cores.size(), -1), core_s(cores.size(), -1), node_s(nodes.size(), -1), core_cnt(cores.size(), 0);
  for (int c = 0; c < nc; ++c) {
    const int k = idx(cores, in.core[c]), nn = idx(nodes, in.numa_node[c]), ss = idx(socks, in.socket[c]);
    t.core_of[c] = (uint8_t)k;
    t.node_of[c] = (uint8_t)nn;
    t.sock_of[c] = (uint8_t)ss;
    if ((core_n[k] >= 0 && core_n[k] != nn) || (core_s[k] >= 0 && core_s[k] != ss) || (node_s[nn] >= 0 && node_s[nn] != ss))
      KS_FAIL(ctx, KS_EUNSUPPORTED, "cpu topology %d: a core spans NUMA nodes / sockets or a NUMA node spans sockets", ti);
    core_n[k] = nn;
    core_s[k] = ss;
    node_s[nn] = ss;
    if (++core_cnt[k] > 8) KS_FAIL(ctx, KS_EUNSUPPORTED, "cpu topology %d: more than 8 CPUs per core", ti);
    cs_add(t.core_mask[k], c);
    cs_add(t.node_mask[nn], c);
    cs_add(t.sock_mask[ss], c);
    cs_add(t.all, c);
  }
  for (size_t k = 0; k < cores.size(); ++k) {
    t.core_node[k] = (uint8_t)core_n[k];
    t.core_sock[k] = (uint8_t)core_s[k];
  }
  for (size_t nn = 0; nn < nodes.size(); ++nn) t.node_sock[nn] = (uint8_t)node_s[nn];
  // CPUTopologyBuilder counts (cpu_topology.go:45-70): cores are distinct per (socket, node, core)
  std::vector<std::tuple<int, int, int>> trip;
  std::vector<std::pair<int, int>> pairs;
  for (int c = 0; c < nc; ++c) {
    trip.emplace_back(in.socket[c], in.numa_node[c], in.core[c]);
    pairs.emplace_back(in.socket[c], in.numa_node[c]);
  }
  std::sort(trip.begin(), trip.end());
  trip.erase(std::unique(trip.begin(), trip.end()), trip.end());
  std::sort(pairs.begin(), pairs.end());
  pairs.erase(std::unique(pairs.begin(), pairs.end()), pairs.end());
  t.ncpus = nc;
  t.ncores = (int32_t)cores.size();
  t.nnodes = (int32_t)nodes.size();
  t.nsockets = (int32_t)socks.size();
  if ((int)trip.size() != t.ncores || (int)pairs.size() != t.nnodes)
    KS_FAIL(ctx, KS_EUNSUPPORTED, "cpu topology %d: core / NUMA ids are not unique across sockets", ti);
  t.cpc = nc / t.ncores;
  t.cpn = nc / t.nnodes;
  t.cps = nc / t.nsockets;
  return KS_OK;
}

// One node's CPU state from row i of st (validated against topology table tt): topology index, CPU sets, the
// CPUs available to cpuset pods and |allocated| (the cpuset millicores of filterAmplifiedCPUs / 1000).
static int cpu_encode_row(ks_ctx* ctx, const ks_cpu_state_cols* st, int64_t i, int64_t node, int32_t ntopo,
                          const std::vector<CpuTopo>& tt, int32_t& tid, CpuSet& al, CpuSet& xp, CpuSet& xn, CpuSet& rs,
                          int32_t& freec, int32_t& ncpu) {
  const int32_t ti = st->topology[i];
  if (ti < -1 || ti >= ntopo) KS_FAIL(ctx, KS_EINVAL, "node %lld: cpu topology %d out of range", (long long)node, ti);
  auto rd = [&](const uint64_t* p) {
    CpuSet c = cs_zero();
    if (p) memcpy(c.w, p + i * kCpuW, sizeof(c.w));
    return c;
  };
  al = rd(st->allocated);
  xp = rd(st->excl_pcpu);
  xn = rd(st->excl_numa);
  rs = rd(st->reserved);
  tid = ti;
  freec = -1;
  if (ti >= 0) {
    const CpuSet& all = tt[ti].all;
    if (cs_count(cs_andnot(cs_or(cs_or(al, xp), cs_or(xn, rs)), all)) != 0)
      KS_FAIL(ctx, KS_EINVAL, "node %lld: CPU set outside its topology", (long long)node);
    if (cs_count(cs_andnot(cs_or(xp, xn), al)) != 0 || cs_count(cs_and(xp, xn)) != 0)
      KS_FAIL(ctx, KS_EINVAL, "node %lld: exclusive CPU sets must be disjoint subsets of allocated", (long long)node);
    freec = cs_count(cs_andnot(all, cs_or(al, rs)));
  } else if (cs_count(al) != 0) {
    KS_FAIL(ctx, KS_EINVAL, "node %lld: allocated CPUs without a topology", (long long)node);
  }
  ncpu = cs_count(al);
  return KS_OK;
}

int ks_load_cpu_state(ks_ctx* ctx, const ks_cpu_topology* topos, int32_t ntopo, const ks_cpu_state_cols* st) {
  if (!ctx || ntopo < 0 || (ntopo > 0 && !topos) || !st || !st->topology || !st->allocated)
    return ctx ? (ctx->err = "ks_load_cpu_state: bad args", KS_EINVAL) : KS_EINVAL;
  if (!ctx->node_blob) KS_FAIL(ctx, KS_ESTATE, "ks_load_cpu_state before ks_load_nodes");
  if (!ctx->cfg.numa.enable) KS_FAIL(ctx, KS_ESTATE, "ks_load_cpu_state: the NodeNUMAResource plugin is not enabled");
  HIPCHK(ctx, hipSetDevice(ctx->device));
  const int64_t n = ctx->n, np = ctx->npad;
  std::vector<CpuTopo> tt((size_t)std::max(ntopo, 1));
  std::vector<int32_t> cpc;
  std::vector<int8_t> dense((size_t)std::max(ntopo, 1), 1);
  for (int32_t i = 0; i < ntopo; ++i) {
    if (int rc = build_cpu_topo(ctx, topos[i], i, tt[i]); rc != KS_OK) return rc;
    cpc.push_back(tt[i].cpc);
    int32_t mx = 0;
    for (int c = 0; c < topos[i].ncpus; ++c) mx = std::max(mx, topos[i].numa_node[c]);
    dense[(size_t)i] = mx + 1 == tt[i].nnodes;  // NUMA ids 0..nnodes-1: topology index == NUMA id
  }
  std::vector<int32_t> tid((size_t)np, -1), freec((size_t)np, -1), ncpu((size_t)np, 0);
  std::vector<CpuSet> al((size_t)np, cs_zero()), xp((size_t)np, cs_zero()), xn((size_t)np, cs_zero()), rs((size_t)np, cs_zero());
  for (int64_t i = 0; i < n; ++i)
    if (int rc = cpu_encode_row(ctx, st, i, i, ntopo, tt, tid[i], al[i], xp[i], xn[i], rs[i], freec[i], ncpu[i]); rc != KS_OK)
      return rc;
  dev_free(ctx->cpu_blob);
  ctx->cpu_loaded = false;
  const size_t tb = align16(tt.size() * sizeof(CpuTopo)), ib = align16((size_t)np * 4), sb = (size_t)np * sizeof(CpuSet);
  if (dev_alloc(ctx, &ctx->cpu_blob, tb + ib + sb * 7) != KS_OK) return KS_ENOMEM;
  char* b = (char*)ctx->cpu_blob;
  DevCpu& c = ctx->cpu;
  c.topo = (const CpuTopo*)b;
  HIPCHK(ctx, hipMemcpyAsync(b, tt.data(), tt.size() * sizeof(CpuTopo), hipMemcpyHostToDevice, ctx->stream));
  b += tb;
  c.topo_id = (const int32_t*)b;
  HIPCHK(ctx, hipMemcpyAsync(b, tid.data(), (size_t)np * 4, hipMemcpyHostToDevice, ctx->stream));
  b += ib;
  CpuSet* sets[4] = {nullptr, nullptr, nullptr, nullptr};
  const std::vector<CpuSet>* srcs[4] = {&al, &xp, &xn, &rs};
  for (int q = 0; q < 4; ++q) {
    sets[q] = (CpuSet*)b;
    HIPCHK(ctx, hipMemcpyAsync(b, srcs[q]->data(), sb, hipMemcpyHostToDevice, ctx->stream));
    b += sb;
  }
  c.allocated = sets[0];
  c.excl_pcpu = sets[1];
  c.excl_numa = sets[2];
  c.reserved = sets[3];
  ctx->cpu_ckpt = (CpuSet*)b;  // 3 x [npad]
  HIPCHK(ctx, hipMemcpyAsync(ctx->cpu_ckpt, c.allocated, sb * 3, hipMemcpyDeviceToDevice, ctx->stream));
  c.npad = np;
  c.ntopo = ntopo;
  HIPCHK(ctx, hipMemcpyAsync(ctx->d.cpu_free, freec.data(), (size_t)np * 4, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(ctx, hipMemcpyAsync(ctx->d.numa_cpus, ncpu.data(), (size_t)np * 4, hipMemcpyHostToDevice, ctx->stream));
  if (upload_prep_nodes(ctx) != KS_OK) return KS_EHIP;  // re-derive the cpuset millicores and offsets
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  ctx->cpu_cpc = cpc;
  ctx->cpu_loaded = true;
  ctx->h_topos = tt;
  ctx->h_topo_dense = dense;
  ctx->h_cpu_nn.assign((size_t)n, 0);
  for (int64_t i = 0; i < n; ++i)
    if (const int32_t ti = tid[(size_t)i]; ti >= 0) ctx->h_cpu_nn[(size_t)i] = dense[(size_t)ti] ? (int8_t)tt[(size_t)ti].nnodes : (int8_t)-1;
  if (int rc = numa_refresh_free(ctx); rc != KS_OK) return rc;
  if (int rc = cores_refresh(ctx); rc != KS_OK) return rc;
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  return KS_OK;
}

int ks_read_cpu_state(ks_ctx* ctx, uint64_t* allocated, uint64_t* excl_pcpu, uint64_t* excl_numa) {
  if (!ctx) return KS_EINVAL;
  if (!ctx->cpu_loaded) return KS_OK;
  const size_t n = (size_t)ctx->n;
  uint64_t* outs[3] = {allocated, excl_pcpu, excl_numa};
  const CpuSet* srcs[3] = {ctx->cpu.allocated, ctx->cpu.excl_pcpu, ctx->cpu.excl_numa};
  for (int q = 0; q < 3; ++q)
    if (outs[q] && n) HIPCHK(ctx, hipMemcpyAsync(outs[q], srcs[q], n * sizeof(CpuSet), hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  return KS_OK;
}

int ks_fetch_cpusets(ks_ctx* ctx, uint64_t* out, int32_t p) {
  if (!ctx || (p > 0 && !out) || p < 0) return ctx ? (ctx->err = "ks_fetch_cpusets: bad args", KS_EINVAL) : KS_EINVAL;
  if (p > ctx->np) KS_FAIL(ctx, KS_EINVAL, "ks_fetch_cpusets: %d pods requested, %d scheduled", p, ctx->np);
  if (p > 0 && ctx->cpusets_clobbered) KS_FAIL(ctx, KS_ESTATE, "ks_fetch_cpusets: a ks_assume since the last schedule overwrote them");
  if (p == 0) return KS_OK;
  if (!ctx->cpuset_out || ctx->cpuset_cap < p) {
    memset(out, 0, (size_t)p * sizeof(CpuSet));
    return KS_OK;
  }
  HIPCHK(ctx, hipMemcpyAsync(out, ctx->cpuset_out, (size_t)p * sizeof(CpuSet), hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  return KS_OK;
}

// NUMA nodes' available CPUs from the CPU state (numa_free_kernel); zero without a loaded CPU state
static int numa_refresh_free(ks_ctx* ctx) {
  if (!ctx->numa_blob) return KS_OK;
  const size_t np = (size_t)ctx->npad;
  if (!ctx->cpu_loaded) {
    HIPCHK(ctx, hipMemsetAsync(ctx->nv.free, 0, (size_t)kNumaDev * np * 4, ctx->stream));
    return KS_OK;
  }
  // the per-NUMA cpuset takes index the topology's NUMA nodes by NUMA id, and a cpu-bind pod admitted with a nil
  // affinity (single NUMA node) takes from NUMA node 0: the CPU topology's NUMA ids are 0..m-1 with m <= the count
  for (int64_t i = 0; i < ctx->n && i < (int64_t)ctx->h_numa_k.size() && i < (int64_t)ctx->h_cpu_nn.size(); ++i) {
    const int k = ctx->h_numa_k[(size_t)i], m = ctx->h_cpu_nn[(size_t)i];
    if (k > 0 && m != 0 && (m < 0 || m > k))
      KS_FAIL(ctx, KS_EUNSUPPORTED, "node %lld: NUMA-policy node whose CPU topology NUMA ids are not 0..m-1 with m <= %d",
              (long long)i, k);
  }
  if (ctx->n > 0)
    hipLaunchKernelGGL(numa_free_kernel, dim3((unsigned)((ctx->n + 255) / 256)), dim3(256), 0, ctx->stream, ctx->cpu, ctx->nv,
                       ctx->n);
  HIPCHK(ctx, hipGetLastError());
  // a load re-bases the checkpoint (as the CPU state's own checkpoint is re-based by ks_load_cpu_state)
  char* ck_free = ctx->numa_ckpt + ((char*)ctx->nv.free - (char*)ctx->nv.used);
  HIPCHK(ctx, hipMemcpyAsync(ck_free, ctx->nv.free, (size_t)kNumaDev * np * 4, hipMemcpyDeviceToDevice, ctx->stream));
  return KS_OK;
}

// DeviceShare as a hint provider on NUMA-policy nodes: its hint masks range over the device topology's NUMA nodes,
// which must be NUMA nodes of the node (ids < its NUMA count), at most kDevHintIds of them, on nodes with at most
// kDevHintIds NUMA nodes (this bounds the merge's cartesian product, ks_numa.h).
static int check_dev_numa(ks_ctx* ctx) {
  if (!ctx->cfg.deviceshare.enable || ctx->h_numa_k.empty() || ctx->h_dev_ids.empty()) return KS_OK;
  for (int64_t i = 0; i < ctx->n; ++i) {
    const int k = ctx->h_numa_k[(size_t)i];
    const uint32_t ids = ctx->h_dev_ids[(size_t)i];
    if (k == 0 || ids == 0) continue;
    if (k > kDevHintIds || __builtin_popcount(ids) > kDevHintIds || (ids >> k) != 0)
      KS_FAIL(ctx, KS_EUNSUPPORTED,
              "node %lld: DeviceShare NUMA hints need the devices on at most %d NUMA nodes of a node with at most %d "
              "(%d NUMA nodes, device NUMA ids 0x%x)", (long long)i, kDevHintIds, kDevHintIds, k, ids);
  }
  return KS_OK;
}

// NUMA node resources of the policy nodes; nc == nullptr installs an empty table (every policy node
// then reports "missing NUMA resources", as the reference does without a NodeResourceTopology).
// Layout: count | total | mutable {used, off, cs, free, present} | checkpoint copy of the mutable block.
static size_t numa_mut_bytes(size_t np) {
  constexpr int K = kNumaDev;
  return 2 * K * np * 8 + K * np * 8 + 2 * K * np * 4 + align16(np * 4);
}

// One node's NUMA-node table words (ks_numa.h layout): row r of nc describes node `node` (numa_flags f, cpu
// amplification ratio).  Only NUMA-policy nodes carry resources; the policy-None path never reads them.
struct NumaRow {
  int32_t cnt = 0;
  uint32_t pres = 0;
  int64_t tot[2 * kNumaDev] = {}, used[2 * kNumaDev] = {}, off[kNumaDev] = {};
  int32_t cs[kNumaDev] = {};
};
static int numa_encode(ks_ctx* ctx, const ks_numa_node_cols* nc, int64_t r, int64_t node, uint32_t f, double ratio,
                       NumaRow& w) {
  constexpr int K = kNumaDev;
  w = NumaRow{};
  const uint32_t pol = (f >> KS_NUMA_POLICY_SHIFT) & 3u;
  const int32_t c = nc->count[r];
  if (c < 0 || c > KS_MAX_NUMA) KS_FAIL(ctx, KS_EINVAL, "node %lld: NUMA node count %d", (long long)node, c);
  if (pol == 0) return KS_OK;
  if (c > K) KS_FAIL(ctx, KS_EUNSUPPORTED, "node %lld: %d NUMA nodes with a NUMA policy (the device evaluates up to %d)", (long long)node, c, K);
  w.cnt = c;
  for (int k = 0; k < c; ++k) {
    const size_t o = (size_t)r * KS_MAX_NUMA + k;
    const int64_t ac = nc->alloc_cpu ? nc->alloc_cpu[o] : 0, am = nc->alloc_memory ? nc->alloc_memory[o] : 0;
    const int64_t uc = nc->used_cpu ? nc->used_cpu[o] : 0, um = nc->used_memory ? nc->used_memory[o] : 0;
    const int32_t cpus = nc->cpuset_cpus ? nc->cpuset_cpus[o] : 0;
    const int64_t cs = (int64_t)cpus * 1000;
    const int64_t lim = (int64_t)1 << 50;
    if (ac < 0 || am < 0 || uc < 0 || um < 0 || cs < 0 || ac > lim || am > lim || uc > lim || um > lim || cs > lim)
      KS_FAIL(ctx, KS_EINVAL, "node %lld NUMA %d: quantity out of range", (long long)node, k);
    // amplifyNUMANodeResources / extension.Amplify: int64(math.Ceil(float64(v) * ratio)) for ratio > 1
    w.tot[0 * K + k] = ratio > 1.0 ? (int64_t)std::ceil((double)ac * ratio) : ac;
    w.tot[1 * K + k] = am;
    w.used[0 * K + k] = uc;
    w.used[1 * K + k] = um;
    w.off[k] = ratio > 1.0 ? (int64_t)std::ceil((double)cs * ratio) - cs : 0;
    w.cs[k] = cpus;
    const bool present = nc->used_present ? nc->used_present[o] != 0 : (uc != 0 || um != 0);
    if (present) w.pres |= 1u << k;
  }
  return KS_OK;
}

static int numa_install(ks_ctx* ctx, const ks_numa_node_cols* nc, const uint32_t* flags_h, const double* ratio_h) {
  const size_t np = (size_t)ctx->npad;
  constexpr int K = kNumaDev;
  const size_t o_cnt = 0, o_tot = align16(np * 4), o_used = o_tot + 2 * K * np * 8, o_off = o_used + 2 * K * np * 8,
               o_cs = o_off + K * np * 8, o_free = o_cs + K * np * 4, o_pres = o_free + K * np * 4,
               o_ck = o_pres + align16(np * 4), bytes = o_ck + numa_mut_bytes(np);
  std::vector<char> h(bytes, 0);
  int32_t* cnt = (int32_t*)(h.data() + o_cnt);
  int64_t* tot = (int64_t*)(h.data() + o_tot);
  int64_t* used = (int64_t*)(h.data() + o_used);
  int64_t* off = (int64_t*)(h.data() + o_off);
  int32_t* csv = (int32_t*)(h.data() + o_cs);
  uint32_t* pres = (uint32_t*)(h.data() + o_pres);
  ctx->h_numa_k.assign((size_t)ctx->n, 0);
  for (int64_t i = 0; nc && i < ctx->n; ++i) {
    NumaRow w;
    if (int rc = numa_encode(ctx, nc, i, i, flags_h[i], ratio_h ? ratio_h[i] : 0.0, w); rc != KS_OK) return rc;
    cnt[i] = w.cnt;
    ctx->h_numa_k[(size_t)i] = (int8_t)w.cnt;
    pres[i] = w.pres;
    for (int k = 0; k < K; ++k) {
      for (int q = 0; q < 2; ++q) {
        tot[(size_t)(q * K + k) * np + i] = w.tot[q * K + k];
        used[(size_t)(q * K + k) * np + i] = w.used[q * K + k];
      }
      off[(size_t)k * np + i] = w.off[k];
      csv[(size_t)k * np + i] = w.cs[k];
    }
  }
  dev_free(ctx->numa_blob);
  if (dev_alloc(ctx, &ctx->numa_blob, bytes) != KS_OK) return KS_ENOMEM;
  char* b = (char*)ctx->numa_blob;
  HIPCHK(ctx, hipMemcpyAsync(b, h.data(), bytes, hipMemcpyHostToDevice, ctx->stream));
  DevNuma& v = ctx->nv;
  v.count = (const int32_t*)(b + o_cnt);
  v.total = (const int64_t*)(b + o_tot);
  v.used = (int64_t*)(b + o_used);
  v.off = (int64_t*)(b + o_off);
  v.cs = (int32_t*)(b + o_cs);
  v.free = (int32_t*)(b + o_free);
  v.present = (uint32_t*)(b + o_pres);
  v.flags = ctx->d.numa_flags;
  v.npad = ctx->npad;
  ctx->numa_ckpt = b + o_ck;
  HIPCHK(ctx, hipMemcpyAsync(ctx->dnv, &v, sizeof(DevNuma), hipMemcpyHostToDevice, ctx->stream));
  if (int rc = numa_refresh_free(ctx); rc != KS_OK) return rc;
  HIPCHK(ctx, hipMemcpyAsync(ctx->numa_ckpt, v.used, numa_mut_bytes(np), hipMemcpyDeviceToDevice, ctx->stream));
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  return check_dev_numa(ctx);
}

int ks_load_numa_nodes(ks_ctx* ctx, const ks_numa_node_cols* nc) {
  if (!ctx || !nc || !nc->count) return ctx ? (ctx->err = "ks_load_numa_nodes: bad args", KS_EINVAL) : KS_EINVAL;
  if (!ctx->node_blob) KS_FAIL(ctx, KS_ESTATE, "ks_load_numa_nodes before ks_load_nodes");
  if (!ctx->cfg.numa.enable) KS_FAIL(ctx, KS_ESTATE, "ks_load_numa_nodes: the NodeNUMAResource plugin is not enabled");
  HIPCHK(ctx, hipSetDevice(ctx->device));
  const size_t n = (size_t)ctx->n;
  std::vector<uint32_t> flags(n ? n : 1);
  std::vector<double> ratio(n ? n : 1);
  if (n) {
    HIPCHK(ctx, hipMemcpyAsync(flags.data(), ctx->d.numa_flags, n * 4, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(ratio.data(), ctx->d.numa_ratio, n * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  }
  return numa_install(ctx, nc, flags.data(), ratio.data());
}

// NodeResourceTopology / NodeAllocation changes of m nodes (topology_eventhandler.go, node_allocation.go): row i
// of rows ([i * KS_MAX_NUMA + k]) replaces node idx[i]'s NUMA-node resources, allocated resources and cpuset CPUs;
// the available CPUs per NUMA node follow from the CPU state (numa_refresh_free).
static int scatter_words(ks_ctx* ctx, void* dst, size_t elem, int64_t rs, int64_t cs, int32_t W,
                         const std::vector<int32_t>& idx, const void* src);
static int check_idx(ks_ctx* ctx, const int32_t* idx, int64_t m, int64_t lim, const char* what, std::vector<int32_t>& out);

int ks_update_numa_nodes(ks_ctx* ctx, const int32_t* idx, const ks_numa_node_cols* rows, int64_t m) {
  if (!ctx || !rows || m < 0 || (m > 0 && (!idx || !rows->count)))
    return ctx ? (ctx->err = "ks_update_numa_nodes: bad args", KS_EINVAL) : KS_EINVAL;
  if (!ctx->numa_blob) KS_FAIL(ctx, KS_ESTATE, "ks_update_numa_nodes: no NUMA-node table (no node has a NUMA policy)");
  std::vector<int32_t> ix;
  if (int rc = check_idx(ctx, idx, m, ctx->n, "ks_update_numa_nodes", ix); rc != KS_OK) return rc;
  if (m == 0) return KS_OK;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  const size_t n = (size_t)ctx->n;
  std::vector<uint32_t> flags(n);
  std::vector<double> ratio(n);
  HIPCHK(ctx, hipMemcpyAsync(flags.data(), ctx->d.numa_flags, n * 4, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(ctx, hipMemcpyAsync(ratio.data(), ctx->d.numa_ratio, n * 8, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  constexpr int K = kNumaDev;
  std::vector<int32_t> cnt((size_t)m), cs((size_t)m * K);
  std::vector<uint32_t> pres((size_t)m);
  std::vector<int64_t> tot((size_t)m * 2 * K), used((size_t)m * 2 * K), off((size_t)m * K);
  for (int64_t i = 0; i < m; ++i) {
    const int32_t node = ix[(size_t)i];
    NumaRow w;
    if (int rc = numa_encode(ctx, rows, i, node, flags[(size_t)node], ratio[(size_t)node], w); rc != KS_OK) return rc;
    cnt[(size_t)i] = w.cnt;
    pres[(size_t)i] = w.pres;
    // word-major [w][m] (scatter_words)
    for (int q = 0; q < 2 * K; ++q) {
      tot[(size_t)q * m + i] = w.tot[q];
      used[(size_t)q * m + i] = w.used[q];
    }
    for (int q = 0; q < K; ++q) {
      off[(size_t)q * m + i] = w.off[q];
      cs[(size_t)q * m + i] = w.cs[q];
    }
  }
  const int64_t np = ctx->npad;
  DevNuma& v = ctx->nv;
  if (scatter_words(ctx, (void*)v.count, 4, 1, np, 1, ix, cnt.data()) != KS_OK ||
      scatter_words(ctx, (void*)v.present, 4, 1, np, 1, ix, pres.data()) != KS_OK ||
      scatter_words(ctx, (void*)v.total, 8, 1, np, 2 * K, ix, tot.data()) != KS_OK ||
      scatter_words(ctx, (void*)v.used, 8, 1, np, 2 * K, ix, used.data()) != KS_OK ||
      scatter_words(ctx, (void*)v.off, 8, 1, np, K, ix, off.data()) != KS_OK ||
      scatter_words(ctx, (void*)v.cs, 4, 1, np, K, ix, cs.data()) != KS_OK)
    return KS_EHIP;
  for (int64_t i = 0; i < m; ++i) ctx->h_numa_k[(size_t)ix[(size_t)i]] = (int8_t)cnt[(size_t)i];
  if (int rc = numa_refresh_free(ctx); rc != KS_OK) return rc;
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  return check_dev_numa(ctx);
}

int ks_read_numa_nodes(ks_ctx* ctx, int64_t* used_cpu, int64_t* used_memory) {
  if (!ctx) return KS_EINVAL;
  const size_t n = (size_t)ctx->n, np = (size_t)ctx->npad;
  std::vector<int64_t> u(2 * kNumaDev * (np ? np : 1), 0);
  std::vector<uint32_t> pr(np ? np : 1, 0);
  if (ctx->numa_blob && n) {
    HIPCHK(ctx, hipMemcpyAsync(u.data(), ctx->nv.used, u.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  }
  int64_t* outs[2] = {used_cpu, used_memory};
  for (int r = 0; r < 2; ++r)
    if (outs[r])
      for (size_t i = 0; i < n; ++i)
        for (int k = 0; k < KS_MAX_NUMA; ++k)
          outs[r][i * KS_MAX_NUMA + k] = k < kNumaDev ? u[((size_t)r * kNumaDev + k) * np + i] : 0;
  return KS_OK;
}

// rows of rc appended to the host mirror (NULL columns as rsv_install reads them; the reserve pod's NonZeroRequested
// resolved the same way)
static void rsv_mirror_append(ks_ctx* ctx, const ks_reservation_cols* rc, int32_t nr) {
  auto& M = ctx->rmir;
  for (int32_t r = 0; r < nr; ++r) {
    M.node.push_back(rc->node[r]);
    M.cls.push_back(rc->owner_classes[r]);
    M.flags.push_back(rc->flags ? rc->flags[r] : 0u);
    M.policy.push_back(rc->policy ? rc->policy[r] : 0u);
    M.key_mask.push_back(rc->key_mask[r]);
    M.order.push_back(rc->order ? rc->order[r] : 0);
    M.assigned.push_back(rc->assigned ? rc->assigned[r] : 0);
    for (int d = 0; d < kRsvDims; ++d) {
      M.alloc[d].push_back(rc->allocatable[d] ? rc->allocatable[d][r] : 0);
      M.allocd[d].push_back(rc->allocated[d] ? rc->allocated[d][r] : 0);
    }
    const uint32_t keys = rc->key_mask[r];
    M.rnz_cpu.push_back(rc->reserve_nonzero_milli_cpu ? rc->reserve_nonzero_milli_cpu[r]
                                                      : ((keys & 1u) ? M.alloc[0].back() : kDefaultMilliCPU));
    M.rnz_mem.push_back(rc->reserve_nonzero_memory ? rc->reserve_nonzero_memory[r]
                                                   : ((keys & 2u) ? M.alloc[1].back() : kDefaultMemory));
    for (int w = 0; w < KS_DEV_WORDS; ++w) {
      M.dal.push_back(rc->dev_allocatable ? rc->dev_allocatable[(size_t)r * KS_DEV_WORDS + w] : 0);
      M.dald.push_back(rc->dev_allocatable && rc->dev_allocated ? rc->dev_allocated[(size_t)r * KS_DEV_WORDS + w] : 0);
    }
    M.live.push_back(1);
  }
}

int ks_load_reservations(ks_ctx* ctx, const ks_reservation_cols* rsv, int32_t r) {
  if (!ctx || r < 0 || (r > 0 && !rsv)) return ctx ? (ctx->err = "ks_load_reservations: bad args", KS_EINVAL) : KS_EINVAL;
  if (!ctx->node_blob) KS_FAIL(ctx, KS_ESTATE, "ks_load_reservations before ks_load_nodes");
  if (!ctx->cfg.reservation.enable) KS_FAIL(ctx, KS_ESTATE, "ks_load_reservations: the Reservation plugin is not enabled");
  HIPCHK(ctx, hipSetDevice(ctx->device));
  if (int rc = rsv_install(ctx, rsv, r); rc != KS_OK) return rc;
  ctx->rmir = ks_ctx::RsvMirror{};
  rsv_mirror_append(ctx, rsv, r);
  return KS_OK;
}

// Reservation informer events between scheduling cycles (reservationCache.updateReservation /
// deleteReservation, reservation/cache.go:104-216): rows are added to or removed from the host mirror, the
// device's Allocated / assigned counts are read back into it, and the table is re-installed (the node
// columns' base restore follows, rsv_install).  Caller row numbers stay stable: added rows get the next numbers,
// deleted rows leave gaps.
static int rsv_reinstall(ks_ctx* ctx) {
  auto& M = ctx->rmir;
  const int32_t total = (int32_t)M.node.size();
  if (ctx->rsv_blob && ctx->rsv_live > 0) {
    // the device's Allocated / assigned (commits since the last install) into the mirror
    const size_t m = (size_t)ctx->rv.nr;
    std::vector<int64_t> ad(kRsvDims * m);
    std::vector<int32_t> as(m);
    HIPCHK(ctx, hipMemcpyAsync(ad.data(), ctx->rv.allocd, ad.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(as.data(), ctx->rv.assigned, m * 4, hipMemcpyDeviceToHost, ctx->stream));
    std::vector<int64_t> dd((size_t)kDevQW * m);
    HIPCHK(ctx, hipMemcpyAsync(dd.data(), ctx->rv.dald, dd.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    for (int32_t i = 0; i < ctx->rsv_live; ++i) {
      const int32_t r = ctx->rsv_perm[(size_t)i];
      for (int d = 0; d < kRsvDims; ++d) M.allocd[d][(size_t)r] = ad[(size_t)d * m + i];
      M.assigned[(size_t)r] = as[(size_t)i];
      for (int w = 0; w < kDevQW; ++w) M.dald[(size_t)r * KS_DEV_WORDS + w] = dd[(size_t)w * m + i];
    }
  }
  std::vector<int32_t> caller;
  for (int32_t r = 0; r < total; ++r)
    if (M.live[(size_t)r]) caller.push_back(r);
  const int32_t nl = (int32_t)caller.size();
  auto pick64 = [&](const std::vector<int64_t>& v) {
    std::vector<int64_t> o((size_t)nl);
    for (int32_t i = 0; i < nl; ++i) o[(size_t)i] = v[(size_t)caller[(size_t)i]];
    return o;
  };
  auto pick32 = [&](const auto& v) {
    std::vector<typename std::decay_t<decltype(v)>::value_type> o((size_t)nl);
    for (int32_t i = 0; i < nl; ++i) o[(size_t)i] = v[(size_t)caller[(size_t)i]];
    return o;
  };
  auto node = pick32(M.node), assigned = pick32(M.assigned);
  auto cls = pick32(M.cls);
  auto flags = pick32(M.flags), policy = pick32(M.policy), key_mask = pick32(M.key_mask);
  auto order = pick64(M.order), rnzc = pick64(M.rnz_cpu), rnzm = pick64(M.rnz_mem);
  std::vector<int64_t> alloc[kRsvDims], allocd[kRsvDims];
  ks_reservation_cols rc{};
  rc.node = node.data();
  rc.owner_classes = cls.data();
  rc.flags = flags.data();
  rc.policy = policy.data();
  rc.order = order.data();
  rc.key_mask = key_mask.data();
  rc.assigned = assigned.data();
  rc.reserve_nonzero_milli_cpu = rnzc.data();
  rc.reserve_nonzero_memory = rnzm.data();
  for (int d = 0; d < kRsvDims; ++d) {
    alloc[d] = pick64(M.alloc[d]);
    allocd[d] = pick64(M.allocd[d]);
    rc.allocatable[d] = alloc[d].data();
    rc.allocated[d] = allocd[d].data();
  }
  std::vector<int64_t> dal((size_t)nl * KS_DEV_WORDS), dald((size_t)nl * KS_DEV_WORDS);
  bool anyd = false;
  for (int32_t i = 0; i < nl; ++i)
    for (int w = 0; w < KS_DEV_WORDS; ++w) {
      dal[(size_t)i * KS_DEV_WORDS + w] = M.dal[(size_t)caller[(size_t)i] * KS_DEV_WORDS + w];
      dald[(size_t)i * KS_DEV_WORDS + w] = M.dald[(size_t)caller[(size_t)i] * KS_DEV_WORDS + w];
      anyd |= dal[(size_t)i * KS_DEV_WORDS + w] != 0;
    }
  if (anyd) {
    rc.dev_allocatable = dal.data();
    rc.dev_allocated = dald.data();
  }
  return rsv_install(ctx, &rc, nl, caller.data(), total);
}

int ks_add_reservations(ks_ctx* ctx, const ks_reservation_cols* rsv, int32_t r, int32_t* first_row) {
  if (!ctx || r < 0 || (r > 0 && !rsv)) return ctx ? (ctx->err = "ks_add_reservations: bad args", KS_EINVAL) : KS_EINVAL;
  if (!ctx->node_blob) KS_FAIL(ctx, KS_ESTATE, "ks_add_reservations before ks_load_nodes");
  if (!ctx->cfg.reservation.enable) KS_FAIL(ctx, KS_ESTATE, "ks_add_reservations: the Reservation plugin is not enabled");
  HIPCHK(ctx, hipSetDevice(ctx->device));
  const int32_t first = (int32_t)ctx->rmir.node.size();
  if (first_row) *first_row = first;
  if (r == 0) return KS_OK;
  const ks_ctx::RsvMirror saved = ctx->rmir;
  rsv_mirror_append(ctx, rsv, r);
  if (int rc = rsv_reinstall(ctx); rc != KS_OK) {
    ctx->rmir = saved;  // the previous table stays installed when validation refused the new rows
    return rc;
  }
  return KS_OK;
}

int ks_delete_reservations(ks_ctx* ctx, const int32_t* rows, int32_t m) {
  if (!ctx || m < 0 || (m > 0 && !rows)) return ctx ? (ctx->err = "ks_delete_reservations: bad args", KS_EINVAL) : KS_EINVAL;
  if (!ctx->cfg.reservation.enable) KS_FAIL(ctx, KS_ESTATE, "ks_delete_reservations: the Reservation plugin is not enabled");
  auto& M = ctx->rmir;
  for (int32_t i = 0; i < m; ++i)
    if (rows[i] < 0 || (size_t)rows[i] >= M.live.size() || !M.live[(size_t)rows[i]])
      KS_FAIL(ctx, KS_EINVAL, "ks_delete_reservations: row %d is not a loaded reservation", rows[i]);
  if (m == 0) return KS_OK;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  for (int32_t i = 0; i < m; ++i) M.live[(size_t)rows[i]] = 0;
  return rsv_reinstall(ctx);
}

int ks_read_reservations(ks_ctx* ctx, int64_t* allocated, int32_t* assigned) {
  if (!ctx) return KS_EINVAL;
  const int32_t nr = ctx->rsv_live;
  if (nr == 0 || !ctx->rsv_blob) return KS_OK;
  const size_t m = (size_t)ctx->rv.nr;
  std::vector<int64_t> ad(kRsvDims * m);
  std::vector<int32_t> as(m);
  HIPCHK(ctx, hipMemcpyAsync(ad.data(), ctx->rv.allocd, ad.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(ctx, hipMemcpyAsync(as.data(), ctx->rv.assigned, m * 4, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  for (int32_t i = 0; i < nr; ++i) {
    const int32_t r = ctx->rsv_perm[i];
    if (allocated)
      for (int d = 0; d < kRsvDims; ++d) allocated[(size_t)r * kRsvDims + d] = ad[(size_t)d * m + i];
    if (assigned) assigned[r] = as[i];
  }
  return KS_OK;
}

int ks_read_reservation_devices(ks_ctx* ctx, int64_t* dev_allocated) {
  if (!ctx) return KS_EINVAL;
  const int32_t nr = ctx->rsv_live;
  if (!dev_allocated || nr == 0 || !ctx->rsv_blob) return KS_OK;
  const size_t m = (size_t)ctx->rv.nr;
  std::vector<int64_t> dd((size_t)kDevQW * m);
  HIPCHK(ctx, hipMemcpyAsync(dd.data(), ctx->rv.dald, dd.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  for (int32_t i = 0; i < nr; ++i) {
    const int32_t r = ctx->rsv_perm[(size_t)i];
    for (int w = 0; w < KS_DEV_WORDS; ++w) dev_allocated[(size_t)r * KS_DEV_WORDS + w] = dd[(size_t)w * m + i];
  }
  return KS_OK;
}

int ks_update_nodes(ks_ctx* ctx, const int32_t* idx, const ks_node_cols* rows, int64_t m) {
  if (!ctx || !idx || !rows || m < 0) return ctx ? (ctx->err = "ks_update_nodes: bad args", KS_EINVAL) : KS_EINVAL;
  for (int64_t i = 0; ctx->cfg.numa.enable && rows->numa_flags && i < m; ++i)
    if (idx[i] >= 0 && (size_t)idx[i] < ctx->h_dev_held.size() && ctx->h_dev_held[(size_t)idx[i]] &&
        ((rows->numa_flags[i] >> KS_NUMA_POLICY_SHIFT) & 3u))
      KS_FAIL(ctx, KS_EUNSUPPORTED, "node %d: a NUMA topology policy on a node whose reservations hold devices", idx[i]);
  if (!ctx->node_blob) KS_FAIL(ctx, KS_ESTATE, "ks_update_nodes before ks_load_nodes");
  if (m == 0) return KS_OK;
  for (int64_t i = 0; i < m; ++i)
    if (idx[i] < 0 || idx[i] >= ctx->n) KS_FAIL(ctx, KS_EINVAL, "ks_update_nodes: idx[%lld]=%d out of range", (long long)i, idx[i]);
  if (ctx->rsv_based) {
    std::vector<int32_t> sorted(idx, idx + m);
    std::sort(sorted.begin(), sorted.end());
    if (std::adjacent_find(sorted.begin(), sorted.end()) != sorted.end())
      KS_FAIL(ctx, KS_EINVAL, "ks_update_nodes: duplicate node index with reservations loaded");
  }
  if (int rc = validate_nodes(ctx, rows, m); rc != KS_OK) return rc;
  if (ctx->cfg.topology.enable && (rows->topo_nkeys != ctx->topo_nkeys || rows->topo_nprops != ctx->topo_nprops ||
                                   rows->topo_ndomains > ctx->topo_ndom))
    KS_FAIL(ctx, KS_EINVAL, "ks_update_nodes: topology sizes differ from the loaded table's (%d keys, %d properties, "
            "%d domains)", ctx->topo_nkeys, ctx->topo_nprops, ctx->topo_ndom);
  std::vector<const void*> src = host_cols(ctx, rows, m);
  std::vector<void*> dst;
  std::vector<int32_t> widths;
  std::vector<size_t> offs;
  size_t bytes = 0;
  for (size_t i = 0; i < ctx->cols.size(); ++i) {
    if (!src[i]) continue;
    dst.push_back(*ctx->cols[i].dev);
    widths.push_back(ctx->cols[i].width);
    offs.push_back(bytes);
    bytes += ((size_t)m * ctx->cols[i].width + 15) / 16 * 16;
  }
  const size_t ncols = dst.size();
  const size_t meta = ncols * (sizeof(void*) * 2 + 4) + (size_t)m * 4 + 64;
  std::vector<char> host(bytes + meta);
  void* dbuf = nullptr;
  if (dev_alloc(ctx, &dbuf, bytes + meta) != KS_OK) return KS_ENOMEM;
  std::vector<const void*> srcdev(ncols);
  size_t j = 0;
  for (size_t i = 0; i < ctx->cols.size(); ++i) {
    if (!src[i]) continue;
    memcpy(host.data() + offs[j], src[i], (size_t)m * ctx->cols[i].width);
    srcdev[j] = (char*)dbuf + offs[j];
    ++j;
  }
  char* mp = host.data() + bytes;
  memcpy(mp, dst.data(), ncols * sizeof(void*));
  memcpy(mp + ncols * sizeof(void*), srcdev.data(), ncols * sizeof(void*));
  memcpy(mp + 2 * ncols * sizeof(void*), widths.data(), ncols * 4);
  const size_t idx_off = bytes + 2 * ncols * sizeof(void*) + ((ncols * 4 + 15) / 16) * 16;
  memcpy(host.data() + idx_off, idx, (size_t)m * 4);
  HIPCHK(ctx, hipMemcpyAsync(dbuf, host.data(), host.size(), hipMemcpyHostToDevice, ctx->stream));
  char* dm = (char*)dbuf + bytes;
  const int threads = 256;
  hipLaunchKernelGGL(scatter_rows_kernel, dim3((unsigned)((m + threads - 1) / threads)), dim3(threads), 0, ctx->stream,
                     (void* const*)dm, (const void* const*)(dm + ncols * sizeof(void*)),
                     (const int32_t*)(dm + 2 * ncols * sizeof(void*)), (int32_t)ncols,
                     (const int32_t*)((char*)dbuf + idx_off), m);
  HIPCHK(ctx, hipGetLastError());
  // the replaced rows are the reference's NodeInfo: add the reservation base restore again
  if (ctx->rsv_based && rsv_launch_base(ctx, (const int32_t*)((char*)dbuf + idx_off), m, +1, 0) != KS_OK) return KS_EHIP;
  if (upload_prep_nodes(ctx) != KS_OK) return KS_EHIP;
  for (int64_t i = 0; ctx->cfg.numa.enable && rows->numa_flags && i < m; ++i) {
    ctx->cpu_bind_labels |= ((rows->numa_flags[i] >> KS_NUMA_CPU_BIND_SHIFT) & 3u) != 0;
    if ((size_t)idx[i] < ctx->h_pol.size()) ctx->h_pol[(size_t)idx[i]] = ((rows->numa_flags[i] >> KS_NUMA_POLICY_SHIFT) & 3u) != 0;
  }
  // (the union only grows: a stale bit only withholds the fast path from a pod)
  for (int64_t i = 0; rows->taints_soft && i < m; ++i) ctx->soft_union |= rows->taints_soft[i];
  cores_mode(ctx);
  if (rows->numa_flags && cores_refresh(ctx) != KS_OK) return KS_EHIP;
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  (void)hipFree(dbuf);
  return KS_OK;
}

int ks_load_quotas(ks_ctx* ctx, const ks_quota_cols* qc, int32_t nq) {
  if (!ctx || !qc || nq < 0) return ctx ? (ctx->err = "ks_load_quotas: bad args", KS_EINVAL) : KS_EINVAL;
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  dev_free(ctx->quota_blob);
  const size_t rows = (size_t)(nq > 0 ? nq : 1);
  const size_t tbl = rows * KS_QUOTA_DIMS * 8;
  const size_t bytes = rows * 12 + 16 + tbl * 6;
  if (dev_alloc(ctx, &ctx->quota_blob, bytes) != KS_OK) return KS_ENOMEM;
  std::vector<char> h(bytes, 0);
  char* b = h.data();
  int32_t* parent = (int32_t*)b;
  uint32_t* lmask = (uint32_t*)(b + rows * 4);
  uint32_t* mmask = (uint32_t*)(b + rows * 8);
  const size_t toff = (rows * 12 + 15) / 16 * 16;
  int64_t* limit = (int64_t*)(b + toff);
  int64_t* used = limit + rows * KS_QUOTA_DIMS;
  int64_t* mn = used + rows * KS_QUOTA_DIMS;
  int64_t* np = mn + rows * KS_QUOTA_DIMS;
  for (int32_t i = 0; i < nq; ++i) {
    parent[i] = qc->parent ? qc->parent[i] : -1;
    if (parent[i] >= nq || parent[i] == i) KS_FAIL(ctx, KS_EINVAL, "quota %d: bad parent %d", i, parent[i]);
    lmask[i] = qc->limit_mask ? qc->limit_mask[i] : 0;
    mmask[i] = qc->min_mask ? qc->min_mask[i] : 0;
    for (int d = 0; d < KS_QUOTA_DIMS; ++d) {
      const size_t o = (size_t)i * KS_QUOTA_DIMS + d;
      limit[o] = qc->limit[d] ? qc->limit[d][i] : 0;
      used[o] = qc->used[d] ? qc->used[d][i] : 0;
      mn[o] = qc->min[d] ? qc->min[d][i] : 0;
      np[o] = qc->nonpreemptible_used[d] ? qc->nonpreemptible_used[d][i] : 0;
    }
  }
  // parent chains must terminate (no cycles)
  for (int32_t i = 0; i < nq; ++i) {
    int32_t cur = i, steps = 0;
    while (cur >= 0 && steps <= nq) cur = parent[cur], ++steps;
    if (cur >= 0) KS_FAIL(ctx, KS_EINVAL, "quota %d: parent chain has a cycle", i);
  }
  HIPCHK(ctx, hipMemcpyAsync(ctx->quota_blob, h.data(), bytes, hipMemcpyHostToDevice, ctx->stream));
  char* d = (char*)ctx->quota_blob;
  ctx->q.q = nq;
  ctx->q.parent = (int32_t*)d;
  ctx->q.limit_mask = (uint32_t*)(d + rows * 4);
  ctx->q.min_mask = (uint32_t*)(d + rows * 8);
  ctx->q.limit = (int64_t*)(d + toff);
  ctx->q.used = ctx->q.limit + rows * KS_QUOTA_DIMS;
  ctx->q.min = ctx->q.used + rows * KS_QUOTA_DIMS;
  ctx->q.npused = ctx->q.min + rows * KS_QUOTA_DIMS;
  ctx->quota_used_ckpt = ctx->q.npused + rows * KS_QUOTA_DIMS;
  ctx->quota_npused_ckpt = ctx->quota_used_ckpt + rows * KS_QUOTA_DIMS;
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  return KS_OK;
}

int ks_refresh_quota_runtime(ks_ctx* ctx, const ks_quota_tree* t, int32_t nq, int64_t* runtime, uint32_t* runtime_mask) {
  if (!ctx || !t || nq < 0) return ctx ? (ctx->err = "ks_refresh_quota_runtime: bad args", KS_EINVAL) : KS_EINVAL;
  if (nq == 0) return KS_OK;
  if (!t->parent || !t->max_mask) KS_FAIL(ctx, KS_EINVAL, "ks_quota_tree: parent and max_mask are required");
  const int D = KS_QUOTA_DIMS;
  // breadth-first layout: sibling groups contiguous, depth levels
  std::vector<std::vector<int32_t>> kids(nq + 1);  // kids[nq] = children of the root
  for (int32_t i = 0; i < nq; ++i) {
    const int32_t p = t->parent[i];
    if (p < -1 || p >= nq || p == i) KS_FAIL(ctx, KS_EINVAL, "quota %d: bad parent %d", i, p);
    kids[p < 0 ? nq : p].push_back(i);
  }
  std::vector<int32_t> order, level_off, grp_parent, grp_off, depth(nq, -1);
  order.reserve(nq);
  grp_parent.push_back(-1);
  grp_off.push_back(0);
  for (int32_t c : kids[nq]) order.push_back(c), depth[c] = 0;
  grp_off.push_back((int32_t)order.size());
  for (size_t i = 0; i < order.size(); ++i) {
    const int32_t q = order[i];
    if (kids[q].empty()) continue;
    grp_parent.push_back(q);
    for (int32_t c : kids[q]) order.push_back(c), depth[c] = depth[q] + 1;
    grp_off.push_back((int32_t)order.size());
  }
  if ((int32_t)order.size() != nq) KS_FAIL(ctx, KS_EINVAL, "ks_quota_tree: parent links form a cycle");
  int32_t nlevels = 0;
  for (int32_t q : order) nlevels = std::max(nlevels, depth[q] + 1);
  level_off.assign(nlevels + 1, 0);
  {
    // `order` is breadth-first, so depths are non-decreasing along it
    int32_t l = 0;
    for (int32_t i = 0; i < nq; ++i)
      while (depth[order[i]] >= l) level_off[l++] = i;
    while (l <= nlevels) level_off[l++] = nq;
  }
  const int32_t ngroups = (int32_t)grp_parent.size();
  uint32_t keys = 0;
  for (int32_t i = 0; i < nq; ++i) keys |= t->max_mask[i];
  keys &= (1u << D) - 1u;
  // pack: int64 tables first, then int32/u8 metadata
  const size_t tbl = (size_t)nq * D;
  std::vector<int64_t> h64(tbl * 6 + D, 0);
  int64_t* mx = h64.data();
  int64_t* mn = mx + tbl;
  int64_t* sw = mn + tbl;
  int64_t* gu = sw + tbl;
  int64_t* sr = gu + tbl;
  int64_t* rtout = sr + tbl;
  int64_t* tot = rtout + tbl;
  for (int32_t i = 0; i < nq; ++i)
    for (int d = 0; d < D; ++d) {
      const size_t o = (size_t)i * D + d;
      mx[o] = t->max[d] ? t->max[d][i] : 0;
      mn[o] = t->min[d] ? t->min[d][i] : 0;
      sw[o] = t->shared_weight[d] ? t->shared_weight[d][i] : mx[o];
      gu[o] = t->guaranteed[d] ? t->guaranteed[d][i] : 0;
      sr[o] = t->self_request[d] ? t->self_request[d][i] : 0;
      for (int64_t v : {mx[o], mn[o], sw[o], gu[o], sr[o]})
        if (v < 0 || v >= ((int64_t)1 << 56)) KS_FAIL(ctx, KS_EINVAL, "quota %d dim %d: value outside [0, 2^56)", i, d);
    }
  for (int d = 0; d < D; ++d) tot[d] = t->cluster_total[d];
  std::vector<int32_t> h32;
  auto put = [&](const std::vector<int32_t>& v) { size_t o = h32.size(); h32.insert(h32.end(), v.begin(), v.end()); return o; };
  const size_t o_order = put(order), o_lvl = put(level_off), o_gp = put(grp_parent), o_go = put(grp_off);
  const size_t o_par = put(std::vector<int32_t>(t->parent, t->parent + nq));
  std::vector<int32_t> mm(nq);
  for (int32_t i = 0; i < nq; ++i) mm[i] = (int32_t)t->max_mask[i];
  const size_t o_mm = put(mm);
  std::vector<int32_t> al(nq);
  for (int32_t i = 0; i < nq; ++i) al[i] = t->allow_lent ? (t->allow_lent[i] ? 1 : 0) : 1;
  const size_t o_al = h32.size();
  h32.resize(h32.size() + (nq + 3) / 4, 0);
  memcpy(h32.data() + o_al, std::vector<uint8_t>(al.begin(), al.end()).data(), nq);
  const size_t b64 = h64.size() * 8, b32 = h32.size() * 4;
  void* dbuf = nullptr;
  if (dev_alloc(ctx, &dbuf, b64 + b32) != KS_OK) return KS_ENOMEM;
  HIPCHK(ctx, hipMemcpyAsync(dbuf, h64.data(), b64, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(ctx, hipMemcpyAsync((char*)dbuf + b64, h32.data(), b32, hipMemcpyHostToDevice, ctx->stream));
  const int64_t* d64 = (const int64_t*)dbuf;
  const int32_t* d32 = (const int32_t*)((char*)dbuf + b64);
  QrtArgs qa;
  qa.n = nq;
  qa.ngroups = ngroups;
  qa.nlevels = nlevels;
  qa.keys = keys;
  qa.order = d32 + o_order;
  qa.level_off = d32 + o_lvl;
  qa.grp_parent = d32 + o_gp;
  qa.grp_off = d32 + o_go;
  qa.parent = d32 + o_par;
  qa.maxmask = (const uint32_t*)(d32 + o_mm);
  qa.allow = (const uint8_t*)(d32 + o_al);
  qa.mx = d64;
  qa.mn = d64 + tbl;
  qa.sw = d64 + 2 * tbl;
  qa.guar = d64 + 3 * tbl;
  qa.selfreq = d64 + 4 * tbl;
  qa.runtime = (int64_t*)d64 + 5 * tbl;
  qa.total = d64 + 6 * tbl;
  // one wave per dimension; as many dimensions per launch as LDS holds (3 x int64 per quota)
  const size_t per_dim = (size_t)nq * 3 * 8;
  int dims_per = (int)std::min<size_t>(D, (160 * 1024) / per_dim);
  if (dims_per < 1) {
    (void)hipFree(dbuf);
    KS_FAIL(ctx, KS_EUNSUPPORTED, "quota tree too large for the runtime kernel's LDS (%d quotas)", nq);
  }
  hipError_t e = hipFuncSetAttribute((const void*)quota_runtime_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)(per_dim * dims_per));
  for (int d0 = 0; e == hipSuccess && d0 < D; d0 += dims_per) {
    qa.dim0 = d0;
    qa.ndims = std::min(dims_per, D - d0);
    hipLaunchKernelGGL(quota_runtime_kernel, dim3(1), dim3(64 * qa.ndims), per_dim * qa.ndims, ctx->stream, qa);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpyAsync(rtout, qa.runtime, tbl * 8, hipMemcpyDeviceToHost, ctx->stream);
  // install as the admission limit of the loaded quota table (EnableRuntimeQuota)
  if (e == hipSuccess && ctx->quota_blob && ctx->q.q == nq) {
    e = hipMemcpyAsync(ctx->q.limit, qa.runtime, tbl * 8, hipMemcpyDeviceToDevice, ctx->stream);
    std::vector<uint32_t> lm(nq, keys);
    if (e == hipSuccess) e = hipMemcpyAsync(ctx->q.limit_mask, lm.data(), (size_t)nq * 4, hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  (void)hipFree(dbuf);
  if (e != hipSuccess) KS_FAIL(ctx, KS_EHIP, "ks_refresh_quota_runtime: %s", hipGetErrorString(e));
  if (runtime) memcpy(runtime, rtout, tbl * 8);
  if (runtime_mask)
    for (int32_t i = 0; i < nq; ++i) runtime_mask[i] = keys;
  return KS_OK;
}

// Pod staging area: the raw pod columns as the caller gave them (HBM) and the PodRec / result arrays built from
// them.  The schedule's own stage (ctx->st) is rebuilt into PodRec by prep_pods_kernel at the start of every
// ks_schedule_staged (PreFilter / EstimatePod work is part of the scheduling call); single-pod evaluation has its
// own stage (ctx->est) so it never disturbs staged pods.
static int ensure_stage(ks_ctx* ctx, PodStage& st, int32_t p) {
  if (p <= st.cap && st.blob) return KS_OK;
  dev_free(st.blob);
  st.cap = 0;
  const int32_t cap = std::max<int32_t>(p, 64);
  const size_t rec = (size_t)cap * sizeof(PodRec);
  const size_t res = ((size_t)cap * sizeof(ks_result) + 255) / 256 * 256;
  const size_t col8 = ((size_t)cap * 8 + 255) / 256 * 256;
  const size_t col4 = ((size_t)cap * 4 + 255) / 256 * 256;
  // stage: cpu mem eph nzcpu nzmem sc[4] la x6 gpu x3 rdma qreq[8] = 27 int64 cols; flags quota qmask rsv_class
  // cpu_bind joint(u8) = 6 x32
  const size_t pst = (size_t)cap * sizeof(PodStat);
  const size_t bytes = rec + pst + res + col8 * 27 + col4 * 7;
  if (dev_alloc(ctx, &st.blob, bytes) != KS_OK) return KS_ENOMEM;
  char* b = (char*)st.blob;
  st.recs = (PodRec*)b;
  b += rec;
  st.stat = (PodStat*)b;
  b += pst;
  st.results = (ks_result*)b;
  b += res;
  st.col8 = col8;
  st.col4 = col4;
  DevPodCols& s = st.cols;
  int64_t** c8[] = {&s.cpu, &s.mem, &s.eph, &s.nzcpu, &s.nzmem, &s.sc[0], &s.sc[1], &s.sc[2], &s.sc[3],
                    &s.la_req_cpu, &s.la_lim_cpu, &s.la_dflt_cpu, &s.la_req_mem, &s.la_lim_mem, &s.la_dflt_mem,
                    &s.gpu_core, &s.gpu_mem, &s.gpu_ratio, &s.rdma};
  for (int64_t** f : c8) {
    *f = (int64_t*)b;
    b += col8;
  }
  for (int d = 0; d < KS_QUOTA_DIMS; ++d) {
    st.pq.req[d] = (int64_t*)b;
    b += col8;
  }
  s.flags = (uint32_t*)b;
  b += col4;
  s.quota = (int32_t*)b;
  b += col4;
  st.pq.mask = (uint32_t*)b;
  b += col4;
  s.rsv_class = (int32_t*)b;
  b += col4;
  s.cpu_bind = (uint32_t*)b;
  b += col4;
  s.stat_dyn = (uint8_t*)b;
  b += col4;
  s.joint = (uint8_t*)b;
  st.cap = cap;
  return KS_OK;
}

// host columns -> the stage's HBM columns (async on the ctx stream)
// The column region of stage st for p <= kPackPods pods, packed on the host in the device layout (ensure_stage: 27
// int64 columns, then 7 x 32-bit ones, each st.col8 / st.col4 bytes apart) and copied once.
static int stage_cols_packed(ks_ctx* ctx, PodStage& st, const ks_pod_cols* pc, int32_t p) {
  const size_t bytes = st.col8 * 27 + st.col4 * 7;
  if (!st.h_pack || st.pack_bytes < bytes) {
    if (st.h_pack) (void)hipHostFree(st.h_pack);
    st.h_pack = nullptr;
    st.pack_bytes = 0;
    HIPCHK(ctx, hipHostMalloc(&st.h_pack, bytes, hipHostMallocDefault));
    st.pack_bytes = bytes;
  }
  // the previous call's copy out of the pinned buffer must be done before it is rewritten
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  unsigned char* h = (unsigned char*)st.h_pack;
  const int64_t* c8[27] = {pc->req_milli_cpu, pc->req_memory, pc->req_ephemeral, pc->nonzero_milli_cpu, pc->nonzero_memory,
                           pc->req_scalar[0], pc->req_scalar[1], pc->req_scalar[2], pc->req_scalar[3], pc->la_req_cpu,
                           pc->la_lim_cpu, pc->la_dflt_cpu, pc->la_req_memory, pc->la_lim_memory, pc->la_dflt_memory,
                           pc->gpu_core, pc->gpu_memory, pc->gpu_memory_ratio, pc->rdma};
  for (int d = 0; d < KS_QUOTA_DIMS; ++d) c8[19 + d] = pc->quota_req[d];
  for (int c = 0; c < 27; ++c) {
    unsigned char* dst = h + (size_t)c * st.col8;
    if (c8[c]) memcpy(dst, c8[c], (size_t)p * 8);
    else memset(dst, 0, (size_t)p * 8);
  }
  unsigned char* b4 = h + st.col8 * 27;
  // flags, quota, quota mask, reservation class, cpu_bind, stat_dyn (u8), joint (u8)
  const void* c4[5] = {pc->flags, pc->quota, pc->quota_mask, pc->rsv_class, pc->cpu_bind};
  const int fill4[5] = {0, 0xFF, 0, 0xFF, 0};
  for (int c = 0; c < 5; ++c) {
    unsigned char* dst = b4 + (size_t)c * st.col4;
    if (c4[c]) memcpy(dst, c4[c], (size_t)p * 4);
    else memset(dst, fill4[c], (size_t)p * 4);
  }
  memset(b4 + 5 * st.col4, 0, (size_t)p);  // stat_dyn: stage_cols fills it with the PodStat records
  if (pc->joint) memcpy(b4 + 6 * st.col4, pc->joint, (size_t)p);
  else memset(b4 + 6 * st.col4, 0, (size_t)p);
  HIPCHK(ctx, hipMemcpyAsync(st.cols.cpu, h, bytes, hipMemcpyHostToDevice, ctx->stream));
  return KS_OK;
}

static int stage_cols(ks_ctx* ctx, PodStage& st, const ks_pod_cols* pc, int32_t p) {
  DevPodCols& s = st.cols;
  if (p <= kPackPods && st.col8 && !ctx->kc.stat && !ctx->cfg.topology.enable) {
    st.cols.topo = nullptr;
    st.ndyn = 0;
    return stage_cols_packed(ctx, st, pc, p);
  }
  auto cp8 = [&](int64_t* d, const int64_t* h) -> hipError_t {
    if (h) return hipMemcpyAsync(d, h, (size_t)p * 8, hipMemcpyHostToDevice, ctx->stream);
    return hipMemsetAsync(d, 0, (size_t)p * 8, ctx->stream);
  };
  HIPCHK(ctx, cp8(s.cpu, pc->req_milli_cpu));
  HIPCHK(ctx, cp8(s.mem, pc->req_memory));
  HIPCHK(ctx, cp8(s.eph, pc->req_ephemeral));
  HIPCHK(ctx, cp8(s.nzcpu, pc->nonzero_milli_cpu));
  HIPCHK(ctx, cp8(s.nzmem, pc->nonzero_memory));
  for (int k = 0; k < KS_MAX_SCALARS; ++k) HIPCHK(ctx, cp8(s.sc[k], pc->req_scalar[k]));
  HIPCHK(ctx, cp8(s.la_req_cpu, pc->la_req_cpu));
  HIPCHK(ctx, cp8(s.la_lim_cpu, pc->la_lim_cpu));
  HIPCHK(ctx, cp8(s.la_dflt_cpu, pc->la_dflt_cpu));
  HIPCHK(ctx, cp8(s.la_req_mem, pc->la_req_memory));
  HIPCHK(ctx, cp8(s.la_lim_mem, pc->la_lim_memory));
  HIPCHK(ctx, cp8(s.la_dflt_mem, pc->la_dflt_memory));
  HIPCHK(ctx, cp8(s.gpu_core, pc->gpu_core));
  HIPCHK(ctx, cp8(s.gpu_mem, pc->gpu_memory));
  HIPCHK(ctx, cp8(s.gpu_ratio, pc->gpu_memory_ratio));
  HIPCHK(ctx, cp8(s.rdma, pc->rdma));
  if (pc->joint) HIPCHK(ctx, hipMemcpyAsync(s.joint, pc->joint, (size_t)p, hipMemcpyHostToDevice, ctx->stream));
  else HIPCHK(ctx, hipMemsetAsync(s.joint, 0, (size_t)p, ctx->stream));
  for (int d = 0; d < KS_QUOTA_DIMS; ++d) HIPCHK(ctx, cp8(st.pq.req[d], pc->quota_req[d]));
  if (pc->flags) HIPCHK(ctx, hipMemcpyAsync(s.flags, pc->flags, (size_t)p * 4, hipMemcpyHostToDevice, ctx->stream));
  else HIPCHK(ctx, hipMemsetAsync(s.flags, 0, (size_t)p * 4, ctx->stream));
  if (pc->quota) HIPCHK(ctx, hipMemcpyAsync(s.quota, pc->quota, (size_t)p * 4, hipMemcpyHostToDevice, ctx->stream));
  else HIPCHK(ctx, hipMemsetAsync(s.quota, 0xFF, (size_t)p * 4, ctx->stream));
  if (pc->quota_mask) HIPCHK(ctx, hipMemcpyAsync(st.pq.mask, pc->quota_mask, (size_t)p * 4, hipMemcpyHostToDevice, ctx->stream));
  else HIPCHK(ctx, hipMemsetAsync(st.pq.mask, 0, (size_t)p * 4, ctx->stream));
  if (pc->rsv_class) HIPCHK(ctx, hipMemcpyAsync(s.rsv_class, pc->rsv_class, (size_t)p * 4, hipMemcpyHostToDevice, ctx->stream));
  else HIPCHK(ctx, hipMemsetAsync(s.rsv_class, 0xFF, (size_t)p * 4, ctx->stream));
  if (pc->cpu_bind) HIPCHK(ctx, hipMemcpyAsync(s.cpu_bind, pc->cpu_bind, (size_t)p * 4, hipMemcpyHostToDevice, ctx->stream));
  else HIPCHK(ctx, hipMemsetAsync(s.cpu_bind, 0, (size_t)p * 4, ctx->stream));
  // TaintToleration / NodeAffinity: the pods' PodStat records and normalization flags, built here from the columns
  // (a pod whose raw scores are 0 on every node normalizes the same under every max: not kPodNormDyn)
  // PodTopologySpread / InterPodAffinity: the pods' query terms (TopoRec) next to the columns
  st.cols.topo = nullptr;
  st.ndyn = 0;
  if (ctx->cfg.topology.enable) {
    const int64_t nt = (pc->topo_term_beg && pc->topo_terms) ? pc->topo_term_beg[p] : 0;
    const int64_t npr = (pc->topo_prop_beg && pc->topo_props) ? pc->topo_prop_beg[p] : 0;
    auto grow = [&](void** buf, int64_t& cap, int64_t want, size_t elem) -> int {
      if (want <= cap && *buf) return KS_OK;
      dev_free(*buf);
      *buf = nullptr;
      cap = 0;
      const int64_t c = std::max<int64_t>(want, 64);
      if (dev_alloc(ctx, buf, (size_t)c * elem) != KS_OK) return KS_ENOMEM;
      cap = c;
      return KS_OK;
    };
    int64_t rcap = st.topo_cap;
    if (grow((void**)&st.topo, rcap, p, sizeof(TopoRec)) != KS_OK || grow((void**)&st.topo_terms, st.topo_tcap, nt, 8) != KS_OK ||
        grow((void**)&st.topo_props, st.topo_pcap, npr, 4) != KS_OK)
      return KS_ENOMEM;
    st.topo_cap = (int32_t)rcap;
    std::vector<TopoRec>& ht = st.h_topo;
    ht.assign((size_t)p, TopoRec{});
    for (int32_t i = 0; i < p; ++i) {
      TopoRec& r = ht[(size_t)i];
      r.flags = pc->topo_flags ? pc->topo_flags[i] : 0;
      if (nt) {
        r.tbeg = pc->topo_term_beg[i];
        r.nterms = pc->topo_term_beg[i + 1] - pc->topo_term_beg[i];
      }
      if (npr) {
        r.pbeg = pc->topo_prop_beg[i];
        r.nprops = pc->topo_prop_beg[i + 1] - pc->topo_prop_beg[i];
      }
      if (r.nterms == 0) r.flags &= ~KS_TOPO_DYN;  // (no query term: nothing the step would ask)
      st.ndyn += (r.flags & KS_TOPO_DYN) ? 1 : 0;
    }
    if (p > 0) HIPCHK(ctx, hipMemcpyAsync(st.topo, ht.data(), (size_t)p * sizeof(TopoRec), hipMemcpyHostToDevice, ctx->stream));
    if (nt) HIPCHK(ctx, hipMemcpyAsync(st.topo_terms, pc->topo_terms, (size_t)nt * 8, hipMemcpyHostToDevice, ctx->stream));
    if (npr) HIPCHK(ctx, hipMemcpyAsync(st.topo_props, pc->topo_props, (size_t)npr * 4, hipMemcpyHostToDevice, ctx->stream));
    st.cols.topo = st.topo;
  }
  if (ctx->kc.stat || ctx->cfg.topology.enable) {
    std::vector<PodStat>& hs = st.h_stat;
    std::vector<uint8_t>& hd = st.h_dyn;
    hs.assign((size_t)p, PodStat{});
    hd.assign((size_t)p, 0);
    for (int32_t i = 0; i < p; ++i) {
      PodStat& r = hs[(size_t)i];
      r.tol = pc->tolerated ? pc->tolerated[i] : 0;
      r.nreq = pc->affinity_required_n ? pc->affinity_required_n[i] : 0;
      bool dyn = (ctx->kc.taint & 2) && (ctx->soft_union & ~r.tol) != 0;
      for (int t = 0; t < KS_AFFINITY_TERMS; ++t) {
        r.req[t] = pc->affinity_required[t] ? pc->affinity_required[t][i] : 0;
        r.pref[t] = pc->affinity_preferred[t] ? pc->affinity_preferred[t][i] : 0;
        r.w[t] = pc->affinity_weight[t] ? pc->affinity_weight[t][i] : 0;
        dyn |= (ctx->kc.aff & 2) && r.w[t] != 0;
      }
      r.pwant = pc->host_ports ? pc->host_ports[i] : 0;
      r.pconf = pc->host_ports_conflict ? pc->host_ports_conflict[i] : 0;
      hd[(size_t)i] = dyn ? 1 : 0;
    }
    if (p > 0) {
      HIPCHK(ctx, hipMemcpyAsync(st.stat, hs.data(), (size_t)p * sizeof(PodStat), hipMemcpyHostToDevice, ctx->stream));
      HIPCHK(ctx, hipMemcpyAsync(s.stat_dyn, hd.data(), (size_t)p, hipMemcpyHostToDevice, ctx->stream));
    }
    if (p > 0) {
      HIPCHK(ctx, hipStreamSynchronize(ctx->stream));  // pageable sources
    }
  } else {
    HIPCHK(ctx, hipMemsetAsync(s.stat_dyn, 0, (size_t)p, ctx->stream));
  }
  return KS_OK;
}

// PreFilter / EstimatePod: the stage's columns -> PodRec (prep_pods_kernel)
static int prep_stage(ks_ctx* ctx, PodStage& st, int32_t p) {
  if (p <= 0) return KS_OK;
  const int threads = 256;
  hipLaunchKernelGGL(prep_pods_kernel, dim3((p + threads - 1) / threads), dim3(threads), 0, ctx->stream, st.cols,
                     st.recs, p, ctx->cfg.loadaware.scaling_cpu, ctx->cfg.loadaware.scaling_memory,
                     (int32_t)(ctx->cfg.deviceshare.enable != 0));
  HIPCHK(ctx, hipGetLastError());
  return KS_OK;
}

static int validate_pods(ks_ctx* ctx, const ks_pod_cols* pc, int32_t p) {
  if (ctx->cfg.topology.enable) {
    // the CSR lists: monotone offsets from 0, at most KS_TOPO_MAX_TERMS terms per pod, properties / keys in range
    if ((pc->topo_term_beg == nullptr) != (pc->topo_terms == nullptr) || (pc->topo_prop_beg == nullptr) != (pc->topo_props == nullptr))
      KS_FAIL(ctx, KS_EINVAL, "topology lists: an offset array without its list (or the reverse)");
    for (int32_t i = 0; pc->topo_term_beg && i < p; ++i) {
      const int32_t b = pc->topo_term_beg[i], e = pc->topo_term_beg[i + 1];
      if ((i == 0 && b != 0) || e < b || e - b > KS_TOPO_MAX_TERMS)
        KS_FAIL(ctx, KS_EINVAL, "pod %d: topology term offsets [%d, %d) (at most %d terms)", i, b, e, KS_TOPO_MAX_TERMS);
      for (int32_t t = b; t < e; ++t) {
        const uint64_t w = pc->topo_terms[t];
        const int kind = (int)(w & 0xF), key = (int)((w >> 8) & 0xFF), prop = (int)((w >> 16) & 0xFFFF);
        const int32_t param = (int32_t)(uint32_t)(w >> 32);
        if (kind < KS_TOPO_K_SPREAD_HARD || kind > KS_TOPO_K_SCORE || prop >= ctx->topo_nprops || key > ctx->topo_nkeys ||
            ((w >> 5) & 0x7) != 0 ||
            ((kind == KS_TOPO_K_SPREAD_HARD || kind == KS_TOPO_K_SPREAD_SOFT) && param < 1) ||
            (kind == KS_TOPO_K_SCORE && (param < -1000000 || param > 1000000)))
          KS_FAIL(ctx, KS_EINVAL, "pod %d: topology term %d (%#llx) malformed", i, t - b, (unsigned long long)w);
      }
    }
    for (int32_t i = 0; pc->topo_prop_beg && i < p; ++i) {
      const int32_t b = pc->topo_prop_beg[i], e = pc->topo_prop_beg[i + 1];
      if ((i == 0 && b != 0) || e < b) KS_FAIL(ctx, KS_EINVAL, "pod %d: topology property offsets [%d, %d)", i, b, e);
      for (int32_t k = b; k < e; ++k)
        if (pc->topo_props[k] < 0 || pc->topo_props[k] >= ctx->topo_nprops)
          KS_FAIL(ctx, KS_EINVAL, "pod %d: topology property %d outside [0, %d)", i, pc->topo_props[k], ctx->topo_nprops);
    }
  }
  for (int32_t i = 0; pc->flags && i < p; ++i)
    if (pc->flags[i] & KS_POD_UNMODELLED)
      KS_FAIL(ctx, KS_EUNSUPPORTED, "pod %d: requests the library does not model (FPGA, DeviceShare allocate hints, "
                                    "a reserve pod as the scheduling subject)", i);
  for (int32_t i = 0; pc->affinity_required_n && i < p; ++i)
    if (pc->affinity_required_n[i] < 0 || pc->affinity_required_n[i] > KS_AFFINITY_TERMS)
      KS_FAIL(ctx, KS_EUNSUPPORTED, "pod %d: %d required node affinity terms (the device evaluates up to %d)", i,
              pc->affinity_required_n[i], KS_AFFINITY_TERMS);
  for (int t = 0; t < KS_AFFINITY_TERMS; ++t)
    for (int32_t i = 0; pc->affinity_weight[t] && i < p; ++i)
      if (pc->affinity_weight[t][i] < 0 || pc->affinity_weight[t][i] > 100)
        KS_FAIL(ctx, KS_EINVAL, "pod %d: preferred node affinity weight %d outside [0, 100]", i, pc->affinity_weight[t][i]);
  const int64_t* cols[] = {pc->req_milli_cpu, pc->req_memory, pc->req_ephemeral, pc->nonzero_milli_cpu,
                           pc->nonzero_memory, pc->la_req_cpu, pc->la_lim_cpu, pc->la_req_memory, pc->la_lim_memory,
                           pc->gpu_core, pc->gpu_memory, pc->gpu_memory_ratio, pc->rdma};
  for (const int64_t* c : cols)
    if (check_range64(ctx, c, p, "pod quantity") != KS_OK) return KS_EINVAL;
  for (int k = 0; k < KS_MAX_SCALARS; ++k)
    if (check_range64(ctx, pc->req_scalar[k], p, "pod scalar") != KS_OK) return KS_EINVAL;
  bool any_req = false;
  if (ctx->cfg.numa.enable && pc->flags) {
    for (int32_t i = 0; i < p; ++i) {
      if (!(pc->flags[i] & KS_POD_CPU_BIND)) continue;
      if (!pc->cpu_bind) KS_FAIL(ctx, KS_EINVAL, "pod %d: KS_POD_CPU_BIND without ks_pod_cols.cpu_bind", i);
      const uint32_t cb = pc->cpu_bind[i], pol = cb & KS_CPU_BIND_POLICY_MASK, ex = (cb >> KS_CPU_EXCL_SHIFT) & 3u;
      const int64_t cpu = pc->req_milli_cpu ? pc->req_milli_cpu[i] : 0;
      if ((pol != KS_CPU_BIND_FULL_PCPUS && pol != KS_CPU_BIND_SPREAD_BY_PCPUS) || ex > KS_CPU_EXCL_NUMA_NODE_LEVEL || (cb >> 5))
        KS_FAIL(ctx, KS_EINVAL, "pod %d: cpu_bind 0x%x invalid", i, cb);
      const bool req = (cb & KS_CPU_BIND_REQUIRED) != 0;
      any_req |= req;
      if (cpu <= 0 || cpu % 1000 != 0 || cpu / 1000 > KS_MAX_CPUS)
        KS_FAIL(ctx, KS_EINVAL, "pod %d: a cpu-bind pod needs a whole-CPU request in (0, %d] CPUs (PreFilter ErrInvalidRequestedCPUs)", i, KS_MAX_CPUS);
      // (a preferred FullPCPUs request that is not a whole number of cores takes a split core in takeCPUs'
      // freeCoresInNode / freeCoresInSocket prefixes or the fallbacks, as ks_cpuset.h does; a required one fails the
      // Filter's SMT alignment check per node, plugin.go:314-317)
    }
  }
  if (pc->joint) {
    for (int32_t i = 0; i < p; ++i) {
      const uint8_t j = pc->joint[i];
      if (j > KS_JOINT_GPU_RDMA_SAME_PCIE) KS_FAIL(ctx, KS_EINVAL, "pod %d: joint %u invalid", i, (unsigned)j);
      // (without an RDMA request jointAllocate still takes RDMA devices, with a nil request: ks_dev.h dev_eval)
    }
  }
  if (pc->rsv_class) {
    for (int32_t i = 0; i < p; ++i)
      if (pc->rsv_class[i] < -1 || pc->rsv_class[i] >= KS_RSV_CLASSES)
        KS_FAIL(ctx, KS_EINVAL, "pod %d: reservation class %d outside [-1, %d)", i, pc->rsv_class[i], KS_RSV_CLASSES);
  }
  if (pc->quota) {
    for (int32_t i = 0; i < p; ++i)
      if (pc->quota[i] >= ctx->q.q || pc->quota[i] < -1)
        KS_FAIL(ctx, KS_EINVAL, "pod %d: quota row %d out of range (loaded %d)", i, pc->quota[i], ctx->q.q);
  }
  // a pod requesting a scalar slot no node advertises still has to be evaluated against the
  // (zero) allocatable of that slot: widen the kernels' scalar template to cover it
  int need = ctx->nsc;
  for (int k = ctx->nsc; k < KS_MAX_SCALARS; ++k) {
    if (!pc->req_scalar[k]) continue;
    for (int32_t i = 0; i < p; ++i)
      if (pc->req_scalar[k][i] != 0) {
        need = k + 1;
        break;
      }
  }
  if (need > ctx->nsc) {
    ctx->nsc = need <= 2 ? 2 : 4;
    ctx->kc.nsc = ctx->nsc;
  }
  // only a batch (or pod) that passed every check decides the core-count mode, and only for its own operation
  // (bind_mode): a rejected or probed pod leaves later schedules as they were
  ctx->val_bind_required = any_req;
  return KS_OK;
}

// Cfg.cores for the operation about to run: node CPU bind labels, or a required policy among its pods
static void bind_mode(ks_ctx* ctx, bool required) {
  ctx->cpu_bind_required = required;
  cores_mode(ctx);
}

int ks_stage_pods(ks_ctx* ctx, const ks_pod_cols* pods, int32_t p) {
  if (!ctx || !pods || p < 0) return ctx ? (ctx->err = "ks_stage_pods: bad args", KS_EINVAL) : KS_EINVAL;
  if (!ctx->node_blob) KS_FAIL(ctx, KS_ESTATE, "ks_stage_pods before ks_load_nodes");
  if (ctx->cfg.quota.enable && pods->quota && !ctx->quota_blob)
    KS_FAIL(ctx, KS_ESTATE, "ElasticQuota enabled but ks_load_quotas not called");
  if (int rc = validate_pods(ctx, pods, p); rc != KS_OK) return rc;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  if (ensure_stage(ctx, ctx->st, p) != KS_OK) return KS_ENOMEM;
  if (p > 0 && stage_cols(ctx, ctx->st, pods, p) != KS_OK) return KS_EHIP;
  ctx->np = p;
  ctx->staged_bind_required = ctx->val_bind_required;
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  return KS_OK;
}

static hipEvent_t take_event(ks_ctx* ctx, size_t i) {
  while (ctx->ev_pool.size() <= i) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    ctx->ev_pool.push_back(e);
  }
  return ctx->ev_pool[i];
}

static size_t dev_cache_bytes(const ks_ctx* ctx);
static int kernel_feat(const ks_ctx* ctx);
// the context's commit variant runs the helper waves (NUMA policies + DeviceShare compiled in, ks_pass.h)
static bool commit_hint_variant(const ks_ctx* ctx) { return (kernel_feat(ctx) & 12) == 12; }
static size_t numa_cache_bytes(const ks_ctx* ctx) {
  return ctx->kc.numa_pol ? (size_t)kMaxBatch * kNumaSlotWords * 8 : 0;
}

// Quota rows are cached in LDS for the pass when the table is small enough and the LDS image fits.
static int kernel_feat(const ks_ctx* ctx);

static bool commit_qcache(const ks_ctx* ctx) {
  if (!(ctx->kc.quota_enable && ctx->q.q > 0 && ctx->q.q <= kQuotaLdsRows)) return false;
  return commit_layout(ctx->k, ctx->nchunks, true, 0, dev_cache_bytes(ctx), numa_cache_bytes(ctx), ctx->q.q, kernel_feat(ctx) == 0,
                       commit_hint_variant(ctx)).total <= 160 * 1024;
}

// Kernel variant (FEAT bits, ks_pass.h): 1 Reservation, 2 NodeNUMAResource, 4 the normalized plugins (DeviceShare,
// TaintToleration / NodeAffinity / NodePorts), 8 NUMA topology policies (with 2), 16 reservations holding devices (with
// 1 and 4: DeviceShare's restore state, ks_rsv.h; without it the restore code costs the 7 / 15 kernels ~30 % at c3r,
// though no node runs it).  A context runs the smallest built
// variant whose bits cover the plugins it enables: a bit that is compiled in but unused still costs registers -- the
// variants with Reservation and the normalized plugins together spill 180-320 B/lane in the commit kernel, those
// without Reservation (4, 6, 14) none (hipcc -Rpass-analysis=kernel-resource-usage).
constexpr int kBuiltFeats[] = {0, 1, 3, 4, 6, 7, 11, 14, 15, 23, 31};  // ascending (koordinator_amd/csrc/Makefile FEATS)

static int kernel_feat(const ks_ctx* ctx) {
  const int need = (ctx->kc.rsv ? 1 : 0) | (ctx->kc.numa ? 2 : 0) | ((ctx->kc.dev || ctx->kc.stat) ? 4 : 0) |
                   (ctx->kc.numa_pol ? 10 : 0) | ((ctx->kc.rsv && ctx->kc.dev && ctx->dev_held_any) ? 21 : 0);
  for (int f : kBuiltFeats)
    if ((f & need) == need) return f;
  return 31;
}

// the slot device region of the commit kernel: GPU state (DeviceShare), then the TaintToleration / NodeAffinity words
// and NodePorts words (4 x u64 per slot, the region's last kMaxBatch * 32 B) after the pass's PodStat records and the
// normalization maxima table (ks_pass.h commit_kernel)
static size_t dev_cache_bytes_with(const ks_ctx* ctx, bool stat_lds) {
  return (ctx->kc.dev ? (size_t)kDevLdsStride * (kDevTW + kDevQW) * 8 + (size_t)kMaxBatch * 4 : 0) +
         ((ctx->kc.dev || ctx->kc.stat) ? (size_t)kNormRows * kMaxBatch * 8 : 0) +
         (ctx->kc.stat ? (size_t)kMaxBatch * 32 : 0) + (stat_lds ? (size_t)kMaxBatch * sizeof(PodStat) : 0);
}

// The pass's PodStat records go to LDS when the commit image still fits with them (before the quota-row and
// reservation caches are sized); otherwise the commit reads them from HBM (CommitArgs.stat_lds)
static bool commit_stat_lds(const ks_ctx* ctx) {
  if (!ctx->kc.stat) return false;
  return commit_layout(ctx->k, ctx->nchunks, false, 0, dev_cache_bytes_with(ctx, true), numa_cache_bytes(ctx), ctx->q.q,
                       kernel_feat(ctx) == 0, commit_hint_variant(ctx)).total + 64 <= 160 * 1024;
}

static size_t dev_cache_bytes(const ks_ctx* ctx) { return dev_cache_bytes_with(ctx, commit_stat_lds(ctx)); }

static size_t rsv_cache_bytes(const ks_ctx* ctx, int32_t rcap) {
  return (size_t)kMaxBatch * rcap * 8 * (size_t)(3 + 2 * (3 + ctx->nsc) + 2);  // sizeof(RsvRec<3+nsc>)
}

// Reservations cached per commit slot: as many as fit next to the rest of the commit layout (<= 8);
// the quota-row cache yields to it when both do not fit.
static int32_t commit_rcap(const ks_ctx* ctx, bool* qcache) {
  *qcache = commit_qcache(ctx);
  if (!ctx->kc.rsv) return 0;
  auto fit = [&](bool qc) {
    const size_t base = commit_layout(ctx->k, ctx->nchunks, qc, 0, dev_cache_bytes(ctx), numa_cache_bytes(ctx), ctx->q.q,
                                      kernel_feat(ctx) == 0, commit_hint_variant(ctx)).total + 64;
    const size_t avail = base < 160 * 1024 ? 160 * 1024 - base : 0;
    return (int32_t)std::min<size_t>(8, avail / rsv_cache_bytes(ctx, 1));
  };
  int32_t r = fit(*qcache);
  if (*qcache && r < 4) {
    *qcache = false;
    r = fit(false);
  }
  return r;
}

// the launch wrappers of the FEAT variant (ks_variant.hip)
static PassLaunch pass_launcher(int feat, int nsc) {
#define KS_PICK(F) return nsc == 0 ? pass_launch_f##F##_n0() : (nsc == 2 ? pass_launch_f##F##_n2() : pass_launch_f##F##_n4())
  switch (feat) {
    case 31: KS_PICK(31);
    case 23: KS_PICK(23);
    case 15: KS_PICK(15);
    case 14: KS_PICK(14);
    case 11: KS_PICK(11);
    case 7: KS_PICK(7);
    case 6: KS_PICK(6);
    case 4: KS_PICK(4);
    case 3: KS_PICK(3);
    case 1: KS_PICK(1);
    default: KS_PICK(0);
  }
#undef KS_PICK
}

// The commit kernel's arguments for the pods of stage st (cursor ctx->cursor, `total` pods, `batch` per pass).
// Candidate-list set i (0 or 1) of the context's double buffer; set 0 unless passes are pipelined.
struct CandSet {
  uint32_t* chunk;
  uint2* t;
  uint64_t *bound, *top, *second;
  int32_t *count, *total;
};
static CandSet cand_set(const ks_ctx* ctx, int i) {
  const size_t e = (size_t)i * kMaxBatch * kMaxCand, r = (size_t)i * kMaxBatch;
  return CandSet{ctx->cand_chunk + e, ctx->cand_t + e, ctx->cand_bound + r, ctx->cand_top + r, ctx->cand_second + r,
                 ctx->cand_count + r, ctx->cand_total + r};
}

static CommitArgs commit_args(ks_ctx* ctx, PodStage& st, int32_t total, int32_t batch, bool* qcache, size_t* smem) {
  CommitArgs ca;
  ca.dn = ctx->dnodes;
  ca.rv = ctx->drv;
  ca.c = ctx->kc;
  ca.pods = st.recs;
  ca.pstat = st.stat;
  ca.pq = st.pq;
  ca.q = ctx->q;
  ca.cursor = ctx->cursor;
  ca.cand_chunk = ctx->cand_chunk;
  ca.cand_t = ctx->cand_t;
  ca.cand_bound = ctx->cand_bound;
  ca.cand_top = ctx->cand_top;
  ca.cand_second = ctx->cand_second;
  ca.cand_count = ctx->cand_count;
  ca.results = st.results;
  ca.counters = ctx->counters;
  ca.n = ctx->n;
  ca.nchunks = ctx->nchunks;
  ca.total_pods = total;
  ca.batch = batch;
  ca.k = ctx->k;
  ca.rowcols = ctx->rowcols;
  ca.rcap = commit_rcap(ctx, qcache);
  ca.rsv_bytes = (int32_t)rsv_cache_bytes(ctx, ca.rcap);
  ca.dev_bytes = (int32_t)dev_cache_bytes(ctx);
  ca.stat_lds = commit_stat_lds(ctx) ? 1 : 0;
  ca.dv = ctx->ddv;
  ca.dev_M = ctx->dev_M;
  ca.cpuset_list = ctx->cpuset_list;
  ca.cpuset_n = ctx->cpuset_n;
  ca.cpuset_split = ctx->cpuset_split;
  ca.numa_alloc = ctx->numa_alloc;
  ca.force = 0;
  ca.numa_bytes = (int32_t)numa_cache_bytes(ctx);
  ca.nv = ctx->dnv;
  ca.pipe_base = nullptr;
  ca.carry = nullptr;
  ca.pipe_follow = nullptr;
  ca.pipe_after = nullptr;
  ca.top_reset = nullptr;
  ca.pre_rsv = nullptr;
  ca.topo = ctx->cfg.topology.enable && st.topo ? 1 : 0;
  ca.topo_const = (int32_t)(100 * ctx->cfg.topology.spread_weight);
  ca.topo_rec = st.topo;
  ca.topo_props = st.topo_props;
  ca.topo_count = ctx->topo_count;
  ca.topo_npad = ctx->npad;
  ca.topo_best = ctx->topo_scr ? &ctx->topo_scr->best_total : nullptr;
  *smem = commit_layout(ctx->k, ctx->nchunks, *qcache, (size_t)ca.rsv_bytes, (size_t)ca.dev_bytes, (size_t)ca.numa_bytes,
                        ctx->q.q, kernel_feat(ctx) == 0, commit_hint_variant(ctx)).total;
  return ca;
}

// The monotone commit kernel (ks_mono.h) runs the passes of a plugin set without Reservation, NodeNUMAResource or
// DeviceShare whose keys commits can only lower (Fit LeastAllocated + LoadAware) when its LDS fits.  With
// ElasticQuota the general kernel runs instead: its admission look-ahead for pod j + 1 overlaps pod j's Reserve,
// and that measured faster than the mono kernel's prebuilt rows at C2 (MI355X, commit 20.6 vs 21.4 ms/step;
// C5 without quota: mono 275.6 vs general 281.3 ms per 200k pods, profiles/r02_commit_ab.txt).
// KS_COMMIT_GENERAL=1 keeps the general kernel, =2 forces the mono kernel with quota too (A/B).  ks_assume always
// uses the general kernel.
static bool mono_commit(const ks_ctx* ctx, bool qcache, size_t* smem) {
  static const int64_t mode = env_i64("KS_COMMIT_GENERAL", 0, 0, 2);
  if (mode == 1 || kernel_feat(ctx) != 0 || !ctx->kc.monotone || ctx->kc.fit_most) return false;
  if (mode == 0 && ctx->kc.quota_enable) return false;
  *smem = mono_layout(ctx->k, ctx->nchunks, qcache, ctx->q.q).total;
  return *smem <= 160 * 1024;
}

// Reserve's NodeNUMAResource / DeviceShare allocations ahead of the commit (reserve_pre_kernel): on for
// the NUMA topology policy variants when policy nodes are loaded; KS_PRE_RSV=0 turns it off (A/B).
static bool pre_reserve(const ks_ctx* ctx) {
  static const int64_t env_pre = env_i64("KS_PRE_RSV", 1, 0, 1);
  return env_pre != 0 && ctx->kc.numa_pol;
}

// the commit kernel's LDS size for this context: checked against the CU's 160 KB and set on the variant
static int commit_attr_set(ks_ctx* ctx) {
  bool qcache = false;
  const int32_t rcap = commit_rcap(ctx, &qcache);
  const size_t smem = commit_layout(ctx->k, ctx->nchunks, qcache, rsv_cache_bytes(ctx, rcap), dev_cache_bytes(ctx),
                                    numa_cache_bytes(ctx), ctx->q.q, kernel_feat(ctx) == 0, commit_hint_variant(ctx)).total;
  if (smem > 160 * 1024)
    KS_FAIL(ctx, KS_EUNSUPPORTED, "too many nodes for the commit kernel's LDS (%lld nodes, %zu B)", (long long)ctx->n, smem);
  hipError_t e = pass_launcher(kernel_feat(ctx), ctx->nsc).commit_attr(qcache, smem);
  if (e != hipSuccess) KS_FAIL(ctx, KS_EHIP, "hipFuncSetAttribute(commit LDS %zu): %s", smem, hipGetErrorString(e));
  size_t msmem = 0;
  if (mono_commit(ctx, qcache, &msmem)) {
    e = pass_launcher(0, ctx->nsc).commit_mono_attr(qcache, msmem);
    if (e != hipSuccess) KS_FAIL(ctx, KS_EHIP, "hipFuncSetAttribute(mono commit LDS %zu): %s", msmem, hipGetErrorString(e));
  }
  return KS_OK;
}

// (pod, node) list + count + per-pod CPU sets / NUMA split / NUMA allocation of one call, for np pods
static int ensure_cpuset_bufs(ks_ctx* ctx, int32_t np) {
  if (!ctx->cfg.numa.enable || ctx->cpuset_cap >= np) return KS_OK;
  void* p = ctx->cpuset_list;
  dev_free(p);
  ctx->cpuset_list = nullptr;
  const int32_t cap = std::max<int32_t>(np, 64);
  const size_t o_n = (size_t)cap * 8, o_out = o_n + 16, o_split = o_out + (size_t)cap * sizeof(CpuSet),
               o_alloc = align16(o_split + (size_t)cap * 4), bytes = o_alloc + (size_t)cap * 2 * kNumaDev * 8;
  if (dev_alloc(ctx, &p, bytes) != KS_OK) return KS_ENOMEM;
  ctx->cpuset_list = (int2*)p;
  ctx->cpuset_n = (int32_t*)((char*)p + o_n);
  ctx->cpuset_out = (CpuSet*)((char*)p + o_out);
  ctx->cpuset_split = (uint32_t*)((char*)p + o_split);
  ctx->numa_alloc = (int64_t*)((char*)p + o_alloc);
  ctx->cpuset_cap = cap;
  return KS_OK;
}

constexpr int kPipeWords = 4 + 1 + kMaxBatch;  // ks_ctx.pipe: bases [0..1], carry list at [4]

// Pipelined passes are used for plugin sets whose sweep output depends on nothing but the node rows
// (and reservations) a commit writes: no DeviceShare (its normalization max spans every node) and no
// NodeNUMAResource (core counts are refreshed by cpuset_kernel).  KS_PIPE=0 turns them off (A/B).
// The re-sweep, the select and two cross-stream hops then sit between consecutive commits instead of the sweep, so it
// pays only when the sweep is long: clusters of at least KS_PIPE_MIN_NODES nodes (default 32,768; C5's 100k, not
// C2's 5k: measured on MI355X, profiles/r03_pipe_ab.txt).
static bool pipelined(const ks_ctx* ctx) {
  static const int64_t env_pipe = env_i64("KS_PIPE", 1, 0, 2);
  static const int64_t env_min = env_i64("KS_PIPE_MIN_NODES", 32768, 0, (int64_t)1 << 40);
  const int64_t mode = ctx->pipe_mode >= 0 ? ctx->pipe_mode : env_pipe;
  const int feat = kernel_feat(ctx);
  if (mode == 0 || !(feat == 0 || feat == 1) || ctx->kc.dev || ctx->kc.cores) return false;
  if (ctx->cfg.topology.enable && ctx->st.ndyn > 0) return false;  // topology pods: the topology step between passes
  return mode == 2 || ctx->n >= env_min;
}

// The pipelined passes' two streams per device, shared by the process's contexts for the life of the process
// (DESIGN §5a "Streams"): each CU-masked stream owns a hardware queue of its own (a queue carries one CU mask), and
// the process has GPU_MAX_HW_QUEUES = 4 of them, so per-context masked streams would run out as soon as two contexts
// pipeline (two scheduler profiles, the loopback ranks).  ks_destroy waits only for its own context's events on them.
struct PipeStreams {
  hipStream_t s = nullptr, c = nullptr;
};
static std::mutex g_pipe_mu;
static std::vector<PipeStreams> g_pipe;

// At process exit the shared streams are released before the HIP runtime's own teardown (atexit handlers run in
// reverse order of registration, and the runtime registers its handlers before the first stream exists): left to the
// runtime's teardown, the CU-masked streams crashed a rocprofv3 --kernel-trace run in __cxa_finalize after its output
// was written.  By then no context may still be using them.
static void release_pipe_streams() {
  std::lock_guard<std::mutex> lock(g_pipe_mu);
  for (PipeStreams& st : g_pipe) {
    if (st.c) (void)hipStreamDestroy(st.c);
    if (st.s) (void)hipStreamDestroy(st.s);
    st.s = st.c = nullptr;
  }
}

// The sweep stream (CU-masked to all but KS_PIPE_COMMIT_CUS = 32 CUs, which the commit stream gets: the one-workgroup
// commit and the patched passes' list re-evaluation never share a CU with sweep waves; KS_PIPE_CUMASK=0: no masks), the
// pipe words and the event ring.
static int ensure_pipe(ks_ctx* ctx) {
  if (!ctx->pipe) {
    void* p = nullptr;
    if (dev_alloc(ctx, &p, kPipeWords * 4) != KS_OK) return KS_ENOMEM;
    ctx->pipe = (int32_t*)p;
    if (dev_alloc(ctx, &p, 2 * kMaxBatch * 8) != KS_OK) return KS_ENOMEM;
    ctx->pipe_top = (unsigned long long*)p;
  }
  if (!ctx->sstream) {
    // One sweep stream and one commit stream per device for the whole process, shared by every context: a
    // CU-masked stream owns a hardware queue of its own, and creating them per context exhausts the process's
    // queues.  Sharing only orders the passes of different contexts; each context's own events order its passes.
    // The commit stream runs on the KS_PIPE_COMMIT_CUS CUs the sweep stream leaves out, so the one-workgroup commit
    // never shares a CU (and its SIMDs' issue slots) with sweep waves.
    std::lock_guard<std::mutex> lock(g_pipe_mu);
    static const bool at_exit = std::atexit(release_pipe_streams) == 0;
    (void)at_exit;
    if (g_pipe.size() <= (size_t)ctx->device) g_pipe.resize((size_t)ctx->device + 1);
    PipeStreams& st = g_pipe[(size_t)ctx->device];
    if (!st.s) {
      static const int64_t env_mask = env_i64("KS_PIPE_CUMASK", 1, 0, 1);
      int ncu = 0;
      (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, ctx->device);
      bool masked = false;
      if (env_mask && ncu > 8) {
        std::vector<uint32_t> smask((size_t)(ncu + 31) / 32, 0u), cmask((size_t)(ncu + 31) / 32, 0u);
        // the commit stream's CUs: the one-workgroup commit and, for patched passes, the re-sweep and list patch
        // that run between two commits
        static const int64_t env_ccus = env_i64("KS_PIPE_COMMIT_CUS", 32, 1, 128);
        const int rc = (int)std::min<int64_t>(env_ccus, ncu / 2);
        for (int c = 0; c < ncu; ++c) (c < rc ? cmask : smask)[(size_t)c / 32] |= 1u << (c % 32);
        hipStream_t a = nullptr, b = nullptr;
        if (hipExtStreamCreateWithCUMask(&a, (uint32_t)smask.size(), smask.data()) == hipSuccess) {
          if (hipExtStreamCreateWithCUMask(&b, (uint32_t)cmask.size(), cmask.data()) == hipSuccess) {
            st.s = a;
            st.c = b;
            masked = true;
          } else {
            (void)hipStreamDestroy(a);
          }
        }
      }
      if (!masked) HIPCHK(ctx, hipStreamCreateWithFlags(&st.s, hipStreamNonBlocking));
    }
    ctx->sstream = st.s;
    ctx->cstream = st.c ? st.c : ctx->stream;
  }
  for (int i = 0; i < kPipeEvents; ++i) {
    if (!ctx->pev_sel[i]) HIPCHK(ctx, hipEventCreateWithFlags(&ctx->pev_sel[i], hipEventDisableTiming));
    if (!ctx->pev_com[i]) HIPCHK(ctx, hipEventCreateWithFlags(&ctx->pev_com[i], hipEventDisableTiming));
  }
  return KS_OK;
}

// ---- the candidate exchange between ranks: RCCL (ks_shard_init), or the loopback test transport ----

static bool loop_barrier(LoopGroup* g) {
  std::unique_lock<std::mutex> lk(g->mu);
  if (g->broken) return false;
  const int64_t my = g->gen;
  if (++g->arrived == g->n) {
    g->arrived = 0;
    ++g->gen;
    g->cv.notify_all();
    return true;
  }
  const bool ok = g->cv.wait_for(lk, std::chrono::seconds(120), [&] { return g->gen != my || g->broken; });
  if (!ok || g->broken) {
    g->broken = true;
    g->cv.notify_all();
    return false;
  }
  return true;
}

static void loop_break(LoopGroup* g) {
  std::lock_guard<std::mutex> lk(g->mu);
  g->broken = true;
  g->cv.notify_all();
}

// The loopback exchange's two phases around `pull` (the device copies of the peers' blocks, on stream s).
template <typename Pull>
static int loop_exchange(ks_ctx* ctx, hipStream_t s, Pull pull) {
  LoopGroup* g = ctx->loop;
  const int par = (int)(ctx->loop_seq++ & 1);
  auto fail = [&](const char* what) {
    loop_break(g);
    KS_FAIL(ctx, KS_EHIP, "loopback exchange: %s", what);
  };
  if (hipEventRecord(ctx->lev[par][0], s) != hipSuccess) return fail("hipEventRecord");
  if (!loop_barrier(g)) return fail("a peer rank failed or timed out");
  for (int32_t p = 0; p < g->n; ++p) {
    if (p == ctx->rank) continue;
    ks_ctx* peer = g->ranks[(size_t)p];
    if (!peer) return fail("a peer rank was destroyed");
    if (hipStreamWaitEvent(s, peer->lev[par][0], 0) != hipSuccess) return fail("hipStreamWaitEvent");
    if (pull(peer, p) != hipSuccess) return fail("device copy of a peer's block");
  }
  if (hipEventRecord(ctx->lev[par][1], s) != hipSuccess) return fail("hipEventRecord");
  if (!loop_barrier(g)) return fail("a peer rank failed or timed out");
  for (int32_t p = 0; p < g->n; ++p) {
    if (p == ctx->rank) continue;
    ks_ctx* peer = g->ranks[(size_t)p];
    if (!peer) return fail("a peer rank was destroyed");
    if (hipStreamWaitEvent(s, peer->lev[par][1], 0) != hipSuccess) return fail("hipStreamWaitEvent");
  }
  return KS_OK;
}

// In-place allgather of the ranks' candidate-slot blocks: rank r's `bytes` at gather + r * bytes.
static int exchange_allgather(ks_ctx* ctx, size_t bytes, hipStream_t s) {
  if (ctx->loop)
    return loop_exchange(ctx, s, [&](ks_ctx* peer, int32_t p) {
      return hipMemcpyAsync(ctx->gather + (size_t)p * bytes, peer->gather + (size_t)p * bytes, bytes,
                            hipMemcpyDeviceToDevice, s);
    });
  const ncclResult_t r = ncclAllGather(ctx->gather + (size_t)ctx->rank * bytes, ctx->gather, bytes, ncclUint8, ctx->comm, s);
  if (r != ncclSuccess) KS_FAIL(ctx, KS_EHIP, "ncclAllGather (candidate slots): %s", ncclGetErrorString(r));
  return KS_OK;
}

__global__ void max_reduce_kernel(unsigned long long* buf, const unsigned long long* peers, int32_t nranks, int32_t rank,
                                   int32_t count) {
  const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  unsigned long long m = buf[i];
  for (int32_t p = 0; p < nranks; ++p)
    if (p != rank) m = max(m, peers[(size_t)p * count + i]);
  buf[i] = m;
}

// In-place max all-reduce of the pass's normalization maxima (count u64 words at buf = ctx->dev_M).
static int exchange_allreduce_max(ks_ctx* ctx, unsigned long long* buf, int32_t count, hipStream_t s) {
  if (ctx->loop) {
    if (int rc = loop_exchange(ctx, s, [&](ks_ctx* peer, int32_t p) {
          return hipMemcpyAsync(ctx->loop_scratch + (size_t)p * count, peer->dev_M, (size_t)count * 8,
                                hipMemcpyDeviceToDevice, s);
        });
        rc != KS_OK)
      return rc;
    hipLaunchKernelGGL(max_reduce_kernel, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, s, buf,
                       (const unsigned long long*)ctx->loop_scratch, ctx->nranks, ctx->rank, count);
    HIPCHK(ctx, hipGetLastError());
    return KS_OK;
  }
  const ncclResult_t r = ncclAllReduce(buf, buf, count, ncclUint64, ncclMax, ctx->comm, s);
  if (r != ncclSuccess) KS_FAIL(ctx, KS_EHIP, "ncclAllReduce (normalization maxima): %s", ncclGetErrorString(r));
  return KS_OK;
}

// Launch shape of the dirty-chunk re-sweep of a pipelined pass; pipe == nullptr: not pipelined.
struct PipeShape {
  int32_t fix_ppw;
  int fix_blocks;
  int list_blocks;  // patched: one wave per (pod, list entry)
  bool patch;  // monotone plugin sets: select before the previous commit ends, re-evaluate the listed chunks after
};

// The per-node outputs of one pod's full evaluation (ks_eval_pod, the topology step) in a scratch buffer that lives
// with the context (grown, never freed per call): reasons, the per-plugin score matrix, totals, raw scores
struct EvBuf {
  uint32_t* dr;
  int64_t *ds, *dt;
  int32_t *draw, *dhi, *ddraw, *dtraw, *daraw;
};
static int ev_buffers(ks_ctx* ctx, EvBuf& b) {
  const int64_t n = ctx->n;
  const size_t bytes = (size_t)(n > 0 ? n : 1) * (4 + 8 * KS_NUM_SCORE_PLUGINS + 8 + 8 + 4 + 8) + 64;
  if (ctx->evbuf_bytes < bytes) {
    dev_free(ctx->evbuf);
    ctx->evbuf_bytes = 0;
    if (dev_alloc(ctx, &ctx->evbuf, bytes) != KS_OK) return KS_ENOMEM;
    ctx->evbuf_bytes = bytes;
  }
  void* buf = ctx->evbuf;
  b.dr = (uint32_t*)buf;
  b.ds = (int64_t*)((char*)buf + ((size_t)n * 4 + 15) / 16 * 16);
  b.dt = b.ds + (size_t)n * KS_NUM_SCORE_PLUGINS;
  b.draw = (int32_t*)(b.dt + n);
  b.dhi = b.draw + n;
  b.ddraw = b.dhi + n;
  b.dtraw = b.ddraw + n;
  b.daraw = b.dtraw + n;
  return KS_OK;
}

// The topology kernels' arguments for stage st: the pod at *cursor (the batch step) or pod 0 (cursor NULL,
// ks_eval_pod)
static TopoKArgs topo_args(ks_ctx* ctx, PodStage& st, const int32_t* cursor, const EvBuf& eb) {
  TopoKArgs a{};
  a.t = dev_topo(ctx);
  a.labels = ctx->d.labels;
  a.stat = st.stat;
  a.trec = st.topo;
  a.terms = st.topo_terms;
  a.cursor = cursor;
  a.total_pods = cursor ? ctx->np : 1;
  a.n = ctx->n;
  a.reasons = eb.dr;
  a.scores = eb.ds;
  a.total = eb.dt;
  a.rraw = eb.draw;
  a.rhi = eb.dhi;
  a.draw = eb.ddraw;
  a.traw = eb.dtraw;
  a.araw = eb.daraw;
  a.sraw = ctx->topo_sraw;
  a.iraw = ctx->topo_iraw;
  a.dev_on = ctx->kc.dev;
  a.taint_on = (ctx->kc.taint & 2) != 0;
  a.aff_on = (ctx->kc.aff & 2) != 0;
  a.rsv_on = ctx->kc.rsv;
  a.dev_w = ctx->cfg.deviceshare.plugin_weight;
  a.taint_w = ctx->cfg.taint.plugin_weight;
  a.aff_w = ctx->cfg.affinity.plugin_weight;
  a.rsv_w = ctx->cfg.reservation.plugin_weight;
  a.spread_w = ctx->cfg.topology.spread_weight;
  a.ipa_w = ctx->cfg.topology.affinity_weight;
  a.scr = ctx->topo_scr;
  if (cursor) {
    a.cand_chunk = ctx->topo_cchunk;
    a.cand_t = ctx->topo_ct;
    a.cand_count = ctx->topo_ccount;
    a.cand_bound = ctx->topo_cbound;
    a.cand_top = ctx->topo_ctop;
    a.cand_second = ctx->topo_csecond;
  }
  return a;
}

// the pass's CPU ids (cores mode): exact per-node core counts for the next sweep (Cfg.cores)
static int cores_pass_refresh(ks_ctx* ctx) {
  if (!(ctx->kc.cores && ctx->cpu_loaded)) return KS_OK;
  hipLaunchKernelGGL(cpuset_kernel, dim3((unsigned)((ctx->n + 255) / 256)), dim3(256), 0, ctx->stream, ctx->cpu,
                     (const int2*)ctx->cpuset_list, (const int32_t*)ctx->cpuset_n, (const uint32_t*)ctx->cpuset_split,
                     (const PodRec*)ctx->st.recs, ctx->cpuset_out, (const uint32_t*)ctx->d.numa_flags,
                     ctx->d.cpu_cores, (int32_t)(ctx->cfg.numa.numa_scoring_strategy == KS_MOST_ALLOCATED),
                     numa_words(ctx), ctx->nv.npad, ctx->n);
  HIPCHK(ctx, hipMemsetAsync(ctx->cpuset_n, 0, 4, ctx->stream));
  return KS_OK;
}

// The topology step (ks_topo.h): when the pod at the cursor is a topology pod, every plugin's Filter / Score on every
// node, the two plugins' PreFilter / Filter / PreScore / Score and every normalization, selectHost, and the commit of
// that one pod on the chosen node (admission, every Reserve, the counters); otherwise every kernel returns at once.
static int topo_step(ks_ctx* ctx) {
  EvBuf eb;
  if (ev_buffers(ctx, eb) != KS_OK) return KS_ENOMEM;
  const int64_t n = ctx->n;
  TopoKArgs ta = topo_args(ctx, ctx->st, ctx->cursor, eb);
  ta.scores = nullptr;  // (the batch step returns no per-plugin score matrix)
  HIPCHK(ctx, launch_topo_sums(ctx->stream, ta));
  HIPCHK(ctx, launch_eval_debug(ctx->nsc, (int)((n + 255) / 256), ctx->stream, ctx->d, ctx->drv, ctx->ddv, ctx->dnv,
                                ctx->kc, ctx->st.recs, n, eb.dr, nullptr, eb.dt, eb.draw, eb.dhi, eb.ddraw, ctx->st.stat,
                                eb.dtraw, eb.daraw, &ta, kernel_feat(ctx)));
  HIPCHK(ctx, launch_topo_pts(ctx->stream, ta));
  const int feat = kernel_feat(ctx);
  if ((feat == 0 || feat == 4) && !ctx->kc.dev && !ctx->kc.rsv && !ctx->kc.numa && !ctx->cpu_loaded) {
    // Reserve = NodeInfo.AddPod + the LoadAware assign cache + ElasticQuota: the lean commit, by the normalize
    // kernel's last workgroup
    TopoCommitArgs tc;
    tc.d = ctx->d;
    tc.q = ctx->q;
    tc.pq = ctx->st.pq;
    tc.pods = ctx->st.recs;
    tc.pstat = ctx->st.stat;
    tc.trec = ctx->st.topo;
    tc.props = ctx->st.topo_props;
    tc.cursor = ctx->cursor;
    tc.total_pods = ctx->np;
    tc.quota_enable = ctx->kc.quota_enable;
    tc.quota_parent = ctx->kc.quota_parent;
    tc.ports = ctx->kc.ports;
    tc.results = ctx->st.results;
    tc.counters = ctx->counters;
    tc.topo_count = ctx->topo_count;
    tc.topo_npad = ctx->npad;
    tc.scr = ctx->topo_scr;
    HIPCHK(ctx, launch_topo_norm(ctx->stream, ta, &tc));
    return KS_OK;
  }
  HIPCHK(ctx, launch_topo_norm(ctx->stream, ta));
  bool qcache = false;
  size_t smem = 0;
  CommitArgs ca = commit_args(ctx, ctx->st, ctx->np, 1, &qcache, &smem);
  if (qcache) {
    // one pod: the quota rows are read from HBM (copying the table into LDS would cost more than the pod's reads)
    qcache = false;  // (the reservation cache that fit next to the quota rows fits without them)
    smem = commit_layout(ctx->k, ctx->nchunks, false, (size_t)ca.rsv_bytes, (size_t)ca.dev_bytes, (size_t)ca.numa_bytes,
                         ctx->q.q, kernel_feat(ctx) == 0, commit_hint_variant(ctx)).total;
  }
  ca.topo = 2;
  ca.cand_chunk = ctx->topo_cchunk;
  ca.cand_t = ctx->topo_ct;
  ca.cand_count = ctx->topo_ccount;
  ca.cand_bound = ctx->topo_cbound;
  ca.cand_top = ctx->topo_ctop;
  ca.cand_second = ctx->topo_csecond;
  HIPCHK(ctx, pass_launcher(kernel_feat(ctx), ctx->nsc).commit(qcache, smem, ctx->stream, ca));
  return cores_pass_refresh(ctx);
}

template <int NSC>
static int launch_pass(ks_ctx* ctx, int32_t ppw, int sweep_blocks, const PipeShape* pipe,
                       std::vector<std::pair<int, size_t>>* evs, size_t* evn) {
  // Pipelined: the sweep and the select run on sstream; the sweep of pass k runs while commit k-1 does
  // (for the pods after commit k-1's, speculatively), then the chunks commit k-1 wrote are re-swept, so the select
  // and commit k see exactly what a sweep after commit k-1 gives.  Otherwise everything runs on ctx->stream.
  // Patched (monotone plugin sets on one shard): sweep k and select k run on sstream as soon as commit k-2 is done
  // (concurrently with commit k-1), into the sweep output and list set of parity k & 1; after commit k-1 the fix
  // stream re-evaluates the listed chunks it wrote in place (sweep_kernel's list mode), and commit k runs on them.
  hipStream_t ss = pipe ? ctx->sstream : ctx->stream;
  const int64_t k = ctx->pipe_k;
  const int32_t S = ctx->nranks * ctx->vshards;
  const bool patch = pipe && pipe->patch;
  // the re-sweep (and patch): patched passes run it on the commit stream, between commit k-1 and commit k
  hipStream_t fs = patch ? ctx->cstream : ss;
  const CandSet cset = cand_set(ctx, patch ? (int)(k & 1) : 0);
  uint2* sout = ctx->sweep_out + (patch ? (size_t)(k & 1) * kMaxBatch * ctx->nchunks : 0);
  int32_t* base = pipe ? ctx->pipe + (k & 1) : ctx->cursor;  // the first pod this pass sweeps
  int32_t* carry = ctx->pipe + 4;
  auto rec = [&](int kind, hipStream_t s) {
    if (!evs) return;
    hipEvent_t e = take_event(ctx, *evn);
    (void)hipEventRecord(e, s);
    evs->push_back({kind, (*evn)++});
  };
  auto shard_lo = [&](int32_t sh) { return ctx->nchunks * sh / S; };
  if (ctx->cfg.topology.enable && ctx->st.ndyn > 0 && !pipe) {
    // the topology pods at the cursor are scheduled alone first, up to topo_k of them in a row (timed with the
    // commits); a step whose cursor pod is not one costs its launches only
    rec(2, ctx->stream);
    for (int32_t t = 0; t < ctx->topo_k; ++t)
      if (int rc = topo_step(ctx); rc != KS_OK) return rc;
    rec(2, ctx->stream);
  }
  SweepArgs sa;
  sa.dn = ctx->dnodes;
  sa.rv = ctx->drv;
  sa.c = ctx->kc;
  sa.pods = ctx->st.recs;
  sa.cursor = base;
  sa.out = sout;
  sa.n = ctx->n;
  sa.nchunks = ctx->nchunks;
  sa.c0 = shard_lo(ctx->rank * ctx->vshards);
  sa.c1 = shard_lo((ctx->rank + 1) * ctx->vshards);
  sa.total_pods = ctx->np;
  sa.batch = ctx->batch;
  sa.ppw = ppw;
  sa.fix = nullptr;
  sa.fix_cursor = nullptr;
  sa.list_t = nullptr;
  sa.list_chunk = nullptr;
  sa.list_count = nullptr;
  sa.list_bound = nullptr;
  sa.list_top = nullptr;
  sa.list_k = 0;
  const int feat = kernel_feat(ctx);
  sa.dv = ctx->ddv;
  sa.nv = ctx->dnv;
  sa.dev_M = ctx->dev_M;
  sa.dcache = (ctx->kc.dev && !ctx->kc.rsv && !ctx->kc.stat && ctx->dcache_words >= (int64_t)kMaxBatch * ctx->npad)
                  ? ctx->dcache : nullptr;
  sa.pstat = ctx->st.stat;
  sa.dstride = ctx->npad;
  sa.phase = 1;
  // One sweep launch per virtual shard (a rank's virtual shards are swept as separate chunk ranges, so the
  // c0 > 0 decode of every non-first shard runs on one GPU too); timed together as one launch.
  const PassLaunch pl = pass_launcher(feat, NSC);
  hipError_t le = hipSuccess;
  auto sweep = [&](int blocks, hipStream_t st) {
    for (int32_t v = 0; v < ctx->vshards && le == hipSuccess; ++v) {
      const int32_t sh = ctx->rank * ctx->vshards + v;
      sa.c0 = shard_lo(sh);
      sa.c1 = shard_lo(sh + 1);
      le = pl.sweep(blocks, st, sa);
    }
  };
  // patched: commit k-2 wrote this pass's first pod and its rows are final
  if (patch && k >= 2) HIPCHK(ctx, hipStreamWaitEvent(ss, ctx->pev_com[(k - 2) % kPipeEvents], 0));
  if (feat & 4) {
    // DeviceShare: phase 0 reduces the per-pod normalization max, (RCCL max over the ranks), phase 1 keys;
    // each launch is timed on its own (the roofline is per sweep launch)
    HIPCHK(ctx, hipMemsetAsync(ctx->dev_M, 0, kNormRows * kMaxBatch * 8, ss));
    sa.phase = 0;
    rec(0, ss);
    sweep(sweep_blocks, ss);
    rec(0, ss);
    if (ctx->comm || ctx->loop)
      if (int rc = exchange_allreduce_max(ctx, ctx->dev_M, kNormRows * kMaxBatch, ss); rc != KS_OK) return rc;
    sa.phase = 1;
    rec(0, ss);
    sweep(sweep_blocks, ss);
  } else {
    rec(0, ss);
    sweep(sweep_blocks, ss);
  }
  HIPCHK(ctx, le);
  rec(0, ss);
  auto fix = [&]() -> int {
    // after commit k-1: its rows' chunks again, for the same pods (nothing when the sweep's pods are not where
    // commit k-1 left the cursor: commit k is then a bubble)
    if (patch) {
      // the select must have read the stale keys before the re-sweep overwrites them (commit k-1 is ahead of
      // the re-sweep on the same stream)
      HIPCHK(ctx, hipEventRecord(ctx->pev_sel[k % kPipeEvents], ss));
      HIPCHK(ctx, hipStreamWaitEvent(fs, ctx->pev_sel[k % kPipeEvents], 0));
    } else if (k > 0) {
      HIPCHK(ctx, hipStreamWaitEvent(fs, ctx->pev_com[(k - 1) % kPipeEvents], 0));
    }
    sa.fix = carry;
    sa.fix_cursor = ctx->cursor;
    sa.ppw = pipe->fix_ppw;
    rec(3, fs);
    if (patch) {
      // the listed chunks commit k-1 wrote, re-evaluated in place; the pods' tops rebuilt (ks_pass.h)
      sa.list_t = cset.t;
      sa.list_chunk = cset.chunk;
      sa.list_count = cset.count;
      sa.list_bound = cset.bound;
      sa.list_top = ctx->pipe_top + (size_t)(k & 1) * kMaxBatch;
      sa.list_k = ctx->k;
      le = pl.sweep(pipe->list_blocks, fs, sa);  // once: the (merged) lists span every shard's chunks
    } else {
      sweep(pipe->fix_blocks, fs);
    }
    HIPCHK(ctx, le);
    rec(3, fs);
    return KS_OK;
  };
  if (pipe && !patch)
    if (int rc = fix(); rc != KS_OK) return rc;
  SelectArgs se;
  se.in = sout;
  se.cursor = base;
  se.nchunks = ctx->nchunks;
  se.total_pods = ctx->np;
  se.batch = ctx->batch;
  se.k = ctx->k;
  se.real_cursor = ctx->cursor;
  se.pods = ctx->st.recs;
  const CandSlot L = cand_slot_layout(ctx->k);
  rec(1, ss);
  for (int32_t v = 0; v < ctx->vshards; ++v) {
    const int32_t sh = ctx->rank * ctx->vshards + v;
    se.c0 = shard_lo(sh);
    se.c1 = shard_lo(sh + 1);
    se.next_base = (pipe && !patch && v == 0) ? ctx->pipe + ((k + 1) & 1) : nullptr;
    if (S == 1) {
      se.cand_chunk = cset.chunk;
      se.cand_t = cset.t;
      se.cand_bound = cset.bound;
      se.cand_top = cset.top;
      se.cand_second = cset.second;
      se.cand_count = cset.count;
      se.cand_total = cset.total;
    } else {
      unsigned char* b = ctx->gather + (size_t)sh * L.bytes;
      se.cand_chunk = (uint32_t*)(b + L.chunk);
      se.cand_t = (uint2*)(b + L.t);
      se.cand_bound = cset.bound;  // scratch: recomputed by the merge
      se.cand_top = (uint64_t*)(b + L.top);
      se.cand_second = cset.second;  // scratch: recomputed by the merge
      se.cand_count = (int32_t*)(b + L.count);
      se.cand_total = (int32_t*)(b + L.total);
    }
    hipLaunchKernelGGL(select_kernel, dim3(kSelBlocks), dim3(kSelThreads), select_smem(se.c1 - se.c0), ss, se);
  }
  if (S > 1) {
    if (ctx->comm || ctx->loop)  // every rank's candidate slots to every rank (one RCCL allgather per pass over xGMI)
      if (int rc = exchange_allgather(ctx, (size_t)ctx->vshards * L.bytes, ss); rc != KS_OK) return rc;
    MergeArgs ma;
    ma.gather = ctx->gather;
    ma.cursor = base;
    ma.cand_chunk = cset.chunk;
    ma.cand_t = cset.t;
    ma.cand_bound = cset.bound;
    ma.cand_top = cset.top;
    ma.cand_second = cset.second;
    ma.cand_count = cset.count;
    ma.nslots = S;
    ma.total_pods = ctx->np;
    ma.batch = ctx->batch;
    ma.k = ctx->k;
    hipLaunchKernelGGL(merge_kernel, dim3(ctx->batch), dim3(64), 0, ss, ma);
  }
  rec(1, ss);
  if (patch)
    if (int rc = fix(); rc != KS_OK) return rc;
  hipStream_t cs = pipe ? ctx->cstream : ctx->stream;
  if (patch) {
    // the re-sweep and the patch ran on cs
  } else if (pipe) {
    HIPCHK(ctx, hipEventRecord(ctx->pev_sel[k % kPipeEvents], ss));
    HIPCHK(ctx, hipStreamWaitEvent(cs, ctx->pev_sel[k % kPipeEvents], 0));
  }
  bool qcache = false;
  size_t smem = 0;
  CommitArgs ca = commit_args(ctx, ctx->st, ctx->np, ctx->batch, &qcache, &smem);
  if (pipe) {
    ca.pipe_base = base;
    ca.carry = carry;
  }
  ca.cand_chunk = cset.chunk;
  ca.cand_t = cset.t;
  ca.cand_bound = cset.bound;
  ca.cand_top = cset.top;
  ca.cand_second = cset.second;
  ca.cand_count = cset.count;
  if (patch) {
    ca.pipe_follow = ctx->pipe + ((k + 1) & 1);
    ca.pipe_after = base;
    ca.cand_top = (const uint64_t*)(ctx->pipe_top + (size_t)(k & 1) * kMaxBatch);  // rebuilt by the list re-evaluation
    ca.top_reset = ctx->pipe_top + (size_t)(k & 1) * kMaxBatch;
  }
  size_t msmem = 0;
  const bool mono = mono_commit(ctx, qcache, &msmem);
  if (!mono && !pipe && pl.reserve_pre && pre_reserve(ctx)) ca.pre_rsv = ctx->pre_rsv;
  rec(2, cs);
  if (ca.pre_rsv) HIPCHK(ctx, pl.reserve_pre(ctx->batch, cs, ca));  // (timed with the commit)
  if (mono) HIPCHK(ctx, pl.commit_mono(qcache, msmem, cs, ca));
  else HIPCHK(ctx, pl.commit(qcache, smem, cs, ca));
  rec(2, cs);
  if (pipe) HIPCHK(ctx, hipEventRecord(ctx->pev_com[k % kPipeEvents], cs));
  ctx->pipe_k = k + 1;
  // the pass's CPU ids now, so that the next sweep sees exact per-node core counts (Cfg.cores)
  return cores_pass_refresh(ctx);
}

static int schedule_staged_impl(ks_ctx* ctx) {
  if (!ctx->node_blob) KS_FAIL(ctx, KS_ESTATE, "schedule before ks_load_nodes");
  HIPCHK(ctx, hipSetDevice(ctx->device));
  bind_mode(ctx, ctx->staged_bind_required);
  ctx->cpusets_clobbered = false;
  ctx->stats = ks_stats{};
  const int32_t np = ctx->np;
  if (np == 0) return KS_OK;
  {
    if (int rc = commit_attr_set(ctx); rc != KS_OK) return rc;
    hipError_t e = hipSuccess;
    const size_t sel_smem = select_smem(ctx->nchunks);
    if (sel_smem > 160 * 1024) KS_FAIL(ctx, KS_EUNSUPPORTED, "too many nodes for the select kernel's LDS (%lld nodes)", (long long)ctx->n);
    e = hipFuncSetAttribute((const void*)select_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sel_smem);
    if (e != hipSuccess) KS_FAIL(ctx, KS_EHIP, "hipFuncSetAttribute(select LDS %zu): %s", sel_smem, hipGetErrorString(e));
    if (ctx->kc.dev && !ctx->kc.rsv && !ctx->kc.stat && ctx->dcache_words < (int64_t)kMaxBatch * ctx->npad) {
      void* q = ctx->dcache;
      dev_free(q);
      ctx->dcache = nullptr;
      ctx->dcache_words = 0;
      if (dev_alloc(ctx, &q, (size_t)kMaxBatch * ctx->npad * 8) != KS_OK) return KS_ENOMEM;
      ctx->dcache = (unsigned long long*)q;
      ctx->dcache_words = (int64_t)kMaxBatch * ctx->npad;
    }
    const size_t gb = (size_t)ctx->nranks * ctx->vshards * cand_slot_layout(ctx->k).bytes;
    if (ctx->nranks * ctx->vshards > 1 && ctx->gather_bytes < gb) {
      void* g = ctx->gather;
      dev_free(g);
      ctx->gather = nullptr;
      if (dev_alloc(ctx, &g, gb) != KS_OK) return KS_ENOMEM;
      HIPCHK(ctx, hipMemsetAsync(g, 0, gb, ctx->stream));
      ctx->gather = (unsigned char*)g;
      ctx->gather_bytes = gb;
    }
  }
  // topology steps per regular pass: about the queue's topology pods per other pod (a regular pass that meets a
  // topology pod at the cursor costs its launches for nothing), 1..8
  ctx->topo_k = 1;
  if (ctx->cfg.topology.enable && ctx->st.ndyn > 0)
    ctx->topo_k = (int32_t)std::min<int64_t>(8, 1 + (int64_t)ctx->st.ndyn / std::max<int64_t>(1, (int64_t)np - ctx->st.ndyn));
  // pods per wave: aim for >= ~4096 waves per sweep
  const int64_t S = (int64_t)ctx->nranks * ctx->vshards;
  const int64_t local_chunks = ctx->nchunks * (ctx->rank + 1) * ctx->vshards / S - ctx->nchunks * ctx->rank * ctx->vshards / S;
  static const int64_t env_waves = env_i64("KS_SWEEP_WAVES", 4096, 64, (int64_t)1 << 24);
  static const int64_t env_ppw = env_i64("KS_SWEEP_PPW", 0, 1, kMaxBatch);
  static const int64_t env_cap = env_i64("KS_SWEEP_BLOCK_CAP", 2048, 8, 65535 * 8);
  int32_t ppw = 64;
  while (ppw > 4 && local_chunks * (ctx->batch / ppw) < env_waves) ppw >>= 1;
  if (env_ppw > 0) ppw = (int32_t)env_ppw;
  if (ppw > ctx->batch) ppw = ctx->batch;
  const int64_t nwork = std::max<int64_t>(local_chunks, 1) * ((ctx->batch + ppw - 1) / ppw);
  const int sweep_blocks = (int)((std::max<int64_t>(1, std::min<int64_t>((nwork + 3) / 4, env_cap)) + 7) & ~7ll);  // % 8 == 0 (XCD swizzle)
  if (ensure_cpuset_bufs(ctx, np) != KS_OK) return KS_ENOMEM;
  hipEvent_t t0 = take_event(ctx, 0), t1 = take_event(ctx, 1);
  if (ctx->cpuset_list) {
    HIPCHK(ctx, hipMemsetAsync(ctx->cpuset_n, 0, 4, ctx->stream));
    HIPCHK(ctx, hipMemsetAsync(ctx->cpuset_out, 0, (size_t)np * sizeof(CpuSet), ctx->stream));
    HIPCHK(ctx, hipMemsetAsync(ctx->numa_alloc, 0, (size_t)np * 2 * kNumaDev * 8, ctx->stream));
  }
  HIPCHK(ctx, hipMemsetAsync(ctx->cursor, 0, 4, ctx->stream));
  HIPCHK(ctx, hipMemsetAsync(ctx->counters, 0, 256, ctx->stream));
  // pipelined passes: pass 0 sweeps from pod 0, no commit has written rows yet
  PipeShape pshape{};
  const PipeShape* pipe = nullptr;
  if (pipelined(ctx)) {
    if (ensure_pipe(ctx) != KS_OK) return KS_EHIP;
    static const int64_t env_patch = env_i64("KS_PIPE_PATCH", 1, 0, 1);
    pshape.patch = env_patch != 0 && ctx->kc.monotone;
    // the re-sweep runs on the commit stream's few CUs when patched: more pods per wave, fewer waves
    static const int64_t env_fix_ppw = env_i64("KS_PIPE_FIX_PPW", 0, 1, kMaxBatch);
    pshape.fix_ppw = (int32_t)std::min<int64_t>(env_fix_ppw > 0 ? env_fix_ppw : (pshape.patch ? 16 : 2), ctx->batch);
    const int64_t fwork = (int64_t)kMaxBatch * ((ctx->batch + pshape.fix_ppw - 1) / pshape.fix_ppw);
    pshape.fix_blocks = (int)((std::max<int64_t>(1, (fwork + 3) / 4) + 7) & ~7ll);
    pshape.list_blocks = (int)((((int64_t)ctx->batch * ctx->k + 3) / 4 + 7) & ~7ll);
    pipe = &pshape;
    HIPCHK(ctx, hipMemsetAsync(ctx->pipe, 0, kPipeWords * 4, ctx->stream));
    // patched: pass 1's sweep starts before commit 0 has decided anything, behind pass 0's pods
    if (pshape.patch) {
      HIPCHK(ctx, hipMemsetD32Async((hipDeviceptr_t)(ctx->pipe + 1), std::min(ctx->batch, np), 1, ctx->stream));
      HIPCHK(ctx, hipMemsetAsync(ctx->pipe_top, 0, 2 * kMaxBatch * 8, ctx->stream));
    }
    ctx->pipe_k = 0;
  }
  HIPCHK(ctx, hipEventRecord(t0, ctx->stream));
  // PreFilter / EstimatePod for the staged queue (the pods' request vectors, estimates, flags)
  if (prep_stage(ctx, ctx->st, np) != KS_OK) return KS_EHIP;
  hipStream_t cs = pipe ? ctx->cstream : ctx->stream;  // where the commits (and the cursor read-back) run
  if (pipe) {
    // the sweep and commit streams start after everything before them on the context's stream
    HIPCHK(ctx, hipEventRecord(ctx->pev_com[kPipeEvents - 1], ctx->stream));
    HIPCHK(ctx, hipStreamWaitEvent(ctx->sstream, ctx->pev_com[kPipeEvents - 1], 0));
    if (cs != ctx->stream) HIPCHK(ctx, hipStreamWaitEvent(cs, ctx->pev_com[kPipeEvents - 1], 0));
  }
  std::vector<std::pair<int, size_t>> evs;
  size_t evn = 2;
  int32_t host_cursor = 0;
  int rounds = 0;
  auto one_pass = [&](std::vector<std::pair<int, size_t>>* ev) -> int {
    switch (ctx->nsc) {
      case 0: return launch_pass<0>(ctx, ppw, sweep_blocks, pipe, ev, &evn);
      case 2: return launch_pass<2>(ctx, ppw, sweep_blocks, pipe, ev, &evn);
      default: return launch_pass<4>(ctx, ppw, sweep_blocks, pipe, ev, &evn);
    }
  };
  // Topology pods (ks_topo.h): an iteration is topo_k topology steps + a regular pass, ~10 launches per pod, which the
  // host's launch rate would bound; kGraphIters iterations are captured into one HIP graph and launched as one (not
  // with per-kernel profiling events, not pipelined)
  hipGraphExec_t gexec = nullptr;
  static const int64_t env_graph = env_i64("KS_TOPO_GRAPH", 1, 0, 1);
  constexpr int32_t kGraphIters = 4;
  if (ctx->cfg.topology.enable && ctx->st.ndyn > 0 && !pipe && !ctx->cfg.profile && env_graph && !ctx->comm && !ctx->loop) {
    EvBuf eb;
    if (ev_buffers(ctx, eb) != KS_OK) return KS_ENOMEM;  // (allocated before the capture)
    hipGraph_t graph = nullptr;
    HIPCHK(ctx, hipStreamBeginCapture(ctx->stream, hipStreamCaptureModeThreadLocal));
    int rc = KS_OK;
    for (int32_t i = 0; i < kGraphIters && rc == KS_OK; ++i) rc = one_pass(nullptr);
    const hipError_t ee = hipStreamEndCapture(ctx->stream, &graph);
    if (rc != KS_OK) {
      if (graph) (void)hipGraphDestroy(graph);
      return rc;
    }
    HIPCHK(ctx, ee);
    const hipError_t ie = hipGraphInstantiate(&gexec, graph, nullptr, nullptr, 0);
    (void)hipGraphDestroy(graph);
    HIPCHK(ctx, ie);
  }
  struct GraphGuard {
    hipGraphExec_t& g;
    ~GraphGuard() {
      if (g) (void)hipGraphExecDestroy(g);
    }
  } graph_guard{gexec};
  while (host_cursor < np) {
    const int32_t remaining = np - host_cursor;
    const int32_t g = std::min<int32_t>((remaining + ctx->batch - 1) / ctx->batch, 256);
    for (int32_t i = 0; i < g; i += gexec ? kGraphIters : 1) {
      if (gexec) {
        HIPCHK(ctx, hipGraphLaunch(gexec, ctx->stream));
        continue;
      }
      if (int rc = one_pass(ctx->cfg.profile ? &evs : nullptr); rc != KS_OK) return rc;
    }
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, hipMemcpyAsync(&host_cursor, ctx->cursor, 4, hipMemcpyDeviceToHost, cs));
    HIPCHK(ctx, hipStreamSynchronize(cs));
    if (++rounds > 1000000) KS_FAIL(ctx, KS_EHIP, "schedule made no progress");
  }
  if (cs != ctx->stream) {
    // everything after the passes runs on the context's stream again
    HIPCHK(ctx, hipEventRecord(ctx->pev_com[0], cs));
    HIPCHK(ctx, hipStreamWaitEvent(ctx->stream, ctx->pev_com[0], 0));
  }
  if (ctx->cpu_loaded && ctx->n > 0) {
    // the CPU ids of the pass's cpu-bind Reserves (ks_cpuset.h), per node in placement order
    hipLaunchKernelGGL(cpuset_kernel, dim3((unsigned)((ctx->n + 255) / 256)), dim3(256), 0, ctx->stream, ctx->cpu,
                       (const int2*)ctx->cpuset_list, (const int32_t*)ctx->cpuset_n, (const uint32_t*)ctx->cpuset_split,
                       (const PodRec*)ctx->st.recs, ctx->cpuset_out, (const uint32_t*)ctx->d.numa_flags,
                       ctx->d.cpu_cores, (int32_t)(ctx->cfg.numa.numa_scoring_strategy == KS_MOST_ALLOCATED),
                       numa_words(ctx), ctx->nv.npad, ctx->n);
    HIPCHK(ctx, hipGetLastError());
  }
  HIPCHK(ctx, hipEventRecord(t1, ctx->stream));
  unsigned long long cnt[16] = {0};
  HIPCHK(ctx, hipMemcpyAsync(cnt, ctx->counters, sizeof(cnt), hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  float ms = 0;
  (void)hipEventElapsedTime(&ms, t0, t1);
  ctx->stats.total_ms = ms;
  ctx->stats.passes = (int64_t)cnt[0];
  ctx->stats.cut_passes = (int64_t)cnt[1];
  ctx->stats.rescans = (int64_t)cnt[2];
  ctx->stats.slot_misses = (int64_t)cnt[3];
  ctx->stats.bubble_passes = (int64_t)cnt[4];
  ctx->stats.pre_reserves = (int64_t)cnt[5];
  ctx->stats.pipelined = pipe ? (pipe->patch ? 2 : 1) : 0;
  {
    bool qc = false;
    const int32_t rcap = commit_rcap(ctx, &qc);
    const CommitLayout L = commit_layout(ctx->k, ctx->nchunks, qc, rsv_cache_bytes(ctx, rcap), dev_cache_bytes(ctx),
                                         numa_cache_bytes(ctx), ctx->q.q, kernel_feat(ctx) == 0, commit_hint_variant(ctx));
    ctx->stats.commit_lds_bytes = (int64_t)L.total;
    ctx->stats.commit_helpers = L.hint ? 1 : 0;
  }
  for (int i = 0; i < 8; ++i) ctx->stats.diag[i] = (int64_t)cnt[8 + i];
  for (size_t i = 0; i + 1 < evs.size(); i += 2) {
    float e = 0;
    (void)hipEventElapsedTime(&e, ctx->ev_pool[evs[i].second], ctx->ev_pool[evs[i + 1].second]);
    if (evs[i].first == 0) {
      ctx->stats.sweep_ms += e;
      ctx->stats.sweep_launches += 1;
    } else if (evs[i].first == 1) {
      ctx->stats.select_ms += e;
    } else if (evs[i].first == 3) {
      ctx->stats.fixup_ms += e;
    } else {
      ctx->stats.commit_ms += e;
    }
  }
  // algorithmic bytes of one full sweep launch: node columns read once per pod group + outputs
  int64_t b_node = 8 * 15 + 4 * 3 + (int64_t)ctx->nsc * 16 + (ctx->kc.rsv ? 8 : 0) + (ctx->kc.numa ? 16 : 0) +
                   (ctx->kc.dev ? 4 + (kDevTW + kDevQW) * 8 : 0);
  const int64_t groups = (ctx->batch + ppw - 1) / ppw;
  ctx->stats.sweep_bytes = local_chunks * 64 * b_node * groups + (int64_t)ctx->batch * sizeof(PodRec) + local_chunks * 64 * 4;
  return KS_OK;
}

int ks_schedule_staged(ks_ctx* ctx) {
  if (!ctx) return KS_EINVAL;
  return schedule_staged_impl(ctx);
}

int ks_fetch_results(ks_ctx* ctx, ks_result* out, int32_t p) {
  if (!ctx || !out || p < 0 || p > ctx->np) return ctx ? (ctx->err = "ks_fetch_results: bad args", KS_EINVAL) : KS_EINVAL;
  if (p == 0) return KS_OK;
  HIPCHK(ctx, hipMemcpyAsync(out, ctx->st.results, (size_t)p * sizeof(ks_result), hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  return KS_OK;
}

int ks_schedule(ks_ctx* ctx, const ks_pod_cols* pods, int32_t p, ks_result* out) {
  int rc = ks_stage_pods(ctx, pods, p);
  if (rc != KS_OK) return rc;
  rc = ks_schedule_staged(ctx);
  if (rc != KS_OK) return rc;
  return ks_fetch_results(ctx, out, p);
}

int ks_checkpoint(ks_ctx* ctx) {
  if (!ctx || !ctx->node_blob) return ctx ? (ctx->err = "ks_checkpoint before ks_load_nodes", KS_ESTATE) : KS_EINVAL;
  if (!ctx->ckpt_blob && dev_alloc(ctx, &ctx->ckpt_blob, ctx->mut_bytes) != KS_OK) return KS_ENOMEM;
  HIPCHK(ctx, hipMemcpyAsync(ctx->ckpt_blob, ctx->node_blob, ctx->mut_bytes, hipMemcpyDeviceToDevice, ctx->stream));
  if (ctx->quota_blob) {
    const size_t tb = (size_t)(ctx->q.q > 0 ? ctx->q.q : 1) * KS_QUOTA_DIMS * 8;
    HIPCHK(ctx, hipMemcpyAsync(ctx->quota_used_ckpt, ctx->q.used, tb, hipMemcpyDeviceToDevice, ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(ctx->quota_npused_ckpt, ctx->q.npused, tb, hipMemcpyDeviceToDevice, ctx->stream));
  }
  if (ctx->dev_blob)
    HIPCHK(ctx, hipMemcpyAsync(ctx->dev_used_ckpt, ctx->dv.used, (size_t)kDevQW * ctx->dv.npad * 8, hipMemcpyDeviceToDevice, ctx->stream));
  if (ctx->cpu_loaded)
    HIPCHK(ctx, hipMemcpyAsync(ctx->cpu_ckpt, ctx->cpu.allocated, (size_t)3 * ctx->cpu.npad * sizeof(CpuSet), hipMemcpyDeviceToDevice, ctx->stream));
  if (ctx->numa_blob)
    HIPCHK(ctx, hipMemcpyAsync(ctx->numa_ckpt, ctx->nv.used, numa_mut_bytes((size_t)ctx->npad), hipMemcpyDeviceToDevice, ctx->stream));
  if (ctx->rsv_blob) {
    HIPCHK(ctx, hipMemcpyAsync(ctx->rsv_allocd_ckpt, ctx->rv.allocd, (size_t)kRsvDims * ctx->rv.nr * 8, hipMemcpyDeviceToDevice, ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(ctx->rsv_dald_ckpt, ctx->rv.dald, (size_t)kDevQW * ctx->rv.nr * 8, hipMemcpyDeviceToDevice, ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(ctx->rsv_assigned_ckpt, ctx->rv.assigned, (size_t)ctx->rv.nr * 4, hipMemcpyDeviceToDevice, ctx->stream));
  }
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  ctx->h_dev_assumed_ckpt = ctx->h_dev_assumed;
  return KS_OK;
}

int ks_restore(ks_ctx* ctx) {
  if (!ctx || !ctx->ckpt_blob) return ctx ? (ctx->err = "ks_restore without ks_checkpoint", KS_ESTATE) : KS_EINVAL;
  HIPCHK(ctx, hipMemcpyAsync(ctx->node_blob, ctx->ckpt_blob, ctx->mut_bytes, hipMemcpyDeviceToDevice, ctx->stream));
  if (ctx->quota_blob) {
    const size_t tb = (size_t)(ctx->q.q > 0 ? ctx->q.q : 1) * KS_QUOTA_DIMS * 8;
    HIPCHK(ctx, hipMemcpyAsync(ctx->q.used, ctx->quota_used_ckpt, tb, hipMemcpyDeviceToDevice, ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(ctx->q.npused, ctx->quota_npused_ckpt, tb, hipMemcpyDeviceToDevice, ctx->stream));
  }
  if (ctx->dev_blob)
    HIPCHK(ctx, hipMemcpyAsync(ctx->dv.used, ctx->dev_used_ckpt, (size_t)kDevQW * ctx->dv.npad * 8, hipMemcpyDeviceToDevice, ctx->stream));
  if (ctx->cpu_loaded)
    HIPCHK(ctx, hipMemcpyAsync(ctx->cpu.allocated, ctx->cpu_ckpt, (size_t)3 * ctx->cpu.npad * sizeof(CpuSet), hipMemcpyDeviceToDevice, ctx->stream));
  if (ctx->numa_blob)
    HIPCHK(ctx, hipMemcpyAsync(ctx->nv.used, ctx->numa_ckpt, numa_mut_bytes((size_t)ctx->npad), hipMemcpyDeviceToDevice, ctx->stream));
  if (ctx->rsv_blob) {
    HIPCHK(ctx, hipMemcpyAsync(ctx->rv.allocd, ctx->rsv_allocd_ckpt, (size_t)kRsvDims * ctx->rv.nr * 8, hipMemcpyDeviceToDevice, ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(ctx->rv.dald, ctx->rsv_dald_ckpt, (size_t)kDevQW * ctx->rv.nr * 8, hipMemcpyDeviceToDevice, ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(ctx->rv.assigned, ctx->rsv_assigned_ckpt, (size_t)ctx->rv.nr * 4, hipMemcpyDeviceToDevice, ctx->stream));
  }
  ctx->h_dev_assumed = ctx->h_dev_assumed_ckpt;
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  return KS_OK;
}

// ---- informer deltas (f1): rows of the device, CPU-state, quota and reservation-usage tables replaced in place
// (the node rows have ks_update_nodes); a delta re-bases nothing else, so ks_checkpoint after a batch of them ----

// dst[idx[i] * rs + w * cs] = src[w * m + i] for the m rows and W words (elem = 4 or 8 bytes)
template <typename T>
__global__ void scatter_words_kernel(T* dst, int64_t rs, int64_t cs, int32_t W, const int32_t* idx, const T* src, int64_t m) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= m * W) return;
  const int64_t w = t / m, i = t - w * m;
  dst[(int64_t)idx[i] * rs + w * cs] = src[t];
}

static int scatter_words(ks_ctx* ctx, void* dst, size_t elem, int64_t rs, int64_t cs, int32_t W,
                         const std::vector<int32_t>& idx, const void* src) {
  const int64_t m = (int64_t)idx.size();
  if (m == 0 || W == 0) return KS_OK;
  const size_t need = align16((size_t)m * 4) + (size_t)m * W * elem;
  if (ctx->dscratch_bytes < need) {
    dev_free(ctx->dscratch);
    ctx->dscratch_bytes = 0;
    if (dev_alloc(ctx, &ctx->dscratch, need) != KS_OK) return KS_ENOMEM;
    ctx->dscratch_bytes = need;
  }
  char* b = (char*)ctx->dscratch;
  HIPCHK(ctx, hipMemcpyAsync(b, idx.data(), (size_t)m * 4, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(ctx, hipMemcpyAsync(b + align16((size_t)m * 4), src, (size_t)m * W * elem, hipMemcpyHostToDevice, ctx->stream));
  const unsigned blocks = (unsigned)((m * W + 255) / 256);
  if (elem == 8)
    hipLaunchKernelGGL(scatter_words_kernel<int64_t>, dim3(blocks), dim3(256), 0, ctx->stream, (int64_t*)dst, rs, cs, W,
                       (const int32_t*)b, (const int64_t*)(b + align16((size_t)m * 4)), m);
  else
    hipLaunchKernelGGL(scatter_words_kernel<int32_t>, dim3(blocks), dim3(256), 0, ctx->stream, (int32_t*)dst, rs, cs, W,
                       (const int32_t*)b, (const int32_t*)(b + align16((size_t)m * 4)), m);
  HIPCHK(ctx, hipGetLastError());
  // the scratch is reused by the next call: let this one finish reading it
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  return KS_OK;
}

static int check_idx(ks_ctx* ctx, const int32_t* idx, int64_t m, int64_t lim, const char* what, std::vector<int32_t>& out) {
  out.assign(idx, idx + m);
  std::vector<int32_t> sorted(out);
  std::sort(sorted.begin(), sorted.end());
  for (int64_t i = 0; i < m; ++i) {
    if (sorted[i] < 0 || sorted[i] >= lim) KS_FAIL(ctx, KS_EINVAL, "%s: index %d out of range", what, sorted[i]);
    if (i && sorted[i] == sorted[i - 1]) KS_FAIL(ctx, KS_EINVAL, "%s: index %d repeated", what, sorted[i]);
  }
  return KS_OK;
}

// deviceshare nodeDeviceCache.updateNodeDevice (device_cache.go:489-527): the device rows of m nodes
int ks_update_devices(ks_ctx* ctx, const int32_t* idx, const ks_device_cols* rows, int64_t m) {
  if (!ctx || !rows || m < 0 || (m > 0 && !idx)) return ctx ? (ctx->err = "ks_update_devices: bad args", KS_EINVAL) : KS_EINVAL;
  if (!ctx->dev_blob || !ctx->cfg.deviceshare.enable) KS_FAIL(ctx, KS_ESTATE, "ks_update_devices without a device table");
  std::vector<int32_t> ix;
  if (int rc = check_idx(ctx, idx, m, ctx->n, "ks_update_devices", ix); rc != KS_OK) return rc;
  for (int32_t i : ix)
    if ((size_t)i < ctx->h_dev_assumed.size() && ctx->h_dev_assumed[(size_t)i] > 0)
      KS_FAIL(ctx, KS_ESTATE, "ks_update_devices: node %d holds %d assumed device pod(s); ks_unreserve them first (their "
              "Unreserve subtracts the request derived from the current device totals)", i, ctx->h_dev_assumed[(size_t)i]);
  HIPCHK(ctx, hipSetDevice(ctx->device));
  std::vector<uint32_t> flags((size_t)m, 0);
  std::vector<int64_t> total((size_t)kDevTW * m, 0), used((size_t)kDevQW * m, 0);
  std::vector<uint16_t> ids((size_t)m, 0);
  if (int rc = dev_encode(ctx, rows, m, (size_t)m, flags.data(), total.data(), used.data(), ids.data()); rc != KS_OK) return rc;
  const int64_t np = ctx->npad;
  if (scatter_words(ctx, (void*)ctx->dv.flags, 4, 1, np, 1, ix, flags.data()) != KS_OK ||
      scatter_words(ctx, (void*)ctx->dv.total, 8, 1, np, kDevTW, ix, total.data()) != KS_OK ||
      scatter_words(ctx, (void*)ctx->dv.used, 8, 1, np, kDevQW, ix, used.data()) != KS_OK)
    return KS_EHIP;
  for (int64_t i = 0; i < m; ++i) ctx->h_dev_ids[(size_t)ix[i]] = ids[(size_t)i];
  ctx->dev_loaded = true;
  if (dev_apply_held(ctx) != KS_OK) return KS_EHIP;
  return check_dev_numa(ctx);
}

// nodenumaresource NodeResourceTopology / pod events (topology_eventhandler.go, resource_manager.go Update /
// Release): the CPU state of m nodes, against the loaded topology table
int ks_update_cpu_state(ks_ctx* ctx, const int32_t* idx, const ks_cpu_state_cols* rows, int64_t m) {
  if (!ctx || !rows || m < 0 || (m > 0 && (!idx || !rows->topology || !rows->allocated)))
    return ctx ? (ctx->err = "ks_update_cpu_state: bad args", KS_EINVAL) : KS_EINVAL;
  if (!ctx->cpu_loaded) KS_FAIL(ctx, KS_ESTATE, "ks_update_cpu_state before ks_load_cpu_state");
  std::vector<int32_t> ix;
  if (int rc = check_idx(ctx, idx, m, ctx->n, "ks_update_cpu_state", ix); rc != KS_OK) return rc;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  const int32_t ntopo = (int32_t)ctx->cpu_cpc.size();
  std::vector<int32_t> tid((size_t)m), freec((size_t)m), ncpu((size_t)m);
  std::vector<CpuSet> sets((size_t)4 * m);
  for (int64_t i = 0; i < m; ++i) {
    if (int rc = cpu_encode_row(ctx, rows, i, ix[(size_t)i], ntopo, ctx->h_topos, tid[(size_t)i], sets[(size_t)i],
                                sets[(size_t)m + i], sets[(size_t)2 * m + i], sets[(size_t)3 * m + i], freec[(size_t)i],
                                ncpu[(size_t)i]);
        rc != KS_OK)
      return rc;
    const int32_t k = (size_t)ix[(size_t)i] < ctx->h_numa_k.size() ? ctx->h_numa_k[(size_t)ix[(size_t)i]] : 0;
    const int32_t nn = tid[(size_t)i] >= 0 ? (ctx->h_topo_dense[(size_t)tid[(size_t)i]] ? ctx->h_topos[(size_t)tid[(size_t)i]].nnodes : -1) : 0;
    if (k > 0 && nn != 0 && (nn < 0 || nn > k))
      KS_FAIL(ctx, KS_EUNSUPPORTED, "node %d: NUMA-policy node whose CPU topology NUMA ids are not 0..m-1 with m <= %d", ix[(size_t)i], k);
    ctx->h_cpu_nn[(size_t)ix[(size_t)i]] = (int8_t)nn;
  }
  // CpuSet rows: 4 tables of [npad] CpuSet, kCpuW u64 words each, row-major
  std::vector<int64_t> words((size_t)kCpuW * m);
  CpuSet* tables[4] = {ctx->cpu.allocated, ctx->cpu.excl_pcpu, ctx->cpu.excl_numa, const_cast<CpuSet*>(ctx->cpu.reserved)};
  for (int q = 0; q < 4; ++q) {
    for (int64_t i = 0; i < m; ++i)
      for (int w = 0; w < kCpuW; ++w) words[(size_t)w * m + i] = (int64_t)sets[(size_t)q * m + i].w[w];
    if (scatter_words(ctx, tables[q], 8, kCpuW, 1, kCpuW, ix, words.data()) != KS_OK) return KS_EHIP;
  }
  if (scatter_words(ctx, (void*)ctx->cpu.topo_id, 4, 1, 0, 1, ix, tid.data()) != KS_OK ||
      scatter_words(ctx, ctx->d.cpu_free, 4, 1, 0, 1, ix, freec.data()) != KS_OK ||
      scatter_words(ctx, ctx->d.numa_cpus, 4, 1, 0, 1, ix, ncpu.data()) != KS_OK)
    return KS_EHIP;
  if (upload_prep_nodes(ctx) != KS_OK || numa_refresh_free(ctx) != KS_OK || cores_refresh(ctx) != KS_OK)
    return KS_EHIP;  // cpuset millicores, offsets, per-NUMA free CPUs, core counts
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  return KS_OK;
}

// elasticquota GroupQuotaManager.OnQuotaUpdate / OnPodAdd-Update-Delete (group_quota_manager.go:736-870): the
// limit / min / used / non-preemptible used / masks of m quotas (the tree, i.e. the parents, is fixed: a parent
// change is a ks_load_quotas)
int ks_update_quotas(ks_ctx* ctx, const int32_t* idx, const ks_quota_cols* rows, int32_t m) {
  if (!ctx || !rows || m < 0 || (m > 0 && !idx)) return ctx ? (ctx->err = "ks_update_quotas: bad args", KS_EINVAL) : KS_EINVAL;
  if (!ctx->quota_blob) KS_FAIL(ctx, KS_ESTATE, "ks_update_quotas before ks_load_quotas");
  std::vector<int32_t> ix;
  if (int rc = check_idx(ctx, idx, m, ctx->q.q, "ks_update_quotas", ix); rc != KS_OK) return rc;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  std::vector<int32_t> lm((size_t)m), mm((size_t)m);
  std::vector<int64_t> t[4];
  for (auto& v : t) v.assign((size_t)KS_QUOTA_DIMS * m, 0);
  const int64_t* const* src[4] = {rows->limit, rows->used, rows->min, rows->nonpreemptible_used};
  for (int32_t i = 0; i < m; ++i) {
    lm[(size_t)i] = (int32_t)(rows->limit_mask ? rows->limit_mask[i] : 0);
    mm[(size_t)i] = (int32_t)(rows->min_mask ? rows->min_mask[i] : 0);
    for (int q = 0; q < 4; ++q)
      for (int d = 0; d < KS_QUOTA_DIMS; ++d) t[q][(size_t)d * m + i] = src[q][d] ? src[q][d][i] : 0;
  }
  int64_t* dst[4] = {ctx->q.limit, ctx->q.used, ctx->q.min, ctx->q.npused};
  if (scatter_words(ctx, ctx->q.limit_mask, 4, 1, 0, 1, ix, lm.data()) != KS_OK ||
      scatter_words(ctx, ctx->q.min_mask, 4, 1, 0, 1, ix, mm.data()) != KS_OK)
    return KS_EHIP;
  for (int q = 0; q < 4; ++q)
    if (scatter_words(ctx, dst[q], 8, KS_QUOTA_DIMS, 1, KS_QUOTA_DIMS, ix, t[q].data()) != KS_OK) return KS_EHIP;
  return KS_OK;
}

// reservation cache updates of reservations already loaded (reservation/cache.go:104-216 updateReservation:
// Allocated and the assigned pods change as pods bind / terminate): allocated [kRsvDims][m] and assigned [m] of
// m caller rows; the nodes' reservation base restore follows.  A reservation added or removed is a
// ks_load_reservations.
int ks_update_reservation_usage(ks_ctx* ctx, const int32_t* rows, const int64_t* const* allocated, const int32_t* assigned,
                                int32_t m) {
  if (!ctx || m < 0 || (m > 0 && (!rows || !allocated || !assigned)))
    return ctx ? (ctx->err = "ks_update_reservation_usage: bad args", KS_EINVAL) : KS_EINVAL;
  if (!ctx->rsv_blob) KS_FAIL(ctx, KS_ESTATE, "ks_update_reservation_usage before ks_load_reservations");
  std::vector<int32_t> ix;
  if (int rc = check_idx(ctx, rows, m, (int64_t)ctx->h_rsv_gi.size(), "ks_update_reservation_usage", ix); rc != KS_OK) return rc;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  std::vector<int32_t> gi((size_t)m), nodes;
  for (int32_t i = 0; i < m; ++i) {
    gi[(size_t)i] = ctx->h_rsv_gi[(size_t)ix[(size_t)i]];
    if (gi[(size_t)i] < 0) KS_FAIL(ctx, KS_EINVAL, "ks_update_reservation_usage: row %d was deleted", ix[(size_t)i]);
    nodes.push_back(ctx->h_rsv_node[(size_t)gi[(size_t)i]]);
    for (int d = 0; d < kRsvDims; ++d)
      if (allocated[d] && (allocated[d][i] < 0 || allocated[d][i] >= ((int64_t)1 << 56)))
        KS_FAIL(ctx, KS_EINVAL, "reservation row %d: allocated out of range", ix[(size_t)i]);
    if (assigned[i] < 0) KS_FAIL(ctx, KS_EINVAL, "reservation row %d: assigned < 0", ix[(size_t)i]);
  }
  std::sort(nodes.begin(), nodes.end());
  nodes.erase(std::unique(nodes.begin(), nodes.end()), nodes.end());
  std::vector<int64_t> al((size_t)kRsvDims * m, 0);
  for (int d = 0; d < kRsvDims; ++d)
    for (int32_t i = 0; i < m; ++i) al[(size_t)d * m + i] = allocated[d] ? allocated[d][i] : 0;
  // the affected nodes' base restore out, the usage in, the restore (and the nodes' owner classes) back
  int32_t* dn = nullptr;
  {
    void* p = nullptr;
    if (dev_alloc(ctx, &p, nodes.size() * 4 + 16) != KS_OK) return KS_ENOMEM;
    dn = (int32_t*)p;
  }
  auto done = [&](int rc) {
    void* p = dn;
    (void)hipStreamSynchronize(ctx->stream);
    dev_free(p);
    return rc;
  };
  HIPCHK(ctx, hipMemcpyAsync(dn, nodes.data(), nodes.size() * 4, hipMemcpyHostToDevice, ctx->stream));
  if (ctx->rsv_based && rsv_launch_base(ctx, dn, (int64_t)nodes.size(), -1, 0) != KS_OK) return done(KS_EHIP);
  if (scatter_words(ctx, ctx->rv.allocd, 8, 1, ctx->rv.nr, kRsvDims, gi, al.data()) != KS_OK ||
      scatter_words(ctx, ctx->rv.assigned, 4, 1, 0, 1, gi, assigned) != KS_OK)
    return done(KS_EHIP);
  if (ctx->rsv_based && rsv_launch_base(ctx, dn, (int64_t)nodes.size(), +1, 1) != KS_OK) return done(KS_EHIP);
  return done(KS_OK);
}

int ks_eval_pod(ks_ctx* ctx, const ks_pod_cols* pod, uint32_t* reasons, int64_t* scores, int64_t* total) {
  if (!ctx || !pod) return ctx ? (ctx->err = "ks_eval_pod: bad args", KS_EINVAL) : KS_EINVAL;
  if (!ctx->node_blob) KS_FAIL(ctx, KS_ESTATE, "ks_eval_pod before ks_load_nodes");
  if (int rc = validate_pods(ctx, pod, 1); rc != KS_OK) return rc;
  bind_mode(ctx, ctx->val_bind_required);
  HIPCHK(ctx, hipSetDevice(ctx->device));
  if (ensure_stage(ctx, ctx->est, 1) != KS_OK) return KS_ENOMEM;
  if (stage_cols(ctx, ctx->est, pod, 1) != KS_OK || prep_stage(ctx, ctx->est, 1) != KS_OK) return KS_EHIP;
  const int64_t n = ctx->n;
  EvBuf eb;
  if (ev_buffers(ctx, eb) != KS_OK) return KS_ENOMEM;
  uint32_t* dr = eb.dr;
  int64_t* ds = eb.ds;
  int64_t* dt = eb.dt;
  int32_t *draw = eb.draw, *dhi = eb.dhi, *ddraw = eb.ddraw, *dtraw = eb.dtraw, *daraw = eb.daraw;
  const int threads = 256;
  const int blocks = (int)((n + threads - 1) / threads);
  if (blocks > 0 && ctx->cfg.topology.enable && ctx->est.topo) {
    // PodTopologySpread / InterPodAffinity: their PreFilter sums, every Filter (theirs folded into the evaluation
    // kernel), then every normalization over the nodes all Filters leave (the topology step's kernels)
    const TopoKArgs ta = topo_args(ctx, ctx->est, nullptr, eb);
    HIPCHK(ctx, launch_topo_sums(ctx->stream, ta));
    HIPCHK(ctx, launch_eval_debug(ctx->nsc, blocks, ctx->stream, ctx->d, ctx->drv, ctx->ddv, ctx->dnv, ctx->kc,
                                  ctx->est.recs, n, dr, ds, dt, draw, dhi, ddraw, ctx->est.stat, dtraw, daraw, &ta,
                                  kernel_feat(ctx)));
    HIPCHK(ctx, launch_topo_pts(ctx->stream, ta));
    HIPCHK(ctx, launch_topo_norm(ctx->stream, ta));
  } else if (blocks > 0) {
    HIPCHK(ctx, launch_eval_debug(ctx->nsc, blocks, ctx->stream, ctx->d, ctx->drv, ctx->ddv, ctx->dnv, ctx->kc,
                                  ctx->est.recs, n, dr, ds, dt, draw, dhi, ddraw, ctx->est.stat, dtraw, daraw, nullptr,
                                  kernel_feat(ctx)));
    if (ctx->kc.dev)
      hipLaunchKernelGGL(dev_normalize_debug_kernel, dim3(1), dim3(1024), 0, ctx->stream, n, dr, ddraw, ds, dt,
                         ctx->cfg.deviceshare.plugin_weight);
    if (ctx->kc.taint & 2)
      hipLaunchKernelGGL(stat_normalize_debug_kernel, dim3(1), dim3(1024), 0, ctx->stream, n, dr, dtraw, ds, dt,
                         ctx->cfg.taint.plugin_weight, KS_SCORE_TAINT, 1);
    if (ctx->kc.aff & 2)
      hipLaunchKernelGGL(stat_normalize_debug_kernel, dim3(1), dim3(1024), 0, ctx->stream, n, dr, daraw, ds, dt,
                         ctx->cfg.affinity.plugin_weight, KS_SCORE_NODE_AFFINITY, 0);
    if (ctx->kc.rsv)
      hipLaunchKernelGGL(rsv_normalize_debug_kernel, dim3(1), dim3(1024), 0, ctx->stream, n, dr, draw, dhi, ds, dt,
                         ctx->cfg.reservation.plugin_weight);
  }
  HIPCHK(ctx, hipGetLastError());
  if (reasons && n) HIPCHK(ctx, hipMemcpyAsync(reasons, dr, (size_t)n * 4, hipMemcpyDeviceToHost, ctx->stream));
  if (scores && n) HIPCHK(ctx, hipMemcpyAsync(scores, ds, (size_t)n * 8 * KS_NUM_SCORE_PLUGINS, hipMemcpyDeviceToHost, ctx->stream));
  if (total && n) HIPCHK(ctx, hipMemcpyAsync(total, dt, (size_t)n * 8, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  return KS_OK;
}

int ks_eval_pod_debug(ks_ctx* ctx, const ks_pod_cols* pod, uint32_t* reasons, int64_t* scores, int64_t* total) {
  return ks_eval_pod(ctx, pod, reasons, scores, total);
}

// Unreserve of every plugin + the scheduler cache's ForgetPod for one pod (ks_unreserve; one thread, a few dozen
// read-modify-writes on the node's, the quota chain's, the reservation's and the devices' rows).
struct UnreserveArgs {
  DevNodes d;
  DevRsv rv;
  DevDev dv;
  DevNuma nv;
  DevCpu cpu;
  DevQuotas q;
  DevPodQuota pq;
  const PodRec* pod;
  const PodStat* pstat;    // NodePorts: the pod's host ports (Cfg.ports)
  Cfg c;
  int32_t node, gi;        // node; the reservation's CSR position (-1 = none)
  uint32_t gmin, rmin;     // DeviceShare minors of the allocation
  const uint64_t* cpuset;  // [KS_CPU_WORDS] the pod's CPUs
  const int64_t* nalloc;   // [2][kNumaDev] its NUMA-node allocation (cpu milli, memory)
  int32_t quota, dev, cpu_loaded, numa_pol, ratio_amp;
  const TopoRec* topo;     // PodTopologySpread / InterPodAffinity: the pod's properties leave the node's counters
  const int32_t* topo_props;
  int32_t* topo_count;
  int64_t topo_npad;
};

__global__ void unreserve_kernel(UnreserveArgs a) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const PodRec p = a.pod[0];
  const int64_t n = a.node;
  DevNodes& d = a.d;
  // ElasticQuota UnreservePod (group_quota_manager.go updatePodUsedNoLock with the pod removed)
  if (a.quota && p.quota >= 0) {
    const uint32_t mask = a.pq.mask[0];
    for (int32_t cur = p.quota; cur >= 0; cur = a.q.parent[cur])
      for (int dd = 0; dd < KS_QUOTA_DIMS; ++dd) {
        if (!((mask >> dd) & 1u)) continue;
        a.q.used[(size_t)cur * KS_QUOTA_DIMS + dd] -= a.pq.req[dd][0];
        if (p.flags & KS_POD_NONPREEMPTIBLE) a.q.npused[(size_t)cur * KS_QUOTA_DIMS + dd] -= a.pq.req[dd][0];
      }
  }
  // ForgetPod (NodeInfo.RemovePod) + podAssignCache.unAssign (load_aware.go:265)
  d.req_cpu[n] -= p.cpu;
  d.req_mem[n] -= p.mem;
  d.req_eph[n] -= p.eph;
  for (int k = 0; k < KS_MAX_SCALARS; ++k) d.req_sc[k][n] -= p.sc[k];
  d.nz_cpu[n] -= p.nzcpu;
  d.nz_mem[n] -= p.nzmem;
  d.pod_count[n] -= 1;
  d.la_term_cpu[n] -= p.est_cpu;
  d.la_term_mem[n] -= p.est_mem;
  if (p.flags & KS_POD_PROD) {
    d.la_pterm_cpu[n] -= p.est_cpu;
    d.la_pterm_mem[n] -= p.est_mem;
  }
  // NodeInfo.RemovePod: the pod's host ports (a used entry conflicts with itself, so no other pod holds it)
  if (a.c.ports & 1) d.host_ports[n] &= ~a.pstat[0].pwant;
  if (a.topo) topo_count_pod(a.topo_count, a.topo_npad, a.topo_props, a.topo[0], n, -1);
  // reservationCache.forgetPod: Allocated -= Mask(requests, ResourceNames); the pod leaves the assigned set
  if (a.gi >= 0) {
    const uint32_t keys = rsv_keys(a.rv.meta[a.gi]);
    for (int dd = 0; dd < kRsvDims; ++dd)
      if ((keys >> dd) & 1u) a.rv.allocd[(int64_t)dd * a.rv.nr + a.gi] -= pod_dim(p, dd);
    a.rv.assigned[a.gi] -= 1;
  }
  // DeviceShare: nodeDevice.updateCacheUsed(allocation, pod, false)
  if (a.dev && (a.gmin | a.rmin)) {
    GpuReq g;
    if (dev_prepare(p, DevGView{a.dv, n}, g) == 0) {
      for (int k = 0; k < kGpus; ++k) {
        if (!((a.gmin >> k) & 1u)) continue;
        a.dv.used[(int64_t)(0 * kGpus + k) * a.dv.npad + n] -= g.core;
        a.dv.used[(int64_t)(1 * kGpus + k) * a.dv.npad + n] -= g.mem;
        a.dv.used[(int64_t)(2 * kGpus + k) * a.dv.npad + n] -= g.ratio;
      }
      for (int j = 0; j < kRdma; ++j)
        if ((a.rmin >> j) & 1u) a.dv.used[(int64_t)(kDevRdmaW + j) * a.dv.npad + n] -= g.rdma;
      // the pod leaves its reservation's AssignedPods: its allocation on the reservation's minors too
      if (a.gi >= 0 && (a.rv.meta[a.gi] & kRsvMetaDev)) {
        const RsvG<true> gv(a.rv, n);
        rsv_dev_assign(a.rv, gv, a.gi - gv.b, g, a.gmin, a.rmin, -1);
      }
    }
  }
  // NodeAllocation.release (node_allocation.go:105-131): the CPUs (reference count 1 -> removed) and the
  // NUMA-node resources (SubtractWithNonNegativeResult; the entries stay)
  if (a.cpu_loaded && a.cpuset) {
    CpuSet cs;
    int32_t cnt = 0;
    for (int w = 0; w < kCpuW; ++w) cs.w[w] = a.cpuset[w] & a.cpu.allocated[n].w[w];
    for (int w = 0; w < kCpuW; ++w) cnt += __builtin_popcountll(cs.w[w]);
    if (cnt) {
      a.cpu.allocated[n] = cs_andnot(a.cpu.allocated[n], cs);
      a.cpu.excl_pcpu[n] = cs_andnot(a.cpu.excl_pcpu[n], cs);
      a.cpu.excl_numa[n] = cs_andnot(a.cpu.excl_numa[n], cs);
      const int32_t cpus = d.numa_cpus[n] - cnt;
      d.numa_cpus[n] = cpus;
      const int64_t A = (int64_t)cpus * 1000;
      const double ratio = d.numa_ratio[n];
      d.numa_amilli[n] = A;
      d.numa_off[n] = (a.ratio_amp && ratio > 1.0) ? (int64_t)::ceil((double)A * ratio) - A : 0;
      if (d.cpu_free[n] >= 0) d.cpu_free[n] += cnt;
      const int32_t tid = a.cpu.topo_id[n];
      if (tid >= 0) {
        const CpuTopo& tp = a.cpu.topo[tid];
        d.cpu_cores[n] = cores_word(tp, cs_andnot(cs_andnot(tp.all, a.cpu.allocated[n]), a.cpu.reserved[n]),
                                    (d.numa_flags[n] >> KS_NUMA_CPU_BIND_SHIFT) & 3u);
      }
      if (a.numa_pol && tid >= 0 && a.nv.count[n] > 0) {
        const CpuTopo& t = a.cpu.topo[tid];
        for (int k = 0; k < kNumaDev && k < a.nv.count[n]; ++k) {
          const int32_t ck = cs_count(cs_and(cs, t.node_mask[k]));
          if (!ck) continue;
          const int64_t o = (int64_t)k * a.nv.npad + n;
          const int32_t c1 = a.nv.cs[o] - ck;
          a.nv.cs[o] = c1;
          a.nv.free[o] = numa_free_word(t, cs_andnot(cs_andnot(t.all, a.cpu.allocated[n]), a.cpu.reserved[n]), k);
          const int64_t m = (int64_t)c1 * 1000;
          a.nv.off[o] = ratio > 1.0 ? (int64_t)::ceil((double)m * ratio) - m : 0;
        }
      }
    }
  }
  if (a.numa_pol && a.nalloc && a.nv.count[n] > 0) {
    for (int k = 0; k < kNumaDev && k < a.nv.count[n]; ++k)
      for (int r = 0; r < 2; ++r) {
        const int64_t o = ((int64_t)r * kNumaDev + k) * a.nv.npad + n;
        const int64_t v = a.nv.used[o] - a.nalloc[r * kNumaDev + k];
        a.nv.used[o] = v < 0 ? 0 : v;
      }
  }
}

// ---- per-pod framework mode: the framework runs Filter/Score through ks_eval_pod, picks the node, and
// reports its Reserve / Unreserve here ----

int ks_assume(ks_ctx* ctx, const ks_pod_cols* pod, int32_t node, ks_result* out, uint64_t* cpuset, int64_t* numa_alloc) {
  if (!ctx || !pod || !out) return ctx ? (ctx->err = "ks_assume: bad args", KS_EINVAL) : KS_EINVAL;
  if (!ctx->node_blob) KS_FAIL(ctx, KS_ESTATE, "ks_assume before ks_load_nodes");
  if (node < 0 || node >= ctx->n) KS_FAIL(ctx, KS_EINVAL, "ks_assume: node %d out of range", node);
  if (ctx->cfg.quota.enable && pod->quota && !ctx->quota_blob) KS_FAIL(ctx, KS_ESTATE, "ks_assume: quotas not loaded");
  if (int rc = validate_pods(ctx, pod, 1); rc != KS_OK) return rc;
  bind_mode(ctx, ctx->val_bind_required);
  HIPCHK(ctx, hipSetDevice(ctx->device));
  if (int rc = commit_attr_set(ctx); rc != KS_OK) return rc;
  if (ensure_stage(ctx, ctx->ast, 1) != KS_OK || ensure_cpuset_bufs(ctx, 1) != KS_OK) return KS_ENOMEM;
  if (stage_cols(ctx, ctx->ast, pod, 1) != KS_OK || prep_stage(ctx, ctx->ast, 1) != KS_OK) return KS_EHIP;
  // one pass of one pod whose only candidate is `node` (an untouched node's snapshot key is taken as is): the
  // commit kernel's Reserve path of every plugin runs on it; force skips the quota admission
  struct {
    uint32_t chunk;
    uint2 t;
    int32_t count;
    uint64_t bound, top;
  } h{(uint32_t)(node >> 6), make_uint2((1u << 6) | (uint32_t)(63 - (node & 63)), 0u), 1, 0ull, 0ull};
  HIPCHK(ctx, hipMemcpyAsync(ctx->cand_chunk, &h.chunk, 4, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(ctx, hipMemcpyAsync(ctx->cand_t, &h.t, 8, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(ctx, hipMemcpyAsync(ctx->cand_count, &h.count, 4, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(ctx, hipMemcpyAsync(ctx->cand_bound, &h.bound, 8, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(ctx, hipMemcpyAsync(ctx->cand_top, &h.top, 8, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(ctx, hipMemcpyAsync(ctx->cand_second, &h.top, 8, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(ctx, hipMemsetAsync(ctx->cursor, 0, 4, ctx->stream));
  HIPCHK(ctx, hipMemsetAsync(ctx->dev_M, 0, kNormRows * kMaxBatch * 8, ctx->stream));
  if (ctx->cpuset_list) {
    HIPCHK(ctx, hipMemsetAsync(ctx->cpuset_n, 0, 4, ctx->stream));
    HIPCHK(ctx, hipMemsetAsync(ctx->cpuset_out, 0, sizeof(CpuSet), ctx->stream));
    HIPCHK(ctx, hipMemsetAsync(ctx->numa_alloc, 0, 2 * kNumaDev * 8, ctx->stream));
  }
  bool qcache = false;
  size_t smem = 0;
  CommitArgs ca = commit_args(ctx, ctx->ast, 1, 1, &qcache, &smem);
  ca.force = 1;
  if (ca.topo) ca.topo = 3;  // count the pod's properties on the node
  HIPCHK(ctx, pass_launcher(kernel_feat(ctx), ctx->nsc).commit(qcache, smem, ctx->stream, ca));
  if (ctx->cpu_loaded && ctx->n > 0) {
    hipLaunchKernelGGL(cpuset_kernel, dim3((unsigned)((ctx->n + 255) / 256)), dim3(256), 0, ctx->stream, ctx->cpu,
                       (const int2*)ctx->cpuset_list, (const int32_t*)ctx->cpuset_n, (const uint32_t*)ctx->cpuset_split,
                       (const PodRec*)ctx->ast.recs, ctx->cpuset_out, (const uint32_t*)ctx->d.numa_flags,
                       ctx->d.cpu_cores, (int32_t)(ctx->cfg.numa.numa_scoring_strategy == KS_MOST_ALLOCATED),
                       numa_words(ctx), ctx->nv.npad, ctx->n);
    HIPCHK(ctx, hipGetLastError());
  }
  HIPCHK(ctx, hipMemcpyAsync(out, ctx->ast.results, sizeof(ks_result), hipMemcpyDeviceToHost, ctx->stream));
  int64_t na[2 * kNumaDev] = {0};
  if (cpuset) {
    if (ctx->cpuset_list) HIPCHK(ctx, hipMemcpyAsync(cpuset, ctx->cpuset_out, sizeof(CpuSet), hipMemcpyDeviceToHost, ctx->stream));
    else memset(cpuset, 0, sizeof(CpuSet));
  }
  if (numa_alloc && ctx->cpuset_list)
    HIPCHK(ctx, hipMemcpyAsync(na, ctx->numa_alloc, sizeof(na), hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  if (numa_alloc) {
    memset(numa_alloc, 0, sizeof(int64_t) * KS_MAX_NUMA * 2);
    for (int k = 0; k < kNumaDev; ++k)
      for (int r = 0; r < 2; ++r) numa_alloc[k * 2 + r] = na[r * kNumaDev + k];
  }
  // the assume wrote pod 0's slots of the batch's cpuset and NUMA-allocation buffers: the last ks_schedule*'s
  // CPU sets are gone, so ks_fetch_cpusets / ks_fetch_numa_alloc refuse until the next schedule
  ctx->cpusets_clobbered = true;
  if (out->status == KS_S_SCHEDULED && (out->gpu_minors | out->rdma_minors)) {
    if (ctx->h_dev_assumed.size() < (size_t)ctx->n) ctx->h_dev_assumed.resize((size_t)ctx->n, 0);
    ++ctx->h_dev_assumed[(size_t)node];
  }
  if (out->node != node && out->status == KS_S_SCHEDULED)
    KS_FAIL(ctx, KS_EHIP, "ks_assume: placed on node %d instead of %d", out->node, node);
  return KS_OK;
}

int ks_unreserve(ks_ctx* ctx, const ks_pod_cols* pod, const ks_result* r, const uint64_t* cpuset, const int64_t* numa_alloc) {
  if (!ctx || !pod || !r) return ctx ? (ctx->err = "ks_unreserve: bad args", KS_EINVAL) : KS_EINVAL;
  if (!ctx->node_blob) KS_FAIL(ctx, KS_ESTATE, "ks_unreserve before ks_load_nodes");
  if (r->status != KS_S_SCHEDULED || r->node < 0 || r->node >= ctx->n)
    KS_FAIL(ctx, KS_EINVAL, "ks_unreserve: the result is not a placement (status %u, node %d)", r->status, r->node);
  if (int rc = validate_pods(ctx, pod, 1); rc != KS_OK) return rc;
  int32_t gi = -1;
  if (r->reservation >= 0) {
    if (!ctx->cfg.reservation.enable || (size_t)r->reservation >= ctx->h_rsv_gi.size())
      KS_FAIL(ctx, KS_EINVAL, "ks_unreserve: reservation row %d unknown", r->reservation);
    gi = ctx->h_rsv_gi[(size_t)r->reservation];
    if (gi < 0) KS_FAIL(ctx, KS_EINVAL, "ks_unreserve: reservation row %d was deleted", r->reservation);
  }
  HIPCHK(ctx, hipSetDevice(ctx->device));
  if (ensure_stage(ctx, ctx->ast, 1) != KS_OK) return KS_ENOMEM;
  if (!ctx->ures && dev_alloc(ctx, &ctx->ures, 16 + sizeof(CpuSet) + 2 * kNumaDev * 8) != KS_OK) return KS_ENOMEM;
  if (stage_cols(ctx, ctx->ast, pod, 1) != KS_OK || prep_stage(ctx, ctx->ast, 1) != KS_OK) return KS_EHIP;
  char* u = (char*)ctx->ures;
  int32_t* d_idx = (int32_t*)u;
  uint64_t* d_cs = (uint64_t*)(u + 16);
  int64_t* d_na = (int64_t*)(u + 16 + sizeof(CpuSet));
  const int32_t node = r->node;
  HIPCHK(ctx, hipMemcpyAsync(d_idx, &node, 4, hipMemcpyHostToDevice, ctx->stream));
  if (cpuset) HIPCHK(ctx, hipMemcpyAsync(d_cs, cpuset, sizeof(CpuSet), hipMemcpyHostToDevice, ctx->stream));
  int64_t na[2 * kNumaDev] = {0};
  if (numa_alloc)
    for (int k = 0; k < kNumaDev; ++k)
      for (int q = 0; q < 2; ++q) na[q * kNumaDev + k] = numa_alloc[k * 2 + q];
  HIPCHK(ctx, hipMemcpyAsync(d_na, na, sizeof(na), hipMemcpyHostToDevice, ctx->stream));
  // the node's reservation base restore follows the reservation's state: out before, back in after
  const bool rb = gi >= 0 && ctx->rsv_based;
  if (rb && rsv_launch_base(ctx, d_idx, 1, -1, 0) != KS_OK) return KS_EHIP;
  UnreserveArgs ua;
  ua.d = ctx->d;
  ua.rv = ctx->rv;
  ua.dv = ctx->dv;
  ua.nv = ctx->nv;
  ua.cpu = ctx->cpu;
  ua.q = ctx->q;
  ua.pq = ctx->ast.pq;
  ua.pod = ctx->ast.recs;
  ua.pstat = ctx->ast.stat;
  ua.c = ctx->kc;
  ua.node = node;
  ua.gi = gi;
  ua.gmin = r->gpu_minors;
  ua.rmin = r->rdma_minors;
  ua.cpuset = cpuset ? d_cs : nullptr;
  ua.nalloc = numa_alloc ? d_na : nullptr;
  ua.quota = ctx->kc.quota_enable && ctx->quota_blob;
  ua.dev = ctx->kc.dev && ctx->dev_loaded;
  ua.cpu_loaded = ctx->cpu_loaded;
  ua.numa_pol = ctx->kc.numa_pol && ctx->numa_blob;
  ua.ratio_amp = ctx->cfg.numa.enable;
  ua.topo = ctx->cfg.topology.enable ? ctx->ast.topo : nullptr;
  ua.topo_props = ctx->ast.topo_props;
  ua.topo_count = ctx->topo_count;
  ua.topo_npad = ctx->npad;
  hipLaunchKernelGGL(unreserve_kernel, dim3(1), dim3(64), 0, ctx->stream, ua);
  HIPCHK(ctx, hipGetLastError());
  if (rb && rsv_launch_base(ctx, d_idx, 1, +1, 1) != KS_OK) return KS_EHIP;
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  if ((r->gpu_minors | r->rdma_minors) && (size_t)node < ctx->h_dev_assumed.size() && ctx->h_dev_assumed[(size_t)node] > 0)
    --ctx->h_dev_assumed[(size_t)node];
  return KS_OK;
}

int ks_fetch_numa_alloc(ks_ctx* ctx, int64_t* out, int32_t p) {
  if (!ctx || (p > 0 && !out) || p < 0) return ctx ? (ctx->err = "ks_fetch_numa_alloc: bad args", KS_EINVAL) : KS_EINVAL;
  if (p > ctx->np) KS_FAIL(ctx, KS_EINVAL, "ks_fetch_numa_alloc: %d pods requested, %d scheduled", p, ctx->np);
  if (p > 0 && ctx->cpusets_clobbered) KS_FAIL(ctx, KS_ESTATE, "ks_fetch_numa_alloc: a ks_assume since the last schedule overwrote it");
  if (p == 0) return KS_OK;
  memset(out, 0, (size_t)p * KS_MAX_NUMA * 2 * 8);
  if (!ctx->numa_alloc || ctx->cpuset_cap < p) return KS_OK;
  std::vector<int64_t> h((size_t)p * 2 * kNumaDev);
  HIPCHK(ctx, hipMemcpyAsync(h.data(), ctx->numa_alloc, h.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  for (int32_t i = 0; i < p; ++i)
    for (int k = 0; k < kNumaDev; ++k)
      for (int q = 0; q < 2; ++q) out[((size_t)i * KS_MAX_NUMA + k) * 2 + q] = h[((size_t)i * 2 + q) * kNumaDev + k];
  return KS_OK;
}

int ks_read_nodes(ks_ctx* ctx, ks_node_state* o) {
  if (!ctx || !o) return ctx ? (ctx->err = "ks_read_nodes: bad args", KS_EINVAL) : KS_EINVAL;
  if (!ctx->node_blob) KS_FAIL(ctx, KS_ESTATE, "ks_read_nodes before ks_load_nodes");
  const size_t n = (size_t)ctx->n;
  auto cp = [&](void* h, const void* d, size_t w) -> hipError_t {
    if (!h || !n) return hipSuccess;
    return hipMemcpyAsync(h, d, n * w, hipMemcpyDeviceToHost, ctx->stream);
  };
  // the columns hold the reservation base restore: the reference's NodeInfo is computed into a scratch copy of
  // the restored columns (the live columns are never touched)
  DevNodes v = ctx->d;
  if (ctx->rsv_based && n) {
    const size_t bytes = n * 8 * (5 + KS_MAX_SCALARS);
    if (!ctx->rdscratch && dev_alloc(ctx, &ctx->rdscratch, (size_t)ctx->npad * 8 * (5 + KS_MAX_SCALARS)) != KS_OK)
      return KS_ENOMEM;
    (void)bytes;
    int64_t* sc = (int64_t*)ctx->rdscratch;
    int64_t** cols[5 + KS_MAX_SCALARS] = {&v.req_cpu, &v.req_mem, &v.req_eph, &v.nz_cpu, &v.nz_mem};
    for (int k = 0; k < KS_MAX_SCALARS; ++k) cols[5 + k] = &v.req_sc[k];
    for (int c = 0; c < 5 + KS_MAX_SCALARS; ++c) {
      int64_t* dst = sc + (size_t)c * ctx->npad;
      HIPCHK(ctx, hipMemcpyAsync(dst, *cols[c], n * 8, hipMemcpyDeviceToDevice, ctx->stream));
      *cols[c] = dst;
    }
    hipLaunchKernelGGL(rsv_base_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream, v, ctx->rv,
                       (const int32_t*)nullptr, (int64_t)n, (int64_t)-1, 0);
    HIPCHK(ctx, hipGetLastError());
  }
  HIPCHK(ctx, cp(o->req_milli_cpu, v.req_cpu, 8));
  HIPCHK(ctx, cp(o->req_memory, v.req_mem, 8));
  HIPCHK(ctx, cp(o->req_ephemeral, v.req_eph, 8));
  HIPCHK(ctx, cp(o->pod_count, v.pod_count, 4));
  HIPCHK(ctx, cp(o->nonzero_milli_cpu, v.nz_cpu, 8));
  HIPCHK(ctx, cp(o->nonzero_memory, v.nz_mem, 8));
  for (int k = 0; k < KS_MAX_SCALARS; ++k) HIPCHK(ctx, cp(o->req_scalar[k], v.req_sc[k], 8));
  HIPCHK(ctx, cp(o->la_term_milli_cpu, v.la_term_cpu, 8));
  HIPCHK(ctx, cp(o->la_term_memory, v.la_term_mem, 8));
  HIPCHK(ctx, cp(o->la_prod_term_milli_cpu, v.la_pterm_cpu, 8));
  HIPCHK(ctx, cp(o->la_prod_term_memory, v.la_pterm_mem, 8));
  HIPCHK(ctx, cp(o->host_ports, v.host_ports, 8));
  for (size_t q = 0; o->topo_count && q < ctx->topo_count_v.size(); ++q)
    HIPCHK(ctx, cp(o->topo_count + q * n, ctx->topo_count_v[q], 4));
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  return KS_OK;
}

int ks_read_quota_used(ks_ctx* ctx, int64_t* used) {
  if (!ctx || !used) return ctx ? (ctx->err = "ks_read_quota_used: bad args", KS_EINVAL) : KS_EINVAL;
  if (!ctx->quota_blob || ctx->q.q == 0) return KS_OK;
  HIPCHK(ctx, hipMemcpyAsync(used, ctx->q.used, (size_t)ctx->q.q * KS_QUOTA_DIMS * 8, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  return KS_OK;
}

// ---- preemption: the ElasticQuota PostFilter (ks_preempt.h) ----

int ks_load_node_pods(ks_ctx* ctx, const ks_node_pod_cols* pc, int64_t m, const int32_t* pdb_allowed, int32_t npdb) {
  if (!ctx || !pc || m < 0 || npdb < 0 || (m > 0 && !pc->node) || (npdb > 0 && !pdb_allowed))
    return ctx ? (ctx->err = "ks_load_node_pods: bad args", KS_EINVAL) : KS_EINVAL;
  if (!ctx->node_blob) KS_FAIL(ctx, KS_ESTATE, "ks_load_node_pods before ks_load_nodes");
  if (m >= ((int64_t)1 << 31)) KS_FAIL(ctx, KS_EINVAL, "ks_load_node_pods: too many pods");
  const int64_t n = ctx->n;
  std::vector<int64_t> beg((size_t)n + 1, 0);
  for (int64_t i = 0; i < m; ++i) {
    const int32_t nd = pc->node[i];
    if (nd < 0 || nd >= n) KS_FAIL(ctx, KS_EINVAL, "ks_load_node_pods: pod %lld on node %d outside [0, %lld)", (long long)i, nd, (long long)n);
    int32_t qs[kPreemptPdbs];
    for (int k = 0; k < kPreemptPdbs; ++k) {
      const int32_t* col = k == 0 ? pc->pdb : pc->pdb_more[k - 1];
      const int32_t q = qs[k] = col ? col[i] : -1;
      if (q < -1 || q >= npdb) KS_FAIL(ctx, KS_EINVAL, "ks_load_node_pods: pod %lld: PDB index %d outside [-1, %d)", (long long)i, q, npdb);
      for (int k2 = 0; k2 < k; ++k2)
        if (q >= 0 && qs[k2] == q) KS_FAIL(ctx, KS_EINVAL, "ks_load_node_pods: pod %lld lists PDB %d twice", (long long)i, q);
    }
    ++beg[(size_t)nd + 1];
  }
  int32_t maxc = 0;
  for (int64_t v = 0; v < n; ++v) {
    maxc = std::max<int32_t>(maxc, (int32_t)beg[(size_t)v + 1]);
    beg[(size_t)v + 1] += beg[(size_t)v];
  }
  if (maxc > kPreemptMaxPods)
    KS_FAIL(ctx, KS_EUNSUPPORTED, "ks_load_node_pods: a node holds %d pods (the dry run holds up to %d)", maxc, kPreemptMaxPods);
  for (int32_t i = 0; i < npdb; ++i)
    if (pdb_allowed[i] < -(1 << 30) || pdb_allowed[i] > (1 << 30)) KS_FAIL(ctx, KS_EINVAL, "ks_load_node_pods: DisruptionsAllowed out of range");
  const int64_t* reqc[kRsvDims] = {pc->req_milli_cpu, pc->req_memory, pc->req_ephemeral, pc->req_scalar[0],
                                   pc->req_scalar[1], pc->req_scalar[2], pc->req_scalar[3]};
  for (int dd = 0; dd < kRsvDims; ++dd)
    if (int rc = check_range64(ctx, reqc[dd], m, "node pod request"); rc != KS_OK) return rc;
  for (int dd = 0; dd < KS_QUOTA_DIMS; ++dd)
    if (int rc = check_range64(ctx, pc->quota_req[dd], m, "node pod quota request"); rc != KS_OK) return rc;
  // positions: per node, util.MoreImportantPod order (priority desc, start time asc), equal pairs in caller order
  std::vector<int32_t> order((size_t)m);
  for (int64_t i = 0; i < m; ++i) order[(size_t)i] = (int32_t)i;
  auto prio = [&](int32_t i) { return pc->priority ? pc->priority[i] : 0; };
  auto start = [&](int32_t i) { return pc->start_time ? pc->start_time[i] : (int64_t)0; };
  std::sort(order.begin(), order.end(), [&](int32_t x, int32_t y) {
    if (pc->node[x] != pc->node[y]) return pc->node[x] < pc->node[y];
    if (prio(x) != prio(y)) return prio(x) > prio(y);
    if (start(x) != start(y)) return start(x) < start(y);
    return x < y;
  });
  const size_t mm = (size_t)std::max<int64_t>(m, 1), nn = (size_t)n + 1;
  // one blob: beg, then the position columns, the PDB budgets and the per-call scratch
  size_t off = 0;
  auto take = [&](size_t bytes) { const size_t o = off; off = align16(off + bytes); return o; };
  const size_t o_beg = take(nn * 8), o_prio = take(mm * 4), o_start = take(mm * 8), o_flags = take(mm * 4),
               o_quota = take(mm * 4), o_pdb = take(mm * 4 * kPreemptPdbs), o_row = take(mm * 4), o_req = take(mm * 8 * kRsvDims),
               o_qreq = take(mm * 8 * KS_QUOTA_DIMS), o_pdba = take((size_t)std::max(npdb, 1) * 4),
               o_cand = take(nn * sizeof(PreemptCand)), o_vrank = take(mm * 4), o_status = take(nn),
               o_out = take(sizeof(PreemptOut)), o_vic = take((size_t)kPreemptMaxPods * 4);
  std::vector<unsigned char> h(off, 0);
  auto put = [&](size_t o, size_t i, const void* v, size_t w) { memcpy(h.data() + o + i * w, v, w); };
  memcpy(h.data() + o_beg, beg.data(), nn * 8);
  for (size_t pos = 0; pos < (size_t)m; ++pos) {
    const int32_t i = order[pos];
    const int32_t pr = prio(i);
    const int64_t st = start(i);
    const uint32_t fl = pc->flags ? pc->flags[i] : KS_NPOD_IN_QUOTA;
    const int32_t q = pc->quota ? pc->quota[i] : -1;
    put(o_prio, pos, &pr, 4);
    put(o_start, pos, &st, 8);
    put(o_flags, pos, &fl, 4);
    put(o_quota, pos, &q, 4);
    for (int k = 0; k < kPreemptPdbs; ++k) {  // [k][m]
      const int32_t* col = k == 0 ? pc->pdb : pc->pdb_more[k - 1];
      const int32_t pd = col ? col[i] : -1;
      put(o_pdb, (size_t)k * mm + pos, &pd, 4);
    }
    put(o_row, pos, &i, 4);
    for (int dd = 0; dd < kRsvDims; ++dd) {
      const int64_t v = reqc[dd] ? reqc[dd][i] : 0;
      put(o_req, (size_t)dd * mm + pos, &v, 8);
    }
    for (int dd = 0; dd < KS_QUOTA_DIMS; ++dd) {
      const int64_t v = pc->quota_req[dd] ? pc->quota_req[dd][i] : 0;
      put(o_qreq, (size_t)dd * mm + pos, &v, 8);
    }
  }
  if (npdb) memcpy(h.data() + o_pdba, pdb_allowed, (size_t)npdb * 4);
  HIPCHK(ctx, hipSetDevice(ctx->device));
  dev_free(ctx->npod_blob);
  if (dev_alloc(ctx, &ctx->npod_blob, off) != KS_OK) return KS_ENOMEM;
  HIPCHK(ctx, hipMemcpyAsync(ctx->npod_blob, h.data(), off, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  unsigned char* b = (unsigned char*)ctx->npod_blob;
  DevNodePods& t = ctx->npt;
  t.beg = (const int64_t*)(b + o_beg);
  t.prio = (const int32_t*)(b + o_prio);
  t.start = (const int64_t*)(b + o_start);
  t.flags = (const uint32_t*)(b + o_flags);
  t.quota = (const int32_t*)(b + o_quota);
  t.pdb = (const int32_t*)(b + o_pdb);
  t.row = (const int32_t*)(b + o_row);
  t.req = (const int64_t*)(b + o_req);
  t.qreq = (const int64_t*)(b + o_qreq);
  t.pdb_allowed = (const int32_t*)(b + o_pdba);
  t.m = (int64_t)mm;
  t.npdb = npdb;
  ctx->pre_cand = (PreemptCand*)(b + o_cand);
  ctx->pre_vrank = (int32_t*)(b + o_vrank);
  ctx->pre_status = (uint8_t*)(b + o_status);
  ctx->pre_out = (PreemptOut*)(b + o_out);
  ctx->pre_victims = (int32_t*)(b + o_vic);
  ctx->npod_slots = maxc <= 64 ? 1 : (maxc <= 128 ? 2 : 4);
  return KS_OK;
}

int ks_preempt(ks_ctx* ctx, const ks_pod_cols* pod, int32_t priority, uint32_t flags, int32_t nominated,
               const uint8_t* unresolvable, ks_preempt_result* out, int32_t* victims, int32_t victims_cap,
               uint8_t* node_status) {
  if (!ctx || !pod || !out || victims_cap < 0 || (victims_cap > 0 && !victims))
    return ctx ? (ctx->err = "ks_preempt: bad args", KS_EINVAL) : KS_EINVAL;
  if (!ctx->npod_blob) KS_FAIL(ctx, KS_ESTATE, "ks_preempt before ks_load_node_pods");
  if (!ctx->cfg.quota.enable || !ctx->quota_blob || ctx->q.q == 0)
    KS_FAIL(ctx, KS_EUNSUPPORTED, "ks_preempt: the ElasticQuota PostFilter needs ElasticQuota and a loaded quota table");
  if (ctx->kc.rsv || ctx->kc.numa || ctx->kc.dev || (ctx->kc.ports & 1))
    KS_FAIL(ctx, KS_EUNSUPPORTED, "ks_preempt: Reservation / NodeNUMAResource / DeviceShare / NodePorts filters read the "
                                  "node's other pods (their PreFilter extensions are not modelled)");
  const int32_t q = pod->quota ? pod->quota[0] : -1;
  if (q < 0 || q >= ctx->q.q)
    KS_FAIL(ctx, KS_EUNSUPPORTED, "ks_preempt: the pod has no quota row (the reference's cloned PostFilterState has no "
                                  "QuotaInfo then)");
  if (nominated < -1 || nominated >= ctx->n) KS_FAIL(ctx, KS_EINVAL, "ks_preempt: nominated node %d out of range", nominated);
  if (ctx->cfg.topology.enable && pod->topo_flags && (pod->topo_flags[0] & KS_TOPO_DYN))
    KS_FAIL(ctx, KS_EUNSUPPORTED, "ks_preempt: the dry runs do not model PodTopologySpread / InterPodAffinity (the pod "
                                  "has topology terms)");
  if (int rc = validate_pods(ctx, pod, 1); rc != KS_OK) return rc;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  if (ensure_stage(ctx, ctx->est, 1) != KS_OK) return KS_ENOMEM;
  if (stage_cols(ctx, ctx->est, pod, 1) != KS_OK || prep_stage(ctx, ctx->est, 1) != KS_OK) return KS_EHIP;
  const int64_t n = ctx->n;
  uint8_t* dunres = nullptr;
  if (unresolvable && n > 0) {
    // the caller's per-node statuses, staged through the ks_eval_pod scratch
    if (ctx->evbuf_bytes < (size_t)n) {
      dev_free(ctx->evbuf);
      ctx->evbuf_bytes = 0;
      if (dev_alloc(ctx, &ctx->evbuf, (size_t)n) != KS_OK) return KS_ENOMEM;
      ctx->evbuf_bytes = (size_t)n;
    }
    dunres = (uint8_t*)ctx->evbuf;
    HIPCHK(ctx, hipMemcpyAsync(dunres, unresolvable, (size_t)n, hipMemcpyHostToDevice, ctx->stream));
  }
  PreemptArgs a;
  a.dn = ctx->dnodes;
  a.t = ctx->npt;
  a.q = ctx->q;
  a.pq = ctx->est.pq;
  a.c = ctx->kc;
  a.pod = ctx->est.recs;
  a.pst = ctx->est.stat;
  a.prio = priority;
  a.pflags = flags;
  a.nominated = nominated;
  a.unresolvable = dunres;
  a.n = n;
  a.cand = ctx->pre_cand;
  a.vrank = ctx->pre_vrank;
  a.status = ctx->pre_status;
  a.out = ctx->pre_out;
  a.victims = ctx->pre_victims;
  // with ks_set_profile on: the dry-run kernel in stats.sweep_ms, the selection in stats.select_ms
  const bool prof = ctx->cfg.profile != 0;
  hipEvent_t e0 = prof ? take_event(ctx, 0) : nullptr, e1 = prof ? take_event(ctx, 1) : nullptr,
             e2 = prof ? take_event(ctx, 2) : nullptr;
  if (prof) HIPCHK(ctx, hipEventRecord(e0, ctx->stream));
  if (n > 0) {
    const dim3 grid((unsigned)((n + 3) / 4)), block(256);
    if (ctx->npod_slots == 1) hipLaunchKernelGGL(preempt_dry_run_kernel<1>, grid, block, 0, ctx->stream, a);
    else if (ctx->npod_slots == 2) hipLaunchKernelGGL(preempt_dry_run_kernel<2>, grid, block, 0, ctx->stream, a);
    else hipLaunchKernelGGL(preempt_dry_run_kernel<4>, grid, block, 0, ctx->stream, a);
  }
  if (prof) HIPCHK(ctx, hipEventRecord(e1, ctx->stream));
  hipLaunchKernelGGL(preempt_select_kernel, dim3(1), dim3(kPreemptSelThreads), 0, ctx->stream, a);
  HIPCHK(ctx, hipGetLastError());
  if (prof) HIPCHK(ctx, hipEventRecord(e2, ctx->stream));
  // the result and the victims (adjacent in the blob) in one read-back
  struct {
    PreemptOut o;
    unsigned char pad[16 - sizeof(PreemptOut) % 16];
    int32_t v[kPreemptMaxPods];
  } rb;
  static_assert(sizeof(PreemptOut) % 16 != 0, "PreemptOut padding");
  const size_t rbytes = (size_t)((const unsigned char*)ctx->pre_victims - (const unsigned char*)ctx->pre_out) +
                        (size_t)kPreemptMaxPods * 4;
  if (rbytes != sizeof(rb)) KS_FAIL(ctx, KS_EHIP, "ks_preempt: read-back layout");
  HIPCHK(ctx, hipMemcpyAsync(&rb, ctx->pre_out, rbytes, hipMemcpyDeviceToHost, ctx->stream));
  if (node_status && n > 0) HIPCHK(ctx, hipMemcpyAsync(node_status, ctx->pre_status, (size_t)n, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  const PreemptOut o = rb.o;
  const int32_t nv = std::min(o.nvict, victims_cap);
  if (nv > 0) memcpy(victims, rb.v, (size_t)nv * 4);
  ctx->stats = ks_stats{};
  if (prof) {
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ctx->stats.sweep_ms = ms;
    ctx->stats.sweep_launches = n > 0 ? 1 : 0;
    (void)hipEventElapsedTime(&ms, e1, e2);
    ctx->stats.select_ms = ms;
    (void)hipEventElapsedTime(&ms, e0, e2);
    ctx->stats.total_ms = ms;
  }
  // algorithmic bytes of the dry-run launch: every node's pod positions (priority, start, flags, quota, 4 PDB, 7 request
  // and 8 quota-request words: 160 B) and node words (allocatable + requested x 7, pod count, allowed, LoadAware bits;
  // the taint / label words with the dictionary plugins) once, the per-node outcome written
  ctx->stats.sweep_bytes = ctx->npt.m * 160 + n * (int64_t)(7 * 16 + 12 + (ctx->kc.stat ? 16 : 0) + sizeof(PreemptCand) + 1);
  out->node = o.node;
  out->status = o.status;
  out->num_victims = o.nvict;
  out->num_pdb_violations = o.nviol;
  out->candidates = o.candidates;
  out->potential_nodes = o.potential;
  return KS_OK;
}

int ks_shard_unique_id(uint8_t* out) {
  if (!out) return KS_EINVAL;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return KS_EHIP;
  static_assert(sizeof(id) == KS_SHARD_ID_BYTES, "ncclUniqueId size");
  memcpy(out, &id, sizeof(id));
  return KS_OK;
}

int ks_shard_init(ks_ctx* ctx, int32_t nranks, int32_t rank, const uint8_t* unique_id, int32_t virtual_shards) {
  if (!ctx || nranks < 1 || rank < 0 || rank >= nranks || virtual_shards < 1 || nranks * virtual_shards > 1024)
    return ctx ? (ctx->err = "ks_shard_init: bad args", KS_EINVAL) : KS_EINVAL;
  if (nranks > 1 && !unique_id) KS_FAIL(ctx, KS_EINVAL, "ks_shard_init: nranks > 1 needs the rank-0 unique id");
  HIPCHK(ctx, hipSetDevice(ctx->device));
  if (ctx->comm) {
    (void)ncclCommDestroy(ctx->comm);
    ctx->comm = nullptr;
  }
  loop_leave(ctx);
  if (nranks > 1 || unique_id) {
    // (nranks == 1 with an id: a one-rank communicator, so the RCCL exchange calls run on one GPU -- the test of the
    // production transport that needs no second GPU)
    ncclUniqueId id;
    memcpy(&id, unique_id, sizeof(id));
    const ncclResult_t r = ncclCommInitRank(&ctx->comm, nranks, id, rank);
    if (r != ncclSuccess) KS_FAIL(ctx, KS_EHIP, "ncclCommInitRank: %s", ncclGetErrorString(r));
  }
  ctx->nranks = nranks;
  ctx->rank = rank;
  ctx->vshards = virtual_shards;
  return KS_OK;
}

int ks_shard_init_loopback(ks_ctx* const* ctxs, int32_t nranks, int32_t virtual_shards) {
  if (!ctxs || nranks < 2 || nranks > 64 || virtual_shards < 1 || nranks * virtual_shards > 1024) return KS_EINVAL;
  for (int32_t r = 0; r < nranks; ++r) {
    if (!ctxs[r]) return KS_EINVAL;
    for (int32_t q = 0; q < r; ++q)
      if (ctxs[q] == ctxs[r]) KS_FAIL(ctxs[r], KS_EINVAL, "ks_shard_init_loopback: a context is given twice");
    if (ctxs[r]->n != ctxs[0]->n || ctxs[r]->k != ctxs[0]->k || ctxs[r]->batch != ctxs[0]->batch)
      KS_FAIL(ctxs[r], KS_EINVAL, "ks_shard_init_loopback: the ranks must load the same node count, batch and candidates");
  }
  LoopGroup* g = new LoopGroup();
  g->n = nranks;
  g->ranks.assign(ctxs, ctxs + nranks);
  for (int32_t r = 0; r < nranks; ++r) {
    ks_ctx* ctx = ctxs[r];
    auto undo = [&](int rc) {
      loop_break(g);
      if (g->refs == 0) delete g;
      return rc;
    };
    if (int rc = ks_shard_init(ctx, 1, 0, nullptr, 1); rc != KS_OK) return undo(rc);
    void* p = nullptr;
    if (dev_alloc(ctx, &p, (size_t)nranks * kNormRows * kMaxBatch * 8) != KS_OK) return undo(KS_ENOMEM);
    ctx->loop_scratch = (unsigned long long*)p;
    for (auto& pr : ctx->lev)
      for (hipEvent_t& e : pr)
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
          ctx->err = "ks_shard_init_loopback: hipEventCreate failed";
          return undo(KS_EHIP);
        }
    ctx->loop = g;
    ++g->refs;
    ctx->nranks = nranks;
    ctx->rank = r;
    ctx->vshards = virtual_shards;
  }
  return KS_OK;
}

int ks_get_stats(const ks_ctx* ctx, ks_stats* out) {
  if (!ctx || !out) return KS_EINVAL;
  *out = ctx->stats;
  return KS_OK;
}

int ks_set_profile(ks_ctx* ctx, int32_t on) {
  if (!ctx) return KS_EINVAL;
  ctx->cfg.profile = on ? 1 : 0;
  return KS_OK;
}

int ks_set_pipeline(ks_ctx* ctx, int32_t mode) {
  if (!ctx) return KS_EINVAL;
  if (mode < 0 || mode > 2) KS_FAIL(ctx, KS_EINVAL, "ks_set_pipeline: mode %d (0 off, 1 automatic, 2 always)", mode);
  ctx->pipe_mode = mode;
  return KS_OK;
}

