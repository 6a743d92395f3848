// ks_device.h — device-side data layout and per-(pod, node) evaluation for gfx950.
//
// One lane evaluates one node; the pod being evaluated is wave-uniform, so its
// record is read with scalar loads (SGPRs) and every Filter/Score formula below
// runs on the node's registers.  The formulas are the reference's, restated:
//
//   NodeResourcesFit Filter  upstream noderesources/fit.go fitsRequest
//                            (in-tree proxy pkg/scheduler/plugins/reservation/plugin.go:445-496)
//   NodeResourcesFit Score   upstream resource_allocation.go + least/most_allocated.go
//                            (in-tree copies nodenumaresource/least_allocated.go:30-58, most_allocated.go:30-62)
//   LoadAware Filter         pkg/scheduler/plugins/loadaware/load_aware.go:123-254 (pre-reduced per
//                            node by prep_nodes_kernel into fail bits; pod-dependent only via prod/daemonset)
//   LoadAware Score          load_aware.go:269-397
//
// Integer division note: every score divides by a per-node capacity.  A 64-bit
// divide is ~40 VALU ops on CDNA; instead q = floor(d*100/cap) is estimated in
// f32 with a per-node reciprocal (relative error < 2^-20, so |q_est - q| <= 1)
// and corrected exactly with one int64 multiply-subtract.  Results are bit-exact
// with Go's int64 arithmetic for every 0 <= d <= cap < 2^56.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/koordgpu.h"

namespace ks {

constexpr int kWave = 64;
constexpr int kMaxBatch = 64;  // pods per sweep pass (one lane per pod in the pass result)
constexpr int kMaxCand = 64;   // candidate chunks per pod

// internal pod flag: podRequest is all-zero with no scalar keys (fitsRequest early return)
constexpr uint32_t kPodAllZero = 0x100u;

// la_bits (prep_nodes_kernel output)
constexpr uint32_t kLaZeroScore = 0x1u;     // Score returns 0 (no NodeMetric / expired)
constexpr uint32_t kLaFailNonProd = 0x2u;   // Filter fails for non-prod (or no prod thresholds) pods
constexpr uint32_t kLaFailProd = 0x4u;      // Filter fails for prod pods when prod thresholds exist
constexpr int kLaReasonNonProdShift = 8;    // KS_R_LA_* reason bits for the non-prod case
constexpr int kLaReasonProdShift = 20;      // KS_R_LA_* reason bits for the prod case

// Kernel-constant view of ks_config.
struct Cfg {
  int32_t fit_filter, fit_score, fit_most, nsc;
  int64_t fw_cpu, fw_mem, fw_eph, fw_sc[KS_MAX_SCALARS], fit_pw;
  int32_t la_filter, la_score, la_filter_expired, la_prod_usage;
  int64_t lw_cpu, lw_mem, la_pw;
  int64_t scaling_cpu, scaling_mem;
  int32_t quota_enable, quota_parent;
  int32_t monotone;  // commits can only lower a node's key (LeastAllocated + LoadAware)
};

// Device node columns (SoA, length npad = nchunks*64, zero padded).
struct DevNodes {
  int64_t *alloc_cpu, *alloc_mem, *alloc_eph;
  int32_t *allowed_pods;
  int64_t *req_cpu, *req_mem, *req_eph;
  int32_t *pod_count;
  int64_t *nz_cpu, *nz_mem;
  int64_t *alloc_sc[KS_MAX_SCALARS], *req_sc[KS_MAX_SCALARS];
  uint32_t *la_flags;
  int64_t *la_alloc_cpu, *la_alloc_mem;
  int64_t *la_term_cpu, *la_term_mem, *la_pterm_cpu, *la_pterm_mem;
  int32_t *la_thr_cpu, *la_thr_mem, *la_pthr_cpu, *la_pthr_mem;
  int64_t *la_total_cpu, *la_total_mem, *la_usage_cpu, *la_usage_mem, *la_pusage_cpu, *la_pusage_mem;
  uint32_t *la_bits;  // derived by prep_nodes_kernel
};

// Per-pod record read by the sweep with scalar loads (AoS, 128 B).
struct __attribute__((aligned(16))) PodRec {
  int64_t cpu, mem, eph, nzcpu, nzmem, est_cpu, est_mem;
  int64_t sc[KS_MAX_SCALARS];
  uint32_t flags;
  int32_t quota;
  int64_t _pad[3];
};
static_assert(sizeof(PodRec) == 128, "PodRec must stay 128 B");

// Quota request columns for the commit kernel (SoA).
struct DevPodQuota {
  uint32_t *mask;
  int64_t *req[KS_QUOTA_DIMS];
};

struct DevQuotas {
  int32_t q;
  int32_t *parent;
  uint32_t *limit_mask, *min_mask;
  int64_t *limit, *used, *min, *npused;  // [q][KS_QUOTA_DIMS]
};

// One node in registers, with node-only precomputation done once per pass.
template <int NSC>
struct __attribute__((aligned(16))) NodeReg {
  int64_t alloc_cpu, alloc_mem, alloc_eph;
  int64_t free_cpu, free_mem, free_eph;
  int64_t nz_cpu, nz_mem, req_eph;
  int64_t alloc_sc[NSC > 0 ? NSC : 1], req_sc[NSC > 0 ? NSC : 1];
  int64_t la_alloc_cpu, la_alloc_mem, term_cpu, term_mem, pterm_cpu, pterm_mem;
  float rcp_cpu, rcp_mem, rcp_eph, rcp_lcpu, rcp_lmem;
  float rcp_sc[NSC > 0 ? NSC : 1];
  uint32_t la_bits;
  int32_t pods_full;
  int32_t allowed;
  int32_t pod_count;
  int32_t valid;
};

__device__ __forceinline__ float rcp100(int64_t cap) {
  // 100 / cap in f32; cap == 0 never reaches the divide (guarded by callers)
  uint64_t u = (uint64_t)cap;
  float f = (float)(uint32_t)(u >> 32) * 4294967296.0f + (float)(uint32_t)u;
  return cap > 0 ? 100.0f / f : 0.0f;
}

// floor(d * 100 / cap) for 0 <= d <= cap < 2^56, rcp = rcp100(cap).
__device__ __forceinline__ int64_t div100(int64_t d, int64_t cap, float rcp) {
  uint64_t u = (uint64_t)d;
  float df = (float)(uint32_t)(u >> 32) * 4294967296.0f + (float)(uint32_t)u;
  int32_t q = (int32_t)(df * rcp);
  int64_t r = d * 100 - (int64_t)q * cap;
  q += (r >= cap) ? 1 : 0;
  q -= (r < 0) ? 1 : 0;
  return q;
}

// leastRequestedScore (load_aware.go:388-397; least_allocated.go:45-54)
__device__ __forceinline__ int64_t least_req(int64_t requested, int64_t cap, float rcp) {
  if (cap == 0 || requested > cap) return 0;
  return div100(cap - requested, cap, rcp);
}

// mostRequestedScore (most_allocated.go:50-62)
__device__ __forceinline__ int64_t most_req(int64_t requested, int64_t cap, float rcp) {
  if (cap == 0) return 0;
  if (requested > cap) requested = cap;
  return div100(requested, cap, rcp);
}

// exact floor(num / den) for the weighted means of [0,100] scores
// (0 <= num < 2^24, 0 < den, quotient <= 100): f32 estimate + exact correction
__device__ __forceinline__ int64_t small_div(int64_t num, int64_t den) {
  const int32_t n32 = (int32_t)num, d32 = (int32_t)den;
  int32_t q = (int32_t)((float)n32 * __builtin_amdgcn_rcpf((float)d32));
  const int32_t r = n32 - q * d32;
  q += (r >= d32) ? 1 : 0;
  q -= (r < 0) ? 1 : 0;
  return q;
}

template <int NSC>
__device__ __forceinline__ void load_node(const DevNodes& d, int64_t n, int valid, NodeReg<NSC>& r) {
  r.valid = valid;
  if (!valid) n = 0;
  r.alloc_cpu = d.alloc_cpu[n];
  r.alloc_mem = d.alloc_mem[n];
  r.alloc_eph = d.alloc_eph[n];
  const int64_t req_cpu = d.req_cpu[n], req_mem = d.req_mem[n];
  r.req_eph = d.req_eph[n];
  r.free_cpu = r.alloc_cpu - req_cpu;
  r.free_mem = r.alloc_mem - req_mem;
  r.free_eph = r.alloc_eph - r.req_eph;
  r.allowed = d.allowed_pods[n];
  r.pod_count = d.pod_count[n];
  r.pods_full = ((int64_t)r.pod_count + 1 > (int64_t)r.allowed) || !valid;
  r.nz_cpu = d.nz_cpu[n];
  r.nz_mem = d.nz_mem[n];
#pragma unroll
  for (int k = 0; k < NSC; ++k) {
    r.alloc_sc[k] = d.alloc_sc[k][n];
    r.req_sc[k] = d.req_sc[k][n];
    r.rcp_sc[k] = rcp100(r.alloc_sc[k]);
  }
  r.la_bits = d.la_bits[n];
  r.la_alloc_cpu = d.la_alloc_cpu[n];
  r.la_alloc_mem = d.la_alloc_mem[n];
  r.term_cpu = d.la_term_cpu[n];
  r.term_mem = d.la_term_mem[n];
  r.pterm_cpu = d.la_pterm_cpu[n];
  r.pterm_mem = d.la_pterm_mem[n];
  r.rcp_cpu = rcp100(r.alloc_cpu);
  r.rcp_mem = rcp100(r.alloc_mem);
  r.rcp_eph = rcp100(r.alloc_eph);
  r.rcp_lcpu = rcp100(r.la_alloc_cpu);
  r.rcp_lmem = rcp100(r.la_alloc_mem);
}

// Reserve: NodeInfo.AddPod (upstream framework/types.go) + podAssignCache.assign
// (load_aware.go:260, pod_assign_cache.go:53): the new pod has no PodMetric, so its
// estimate counts in every later Score on this node (load_aware.go:350-355).
template <int NSC>
__device__ __forceinline__ void reserve_row(NodeReg<NSC>& r, const PodRec& p) {
  r.free_cpu -= p.cpu;
  r.free_mem -= p.mem;
  r.free_eph -= p.eph;
  r.req_eph += p.eph;
#pragma unroll
  for (int k = 0; k < NSC; ++k) r.req_sc[k] += p.sc[k];
  r.nz_cpu += p.nzcpu;
  r.nz_mem += p.nzmem;
  r.pod_count += 1;
  r.pods_full = ((int64_t)r.pod_count + 1 > (int64_t)r.allowed) || !r.valid;
  r.term_cpu += p.est_cpu;
  r.term_mem += p.est_mem;
  if (p.flags & KS_POD_PROD) {
    r.pterm_cpu += p.est_cpu;
    r.pterm_mem += p.est_mem;
  }
}

struct EvalOut {
  uint32_t reasons;  // KS_R_* (0 = feasible)
  int64_t fit, la, total;
};

// Filter + Score of one (pod, node).  DEBUG=false computes only what the sweep
// needs (feasible + total); DEBUG=true also fills reasons and per-plugin scores.
template <int NSC, bool DEBUG>
__device__ __forceinline__ EvalOut eval_pod_node(const Cfg& c, const PodRec& p, const NodeReg<NSC>& r) {
  EvalOut o;
  o.reasons = 0;
  o.fit = 0;
  o.la = 0;
  o.total = 0;
  uint32_t rs = 0;
  if (c.fit_filter) {
    if (r.pods_full) rs |= KS_R_FIT_PODS;
    if (!(p.flags & kPodAllZero)) {
      if (p.cpu > r.free_cpu) rs |= KS_R_FIT_CPU;
      if (p.mem > r.free_mem) rs |= KS_R_FIT_MEMORY;
      if (p.eph > r.free_eph) rs |= KS_R_FIT_EPHEMERAL;
#pragma unroll
      for (int k = 0; k < NSC; ++k)
        if (p.sc[k] != 0 && p.sc[k] > r.alloc_sc[k] - r.req_sc[k]) rs |= KS_R_FIT_SCALAR;
    }
  } else if (!r.valid) {
    rs |= KS_R_FIT_PODS;
  }
  if (c.la_filter && !(p.flags & KS_POD_DAEMONSET)) {
    const bool prod_path = (p.flags & KS_POD_PROD) != 0;
    const uint32_t failbit = prod_path ? kLaFailProd : kLaFailNonProd;
    if (r.la_bits & failbit) {
      if (DEBUG)
        rs |= (r.la_bits >> (prod_path ? kLaReasonProdShift : kLaReasonNonProdShift)) & 0x1ffu;
      else
        rs |= KS_R_LA_CPU;
    }
  }
  o.reasons = rs;
  if (!DEBUG && rs) return o;
  if (c.fit_score) {
    int64_t ns = 0, ws = 0;
    auto term = [&](int64_t w, int64_t alloc, int64_t req, float rcp) {
      if (w != 0 && alloc != 0) {
        ns += (c.fit_most ? most_req(req, alloc, rcp) : least_req(req, alloc, rcp)) * w;
        ws += w;
      }
    };
    term(c.fw_cpu, r.alloc_cpu, r.nz_cpu + p.nzcpu, r.rcp_cpu);
    term(c.fw_mem, r.alloc_mem, r.nz_mem + p.nzmem, r.rcp_mem);
    term(c.fw_eph, r.alloc_eph, r.req_eph + p.eph, r.rcp_eph);
#pragma unroll
    for (int k = 0; k < NSC; ++k)
      if (p.sc[k] != 0) term(c.fw_sc[k], r.alloc_sc[k], r.req_sc[k] + p.sc[k], r.rcp_sc[k]);
    o.fit = ws ? small_div(ns, ws) : 0;
    o.total += o.fit * c.fit_pw;
  }
  if (c.la_score && !(r.la_bits & kLaZeroScore)) {
    const bool prod = (p.flags & KS_POD_PROD) && c.la_prod_usage;
    const int64_t ucpu = p.est_cpu + (prod ? r.pterm_cpu : r.term_cpu);
    const int64_t umem = p.est_mem + (prod ? r.pterm_mem : r.term_mem);
    int64_t ns = 0, ws = 0;
    if (c.lw_cpu) {
      ns += least_req(ucpu, r.la_alloc_cpu, r.rcp_lcpu) * c.lw_cpu;
      ws += c.lw_cpu;
    }
    if (c.lw_mem) {
      ns += least_req(umem, r.la_alloc_mem, r.rcp_lmem) * c.lw_mem;
      ws += c.lw_mem;
    }
    o.la = ws ? small_div(ns, ws) : 0;
    o.total += o.la * c.la_pw;
  }
  return o;
}

// Wave-wide reductions (64 lanes), result wave-uniform.
// DPP within each 16-lane row (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror),
// then the four row maxima through readlane into SGPRs.  Requires all 64 lanes active.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}

__device__ __forceinline__ uint32_t umax32(uint32_t a, uint32_t b) { return a > b ? a : b; }
__device__ __forceinline__ uint64_t umax64(uint64_t a, uint64_t b) { return a > b ? a : b; }

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  v = umax32(v, dpp32<0xB1>(v));
  v = umax32(v, dpp32<0x4E>(v));
  v = umax32(v, dpp32<0x141>(v));
  v = umax32(v, dpp32<0x140>(v));
  const uint32_t r0 = __builtin_amdgcn_readlane(v, 0), r1 = __builtin_amdgcn_readlane(v, 16);
  const uint32_t r2 = __builtin_amdgcn_readlane(v, 32), r3 = __builtin_amdgcn_readlane(v, 48);
  return umax32(umax32(r0, r1), umax32(r2, r3));
}

template <int CTRL>
__device__ __forceinline__ uint64_t dpp64(uint64_t v) {
  const uint32_t lo = dpp32<CTRL>((uint32_t)v), hi = dpp32<CTRL>((uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, l), hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
  v = umax64(v, dpp64<0xB1>(v));
  v = umax64(v, dpp64<0x4E>(v));
  v = umax64(v, dpp64<0x141>(v));
  v = umax64(v, dpp64<0x140>(v));
  return umax64(umax64(readlane64(v, 0), readlane64(v, 16)), umax64(readlane64(v, 32), readlane64(v, 48)));
}

__device__ __forceinline__ int32_t wave_sum_i32(int32_t v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// global candidate key: higher is better; (score+1) in the high word, ~node in the low word
__device__ __forceinline__ uint64_t gkey(int64_t total, int64_t node) {
  return ((uint64_t)(total + 1) << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)node);
}
__device__ __forceinline__ int64_t gkey_node(uint64_t k) { return (int64_t)(0xFFFFFFFFu - (uint32_t)k); }
__device__ __forceinline__ int64_t gkey_score(uint64_t k) { return (int64_t)(k >> 32) - 1; }

}  // namespace ks
