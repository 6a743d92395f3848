// ks_dev.h — DeviceShare (GPU) on the device (pkg/scheduler/plugins/deviceshare).
//
// Per (pod, node): GPUHandler.CalcDesiredRequestsAndCount after fillGPUTotalMem
// (devicehandler_gpu.go:40-98: the request per instance and the instance count), the
// defaultAllocateDevices feasibility (device_allocator.go:392-462: enough free minors satisfy
// LessThanOrEqual(request, free)), and the node score scoreNode (scoring.go:228-253) over the summed
// totals / free amounts.  Reserve picks the minors in sortDeviceResourcesByMinor order (score desc,
// minor asc; device_resources.go:171-208) and adds the request to each (updateCacheUsed).
//
// NormalizeScore is DefaultNormalizeScore(100) over the feasible nodes (scoring.go:95-97): a
// cross-node max M.  The sweep runs twice when DeviceShare is on — phase 0 reduces, per pod, the
// key (M << 32 | ~witness) where the witness is the lowest-index feasible node holding M; phase 1
// scores with floor(100 * raw / M).  The commit kernel keeps M valid: the untouched nodes'
// maximum is still M while the witness is untouched, the touched nodes are re-scored, and a pass
// whose M would change is cut so the next pass re-sweeps from that pod.
#pragma once

#include "ks_device.h"

namespace ks {

constexpr int kGpus = KS_MAX_GPUS;

struct DevDev {
  const uint32_t* flags;  // [npad] KS_DEV_*
  const int64_t* total;   // [3][kGpus][npad]  q = 0 core, 1 memory, 2 ratio
  int64_t* used;          // [3][kGpus][npad]  mutable (Reserve)
  int64_t npad;
};

// A GPU instance request for one node: per-instance (core, memory, ratio), count, core key present.
struct GpuReq {
  int64_t core, mem, ratio;
  int32_t desired;
  bool has_core;
  bool no_gpu;  // no healthy GPU on the node (UnschedulableAndUnresolvable)
};

// views of one node's GPUs: HBM columns or the commit kernel's LDS copy (tot/use[q*kGpus+k])
struct DevGView {
  const DevDev& d;
  int64_t n;
  __device__ __forceinline__ bool present() const { return (gld(d.flags + n) & KS_DEV_PRESENT) != 0; }
  __device__ __forceinline__ int64_t total(int q, int k) const { return gld(d.total + ((int64_t)q * kGpus + k) * d.npad + n); }
  __device__ __forceinline__ int64_t used(int q, int k) const { return gld(d.used + ((int64_t)q * kGpus + k) * d.npad + n); }
};

struct DevLView {
  const int64_t* tot;  // [3*kGpus]
  const int64_t* use;  // [3*kGpus]
  bool pres;
  __device__ __forceinline__ bool present() const { return pres; }
  __device__ __forceinline__ int64_t total(int q, int k) const { return tot[q * kGpus + k]; }
  __device__ __forceinline__ int64_t used(int q, int k) const { return use[q * kGpus + k]; }
};

template <typename V>
__device__ __forceinline__ GpuReq gpu_request(const PodRec& p, const V& v) {
  GpuReq g{0, 0, 0, 1, (p.flags & KS_POD_GPU_CORE) != 0, false};
  int64_t total_mem = -1;
#pragma unroll
  for (int k = kGpus - 1; k >= 0; --k) {  // the first healthy minor (all GPUs of a node are the same model)
    const int64_t tc = v.total(0, k), tm = v.total(1, k), tr = v.total(2, k);
    if (tc || tm || tr) total_mem = tm;
  }
  if (total_mem < 0) {
    g.no_gpu = true;
    return g;
  }
  int64_t core = p.gpu_core, mem = p.gpu_mem, ratio = p.gpu_ratio;
  if (p.flags & KS_POD_GPU_MEMORY)
    ratio = (int64_t)((double)mem / (double)total_mem * 100.0);  // memoryBytesToRatio
  else
    mem = ratio * total_mem / 100;  // memoryRatioToBytes
  if (ratio > 100 && ratio % 100 == 0) {
    g.desired = (int32_t)(ratio / 100);
    core /= g.desired;
    mem /= g.desired;
    ratio /= g.desired;
  }
  g.core = core;
  g.mem = mem;
  g.ratio = ratio;
  return g;
}

// one resource of the scorer: Least/MostAllocated of (requested, capacity) (scoring.go:278-308)
__device__ __forceinline__ int32_t dev_term(bool most, int64_t req, int64_t cap) {
  if (most) return pct_floor_i64(req > cap ? cap : req, cap);
  return req > cap ? 0 : pct_floor_i64(cap - req, cap);
}

// scoreDevice / scoreNode body: requested = total - free + pod (total >= free), allocatable = total
__device__ __forceinline__ int32_t dev_score3(const Cfg& c, const int64_t* tot, const int64_t* fre, const int64_t* pod) {
  const int32_t w[3] = {c.dw_core, c.dw_mem, c.dw_ratio};
  int32_t ns = 0, ws = 0;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    if (w[q] == 0 || tot[q] == 0) continue;
    const int64_t req = tot[q] >= fre[q] ? tot[q] - fre[q] + pod[q] : tot[q];
    ns += dev_term(c.dev_most != 0, req, tot[q]) * w[q];
    ws += w[q];
  }
  return ws ? small_div(ns, ws) : 0;
}

struct DevOut {
  uint32_t reasons;  // KS_R_DEV_*
  int32_t raw;       // scoreNode (feasible only)
  uint32_t minors;   // allocation (ALLOC only)
};

// DeviceShare Filter + Score (+ the allocation with ALLOC) of one (pod, node).
template <bool ALLOC, typename V>
__device__ __forceinline__ DevOut dev_eval(const Cfg& c, const PodRec& p, const V& v, GpuReq* req_out = nullptr) {
  DevOut o{0u, 0, 0u};
  if (!v.present()) return o;  // no device info: Filter passes, Score 0
  const GpuReq g = gpu_request(p, v);
  if (req_out) *req_out = g;
  if (g.no_gpu) {
    o.reasons = KS_R_DEV_NO_GPU;
    return o;
  }
  const int64_t pod[3] = {g.has_core ? g.core : 0, g.mem, g.ratio};
  int64_t tsum[3] = {0, 0, 0}, fsum[3] = {0, 0, 0};
  int32_t nfit = 0;
  int32_t sc[kGpus];
  uint32_t fitmask = 0;
#pragma unroll
  for (int k = 0; k < kGpus; ++k) {
    const int64_t t[3] = {v.total(0, k), v.total(1, k), v.total(2, k)};
    const int64_t f[3] = {t[0] - v.used(0, k), t[1] - v.used(1, k), t[2] - v.used(2, k)};
    const bool exists = t[0] || t[1] || t[2];
    const bool has_free = exists && (f[0] || f[1] || f[2]);
    const bool fits = has_free && (!g.has_core || g.core <= f[0]) && g.mem <= f[1] && g.ratio <= f[2];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      tsum[q] += exists ? t[q] : 0;
      fsum[q] += has_free ? f[q] : 0;
    }
    nfit += fits ? 1 : 0;
    fitmask |= fits ? (1u << k) : 0u;
    sc[k] = (ALLOC && fits) ? dev_score3(c, t, f, pod) : 0;
  }
  if (nfit < g.desired) {
    o.reasons = KS_R_DEV_INSUFFICIENT;
    return o;
  }
  o.raw = dev_score3(c, tsum, fsum, pod);
  if (ALLOC) {
    uint32_t mask = 0;
    for (int got = 0; got < g.desired; ++got) {
      int best = -1;
      int32_t bs = -1;
#pragma unroll
      for (int k = 0; k < kGpus; ++k) {
        const bool cand = ((fitmask >> k) & 1u) && !((mask >> k) & 1u) && sc[k] > bs;
        best = cand ? k : best;
        bs = cand ? sc[k] : bs;
      }
      mask |= 1u << best;
    }
    o.minors = mask;
  }
  return o;
}

}  // namespace ks
