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
// divide is ~40 VALU ops on CDNA; the score terms instead compute
// q = floor(100*d/cap) as one f64 fma, trunc(fma(100*d, 1/cap, 2^-44)), exact for
// cap < 2^43 and 100*|d| < 2^53 (see term_least); other nodes / pods take the
// int64 path (f32 estimate corrected by one int64 multiply-subtract, exact for
// 0 <= d <= cap < 2^56).  Results are bit-exact with Go's int64 arithmetic.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/koordgpu.h"

namespace ks {

constexpr int kWave = 64;
constexpr int kMaxBatch = 64;  // pods per sweep pass (one lane per pod in the pass result)
constexpr int kMaxCand = 64;   // candidate chunks per pod

// internal pod flag: podRequest is all-zero with no scalar keys (fitsRequest early return)
constexpr uint32_t kPodAllZero = 0x100u;
// internal pod flag: every request value is zero (quotav1.IsZero, NodeNUMAResource PreFilter skip)
constexpr uint32_t kPodReqZero = 0x200u;
// internal pod flag: the pod has a device request, GPU or RDMA (DeviceShare preparePod: skip = false)
constexpr uint32_t kPodHasGpu = 0x400u;
// internal pod flag: the pod has a GPU request
constexpr uint32_t kPodGpuReq = 0x800u;
// internal pod flag: a score-term request >= kBigReq: the pod's terms take the int64 path
constexpr uint32_t kPodBigReq = 0x1000u;
// internal pod flag: a normalized score (DeviceShare, TaintToleration, NodeAffinity) can differ between nodes for the
// pod, so a commit may change its normalization max (the monotone fast path does not hold for it)
constexpr uint32_t kPodNormDyn = 0x2000u;
// internal pod flag: DeviceShare (enabled) has the pod's device requests, so its FilterReservation (plugin.go:322-358)
// rejects every reservation holding no device -- every reservation the library models: none is nominated
// (nominator.go:163-168), the pod is never assumed into one (reservation/plugin.go:546-560)
constexpr uint32_t kPodDevNoNom = 0x8000u;

// la_bits (prep_nodes_kernel output)
constexpr uint32_t kLaZeroScore = 0x1u;     // Score returns 0 (no NodeMetric / expired)
constexpr uint32_t kLaFailNonProd = 0x2u;   // Filter fails for non-prod (or no prod thresholds) pods
constexpr uint32_t kLaFailProd = 0x4u;      // Filter fails for prod pods when prod thresholds exist
constexpr int kLaReasonNonProdShift = 8;    // KS_R_LA_* reason bits for the non-prod case
constexpr int kLaReasonProdShift = 20;      // KS_R_LA_* reason bits for the prod case
constexpr uint32_t kNodeBigCap = 0x8u;      // a score-term capacity >= kBigCap: the node's terms take the int64 path
constexpr uint32_t kNumaPolNode = 1u << 29; // NodeNUMAResource: the node has a NUMA topology policy (numa_flags bits 5-6)
constexpr uint32_t kNumaAmp = 1u << 30;     // NodeNUMAResource: cpu amplification ratio > 1
constexpr uint32_t kNumaInvalid = 1u << 31; // NodeNUMAResource: invalid amplification annotation

// Kernel-constant view of ks_config (int32: weights are validated to small ranges in ks_create,
// which keeps the sweep's SGPR footprint small).
struct Cfg {
  int32_t fit_filter, fit_score, fit_most, nsc;
  int32_t fw_cpu, fw_mem, fw_eph, fw_sc[KS_MAX_SCALARS], fit_pw;
  int32_t la_filter, la_score, la_filter_expired, la_prod_usage;
  int32_t lw_cpu, lw_mem, la_pw;
  int32_t quota_enable, quota_parent;
  int32_t monotone;  // commits can only lower a node's key (LeastAllocated + LoadAware)
  int32_t rsv;       // Reservation plugin enabled
  int32_t rsv_F;     // key radix: key total = hi * rsv_F + (Fit + LoadAware + NUMA weighted total), see ks_rsv.h
  int32_t numa, numa_most, nw_cpu, nw_mem, numa_pw;  // NodeNUMAResource
  int32_t cpuset;    // CPU state loaded: cpu-bind pods are evaluated (ks_cpuset.h)
  int32_t numa_pol;  // nodes with a NUMA topology policy exist (ks_numa.h)
  int32_t numa_sc_most;  // NUMAScoringStrategy MostAllocated (hint scores)
  int32_t dev, dev_most, dw_core, dw_mem, dw_ratio, dev_pw, dw_rdma;  // DeviceShare (GPU, RDMA)
  int32_t monotone_nd;  // monotone for pods without device requests (DeviceShare skips them: no normalization max)
  int32_t cores;        // node CPU bind policies or required pod policies: the per-node core counts are read
  int32_t bal, bal_pw;  // upstream NodeResourcesBalancedAllocation: KS_BAL_* resources (0 = off), plugin weight
  int32_t taint, taint_pw;  // upstream TaintToleration: bit 0 Filter, bit 1 Score; plugin weight
  int32_t aff, aff_pw;      // upstream NodeAffinity: bit 0 Filter, bit 1 Score; plugin weight
  int32_t ports;            // upstream NodePorts Filter (bit 0)
  int32_t stat;             // taint | aff | ports: the dictionary-bit plugins are on (kernel variant FEAT & 4, PodStat)
  // Reservation with an otherwise monotone plugin set: monotone for the pods that match no reservation (class -1)
  // while no commit of the pass lowered a node's restored Requested (ks_pass.h commit_kernel)
  int32_t monotone_rsv;
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
  uint64_t *rsv_cls;  // union of the owner classes of the node's matchable reservations (ks_rsv.h)
  double *numa_ratio;       // NodeNUMAResource inputs: cpu amplification ratio, cpuset CPUs, flags
  int32_t *numa_cpus;
  uint32_t *numa_flags;
  int64_t *numa_amilli;     // derived: cpuset CPUs x 1000
  int64_t *numa_off;        // derived: Amplify(cpuset milli, ratio) - cpuset milli (ratio > 1), else 0
  int32_t *cpu_free;        // available CPUs for cpuset pods (ks_cpuset.h), -1 = no valid CPU topology
  uint32_t *cpu_cores;      // derived: CoresWord (fully available / partly available cores, CPUsPerCore, CPU bind label)
  uint64_t *taints_hard, *taints_soft, *labels;  // TaintToleration / NodeAffinity dictionary bits (static per node)
  uint64_t *host_ports;                          // NodePorts dictionary bits in use (mutable: every Reserve adds)
};

// Per-node word of the required CPU bind policies (Cfg.cores): the cores whose CPUs are all available
// (filterCPUsByRequiredCPUBindPolicy FullPCPUs keeps exactly these), the cores with any available CPU
// (SpreadByPCPUs keeps one CPU of each), CPUsPerCore, and the node's CPU bind policy (KS_NODE_CPU_BIND_*).
// Bit 26 is the commit kernel's per-slot "cores changed in this pass" flag.
constexpr uint32_t kCoresCount = 0x1FFu;
constexpr int kCoresAnyShift = 9, kCoresCpcShift = 18, kCoresLabelShift = 24;
constexpr uint32_t kCoresDirty = 1u << 26;
__device__ __forceinline__ uint32_t cores_full(uint32_t w) { return w & kCoresCount; }
__device__ __forceinline__ uint32_t cores_any(uint32_t w) { return (w >> kCoresAnyShift) & kCoresCount; }
__device__ __forceinline__ uint32_t cores_cpc(uint32_t w) { return (w >> kCoresCpcShift) & 31u; }
__device__ __forceinline__ uint32_t cores_label(uint32_t w) { return (w >> kCoresLabelShift) & 3u; }

// Per-pod record read by the sweep with scalar loads (AoS, 192 B).  The x100 and f32 copies feed
// the exact score terms (see term_least below).
struct __attribute__((aligned(16))) PodRec {
  int64_t cpu, mem, eph, nzcpu, nzmem, est_cpu, est_mem;  // words 0..6
  int64_t sc[KS_MAX_SCALARS];                              // words 7..10
  uint32_t flags;                                          // word 11 (lo)
  int32_t quota;                                           // word 11 (hi)
  // 100 x the score-term requests (nzcpu, nzmem, eph, est_cpu, est_mem, sc[k]) as f64 (exact: kPodBigReq otherwise)
  double h_nzcpu, h_nzmem, h_eph, h_est_cpu, h_est_mem;    // words 12..16
  double h_sc[KS_MAX_SCALARS];                             // words 17..20
  int32_t rsv_class;  // reservation match class (-1 = none)
  uint32_t rsv_keys;  // bit d: request dimension d is non-zero (a key of the pod's requests)
  uint32_t cpu_bind;  // KS_POD_CPU_BIND pods: KS_CPU_BIND_* | exclusive << KS_CPU_EXCL_SHIFT | numCPUsNeeded << 8
  int32_t _pad1;
  double h_cpu, h_mem;  // 100 x the Requested cpu / memory (NodeNUMAResource score)
  int64_t gpu_core, gpu_mem, gpu_ratio;  // DeviceShare: converted GPU request
  int64_t rdma;                          // DeviceShare: koordinator.sh/rdma request
  uint32_t joint;                        // DeviceShare: KS_JOINT_*
  int32_t _pad0;
};
static_assert(sizeof(PodRec) == 240, "PodRec layout");
// PodRec int64 word indices read by the commit kernel's lane-parallel Reserve
constexpr int kPodWordHCpu = (int)(offsetof(PodRec, h_cpu) / 8), kPodWordHMem = (int)(offsetof(PodRec, h_mem) / 8);
static_assert(offsetof(PodRec, h_nzcpu) == 12 * 8 && offsetof(PodRec, h_sc) == 17 * 8, "PodRec word layout");

// Explicit global (addrspace 1) accesses for pointers read from memory: without the cast hipcc
// emits flat_load, which counts on lgkmcnt too, so every later LDS wait would also wait for the
// HBM load (the commit kernel overlaps its row prefetch with LDS work).
template <typename T>
__device__ __forceinline__ T gld(const T* p) {
#if defined(__HIP_DEVICE_COMPILE__)
  return *(const __attribute__((address_space(1))) T*)p;
#else
  return *p;
#endif
}
template <typename T>
__device__ __forceinline__ void gst(T* p, T v) {
#if defined(__HIP_DEVICE_COMPILE__)
  *(__attribute__((address_space(1))) T*)p = v;
#else
  *p = v;
#endif
}

// Wave-uniform pod record through the constant address space: the compiler emits scalar loads
// (s_load) into SGPRs, so every branch on pod fields is a scalar branch.
__device__ __forceinline__ PodRec load_pod_uniform(const PodRec* p) {
  PodRec r;
#if defined(__HIP_DEVICE_COMPILE__)
  typedef const __attribute__((address_space(4))) int64_t* ConstWords;
  const ConstWords src = (ConstWords)p;
  int64_t* dst = reinterpret_cast<int64_t*>(&r);
#pragma unroll
  for (int i = 0; i < (int)(sizeof(PodRec) / 8); ++i) dst[i] = src[i];
#else
  r = *p;
#endif
  return r;
}

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

// One score term's node side: capacity c and headroom h = c - requested_on_node (offset by -2^62 when
// c == 0, so the int64 path scores 0 without a branch while the requested value stays recoverable,
// term_requested), and for the f64 path hd = 100*h and r = 1/c (both 0 when c == 0).
struct Term {
  int64_t c, h;
  double hd, r;
};

__device__ __forceinline__ float i64_to_f32(int64_t v) {
  // |v| < 2^62: hi part exact in f32 up to 2^24, the sum within 2^-23 relative
  return __builtin_fmaf((float)(int32_t)(v >> 32), 4294967296.0f, (float)(uint32_t)v);
}

// exact floor(100 * num / cap) for 0 <= num <= cap < 2^56, cap > 0 (f32 estimate + int64 correction)
__device__ __forceinline__ int32_t pct_floor_i64(int64_t num, int64_t cap) {
  int32_t q = (int32_t)(i64_to_f32(num) * 100.0f * __builtin_amdgcn_rcpf(i64_to_f32(cap)));
  const int64_t r = num * 100 - (int64_t)q * cap;
  q += (r >= cap) ? 1 : 0;
  q -= (r < 0) ? 1 : 0;
  return q;
}

constexpr int64_t kNoCap = -((int64_t)1 << 62);
// f64 score path limits (term_least): capacities below kBigCap, requests below kBigReq
constexpr int64_t kBigCap = (int64_t)1 << 43;
constexpr int64_t kBigReq = (int64_t)1 << 46;
constexpr double kScoreBias = 0x1p-44;

__device__ __forceinline__ void term_set(Term& t, int64_t cap, int64_t requested) {
  t.c = cap;
  t.h = cap - requested + (cap != 0 ? 0 : kNoCap);
  t.hd = cap != 0 ? (double)(cap - requested) * 100.0 : 0.0;
  t.r = cap != 0 ? 1.0 / (double)cap : 0.0;
}

__device__ __forceinline__ int64_t term_requested(const Term& t) { return t.c - t.h + (t.c != 0 ? 0 : kNoCap); }

// Reserve: the node's requested grows by r (rd = 100 r as f64).
__device__ __forceinline__ void term_take(Term& t, int64_t r, double rd) {
  t.h -= r;
  t.hd -= rd;
}

// leastRequestedScore(requested = c - h + p, c) (load_aware.go:388-397, least_allocated.go:45-54):
// 0 if c == 0 or requested > c, else floor(100 (h - p) / c).
// f64 path: x = fma(100 (h - p), r, B) with r = fl(1/c), B = 2^-44, then trunc(max(x, 0)).  100(h-p) is an
// exact f64 integer (100|h|, 100 p < 2^53).  For 0 <= h - p <= c the exact quotient x* lies in [0, 100] and
// |x - (x* + B)| <= |100(h-p)| |r - 1/c| + ulp(x)/2 <= 100 * 2^-53 + 2^-47 < 2^-45, so an integral x*
// truncates to itself (x >= x* + B - 2^-45 > x*), and a non-integral one is at least 1/c > 2^-43 below the
// next integer (c < 2^43), which B + 2^-45 < 2^-43 cannot cross.  For h < p, x* <= -100/c and x < 1, so the
// result is 0.  tests/test_score_f64.py replays the formula on the boundary cases with exact rational
// arithmetic.
__device__ __forceinline__ int32_t term_least(const Term& t, double pd) {
  return (int32_t)fmax(fma(t.hd - pd, t.r, kScoreBias), 0.0);
}
__device__ __forceinline__ int32_t term_least_i64(const Term& t, int64_t p) {
  return t.h >= p ? pct_floor_i64(t.h - p, t.c) : 0;
}

// mostRequestedScore(requested, c) (most_allocated.go:50-62): requested clamped to c, then
// floor(requested * 100 / c); requested = c - (h - p).  f64 path: y = fma(100 (p - h), r, 100 + B), exact by
// the same argument (y* = 100 requested / c >= 0), clamped to 100 for requested > c; 0 when c == 0.
__device__ __forceinline__ int32_t term_most(const Term& t, double pd) {
  const int32_t q = (int32_t)fmin(fma(pd - t.hd, t.r, 100.0 + kScoreBias), 100.0);
  return t.r != 0.0 ? q : 0;
}
__device__ __forceinline__ int32_t term_most_i64(const Term& t, int64_t p) {
  if (t.c == 0) return 0;
  if (p > t.h) return 100;
  return pct_floor_i64(t.c - (t.h - p), t.c);
}

// One node in registers, with node-only precomputation done once per load.
template <int NSC>
struct __attribute__((aligned(16))) NodeReg {
  int64_t free_cpu, free_mem, free_eph;       // Allocatable - Requested (Fit Filter)
  int64_t free_sc[NSC > 0 ? NSC : 1];
  Term t_cpu, t_mem;                           // Fit cpu/memory: NonZeroRequested (upstream resource_allocation.go)
  Term t_eph;                                  // Fit ephemeral-storage: Requested
  Term t_sc[NSC > 0 ? NSC : 1];                // Fit scalars: Requested
  Term t_lcpu, t_lmem, t_plcpu, t_plmem;       // LoadAware: EstimateNode alloc - node term (all / prod)
  Term t_ncpu, t_nmem;                         // NodeNUMAResource: Requested (+ amplified cpuset part for cpu)
  int64_t numa_A, numa_off;                    // cpuset milli-CPUs, Amplify(A) - A
  double numa_ratio;                           // cpu amplification ratio (amplifies a cpu-bind pod's request)
  int32_t cpu_free;                            // available CPUs for cpuset pods, -1 = no valid CPU topology
  uint32_t cpu_cores;                          // CoresWord (Cfg.cores), else 0
  uint32_t la_bits;
  int32_t fit_ws;                              // Σ weights of cpu/mem/eph terms with capacity != 0
  int32_t pods_full;
  int32_t allowed;
  int32_t pod_count;
  int32_t valid;
  uint64_t rsv_cls;                            // owner classes of matchable reservations (0 = none)
};

template <int NSC>
__device__ __forceinline__ int32_t node_fit_ws(const Cfg& c, const NodeReg<NSC>& r) {
  return (r.t_cpu.c != 0 ? c.fw_cpu : 0) + (r.t_mem.c != 0 ? c.fw_mem : 0) + (r.t_eph.c != 0 ? c.fw_eph : 0);
}

// exact floor(num / den) for the weighted means of [0,100] scores
// (0 <= num < 2^24, 0 < den, quotient <= 100): f32 estimate + exact correction
__device__ __forceinline__ int32_t small_div(int32_t n32, int32_t d32) {
  int32_t q = (int32_t)((float)n32 * __builtin_amdgcn_rcpf((float)d32));
  const int32_t r = n32 - q * d32;
  q += (r >= d32) ? 1 : 0;
  q -= (r < 0) ? 1 : 0;
  return q;
}

// Build a NodeReg from the node's fields (shared by load_node and the commit's raw rows).
template <int NSC>
__device__ __forceinline__ void make_node(const Cfg& c, NodeReg<NSC>& r, int valid, int64_t alloc_cpu,
                                          int64_t alloc_mem, int64_t alloc_eph, int64_t req_cpu, int64_t req_mem,
                                          int64_t req_eph, int64_t nz_cpu, int64_t nz_mem, const int64_t* alloc_sc,
                                          const int64_t* req_sc, int64_t la_alloc_cpu, int64_t la_alloc_mem,
                                          int64_t term_cpu, int64_t term_mem, int64_t pterm_cpu, int64_t pterm_mem,
                                          uint32_t la_bits, int32_t allowed, int32_t pod_count, int64_t numa_A = 0,
                                          int64_t numa_off = 0, double numa_ratio = 0.0, int32_t cpu_free = -1) {
  r.valid = valid;
  r.free_cpu = alloc_cpu - req_cpu;
  r.free_mem = alloc_mem - req_mem;
  r.free_eph = alloc_eph - req_eph;
  term_set(r.t_cpu, alloc_cpu, nz_cpu);
  term_set(r.t_mem, alloc_mem, nz_mem);
  term_set(r.t_eph, alloc_eph, req_eph);
#pragma unroll
  for (int k = 0; k < NSC; ++k) {
    r.free_sc[k] = alloc_sc[k] - req_sc[k];
    term_set(r.t_sc[k], alloc_sc[k], req_sc[k]);
  }
  term_set(r.t_lcpu, la_alloc_cpu, term_cpu);
  term_set(r.t_lmem, la_alloc_mem, term_mem);
  term_set(r.t_plcpu, la_alloc_cpu, pterm_cpu);
  term_set(r.t_plmem, la_alloc_mem, pterm_mem);
  r.la_bits = la_bits;
  r.allowed = allowed;
  r.pod_count = pod_count;
  r.pods_full = ((int64_t)pod_count + 1 > (int64_t)allowed) || !valid;
  r.fit_ws = node_fit_ws<NSC>(c, r);
  r.rsv_cls = 0;
  r.numa_A = numa_A;
  r.numa_off = numa_off;
  r.numa_ratio = numa_ratio;
  r.cpu_free = cpu_free;
  r.cpu_cores = 0;
  term_set(r.t_ncpu, alloc_cpu, req_cpu + numa_off);
  term_set(r.t_nmem, alloc_mem, req_mem);
}

template <int NSC>
__device__ __forceinline__ void load_node(const Cfg& c, const DevNodes& d, int64_t n, int valid, NodeReg<NSC>& r) {
  if (!valid) n = 0;
  int64_t asc[NSC > 0 ? NSC : 1], rsc[NSC > 0 ? NSC : 1];
#pragma unroll
  for (int k = 0; k < NSC; ++k) {
    asc[k] = gld(d.alloc_sc[k] + n);
    rsc[k] = gld(d.req_sc[k] + n);
  }
  int64_t na = 0, no = 0;
  double nr = 0.0;
  int32_t cf = -1;
  if (c.numa) {
    na = gld(d.numa_amilli + n);
    no = gld(d.numa_off + n);
    if (c.cpuset) {
      nr = gld(d.numa_ratio + n);
      cf = gld(d.cpu_free + n);
    }
  }
  make_node<NSC>(c, r, valid, gld(d.alloc_cpu + n), gld(d.alloc_mem + n), gld(d.alloc_eph + n), gld(d.req_cpu + n),
                 gld(d.req_mem + n), gld(d.req_eph + n), gld(d.nz_cpu + n), gld(d.nz_mem + n), asc, rsc,
                 gld(d.la_alloc_cpu + n), gld(d.la_alloc_mem + n), gld(d.la_term_cpu + n), gld(d.la_term_mem + n),
                 gld(d.la_pterm_cpu + n), gld(d.la_pterm_mem + n), gld(d.la_bits + n), gld(d.allowed_pods + n),
                 gld(d.pod_count + n), na, no, nr, cf);
  if (c.rsv && valid) r.rsv_cls = gld(d.rsv_cls + n);
  if (c.cores) r.cpu_cores = gld(d.cpu_cores + n);
}

// Reserve: NodeInfo.AddPod (upstream framework/types.go) + podAssignCache.assign
// (load_aware.go:260, pod_assign_cache.go:53): the new pod has no PodMetric, so its
// estimate counts in every later Score on this node (load_aware.go:350-355).
template <int NSC>
__device__ __forceinline__ void reserve_row(NodeReg<NSC>& r, const PodRec& p) {
  r.free_cpu -= p.cpu;
  r.free_mem -= p.mem;
  r.free_eph -= p.eph;
  term_take(r.t_cpu, p.nzcpu, p.h_nzcpu);
  term_take(r.t_mem, p.nzmem, p.h_nzmem);
  term_take(r.t_eph, p.eph, p.h_eph);
#pragma unroll
  for (int k = 0; k < NSC; ++k) {
    r.free_sc[k] -= p.sc[k];
    term_take(r.t_sc[k], p.sc[k], p.h_sc[k]);
  }
  r.pod_count += 1;
  r.pods_full = ((int64_t)r.pod_count + 1 > (int64_t)r.allowed) || !r.valid;
  term_take(r.t_ncpu, p.cpu, p.h_cpu);
  term_take(r.t_nmem, p.mem, p.h_mem);
  term_take(r.t_lcpu, p.est_cpu, p.h_est_cpu);
  term_take(r.t_lmem, p.est_mem, p.h_est_mem);
  if (p.flags & KS_POD_PROD) {
    term_take(r.t_plcpu, p.est_cpu, p.h_est_cpu);
    term_take(r.t_plmem, p.est_mem, p.h_est_mem);
  }
}

struct EvalOut {
  uint32_t reasons;  // KS_R_* (0 = feasible)
  int32_t fit, la, total;  // total: Fit + LoadAware + NodeNUMAResource (weighted)
  int32_t numa;
  int32_t dev_raw;         // DeviceShare raw score (normalized in key_total)
  int32_t hi;              // Reservation ranking component (ks_rsv.h)
  int32_t bal;             // NodeResourcesBalancedAllocation score
  uint32_t numa_rs;        // NodeNUMAResource reasons of the policy-None checks (before the policy path)
  int32_t traw, araw;      // TaintToleration / NodeAffinity raw scores (normalized in key_total)
};

// TaintToleration / NodeAffinity inputs of one pod over the context's dictionaries (ks_static_plugin_args), built by
// the host at staging; read wave-uniform (scalar loads) by the kernels of the FEAT & 4 variants.
struct __attribute__((aligned(16))) PodStat {
  uint64_t tol;                       // dictionary taints some toleration tolerates
  uint64_t req[KS_AFFINITY_TERMS];    // required terms (nodeSelector folded in); KS_LABEL_NEVER = an empty term
  uint64_t pref[KS_AFFINITY_TERMS];   // preferred terms
  int32_t w[KS_AFFINITY_TERMS];       // preferred weights (0 = unused)
  int32_t nreq;                       // required terms (0 = no required node affinity / selector)
  int32_t _pad;
  uint64_t pwant, pconf;              // NodePorts: the pod's host-port bits, the bits any of them conflicts with
};
static_assert(sizeof(PodStat) == 112, "PodStat layout");

__device__ __forceinline__ PodStat load_stat_uniform(const PodStat* p) {
  PodStat r;
#if defined(__HIP_DEVICE_COMPILE__)
  typedef const __attribute__((address_space(4))) int64_t* ConstWords;
  const ConstWords src = (ConstWords)p;
  int64_t* dst = reinterpret_cast<int64_t*>(&r);
#pragma unroll
  for (int i = 0; i < (int)(sizeof(PodStat) / 8); ++i) dst[i] = src[i];
#else
  r = *p;
#endif
  return r;
}

// Upstream TaintToleration and NodeAffinity (kube-scheduler v1.24.15, plugins/tainttoleration/taint_toleration.go and
// plugins/nodeaffinity/node_affinity.go; not on disk: parity unpinned, restated in oracle/static_plugins_ref.py) on
// the node's dictionary words: Filter -- an untolerated NoSchedule / NoExecute taint (FindMatchingUntoleratedTaint),
// no required term whose requirement bits the node has (RequiredNodeAffinity.Match); Score raw values -- untolerated
// PreferNoSchedule taints (countIntolerableTaintsPreferNoSchedule) and the weights of the matching preferred terms.
// Every node is evaluated the same way whatever other Filters said (reasons are OR-ed).
__device__ __forceinline__ void stat_eval(const Cfg& c, const PodStat& s, uint64_t hard, uint64_t soft, uint64_t labels,
                                          uint64_t ports, EvalOut& o) {
  if ((c.taint & 1) && (hard & ~s.tol)) o.reasons |= KS_R_TAINT;
  // upstream NodePorts Filter (plugins/nodeports/node_ports.go fitsPorts: UsedPorts.CheckConflict per wanted port)
  if ((c.ports & 1) && (ports & s.pconf)) o.reasons |= KS_R_NODE_PORTS;
  if ((c.aff & 1) && s.nreq > 0) {
    bool ok = false;
#pragma unroll
    for (int t = 0; t < KS_AFFINITY_TERMS; ++t) ok |= t < s.nreq && (labels & s.req[t]) == s.req[t];
    if (!ok) o.reasons |= KS_R_NODE_AFFINITY;
  }
  o.traw = (c.taint & 2) ? __builtin_popcountll(soft & ~s.tol) : 0;
  int32_t a = 0;
  if (c.aff & 2) {
#pragma unroll
    for (int t = 0; t < KS_AFFINITY_TERMS; ++t) a += (s.w[t] != 0 && (labels & s.pref[t]) == s.pref[t]) ? s.w[t] : 0;
  }
  o.araw = a;
}

// Normalization maxima of one pod: DeviceShare, TaintToleration, NodeAffinity (DefaultNormalizeScore over the feasible
// nodes, normalize_score.go:24-52)
struct NormM {
  int32_t dev, taint, aff;
};
constexpr int kNormRows = 3;  // rows of the per-pass maxima table (SweepArgs.dev_M)

// Upstream NodeResourcesBalancedAllocation (kube-scheduler v1.24 noderesources/balanced_allocation.go,
// balancedResourceScorer with useRequested = true): fraction = float64(Requested + pod request) / float64(Allocatable)
// for each listed resource with Allocatable != 0, capped at 1; std = |f0 - f1| / 2 for two fractions, 0 for fewer;
// score = int64((1 - std) * 100).  Plain f64 operations in Go's order (-ffp-contract=off: no fused multiply-add).
__device__ __forceinline__ int32_t balanced_score(int32_t res, int64_t acpu, int64_t rcpu, int64_t amem, int64_t rmem) {
  double f0 = 0.0, f1 = 0.0;
  int n = 0;
  if ((res & KS_BAL_CPU) && acpu != 0) {
    const double x = (double)rcpu / (double)acpu;
    f0 = x > 1.0 ? 1.0 : x;
    n = 1;
  }
  if ((res & KS_BAL_MEMORY) && amem != 0) {
    const double x = (double)rmem / (double)amem;
    if (n == 0) f0 = x > 1.0 ? 1.0 : x;
    else f1 = x > 1.0 ? 1.0 : x;
    ++n;
  }
  const double sd = n == 2 ? fabs((f0 - f1) / 2.0) : 0.0;
  return (int32_t)((1.0 - sd) * 100.0);
}

// Filter + Score of one (pod, node).  DEBUG=false computes feasibility (reasons != 0) and the
// total without branches on node data; DEBUG=true also fills every reason bit and the
// per-plugin scores (which it computes for infeasible nodes too; callers mask them).
template <int NSC, bool DEBUG>
__device__ __forceinline__ EvalOut eval_pod_node(const Cfg& c, const PodRec& p, const NodeReg<NSC>& r) {
  EvalOut o;
  uint32_t rs = 0;
  if (c.fit_filter) {
    if (DEBUG) {
      if (r.pods_full) rs |= KS_R_FIT_PODS;
      if (!(p.flags & kPodAllZero)) {
        if (p.cpu > r.free_cpu) rs |= KS_R_FIT_CPU;
        if (p.mem > r.free_mem) rs |= KS_R_FIT_MEMORY;
        if (p.eph > r.free_eph) rs |= KS_R_FIT_EPHEMERAL;
#pragma unroll
        for (int k = 0; k < NSC; ++k)
          if (p.sc[k] != 0 && p.sc[k] > r.free_sc[k]) rs |= KS_R_FIT_SCALAR;
      }
    } else {
      bool bad = r.pods_full != 0;
      if (!(p.flags & kPodAllZero)) {
        bad |= (p.cpu > r.free_cpu) | (p.mem > r.free_mem) | (p.eph > r.free_eph);
#pragma unroll
        for (int k = 0; k < NSC; ++k)
          if (p.sc[k] != 0) bad |= p.sc[k] > r.free_sc[k];
      }
      rs = bad ? KS_R_FIT_PODS : 0u;
    }
  } else {
    rs = r.valid ? 0u : KS_R_FIT_PODS;
  }
  if (c.la_filter && !(p.flags & KS_POD_DAEMONSET)) {
    const bool prod_path = (p.flags & KS_POD_PROD) != 0;
    const uint32_t failbit = prod_path ? kLaFailProd : kLaFailNonProd;
    if (DEBUG) {
      if (r.la_bits & failbit) rs |= (r.la_bits >> (prod_path ? kLaReasonProdShift : kLaReasonNonProdShift)) & 0x1ffu;
    } else {
      rs |= (r.la_bits & failbit) ? KS_R_LA_CPU : 0u;
    }
  }
  o.reasons = rs;
  o.fit = 0;
  o.la = 0;
  o.numa = 0;
  o.dev_raw = 0;
  o.traw = 0;
  o.araw = 0;
  o.hi = 0;
  o.numa_rs = 0;
  o.bal = 0;
  int32_t total = 0;
  // the score terms: the f64 path everywhere, then the int64 path for the lanes it does not cover
  // (a divergent branch the wave skips when no lane needs it)
  const bool exact64 = (r.la_bits & kNodeBigCap) || (p.flags & kPodBigReq);
  auto fit_score = [&](auto least, auto most) -> int32_t {
    int32_t ns = 0, ws = r.fit_ws;
    auto term = [&](int32_t w, const Term& t, int64_t pr, double prd) {
      if (w != 0) {
        const int32_t s = c.fit_most ? most(t, pr, prd) : least(t, pr, prd);
        ns += (w == 1) ? s : s * w;
      }
    };
    term(c.fw_cpu, r.t_cpu, p.nzcpu, p.h_nzcpu);
    term(c.fw_mem, r.t_mem, p.nzmem, p.h_nzmem);
    term(c.fw_eph, r.t_eph, p.eph, p.h_eph);
#pragma unroll
    for (int k = 0; k < NSC; ++k) {
      if (p.sc[k] != 0 && c.fw_sc[k] != 0) {  // scalar skipped when the pod does not request it
        term(c.fw_sc[k], r.t_sc[k], p.sc[k], p.h_sc[k]);
        ws += r.t_sc[k].c != 0 ? c.fw_sc[k] : 0;
      }
    }
    return ws > 0 ? small_div(ns, ws > 0 ? ws : 1) : 0;
  };
  const bool prod = (p.flags & KS_POD_PROD) && c.la_prod_usage;
  const Term& tc = prod ? r.t_plcpu : r.t_lcpu;
  const Term& tm = prod ? r.t_plmem : r.t_lmem;
  auto la_score = [&](auto least) -> int32_t {
    int32_t ns = 0;
    if (c.lw_cpu) ns += least(tc, p.est_cpu, p.h_est_cpu) * c.lw_cpu;
    if (c.lw_mem) ns += least(tm, p.est_mem, p.h_est_mem) * c.lw_mem;
    return small_div(ns, c.lw_cpu + c.lw_mem);
  };
  auto least_f = [](const Term& t, int64_t, double pd) { return term_least(t, pd); };
  auto most_f = [](const Term& t, int64_t, double pd) { return term_most(t, pd); };
  auto least_i = [](const Term& t, int64_t pv, double) { return term_least_i64(t, pv); };
  auto most_i = [](const Term& t, int64_t pv, double) { return term_most_i64(t, pv); };
  int32_t fit = 0, la = 0;
  if (c.fit_score) fit = fit_score(least_f, most_f);
  if (c.la_score) la = la_score(least_f);
  if (exact64) {
    if (c.fit_score) fit = fit_score(least_i, most_i);
    if (c.la_score) la = la_score(least_i);
  }
  if (c.fit_score) {
    o.fit = fit;
    total += o.fit * c.fit_pw;
  }
  if (c.la_score) {
    o.la = (r.la_bits & kLaZeroScore) ? 0 : la;
    total += o.la * c.la_pw;
  }
  if (c.bal) {
    // Requested + pod = Allocatable - (Allocatable - Requested) + pod request
    o.bal = balanced_score(c.bal, r.t_cpu.c, r.t_cpu.c - r.free_cpu + p.cpu, r.t_mem.c, r.t_mem.c - r.free_mem + p.mem);
    total += o.bal * c.bal_pw;
  }
  o.total = total;
  return o;
}

// NodeNUMAResource on a topology-policy-None node: filterAmplifiedCPUs (nodenumaresource/plugin.go:340-373),
// for a cpu-bind pod the CPU topology check (:296-301; the trial Allocate runs only for a required bind
// policy, :318-327), and scoreWithAmplifiedCPUs (scoring.go:98-114) with the resourceAllocationScorer over
// cpu / memory Requested (:206-242).  A cpu-bind pod's request is amplified on a node with ratio > 1
// (plugin.go:357-359 and getResourceOptions :503-506).
template <int NSC, bool DEBUG>
__device__ __forceinline__ void numa_eval(const Cfg& c, const PodRec& p, const NodeReg<NSC>& r, EvalOut& o) {
  if (p.flags & kPodReqZero) return;  // PreFilter skip
  bool bind = c.cpuset && (p.flags & KS_POD_CPU_BIND);
  uint32_t rs = 0;
  // requestCPUBind (util.go:105-122): a node CPU bind policy makes a whole-CPU pod cpu-bind
  const uint32_t label = c.cores ? cores_label(r.cpu_cores) : 0u;
  if (label && !bind && p.cpu > 0) {
    if (p.cpu % 1000 != 0) rs = KS_R_NUMA_INVALID_CPUS;
    else bind = true;
  }
  int64_t pc = p.cpu;
  double pcd = p.h_cpu;
  if (bind && (r.la_bits & kNumaAmp)) {
    pc = (int64_t)::ceil((double)p.cpu * r.numa_ratio);  // extension.Amplify
    pcd = (double)(pc * 100);
  }
  if (rs == 0 && p.cpu != 0) {
    if (r.la_bits & kNumaInvalid) {
      rs = KS_R_NUMA_INVALID_RATIO;
    } else if (r.la_bits & kNumaAmp) {
      const int64_t requested = r.t_ncpu.c - r.free_cpu;  // alloc - (alloc - Requested)
      const bool amp = requested >= r.numa_A && r.numa_A > 0;
      if (pc > r.free_cpu - (amp ? r.numa_off : 0)) rs = KS_R_NUMA_AMPLIFIED_CPU;
    }
  }
  if (bind && rs == 0 && r.cpu_free < 0) rs = KS_R_NUMA_INVALID_TOPOLOGY;
  if (c.cores && bind && rs == 0) {
    // the Filter's required policy: the node's, else the pod's required one (plugin.go:303-312); FullPCPUs needs
    // whole cores (:314-317); the trial Allocate keeps the cores the policy allows (resource_manager.go:322-335) --
    // only on a node without a NUMA topology policy (:318): on a policy node FilterByNUMANode's Allocate runs instead
    // (numa_policy_eval)
    const bool pol_node = c.numa_pol && (r.la_bits & kNumaPolNode);
    const bool preq = (p.flags & KS_POD_CPU_BIND) && (p.cpu_bind & KS_CPU_BIND_REQUIRED);
    const uint32_t ppol = p.cpu_bind & KS_CPU_BIND_POLICY_MASK;
    const uint32_t req = label ? label : (preq ? ppol : 0u);
    if (preq && ppol != req) {
      rs = KS_R_NUMA_BIND_CONFLICT;
    } else if (req) {
      const int32_t need = (int32_t)(p.cpu / 1000), cpc = max((int32_t)cores_cpc(r.cpu_cores), 1);
      if (req == KS_CPU_BIND_FULL_PCPUS) {
        if (need % cpc != 0) rs = KS_R_NUMA_SMT;
        else if (!pol_node && (int32_t)cores_full(r.cpu_cores) * cpc < need) rs = KS_R_NUMA_CPUSET;
      } else if (!pol_node && (int32_t)cores_any(r.cpu_cores) < need) {
        rs = KS_R_NUMA_CPUSET;
      }
    }
  }
  o.reasons |= DEBUG ? rs : (rs ? KS_R_FIT_PODS : 0u);
  o.numa_rs = rs;
  Term tc = r.t_ncpu;
  if (p.cpu == 0) term_take(tc, -r.numa_off, (double)(-r.numa_off * 100));  // a cpu-less pod scores the plain Requested
  int32_t ns = 0, ws = 0;
  if (c.nw_cpu && tc.c != 0) ws += c.nw_cpu;
  if (c.nw_mem && r.t_nmem.c != 0) ws += c.nw_mem;
  const bool exact64 = (r.la_bits & kNodeBigCap) || (p.flags & kPodBigReq) || pc >= kBigReq;
  if (c.nw_cpu && tc.c != 0) ns += (c.numa_most ? term_most(tc, pcd) : term_least(tc, pcd)) * c.nw_cpu;
  if (c.nw_mem && r.t_nmem.c != 0)
    ns += (c.numa_most ? term_most(r.t_nmem, p.h_mem) : term_least(r.t_nmem, p.h_mem)) * c.nw_mem;
  if (exact64) {
    ns = 0;
    if (c.nw_cpu && tc.c != 0) ns += (c.numa_most ? term_most_i64(tc, pc) : term_least_i64(tc, pc)) * c.nw_cpu;
    if (c.nw_mem && r.t_nmem.c != 0)
      ns += (c.numa_most ? term_most_i64(r.t_nmem, p.mem) : term_least_i64(r.t_nmem, p.mem)) * c.nw_mem;
  }
  o.numa = ws > 0 ? small_div(ns, ws) : 0;
  o.total += o.numa * c.numa_pw;
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

// DPP sum over the wave (the same exchange pattern as wave_max_u32: each step combines disjoint groups)
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
  v += dpp32<0xB1>(v);
  v += dpp32<0x4E>(v);
  v += dpp32<0x141>(v);
  v += dpp32<0x140>(v);
  return __builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16) + __builtin_amdgcn_readlane(v, 32) +
         __builtin_amdgcn_readlane(v, 48);
}

__device__ __forceinline__ uint64_t wave_or_u64(uint64_t v) {
  v |= dpp64<0xB1>(v);
  v |= dpp64<0x4E>(v);
  v |= dpp64<0x141>(v);
  v |= dpp64<0x140>(v);
  return readlane64(v, 0) | readlane64(v, 16) | readlane64(v, 32) | readlane64(v, 48);
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
