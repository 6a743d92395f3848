// ks_dev.h — DeviceShare (GPU + RDMA, joint allocation) on the device (pkg/scheduler/plugins/deviceshare).
//
// Per (pod, node): AutopilotAllocator.Prepare (GPUHandler.CalcDesiredRequestsAndCount after fillGPUTotalMem,
// devicehandler_gpu.go:40-98; DefaultDeviceHandler for RDMA, devicehandler_default.go:44-93), the Allocate
// feasibility (device_allocator.go:94-132: tryJointAllocate for [gpu, rdma] pods, then defaultAllocateDevices
// per remaining type, :392-462), and the node score AutopilotAllocator.score (:507-530: scoreNode per requested
// type, summed).  Reserve takes the minors the same Allocate picks and adds the request per instance to each
// (updateCacheUsed).
//
// Minors are bit masks.  defaultAllocateDevices' sort (sortDeviceResourcesByPreferredPCIe then
// sortDeviceResourcesByMinor: preferred switch first, score desc, minor asc; device_resources.go:187-220) is
// a repeated arg-max over the key (preferred << 12 | score << 4 | 15 - minor).  The topology walk of
// allocateByTopology (:210-253) runs over at most KS_MAX_PCIE switches (numbered per node in (socket, NUMA
// node, pcieID) order, so the stable sort of freeNodeDevicesInPCIe is "preferred first, then index order") and
// the NUMA-node groups of freeNodeDevicesInNode (numa_topology.go:185-240: |preferred switches| desc, preferred
// desc, node asc).
//
// NormalizeScore is DefaultNormalizeScore(100) over the feasible nodes (scoring.go:95-97): a cross-node max M.
// The sweep runs twice when DeviceShare is on — phase 0 reduces, per pod, the key (M << 32 | ~witness) where
// the witness is the lowest-index feasible node holding M; phase 1 scores with floor(100 * raw / M).  The
// commit kernel keeps M valid: the untouched nodes' maximum is still M while the witness is untouched, the
// touched nodes are re-scored, and a pass whose M would change is cut so the next pass re-sweeps from that pod.
#pragma once

#include "ks_device.h"

namespace ks {

constexpr int kGpus = KS_MAX_GPUS;
constexpr int kRdma = KS_MAX_RDMA;
constexpr int kPcie = KS_MAX_PCIE;
// int64 words per node: totals [0, 3*kGpus) GPU (q * kGpus + k), [kDevRdmaW, +kRdma) RDMA, then the packed
// topology (kDevTopoW: 4-bit switch of GPU k at bit 4k, of RDMA j at bit 32 + 4j, 0xF = none; kDevMetaW: NUMA
// node of switch p at bit 8p, socket at bit 8p + 4).  Used amounts cover the quantity words only.
constexpr int kDevRdmaW = 3 * kGpus;
constexpr int kDevQW = 3 * kGpus + kRdma;  // quantity words (totals and used)
constexpr int kDevTopoW = kDevQW;
constexpr int kDevMetaW = kDevQW + 1;
constexpr int kDevTW = kDevQW + 2;  // total-table words
static_assert(kDevQW == KS_DEV_WORDS, "the reservation device words (ks_reservation_cols.dev_*) are the quantity words");

// internal node flag (DevDev.flags): a reservation on the node holds devices -- DeviceShare then runs with the
// node's reservation restore state (ks_rsv.h dev_rsv_*)
constexpr uint32_t kDevRsvHeld = 0x100u;

struct DevDev {
  const uint32_t* flags;  // [npad] KS_DEV_* | kDevRsvHeld
  const int64_t* total;   // [kDevTW][npad]
  int64_t* used;          // [kDevQW][npad]  mutable (Reserve)
  int64_t npad;
};

// views of one node's devices: HBM columns or the commit kernel's LDS copy
struct DevGView {
  const DevDev& d;
  int64_t n;
  __device__ __forceinline__ bool present() const { return (gld(d.flags + n) & KS_DEV_PRESENT) != 0; }
  __device__ __forceinline__ bool held() const { return (gld(d.flags + n) & kDevRsvHeld) != 0; }
  __device__ __forceinline__ int64_t tot(int w) const { return gld(d.total + (int64_t)w * d.npad + n); }
  __device__ __forceinline__ int64_t ptot(int w) const { return tot(w); }  // (Prepare's unfiltered node device)
  __device__ __forceinline__ int64_t use(int w) const { return gld(d.used + (int64_t)w * d.npad + n); }
};

// LDS slot copies are word-major with this row stride (an odd multiple of 8 B: conflict-free lane = slot reads)
constexpr int kDevLdsStride = kMaxBatch + 1;

struct DevLView {
  const int64_t* t;  // word w at t[w * kDevLdsStride]  (kDevTW words)
  const int64_t* u;  // (kDevQW words)
  uint32_t fl;       // the node's flags
  __device__ __forceinline__ bool present() const { return (fl & KS_DEV_PRESENT) != 0; }
  __device__ __forceinline__ bool held() const { return (fl & kDevRsvHeld) != 0; }
  __device__ __forceinline__ int64_t tot(int w) const { return t[w * kDevLdsStride]; }
  __device__ __forceinline__ int64_t ptot(int w) const { return tot(w); }
  __device__ __forceinline__ int64_t use(int w) const { return u[w * kDevLdsStride]; }
};

// defaultAllocateDevices' minor sets from a reservation (deviceshare/reservation.go:201-240): preferred minors per
// type (0 = none: the preferred-PCIe order applies; non-empty they replace it, sortDeviceResourcesByMinor) and
// required minors (0xFF = every minor)
struct DevPick {
  uint32_t gpref, rpref, greq, rreq;
};
constexpr DevPick kNoPick{0u, 0u, 0xFFu, 0xFFu};

// The pod's request per instance and desired count per device type on one node.
struct GpuReq {
  int64_t core, mem, ratio;  // GPU per instance (core 0 without a gpu-core key)
  int64_t rdma;              // RDMA per instance
  int32_t desired, rdesired;
  bool has_core;
};

template <typename V>
__device__ __forceinline__ uint32_t dev_prepare(const PodRec& p, const V& v, GpuReq& g) {
  g = GpuReq{0, 0, 0, 0, 1, 1, (p.flags & KS_POD_GPU_CORE) != 0};
  if (p.flags & kPodGpuReq) {
    int64_t total_mem = -1;
#pragma unroll
    for (int k = kGpus - 1; k >= 0; --k) {  // the first healthy minor (all GPUs of a node are the same model)
      const int64_t tc = v.ptot(k), tm = v.ptot(kGpus + k), tr = v.ptot(2 * kGpus + k);
      if (tc || tm || tr) total_mem = tm;
    }
    if (total_mem < 0) return KS_R_DEV_NO_GPU;
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
    g.core = g.has_core ? core : 0;
    g.mem = mem;
    g.ratio = ratio;
  }
  if (p.rdma > 0) {
    bool any = false;
#pragma unroll
    for (int j = 0; j < kRdma; ++j) any |= v.ptot(kDevRdmaW + j) != 0;
    if (!any) return KS_R_DEV_NO_RDMA;
    int64_t q = p.rdma;
    if (q > 100 && q % 100 == 0) {
      g.rdesired = (int32_t)(q / 100);
      q /= g.rdesired;
    }
    g.rdma = q;
  }
  return 0u;
}

// one resource of the scorer: Least/MostAllocated of (requested, capacity) (scoring.go:270-308)
__device__ __forceinline__ int32_t dev_term(bool most, int64_t req, int64_t cap) {
  if (most) return pct_floor_i64(req > cap ? cap : req, cap);
  return req > cap ? 0 : pct_floor_i64(cap - req, cap);
}

// scoreDevice / scoreNode body for GPUs: requested = total - free + pod (total >= free), allocatable = total
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

// the same for RDMA (one resource, koordinator.sh/rdma)
__device__ __forceinline__ int32_t dev_score1(const Cfg& c, int64_t tot, int64_t fre, int64_t pod) {
  if (c.dw_rdma == 0 || tot == 0) return 0;
  const int64_t req = tot >= fre ? tot - fre + pod : tot;
  return dev_term(c.dev_most != 0, req, tot);  // (s * w) / w
}

struct DevOut {
  uint32_t reasons;  // KS_R_DEV_*
  int32_t raw;       // AutopilotAllocator.score (feasible only)
  uint32_t minors;   // GPU allocation (ALLOC only)
  uint32_t rminors;  // RDMA allocation (ALLOC only)
};

// per-type state of one node for one pod, packed to keep the sweep's register footprint small
struct DevType {
  uint32_t fit;  // minors with non-zero free that satisfy the request per instance
  uint32_t pcw;  // 4-bit switch of each minor (0xF = none)
  uint64_t sc;   // 8-bit scoreDevice of each minor (only with scores; <= 100)
  __device__ __forceinline__ uint32_t pcie(int k) const { return (pcw >> (4 * k)) & 0xFu; }
  __device__ __forceinline__ int score(int k) const { return (int)((sc >> (8 * k)) & 0xFFu); }
};

// defaultAllocateDevices over the fitting minors in `sub` and the required set `rq`: up to maxd minors in (preferred,
// score desc, minor asc) order -- preferred = the minor in `pm` when pm != 0, else its switch in `pref` --, at least
// `desired`; 0 = "Insufficient <type> devices"
__device__ __forceinline__ uint32_t dev_take(const DevType& t, int nm, uint32_t sub, int desired, uint32_t pref,
                                             uint32_t pm = 0u, uint32_t rq = 0xFFu) {
  int maxd = desired;
  const int npref = __builtin_popcount(pref);
  maxd = npref > maxd ? npref : maxd;
  desired = desired == 0 ? 1 : desired;
  maxd = maxd < desired ? desired : maxd;
  const uint32_t cand = t.fit & sub & rq;
  uint32_t mask = 0;
  int got = 0;
  for (int r = 0; r < maxd; ++r) {
    int best = -1, bk = -1;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (k >= nm) break;
      const bool ok = ((cand >> k) & 1u) && !((mask >> k) & 1u);
      const uint32_t pc = t.pcie(k);
      const bool pr = pm ? ((pm >> k) & 1u) != 0 : (pc < 8u && ((pref >> pc) & 1u));
      const int key = (pr ? (1 << 12) : 0) | (t.score(k) << 4) | (15 - k);
      best = (ok && key > bk) ? k : best;
      bk = (ok && key > bk) ? key : bk;
    }
    if (best < 0) break;
    mask |= 1u << best;
    ++got;
  }
  return got >= desired ? mask : 0u;
}

__device__ __forceinline__ uint32_t dev_pcies_of(const DevType& t, int nm, uint32_t mask) {
  uint32_t p = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k)
    if (k < nm && ((mask >> k) & 1u) && t.pcie(k) < 8u) p |= 1u << t.pcie(k);
  return p;
}

__device__ __forceinline__ uint32_t dev_sub_of(const DevType& t, int nm, uint32_t pcies) {
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k)
    if (k < nm && t.pcie(k) < 8u && ((pcies >> t.pcie(k)) & 1u)) s |= 1u << k;
  return s;
}

// jointAllocate (device_allocator.go:286-339) restricted to the switches `sw` (all minors if sw == ~0)
__device__ __forceinline__ bool dev_joint(const DevType& G, const DevType& R, const GpuReq& g, bool same, uint32_t sw,
                                          uint32_t pref, uint32_t& om, uint32_t& orm, const DevPick& pk = kNoPick) {
  const uint32_t gs = sw == ~0u ? 0xFFu : dev_sub_of(G, kGpus, sw);
  const uint32_t rs = sw == ~0u ? 0xFFu : dev_sub_of(R, kRdma, sw);
  const uint32_t prim = dev_take(G, kGpus, gs, g.desired, pref, pk.gpref, pk.greq);
  if (!prim) return false;
  const uint32_t pc = dev_pcies_of(G, kGpus, prim);
  const uint32_t sec = dev_take(R, kRdma, rs, same ? __builtin_popcount(pc) : 1, pc, pk.rpref, pk.rreq);
  if (!sec) return false;
  om = prim;
  orm = sec;
  return true;
}

// tryJointAllocate -> allocateByTopology with DeviceTypes [gpu, rdma] (device_allocator.go:188-253).  rpref: the pod
// requests RDMA -- only then is a switch or a NUMA-node group `preferred` (newDeviceTopologyGuide splits the free devices
// per requested type, numa_topology.go:109-135; a joint pod without an RDMA request has no RDMA entry there)
__device__ __forceinline__ bool dev_by_topology(const DevType& G, const DevType& R, const GpuReq& g, bool same,
                                                uint64_t meta, uint32_t& om, uint32_t& orm, bool rpref = true,
                                                const DevPick& pk = kNoPick) {
  uint32_t exist = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    exist |= G.pcie(k) < 8u ? (1u << G.pcie(k)) : 0u;
    exist |= R.pcie(k) < 8u ? (1u << R.pcie(k)) : 0u;
  }
  // per switch: preferred = a fitting RDMA instance on it (freeDevices[rdma] of the last joint type)
  uint32_t swpref = 0;
#pragma unroll
  for (int p = 0; p < kPcie; ++p)
    if (rpref && ((exist >> p) & 1u) && (R.fit & dev_sub_of(R, kRdma, 1u << p))) swpref |= 1u << p;
  // freeNodeDevicesInPCIe: preferred switches first (with an RDMA request a switch without a fitting RDMA device fails
  // jointAllocate, so only those are tried); without one no switch is preferred and every switch is tried in
  // (socket, node, pcie) = index order
  const uint32_t tryset = rpref ? swpref : exist;
  for (int p = 0; p < kPcie; ++p) {
    if (!((tryset >> p) & 1u)) continue;
    if (__builtin_popcount(G.fit & dev_sub_of(G, kGpus, 1u << p)) >= g.desired &&
        dev_joint(G, R, g, same, 1u << p, 1u << p, om, orm, pk))
      return true;
  }
  // freeNodeDevicesInNode: one group per NUMA node, ordered by (|preferred switches| desc, preferred desc,
  // node asc)
  uint32_t gsw[kPcie], gkey[kPcie];
  int ng = 0;
  uint32_t seen = 0;
  for (int p = 0; p < kPcie; ++p) {
    if (!((exist >> p) & 1u)) continue;
    const uint32_t node = (uint32_t)(meta >> (8 * p)) & 0xFu;
    if ((seen >> node) & 1u) continue;
    seen |= 1u << node;
    uint32_t sw = 0;
    for (int q = p; q < kPcie; ++q)
      if (((exist >> q) & 1u) && ((uint32_t)(meta >> (8 * q)) & 0xFu) == node) sw |= 1u << q;
    const bool pr = rpref && (R.fit & dev_sub_of(R, kRdma, sw)) != 0;
    gsw[ng] = sw;
    gkey[ng] = ((uint32_t)__builtin_popcount(sw & swpref) << 8) | (pr ? 16u : 0u) | (15u - node);
    ++ng;
  }
  uint32_t done = 0;
  for (int r = 0; r < ng; ++r) {
    int bi = -1;
    uint32_t bk = 0;
    for (int i = 0; i < ng; ++i)
      if (!((done >> i) & 1u) && (bi < 0 || gkey[i] > bk)) {
        bi = i;
        bk = gkey[i];
      }
    done |= 1u << bi;
    const uint32_t sw = gsw[bi];
    if (__builtin_popcount(G.fit & dev_sub_of(G, kGpus, sw)) >= g.desired &&
        dev_joint(G, R, g, same, sw, sw & swpref, om, orm, pk))
      return true;
  }
  // the whole node, preferring every preferred switch
  return dev_joint(G, R, g, same, ~0u, swpref, om, orm, pk);
}

// The minors of each type on the NUMA nodes of `allow` (a bit per NUMA node id; ~0u = every minor): with a
// topology-manager affinity, filterNodeDevice keeps only devices with a topology on an allowed NUMA node
// (device_allocator.go:134-158).
template <typename V>
__device__ __forceinline__ void dev_allowed(const V& v, uint32_t allow, uint32_t& gin, uint32_t& rin) {
  gin = 0xFFu;
  rin = 0xFFu;
  if (allow == ~0u) return;
  const uint64_t topo = (uint64_t)v.tot(kDevTopoW), meta = (uint64_t)v.tot(kDevMetaW);
  gin = rin = 0u;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint32_t pg = (uint32_t)(topo >> (4 * k)) & 0xFu, pr = (uint32_t)(topo >> (32 + 4 * k)) & 0xFu;
    gin |= (pg < 8u && ((allow >> ((uint32_t)(meta >> (8 * pg)) & 0xFu)) & 1u)) ? (1u << k) : 0u;
    rin |= (pr < 8u && ((allow >> ((uint32_t)(meta >> (8 * pr)) & 0xFu)) & 1u)) ? (1u << k) : 0u;
  }
}

// DeviceShare Filter + Score (+ the allocation with ALLOC) of one (pod, node); allow restricts the devices to a
// NUMA affinity (dev_allowed).
template <bool ALLOC, typename V>
__device__ __forceinline__ DevOut dev_eval(const Cfg& c, const PodRec& p, const V& v, GpuReq* req_out = nullptr,
                                           uint32_t allow = ~0u, const DevPick& pk = kNoPick) {
  DevOut o{0u, 0, 0u, 0u};
  if (!v.present()) return o;  // no device info: Filter passes, Score 0
  GpuReq g;
  o.reasons = dev_prepare(p, v, g);
  if (req_out) *req_out = g;
  if (o.reasons) return o;
  const bool has_gpu = (p.flags & kPodGpuReq) != 0, has_rdma = p.rdma > 0;
  // jointAllocate's secondary type without an RDMA request (device_allocator.go:308-330): allocateDevices with a nil
  // request per instance -- every RDMA device with non-zero free fits, none is used up, none scores the node
  const bool jr = has_gpu && !has_rdma && p.joint != KS_JOINT_NONE;
  const bool joint = has_gpu && (has_rdma || jr) && p.joint != KS_JOINT_NONE;
  const bool same = p.joint == KS_JOINT_GPU_RDMA_SAME_PCIE;
  // A best-effort joint pod asking for one RDMA device (or none) is feasible iff the per-type counts are: a joint
  // success takes >= desired GPUs and one RDMA device, a joint failure falls back to allocateDevices.  Only
  // the allocation itself (Reserve) needs the walk then.
  const bool walk = joint && (ALLOC || same || g.rdesired > 1);
  // only Reserve's allocator has a scorer (deviceshare/plugin.go:404); Filter's walk sorts minors with score 0
  const bool scores = ALLOC;
  uint32_t gin, rin;
  dev_allowed(v, allow, gin, rin);
  const uint64_t topo = (walk || ALLOC) ? (uint64_t)v.tot(kDevTopoW) : 0ull;
  DevType G, R;
  G.fit = R.fit = 0;
  G.sc = R.sc = 0;
  G.pcw = (uint32_t)topo;
  R.pcw = (uint32_t)(topo >> 32);
  int32_t raw = 0;
  if (has_gpu) {
    const int64_t pod[3] = {g.core, g.mem, g.ratio};
    int64_t tsum[3] = {0, 0, 0}, fsum[3] = {0, 0, 0};
#pragma unroll
    for (int k = 0; k < kGpus; ++k) {
      const int64_t t[3] = {v.tot(k), v.tot(kGpus + k), v.tot(2 * kGpus + k)};
      const int64_t u[3] = {v.use(k), v.use(kGpus + k), v.use(2 * kGpus + k)};
      const int64_t f[3] = {t[0] > u[0] ? t[0] - u[0] : 0, t[1] > u[1] ? t[1] - u[1] : 0, t[2] > u[2] ? t[2] - u[2] : 0};
      const bool exists = (t[0] || t[1] || t[2]) && ((gin >> k) & 1u);
      const bool has_free = exists && (f[0] || f[1] || f[2]);
      const bool fits = has_free && (!g.has_core || g.core <= f[0]) && g.mem <= f[1] && g.ratio <= f[2];
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        tsum[q] += exists ? t[q] : 0;
        fsum[q] += exists ? f[q] : 0;
      }
      G.fit |= fits ? (1u << k) : 0u;
      if (scores && fits) G.sc |= (uint64_t)dev_score3(c, t, f, pod) << (8 * k);
    }
    raw += dev_score3(c, tsum, fsum, pod);
  }
  if (has_rdma || (jr && walk)) {
    int64_t tsum = 0, fsum = 0;
#pragma unroll
    for (int j = 0; j < kRdma; ++j) {
      const bool in = ((rin >> j) & 1u) != 0;
      const int64_t t = in ? v.tot(kDevRdmaW + j) : 0, u = in ? v.use(kDevRdmaW + j) : 0;
      const int64_t f = t > u ? t - u : 0;
      tsum += t;
      fsum += f;
      const bool fits = t != 0 && f != 0 && g.rdma <= f;  // (g.rdma == 0 without a request)
      R.fit |= fits ? (1u << j) : 0u;
      if (scores && fits) R.sc |= (uint64_t)dev_score1(c, t, f, g.rdma) << (8 * j);
    }
    if (has_rdma) raw += dev_score1(c, tsum, fsum, g.rdma);
  }
  uint32_t om = 0, orm = 0;
  bool jdone = false;
  if (walk) {
    if (dev_by_topology(G, R, g, same, (uint64_t)v.tot(kDevMetaW), om, orm, has_rdma, pk)) {
      // validateJointAllocation (device_allocator.go:255-284)
      if (same && dev_pcies_of(G, kGpus, om) != dev_pcies_of(R, kRdma, orm)) {
        o.reasons = KS_R_DEV_JOINT;
        return o;
      }
      jdone = true;
    } else if (same) {
      o.reasons = KS_R_DEV_JOINT;
      return o;
    }
  }
  if (!jdone) {
    // allocateDevices per remaining type: feasibility is a count; the minors only with ALLOC
    if ((has_gpu && __builtin_popcount(G.fit & pk.greq) < g.desired) ||
        (has_rdma && __builtin_popcount(R.fit & pk.rreq) < g.rdesired)) {
      o.reasons = KS_R_DEV_INSUFFICIENT;
      return o;
    }
    if (ALLOC) {
      om = has_gpu ? dev_take(G, kGpus, 0xFFu, g.desired, 0u, pk.gpref, pk.greq) : 0u;
      orm = has_rdma ? dev_take(R, kRdma, 0xFFu, g.rdesired, 0u, pk.rpref, pk.rreq) : 0u;
    }
  }
  o.raw = raw;
  if (ALLOC) {
    o.minors = om;
    o.rminors = orm;
  }
  return o;
}

// AutopilotAllocator.score alone (device_allocator.go:507-530): scoreNode per requested type over the view; a type
// whose devices all have zero free is left out of the filtered node device (nodeDevice.filter, device_cache.go:351-353)
template <typename V>
__device__ __forceinline__ int32_t dev_raw(const Cfg& c, const PodRec& p, const V& v, const GpuReq& g) {
  int32_t raw = 0;
  if (p.flags & kPodGpuReq) {
    const int64_t pod[3] = {g.core, g.mem, g.ratio};
    int64_t tsum[3] = {0, 0, 0}, fsum[3] = {0, 0, 0};
    bool anyf = false;
    for (int k = 0; k < kGpus; ++k) {
      const int64_t t[3] = {v.tot(k), v.tot(kGpus + k), v.tot(2 * kGpus + k)};
      const int64_t u[3] = {v.use(k), v.use(kGpus + k), v.use(2 * kGpus + k)};
      const bool exists = t[0] || t[1] || t[2];
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int64_t f = t[q] > u[q] ? t[q] - u[q] : 0;
        tsum[q] += exists ? t[q] : 0;
        fsum[q] += exists ? f : 0;
        anyf |= exists && f != 0;
      }
    }
    if (anyf) raw += dev_score3(c, tsum, fsum, pod);
  }
  if (p.rdma > 0) {
    int64_t tsum = 0, fsum = 0;
    for (int j = 0; j < kRdma; ++j) {
      const int64_t t = v.tot(kDevRdmaW + j), u = v.use(kDevRdmaW + j);
      tsum += t;
      fsum += t > u ? t - u : 0;
    }
    if (fsum) raw += dev_score1(c, tsum, fsum, g.rdma);
  }
  return raw;
}

// DeviceShare's Filter under several NUMA restrictions (generateTopologyHints' trial allocations): the per-minor
// fits and scores do not depend on the restriction, so they are computed once; under a restriction the fit sets
// are masked to its minors and dev_eval's feasibility logic runs on them.  dev_fits_ok(f, gin, rin) ==
// (dev_eval<false>(c, p, v, nullptr, allow).reasons == 0) for dev_allowed(v, allow) = (gin, rin).
struct DevFits {
  DevType G, R;
  GpuReq g;
  uint64_t meta;
  bool walk, same, has_gpu, has_rdma, jr;
};

template <typename V>
__device__ __forceinline__ DevFits dev_fits(const Cfg& c, const PodRec& p, const V& v, const GpuReq& g) {
  DevFits f;
  f.g = g;
  f.has_gpu = (p.flags & kPodGpuReq) != 0;
  f.has_rdma = p.rdma > 0;
  f.jr = f.has_gpu && !f.has_rdma && p.joint != KS_JOINT_NONE;  // (dev_eval: joint without an RDMA request)
  const bool joint = f.has_gpu && (f.has_rdma || f.jr) && p.joint != KS_JOINT_NONE;
  f.same = p.joint == KS_JOINT_GPU_RDMA_SAME_PCIE;
  f.walk = joint && (f.same || g.rdesired > 1);
  const uint64_t topo = (uint64_t)v.tot(kDevTopoW);
  f.meta = (uint64_t)v.tot(kDevMetaW);
  f.G.fit = f.R.fit = 0;
  f.G.sc = f.R.sc = 0;
  f.G.pcw = (uint32_t)topo;
  f.R.pcw = (uint32_t)(topo >> 32);
  if (f.has_gpu) {
#pragma unroll
    for (int k = 0; k < kGpus; ++k) {
      const int64_t t[3] = {v.tot(k), v.tot(kGpus + k), v.tot(2 * kGpus + k)};
      const int64_t u[3] = {v.use(k), v.use(kGpus + k), v.use(2 * kGpus + k)};
      const int64_t fr[3] = {t[0] > u[0] ? t[0] - u[0] : 0, t[1] > u[1] ? t[1] - u[1] : 0, t[2] > u[2] ? t[2] - u[2] : 0};
      const bool exists = t[0] || t[1] || t[2];
      const bool fits = exists && (fr[0] || fr[1] || fr[2]) && (!g.has_core || g.core <= fr[0]) && g.mem <= fr[1] &&
                        g.ratio <= fr[2];
      f.G.fit |= fits ? (1u << k) : 0u;  // (the hints' trial allocator has no scorer: every minor scores 0)
    }
  }
  if (f.has_rdma || (f.jr && f.walk)) {
#pragma unroll
    for (int j = 0; j < kRdma; ++j) {
      const int64_t t = v.tot(kDevRdmaW + j), u = v.use(kDevRdmaW + j);
      const int64_t fr = t > u ? t - u : 0;
      const bool fits = t != 0 && fr != 0 && g.rdma <= fr;
      f.R.fit |= fits ? (1u << j) : 0u;
    }
  }
  return f;
}

__device__ __forceinline__ uint64_t dev_byte_mask(uint32_t bits) {
  uint64_t m = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) m |= ((bits >> k) & 1u) ? (0xFFull << (8 * k)) : 0ull;
  return m;
}

__device__ __forceinline__ bool dev_fits_ok(const DevFits& f, uint32_t gin, uint32_t rin) {
  DevType G = f.G, R = f.R;
  G.fit &= gin;
  R.fit &= rin;
  G.sc &= dev_byte_mask(G.fit);
  R.sc &= dev_byte_mask(R.fit);
  if (f.walk) {
    uint32_t om = 0, orm = 0;
    if (dev_by_topology(G, R, f.g, f.same, f.meta, om, orm, f.has_rdma))
      return !(f.same && dev_pcies_of(G, kGpus, om) != dev_pcies_of(R, kRdma, orm));
    if (f.same) return false;
  }
  return !((f.has_gpu && __builtin_popcount(G.fit) < f.g.desired) || (f.has_rdma && __builtin_popcount(R.fit) < f.g.rdesired));
}

}  // namespace ks
