// ks_rsv.h — Reservation plugin on the device (pkg/scheduler/plugins/reservation).
//
// Node columns hold the "base" NodeInfo: the reference's NodeInfo (reserve pods included) with
// every eligible reservation that has assigned pods already replaced by its remainder, i.e. the
// restoreUnmatchedReservations step (transformer.go:266-307) applied as if no reservation matched
// the pod.  That part is pod-independent.  For a (pod, node) pair whose pod class matches some of
// the node's reservations, rsv_eval turns the base into the pod's restored NodeInfo
// (restoreMatchedReservation :241-264 for the matched ones, undoing their unmatched step), and
// derives nodeRState.podRequested / rAllocated for fitsNode (plugin.go:445-496), the Reservation
// Filter (:311-440), the nomination (nominator.go:134-192, FilterReservation plugin.go:503-530)
// and scoreReservation (scoring.go:183-203).
//
// Score ranking.  Reservation's Score is 1000 on the PreScore-preferred node (lowest order label
// among feasible nodes, scoring.go:87-96), the nominated reservation's score elsewhere, then
// DefaultNormalizeScore(100) and weight w (5000).  With w > 100 * (Fit + LoadAware weights) the
// weighted totals order nodes exactly by (hi, Fit+LoadAware total, lowest index) where
// hi = 101 + rank of the node's best order label (larger for smaller labels) when it has an ordered
// matched reservation, else the raw score (0..100): the preferred node scores 100*w and every other
// node at most 10*w + (Fit+LA), and without a preferred node floor(100*raw/max) is strictly
// increasing in raw for max <= 100.  So the key total is hi * F + (Fit+LA) with F = max(Fit+LA)+1,
// which depends on the node alone: untouched nodes keep their snapshot keys under commits exactly
// as for the other plugins.  Ordered nodes drop the Fit+LA part (hi * F alone): among equal order
// labels the preferred node is the lowest index (scoring.go:87-96), not the best Fit+LA.  The
// chosen node's reference total is (Fit+LA) + 100*w when hi > 0 (it holds the maximum raw score or
// is the preferred node) and (Fit+LA) otherwise.
#pragma once

#include <type_traits>

#include "ks_device.h"
#include "ks_numa.h"

namespace ks {

constexpr int kRsvDims = KS_RSV_DIMS;
constexpr int64_t kDefaultMilliCPU = 100;                 // schedutil.DefaultMilliCPURequest
constexpr int64_t kDefaultMemory = 200ll * 1024 * 1024;   // schedutil.DefaultMemoryRequest
constexpr int32_t kRsvOrderBase = 101;                    // hi of an ordered node > any raw score

// meta word: flags (KS_RSV_*) | policy << 4 | key_mask << 8 | ndims << 16 | kRsvMetaDev
constexpr uint32_t kRsvMetaDev = 1u << 20;  // the reservation holds devices (DevRsv.dal row non-zero)
__device__ __forceinline__ uint32_t rsv_policy(uint32_t m) { return (m >> 4) & 0xfu; }
__device__ __forceinline__ uint32_t rsv_keys(uint32_t m) { return (m >> 8) & 0xffu; }

// Reservation table in CSR order (rows of node n at [beg[n], beg[n+1]), table order within a node).
struct DevRsv {
  const int32_t* beg;     // [npad + 1]
  const uint64_t* cls;    // owner classes
  const uint32_t* meta;
  const int32_t* ohi;     // kRsvOrderBase + (#distinct orders - 1 - rank of the order label); 0 = none
  const int64_t* alloc;   // [kRsvDims][nr]
  int64_t* allocd;        // [kRsvDims][nr]  mutable (Reserve)
  int32_t* assigned;      // [nr]            mutable (Reserve)
  const int64_t* rnz;     // [2][nr] reserve pod NonZeroRequested cpu / memory
  uint64_t* ncls;         // = DevNodes.rsv_cls
  const int32_t* rowid;   // CSR position -> caller row
  // DeviceShare (deviceshare/reservation.go): the reserve pod's device allocation and its assigned pods' allocations
  // on those minors, [kDevQW][nr] (ks_dev.h word layout); NULL when no reservation holds a device
  const int64_t* dal;
  int64_t* dald;          // mutable (Reserve)
  const uint32_t* dmask;  // [nr] bit w: dal word w is non-zero (a device word the reservation holds)
  int64_t nr;
  int64_t w100;           // 100 * plugin weight
};

// Mutable reservation fields read inside the commit kernel go around the CU's L1 (agent-scope
// relaxed loads = global_load sc1): the same wave wrote them a few pods earlier.
template <bool FRESH, typename T>
__device__ __forceinline__ T rld(const T* p) {
  if (FRESH) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return gld(p);
}

__device__ __forceinline__ int64_t pod_dim(const PodRec& p, int d) {
  return d == 0 ? p.cpu : d == 1 ? p.mem : d == 2 ? p.eph : p.sc[d - 3];
}

__device__ __forceinline__ int32_t pct_floor(int64_t req, int64_t cap) { return pct_floor_i64(req, cap); }

// Per-(pod, node) restore deltas relative to the base NodeInfo.
template <int NSC>
struct RsvDelta {
  int64_t dreq[3 + NSC];  // Requested (cpu, memory, ephemeral, scalars)
  int64_t dnz[2];         // NonZeroRequested
  int32_t nm;             // len(matched)
};

struct RsvOut {
  uint32_t reasons;  // KS_R_RSV_*
  int32_t hi;        // ranking key component (see header)
  int32_t raw;       // scoreReservation of the nominated reservation (0 = none)
  int32_t hiord;     // kRsvOrderBase+... of the node's best order label over matched (0 = none)
  int32_t nom;       // nominated reservation, CSR position (-1 = none)
  int32_t dds;       // 1 + DeviceShare's ScoreReservation of the nominated reservation when its FilterReservation
                     // nominated it (a reservation holding devices the pod allocates from), else 0
};

// ---- views of one node's reservations ----
// RsvG: the CSR table in HBM (FRESH: the mutable fields around the CU's L1).
// RsvL: the commit kernel's LDS copy of a touched node's reservations (D = 3 + NSC dims kept; a node
// whose reservations use a dimension beyond D stays on RsvG).  Index i runs over [0, n()).
template <bool FRESH>
struct RsvG {
  const DevRsv& rv;
  int64_t b, e;
  __device__ __forceinline__ RsvG(const DevRsv& r, int64_t node) : rv(r), b(gld(r.beg + node)), e(gld(r.beg + node + 1)) {}
  __device__ __forceinline__ int64_t n() const { return e - b; }
  __device__ __forceinline__ uint32_t meta(int64_t i) const { return gld(rv.meta + b + i); }
  __device__ __forceinline__ int32_t assigned(int64_t i) const { return rld<FRESH>(rv.assigned + b + i); }
  __device__ __forceinline__ uint64_t cls(int64_t i) const { return gld(rv.cls + b + i); }
  __device__ __forceinline__ int32_t ohi(int64_t i) const { return gld(rv.ohi + b + i); }
  __device__ __forceinline__ int64_t alloc(int d, int64_t i) const { return gld(rv.alloc + d * rv.nr + b + i); }
  __device__ __forceinline__ int64_t allocd(int d, int64_t i) const { return rld<FRESH>(rv.allocd + d * rv.nr + b + i); }
  __device__ __forceinline__ int64_t rnz(int k, int64_t i) const { return gld(rv.rnz + k * rv.nr + b + i); }
  __device__ __forceinline__ int32_t csr(int64_t i) const { return (int32_t)(b + i); }
  __device__ __forceinline__ int64_t dal(int w, int64_t i) const { return gld(rv.dal + (int64_t)w * rv.nr + b + i); }
  __device__ __forceinline__ uint32_t dmask(int64_t i) const { return gld(rv.dmask + b + i); }
  __device__ __forceinline__ int64_t dald(int w, int64_t i) const { return rld<FRESH>(rv.dald + (int64_t)w * rv.nr + b + i); }
};

template <int D>
struct __attribute__((aligned(8))) RsvRec {
  uint64_t cls;
  uint32_t meta;
  int32_t ohi;
  int32_t assigned, _pad;
  int64_t alloc[D], allocd[D], rnz[2];
};

template <int D>
struct RsvL {
  const RsvRec<D>* rec;
  int32_t cnt, b;
  const DevRsv* rvp;  // the device allocations stay in HBM
  __device__ __forceinline__ int64_t n() const { return cnt; }
  __device__ __forceinline__ uint32_t meta(int64_t i) const { return rec[i].meta; }
  __device__ __forceinline__ int32_t assigned(int64_t i) const { return rec[i].assigned; }
  __device__ __forceinline__ uint64_t cls(int64_t i) const { return rec[i].cls; }
  __device__ __forceinline__ int32_t ohi(int64_t i) const { return rec[i].ohi; }
  __device__ __forceinline__ int64_t alloc(int d, int64_t i) const { return d < D ? rec[i].alloc[d] : 0; }
  __device__ __forceinline__ int64_t allocd(int d, int64_t i) const { return d < D ? rec[i].allocd[d] : 0; }
  __device__ __forceinline__ int64_t rnz(int k, int64_t i) const { return rec[i].rnz[k]; }
  __device__ __forceinline__ int32_t csr(int64_t i) const { return b + (int32_t)i; }
  __device__ __forceinline__ int64_t dal(int w, int64_t i) const { return gld(rvp->dal + (int64_t)w * rvp->nr + b + i); }
  __device__ __forceinline__ uint32_t dmask(int64_t i) const { return gld(rvp->dmask + b + i); }
  __device__ __forceinline__ int64_t dald(int w, int64_t i) const {
    return rld<true>(rvp->dald + (int64_t)w * rvp->nr + b + i);
  }
};

// meta bits 16..19: 1 + the highest dimension with a non-zero allocatable / allocated (0 = none)
__device__ __forceinline__ int32_t rsv_ndims(uint32_t m) { return (int32_t)((m >> 16) & 0xfu); }

template <typename V>
__device__ __forceinline__ bool rsv_matches(const V& v, int64_t i, int32_t cls, uint32_t& meta, int32_t& a) {
  meta = v.meta(i);
  a = v.assigned(i);
  const bool eligible = !((meta & KS_RSV_ALLOCATE_ONCE) && a > 0);  // transformer.go:109
  return eligible && !(meta & KS_RSV_UNSCHEDULABLE) && ((v.cls(i) >> cls) & 1ull);
}

// scoreReservation (scoring.go:183-203): MostAllocated over the non-zero allocatable dims
template <typename V>
__device__ __forceinline__ int32_t rsv_score(const V& v, const PodRec& p, int64_t i) {
  int32_t s = 0, w = 0;
#pragma unroll
  for (int d = 0; d < kRsvDims; ++d) {
    const int64_t al = v.alloc(d, i);
    if (al == 0) continue;
    ++w;
    const int64_t req = pod_dim(p, d) + v.allocd(d, i);
    if (req <= al) s += pct_floor(req, al);
  }
  return w ? s / w : 0;
}

// ---- DeviceShare with reservations holding devices (deviceshare/reservation.go) ----
// RestoreReservation (:118-171) keeps the transformer's matched reservations that hold devices (allocatable = the
// reserve pod's allocation, allocated = its assigned pods' on those minors, remained = allocatable - allocated) and the
// unmatched ones with assigned pods; the allocator then sees used' = max(0, used - preemptible) (calcFreeWithPreemptible)
// with preemptible = mergedUnmatchedUsed + mergedMatchedAllocatable (the node outside any reservation's preference) or
// mergedUnmatchedUsed + mergedMatchedAllocated + remained(r) (allocating from reservation r).  The node columns hold
// nodeDeviceCache's used (reserve pods and assigned pods both counted); the views below subtract the per-pod part.
constexpr int kDrsFallback = 0, kDrsTry = 1;

// a reservation the pod's restore treats as matched and holding devices
template <typename V>
__device__ __forceinline__ bool rsv_dev_matched(const V& v, int64_t i, int32_t cls) {
  uint32_t meta;
  int32_t a;
  return cls >= 0 && cls < 64 && rsv_matches(v, i, cls, meta, a) && (meta & kRsvMetaDev);
}

// the reservation's minors of each type (newDeviceMinorMap(allocatable))
template <typename V>
__device__ __forceinline__ void rsv_dev_minors(const V& v, int64_t i, uint32_t& gm, uint32_t& rm) {
  gm = rm = 0u;
  for (int k = 0; k < kGpus; ++k)
    gm |= (v.dal(k, i) | v.dal(kGpus + k, i) | v.dal(2 * kGpus + k, i)) != 0 ? (1u << k) : 0u;
  for (int j = 0; j < kRdma; ++j) rm |= v.dal(kDevRdmaW + j, i) != 0 ? (1u << j) : 0u;
}

// The node's reservations as one pod's restore sees them, classified once per call: mm = the matched ones holding
// devices (rsv_dev_matched), um = the unmatched ones holding devices with assigned pods, hm = the device words any
// reservation holds (other words need no restore).  View positions >= 64 are classified on the spot (drs_matched).
struct DrsSet {
  uint64_t mm, um;
  uint32_t hm;
};
template <typename V>
__device__ __forceinline__ DrsSet drs_set(const V& v, int32_t cls) {
  DrsSet s{0ull, 0ull, 0u};
  const int64_t n = v.n();
  for (int64_t i = 0; i < n; ++i) {
    s.hm |= v.dmask(i);
    if (i >= 64) continue;
    const uint32_t meta = v.meta(i);
    if (!(meta & kRsvMetaDev)) continue;
    const int32_t a = v.assigned(i);
    if ((meta & KS_RSV_ALLOCATE_ONCE) && a > 0) continue;  // (not restored at all)
    const bool matched = !(meta & KS_RSV_UNSCHEDULABLE) && cls >= 0 && cls < 64 && ((v.cls(i) >> cls) & 1ull);
    s.mm |= matched ? (1ull << i) : 0ull;
    s.um |= (!matched && a > 0) ? (1ull << i) : 0ull;
  }
  return s;
}
template <typename V>
__device__ __forceinline__ bool drs_matched(const DrsSet& s, const V& v, int64_t i, int32_t cls) {
  return i < 64 ? ((s.mm >> i) & 1ull) != 0 : rsv_dev_matched(v, i, cls);
}

// The node device of one allocator call (see above).  r: the reservation allocated from (kDrsTry); gq / rq: the types
// of requiredDeviceResources (calcRequiredDeviceResources, reservation.go:273-292) -- only those minors exist, with
// free = r's remained (zero when `zero`: nothing remained anywhere).
template <typename DV, typename V>
struct DevRView {
  const DV& d;
  const V& v;
  int32_t cls;
  int64_t r;
  int mode;
  uint32_t gq, rq;
  bool zero;
  const DrsSet& s;
  __device__ __forceinline__ bool present() const { return d.present(); }
  __device__ __forceinline__ int64_t ptot(int w) const { return d.tot(w); }
  // the word's required-type minor mask (0 = the type is not required)
  __device__ __forceinline__ uint32_t req_of(int w, int& k) const {
    if (w < kDevRdmaW) {
      k = w % kGpus;
      return gq;
    }
    k = w - kDevRdmaW;
    return rq;
  }
  __device__ __forceinline__ int64_t tot(int w) const {
    if (w >= kDevQW) return d.tot(w);  // (topology words)
    int k;
    const uint32_t q = req_of(w, k);
    return (q && !((q >> k) & 1u)) ? 0 : d.tot(w);
  }
  __device__ __forceinline__ int64_t use(int w) const {
    int k;
    if (req_of(w, k)) {  // nodeDevice.filter: used = max(0, total - free)
      const int64_t f = zero ? 0 : v.dal(w, r) - v.dald(w, r), u = d.tot(w) - f;
      return u > 0 ? u : 0;
    }
    if (!((s.hm >> w) & 1u)) return d.use(w);
    // preemptible: the matched ones' allocatable (fallback) or allocated plus r's remained (kDrsTry), the unmatched
    // ones' allocated (their assigned pods' part of the reserve pod's use)
    int64_t pre = 0;
    for (uint64_t m = s.mm; m; m &= m - 1ull) {
      const int i = __builtin_ctzll(m);
      pre += mode == kDrsFallback ? v.dal(w, i) : v.dald(w, i);
    }
    if (mode == kDrsTry && r < 64) pre += v.dal(w, r) - v.dald(w, r);
    for (uint64_t m = s.um; m; m &= m - 1ull) {
      const int64_t x = v.dald(w, __builtin_ctzll(m));
      pre += x > 0 ? x : 0;
    }
    for (int64_t i = 64; i < v.n(); ++i) {
      const uint32_t meta = v.meta(i);
      const int32_t a = v.assigned(i);
      if (!(meta & kRsvMetaDev) || ((meta & KS_RSV_ALLOCATE_ONCE) && a > 0)) continue;
      const bool matched = !(meta & KS_RSV_UNSCHEDULABLE) && cls >= 0 && cls < 64 && ((v.cls(i) >> cls) & 1ull);
      if (matched) {
        pre += mode == kDrsFallback ? v.dal(w, i) : v.dald(w, i) + (i == r ? v.dal(w, i) - v.dald(w, i) : 0);
      } else if (a > 0) {
        const int64_t x = v.dald(w, i);  // used = max(0, allocatable - remained)
        pre += x > 0 ? x : 0;
      }
    }
    const int64_t u = d.use(w) - pre;
    return u > 0 ? u : 0;
  }
};

// tryAllocateFromReservation's body for reservation i (reservation.go:201-240): Default / Aligned allocate with its
// minors preferred; Restricted requires them, then allocates again with its remained as the free amounts.  ALLOC:
// with Reserve's scorer and the minors.
template <bool ALLOC, typename DV, typename V>
__device__ __forceinline__ DevOut dev_rsv_try(const Cfg& c, const PodRec& p, const DV& dv, const V& v, const DrsSet& s,
                                              int64_t i, GpuReq* req_out) {
  const int32_t cls = p.rsv_class;
  uint32_t gm, rm;
  rsv_dev_minors(v, i, gm, rm);
  DevPick pk{gm, rm, 0xFFu, 0xFFu};
  const DevRView<DV, V> tv{dv, v, cls, i, kDrsTry, 0u, 0u, false, s};
  const uint32_t pol = rsv_policy(v.meta(i));
  if (pol == KS_RSV_POLICY_DEFAULT || pol == KS_RSV_POLICY_ALIGNED) return dev_eval<ALLOC>(c, p, tv, req_out, ~0u, pk);
  if (pol != KS_RSV_POLICY_RESTRICTED) return DevOut{KS_R_DEV_INSUFFICIENT, 0, 0u, 0u};
  pk.greq = gm ? gm : 0xFFu;  // (a type the reservation holds none of is not required: an empty minor set)
  pk.rreq = rm ? rm : 0xFFu;
  const DevOut d = dev_eval<false>(c, p, tv, nullptr, ~0u, pk);
  if (d.reasons) return d;
  // calcRequiredDeviceResources: the minors whose remained is not all-zero, else every minor with nothing
  uint32_t gq = 0u, rq = 0u;
  for (int k = 0; k < kGpus; ++k)
    if ((gm >> k) & 1u) {
      bool nz = false;
#pragma unroll
      for (int q = 0; q < 3; ++q) nz |= v.dal(q * kGpus + k, i) != v.dald(q * kGpus + k, i);
      gq |= nz ? (1u << k) : 0u;
    }
  for (int j = 0; j < kRdma; ++j)
    if (((rm >> j) & 1u) && v.dal(kDevRdmaW + j, i) != v.dald(kDevRdmaW + j, i)) rq |= 1u << j;
  const bool zero = !gq && !rq;
  const DevRView<DV, V> qv{dv, v, cls, i, kDrsTry, zero ? gm : gq, zero ? rm : rq, zero, s};
  return dev_eval<ALLOC>(c, p, qv, req_out, ~0u, pk);
}

// scoreWithReservation (reservation.go:249-271) on reservation i's view, or (i < 0) the node outside every
// reservation's preference -- DeviceShare Score (scoring.go:30-90)
template <typename DV, typename V>
__device__ __forceinline__ int32_t dev_rsv_score(const Cfg& c, const PodRec& p, const DV& dv, const V& v, const DrsSet& s,
                                                int64_t i, const GpuReq& g) {
  const int32_t cls = p.rsv_class;
  if (i < 0) return dev_raw(c, p, DevRView<DV, V>{dv, v, cls, -1, kDrsFallback, 0u, 0u, false, s}, g);
  if (rsv_policy(v.meta(i)) != KS_RSV_POLICY_RESTRICTED)
    return dev_raw(c, p, DevRView<DV, V>{dv, v, cls, i, kDrsTry, 0u, 0u, false, s}, g);
  uint32_t gm, rm, gq = 0u, rq = 0u;
  rsv_dev_minors(v, i, gm, rm);
  for (int k = 0; k < kGpus; ++k)
    if ((gm >> k) & 1u) {
      bool nz = false;
#pragma unroll
      for (int q = 0; q < 3; ++q) nz |= v.dal(q * kGpus + k, i) != v.dald(q * kGpus + k, i);
      gq |= nz ? (1u << k) : 0u;
    }
  for (int j = 0; j < kRdma; ++j)
    if (((rm >> j) & 1u) && v.dal(kDevRdmaW + j, i) != v.dald(kDevRdmaW + j, i)) rq |= 1u << j;
  const bool zero = !gq && !rq;
  return dev_raw(c, p, DevRView<DV, V>{dv, v, cls, i, kDrsTry, zero ? gm : gq, zero ? rm : rq, zero, s}, g);
}

// DeviceShare Filter + Score on a node whose reservations hold devices (deviceshare/plugin.go:271-320): a matched
// reservation to allocate from (required for a reservation-affinity pod: KS_R_RSV_NO_FIT, "no reservation(s) to meet
// the device requirements"), else the fallback view; the score on the nominated reservation's view (nom: view index)
template <typename DV, typename V>
__device__ __forceinline__ DevOut dev_rsv_eval(const Cfg& c, const PodRec& p, const DV& dv, const V& v, int32_t nom) {
  DevOut o{0u, 0, 0u, 0u};
  if (!dv.present()) return o;
  GpuReq g;
  o.reasons = dev_prepare(p, dv, g);
  if (o.reasons) return o;
  const int32_t cls = p.rsv_class;
  const DrsSet s = drs_set(v, cls);
  bool ok = false, any = false;
  for (int64_t i = 0; i < v.n() && !ok; ++i) {
    if (!drs_matched(s, v, i, cls)) continue;
    any = true;
    ok = dev_rsv_try<false>(c, p, dv, v, s, i, nullptr).reasons == 0;
  }
  if (!ok) {
    if (any && (p.flags & KS_POD_RSV_AFFINITY)) {
      o.reasons = KS_R_RSV_NO_FIT;
      return o;
    }
    const DevOut f = dev_eval<false>(c, p, DevRView<DV, V>{dv, v, cls, -1, kDrsFallback, 0u, 0u, false, s});
    o.reasons = f.reasons;
    if (o.reasons) return o;
    if (!(nom >= 0 && drs_matched(s, v, nom, cls))) {
      o.raw = f.raw;  // (the Score's view is this one: its raw is the Filter's)
      return o;
    }
  }
  o.raw = dev_rsv_score(c, p, dv, v, s, (nom >= 0 && drs_matched(s, v, nom, cls)) ? nom : -1, g);
  return o;
}

// DeviceShare's FilterReservation + ScoreReservation of reservation i (plugin.go:322-358, scoring.go:99-142): it holds
// devices and tryAllocateFromReservation([i], required) allocates; *ds = its scoreWithReservation
template <typename DV, typename V>
__device__ __forceinline__ bool dev_rsv_candidate(const Cfg& c, const PodRec& p, const DV& dv, const V& v, const DrsSet& s,
                                                  int64_t i, int32_t* ds) {
  *ds = 0;
  if (!dv.present() || !rsv_dev_matched(v, i, p.rsv_class)) return false;
  GpuReq g;
  if (dev_prepare(p, dv, g)) return false;
  if (dev_rsv_try<false>(c, p, dv, v, s, i, nullptr).reasons) return false;
  *ds = dev_rsv_score(c, p, dv, v, s, i, g);
  return true;
}

// Reserve (plugin.go:377-430): allocateWithNominatedReservation on the nominated reservation (view index nom), else
// the fallback view, with the scorer; the minors in the result
template <typename DV, typename V>
__device__ __forceinline__ DevOut dev_rsv_reserve(const Cfg& c, const PodRec& p, const DV& dv, const V& v, int32_t nom, GpuReq* req_out) {
  const DrsSet s = drs_set(v, p.rsv_class);
  if (nom >= 0 && drs_matched(s, v, nom, p.rsv_class)) {
    const DevOut d = dev_rsv_try<true>(c, p, dv, v, s, nom, req_out);
    if (d.reasons == 0) return d;
  }
  return dev_eval<true>(c, p, DevRView<DV, V>{dv, v, p.rsv_class, -1, kDrsFallback, 0u, 0u, false, s}, req_out);
}

// the assigned pod's allocation on reservation i's minors: allocated += (sign) the request per instance there
template <typename V>
__device__ __forceinline__ void rsv_dev_assign(const DevRsv& rv, const V& v, int64_t i, const GpuReq& g, uint32_t gmin,
                                               uint32_t rmin, int64_t sign) {
  uint32_t gm, rm;
  rsv_dev_minors(v, i, gm, rm);
  const int64_t col = v.csr(i);
  for (int k = 0; k < kGpus; ++k)
    if ((gm & gmin) >> k & 1u) {
      rv.dald[(int64_t)(0 * kGpus + k) * rv.nr + col] += sign * g.core;
      rv.dald[(int64_t)(1 * kGpus + k) * rv.nr + col] += sign * g.mem;
      rv.dald[(int64_t)(2 * kGpus + k) * rv.nr + col] += sign * g.ratio;
    }
  for (int j = 0; j < kRdma; ++j)
    if ((rm & rmin) >> j & 1u) rv.dald[(int64_t)(kDevRdmaW + j) * rv.nr + col] += sign * g.rdma;
}

// DeviceShare's FilterReservation where no reservation holds a device: it rejects every one for a pod it restores
struct NoDevNom {
  template <typename V>
  __device__ __forceinline__ bool operator()(const V&, int64_t, int32_t* ds) const {
    *ds = 0;
    return false;
  }
};

// BeforePreFilter restore + Reservation Filter + nomination for one (pod, node); r is the base row.
// RsvOut.nom is the view index of the nominated reservation.  dn(v, i, &ds): DeviceShare's FilterReservation of
// reservation i for a pod it restores (kPodDevNoNom), with its ScoreReservation in ds.
template <int NSC, typename V, typename DN = NoDevNom>
__device__ __forceinline__ RsvOut rsv_eval(const V& v, const PodRec& p, const NodeReg<NSC>& r, RsvDelta<NSC>& dl,
                                           DN dn = DN{}) {
  constexpr int D = 3 + NSC;
  const int32_t cls = p.rsv_class;
  const int64_t cnt = v.n();
  int64_t dpre[D], ral[D];
#pragma unroll
  for (int d = 0; d < D; ++d) dl.dreq[d] = dpre[d] = ral[d] = 0;
  dl.dnz[0] = dl.dnz[1] = 0;
  int32_t nm = 0, hiord = 0;
  for (int64_t i = 0; i < cnt; ++i) {
    uint32_t meta;
    int32_t a;
    if (!rsv_matches(v, i, cls, meta, a)) continue;
    ++nm;
    hiord = max(hiord, v.ohi(i));
    int64_t rem[kRsvDims];
    bool nzr = false;
#pragma unroll
    for (int d = 0; d < kRsvDims; ++d) {
      const int64_t x = v.alloc(d, i) - v.allocd(d, i);
      rem[d] = x > 0 ? x : 0;  // quotav1.SubtractWithNonNegativeResult
      nzr |= rem[d] != 0;
    }
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int64_t al = v.alloc(d, i);
      const int64_t kept = nzr ? rem[d] : 0;
      dl.dreq[d] -= a > 0 ? kept : al;  // matched: reserve pod removed; base had it replaced by `kept`
      dpre[d] += a > 0 ? al - kept : 0; // podRequested: this one is not in the pod's unmatched set
      ral[d] += v.allocd(d, i);
    }
    const uint32_t keys = rsv_keys(meta);
    const int64_t nzc = nzr ? ((keys & 1u) ? rem[0] : kDefaultMilliCPU) : 0;
    const int64_t nzm = nzr ? ((keys & 2u) ? rem[1] : kDefaultMemory) : 0;
    dl.dnz[0] -= a > 0 ? nzc : v.rnz(0, i);
    dl.dnz[1] -= a > 0 ? nzm : v.rnz(1, i);
  }
  dl.nm = nm;
  RsvOut o{0u, 0, 0, hiord, -1};
  const bool aff = (p.flags & KS_POD_RSV_AFFINITY) != 0;
  if (nm == 0) {
    o.reasons = aff ? KS_R_RSV_AFFINITY : 0u;
    return o;
  }
  // fitsNode (plugin.go:445-496): pods check on the restored NodeInfo, resources against
  // Allocatable - (podRequested - rRemained - rAllocated)
  const bool pods_bad = (int64_t)(r.pod_count - nm) - nm + 1 > (int64_t)r.allowed;
  const bool all_zero = (p.flags & kPodAllZero) != 0;
  int64_t slack[D];
  slack[0] = r.free_cpu - dpre[0] + ral[0];
  slack[1] = r.free_mem - dpre[1] + ral[1];
  slack[2] = r.free_eph - dpre[2] + ral[2];
#pragma unroll
  for (int k = 0; k < NSC; ++k) slack[3 + k] = r.free_sc[k] - dpre[3 + k] + ral[3 + k];
  // DeviceShare's FilterReservation for a pod it restores: dn, or (NoDevNom) none of them passes
  constexpr bool DSN = !std::is_same<DN, NoDevNom>::value;
  const bool dnom = (p.flags & kPodDevNoNom) != 0;
  int32_t best_o = 0, best_s = -1, nom_o = -1, nom_s = -1, raw_o = 0, dmax = 0, ds_o = 0, ds_s = 0;
  bool any_ok = false;
  // filterWithReservations body for one reservation (plugin.go:386-422)
  auto satisfies = [&](int64_t i) {
    const uint32_t meta = v.meta(i);
    const uint32_t names = rsv_keys(meta) & p.rsv_keys;
    bool ok = names != 0 && !pods_bad;
    if (ok && !all_zero) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const int64_t pd = pod_dim(p, d);
        if (d >= 3 && pd == 0) continue;  // podRequest.ScalarResources keys
        const int64_t rrem = v.alloc(d, i) - v.allocd(d, i);
        ok = ok && !(pd > slack[d] + rrem);
      }
    }
    const uint32_t pol = rsv_policy(meta);
    if (pol == KS_RSV_POLICY_RESTRICTED) {
#pragma unroll
      for (int d = 0; d < kRsvDims; ++d) {
        if (!((names >> d) & 1u)) continue;
        int64_t rem = v.alloc(d, i) - v.allocd(d, i);
        rem = rem > 0 ? rem : 0;
        ok = ok && !(pod_dim(p, d) > rem);
      }
    } else if (pol != KS_RSV_POLICY_DEFAULT && pol != KS_RSV_POLICY_ALIGNED) {
      ok = false;
    }
    return ok;
  };
  // DeviceShare's verdicts of the first 8 reservations, kept for the second pass (ok bit, 8-bit score: <= 200)
  uint32_t dok = 0u;
  uint64_t dsv = 0ull;
  for (int64_t i = 0; i < cnt; ++i) {
    uint32_t meta;
    int32_t a;
    if (!rsv_matches(v, i, cls, meta, a)) continue;
    if (!satisfies(i)) continue;
    any_ok = true;
    // NominateReservation: RunReservationFilterPlugins (Reservation's FilterReservation = the body above, then
    // DeviceShare's for a pod it restores), lowest order label first (strict, table order), else the best score
    int32_t ds = 0;
    if (dnom) {
      if constexpr (!DSN) continue;
      const bool pass = dn(v, i, &ds);
      if (i < 8 && pass) {
        dok |= 1u << i;
        dsv |= (uint64_t)(uint32_t)ds << (8 * i);
      }
      if (!pass) continue;
    }
    const int32_t oh = v.ohi(i);
    const int32_t sc = rsv_score(v, p, i);
    if (oh > best_o) {
      best_o = oh;
      nom_o = (int32_t)i;
      raw_o = sc;
      ds_o = ds;
    }
    dmax = max(dmax, ds);
    if (!dnom && sc > best_s) {
      best_s = sc;
      nom_s = (int32_t)i;
    }
  }
  int32_t raw_s = best_s;
  if (DSN && dnom && nom_o < 0) {
    // prioritizeReservations (nominator.go:218-262): Reservation's ScoreReservation (no normalization) + DeviceShare's
    // after DefaultReservationNormalizeScore(100); the highest sum, ties in table order
    for (int64_t i = 0; i < cnt; ++i) {
      uint32_t meta;
      int32_t a;
      if (!rsv_matches(v, i, cls, meta, a) || !satisfies(i)) continue;
      int32_t ds = 0;
      if (i < 8) {
        if (!((dok >> i) & 1u)) continue;
        ds = (int32_t)((dsv >> (8 * i)) & 0xFFull);
      } else if (!dn(v, i, &ds)) {
        continue;
      }
      const int32_t sc = rsv_score(v, p, i);
      const int32_t t = sc + (dmax > 0 ? 100 * ds / dmax : ds);
      if (t > best_s) {
        best_s = t;
        nom_s = (int32_t)i;
        raw_s = sc;
        ds_s = ds;
      }
    }
  }
  o.nom = nom_o >= 0 ? nom_o : nom_s;
  o.raw = nom_o >= 0 ? raw_o : (nom_s >= 0 ? raw_s : 0);
  o.dds = (DSN && dnom && o.nom >= 0) ? 1 + (nom_o >= 0 ? ds_o : ds_s) : 0;
  // the Reservation Filter passes on any satisfying reservation (DeviceShare's FilterReservation runs in the
  // nomination only)
  o.reasons = (aff && !any_ok) ? KS_R_RSV_NO_FIT : 0u;
  o.hi = hiord > 0 ? hiord : o.raw;
  return o;
}

// ---- the restore path's call boundary: these run out of line (one instance per view pair) with their inputs by
// value, so the kernels keep their registers and nothing is copied to the stack per call ----
struct DevRsvArgs {
  int32_t dev_most, dw_core, dw_mem, dw_ratio, dw_rdma;
  uint32_t flags;
  int32_t rsv_class;
  uint32_t joint;
  int64_t gpu_core, gpu_mem, gpu_ratio, rdma;
};
__device__ __forceinline__ DevRsvArgs dev_rsv_args(const Cfg& c, const PodRec& p) {
  return DevRsvArgs{c.dev_most, c.dw_core, c.dw_mem, c.dw_ratio, c.dw_rdma, p.flags, p.rsv_class, p.joint,
                    p.gpu_core, p.gpu_mem, p.gpu_ratio, p.rdma};
}
__device__ __forceinline__ void dev_rsv_unpack(const DevRsvArgs& x, Cfg& c, PodRec& p) {
  c = Cfg{};
  c.dev = 1;
  c.dev_most = x.dev_most;
  c.dw_core = x.dw_core;
  c.dw_mem = x.dw_mem;
  c.dw_ratio = x.dw_ratio;
  c.dw_rdma = x.dw_rdma;
  p = PodRec{};
  p.flags = x.flags;
  p.rsv_class = x.rsv_class;
  p.joint = x.joint;
  p.gpu_core = x.gpu_core;
  p.gpu_mem = x.gpu_mem;
  p.gpu_ratio = x.gpu_ratio;
  p.rdma = x.rdma;
}
template <typename DV, typename V>
__device__ __attribute__((noinline)) DevOut dev_rsv_eval_x(DevRsvArgs x, DV dv, V v, int32_t nom) {
  Cfg c;
  PodRec p;
  dev_rsv_unpack(x, c, p);
  return dev_rsv_eval(c, p, dv, v, nom);
}
// (ok << 32) | ds
template <typename DV, typename V>
__device__ __attribute__((noinline)) uint64_t dev_rsv_candidate_x(DevRsvArgs x, DV dv, V v, DrsSet s, int64_t i) {
  Cfg c;
  PodRec p;
  dev_rsv_unpack(x, c, p);
  int32_t ds = 0;
  const bool ok = dev_rsv_candidate(c, p, dv, v, s, i, &ds);
  return ((uint64_t)(ok ? 1u : 0u) << 32) | (uint32_t)ds;
}

// A reservation visitor with the pod's rsv_eval on it already computed (the commit's nomination, reused by eval_full)
template <int NSC, typename F>
struct RsvWithOut {
  F f;
  RsvOut ro;
  RsvDelta<NSC> dl;
  template <typename G>
  __device__ __forceinline__ auto operator()(G&& g) const {
    return f(g);
  }
};
template <typename T>
struct RsvKnown : std::false_type {};
template <int NSC, typename F>
struct RsvKnown<RsvWithOut<NSC, F>> : std::true_type {};

// base row <-> the pod's restored row (sign = +1 apply, -1 undo; exact in int64)
template <int NSC>
__device__ __forceinline__ void rsv_apply(NodeReg<NSC>& r, const RsvDelta<NSC>& dl, int64_t sign) {
  r.free_cpu -= sign * dl.dreq[0];
  r.free_mem -= sign * dl.dreq[1];
  r.free_eph -= sign * dl.dreq[2];
  term_take(r.t_eph, sign * dl.dreq[2], (double)(sign * dl.dreq[2]) * 100.0);
#pragma unroll
  for (int k = 0; k < NSC; ++k) {
    r.free_sc[k] -= sign * dl.dreq[3 + k];
    term_take(r.t_sc[k], sign * dl.dreq[3 + k], (double)(sign * dl.dreq[3 + k]) * 100.0);
  }
  term_take(r.t_cpu, sign * dl.dnz[0], (double)(sign * dl.dnz[0]) * 100.0);
  term_take(r.t_mem, sign * dl.dnz[1], (double)(sign * dl.dnz[1]) * 100.0);
  term_take(r.t_ncpu, sign * dl.dreq[0], (double)(sign * dl.dreq[0]) * 100.0);
  term_take(r.t_nmem, sign * dl.dreq[1], (double)(sign * dl.dreq[1]) * 100.0);
  r.pod_count -= (int32_t)sign * dl.nm;
  r.pods_full = ((int64_t)r.pod_count + 1 > (int64_t)r.allowed) || !r.valid;
}

// Filter + Score of one (pod, node) with the Reservation plugin: total = hi * F + Fit/LA total.
// r must be the base row; with UNDO it is returned unchanged (the sweep reuses it across pods).
// rsv(f) calls f on the node's reservation view (RsvG / RsvL): rsv_eval when the pod's class matches one of them,
// DeviceShare's restore-state evaluation (dev_rsv_eval) on a node whose reservations hold devices.
// FEAT: bit 0 Reservation, bit 1 NodeNUMAResource, bit 2 DeviceShare, bit 3 NUMA topology policies compiled in
// (the Cfg flags switch them at run time).  devv() / numav() return the node's device view (ks_dev.h) and NUMA
// view (ks_numa.h).  Filter order as in the profile: Fit, LoadAware, NodeNUMAResource (on a node with a NUMA
// topology policy its topology-manager Admit, whose affinity then restricts DeviceShare), DeviceShare,
// Reservation.  The key total is key_total(c, o, M) with M the pod's normalization maxima (NormM).
// dhf / dff: DeviceShare's topology hints and its Filter / Score under a NUMA restriction from elsewhere (the commit
// kernel's helper waves, ks_pass.h); NoDevHints = computed here.
template <int NSC, bool DEBUG, bool UNDO, int FEAT, typename F, typename G, typename H, typename DHF = NoDevHints,
          typename DFF = NoDevHints>
__device__ __forceinline__ EvalOut eval_full(const Cfg& c, const PodRec& p, NodeReg<NSC>& r, F&& rsv, G&& devv,
                                             H&& numav, RsvOut* info = nullptr, DHF dhf = DHF{}, DFF dff = DFF{}) {
  constexpr bool RSV = (FEAT & 1) != 0, NUMA = (FEAT & 2) != 0, DEV = (FEAT & 4) != 0, POL = (FEAT & 8) != 0;
  constexpr bool HELD = RSV && DEV && (FEAT & 16) != 0;  // reservations holding devices (DeviceShare's restore state)
  const bool dev_pod = DEV && c.dev && (p.flags & kPodHasGpu);
  // NodeNUMAResource (policy None part, then the topology-manager path on a policy node); returns DeviceShare's
  // NUMA restriction
  // (without DEBUG a node some earlier Filter already rejected skips the expensive paths: its key is 0)
  bool dev_pol = false;  // the policy path reached DeviceShare's Allocate under the same restriction as dev()
  bool dev_pre = false;  // ... and dpre is its result
  DevOut dpre = DevOut{0u, 0, 0u, 0u};
  auto numa = [&](EvalOut& o) __attribute__((always_inline)) -> uint32_t {
    if (!(NUMA && c.numa)) return ~0u;
    numa_eval<NSC, DEBUG>(c, p, r, o);
    if (!(POL && c.numa_pol) || (p.flags & kPodReqZero)) return ~0u;
    if (!DEBUG && o.reasons) return ~0u;
    const auto nv = numav();
    if (nv.policy() == 0) return ~0u;
    using DVT = decltype(devv());
    NumaPolOut pr;
    if (dev_pod) {
      const DVT dv = devv();
      pr = numa_policy_eval<!DEBUG>(c, p, nv, numa_node_ctx<NSC>(r), &dv, dhf);
    } else {
      pr = numa_policy_eval<!DEBUG>(c, p, nv, numa_node_ctx<NSC>(r), (const DVT*)nullptr);
    }
    numa_policy_apply<DEBUG>(c, p, o, o.numa_rs, pr);
    const uint32_t allow = (o.numa_rs == 0 && pr.admitted && pr.affinity) ? pr.affinity : ~0u;
    dev_pol = pr.dev_done && allow == (pr.affinity ? pr.affinity : ~0u);
    dev_pre = dev_pol && pr.dev_hit;
    dpre = pr.dev;
    return allow;
  };
  auto dev_apply = [&](EvalOut& o, const DevOut& d) __attribute__((always_inline)) {
    o.reasons |= DEBUG ? d.reasons : (d.reasons ? KS_R_FIT_PODS : 0u);
    o.dev_raw = d.raw;
    if (!DEBUG && dev_pol && d.reasons) {  // the deferred policy-path failure: no NUMA score (numa_policy_eval)
      o.total -= o.numa * c.numa_pw;
      o.numa = 0;
    }
  };
  auto dev = [&](EvalOut& o, uint32_t allow, int32_t nom, int32_t dds) __attribute__((always_inline)) {
    if (!dev_pod) return;
    if (!DEBUG && o.reasons) return;
    if constexpr (HELD) {
      // reservations holding devices on the node (never one with a NUMA policy): the restore state's views
      if (c.rsv) {
        const auto dv = devv();
        if (dv.held()) {
          // a reservation DeviceShare's FilterReservation nominated: the pod allocates from it (Filter passes) and
          // the Score is its ScoreReservation's view, both computed in the nomination
          if (dds > 0) dev_apply(o, DevOut{0u, dds - 1, 0u, 0u});
          else dev_apply(o, rsv([&](const auto& v) { return dev_rsv_eval_x(dev_rsv_args(c, p), dv, v, nom); }));
          return;
        }
      }
    }
    DevOut d;
    if (dev_pre) {
      d = dpre;
    } else {
      if constexpr (LateDevHints<DFF>::value) d = dff(allow);
      else d = dev_eval<false>(c, p, devv(), nullptr, allow);
    }
    dev_apply(o, d);
  };
  if (!RSV || !c.rsv || (p.rsv_class < 0 && !(p.flags & KS_POD_RSV_AFFINITY))) {
    if (info) *info = RsvOut{0u, 0, 0, 0, -1};
    EvalOut o = eval_pod_node<NSC, DEBUG>(c, p, r);
    const uint32_t allow = numa(o);
    dev(o, allow, -1, 0);
    return o;
  }
  const bool slow = p.rsv_class >= 0 && p.rsv_class < 64 && ((r.rsv_cls >> p.rsv_class) & 1ull);
  RsvDelta<NSC> dl;
  RsvOut ro{(p.flags & KS_POD_RSV_AFFINITY) ? KS_R_RSV_AFFINITY : 0u, 0, 0, 0, -1};
  if (slow) {
    // DeviceShare's FilterReservation / ScoreReservation in the nomination (a pod it restores); the view's
    // classification once per nomination
    DrsSet dset{0ull, 0ull, 0u};
    bool dset_on = false;
    auto dnom = [&](const auto& v, int64_t i, int32_t* ds) -> bool {
      *ds = 0;
      if constexpr (HELD) {
        const auto dv = devv();
        if (!dv.held()) return false;
        if (!dset_on) {
          dset = drs_set(v, p.rsv_class);
          dset_on = true;
        }
        const uint64_t r = dev_rsv_candidate_x(dev_rsv_args(c, p), dv, v, dset, i);
        *ds = (int32_t)(uint32_t)r;
        return (r >> 32) != 0;
      }
      return false;
    };
    if constexpr (RsvKnown<std::decay_t<F>>::value) {
      ro = rsv.ro;  // (the caller's nomination on the same row)
      dl = rsv.dl;
    } else if constexpr (HELD) {
      ro = rsv([&](const auto& v) { return rsv_eval<NSC>(v, p, r, dl, dnom); });
    } else {
      ro = rsv([&](const auto& v) { return rsv_eval<NSC>(v, p, r, dl); });
    }
    rsv_apply<NSC>(r, dl, 1);
  }
  EvalOut o = eval_pod_node<NSC, DEBUG>(c, p, r);
  const uint32_t allow = numa(o);
  if (UNDO && slow) rsv_apply<NSC>(r, dl, -1);
  dev(o, allow, ro.nom, ro.dds);
  // a node without matched reservations is cut by the Reservation PreFilter (PreFilterResult
  // NodeNames, plugin.go:235-246) before any Filter plugin runs
  o.reasons = ro.reasons == KS_R_RSV_AFFINITY ? ro.reasons : (o.reasons | ro.reasons);
  o.hi = ro.hi;
  if (info) *info = ro;
  return o;
}

// Key total of a feasible node: Fit + LoadAware + NUMA + the normalized plugins with the pod's maxima M,
// then the Reservation ranking.  The preferred node is the lowest INDEX among equal order labels,
// whatever its other scores: ordered nodes rank by hi alone (ties to the lower index through the
// key's node bits).
__device__ __forceinline__ int32_t norm_terms(const Cfg& c, const EvalOut& o, const NormM& M) {
  int32_t t = 0;
  if (c.dev) t += c.dev_pw * (M.dev == 0 ? o.dev_raw : small_div(100 * o.dev_raw, M.dev));
  // TaintToleration: DefaultNormalizeScore(100, reverse = true); NodeAffinity: DefaultNormalizeScore(100)
  if (c.taint & 2) t += c.taint_pw * (M.taint == 0 ? 100 : 100 - small_div(100 * o.traw, M.taint));
  if (c.aff & 2) t += c.aff_pw * (M.aff == 0 ? o.araw : small_div(100 * o.araw, M.aff));
  return t;
}

__device__ __forceinline__ int32_t key_total(const Cfg& c, const EvalOut& o, const NormM& M) {
  int32_t t = o.total + norm_terms(c, o, M);
  if (c.rsv) t = o.hi >= kRsvOrderBase ? o.hi * c.rsv_F : t + o.hi * c.rsv_F;
  return t;
}

// Reserve into reservation i of the view (plugin.go:532-570 -> reservation_info.go:379-388): the
// change of the node's base restore (unmatched remainder of i before / after) for each Requested /
// NonZero dim, and the Allocated increment.
struct RsvReserve {
  int64_t dreq[kRsvDims];
  int64_t dnz[2];
  int64_t add[kRsvDims];  // Allocated += Mask(pod requests, ResourceNames)
  bool now_ineligible;    // AllocateOnce: skipped from now on (transformer.go:109)
};

template <typename V>
__device__ __forceinline__ RsvReserve rsv_reserve_delta(const V& v, const PodRec& p, int64_t i) {
  RsvReserve o;
  const uint32_t meta = v.meta(i);
  const uint32_t keys = rsv_keys(meta);
  const int32_t a_old = v.assigned(i);
  const bool ao = (meta & KS_RSV_ALLOCATE_ONCE) != 0;
  int64_t al[kRsvDims], ro[kRsvDims], rn[kRsvDims];
  bool nz_old = false, nz_new = false;
#pragma unroll
  for (int d = 0; d < kRsvDims; ++d) {
    al[d] = v.alloc(d, i);
    const int64_t ad = v.allocd(d, i);
    o.add[d] = ((keys >> d) & 1u) ? pod_dim(p, d) : 0;
    const int64_t vo = al[d] - ad, vn = al[d] - (ad + o.add[d]);
    ro[d] = vo > 0 ? vo : 0;
    rn[d] = vn > 0 ? vn : 0;
    nz_old |= ro[d] != 0;
    nz_new |= rn[d] != 0;
  }
  // base contribution U(r) = eligible && assigned > 0 ? [rem != 0] * rem - alloc : 0
#pragma unroll
  for (int d = 0; d < kRsvDims; ++d) {
    const int64_t u_old = a_old > 0 ? (nz_old ? ro[d] : 0) - al[d] : 0;
    const int64_t u_new = !ao ? (nz_new ? rn[d] : 0) - al[d] : 0;
    o.dreq[d] = u_new - u_old;
  }
  const int64_t rnzc = v.rnz(0, i), rnzm = v.rnz(1, i);
  const int64_t oc = nz_old ? ((keys & 1u) ? ro[0] : kDefaultMilliCPU) : 0;
  const int64_t om = nz_old ? ((keys & 2u) ? ro[1] : kDefaultMemory) : 0;
  const int64_t nc = nz_new ? ((keys & 1u) ? rn[0] : kDefaultMilliCPU) : 0;
  const int64_t nmm = nz_new ? ((keys & 2u) ? rn[1] : kDefaultMemory) : 0;
  o.dnz[0] = (!ao ? nc - rnzc : 0) - (a_old > 0 ? oc - rnzc : 0);
  o.dnz[1] = (!ao ? nmm - rnzm : 0) - (a_old > 0 ? om - rnzm : 0);
  o.now_ineligible = ao;
  return o;
}

// union of owner classes of the node's matchable reservations
template <typename V>
__device__ __forceinline__ uint64_t rsv_node_classes(const V& v) {
  uint64_t m = 0;
  for (int64_t i = 0; i < v.n(); ++i) {
    const uint32_t meta = v.meta(i);
    const int32_t a = v.assigned(i);
    if (((meta & KS_RSV_ALLOCATE_ONCE) && a > 0) || (meta & KS_RSV_UNSCHEDULABLE)) continue;
    m |= v.cls(i);
  }
  return m;
}

}  // namespace ks
