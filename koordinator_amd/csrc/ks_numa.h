// ks_numa.h — NodeNUMAResource on nodes with a NUMA topology policy (SURVEY a24 hints, a25 topology manager, a29
// DeviceShare hints).
//
// Per (pod, node) one lane runs the whole FilterByNUMANode -> topology manager Admit path:
//   * NodeNUMAResource hints (generateResourceHints, resource_manager.go:459-593): per NUMA-node mask in
//     IterateBitMasks order, a hint per requested resource (cpu, memory) when the mask's total and free amounts
//     cover the request (a cpu-bind pod's cpu amplified, getResourceOptions plugin.go:495-506); preferred = the
//     narrowest mask size that could hold it; hint score = the NUMAScoringStrategy scorer over the mask;
//   * DeviceShare hints (generateTopologyHints, deviceshare/topology_hint.go:108-210): per mask over the device
//     topology's NUMA nodes, Prepare, the device count of the mask (calcTotalDevicesByNUMA) against each type's
//     desired count, minAffinitySize, a trial Allocate restricted to the mask (dev_eval with a NUMA restriction);
//     one identical list per resource name of the request (gpu-core / gpu-memory / gpu-memory-ratio, rdma);
//   * the merge (filterProvidersHints / mergeFilteredHints, topologymanager/policy.go:96-226) over the cartesian
//     product of the lists, providers in the order NodeNUMAResource, DeviceShare (the reference registers them
//     in plugin construction order, which Go's registry map leaves random), NodeNUMAResource's lists cpu then
//     memory (a Go map there too); the policy's filter and admit rule;
//   * allocateResources: the NUMA plugin's Allocate (tryBestToDistributeEvenly, resource_manager.go:221-283,
//     including its sort that compares totalAvailable by slice position; a cpu-bind pod distributes its original
//     request in whole CPUs, and allocateCPUSet :314-401 needs, per allocated NUMA node, min(available CPUs there,
//     the node's whole CPUs) to add up to numCPUsNeeded), then DeviceShare's Allocate restricted to the affinity;
//   * the node score over the allocated NUMA nodes (calculateAllocatableAndRequested, scoring.go:116-163; a
//     cpu-bind pod's requested cpu is the node's amplified cpuset CPUs).
// Up to kNumaDev NUMA nodes per node (15 masks); DeviceShare hints over at most 2 device NUMA nodes on nodes
// with at most 2 NUMA nodes (ks_load_* refuses more), so the product is at most 3 x 3 x 3^4 = 729 permutations.
// The oracle (oracle/koord_oracle.c numa_policy_eval, ko_merge_hints, dev_hints) restates the same code with
// per-NUMA arrays and explicit hint lists; its merge is pinned by the reference's policy_test.go tables.
#pragma once

#include "ks_device.h"
#include "ks_dev.h"

namespace ks {

constexpr int kNumaDev = 4;  // NUMA nodes per node the device evaluates
constexpr int kNumaMasks = (1 << kNumaDev) - 1;
constexpr int kDevHintIds = 2;  // device-topology NUMA nodes DeviceShare hints are generated over

struct DevNuma {
  const int32_t* count;  // [npad] NUMA nodes with resources
  const int64_t* total;  // [2][kNumaDev][npad] amplified NUMANodeResources (cpu milli, memory)
  int64_t* used;         // [2][kNumaDev][npad] allocatedResources (raw; mutable)
  int64_t* off;          // [kNumaDev][npad] cpuset amplification of the allocated cpu: Amplify(cs) - cs (mutable)
  int32_t* cs;           // [kNumaDev][npad] allocated cpuset CPUs on the NUMA node (mutable)
  int32_t* free;         // [kNumaDev][npad] CPUs of the NUMA node available to cpuset pods (mutable)
  uint32_t* present;     // [npad] bit k: an allocatedResources entry exists (mutable)
  const uint32_t* flags; // [npad] ks_node_cols.numa_flags (policy in bits 5-6)
  int64_t npad;
};

// node view: HBM columns or the commit kernel's LDS copy
struct NumaGView {
  const DevNuma& d;
  int64_t n;
  __device__ __forceinline__ int policy() const { return (int)((gld(d.flags + n) >> KS_NUMA_POLICY_SHIFT) & 3u); }
  __device__ __forceinline__ int count() const { return gld(d.count + n); }
  __device__ __forceinline__ uint32_t present() const { return gld(d.present + n); }
  __device__ __forceinline__ int64_t total(int r, int k) const { return gld(d.total + ((int64_t)r * kNumaDev + k) * d.npad + n); }
  __device__ __forceinline__ int64_t used(int r, int k) const { return gld(d.used + ((int64_t)r * kNumaDev + k) * d.npad + n); }
  __device__ __forceinline__ int64_t off(int k) const { return gld(d.off + (int64_t)k * d.npad + n); }
  __device__ __forceinline__ int32_t freec(int k) const { return gld(d.free + (int64_t)k * d.npad + n); }
};

// LDS slot words: [2K total | 2K used | K off | K (cs << 32 | free) | meta (policy | count << 8 | present << 32)]
constexpr int kNumaWTot = 0, kNumaWUsed = 2 * kNumaDev, kNumaWOff = 4 * kNumaDev, kNumaWCpu = 5 * kNumaDev,
              kNumaWMeta = 6 * kNumaDev;
constexpr int kNumaSlotWords = 6 * kNumaDev + 1;

struct NumaLView {
  const int64_t* w;
  __device__ __forceinline__ int policy() const { return (int)(w[kNumaWMeta] & 3); }
  __device__ __forceinline__ int count() const { return (int)((w[kNumaWMeta] >> 8) & 0xFF); }
  __device__ __forceinline__ uint32_t present() const { return (uint32_t)(w[kNumaWMeta] >> 32); }
  __device__ __forceinline__ int64_t total(int r, int k) const { return w[kNumaWTot + r * kNumaDev + k]; }
  __device__ __forceinline__ int64_t used(int r, int k) const { return w[kNumaWUsed + r * kNumaDev + k]; }
  __device__ __forceinline__ int64_t off(int k) const { return w[kNumaWOff + k]; }
  __device__ __forceinline__ int32_t freec(int k) const { return (int32_t)(uint32_t)w[kNumaWCpu + k]; }
};

// node-level inputs of the policy path (NodeInfo and the node's cpuset state)
struct NumaNodeCtx {
  int64_t plain_req_cpu, plain_req_mem, plain_alloc_cpu, plain_alloc_mem;  // NodeInfo Requested / Allocatable
  double ratio;     // cpu amplification ratio
  int64_t cs_milli; // the node's allocated cpuset CPUs x 1000
  int64_t cs_off;   // Amplify(cs_milli) - cs_milli
  int32_t cpu_free; // CPUs available to cpuset pods on the node (-1 = no valid CPU topology)
};

struct NumaPolOut {
  uint32_t reasons;
  int32_t score;
  int64_t alloc[2][kNumaDev];  // the pod's NUMA allocation (cpu milli, memory)
  int32_t cpus[kNumaDev];      // cpu-bind pod: CPUs allocateCPUSet takes per allocated NUMA node
  uint32_t affinity;           // merged NUMANodeAffinity (0 = nil)
  bool admitted;               // Admit stored the affinity (DeviceShare's Filter / Score / Reserve read it)
};

// resourceAllocationScorer.score over cpu / memory with the plugin weights (scoring.go:206-242)
__device__ __forceinline__ int32_t numa_res_score(const Cfg& c, bool most, int64_t rq_cpu, int64_t rq_mem,
                                                  int64_t al_cpu, int64_t al_mem, int64_t pod_cpu, int64_t pod_mem) {
  int32_t ns = 0, ws = 0;
  if (c.nw_cpu && al_cpu != 0) {
    const int64_t rq = rq_cpu + pod_cpu;
    ns += (most ? pct_floor_i64(rq > al_cpu ? al_cpu : rq, al_cpu) : (rq > al_cpu ? 0 : pct_floor_i64(al_cpu - rq, al_cpu))) * c.nw_cpu;
    ws += c.nw_cpu;
  }
  if (c.nw_mem && al_mem != 0) {
    const int64_t rq = rq_mem + pod_mem;
    ns += (most ? pct_floor_i64(rq > al_mem ? al_mem : rq, al_mem) : (rq > al_mem ? 0 : pct_floor_i64(al_mem - rq, al_mem))) * c.nw_mem;
    ws += c.nw_mem;
  }
  return ws ? small_div(ns, ws) : 0;
}

// IterateBitMasks order for K NUMA nodes: size 1..K, lexicographic index lists (bitmask.go:206-222)
__device__ __forceinline__ int numa_masks(int K, uint32_t* m) {
  int n = 0;
  for (int size = 1; size <= K; ++size) {
    for (int i0 = 0; i0 < K; ++i0) {
      if (size == 1) { m[n++] = 1u << i0; continue; }
      for (int i1 = i0 + 1; i1 < K; ++i1) {
        if (size == 2) { m[n++] = (1u << i0) | (1u << i1); continue; }
        for (int i2 = i1 + 1; i2 < K; ++i2) {
          if (size == 3) { m[n++] = (1u << i0) | (1u << i1) | (1u << i2); continue; }
          for (int i3 = i2 + 1; i3 < K; ++i3) m[n++] = (1u << i0) | (1u << i1) | (1u << i2) | (1u << i3);
        }
      }
    }
  }
  return n;
}

__device__ __forceinline__ bool numa_narrower(uint32_t a, uint32_t b) {
  const int ca = __builtin_popcount(a), cb = __builtin_popcount(b);
  return ca == cb ? a < b : ca < cb;
}

// DeviceShare's topology hints on one node (generateTopologyHints): the hint masks (NUMA-id bit masks, IterateBitMasks
// order over the device topology's NUMA nodes), which of them allocate (ok bits), minAffinitySize, and the number
// of identical resource lists (0 = the provider expresses no preference).
struct DevHints {
  int lists;
  int nm;
  uint32_t masks[3];
  uint32_t ok;
  int minaff;
};

template <typename V>
__device__ __forceinline__ DevHints dev_hints(const Cfg& c, const PodRec& p, const V& v) {
  DevHints h;
  h.lists = 0;
  h.nm = 0;
  h.ok = 0;
  h.minaff = -1;
  if (!v.present()) return h;
  const uint64_t topo = (uint64_t)v.tot(kDevTopoW), meta = (uint64_t)v.tot(kDevMetaW);
  // numaTopology.nodes: NUMA nodes of the switches holding a device with a topology
  uint32_t ids = 0, gin[2] = {0u, 0u}, rin[2] = {0u, 0u};
  int idl[kDevHintIds];
  int nid = 0;
#pragma unroll
  for (int k = 0; k < kGpus; ++k) {
    const uint32_t pc = (uint32_t)(topo >> (4 * k)) & 0xFu;
    const bool ex = v.tot(k) != 0 || v.tot(kGpus + k) != 0 || v.tot(2 * kGpus + k) != 0;
    if (ex && pc < 8u) ids |= 1u << ((uint32_t)(meta >> (8 * pc)) & 0xFu);
  }
#pragma unroll
  for (int j = 0; j < kRdma; ++j) {
    const uint32_t pc = (uint32_t)(topo >> (32 + 4 * j)) & 0xFu;
    if (v.tot(kDevRdmaW + j) != 0 && pc < 8u) ids |= 1u << ((uint32_t)(meta >> (8 * pc)) & 0xFu);
  }
  for (uint32_t b = ids; b && nid < kDevHintIds; b &= b - 1) idl[nid++] = __builtin_ctz(b);
  GpuReq g;
  if (dev_prepare(p, v, g)) return h;  // every mask returns before minAffinitySize is set: no preference
  // minors of each type per position of the id list (existing, with a topology)
#pragma unroll
  for (int k = 0; k < kGpus; ++k) {
    const uint32_t pc = (uint32_t)(topo >> (4 * k)) & 0xFu;
    const bool ex = v.tot(k) != 0 || v.tot(kGpus + k) != 0 || v.tot(2 * kGpus + k) != 0;
    const uint32_t id = (uint32_t)(meta >> (8 * (pc & 7u))) & 0xFu;
    for (int i = 0; i < nid; ++i) gin[i] |= (ex && pc < 8u && (int)id == idl[i]) ? (1u << k) : 0u;
  }
#pragma unroll
  for (int j = 0; j < kRdma; ++j) {
    const uint32_t pc = (uint32_t)(topo >> (32 + 4 * j)) & 0xFu;
    const uint32_t id = (uint32_t)(meta >> (8 * (pc & 7u))) & 0xFu;
    for (int i = 0; i < nid; ++i) rin[i] |= (v.tot(kDevRdmaW + j) != 0 && pc < 8u && (int)id == idl[i]) ? (1u << j) : 0u;
  }
  const bool has_gpu = (p.flags & kPodGpuReq) != 0, has_rdma = p.rdma > 0;
  // masks over positions: {0}, {1}, {0, 1} (IterateBitMasks over the sorted id list)
  const uint32_t pos[3] = {1u, 2u, 3u};
  const int npos = nid == 0 ? 0 : (nid == 1 ? 1 : 3);
  for (int i = 0; i < npos; ++i) {
    uint32_t mask = 0, gm = 0, rm = 0;
    for (int q = 0; q < nid; ++q)
      if ((pos[i] >> q) & 1u) {
        mask |= 1u << idl[q];
        gm |= gin[q];
        rm |= rin[q];
      }
    h.masks[h.nm++] = mask;
    if ((has_gpu && __builtin_popcount(gm) < g.desired) || (has_rdma && __builtin_popcount(rm) < g.rdesired)) continue;
    const int cnt = __builtin_popcount(pos[i]);
    h.minaff = h.minaff < 0 ? (cnt < nid ? cnt : nid) : (cnt < h.minaff ? cnt : h.minaff);
    if (dev_eval<false>(c, p, v, nullptr, mask).reasons == 0) h.ok |= 1u << i;
  }
  if (h.minaff >= 0)
    h.lists = (has_gpu ? ((g.has_core || g.desired > 1) ? 3 : 2) : 0) + (has_rdma ? 1 : 0);
  return h;
}

// Filter (FilterByNUMANode -> Admit -> allocateResources) and Score of one (pod, node) with a NUMA policy.
// dv: the node's device view when DeviceShare is a hint provider for this pod, else nullptr.
template <typename V, typename DV>
__device__ __forceinline__ NumaPolOut numa_policy_eval(const Cfg& c, const PodRec& p, const V& v, const NumaNodeCtx& nc,
                                                       const DV* dv) {
  NumaPolOut o;
  o.reasons = 0;
  o.score = 0;
  o.affinity = 0;
  o.admitted = false;
#pragma unroll
  for (int k = 0; k < kNumaDev; ++k) {
    o.alloc[0][k] = o.alloc[1][k] = 0;
    o.cpus[k] = 0;
  }
  const int K = v.count();
  if (K == 0) {
    o.reasons = KS_R_NUMA_MISSING;
    return o;
  }
  const int pol = v.policy();
  const uint32_t pres = v.present();
  const bool bind = c.cpuset && (p.flags & KS_POD_CPU_BIND);
  int64_t tot[2][kNumaDev], use[2][kNumaDev], av[2][kNumaDev];
#pragma unroll
  for (int k = 0; k < kNumaDev; ++k) {
    const bool in = k < K, pr = in && ((pres >> k) & 1u);
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      tot[r][k] = in ? v.total(r, k) : 0;
      use[r][k] = pr ? v.used(r, k) + (r == 0 ? v.off(k) : 0) : 0;
      const int64_t a = tot[r][k] - use[r][k];
      av[r][k] = a < 0 ? 0 : a;
    }
  }
  // options.requests: a cpu-bind pod's cpu amplified (hints and score); originalRequests for the allocation
  const int64_t req_cpu = (bind && nc.ratio > 1.0) ? (int64_t)::ceil((double)p.cpu * nc.ratio) : p.cpu;
  const int64_t req[2] = {req_cpu, p.mem};
  const bool want[2] = {p.cpu != 0, p.mem != 0};
  uint32_t masks[kNumaMasks];
  const int nm = numa_masks(K, masks);
  uint32_t lack[2] = {0u, 0u};
#pragma unroll
  for (int k = 0; k < kNumaDev; ++k)
#pragma unroll
    for (int r = 0; r < 2; ++r)
      if (k < K && av[r][k] == 0) lack[r] |= 1u << k;
  // NodeNUMAResource hints: bit i of hset[r] = mask i is a hint of resource r; one score per mask
  uint32_t hset[2] = {0u, 0u};
  int min_size[2] = {K, K};
  int32_t hsc[kNumaMasks];
  const bool nmost = c.numa_sc_most != 0;
  for (int i = 0; i < nm; ++i) {
    int64_t ts[2] = {0, 0}, fs[2] = {0, 0};
#pragma unroll
    for (int k = 0; k < kNumaDev; ++k)
      if ((masks[i] >> k) & 1u)
#pragma unroll
        for (int r = 0; r < 2; ++r) {
          ts[r] += tot[r][k];
          fs[r] += av[r][k];
        }
    hsc[i] = numa_res_score(c, nmost, ts[0] - fs[0], ts[1] - fs[1], ts[0], ts[1], req[0], req[1]);
    const int cnt = __builtin_popcount(masks[i]);
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      if (!want[r] || ts[r] < req[r] || (masks[i] & lack[r])) continue;
      min_size[r] = cnt < min_size[r] ? cnt : min_size[r];
      if (fs[r] >= req[r]) hset[r] |= 1u << i;
    }
  }
  auto pref_of = [&](int r, int i) { return __builtin_popcount(masks[i]) == min_size[r]; };
  const bool single = pol == KS_NUMA_POLICY_SINGLE_NUMA_NODE;
  // DeviceShare's hints
  DevHints dh;
  dh.lists = 0;
  dh.nm = 0;
  dh.ok = 0;
  if (dv) dh = dev_hints(c, p, *dv);
  // the lists after filterProvidersHints (and filterSingleNumaHints): a list is a bit set of entries; entry 15 is
  // the list's nil entry.  lkind: 0 / 1 = NodeNUMAResource cpu / memory, 2 = DeviceShare
  constexpr int kNil = 15, kMaxLists = 2 + 4;
  uint32_t bits[kMaxLists];
  int lkind[kMaxLists];
  bool nilpref[kMaxLists];
  int nl = 0;
  bool any_numa = false;
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    if (!want[r]) continue;
    any_numa = true;
    lkind[nl] = r;
    if (hset[r] == 0) {
      bits[nl] = 1u << kNil;  // {nil, false}: "no possible NUMA affinities"
      nilpref[nl] = false;
    } else {
      uint32_t s = hset[r];
      if (single) {
        uint32_t f = 0;
        for (int i = 0; i < nm; ++i)
          if (((s >> i) & 1u) && __builtin_popcount(masks[i]) == 1 && pref_of(r, i)) f |= 1u << i;
        s = f;
      }
      bits[nl] = s;
      nilpref[nl] = false;
    }
    ++nl;
  }
  if (!any_numa) {  // the NUMA provider returns no hints: one preferred any-numa hint
    lkind[nl] = 0;
    bits[nl] = 1u << kNil;
    nilpref[nl] = true;
    ++nl;
  }
  uint32_t dbits = 0;  // DeviceShare entries (positions of dh.masks), after the single-numa-node filter
  if (dh.lists) {
    for (int i = 0; i < dh.nm; ++i) {
      if (!((dh.ok >> i) & 1u)) continue;
      const bool pr = __builtin_popcount(dh.masks[i]) == dh.minaff;
      if (!single || (__builtin_popcount(dh.masks[i]) == 1 && pr)) dbits |= 1u << i;
    }
    const bool none = dh.ok == 0;  // no allocating mask: {nil, false} per list (dropped by single-numa-node)
    for (int l = 0; l < dh.lists; ++l) {
      lkind[nl] = 2;
      bits[nl] = none ? (single ? 0u : (1u << kNil)) : dbits;
      nilpref[nl] = false;
      ++nl;
    }
  } else {
    lkind[nl] = 2;
    bits[nl] = 1u << kNil;
    nilpref[nl] = true;
    ++nl;
  }
  if (single)
    for (int l = 0; l < nl; ++l)
      if (bits[l] == (1u << kNil) && !nilpref[l]) bits[l] = 0;
  // mergeFilteredHints over the cartesian product, first list outermost
  const uint32_t dflt = (1u << K) - 1u;
  uint32_t best_mask = dflt;
  bool best_pref = false;
  int32_t best_score = 0;
  bool empty = false;
  for (int l = 0; l < nl; ++l) empty |= bits[l] == 0;
  if (!empty) {
    uint32_t rest[kMaxLists];
    int cur[kMaxLists];
    for (int l = 0; l < nl; ++l) {
      cur[l] = __builtin_ctz(bits[l]);
      rest[l] = bits[l] & (bits[l] - 1);
    }
    for (;;) {
      // mergePermutation
      uint32_t merged = dflt, first = 0;
      bool pref = true, have = false;
      for (int l = 0; l < nl; ++l) {
        const int e = cur[l];
        uint32_t m = 0;
        bool hp;
        if (e == kNil) {
          hp = nilpref[l];
        } else if (lkind[l] < 2) {
          m = masks[e];
          hp = pref_of(lkind[l], e);
        } else {
          m = dh.masks[e];
          hp = __builtin_popcount(m) == dh.minaff;
        }
        if (m) {
          if (!have) first = m;
          else if (m != first) pref = false;
          have = true;
          merged &= m;
        }
        if (!hp) pref = false;
      }
      if (merged != 0) {
        int32_t msc = 0;
        for (int l = 0; l < nl; ++l) {
          const int e = cur[l];
          if (e != kNil && lkind[l] < 2 && masks[e] == merged && hsc[e] > msc) msc = hsc[e];
        }
        if (pref && !best_pref) {
          best_mask = merged; best_pref = true; best_score = msc;
        } else if (!pref && best_pref) {
        } else if (!numa_narrower(merged, best_mask)) {
          if (__builtin_popcount(merged) == __builtin_popcount(best_mask) && msc > best_score) {
            best_mask = merged; best_pref = pref; best_score = msc;
          }
        } else {
          best_mask = merged; best_pref = pref; best_score = msc;
        }
      }
      int l = nl - 1;
      for (; l >= 0; --l) {
        if (rest[l]) {
          cur[l] = __builtin_ctz(rest[l]);
          rest[l] &= rest[l] - 1;
          break;
        }
        cur[l] = __builtin_ctz(bits[l]);
        rest[l] = bits[l] & (bits[l] - 1);
      }
      if (l < 0) break;
    }
  }
  uint32_t affinity = best_mask;
  bool admit = true;
  if (single) {
    if (affinity == dflt) affinity = 0u;
    admit = best_pref;
  } else if (pol == KS_NUMA_POLICY_RESTRICTED) {
    admit = best_pref;
  }
  if (!admit) {
    o.reasons = KS_R_NUMA_AFFINITY;
    return o;
  }
  o.admitted = true;
  o.affinity = affinity;
  // the NUMA plugin's Allocate
  if (affinity) {
    int bitsk[kNumaDev], nb = 0;
#pragma unroll
    for (int k = 0; k < kNumaDev; ++k)
      if ((affinity >> k) & 1u) bitsk[nb++] = k;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      if (!want[r]) continue;
      int ord[kNumaDev];
#pragma unroll
      for (int i = 0; i < kNumaDev; ++i) ord[i] = i < nb ? bitsk[i] : 0;
      // sort.Slice insertion sort with less(i, j) comparing totalAvailable by slice position
      for (int i = 1; i < nb; ++i)
        for (int j = i; j > 0; --j) {
          const int64_t aj = j < K ? av[r][j] : 0, ai = (j - 1) < K ? av[r][j - 1] : 0;
          if (!(aj < ai)) break;
          const int t = ord[j];
          ord[j] = ord[j - 1];
          ord[j - 1] = t;
        }
      int64_t q = r == 0 ? p.cpu : p.mem;  // originalRequests
      for (int i = 0; i < nb; ++i) {
        // splitQuantity: a cpu-bind pod's cpu in whole CPUs (Quantity.Value() rounds up)
        const int64_t split = (r == 0 && bind) ? ((q + 999) / 1000) / (nb - i) * 1000 : q / (nb - i);
        const int64_t a = av[r][ord[i]];
        const int64_t got = a > split ? split : a;
        o.alloc[r][ord[i]] = got;
        q -= got;
      }
      if (q != 0) {
        o.reasons = KS_R_NUMA_INSUFFICIENT;
        return o;
      }
    }
  }
  bool any_alloc = false;
#pragma unroll
  for (int k = 0; k < kNumaDev; ++k) any_alloc |= o.alloc[0][k] != 0 || o.alloc[1][k] != 0;
  if (bind) {
    // allocateCPUSet: the node's available CPUs, then per allocated NUMA node min(available there, whole CPUs)
    const int32_t need = (int32_t)(p.cpu_bind >> 8);
    if (nc.cpu_free < need) {
      o.reasons = KS_R_NUMA_CPUSET;
      return o;
    }
    if (any_alloc) {
      int32_t taken = 0;
#pragma unroll
      for (int k = 0; k < kNumaDev; ++k) {
        if (o.alloc[0][k] == 0 && o.alloc[1][k] == 0) continue;
        const int32_t f = v.freec(k), w = (int32_t)(o.alloc[0][k] / 1000);
        o.cpus[k] = f < w ? f : w;
        taken += o.cpus[k];
      }
      if (taken != need) {
        o.reasons = KS_R_NUMA_CPUSET;
        return o;
      }
    }
  }
  // DeviceShare's Allocate with the affinity
  if (dv) {
    const uint32_t dr = dev_eval<false>(c, p, *dv, nullptr, affinity ? affinity : ~0u).reasons;
    if (dr) {
      o.reasons = dr;
      return o;
    }
  }
  int64_t trq[2] = {0, 0}, tal[2] = {0, 0};
#pragma unroll
  for (int k = 0; k < kNumaDev; ++k) {
    if (o.alloc[0][k] == 0 && o.alloc[1][k] == 0) continue;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      tal[r] += tot[r][k];
      trq[r] += use[r][k];
    }
  }
  if (!any_alloc) {
    trq[0] = nc.plain_req_cpu;
    trq[1] = nc.plain_req_mem;
    tal[0] = nc.plain_alloc_cpu;
    tal[1] = nc.plain_alloc_mem;
  }
  if (bind) trq[0] = nc.cs_milli + nc.cs_off;  // Amplify(allocated cpuset CPUs x 1000)
  o.score = numa_res_score(c, c.numa_most != 0, trq[0], trq[1], tal[0], tal[1], req[0], req[1]);
  return o;
}

// Replace the policy-None NodeNUMAResource result of eval with the policy path's (the amplified-CPU filter and a
// cpu-bind topology failure come first, plugin.go:275-338).
template <bool DEBUG>
__device__ __forceinline__ void numa_policy_apply(const Cfg& c, const PodRec& p, EvalOut& o, uint32_t numa_rs,
                                                  const NumaPolOut& pr) {
  if (p.flags & kPodReqZero) return;
  if (numa_rs == 0) o.reasons |= DEBUG ? pr.reasons : (pr.reasons ? KS_R_FIT_PODS : 0u);
  o.total += (pr.score - o.numa) * c.numa_pw;
  o.numa = pr.score;
}

template <int NSC>
__device__ __forceinline__ NumaNodeCtx numa_node_ctx(const NodeReg<NSC>& r) {
  NumaNodeCtx nc;
  nc.plain_req_cpu = r.t_ncpu.c - r.free_cpu;
  nc.plain_req_mem = r.t_nmem.c - r.free_mem;
  nc.plain_alloc_cpu = r.t_ncpu.c;
  nc.plain_alloc_mem = r.t_nmem.c;
  nc.ratio = r.numa_ratio;
  nc.cs_milli = r.numa_A;
  nc.cs_off = r.numa_off;
  nc.cpu_free = r.cpu_free;
  return nc;
}

}  // namespace ks
