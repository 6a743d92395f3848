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
// with at most 2 NUMA nodes (ks_load_* refuses more); its identical per-resource lists merge as one list, so the
// product is at most 15 x 15 permutations (3 x 3 x 3 with device hints).
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
  int32_t* free;         // [kNumaDev][npad] numa_free_word (ks_cpuset.h): CPUs of the NUMA node available to cpuset pods
                         // (bits 0-11), its whole free cores (12-21) and cores with a free CPU (22-31) (mutable)
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
  __device__ __forceinline__ int32_t freew(int k) const { return gld(d.free + (int64_t)k * d.npad + n); }
  __device__ __forceinline__ int32_t freec(int k) const { return freew(k) & 0xFFF; }
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
  __device__ __forceinline__ int32_t freew(int k) const { return (int32_t)(uint32_t)w[kNumaWCpu + k]; }
  __device__ __forceinline__ int32_t freec(int k) const { return freew(k) & 0xFFF; }
};

// a NUMA-node word's CPUs left by filterCPUsByRequiredCPUBindPolicy (resource_manager.go:595-627): FullPCPUs the CPUs
// of the whole free cores, SpreadByPCPUs one CPU per core with a free CPU
__device__ __forceinline__ int32_t numa_filtered(int32_t w, uint32_t policy, int32_t cpc) {
  return policy == KS_CPU_BIND_FULL_PCPUS ? (int32_t)(((uint32_t)w >> 12) & 0x3FFu) * cpc : (int32_t)(((uint32_t)w >> 22) & 0x3FFu);
}

// node-level inputs of the policy path (NodeInfo and the node's cpuset state)
struct NumaNodeCtx {
  int64_t plain_req_cpu, plain_req_mem, plain_alloc_cpu, plain_alloc_mem;  // NodeInfo Requested / Allocatable
  double ratio;     // cpu amplification ratio
  int64_t cs_milli; // the node's allocated cpuset CPUs x 1000
  int64_t cs_off;   // Amplify(cs_milli) - cs_milli
  int32_t cpu_free; // CPUs available to cpuset pods on the node (-1 = no valid CPU topology)
  uint32_t cores;   // the node's CoresWord (Cfg.cores: core counts, CPUsPerCore, CPU bind label; ks_device.h)
};

struct NumaPolOut {
  uint32_t reasons;
  int32_t score;
  int64_t alloc[2][kNumaDev];  // the pod's NUMA allocation (cpu milli, memory)
  int32_t cpus[kNumaDev];      // cpu-bind pod: CPUs allocateCPUSet takes per allocated NUMA node
  uint32_t affinity;           // merged NUMANodeAffinity (0 = nil)
  bool admitted;               // Admit stored the affinity (DeviceShare's Filter / Score / Reserve read it)
  bool dev_done;               // reached DeviceShare's Allocate under the affinity (allow = affinity, or all if nil)
  bool dev_hit;                // ... and dev is its result (a hint's trial allocation, or computed without DEFER_DEV)
  DevOut dev;
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

// IterateBitMasks order (bitmask.go:206-222) for K <= 4 NUMA nodes: size 1..K, lexicographic index lists; mask i
// in bits [4i, 4i + 4) of the table
__device__ __forceinline__ uint64_t numa_mask_table(int K) {
  return K <= 1 ? 0x1ull : (K == 2 ? 0x321ull : (K == 3 ? 0x7653421ull : 0xFEDB7CA69538421ull));
}
__device__ __forceinline__ uint32_t numa_mask_at(uint64_t tab, int i) { return (uint32_t)(tab >> (4 * i)) & 0xFu; }

__device__ __forceinline__ bool numa_narrower(uint32_t a, uint32_t b) {
  const int ca = __builtin_popcount(a), cb = __builtin_popcount(b);
  return ca == cb ? a < b : ca < cb;
}

// DeviceShare's topology hints on one node (generateTopologyHints): hint positions 0: {id0}, 1: {id1}, 2: {id0, id1}
// over the device topology's (at most kDevHintIds) NUMA ids, which of them allocate, minAffinitySize and the
// number of identical resource lists (0 = the provider expresses no preference).
struct DevHints {
  int lists;
  int npos;
  int id0, id1;
  uint32_t ok;
  int minaff;
};

__device__ __forceinline__ uint32_t dev_hint_mask(const DevHints& h, int i) {
  const uint32_t pos = (uint32_t)i + 1u;
  return ((pos & 1u) ? (1u << h.id0) : 0u) | ((pos & 2u) ? (1u << h.id1) : 0u);
}

// numaTopology.nodes of a node's devices: the NUMA ids (a bit each) of the switches holding a device with a topology
template <typename V>
__device__ __forceinline__ uint32_t dev_topo_ids(const V& v) {
  const uint64_t topo = (uint64_t)v.tot(kDevTopoW), meta = (uint64_t)v.tot(kDevMetaW);
  uint32_t ids = 0;
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
  return ids;
}

template <typename V>
__device__ __forceinline__ DevHints dev_hints(const Cfg& c, const PodRec& p, const V& v) {
  DevHints h;
  h.lists = 0;
  h.npos = 0;
  h.id0 = h.id1 = 0;
  h.ok = 0;
  h.minaff = -1;
  if (!v.present()) return h;
  const uint64_t topo = (uint64_t)v.tot(kDevTopoW), meta = (uint64_t)v.tot(kDevMetaW);
  const uint32_t ids = dev_topo_ids(v);
  const int nid = __builtin_popcount(ids) < kDevHintIds ? __builtin_popcount(ids) : kDevHintIds;  // ks_load_* checks <= 2
  const uint32_t rest = ids & (ids - 1u);
  h.id0 = ids ? __builtin_ctz(ids) : 0;
  h.id1 = rest ? __builtin_ctz(rest) : 0;
  GpuReq g;
  if (dev_prepare(p, v, g)) return h;  // every mask returns before minAffinitySize is set: no preference
  // minors of each type on id0 / id1 (existing, with a topology)
  uint32_t gin0 = 0, gin1 = 0, rin0 = 0, rin1 = 0;
#pragma unroll
  for (int k = 0; k < kGpus; ++k) {
    const uint32_t pc = (uint32_t)(topo >> (4 * k)) & 0xFu;
    const bool ex = pc < 8u && (v.tot(k) != 0 || v.tot(kGpus + k) != 0 || v.tot(2 * kGpus + k) != 0);
    const int id = (int)((uint32_t)(meta >> (8 * (pc & 7u))) & 0xFu);
    gin0 |= (ex && nid >= 1 && id == h.id0) ? (1u << k) : 0u;
    gin1 |= (ex && nid >= 2 && id == h.id1) ? (1u << k) : 0u;
  }
#pragma unroll
  for (int j = 0; j < kRdma; ++j) {
    const uint32_t pc = (uint32_t)(topo >> (32 + 4 * j)) & 0xFu;
    const bool ex = pc < 8u && v.tot(kDevRdmaW + j) != 0;
    const int id = (int)((uint32_t)(meta >> (8 * (pc & 7u))) & 0xFu);
    rin0 |= (ex && nid >= 1 && id == h.id0) ? (1u << j) : 0u;
    rin1 |= (ex && nid >= 2 && id == h.id1) ? (1u << j) : 0u;
  }
  const bool has_gpu = (p.flags & kPodGpuReq) != 0, has_rdma = p.rdma > 0;
  h.npos = nid == 0 ? 0 : (nid == 1 ? 1 : 3);
  const DevFits fits = dev_fits(c, p, v, g);  // the trial allocations share the unrestricted per-minor fits
  for (int i = 0; i < h.npos; ++i) {
    const uint32_t pos = (uint32_t)i + 1u;
    const uint32_t gm = ((pos & 1u) ? gin0 : 0u) | ((pos & 2u) ? gin1 : 0u);
    const uint32_t rm = ((pos & 1u) ? rin0 : 0u) | ((pos & 2u) ? rin1 : 0u);
    if ((has_gpu && __builtin_popcount(gm) < g.desired) || (has_rdma && __builtin_popcount(rm) < g.rdesired)) continue;
    const int cnt = __builtin_popcount(pos);
    h.minaff = h.minaff < 0 ? (cnt < nid ? cnt : nid) : (cnt < h.minaff ? cnt : h.minaff);
    // the restriction to dev_hint_mask(h, i) keeps exactly the minors in gm / rm (dev_allowed)
    if (dev_fits_ok(fits, gm, rm)) h.ok |= 1u << i;
  }
  if (h.minaff >= 0)
    h.lists = (has_gpu ? ((g.has_core || g.desired > 1) ? 3 : 2) : 0) + (has_rdma ? 1 : 0);
  return h;
}

// Filter (FilterByNUMANode -> Admit -> allocateResources) and Score of one (pod, node) with a NUMA policy.
// dv: the node's device view when DeviceShare is a hint provider for this pod, else nullptr.  DEFER_DEV leaves
// DeviceShare's Allocate under the affinity to the caller (eval_full's DeviceShare Filter runs it with the same
// restriction; one inlined copy of dev_eval less), which then owns the score rule "a DeviceShare failure there
// returns before the NUMA score".
// Register-resident: hint sets are bit sets over mask indices, per-mask hint scores are packed bytes, the merge is
// three nested bit-set walks; no dynamically indexed local arrays (those would live in scratch memory).
// dhf: DeviceShare's hints from elsewhere (the commit kernel's hint wave, ks_pass.h), fetched after the NodeNUMAResource
// hints instead of computed first; NoDevHints = compute them here.
struct NoDevHints {};
template <typename T> struct LateDevHints { static constexpr bool value = true; };
template <> struct LateDevHints<NoDevHints> { static constexpr bool value = false; };

template <bool DEFER_DEV = false, typename V, typename DV, typename DHF = NoDevHints>
__device__ __forceinline__ NumaPolOut numa_policy_eval(const Cfg& c, const PodRec& p, const V& v, const NumaNodeCtx& nc,
                                                       const DV* dv, DHF dhf = DHF{}) {
  constexpr bool LATE = LateDevHints<DHF>::value;
  NumaPolOut o;
  o.reasons = 0;
  o.score = 0;
  o.affinity = 0;
  o.admitted = false;
  o.dev_done = o.dev_hit = false;
  o.dev = DevOut{0u, 0, 0u, 0u};
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
  // DeviceShare's hints first: its trial allocations are the register-heaviest part, nothing else is live yet
  DevHints dh;
  dh.lists = 0;
  dh.npos = 0;
  dh.ok = 0;
  dh.minaff = -1;
  if (!LATE && dv) dh = dev_hints(c, p, *dv);
  const int pol = v.policy();
  const uint32_t pres = v.present();
  // requestCPUBind / getCPUBindPolicy on this node (util.go:85-122): a node CPU bind policy makes a whole-CPU pod
  // cpu-bind with that policy required; else the pod's own policy, required or preferred (the Filter rejected a
  // fractional request and a conflicting policy before: numa_eval)
  const uint32_t label = c.cores ? cores_label(nc.cores) : 0u;
  const bool pbind = c.cpuset && (p.flags & KS_POD_CPU_BIND);
  const bool bind = pbind || (label != 0u && p.cpu > 0);
  const uint32_t rpol = label ? label
                              : ((pbind && (p.cpu_bind & KS_CPU_BIND_REQUIRED)) ? (p.cpu_bind & KS_CPU_BIND_POLICY_MASK) : 0u);
  const int32_t cpc = max((int32_t)cores_cpc(nc.cores), 1);
  // used (with the cpuset amplification) is re-read for the score; total and available stay live
  auto used_of = [&](int r, int k) -> int64_t {
    return (k < K && ((pres >> k) & 1u)) ? v.used(r, k) + (r == 0 ? v.off(k) : 0) : 0;
  };
  int64_t tot[2][kNumaDev], av[2][kNumaDev];
#pragma unroll
  for (int k = 0; k < kNumaDev; ++k) {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      tot[r][k] = k < K ? v.total(r, k) : 0;
      const int64_t a = tot[r][k] - used_of(r, k);
      av[r][k] = a < 0 ? 0 : a;
    }
    // trimNUMANodeResources (resource_manager.go:144-167): under a required policy a NUMA node offers at most the
    // CPUs the policy leaves there (for the hints and for the allocation)
    if (rpol && k < K && av[0][k] != 0) {
      const int64_t fk = (int64_t)numa_filtered(v.freew(k), rpol, cpc) * 1000;
      if (fk < av[0][k]) av[0][k] = fk;
    }
  }
  // options.requests: a cpu-bind pod's cpu amplified (hints and score); originalRequests for the allocation
  const int64_t req_cpu = (bind && nc.ratio > 1.0) ? (int64_t)::ceil((double)p.cpu * nc.ratio) : p.cpu;
  const int64_t req[2] = {req_cpu, p.mem};
  const bool want[2] = {p.cpu != 0, p.mem != 0};
  const uint64_t tab = numa_mask_table(K);
  const int nm = (1 << K) - 1;
  uint32_t lack[2] = {0u, 0u};
#pragma unroll
  for (int k = 0; k < kNumaDev; ++k)
#pragma unroll
    for (int r = 0; r < 2; ++r)
      if (k < K && av[r][k] == 0) lack[r] |= 1u << k;
  // NodeNUMAResource hints: bit i of hset[r] = mask i is a hint of resource r; one score per mask (byte i)
  uint32_t hset[2] = {0u, 0u};
  int min_size[2] = {K, K};
  uint64_t hsc_lo = 0, hsc_hi = 0;
  const bool nmost = c.numa_sc_most != 0;
  for (int i = 0; i < nm; ++i) {
    const uint32_t mk = numa_mask_at(tab, i);
    int64_t ts[2] = {0, 0}, fs[2] = {0, 0};
#pragma unroll
    for (int k = 0; k < kNumaDev; ++k)
      if ((mk >> k) & 1u)
#pragma unroll
        for (int r = 0; r < 2; ++r) {
          ts[r] += tot[r][k];
          fs[r] += av[r][k];
        }
    const uint64_t sc = (uint64_t)(uint32_t)numa_res_score(c, nmost, ts[0] - fs[0], ts[1] - fs[1], ts[0], ts[1], req[0], req[1]);
    if (i < 8) hsc_lo |= sc << (8 * i);
    else hsc_hi |= sc << (8 * (i - 8));
    const int cnt = __builtin_popcount(mk);
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      if (!want[r] || ts[r] < req[r] || (mk & lack[r])) continue;
      min_size[r] = cnt < min_size[r] ? cnt : min_size[r];
      if (fs[r] >= req[r]) hset[r] |= 1u << i;
    }
  }
  auto hscore = [&](int i) -> int32_t {
    return (int32_t)(((i < 8 ? (hsc_lo >> (8 * i)) : (hsc_hi >> (8 * (i - 8))))) & 0xFFu);
  };
  const bool single = pol == KS_NUMA_POLICY_SINGLE_NUMA_NODE;
  // The lists after filterProvidersHints (and filterSingleNumaHints), as bit sets of entries; bit kNil is the
  // list's nil entry.  A list holding only a preferred nil entry (a provider / resource without preference) is a
  // no-op in mergePermutation, so it stands for "no list".  Lists, outermost first: NodeNUMAResource cpu, memory,
  // then DeviceShare.  DeviceShare returns one identical list per requested device resource; the merge over L
  // identical lists equals the merge over one of them (checked exhaustively for K <= 2, the only case with device
  // hints: tools/merge_collapse_check.c), so one list is walked.
  constexpr int kNil = 15;
  uint32_t lb[2];
  bool lnp[2];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    lnp[r] = !want[r];
    if (!want[r]) {
      lb[r] = 1u << kNil;  // no hints for this resource (the provider returns none when neither is requested)
    } else if (hset[r] == 0) {
      lb[r] = single ? 0u : (1u << kNil);  // {nil, false}: "no possible NUMA affinities"
    } else {
      uint32_t s = hset[r];
      if (single) {
        uint32_t f = 0;
        for (int i = 0; i < nm; ++i) {
          const uint32_t mk = numa_mask_at(tab, i);
          if (((s >> i) & 1u) && __builtin_popcount(mk) == 1 && __builtin_popcount(mk) == min_size[r]) f |= 1u << i;
        }
        s = f;
      }
      lb[r] = s;
    }
  }
  if constexpr (LATE) {
    if (dv) dh = dhf();
  }
  uint32_t db = 1u << kNil;
  bool dnp = true;
  if (dh.lists) {
    dnp = false;
    if (dh.ok == 0) {
      db = single ? 0u : (1u << kNil);  // no allocating mask: {nil, false}
    } else {
      db = 0;
      for (int i = 0; i < dh.npos; ++i) {
        if (!((dh.ok >> i) & 1u)) continue;
        const int pc = __builtin_popcount(dev_hint_mask(dh, i));
        if (!single || (pc == 1 && pc == dh.minaff)) db |= 1u << i;
      }
    }
  }
  // mergeFilteredHints over the cartesian product, first list outermost (policy.go:129-226)
  const uint32_t dflt = (1u << K) - 1u;
  uint32_t best_mask = dflt;
  bool best_pref = false;
  int32_t best_score = 0;
  if (lb[0] && lb[1] && db) {
    for (uint32_t b0 = lb[0]; b0; b0 &= b0 - 1u) {
      const int e0 = __builtin_ctz(b0);
      const uint32_t m0 = e0 == kNil ? 0u : numa_mask_at(tab, e0);
      const bool h0 = e0 == kNil ? lnp[0] : __builtin_popcount(m0) == min_size[0];
      const int32_t s0 = e0 == kNil ? 0 : hscore(e0);
      for (uint32_t b1 = lb[1]; b1; b1 &= b1 - 1u) {
        const int e1 = __builtin_ctz(b1);
        const uint32_t m1 = e1 == kNil ? 0u : numa_mask_at(tab, e1);
        const bool h1 = e1 == kNil ? lnp[1] : __builtin_popcount(m1) == min_size[1];
        const int32_t s1 = e1 == kNil ? 0 : hscore(e1);
        for (uint32_t b2 = db; b2; b2 &= b2 - 1u) {
          const int e2 = __builtin_ctz(b2);
          const uint32_t m2 = e2 == kNil ? 0u : dev_hint_mask(dh, e2);
          const bool h2 = e2 == kNil ? dnp : __builtin_popcount(m2) == dh.minaff;
          // mergePermutation
          uint32_t merged = dflt, first = 0;
          bool pref = h0 && h1 && h2, have = false;
          if (m0) { first = m0; have = true; merged &= m0; }
          if (m1) { if (have && m1 != first) pref = false; if (!have) first = m1; have = true; merged &= m1; }
          if (m2) { if (have && m2 != first) pref = false; have = true; merged &= m2; }
          if (merged == 0) continue;
          int32_t msc = 0;
          if (m0 == merged && s0 > msc) msc = s0;
          if (m1 == merged && s1 > msc) msc = s1;
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
      }
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
  // the NUMA plugin's Allocate (tryBestToDistributeEvenly)
  if (affinity) {
    const int nb = __builtin_popcount(affinity);
    int ord0[kNumaDev];  // the affinity's NUMA ids ascending
    {
      uint32_t b = affinity;
#pragma unroll
      for (int i = 0; i < kNumaDev; ++i) {
        ord0[i] = b ? __builtin_ctz(b) : 0;
        b &= b - 1u;
      }
    }
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      if (!want[r]) continue;
      int ord[kNumaDev];
#pragma unroll
      for (int i = 0; i < kNumaDev; ++i) ord[i] = ord0[i];
      // sort.Slice insertion sort with less(i, j) comparing totalAvailable by slice position (fixed per position)
#pragma unroll
      for (int i = 1; i < kNumaDev; ++i) {
        bool go = i < nb;
#pragma unroll
        for (int j = i; j > 0; --j) {
          const int64_t aj = j < K ? av[r][j] : 0, ai = (j - 1) < K ? av[r][j - 1] : 0;
          go = go && aj < ai;
          if (go) {
            const int t = ord[j];
            ord[j] = ord[j - 1];
            ord[j - 1] = t;
          }
        }
      }
      int64_t q = r == 0 ? p.cpu : p.mem;  // originalRequests
#pragma unroll
      for (int i = 0; i < kNumaDev; ++i) {
        if (i >= nb) break;
        // splitQuantity (:285-300): a cpu-bind pod's cpu in whole CPUs (Quantity.Value() rounds up); under a required
        // FullPCPUs policy in whole cores
        int64_t split = q / (nb - i);
        if (r == 0 && bind)
          split = rpol == KS_CPU_BIND_FULL_PCPUS ? ((q + 999) / 1000) / cpc / (nb - i) * cpc * 1000
                                                 : ((q + 999) / 1000) / (nb - i) * 1000;
        int64_t a = 0;
#pragma unroll
        for (int k = 0; k < kNumaDev; ++k) a = ord[i] == k ? av[r][k] : a;
        const int64_t got = a > split ? split : a;
#pragma unroll
        for (int k = 0; k < kNumaDev; ++k)
          if (ord[i] == k) o.alloc[r][k] = got;
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
    // allocateCPUSet (:314-401): the node's available CPUs (under a required policy the ones it keeps), then per
    // allocated NUMA node min(available there, whole CPUs); a required policy's satisfiedRequiredCPUBindPolicy on the
    // union: FullPCPUs takes whole cores of a NUMA node only for a multiple of CPUsPerCore (SpreadByPCPUs' one CPU
    // per core always satisfies it)
    const int32_t need = pbind ? (int32_t)(p.cpu_bind >> 8) : (int32_t)(p.cpu / 1000);
    const int32_t have = !rpol ? nc.cpu_free
                               : (rpol == KS_CPU_BIND_FULL_PCPUS ? (int32_t)cores_full(nc.cores) * cpc
                                                                 : (int32_t)cores_any(nc.cores));
    if (nc.cpu_free < 0 || have < need) {
      o.reasons = KS_R_NUMA_CPUSET;
      return o;
    }
    if (any_alloc) {
      int32_t taken = 0;
      bool whole = true;
#pragma unroll
      for (int k = 0; k < kNumaDev; ++k) {
        if (o.alloc[0][k] == 0 && o.alloc[1][k] == 0) continue;
        const int32_t f = rpol ? numa_filtered(v.freew(k), rpol, cpc) : v.freec(k), w = (int32_t)(o.alloc[0][k] / 1000);
        o.cpus[k] = f < w ? f : w;
        taken += o.cpus[k];
        whole = whole && (o.cpus[k] % cpc == 0);
      }
      if (taken != need || (rpol == KS_CPU_BIND_FULL_PCPUS && !whole)) {
        o.reasons = KS_R_NUMA_CPUSET;
        return o;
      }
    }
  }
  // DeviceShare's Allocate with the affinity (with DEFER_DEV the caller's DeviceShare Filter, same restriction)
  if (dv) {
    o.dev_done = true;
    if (!DEFER_DEV) {
      o.dev = dev_eval<false>(c, p, *dv, nullptr, affinity ? affinity : ~0u);
      o.dev_hit = true;
      if (o.dev.reasons) {
        o.reasons = o.dev.reasons;
        return o;
      }
    }
  }
  int64_t trq[2] = {0, 0}, tal[2] = {0, 0};
#pragma unroll
  for (int k = 0; k < kNumaDev; ++k) {
    if (o.alloc[0][k] == 0 && o.alloc[1][k] == 0) continue;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      tal[r] += tot[r][k];
      trq[r] += used_of(r, k);
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
  nc.cores = r.cpu_cores;
  return nc;
}

}  // namespace ks
