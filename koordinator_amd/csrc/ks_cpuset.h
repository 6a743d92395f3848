// ks_cpuset.h — NodeNUMAResource cpuset allocation on the device (pkg/scheduler/plugins/nodenumaresource).
//
// A cpu-bind pod's node choice depends only on CPU counts (maxRefCount 1, topology policy None): the
// Filter checks the topology and the amplified request, Reserve checks |available| >= numCPUsNeeded
// (resourceManager.allocateCPUSet, resource_manager.go:314-335) and always takes exactly that many CPUs.
// So the sweep and the commit kernel track counts (cpu_free, the cpuset millicores A), and the CPU ids
// are chosen afterwards, per node in placement order, by the CPU accumulator below (takeCPUs,
// cpu_accumulator.go:86-232) in `cpuset_kernel` — one thread per node, CPU sets as 4 x u64 bit masks.
//
// Topology ids are mapped to dense indices in ascending id order, so "lower id first" tie-breaks are
// index compares.  Every sort of the accumulator has a total order, except the two len-only
// sort.Slice calls of the FullPCPUs fallback, which Go runs as a stable insertion sort for up to 12
// sockets; the restatement is stable.
#pragma once

#include "ks_device.h"

namespace ks {

constexpr int kCpuW = KS_CPU_WORDS;
constexpr int kMaxNumaNodes = 64;  // dense NUMA nodes / sockets per topology

struct CpuSet {
  uint64_t w[kCpuW];
};

__host__ __device__ inline CpuSet cs_zero() { return CpuSet{{0, 0, 0, 0}}; }
__host__ __device__ inline CpuSet cs_and(const CpuSet& a, const CpuSet& b) {
  return CpuSet{{a.w[0] & b.w[0], a.w[1] & b.w[1], a.w[2] & b.w[2], a.w[3] & b.w[3]}};
}
__host__ __device__ inline CpuSet cs_andnot(const CpuSet& a, const CpuSet& b) {
  return CpuSet{{a.w[0] & ~b.w[0], a.w[1] & ~b.w[1], a.w[2] & ~b.w[2], a.w[3] & ~b.w[3]}};
}
__host__ __device__ inline CpuSet cs_or(const CpuSet& a, const CpuSet& b) {
  return CpuSet{{a.w[0] | b.w[0], a.w[1] | b.w[1], a.w[2] | b.w[2], a.w[3] | b.w[3]}};
}
__host__ __device__ inline int cs_count(const CpuSet& a) {
  return __builtin_popcountll(a.w[0]) + __builtin_popcountll(a.w[1]) + __builtin_popcountll(a.w[2]) +
         __builtin_popcountll(a.w[3]);
}
__host__ __device__ inline bool cs_has(const CpuSet& a, int c) { return (a.w[c >> 6] >> (c & 63)) & 1ull; }
__host__ __device__ inline void cs_add(CpuSet& a, int c) { a.w[c >> 6] |= 1ull << (c & 63); }
// the lowest CPU of a non-empty set
__host__ __device__ inline int cs_first(const CpuSet& a) {
  for (int i = 0; i < kCpuW; ++i)
    if (a.w[i]) return i * 64 + __builtin_ctzll(a.w[i]);
  return -1;
}

// One CPU topology in dense form (host-built from ks_cpu_topology, read-only on the device).
struct CpuTopo {
  int32_t ncpus, ncores, nnodes, nsockets;
  int32_t cpc, cpn, cps;             // CPUsPerCore / CPUsPerNode / CPUsPerSocket (integer division)
  int32_t _pad;
  uint8_t core_of[KS_MAX_CPUS];      // dense core of each CPU
  uint8_t node_of[KS_MAX_CPUS];      // dense NUMA node of each CPU
  uint8_t sock_of[KS_MAX_CPUS];      // dense socket of each CPU
  uint8_t core_node[KS_MAX_CPUS];    // dense NUMA node / socket of each core
  uint8_t core_sock[KS_MAX_CPUS];
  uint8_t node_sock[kMaxNumaNodes];  // dense socket of each NUMA node
  CpuSet all;
  CpuSet core_mask[KS_MAX_CPUS];
  CpuSet node_mask[kMaxNumaNodes];
  CpuSet sock_mask[kMaxNumaNodes];
};

// Per-node CPU state ([npad] sets each), mutable by cpuset_kernel; cpu_free lives in DevNodes.
struct DevCpu {
  const CpuTopo* topo;     // [ntopo]
  const int32_t* topo_id;  // [npad], -1 = none
  CpuSet* allocated;       // [npad]
  CpuSet* excl_pcpu;       // [npad]
  CpuSet* excl_numa;       // [npad]
  const CpuSet* reserved;  // [npad]
  int64_t npad;
  int32_t ntopo;
};

// The accumulator state of one takeCPUs call (newCPUAccumulator, cpu_accumulator.go:247-286).
struct CpuAcc {
  const CpuTopo* t;
  CpuSet al;         // allocatableCPUs
  CpuSet res;        // result
  CpuSet exc_cores;  // bit k: dense core k in exclusiveInCores
  uint64_t exc_nodes;
  int32_t excl;      // request exclusive policy (KS_CPU_EXCL_*)
  bool most;         // NUMAMostAllocated
  int32_t needed;
};

__device__ inline CpuSet cpus_of_cores(const CpuTopo& t, const CpuSet& cores) {
  CpuSet m = cs_zero();
  for (int i = 0; i < kCpuW; ++i)
    for (uint64_t b = cores.w[i]; b; b &= b - 1) m = cs_or(m, t.core_mask[i * 64 + __builtin_ctzll(b)]);
  return m;
}
__device__ inline CpuSet cpus_of_nodes(const CpuTopo& t, uint64_t nodes) {
  CpuSet m = cs_zero();
  for (uint64_t b = nodes; b; b &= b - 1) m = cs_or(m, t.node_mask[__builtin_ctzll(b)]);
  return m;
}

// take (cpu_accumulator.go:288-302)
__device__ inline void acc_take(CpuAcc& a, const CpuSet& m) {
  a.res = cs_or(a.res, m);
  a.al = cs_andnot(a.al, m);
  a.needed -= cs_count(m);
  if (a.excl == KS_CPU_EXCL_PCPU_LEVEL || a.excl == KS_CPU_EXCL_NUMA_NODE_LEVEL) {
    for (int i = 0; i < kCpuW; ++i)
      for (uint64_t b = m.w[i]; b; b &= b - 1) {
        const int c = i * 64 + __builtin_ctzll(b);
        if (a.excl == KS_CPU_EXCL_PCPU_LEVEL) cs_add(a.exc_cores, a.t->core_of[c]);
        else a.exc_nodes |= 1ull << a.t->node_of[c];
      }
  }
}

// strategy order of free counts: NUMAMostAllocated ascending, else descending; returns x before y
__device__ inline int strat_cmp(bool most, int x, int y) { return x == y ? 0 : ((most ? x < y : x > y) ? -1 : 1); }

// the eligible CPUs of freeCPUsInNode / freeCPUs (PCPU- or NUMA-level exclusive filtering)
__device__ inline CpuSet excl_filtered(const CpuAcc& a, bool filter_exclusive) {
  if (!filter_exclusive) return a.al;
  if (a.excl == KS_CPU_EXCL_PCPU_LEVEL) return cs_andnot(a.al, cpus_of_cores(*a.t, a.exc_cores));
  if (a.excl == KS_CPU_EXCL_NUMA_NODE_LEVEL) return cs_andnot(a.al, cpus_of_nodes(*a.t, a.exc_nodes));
  return a.al;
}

// Take the first n CPUs of a group whose cores are ordered (count desc, core asc) with CPUs ascending
// (freeCoresInNode / freeCoresInSocket lists).  `grp` = the group's eligible CPUs, full = only full cores.
__device__ inline void take_cores_in_order(CpuAcc& a, const CpuSet& grp, bool full, int n) {
  const CpuTopo& t = *a.t;
  CpuSet m = cs_zero();
  int got = 0;
  for (int cnt = t.cpc; cnt >= 1 && got < n; --cnt) {
    if (full && cnt != t.cpc) break;
    for (int k = 0; k < t.ncores && got < n; ++k) {
      const CpuSet ck = cs_and(grp, t.core_mask[k]);
      if (cs_count(ck) != cnt) continue;
      for (int i = 0; i < kCpuW && got < n; ++i)
        for (uint64_t b = ck.w[i]; b && got < n; b &= b - 1) {
          cs_add(m, i * 64 + __builtin_ctzll(b));
          ++got;
        }
    }
  }
  acc_take(a, m);
}

// per-core eligible counts of a set, and the group sums over full (or all non-empty) cores
__device__ inline void group_core_sums(const CpuTopo& t, const CpuSet& e, bool full, bool by_socket, int* len) {
  const int ng = by_socket ? t.nsockets : t.nnodes;
  for (int g = 0; g < ng; ++g) len[g] = 0;
  for (int k = 0; k < t.ncores; ++k) {
    const int cnt = cs_count(cs_and(e, t.core_mask[k]));
    if (cnt == 0 || (full && cnt != t.cpc)) continue;
    len[by_socket ? t.core_sock[k] : t.core_node[k]] += cnt;
  }
}

// the full cores of a group as a CPU set
__device__ inline CpuSet group_full_cores(const CpuTopo& t, const CpuSet& e, const CpuSet& gm) {
  CpuSet m = cs_zero();
  for (int k = 0; k < t.ncores; ++k) {
    const CpuSet ck = cs_and(cs_and(e, gm), t.core_mask[k]);
    if (cs_count(ck) == t.cpc) m = cs_or(m, ck);
  }
  return m;
}

// freeCoresInNode(true, fe) (cpu_accumulator.go:370-455): the first node in order with enough CPUs
__device__ inline bool try_full_cores_in_node(CpuAcc& a, bool fe) {
  const CpuTopo& t = *a.t;
  const CpuSet e = (fe && a.excl == KS_CPU_EXCL_NUMA_NODE_LEVEL) ? cs_andnot(a.al, cpus_of_nodes(t, a.exc_nodes)) : a.al;
  int len[kMaxNumaNodes], sfree[kMaxNumaNodes];
  group_core_sums(t, e, true, false, len);
  for (int s = 0; s < t.nsockets; ++s) sfree[s] = cs_count(cs_and(e, t.sock_mask[s]));
  int best = -1;
  for (int n = 0; n < t.nnodes; ++n) {
    if (len[n] < a.needed || len[n] == 0) continue;
    if (best < 0) { best = n; continue; }
    int r = strat_cmp(a.most, len[n], len[best]);
    if (r == 0) r = strat_cmp(a.most, sfree[t.node_sock[n]], sfree[t.node_sock[best]]);
    if (r < 0) best = n;  // equal keys keep the lower node id
  }
  if (best < 0) return false;
  take_cores_in_order(a, cs_and(e, t.node_mask[best]), true, a.needed);
  return true;
}

// freeCoresInSocket(true) (:458-519): the first socket in order with enough CPUs
__device__ inline bool try_full_cores_in_socket(CpuAcc& a) {
  const CpuTopo& t = *a.t;
  int len[kMaxNumaNodes];
  group_core_sums(t, a.al, true, true, len);
  int best = -1;
  for (int s = 0; s < t.nsockets; ++s) {
    if (len[s] < a.needed || len[s] == 0) continue;
    if (best < 0 || strat_cmp(a.most, len[s], len[best]) < 0) best = s;
  }
  if (best < 0) return false;
  take_cores_in_order(a, cs_and(a.al, t.sock_mask[best]), true, a.needed);
  return true;
}

// The FullPCPUs fallback (:139-176): whole sockets of free cores by size, then single cores from the
// smallest remaining sockets.  Returns true when satisfied.
__device__ inline bool full_pcpus_fallback(CpuAcc& a) {
  const CpuTopo& t = *a.t;
  int len[kMaxNumaNodes];
  group_core_sums(t, a.al, true, true, len);
  int ord[kMaxNumaNodes], n = 0;
  for (int s = 0; s < t.nsockets; ++s)
    if (len[s] > 0) ord[n++] = s;
  // (len desc, socket asc): the stable len-desc sort of the (len strategy, socket) order
  for (int i = 1; i < n; ++i) {
    const int x = ord[i];
    int j = i - 1;
    while (j >= 0 && (len[ord[j]] < len[x] || (len[ord[j]] == len[x] && ord[j] > x))) { ord[j + 1] = ord[j]; --j; }
    ord[j + 1] = x;
  }
  int uns[kMaxNumaNodes], nu = 0;
  for (int i = 0; i < n; ++i) {
    const int s = ord[i];
    if (a.needed < len[s]) {
      uns[nu++] = s;
    } else {
      acc_take(a, group_full_cores(t, a.al, t.sock_mask[s]));
      if (a.needed < 1) return true;
    }
  }
  if (a.needed >= t.cpc) {
    // (len asc, socket asc) — the stable len-asc sort of the list above
    for (int i = 1; i < nu; ++i) {
      const int x = uns[i];
      int j = i - 1;
      while (j >= 0 && (len[uns[j]] > len[x] || (len[uns[j]] == len[x] && uns[j] > x))) { uns[j + 1] = uns[j]; --j; }
      uns[j + 1] = x;
    }
    for (int i = 0; i < nu; ++i) {
      const CpuSet g = cs_and(a.al, t.sock_mask[uns[i]]);
      for (int k = 0; k < t.ncores; ++k) {
        const CpuSet ck = cs_and(g, t.core_mask[k]);
        if (cs_count(ck) != t.cpc) continue;
        acc_take(a, ck);
        if (a.needed < 1) return true;
        if (a.needed < t.cpc) break;
      }
    }
  }
  return false;
}

// rank of CPU c among the set's CPUs of its core (0 = lowest)
__device__ inline int rank_in_core(const CpuTopo& t, const CpuSet& e, int c) {
  const CpuSet ck = cs_and(e, t.core_mask[t.core_of[c]]);
  int r = 0;
  for (int i = 0; i < (c >> 6); ++i) r += __builtin_popcountll(ck.w[i]);
  r += __builtin_popcountll(ck.w[c >> 6] & ((1ull << (c & 63)) - 1ull));
  return r;
}

// Take the first n CPUs of spreadCPUs(list) where list = the group's CPUs ascending, or, with
// extraction, the lowest eligible CPU of each core (extractCPU); spread only when len > CPUsPerCore.
__device__ inline void take_spread_ascending(CpuAcc& a, const CpuSet& g, bool extracted, int n) {
  const CpuTopo& t = *a.t;
  const int len = extracted ? 0 : cs_count(g);
  CpuSet m = cs_zero();
  int got = 0;
  if (extracted) {
    // one CPU per core in ascending CPU order: spread is the identity
    for (int i = 0; i < kCpuW && got < n; ++i)
      for (uint64_t b = g.w[i]; b && got < n; b &= b - 1) {
        const int c = i * 64 + __builtin_ctzll(b);
        if (rank_in_core(t, g, c) == 0) { cs_add(m, c); ++got; }
      }
  } else if (len <= t.cpc) {
    for (int i = 0; i < kCpuW && got < n; ++i)
      for (uint64_t b = g.w[i]; b && got < n; b &= b - 1) { cs_add(m, i * 64 + __builtin_ctzll(b)); ++got; }
  } else {
    for (int pass = 0; got < n && pass < 8; ++pass)
      for (int i = 0; i < kCpuW && got < n; ++i)
        for (uint64_t b = g.w[i]; b && got < n; b &= b - 1) {
          const int c = i * 64 + __builtin_ctzll(b);
          if (rank_in_core(t, g, c) == pass) { cs_add(m, c); ++got; }
        }
  }
  acc_take(a, m);
}

__device__ inline int distinct_cores(const CpuTopo& t, const CpuSet& g) {
  int k = 0;
  for (int i = 0; i < kCpuW; ++i)
    for (uint64_t b = g.w[i]; b; b &= b - 1)
      if (rank_in_core(t, g, i * 64 + __builtin_ctzll(b)) == 0) ++k;
  return k;
}

// freeCPUsInNode(fe) (:522-595)
__device__ inline bool try_cpus_in_node(CpuAcc& a, bool fe) {
  const CpuTopo& t = *a.t;
  const CpuSet e = excl_filtered(a, fe);
  int sfree[kMaxNumaNodes];
  for (int s = 0; s < t.nsockets; ++s) sfree[s] = cs_count(cs_and(e, t.sock_mask[s]));
  int best = -1, bfree = 0;
  for (int n = 0; n < t.nnodes; ++n) {
    const CpuSet g = cs_and(e, t.node_mask[n]);
    const int nfree = cs_count(g);
    if (nfree == 0) continue;
    const int len = fe ? distinct_cores(t, g) : nfree;
    if (len < a.needed) continue;
    int r = best < 0 ? -1 : strat_cmp(a.most, nfree, bfree);
    if (r == 0) r = strat_cmp(a.most, sfree[t.node_sock[n]], sfree[t.node_sock[best]]);
    if (r < 0) { best = n; bfree = nfree; }
  }
  if (best < 0) return false;
  take_spread_ascending(a, cs_and(e, t.node_mask[best]), fe, a.needed);
  return true;
}

// freeCPUsInSocket(fe) (:598-640)
__device__ inline bool try_cpus_in_socket(CpuAcc& a, bool fe) {
  const CpuTopo& t = *a.t;
  const CpuSet e = (fe && a.excl == KS_CPU_EXCL_PCPU_LEVEL) ? cs_andnot(a.al, cpus_of_cores(t, a.exc_cores)) : a.al;
  int best = -1, blen = 0;
  for (int s = 0; s < t.nsockets; ++s) {
    const CpuSet g = cs_and(e, t.sock_mask[s]);
    const int nfree = cs_count(g);
    if (nfree == 0) continue;
    const int len = fe ? distinct_cores(t, g) : nfree;
    if (len < a.needed) continue;
    if (best < 0 || strat_cmp(a.most, len, blen) < 0) { best = s; blen = len; }
  }
  if (best < 0) return false;
  take_spread_ascending(a, cs_and(e, t.sock_mask[best]), fe, a.needed);
  return true;
}

// freeCPUs(fe) + spreadCPUs + take one by one (:214-229, :650-770)
__device__ inline bool take_free_cpus(CpuAcc& a, bool fe, uint64_t* keys) {
  const CpuTopo& t = *a.t;
  const CpuSet e = excl_filtered(a, fe);
  int nfree[kMaxNumaNodes], sfree[kMaxNumaNodes], colo[kMaxNumaNodes];
  for (int n = 0; n < t.nnodes; ++n) nfree[n] = cs_count(cs_and(e, t.node_mask[n]));
  for (int s = 0; s < t.nsockets; ++s) {
    sfree[s] = cs_count(cs_and(e, t.sock_mask[s]));
    colo[s] = cs_count(cs_and(a.res, t.sock_mask[s]));
  }
  // cores ordered by (colocation desc, socket free by strategy, node free by strategy, core free asc,
  // socket asc, core asc) as one ascending 64-bit key
  int nc = 0, total = 0;
  for (int k = 0; k < t.ncores; ++k) {
    const int cnt = cs_count(cs_and(e, t.core_mask[k]));
    if (cnt == 0) continue;
    const int s = t.core_sock[k], n = t.core_node[k];
    const uint64_t kc = (uint64_t)(511 - colo[s]);
    const uint64_t ks = (uint64_t)(a.most ? sfree[s] : 511 - sfree[s]);
    const uint64_t kn = (uint64_t)(a.most ? nfree[n] : 511 - nfree[n]);
    uint64_t key = (kc << 50) | (ks << 41) | (kn << 32) | ((uint64_t)cnt << 24) | ((uint64_t)s << 16) | (uint64_t)k;
    int j = nc - 1;
    while (j >= 0 && keys[j] > key) { keys[j + 1] = keys[j]; --j; }
    keys[j + 1] = key;
    ++nc;
    total += cnt;
  }
  // spreadCPUs over the core-grouped list: pass p takes the p-th CPU of every core in order
  const bool spread = total > t.cpc;
  for (int pass = 0; pass < (spread ? t.cpc : 1); ++pass) {
    for (int i = 0; i < nc; ++i) {
      const int k = (int)(keys[i] & 0xFFFF);
      const CpuSet ck = cs_and(e, t.core_mask[k]);
      int r = 0;
      for (int w = 0; w < kCpuW; ++w)
        for (uint64_t b = ck.w[w]; b; b &= b - 1, ++r) {
          if (spread && r != pass) continue;
          if (a.needed >= 1) {
            CpuSet one = cs_zero();
            cs_add(one, w * 64 + __builtin_ctzll(b));
            acc_take(a, one);
          }
          if (a.needed < 1) return true;
        }
    }
  }
  return false;
}

// takeCPUs (cpu_accumulator.go:86-232) with maxRefCount 1; `keys` is scratch for 256 entries.
__device__ inline bool take_cpus(CpuAcc& a, int bind, uint64_t* keys) {
  const CpuTopo& t = *a.t;
  if (a.needed < 1) return true;
  if (a.needed > cs_count(a.al)) return false;
  const bool full = bind == KS_CPU_BIND_FULL_PCPUS;
  if (full || t.cpc == 1) {
    if (a.needed <= t.cpn) {
      if (try_full_cores_in_node(a, true)) return true;
      if (try_full_cores_in_node(a, false)) return true;
    }
    if (a.needed <= t.cps && try_full_cores_in_socket(a)) return true;
    if (full_pcpus_fallback(a)) return true;
  }
  if (!full) {
    if (a.needed <= t.cpn) {
      if (try_cpus_in_node(a, true)) return true;
      if (try_cpus_in_node(a, false)) return true;
    }
    if (a.needed <= t.cps) {
      if (try_cpus_in_socket(a, true)) return true;
      if (try_cpus_in_socket(a, false)) return true;
    }
  }
  if (take_free_cpus(a, true, keys)) return true;
  return take_free_cpus(a, false, keys);
}

// filterCPUsByRequiredCPUBindPolicy (resource_manager.go:595-627): FullPCPUs keeps the cores whose CPUs are all in
// `avail` (CPUsPerCore of them), SpreadByPCPUs the lowest CPU of `avail` in every core.
__device__ inline CpuSet filter_required(const CpuTopo& t, const CpuSet& avail, int policy) {
  CpuSet r = cs_zero();
  for (int k = 0; k < t.ncores; ++k) {
    const CpuSet m = cs_and(avail, t.core_mask[k]);
    const int c = cs_count(m);
    if (policy == KS_CPU_BIND_FULL_PCPUS) {
      if (c == t.cpc) r = cs_or(r, m);
    } else if (c > 0) {
      for (int w = 0; w < kCpuW; ++w)
        if (m.w[w]) {
          r.w[w] |= m.w[w] & (~m.w[w] + 1ull);
          break;
        }
    }
  }
  return r;
}

// NUMA node k's word of the NUMA-policy path (DevNuma.free, ks_numa.h): its available CPUs (bits 0-11), the cores
// of the NUMA node whose CPUs are all available (bits 12-21: filterCPUsByRequiredCPUBindPolicy FullPCPUs keeps them)
// and its cores with any available CPU (bits 22-31: SpreadByPCPUs keeps one CPU of each) -- trimNUMANodeResources
// and allocateCPUSet of a required CPU bind policy read the latter two (resource_manager.go:144-167, :322-330).
__device__ inline int32_t numa_free_word(const CpuTopo& t, const CpuSet& avail, int k) {
  if (k >= t.nnodes) return 0;
  const int32_t f = cs_count(cs_and(avail, t.node_mask[k]));
  uint32_t full = 0, any = 0;
  for (int c = 0; c < t.ncores; ++c) {
    if (cs_count(cs_and(t.core_mask[c], t.node_mask[k])) == 0) continue;  // (a core lies in one NUMA node)
    const int n = cs_count(cs_and(avail, t.core_mask[c]));
    full += n == t.cpc ? 1u : 0u;
    any += n > 0 ? 1u : 0u;
  }
  return (int32_t)((uint32_t)f | (full << 12) | (any << 22));
}

// CoresWord (ks_device.h) of a node whose available CPUs are `avail`.
__device__ inline uint32_t cores_word(const CpuTopo& t, const CpuSet& avail, uint32_t label) {
  uint32_t full = 0, any = 0;
  for (int k = 0; k < t.ncores; ++k) {
    const int c = cs_count(cs_and(avail, t.core_mask[k]));
    full += c == t.cpc ? 1u : 0u;
    any += c > 0 ? 1u : 0u;
  }
  return full | (any << kCoresAnyShift) | ((uint32_t)min(t.cpc, 31) << kCoresCpcShift) | (label << kCoresLabelShift);
}

}  // namespace ks
