// ks_topo.h — upstream PodTopologySpread and InterPodAffinity (kube-scheduler v1.24.15 plugins/podtopologyspread,
// plugins/interpodaffinity) on the device: the node counters and pod query terms of include/koordgpu.h
// ks_topology_args (compiled on the host by koordinator_amd/topology_plugins.py), the kernels that schedule a
// topology pod (KS_TOPO_DYN) alone against them, and the commit kernels' hooks.
//
// A topology pod's Filter needs per-domain sums over every eligible node (PreFilter) and its Score a normalization
// over every feasible node, so it cannot share a pass with other pods: the pass loop runs, before each regular pass,
// a topology step that acts only when the pod at the cursor is one --
//   eval_debug_kernel   every other plugin's Filter / Score on every node (ks_debug.hip, the ks_eval_pod path)
//   topo_filter_kernel  PreFilter domain sums (one workgroup, LDS) + both plugins' Filters, OR-ed into the reasons
//   topo_norm_kernel    the other plugins' normalizations, PodTopologySpread PreScore / Score / NormalizeScore and
//                       InterPodAffinity Score / NormalizeScore over the feasible nodes, the best node (max total,
//                       lowest index) as a one-candidate set
//   commit_kernel       (CommitArgs.topo = 2) admission + every Reserve on that node, the counters of the pod's
//                       properties
// -- and every regular pass ends before its first topology pod (CommitArgs.topo = 1).
#pragma once

#include <hip/hip_runtime.h>

#include "ks_device.h"

namespace ks {

// internal pod flag (PodRec.flags): the pod has topology query terms (KS_TOPO_DYN)
constexpr uint32_t kPodTopoDyn = 0x4000u;

// Per pending pod, queue order (staged with the pod columns): the query terms and properties.
struct __attribute__((aligned(16))) TopoRec {
  uint64_t term[KS_TOPO_TERMS];
  uint32_t props, flags;
  int32_t nterms, _pad;
};
static_assert(sizeof(TopoRec) == 80, "TopoRec layout");

// Node side: zonal domain, per-property counters ([p][npad]), the topologyNormalizingWeight table
// lw[s] = log(s + 2) for s in [0, nlw) (computed by the host's libm, the oracle's log)
struct DevTopo {
  int32_t* zone;
  int32_t* count;
  int64_t npad;
  const double* lw;
  int32_t nlw;
};

// The topology step's scratch (HBM, one per context)
struct TopoScratch {
  int64_t zsum[KS_TOPO_TERMS][KS_TOPO_ZONES];  // per term: the zone's counted pods over the term's eligible nodes
  unsigned long long zpres[KS_TOPO_TERMS];      // hard spread: zones with an eligible node
  int64_t best_total;                           // the chosen node's total (the pod's result score)
};

__device__ __forceinline__ int tp_kind(uint64_t w) { return (int)(w & 0xFF); }
__device__ __forceinline__ int tp_prop(uint64_t w) { return (int)((w >> 8) & 0xFF); }
__device__ __forceinline__ int tp_key(uint64_t w) { return (int)((w >> 16) & 0xFF); }
__device__ __forceinline__ uint32_t tp_flags(uint64_t w) { return (uint32_t)((w >> 24) & 0xFF); }
__device__ __forceinline__ int32_t tp_param(uint64_t w) { return (int32_t)(uint32_t)(w >> 32); }

// nodeaffinity.GetRequiredNodeAffinity(pod).Match(node) over the label dictionary (NodeAffinity's Filter test)
__device__ __forceinline__ bool tp_node_aff(const PodStat* s, uint64_t labels) {
  if (!s || s->nreq <= 0) return true;
  bool ok = false;
  for (int t = 0; t < KS_AFFINITY_TERMS; ++t) ok |= t < s->nreq && (labels & s->req[t]) == s->req[t];
  return ok;
}

// ---- commit kernel hooks (ks_pass.h commit_kernel, ks_mono.h commit_mono_kernel) ----

// The pods the pass commits: mode 1 ends it before its first topology pod (0: the kernel returns, the topology step
// of the next iteration takes that pod), mode 2 (the topology step's commit) is the pod at the cursor if it is one,
// else nothing; mode 3 (ks_assume) and 0 leave np.  Wave-uniform (every wave computes the same ballot).
template <typename A>
__device__ __forceinline__ int32_t topo_pass_pods(const A& a, int32_t cursor0, int32_t np) {
  if (a.topo == 0 || a.topo == 3) return np;
  const int lane = threadIdx.x & 63;
  const uint32_t f = lane < np ? a.topo_rec[cursor0 + lane].flags : 0u;
  const uint64_t dyn = __ballot((f & KS_TOPO_DYN) != 0u);
  if (a.topo == 2) return (dyn & 1ull) ? 1 : 0;
  return dyn ? (int32_t)(__ffsll((long long)dyn) - 1) : np;
}

// Write-back of one result: the counters of the placed pod's properties (NodeInfo.AddPod), its score (the topology
// step's total; a pod without query terms gets PodTopologySpread's constant 100 x weight on every node)
template <typename A>
__device__ __forceinline__ void topo_writeback(const A& a, int32_t pod, ks_result& r) {
  if (a.topo == 0 || r.status != KS_S_SCHEDULED || r.node < 0) return;
  const TopoRec& t = a.topo_rec[pod];
  if (a.topo == 2) r.score = *a.topo_best;
  else if (a.topo == 1 && !(t.flags & KS_TOPO_DYN)) r.score += a.topo_const;
  uint32_t m = t.props;
  while (m) {
    const int q = __ffs((int)m) - 1;
    m &= m - 1u;
    atomicAdd(a.topo_count + (int64_t)q * a.topo_npad + r.node, 1);
  }
}

// ---- topology step kernels (ks_topo.hip) ----

struct TopoKArgs {
  DevTopo t;
  const uint64_t* labels;  // DevNodes.labels (required node affinity of the spread constraints)
  const PodRec* recs;      // the stage, queue order
  const PodStat* stat;     // NULL = no node affinity
  const TopoRec* trec;
  const int32_t* cursor;   // the pod at *cursor, only if it is a topology pod; NULL = pod 0, always (ks_eval_pod)
  int32_t total_pods;
  int64_t n;
  uint32_t* reasons;       // [n] every plugin's KS_R_* (eval_debug_kernel's), topology bits OR-ed in
  int64_t* scores;         // [n][KS_NUM_SCORE_PLUGINS]
  int64_t* total;          // [n] weighted total, -1 = infeasible
  const int32_t* rraw;     // Reservation raw score, order rank (eval_debug_kernel's)
  const int32_t* rhi;
  const int32_t* draw;     // DeviceShare raw
  const int32_t* traw;     // TaintToleration raw
  const int32_t* araw;     // NodeAffinity raw
  int32_t norm_others;     // topo_norm_kernel also runs the DeviceShare / TaintToleration / NodeAffinity /
                           // Reservation normalizations (the batch step; ks_eval_pod launches their own kernels)
  int32_t dev_on, taint_on, aff_on, rsv_on;
  int64_t dev_w, taint_w, aff_w, rsv_w, spread_w, ipa_w;
  TopoScratch* scr;
  // the batch step's one-candidate set of the chosen node (commit_kernel's lists, pod 0 of a one-pod pass)
  uint32_t* cand_chunk;
  uint2* cand_t;
  int32_t* cand_count;
  uint64_t *cand_bound, *cand_top, *cand_second;
};

hipError_t launch_topo_filter(hipStream_t s, const TopoKArgs& a);
hipError_t launch_topo_norm(hipStream_t s, const TopoKArgs& a);

}  // namespace ks
