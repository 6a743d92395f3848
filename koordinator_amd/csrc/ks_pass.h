// ks_pass.h — the per-pass kernels that exist in one variant per plugin set (FEAT) and scalar-slot count
// (NSC): the node sweep and the sequential commit.  Each FEAT is compiled in its own translation unit
// (ks_variant.hip, -DKS_FEAT=F) so the variants build in parallel; koordgpu.hip launches them through
// the plain host wrappers declared at the end of this header.
#pragma once

#include <hip/hip_runtime.h>

#include <type_traits>

#include "ks_device.h"
#include "ks_rsv.h"
#include "ks_dev.h"
#include "ks_cpuset.h"
#include "ks_numa.h"
#include "ks_topo.h"

namespace ks {

// global candidate key of a chunk-local key: (score + 1) << 32 | ~node
__device__ __forceinline__ uint64_t local_gkey(uint32_t loc, int64_t chunk) {
  if (loc == 0) return 0;
  const int64_t node = chunk * 64 + (63 - (int64_t)(loc & 63u));
  return ((uint64_t)(loc >> 6) << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)node);
}

// ------------------------------------------------------------------------------------------
// sweep: per (pod, 64-node chunk) best and runner-up
// ------------------------------------------------------------------------------------------

struct SweepArgs {
  const DevNodes* __restrict__ dn;
  const DevRsv* __restrict__ rv;
  const DevDev* __restrict__ dv;
  const DevNuma* __restrict__ nv;
  // [3][64] normalization maxima per pod of the pass: (max raw << 32) | ~witness node of DeviceShare, TaintToleration,
  // NodeAffinity (kNormPlugins rows)
  unsigned long long* dev_M;
  int32_t phase;              // 0: reduce dev_M only (normalized plugins), 1: chunk keys
  const PodStat* __restrict__ pstat;  // TaintToleration / NodeAffinity per pod (Cfg.stat), queue order
  // DeviceShare without Reservation: phase 0 keeps each (pod, node)'s (feasible, Fit + LoadAware + NUMA
  // total, DeviceShare raw) here and phase 1 only applies the normalization ([64][dstride]); NULL = re-evaluate
  unsigned long long* dcache;
  int64_t dstride;
  Cfg c;
  const PodRec* __restrict__ pods;
  const int32_t* __restrict__ cursor;
  // [nchunks][64 pods]: {best, runner-up} local keys, chunk-major so that a work item's pods (consecutive lanes) write
  // consecutive words -- ppw x 8 B in one store instruction instead of ppw lone 8-byte writes into ppw rows
  uint2* __restrict__ out;
  int64_t n, nchunks;
  int64_t c0, c1;  // this shard's chunk range
  int32_t total_pods, batch, ppw;
  // Pipelined passes: the re-sweep of the chunks the previous commit wrote.  fix = that commit's
  // node list ([0] count, [1..64] nodes); only chunks of those nodes inside [c0, c1) are swept, and nothing
  // when the pass's speculative first pod (*cursor) is not where the real cursor (*fix_cursor) stands.
  // NULL = a full sweep.
  const int32_t* fix;
  const int32_t* fix_cursor;
  // Patched pipelined passes: instead of whole chunks, re-evaluate each pod's listed chunks that the
  // previous commit wrote (the fix list's chunks), in place in the pass's candidate lists (select_kernel ran on the
  // speculative sweep), and rebuild each pod's top into list_top (atomic max, zeroed by the commit that read it).
  // NULL = off.
  uint2* list_t;
  const uint32_t* list_chunk;
  const int32_t* list_count;
  const uint64_t* list_bound;
  unsigned long long* list_top;
  int32_t list_k;
};

// local key: ((total+1) << 6) | (63 - lane); 0 = no feasible node.  Max = best score, lowest lane.
// Fit + LoadAware (FEAT 0, C2 / C5) with up to two scalar slots: 4 waves per SIMD (<= 128 VGPRs; the kernel is
// latency-bound, more waves in flight hide the HBM round trips), the other variants as many as their registers allow
// (NSC 4 would spill inside the node loop at 128).
#ifndef KS_SWEEP_WAVES
#define KS_SWEEP_WAVES 4  // (profiles/r03_sweep_w4_ab.txt: C5 sweep 51.1 -> 43.1 us per launch)
#endif
template <int NSC, int FEAT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu((FEAT == 0 && NSC <= 2) ? KS_SWEEP_WAVES : 1)))
void sweep_kernel(SweepArgs a) {
  const int lane = threadIdx.x & 63;
  // wave-uniform work indices (readfirstlane: the compiler keeps the pod loop and its records scalar).
  // XCD-aware: blocks are dealt round-robin over the 8 XCDs, so block b works as virtual block
  // (b % 8) * (grid / 8) + b / 8 — each XCD gets a contiguous run of work items, i.e. every pod
  // group of a node chunk is swept on one XCD and the chunk's columns are fetched into one L2 only.
  // The host launches a multiple of 8 blocks.
  const uint32_t vblock = (blockIdx.x & 7u) * (gridDim.x >> 3) + (blockIdx.x >> 3);
  const int64_t wave = (int64_t)vblock * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
  if (a.list_t) {
    // one wave per (pod, list entry): a monotone commit only lowered the keys of the nodes it wrote, so an entry
    // whose chunk it did not write keeps its keys, a written one takes fresh keys, and a chunk outside the list
    // stays below the bound.  The pod's top is the largest listed key when that is at least the bound (else 0:
    // the best node may lie outside the list, and the commit's resolution then cuts the pass there).
    // A written chunk whose best and runner-up nodes were both left alone keeps them: their keys are exact, and
    // every other node's key was at most the runner-up's when swept (a half-written row included) and has only
    // dropped since.  Most waves have nothing to re-evaluate, so every input load is issued before the first use
    // (one HBM round trip instead of one per dependent read); the host launches >= kMaxBatch * K waves.
    const int32_t K = a.list_k;
    if (wave >= (int64_t)kMaxBatch * K) return;
    const int32_t p = (int32_t)(wave / K), e = (int32_t)(wave - (int64_t)p * K);
    const int32_t c_raw = *a.cursor, fc_raw = *a.fix_cursor, m_raw = a.fix[0];
    const int32_t wn_raw = a.fix[1 + lane];                 // the list has kMaxBatch node words
    const int32_t cnt_raw = a.list_count[p];
    const uint32_t ch_raw = a.list_chunk[p * K + e];
    const uint2 v = a.list_t[p * K + e];
    const uint64_t b = a.list_bound[p];
    const int32_t cursor = __builtin_amdgcn_readfirstlane(c_raw);
    if (cursor >= a.total_pods || __builtin_amdgcn_readfirstlane(fc_raw) != cursor) return;  // done / a bubble
    const int32_t np = min(a.batch, a.total_pods - cursor);
    if (p >= np || e >= __builtin_amdgcn_readfirstlane(cnt_raw)) return;
    const int32_t m = min(__builtin_amdgcn_readfirstlane(m_raw), kMaxBatch);
    const int32_t wn = lane < m ? wn_raw : -1;  // lane i: written node i
    const int64_t c = (int64_t)__builtin_amdgcn_readfirstlane(ch_raw);
    uint2 t = make_uint2(__builtin_amdgcn_readfirstlane(v.x), __builtin_amdgcn_readfirstlane(v.y));
    const int32_t nb = (int32_t)(c * 64 + 63 - (int64_t)(t.x & 63u));
    const int32_t nr = t.y ? (int32_t)(c * 64 + 63 - (int64_t)(t.y & 63u)) : -2;
    if (__ballot(wn >= 0 && (wn == nb || wn == nr))) {
      const int64_t node = c * 64 + lane;
      NodeReg<NSC> r;
      {
        const DevNodes d = *a.dn;
        load_node<NSC>(a.c, d, node, node < a.n, r);
      }
      const PodRec pod = load_pod_uniform(a.pods + cursor + p);
      EvalOut o = eval_full<NSC, false, true, FEAT>(
          a.c, pod, r, [&](auto&& f) { return f(RsvG<false>(*a.rv, node)); },
          [&]() { return DevGView{*a.dv, node}; }, [&]() { return NumaGView{*a.nv, node}; });
      const uint32_t key = o.reasons ? 0u : (((uint32_t)(key_total(a.c, o, NormM{0, 0, 0}) + 1) << 6) | (uint32_t)(63 - lane));
      t.x = wave_max_u32(key);
      t.y = wave_max_u32(key == t.x ? 0u : key);
      if (lane == 0) a.list_t[p * K + e] = t;
    }
    const uint64_t g = t.x ? local_gkey(t.x, c) : 0ull;
    if (lane == 0 && g && (b == 0ull || g >= b)) atomicMax(a.list_top + p, (unsigned long long)g);
    return;
  }
  const int32_t cursor = __builtin_amdgcn_readfirstlane(*a.cursor);
  if (cursor >= a.total_pods) return;
  // a topology pod at the cursor (ks_topo.h): the topology step takes it and this pass commits nothing
  if (__builtin_amdgcn_readfirstlane(a.pods[cursor].flags) & kPodTopoDyn) return;
  const int32_t np = min(a.batch, a.total_pods - cursor);
  const int32_t groups = (np + a.ppw - 1) / a.ppw;
  int64_t nitems = a.c1 - a.c0;
  if (a.fix) {
    if (__builtin_amdgcn_readfirstlane(*a.fix_cursor) != cursor) return;  // the next commit will not use it
    nitems = min(__builtin_amdgcn_readfirstlane(a.fix[0]), kMaxBatch);
  }
  const int64_t nwork = nitems * groups;
  // The work loop, instantiated separately for the full sweep and the re-sweep of a commit's chunks (FIX): a run-time
  // flag tested inside the loop was kept in a VGPR across it and spilled to scratch at 4 waves per SIMD (one scratch
  // write per wave, written back to HBM at the kernel's end: most of the launch's write traffic).
  auto items = [&](auto fixc) __attribute__((always_inline)) {
    constexpr bool FIX = decltype(fixc)::value;
    for (int64_t w = wave; w < nwork; w += nwaves) {
      // (32-bit, with the divisor opaque per item: a hoisted reciprocal would be one more value live across the loop)
      // (readfirstlane, not an "s" asm constraint: under SGPR pressure the allocator may keep the value in a VGPR)
      const int32_t gdiv = __builtin_amdgcn_readfirstlane(groups);
      const int64_t lc = (int64_t)((uint32_t)w / (uint32_t)gdiv);  // chunk within this shard's range (or fix-list entry)
      const int64_t c = FIX ? (int64_t)(__builtin_amdgcn_readfirstlane(a.fix[1 + lc]) >> 6) : a.c0 + lc;
      if (FIX && (c < a.c0 || c >= a.c1)) continue;  // another shard's chunk
      const int32_t g = (int32_t)(w - lc * groups);
      const int64_t node = c * 64 + lane;
      if ((FEAT & 4) && a.phase == 1 && a.dcache) {
        const int32_t p0 = g * a.ppw, p1 = min(np, p0 + a.ppw);
        uint32_t best = 0, second = 0;
        for (int32_t p = p0; p < p1; ++p) {
          const unsigned long long e = a.dcache[(size_t)p * a.dstride + node];
          EvalOut o{};
          o.total = (int32_t)(uint32_t)e;
          o.dev_raw = (int32_t)((e >> 32) & 0xFFFFull);
          const NormM M{(int32_t)(a.dev_M[p] >> 32), 0, 0};  // (no dcache with the dictionary-bit plugins)
          const uint32_t key = (e >> 63) ? (((uint32_t)(key_total(a.c, o, M) + 1) << 6) | (uint32_t)(63 - lane)) : 0u;
          const uint32_t m1 = wave_max_u32(key);
          const uint32_t m2 = wave_max_u32(key == m1 ? 0u : key);
          best = (lane == p) ? m1 : best;
          second = (lane == p) ? m2 : second;
        }
        if (lane >= p0 && lane < p1) a.out[(size_t)c * kMaxBatch + lane] = make_uint2(best, second);
        continue;
      }
      NodeReg<NSC> r;
      uint64_t st_hard = 0, st_soft = 0, st_lab = 0, st_port = 0;  // dictionary-bit plugin words (FEAT & 4 variants)
      {
        const DevNodes d = *a.dn;
        load_node<NSC>(a.c, d, node, node < a.n, r);
        if ((FEAT & 4) && a.c.stat && node < a.n) {
          st_hard = gld(d.taints_hard + node);
          st_soft = gld(d.taints_soft + node);
          st_lab = gld(d.labels + node);
          st_port = gld(d.host_ports + node);
        }
      }
      const int32_t p0 = g * a.ppw, p1 = min(np, p0 + a.ppw);
      uint32_t best = 0, second = 0;
      for (int32_t p = p0; p < p1; ++p) {
        const PodRec pod = load_pod_uniform(a.pods + cursor + p);
        EvalOut o = eval_full<NSC, false, true, FEAT>(
            a.c, pod, r, [&](auto&& f) { return f(RsvG<false>(*a.rv, node)); },
            [&]() { return DevGView{*a.dv, node}; }, [&]() { return NumaGView{*a.nv, node}; });
        if ((FEAT & 4) && a.c.stat) stat_eval(a.c, load_stat_uniform(a.pstat + cursor + p), st_hard, st_soft, st_lab, st_port, o);
        if ((FEAT & 4) && a.phase == 0) {
          // normalization maxima over the feasible nodes, witness = lowest index holding each
          const uint64_t wit = 0xFFFFFFFFull - (uint64_t)node;
          const uint64_t mk = o.reasons ? 0ull : (((uint64_t)(uint32_t)o.dev_raw << 32) | wit);
          const uint64_t m = wave_max_u64(mk);
          if (lane == 0 && m) atomicMax(a.dev_M + p, (unsigned long long)m);
          if (a.c.stat) {
            const uint64_t mt = wave_max_u64(o.reasons ? 0ull : (((uint64_t)(uint32_t)o.traw << 32) | wit));
            const uint64_t ma = wave_max_u64(o.reasons ? 0ull : (((uint64_t)(uint32_t)o.araw << 32) | wit));
            if (lane == 0 && mt) atomicMax(a.dev_M + kMaxBatch + p, (unsigned long long)mt);
            if (lane == 0 && ma) atomicMax(a.dev_M + 2 * kMaxBatch + p, (unsigned long long)ma);
          }
          if (a.dcache)
            a.dcache[(size_t)p * a.dstride + node] =
                (node < a.n && !o.reasons) ? ((1ull << 63) | ((unsigned long long)(uint32_t)o.dev_raw << 32) | (uint32_t)o.total)
                                           : 0ull;
          continue;
        }
        NormM M{0, 0, 0};
        if (FEAT & 4) {
          M.dev = (int32_t)(a.dev_M[p] >> 32);
          if (a.c.stat) {
            M.taint = (int32_t)(a.dev_M[kMaxBatch + p] >> 32);
            M.aff = (int32_t)(a.dev_M[2 * kMaxBatch + p] >> 32);
          }
        }
        const uint32_t key = o.reasons ? 0u : (((uint32_t)(key_total(a.c, o, M) + 1) << 6) | (uint32_t)(63 - lane));
        const uint32_t m1 = wave_max_u32(key);
        const uint32_t m2 = wave_max_u32(key == m1 ? 0u : key);
        best = (lane == p) ? m1 : best;
        second = (lane == p) ? m2 : second;
      }
      if ((FEAT & 4) && a.phase == 0) continue;
      if (lane >= p0 && lane < p1) {
        // (the lane's offset is rematerialised per work item: hoisted out of the loop it is one more value live across
        // it, which at 4 waves per SIMD the compiler spills to scratch -- one scratch write per wave, in HBM traffic)
        int32_t ln = lane;
        asm volatile("" : "+v"(ln));
        a.out[(size_t)c * kMaxBatch + ln] = make_uint2(best, second);
      }
    }
  };
  if (a.fix) items(std::true_type{});
  else items(std::false_type{});
}

struct CandSlot {  // one shard's select output inside the gather buffer (byte offsets)
  size_t chunk, t, count, total, top, bytes;
};

__host__ __device__ inline CandSlot cand_slot_layout(int32_t k) {
  CandSlot L;
  size_t o = 0;
  L.chunk = o;
  o += (size_t)kMaxBatch * k * 4;
  L.t = o;
  o += (size_t)kMaxBatch * k * 8;
  L.count = o;
  o += kMaxBatch * 4;
  L.total = o;
  o += kMaxBatch * 4;
  L.top = o;
  o += kMaxBatch * 8;
  L.bytes = (o + 255) / 256 * 256;
  return L;
}

// ------------------------------------------------------------------------------------------
// commit: sequential exact selection + Reserve, one wave, pass state resident in LDS
// ------------------------------------------------------------------------------------------
//
// Slot s (the s-th node touched in this pass) is an LDS row of score Terms + Filter headrooms,
// updated in place by every Reserve.  Building a slot and Reserve are lane-parallel (lane t owns
// term t).  For pod j the wave evaluates every slot at once (lane = slot; touched nodes exact)
// and takes the best untouched node from the candidate lists (snapshot keys, exact for untouched
// nodes).  Monotone profiles skip the slot evaluation whenever the pod's snapshot-best node is
// still untouched (a commit can only lower keys).  Pod j+1's quota admission and candidate
// resolution depend only on state pod j has finished changing, so they run right after pod j's
// Reserve, and the row of pod j+1's best untouched candidate is put in flight from HBM then.

constexpr int kQuotaLdsRows = 128;  // quota tables up to this size are cached in LDS for the pass
static_assert(kQuotaLdsRows < 0xFFFF && KS_QUOTA_DIMS <= 8, "commit_kernel's packed per-pod quota words");
// Threads of a commit workgroup: its waves load the pass into LDS together, then wave 0 alone runs the sequential
// loop.  The Fit + LoadAware [+ ElasticQuota] kernels fit 2 waves per SIMD (<= 256 VGPRs), so they load with 8 waves;
// the other variants use every register of a SIMD (1 wave each).
constexpr int kCommitThreads = 256;
#ifndef KS_COMMIT_THREADS0
#define KS_COMMIT_THREADS0 512
#endif
__host__ __device__ constexpr int commit_threads(int feat) { return feat == 0 ? KS_COMMIT_THREADS0 : 256; }

// fields of a raw node row (lane f of a row load holds field f)
enum RowField : int {
  RF_REQ_CPU = 0, RF_REQ_MEM = 1, RF_REQ_EPH = 2, RF_NZ_CPU = 3, RF_NZ_MEM = 4, RF_REQ_SC = 5,  // 5..8
  RF_TERM_CPU = 9, RF_TERM_MEM = 10, RF_PTERM_CPU = 11, RF_PTERM_MEM = 12, RF_POD_COUNT = 13,
  RF_ALLOC_CPU = 14, RF_ALLOC_MEM = 15, RF_ALLOC_EPH = 16, RF_ALLOC_SC = 17,  // 17..20
  RF_LA_ALLOC_CPU = 21, RF_LA_ALLOC_MEM = 22, RF_ALLOWED = 23, RF_LA_BITS = 24, RF_RSV_CLS = 25,
  RF_RSV_BEG = 26, RF_RSV_END = 27,  // the node's reservation range [beg, end) in the CSR table
  RF_NUMA_A = 28, RF_NUMA_OFF = 29,   // NodeNUMAResource cpuset milli-CPUs and amplification offset
  RF_NUMA_RATIO = 30, RF_CPU_FREE = 31,  // cpu amplification ratio (f64 bits), available CPUs (i32, -1 = no topology)
  RF_N = 32
};

// slot-row terms: score terms 0..10, then the Filter headrooms (Allocatable - Requested) stored as
// Terms too (only .h is read), so building a row and Reserve are one lane-uniform code path
enum SlotTerm : int {
  ST_CPU = 0, ST_MEM = 1, ST_EPH = 2, ST_SC = 3, ST_LCPU = 7, ST_LMEM = 8, ST_PLCPU = 9, ST_PLMEM = 10,
  ST_FREE_CPU = 11, ST_FREE_MEM = 12, ST_FREE_EPH = 13, ST_FREE_SC = 14,  // 14..17
  ST_NCPU = 18, ST_NMEM = 19,  // NodeNUMAResource: Requested (+ amplified cpuset part) cpu / memory
  ST_N = 20
};

struct __attribute__((aligned(16))) SlotRow {
  Term t[ST_N];
  uint32_t la_bits;
  int32_t fit_ws, allowed, pod_count;
};
// 656 B = 41 x 16 B (an odd number of 16 B units): lane = slot ds_read_b128 is conflict-free
static_assert(sizeof(SlotRow) == 656, "SlotRow layout");

// Device column of each row field (built by the host at ks_load_nodes).
struct RowCol {
  const void* p;
  int32_t width;
  int32_t _pad;
};

struct CommitArgs {
  const DevNodes* __restrict__ dn;
  const DevRsv* __restrict__ rv;
  const DevDev* __restrict__ dv;
  const DevNuma* __restrict__ nv;
  const unsigned long long* __restrict__ dev_M;  // [3][64] normalization maxima + witnesses (sweep phase 0)
  const PodStat* __restrict__ pstat;             // TaintToleration / NodeAffinity per pod (Cfg.stat), queue order
  Cfg c;
  const PodRec* __restrict__ pods;
  DevPodQuota pq;
  DevQuotas q;
  const RowCol* __restrict__ rowcols;  // [RF_N]
  int32_t* cursor;
  const uint32_t* __restrict__ cand_chunk;
  const uint2* __restrict__ cand_t;
  const uint64_t* __restrict__ cand_bound;
  const uint64_t* __restrict__ cand_top;
  const uint64_t* __restrict__ cand_second;  // [64] each pod's second-best key (select_kernel)
  const int32_t* __restrict__ cand_count;
  ks_result* results;
  unsigned long long* counters;  // [0] passes [1] cut passes [2] rescans [3] new-slot row misses [14] fast picks
  int64_t n, nchunks;
  int32_t total_pods, batch, k;
  int2* cpuset_list;   // (pod, node) of every cpu-bind Reserve, in placement order (ks_cpuset.h)
  int32_t* cpuset_n;
  uint32_t* cpuset_split;  // [pod] CPUs per NUMA node of a cpu-bind Reserve on a NUMA-policy node (0 = whole node)
  int64_t* numa_alloc;     // [pod][2][kNumaDev] NUMA-policy Reserve: the pod's NUMANodeResources (cpu milli, memory)
  int32_t force;           // ks_assume: the framework chose the node; no quota admission (Reserve only)
  int32_t rcap;        // reservations cached in LDS per slot (0 = none)
  int32_t rsv_bytes;   // LDS bytes of the slot reservation cache (commit_layout)
  int32_t dev_bytes;   // LDS bytes of the slot GPU state (commit_layout)
  int32_t numa_bytes;  // LDS bytes of the slot NUMA-node state (commit_layout)
  int32_t stat_lds;    // the pass's PodStat records are staged in LDS (else read from pstat in HBM)
  // Pipelined passes: the first pod the pass's sweep was run for; the pass is a no-op (a bubble) when
  // the real cursor is elsewhere (the previous pass was cut).  NULL = not pipelined.
  const int32_t* pipe_base;
  // [0] count, [1..64] nodes whose rows this pass wrote back (the next pass re-sweeps their chunks); NULL = not kept
  int32_t* carry;
  // Patched pipelined passes: the commit of pass k decides where pass k+2's speculative sweep starts,
  // from pass k+1's start (pipe_follow) and the cursor it leaves, into pipe_after (pass k's own start word, read by
  // nobody after this commit's prologue).  NULL = the select / patch kernels write it.
  const int32_t* pipe_follow;
  int32_t* pipe_after;
  // patched passes: cand_top is the list re-evaluation's atomic max, which the commit zeroes after reading
  unsigned long long* top_reset;
  // NUMA topology policy variants: Reserve's NodeNUMAResource / DeviceShare allocations on each pod's snapshot-best
  // nodes, computed before the commit by reserve_pre_kernel ([64][kPreRsvM]); NULL = the commit computes every Reserve
  const struct PreRsv* pre_rsv;
  // PodTopologySpread / InterPodAffinity (ks_topo.h): 0 off; 1 the pass ends before its first topology pod; 2 the
  // topology step's one-pod commit; 3 ks_assume.  Every placed pod's properties are counted on its node.
  int32_t topo;
  int32_t topo_const;        // 100 x the PodTopologySpread weight: the score of a pod without query terms
  const TopoRec* topo_rec;   // [pod] queue order
  const int32_t* topo_props; // the stage's property list (TopoRec.pbeg / nprops)
  int32_t* topo_count;       // [nprops][topo_npad]
  int64_t topo_npad;
  const long long* topo_best;  // mode 2: the topology step's total of the chosen node
};

// One pod's NodeNUMAResource + DeviceShare Reserve on one node of its snapshot ranking, computed on the snapshot state
// (what the commit's Reserve computes on the slot state of a node no earlier pod of the pass touched).
constexpr int kPreRsvM = 16;  // ranks per pod (C3: the winner is within the snapshot top-16 for 97.7% of pods)
struct __attribute__((aligned(16))) PreRsv {
  int32_t node;     // -1 = none
  uint32_t flags;   // bit 0: the node has a NUMA policy (npr valid), bit 1: npr.admitted
  uint32_t reasons, affinity;
  int64_t alloc[2][kNumaDev];
  int32_t cpus[kNumaDev];
  uint32_t gminors, rminors;
  int32_t _pad[2];
  int64_t g_core, g_mem, g_ratio, g_rdma;  // GpuReq per instance
};
static_assert(sizeof(PreRsv) == 144, "PreRsv layout");

// The first pod of the pass after next: pass k+1 commits iff it was swept for the pods at the cursor this commit
// leaves (rc), and then the pass after it starts behind its pods; otherwise pass k+1 is a bubble and k+2 starts at rc.
__device__ __forceinline__ void pipe_next(const CommitArgs& a, int32_t rc) {
  if (!a.pipe_after) return;
  const int32_t b1 = *a.pipe_follow;
  *a.pipe_after = (b1 == rc && b1 < a.total_pods) ? b1 + min(a.batch, a.total_pods - b1) : rc;
}

// Pipelined pass prologue: a pass whose sweep ran for other pods than the ones at the cursor does nothing (its
// successor's sweep starts at the cursor).  Returns true when the calling kernel must return.
__device__ __forceinline__ bool pipe_bubble(const CommitArgs& a, int32_t cursor0) {
  if (!a.pipe_base || __builtin_amdgcn_readfirstlane(*a.pipe_base) == cursor0) return false;
  if (threadIdx.x == 0) {
    a.carry[0] = 0;
    atomicAdd(&a.counters[4], 1ull);
    pipe_next(a, cursor0);
  }
  return true;
}

// Pipelined pass epilogue: the nodes of the pass's slots (lane s holds slot s's node)
__device__ __forceinline__ void pipe_carry(const CommitArgs& a, int32_t nslots, int32_t snode) {
  if (!a.carry) return;
  const int lane = threadIdx.x & 63;
  if (lane < nslots) a.carry[1 + lane] = snode;
  if (lane == 0) a.carry[0] = nslots;
}

// The pass's quota rows in LDS, sized by the loaded table (q <= kQuotaLdsRows rows): a view of pointers into the
// commit kernel's dynamic LDS (quota_lds).
struct QuotaRowsLds {
  int32_t* parent;
  uint32_t *limit_mask, *min_mask;
  int64_t *limit, *used, *min, *npused;
};

__host__ __device__ inline size_t quota_lds_bytes(int32_t q) {
  const size_t r = (size_t)(q > 0 ? q : 1);
  return (r * 12 + 15) / 16 * 16 + r * KS_QUOTA_DIMS * 32;
}

__device__ __forceinline__ QuotaRowsLds quota_lds(unsigned char* p, int32_t q) {
  const size_t r = (size_t)(q > 0 ? q : 1);
  QuotaRowsLds v;
  v.parent = reinterpret_cast<int32_t*>(p);
  v.limit_mask = reinterpret_cast<uint32_t*>(p + r * 4);
  v.min_mask = reinterpret_cast<uint32_t*>(p + r * 8);
  int64_t* w = reinterpret_cast<int64_t*>(p + (r * 12 + 15) / 16 * 16);
  v.limit = w;
  v.used = w + r * KS_QUOTA_DIMS;
  v.min = w + 2 * r * KS_QUOTA_DIMS;
  v.npused = w + 3 * r * KS_QUOTA_DIMS;
  return v;
}

// FEAT 0: the builder wave's descriptors, counts and ready mask
constexpr size_t kHelpBytes = (size_t)kMaxBatch * 8 + 16 + 16;
// NUMA policies + DeviceShare (the commit's LDS holds both slot caches): the helper waves' per-slot DevHints, four
// DeviceShare Filter / Score variants per slot (DevVar) and the request words
struct DevVar {
  uint32_t sel;  // bit 31: valid; GPU minors allowed in bits 0-7, RDMA minors in bits 8-15 (dev_allowed)
  uint32_t reasons;
  int32_t raw;
  uint32_t _pad;
};
constexpr int kDevVars = 4;
constexpr size_t kHelpHintBytes = (size_t)kMaxBatch * (24 + kDevVars * 16) + 64;
static_assert(sizeof(DevHints) == 24 && sizeof(DevVar) == 16, "help region");

struct CommitLayout {
  size_t rows, pods, res, raw, rawtop, rawrun, pqreq, cand_t, cand_chunk, scls, snuma, srcnt, srec, sdev, snp, quota, help,
      touched, total;
  bool hint;  // the helper waves' region is in the layout (the commit kernel runs them)
};

__host__ __device__ inline size_t align16(size_t x) { return (x + 15) / 16 * 16; }

// hint_ok: the variant runs the helper waves (NUMA policies + DeviceShare compiled in, (FEAT & 12) == 12)
__host__ __device__ inline CommitLayout commit_layout(int32_t k, int64_t nchunks, bool qc, size_t rsv_bytes = 0,
                                                      size_t dev_bytes = 0, size_t numa_bytes = 0,
                                                      int32_t qrows = kQuotaLdsRows, bool run = false,
                                                      bool hint_ok = false) {
  CommitLayout L;
  size_t o = 0;
  L.rows = o;
  o += (size_t)kMaxBatch * sizeof(SlotRow);
  L.pods = o;
  o += (size_t)kMaxBatch * sizeof(PodRec);
  L.res = o;
  o += align16((size_t)kMaxBatch * sizeof(ks_result));
  L.raw = o;
  o += 32 * 8;  // one raw row being turned into a slot row
  L.rawtop = o;
  o += (size_t)kMaxBatch * 32 * 8;  // raw row of each pod's snapshot-best node, prefetched per pass
  L.rawrun = o;
  // raw row of each pod's second-best node (its likely winner once the top is taken); Fit + LoadAware
  // [+ ElasticQuota] only (FEAT 0: the other plugin sets need the LDS for their slot state)
  if (run) o += (size_t)kMaxBatch * 32 * 8;
  L.pqreq = o;
  o += (size_t)kMaxBatch * KS_QUOTA_DIMS * 8;
  L.cand_t = o;
  o += (size_t)kMaxBatch * k * sizeof(uint2);
  L.cand_chunk = o;
  o += align16((size_t)kMaxBatch * k * 4);
  L.scls = o;
  o += (size_t)kMaxBatch * 8;  // per slot: owner classes of the node's matchable reservations
  L.snuma = o;
  o += (size_t)kMaxBatch * 32;  // per slot: NodeNUMAResource cpuset milli-CPUs, amplification offset, ratio, free CPUs
  L.srcnt = o;
  o += (size_t)kMaxBatch * 8;  // per slot: reservations cached (-1 = on the HBM table), CSR begin
  L.srec = o;
  o += align16(rsv_bytes);     // per slot: the node's reservations (RsvRec, rcap each)
  L.sdev = o;
  o += align16(dev_bytes);     // per slot: GPU totals / used [3][kGpus] + present flag
  L.snp = o;
  o += align16(numa_bytes);    // per slot: NUMA-node totals / used / offsets + policy, count, present (ks_numa.h)
  L.quota = o;
  if (qc) o += align16(quota_lds_bytes(qrows));
  L.help = o;
  // slot-row hand-off to the builder wave (FEAT 0): descriptors, issued count, done flag, ready mask; with both the
  // device and the NUMA slot caches, the helper waves' hints and DeviceShare variants when they still fit the CU's LDS
  L.hint = hint_ok && dev_bytes && numa_bytes && o + kHelpHintBytes + (size_t)nchunks * 8 <= (size_t)160 * 1024;
  o += L.hint ? kHelpHintBytes : kHelpBytes;
  L.touched = o;
  o += (size_t)nchunks * 8;  // u64 per chunk: lanes touched in this pass
  L.total = o;
  return L;
}

// ElasticQuota PreFilter (plugin.go:210-255, plugin_helper.go:281-319); lane d checks dimension d.
// The leaf's used/limit/mask reads are independent, so they are issued together.
template <typename P32, typename PU32, typename P64>
__device__ __forceinline__ uint32_t quota_admit(P32 parent, PU32 limit_mask, PU32 min_mask, P64 limit, P64 used,
                                                P64 minv, P64 npused, bool check_parent, int32_t quota,
                                                uint32_t flags, uint32_t pmask, int64_t req,
                                                bool skip_leaf = false) {
  const int lane = threadIdx.x & 63;
  const bool in_pod = lane < KS_QUOTA_DIMS && ((pmask >> lane) & 1u);
  const int ld = lane < KS_QUOTA_DIMS ? lane : 0;
  const size_t o = (size_t)quota * KS_QUOTA_DIMS + ld;
  if (!skip_leaf) {
    const uint32_t lm = limit_mask[quota];
    const int64_t u = used[o], l = limit[o];
    const bool bad = in_pod && ((lm >> lane) & 1u) && (req + u > l);
    if (__ballot(bad)) return KS_S_QUOTA;
  }
  if (flags & KS_POD_NONPREEMPTIBLE) {
    const uint32_t mm = min_mask[quota];
    const int64_t u = npused[o], m = minv[o];
    const bool bad = in_pod && ((mm >> lane) & 1u) && (req + u > m);
    if (__ballot(bad)) return KS_S_QUOTA_NONPREEMPTIBLE;
  }
  if (check_parent) {
    for (int32_t cur = parent[quota]; cur >= 0; cur = parent[cur]) {
      const size_t oc = (size_t)cur * KS_QUOTA_DIMS + ld;
      const bool bad = in_pod && ((limit_mask[cur] >> lane) & 1u) && (req + used[oc] > limit[oc]);
      if (__ballot(bad)) return KS_S_QUOTA | KS_S_QUOTA_PARENT;
    }
  }
  return 0;
}

// One row field of node `node`, lane f loading field f (4-byte columns zero-extended).  Two 32-bit loads and no branch:
// the high word of a 4-byte column re-reads the low word and is dropped when the value is used.  (A per-lane
// `w == 8 ? 64-bit load : 32-bit load + zero-extension` is a divergent branch whose extension sits right behind the
// 32-bit load, so the compiler waits for that load on the spot: every prefetch through it was a synchronous load.)
struct FieldLd {
  uint32_t lo, hi;
  bool wide;
};
__device__ __forceinline__ FieldLd field_issue(const void* p, int32_t w, int64_t node) {
  const uint32_t* q = reinterpret_cast<const uint32_t*>(static_cast<const char*>(p) + node * (int64_t)w);
  FieldLd f;
  f.wide = w == 8;
  f.lo = gld(q);
  f.hi = gld(q + (f.wide ? 1 : 0));
  return f;
}
__device__ __forceinline__ int64_t field_value(const FieldLd& f) {
  return (int64_t)(((uint64_t)(f.wide ? f.hi : 0u) << 32) | f.lo);
}
__device__ __forceinline__ int64_t load_field(const void* p, int32_t w, int64_t node) {
  return field_value(field_issue(p, w, node));
}

// NodeReg of one slot row (lane-private LDS reads).
template <int NSC>
__device__ __forceinline__ void slot_to_reg(const SlotRow& s, NodeReg<NSC>& r) {
  r.free_cpu = s.t[ST_FREE_CPU].h;
  r.free_mem = s.t[ST_FREE_MEM].h;
  r.free_eph = s.t[ST_FREE_EPH].h;
  r.t_cpu = s.t[ST_CPU];
  r.t_mem = s.t[ST_MEM];
  r.t_eph = s.t[ST_EPH];
#pragma unroll
  for (int k = 0; k < NSC; ++k) {
    r.free_sc[k] = s.t[ST_FREE_SC + k].h;
    r.t_sc[k] = s.t[ST_SC + k];
  }
  r.t_lcpu = s.t[ST_LCPU];
  r.t_lmem = s.t[ST_LMEM];
  r.t_plcpu = s.t[ST_PLCPU];
  r.t_plmem = s.t[ST_PLMEM];
  r.t_ncpu = s.t[ST_NCPU];
  r.t_nmem = s.t[ST_NMEM];
  r.numa_A = 0;
  r.numa_off = 0;
  r.la_bits = s.la_bits;
  r.fit_ws = s.fit_ws;
  r.allowed = s.allowed;
  r.pod_count = s.pod_count;
  r.pods_full = (int64_t)s.pod_count + 1 > (int64_t)s.allowed;
  r.valid = 1;
  r.rsv_cls = 0;
  r.cpu_cores = 0;
}

// Untouched-candidate resolution of one pod (lane k = candidate k), against the current touched masks.
struct Cands {
  uint64_t u;      // exact best untouched key of the lane's chunk (0 = none / unknown)
  uint64_t ub;     // upper bound when inexact (best and runner-up both touched)
  uint32_t chunk;
  bool exact, valid;
  uint64_t umax;   // wave max of the exact u
  bool fast;       // monotone profile and the pod's snapshot-best node is untouched
};

__device__ __forceinline__ Cands resolve_cands(const uint32_t* cand_chunk, const uint2* cand_t,
                                               const unsigned long long* touched, int32_t j, int32_t K,
                                               int32_t cnt) {
  const int lane = threadIdx.x & 63;
  Cands r;
  r.valid = lane < cnt;
  r.chunk = r.valid ? cand_chunk[j * K + lane] : 0u;
  const uint2 t = r.valid ? cand_t[j * K + lane] : make_uint2(0u, 0u);
  r.valid = r.valid && t.x != 0u;  // a patched list's chunk whose nodes all became infeasible
  const uint64_t tm = r.valid ? touched[r.chunk] : 0ull;
  r.u = local_gkey(t.x, r.chunk);
  r.fast = false;
  r.ub = 0;
  r.exact = r.valid;
  if (r.valid && ((tm >> (63 - (t.x & 63u))) & 1ull)) {  // chunk best touched
    if (t.y == 0) {
      r.u = 0;                                           // no other feasible node in the chunk
    } else if (!((tm >> (63 - (t.y & 63u))) & 1ull)) {
      r.u = local_gkey(t.y, r.chunk);                    // runner-up untouched: exact
    } else {
      r.exact = false;                                   // both touched: below the runner-up, unknown
      r.ub = local_gkey(t.y, r.chunk);
      r.u = 0;
    }
  }
  r.umax = wave_max_u64(r.exact ? r.u : 0ull);
  return r;
}

// Re-scan a candidate chunk's untouched nodes exactly for one pod (lane = node); touched nodes are
// covered by the slot evaluation.
template <int NSC, int FEAT>
__device__ __forceinline__ uint64_t rescan_untouched(const CommitArgs& a, const Cfg& cfg, const PodRec& pod,
                                                     int64_t chunk, uint64_t touched_mask, const NormM& M,
                                                     const PodStat* ps) {
  const int lane = threadIdx.x & 63;
  const int64_t node = chunk * 64 + lane;
  NodeReg<NSC> r;
  uint64_t sh = 0, ss = 0, sl = 0, sp = 0;
  {
    const DevNodes d = *a.dn;
    load_node<NSC>(cfg, d, node, node < a.n, r);
    if ((FEAT & 4) && cfg.stat && node < a.n) {
      sh = gld(d.taints_hard + node);
      ss = gld(d.taints_soft + node);
      sl = gld(d.labels + node);
      sp = gld(d.host_ports + node);
    }
  }
  EvalOut o = eval_full<NSC, false, false, FEAT>(
      cfg, pod, r, [&](auto&& f) { return f(RsvG<false>(*a.rv, node)); },
      [&]() { return DevGView{*a.dv, node}; }, [&]() { return NumaGView{*a.nv, node}; });
  if ((FEAT & 4) && cfg.stat) stat_eval(cfg, *ps, sh, ss, sl, sp, o);
  const bool skip = o.reasons || ((touched_mask >> lane) & 1ull);
  return wave_max_u64(skip ? 0ull : gkey(key_total(cfg, o, M), node));
}

// Prologue copies into LDS with every load of a thread issued before its first LDS store (kPro loads in flight per
// thread), so a pass's candidate lists, pod records and top-node raw rows arrive in a few HBM round trips rather
// than one per 256 elements.
constexpr int kPro = 8;
template <int NT = kCommitThreads, typename T>
__device__ __forceinline__ void lds_copy(T* dst, const T* src, int32_t n, int tid) {
  for (int32_t i0 = tid; i0 < n; i0 += NT * kPro) {
    T v[kPro];
#pragma unroll
    for (int u = 0; u < kPro; ++u) {
      const int32_t i = i0 + u * NT;
      if (i < n) v[u] = src[i];
    }
#pragma unroll
    for (int u = 0; u < kPro; ++u) {
      const int32_t i = i0 + u * NT;
      if (i < n) dst[i] = v[u];
    }
  }
}

// rawtop[p * 32 + f] = raw row field f of pod p's snapshot-best node (pods without a feasible node: untouched)
template <int NT = kCommitThreads>
__device__ __forceinline__ void lds_rawtop(int64_t* rawtop, const uint64_t* cand_top, const RowCol* rowcols, int32_t np,
                                           int tid) {
  const int32_t n = np * RF_N;
  for (int32_t i0 = tid; i0 < n; i0 += NT * kPro) {
    uint64_t t[kPro];
    RowCol rc[kPro];
#pragma unroll
    for (int u = 0; u < kPro; ++u) {
      const int32_t i = i0 + u * NT;
      const int32_t ii = i < n ? i : 0;  // (no branch: every load of the batch stays in flight together)
      const int32_t p = ii / RF_N, f = ii - p * RF_N;
      t[u] = i < n ? cand_top[p] : 0ull;
      rc[u] = rowcols[f];
    }
    FieldLd v[kPro];
#pragma unroll
    for (int u = 0; u < kPro; ++u) v[u] = field_issue(rc[u].p, rc[u].width, t[u] ? gkey_node(t[u]) : 0);
#pragma unroll
    for (int u = 0; u < kPro; ++u) {
      const int32_t i = i0 + u * NT;
      if (i < n && t[u]) {
        const int32_t p = i / RF_N, f = i - p * RF_N;
        rawtop[p * 32 + f] = field_value(v[u]);
      }
    }
  }
}

template <int NSC, bool QC, int FEAT>
__global__ __launch_bounds__(commit_threads(FEAT)) void commit_kernel(CommitArgs a) {
  constexpr int NT = commit_threads(FEAT);
  constexpr bool RSV = (FEAT & 1) != 0;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const int32_t K = a.k;
  const CommitLayout lay = commit_layout(K, a.nchunks, QC, (size_t)a.rsv_bytes, (size_t)a.dev_bytes, (size_t)a.numa_bytes, a.q.q,
                                         FEAT == 0, (FEAT & 12) == 12);
  SlotRow* rows = reinterpret_cast<SlotRow*>(smem_raw + lay.rows);
  PodRec* spods = reinterpret_cast<PodRec*>(smem_raw + lay.pods);
  ks_result* sres = reinterpret_cast<ks_result*>(smem_raw + lay.res);
  int64_t* raw = reinterpret_cast<int64_t*>(smem_raw + lay.raw);
  int64_t* rawtop = reinterpret_cast<int64_t*>(smem_raw + lay.rawtop);
  int64_t* pqreq = reinterpret_cast<int64_t*>(smem_raw + lay.pqreq);
  uint2* cand_t = reinterpret_cast<uint2*>(smem_raw + lay.cand_t);
  uint32_t* cand_chunk = reinterpret_cast<uint32_t*>(smem_raw + lay.cand_chunk);
  QuotaRowsLds qview = quota_lds(smem_raw + lay.quota, a.q.q);
  QuotaRowsLds* qlds = &qview;
  unsigned long long* touched = reinterpret_cast<unsigned long long*>(smem_raw + lay.touched);
  int64_t* rawrun = reinterpret_cast<int64_t*>(smem_raw + lay.rawrun);
  uint64_t* scls = reinterpret_cast<uint64_t*>(smem_raw + lay.scls);
  int64_t* snuma = reinterpret_cast<int64_t*>(smem_raw + lay.snuma);
  int32_t* srcnt = reinterpret_cast<int32_t*>(smem_raw + lay.srcnt);
  int32_t* srbeg = srcnt + kMaxBatch;
  constexpr int RD = 3 + NSC;
  RsvRec<RD>* srec = reinterpret_cast<RsvRec<RD>*>(smem_raw + lay.srec);
  constexpr bool DEV = (FEAT & 4) != 0;
  constexpr int DW = kDevTW;   // int64 words of one slot's device totals + topology (ks_dev.h)
  constexpr int DU = kDevQW;   // int64 words of its used amounts
  // word-major [w][kDevLdsStride] (slot s at column s): the slot-parallel reads (lane = slot) are
  // bank-conflict free, the lane = word row fills hit distinct bank pairs
  int64_t* sdev_tot = reinterpret_cast<int64_t*>(smem_raw + lay.sdev);
  int64_t* sdev_use = sdev_tot + kDevLdsStride * DW;
  int32_t* sdev_pres = reinterpret_cast<int32_t*>(sdev_use + kDevLdsStride * DU);
  int64_t* snp = reinterpret_cast<int64_t*>(smem_raw + lay.snp);  // [slot][kNumaSlotWords]
  // per slot: the node's dictionary-bit plugin words (taints hard, soft, labels, host ports -- the last one updated
  // by every Reserve of the pass): the last kMaxBatch * 32 B of the slot device region (dev_cache_bytes)
  // and before them the pass's PodStat records (Cfg.stat), and before those the normalization maxima table
  // ([kNormRows][kMaxBatch], DeviceShare variants): dev_cache_bytes
  // (the PodStat records only with CommitArgs.stat_lds)
  unsigned char* const sdev_end = smem_raw + lay.sdev + a.dev_bytes;
  uint64_t* sstat = reinterpret_cast<uint64_t*>(sdev_end - (size_t)kMaxBatch * 32);
  unsigned char* sp = a.c.stat ? reinterpret_cast<unsigned char*>(sstat) : sdev_end;
  PodStat* spstat = reinterpret_cast<PodStat*>(sp - (size_t)kMaxBatch * sizeof(PodStat));
  if (a.stat_lds) sp = reinterpret_cast<unsigned char*>(spstat);
  uint64_t* snorm = reinterpret_cast<uint64_t*>(sp - (size_t)kNormRows * kMaxBatch * 8);
  // Fit + LoadAware [+ ElasticQuota] (FEAT 0): wave 1 builds the slot rows of new slots whose node row was
  // prefetched (the pod's top or second-best node) while wave 0 goes on with the next pods; wave 0 waits for a
  // row only where it reads one (a later pod's slot evaluation, a Reserve onto the slot, the write-back).
#ifdef KS_NO_HELP
  constexpr bool HELP = false;  // (A/B builds)
#else
  constexpr bool HELP = FEAT == 0;
#endif
  int2* hdesc = reinterpret_cast<int2*>(smem_raw + lay.help);  // [issue order] {node, slot | pod << 8 | second << 16}
  int32_t* hpend = reinterpret_cast<int32_t*>(smem_raw + lay.help + (size_t)kMaxBatch * 8);  // descriptors issued
  int32_t* hdone = hpend + 1;                                                                // wave 0 is done
  unsigned long long* hready = reinterpret_cast<unsigned long long*>(smem_raw + lay.help + (size_t)kMaxBatch * 8 + 16);
  // NUMA topology policies + DeviceShare: wave 1 computes DeviceShare's topology hints of every touched slot for the
  // pod wave 0 is evaluating (lane = slot, the same dev_hints on the same LDS state), while wave 0 runs the other
  // plugins and the NodeNUMAResource hints; wave 0 takes them at the merge (numa_policy_eval's dhf)
  // (waves 2 and 3 compute DeviceShare's Filter / Score of every touched slot under the restrictions an affinity can
  // give: the device NUMA ids one by one, both, none -- wave 0 takes the one matching its merged affinity)
  constexpr bool HINTW = (FEAT & 12) == 12;
  const bool hintw = HINTW && lay.hint;  // (the layout holds the helper region)
  DevHints* shint = reinterpret_cast<DevHints*>(smem_raw + lay.help);                                // [slot]
  DevVar* sdv = reinterpret_cast<DevVar*>(smem_raw + lay.help + (size_t)kMaxBatch * 24);             // [k][slot]
  // seq, pod, n, done (wave 1), quit, done (wave 2), done (wave 3)
  int32_t* hw = reinterpret_cast<int32_t*>(smem_raw + lay.help + (size_t)kMaxBatch * (24 + kDevVars * 16));
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int32_t cursor0 = __builtin_amdgcn_readfirstlane(*a.cursor);
  if (cursor0 >= a.total_pods) {
    if (threadIdx.x == 0) pipe_next(a, cursor0);  // the queue is done: so are the speculative sweeps after it
    return;
  }
  if (pipe_bubble(a, cursor0)) return;
  const int32_t np = topo_pass_pods(a, cursor0, min(a.batch, a.total_pods - cursor0));
  if (np == 0) return;  // a topology pod at the cursor: the next topology step takes it
#ifdef KS_COMMIT_STAMPS
  uint64_t ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t tlast = __builtin_amdgcn_s_memtime();
#ifdef KS_SLOT_SPLIT
  uint64_t split[4] = {0, 0, 0, 0}, split_sink = 0;
#endif
#define KS_STAMP(i)                                    \
  do {                                                 \
    const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
    ph[i] += t_ - tlast;                               \
    tlast = t_;                                        \
  } while (0)
#else
#define KS_STAMP(i) \
  do {              \
  } while (0)
#endif
#ifdef KS_COMMIT_CAT
  // diagnostic build: whole-iteration cycles per pod category (0 quota-rejected, 1 fast, 2 slow onto a new slot,
  // 3 slow onto a touched slot, 4 unschedulable) in diag[0..4]; counts of categories 2 and 3 in diag[5..6]
  uint64_t ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t tcat = __builtin_amdgcn_s_memtime();
  int32_t cat = 0;
#define KS_CAT(c) cat = (c)
#else
#define KS_CAT(c) \
  do {            \
  } while (0)
#endif

  // ---- load the pass into LDS with all four waves (independent loads, one burst) ----
  lds_copy<NT>(cand_chunk, a.cand_chunk, np * K, tid);
  lds_copy<NT>(cand_t, a.cand_t, np * K, tid);
  for (int32_t i = tid; i < np * KS_QUOTA_DIMS; i += NT) {
    const int32_t p = i / KS_QUOTA_DIMS, dd = i - p * KS_QUOTA_DIMS;
    pqreq[i] = a.pq.req[dd][cursor0 + p];
  }
  if (DEV) {
    // the normalization maxima and the PodStat records in LDS (read per pod, not held in registers: these variants
    // are register-bound)
    lds_copy<NT>(snorm, reinterpret_cast<const uint64_t*>(a.dev_M), kNormRows * kMaxBatch, tid);
    if (a.stat_lds)
      lds_copy<NT>(reinterpret_cast<int64_t*>(spstat), reinterpret_cast<const int64_t*>(a.pstat + cursor0),
                   np * (int32_t)(sizeof(PodStat) / 8), tid);
  }
  {
    const int64_t* src = reinterpret_cast<const int64_t*>(a.pods + cursor0);
    int64_t* dst = reinterpret_cast<int64_t*>(spods);
    const int32_t words = np * (int32_t)(sizeof(PodRec) / 8);
    lds_copy<NT>(dst, src, words, tid);
  }
  for (int64_t c = tid; c < a.nchunks; c += NT) touched[c] = 0ull;
  // raw rows of every pod's snapshot-best node (the monotone fast path's winner) and second-best node (the usual
  // winner of a pod whose top an earlier pod took): all loads in flight together
  lds_rawtop<NT>(rawtop, a.cand_top, a.rowcols, np, tid);
  if (FEAT == 0) lds_rawtop<NT>(rawrun, a.cand_second, a.rowcols, np, tid);
  if (QC) {
    for (int32_t r = tid; r < a.q.q; r += NT) {
      qlds->parent[r] = a.q.parent[r];
      qlds->limit_mask[r] = a.q.limit_mask[r];
      qlds->min_mask[r] = a.q.min_mask[r];
    }
    for (int32_t i = tid; i < a.q.q * KS_QUOTA_DIMS; i += NT) {
      qlds->limit[i] = a.q.limit[i];
      qlds->used[i] = a.q.used[i];
      qlds->min[i] = a.q.min[i];
      qlds->npused[i] = a.q.npused[i];
    }
  }
  // wave 0, lane j: pod j's small per-pod values (read back with v_readlane in the loop)
  int32_t my_cnt = 0, my_quota = -1, my_cls = -1;
  uint32_t my_flags = 0, my_pmask = 0;
  // QC: the pod's leaf quota row's static words -- parent (0xFFFF = none) | limit_mask << 16 | min_mask << 24 (the
  // look-ahead's admission then reads only the per-dimension amounts from LDS, in one batch)
  uint32_t my_qmeta = 0xFFFFu;
  uint64_t my_bound = 0, my_top = 0, my_second = 0;
  if (tid < 64 && lane < np) {
    my_cnt = a.cand_count[lane];
    my_bound = a.cand_bound[lane];
    my_top = a.cand_top[lane];
    if (FEAT == 0) my_second = a.cand_second[lane];

    my_pmask = a.pq.mask[cursor0 + lane];
    my_quota = a.pods[cursor0 + lane].quota;
    if (QC && my_quota >= 0) {
      const int32_t pp = a.q.parent[my_quota];
      my_qmeta = (uint32_t)(pp < 0 ? 0xFFFF : pp) | ((a.q.limit_mask[my_quota] & 0xFFu) << 16) |
                 ((a.q.min_mask[my_quota] & 0xFFu) << 24);
    }
    my_flags = a.pods[cursor0 + lane].flags;
    if (RSV) my_cls = a.pods[cursor0 + lane].rsv_class;
  }
  // lane f < RF_N: the column of row field f
  const void* my_col = nullptr;
  int32_t my_w = 8;
  if (tid < RF_N) {
    my_col = a.rowcols[lane].p;
    my_w = a.rowcols[lane].width;
  }
  if (HELP && tid == 0) {
    *hpend = 0;
    *hdone = 0;
    *hready = 0ull;
  }
  if (hintw && tid < 7) hw[tid] = 0;
  __syncthreads();
  if (tid >= (HELP ? 128 : (hintw ? 256 : 64))) return;  // the other waves are done; wave 0 runs the sequential loop
  KS_STAMP(0);
  // Opaque copy of the profile: hipcc otherwise re-loads kernel-argument words inside the loop
  // (s_load + s_waitcnt lgkmcnt(0)), which would drain every LDS read in flight.
  // (The Reservation + DeviceShare variants run at the SGPR limit, where an "s" constraint can meet a value the
  // allocator keeps in a VGPR -- an illegal copy: they take readfirstlane, which stays legal.)
  Cfg cfg = a.c;
  int32_t Kc = K;
  {
    int32_t* w = reinterpret_cast<int32_t*>(&cfg);
    if constexpr ((FEAT & 5) == 5) {
#pragma unroll
      for (int i = 0; i < (int)(sizeof(Cfg) / 4); ++i) w[i] = __builtin_amdgcn_readfirstlane(w[i]);
      Kc = __builtin_amdgcn_readfirstlane(Kc);
    } else {
#pragma unroll
      for (int i = 0; i < (int)(sizeof(Cfg) / 4); ++i) asm volatile("" : "+s"(w[i]));
      asm volatile("" : "+s"(Kc));
    }
  }

  // ---- per-lane roles in slot construction and Reserve: lane t < ST_N owns slot term t ----
  // capacity / requested raw fields, the PodRec words of its Reserve delta (x1, x100), and whether a
  // zero capacity disables the term (score terms) or not (headrooms)
  // (t_pw100: the PodRec word of 100 x the request as f64; headroom lanes only use .h, so theirs is a dummy)
  int32_t t_cap = 0, t_req = 0, t_pw = 0, t_pw100 = 0;
  int32_t t_rdim = -1;  // reservation restore dimension of the lane's term: 0..6 Requested, 8/9 NonZero cpu/memory
  bool t_prod_only = false, t_score = true;
  switch (lane) {
    case ST_CPU: t_cap = RF_ALLOC_CPU; t_req = RF_NZ_CPU; t_pw = 3; t_pw100 = 12; t_rdim = 8; break;
    case ST_MEM: t_cap = RF_ALLOC_MEM; t_req = RF_NZ_MEM; t_pw = 4; t_pw100 = 13; t_rdim = 9; break;
    case ST_EPH: t_cap = RF_ALLOC_EPH; t_req = RF_REQ_EPH; t_pw = 2; t_pw100 = 14; t_rdim = 2; break;
    case ST_SC + 0: case ST_SC + 1: case ST_SC + 2: case ST_SC + 3:
      t_cap = RF_ALLOC_SC + (lane - ST_SC); t_req = RF_REQ_SC + (lane - ST_SC); t_pw = 7 + (lane - ST_SC); t_pw100 = 17 + (lane - ST_SC);
      t_rdim = 3 + (lane - ST_SC); break;
    case ST_LCPU: t_cap = RF_LA_ALLOC_CPU; t_req = RF_TERM_CPU; t_pw = 5; t_pw100 = 15; break;
    case ST_LMEM: t_cap = RF_LA_ALLOC_MEM; t_req = RF_TERM_MEM; t_pw = 6; t_pw100 = 16; break;
    case ST_PLCPU: t_cap = RF_LA_ALLOC_CPU; t_req = RF_PTERM_CPU; t_pw = 5; t_pw100 = 15; t_prod_only = true; break;
    case ST_PLMEM: t_cap = RF_LA_ALLOC_MEM; t_req = RF_PTERM_MEM; t_pw = 6; t_pw100 = 16; t_prod_only = true; break;
    case ST_FREE_CPU: t_cap = RF_ALLOC_CPU; t_req = RF_REQ_CPU; t_pw = 0; t_pw100 = 0; t_score = false; t_rdim = 0; break;
    case ST_FREE_MEM: t_cap = RF_ALLOC_MEM; t_req = RF_REQ_MEM; t_pw = 1; t_pw100 = 1; t_score = false; t_rdim = 1; break;
    case ST_FREE_EPH: t_cap = RF_ALLOC_EPH; t_req = RF_REQ_EPH; t_pw = 2; t_pw100 = 2; t_score = false; t_rdim = 2; break;
    case ST_FREE_SC + 0: case ST_FREE_SC + 1: case ST_FREE_SC + 2: case ST_FREE_SC + 3:
      t_cap = RF_ALLOC_SC + (lane - ST_FREE_SC); t_req = RF_REQ_SC + (lane - ST_FREE_SC);
      t_pw = 7 + (lane - ST_FREE_SC); t_pw100 = t_pw; t_score = false; t_rdim = 3 + (lane - ST_FREE_SC); break;
    case ST_NCPU: t_cap = RF_ALLOC_CPU; t_req = RF_REQ_CPU; t_pw = 0; t_pw100 = kPodWordHCpu; t_rdim = 0; break;
    case ST_NMEM: t_cap = RF_ALLOC_MEM; t_req = RF_REQ_MEM; t_pw = 1; t_pw100 = kPodWordHMem; t_rdim = 1; break;
    default: break;
  }
  constexpr int kLaneCounts = ST_N;  // lane: pod count / flags of the row
  const bool monotone = cfg.monotone != 0;

  if (HELP && tid >= 64) {
    // ---- wave 1: the slot-row builder (runs until wave 0 is done and every descriptor is built) ----
    int32_t next = 0;
    for (;;) {
      const int32_t pend =
          __builtin_amdgcn_readfirstlane(__hip_atomic_load(hpend, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
      if (next < pend) {
        const int2 d = hdesc[next];
        const int32_t w = __builtin_amdgcn_readfirstlane(d.y);
        const int32_t s = w & 0xFF, jj = (w >> 8) & 0xFF;
        const int64_t* src = (((w >> 16) & 1) ? rawrun : rawtop) + jj * 32;
        const int64_t* podw = reinterpret_cast<const int64_t*>(&spods[jj]);
        const uint32_t pflags = __builtin_amdgcn_readfirstlane(spods[jj].flags);
        const bool take = !t_prod_only || (pflags & KS_POD_PROD);
        const int64_t f_cap = src[t_cap], f_req = src[t_req], f_pw = podw[t_pw];
        const int64_t u_bits = src[RF_LA_BITS], u_allowed = src[RF_ALLOWED], u_pods = src[RF_POD_COUNT];
        const int64_t u_acpu = src[RF_ALLOC_CPU], u_amem = src[RF_ALLOC_MEM], u_aeph = src[RF_ALLOC_EPH];
        SlotRow* row = &rows[s];
        const int64_t cap = f_cap, req = f_req + (take ? f_pw : 0);
        if (lane < ST_N) {
          Term t;
          t.c = cap;
          t.h = cap - req + ((cap != 0 || !t_score) ? 0 : kNoCap);
          t.hd = cap != 0 ? (double)(cap - req) * 100.0 : 0.0;
          t.r = cap != 0 ? 1.0 / (double)cap : 0.0;
          row->t[lane] = t;
        } else if (lane == kLaneCounts) {
          row->la_bits = (uint32_t)u_bits;
          row->allowed = (int32_t)u_allowed;
          row->pod_count = (int32_t)u_pods + 1;
          row->fit_ws = (u_acpu != 0 ? cfg.fw_cpu : 0) + (u_amem != 0 ? cfg.fw_mem : 0) + (u_aeph != 0 ? cfg.fw_eph : 0);
        }
        if (lane == 0)
          __hip_atomic_fetch_or(hready, 1ull << s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        ++next;
        continue;
      }
      if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(hdone, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) &&
          next >= __builtin_amdgcn_readfirstlane(__hip_atomic_load(hpend, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)))
        break;
      __builtin_amdgcn_s_sleep(1);
    }
    return;
  }
  if (hintw && tid >= 64) {
    const int wv = tid >> 6;  // 1: hints, 2 / 3: DeviceShare variants 0-1 / 2-3
    // ---- wave 1: the hint wave (serves wave 0's requests in order until told to quit; an idle ~0.1 s, far
    // beyond any pass, also ends it: wave 0's wait is bounded the same way and then computes the hints itself) ----
    int32_t last = 0;
    uint32_t idle = 0;
    for (;;) {
      const int32_t sq = __builtin_amdgcn_readfirstlane(__hip_atomic_load(hw, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
      if (sq != last) {
        const int32_t jj = __builtin_amdgcn_readfirstlane(hw[1]), ns = __builtin_amdgcn_readfirstlane(hw[2]);
        if (lane < ns) {
          PodRec pod = spods[jj];
          pod.flags = __builtin_amdgcn_readfirstlane(pod.flags);
          pod.rsv_class = __builtin_amdgcn_readfirstlane(pod.rsv_class);
          const DevLView v{sdev_tot + lane, sdev_use + lane, (uint32_t)sdev_pres[lane]};
          if (wv == 1) {
            shint[lane] = dev_hints(cfg, pod, v);
          } else {
            const uint32_t ids = v.present() ? dev_topo_ids(v) : 0u;
            const uint32_t rest = ids & (ids - 1u);
            const uint32_t m0 = ids ? (1u << __builtin_ctz(ids)) : 0u, m1 = rest ? (1u << __builtin_ctz(rest)) : 0u;
#pragma unroll
            for (int q = 0; q < 2; ++q) {
              const int k = 2 * (wv - 2) + q;
              // the restrictions: {id0}, {id1}, {id0, id1} (with two ids), none
              const uint32_t allow = k == 0 ? m0 : (k == 1 ? m1 : (k == 2 ? (m1 ? (m0 | m1) : 0u) : ~0u));
              DevVar dv{0u, 0u, 0, 0u};
              if (allow) {
                uint32_t gin, rin;
                dev_allowed(v, allow, gin, rin);
                const DevOut d = dev_eval<false>(cfg, pod, v, nullptr, allow);
                dv.sel = (1u << 31) | (gin & 0xFFu) | ((rin & 0xFFu) << 8);
                dv.reasons = d.reasons;
                dv.raw = d.raw;
              }
              sdv[k * kMaxBatch + lane] = dv;
            }
          }
        }
        if (lane == 0)
          __hip_atomic_store(hw + (wv == 1 ? 3 : (wv == 2 ? 5 : 6)), sq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        last = sq;
        idle = 0;
        continue;
      }
      if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(hw + 4, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP))) break;
      if (++idle > (1u << 22)) break;
      __builtin_amdgcn_s_sleep(1);
    }
    return;
  }
  int32_t hseq = 0;      // hint-wave requests issued
  int32_t hn = 0;        // descriptors issued to wave 1
  uint64_t hown = 0;     // slots whose rows wave 0 built itself
  // wave 0: every row of `need` is built (wave 1's ready mask or its own)
  auto wait_rows = [&](uint64_t need) {
    if (!HELP || (hown & need) == need) return;
    for (;;) {
      const uint64_t r =
          readlane64(__hip_atomic_load(hready, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP), 0) | hown;
      if ((r & need) == need) break;
      __builtin_amdgcn_s_sleep(1);
    }
  };

  int32_t snode = -1;  // lane s: node of slot s
  int32_t nslots = 0;
  int32_t processed = np;
  uint32_t rescans = 0, misses = 0, fast = 0, prehits = 0;
#ifdef KS_SPEC
  // speculative raw row of the next pod's best untouched candidate (lane f = field f), two 32-bit halves in flight
  FieldLd spec_val{0u, 0u, false};
  int32_t spec_node = -1;
#endif

  auto admit = [&](int32_t j) -> uint32_t {
    const int32_t qrow = __builtin_amdgcn_readlane(my_quota, j);
    if (!cfg.quota_enable || qrow < 0) return 0u;
    const uint32_t flags = __builtin_amdgcn_readlane(my_flags, j);
    const uint32_t pmask = __builtin_amdgcn_readlane(my_pmask, j);
    const int64_t req = pqreq[j * KS_QUOTA_DIMS + (lane & (KS_QUOTA_DIMS - 1))];
    return QC ? quota_admit(qlds->parent, qlds->limit_mask, qlds->min_mask, qlds->limit, qlds->used, qlds->min,
                            qlds->npused, cfg.quota_parent, qrow, flags, pmask, req)
              : quota_admit(a.q.parent, a.q.limit_mask, a.q.min_mask, a.q.limit, a.q.used, a.q.min, a.q.npused,
                            cfg.quota_parent, qrow, flags, pmask, req);
  };
  uint32_t st_next = 0;
  int32_t par_next = -1;  // QC: the quota parent of the pod the look-ahead ran for (read with its admission)
  int64_t req_next = 0;   // QC: its request in dimension lane & 7 (the admission's read, reused by its usage update)
  // NUMA-policy variants: the node ids of the look-ahead pod's reserve_pre_kernel records (lane < kPreRsvM) and, with
  // Cfg.cores, the core word of its best untouched candidate; both loads in flight across the pod's slot evaluation
  int32_t pre_nodes = -1, cw_node = -1;
  uint32_t cw_next = 0;
  Cands cn{};
  // Reservation: set once a commit of this pass lowered a node's restored Requested (the class -1 fast path is off then)
  bool rsv_raised = false;
  auto lookahead = [&](int32_t j) {
    if ((FEAT & 8) && a.pre_rsv) pre_nodes = lane < kPreRsvM ? a.pre_rsv[j * kPreRsvM + lane].node : -1;
    // the fast path also holds for a pod without device requests when only DeviceShare's normalization
    // max made the profile non-monotone (its DeviceShare score is 0 on every node), and, with Reservation, for a pod
    // that matches no reservation: it sees every node through the base restore, whose Requested a commit only raises
    // (NodeInfo.AddPod) unless the commit shrank a reservation's remainder by more than the pod adds -- rsv_raised
    const bool mono = monotone || (cfg.monotone_nd && !(__builtin_amdgcn_readlane(my_flags, j) & kPodNormDyn)) ||
                      (RSV && cfg.monotone_rsv && !rsv_raised && __builtin_amdgcn_readlane(my_cls, j) < 0);
    const uint64_t top = mono ? readlane64(my_top, j) : 0ull;
    const int32_t tn = top ? (int32_t)gkey_node(top) : 0;
    if (QC) {
      // every LDS read of the admission and of the fast check issued together (one latency)
      const int32_t qrow = __builtin_amdgcn_readlane(my_quota, j);
      const bool has_q = cfg.quota_enable && qrow >= 0;
      const int32_t qr = has_q ? qrow : 0;
      const int ld = lane & (KS_QUOTA_DIMS - 1);
      const size_t o = (size_t)qr * KS_QUOTA_DIMS + ld;
      const int64_t req = pqreq[j * KS_QUOTA_DIMS + ld];
      req_next = req;
      const int64_t u = qlds->used[o], l = qlds->limit[o];
      // the leaf's min check (non-preemptible pods), in the same batch of reads; masks and parent from registers
      const int64_t nu = qlds->npused[o], mn = qlds->min[o];
      const uint32_t qm = __builtin_amdgcn_readlane(my_qmeta, j);
      const uint32_t lm = (qm >> 16) & 0xFFu, mm = qm >> 24;
      const int32_t par = (qm & 0xFFFFu) == 0xFFFFu ? -1 : (int32_t)(qm & 0xFFFFu);
      const uint64_t tw = touched[tn >> 6];
      st_next = 0;
      par_next = par;
      if (has_q && !a.force) {
        // quota_admit's three checks in its order: the leaf's limits, the leaf's min for a non-preemptible pod, the
        // ancestors' limits
        const uint32_t pmask = __builtin_amdgcn_readlane(my_pmask, j);
        const bool in_pod = lane < KS_QUOTA_DIMS && ((pmask >> lane) & 1u);
        const uint32_t flags = __builtin_amdgcn_readlane(my_flags, j);
        if (__ballot(in_pod && ((lm >> lane) & 1u) && (req + u > l))) {
          st_next = KS_S_QUOTA;
        } else if ((flags & KS_POD_NONPREEMPTIBLE) && __ballot(in_pod && ((mm >> lane) & 1u) && (req + nu > mn))) {
          st_next = KS_S_QUOTA_NONPREEMPTIBLE;
        } else if (cfg.quota_parent && par >= 0) {
          st_next = quota_admit(qlds->parent, qlds->limit_mask, qlds->min_mask, qlds->limit, qlds->used, qlds->min,
                                qlds->npused, true, qrow, 0u, pmask, req, /*skip_leaf=*/true);
        }
      }
      KS_STAMP(6);  // (diagnostic builds: the admission part of the look-ahead)
      if (st_next) return;
      if (top && !((tw >> (tn & 63)) & 1ull)) {
        cn.fast = true;  // its row is in rawtop[j]
        cn.umax = top;
        return;
      }
    } else {
      st_next = a.force ? 0u : admit(j);
      KS_STAMP(6);
      if (st_next) return;
      if (top && !((touched[tn >> 6] >> (tn & 63)) & 1ull)) {
        cn.fast = true;
        cn.umax = top;
        return;
      }
    }
    cn = resolve_cands(cand_chunk, cand_t, touched, j, Kc, __builtin_amdgcn_readlane(my_cnt, j));
    if ((FEAT & 2) && cfg.cores && cn.umax) {
      cw_node = (int32_t)gkey_node(cn.umax);
      cw_next = gld(a.dn->cpu_cores + cw_node);
    }
#ifdef KS_SPEC
    if (cn.umax) {
      const int32_t node = (int32_t)gkey_node(cn.umax);
      // (the top's and the second-best node's rows are in LDS already)
      if (node != spec_node && node != (int32_t)gkey_node(readlane64(my_top, j)) &&
          node != (int32_t)gkey_node(readlane64(my_second, j))) {
        spec_node = node;
        if (lane < RF_N) spec_val = field_issue(my_col, my_w, node);
      }
    }
#endif
  };
  lookahead(0);
  KS_STAMP(1);
#ifdef KS_COMMIT_CAT
  tcat = __builtin_amdgcn_s_memtime();
#endif

  for (int32_t j = 0; j < np; ++j) {
    const uint32_t st = st_next;
    const Cands cj = cn;
    const int32_t qpar = par_next;
    const int64_t qreq_j = req_next;
    KS_CAT(0);
    if (st) {
      if (lane == 0) sres[j] = ks_result{-1, st, 0, -1, 0, 0, 0};
      goto next_pod;
    }
    {
    uint64_t best;
    NormM Muse{0, 0, 0};  // normalization maxima used for this pod
    // TaintToleration / NodeAffinity / NodePorts inputs (Cfg.stat), in LDS when they fit
    const PodStat& pst = a.stat_lds ? spstat[j] : a.pstat[cursor0 + j];
    if (cj.fast) {
      best = cj.umax;  // the snapshot-best node is untouched: commits only lower keys, so it wins
      ++fast;
      KS_CAT(1);
      KS_STAMP(2);
    } else {
      // pod j: LDS broadcast into VGPRs; flags scalar so the plugin branches stay wave-uniform
      PodRec pod = spods[j];
      pod.flags = __builtin_amdgcn_readfirstlane(pod.flags);
      pod.rsv_class = __builtin_amdgcn_readfirstlane(pod.rsv_class);
      // ---- every touched node exactly (lane = slot), untouched from the candidates ----
      uint64_t key_mod = 0;
      EvalOut o{};
      bool feas = false;
      bool unk = false;  // Cfg.cores: feasible only if the slot's core counts, changed in this pass, allow it
      bool unk_pol = false;  // ... a NUMA-policy slot whose evaluation depends on them (numa_policy_eval)
      wait_rows(nslots >= 64 ? ~0ull : ((1ull << nslots) - 1));
      bool use_hw = false;
      if constexpr (HINTW) {
        use_hw = hintw && cfg.dev && cfg.numa_pol && (pod.flags & kPodHasGpu) && !(pod.flags & kPodReqZero) && nslots > 0;
        if (use_hw) {
          ++hseq;
          if (lane == 0) {
            hw[1] = j;
            hw[2] = nslots;
            __hip_atomic_store(hw, hseq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
          }
        }
      }
#ifdef KS_SLOT_SPLIT
      // diagnostic build (with KS_COMMIT_STAMPS): the slot evaluation's parts timed separately, each run once more on
      // the same slots ahead of the real evaluation; cycles in diag[0] Fit / LoadAware / NUMA policy None,
      // diag[1] the NUMA policy path (with DeviceShare's hints), diag[2] DeviceShare's Filter / Score
      if (lane < nslots) {
        NodeReg<NSC> r;
        slot_to_reg<NSC>(rows[lane], r);
        r.numa_A = snuma[4 * lane];
        r.numa_off = snuma[4 * lane + 1];
        r.numa_ratio = __longlong_as_double(snuma[4 * lane + 2]);
        r.cpu_free = (int32_t)snuma[4 * lane + 3];
        uint64_t t0 = __builtin_amdgcn_s_memtime();
        EvalOut e = eval_pod_node<NSC, false>(cfg, pod, r);
        if ((FEAT & 2) && cfg.numa) numa_eval<NSC, false>(cfg, pod, r, e);
        split_sink ^= (uint64_t)e.total ^ e.reasons;
        uint64_t t1 = __builtin_amdgcn_s_memtime();
        split[0] += t1 - t0;
        const DevLView dvl{sdev_tot + lane, sdev_use + lane, (uint32_t)sdev_pres[lane]};
        if ((FEAT & 8) && cfg.numa_pol && !(pod.flags & kPodReqZero)) {
          const NumaLView nl{snp + lane * kNumaSlotWords};
          if (nl.policy() != 0) {
            const NumaPolOut pr = (DEV && cfg.dev && (pod.flags & kPodHasGpu))
                                      ? numa_policy_eval<true>(cfg, pod, nl, numa_node_ctx<NSC>(r), &dvl)
                                      : numa_policy_eval(cfg, pod, nl, numa_node_ctx<NSC>(r), (const DevLView*)nullptr);
            split_sink ^= (uint64_t)pr.score ^ pr.affinity ^ pr.reasons;
          }
        }
        uint64_t t2 = __builtin_amdgcn_s_memtime();
        split[1] += t2 - t1;
        if (DEV && cfg.dev && (pod.flags & kPodHasGpu)) {
          const DevOut d = dev_eval<false>(cfg, pod, dvl, nullptr, ~0u);
          split_sink ^= (uint64_t)d.raw ^ d.reasons;
        }
        uint64_t t3 = __builtin_amdgcn_s_memtime();
        split[2] += t3 - t2;
        if ((FEAT & 8) && DEV && cfg.dev && (pod.flags & kPodHasGpu)) {
          const DevHints dh = dev_hints(cfg, pod, dvl);
          split_sink ^= (uint64_t)dh.ok ^ dh.minaff ^ dh.lists;
        }
        split[3] += __builtin_amdgcn_s_memtime() - t3;
      }
#endif
      if (lane < nslots) {
        // the dictionary-bit plugins first: three words out, their temporaries dead before eval_full's peak
        EvalOut so{};
        if (DEV && cfg.stat)
          stat_eval(cfg, pst, sstat[4 * lane], sstat[4 * lane + 1], sstat[4 * lane + 2], sstat[4 * lane + 3], so);
        NodeReg<NSC> r;
        slot_to_reg<NSC>(rows[lane], r);
        r.rsv_cls = scls[lane];
        r.numa_A = snuma[4 * lane];
        r.numa_off = snuma[4 * lane + 1];
        r.numa_ratio = __longlong_as_double(snuma[4 * lane + 2]);
        r.cpu_free = (int32_t)snuma[4 * lane + 3];
        uint32_t cw = 0;
        if ((FEAT & 2) && cfg.cores) {
          // a cpu-bind Reserve on the slot in this pass moved its core counts (the CPU ids come after the pass):
          // evaluate optimistically and cut the pass if that decides the pod
          cw = (uint32_t)((uint64_t)snuma[4 * lane + 3] >> 32);
          r.cpu_cores = (cw & kCoresDirty) ? (cw | kCoresCount | (kCoresCount << kCoresAnyShift)) : cw;
        }
        auto rsvf = [&](auto&& f) {
          const int32_t c = srcnt[lane];
          if (c >= 0) return f(RsvL<RD>{srec + lane * a.rcap, c, srbeg[lane], a.rv});
          return f(RsvG<true>(*a.rv, snode));
        };
        auto devf = [&]() { return DevLView{sdev_tot + lane, sdev_use + lane, (uint32_t)sdev_pres[lane]}; };
        auto numaf = [&]() { return NumaLView{snp + lane * kNumaSlotWords}; };
        if constexpr (HINTW) {
          // the slot's DeviceShare hints: the hint wave's (use_hw), else computed here
          auto dhf = [&]() -> DevHints {
            if (use_hw) {
              for (uint32_t it = 0; it <= (1u << 22); ++it) {
                if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(hw + 3, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) ==
                    hseq)
                  return shint[lane];
                __builtin_amdgcn_s_sleep(1);
              }
            }
            return dev_hints(cfg, pod, DevLView{sdev_tot + lane, sdev_use + lane, (uint32_t)sdev_pres[lane]});
          };
          // the slot's DeviceShare Filter / Score under `allow`: a helper wave's variant with the same allowed minors (the
          // result depends on the restriction only through them), else computed here
          auto dff = [&](uint32_t allow) -> DevOut {
            const DevLView v{sdev_tot + lane, sdev_use + lane, (uint32_t)sdev_pres[lane]};
            if (use_hw) {
              uint32_t gin, rin;
              dev_allowed(v, allow, gin, rin);
              const uint32_t want = (1u << 31) | (gin & 0xFFu) | ((rin & 0xFFu) << 8);
              bool ready = false;
              for (uint32_t it = 0; it <= (1u << 22); ++it) {
                if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(hw + 5, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) == hseq &&
                    __builtin_amdgcn_readfirstlane(__hip_atomic_load(hw + 6, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) == hseq) {
                  ready = true;
                  break;
                }
                __builtin_amdgcn_s_sleep(1);
              }
              if (ready) {
    #pragma unroll
                for (int k = 0; k < kDevVars; ++k) {
                  const DevVar dv = sdv[k * kMaxBatch + lane];
                  if (dv.sel == want) return DevOut{dv.reasons, dv.raw, 0u, 0u};
                }
              }
            }
            return dev_eval<false>(cfg, pod, v, nullptr, allow);
          };
          o = eval_full<NSC, false, false, FEAT>(cfg, pod, r, rsvf, devf, numaf, nullptr, dhf, dff);
        } else {
          o = eval_full<NSC, false, false, FEAT>(cfg, pod, r, rsvf, devf, numaf);
        }
        if (DEV && cfg.stat) {
          o.reasons |= so.reasons;
          o.traw = so.traw;
          o.araw = so.araw;
        }
        feas = o.reasons == 0;
        const bool needs_cores = ((pod.flags & KS_POD_CPU_BIND) && (pod.cpu_bind & KS_CPU_BIND_REQUIRED)) ||
                                 (cores_label(cw) != 0 && pod.cpu > 0);
        if ((FEAT & 2) && cfg.cores && (cw & kCoresDirty) && feas) unk = needs_cores;
        // on a node with a NUMA topology policy a required policy's NUMA-node core counts shape the hints, the
        // allocation and the score, not only feasibility: a slot whose CPU ids are not chosen yet is unknown either way
        if ((FEAT & 8) && cfg.cores && cfg.numa_pol && (cw & kCoresDirty) && (r.la_bits & kNumaPolNode) && needs_cores)
          unk_pol = true;
      }
      if ((FEAT & 8) && cfg.cores && cfg.numa_pol && __ballot(unk_pol)) {
        processed = j;  // the next pass sees the CPU ids cpuset_kernel chose
        break;
      }
      if ((FEAT & 2) && DEV && (cfg.dev || cfg.stat) && cfg.cores && __ballot(unk)) {
        processed = j;  // a normalization max over the feasible nodes would depend on it
        break;
      }
      if (DEV && (cfg.dev || cfg.stat) && (pod.flags & kPodNormDyn)) {
        // Normalization (DeviceShare, TaintToleration, NodeAffinity): the untouched nodes' max is the sweep's M
        // while its witness is untouched; the touched nodes are current.  If a pod's max changes, cut the pass
        // here.  (A pod without kPodNormDyn has raw 0 everywhere: every M normalizes it the same.)
        bool cut = false;
        auto norm1 = [&](uint64_t mk, int32_t raw) -> int32_t {
          const int32_t Msw = (int32_t)(mk >> 32);
          const int32_t Mt = (int32_t)wave_max_u32(feas ? (uint32_t)raw + 1u : 0u) - 1;
          if (mk == 0) return Mt < 0 ? 0 : Mt;  // no untouched node is feasible: only the touched ones compete
          const int64_t wn = (int64_t)(0xFFFFFFFFull - (mk & 0xFFFFFFFFull));
          const bool wt = ((touched[wn >> 6] >> (wn & 63)) & 1ull) != 0;
          if (wt ? (Mt != Msw) : (Mt > Msw)) cut = true;
          return Msw;
        };
        if (cfg.dev) Muse.dev = norm1(snorm[j], o.dev_raw);
        if (cfg.taint & 2) Muse.taint = norm1(snorm[kMaxBatch + j], o.traw);
        if (cfg.aff & 2) Muse.aff = norm1(snorm[2 * kMaxBatch + j], o.araw);
        if (cut) {
          processed = j;
          break;
        }
      }
      if (feas) key_mod = gkey(key_total(cfg, o, Muse), snode);
      best = umax64(cj.umax, wave_max_u64(key_mod));
      KS_STAMP(2);
      uint64_t need = __ballot(!cj.exact && cj.valid && cj.ub > best);
      while (need) {
        const uint64_t kmax = wave_max_u64(((need >> lane) & 1ull) ? cj.ub : 0ull);
        const int sel = __ffsll((long long)__ballot(((need >> lane) & 1ull) && cj.ub == kmax)) - 1;
        const int64_t c = (int64_t)(uint32_t)__shfl((int)cj.chunk, sel, 64);
        const uint64_t v = rescan_untouched<NSC, FEAT>(a, cfg, pod, c, touched[c], Muse, &pst);
        ++rescans;
        best = umax64(best, v);
        need &= ~(1ull << sel);
        need &= __ballot(cj.ub > best);
      }
      if (best < readlane64(my_bound, j)) {
        processed = j;  // an untouched chunk outside the list may hold a better node: re-sweep from j
        break;
      }
      if ((FEAT & 2) && cfg.cores && __ballot(unk && key_mod == best)) {
        processed = j;  // the winner's feasibility depends on core counts the next pass will have exact
        break;
      }
      KS_STAMP(3);
    }
    if (best == 0) {
      KS_CAT(4);
      if (lane == 0) sres[j] = ks_result{-1, KS_S_UNSCHEDULABLE, 0, -1, 0, 0, 0};
      goto next_pod;
    }
    const int32_t node = (int32_t)gkey_node(best);
    const int64_t score = gkey_score(best);
    const uint32_t pflags = __builtin_amdgcn_readlane(my_flags, j);
    const int64_t* podw = reinterpret_cast<const int64_t*>(&spods[j]);
    // ---- Reserve: NodeInfo.AddPod + podAssignCache.assign on the slot row (lane = term) ----
    // a cpu-bind pod first needs numCPUsNeeded available CPUs on the node (resource_manager.go:333-335)
    bool cpubind = (FEAT & 2) && cfg.cpuset && (pflags & KS_POD_CPU_BIND);
    int32_t cpu_need = cpubind ? (int32_t)(__builtin_amdgcn_readfirstlane(spods[j].cpu_bind) >> 8) : 0;
    int32_t s = __ffsll((long long)__ballot(snode == node)) - 1;
    uint32_t ncw = 0;  // Cfg.cores: the node's CoresWord
    if ((FEAT & 2) && cfg.cores) {
      ncw = __builtin_amdgcn_readfirstlane(s >= 0 ? (uint32_t)((uint64_t)snuma[4 * s + 3] >> 32)
                                                  : (node == cw_node ? cw_next : gld(a.dn->cpu_cores + node)));
      // a whole-CPU pod is cpu-bind on a node with a CPU bind policy (requestCPUBind, util.go:105-122)
      const int64_t pcpu = podw[0];  // PodRec.cpu
      if (!cpubind && cfg.cpuset && cores_label(ncw) != 0 && pcpu > 0) {
        cpubind = true;
        cpu_need = __builtin_amdgcn_readfirstlane((int32_t)(pcpu / 1000));
      }
    }
    SlotRow* row;
    // Reservation Reserve needs the node's pre-pod row: when the pod's class matches one of the
    // node's reservations the row is built / kept without the pod, nominated on, then taken.
    const int32_t pcls = (RSV && cfg.rsv) ? __builtin_amdgcn_readfirstlane(spods[j].rsv_class) : -1;
    bool rsvc = false;
    bool fresh = false;  // the slot is created by this pod: its state is the snapshot's
    if (s < 0) {
      if (!cj.fast) KS_CAT(2);
      fresh = true;
      s = nslots++;
      row = &rows[s];
      // the node's NUMA-node, dictionary and device words: loads issued before the raw row's, one HBM round trip
      int64_t ld_numa = 0, ld_stat = 0, ld_dtot = 0, ld_duse = 0;
      if ((FEAT & 8) && cfg.numa_pol) {
        const DevNuma& nv = *a.nv;
        if (lane < kNumaWUsed) ld_numa = gld(nv.total + (int64_t)lane * nv.npad + node);
        else if (lane < kNumaWOff) ld_numa = gld(nv.used + (int64_t)(lane - kNumaWUsed) * nv.npad + node);
        else if (lane < kNumaWCpu) ld_numa = gld(nv.off + (int64_t)(lane - kNumaWOff) * nv.npad + node);
        else if (lane < kNumaWMeta)
          ld_numa = ((int64_t)gld(nv.cs + (int64_t)(lane - kNumaWCpu) * nv.npad + node) << 32) |
                    (int64_t)(uint32_t)gld(nv.free + (int64_t)(lane - kNumaWCpu) * nv.npad + node);
        else if (lane == kNumaWMeta)
          ld_numa = (int64_t)((gld(nv.flags + node) >> KS_NUMA_POLICY_SHIFT) & 3u) |
                    ((int64_t)gld(nv.count + node) << 8) | ((int64_t)gld(nv.present + node) << 32);
      }
      if (DEV && cfg.stat && lane < 4) {
        const DevNodes d = *a.dn;
        const uint64_t* col = lane == 0 ? d.taints_hard : (lane == 1 ? d.taints_soft : (lane == 2 ? d.labels : d.host_ports));
        ld_stat = (int64_t)gld(col + node);
      }
      if (DEV && cfg.dev) {
        const DevDev& dv = *a.dv;
        if (lane < DW) ld_dtot = gld(dv.total + (int64_t)lane * dv.npad + node);
        else if (lane == DW) ld_dtot = (int64_t)(gld(dv.flags + node) & (KS_DEV_PRESENT | kDevRsvHeld));
        if (lane < DU) ld_duse = gld(dv.used + (int64_t)lane * dv.npad + node);
      }
      const int64_t* src = raw;
      if (node == (int32_t)gkey_node(readlane64(my_top, j))) {
        src = rawtop + j * 32;  // prefetched at pass start
      } else if (node == (int32_t)gkey_node(readlane64(my_second, j))) {
        src = rawrun + j * 32;  // prefetched at pass start
      } else {
#ifdef KS_SPEC
        if (node == spec_node) {
          if (lane < RF_N) raw[lane] = field_value(spec_val);
        } else
#endif
        {
          ++misses;
          if (lane < RF_N) raw[lane] = load_field(my_col, my_w, node);
        }
      }
      if (HELP && src != raw) {
        // the row comes from a prefetched node row: wave 1 builds it
        if (lane == s) snode = node;
        if (lane == 0) {
          atomicOr(&touched[node >> 6], 1ull << (node & 63));
          hdesc[hn] = make_int2(node, s | (j << 8) | (src == rawtop + j * 32 ? 0 : (1 << 16)));
          __hip_atomic_store(hpend, hn + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        ++hn;
        goto row_done;
      }
      if (HELP) hown |= 1ull << s;
      // Every field this slot needs is read before the first LDS write: the compiler cannot prove the
      // slot writes do not alias `src`, so each read after a write would cost a full LDS round trip.
      const bool take = !t_prod_only || (pflags & KS_POD_PROD);  // (before the Reservation match below)
      const int64_t f_cap = src[t_cap], f_req = src[t_req], f_pw = podw[t_pw];
      const int64_t u_bits = src[RF_LA_BITS], u_allowed = src[RF_ALLOWED], u_pods = src[RF_POD_COUNT];
      const int64_t u_acpu = src[RF_ALLOC_CPU], u_amem = src[RF_ALLOC_MEM], u_aeph = src[RF_ALLOC_EPH];
      const uint64_t ncl = RSV ? (uint64_t)src[RF_RSV_CLS] : 0ull;
      const int32_t u_rb = RSV ? (int32_t)src[RF_RSV_BEG] : 0, u_re = RSV ? (int32_t)src[RF_RSV_END] : 0;
      const int64_t u_A = (FEAT & 2) ? src[RF_NUMA_A] : 0, u_off = (FEAT & 2) ? src[RF_NUMA_OFF] : 0;
      const int64_t u_ratio = (FEAT & 2) ? src[RF_NUMA_RATIO] : 0;
      const int32_t u_free = (FEAT & 2) ? (int32_t)src[RF_CPU_FREE] : 0;
      if (cpubind && u_free < cpu_need) {
        // NodeNUMAResource Reserve -> Allocate: not enough CPUs; every plugin unreserves
        --nslots;
        if (lane == 0) sres[j] = ks_result{node, KS_S_RESERVE_FAILED, 0, -1, 0, 0, 0};
        goto next_pod;
      }
      if (lane == s) snode = node;
      if (lane == 0) atomicOr(&touched[node >> 6], 1ull << (node & 63));
      rsvc = pcls >= 0 && pcls < 64 && ((ncl >> pcls) & 1ull);
      if (lane == 0) {
        if (RSV) scls[s] = ncl;
        if (FEAT & 2) {
          snuma[4 * s] = u_A;
          snuma[4 * s + 1] = u_off;
          snuma[4 * s + 2] = u_ratio;
          snuma[4 * s + 3] = cfg.cores ? (int64_t)(((uint64_t)(ncw & ~kCoresDirty) << 32) | (uint32_t)u_free)
                                       : (int64_t)u_free;
        }
      }
      // the slot's NUMA-node state (lane = word, NumaLView layout), dictionary words and device totals + topology /
      // used / present flag into LDS (loaded above)
      if ((FEAT & 8) && cfg.numa_pol && lane < kNumaSlotWords) snp[s * kNumaSlotWords + lane] = ld_numa;
      if (DEV && cfg.stat && lane < 4) sstat[4 * s + lane] = (uint64_t)ld_stat;
      if (DEV && cfg.dev) {
        if (lane < DW) sdev_tot[lane * kDevLdsStride + s] = ld_dtot;
        else if (lane == DW) sdev_pres[s] = (int32_t)ld_dtot;
        if (lane < DU) sdev_use[lane * kDevLdsStride + s] = ld_duse;
      }
      if (RSV && cfg.rsv) {
        // the node's reservations into LDS (lane = record word), unless too many or too wide
        const int32_t rb = u_rb, cnt = u_re - u_rb;
        int32_t mode = -1;
        if (cnt <= a.rcap) {
          constexpr int W = (int)(sizeof(RsvRec<RD>) / 8);
          int64_t* dst = reinterpret_cast<int64_t*>(srec + s * a.rcap);
          const DevRsv& rv = *a.rv;
          for (int t = lane; t < cnt * W; t += 64) {
            const int rr = t / W, w = t - rr * W;
            const int64_t i = rb + rr;
            int64_t v;
            if (w == 0) v = (int64_t)gld(rv.cls + i);
            else if (w == 1) v = (int64_t)(((uint64_t)(uint32_t)gld(rv.ohi + i) << 32) | gld(rv.meta + i));
            else if (w == 2) v = (int64_t)(uint32_t)gld(rv.assigned + i);
            else if (w < 3 + RD) v = gld(rv.alloc + (int64_t)(w - 3) * rv.nr + i);
            else if (w < 3 + 2 * RD) v = gld(rv.allocd + (int64_t)(w - 3 - RD) * rv.nr + i);
            else v = gld(rv.rnz + (int64_t)(w - 3 - 2 * RD) * rv.nr + i);
            dst[t] = v;
          }
          const bool wide = __ballot(lane < cnt && rsv_ndims(srec[s * a.rcap + (lane < cnt ? lane : 0)].meta) > RD) != 0;
          mode = wide ? -1 : cnt;
        }
        if (lane == 0) {
          srcnt[s] = mode;
          srbeg[s] = rb;
        }
      }
      // build the slot row with the pod already reserved on it (lane-parallel, one code path)
      const bool take_here = take && !rsvc;
      const int64_t cap = f_cap, req = f_req + (take_here ? f_pw : 0) + (lane == ST_NCPU ? u_off : 0);
      if (lane < ST_N) {
        Term t;
        t.c = cap;
        t.h = cap - req + ((cap != 0 || !t_score) ? 0 : kNoCap);
        t.hd = cap != 0 ? (double)(cap - req) * 100.0 : 0.0;
        t.r = cap != 0 ? 1.0 / (double)cap : 0.0;
        row->t[lane] = t;
      } else if (lane == kLaneCounts) {
        row->la_bits = (uint32_t)u_bits;
        row->allowed = (int32_t)u_allowed;
        row->pod_count = (int32_t)u_pods + (rsvc ? 0 : 1);
        row->fit_ws = (u_acpu != 0 ? cfg.fw_cpu : 0) + (u_amem != 0 ? cfg.fw_mem : 0) + (u_aeph != 0 ? cfg.fw_eph : 0);
      }
    } else {
      KS_CAT(3);
      wait_rows(1ull << s);
      if (cpubind && (int32_t)snuma[4 * s + 3] < cpu_need) {
        if (lane == 0) sres[j] = ks_result{node, KS_S_RESERVE_FAILED, 0, -1, 0, 0, 0};
        goto next_pod;
      }
      row = &rows[s];
      rsvc = pcls >= 0 && pcls < 64 && ((scls[s] >> pcls) & 1ull);
      const bool take = !rsvc && (!t_prod_only || (pflags & KS_POD_PROD));
      if (lane < ST_N) {
        if (take) term_take(row->t[lane], podw[t_pw], __longlong_as_double(podw[t_pw100]));
      } else if (lane == kLaneCounts) {
        if (!rsvc) row->pod_count += 1;
      }
    }
  row_done:
    KS_STAMP(4);
    int32_t nom_row = -1;
    int64_t fitla_pref = -1;  // Fit + LoadAware total of a preferred (ordered) chosen node
    // DeviceShare Reserve on a node whose reservations hold devices (computed with the nomination)
    const bool want_dev0 = DEV && cfg.dev && (pflags & kPodHasGpu);
    bool dev_rsv_done = false;
    uint32_t gmin_rsv = 0, rmin_rsv = 0;
    GpuReq g_rsv{};
    if (RSV && rsvc) {
      // NominateReservation on the pre-pod state, Reserve into it (AddAssignedPod), then the pod
      PodRec pod = spods[j];
      pod.flags = __builtin_amdgcn_readfirstlane(pod.flags);
      pod.rsv_class = pcls;
      NodeReg<NSC> nr;
      slot_to_reg<NSC>(*row, nr);
      nr.rsv_cls = scls[s];
      nr.numa_A = snuma[4 * s];
      nr.numa_off = snuma[4 * s + 1];
      nr.numa_ratio = __longlong_as_double(snuma[4 * s + 2]);
      nr.cpu_free = (int32_t)snuma[4 * s + 3];
      if ((FEAT & 2) && cfg.cores) nr.cpu_cores = (uint32_t)((uint64_t)snuma[4 * s + 3] >> 32);  // (score: the label)
      RsvDelta<NSC> dl;
      const int32_t mode = srcnt[s];
      const RsvL<RD> lv{srec + s * a.rcap, mode, srbeg[s], a.rv};
      const DevLView sdv{sdev_tot + s, sdev_use + s, DEV && cfg.dev ? (uint32_t)sdev_pres[s] : 0u};
      // DeviceShare's FilterReservation / ScoreReservation in the nomination (reservations holding devices); the
      // view's classification once per nomination
      DrsSet dset{0ull, 0ull, 0u};
      bool dset_on = false;
      auto dnom = [&](const auto& v, int64_t i, int32_t* ds) -> bool {
        *ds = 0;
        if constexpr (DEV && (FEAT & 16) != 0) {
          if (!sdv.held()) return false;
          if (!dset_on) {
            dset = drs_set(v, pod.rsv_class);
            dset_on = true;
          }
          const uint64_t r = dev_rsv_candidate_x(dev_rsv_args(cfg, pod), sdv, v, dset, i);
          *ds = (int32_t)(uint32_t)r;
          return (r >> 32) != 0;
        }
        return false;
      };
      RsvOut ro;
      if constexpr ((FEAT & 16) != 0) {
        if (mode >= 0) ro = rsv_eval<NSC>(lv, pod, nr, dl, dnom);
        else ro = rsv_eval<NSC>(RsvG<true>(*a.rv, node), pod, nr, dl, dnom);
      } else {
        if (mode >= 0) ro = rsv_eval<NSC>(lv, pod, nr, dl);
        else ro = rsv_eval<NSC>(RsvG<true>(*a.rv, node), pod, nr, dl);
      }
      const int32_t nom = __builtin_amdgcn_readfirstlane(ro.nom);  // view index
      if (ro.hi >= kRsvOrderBase) {
        // the whole Filter / Score of the slot with this restore (eval_full: on a node with a NUMA topology policy the
        // score over the allocated NUMA nodes and DeviceShare under the admitted affinity, not the policy-None parts)
        NodeReg<NSC> n2 = nr;
        auto rv2 = [&](auto&& f) {
          if (mode >= 0) return f(lv);
          return f(RsvG<true>(*a.rv, node));
        };
        EvalOut e2 = eval_full<NSC, false, false, FEAT>(
            cfg, pod, n2, RsvWithOut<NSC, decltype(rv2)>{rv2, ro, dl},
            [&]() { return DevLView{sdev_tot + s, sdev_use + s, (uint32_t)sdev_pres[s]}; },
            [&]() { return NumaLView{snp + s * kNumaSlotWords}; });
        if (DEV && cfg.stat) stat_eval(cfg, pst, sstat[4 * s], sstat[4 * s + 1], sstat[4 * s + 2], sstat[4 * s + 3], e2);
        fitla_pref = e2.total + norm_terms(cfg, e2, Muse);
      }
      if ((FEAT & 16) && DEV && want_dev0 && sdv.held()) {
        // DeviceShare Reserve on the cycle's restore state, before the Reservation plugin's own Reserve changes it
        // (the ordered node's full evaluation above ran on the same state)
        const DevOut rd = mode >= 0 ? dev_rsv_reserve(cfg, pod, sdv, lv, nom, &g_rsv)
                                    : dev_rsv_reserve(cfg, pod, sdv, RsvG<true>(*a.rv, node), nom, &g_rsv);
        gmin_rsv = __builtin_amdgcn_readfirstlane(rd.minors);
        rmin_rsv = __builtin_amdgcn_readfirstlane(rd.rminors);
        dev_rsv_done = true;
        if (nom >= 0 && lane == 0) {
          if (mode >= 0) rsv_dev_assign(*a.rv, lv, nom, g_rsv, gmin_rsv, rmin_rsv, +1);
          else rsv_dev_assign(*a.rv, RsvG<true>(*a.rv, node), nom, g_rsv, gmin_rsv, rmin_rsv, +1);
        }
      }
      int64_t dd = 0;
      if (nom >= 0) {
        RsvReserve rr;
        int64_t gi;
        if (mode >= 0) {
          rr = rsv_reserve_delta(lv, pod, nom);
          gi = lv.csr(nom);
        } else {
          const RsvG<true> gv(*a.rv, node);
          rr = rsv_reserve_delta(gv, pod, nom);
          gi = gv.csr(nom);
        }
        RsvRec<RD>* rec = srec + s * a.rcap + nom;
#pragma unroll
        for (int d = 0; d < kRsvDims; ++d) {
          dd = (t_rdim == d) ? rr.dreq[d] : dd;
          if (lane == d && rr.add[d] != 0) {
            // the HBM table stays current for the next pass; the LDS copy for this one
            atomicAdd((unsigned long long*)(a.rv->allocd + (int64_t)d * a.rv->nr + gi), (unsigned long long)rr.add[d]);
            if (mode >= 0 && d < RD) rec->allocd[d] += rr.add[d];
          }
        }
        dd = (t_rdim == 8) ? rr.dnz[0] : (t_rdim == 9) ? rr.dnz[1] : dd;
        if (lane == 0) {
          atomicAdd(a.rv->assigned + gi, 1);
          if (mode >= 0) rec->assigned += 1;
        }
        if (mode < 0) __threadfence();
        if (rr.now_ineligible) {
          const uint64_t ncl = mode >= 0 ? rsv_node_classes(lv) : rsv_node_classes(RsvG<true>(*a.rv, node));
          if (lane == 0) {
            scls[s] = ncl;
            atomicExch((unsigned long long*)(a.rv->ncls + node), (unsigned long long)ncl);
          }
        }
        nom_row = (int32_t)gi;  // CSR position: the caller's row is looked up at the write-back (off the sequential path)
      }
      const bool take = !t_prod_only || (pflags & KS_POD_PROD);
      int64_t v = 0;
      if (lane < ST_N) {
        v = (take ? podw[t_pw] : 0) + dd;
        const double v100 = (take ? __longlong_as_double(podw[t_pw100]) : 0.0) + (double)dd * 100.0;
        if (take || dd != 0) term_take(row->t[lane], v, v100);
      } else if (lane == kLaneCounts) {
        row->pod_count += 1;
      }
      // a restored Requested went down: this node's key may rise for the pods of class -1 (no fast path for them)
      if (__ballot(lane < ST_N && v < 0)) rsv_raised = true;
    }
    int64_t score_out = score;
    if (RSV && cfg.rsv) {
      // the chosen node holds the maximum normalized Reservation score: 100 if hi > 0, else 0
      const int64_t hi = score / cfg.rsv_F;
      const int64_t fitla = hi >= kRsvOrderBase ? fitla_pref : score - hi * cfg.rsv_F;
      score_out = fitla + (hi > 0 ? a.rv->w100 : 0);
    }
    uint32_t gminors = 0, rminors = 0;
    // NodeNUMAResource Reserve on a node with a NUMA policy: Allocate with the Filter's hint on the pre-pod state
    // (the topology manager's stored affinity also restricts DeviceShare's Reserve)
    NumaPolOut npr;
    npr.admitted = false;
    npr.affinity = 0;
    bool npol = false;
    const bool want_npol = (FEAT & 8) && cfg.numa_pol && !(pflags & kPodReqZero);
    const bool want_dev = DEV && cfg.dev && (pflags & kPodHasGpu);
    // a slot created by this pod holds the snapshot state: reserve_pre_kernel's allocation for the node, if it ranked
    const PreRsv* pre = nullptr;
    const bool held_here = (FEAT & 16) && DEV && cfg.dev && RSV && cfg.rsv && ((uint32_t)sdev_pres[s] & kDevRsvHeld);
    if ((FEAT & 8) && a.pre_rsv && fresh && (want_npol || want_dev) && !held_here) {
      const uint64_t hit = __ballot(pre_nodes == node);  // (read by the look-ahead)
      if (hit) pre = a.pre_rsv + j * kPreRsvM + (__ffsll((long long)hit) - 1);
    }
    GpuReq g;
    if (pre) {
      const uint32_t pf = pre->flags;
      npol = (pf & 1u) != 0;
      npr.admitted = (pf & 2u) != 0;
      npr.reasons = pre->reasons;
      npr.affinity = pre->affinity;
#pragma unroll
      for (int k = 0; k < kNumaDev; ++k) {
        npr.alloc[0][k] = pre->alloc[0][k];
        npr.alloc[1][k] = pre->alloc[1][k];
        npr.cpus[k] = pre->cpus[k];
      }
      gminors = pre->gminors;
      rminors = pre->rminors;
      g.core = pre->g_core;
      g.mem = pre->g_mem;
      g.ratio = pre->g_ratio;
      g.rdma = pre->g_rdma;
      ++prehits;
    } else if (want_npol) {
      const NumaLView nl{snp + s * kNumaSlotWords};
      if (nl.policy() != 0) {
        PodRec pod = spods[j];
        pod.flags = pflags;
        NumaNodeCtx nc;
        nc.plain_req_cpu = nc.plain_req_mem = nc.plain_alloc_cpu = nc.plain_alloc_mem = 0;  // (score only)
        nc.cs_milli = snuma[4 * s];
        nc.cs_off = snuma[4 * s + 1];
        nc.ratio = __longlong_as_double(snuma[4 * s + 2]);
        nc.cpu_free = (int32_t)snuma[4 * s + 3];
        nc.cores = cfg.cores ? ((uint32_t)((uint64_t)snuma[4 * s + 3] >> 32) & ~kCoresDirty) : 0u;
        if (DEV && cfg.dev && (pflags & kPodHasGpu)) {
          const DevLView dvl{sdev_tot + s, sdev_use + s, (uint32_t)sdev_pres[s]};
          npr = numa_policy_eval<true>(cfg, pod, nl, nc, &dvl);  // the Filter passed on this state: DeviceShare follows
        } else {
          npr = numa_policy_eval(cfg, pod, nl, nc, (const DevLView*)nullptr);
        }
        npol = true;
      }
    }
    const uint32_t dev_allow = (npol && npr.admitted && npr.affinity) ? npr.affinity : ~0u;
    if (want_dev) {
      // DeviceShare Reserve: allocate the minors on the pre-pod GPU state, add the request per instance
      if (dev_rsv_done) {
        gminors = gmin_rsv;
        rminors = rmin_rsv;
        g = g_rsv;
      } else if (held_here) {
        // reservations holding devices, none matching the pod: the unmatched ones' restore still applies
        PodRec pod = spods[j];
        pod.flags = pflags;
        const DevLView sdv{sdev_tot + s, sdev_use + s, (uint32_t)sdev_pres[s]};
        const int32_t mode = srcnt[s];
        const DevOut dd = mode >= 0 ? dev_rsv_reserve(cfg, pod, sdv, RsvL<RD>{srec + s * a.rcap, mode, srbeg[s], a.rv}, -1, &g)
                                    : dev_rsv_reserve(cfg, pod, sdv, RsvG<true>(*a.rv, node), -1, &g);
        gminors = __builtin_amdgcn_readfirstlane(dd.minors);
        rminors = __builtin_amdgcn_readfirstlane(dd.rminors);
      } else if (!pre) {
        PodRec pod = spods[j];
        pod.flags = pflags;
        const DevOut dd = dev_eval<true>(cfg, pod, DevLView{sdev_tot + s, sdev_use + s, (uint32_t)sdev_pres[s]}, &g, dev_allow);
        gminors = __builtin_amdgcn_readfirstlane(dd.minors);
        rminors = __builtin_amdgcn_readfirstlane(dd.rminors);
      }
      // used word `lane`: GPU (q, k) for lane < 3 * kGpus, RDMA j = lane - kDevRdmaW after
      const bool is_gpu = lane < kDevRdmaW;
      const int k = is_gpu ? lane % kGpus : lane - kDevRdmaW;
      const uint32_t m = is_gpu ? gminors : rminors;
      if (lane < DU && ((m >> k) & 1u)) {
        const int q = lane / kGpus;
        const int64_t add = !is_gpu ? g.rdma : (q == 0 ? g.core : (q == 1 ? g.mem : g.ratio));
        const int64_t nv = sdev_use[lane * kDevLdsStride + s] + add;
        sdev_use[lane * kDevLdsStride + s] = nv;
        gst(a.dv->used + (int64_t)lane * a.dv->npad + node, nv);  // the HBM table for the next pass
      }
    }
    if ((FEAT & 8) && a.numa_alloc && lane < 2 * kNumaDev) {
      int64_t v = 0;
#pragma unroll
      for (int q = 0; q < 2 * kNumaDev; ++q) v = (q == lane) ? npr.alloc[q / kNumaDev][q % kNumaDev] : v;
      a.numa_alloc[(int64_t)(cursor0 + j) * 2 * kNumaDev + lane] = (npol && npr.reasons == 0) ? v : 0;
    }
    uint32_t cpu_split = 0;  // cpu-bind pod: CPUs per NUMA node (8 bits each), 0 = takeCPUs over the whole node
    if (npol && npr.reasons == 0) {
      // addPodAllocation: the NUMANodeResources to allocatedResources (node_allocation.go:86-99); a cpu-bind pod's
      // CPUs to the NUMA nodes' cpuset counts (and their amplification offsets) and available CPUs
      int64_t* w = snp + s * kNumaSlotWords;
      uint32_t bits = 0;
#pragma unroll
      for (int k = 0; k < kNumaDev; ++k) bits |= (npr.alloc[0][k] != 0 || npr.alloc[1][k] != 0) ? (1u << k) : 0u;
      int32_t cpus[kNumaDev];
#pragma unroll
      for (int k = 0; k < kNumaDev; ++k) cpus[k] = 0;
      if (cpubind) {
        if (bits) {
#pragma unroll
          for (int k = 0; k < kNumaDev; ++k) cpus[k] = npr.cpus[k];
        } else {
          cpus[0] = cpu_need;  // no NUMA allocation: admitted with a nil affinity, i.e. one NUMA node (count 1)
        }
#pragma unroll
        for (int k = 0; k < kNumaDev; ++k) cpu_split |= bits ? ((uint32_t)cpus[k] << (8 * k)) : 0u;
      }
      const int rr = lane / kNumaDev, kk = lane % kNumaDev;
      const double ratio = __longlong_as_double(snuma[4 * s + 2]);
      if (lane < 2 * kNumaDev) {
        int64_t add = 0;
#pragma unroll
        for (int q = 0; q < 2 * kNumaDev; ++q) add = (q == lane) ? npr.alloc[q / kNumaDev][q % kNumaDev] : add;
        if (add != 0) {
          const int64_t nvv = w[kNumaWUsed + lane] + add;
          w[kNumaWUsed + lane] = nvv;
          gst(a.nv->used + ((int64_t)rr * kNumaDev + kk) * a.nv->npad + node, nvv);
        }
      } else if (lane == 2 * kNumaDev && bits) {
        const int64_t meta = w[kNumaWMeta] | ((int64_t)bits << 32);
        w[kNumaWMeta] = meta;
        gst(a.nv->present + node, (uint32_t)(meta >> 32));
      } else if (lane >= 3 * kNumaDev && lane < 4 * kNumaDev) {
        const int k = lane - 3 * kNumaDev;
        int32_t c = 0;
#pragma unroll
        for (int q = 0; q < kNumaDev; ++q) c = (q == k) ? cpus[q] : c;
        if (c != 0) {
          const int64_t cw = w[kNumaWCpu + k];
          const int32_t cs1 = (int32_t)(cw >> 32) + c, fr1 = (int32_t)(uint32_t)cw - c;
          const int64_t m = (int64_t)cs1 * 1000;
          const int64_t off1 = ratio > 1.0 ? (int64_t)::ceil((double)m * ratio) - m : 0;
          w[kNumaWCpu + k] = ((int64_t)cs1 << 32) | (int64_t)(uint32_t)fr1;
          w[kNumaWOff + k] = off1;
          gst(a.nv->cs + (int64_t)k * a.nv->npad + node, cs1);
          gst(a.nv->free + (int64_t)k * a.nv->npad + node, fr1);
          gst(a.nv->off + (int64_t)k * a.nv->npad + node, off1);
        }
      }
    }
    if (cpubind) {
      // NodeAllocation.addPodAllocation of numCPUsNeeded CPUs: the cpuset millicores A grow, the
      // amplification offset Amplify(A) - A is re-derived (the CPU ids are chosen by cpuset_kernel)
      const int64_t A0 = snuma[4 * s], off0 = snuma[4 * s + 1];
      const double ratio = __longlong_as_double(snuma[4 * s + 2]);
      const int64_t A1 = A0 + (int64_t)cpu_need * 1000;
      const int64_t off1 = ratio > 1.0 ? (int64_t)::ceil((double)A1 * ratio) - A1 : 0;
      if (lane == ST_NCPU) term_take(row->t[ST_NCPU], off1 - off0, (double)(off1 - off0) * 100.0);
      if (lane == 0) {
        snuma[4 * s] = A1;
        snuma[4 * s + 1] = off1;
        snuma[4 * s + 3] -= cpu_need;
        if (cfg.cores) snuma[4 * s + 3] |= (int64_t)((uint64_t)kCoresDirty << 32);
        a.cpuset_list[atomicAdd(a.cpuset_n, 1)] = make_int2(cursor0 + j, node);
        a.cpuset_split[cursor0 + j] = cpu_split;
      }
    }
    // NodePorts: NodeInfo.AddPod adds the pod's host ports (written back with the slot)
    if (DEV && (cfg.ports & 1) && lane == 0) sstat[4 * s + 3] |= pst.pwant;
    if (lane == 0) sres[j] = ks_result{node, KS_S_SCHEDULED, score_out, nom_row, gminors, rminors, 0};
    {
      const int32_t qrow = __builtin_amdgcn_readlane(my_quota, j);
      if (cfg.quota_enable && qrow >= 0) {
        const uint32_t pmask = __builtin_amdgcn_readlane(my_pmask, j);
        if (lane < KS_QUOTA_DIMS && ((pmask >> lane) & 1u)) {
          // updatePodUsedNoLock -> updateGroupDeltaUsedNoLock (group_quota_manager.go:620-655)
          // (QC: the look-ahead's read of the pod's request; no LDS round trip in front of the atomics)
          const int64_t qreq = QC ? qreq_j : pqreq[j * KS_QUOTA_DIMS + lane];
          const bool np_ = (pflags & KS_POD_NONPREEMPTIBLE) != 0;
          if (QC) {
            // LDS atomics: no read-back on the sequential path (the next pod's admission reads after them)
            for (int32_t cur = qrow; cur >= 0;) {
              const int32_t up = cur == qrow ? qpar : qlds->parent[cur];  // (the leaf's parent: read by the look-ahead)
              atomicAdd((unsigned long long*)&qlds->used[(size_t)cur * KS_QUOTA_DIMS + lane], (unsigned long long)qreq);
              if (np_) atomicAdd((unsigned long long*)&qlds->npused[(size_t)cur * KS_QUOTA_DIMS + lane], (unsigned long long)qreq);
              cur = up;
            }
          } else {
            for (int32_t cur = qrow; cur >= 0; cur = a.q.parent[cur]) {
              a.q.used[(size_t)cur * KS_QUOTA_DIMS + lane] += qreq;
              if (np_) a.q.npused[(size_t)cur * KS_QUOTA_DIMS + lane] += qreq;
            }
          }
        }
      }
    }
    KS_STAMP(5);
    }
  next_pod:
    if (j + 1 < np) lookahead(j + 1);
    KS_STAMP(1);
#ifdef KS_COMMIT_CAT
    {
      const uint64_t t_ = __builtin_amdgcn_s_memtime();
      ph[cat] += t_ - tcat;
      tcat = t_;
      if (cat == 2) ph[5] += 1;
      if (cat == 3) ph[6] += 1;
    }
#endif
  }
  KS_STAMP(6);
  if (hintw && lane == 0) __hip_atomic_store(hw + 4, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  if (HELP) {
    if (lane == 0) __hip_atomic_store(hdone, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    wait_rows(nslots >= 64 ? ~0ull : ((1ull << nslots) - 1));
  }
  // ---- write back: results, touched rows, quota usage ----
  if (lane < processed) {
    ks_result r = sres[lane];
    if (RSV && r.reservation >= 0) r.reservation = a.rv->rowid[r.reservation];
    topo_writeback(a, cursor0 + lane, r);
    a.results[cursor0 + lane] = r;
  }
  if (lane < nslots) {
    const DevNodes d = *a.dn;
    const SlotRow& r = rows[lane];
    const int64_t node = snode;
    gst(d.req_cpu + node, r.t[ST_FREE_CPU].c - r.t[ST_FREE_CPU].h);
    gst(d.req_mem + node, r.t[ST_FREE_MEM].c - r.t[ST_FREE_MEM].h);
    gst(d.req_eph + node, r.t[ST_FREE_EPH].c - r.t[ST_FREE_EPH].h);
    gst(d.nz_cpu + node, term_requested(r.t[ST_CPU]));
    gst(d.nz_mem + node, term_requested(r.t[ST_MEM]));
#pragma unroll
    for (int k = 0; k < KS_MAX_SCALARS; ++k) gst(d.req_sc[k] + node, r.t[ST_FREE_SC + k].c - r.t[ST_FREE_SC + k].h);
    gst(d.pod_count + node, r.pod_count);
    gst(d.la_term_cpu + node, term_requested(r.t[ST_LCPU]));
    gst(d.la_term_mem + node, term_requested(r.t[ST_LMEM]));
    gst(d.la_pterm_cpu + node, term_requested(r.t[ST_PLCPU]));
    gst(d.la_pterm_mem + node, term_requested(r.t[ST_PLMEM]));
    if (DEV && (cfg.ports & 1)) gst(d.host_ports + node, sstat[4 * lane + 3]);
    if ((FEAT & 2) && cfg.cpuset) {
      gst(d.numa_amilli + node, snuma[4 * lane]);
      gst(d.numa_off + node, snuma[4 * lane + 1]);
      gst(d.numa_cpus + node, (int32_t)(snuma[4 * lane] / 1000));
      gst(d.cpu_free + node, (int32_t)snuma[4 * lane + 3]);
    }
  }
  if (QC) {
    for (int32_t i = lane; i < a.q.q * KS_QUOTA_DIMS; i += 64) {
      a.q.used[i] = qlds->used[i];
      a.q.npused[i] = qlds->npused[i];
    }
  }
  pipe_carry(a, nslots, snode);
  if (a.top_reset) a.top_reset[lane] = 0ull;
  if (lane == 0) {
    *a.cursor = cursor0 + processed;
    pipe_next(a, cursor0 + processed);
    atomicAdd(&a.counters[0], 1ull);
    if (processed < np) atomicAdd(&a.counters[1], 1ull);
    atomicAdd(&a.counters[2], (unsigned long long)rescans);
    atomicAdd(&a.counters[3], (unsigned long long)misses);
    atomicAdd(&a.counters[15], (unsigned long long)fast);  // ks_stats.diag[7]: monotone fast picks
    if (FEAT & 8) atomicAdd(&a.counters[5], (unsigned long long)prehits);
#if defined(KS_COMMIT_STAMPS) || defined(KS_COMMIT_CAT)
#ifdef KS_SLOT_SPLIT
    // (the slowest lane of each part: the wave's time; the sink keeps the timed evaluations)
    ph[0] = split[0] + (split_sink == 0x5eedull ? 1 : 0);
    ph[1] = split[1];
    ph[2] = split[2];
    ph[3] = split[3];
    ph[4] = ph[5] = ph[6] = 0;
#endif
    for (int i = 0; i < 7; ++i) atomicAdd(&a.counters[8 + i], (unsigned long long)ph[i]);
#endif
  }
#undef KS_STAMP
#undef KS_CAT
}

// ---- host launch wrappers (one set per (FEAT, NSC) translation unit of ks_variant.hip) ----
// Reserve ahead of the commit (NUMA topology policy variants, FEAT bit 8; in the DeviceShare-only variants the extra
// registers of the commit's look-up cost more than the device Reserve it saves): one workgroup per pod of the pass ranks the
// pod's candidate-list keys (each listed chunk's best and runner-up, the snapshot-best nodes of SelectArgs) and computes,
// for the kPreRsvM highest, what the commit's Reserve computes for a node no earlier pod of the pass touched --
// numa_policy_eval<ALLOC> (NodeNUMAResource Reserve -> Allocate with the Filter's hint) and dev_eval<ALLOC>
// (DeviceShare Reserve) -- on the snapshot state, all ranks in parallel.  It runs on the commit's stream right before
// the commit, so the state it reads is the state the commit loads into a new slot; the commit takes the record when
// the pod lands on one of these nodes as a new slot and computes the Reserve itself otherwise.
template <int FEAT>
__global__ __launch_bounds__(64) void reserve_pre_kernel(CommitArgs a) {
  constexpr bool DEV = (FEAT & 4) != 0;
  __shared__ int32_t sel[kPreRsvM];
  const int lane = threadIdx.x;
  const int32_t j = blockIdx.x;
  const int32_t cursor0 = __builtin_amdgcn_readfirstlane(*a.cursor);
  if (cursor0 >= a.total_pods) return;
  // the pods the commit will take: with the topology plugins the pass ends before its first topology pod, and when the
  // cursor's pod is one the sweep and the select return at once, so no list of this pass exists from that pod on (the
  // lists there are an earlier pass's, or never written)
  const int32_t np = topo_pass_pods(a, cursor0, min(a.batch, a.total_pods - cursor0));
  if (j >= np) return;
  const Cfg& cfg = a.c;
  const int32_t K = a.k, cnt = min(a.cand_count[j], K);
  // lane i: list entry i (K <= kMaxCand = 64)
  uint64_t kb = 0, kr = 0;
  if (lane < cnt) {
    const uint32_t ch = a.cand_chunk[j * K + lane];
    const uint2 t = a.cand_t[j * K + lane];
    // (a list entry outside the cluster is not a node: never read as one, whatever the list memory holds)
    if (ch < (uint32_t)a.nchunks) {
      kb = local_gkey(t.x, ch);
      kr = local_gkey(t.y, ch);
    }
  }
  int32_t rb = 0, rr = 0;  // ranks: keys are distinct (the node is in the low word)
  for (int l = 0; l < 64; ++l) {
    const uint64_t ob = readlane64(kb, l), orr = readlane64(kr, l);
    rb += (ob > kb) + (orr > kb);
    rr += (ob > kr) + (orr > kr);
  }
  if (lane < kPreRsvM) sel[lane] = -1;
  __syncthreads();
  if (kb && rb < kPreRsvM) sel[rb] = (int32_t)gkey_node(kb);
  if (kr && rr < kPreRsvM) sel[rr] = (int32_t)gkey_node(kr);
  __syncthreads();
  if (lane >= kPreRsvM) return;
  PreRsv o;
  o.node = sel[lane];
  o.flags = 0;
  o.reasons = 0;
  o.affinity = 0;
#pragma unroll
  for (int k = 0; k < kNumaDev; ++k) {
    o.alloc[0][k] = o.alloc[1][k] = 0;
    o.cpus[k] = 0;
  }
  o.gminors = o.rminors = 0;
  o._pad[0] = o._pad[1] = 0;
  o.g_core = o.g_mem = o.g_ratio = o.g_rdma = 0;
  if (o.node >= a.n) o.node = -1;
  if (o.node >= 0) {
    const int64_t node = o.node;
    const PodRec pod = a.pods[cursor0 + j];
    const uint32_t pflags = pod.flags;
    NumaPolOut npr;
    npr.admitted = false;
    npr.affinity = 0;
    npr.reasons = 0;
    bool npol = false;
    const DevGView dvg{*a.dv, node};
    if ((FEAT & 8) && cfg.numa_pol && !(pflags & kPodReqZero)) {
      const NumaGView nv{*a.nv, node};
      if (nv.policy() != 0) {
        // the commit's slot copy of the node's cpuset state (RF_NUMA_* row fields)
        NumaNodeCtx nc;
        nc.plain_req_cpu = nc.plain_req_mem = nc.plain_alloc_cpu = nc.plain_alloc_mem = 0;
        nc.cs_milli = load_field(a.rowcols[RF_NUMA_A].p, a.rowcols[RF_NUMA_A].width, node);
        nc.cs_off = load_field(a.rowcols[RF_NUMA_OFF].p, a.rowcols[RF_NUMA_OFF].width, node);
        nc.ratio = __longlong_as_double(load_field(a.rowcols[RF_NUMA_RATIO].p, a.rowcols[RF_NUMA_RATIO].width, node));
        nc.cpu_free = (int32_t)load_field(a.rowcols[RF_CPU_FREE].p, a.rowcols[RF_CPU_FREE].width, node);
        nc.cores = cfg.cores ? gld(a.dn->cpu_cores + node) : 0u;
        if (DEV && cfg.dev && (pflags & kPodHasGpu)) npr = numa_policy_eval<true>(cfg, pod, nv, nc, &dvg);
        else npr = numa_policy_eval(cfg, pod, nv, nc, (const DevGView*)nullptr);
        npol = true;
      }
    }
    if (npol) {
      o.flags = 1u | (npr.admitted ? 2u : 0u);
      o.reasons = npr.reasons;
      o.affinity = npr.affinity;
#pragma unroll
      for (int k = 0; k < kNumaDev; ++k) {
        o.alloc[0][k] = npr.alloc[0][k];
        o.alloc[1][k] = npr.alloc[1][k];
        o.cpus[k] = npr.cpus[k];
      }
    }
    if (DEV && cfg.dev && (pflags & kPodHasGpu)) {
      const uint32_t dev_allow = (npol && npr.admitted && npr.affinity) ? npr.affinity : ~0u;
      GpuReq g;
      const DevOut dd = dev_eval<true>(cfg, pod, dvg, &g, dev_allow);
      o.gminors = dd.minors;
      o.rminors = dd.rminors;
      o.g_core = g.core;
      o.g_mem = g.mem;
      o.g_ratio = g.ratio;
      o.g_rdma = g.rdma;
    }
  }
  const_cast<PreRsv*>(a.pre_rsv)[j * kPreRsvM + lane] = o;
}

struct PassLaunch {
  hipError_t (*sweep)(int blocks, hipStream_t s, const SweepArgs& a);
  hipError_t (*commit)(bool qc, size_t smem, hipStream_t s, const CommitArgs& a);
  hipError_t (*commit_attr)(bool qc, size_t smem);
  // FEAT 0 only (else null): the monotone commit kernel (ks_mono.h)
  hipError_t (*commit_mono)(bool qc, size_t smem, hipStream_t s, const CommitArgs& a);
  hipError_t (*commit_mono_attr)(bool qc, size_t smem);
  // NUMA topology policy variants only (else null): reserve_pre_kernel, one workgroup per pod of the pass
  hipError_t (*reserve_pre)(int blocks, hipStream_t s, const CommitArgs& a);
};
#define KS_DECLARE_VARIANT(F) PassLaunch pass_launch_f##F##_n0(); PassLaunch pass_launch_f##F##_n2(); PassLaunch pass_launch_f##F##_n4();
KS_DECLARE_VARIANT(0)
KS_DECLARE_VARIANT(1)
KS_DECLARE_VARIANT(3)
KS_DECLARE_VARIANT(4)
KS_DECLARE_VARIANT(6)
KS_DECLARE_VARIANT(7)
KS_DECLARE_VARIANT(11)
KS_DECLARE_VARIANT(14)
KS_DECLARE_VARIANT(15)
KS_DECLARE_VARIANT(23)
KS_DECLARE_VARIANT(31)
#undef KS_DECLARE_VARIANT

}  // namespace ks
