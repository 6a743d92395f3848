// ks_debug.hip — ks_eval_pod_debug's per-node evaluation (every reason bit and per-plugin score of one pod on
// every node, no Reserve), in its own translation unit.
#include "ks_pass.h"
#include "ks_debug.h"
#include "ks_topo.h"

namespace ks {
// ------------------------------------------------------------------------------------------
// debug evaluation of one pod over every node (no Reserve)
// ------------------------------------------------------------------------------------------

template <int NSC, int FEAT>
__global__ __launch_bounds__(256) void eval_debug_kernel(DevNodes d, const DevRsv* rv, const DevDev* dv, const DevNuma* nv, Cfg c, const PodRec* pod, int64_t n,
                                  uint32_t* reasons, int64_t* scores, int64_t* total, int32_t* raw, int32_t* hiord,
                                  int32_t* draw, const PodStat* pstat, int32_t* traw, int32_t* araw,
                                  TopoKArgs tk, int32_t topo) {
  __shared__ TopoLds tl;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool valid = i < n;
  // the topology step (ks_topo.h): the pod at the cursor, only if it is a topology pod
  int64_t pi = 0;
  TopoRec tr;
  TopoTerms tt;
  NodeReg<NSC> r;
  load_node<NSC>(c, d, i, valid ? 1 : 0, r);  // (issued with the step's pod record)
  const int64_t i0 = valid ? i : 0;
  const TopoNodeDom nd = topo ? topo_node_dom(tk.t, i0) : TopoNodeDom{};
  const uint64_t th = c.stat ? d.taints_hard[i0] : 0ull, ts = c.stat ? d.taints_soft[i0] : 0ull,
                 lb = c.stat ? d.labels[i0] : 0ull, hp = c.stat ? d.host_ports[i0] : 0ull;
  if (topo) {
    pi = topo_cur(tk, tr);
    tt = topo_terms_cur(tk);
    if (pi < 0) return;
    if (tr.flags & KS_TOPO_DYN) topo_stage(tk, tr, tt, tl);
  }
  TopoNodeIn tin{1u, 0, 0, 0, 0};
  if (valid) {
    const PodRec p = pod[pi];
    const PodStat* ps = pstat ? pstat + pi : nullptr;
    RsvOut ro;
    EvalOut o = eval_full<NSC, true, false, FEAT>(
        c, p, r, [&](auto&& f) { return f(RsvG<false>(*rv, i)); },
        [&]() { return DevGView{*dv, i}; }, [&]() { return NumaGView{*nv, i}; }, &ro);
    if (c.stat) stat_eval(c, *ps, th, ts, lb, hp, o);
    reasons[i] = o.reasons;
    // Fit + LoadAware + NUMA + BalancedAllocation part (the normalized plugins are added by the normalize kernels)
    total[i] = o.reasons ? -1
                         : (int64_t)o.fit * c.fit_pw + (int64_t)o.la * c.la_pw + (int64_t)o.numa * c.numa_pw +
                               (int64_t)o.bal * c.bal_pw;
    raw[i] = ro.raw;
    hiord[i] = ro.hiord;
    draw[i] = o.dev_raw;
    traw[i] = o.traw;
    araw[i] = o.araw;
    if (scores) {  // (NULL in the batch's topology step: only ks_eval_pod returns the per-plugin matrix)
      int64_t* sc = scores + i * KS_NUM_SCORE_PLUGINS;
      sc[KS_SCORE_FIT] = o.reasons ? 0 : o.fit;
      sc[KS_SCORE_LOADAWARE] = o.reasons ? 0 : o.la;
      sc[KS_SCORE_RESERVATION] = 0;
      sc[KS_SCORE_NUMA] = o.reasons ? 0 : o.numa;
      sc[KS_SCORE_BALANCED] = o.reasons ? 0 : o.bal;
      sc[KS_SCORE_DEVICESHARE] = 0;
      sc[KS_SCORE_TAINT] = 0;
      sc[KS_SCORE_NODE_AFFINITY] = 0;
      sc[KS_SCORE_TOPOLOGY_SPREAD] = 0;
      sc[KS_SCORE_POD_AFFINITY] = 0;
    }
    tin = TopoNodeIn{o.reasons, o.dev_raw, o.traw, o.araw, ro.hiord};
  }
  // PodTopologySpread / InterPodAffinity Filters and the normalizations' reductions (every lane, converged)
  if (topo) topo_eval_node(tk, tr, tt, nd, (int32_t)pi, i, valid, tl, tin);
}


// The plugin-set variant the context's kernels use (FEAT 0: Fit + LoadAware [+ quota], FEAT 4: + DeviceShare / the
// dictionary plugins) or the generic one
template <int NSC>
static void launch_nsc(int feat, int blocks, hipStream_t s, DevNodes d, const DevRsv* rv, const DevDev* dv,
                       const DevNuma* nv, Cfg c, const PodRec* pod, int64_t n, uint32_t* reasons, int64_t* scores,
                       int64_t* total, int32_t* raw, int32_t* hiord, int32_t* draw, const PodStat* pstat, int32_t* traw,
                       int32_t* araw, const TopoKArgs& t, int32_t on) {
  if (feat == 0)
    hipLaunchKernelGGL((eval_debug_kernel<NSC, 0>), dim3(blocks), dim3(256), 0, s, d, rv, dv, nv, c, pod, n, reasons, scores, total, raw, hiord, draw, pstat, traw, araw, t, on);
  else if (feat == 4)
    hipLaunchKernelGGL((eval_debug_kernel<NSC, 4>), dim3(blocks), dim3(256), 0, s, d, rv, dv, nv, c, pod, n, reasons, scores, total, raw, hiord, draw, pstat, traw, araw, t, on);
  else
    hipLaunchKernelGGL((eval_debug_kernel<NSC, 31>), dim3(blocks), dim3(256), 0, s, d, rv, dv, nv, c, pod, n, reasons, scores, total, raw, hiord, draw, pstat, traw, araw, t, on);
}

hipError_t launch_eval_debug(int nsc, int blocks, hipStream_t s, DevNodes d, const DevRsv* rv, const DevDev* dv,
                             const DevNuma* nv, Cfg c, const PodRec* pod, int64_t n, uint32_t* reasons,
                             int64_t* scores, int64_t* total, int32_t* raw, int32_t* hiord, int32_t* draw,
                             const PodStat* pstat, int32_t* traw, int32_t* araw, const TopoKArgs* tk, int feat) {
  const TopoKArgs t = tk ? *tk : TopoKArgs{};
  const int32_t on = tk ? 1 : 0;
  const int f = (feat == 0 || feat == 4) ? feat : 15;
  if (nsc == 0) launch_nsc<0>(f, blocks, s, d, rv, dv, nv, c, pod, n, reasons, scores, total, raw, hiord, draw, pstat, traw, araw, t, on);
  else if (nsc == 2) launch_nsc<2>(f, blocks, s, d, rv, dv, nv, c, pod, n, reasons, scores, total, raw, hiord, draw, pstat, traw, araw, t, on);
  else launch_nsc<4>(f, blocks, s, d, rv, dv, nv, c, pod, n, reasons, scores, total, raw, hiord, draw, pstat, traw, araw, t, on);
  return hipGetLastError();
}

}  // namespace ks
