// ks_variant.hip — one plugin-set (FEAT = KS_FEAT) x scalar-slot (NSC = KS_NSC) variant of the pass kernels (ks_pass.h) and its host launch
// wrappers.  The Makefile compiles this file once per (FEAT, NSC) so the variants build in parallel.
#include "ks_pass.h"
#include "ks_mono.h"

#if !defined(KS_FEAT) || !defined(KS_NSC)
#error "compile with -DKS_FEAT=<feature bits> -DKS_NSC=<0|2|4>"
#endif

#define KS_CAT2(a, b) a##b
#define KS_CAT(a, b) KS_CAT2(a, b)

namespace ks {
namespace {

constexpr int F = KS_FEAT;

constexpr int NSC = KS_NSC;

hipError_t sweep(int blocks, hipStream_t s, const SweepArgs& a) {
  hipLaunchKernelGGL((sweep_kernel<NSC, F>), dim3(blocks), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t commit(bool qc, size_t smem, hipStream_t s, const CommitArgs& a) {
  if (qc) hipLaunchKernelGGL((commit_kernel<NSC, true, F>), dim3(1), dim3(commit_threads(F)), smem, s, a);
  else hipLaunchKernelGGL((commit_kernel<NSC, false, F>), dim3(1), dim3(commit_threads(F)), smem, s, a);
  return hipGetLastError();
}

hipError_t commit_attr(bool qc, size_t smem) {
  const void* fn = qc ? (const void*)commit_kernel<NSC, true, F> : (const void*)commit_kernel<NSC, false, F>;
  return hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
}

#if KS_FEAT == 0
// the monotone Fit + LoadAware [+ ElasticQuota] commit (ks_mono.h)
hipError_t commit_mono(bool qc, size_t smem, hipStream_t s, const CommitArgs& a) {
  if (qc) hipLaunchKernelGGL((commit_mono_kernel<NSC, true>), dim3(1), dim3(commit_threads(0)), smem, s, a);
  else hipLaunchKernelGGL((commit_mono_kernel<NSC, false>), dim3(1), dim3(commit_threads(0)), smem, s, a);
  return hipGetLastError();
}

hipError_t commit_mono_attr(bool qc, size_t smem) {
  const void* fn = qc ? (const void*)commit_mono_kernel<NSC, true> : (const void*)commit_mono_kernel<NSC, false>;
  return hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
}
#endif

#if (KS_FEAT & 8) != 0
hipError_t reserve_pre(int blocks, hipStream_t s, const CommitArgs& a) {
  hipLaunchKernelGGL((reserve_pre_kernel<F>), dim3(blocks), dim3(64), 0, s, a);
  return hipGetLastError();
}
#endif

}  // namespace

PassLaunch KS_CAT(KS_CAT(KS_CAT(pass_launch_f, KS_FEAT), _n), KS_NSC)() {
#if KS_FEAT == 0
  return PassLaunch{sweep, commit, commit_attr, commit_mono, commit_mono_attr, nullptr};
#elif (KS_FEAT & 8) != 0
  return PassLaunch{sweep, commit, commit_attr, nullptr, nullptr, reserve_pre};
#else
  return PassLaunch{sweep, commit, commit_attr, nullptr, nullptr, nullptr};
#endif
}

}  // namespace ks
