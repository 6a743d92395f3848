// ks_debug.h — host wrapper of the debug evaluation kernel (ks_debug.hip).
#pragma once

#include "ks_pass.h"
#include "ks_topo.h"

namespace ks {

hipError_t launch_eval_debug(int nsc, int blocks, hipStream_t s, DevNodes d, const DevRsv* rv, const DevDev* dv,
                             const DevNuma* nv, Cfg c, const PodRec* pod, int64_t n, uint32_t* reasons,
                             int64_t* scores, int64_t* total, int32_t* raw, int32_t* hiord, int32_t* draw,
                             const PodStat* pstat, int32_t* traw, int32_t* araw, const TopoKArgs* tk = nullptr,
                             int feat = 15);

}  // namespace ks
