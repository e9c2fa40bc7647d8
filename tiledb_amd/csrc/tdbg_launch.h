// tdbg_launch.h -- kernel dispatch for the launch shims.
//
// Launch timing (tdbg_context_time_launches) binds its HIP events to kernel
// dispatches instead of recording them as separate marker packets: each
// hipEventRecord on the launch stream cost ~4 us of stream time per event
// (three per launch: ~12 us of a 330 us 12,500-tile C5 step), a bound event
// costs nothing extra.  The host arms a start and/or stop event for the next
// dispatch; the next TDBG_LAUNCH takes and disarms them.
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

namespace tdbg {
struct EvArm {
  hipEvent_t start;  // time of the next dispatch's start
  hipEvent_t stop;   // time of the next dispatch's end
};
extern thread_local EvArm ev_arm;
}  // namespace tdbg

#define TDBG_LAUNCH(KERNEL, GRID, BLOCK, STREAM, ...)                                    \
  do {                                                                                   \
    const tdbg::EvArm ev_ = tdbg::ev_arm;                                                \
    tdbg::ev_arm = tdbg::EvArm{nullptr, nullptr};                                        \
    hipExtLaunchKernelGGL(KERNEL, GRID, BLOCK, 0, STREAM, ev_.start, ev_.stop, 0u, __VA_ARGS__); \
  } while (0)
