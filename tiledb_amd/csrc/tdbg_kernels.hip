// tdbg_kernels.hip -- gfx950 (MI355X / CDNA4) tile unfilter kernels.
//
// Reverse ("unfilter") direction of TileDB's filter pipeline
// (tiledb/sm/filter/filter_pipeline.cc:439-517) for byteshuffle, bitshuffle,
// bit-width reduction, positive delta, double delta and fixed-size RLE, on
// whole tiles in the on-disk layout (format_spec/tile.md).
//
// Work decomposition: a persistent grid; each workgroup owns one scratch slot
// and walks tiles t = blockIdx.x, blockIdx.x + gridDim.x, ...  A tile's chunk
// directory (tile.cc:280-313) is walked by the whole workgroup (uniform
// loads), then each chunk runs through the filters in reverse, every filter
// block-parallel.  The general interpreter below keeps intermediates in a
// per-workgroup global scratch slot (L2/MALL resident) and is correct for any
// combination of the six filters and any chunk size; the fused LDS fast paths
// (tdbg_fast.hip) take over for the hot pipelines.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/tiledb_amd.h"
#include "tdbg_desc.h"
#include "tdbg_launch.h"
#include "tdbg_device.h"
#include "tdbg_general.h"

namespace tdbg {

__device__ __attribute__((noinline)) void general_body(const KParams& kp) {
  __shared__ Shared<GEN_NT> sh;
  Slot sl;
  uint8_t* base = kp.scratch + (uint64_t)blockIdx.x * kp.slot_bytes;
  sl.slot_cap = kp.slot_cap;
  sl.md_cap = kp.md_cap;
  sl.tab_cap = kp.tab_cap;
  sl.buf[0] = base;
  sl.buf[1] = base + kp.slot_cap;
  sl.md[0] = base + 2ull * kp.slot_cap;
  sl.md[1] = sl.md[0] + kp.md_cap;
  sl.tab = sl.md[1] + kp.md_cap;
  uint64_t n = kp.ntiles;
  const uint32_t* list = kp.tile_list;
  if (kp.fixup) {  // only the tiles the fused kernel queued
    n = kp.fbq[0];
    if (n > kp.fbq_cap) n = kp.fbq_cap;
    list = kp.fbq + 1;
  }
  uint64_t ok_tiles = 0, ok_bytes = 0;
  for (uint64_t j = blockIdx.x; j < n; j += gridDim.x) {
    const uint64_t t = list ? list[j] : j;
    uint64_t need = 0;
    const int rc = g_tile<GEN_NT>(kp, kp.in[t], kp.in_size[t], kp.out[t], kp.out_size[t], sl, sh, &need);
    __syncthreads();
    if (rc == TDBG_OK) {
      ok_tiles++;
      ok_bytes += kp.out_size[t];
    }
    if (threadIdx.x == 0) {
      if (kp.status) kp.status[t] = rc;
      if (kp.need) kp.need[t] = need;
    }
  }
  if (kp.stats && threadIdx.x == 0 && ok_tiles) {
    atomicAdd((unsigned long long*)&kp.stats[TDBG_STAT_GENERAL_TILES], (unsigned long long)ok_tiles);
    atomicAdd((unsigned long long*)&kp.stats[TDBG_STAT_GENERAL_BYTES], (unsigned long long)ok_bytes);
  }
}

__global__ void __launch_bounds__(GEN_NT)
unfilter_general_kernel(const KParams kp) {
  general_body(kp);
}

// Fixup launch after the fused kernel: the general interpreter over the
// tiles the fused kernel queued.  The queue is almost always empty, so the
// entry only reads its count (the interpreter's prologue sits behind the call).
__global__ void __launch_bounds__(GEN_NT)
unfilter_fixup_kernel(const KParams kp) {
  // streamed launches: the streaming kernel's queue was consumed by the fused
  // kernel before this launch started; its count is reset for the next launch
  if (kp.sq && blockIdx.x == 0 && threadIdx.x == 0) kp.sq[0] = 0;
  const uint32_t queued = kp.fbq[0];
  if (queued == 0) return;
  if (blockIdx.x == 0 && threadIdx.x == 0 && kp.stats)
    atomicAdd((unsigned long long*)&kp.stats[TDBG_STAT_FALLBACK],
              (unsigned long long)(queued < kp.fbq_cap ? queued : kp.fbq_cap));
  const KParams local = kp;  // copied only past the early exit
  general_body(local);
}

}  // namespace tdbg

// ---------------------------------------------------------------------------
// host-side launch shims (called from tdbg_host.cpp)
// ---------------------------------------------------------------------------
extern "C" hipError_t tdbg_launch_general(const tdbg::KParams* kp, uint32_t grid,
                                          hipStream_t stream) {
  TDBG_LAUNCH(tdbg::unfilter_general_kernel, dim3(grid), dim3(GEN_NT), stream, *kp);
  return hipGetLastError();
}

extern "C" hipError_t tdbg_launch_fixup(const tdbg::KParams* kp, uint32_t grid,
                                        hipStream_t stream) {
  TDBG_LAUNCH(tdbg::unfilter_fixup_kernel, dim3(grid), dim3(GEN_NT), stream, *kp);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Tile::add_extra_offset (tile.h:144-146) for unfiltered offsets tiles: the
// last u64 of the tile (the slot TDBG_TILE_OFFSETS reserves) becomes the size
// of its var-data tile.  One thread per tile; tiles whose status is an error
// are left alone.
// ---------------------------------------------------------------------------
__global__ void extra_offset_kernel(uint64_t ntiles, uint8_t* const* out, const uint64_t* out_size,
                                    const uint64_t* var_size, const int32_t* status) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntiles) return;
  if (status && status[t] != TDBG_OK) return;
  const uint64_t os = out_size[t];
  if (os < 8) return;
  uint8_t* p = out[t] + os - 8;
  const uint64_t v = var_size[t];
  if ((((uintptr_t)p) & 7) == 0) {
    *(uint64_t*)p = v;
  } else {
    for (int b = 0; b < 8; b++) p[b] = (uint8_t)(v >> (8 * b));
  }
}

extern "C" hipError_t tdbg_launch_extra_offset(uint64_t ntiles, uint8_t* const* out, const uint64_t* out_size,
                                               const uint64_t* var_size, const int32_t* status,
                                               hipStream_t stream) {
  if (ntiles == 0) return hipSuccess;
  const uint32_t grid = (uint32_t)((ntiles + 255) / 256);
  hipLaunchKernelGGL(extra_offset_kernel, dim3(grid), dim3(256), 0, stream, ntiles, out, out_size, var_size,
                     status);
  return hipGetLastError();
}
