// tdbg_stream_common.h -- pieces shared by the streaming C5 kernels
// (tdbg_stream.hip: DoubleDelta bit-packed; tdbg_stream_raw.hip: DoubleDelta
// raw): persistent-grid tile walk with descriptors batched 64 at a time, the
// LDS-DMA of 16-B units, and the LDS-only workgroup barrier.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tdbg_desc.h"

namespace tdbg {
namespace sc {

// Tile images of at most this many bytes belong to the coded kernel
// (tdbg_stream.hip stages whole images of this size in LDS); bigger ones to
// the raw-DoubleDelta kernel (tdbg_stream_raw.hip).  Each kernel queues the
// tiles of its class it does not decode and skips the other class.
constexpr uint32_t CODED_CAP = 22016;

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) v4u g_u4;

__device__ __forceinline__ uint32_t lane_() {
  uint32_t l = threadIdx.x & 63;
  asm volatile("" : "+v"(l));
  return l;
}
__device__ __forceinline__ uint32_t wave_() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// one tile of the launch
struct Desc {
  uint64_t t, fs, os;
  const uint8_t* in;
  uint8_t* out;
};

// Descriptors of the workgroup's tiles, 64 at a time: lane i holds those of
// its (base + i)-th tile, loaded once (one HBM latency per 64 tiles instead
// of one per tile) and read back with v_readlane at a uniform index.  The
// workgroup's k-th tile is blockIdx.x + k * gridDim.x.
struct Batch {
  uint32_t fs, os;  // saturated at 2^32 - 1 (such a tile fits no streaming kernel)
  uint64_t in, out;
};
// Chunk mode (kp.chunks set: a chunk-parallel launch, tdbg_chunkdir.hip):
// the work items are the records of the device chunk directory, and a
// descriptor is one chunk: its image starts at the chunk's 12-byte header
// ([u32 orig][u32 filtered][u32 md], tile.cc:280-313) and its output at the
// chunk's offset in the tile's buffer.
// (bid: the workgroup's index in the launch's deal of work items; blockIdx.x
// unless a kernel remaps it)
__device__ __forceinline__ Batch batch_load(const KParams& kp, uint64_t base, uint64_t ntl, uint32_t bid) {
  const uint64_t j = bid + (base + (threadIdx.x & 63)) * (uint64_t)gridDim.x;
  Batch b{0, 0, 0, 0};
  if (j < ntl) {
    if (kp.chunks) {
      const ChunkRec r = kp.chunks[j];
      const uint64_t fs = 12ull + r.ml + r.fl;
      b.fs = fs < 0xffffffffull ? (uint32_t)fs : 0xffffffffu;
      b.os = r.orig;
      b.in = (uint64_t)kp.in[r.tile] + r.in_off - 12;
      b.out = (uint64_t)kp.out[r.tile] + r.out_off;
    } else {
      const uint64_t fs = kp.in_size[j], os = kp.out_size[j];
      b.fs = fs < 0xffffffffull ? (uint32_t)fs : 0xffffffffu;
      b.os = os < 0xffffffffull ? (uint32_t)os : 0xffffffffu;
      b.in = (uint64_t)kp.in[j];
      b.out = (uint64_t)kp.out[j];
    }
  }
  return b;
}
__device__ __forceinline__ Batch batch_load(const KParams& kp, uint64_t base, uint64_t ntl) {
  return batch_load(kp, base, ntl, blockIdx.x);
}

// work items of a launch: tiles, or (chunk mode / a queue) a device count
__device__ __forceinline__ uint64_t work_items(const KParams& kp) {
  uint64_t ntl = kp.ntiles;
  if (kp.ntiles_dev) {
    const uint64_t c = (uint32_t)__builtin_amdgcn_readfirstlane(*kp.ntiles_dev);
    ntl = c < ntl ? c : ntl;
  }
  return ntl;
}
// (the builtin returns int: each half goes through uint32_t, or the low half
// of a pointer would be sign-extended over the high one)
__device__ __forceinline__ uint64_t rl64(uint64_t v, uint32_t k) {
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((uint32_t)(v >> 32), k);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((uint32_t)v, k);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ Desc batch_get(const Batch& b, uint32_t k, uint64_t t) {
  Desc d;
  d.t = t;
  d.fs = (uint32_t)__builtin_amdgcn_readlane(b.fs, k);
  d.os = (uint32_t)__builtin_amdgcn_readlane(b.os, k);
  d.in = (const uint8_t*)rl64(b.in, k);
  d.out = (uint8_t*)rl64(b.out, k);
  return d;
}

// LDS byte address of a __shared__ object (for M0)
template <typename T>
__device__ __forceinline__ uint32_t lds_addr(T* p) {
  return (uint32_t)(uintptr_t)((__attribute__((address_space(3))) uint8_t*)p);
}

// One LDS-DMA instruction: every active lane moves the 16-B unit at `src`
// to LDS byte dst_wave + 16 * lane (dst_wave wave-uniform).  Inline asm, not
// the builtin: the compiler would otherwise wait for the DMA (vmcnt(0),
// which on gfx950 also drains every store before it) at the next LDS read
// of any address; the kernels wait for it explicitly with counted vmcnt.
// The instruction is issued iff at least one lane is active: callers count
// only instructions they know have an active lane.
// TDBG_DMA_NT: the loads carry the nontemporal hint (experiment builds).
#ifndef TDBG_DMA_NT
#define TDBG_DMA_NT 0
#endif
#if TDBG_DMA_NT
#define TDBG_DMA_POLICY " nt"
#else
#define TDBG_DMA_POLICY ""
#endif
__device__ __forceinline__ void dma16(uint64_t src, uint32_t dst_wave) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off" TDBG_DMA_POLICY "\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(__builtin_amdgcn_readfirstlane(dst_wave))
      : "memory");
}

// Workgroup barrier for LDS only: no vmcnt drain (outstanding stores and the
// next tile's DMA stay in flight); "memory" keeps LDS accesses on their side.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

}  // namespace sc
}  // namespace tdbg
