// tdbg_stream_common.h -- pieces shared by the streaming / tile kernels
// (tdbg_c5tile.hip, tdbg_c2tile.hip, tdbg_stream_small.hip, and the retired
// tdbg_stream*.hip of the experiments build): tile descriptors, the LDS-DMA
// of 16-B units, the LDS-only workgroup barrier, and the tile kernels' BWR
// window table and in-LDS BWR^-1.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tdbg_desc.h"
#include "tdbg_device.h"

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

// ---------------------------------------------------------------------------
// Pieces of the one-workgroup-per-tile kernels (tdbg_c5tile.hip,
// tdbg_c2tile.hip): the whole filtered image staged in LDS as dwords, BWR
// windows described by a table of {image offset of the window's data |
// kind << 20, window minimum} (kind 0: 8-bit, 1: 16-bit, 2: raw)
// ---------------------------------------------------------------------------
constexpr uint32_t OFFM = (1u << 20) - 1;

// bytes [o, o + 4) of a dword array (any alignment)
__device__ __forceinline__ uint32_t rd32(const uint32_t* a, uint32_t o) {
  return __builtin_amdgcn_alignbyte(a[(o >> 2) + 1], a[o >> 2], o & 3);
}

// bits [o, o + w) of x, sign- or zero-extended (BWR's stored values are
// signed for signed T, bit_width_reduction_filter.cc:491-528)
template <bool SGN>
__device__ __forceinline__ uint32_t ext(uint32_t x, uint32_t o, uint32_t w) {
  return SGN ? (uint32_t)__builtin_amdgcn_sbfe((int32_t)x, o, w) : __builtin_amdgcn_ubfe(x, o, w);
}

// The BWR window table of a chunk (one wave): window q's header [T min][u8
// bits][u32 bytes] sits at image byte e0 - 45 l + 9 q (lane l reads windows
// 5 l .. 5 l + 4, 45 bytes from e0); window sizes must be ws except the last
// (Lb bytes in all), stored widths 8 / 16 or raw (bits >= 32, or a byte count
// that is not a multiple of 4: bit_width_reduction_filter.cc:353-404); the
// compressed sizes' DPP scan places each window's data from image byte dst.
// Returns false (every lane) when a header is off or the sizes do not sum to
// fl; TAB[0 .. nwin) is written either way.  k0 / mn0: window 0's kind and
// minimum (lane 0's).
struct WinTab {
  bool ok;
  uint32_t k0, mn0;
};
__device__ __forceinline__ WinTab bwr_window_table(const uint32_t* P, uint2* TAB, uint32_t e0, uint32_t nwin,
                                                   uint32_t ws, uint32_t Lb, uint32_t fl, uint32_t dst, uint32_t l) {
  uint32_t R[13];
#pragma unroll
  for (int k = 0; k < 13; k++) R[k] = P[(e0 >> 2) + k];
  const uint32_t sh = e0 & 3;
  // (the byte shift sh + (o & 3) may reach 6: alignbyte takes it mod 4, so
  // the dword index steps by hand)
  auto rw = [&](int o) -> uint32_t {
    const uint32_t lo0 = R[o >> 2], hi0 = R[(o >> 2) + 1], hi1 = R[(o >> 2) + 2];
    const uint32_t s = sh + (uint32_t)(o & 3);
    return s < 4 ? __builtin_amdgcn_alignbyte(hi0, lo0, s) : __builtin_amdgcn_alignbyte(hi1, hi0, s - 4);
  };
  uint32_t cs[5], kind[5], mn[5];
  bool bad = false;
#pragma unroll
  for (int q = 0; q < 5; q++) {
    const uint32_t wi = 5 * l + q;
    const uint32_t vmin = rw(9 * q), bits = rw(9 * q + 4) & 0xffu, nb = rw(9 * q + 5);
    const bool in = wi < nwin;
    const uint32_t want = wi + 1 < nwin ? ws : Lb - ws * (nwin - 1);
    bad = bad || (in && nb != want);
    const bool raw = bits >= 32 || (nb & 3) != 0;
    bad = bad || (in && !raw && bits != 8 && bits != 16);
    kind[q] = raw ? 2 : bits == 8 ? 0 : 1;
    cs[q] = !in ? 0 : raw ? nb : bits == 8 ? nb >> 2 : nb >> 1;
    mn[q] = raw ? 0 : vmin;
  }
  const uint32_t s5 = cs[0] + cs[1] + cs[2] + cs[3] + cs[4];
  const uint32_t inc = wave_incscan_u32(s5);
  const bool ok = !__builtin_amdgcn_ballot_w64(bad) && __builtin_amdgcn_readlane(inc, 63) == fl;
  uint32_t off = dst + inc - s5;
#pragma unroll
  for (int q = 0; q < 5; q++) {
    if (5 * l + q < nwin) TAB[5 * l + q] = make_uint2(off | (kind[q] << 20), mn[q]);
    off += cs[q];
  }
  return WinTab{ok, (uint32_t)__builtin_amdgcn_readfirstlane(kind[0]), (uint32_t)__builtin_amdgcn_readfirstlane(mn[0])};
}

// BWR^-1 of a whole chunk's stream (bit_width_reduction_filter.cc:353-404)
// into LDS, in place over the image, in 16-B units of 4 elements: thread T of
// a 1,024-thread workgroup decodes units T + 1024 j (j < 4: at most 64 KiB of
// output).  A unit's 4 elements lie in one window (windows are >= 64
// elements), looked up per lane (esh = log2(elements per window), wlast =
// the last window).  Per round one wave-uniform decoder: every lane's window
// 8-bit (one dword read gives the unit), or the general form (five dwords
// realigned, then per element the window's kind: raw dword, 8-bit byte or
// 16-bit half, plus the minimum).  Every compressed read lands in registers
// before the one barrier after which the decoded units overwrite the image.
// NR: the wave's rounds with a unit below nun (all of them lie in the chunk),
// one instantiation each -- a round skipped behind a branch left its
// registers to be zeroed at every exit (40 VALU per wave, measured in the
// ISA); every path holds exactly one barrier.
template <bool SGN, int NR>
__device__ __forceinline__ void bwr_materialize_n(uint32_t* IMG, const uint2* TAB, uint32_t b, uint32_t esh,
                                                  uint32_t wlast, uint32_t w, uint32_t l) {
  v4u dv[NR];
  uint2 te[NR];
  uint32_t ea[NR];
#pragma unroll
  for (uint32_t j = 0; j < NR; j++) {
    const uint32_t e = 4 * (1024 * j + 64 * w + l);
    uint32_t W = e >> esh;
    W = W < wlast ? W : wlast;
    te[j] = TAB[W];
    const uint32_t kind = te[j].x >> 20;
    ea[j] = (te[j].x & OFFM) + b + ((e - (W << esh)) << kind);  // LDS byte of element e's compressed value
  }
  // (every round's five dwords first, so that all the reads are in flight
  // together; the decoders below pick from them)
  uint32_t D[NR][5];
#pragma unroll
  for (uint32_t j = 0; j < NR; j++) {
    const uint32_t* p = IMG + (ea[j] >> 2);
#pragma unroll
    for (int k = 0; k < 5; k++) D[j][k] = p[k];
  }
#pragma unroll
  for (uint32_t j = 0; j < NR; j++) {
    const uint32_t kind = te[j].x >> 20, mn = te[j].y, sh = ea[j] & 3;
    if (__builtin_amdgcn_ballot_w64(kind != 0) == 0) {
      const uint32_t y = __builtin_amdgcn_alignbyte(D[j][1], D[j][0], sh);
      dv[j] = v4u{ext<SGN>(y, 0, 8) + mn, ext<SGN>(y, 8, 8) + mn, ext<SGN>(y, 16, 8) + mn, ext<SGN>(y, 24, 8) + mn};
    } else {
      const uint32_t r0 = __builtin_amdgcn_alignbyte(D[j][1], D[j][0], sh), r1 = __builtin_amdgcn_alignbyte(D[j][2], D[j][1], sh);
      const uint32_t r2 = __builtin_amdgcn_alignbyte(D[j][3], D[j][2], sh), r3 = __builtin_amdgcn_alignbyte(D[j][4], D[j][3], sh);
      const bool b8 = kind == 0, raw = kind == 2;
      // element i: 8-bit -> byte i of r0; 16-bit -> half (i & 1) of r(i >> 1)
      const uint32_t e0 = ext<SGN>(r0, 0, b8 ? 8 : 16) + mn;
      const uint32_t e1 = ext<SGN>(r0, b8 ? 8 : 16, b8 ? 8 : 16) + mn;
      const uint32_t e2 = ext<SGN>(b8 ? r0 : r1, b8 ? 16 : 0, b8 ? 8 : 16) + mn;
      const uint32_t e3 = ext<SGN>(b8 ? r0 : r1, b8 ? 24 : 16, b8 ? 8 : 16) + mn;
      dv[j] = v4u{raw ? r0 : e0, raw ? r1 : e1, raw ? r2 : e2, raw ? r3 : e3};
    }
  }
  lds_barrier();  // every compressed byte is in registers: the stream may overwrite the image
#pragma unroll
  for (uint32_t j = 0; j < NR; j++) *(v4u*)(IMG + 4 * (1024 * j + 64 * w + l)) = dv[j];
}

template <bool SGN>
__device__ __forceinline__ void bwr_materialize(uint32_t* IMG, const uint2* TAB, uint32_t b, uint32_t esh,
                                                uint32_t wlast, uint32_t w, uint32_t l, uint32_t nun) {
  // (wave-uniform: round j has a unit below nun iff 1024 j + 64 w < nun)
  const uint32_t nr = nun <= 64 * w ? 0u : min(4u, (nun - 64 * w + 1023) >> 10);
  switch (__builtin_amdgcn_readfirstlane(nr)) {
    case 4: bwr_materialize_n<SGN, 4>(IMG, TAB, b, esh, wlast, w, l); break;
    case 3: bwr_materialize_n<SGN, 3>(IMG, TAB, b, esh, wlast, w, l); break;
    case 2: bwr_materialize_n<SGN, 2>(IMG, TAB, b, esh, wlast, w, l); break;
    case 1: bwr_materialize_n<SGN, 1>(IMG, TAB, b, esh, wlast, w, l); break;
    default: lds_barrier(); break;
  }
}

}  // namespace sc
}  // namespace tdbg
