// tdbg_view.hip -- LDS-free streaming unfilter for "view" tiles (gfx950).
//
// For pipelines whose filter 0 is BYTESHUFFLE and whose later filters are
// DOUBLE_DELTA and/or BIT_WIDTH_REDUCTION (the C1 and C5 shapes), a tile is a
// *view tile* when every stage before the final byteshuffle is the identity
// on the bytes it keeps:
//   - BWR with every window raw (bits >= 8*sizeof(T) or nbytes % sizeof(T),
//     bit_width_reduction_filter.cc:380-386): the reference copies window
//     after window, so the output is the first orig bytes of the input;
//   - DD whose data part took the raw fallback (bitsize >= 8*sizeof(T) - 1,
//     dd_compressor.cc:233-236,327-331) and whose metadata part (the 8-byte
//     byteshuffle header) holds n <= 2 values, which DoubleDelta stores
//     verbatim after its 9-byte header (dd_compressor.cc:238-248).
// Incompressible data (C5 "rand") is all view tiles.  The byteshuffle
// inverse then reads its TS planes straight from the filtered tile in HBM,
// so a wave streams 16-B output units with plane loads at arbitrary byte
// alignment and no LDS, no barriers: the kernel runs at copy speed.
//
// Work unit = (tile, 16 KiB output slice); waves are independent.  Every
// wave of a tile resolves the tile's metadata itself (the same bytes, so the
// same verdict).  A tile that is not a view tile -- any other metadata
// shape, any malformed field, any error the reference would report -- is
// appended to the LDS queue by its slice-0 wave and unfiltered by the fused
// LDS kernel next on the stream (then the general interpreter), which
// reproduces the reference's results and error precedence.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/tiledb_amd.h"
#include "tdbg_desc.h"
#include "tdbg_device.h"

namespace tdbg {

constexpr int VNT = 256;             // threads per workgroup (4 independent waves)
constexpr uint32_t VSLICE = 16384;   // output bytes per work unit
constexpr uint32_t VSLICES = 4;      // units per tile (view tiles are <= 64 KiB)
constexpr int VSTEPS = 8;            // 16-B units per lane in flight
constexpr uint32_t VMAXWIN = 512;    // BWR windows checked per tile (8 per lane)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const uint32_t vg_cu32;
typedef __attribute__((address_space(1))) const uint16_t vg_cu16;
typedef __attribute__((address_space(1))) const uint8_t vg_cu8;
typedef __attribute__((address_space(1))) v4u vg_u4;
typedef __attribute__((address_space(1))) uint8_t vg_u8;

// Global loads at arbitrary byte offsets, built from naturally aligned dword
// loads (two per value; both hit the same or adjacent cache lines) and
// v_alignbyte.  Only the dwords that hold requested bytes are read.
__device__ __forceinline__ uint32_t u32at(const uint8_t* p) {
  const uintptr_t a = (uintptr_t)p;
  const vg_cu32* q = (const vg_cu32*)(a & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(a & 3);
  const uint32_t lo = q[0];
  const uint32_t hi = sh ? q[1] : 0u;
  return __builtin_amdgcn_alignbyte(hi, lo, sh);
}
__device__ __forceinline__ uint32_t u16at(const uint8_t* p) {
  const uintptr_t a = (uintptr_t)p;
  const vg_cu32* q = (const vg_cu32*)(a & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(a & 3);
  const uint32_t lo = q[0];
  const uint32_t hi = sh == 3 ? q[1] : 0u;
  return __builtin_amdgcn_alignbyte(hi, lo, sh) & 0xffffu;
}
__device__ __forceinline__ uint32_t u8at(const uint8_t* p) { return *(vg_cu8*)p; }
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  return ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32) |
         __builtin_amdgcn_readfirstlane((uint32_t)v);
}

struct ViewSrc {
  const uint8_t* src;  // byteshuffled bytes of the chunk (global)
  uint32_t n;          // unfiltered chunk bytes
};

// Resolves a tile to its byteshuffled byte range, or returns false.  Wave
// uniform.  Stage order follows the reverse pass (filter_pipeline.cc:470-513):
// BWR (filter 2), DD (filter 1), byteshuffle (filter 0).
template <int TS, int DDW, int BW>
__device__ __forceinline__ bool view_resolve(const tdbg_plan& P, const uint8_t* tile, uint64_t fs,
                                             uint64_t expected, ViewSrc& v) {
  const uint32_t lane = threadIdx.x & 63;
  if (fs < 20) return false;
  // Tile::load_chunk_data (tile.cc:280-313): one chunk
  const uint64_t nch = (uint64_t)u32at(tile) | ((uint64_t)u32at(tile + 4) << 32);
  const uint32_t orig = u32at(tile + 8), fl = u32at(tile + 12), ml = u32at(tile + 16);
  if (nch != 1 || ml > fs - 20 || fl > fs - 20 - ml || orig != expected || orig > VSLICES * VSLICE)
    return false;
  const uint8_t* md = tile + 20;
  uint32_t mn = ml;
  const uint8_t* d = md + ml;
  uint32_t dn = fl;
  if constexpr (BW != 0) {
    // BitWidthReductionFilter::run_reverse (bit_width_reduction_filter.cc:352-404)
    const uint32_t dts = P.s[P.nstages - 1].dts;
    if (mn < 8) return false;
    const uint32_t borig = u32at(md), nw = u32at(md + 4), E = dts + 5;
    if (nw == 0 || nw > VMAXWIN || 8 + (uint64_t)nw * E > mn) return false;
    uint32_t bits[VMAXWIN / 64], nb[VMAXWIN / 64];
#pragma unroll
    for (int k = 0; k < (int)(VMAXWIN / 64); k++) {  // all loads first
      const uint32_t w = lane + 64 * k;
      const uint8_t* e = md + 8 + (w < nw ? w : 0) * E;
      bits[k] = u8at(e + dts);
      nb[k] = u32at(e + dts + 1);
    }
    bool nonraw = false;
    uint64_t sum = 0;
#pragma unroll
    for (int k = 0; k < (int)(VMAXWIN / 64); k++) {
      if (lane + 64 * k < nw) {
        nonraw |= !(bits[k] >= 8u * BW || (nb[k] % BW) != 0);
        sum += nb[k];
      }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) sum += __shfl_xor(sum, o, 64);
    if (__ballot(nonraw) != 0 || uni64(sum) != borig || borig > dn) return false;
    md += 8 + nw * E;
    mn -= 8 + nw * E;
    dn = borig;
  }
  if constexpr (DDW != 0) {
    // CompressionFilter::run_reverse (compression_filter.cc:303-347) +
    // DoubleDelta::decompress (dd_compressor.cc:314-404)
    if (mn < 8) return false;
    const uint32_t nmd = u32at(md), nd = u32at(md + 4);
    if (nd != 1 || nmd > 1 || 8 + 8 * (nmd + 1) > mn) return false;
    uint32_t p = 0;
    const uint8_t* nmdp = md;
    uint32_t nmn = 0;
    if (nmd == 1) {
      const uint32_t un0 = u32at(md + 8), cn0 = u32at(md + 12);
      if (un0 % DDW != 0 || cn0 != 9 + un0 || cn0 > dn) return false;
      const uint32_t b0 = u8at(d);
      const uint64_t n0 = (uint64_t)u32at(d + 1) | ((uint64_t)u32at(d + 5) << 32);
      if (n0 * DDW != un0 || !(n0 <= 2 || b0 >= 8u * DDW - 1)) return false;
      nmdp = d + 9;
      nmn = un0;
      p = cn0;
    }
    const uint32_t un1 = u32at(md + 8 + 8 * nmd), cn1 = u32at(md + 12 + 8 * nmd);
    if ((uint64_t)p + cn1 > dn || cn1 < 9 || cn1 - 9 != un1) return false;
    if (u8at(d + p) < 8u * DDW - 1) return false;  // not the raw fallback
    d = d + p + 9;
    dn = un1;
    md = nmdp;
    mn = nmn;
  }
  // ByteshuffleFilter::run_reverse (byteshuffle_filter.cc:111-166): one part
  if (mn < 8) return false;
  const uint32_t np = u32at(md), ps = u32at(md + 4);
  if (np != 1 || ps != dn || ps != orig) return false;
  v.src = d;
  v.n = ps;
  return true;
}

// 16-B output unit k (bytes [16k, 16k+16)) of an inverse byteshuffle with
// N = n / TS elements per plane; requires 16k + 16 <= N * TS.
template <int TS>
__device__ __forceinline__ void unit_load(const uint8_t* s, uint32_t N, uint32_t k, uint32_t (&r)[4]) {
  if constexpr (TS == 4) {
#pragma unroll
    for (int j = 0; j < 4; j++) r[j] = u32at(s + j * N + 4 * k);
  } else if constexpr (TS == 2) {
    r[0] = u32at(s + 8 * k);
    r[1] = u32at(s + 8 * k + 4);
    r[2] = u32at(s + N + 8 * k);
    r[3] = u32at(s + N + 8 * k + 4);
  } else {  // TS == 8: two elements, 8 planes x 2 bytes
#pragma unroll
    for (int j = 0; j < 4; j++) r[j] = u16at(s + (2 * j) * N + 2 * k) | (u16at(s + (2 * j + 1) * N + 2 * k) << 16);
  }
}

template <int TS>
__device__ __forceinline__ v4u unit_mix(const uint32_t (&r)[4]) {
  if constexpr (TS == 4) {
    const uint32_t a = __builtin_amdgcn_perm(r[1], r[0], 0x05010400u), b = __builtin_amdgcn_perm(r[3], r[2], 0x05010400u);
    const uint32_t c = __builtin_amdgcn_perm(r[1], r[0], 0x07030602u), d = __builtin_amdgcn_perm(r[3], r[2], 0x07030602u);
    return v4u{__builtin_amdgcn_perm(b, a, 0x05040100u), __builtin_amdgcn_perm(b, a, 0x07060302u),
               __builtin_amdgcn_perm(d, c, 0x05040100u), __builtin_amdgcn_perm(d, c, 0x07060302u)};
  } else if constexpr (TS == 2) {
    // plane 0 bytes in r[0..1], plane 1 bytes in r[2..3]: interleave
    return v4u{__builtin_amdgcn_perm(r[2], r[0], 0x05010400u), __builtin_amdgcn_perm(r[2], r[0], 0x07030602u),
               __builtin_amdgcn_perm(r[3], r[1], 0x05010400u), __builtin_amdgcn_perm(r[3], r[1], 0x07030602u)};
  } else {
    // r[j] = (plane 2j: e0 e1) | (plane 2j+1: e0 e1) << 16; element e = 8 bytes
    // byte b of element e = plane b, byte e.
    const uint32_t lo01 = __builtin_amdgcn_perm(r[1], r[0], 0x06040200u);  // e0: p0 p1 p2 p3
    const uint32_t lo23 = __builtin_amdgcn_perm(r[3], r[2], 0x06040200u);  // e0: p4 p5 p6 p7
    const uint32_t hi01 = __builtin_amdgcn_perm(r[1], r[0], 0x07050301u);  // e1: p0 p1 p2 p3
    const uint32_t hi23 = __builtin_amdgcn_perm(r[3], r[2], 0x07050301u);  // e1: p4 p5 p6 p7
    return v4u{lo01, lo23, hi01, hi23};
  }
}

// byte o of the unfiltered chunk (slow path: tails, unaligned outputs)
template <int TS>
__device__ __forceinline__ uint32_t unshuf_at(const uint8_t* s, uint32_t n, uint32_t N, uint32_t o) {
  return o < N * TS ? u8at(s + (o % TS) * N + o / TS) : u8at(s + o);
}

template <int TS>
__device__ __forceinline__ void view_slice(const ViewSrc& v, uint8_t* out, uint32_t q, bool plain) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t n = v.n, N = n / TS;
  const uint32_t b0 = q * VSLICE, b1 = n < b0 + VSLICE ? n : b0 + VSLICE;
  if (b0 >= b1) return;
  const uint32_t full = (N * TS) & ~15u;  // bytes covered by whole 16-B units
  uint32_t fast_end = b1 < full ? b1 : full;
  if ((((uintptr_t)out) & 15) != 0) fast_end = b0;  // unaligned output: byte path
  const uint32_t k0 = b0 / 16, k1 = fast_end > b0 ? fast_end / 16 : k0;
  for (uint32_t kb = k0; kb < k1; kb += 64 * VSTEPS) {
    uint32_t r[VSTEPS][4];
#pragma unroll
    for (int s = 0; s < VSTEPS; s++) {
      const uint32_t k = kb + s * 64 + lane;
      unit_load<TS>(v.src, N, k < k1 ? k : k1 - 1, r[s]);
    }
#pragma unroll
    for (int s = 0; s < VSTEPS; s++) {
      const uint32_t k = kb + s * 64 + lane;
      if (k < k1) {
        if (plain) *(vg_u4*)(out + 16 * k) = unit_mix<TS>(r[s]);
        else __builtin_nontemporal_store(unit_mix<TS>(r[s]), (vg_u4*)(out + 16 * k));
      }
    }
  }
  for (uint32_t o = (k1 > k0 ? 16 * k1 : b0) + lane; o < b1; o += 64)
    ((vg_u8*)out)[o] = (uint8_t)unshuf_at<TS>(v.src, n, N, o);
}

template <int TS, int DDW, int BW>
__global__ void __launch_bounds__(VNT) unfilter_view_kernel(const KParams kp) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wid = (uint64_t)blockIdx.x * (VNT / 64) + (threadIdx.x >> 6);
  const uint64_t nwv = (uint64_t)gridDim.x * (VNT / 64);
  const uint64_t nu = kp.ntiles * VSLICES;
  if ((kp.dbg_print & 1) && threadIdx.x == 0 && blockIdx.x < 2)
    printf("view b%u: nu %llu nwv %llu wid %llu\n", (unsigned)blockIdx.x, (unsigned long long)nu,
           (unsigned long long)nwv, (unsigned long long)wid);
  for (uint64_t u = wid; u < nu; u += nwv) {
    const uint64_t t = u / VSLICES;
    const uint32_t q = (uint32_t)(u % VSLICES);
    const uint8_t* in = (const uint8_t*)uni64((uint64_t)kp.in[t]);
    const uint64_t fs = uni64(kp.in_size[t]);
    uint8_t* out = (uint8_t*)uni64((uint64_t)kp.out[t]);
    const uint64_t os = uni64(kp.out_size[t]);
    uint64_t expected = os;
    bool ok = true;
    if (kp.flags & TDBG_TILE_OFFSETS) {
      ok = os >= 8;
      expected = os - 8;
    }
    ViewSrc v{nullptr, 0};
    ok = ok && view_resolve<TS, DDW, BW>(kp.plan, in, fs, expected, v);
    if (!ok) {
      if (q == 0 && lane == 0) kp.ldsq[1 + atomicAdd(kp.ldsq, 1u)] = (uint32_t)t;
      continue;
    }
    if (q == 0 && lane == 0 && kp.status) kp.status[t] = TDBG_OK;
    view_slice<TS>(v, out, q, (kp.dbg_print & 2) != 0);
  }
  if ((kp.dbg_print & 1) && threadIdx.x == 0 && blockIdx.x < 2) printf("view b%u: done\n", (unsigned)blockIdx.x);
}

}  // namespace tdbg

// view kinds: (TS, DD width, BWR width); 0 = stage absent
#define VIEW_SPECS(X) \
  X(1, 4, 0, 0)       \
  X(2, 8, 0, 0)       \
  X(3, 2, 0, 0)       \
  X(4, 4, 4, 4)       \
  X(5, 8, 8, 8)       \
  X(6, 4, 4, 0)       \
  X(7, 8, 8, 0)       \
  X(8, 2, 2, 2)

extern "C" uint32_t tdbg_view_select(const tdbg_plan* P) {
  // filter 0 = BYTESHUFFLE, then optionally DD, then optionally BWR, each
  // of the same element width (the datatype chain of C1/C5 pipelines)
  if (P->nstages < 1 || P->nstages > 3 || P->s[0].kind != TDBG_K_BYTESHUFFLE) return 0;
  const uint32_t ts = P->s[0].w;
  uint32_t dd = 0, bw = 0, i = 1;
  if (i < P->nstages && P->s[i].kind == TDBG_K_DD) dd = P->s[i++].w;
  if (i < P->nstages && P->s[i].kind == TDBG_K_BWR) {
    bw = P->s[i].w;
    if (P->s[i].dts != bw) return 0;
    i++;
  }
  if (i != P->nstages) return 0;
  if ((dd && dd != ts) || (bw && bw != ts)) return 0;
#define SEL(id, a, b, c) \
  if (ts == (a) && dd == (b) && bw == (c)) return id;
  VIEW_SPECS(SEL)
#undef SEL
  return 0;
}

extern "C" hipError_t tdbg_launch_view(const tdbg::KParams* kp, uint32_t grid, hipStream_t stream) {
  switch (kp->plan.view) {
#define LAUNCH(id, a, b, c)                                                                         \
  case id:                                                                                          \
    hipLaunchKernelGGL((tdbg::unfilter_view_kernel<a, b, c>), dim3(grid), dim3(tdbg::VNT), 0, stream, \
                       *kp);                                                                        \
    return hipGetLastError();
    VIEW_SPECS(LAUNCH)
#undef LAUNCH
    default:
      return hipErrorInvalidValue;
  }
}
