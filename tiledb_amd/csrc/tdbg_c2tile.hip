// tdbg_c2tile.hip -- one-workgroup-per-tile unfilter kernel for BASELINE C2 /
// C2i: [BITSHUFFLE] (+ BIT_WIDTH_REDUCTION, a pass-through on FLOAT32) and
// [BITSHUFFLE, BIT_WIDTH_REDUCTION(256..4096)] on 4-byte integers, one chunk
// of 256 B .. 64 KiB (a multiple of 4) per tile; whole 64 KiB chunks take
// their own instantiation.
//
// The C5 tile kernel's shape (tdbg_c5tile.hip): a non-persistent
// 1024-thread workgroup per tile, the launch's workgroups dealt so that each
// XCD works through a contiguous eighth of the tiles; the whole filtered image
// lands in LDS by LDS-DMA; wave 0 parses the prefix while the rest is in
// flight:
//   * the tile + chunk header (Tile::load_chunk_data, tile.cc:280-313);
//   * C2i: the BWR metadata [u32 bytes][u32 nwin] + nwin x [i32 min][u8
//     bits][u32 bytes] (bit_width_reduction_filter.cc:353-380; the window
//     table is a DPP scan of the compressed sizes), then
//   * the bitshuffle metadata [u32 1][u32 65536] (bitshuffle_filter.cc:
//     128-167: one part, transformed in 8,192-B blocks).
// Bitshuffle^-1
// (bitshuffle_filter.cc:168-212): a block of 8,192 B is 32 bit rows of 256 B
// (row 8 b + k = bit k of byte b of each of its 2,048 elements); wave w < 8
// takes block w, lane t' its groups 4 t' .. 4 t' + 3 (elements 32 t' ..
// 32 t' + 31): one dword per row holds the four groups' bytes (C2i: BWR^-1
// on the way -- a 256-B row lies in one window, so the row's read is one
// wave-uniform 8-bit / 16-bit / raw decode from the compressed window).  Per
// byte plane, three bit-swap stages across the plane's eight row registers
// transpose the four groups' 8x8 bit matrices at once (72 VALU operations for
// 4 matrices); a 4x4 byte transpose per element index then assembles the
// elements.  The elements
// go back to LDS (XOR-swizzled 16-B units, after a barrier) and leave as
// lane-consecutive 16-B stores, 1 KiB per wave instruction (outputs 4-B
// aligned).
//
// Other shapes (multi-chunk tiles, windows, malformed, offsets tiles) are
// queued for the fused kernel, which runs on the queue in the same launch.
// Nothing is written to a tile's output before all its checks passed.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "../../include/tiledb_amd.h"
#include "tdbg_desc.h"
#include "tdbg_device.h"
#include "tdbg_launch.h"
#include "tdbg_stream_common.h"
#include "tdbg_hooks.h"

namespace tdbg {
namespace c2t {

using namespace sc;

constexpr int NT = 1024;
constexpr uint32_t OUTB = 65536;
constexpr uint32_t IMGU = 4256;  // 16-B units of the image stage (68,096 B)
constexpr uint32_t IMG_CAP = IMGU * 16 - 15;
constexpr uint32_t TABN = 320;
constexpr uint32_t GRID_CAP = 1u << 22;
constexpr uint32_t PFX = 192;  // 16-B units of the image prefix the parse reads (3 KiB)

struct Lds {
  uint32_t IMG[IMGU * 4];
  uint2 TAB[TABN];  // BWR window: {image offset of its data | kind << 20, minimum}
  uint32_t hd[8];   // verdict, log2(window bytes), nwin - 1, image byte of the bitshuffled data
};

// a 16-B unit at a 4-B aligned address (global_store_dwordx4 needs no more)
typedef uint32_t v4a __attribute__((ext_vector_type(4))) __attribute__((aligned(4)));
typedef __attribute__((address_space(1))) v4a g_a4;

__device__ __forceinline__ void decline(const KParams& kp, uint64_t t) {
  if (threadIdx.x == 0) {
    const uint32_t k = atomicAdd(kp.sq, 1u);
    if (k < kp.sq_cap) kp.sq[1 + k] = (uint32_t)t;
    else if (kp.status) kp.status[t] = TDBG_E_INTERNAL;
  }
}

// MODE 0: [BITSHUFFLE] (a FLOAT32 BWR is a pass-through with no metadata,
// bit_width_reduction_filter.cc:166-176); MODE 1: [BITSHUFFLE, BWR] on 4-byte
// integers.  One wave.
template <int MODE>
__device__ __forceinline__ void parse(Lds& L, uint32_t b, uint64_t fs, uint32_t os, uint32_t l) {
  const uint32_t* P = L.IMG;
  const uint32_t nlo = rd32(P, b), nhi = rd32(P, b + 4), orig = rd32(P, b + 8), fl = rd32(P, b + 12),
                 ml = rd32(P, b + 16);
  const uint32_t m = b + 20;
  // the bitshuffle md: parts [os - os % 8] and, when os % 8 != 0, [os % 8]
  // (bitshuffle_filter.cc:107-126)
  const uint32_t np = (os & 7) ? 2u : 1u, bml = 4 + 4 * np;
  auto bmd_ok = [&](uint32_t f) {
    return rd32(P, f) == np && rd32(P, f + 4) == os - (os & 7) && (np == 1 || rd32(P, f + 8) == (os & 7));
  };
  bool ok = nlo == 1 && nhi == 0 && orig == os && (uint64_t)ml + fl + 20 <= fs;
  if (MODE == 0) {
    ok = ok && ml == bml && fl == os && bmd_ok(m);
    if (l == 0) {
      L.hd[0] = ok ? 1u : 0u;
      L.hd[1] = 8;
      L.hd[2] = 0;
      L.hd[3] = m + bml;
    }
    return;
  }
  // BWR md; lane l: windows 5 l .. 5 l + 4 (45 bytes from e0)
  const uint32_t Lb = rd32(P, m), nwr = rd32(P, m + 4), ws = rd32(P, m + 13);
  ok = ok && Lb == os && nwr >= 1 && nwr <= TABN && ml == 8 + 9 * nwr + bml && ws >= 256 && ws <= 4096 &&
       (ws & (ws - 1)) == 0 && (Lb - 1) / ws + 1 == nwr;
  const uint32_t nwin = ok ? nwr : 1;
  const uint32_t dst = 20 + ml;  // image offset (from b) of the BWR data
  ok = ok && bwr_window_table(P, L.TAB, m + 8 + 45 * l, nwin, ws, Lb, fl, dst, l).ok;
  // the bitshuffle md after the windows' headers
  ok = ok && bmd_ok(m + 8 + 9 * nwin);
  if (l == 0) {
    L.hd[0] = ok ? 1u : 0u;
    L.hd[1] = 31 - __builtin_clz(ws);
    L.hd[2] = nwin - 1;
    L.hd[3] = 0;  // (the stream is decoded to LDS byte 0)
  }
}

__device__ __forceinline__ void tr4(uint32_t p0, uint32_t p1, uint32_t p2, uint32_t p3, uint32_t (&o)[4]) {
  const uint32_t a = __builtin_amdgcn_perm(p1, p0, 0x05010400u);
  const uint32_t b = __builtin_amdgcn_perm(p3, p2, 0x05010400u);
  const uint32_t c = __builtin_amdgcn_perm(p1, p0, 0x07030602u);
  const uint32_t d = __builtin_amdgcn_perm(p3, p2, 0x07030602u);
  o[0] = __builtin_amdgcn_perm(b, a, 0x05040100u);
  o[1] = __builtin_amdgcn_perm(b, a, 0x07060302u);
  o[2] = __builtin_amdgcn_perm(d, c, 0x05040100u);
  o[3] = __builtin_amdgcn_perm(d, c, 0x07060302u);
}

// 16-B unit u of the output at its XOR-swizzled LDS slot (the eight b128
// writes of a lane land in distinct bank groups)
__device__ __forceinline__ uint32_t uslot(uint32_t u) { return u ^ ((u >> 3) & 7u); }

// Everything after the parse: BWR^-1 (C2i), bitshuffle^-1, the stores.
// The chunk: os bytes; its first bitshuffle part n = os - os % 8 in nblk
// blocks of 8,192 B, the last one of nbl bytes whose first n8 = nbl / 4
// rounded down to 8 elements are bit-transposed (rows of R = n8 / 8 bytes);
// bytes [P, os) -- that block's other elements, then the second part -- are
// copied (bitshuffle_filter.cc:128-212).  FULL: os = 65,536.
template <int MODE, bool SGN, bool MAT, bool FULL>
__device__ __forceinline__ void c2_body(Lds& L, uint8_t* out, uint32_t b, uint32_t os, uint32_t w, uint32_t l) {
  if (FULL) os = OUTB;  // (a constant for the optimizer)
  const uint32_t n = os & ~7u, nblk = FULL ? 8u : (n + 8191) >> 13, nbl = n - 8192 * (nblk - 1);
  const uint32_t n8 = (nbl >> 2) & ~7u, R = FULL ? 256u : n8 >> 3, P = FULL ? OUTB : 8192 * (nblk - 1) + 4 * n8;
  uint32_t S = __builtin_amdgcn_readfirstlane(L.hd[3]);
  const uint32_t wsh = __builtin_amdgcn_readfirstlane(L.hd[1]), wlast = __builtin_amdgcn_readfirstlane(L.hd[2]);
  // C2i with a partial last block (its rows are not 256-B aligned windows):
  // BWR^-1 of the whole stream into LDS first, as its own pass (tile-uniform)
  const bool mat = MODE == 1 && (MAT || R != 256);
  if (mat) {
    bwr_materialize<SGN>(L.IMG, L.TAB, b, wsh - 2, wlast, w, l, 4096);
    lds_barrier();  // the bitshuffled stream at LDS byte 0
  }
  // BWR-output element e (C2i, decoded from its window; any lane)
  auto dec = [&](uint32_t e) -> uint32_t {
    uint32_t W = e >> (wsh - 2);
    W = W < wlast ? W : wlast;
    const uint2 te = L.TAB[W];
    const uint32_t kind = te.x >> 20;
    const uint32_t y = rd32(L.IMG, (te.x & OFFM) + b + ((e - (W << (wsh - 2))) << kind));
    return kind == 2 ? y : ext<SGN>(y, 0, 8u << kind) + te.y;
  };
  // the copied bytes [P, os) (at most 32): lane k of the last wave holds
  // dword k, read before the barrier that lets the elements overwrite them
  uint32_t tail = 0;
  if constexpr (!FULL)
    if (w == NT / 64 - 1 && P + 4 * l < os) tail = (MODE == 0 || mat) ? rd32(L.IMG, S + P + 4 * l) : dec((P >> 2) + l);
  // bitshuffle^-1: wave w < nblk takes block w, lane l its groups 4 l ..
  // 4 l + 3 (of the last block, those below R bytes a row are real)
  uint32_t E[4][8];
  if (w < nblk) {
    const bool part = w == nblk - 1 && R != 256;  // (wave-uniform)
    const uint32_t rs = part ? R : 256u;
    const uint32_t rb = S + 8192 * w + 4 * l;
    // row r's dword of lane l.  C2i: decoded from its BWR window on the way
    // (a 256-B row of a whole block is one window or part of one: a
    // wave-uniform decoder; lane q < 32 holds row q's window entry, each row
    // takes it by readlane)
    uint2 tq = make_uint2(0, 0);
    if (MODE == 1 && !mat) {
      const uint32_t Wq = (8192 * w + 256 * (l & 31)) >> wsh;
      tq = L.TAB[Wq < wlast ? Wq : wlast];
    }
    auto row = [&](uint32_t r) -> uint32_t {
      if (MODE == 0 || mat) return (S & 3) == 0 && !part ? L.IMG[(rb + r * 256) >> 2] : rd32(L.IMG, rb + r * rs);
      const uint32_t o = 8192 * w + 256 * r;
      uint32_t W = o >> wsh;
      W = W < wlast ? W : wlast;
      const uint32_t tx = __builtin_amdgcn_readlane(tq.x, r), mn = __builtin_amdgcn_readlane(tq.y, r);
      const uint32_t kind = tx >> 20;  // (scalar: the row's decoder is a wave-uniform branch)
      const uint32_t x = rd32(L.IMG, (tx & OFFM) + b + (((o - (W << wsh)) >> 2) << kind) + (l << kind));
      return kind == 2 ? x : ext<SGN>(x, 0, 8u << kind) + mn;
    };
    // Per byte plane pb: rows 8 pb + k (k = 0..7) in R[pb][k], byte g of
    // each = group g's 8x8 bit matrix (row k, bit e = element e).  Three
    // swap stages across the eight registers (blocks of 4, 2, 1 bits)
    // transpose the four matrices at once: R[pb][e] byte g = byte pb of
    // element 8 g + e.  One 4x4 byte transpose per e then assembles the
    // elements.
    uint32_t Rg[4][8];
    auto sw = [](uint32_t& x, uint32_t& z, int sh, uint32_t m) {
      const uint32_t t = ((x >> sh) ^ z) & m;
      z ^= t;
      x ^= t << sh;
    };
#pragma unroll
    for (int pb = 0; pb < 4; pb++) {
      uint32_t* D = Rg[pb];
#pragma unroll
      for (int k = 0; k < 8; k++) D[k] = row(8 * pb + k);
#pragma unroll
      for (int k = 0; k < 4; k++) sw(D[k], D[k + 4], 4, 0x0F0F0F0Fu);
#pragma unroll
      for (int k = 0; k < 8; k += 4) {
        sw(D[k], D[k + 2], 2, 0x33333333u);
        sw(D[k + 1], D[k + 3], 2, 0x33333333u);
      }
#pragma unroll
      for (int k = 0; k < 8; k += 2) sw(D[k], D[k + 1], 1, 0x55555555u);
    }
#pragma unroll
    for (int e = 0; e < 8; e++) {
      uint32_t o[4];
      tr4(Rg[0][e], Rg[1][e], Rg[2][e], Rg[3][e], o);
#pragma unroll
      for (int g = 0; g < 4; g++) E[g][e] = o[g];
    }
  }
  lds_barrier();  // every row read before the elements overwrite them
  if (w < nblk) {
    // lane bytes [8192 w + 128 l, +128) = units 512 w + 8 l + i
    const uint32_t u0 = 512 * w + 8 * l;
#pragma unroll
    for (int i = 0; i < 8; i++)
      *(v4u*)(L.IMG + 4 * uslot(u0 + i)) =
          v4u{E[i >> 1][4 * (i & 1)], E[i >> 1][4 * (i & 1) + 1], E[i >> 1][4 * (i & 1) + 2], E[i >> 1][4 * (i & 1) + 3]};
  }
  if (!FULL && P < os) {  // (uniform) the copied bytes over the last block's unused element slots
    lds_barrier();
    if (w == NT / 64 - 1 && P + 4 * l < os) {
      const uint32_t o = P + 4 * l;
      L.IMG[4 * uslot(o >> 4) + ((o >> 2) & 3)] = tail;
    }
  }
  lds_barrier();
  const uint32_t T = 64 * w + l;
  const uint32_t nfull = os >> 4;
#pragma unroll
  for (uint32_t r = 0; r < 4; r++) {
    const uint32_t u = 1024 * r + T;
    const v4u v = *(const v4u*)(L.IMG + 4 * uslot(u));
    if (FULL || u < nfull) {
      __builtin_nontemporal_store((v4a)v, (g_a4*)(out + 16 * u));
    } else if (u == nfull && (os & 15)) {  // the last 4, 8 or 12 bytes
      uint32_t* q = (uint32_t*)(out + 16 * u);
      q[0] = v.x;
      if ((os & 15) > 4) q[1] = v.y;
      if ((os & 15) > 8) q[2] = v.z;
    }
  }
}

template <int MODE, bool SGN, bool MAT>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(8, 8)))
unfilter_c2tile_kernel(const KParams kp, uint32_t base, uint32_t cnt) {
  __shared__ Lds L;
  const uint32_t w = wave_(), l = lane_();
  const uint32_t per = (cnt + 7) >> 3;
  const uint32_t j = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
  if (j >= cnt) return;
  const uint64_t t = (uint64_t)base + j;
  if (t >= kp.ntiles) return;
  if (kp.fbq && blockIdx.x == 0 && threadIdx.x == 0) kp.fbq[0] = 0;
  const uint64_t fs = kp.in_size[t];
  const uint8_t* in = kp.in[t];
  uint8_t* out = kp.out[t];
  const uint64_t os64 = kp.out_size[t];
  if ((kp.flags & TDBG_TILE_OFFSETS) || kp.chunks || os64 > OUTB || os64 < 256 || (os64 & 3) ||
      (((uintptr_t)out) & 3) || fs > IMG_CAP || fs < 28 + 8) {
    decline(kp, t);
    return;
  }
  const uint32_t os = __builtin_amdgcn_readfirstlane((uint32_t)os64);
  const uint32_t b = (uint32_t)((uintptr_t)in & 15);
  {
    const uint64_t a0 = (uint64_t)in & ~15ull;
    const uint32_t nu = (uint32_t)((b + fs + 15) >> 4);
    if (w == 0) {
#pragma unroll
      for (uint32_t k = 0; k < PFX / 64; k++)
        if (64 * k < nu && 64 * k + l < nu) dma16(a0 + 16ull * (64 * k + l), lds_addr(L.IMG) + 1024 * k);
    }
    uint32_t after = 0;
#pragma unroll
    for (uint32_t i = 0; i < (IMGU - PFX + NT - 1) / NT; i++) {
      const uint32_t u0 = PFX + 64 * (w + 16 * i);
      if (u0 < nu) {
        after++;
        if (u0 + l < nu) dma16(a0 + 16ull * (u0 + l), lds_addr(L.IMG) + 16 * u0);
      }
    }
    if (w == 0) {
      switch (__builtin_amdgcn_readfirstlane(after)) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
      }
      __builtin_amdgcn_s_setprio(3);
      parse<MODE>(L, b, fs, os, l);
      __builtin_amdgcn_s_setprio(0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  lds_barrier();
  if (__builtin_amdgcn_readfirstlane(L.hd[0]) == 0) {
    decline(kp, t);
    return;
  }
  // (a whole 64 KiB chunk -- the common case -- on its own instantiation)
#ifdef TDBG_C2T_FULLONLY  // (A/B build: no other chunk size)
  c2_body<MODE, SGN, MAT, true>(L, out, b, os, w, l);
#else
  if (os == OUTB) c2_body<MODE, SGN, MAT, true>(L, out, b, os, w, l);
  else c2_body<MODE, SGN, MAT, false>(L, out, b, os, w, l);
#endif
  if (threadIdx.x == 0) {
    if (kp.status) kp.status[t] = TDBG_OK;
    if (kp.stats) {
      uint64_t* s = kp.stats + TDBG_STAT_STRIDE * (1 + (blockIdx.x & 63));
      atomicAdd((unsigned long long*)&s[TDBG_STAT_FUSED_TILES], 1ull);
      atomicAdd((unsigned long long*)&s[TDBG_STAT_FUSED_BYTES], (unsigned long long)os);
      atomicAdd((unsigned long long*)&s[TDBG_STAT_STREAM_TILES], 1ull);
    }
  }
}

}  // namespace c2t
}  // namespace tdbg

// mode 0: [BITSHUFFLE] / [BITSHUFFLE, BWR pass-through]; 1: [BITSHUFFLE, BWR]
// on 4-byte integers (sgn: signed).  One workgroup per tile, launches of at
// most GRID_CAP tiles.
extern "C" hipError_t tdbg_launch_c2tile(const tdbg::KParams* kp, int mode, int sgn, hipStream_t s) {
  using namespace tdbg::c2t;
#ifdef TDBG_EXPERIMENTS
  static const bool mat = tdbg_hook("TDBG_C2T_MAT") != nullptr;  // A/B: BWR^-1 as its own LDS pass
#else
  constexpr bool mat = false;
#endif
  auto k = mode == 0 ? unfilter_c2tile_kernel<0, false, false>
           : mat     ? (sgn ? unfilter_c2tile_kernel<1, true, true> : unfilter_c2tile_kernel<1, false, true>)
                     : (sgn ? unfilter_c2tile_kernel<1, true, false> : unfilter_c2tile_kernel<1, false, false>);
  for (uint64_t b = 0; b < kp->ntiles; b += GRID_CAP) {
    const uint32_t cnt = (uint32_t)std::min<uint64_t>(kp->ntiles - b, GRID_CAP);
    TDBG_LAUNCH(k, dim3(8 * ((cnt + 7) / 8)), dim3(NT), s, *kp, (uint32_t)b, cnt);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}
