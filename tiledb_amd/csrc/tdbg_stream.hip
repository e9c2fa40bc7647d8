// tdbg_stream.hip -- streaming unfilter kernel for the headline pipeline
// [BYTESHUFFLE, DOUBLE_DELTA, BIT_WIDTH_REDUCTION] on 4-byte integers
// (BASELINE C5: dense int32, one 64 KiB chunk per tile), gfx950.
//
// The fused LDS kernel (tdbg_fast.hip) materialises every intermediate of
// a chunk in LDS: BWR's output (the ~59 KB DoubleDelta stream), then DD's
// output (the 64 KiB byteshuffled chunk), each written in place behind a
// workgroup barrier, and the byteshuffle gathers the final bytes from LDS.
// That needs ~80 KB of LDS per tile (two tiles per CU) and a chain of ~8
// barrier-separated phases per tile.  Here nothing but the filtered tile
// (~20 KB) is staged in the workgroup's LDS, so four tiles are in flight per
// CU, and a tile takes three workgroup barriers:
//
//   * Thread ownership follows the OUTPUT.  Byteshuffle⁻¹ of 16,384 int32
//     builds output unit j (16 bytes, elements 4j..4j+3) from dword j of
//     each of the four byte planes, i.e. from DoubleDelta values j, 4096+j,
//     8192+j and 12288+j (byteshuffle_filter.cc:111-166 -> blosc2
//     unshuffle).  Lane l of wave w owns units [1024w + 16l, +16) and so
//     decodes four runs of 16 consecutive DD values, one per plane; its
//     outputs leave registers through v_perm 4x4 byte transposes, straight
//     to HBM.  No DD output or byteshuffle input ever touches LDS.
//   * BWR⁻¹ (bit_width_reduction_filter.cc:353-404) is decoded lazily per
//     wave and per plane: the wave decodes, lane-linearly, the ~1 K dwords
//     of BWR output its 1,024 DD codes sit in, into a wave-private 4 KiB
//     scratch (no workgroup barrier: LDS is in order within a wave); every
//     lane then reads its 19 dwords of the DD bit stream from there.  The
//     window table (LDS) is built once per tile; every wave scans all window
//     headers itself, so the only barrier is the one that publishes it.
//   * DD⁻¹ (dd_compressor.cc:314-404): the lane realigns its 16 codes with
//     per-lane v_alignbyte/v_alignbit, extracts them at compile-time bit
//     positions (one instantiation per code width cb = bitsize+1 in 2..31),
//     and folds them into the affine double-delta aggregate (A = sum dd,
//     B = sum of running deltas); a DPP wave scan and one LDS exchange of
//     the 16 (plane, wave) totals give every lane its start state.  Values
//     0 and 1 (x0, x1 in the DD header) enter the same scan as pseudo codes
//     x0 and x1 - 2 x0.
//   * The next tile's image is copied into LDS by LDS-DMA
//     (global_load_lds_dwordx4, no VGPRs) while the current one computes
//     its values and stores them.
//
// The kernel takes only the tile shape it was built for (one chunk of
// 65,536 bytes, BWR windows of 8/16-bit or raw int32, DD bitsize 1..30, the
// exact metadata layout the reference writes, image <= CCAP bytes); any
// other tile is queued for the fused kernel, which runs on the queue right
// after (and sends what it declines on to the general interpreter), so the
// status and bytes of every tile stay the reference's.  Nothing is written
// to a tile's output before all its checks passed.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/tiledb_amd.h"
#include "tdbg_desc.h"
#include "tdbg_launch.h"
#include "tdbg_device.h"
#include "tdbg_stream_common.h"
#include "tdbg_hooks.h"

namespace tdbg {
namespace stream {

constexpr int NT = 256;              // threads per workgroup (4 wave64)
constexpr int NWV = NT / 64;
constexpr uint32_t NV = 16384;       // int32 values per chunk
constexpr uint32_t CCAP = sc::CODED_CAP;  // tile image bytes staged in LDS (16-B window)
constexpr uint32_t CPAD = 64;        // decode reads past the last window stay inside C
constexpr uint32_t WSD = 1024;       // scratch dwords per wave (256 16-B units)
constexpr uint32_t TABN = 256;       // BWR windows per chunk
#ifndef TDBG_STREAM_RD128
#define TDBG_STREAM_RD128 0  // experiment: 16-B scratch reads for the DD code realignment
#endif

struct Lds {
  uint32_t C[(CCAP + CPAD) / 4];
  uint2 TAB[TABN];                   // {LDS byte address | kind << 16, window minimum}
  uint32_t WS[NWV][WSD];
  uint32_t red[4][NWV][2];           // per plane and wave: DD aggregate (A, B)
  uint32_t wt[NWV];                  // compressed bytes of each wave's 64 windows
  uint32_t vd[NWV];                  // each wave's header verdict (ANDed after B2)
  uint32_t vok[NWV];                 // each wave's DD-header verdict (ANDed after P0)
  uint64_t clk[8];                   // diagnostics: phase clocks (TDBG_PROF)
};

using sc::batch_get;
using sc::batch_load;
using sc::Batch;
using sc::Desc;
using sc::g_u4;
using sc::lane_;
using sc::lds_barrier;
using sc::v4u;
using sc::wave_;

__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}
// bytes [o, o + 4) of C (any alignment)
__device__ __forceinline__ uint32_t c32(const Lds& L, uint32_t o) {
  const uint32_t* p = L.C + (o >> 2);
  return __builtin_amdgcn_alignbyte(p[1], p[0], o & 3);
}
__device__ __forceinline__ uint32_t c8(const Lds& L, uint32_t o) {
  return (L.C[o >> 2] >> (8 * (o & 3))) & 0xffu;
}

// ---------------------------------------------------------------------------
// the LDS-DMA of a tile image
// ---------------------------------------------------------------------------
// the image [in, in + fs) fits the staging window (16-B aligned units)
__device__ __forceinline__ bool fits(const Desc& d) {
  if (d.fs < 20 || d.fs > CCAP) return false;
  const uint64_t a0 = (uint64_t)d.in & ~15ull, a1 = ((uint64_t)d.in + d.fs + 15) & ~15ull;
  return a1 - a0 <= CCAP;
}

// LDS-DMA of the image's 16-B units into C: wave w's instruction r moves
// units [64 (4r + w), +64), lane-linear in LDS.
__device__ __forceinline__ void dma(Lds& L, const Desc& d) {
  const uint64_t a0 = (uint64_t)d.in & ~15ull, a1 = ((uint64_t)d.in + d.fs + 15) & ~15ull;
  const uint32_t n16 = (uint32_t)((a1 - a0) >> 4);
  const uint32_t w = wave_(), l = lane_();
  for (uint32_t r = 0; r * NT < n16; r++) {
    const uint32_t ub = r * NT + 64 * w;  // wave-uniform first unit
    if (ub + l < n16) sc::dma16(a0 + 16ull * (ub + l), sc::lds_addr(L.C) + 16 * ub);
  }
}

// ---------------------------------------------------------------------------
// BWR⁻¹ of one 16-B unit u of the BWR output (dwords 4u..4u+3)
// ---------------------------------------------------------------------------
struct Win {
  uint32_t wsh;    // log2(window bytes / 16)
  uint32_t wlast;  // nwin - 1
  uint32_t sh;     // LDS byte alignment of the data section (window data keep it)
};

template <bool SGN>
__device__ __forceinline__ uint32_t bfe8(uint32_t x, uint32_t o, uint32_t w) {
  return SGN ? (uint32_t)__builtin_amdgcn_sbfe((int32_t)x, o, w) : __builtin_amdgcn_ubfe(x, o, w);
}

template <bool SGN>
__device__ __forceinline__ v4u bwr_unit_te(const Lds& L, const Win& W, uint32_t u, uint32_t w, uint2 te) {
  const uint32_t kind = te.x >> 16;  // 0: 8-bit, 1: 16-bit, 2: raw
  const uint32_t o = (u - (w << W.wsh)) << 4;
  uint32_t a = (te.x & 0xffffu) + (o >> (2 - kind));
  a = a < CCAP + CPAD - 20 ? a : CCAP + CPAD - 20;  // units past the stream: any bytes, in bounds
  const uint32_t* p = L.C + (a >> 2);
  const uint32_t d0 = p[0], d1 = p[1], d2 = p[2], d3 = p[3], d4 = p[4];
  const uint32_t r0 = __builtin_amdgcn_alignbyte(d1, d0, W.sh);
  const uint32_t r1 = __builtin_amdgcn_alignbyte(d2, d1, W.sh);
  const uint32_t r2 = __builtin_amdgcn_alignbyte(d3, d2, W.sh);
  const uint32_t r3 = __builtin_amdgcn_alignbyte(d4, d3, W.sh);
  const uint32_t mn = te.y;
  const bool b8 = kind == 0, raw = kind == 2;
  // element i: 8-bit -> byte i of r0; 16-bit -> half (i & 1) of r(i >> 1)
  const uint32_t e0 = bfe8<SGN>(r0, 0, b8 ? 8 : 16) + mn;
  const uint32_t e1 = bfe8<SGN>(r0, b8 ? 8 : 16, b8 ? 8 : 16) + mn;
  const uint32_t e2 = bfe8<SGN>(b8 ? r0 : r1, b8 ? 16 : 0, b8 ? 8 : 16) + mn;
  const uint32_t e3 = bfe8<SGN>(b8 ? r0 : r1, b8 ? 24 : 16, b8 ? 8 : 16) + mn;
  return v4u{raw ? r0 : e0, raw ? r1 : e1, raw ? r2 : e2, raw ? r3 : e3};
}

template <bool SGN>
__device__ __forceinline__ v4u bwr_unit(const Lds& L, const Win& W, uint32_t u) {
  uint32_t w = u >> W.wsh;
  w = w < W.wlast ? w : W.wlast;
  return bwr_unit_te<SGN>(L, W, u, w, L.TAB[w]);
}

// all-8-bit fast form (the wave checked every lane's window)
template <bool SGN>
__device__ __forceinline__ v4u bwr_unit8(const Lds& L, const Win& W, uint32_t u, uint32_t w, uint2 te) {
  const uint32_t a = (te.x & 0xffffu) + ((u - (w << W.wsh)) << 2);
  const uint32_t* p = L.C + (a >> 2);
  const uint32_t r0 = __builtin_amdgcn_alignbyte(p[1], p[0], W.sh);
  const uint32_t mn = te.y;
  return v4u{bfe8<SGN>(r0, 0, 8) + mn, bfe8<SGN>(r0, 8, 8) + mn, bfe8<SGN>(r0, 16, 8) + mn,
             bfe8<SGN>(r0, 24, 8) + mn};
}

// 8-bit or raw windows (the wave checked that no lane meets a 16-bit window
// or a unit past the stream): the four dwords of a raw window's unit, or the
// four bytes of an 8-bit window's unit widened, chosen per lane
template <bool SGN>
__device__ __forceinline__ v4u bwr_unit8r(const Lds& L, const Win& W, uint32_t u, uint32_t w, uint2 te) {
  const bool raw = (te.x >> 16) != 0;
  const uint32_t a = (te.x & 0xffffu) + ((u - (w << W.wsh)) << (raw ? 4 : 2));
  const uint32_t* p = L.C + (a >> 2);
  const uint32_t d0 = p[0], d1 = p[1], d2 = p[2], d3 = p[3], d4 = p[4];
  const uint32_t r0 = __builtin_amdgcn_alignbyte(d1, d0, W.sh);
  const uint32_t r1 = __builtin_amdgcn_alignbyte(d2, d1, W.sh);
  const uint32_t r2 = __builtin_amdgcn_alignbyte(d3, d2, W.sh);
  const uint32_t r3 = __builtin_amdgcn_alignbyte(d4, d3, W.sh);
  const uint32_t mn = te.y;
  return v4u{raw ? r0 : bfe8<SGN>(r0, 0, 8) + mn, raw ? r1 : bfe8<SGN>(r0, 8, 8) + mn,
             raw ? r2 : bfe8<SGN>(r0, 16, 8) + mn, raw ? r3 : bfe8<SGN>(r0, 24, 8) + mn};
}

// ---------------------------------------------------------------------------
// DD⁻¹ codes of one lane and plane (code width CB = bitsize + 1)
// ---------------------------------------------------------------------------
// G: 20 dwords of BWR output starting at dword 8 + 2 * (Ms >> 1), Ms the
// first MSB-first stream dword needed (p = Ms & 1); n: alignbit amount.
// The stream's u64 words start at BWR-output byte 34 (two 17-byte DD
// headers precede them), so word q = bytes [34 + 8q, 42 + 8q): H[x] =
// alignbyte(G[x+1], G[x], 2) are the dwords at byte offset 2, and the
// MSB-first dword sequence swaps the halves of every word.
template <int CB>
__device__ __forceinline__ void dd_codes(const uint32_t (&H)[18], uint32_t p, uint32_t n, bool first,
                                         uint32_t x0, uint32_t x1, uint32_t (&xl)[16], uint32_t& Aout,
                                         uint32_t& Bout) {
  // M_j = p ? H[(j+1)^1] : H[j^1] as a bit select (v_bfi_b32): a plain
  // ternary lets the optimizer turn the pair into an indexed scratch load
  uint32_t pm = 0u - p;
  asm volatile("" : "+v"(pm));  // (opaque: the select stays one v_bfi_b32, not a cndmask + and_or)
  uint32_t M[17];
#pragma unroll
  for (int j = 0; j < 17; j++) M[j] = (pm & H[(j + 1) ^ 1]) | (~pm & H[j ^ 1]);
  uint32_t A[16];
#pragma unroll
  for (int j = 0; j < 16; j++) A[j] = __builtin_amdgcn_alignbit(M[j], M[j + 1], n);
  constexpr int B = CB - 1;
  uint32_t drun = 0, xrun = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) {
    constexpr int dummy = 0;
    (void)dummy;
    const int pos = i * CB;
    const int j = pos >> 5, o = pos & 31;
    const int32_t sg = __builtin_amdgcn_sbfe((int32_t)A[j], 31 - o, 1);
    const int o1a = o + 1;
    const int jm = j + (o1a >> 5), o1 = o1a & 31;
    uint32_t mag;
    if (o1 + B <= 32) {
      mag = __builtin_amdgcn_ubfe(A[jm], 32 - o1 - B, B);
    } else {
      mag = __builtin_amdgcn_alignbit(A[jm], A[jm + 1], 64 - o1 - B) & ((1u << B) - 1u);
    }
    uint32_t dd = (mag ^ (uint32_t)sg) - (uint32_t)sg;
    if (i == 0) dd = first ? x0 : dd;
    if (i == 1) dd = first ? x1 - 2u * x0 : dd;
    drun += dd;
    xrun += drun;
    xl[i] = xrun;
  }
  Aout = drun;
  Bout = xrun;
}

template <int CB>
__device__ __forceinline__ void dd_codes_at(const uint32_t* wsp, uint32_t g, uint32_t p, uint32_t n,
                                            bool first, uint32_t x0, uint32_t x1, uint32_t (&xl)[16],
                                            uint32_t& A, uint32_t& B) {
  // (H[x] = the dword at byte 2 of scratch dword g + x.  One 2-byte-aligned
  // ds_read_b32 per H[x] instead of the aligned pairs and a v_alignbyte
  // takes 18 VALU off each plane but made the kernel 19 % slower: 0.2782-
  // 0.2806 vs 0.2352-0.2363 ms per 12,500-tile launch, same box, same call,
  // profiles/r04/ab2_*.json -- misaligned LDS reads are slow on gfx950)
  uint32_t H[18];
  uint32_t G[20];
#if TDBG_STREAM_RD128
  // (experiment: six 16-B reads from g rounded down to 4 dwords, then a
  // 2-dword select -- lanes g ~ cb/2 dwords apart make the 8-B reads 2-4-way
  // bank conflicts; g is even, so g - g4 is 0 or 2)
  {
    const uint32_t g4 = g & ~3u;
    uint32_t sm = 0u - ((g >> 1) & 1u);
    asm volatile("" : "+v"(sm));
    uint32_t G4[24];
#pragma unroll
    for (int x = 0; x < 6; x++) {
      const v4u v = *(const v4u*)(wsp + g4 + 4 * x);
      G4[4 * x] = v.x;
      G4[4 * x + 1] = v.y;
      G4[4 * x + 2] = v.z;
      G4[4 * x + 3] = v.w;
    }
#pragma unroll
    for (int k = 0; k < 20; k++) G[k] = (sm & G4[k + 2]) | (~sm & G4[k]);
  }
#else
#pragma unroll
  for (int x = 0; x < 10; x++) {
    const uint2 v = *(const uint2*)(wsp + g + 2 * x);
    G[2 * x] = v.x;
    G[2 * x + 1] = v.y;
  }
#endif
#pragma unroll
  for (int x = 0; x < 18; x++) H[x] = __builtin_amdgcn_alignbyte(G[x + 1], G[x], 2);
  dd_codes<CB>(H, p, n, first, x0, x1, xl, A, B);
}

// ---------------------------------------------------------------------------
// the kernel
// ---------------------------------------------------------------------------
// DD aggregate combine: the block with aggregate (Ap, Bp) precedes `self`
// (nself codes): B = Bp + nself * Ap + B, A = Ap + A.
template <int CTRL, int ROWS>
__device__ __forceinline__ void scan_step(uint32_t& A, uint32_t& B, uint32_t nself) {
  const uint32_t Ap = dpp0<CTRL, ROWS>(A), Bp = dpp0<CTRL, ROWS>(B);
  B = B + Bp + nself * Ap;
  A = A + Ap;
}

#ifndef TDBG_STREAM_OCC
#define TDBG_STREAM_OCC 4  // waves per SIMD = workgroups per CU (128 VGPRs, 40.7 KB LDS)
#endif
// Diagnostics (KParams::prof, TDBG_PROF=1): per-workgroup shader-clock
// cycles per phase in slots 8..15 of the profile rows: 8 wait for the image
// (B1), 9 headers + window table, 10 B2 + DD header, 11 BWR decode into the
// wave scratch, 12 DD codes, 13 wave scans, 14 B3 + next DMA + start states
// + values, 15 byteshuffle transposes and stores.
struct Clock {
  uint64_t* out;
  uint64_t* acc;  // 8 accumulators in the workgroup's LDS (no SGPRs held for them)
  uint64_t t;
  __device__ __forceinline__ void init(uint64_t* o, uint64_t* lds_acc) {
    out = o;
    acc = lds_acc;
    if (!out) return;
    t = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0)
      for (int k = 0; k < 8; k++) acc[k] = 0;
  }
  __device__ __forceinline__ void mark(int k) {
    if (!out) return;
    const uint64_t n = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) acc[k - 8] += n - t;
    t = n;
  }
  __device__ __forceinline__ void flush() {
    if (!out || threadIdx.x != 0) return;
    for (int k = 0; k < 8; k++) out[blockIdx.x * TDBG_PROF_PHASES + 8 + k] = acc[k];
  }
};

// Plane K of one tile for one wave (code width CB): BWR⁻¹ of the wave's
// range into its scratch, the lane's 16 codes straight into xk (local
// running values), the local affine scan and the DPP wave scan.  Returns the
// lane's exclusive wave prefix (ae, be); lane 63 puts the wave total in red.
// The caller folds prefix and block start into xk after the plane's barrier.
template <int CB, int K, bool SGN>
__device__ __forceinline__ void plane(Lds& L, const Win& W, uint32_t w, uint32_t l, uint32_t x0, uint32_t x1,
                                      uint32_t (&xk)[16], uint32_t& ae, uint32_t& be, Clock& pc) {
  uint32_t* wsp = L.WS[w];
  constexpr int32_t cb = CB;
  const int32_t c0w = 4096 * K + 1024 * (int32_t)w - 2;
  const int32_t P0 = (c0w + 16 * (int32_t)l) * cb;
  const int32_t b0 = (P0 + 31) >> 5;
  const uint32_t n = (uint32_t)(32 * b0 - P0);
  const int32_t Ms = b0 - 1;
  const uint32_t p = (uint32_t)Ms & 1u;
  const int32_t es = 8 + 2 * (Ms >> 1);
  // the wave's range starts at lane 0's first dword
  const int32_t P00 = c0w * cb;
  const int32_t es0 = 8 + 2 * ((((P00 + 31) >> 5) - 1) >> 1);
  const uint32_t ulo = (uint32_t)es0 >> 2;
  __builtin_amdgcn_wave_barrier();
  // four rounds of 64 units (the wave needs <= 252 for cb <= 31), batched:
  // every table entry first, one uniform choice of the unit decoder, then
  // the reads
  uint32_t uu[4], wc[4];
  uint2 te[4];
  bool gen = false, k16 = false;
#pragma unroll
  for (int r = 0; r < 4; r++) {
    uu[r] = ulo + 64 * r + l;
    const uint32_t wu = uu[r] >> W.wsh;
    wc[r] = wu < W.wlast ? wu : W.wlast;
    te[r] = L.TAB[wc[r]];
    const uint32_t kind = te[r].x >> 16;
    gen |= kind != 0 || wu > W.wlast;
    k16 |= kind == 1 || wu > W.wlast;
  }
  v4u dv[4];
  if (__builtin_amdgcn_ballot_w64(gen) == 0) {
#pragma unroll
    for (int r = 0; r < 4; r++) dv[r] = bwr_unit8<SGN>(L, W, uu[r], wc[r], te[r]);
  } else if (__builtin_amdgcn_ballot_w64(k16) == 0) {
    // 8-bit and raw windows (C5 'active': most wave-planes meet a raw one)
#pragma unroll
    for (int r = 0; r < 4; r++) dv[r] = bwr_unit8r<SGN>(L, W, uu[r], wc[r], te[r]);
  } else {
    // (rare: one unit at a time, so the general decoder's temporaries do
    // not set the kernel's register count)
#pragma unroll
    for (int r = 0; r < 4; r++) {
      dv[r] = bwr_unit_te<SGN>(L, W, uu[r], wc[r], te[r]);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int r = 0; r < 4; r++) *(v4u*)(wsp + 4 * (64 * r + l)) = dv[r];
  __builtin_amdgcn_wave_barrier();
  pc.mark(11);
  const uint32_t g = (uint32_t)es - 4 * ulo;
  const bool first = K == 0 && w == 0 && l == 0;
  uint32_t A = 0, B = 0;
  dd_codes_at<CB>(wsp, g, p, n, first, x0, x1, xk, A, B);
  __builtin_amdgcn_wave_barrier();
  pc.mark(12);
  // inclusive wave scan of the (A, B) aggregates, 16 codes per lane
  const uint32_t As = A, Bs = B;
  scan_step<DPP_ROW_SHR1, 0xf>(A, B, 16);
  scan_step<DPP_ROW_SHR2, 0xf>(A, B, 32);
  scan_step<DPP_ROW_SHR4, 0xf>(A, B, 64);
  scan_step<DPP_ROW_SHR8, 0xf>(A, B, 128);
  scan_step<DPP_ROW_BCAST15, 0xa>(A, B, 16 * ((l & 15) + 1));
  scan_step<DPP_ROW_BCAST31, 0xc>(A, B, 16 * ((l & 31) + 1));
  // the lane's exclusive wave prefix: x_i = Xs + (16 l + i + 1) Ds + be +
  // (i + 1) ae + xk_i, with (Xs, Ds) the state at the start of the (plane,
  // wave) block
  ae = A - As;
  be = B - Bs - 16 * (A - As);
  if (l == 63) {
    L.red[K][w][0] = A;
    L.red[K][w][1] = B;
  }
  pc.mark(13);
}

// After plane K's barrier: the start state of every (K, wave) block from the
// four wave totals (scalar registers), then the one fold of the lane's
// prefix and its block's start into its 16 values.  (X, D) = state at the
// end of plane K - 1 on entry, of plane K on return.
template <int K>
__device__ __forceinline__ void plane_fold(const Lds& L, uint32_t w, uint32_t l, uint32_t& X, uint32_t& D,
                                          uint32_t ae, uint32_t be, uint32_t (&xk)[16]) {
  uint32_t Xs = 0, Ds = 0;
#pragma unroll
  for (int v = 0; v < NWV; v++) {
    if ((uint32_t)v == w) {
      Xs = X;
      Ds = D;
    }
    const uint32_t A = __builtin_amdgcn_readfirstlane(L.red[K][v][0]);
    const uint32_t B = __builtin_amdgcn_readfirstlane(L.red[K][v][1]);
    X = X + 1024u * D + B;
    D = D + A;
  }
  uint32_t t = Xs + be + 16u * l * Ds;
  const uint32_t st = Ds + ae;
#pragma unroll
  for (int i = 0; i < 16; i++) {
    t += st;
    xk[i] += t;
  }
}

// The four planes of one tile (code width CB).  PB == 4:
// each plane is followed by one workgroup barrier that publishes its (plane,
// wave) totals and its fold; PB == 1: the four planes run back to back and one
// barrier publishes all sixteen totals before the four folds (the lane keeps
// its four (ae, be) prefixes).  After the first barrier the waves' DD-header
// verdicts are ANDed (vok).  The barrier count depends only on PB (the
// caller's default case executes as many).  Measured (profiles/r04/
// barriers/): PB = 1 is 4 % faster on 12,500-tile launches (12 tiles per
// workgroup: shorter tiles, shorter tail), PB = 4 0.8 % faster on 100,000
// (98 per workgroup); the launcher picks by tiles per workgroup.
template <int CB, bool SGN, int PB>
__device__ __forceinline__ void planes4(Lds& L, const Win& W, uint32_t w, uint32_t l, uint32_t x0, uint32_t x1,
                                        uint32_t (&xl)[4][16], bool& ok, Clock& pc) {
  uint32_t X = 0, D = 0;
  auto verdicts = [&] {
    uint32_t all = 1;
#pragma unroll
    for (int v = 0; v < NWV; v++) all &= L.vok[v];
    ok = ok && all != 0;
  };
  if constexpr (PB == 1) {
    uint32_t ae[4], be[4];
    plane<CB, 0, SGN>(L, W, w, l, x0, x1, xl[0], ae[0], be[0], pc);
    plane<CB, 1, SGN>(L, W, w, l, x0, x1, xl[1], ae[1], be[1], pc);
    plane<CB, 2, SGN>(L, W, w, l, x0, x1, xl[2], ae[2], be[2], pc);
    plane<CB, 3, SGN>(L, W, w, l, x0, x1, xl[3], ae[3], be[3], pc);
    sc::lds_barrier();  // (also frees C and TAB for the next tile's DMA)
    verdicts();
    if (ok) {
      plane_fold<0>(L, w, l, X, D, ae[0], be[0], xl[0]);
      plane_fold<1>(L, w, l, X, D, ae[1], be[1], xl[1]);
      plane_fold<2>(L, w, l, X, D, ae[2], be[2], xl[2]);
      plane_fold<3>(L, w, l, X, D, ae[3], be[3], xl[3]);
    }
  } else {
    uint32_t ae = 0, be = 0;
    plane<CB, 0, SGN>(L, W, w, l, x0, x1, xl[0], ae, be, pc);
    sc::lds_barrier();
    verdicts();
    if (ok) plane_fold<0>(L, w, l, X, D, ae, be, xl[0]);
    plane<CB, 1, SGN>(L, W, w, l, x0, x1, xl[1], ae, be, pc);
    sc::lds_barrier();
    if (ok) plane_fold<1>(L, w, l, X, D, ae, be, xl[1]);
    plane<CB, 2, SGN>(L, W, w, l, x0, x1, xl[2], ae, be, pc);
    sc::lds_barrier();
    if (ok) plane_fold<2>(L, w, l, X, D, ae, be, xl[2]);
    plane<CB, 3, SGN>(L, W, w, l, x0, x1, xl[3], ae, be, pc);
    sc::lds_barrier();  // (also frees C and TAB for the next tile's DMA)
    if (ok) plane_fold<3>(L, w, l, X, D, ae, be, xl[3]);
  }
}

// Queue the declined tiles of one batch (bit i of mask: the workgroup's tile
// base + i) for the fused kernel, which writes their statuses.  Wave 0.
__device__ __forceinline__ void queue_batch(const KParams& kp, uint64_t mask, uint32_t base) {
  const uint32_t l = threadIdx.x & 63;
  uint32_t b0 = 0;
  if (l == 0) b0 = atomicAdd(kp.sq, (uint32_t)__builtin_popcountll(mask));
  b0 = __builtin_amdgcn_readfirstlane(b0);
  if ((mask >> l) & 1) {
    const uint32_t k = b0 + (uint32_t)__builtin_popcountll(mask & ((1ull << l) - 1));
    const uint32_t t = (uint32_t)(blockIdx.x + (uint64_t)(base + l) * gridDim.x);
    // (k < sq_cap always holds -- a tile is queued at most once per launch and
    // sq_cap = ntiles -- but a tile that would not fit must not be lost: it
    // gets a status instead of silently keeping whatever its status held)
    if (k < kp.sq_cap) kp.sq[1 + k] = t;
    else if (kp.status) kp.status[kp.chunks ? kp.chunks[t].tile : t] = TDBG_E_INTERNAL;
  }
}

template <bool SGN, int STM, int PB>
__global__ void __launch_bounds__(NT, TDBG_STREAM_OCC) unfilter_stream_kernel(const KParams kp) {
  __shared__ Lds L;
  const uint64_t G = gridDim.x;
  uint64_t ntl = kp.ntiles;
  if (kp.ntiles_dev) {
    const uint64_t c = (uint32_t)__builtin_amdgcn_readfirstlane(*kp.ntiles_dev);
    ntl = c < ntl ? c : ntl;
  }
  // the fused kernel's fallback queue starts empty for this launch (it runs
  // next on the same stream and is the only one to append; chunk mode: the
  // directory's scan kernel cleared it, and may have appended, so fbq is
  // not passed here)
  if (kp.fbq && blockIdx.x == 0 && threadIdx.x == 0) kp.fbq[0] = 0;
  const bool chunked = kp.chunks != nullptr;
  const uint32_t w = wave_();
  Clock pc;
  pc.init(kp.prof, L.clk);
  uint64_t ok_tiles = 0, ok_bytes = 0;
  Desc cur{};
  bool cur_dma = false;
  bool stored = false;  // the last iteration issued its 16 output stores after the DMA
  // The workgroup's k-th tile is blockIdx.x + k G; descriptors come 64 at a
  // time (bt, batch base bbase).  This kernel owns the tiles of at most
  // CCAP bytes (it decodes them or queues them); the bigger ones belong to
  // the raw-DoubleDelta kernel and are skipped a batch at a time (mine: the
  // batch's owned tiles), so a launch of raw tiles costs this kernel two
  // descriptor loads per workgroup, not a walk over every tile.
  Batch bt{0, 0, 0, 0};
  uint64_t bbase = ~0ull, mine = 0;
  // smallest owned tile index >= from (false: none left)
  auto next_owned = [&](uint64_t from, uint64_t& nit) -> bool {
    for (;;) {
      const uint64_t base = from - from % 64;
      if (blockIdx.x + base * G >= ntl) return false;
      if (base != bbase) {
        bt = batch_load(kp, base, ntl);
        const uint64_t jl = blockIdx.x + (base + lane_()) * G;
        mine = __builtin_amdgcn_ballot_w64(jl < ntl && bt.fs <= CCAP);
        bbase = base;
      }
      const uint64_t m = mine & (~0ull << (from - base));
      if (m) {
        nit = base + (uint64_t)__builtin_ctzll(m);
        return true;
      }
      from = base + 64;
    }
  };
  uint64_t it = 0;
  bool have = next_owned(0, it);
  if (have) {
    cur = batch_get(bt, (uint32_t)(it % 64), blockIdx.x + it * G);
    cur_dma = fits(cur);
    if (cur_dma) dma(L, cur);
  }
  // tiles left to the fused kernel, this batch: bit i = batch position i
  // (queued with one atomic per workgroup and batch: a single global counter
  // taking one atomic per tile serialises the whole grid on it)
  uint64_t dmask = 0;
  while (have) {
    const uint32_t l = lane_();
    // A tile whose image does not fit is declined without touching LDS (and
    // without barriers: no wave reads C for it, and the last tile that did
    // passed B3).
    bool ok = cur_dma && !(kp.flags & TDBG_TILE_OFFSETS) && cur.os == NV * 4 &&
              (((uintptr_t)cur.out) & 15) == 0;
    uint32_t xl[4][16];
    if (cur_dma) {
    // B1: this tile's DMA has landed (vmcnt counts in issue order: the last
    // iteration's 16 output stores, issued after the DMA, may stay in flight)
    // (the STM == 3 timing ablation issues its stores under a branch almost
    // never taken, so it waits for everything)
    if (stored && STM != 3) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
    pc.mark(8);
    // ---- tile + chunk header (Tile::load_chunk_data, tile.cc:280-313) -----
    // Every read below is issued speculatively (all addresses lie inside C
    // whatever the bytes say) so the parse is two LDS round trips; the
    // checks then decide.  BWR md: [u32 orig][u32 nwin] + nwin x [i32 min]
    // [u8 bits][u32 nbytes] (bit_width_reduction_filter.cc:353-380), then the
    // compression frame's md (compression_filter.cc:413-486).
    // the chunk header sits after the tile's u64 chunk count, or (chunk mode)
    // the image starts with it
    const uint32_t ho = chunked ? 0u : 8u;
    const uint32_t b = (uint32_t)((uintptr_t)cur.in & 15);
    const uint32_t m = b + ho + 12;
    uint32_t ml = 0, fl = 0, dst = 0, nwin = 0, wsh = 0, ws = 0;
    if (ok) {
      const uint32_t nlo = c32(L, b), nhi = c32(L, b + 4), orig = c32(L, b + ho);
      fl = c32(L, b + ho + 4);
      ml = c32(L, b + ho + 8);
      const uint32_t Lb = c32(L, m), nwr = c32(L, m + 4), ws0 = c32(L, m + 13);
      // Wave w parses windows [64 w, 64 w + 64), lane l window 64 w + l (9
      // bytes at e0), and writes their table entries with offsets relative
      // to its part; the part totals go through LDS (B2) and each wave then
      // adds its part's prefix to its own entries (B2b).
      const uint32_t wi = 64 * w + l;
      const uint32_t e0 = m + 8 + 9 * wi;
      const uint32_t* rp = L.C + (e0 >> 2);
      const uint32_t R0 = rp[0], R1 = rp[1], R2 = rp[2], R3 = rp[3];
      const uint32_t vmin = __builtin_amdgcn_alignbyte(R1, R0, e0 & 3);
      const uint32_t E1 = __builtin_amdgcn_alignbyte(R2, R1, e0 & 3);
      const uint32_t E2 = __builtin_amdgcn_alignbyte(R3, R2, e0 & 3);
      const uint32_t bits = E1 & 0xffu, nb = __builtin_amdgcn_alignbyte(E2, E1, 1);
      nwin = nwr < TABN ? nwr : TABN;
      const uint32_t f = m + 8 + 9 * nwin;
      const uint32_t d0 = c32(L, f), d1 = c32(L, f + 4), d2 = c32(L, f + 8), d3 = c32(L, f + 12),
                     d4 = c32(L, f + 16), d5 = c32(L, f + 20);
      dst = m + ml;
      ws = nwin > 1 ? ws0 : 256;
      ok = (chunked || (nlo == 1 && nhi == 0)) && orig == NV * 4 && (uint64_t)ml + fl + ho + 12 <= cur.fs && nwr >= 1 &&
           nwr <= TABN && ml == 8 + 9 * nwr + 24 && d0 == 1 && d1 == 1 && d2 == 8 && d3 == 17 &&
           d4 == NV * 4 && d5 + 17 == Lb && ws >= 64 && ws <= 4096 && (ws & (ws - 1)) == 0 &&
           (Lb - 1) / ws + 1 == nwin;
      wsh = ok ? 31 - __builtin_clz(ws) - 4 : 0;
      if (ok) {
        const uint32_t want = wi + 1 < nwin ? ws : Lb - ws * (nwin - 1);
        const bool in = wi < nwin;
        const bool raw = bits >= 32 || (nb & 3) != 0;
        const bool bad = in && (nb != want || (!raw && bits != 8 && bits != 16));
        const uint32_t kind = raw ? 2 : bits == 8 ? 0 : 1;
        const uint32_t cs = !in ? 0 : raw ? nb : bits == 8 ? nb >> 2 : nb >> 1;
        const uint32_t inc = wave_incscan_u32(cs);
        ok = !__builtin_amdgcn_ballot_w64(bad);
        if (in) L.TAB[wi] = make_uint2((inc - cs) | (kind << 16), raw ? 0 : vmin);
        if (l == 63) L.wt[w] = inc;
      }
    }
    pc.mark(9);
    // Barrier reachability is uniform by construction: every workgroup
    // barrier below depends only on cur_dma (a function of readlane'd
    // descriptors); the data-dependent verdicts are published through LDS
    // and read back after a barrier, every wave taking the AND of all.
    if (l == 0) L.vd[w] = ok ? 1u : 0u;
    lds_barrier();  // B2: part tables, part totals, header verdicts
    {
      uint32_t all = 1, tot = 0, pre = dst;
#pragma unroll
      for (int v = 0; v < NWV; v++) {
        all &= L.vd[v];
        const uint32_t t = __builtin_amdgcn_readfirstlane(L.wt[v]);
        if ((uint32_t)v < w) pre += t;
        tot += t;
      }
      ok = ok && all != 0 && tot == fl;
      // each wave makes its own entries absolute (image offset of the
      // window's compressed data)
      const uint32_t wi = 64 * w + l;
      if (ok && wi < nwin) L.TAB[wi].x += pre;
    }
    lds_barrier();  // B2b: the window table
    if (!ok) {
      wsh = 0;
      nwin = 1;
    }
    uint32_t cb = 0, x0 = 0, x1 = 0;
    Win W{wsh, nwin - 1, dst & 3};
    if (ok) {
      // DD headers: BWR output bytes [0, 34) = c0 (the byteshuffle md) and c1's
      // header (dd_compressor.cc:314-345); lanes 0..3 decode units 0..3
      const v4u h = bwr_unit<SGN>(L, W, l < 4 ? l : 3);
      auto dw = [&](int k) -> uint32_t { return __builtin_amdgcn_readlane(h[k & 3], k >> 2); };
      auto at = [&](int o) -> uint32_t {
        return __builtin_amdgcn_alignbyte(dw((o >> 2) + 1), dw(o >> 2), o & 3);
      };
      const uint32_t num0lo = at(1), num0hi = at(5), np = at(9), psz = at(13);
      const uint32_t bs = at(17) & 0xffu, num1lo = at(18), num1hi = at(22);
      x0 = at(26);
      x1 = at(30);
      cb = bs + 1;
      const uint32_t comp1 = c32(L, m + 8 + 9 * nwin + 20);
      const uint32_t words = ((NV - 2) * cb + 63) / 64;
      ok = num0lo == 2 && num0hi == 0 && np == 1 && psz == NV * 4 && bs >= 1 && bs <= 30 &&
           num1lo == NV && num1hi == 0 && comp1 == 17 + 8 * words;
    }
    pc.mark(10);
    // ---- four planes: BWR⁻¹ into the wave scratch, codes, wave scan; one
    // barrier per plane publishes the (plane, wave) totals, and the lane's
    // prefix and its block's start fold into its values in one pass -----
    if (l == 0) L.vok[w] = ok ? 1u : 0u;
    // one instantiation per code width: the plane loop unrolls and every
    // plane's codes land directly in their value registers
    switch (ok ? cb : 0u) {
#define TDBG_CB(c) \
  case c: planes4<c, SGN, PB>(L, W, w, l, x0, x1, xl, ok, pc); break;
      TDBG_CB(2) TDBG_CB(3) TDBG_CB(4) TDBG_CB(5) TDBG_CB(6) TDBG_CB(7) TDBG_CB(8) TDBG_CB(9)
      TDBG_CB(10) TDBG_CB(11) TDBG_CB(12) TDBG_CB(13) TDBG_CB(14) TDBG_CB(15) TDBG_CB(16)
      TDBG_CB(17) TDBG_CB(18) TDBG_CB(19) TDBG_CB(20) TDBG_CB(21) TDBG_CB(22) TDBG_CB(23)
      TDBG_CB(24) TDBG_CB(25) TDBG_CB(26) TDBG_CB(27) TDBG_CB(28) TDBG_CB(29) TDBG_CB(30)
      TDBG_CB(31)
#undef TDBG_CB
      default:  // declined (ok is false): the same barriers as planes4
        ok = false;
        // (defined values: an undefined xl here lets the register allocator
        // keep the last tile's values live around the loop)
#pragma unroll
        for (int k = 0; k < 4; k++)
#pragma unroll
          for (int i = 0; i < 16; i++) xl[k][i] = 0;
#pragma unroll
        for (int k = 0; k < PB; k++) lds_barrier();
        break;
    }
    }  // cur_dma
    // tiles bigger than CCAP belong to the raw-DoubleDelta kernel, which runs
    // next on every tile and queues the ones it does not take itself
    if (!ok && cur.fs <= CCAP) dmask |= 1ull << (it % 64);
    const uint64_t cbase = it - it % 64;
    uint64_t nit = 0;
    const bool hn = next_owned(it + 1, nit);  // (may load later batches: before the DMA)
    if (!hn || nit - nit % 64 != cbase) {
      if (dmask && w == 0) queue_batch(kp, dmask, (uint32_t)cbase);
      dmask = 0;
    }
    Desc nxt{};
    bool nxt_dma = false;
    if (hn) {
      nxt = batch_get(bt, (uint32_t)(nit % 64), blockIdx.x + nit * G);
      nxt_dma = fits(nxt);
      if (nxt_dma) dma(L, nxt);
    }
    if (ok) {
      pc.mark(14);
      // byteshuffle⁻¹: unit i of the lane = dword i of the four planes,
      // transposed bytewise (out dword b byte k = plane k value byte b).
      // The lane's 16 units are 256 contiguous bytes, so lane-strided stores
      // would touch 64 lines per instruction; they go through the wave's
      // 4 KiB scratch in four rounds instead: units half u, lanes half h.
      // Lanes [32h, 32h + 32) put units [8u, 8u + 8) in row l & 31 (128 B,
      // slot j at j ^ (row & 7): conflict-free), then each store
      // instruction writes 8 whole 128-B lines (8 lanes per line).
      uint8_t* o = cur.out + 16u * (1024u * w);
      uint32_t* wsp = L.WS[w];
      // the 4x4 byte transposes of all 16 units, every lane active, in place
      // (unit i's four output dwords replace the four plane values they came
      // from); only the scratch writes below run under the half mask
#pragma unroll
      for (int i = 0; i < 16; i++) {
        const uint32_t t0 = __builtin_amdgcn_perm(xl[1][i], xl[0][i], 0x05010400u);
        const uint32_t t1 = __builtin_amdgcn_perm(xl[1][i], xl[0][i], 0x07030602u);
        const uint32_t t2 = __builtin_amdgcn_perm(xl[3][i], xl[2][i], 0x05010400u);
        const uint32_t t3 = __builtin_amdgcn_perm(xl[3][i], xl[2][i], 0x07030602u);
        xl[0][i] = __builtin_amdgcn_perm(t2, t0, 0x05040100u);
        xl[1][i] = __builtin_amdgcn_perm(t2, t0, 0x07060302u);
        xl[2][i] = __builtin_amdgcn_perm(t3, t1, 0x05040100u);
        xl[3][i] = __builtin_amdgcn_perm(t3, t1, 0x07060302u);
      }
#pragma unroll
      for (int u = 0; u < 2; u++) {
#pragma unroll
        for (int h = 0; h < 2; h++) {
          __builtin_amdgcn_wave_barrier();
          if ((l >> 5) == (uint32_t)h) {
            const uint32_t row = l & 31;
#pragma unroll
            for (int j = 0; j < 8; j++) {
              const int i = 8 * u + j;
              *(v4u*)(wsp + 4 * (8 * row + (j ^ (row & 7)))) = v4u{xl[0][i], xl[1][i], xl[2][i], xl[3][i]};
            }
          }
          __builtin_amdgcn_wave_barrier();
#pragma unroll
          for (int q = 0; q < 4; q++) {
            const uint32_t row = 8 * q + (l >> 3), sl = l & 7;
            const v4u y = *(const v4u*)(wsp + 4 * (8 * row + (sl ^ (row & 7))));
            g_u4* dstp = (g_u4*)(o + 16u * (16u * (32u * h + row) + 8u * u + sl));
            if (STM == 1) __builtin_nontemporal_store(y, dstp);
            else if (STM == 3) {  // timing ablation: no stores (output left unwritten)
              if (y.x == 0x9e3779b9u && y.y == 0x7f4a7c15u) *dstp = y;
            } else *dstp = y;
          }
        }
      }
      ok_tiles++;
      ok_bytes += cur.os;
      // (chunk mode: the directory pass wrote the tile's status)
      if (threadIdx.x == 0 && kp.status && !chunked) kp.status[cur.t] = TDBG_OK;
    }
    cur = nxt;
    cur_dma = nxt_dma;
    stored = ok;
    it = nit;
    have = hn;
    pc.mark(15);
  }
  pc.flush();
  if (kp.stats && threadIdx.x == 0 && ok_tiles) {
    if (chunked) {  // (the directory pass counted the tiles)
      atomicAdd((unsigned long long*)&kp.stats[TDBG_STAT_STREAM_CHUNKS], (unsigned long long)ok_tiles);
    } else {
      atomicAdd((unsigned long long*)&kp.stats[TDBG_STAT_FUSED_TILES], (unsigned long long)ok_tiles);
      atomicAdd((unsigned long long*)&kp.stats[TDBG_STAT_FUSED_BYTES], (unsigned long long)ok_bytes);
      atomicAdd((unsigned long long*)&kp.stats[TDBG_STAT_STREAM_TILES], (unsigned long long)ok_tiles);
    }
  }
}

}  // namespace stream
}  // namespace tdbg

// Persistent grid: one workgroup per CU for every TDBG_STREAM_OCC waves per
// SIMD the registers allow (LDS would hold four).
extern "C" uint32_t tdbg_stream_grid(int cus) {
  static const int g = tdbg_hook("TDBG_STREAM_GRID") ? atoi(tdbg_hook("TDBG_STREAM_GRID")) : 0;  // experiments
  return g > 0 ? (uint32_t)g : (uint32_t)cus * TDBG_STREAM_OCC;
}

// Launch: sgn = the BWR stage's integer type is signed.
extern "C" hipError_t tdbg_launch_stream(const tdbg::KParams* kp, uint32_t grid, int sgn, hipStream_t s) {
  using namespace tdbg::stream;
  // store mode: 1 nontemporal (5 % faster than plain stores on C5 active,
  // profiles/r03_*), 3 no stores (timing ablation only, signed tiles)
  static const int stm = tdbg_hook("TDBG_STREAM_STORE") ? atoi(tdbg_hook("TDBG_STREAM_STORE")) : 1;
  // one barrier per tile for short launches, one per plane for long ones
  // (planes4); TDBG_STREAM_PB=1|4 forces one (experiments)
  static const int pbe = tdbg_hook("TDBG_STREAM_PB") ? atoi(tdbg_hook("TDBG_STREAM_PB")) : 0;
  const bool pb1 = pbe ? pbe == 1 : kp->ntiles < 48ull * grid;
  auto k = stm == 3 ? unfilter_stream_kernel<true, 3, 4>
           : sgn    ? (pb1 ? unfilter_stream_kernel<true, 1, 1> : unfilter_stream_kernel<true, 1, 4>)
                    : (pb1 ? unfilter_stream_kernel<false, 1, 1> : unfilter_stream_kernel<false, 1, 4>);
  TDBG_LAUNCH(k, dim3(grid), dim3(NT), s, *kp);
  return hipGetLastError();
}
