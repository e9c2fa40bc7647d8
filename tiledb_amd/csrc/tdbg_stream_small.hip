// tdbg_stream_small.hip -- streaming unfilter kernels for the scan pipelines
// of BASELINE C3a / C3b / C4 on 8-byte values (one 64 KiB chunk per tile):
//
//   M_DD    [DOUBLE_DELTA]                      (C3a, uint64 coords)
//   M_RLE   [RLE], cell size 8                  (C3b, uint64 coords)
//   M_PDBWR [POSITIVE_DELTA, BIT_WIDTH_REDUCTION] on 8-byte integers (C4 offsets)
//
// Their filtered images are small (C3a ~6 KB, C3b ~1.3 KB, C4 ~12 KB) and
// their output is 64 KiB, so the tile's time is the decode chain and the
// 64 KiB of stores.  The fused LDS kernel (tdbg_fast.hip) materialises the
// chunk in an 80 KB LDS image (two workgroups per CU) and runs a chain of
// barrier-separated phases per tile; here ownership follows the output, as
// in the C5 streaming kernels (tdbg_stream*.hip):
//
//   * Only the filtered image is staged in LDS, by LDS-DMA issued as soon as
//     the previous tile's last read of it is done; 256-thread workgroups with
//     24-37 KB of LDS, so 4-6 tiles are in flight per CU.
//   * Lane l of wave w owns the 16 values [4096 h + 1024 w + 16 l, +16) of
//     round h = 0, 1 (128 contiguous output bytes); they are computed in
//     registers and leave through a wave-private 4 KiB scratch so that every
//     store instruction writes 8 whole 128-B lines (nontemporal).
//   * DD⁻¹ (dd_compressor.cc:314-404): the lane reads the dwords of its 16
//     codes, realigns them with v_alignbyte / v_alignbit and extracts each
//     code at a compile-time bit position (one instantiation per code width
//     cb = bitsize + 1 in 2..7: an 8,192-value stream of wider codes does not
//     fit the 8 KB staging); the affine double-delta aggregate of its
//     codes goes through a DPP wave scan and one LDS exchange per round.
//   * RLE⁻¹ (rle_compressor.cc:103-141): one workgroup scan of the run
//     lengths gives the run starts; every run writes its index at each
//     16-cell group start it holds (a run-head scatter: 512 writes per tile),
//     so a lane finds the run of its first cell with one LDS read and walks
//     forward.
//   * BWR⁻¹ then PD⁻¹ (bit_width_reduction_filter.cc:352-404,
//     positive_delta_filter.cc:324-375): one pass over the window headers
//     builds both window tables; a lane's 16 values lie in one BWR window
//     and one PD window, so the PD scan is a segmented DPP scan across the
//     lanes of a window -- no cross-wave exchange.
//
// Anything else (other sizes, multi-chunk tiles, raw DoubleDelta, code
// widths > 7 bits, more than 1,024 runs, non-power-of-two windows,
// malformed metadata, offsets tiles) is queued for the fused kernel, which
// runs on the queue right after and sends what it declines to the general
// interpreter, so every status and byte stays the reference's.  Nothing is
// written to a tile's output before all its checks passed.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>
#include <type_traits>

#include "../../include/tiledb_amd.h"
#include "tdbg_desc.h"
#include "tdbg_launch.h"
#include "tdbg_device.h"
#include "tdbg_stream_common.h"
#include "tdbg_hooks.h"

// Built twice (tiledb_amd/build.py): TDBG_SMALL_NT 256 -- the persistent
// kernel, two rounds of 4,096 values per tile, 4-5 workgroups per CU -- and
// 512 -- one workgroup per tile (non-persistent, the launch's workgroups
// dealt XCD-contiguously as in tdbg_c5tile.hip), one round of 8,192 values.
// (TDBG_SMALL_NP=1 with 256 threads: one tile per workgroup, two rounds;
// an A/B build)
#ifndef TDBG_SMALL_NT
#define TDBG_SMALL_NT 256
#endif
#ifndef TDBG_SMALL_NP
#define TDBG_SMALL_NP (TDBG_SMALL_NT == 512)
#endif
#if TDBG_SMALL_NT == 256 && !TDBG_SMALL_NP
#define TDBG_SSM_NS ssm
#define TDBG_SSM_SYM(x) x
#elif TDBG_SMALL_NT == 256
#define TDBG_SSM_NS ssm256np
#define TDBG_SSM_SYM(x) x##_256np
#elif TDBG_SMALL_NT == 512
#define TDBG_SSM_NS ssm512
#define TDBG_SSM_SYM(x) x##_512
#else
#error "TDBG_SMALL_NT: 256 or 512"
#endif

namespace tdbg {
namespace TDBG_SSM_NS {

using namespace sc;

constexpr int NT = TDBG_SMALL_NT;
constexpr int NWV = NT / 64;      // waves per workgroup
constexpr bool NP = TDBG_SMALL_NP;  // one tile per workgroup, XCD-contiguous deal
constexpr uint32_t NR = 8 / NWV;  // rounds of 1,024 NWV values per tile
constexpr uint32_t OUTB = 65536;   // output bytes per tile
constexpr uint32_t NV = OUTB / 8;  // 8-byte values per tile
constexpr uint32_t CPAD = 128;     // reads past the image stay inside C
constexpr uint32_t WSD = 1024;     // scratch dwords per wave (4 KiB)
constexpr uint32_t RUNCAP = 1024;  // RLE runs per tile
constexpr uint32_t RPT = RUNCAP / NT;  // runs per thread
constexpr uint32_t BWN = 256;      // BWR windows per tile (>= 256 B each)
constexpr uint32_t PDN = 256;      // PD windows per tile (>= 256 B each)

enum : int { M_DD = 0, M_RLE = 1, M_PDBWR = 2 };

template <int MODE>
struct Cfg {
  static constexpr uint32_t CAP = MODE == M_PDBWR ? 16384 : 8192;  // staged image bytes
};

template <int MODE>
struct Tab;
template <>
struct Tab<M_DD> {
  uint64_t red[NR][NWV][2];  // per round and wave: DD aggregate (A, B)
};
template <>
struct Tab<M_RLE> {
  uint32_t RS[RUNCAP + 4];  // run starts in cells; RS[r] = total for r >= nr
  uint16_t HD[NV / 16];     // the run holding cell 16 g
  uint32_t wt[NWV];
};
template <>
struct Tab<M_PDBWR> {
  uint4 BT[BWN];  // BWR window: {image offset, kind (0: 8, 1: 16, 2: 32 bit, 3: raw), min lo, min hi}
  uint2 PT[PDN];  // PD window: first value
  uint32_t wt[NWV];
};

template <int MODE>
struct Lds {
  uint32_t C[(Cfg<MODE>::CAP + CPAD) / 4];
  uint32_t WS[NWV][WSD];
  Tab<MODE> T;
  uint32_t vd[NWV];
};

// bytes [o, o + 4) / [o, o + 8) of C (any alignment)
__device__ __forceinline__ uint32_t c32(const uint32_t* C, uint32_t o) {
  const uint32_t* p = C + (o >> 2);
  return __builtin_amdgcn_alignbyte(p[1], p[0], o & 3);
}
__device__ __forceinline__ uint64_t c64(const uint32_t* C, uint32_t o) {
  const uint32_t* p = C + (o >> 2);
  const uint32_t d0 = p[0], d1 = p[1], d2 = p[2];
  return ((uint64_t)__builtin_amdgcn_alignbyte(d2, d1, o & 3) << 32) | __builtin_amdgcn_alignbyte(d1, d0, o & 3);
}
__device__ __forceinline__ uint32_t c8(const uint32_t* C, uint32_t o) { return (C[o >> 2] >> (8 * (o & 3))) & 0xffu; }

// the image [in, in + fs) fits the staging window (16-B units)
template <int MODE>
__device__ __forceinline__ bool fits(const Desc& d) {
  if (d.fs < 20 || d.fs > Cfg<MODE>::CAP) return false;
  const uint64_t a0 = (uint64_t)d.in & ~15ull, a1 = ((uint64_t)d.in + d.fs + 15) & ~15ull;
  return a1 - a0 <= Cfg<MODE>::CAP;
}

// LDS-DMA of the image's 16-B units into C: wave w's instruction r moves
// units [64 (4r + w), +64), lane-linear in LDS
template <int MODE>
__device__ __forceinline__ void dma(Lds<MODE>& L, const Desc& d) {
  const uint64_t a0 = (uint64_t)d.in & ~15ull, a1 = ((uint64_t)d.in + d.fs + 15) & ~15ull;
  const uint32_t n16 = (uint32_t)((a1 - a0) >> 4);
  const uint32_t w = wave_(), l = lane_();
  for (uint32_t r = 0; r * NT < n16; r++) {
    const uint32_t ub = r * NT + 64 * w;  // wave-uniform first unit
    if (ub + l < n16) dma16(a0 + 16ull * (ub + l), lds_addr(L.C) + 16 * ub);
  }
}

// The lane's 16 values (128 B) to out + 128 * lane, through the wave's
// scratch: lanes [32 hh, 32 hh + 32) put their 8 units in row l & 31 (slot j
// at j ^ (row & 7): conflict-free), then every store instruction writes 8
// whole 128-B lines.  8 store instructions per call, every lane active.
// Values vw + i (vw: the wave's first value of the round) at or past nv (a
// chunk of nv < 8,192 values) are not stored: a 16-B unit holds two.
template <bool FULL>
__device__ __forceinline__ void stage_store_(uint32_t* wsp, const uint64_t (&v)[16], uint8_t* o, uint32_t l,
                                             uint32_t vw, uint32_t nv) {
#pragma unroll
  for (int hh = 0; hh < 2; hh++) {
    __builtin_amdgcn_wave_barrier();
    if ((l >> 5) == (uint32_t)hh) {
      const uint32_t row = l & 31;
#pragma unroll
      for (int j = 0; j < 8; j++)
        *(v4u*)(wsp + 4 * (8 * row + (j ^ (row & 7)))) =
            v4u{(uint32_t)v[2 * j], (uint32_t)(v[2 * j] >> 32), (uint32_t)v[2 * j + 1], (uint32_t)(v[2 * j + 1] >> 32)};
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const uint32_t row = 8 * q + (l >> 3), sl = l & 7;
      const v4u y = *(const v4u*)(wsp + 4 * (8 * row + (sl ^ (row & 7))));
      uint8_t* const dst = o + 128u * (32u * hh + row) + 16u * sl;
      if (FULL) {  // (a whole 64 KiB chunk)
        __builtin_nontemporal_store(y, (g_u4*)dst);
      } else {
        const uint32_t vi = vw + 16u * (32u * hh + row) + 2u * sl;  // the unit's first value
        if (vi + 2 <= nv) __builtin_nontemporal_store(y, (g_u4*)dst);
        else if (vi < nv) *(uint2*)dst = make_uint2(y.x, y.y);
      }
    }
  }
}

__device__ __forceinline__ void stage_store(uint32_t* wsp, const uint64_t (&v)[16], uint8_t* o, uint32_t l,
                                            uint32_t vw, uint32_t nv) {
  if (nv == NV) stage_store_<true>(wsp, v, o, l, vw, nv);  // (uniform)
  else stage_store_<false>(wsp, v, o, l, vw, nv);
}

// ---------------------------------------------------------------------------
// DD⁻¹ codes of one lane (code width CB = bitsize + 1 <= 32; instantiated for <= 7)
// ---------------------------------------------------------------------------
// G: dwords of C from byte S + 8 (Ms >> 1) on, read at dword granularity
// (s3 = S & 3: the stream's u64 words start at LDS byte S); Ms = the first
// MSB-first stream dword needed, p = Ms & 1, n = the alignbit amount.
// (dd_compressor.cc:356-404: a sign bit then bitsize magnitude bits, MSB
// first from bit 63 of each little-endian u64 word.)
// dwords of the lane's codes: NA aligned (16 CB bits + up to 31 of
// alignment), NM MSB-first, NH realigned, NG read
template <int CB>
struct Nd {
  static constexpr int NA = (16 * CB + 31) / 32, NM = NA + 1, NH = NM + 2 - (NM & 1), NG = NH + 1;
};

template <int CB>
__device__ __forceinline__ void dd_codes(const uint32_t (&G)[Nd<CB>::NG], uint32_t s3, uint32_t p, uint32_t n,
                                         int32_t (&dd)[16]) {
  constexpr int NA = Nd<CB>::NA, NM = Nd<CB>::NM, NH = Nd<CB>::NH;
  uint32_t H[NH];
#pragma unroll
  for (int x = 0; x < NH; x++) H[x] = __builtin_amdgcn_alignbyte(G[x + 1], G[x], s3);
  // M_j = p ? H[(j+1)^1] : H[j^1] as a bit select (a ternary would turn the
  // pair into an indexed scratch load)
  const uint32_t pm = 0u - p;
  uint32_t M[NM];
#pragma unroll
  for (int j = 0; j < NM; j++) M[j] = (pm & H[(j + 1) ^ 1]) | (~pm & H[j ^ 1]);
  uint32_t A[NA];
#pragma unroll
  for (int j = 0; j < NA; j++) A[j] = __builtin_amdgcn_alignbit(M[j], M[j + 1], n);
  constexpr int B = CB - 1;
#pragma unroll
  for (int i = 0; i < 16; i++) {
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
    dd[i] = (int32_t)((mag ^ (uint32_t)sg) - (uint32_t)sg);
  }
}

// DD aggregate combine: the block with aggregate (Ap, Bp) precedes `self`
// (nself codes): B = Bp + nself * Ap + B, A = Ap + A (modulo 2^64)
template <int CTRL, int ROWS>
__device__ __forceinline__ void scan_step(uint64_t& A, uint64_t& B, uint32_t nself) {
  const uint64_t Ap = dpp0<CTRL, ROWS>(A), Bp = dpp0<CTRL, ROWS>(B);
  B = B + Bp + (uint64_t)nself * Ap;
  A = A + Ap;
}

// ---------------------------------------------------------------------------
// per-tile parse results
// ---------------------------------------------------------------------------
struct Hdr {
  uint32_t dst;    // image (C) byte offset of the chunk's data section
  uint32_t nr;     // RLE: runs
  uint32_t s;      // DD: C byte offset of the stream's first u64 word
  uint32_t cb;     // DD: code width
  uint64_t x0, x1; // DD: the first two values
  uint32_t bsh;    // PDBWR: log2(BWR window elements)
  uint32_t psh;    // PDBWR: log2(PD window elements)
};

// ---------------------------------------------------------------------------
// rounds: the lane's 16 values of round h into v[]
// ---------------------------------------------------------------------------
// DD: codes, local affine fold, DPP wave scan; the wave total goes to red;
// returns the lane's values without the (round, wave) block's start state
// (added after the exchange)
template <int CB>
__device__ __forceinline__ void dd_round_codes(const Lds<M_DD>& L, const Hdr& hd, uint32_t h, uint32_t w, uint32_t l,
                                               uint64_t (&v)[16], uint64_t& A, uint64_t& B) {
  constexpr int32_t cb = CB;
  const int32_t v0 = (int32_t)(4096 * h + 1024 * w + 16 * l);
  const int32_t P0 = (v0 - 2) * cb;       // stream bit of the lane's first code
  const int32_t b0 = (P0 + 31) >> 5;      // (arithmetic: floor for P0 < 0)
  const uint32_t n = (uint32_t)(32 * b0 - P0);
  const int32_t Ms = b0 - 1;
  const uint32_t p = (uint32_t)Ms & 1u;
  const uint32_t gb = hd.s + (uint32_t)(8 * (Ms >> 1));  // >= s - 16 > 0
  uint32_t G[Nd<CB>::NG];
  const uint32_t* gp = L.C + (gb >> 2);
#pragma unroll
  for (int x = 0; x < Nd<CB>::NG; x++) G[x] = gp[x];
  int32_t dd[16];
  dd_codes<CB>(G, hd.s & 3, p, n, dd);
  const bool first = v0 == 0;  // values 0 and 1 enter as pseudo codes x0, x1 - 2 x0
  uint64_t drun = 0, xrun = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) {
    uint64_t e = (uint64_t)(int64_t)dd[i];
    if (i == 0) e = first ? hd.x0 : e;
    if (i == 1) e = first ? hd.x1 - 2 * hd.x0 : e;
    drun += e;
    xrun += drun;
    v[i] = xrun;
  }
  A = drun;
  B = xrun;
}

template <bool SGN>
__device__ __forceinline__ uint64_t bwr_ext(uint64_t x, uint32_t kind) {
  // kind 0/1/2: 8/16/32-bit compressed values (sign- or zero-extended)
  if (kind == 0) return SGN ? (uint64_t)(int64_t)(int8_t)x : (x & 0xffull);
  if (kind == 1) return SGN ? (uint64_t)(int64_t)(int16_t)x : (x & 0xffffull);
  if (kind == 2) return SGN ? (uint64_t)(int64_t)(int32_t)x : (x & 0xffffffffull);
  return x;
}

// ---------------------------------------------------------------------------
// the kernel
// ---------------------------------------------------------------------------
// workgroups per CU by LDS (24.5 / 28.6 / 38.6 KB); the register budget
// follows (80 / 96 / 128 VGPRs)
// (512 threads: 41 / 46 / 55 KB; 2 per CU -- 3 would need <= 80 VGPRs, and
// DD / RLE then spill)
template <int MODE>
struct Occ {
  static constexpr int v = NT == 512 ? 2 : (MODE == M_DD ? 5 : MODE == M_RLE ? 5 : 4);
};

// Queue the declined tiles of one batch (bit i of mask: the workgroup's tile
// base + i) for the fused kernel.  Wave 0.
__device__ __forceinline__ void queue_batch(const KParams& kp, uint64_t mask, uint32_t base, uint32_t bid) {
  const uint32_t l = threadIdx.x & 63;
  uint32_t b0 = 0;
  if (l == 0) b0 = atomicAdd(kp.sq, (uint32_t)__builtin_popcountll(mask));
  b0 = __builtin_amdgcn_readfirstlane(b0);
  if ((mask >> l) & 1) {
    const uint32_t k = b0 + (uint32_t)__builtin_popcountll(mask & ((1ull << l) - 1));
    const uint32_t t = (uint32_t)(bid + (uint64_t)(base + l) * gridDim.x);
    if (k < kp.sq_cap) kp.sq[1 + k] = t;
    else if (kp.status) kp.status[kp.chunks ? kp.chunks[t].tile : t] = TDBG_E_INTERNAL;
  }
}

// AND of every wave's verdict (published before the barrier the caller
// issued): barrier reachability never depends on data
template <int MODE>
__device__ __forceinline__ bool all_ok(const Lds<MODE>& L) {
  uint32_t a = 1;
#pragma unroll
  for (int v = 0; v < NWV; v++) a &= L.vd[v];
  return a != 0;
}

template <int MODE, bool SGN>
__global__ void __launch_bounds__(NT, Occ<MODE>::v) unfilter_stream_small_kernel(const KParams kp) {
  __shared__ Lds<MODE> L;
  const uint64_t G = gridDim.x;
  // work items: tiles, or (chunk mode, tdbg_stream_common.h) the records of
  // the device chunk directory
  const uint64_t ntl = work_items(kp);
  const bool chunked = kp.chunks != nullptr;
  // the fused kernel's fallback queue starts empty for this launch (it runs
  // next on the same stream and is the only one to append; chunk mode: the
  // directory's scan kernel cleared it, and fbq is not passed here)
  if (kp.fbq && blockIdx.x == 0 && threadIdx.x == 0) kp.fbq[0] = 0;
  // the workgroup's place in the deal: NP, workgroups are dealt over the 8
  // XCDs round-robin, so XCD x takes the contiguous eighth [x G / 8, +G / 8)
  // of the items (G a multiple of 8; a placement assumption for speed only)
  const uint32_t bid = NP ? (blockIdx.x & 7) * (uint32_t)(G >> 3) + (blockIdx.x >> 3) : blockIdx.x;
  const uint32_t w = wave_();
  uint64_t ok_tiles = 0, ok_bytes = 0;
  Desc cur{};
  bool cur_dma = false;
  bool stored = false;  // the last tile issued its 8 round-1 stores after the DMA
  Batch bt{0, 0, 0, 0};
  if (bid < ntl) {
    bt = batch_load(kp, 0, ntl, bid);
    cur = batch_get(bt, 0, bid);
    cur_dma = fits<MODE>(cur);
    if (cur_dma) dma(L, cur);
  }
  uint64_t dmask = 0;
  uint32_t it = 0;
  for (uint64_t j = bid; j < ntl; j += G, it++) {
    const uint64_t jn = j + G;
    const uint32_t l = lane_();
    // a chunk of nv = os / 8 values, 16 <= nv <= 8,192 (short last chunks,
    // tiles under 64 KiB: tile.cc:87-100)
    bool ok = cur_dma && !(kp.flags & TDBG_TILE_OFFSETS) && cur.os >= 128 && cur.os <= OUTB && (cur.os & 7) == 0 &&
              (((uintptr_t)cur.out) & 15) == 0;
    // (uniform: scalar registers)
    const uint32_t os = __builtin_amdgcn_readfirstlane((uint32_t)(ok ? cur.os : OUTB)), nv = os >> 3;
    Hdr hd{};
    Desc nxt{};
    bool nxt_dma = false;
    bool issued = false;  // the next tile's DMA went out inside the tile
    // the next descriptor (and its batch) before anything is stored, so the
    // counted waits below see only the stores issued after the DMA
    auto next_dma = [&]() {
      if ((it + 1) % 64 == 0 && jn < ntl) bt = batch_load(kp, it + 1, ntl, bid);
      nxt = batch_get(bt, (it + 1) % 64, jn);
      nxt_dma = jn < ntl && fits<MODE>(nxt);
      if (nxt_dma) dma(L, nxt);
      issued = true;
    };
    if (cur_dma) {
      // B1: this tile's image has landed (the last tile's 8 round-1 stores,
      // issued after the DMA, may stay in flight) and every wave is past the
      // last tile's reads of the tables
      if (stored) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      lds_barrier();
      const uint32_t* C = L.C;
      const uint32_t b = (uint32_t)((uintptr_t)cur.in & 15);
      // ---- tile + chunk header (Tile::load_chunk_data, tile.cc:280-313) ----
      // (chunk mode: the image starts at the chunk header, no u64 chunk count)
      const uint32_t ho = chunked ? 0u : 8u;
      const uint32_t nlo = c32(C, b), nhi = c32(C, b + 4), orig = c32(C, b + ho), fl = c32(C, b + ho + 4),
                     ml = c32(C, b + ho + 8);
      const uint32_t m = b + ho + 12;
      ok = ok && (chunked || (nlo == 1 && nhi == 0)) && orig == os && (uint64_t)ml + fl + ho + 12 <= cur.fs;
      hd.dst = m + ml;
      if constexpr (MODE == M_DD || MODE == M_RLE) {
        // compression frame (compression_filter.cc:413-486): 0 md parts, one
        // data part of os bytes compressed to fl
        const uint32_t nmd = c32(C, m), ndp = c32(C, m + 4), po = c32(C, m + 8), pc = c32(C, m + 12);
        ok = ok && ml == 16 && nmd == 0 && ndp == 1 && po == os && pc == fl;
        if constexpr (MODE == M_DD) {
          // [u8 bitsize][u64 n][u64 x0][u64 x1][u64 words] (dd_compressor.cc:314-345)
          const uint32_t s0 = hd.dst;
          const uint32_t bs = c8(C, s0), n0 = c32(C, s0 + 1), n1 = c32(C, s0 + 5);
          hd.x0 = c64(C, s0 + 9);
          hd.x1 = c64(C, s0 + 17);
          hd.s = s0 + 25;
          hd.cb = bs + 1;
          const uint32_t words = ((nv - 2) * hd.cb + 63) / 64;
          // (bitsize <= 6: an 8,192-value stream of wider codes is bigger than CAP)
          ok = ok && bs >= 1 && bs <= 6 && n0 == nv && n1 == 0 && fl == 25 + 8 * words;
        } else {
          // runs of [u64 value][u8 len_hi][u8 len_lo] (rle_compressor.cc:103-141)
          hd.nr = fl / 10;
          ok = ok && fl % 10 == 0 && hd.nr >= 1 && hd.nr <= RUNCAP;
        }
      } else {
        // BWR md [u32 orig][u32 nwin] + nwin x [u64 min][u8 bits][u32 nbytes]
        // (bit_width_reduction_filter.cc:353-380), then PD md [u32 nwin] +
        // nwin x [u64 first][u32 nbytes] (positive_delta_filter.cc:324-340)
        const uint32_t bo = c32(C, m), nw = c32(C, m + 4), ws = c32(C, m + 8 + 9);
        const uint32_t m2 = m + 8 + 13 * (nw < BWN ? nw : BWN);
        const uint32_t npw = c32(C, m2), wp = c32(C, m2 + 4 + 8);
        // (windows of ws / wp bytes, the last one holding the rest)
        ok = ok && bo == os && nw >= 1 && nw <= BWN && ws >= 256 && (ws & (ws - 1)) == 0 && nw == (os + ws - 1) / ws &&
             npw >= 1 && npw <= PDN && wp >= 256 && wp <= 8192 && (wp & (wp - 1)) == 0 && npw == (os + wp - 1) / wp &&
             ml == 8 + 13 * nw + 4 + 12 * npw;
        hd.bsh = ok ? 31 - __builtin_clz(ws) - 3 : 5;
        hd.psh = ok ? 31 - __builtin_clz(wp) - 3 : 7;
        hd.nr = nw;    // (reused: window counts)
        hd.cb = npw;
        hd.s = m2;
      }
      // ---- tables (one workgroup pass; barriers reached whatever the bytes) ----
      if constexpr (MODE == M_RLE) {
        // run starts: thread t owns runs 4t..4t+3 (length 0 past nr), an
        // exclusive workgroup scan of the lengths
        uint32_t len[RPT], s4 = 0;
#pragma unroll
        for (int i = 0; i < (int)RPT; i++) {
          const uint32_t r = RPT * threadIdx.x + i;
          uint32_t x = 0;
          if (ok && r < hd.nr) x = c32(C, hd.dst + 10 * r + 8);
          len[i] = ((x & 0xffu) << 8) | ((x >> 8) & 0xffu);
          s4 += len[i];
        }
        const uint32_t inc = wave_incscan_u32(s4);
        if (l == 63) L.T.wt[w] = inc;
        lds_barrier();
        uint32_t pre = 0, tot = 0;
#pragma unroll
        for (int v2 = 0; v2 < NWV; v2++) {
          const uint32_t x = L.T.wt[v2];
          pre += (uint32_t)v2 < w ? x : 0u;
          tot += x;
        }
        ok = ok && tot == nv;
        uint32_t a = pre + inc - s4;
#pragma unroll
        for (int i = 0; i < (int)RPT; i++) {
          L.T.RS[RPT * threadIdx.x + i] = a;
          // run-head scatter: the run holding cell 16 g, for every 16-cell
          // group start inside this run (each written once: the runs tile
          // [0, 8192) when tot == NV; empty runs hold none)
          if (ok)
            for (uint32_t g = (a + 15) >> 4; 16 * g < a + len[i]; g++) L.T.HD[g] = (uint16_t)(RPT * threadIdx.x + i);
          a += len[i];
        }
        if (threadIdx.x == NT - 1) L.T.RS[RUNCAP] = a;
      } else if constexpr (MODE == M_PDBWR) {
        const uint32_t t = threadIdx.x, nw = hd.nr, npw = hd.cb;
        const uint32_t wsz = 8u << hd.bsh, psz = 8u << hd.psh;
        uint32_t cs = 0, kind = 3;
        uint64_t mn = 0;
        bool bad = false;
        if (ok && t < nw) {
          const uint32_t e = m + 8 + 13 * t;
          mn = c64(C, e);
          const uint32_t bits = c8(C, e + 8), nb = c32(C, e + 9);
          const bool raw = bits >= 64 || (nb & 7) != 0;
          bad = nb != (t + 1 < nw ? wsz : os - wsz * (nw - 1)) || (!raw && bits != 8 && bits != 16 && bits != 32);
          kind = raw ? 3u : bits == 8 ? 0u : bits == 16 ? 1u : 2u;
          cs = raw ? nb : (nb >> 3) << kind;
        }
        if (ok && t < npw) {
          const uint32_t e = hd.s + 4 + 12 * t;
          const uint64_t first = c64(C, e);
          bad = bad || c32(C, e + 8) != (t + 1 < npw ? psz : os - psz * (npw - 1));
          L.T.PT[t] = make_uint2((uint32_t)first, (uint32_t)(first >> 32));
        }
        const uint32_t inc = wave_incscan_u32(cs);
        if (l == 63) L.T.wt[w] = inc;
        ok = ok && !__builtin_amdgcn_ballot_w64(bad);
        lds_barrier();
        uint32_t pre = 0, tot = 0;
#pragma unroll
        for (int v2 = 0; v2 < NWV; v2++) {
          const uint32_t x = L.T.wt[v2];
          pre += (uint32_t)v2 < w ? x : 0u;
          tot += x;
        }
        // (every wave's verdict is ANDed at B2 below; a table entry written
        // under a failed verdict is never read)
        ok = ok && tot <= fl;
        if (t < BWN) L.T.BT[t] = make_uint4(hd.dst + pre + inc - cs, kind, (uint32_t)mn, (uint32_t)(mn >> 32));
      }
      // verdicts published, tables visible (B2)
      if (l == 0) L.vd[w] = ok ? 1u : 0u;
      lds_barrier();
      ok = ok && all_ok(L);
      // ---- two rounds of 4,096 values ----
      auto round = [&](auto HC) {
        constexpr uint32_t h = decltype(HC)::value;
        uint64_t v[16];
        uint8_t* obase = cur.out + 32768u * h + 8192u * w;
        if constexpr (MODE == M_DD) {
          uint64_t A = 0, B = 0;
          if (ok) {
            switch (hd.cb) {
#define TDBG_CB(c) \
  case c: dd_round_codes<c>(L, hd, h, w, l, v, A, B); break;
              TDBG_CB(2) TDBG_CB(3) TDBG_CB(4) TDBG_CB(5) TDBG_CB(6) TDBG_CB(7)
#undef TDBG_CB
              default: break;
            }
            // inclusive wave scan of the (A, B) aggregates, 16 codes per lane
            const uint64_t As = A, Bs = B;
            scan_step<DPP_ROW_SHR1, 0xf>(A, B, 16);
            scan_step<DPP_ROW_SHR2, 0xf>(A, B, 32);
            scan_step<DPP_ROW_SHR4, 0xf>(A, B, 64);
            scan_step<DPP_ROW_SHR8, 0xf>(A, B, 128);
            scan_step<DPP_ROW_BCAST15, 0xa>(A, B, 16 * ((l & 15) + 1));
            scan_step<DPP_ROW_BCAST31, 0xc>(A, B, 16 * ((l & 31) + 1));
            // fold the lane's exclusive wave prefix into its values
            const uint64_t ae = A - As, be = B - Bs - 16 * ae;
            uint64_t t = be;
#pragma unroll
            for (int i = 0; i < 16; i++) {
              t += ae;
              v[i] += t;
            }
            if (l == 63) {
              L.T.red[h][w][0] = A;
              L.T.red[h][w][1] = B;
            }
          }
          lds_barrier();  // the round's (wave) totals; in round 1 also: C is free
          if (h == NR - 1) next_dma();
          if (ok) {
            // start state of the (round, wave) block: 1,024 codes per block
            uint64_t X = 0, D = 0;
#pragma unroll
            for (uint32_t hb = 0; hb <= h; hb++)
#pragma unroll
              for (int vb = 0; vb < NWV; vb++) {
                if (hb == h && (uint32_t)vb >= w) continue;
                const uint64_t Ab = L.T.red[hb][vb][0], Bb = L.T.red[hb][vb][1];
                X = X + 1024ull * D + Bb;
                D = D + Ab;
              }
            X = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(X >> 32)) << 32) |
                (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)X);
            D = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(D >> 32)) << 32) |
                (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)D);
            uint64_t t = X + (uint64_t)(16 * l) * D;
#pragma unroll
            for (int i = 0; i < 16; i++) {
              t += D;
              v[i] += t;
            }
            stage_store(L.WS[w], v, obase, l, 4096 * h + 1024 * w, nv);
          }
        } else if constexpr (MODE == M_RLE) {
          const uint32_t c0 = 4096 * h + 1024 * w + 16 * l;
          if (ok && c0 < nv) {
            // the run holding c0 (a multiple of 16): one read of the
            // run-head scatter instead of a dependent binary search
            uint32_t r = L.T.HD[c0 >> 4];
            uint32_t rend = L.T.RS[r + 1];
            uint64_t x = c64(L.C, hd.dst + 10 * r);
            if (c0 + 16 <= nv) {
#pragma unroll
              for (int k = 0; k < 16; k++) {
                if (c0 + k >= rend) {
                  do {
                    r++;
                    rend = L.T.RS[r + 1];
                  } while (c0 + k >= rend);
                  x = c64(L.C, hd.dst + 10 * r);
                }
                v[k] = x;
              }
            } else {
              // (the one lane holding the chunk's end when nv is not a
              // multiple of 16: no run holds the cells past it)
#pragma unroll
              for (int k = 0; k < 16; k++) {
                if (c0 + k < nv && c0 + k >= rend) {
                  do {
                    r++;
                    rend = L.T.RS[r + 1];
                  } while (c0 + k >= rend);
                  x = c64(L.C, hd.dst + 10 * r);
                }
                v[k] = x;
              }
            }
          }
          if (h == NR - 1) {
            lds_barrier();  // every wave is done with C
            next_dma();
          }
          if (ok) stage_store(L.WS[w], v, obase, l, 4096 * h + 1024 * w, nv);
        } else {  // M_PDBWR
          if (ok) {
            const uint32_t e0 = 4096 * h + 1024 * w + 16 * l;
            // (lanes past a short chunk decode values no store takes, from
            // the last windows)
            const uint32_t wi = min(e0 >> hd.bsh, hd.nr - 1);
            const uint4 te = L.T.BT[wi];
            const uint64_t mn = ((uint64_t)te.w << 32) | te.z;
            const uint32_t kind = te.y, j0 = min(e0 - (wi << hd.bsh), (1u << hd.bsh) - 16);
            const uint32_t a = te.x + (j0 << (kind == 3 ? 3 : kind));
            // the lane's 16 deltas (BWR⁻¹: value + window minimum, wrapping)
            uint64_t d[16];
            if (__builtin_amdgcn_ballot_w64(kind != 0) == 0) {
              // every lane's window is 8-bit: 16 bytes
              const uint32_t* p = L.C + (a >> 2);
              uint32_t R[5];
#pragma unroll
              for (int k = 0; k < 5; k++) R[k] = p[k];
              uint32_t q[4];
#pragma unroll
              for (int k = 0; k < 4; k++) q[k] = __builtin_amdgcn_alignbyte(R[k + 1], R[k], a & 3);
#pragma unroll
              for (int k = 0; k < 16; k++) {
                const uint32_t by = (q[k >> 2] >> (8 * (k & 3))) & 0xffu;
                d[k] = (SGN ? (uint64_t)(int64_t)(int8_t)by : (uint64_t)by) + mn;
              }
            } else {
              const uint32_t sh = kind == 3 ? 3 : kind;
#pragma unroll
              for (int k = 0; k < 16; k++) {
                const uint64_t x = c64(L.C, a + ((uint32_t)k << sh));
                d[k] = kind == 3 ? x : bwr_ext<SGN>(x, kind) + mn;
              }
            }
            // PD⁻¹: inclusive prefix in the lane, then a segmented scan of the
            // lane sums over the 2^(psh - 4) lanes of the PD window
#pragma unroll
            for (int k = 1; k < 16; k++) d[k] += d[k - 1];
            const uint64_t s = d[15];
            const uint32_t gl = 1u << (hd.psh - 4), lg = l & (gl - 1);
            uint64_t inc = s;
            {
              // in-row steps (a source in another row reads 0), then the
              // row carries for windows of 32 / 64 lanes
              uint64_t y = dpp0<DPP_ROW_SHR1, 0xf>(inc);
              if (gl > 1 && lg >= 1) inc += y;
              y = dpp0<DPP_ROW_SHR2, 0xf>(inc);
              if (gl > 2 && lg >= 2) inc += y;
              y = dpp0<DPP_ROW_SHR4, 0xf>(inc);
              if (gl > 4 && lg >= 4) inc += y;
              y = dpp0<DPP_ROW_SHR8, 0xf>(inc);
              if (gl > 8 && lg >= 8) inc += y;
              if (gl > 16) inc += dpp0<DPP_ROW_BCAST15, 0xa>(inc);
              if (gl > 32) inc += dpp0<DPP_ROW_BCAST31, 0xc>(inc);
            }
            const uint2 f = L.T.PT[min(e0 >> hd.psh, hd.cb - 1)];
            const uint64_t base = (((uint64_t)f.y << 32) | f.x) + (inc - s);
#pragma unroll
            for (int k = 0; k < 16; k++) v[k] = base + d[k];
          }
          if (h == NR - 1) {
            lds_barrier();  // every wave is done with C
            next_dma();
          }
          if (ok) stage_store(L.WS[w], v, obase, l, 4096 * h + 1024 * w, nv);
        }
      };
      round(std::integral_constant<uint32_t, 0>{});
      if constexpr (NR == 2) round(std::integral_constant<uint32_t, 1>{});
    }  // cur_dma
    // a tile this kernel does not take goes to the fused kernel
    if (!ok) dmask |= 1ull << (it % 64);
    if ((it + 1) % 64 == 0 || jn >= ntl) {
      if (dmask && w == 0) queue_batch(kp, dmask, it - it % 64, bid);
      dmask = 0;
    }
    if (!issued) next_dma();
    if (ok) {
      ok_tiles++;
      ok_bytes += os;
      if (threadIdx.x == 0 && kp.status && !chunked) kp.status[cur.t] = TDBG_OK;
    }
    cur = nxt;
    cur_dma = nxt_dma;
    stored = ok;
  }
  // (one slot of counters per 64 workgroups, summed by the host: a
  // 100,000-workgroup launch on one address would serialise its atomics)
  uint64_t* const sl = kp.stats ? kp.stats + TDBG_STAT_STRIDE * (1 + (blockIdx.x & 63)) : nullptr;
  if (sl && threadIdx.x == 0 && ok_tiles && chunked) {
    atomicAdd((unsigned long long*)&sl[TDBG_STAT_STREAM_CHUNKS], (unsigned long long)ok_tiles);
  } else if (sl && threadIdx.x == 0 && ok_tiles) {
    atomicAdd((unsigned long long*)&sl[TDBG_STAT_FUSED_TILES], (unsigned long long)ok_tiles);
    atomicAdd((unsigned long long*)&sl[TDBG_STAT_FUSED_BYTES], (unsigned long long)ok_bytes);
    atomicAdd((unsigned long long*)&sl[TDBG_STAT_STREAM_TILES], (unsigned long long)ok_tiles);
  }
}

}  // namespace TDBG_SSM_NS
}  // namespace tdbg

// mode: 0 DD (8-byte), 1 RLE (cell size 8), 2 PD + BWR (8-byte); sgn: the
// BWR stage's integer type is signed
extern "C" uint32_t TDBG_SSM_SYM(tdbg_stream_small_grid)(int cus, int mode) {
  using namespace tdbg::TDBG_SSM_NS;
  static const int g = tdbg_hook("TDBG_SMALL_GRID") ? atoi(tdbg_hook("TDBG_SMALL_GRID")) : 0;  // experiments
  const int occ = mode == M_DD ? Occ<M_DD>::v : mode == M_RLE ? Occ<M_RLE>::v : Occ<M_PDBWR>::v;
  return g > 0 ? (uint32_t)g : (uint32_t)(cus * occ);
}

// (512: grid = the items rounded up to 8, at most 2^22 -- workgroups then loop)
extern "C" hipError_t TDBG_SSM_SYM(tdbg_launch_stream_small)(const tdbg::KParams* kp, uint32_t grid, int mode,
                                                             int sgn, hipStream_t s) {
  using namespace tdbg::TDBG_SSM_NS;
  if (NP) grid = 8 * ((std::min<uint64_t>(std::max<uint64_t>(kp->ntiles, 1), 1ull << 22) + 7) / 8);
  if (mode == M_DD) {
    TDBG_LAUNCH((unfilter_stream_small_kernel<M_DD, false>), dim3(grid), dim3(NT), s, *kp);
  } else if (mode == M_RLE) {
    TDBG_LAUNCH((unfilter_stream_small_kernel<M_RLE, false>), dim3(grid), dim3(NT), s, *kp);
  } else if (sgn) {
    TDBG_LAUNCH((unfilter_stream_small_kernel<M_PDBWR, true>), dim3(grid), dim3(NT), s, *kp);
  } else {
    TDBG_LAUNCH((unfilter_stream_small_kernel<M_PDBWR, false>), dim3(grid), dim3(NT), s, *kp);
  }
  return hipGetLastError();
}
