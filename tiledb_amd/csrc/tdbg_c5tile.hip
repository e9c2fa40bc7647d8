// tdbg_c5tile.hip -- one-workgroup-per-tile unfilter kernel for the headline
// pipeline [BYTESHUFFLE, DOUBLE_DELTA, BIT_WIDTH_REDUCTION] on 4-byte
// integers, one 64 KiB chunk, DoubleDelta stored raw (dd_compressor.cc:
// 233-236 on write, :327-331 on read): SURVEY 8(d)'s C5 "rand" and "ramp"
// tiles, whose filtered images (40-68 KB) are above the coded kernel's
// staging cap (tdbg_stream.hip).
//
// Shape (round 5, tools/ceiling3.hip, profiles/r05/): on MI355X a tile moved
// by ONE non-persistent 1024-thread workgroup, with the launch's workgroups
// dealt so that each XCD owns one contiguous eighth of the tiles, streams at
// 0.77 of 8 TB/s on C5-rand-shaped tiles (68 KB in, 64 KiB out), where every
// persistent grid of the same tiles stays at 0.64-0.68 (a wave's loads of
// tile n + 1 wait behind its stores of tile n: gfx950 has one in-order vmcnt
// for both).  So:
//
//   * grid = the launch's work items (rounded up to 8); workgroup b takes
//     item (b & 7) * ceil(n / 8) + (b >> 3) (workgroups are dealt over the 8
//     XCDs round-robin: this keeps each XCD on a contiguous range; a
//     placement assumption for speed only, every item is taken exactly once
//     whatever the placement).  Bigger launches than the grid cap loop.
//   * The whole filtered image (<= 68,080 B at any alignment) lands in LDS
//     by LDS-DMA (1 KiB per wave instruction, five per wave); one wave
//     parses the tile + chunk header, every BWR window header
//     (bit_width_reduction_filter.cc:353-380: the window table is a DPP scan
//     of the compressed sizes), the compression frame (compression_filter.cc:
//     413-486) and the two DD headers (dd_compressor.cc:314-331).
//   * Ownership follows the output: thread T makes output units
//     1024 r + T (r = 0..3; 16 B each, lane-consecutive, so every store
//     instruction writes 1 KiB of whole lines).  Unit j is byteshuffle^-1
//     (byteshuffle_filter.cc:111-166) of dword j of the four byte planes, i.e.
//     of the BWR-output dwords at bytes 26 + 16384 k + 4 j (c0 = 17 B and
//     c1's 9-byte header precede the raw values).  Each wave decodes its
//     256-B plane ranges with one wave-uniform BWR^-1 decoder: all-raw
//     windows (an unaligned dword read), all-8-bit windows (two bytes plus
//     their window minima), or per element (16-bit or mixed windows).
//
// Tiles it does not decode (other sizes, windows not a power of two in
// [256, 4096], a coded DD part, malformed headers, offsets tiles, images
// over the stage) are queued for the fused kernel, which runs on the queue
// in the same launch (and from there the general interpreter), so every
// status and byte stays the reference's.  Nothing is written to a tile's
// output before all its checks passed.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <stdlib.h>

#include <algorithm>

#include "../../include/tiledb_amd.h"
#include "tdbg_desc.h"
#include "tdbg_device.h"
#include "tdbg_launch.h"
#include "tdbg_stream_common.h"
#include "tdbg_hooks.h"

namespace tdbg {
namespace c5t {

using namespace sc;

constexpr int NT = 1024;              // 16 waves
constexpr uint32_t OUTB = 65536;      // output bytes per tile
constexpr uint32_t SMALL = CODED_CAP; // tiles this big or smaller belong to tdbg_stream.hip
constexpr uint32_t IMGU = 4256;       // 16-B units of the image stage (68,096 B)
constexpr uint32_t IMG_CAP = IMGU * 16 - 15;
constexpr uint32_t TABN = 320;        // BWR windows per chunk (nwin <= 257 for windows >= 256 B)
constexpr uint32_t LBWR = 65562;      // BWR output bytes of a raw-DD C5 chunk: 17 + 9 + 65536
constexpr uint32_t GRID_CAP = 1u << 22;
constexpr uint32_t PFX = 192;         // 16-B units of the image prefix the parse reads (3 KiB)

struct Lds {
  uint32_t IMG[IMGU * 4];
  uint2 TAB[TABN];  // {image offset of the window's data | kind << 20, window minimum}
  uint32_t hd[8];   // verdict, log2(window bytes), nwin - 1, code width (0: raw DD), x0, x1, Lb, values
  uint32_t red[16][2];  // coded tiles: each wave's DD aggregate (A, B)
  // multi-chunk tiles (MC): the chunk loop's state, kept here rather than in
  // registers through the loop (its body is the whole decoder).  Per chunk k
  // (buffer k & 1, written by thread 0 during chunk k - 1): the chunk's
  // header byte in the tile, its output byte, its header [orig, filtered,
  // md]; per tile: the chunk count, the tile's input and output pointers
  uint32_t mcs[2][5];
  uint32_t mct[5];
};

// the tile's shape is one this kernel decodes (descriptor checks only)
// (a chunk of 4 n bytes, 16 <= n <= 16384 values; the output 4-B aligned)
__device__ __forceinline__ bool takes(const KParams& kp, const Desc& d) {
  return !(kp.flags & TDBG_TILE_OFFSETS) && d.os >= 64 && d.os <= OUTB && (d.os & 3) == 0 &&
         (((uintptr_t)d.out) & 3) == 0 && d.fs <= IMG_CAP;
}

// a tile of several chunks this kernel may decode in tile mode (its chunks
// are checked one by one as they come)
__device__ __forceinline__ bool mc_tile(const KParams& kp, const Desc& d) {
  return !(kp.flags & TDBG_TILE_OFFSETS) && d.os > OUTB && d.os < (1ull << 32) && d.fs < (1ull << 32) &&
         (d.os & 3) == 0 && (((uintptr_t)d.out) & 3) == 0 && d.fs >= 8 + 2 * 12;
}

__device__ __forceinline__ void decline(const KParams& kp, uint64_t t) {
  if (threadIdx.x == 0) {
    const uint32_t k = atomicAdd(kp.sq, 1u);
    if (k < kp.sq_cap) kp.sq[1 + k] = (uint32_t)t;
    else if (kp.status) kp.status[kp.chunks ? kp.chunks[t].tile : t] = TDBG_E_INTERNAL;
  }
}

// work item t's descriptor (every lane reads the same item)
__device__ __forceinline__ Desc load_desc(const KParams& kp, uint64_t t) {
  Desc d;
  d.t = t;
  if (kp.chunks) {
    const ChunkRec r = kp.chunks[t];
    const uint64_t fs = 12ull + r.ml + r.fl;
    d.fs = fs;
    d.os = r.orig;
    d.in = kp.in[r.tile] + r.in_off - 12;
    d.out = kp.out[r.tile] + r.out_off;
  } else {
    d.fs = kp.in_size[t];
    d.os = kp.out_size[t];
    d.in = kp.in[t];
    d.out = kp.out[t];
  }
  return d;
}

// ---------------------------------------------------------------------------
// header parse (one wave): tile/chunk header, window table, frame, DD headers
// ---------------------------------------------------------------------------
// Two LDS round trips: (1) the tile + chunk header and every window header
// (lane l: windows 5 l .. 5 l + 4, 45 bytes), issued together (the window
// headers' place does not depend on any value read); (2) after the scan of
// the compressed sizes, the compression frame (after the nwin window
// headers) and the DD headers (BWR-output elements 0..8, in window 0).
template <bool SGN>
__device__ __forceinline__ void parse(Lds& L, const Desc& d, uint32_t l, bool chunked) {
  const uint32_t* P = L.IMG;
  // the chunk header follows the tile's u64 chunk count, or (chunk mode: a
  // chunk of a multi-chunk tile) starts the image
  const uint32_t ho = chunked ? 0u : 8u;
  const uint32_t b = (uint32_t)((uintptr_t)d.in & 15);
  const uint32_t m = b + ho + 12;
  const uint32_t e0 = m + 8 + 45 * l;  // m + 8 + 45 * 63 + 52 < 3,000
  // ---- round 1 (the window headers are read inside bwr_window_table; the
  // uniform addresses below are broadcast reads)
  const uint32_t nlo = rd32(P, b), nhi = rd32(P, b + 4), orig = rd32(P, b + ho), fl = rd32(P, b + ho + 4),
                 ml = rd32(P, b + ho + 8);
  const uint32_t Lb = rd32(P, m), nwr = rd32(P, m + 4), ws = rd32(P, m + 13);  // ws: window 0's byte count
  const uint32_t os = (uint32_t)d.os, nv = os >> 2;
  bool ok = (chunked || (nlo == 1 && nhi == 0)) && orig == os && (uint64_t)ml + fl + ho + 12 <= d.fs && nwr >= 1 &&
            nwr <= TABN && ml == 8 + 9 * nwr + 24 && Lb <= LBWR && Lb >= 34 + 8 && ws >= 256 && ws <= 4096 &&
            (ws & (ws - 1)) == 0 && (Lb - 1) / ws + 1 == nwr;
  const uint32_t nwin = ok ? nwr : 2;
  const uint32_t dst = ho + 12 + ml;  // image offset of the BWR data
  const WinTab wt = bwr_window_table(P, L.TAB, e0, nwin, ws, Lb, fl, dst, l);
  ok = ok && wt.ok;
  // ---- round 2: the compression frame md (compression_filter.cc:413-486):
  // 1 md part of 8 B (the byteshuffle header) compressed to 17 B, 1 data part
  // of os bytes compressed to d5 bytes (the BWR output is c0 + c1); the DD
  // headers = BWR-output bytes [0, 34): lane e decodes element e < 9 of
  // window 0
  const uint32_t k0 = wt.k0, mn0 = wt.mn0;
  const uint32_t f = m + 8 + 9 * nwin;
  const uint32_t lf = l < 6 ? l : 5;
  const uint32_t fv = rd32(P, f + 4 * lf);  // lane i < 6: frame dword i
  const uint32_t e = l < 9 ? l : 8;
  uint32_t v = rd32(P, b + dst + (e << k0));
  v = k0 == 2 ? v : (k0 == 0 ? ext<SGN>(v, 0, 8) : ext<SGN>(v, 0, 16)) + mn0;
  auto fr = [&](int k) -> uint32_t { return __builtin_amdgcn_readlane(fv, k); };
  const uint32_t d5 = fr(5);
  ok = ok && fr(0) == 1 && fr(1) == 1 && fr(2) == 8 && fr(3) == 17 && fr(4) == os && d5 + 17 == Lb;
  auto dw = [&](int k) -> uint32_t { return __builtin_amdgcn_readlane(v, k); };
  auto dd = [&](int o) -> uint32_t { return __builtin_amdgcn_alignbyte(dw((o >> 2) + 1), dw(o >> 2), o & 3); };
  // c0 = [u8 bitsize][u64 n = 2][1][os] (any bitsize: two values, or the
  // same 8 bytes copied raw); c1 = [u8 bitsize][u64 nv = os / 4] followed by
  // the raw values (bitsize >= 31, dd_compressor.cc:233-236) or by [x0][x1]
  // and nv - 2 codes of bitsize + 1 bits in u64 words, MSB first (bitsize
  // 1..30, dd_compressor.cc:314-404)
  const uint32_t bs = dd(17) & 0xffu;
  const uint32_t cb = bs + 1, words = ((nv - 2) * cb + 63) / 64;
  const bool raw = bs >= 31;
  ok = ok && dd(1) == 2 && dd(5) == 0 && dd(9) == 1 && dd(13) == os && dd(18) == nv && dd(22) == 0 &&
       (raw ? d5 == 9 + os : bs >= 1 && d5 == 17 + 8 * words);
  if (l == 0) {
    L.hd[0] = ok ? 1u : 0u;
    L.hd[1] = 31 - __builtin_clz(ws);
    L.hd[2] = nwin - 1;
    L.hd[3] = raw ? 0u : cb;
    L.hd[4] = dd(26);
    L.hd[5] = dd(30);
    L.hd[6] = Lb;
    L.hd[7] = nv;
  }
}

// Byteshuffle^-1 of one output unit from dword j of the four planes: out
// dword b, byte k = plane k's byte b
__device__ __forceinline__ v4u unshuffle4(const uint32_t (&x)[4]) {
  const uint32_t t0 = __builtin_amdgcn_perm(x[1], x[0], 0x05010400u);
  const uint32_t t1 = __builtin_amdgcn_perm(x[1], x[0], 0x07030602u);
  const uint32_t t2 = __builtin_amdgcn_perm(x[3], x[2], 0x05010400u);
  const uint32_t t3 = __builtin_amdgcn_perm(x[3], x[2], 0x07030602u);
  return v4u{__builtin_amdgcn_perm(t2, t0, 0x05040100u), __builtin_amdgcn_perm(t2, t0, 0x07060302u),
             __builtin_amdgcn_perm(t3, t1, 0x05040100u), __builtin_amdgcn_perm(t3, t1, 0x07060302u)};
}

// The wave's plane ranges: (r, k) = round r (output units 1024 r + 64 w +
// [0, 64)), plane k = the 256 BWR-output bytes [Q0, Q0 + 256), Q0 = 26 +
// nv k + 4 (1024 r + 64 w) for a chunk of nv values (byte shift s = Q0 & 3,
// the same for a plane's every range: 2 when nv is a multiple of 4).  A range spans at most two windows (windows
// are >= 256 B), W0 and W1; lane i < 16 reads range i = 4 r + k's two table
// entries once, and the decode takes them back with v_readlane (no per-lane
// table lookups).  One wave-uniform BWR^-1 decoder per range:
//   raw     both windows raw: the compressed dword at W0's data offset +
//           (Q - W0's start) (consecutive full raw windows are contiguous);
//   8-bit   both 8-bit: the two element bytes at W0's offset + element index
//           (full 8-bit windows are contiguous too), each plus its window's
//           minimum;
//   general (16-bit or mixed windows) the dword = bytes [s, 4) of element
//           e = Q / 4 and bytes [0, s) of e + 1, each decoded from its own
//           window's entry.
struct Ranges {
  uint32_t x0, x1;  // table words of W0 and W1 ({data offset | kind << 20})
  uint32_t m0, m1;  // their minima
  uint32_t e0, e1;  // their first element indices (e1 = W1's, or ~0 when W1 == W0)
  uint32_t s1;      // the decoded value of element e1 (W1's first element)
  uint32_t base;    // raw / 8-bit ranges: LDS byte of the range's first compressed dword / element byte
  uint32_t is8, gen;  // 16-bit masks over ranges 4 r + k
};

template <bool SGN>
__device__ __forceinline__ Ranges setup_ranges(const Lds& L, uint32_t b, uint32_t w, uint32_t l, uint32_t wsh,
                                               uint32_t wlast, uint32_t nv) {
  const uint32_t esh = wsh - 2;
  const uint32_t i = l & 15, r = i >> 2, k = i & 3;
  const uint32_t Q0 = 26 + nv * k + 4 * (1024 * r + 64 * w);
  // (a range whose units all lie past the chunk is never decoded or stored:
  // it reads at LDS byte 0; the bytes past the BWR output that the last
  // range reads decode to values no store takes, from window wlast)
  const bool valid = 1024 * r + 64 * w < (nv + 3) >> 2;
  const uint32_t W0 = min(Q0 >> wsh, wlast), W1 = min((Q0 + 255) >> wsh, wlast);
  const uint2 t0 = L.TAB[W0], t1 = L.TAB[W1];
  const uint32_t k0 = t0.x >> 20, k1 = t1.x >> 20;
  const bool raw = k0 == 2 && k1 == 2, b8 = k0 == 0 && k1 == 0;
  Ranges g;
  g.x0 = t0.x;
  g.x1 = t1.x;
  g.m0 = t0.y;
  g.m1 = t1.y;
  g.e0 = W0 << esh;
  g.e1 = W1 > W0 ? W1 << esh : 0xffffffffu;
  g.base = !valid ? 0u
           : raw  ? (t0.x & OFFM) + (Q0 - (W0 << wsh)) + b
                  : (t0.x & OFFM) + ((Q0 >> 2) - (W0 << esh)) + b;
  g.is8 = (uint32_t)__builtin_amdgcn_ballot_w64(l < 16 && valid && b8);
  g.gen = (uint32_t)__builtin_amdgcn_ballot_w64(l < 16 && valid && !raw && !b8);
  // W1's first element decoded: only the general decoder uses it (a second
  // dependent LDS round trip the other waves skip)
  g.s1 = 0;
  if (g.gen != 0) {
    const uint32_t y = rd32(L.IMG, (t1.x & OFFM) + b);
    g.s1 = k1 == 2 ? y : (k1 == 0 ? ext<SGN>(y, 0, 8) : ext<SGN>(y, 0, 16)) + t1.y;
  }
  return g;
}

// General ranges (16-bit windows, or two windows of different kinds): lane
// l's dword = bytes [s, 4) of element e and bytes [0, s) of e + 1.  Both
// come from one read at element e's compressed value in its own window (W0's
// below e1, else W1's; raw: from its byte s, so the read holds exactly the
// dword), except for the one lane whose e + 1 is W1's first element: those
// bytes are the range's s1.  The v_readlane's are taken before any select (a
// readlane under a lane-dependent condition becomes an exec-masked branch).
struct GenRange {
  uint32_t x0, x1, m0, m1, e0, e1, s1;
};
__device__ __forceinline__ GenRange gen_range(const Ranges& g, uint32_t i) {
  return GenRange{(uint32_t)__builtin_amdgcn_readlane(g.x0, i), (uint32_t)__builtin_amdgcn_readlane(g.x1, i),
                  (uint32_t)__builtin_amdgcn_readlane(g.m0, i), (uint32_t)__builtin_amdgcn_readlane(g.m1, i),
                  (uint32_t)__builtin_amdgcn_readlane(g.e0, i), (uint32_t)__builtin_amdgcn_readlane(g.e1, i),
                  (uint32_t)__builtin_amdgcn_readlane(g.s1, i)};
}
__device__ __forceinline__ uint32_t gen_addr(const GenRange& q, uint32_t e, uint32_t b, uint32_t s) {
  const bool hi = e >= q.e1;
  const uint32_t tx = hi ? q.x1 : q.x0, st = hi ? q.e1 : q.e0, kind = tx >> 20;
  return (tx & OFFM) + ((e - st) << kind) + b + (kind == 2 ? s : 0u);
}
template <bool SGN>
__device__ __forceinline__ uint32_t gen_dword(const GenRange& q, uint32_t e, uint32_t y, uint32_t s) {
  const bool hi = e >= q.e1;
  const uint32_t tx = hi ? q.x1 : q.x0, mn = hi ? q.m1 : q.m0, kind = tx >> 20;
  const uint32_t v0 = (kind == 0 ? ext<SGN>(y, 0, 8) : ext<SGN>(y, 0, 16)) + mn;
  const uint32_t v1 = (kind == 0 ? ext<SGN>(y, 8, 8) : ext<SGN>(y, 16, 16)) + mn;
  // raw: y = the dword itself (bytes [s, 4) of e, then e + 1's); as values:
  // e's at its bytes [s, 4), e + 1's at [0, s)
  const uint32_t a = kind == 2 ? y << (8 * s) : v0;
  const uint32_t bn = kind == 2 ? __builtin_amdgcn_alignbyte(0u, y, 4 - s) : v1;
  const uint32_t bh = e + 1 == q.e1 ? q.s1 : bn;
  return __builtin_amdgcn_alignbyte(bh, a, s);
}

// Output unit u (16 B at o + 16384 r, u = 1024 r + T) of a chunk of nv
// values: whole below nv / 4, the last one partial (nv mod 4 dwords) when
// nv is not a multiple of 4, nothing past it.  The output is 4-B aligned
// (a chunk of a multi-chunk tile starts at a multiple of its size).
typedef uint32_t v4a __attribute__((ext_vector_type(4))) __attribute__((aligned(4)));
typedef __attribute__((address_space(1))) v4a g_a4;
__device__ __forceinline__ void store_unit(uint8_t* p, const v4u& v, uint32_t u, uint32_t nv, bool whole) {
  // (whole: the wave's 64 units all lie below nv / 4 -- a wave-uniform test
  // that keeps the lane test to the one wave-round holding the chunk's end)
  if (whole) {
    __builtin_nontemporal_store((v4a)v, (g_a4*)p);
  } else if (u < (nv >> 2)) {
    __builtin_nontemporal_store((v4a)v, (g_a4*)p);
  } else if (u < ((nv + 3) >> 2)) {
    uint32_t* q = (uint32_t*)p;
    q[0] = v.x;
    if ((nv & 3) > 1) q[1] = v.y;
    if ((nv & 3) > 2) q[2] = v.z;
  }
}

// NR ranges (NR / 4 rounds from round r0): reads, decode, stores
// (hook: called by every wave once all of its reads are issued, before the
// first store -- the multi-chunk variant's point to issue the next chunk's
// DMA, tdbg_c5tile's chunk loop)
struct NoHook {
  __device__ __forceinline__ void operator()() const {}
};
// FULL: a full 64 KiB chunk (no per-round test, whole-unit stores without a
// lane test); RAW: every range of the wave raw (every rand wave): no
// per-range decoder branch.  (Both measured: the branch-free all-raw full
// path rand 0.739 -> 0.757, same box, profiles/r06/ab_rawf.txt.)
// PAT >= 0: the wave's 8-bit ranges are planes k with bit k of PAT set, in every round (a constant
// high byte plane's windows: ramp-like columns) -- the decoder per range is fixed at compile time.
template <bool SGN, int ABL, bool GEN, int NR, typename Hook = NoHook, bool FULL = false, bool RAW = false,
          int PAT = -1>
__device__ __forceinline__ void decode_store(const Lds& L, const Ranges& g, uint32_t b, uint32_t w, uint32_t l,
                                             uint8_t* o, uint32_t r0, uint32_t nv, const Hook& hook = Hook()) {
  uint32_t y[NR];
#pragma unroll
  for (uint32_t j = 0; j < NR; j++) {
    const uint32_t i = 4 * r0 + j;
    const uint32_t Q0 = 26 + nv * (i & 3) + 4 * (1024 * (i >> 2) + 64 * w);
    const uint32_t e = (Q0 >> 2) + l;
    const bool r8 = PAT >= 0 ? ((PAT >> (i & 3)) & 1) != 0 : (!RAW && ((g.is8 >> i) & 1));
    uint32_t a = __builtin_amdgcn_readlane(g.base, i) + (r8 ? l : 4 * l);
    if (GEN && ((g.gen >> i) & 1)) a = gen_addr(gen_range(g, i), e, b, Q0 & 3);
    y[j] = (ABL == 1 || ABL == 2) ? l + i : rd32(L.IMG, a);
  }
  hook();
#pragma unroll
  for (uint32_t rr = 0; rr < NR / 4; rr++) {
    const uint32_t r = r0 + rr;
    if (!FULL && 1024 * r + 64 * w >= ((nv + 3) >> 2)) break;  // (wave-uniform: no unit of this round is in the chunk)
    uint32_t x[4];
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) {
      const uint32_t i = 4 * r + k;
      x[k] = y[4 * rr + k];
      if (RAW || ABL == 1 || ABL == 2 || ABL == 5) continue;
      const uint32_t Q0 = 26 + nv * k + 4 * (1024 * r + 64 * w);
      const uint32_t e = (Q0 >> 2) + l, sk = Q0 & 3;
      // (wave-uniform branches: all 16 reads are already in flight)
      if (PAT >= 0) {
        if ((PAT >> k) & 1) {
          const uint32_t m0 = __builtin_amdgcn_readlane(g.m0, i), m1 = __builtin_amdgcn_readlane(g.m1, i),
                         e1 = __builtin_amdgcn_readlane(g.e1, i);
          const uint32_t v0 = ext<SGN>(x[k], 0, 8) + (e < e1 ? m0 : m1), v1 = ext<SGN>(x[k], 8, 8) + (e + 1 < e1 ? m0 : m1);
          x[k] = __builtin_amdgcn_alignbyte(v1, v0, sk);
        }
      } else if ((g.is8 >> i) & 1) {
        const uint32_t m0 = __builtin_amdgcn_readlane(g.m0, i), m1 = __builtin_amdgcn_readlane(g.m1, i),
                       e1 = __builtin_amdgcn_readlane(g.e1, i);
        const uint32_t v0 = ext<SGN>(x[k], 0, 8) + (e < e1 ? m0 : m1), v1 = ext<SGN>(x[k], 8, 8) + (e + 1 < e1 ? m0 : m1);
        x[k] = __builtin_amdgcn_alignbyte(v1, v0, sk);
      } else if (GEN && ((g.gen >> i) & 1)) {
        x[k] = gen_dword<SGN>(gen_range(g, i), e, x[k], sk);
      }
    }
    const v4u v = unshuffle4(x);
    if (FULL && ABL == 0)
      __builtin_nontemporal_store((v4a)v, (g_a4*)(o + 16384u * r));
    else if (ABL != 3 || (v.x == 0x9e3779b9u && v.y == 0x7f4a7c15u))
      store_unit(o + 16384u * r, v, 1024 * r + 64 * w + l, nv, 1024 * r + 64 * w + 64 <= (nv >> 2));
  }
}

// ---------------------------------------------------------------------------
// coded DoubleDelta tiles (bitsize 1..30)
// ---------------------------------------------------------------------------
// Thread T owns DD values 16 T .. 16 T + 15 (stream order: plane K = T / 256,
// so each wave's 1,024 values are one block of the scan), i.e. codes
// 16 T - 2 .. 16 T + 13 of the stream (values 0 and 1 are the header's x0
// and x1, which enter as pseudo codes x0 and x1 - 2 x0).  The codes' bits
// lie in BWR-output elements (dwords) es .. es + 19; the lane decodes those
// 20 elements straight from the image (two window entries per lane: 20
// elements span at most two windows of >= 64), realigns them into the
// MSB-first code stream and extracts its 16 codes at compile-time bit
// positions (one instantiation per code width CB = bitsize + 1).

// DD^-1 codes of one lane (CB = bitsize + 1).  H: the dwords at byte 2 of
// the lane's 20 BWR elements (the stream's u64 words start at BWR-output byte
// 34: word q = bytes [34 + 8 q, 42 + 8 q)); the MSB-first dword sequence
// swaps the halves of every word.  p: parity of the first dword, n: alignbit
// amount (dd_compressor.cc:384-399 reads a code as 1 sign bit + bitsize
// magnitude bits).
template <int CB>
__device__ __forceinline__ void dd_codes(const uint32_t (&H)[18], uint32_t p, uint32_t n, bool first,
                                         uint32_t x0, uint32_t x1, uint32_t (&xl)[16], uint32_t& Aout,
                                         uint32_t& Bout) {
  uint32_t pm = 0u - p;
  asm volatile("" : "+v"(pm));  // (opaque: the select stays one v_bfi_b32)
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

// DD aggregate combine: the block with aggregate (Ap, Bp) precedes `self`
// (nself codes): B = Bp + nself * Ap + B, A = Ap + A.
template <int CTRL, int ROWS>
__device__ __forceinline__ void scan_step(uint32_t& A, uint32_t& B, uint32_t nself) {
  const uint32_t Ap = dpp0<CTRL, ROWS>(A), Bp = dpp0<CTRL, ROWS>(B);
  B = B + Bp + nself * Ap;
  A = A + Ap;
}

// The lane's 16 values (local running sums) and its exclusive wave prefix
// (ae, be); lane 63 publishes the wave total.
template <int CB>
__device__ __forceinline__ void coded_lane(Lds& L, uint32_t w, uint32_t l, uint32_t x0, uint32_t x1,
                                           uint32_t (&xk)[16], uint32_t& ae, uint32_t& be, uint32_t nv) {
  if (1024 * w >= nv) {
    // (a wave whose values all lie past the chunk: nothing to decode; its
    // block folds as zeros, after every real value)
#pragma unroll
    for (int i = 0; i < 16; i++) xk[i] = 0;
    ae = be = 0;
    if (l == 63) {
      L.red[w][0] = 0;
      L.red[w][1] = 0;
    }
    return;
  }
  const int32_t T = (int32_t)(64 * w + l);
  const int32_t P0 = (16 * T - 2) * CB;  // stream bit of the lane's first code
  const int32_t b0 = (P0 + 31) >> 5;
  const uint32_t n = (uint32_t)(32 * b0 - P0);
  const int32_t Ms = b0 - 1;              // first MSB-first stream dword needed
  const uint32_t p = (uint32_t)Ms & 1u;
  const uint32_t es = (uint32_t)(8 + 2 * (Ms >> 1));
  // the lane's 20 elements of the decoded stream (es is even: 8-B reads)
  uint32_t G[20];
#pragma unroll
  for (int x = 0; x < 10; x++) {
    const uint2 v = *(const uint2*)(L.IMG + es + 2 * x);
    G[2 * x] = v.x;
    G[2 * x + 1] = v.y;
  }
  // a wave whose codes are all zero (a constant-stride run: the common case
  // in DD streams of run-heavy columns) skips the realignment, extraction
  // and scan: every running sum and the wave's aggregate are 0 (wave 0 never
  // does, its lane 0 injects the two header values)
  uint32_t z = 0;
#pragma unroll
  for (int x = 0; x < 20; x++) z |= G[x];
  if (__builtin_amdgcn_ballot_w64(z != 0 || w == 0) == 0) {
#pragma unroll
    for (int i = 0; i < 16; i++) xk[i] = 0;
    ae = be = 0;
    if (l == 63) {
      L.red[w][0] = 0;
      L.red[w][1] = 0;
    }
    return;
  }
  uint32_t H[18];
#pragma unroll
  for (int x = 0; x < 18; x++) H[x] = __builtin_amdgcn_alignbyte(G[x + 1], G[x], 2);
  uint32_t A = 0, B = 0;
  dd_codes<CB>(H, p, n, T == 0, x0, x1, xk, A, B);
  const uint32_t As = A, Bs = B;
  scan_step<DPP_ROW_SHR1, 0xf>(A, B, 16);
  scan_step<DPP_ROW_SHR2, 0xf>(A, B, 32);
  scan_step<DPP_ROW_SHR4, 0xf>(A, B, 64);
  scan_step<DPP_ROW_SHR8, 0xf>(A, B, 128);
  scan_step<DPP_ROW_BCAST15, 0xa>(A, B, 16 * ((l & 15) + 1));
  scan_step<DPP_ROW_BCAST31, 0xc>(A, B, 16 * ((l & 31) + 1));
  ae = A - As;
  be = B - Bs - 16 * (A - As);
  if (l == 63) {
    L.red[w][0] = A;
    L.red[w][1] = B;
  }
}

// LDS dword of DD value v in the value buffer (written by its owner as four
// 16-B slots, slot q of thread T at 4 T + (q ^ ((T >> 2) & 3)): the b128
// writes of lanes T and T + 4 do not share banks)
__device__ __forceinline__ uint32_t vslot(uint32_t v) {
  const uint32_t T = v >> 4, q = (v >> 2) & 3;
  return 4 * (4 * T + (q ^ ((T >> 2) & 3))) + (v & 3);
}

// A coded tile: codes, scans (one barrier publishes the 16 wave totals and
// frees the image), the fold of each lane's prefix into its values, the
// values into LDS (second barrier), then byteshuffle^-1 and the stores.
template <int CB, bool SGN, int ABL, bool MC, typename Hook>
__device__ __forceinline__ void coded_tile(Lds& L, const Desc& d, uint32_t b, uint32_t esh, uint32_t wlast,
                                           uint32_t w, uint32_t l, uint32_t nv, uint64_t* prof, const Hook& hook) {
  const uint32_t x0 = __builtin_amdgcn_readfirstlane(L.hd[4]), x1 = __builtin_amdgcn_readfirstlane(L.hd[5]);
  uint32_t xk[16], ae, be;
  const uint64_t c3 = prof ? __builtin_amdgcn_s_memtime() : 0;
  bwr_materialize<SGN>(L.IMG, L.TAB, b, esh, wlast, w, l, (__builtin_amdgcn_readfirstlane(L.hd[6]) + 15) >> 4);
  lds_barrier();  // the decoded stream
  coded_lane<CB>(L, w, l, x0, x1, xk, ae, be, nv);
  const uint64_t c4 = prof ? __builtin_amdgcn_s_memtime() : 0;
  lds_barrier();
  // the start state (X, D) of this wave's block: the exclusive fold of the
  // waves before it (1,024 codes each); lane v < 16 holds wave v's total and
  // a DPP scan over the 16 lanes does the fold
  uint32_t X, Dd;
  {
    uint32_t A = l < 16 ? L.red[l][0] : 0u, B = l < 16 ? L.red[l][1] : 0u;
    const uint32_t As = A, Bs = B;
    scan_step<DPP_ROW_SHR1, 0xf>(A, B, 1024);
    scan_step<DPP_ROW_SHR2, 0xf>(A, B, 2048);
    scan_step<DPP_ROW_SHR4, 0xf>(A, B, 4096);
    scan_step<DPP_ROW_SHR8, 0xf>(A, B, 8192);
    // (inclusive over lanes 0..v; exclusive = minus lane v's own block)
    X = __builtin_amdgcn_readlane(B - Bs - 1024u * (A - As), w);
    Dd = __builtin_amdgcn_readlane(A - As, w);
  }
  uint32_t t = X + be + 16u * l * Dd;
  const uint32_t st = Dd + ae;
#pragma unroll
  for (int i = 0; i < 16; i++) {
    t += st;
    xk[i] += t;
  }
  const uint32_t T = 64 * w + l;
#pragma unroll
  for (uint32_t q = 0; q < 4; q++)
    *(v4u*)(L.IMG + 4 * (4 * T + (q ^ ((T >> 2) & 3)))) = v4u{xk[4 * q], xk[4 * q + 1], xk[4 * q + 2], xk[4 * q + 3]};
  const uint64_t c5 = prof ? __builtin_amdgcn_s_memtime() : 0;
  lds_barrier();
  const uint64_t c6 = prof ? __builtin_amdgcn_s_memtime() : 0;
  uint8_t* const o = d.out + 16u * T;
  if (nv == OUTB / 4) {
    // value 4096 k + 1024 r + T sits at dword vslot(T) + 4096 k + 1024 r (the
    // swizzle depends only on bits of T): one base, constant offsets
    const uint32_t* const vb = L.IMG + vslot(T);
    if constexpr (MC) {
      // (every value read before the hook: the next chunk's DMA may then
      // land over the value buffer while these stores go out)
      uint32_t x[16];
#pragma unroll
      for (uint32_t r = 0; r < 4; r++)
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) x[4 * r + k] = vb[4096 * k + 1024 * r];
      hook();
#pragma unroll
      for (uint32_t r = 0; r < 4; r++) {
        const uint32_t y[4] = {x[4 * r], x[4 * r + 1], x[4 * r + 2], x[4 * r + 3]};
        __builtin_nontemporal_store((v4a)unshuffle4(y), (g_a4*)(o + 16384u * r));
      }
    } else {
#pragma unroll
      for (uint32_t r = 0; r < 4; r++) {
        uint32_t x[4];
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) x[k] = vb[4096 * k + 1024 * r];
        const v4u v = unshuffle4(x);
        if (ABL != 3 || (v.x == 0x9e3779b9u && v.y == 0x7f4a7c15u))
          __builtin_nontemporal_store((v4a)v, (g_a4*)(o + 16384u * r));
      }
    }
  } else {
    // nv values: plane k starts at stream byte nv k, so unit u's plane dword
    // is bytes [nv k + 4 u, + 4) of the value stream (two values when nv k is
    // not a multiple of 4)
#pragma unroll
    for (uint32_t r = 0; r < 4; r++) {
      if (1024 * r + 64 * w >= ((nv + 3) >> 2)) break;  // (wave-uniform)
      uint32_t x[4];
#pragma unroll
      for (uint32_t k = 0; k < 4; k++) {
        const uint32_t v0 = ((nv * k) >> 2) + 1024 * r + T;
        if ((nv & 3) == 0)
          x[k] = L.IMG[vslot(v0)];
        else
          x[k] = __builtin_amdgcn_alignbyte(L.IMG[vslot(v0 + 1)], L.IMG[vslot(v0)], (nv * k) & 3);
      }
      const v4u v = unshuffle4(x);
      store_unit(o + 16384u * r, v, 1024 * r + T, nv, 1024 * r + 64 * w + 64 <= (nv >> 2));
    }
  }
  if (prof && l == 0 && (w == 0 || w == 15)) {
    // coded tiles: 2 codes + wave scan, 3 B3 + fold + value writes, 4 B4,
    // 5 transposes + stores (wave 0; wave 15 in 6)
    const uint64_t c7 = __builtin_amdgcn_s_memtime();
    if (w == 0) {
      prof[2] = c4 - c3;
      prof[3] = c5 - c4;
      prof[4] = c6 - c5;
      prof[5] = c7 - c6;
    } else {
      prof[6] = c7 - c3;
    }
  }
}

// ABL (timing ablations, outputs not meaningful): 1 no parse and no decode
// (DMA, barriers, constant stores), 2 parse but no decode, 3 no stores,
// 4 every wave on the one-read path, 5 no 8-bit combine, 6 two halves of 8
// one-read ranges
// MC: the multi-chunk variant (launches flagged TDBG_MULTI_CHUNK): tiles of
// several chunks are decoded chunk after chunk by their workgroup; without
// it they are declined (the fused kernel takes them).
template <bool SGN, int ABL, bool MC, bool PIPE = false>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(8, 8)))
unfilter_c5tile_kernel(const KParams kp, uint32_t base, uint32_t cnt) {
  __shared__ Lds L;
  const uint32_t w0 = wave_(), l0 = lane_();
  // diagnostics (KParams::prof, TDBG_PROF=1): shader clocks of workgroups
  // < 1024 (slots 8.. of the profile buffer's rows; the fused kernel, which runs
  // next, writes 0..7): 0 DMA wait, 1 parse, 2 range setup,
  // 3 / 4 / 5 decode + stores of waves 0 / 1 / 15, 6 whole workgroup
  uint64_t* const prof = kp.prof && blockIdx.x < 1024 ? kp.prof + (uint64_t)blockIdx.x * TDBG_PROF_PHASES + 8 : nullptr;
  const uint64_t c0 = prof ? __builtin_amdgcn_s_memtime() : 0;
  // this workgroup's work item: the XCD-contiguous deal of [base, base + cnt)
  // (chunk mode: cnt is the directory's capacity, the records are [0, device
  // count), so workgroups take them round-robin, which spreads the real ones
  // over every XCD however few they are -- ADVICE r5)
  const uint32_t n8 = (cnt + 7) >> 3;
  const uint32_t j = kp.chunks ? blockIdx.x : (blockIdx.x & 7) * n8 + (blockIdx.x >> 3);
  if (j >= cnt) return;
  const uint64_t t = (uint64_t)base + j;
  if (t >= work_items(kp)) return;
  const bool chunked = kp.chunks != nullptr;
  // the fused kernel's fallback queue starts empty for this launch (the
  // fused kernel runs next on the same stream and is the only one to append;
  // chunk mode: the directory pass cleared it and may have appended, so fbq
  // is not passed here)
  if (kp.fbq && blockIdx.x == 0 && threadIdx.x == 0) kp.fbq[0] = 0;
  const Desc d = load_desc(kp, t);
  // A tile of several chunks (tile mode; TileDB splits tiles over 64 KiB
  // into chunks of at most 64 KiB, tile.cc:87-100): this workgroup decodes
  // its chunks one after the other (FilterPipeline::run_reverse's loop over
  // chunks, filter_pipeline.cc:439-517).  The tile's chunk count and chunk
  // 0's header come from one load; each later chunk's 12-byte header rides
  // at the end of the previous chunk's image DMA.
  const bool mc = MC && !takes(kp, d) && !chunked && mc_tile(kp, d);
  if (!takes(kp, d) && !mc) {
    decline(kp, t);
    return;
  }
  if (mc) {
    // (uniform values: made scalar, so that nothing of the loop below is
    // taken for a per-lane value)
    const uint64_t n = ldn(d.in, 8);
    const uint32_t nlo = __builtin_amdgcn_readfirstlane((uint32_t)n), nhi = __builtin_amdgcn_readfirstlane((uint32_t)(n >> 32));
    if (nhi != 0 || nlo < 2 || nlo > (d.fs - 8) / 12) {
      decline(kp, t);
      return;
    }
    if (threadIdx.x == 0) {
      L.mcs[0][0] = 8;  // chunk 0's header follows the u64 chunk count
      L.mcs[0][1] = 0;
      L.mcs[0][2] = (uint32_t)ldn(d.in + 8, 4);
      L.mcs[0][3] = (uint32_t)ldn(d.in + 12, 4);
      L.mcs[0][4] = (uint32_t)ldn(d.in + 16, 4);
      L.mct[0] = nlo;
      L.mct[1] = (uint32_t)(uintptr_t)d.in;
      L.mct[2] = (uint32_t)((uintptr_t)d.in >> 32);
      L.mct[3] = (uint32_t)(uintptr_t)d.out;
      L.mct[4] = (uint32_t)((uintptr_t)d.out >> 32);
    }
    lds_barrier();
  }
  bool any_raw = false;
  // Multi-chunk tiles, pipelined: once every wave has read a full (64 KiB)
  // chunk out of LDS, the next chunk's image DMA is issued, before this
  // chunk's stores, so that its latency overlaps them (gfx950 counts loads
  // and stores in one in-order vmcnt: a DMA issued after the stores would
  // wait for them).  `issued`: this chunk's DMA went out in the previous
  // iteration, `after` its DMA instructions past the prefix, `pend` the
  // stores this wave issued after it (exact: one per full 16-B unit round).
  bool issued = false, declined = false;
  uint32_t after = 0, pend = 0;
  // (vmcnt wait with a run-time count; counts above 12 cannot occur)
  auto vm_wait = [](uint32_t n) {
    switch (__builtin_amdgcn_readfirstlane(n)) {
      case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
      case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
      case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
      case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
      case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
      case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
      case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
      case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
      case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
      case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
      case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
      case 11: asm volatile("s_waitcnt vmcnt(11)" ::: "memory"); break;
      default: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    }
  };
  for (uint32_t k = 0;; k++) {
    // (the lane index made opaque per chunk: nothing per-lane is computed
    // once before the loop and held in registers through it)
    uint32_t l = l0, w = w0, img = lds_addr(L.IMG);
    if (MC) {
      l = lane_();
      asm volatile("" : "+s"(w), "+s"(img));  // (the same for the wave and the LDS addresses derived from them)
    }
    // The image's aligned cover by LDS-DMA.  Wave 0 moves the prefix first
    // (units [0, PFX): tile and chunk headers, every window header, the frame
    // and the DD headers -- all the parse reads); the rest of the image
    // (units PFX + 64 (w + 16 i) + l) goes out from every wave.  Returns the
    // DMA instructions this wave issued after the prefix.
    auto issue_dma = [&](const Desc& q, uint32_t ex) -> uint32_t {
      const uint64_t a0 = (uint64_t)q.in & ~15ull;
      const uint32_t nu = (uint32_t)((((uint64_t)q.in & 15) + q.fs + ex + 15) >> 4);
      if (w == 0) {
#pragma unroll
        for (uint32_t u = 0; u < PFX / 64; u++)
          if (64 * u < nu && 64 * u + l < nu) dma16(a0 + 16ull * (64 * u + l), img + 1024 * u);
      }
      uint32_t n = 0;
      uint64_t src = a0 + 16ull * (PFX + 64 * w + l);  // (one address, stepped: registers)
#pragma unroll
      for (uint32_t i = 0; i < (IMGU - PFX + NT - 1) / NT; i++) {
        const uint32_t u0 = PFX + 64 * (w + 16 * i);
        if (u0 < nu) {
          n++;
          if (u0 + l < nu) dma16(src, img + 16 * u0);
        }
        src += 16ull * NT;
      }
      return n;
    };
    // (multi-chunk) chunk k of the tile from the loop state; checked: a
    // chunk this kernel decodes, inside the tile, and (the last one)
    // completing the tile's unfiltered size (tile.cc:305-309)
    auto chunk_desc = [&](uint32_t cur, uint32_t out_off, uint32_t ho, uint32_t hf, uint32_t hm, uint32_t kk,
                          uint32_t nch, Desc& q, uint32_t& ex) -> bool {
      const bool last = kk + 1 == nch;
      const uint64_t cfs = 12ull + hm + hf;
      ex = last ? 0u : 12u;
      // (the builtin returns int: each half goes through uint32_t, or a low
      // half with its top bit set would be sign-extended over the high one)
      auto u = [&](int i) -> uint64_t { return (uint32_t)__builtin_amdgcn_readfirstlane(L.mct[i]); };
      const uint64_t tin = (u(2) << 32) | u(1), tout = (u(4) << 32) | u(3);
      q.t = t;
      q.fs = cfs;
      q.os = ho;
      q.in = (const uint8_t*)(tin + cur);
      q.out = (uint8_t*)(tout + out_off);
      return (uint64_t)cur + cfs + ex <= d.fs && ho >= 64 && ho <= OUTB && (ho & 3) == 0 && cfs + ex <= IMG_CAP &&
             (uint64_t)out_off + ho <= d.os && (!last || (uint64_t)out_off + ho == d.os);
    };
    Desc dk = d;
    uint32_t extra = 0;  // bytes DMA'd past the image: the next chunk's header
    if (mc) {
      auto S = [&](int i) -> uint32_t { return __builtin_amdgcn_readfirstlane(L.mcs[k & 1][i]); };
      if (!chunk_desc(S(0), S(1), S(2), S(3), S(4), k, __builtin_amdgcn_readfirstlane(L.mct[0]), dk, extra)) {
        declined = true;
        break;
      }
    }
    uint64_t* const pf = mc ? nullptr : prof;
    if (!issued) {
      after = __builtin_amdgcn_readfirstlane(issue_dma(dk, extra));
      pend = 0;
    }
    if (w == 0 && ABL != 1) {
      // (vmcnt counts in issue order: the prefix has landed when at most
      // `after` DMA instructions and the `pend` stores behind them are left)
      vm_wait(after + pend);
      // (the parse is the one serial step of a tile: it issues first on its
      // SIMD, ahead of the other workgroup's waves)
      __builtin_amdgcn_s_setprio(3);
      parse<SGN>(L, dk, l, chunked || mc);
      __builtin_amdgcn_s_setprio(0);
    }
    const uint64_t c1 = pf ? __builtin_amdgcn_s_memtime() : 0;
    vm_wait(pend);
    lds_barrier();
    const uint64_t c2 = pf ? __builtin_amdgcn_s_memtime() : 0;
    if (ABL != 1 && __builtin_amdgcn_readfirstlane(L.hd[0]) == 0) {
      declined = true;
      break;
    }
    const uint32_t wsh = __builtin_amdgcn_readfirstlane(L.hd[1]);
    const uint32_t b = (uint32_t)((uintptr_t)dk.in & 15);
    const uint32_t cb = __builtin_amdgcn_readfirstlane(L.hd[3]);
    const uint32_t wlast = __builtin_amdgcn_readfirstlane(L.hd[2]);
    const uint32_t nv = __builtin_amdgcn_readfirstlane(L.hd[7]);
    // the next chunk (its header was DMA'd behind this image) and whether its
    // DMA goes out before this chunk's stores
    Desc dn = dk;
    uint32_t extra_n = 0;
    bool pipe = false;
    if (mc && extra) {
      const uint32_t hb = b + (uint32_t)dk.fs;
      const uint32_t nho = __builtin_amdgcn_readfirstlane(rd32(L.IMG, hb)),
                     nhf = __builtin_amdgcn_readfirstlane(rd32(L.IMG, hb + 4)),
                     nhm = __builtin_amdgcn_readfirstlane(rd32(L.IMG, hb + 8));
      const uint32_t ncur = __builtin_amdgcn_readfirstlane(L.mcs[k & 1][0]) + (uint32_t)dk.fs,
                     nout = __builtin_amdgcn_readfirstlane(L.mcs[k & 1][1]) + (uint32_t)dk.os;
      pipe = chunk_desc(ncur, nout, nho, nhf, nhm, k + 1, __builtin_amdgcn_readfirstlane(L.mct[0]), dn, extra_n) &&
             dk.os == OUTB && PIPE;
      // the next chunk's state, into the other buffer (read after the next
      // barrier: the hook's, or the end of this chunk's)
      if (threadIdx.x == 0) {
        uint32_t* const m = L.mcs[(k + 1) & 1];
        m[0] = ncur;
        m[1] = nout;
        m[2] = nho;
        m[3] = nhf;
        m[4] = nhm;
      }
    }
    uint32_t after_n = 0;
    // the next chunk's DMA, once every wave's reads of this chunk are issued
    // and done (the barrier): before this chunk's stores
    auto hook = [&]() {
      if (!pipe) return;
      lds_barrier();
      after_n = __builtin_amdgcn_readfirstlane(issue_dma(dn, extra_n));
    };
    if (cb != 0) {
      // coded DoubleDelta: one instantiation per code width
      switch (cb) {
#define TDBG_CB(c) \
  case c: coded_tile<c, SGN, ABL, MC && PIPE>(L, dk, b, wsh - 2, wlast, w, l, nv, pf, hook); break;
        TDBG_CB(2) TDBG_CB(3) TDBG_CB(4) TDBG_CB(5) TDBG_CB(6) TDBG_CB(7) TDBG_CB(8) TDBG_CB(9)
        TDBG_CB(10) TDBG_CB(11) TDBG_CB(12) TDBG_CB(13) TDBG_CB(14) TDBG_CB(15) TDBG_CB(16)
        TDBG_CB(17) TDBG_CB(18) TDBG_CB(19) TDBG_CB(20) TDBG_CB(21) TDBG_CB(22) TDBG_CB(23)
        TDBG_CB(24) TDBG_CB(25) TDBG_CB(26) TDBG_CB(27) TDBG_CB(28) TDBG_CB(29) TDBG_CB(30)
        TDBG_CB(31)
#undef TDBG_CB
        default: break;
      }
      pend = 4;  // (pipelined: a full chunk's four unit rounds)
      if (pf && threadIdx.x == 0) {
        pf[0] = c1 - c0;
        pf[1] = c2 - c1;
      }
    } else {
      any_raw = true;
      const Ranges g = setup_ranges<SGN>(L, b, w, l, wsh, wlast, nv);
      uint8_t* const o = dk.out + 16u * (64 * w + l);
      // (the wave's ranges inside the chunk: rounds r with 1024 r + 64 w < nv / 4)
      uint32_t vmask = 0;
      if constexpr (!PIPE) {
        const uint32_t nu4 = (nv + 3) >> 2;
        const uint32_t vr = nu4 <= 64 * w ? 0u : min(4u, (nu4 - 64 * w + 1023) >> 10);
        vmask = vr >= 4 ? 0xFFFFu : (1u << (4 * vr)) - 1u;
      }
      const uint64_t c3 = pf ? __builtin_amdgcn_s_memtime() + (uint64_t)(g.x0 & 0) : 0;
      // All 16 ranges' reads first, then the decode and one store per round.
      // Raw and 8-bit ranges read one dword (the decoder picked by a select).
      // The few general ranges (a wave of a ramp tile on a plane boundary)
      // take the per-element decoder under a wave-uniform branch that holds
      // no LDS access, so the reads stay in flight together (8 at a time in
      // such waves, for registers).  (Measured, not kept: the general rounds
      // first, one at a time, then all 16 one-read ranges together -- ramp
      // -0.9 %, rand -1.1 % on one box, profiles/r06/ab_general_first.txt.)
      if (MC && pipe && g.gen == 0) {
        // (pipelined: two halves of 8 ranges, the next chunk's DMA after the
        // second half's reads -- 16 reads held through the DMA issue do not
        // fit the registers)
        decode_store<SGN, ABL, false, 8>(L, g, b, w, l, o, 0, nv);
        decode_store<SGN, ABL, false, 8>(L, g, b, w, l, o, 2, nv, hook);
        pend = 2;
      } else if (ABL == 0 && g.gen == 0 && g.is8 == 0 && nv == OUTB / 4) {
        decode_store<SGN, ABL, false, 16, NoHook, true, true>(L, g, b, w, l, o, 0, nv);
        hook();  // (a no-op unless pipelined)
        pend = 0;
      } else if (ABL == 0 && g.gen == 0 && nv == OUTB / 4) {
        // (the common plane patterns of 8-bit ranges: decoders fixed at compile time)
        switch (g.is8) {
          case 0xCCCCu: decode_store<SGN, ABL, false, 16, NoHook, true, false, 0xC>(L, g, b, w, l, o, 0, nv); break;
          case 0x8888u: decode_store<SGN, ABL, false, 16, NoHook, true, false, 0x8>(L, g, b, w, l, o, 0, nv); break;
          case 0xEEEEu: decode_store<SGN, ABL, false, 16, NoHook, true, false, 0xE>(L, g, b, w, l, o, 0, nv); break;
          case 0xFFFFu: decode_store<SGN, ABL, false, 16, NoHook, true, false, 0xF>(L, g, b, w, l, o, 0, nv); break;
          default: decode_store<SGN, ABL, false, 16, NoHook, true>(L, g, b, w, l, o, 0, nv); break;
        }
        hook();
        pend = 0;
      } else if (ABL == 0 && g.gen == 0 && g.is8 == 0) {
        // (all raw in a shorter chunk: no per-range decoder branch)
        decode_store<SGN, ABL, false, 16, NoHook, false, true>(L, g, b, w, l, o, 0, nv);
        hook();
        pend = 0;
      } else if (ABL == 0 && !PIPE && g.gen == 0 && g.is8 != 0 &&
                 (g.is8 == (0xCCCCu & vmask) || g.is8 == (0x8888u & vmask))) {
        // (shorter chunks: the plane patterns over the wave's rounds inside the chunk)
        if (g.is8 == (0xCCCCu & vmask)) decode_store<SGN, ABL, false, 16, NoHook, false, false, 0xC>(L, g, b, w, l, o, 0, nv);
        else decode_store<SGN, ABL, false, 16, NoHook, false, false, 0x8>(L, g, b, w, l, o, 0, nv);
        hook();
        pend = 0;
      } else if (g.gen == 0 || ABL == 4) {
        decode_store<SGN, ABL, false, 16>(L, g, b, w, l, o, 0, nv);
        hook();  // (a no-op unless pipelined)
        pend = 0;
      } else if (ABL == 6) {
        decode_store<SGN, ABL, false, 8>(L, g, b, w, l, o, 0, nv);
        decode_store<SGN, ABL, false, 8>(L, g, b, w, l, o, 2, nv);
      } else if (ABL == 0 && nv == OUTB / 4) {
        decode_store<SGN, ABL, true, 8, NoHook, true>(L, g, b, w, l, o, 0, nv);
        decode_store<SGN, ABL, true, 8, NoHook, true>(L, g, b, w, l, o, 2, nv);
        hook();
        pend = 0;
      } else {
        decode_store<SGN, ABL, true, 8>(L, g, b, w, l, o, 0, nv);
        decode_store<SGN, ABL, true, 8>(L, g, b, w, l, o, 2, nv);
        // (such a wave -- a ramp tile's plane boundary -- takes part in the
        // next chunk's DMA after its stores: registers)
        hook();
        pend = 0;
      }
      if (pf && l == 0) {
        const uint64_t c4 = __builtin_amdgcn_s_memtime();
        if (w == 0) {
          pf[0] = c1 - c0;
          pf[1] = c2 - c1;
          pf[2] = c3 - c2;
          pf[3] = c4 - c3;
          pf[6] = c4 - c0;
        }
        if (w == 1) pf[4] = c4 - c3;
        if (w == 15) pf[5] = c4 - c3;
      }
    }
    if (!mc || extra == 0) break;  // (the last chunk DMA'd no next header)
    if (!pipe) {
      lds_barrier();  // every wave is done with this chunk's image, table and headers
      pend = 0;
    }
    issued = pipe;
    after = __builtin_amdgcn_readfirstlane(after_n);
    pend = __builtin_amdgcn_readfirstlane(pend);
  }
  if (declined) {
    // (a pipelined DMA may still be in flight into LDS: it drains before the
    // workgroup ends; nothing reads it)
    decline(kp, t);
    return;
  }
  if (threadIdx.x == 0) {
    if (kp.status && !chunked) kp.status[t] = TDBG_OK;
    if (kp.stats) {
      // one slot of 16 counters per 64 workgroups (tdbg_host.cpp read_stats
      // sums the slots): one address for every workgroup of a 100,000-tile
      // launch would serialise its atomics
      uint64_t* s = kp.stats + TDBG_STAT_STRIDE * (1 + (blockIdx.x & 63));
      if (chunked) {
        atomicAdd((unsigned long long*)&s[TDBG_STAT_STREAM_CHUNKS], 1ull);
      } else {
        atomicAdd((unsigned long long*)&s[TDBG_STAT_FUSED_TILES], 1ull);
        atomicAdd((unsigned long long*)&s[TDBG_STAT_FUSED_BYTES], (unsigned long long)d.os);
        atomicAdd((unsigned long long*)&s[TDBG_STAT_STREAM_TILES], 1ull);
        if (any_raw && !mc) atomicAdd((unsigned long long*)&s[TDBG_STAT_STREAM_RAW_TILES], 1ull);
        if (mc) atomicAdd((unsigned long long*)&s[TDBG_STAT_TILE_CHUNKS], (unsigned long long)L.mct[0]);
      }
    }
  }
}

}  // namespace c5t
}  // namespace tdbg

// one workgroup per work item (kp->ntiles of them, or in chunk mode the
// directory's capacity: items past the device count exit at once); launches
// of at most GRID_CAP items
template <typename K>
static hipError_t c5tile_grid(K k, const tdbg::KParams* kp, hipStream_t s) {
  using namespace tdbg::c5t;
  for (uint64_t base = 0; base < kp->ntiles; base += GRID_CAP) {
    const uint32_t cnt = (uint32_t)std::min<uint64_t>(kp->ntiles - base, GRID_CAP);
    const uint32_t grid = 8 * ((cnt + 7) / 8);
    TDBG_LAUNCH(k, dim3(grid), dim3(NT), s, *kp, (uint32_t)base, cnt);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

#ifdef TDBG_C5T_MC_UNIT
// The multi-chunk variant is its own translation unit, compiled with
// -mllvm -disable-machine-licm (tiledb_amd/build.py): its chunk loop holds
// the whole decoder, and loop-invariant code hoisted out of it (LDS
// addresses, kernel-argument tests) outgrew the 64 VGPRs of 8 waves per SIMD
// and spilled to scratch, which the counted vmcnt waits cannot allow.
extern "C" hipError_t tdbg_launch_c5tile_mc(const tdbg::KParams* kp, int sgn, hipStream_t s) {
  using namespace tdbg::c5t;
#ifdef TDBG_EXPERIMENTS
  // A/B: the next chunk's DMA issued before this chunk's stores (measured
  // slower: profiles/r06/c5big_pipe_ab.txt)
  static const bool pipe = tdbg_hook("TDBG_C5T_PIPE") != nullptr;  // experiments
  if (pipe)
    return c5tile_grid(sgn ? unfilter_c5tile_kernel<true, 0, true, true> : unfilter_c5tile_kernel<false, 0, true, true>,
                       kp, s);
#endif
  return c5tile_grid(sgn ? unfilter_c5tile_kernel<true, 0, true> : unfilter_c5tile_kernel<false, 0, true>, kp, s);
}
#else
extern "C" hipError_t tdbg_launch_c5tile_mc(const tdbg::KParams* kp, int sgn, hipStream_t s);

extern "C" hipError_t tdbg_launch_c5tile(const tdbg::KParams* kp, int sgn, int mc, hipStream_t s) {
  using namespace tdbg::c5t;
  if (mc) return tdbg_launch_c5tile_mc(kp, sgn, s);
#ifdef TDBG_EXPERIMENTS
  static const int abl = tdbg_hook("TDBG_C5T_ABL") ? atoi(tdbg_hook("TDBG_C5T_ABL")) : 0;  // experiments
  auto k = sgn ? (abl == 1   ? unfilter_c5tile_kernel<true, 1, false>
                  : abl == 2 ? unfilter_c5tile_kernel<true, 2, false>
                  : abl == 3 ? unfilter_c5tile_kernel<true, 3, false>
                  : abl == 4 ? unfilter_c5tile_kernel<true, 4, false>
                  : abl == 5 ? unfilter_c5tile_kernel<true, 5, false>
                  : abl == 6 ? unfilter_c5tile_kernel<true, 6, false>
                             : unfilter_c5tile_kernel<true, 0, false>)
               : unfilter_c5tile_kernel<false, 0, false>;
#else
  auto k = sgn ? unfilter_c5tile_kernel<true, 0, false> : unfilter_c5tile_kernel<false, 0, false>;
#endif
  return c5tile_grid(k, kp, s);
}
#endif
