// tdbg_stream_raw.hip -- streaming unfilter kernel for headline-pipeline
// tiles whose DoubleDelta stage stored the values raw:
// [BYTESHUFFLE, DOUBLE_DELTA, BIT_WIDTH_REDUCTION] on 4-byte integers, one
// 64 KiB chunk, DD data part = [u8 bitsize >= 31][u64 n][n raw values]
// (dd_compressor.cc:233-236 on write, :327-331 on read: "copy the rest").
// These are the C5 "rand" and "ramp" tiles of SURVEY 8(d): their filtered
// images are 40-68 KB, too big for the coded kernel's whole-image staging
// (tdbg_stream.hip), so this kernel owns every tile above that kernel's
// staging cap and never stages a whole image:
//
//   * Only the tile's prefix (tile + chunk header, BWR and compression-frame
//     metadata, the start of BWR window 0: <= 4 KiB) is staged in LDS, by
//     LDS-DMA issued one tile ahead.  Wave 0 parses it: every window header
//     (bit_width_reduction_filter.cc:353-380), the prefix sums of the windows'
//     compressed sizes (the window table), the compression frame
//     (compression_filter.cc:413-486) and the two DD headers at BWR-output
//     bytes [0, 26) (dd_compressor.cc:314-331); one barrier publishes it.
//   * Ownership follows the output.  Output unit j (16 B, elements 4j..4j+3)
//     is byteshuffle⁻¹ of dword j of the four byte planes
//     (byteshuffle_filter.cc:111-166), i.e. of the four BWR-output dwords at
//     bytes 26 + 16384 k + 4 j: the raw DD part starts at BWR-output byte 26
//     (c0 = 17 B, c1's header = 9 B).  A wave owns 1,024 units and works
//     through them in jobs of 128: for each plane it LDS-DMAs just the
//     compressed bytes of the job's 512-byte plane range (at most 33 16-B
//     units), double-buffered per wave, with counted vmcnt waits -- no
//     workgroup barrier inside a tile.
//   * BWR⁻¹ per dword, with one wave-uniform decoder per job and plane:
//     all-raw windows (a plain unaligned dword read), all-8-bit windows (two
//     bytes, sign/zero extended, plus their window minimum), or the general
//     per-element decode for mixed or 16-bit windows.
//   * Byteshuffle⁻¹ in registers (v_perm 4x4 byte transposes); each store
//     instruction writes 1 KiB of whole lines, nontemporal.
//
// Any other tile it owns (wrong sizes, windows not a power of two in
// [256, 4096], a coded DD part, malformed headers, offsets tiles) is queued
// for the fused kernel (and from there the general interpreter), so every
// status and byte stays the reference's.  Nothing is written to a tile's
// output before all its checks passed.
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
namespace sraw {

using namespace sc;

#ifndef TDBG_RAW_PW
#define TDBG_RAW_PW 0
#endif
// PW: a fifth wave per workgroup (the parser) DMAs and parses tile n + 1's
// prefix while the four job waves decode tile n: one barrier per tile, and the
// parse is off the job waves' path.  Otherwise wave 0 parses between two
// barriers while the other waves wait.
constexpr bool PW = TDBG_RAW_PW != 0;
constexpr int NWV = 4;                    // job waves (wave64)
constexpr int NT = 64 * (NWV + (PW ? 1 : 0));
constexpr int NS = PW ? 2 : 1;            // window-table slots
constexpr uint32_t OUTB = 65536;     // output bytes per tile (one 64 KiB chunk of int32)
constexpr uint32_t SMALL = CODED_CAP;  // tiles this big or smaller belong to tdbg_stream.hip
constexpr uint32_t PFU = 256;        // prefix: 256 16-B units
constexpr uint32_t TABN = 320;       // BWR windows per chunk
constexpr uint32_t LBWR = 65562;     // BWR output bytes of a raw-DD C5 chunk: 17 + 9 + 65536
#ifndef TDBG_RAW_JU
#define TDBG_RAW_JU 128
#endif
constexpr uint32_t JU = TDBG_RAW_JU; // output units per job (128, or 256: 1 KiB plane ranges)
static_assert(JU == 128 || JU == 256, "job size");
constexpr uint32_t NJOB = 1024 / JU; // jobs per wave and tile
constexpr uint32_t NU = JU / 64;     // output units per lane and job
constexpr uint32_t RU = JU / 4 + 1;  // 16-B DMA units per job plane (4 JU bytes at any alignment)
constexpr uint32_t ND = (RU + 63) / 64;  // DMA instructions per job plane
constexpr uint32_t RW = (RU + 1) * 4;  // dwords per job plane region (+1 unit: reads past the range)
#ifndef TDBG_RAW_NB
#define TDBG_RAW_NB 2
#endif
constexpr int NB = TDBG_RAW_NB;      // job buffers per wave (2 or 3)
static_assert(NB == 2 || NB == 3, "job buffers");

struct Lds {
  uint32_t PF[PFU * 4];
  uint2 TAB[NS][TABN];         // {image offset of the window's data | kind << 20, window minimum}
  uint32_t J[NWV][NB][4][RW];  // per wave, buffer and plane: the job's compressed plane bytes
  uint32_t hd[NS][4];          // published by the parse: verdict, log2(window bytes), nwin - 1
};

// bytes [o, o + 4) of a dword array (any alignment)
__device__ __forceinline__ uint32_t rd32(const uint32_t* a, uint32_t o) {
  return __builtin_amdgcn_alignbyte(a[(o >> 2) + 1], a[o >> 2], o & 3);
}

template <bool SGN>
__device__ __forceinline__ uint32_t ext(uint32_t x, uint32_t o, uint32_t w) {
  return SGN ? (uint32_t)__builtin_amdgcn_sbfe((int32_t)x, o, w) : __builtin_amdgcn_ubfe(x, o, w);
}

// ---------------------------------------------------------------------------
// the workgroup's walk over the tiles it owns (fs > SMALL), 64 descriptors at a time
// ---------------------------------------------------------------------------
struct Walk {
  Batch bt;
  uint64_t mine;  // bit i: the batch's i-th tile is ours
  uint64_t base;  // batch index * 64
  uint64_t ntl;
  bool loaded;
};

__device__ __forceinline__ void walk_load(const KParams& kp, Walk& w) {
  w.bt = batch_load(kp, w.base, w.ntl);
  const uint64_t j = blockIdx.x + (w.base + (threadIdx.x & 63)) * (uint64_t)gridDim.x;
  w.mine = __builtin_amdgcn_ballot_w64(j < w.ntl && w.bt.fs > SMALL);
  w.loaded = true;
}

// next owned tile at or after iteration `it`; returns false at the end
__device__ __forceinline__ bool walk_next(const KParams& kp, Walk& w, uint64_t& it, Desc& d) {
  for (;;) {
    if (it >= w.base + 64) {
      w.base = it - it % 64;
      w.loaded = false;
    }
    if (blockIdx.x + w.base * (uint64_t)gridDim.x >= w.ntl) return false;
    if (!w.loaded) walk_load(kp, w);
    const uint64_t m = w.mine & (~0ull << (it - w.base));
    if (m) {
      const uint32_t k = (uint32_t)__builtin_ctzll(m);
      it = w.base + k;
      d = batch_get(w.bt, k, blockIdx.x + it * (uint64_t)gridDim.x);
      return true;
    }
    it = w.base + 64;
  }
}

// the tile's shape is the one this kernel decodes (descriptor checks only)
__device__ __forceinline__ bool takes(const KParams& kp, const Desc& d) {
  return !(kp.flags & TDBG_TILE_OFFSETS) && d.os == OUTB && (((uintptr_t)d.out) & 15) == 0 &&
         d.fs != 0xffffffffu;
}

// decline: the fused kernel runs on the queue after this launch
__device__ __forceinline__ void decline(const KParams& kp, uint64_t t) {
  if (threadIdx.x == 0) {
    const uint32_t k = atomicAdd(kp.sq, 1u);
    if (k < kp.sq_cap) kp.sq[1 + k] = (uint32_t)t;
    else if (kp.status) kp.status[kp.chunks ? kp.chunks[t].tile : t] = TDBG_E_INTERNAL;
  }
}

// prefix DMA: wave w < 3 moves units [64 w, 64 w + 64) of the image's first
// 3 KiB (the image is > SMALL bytes, so all 192 units lie inside it: one
// instruction per wave, every lane active).  The parse reads no byte past
// m + ml + 28 <= 35 + 8 + 9 * 320 + 24 + 28 < 3 KiB - 16 (nwin <= TABN), so
// the rest of PF may hold the last tile's bytes; staging only what the parse
// reads keeps the re-read of window 0's data (the jobs DMA it again) small.
// (PW: the parser wave issues all three, so its own vmcnt covers the prefix)
__device__ __forceinline__ void prefix_dma(Lds& L, const Desc& d, uint32_t w, uint32_t l) {
  const uint64_t a0 = (uint64_t)d.in & ~15ull;
  if constexpr (PW) {
#pragma unroll
    for (uint32_t k = 0; k < 3; k++) dma16(a0 + 16ull * (64 * k + l), lds_addr(L.PF) + 1024 * k);
  } else {
    if (w < 3) dma16(a0 + 16ull * (64 * w + l), lds_addr(L.PF) + 1024 * w);
  }
}

// ---------------------------------------------------------------------------
// header parse (wave 0): tile/chunk header, window table, frame, DD headers
// ---------------------------------------------------------------------------
template <bool SGN>
__device__ __forceinline__ void parse(Lds& L, const Desc& d, uint32_t l, bool chunked, uint32_t slot) {
  const uint32_t* P = L.PF;
  // the chunk header follows the tile's u64 chunk count, or (chunk mode:
  // a chunk of a multi-chunk tile) starts the image
  const uint32_t ho = chunked ? 0u : 8u;
  const uint32_t b = (uint32_t)((uintptr_t)d.in & 15);
  const uint32_t nlo = rd32(P, b), nhi = rd32(P, b + 4), orig = rd32(P, b + ho), fl = rd32(P, b + ho + 4),
                 ml = rd32(P, b + ho + 8);
  const uint32_t m = b + ho + 12;
  const uint32_t Lb = rd32(P, m), nwr = rd32(P, m + 4);
  bool ok = (chunked || (nlo == 1 && nhi == 0)) && orig == OUTB && (uint64_t)ml + fl + ho + 12 <= d.fs && nwr >= 2 &&
            nwr <= TABN &&
            ml == 8 + 9 * nwr + 24 && Lb == LBWR;
  const uint32_t nwin = ok ? nwr : 2;
  // lane l: windows 5l..5l+4 = 45 bytes at e0 (inside PF: m + 8 + 9 * 320 < 4096 - 64)
  const uint32_t e0 = m + 8 + 45 * l;
  uint32_t E[12];
#pragma unroll
  for (int k = 0; k < 12; k++) E[k] = rd32(P, e0 + 4 * k);
  auto byte_at = [&](int o) -> uint32_t { return (E[o >> 2] >> (8 * (o & 3))) & 0xffu; };
  auto dw_at = [&](int o) -> uint32_t {
    return (o & 3) ? __builtin_amdgcn_alignbyte(E[(o >> 2) + 1], E[o >> 2], o & 3) : E[o >> 2];
  };
  const uint32_t ws = __builtin_amdgcn_readfirstlane(dw_at(5));  // window 0's byte count
  ok = ok && ws >= 256 && ws <= 4096 && (ws & (ws - 1)) == 0 && (Lb - 1) / ws + 1 == nwin;
  uint32_t cs[5], kind[5], mn[5];
  bool bad = false;
#pragma unroll
  for (int q = 0; q < 5; q++) {
    const uint32_t wi = 5 * l + q;
    const uint32_t vmin = dw_at(9 * q), bits = byte_at(9 * q + 4), nb = dw_at(9 * q + 5);
    const bool in = wi < nwin;
    const uint32_t want = wi + 1 < nwin ? ws : Lb - ws * (nwin - 1);
    bad |= in && nb != want;
    const bool raw = bits >= 32 || (nb & 3) != 0;
    bad |= in && !raw && bits != 8 && bits != 16;
    kind[q] = raw ? 2 : bits == 8 ? 0 : 1;
    cs[q] = !in ? 0 : raw ? nb : bits == 8 ? nb >> 2 : nb >> 1;
    mn[q] = raw ? 0 : vmin;
  }
  const uint32_t s5 = cs[0] + cs[1] + cs[2] + cs[3] + cs[4];
  const uint32_t inc = wave_incscan_u32(s5);
  ok = ok && !__builtin_amdgcn_ballot_w64(bad) && __builtin_amdgcn_readlane(inc, 63) == fl;
  const uint32_t dst = ho + 12 + ml;  // image offset of the BWR data
  {
    uint32_t off = dst + inc - s5;
#pragma unroll
    for (int q = 0; q < 5; q++) {
      const uint32_t wi = 5 * l + q;
      if (wi < nwin) L.TAB[slot][wi] = make_uint2(off | (kind[q] << 20), mn[q]);
      off += cs[q];
    }
  }
  // compression frame md (compression_filter.cc:413-486): 1 md part of 8 B
  // (the byteshuffle header) compressed to 17 B, 1 data part of 65,536 B
  // compressed to 9 + 65,536 B (raw DoubleDelta)
  const uint32_t f = m + 8 + 9 * nwin;
  ok = ok && rd32(P, f) == 1 && rd32(P, f + 4) == 1 && rd32(P, f + 8) == 8 && rd32(P, f + 12) == 17 &&
       rd32(P, f + 16) == OUTB && rd32(P, f + 20) == 9 + OUTB;
  // DD headers = BWR-output bytes [0, 26): elements 0..6 of window 0 (lane e
  // decodes element e; window 0 lies in the prefix: dst + 28 <= m + ml + 28 < 4096 - 16)
  const uint32_t k0 = __builtin_amdgcn_readfirstlane(kind[0]), mn0 = __builtin_amdgcn_readfirstlane(mn[0]);
  const uint32_t e = l < 7 ? l : 6;
  uint32_t v;
  if (k0 == 2) v = rd32(P, b + dst + 4 * e);
  else if (k0 == 0) v = ext<SGN>(rd32(P, b + dst + e), 0, 8) + mn0;
  else v = ext<SGN>(rd32(P, b + dst + 2 * e), 0, 16) + mn0;
  auto dw = [&](int k) -> uint32_t { return __builtin_amdgcn_readlane(v, k); };
  auto at = [&](int o) -> uint32_t { return __builtin_amdgcn_alignbyte(dw((o >> 2) + 1), dw(o >> 2), o & 3); };
  // c0 = [u8 bitsize][u64 n = 2][1][65536] (any bitsize: two values, or the
  // same 8 bytes copied raw); c1 = [u8 bitsize >= 31][u64 16384] + raw values
  ok = ok && at(1) == 2 && at(5) == 0 && at(9) == 1 && at(13) == OUTB && (at(17) & 0xffu) >= 31 &&
       at(18) == OUTB / 4 && at(22) == 0;
  if (l == 0) {
    L.hd[slot][0] = ok ? 1u : 0u;
    L.hd[slot][1] = 31 - __builtin_clz(ws);
    L.hd[slot][2] = nwin - 1;
  }
}

// ---------------------------------------------------------------------------
// jobs
// ---------------------------------------------------------------------------
constexpr uint32_t OFFM = (1u << 20) - 1;

// compressed image offset of BWR-output byte q in the window starting at
// wstart with table word tx (start of q's element for 8/16-bit windows; its
// end when `end`)
__device__ __forceinline__ uint32_t cpos(uint32_t tx, uint32_t wstart, uint32_t q, bool end) {
  const uint32_t kind = tx >> 20, off = tx & OFFM, dq = q - wstart;
  if (kind == 2) return off + dq + (end ? 1 : 0);
  const uint32_t el = dq >> 2;
  return off + ((el + (end ? 1 : 0)) << kind);
}

// The jobs of one wave and tile: 8 jobs x 4 planes, job i plane k covering
// BWR-output bytes [Q0, Q0 + 512), Q0 = 26 + 16384 k + 4 (1024 w + 128 i).
// Lane 4 i + k computes that plane range's setup once per tile, in vector
// registers: the kernel would otherwise be bound by the CU's one scalar
// unit (~50 scalar instructions per plane range).  A job reads its values
// back with v_readlane.
struct Setup {
  uint32_t g0lo, g0hi;  // 16-B aligned global address of the range's first compressed unit
  uint32_t nu;          // DMA units (1..RU)
  uint32_t rel;         // LDS byte offset, in the plane's region, of the compressed byte of Q0
  uint32_t rb;          // image offset of the region's first byte
  uint64_t k8, gen;     // ballots: bit 4i+k = plane range all 8-bit windows / needs the general decoder
};

template <int ABL>
__device__ __forceinline__ Setup wave_setup(const uint2* TAB, const Desc& d, uint32_t w, uint32_t wsh, uint32_t l) {
  const uint32_t i = (l >> 2) % NJOB, k = l & 3;
  const uint32_t Q0 = 26 + 16384 * k + 4 * (1024 * w + JU * i);
  const uint32_t W0 = Q0 >> wsh, W1 = (Q0 + 4 * JU - 1) >> wsh;  // W1 - W0 <= 4 JU / 256 (windows >= 256 B)
  const uint32_t xA = TAB[W0].x, xL = TAB[W1].x;
  bool all8 = (xA >> 20) == 0 && (xL >> 20) == 0, allraw = (xA >> 20) == 2 && (xL >> 20) == 2;
#pragma unroll
  for (uint32_t q = 1; q < 4 * JU / 256; q++) {
    const uint32_t kq = TAB[W0 + q < W1 ? W0 + q : W1].x >> 20;
    all8 = all8 && kq == 0;
    allraw = allraw && kq == 2;
  }
  Setup st;
  const bool mine = l < 4 * NJOB;
  st.k8 = __builtin_amdgcn_ballot_w64(mine && all8);
  st.gen = __builtin_amdgcn_ballot_w64(mine && !all8 && !allraw);
  const uint32_t c0 = cpos(xA, W0 << wsh, Q0, false);
  const uint32_t c1 = cpos(xL, W1 << wsh, Q0 + 4 * JU - 1, true);
  const uint64_t g0 = ((uint64_t)d.in + c0) & ~15ull;
  st.nu = ABL == 2 ? 1u : (uint32_t)(((((uint64_t)d.in + c1 + 15) & ~15ull) - g0) >> 4);
  st.g0lo = (uint32_t)g0;
  st.g0hi = (uint32_t)(g0 >> 32);
  st.rb = (uint32_t)(g0 - (uint64_t)d.in);  // >= 5: c0 >= 20
  st.rel = c0 - st.rb;
  return st;
}

// One job's uniform values, read back from the setup lanes.
struct Job {
  uint32_t rel[4], rb[4];
  uint32_t k8, gen;  // 4-bit plane masks
};

// the job's planes: LDS-DMA of each plane range into its region (lanes <
// nu; at least one unit, so every instruction is issued) and its values
__device__ __forceinline__ Job job_dma(const Setup& st, uint32_t i, uint32_t R0, uint32_t l) {
  Job jb;
  jb.k8 = (uint32_t)(st.k8 >> (4 * i)) & 15u;
  jb.gen = (uint32_t)(st.gen >> (4 * i)) & 15u;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t s = 4 * i + k;
    const uint32_t nu = __builtin_amdgcn_readlane(st.nu, s);
    const uint64_t g0 = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(st.g0hi, s) << 32) |
                        (uint32_t)__builtin_amdgcn_readlane(st.g0lo, s);
    jb.rel[k] = __builtin_amdgcn_readlane(st.rel, s);
    jb.rb[k] = __builtin_amdgcn_readlane(st.rb, s);
    if (l < nu) dma16(g0 + 16ull * l, R0 + k * (RW * 4));
    // (JU 256: units 64.. by a second instruction, always issued -- the
    // counted waits assume ND per plane; with nu <= 64 lane 0 moves unit 0
    // again into slot 64, which nothing reads)
    if constexpr (ND > 1)
      if (l < (nu > 64 ? nu - 64 : 1u)) dma16(nu > 64 ? g0 + 16ull * (64 + l) : g0, R0 + k * (RW * 4) + 1024);
  }
  return jb;
}

// General decoder (mixed or 16-bit windows): the BWR-output dword at bytes
// [Q0 + 4 v, +4) = the upper half of element e = (Q0 + 4 v) / 4 and the
// lower half of e + 1 (Q0 = 2 mod 4), each looked up in the window table.
template <bool SGN>
__device__ __forceinline__ uint32_t dword_general(const uint2* TAB, const uint32_t* R, uint32_t rb, uint32_t Q0,
                                                  uint32_t v, uint32_t esh) {
  const uint32_t e = (Q0 >> 2) + v;
  uint32_t val[2];
#pragma unroll
  for (int i = 0; i < 2; i++) {
    const uint32_t ei = e + i, wi = ei >> esh;
    const uint2 te = TAB[wi];
    const uint32_t kind = te.x >> 20;
    const uint32_t o = (te.x & OFFM) + ((ei - (wi << esh)) << kind) - rb;
    const uint32_t x = rd32(R, o);
    val[i] = kind == 2 ? x : (kind == 0 ? ext<SGN>(x, 0, 8) : ext<SGN>(x, 0, 16)) + te.y;
  }
  return __builtin_amdgcn_perm(val[1], val[0], 0x05040302u);
}

// Byteshuffle⁻¹ of one output unit from dword j of the four planes: out
// dword b, byte k = plane k's byte b
__device__ __forceinline__ v4u unshuffle4(const uint32_t (&x)[4]) {
  const uint32_t t0 = __builtin_amdgcn_perm(x[1], x[0], 0x05010400u);
  const uint32_t t1 = __builtin_amdgcn_perm(x[1], x[0], 0x07030602u);
  const uint32_t t2 = __builtin_amdgcn_perm(x[3], x[2], 0x05010400u);
  const uint32_t t3 = __builtin_amdgcn_perm(x[3], x[2], 0x07030602u);
  return v4u{__builtin_amdgcn_perm(t2, t0, 0x05040100u), __builtin_amdgcn_perm(t2, t0, 0x07060302u),
             __builtin_amdgcn_perm(t3, t1, 0x05040100u), __builtin_amdgcn_perm(t3, t1, 0x07060302u)};
}

// The four planes' dwords of units J + v (v = 64 u + l, u = 0, 1) of a job
// whose planes are all-raw (bit k of K8 clear) or all-8-bit (set): every LDS
// read is issued first (data dwords; for 8-bit planes also the two
// elements' window minima), then one wait, then the arithmetic.  Raw planes:
// the dword is the compressed dword at rel + 4 v.  8-bit planes (full
// windows, so one compressed byte per element in order): elements e and
// e + 1 are the bytes at rel + v and rel + v + 1.
template <bool SGN, int K8>
__device__ __forceinline__ void job_fast(const uint2* TAB, const Job& jb, const uint32_t* R0, uint32_t J, uint32_t esh,
                                         uint32_t l, uint32_t (&x)[NU][4]) {
  uint32_t lo[NU][4], hi[NU][4], ma[NU][4], mb[NU][4];
#pragma unroll
  for (int u = 0; u < (int)NU; u++)
#pragma unroll
    for (int k = 0; k < 4; k++) {
      constexpr int dummy = 0;
      (void)dummy;
      const bool b8 = (K8 >> k) & 1;
      const uint32_t v = 64 * u + l;
      const uint32_t o = jb.rel[k] + (b8 ? v : 4 * v);
      const uint32_t* R = R0 + k * RW;
      lo[u][k] = R[o >> 2];
      hi[u][k] = R[(o >> 2) + 1];
      if (b8) {
        const uint32_t e = ((26 + 16384 * k + 4 * J) >> 2) + v;
        ma[u][k] = TAB[e >> esh].y;
        mb[u][k] = TAB[(e + 1) >> esh].y;
      }
    }
#pragma unroll
  for (int u = 0; u < (int)NU; u++)
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const bool b8 = (K8 >> k) & 1;
      const uint32_t v = 64 * u + l;
      if (b8) {
        const uint32_t y = __builtin_amdgcn_alignbyte(hi[u][k], lo[u][k], (jb.rel[k] + v) & 3);
        const uint32_t v0 = ext<SGN>(y, 0, 8) + ma[u][k], v1 = ext<SGN>(y, 8, 8) + mb[u][k];
        x[u][k] = __builtin_amdgcn_perm(v1, v0, 0x05040302u);
      } else {
        x[u][k] = __builtin_amdgcn_alignbyte(hi[u][k], lo[u][k], jb.rel[k] & 3);
      }
    }
}

// VMEM operations a wave has issued after job i's DMA when job i waits
// (issue order: D_0 .. D_{NB-1}, then per job i: its compute, D_{i+NB},
// its stores S_i; D = 4 ND DMA instructions, S = NU stores): the D_k with
// i < k <= min(i + NB - 1, NJOB - 1), and the S_j with i - NB <= j < i.
constexpr uint32_t vm_after(uint32_t i) {
  return 4 * ND * ((i + NB - 1 < NJOB - 1 ? i + NB - 1 : NJOB - 1) - i) + NU * (i < (uint32_t)NB ? i : (uint32_t)NB);
}

// s_waitcnt vmcnt(n) for the counts vm_after takes (n uniform)
__device__ __forceinline__ void vm_wait(uint32_t n) {
  switch (n) {
#define TDBG_VMW(c) \
  case c: asm volatile("s_waitcnt vmcnt(" #c ")" ::: "memory"); break;
    TDBG_VMW(4) TDBG_VMW(6) TDBG_VMW(8) TDBG_VMW(10) TDBG_VMW(12) TDBG_VMW(14) TDBG_VMW(16) TDBG_VMW(20)
    TDBG_VMW(24)
#undef TDBG_VMW
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}
constexpr bool vm_case(uint32_t n) { return n == 4 || n == 6 || (n >= 8 && n <= 16 && n % 2 == 0) || n == 20 || n == 24; }
constexpr bool vm_cases_ok() {
  for (uint32_t i = 0; i < NJOB; i++)
    if (!vm_case(vm_after(i))) return false;
  return true;
}
static_assert(vm_cases_ok(), "vm_wait cases");

// The wave's 1,024 output units of one tile, in NJOB jobs of JU units, NB
// job buffers in a ring: job i waits until only the operations issued after
// its DMA are left (vm_after; NB = 2: 4, 6, 8 x 5, 4).  No other VMEM
// instruction is issued meanwhile (no scratch: the build's resource check
// keeps ScratchSize at 0).
template <bool SGN, int ABL>
__device__ __forceinline__ void tile_jobs(Lds& L, const Desc& d, uint32_t w, uint32_t l, uint32_t wsh, uint32_t slot) {
  const uint2* TAB = L.TAB[slot];
  const uint32_t esh = wsh - 2;
  const uint32_t rbase = lds_addr(&L.J[w][0][0][0]);
  constexpr uint32_t RB = 4 * RW * 4;  // bytes per job buffer
  const Setup st = wave_setup<ABL>(TAB, d, w, wsh, l);
  Job jc = job_dma(st, 0, rbase, l);
  Job jn = job_dma(st, 1, rbase + RB, l);
  Job jn2 = jn;
  if constexpr (NB == 3) jn2 = job_dma(st, 2, rbase + 2 * RB, l);
  for (uint32_t i = 0; i < NJOB; i++) {
    const uint32_t buf = i % NB;
    const uint32_t J = 1024 * w + JU * i;
    vm_wait(vm_after(i));
    const uint32_t* R0 = &L.J[w][buf][0][0];
    uint32_t x[NU][4];
    if (jc.gen == 0) {
      switch (jc.k8) {
#define TDBG_K8(m) \
  case m: job_fast<SGN, m>(TAB, jc, R0, J, esh, l, x); break;
        TDBG_K8(0) TDBG_K8(1) TDBG_K8(2) TDBG_K8(3) TDBG_K8(4) TDBG_K8(5) TDBG_K8(6) TDBG_K8(7)
        TDBG_K8(8) TDBG_K8(9) TDBG_K8(10) TDBG_K8(11) TDBG_K8(12) TDBG_K8(13) TDBG_K8(14) TDBG_K8(15)
#undef TDBG_K8
        default: break;
      }
    } else {
#pragma unroll
      for (int u = 0; u < (int)NU; u++)
#pragma unroll
        for (int k = 0; k < 4; k++)
          x[u][k] = dword_general<SGN>(TAB, R0 + k * RW, jc.rb[k], 26 + 16384 * k + 4 * J, 64 * u + l, esh);
    }
    v4u y[NU];
#pragma unroll
    for (int u = 0; u < (int)NU; u++) y[u] = unshuffle4(x[u]);
    // the buffer's reads are consumed: job i + NB's DMA may overwrite it
    Job jw = jc;
    if (i + NB < NJOB) jw = job_dma(st, i + NB, rbase + buf * RB, l);
#pragma unroll
    for (int u = 0; u < (int)NU; u++) {
      g_u4* dst = (g_u4*)(d.out + 16u * (J + 64 * u + l));
      if (ABL == 3) {  // timing ablation: stores issued only under a branch never taken (vmcnt counts off: ABL only)
        if (y[u].x == 0x9e3779b9u && y[u].y == 0x7f4a7c15u) __builtin_nontemporal_store(y[u], dst);
      } else {
        __builtin_nontemporal_store(y[u], dst);
      }
    }
    jc = jn;
    if constexpr (NB == 3) {
      jn = jn2;
      jn2 = jw;
    } else {
      jn = jw;
    }
  }
}

#ifndef TDBG_RAW_OCC
#if TDBG_RAW_PW || TDBG_RAW_JU > 128
#define TDBG_RAW_OCC 4  // workgroups per CU (PW: 5 waves each at <= 96 VGPRs; JU 256: 40 KB LDS)
#else
#define TDBG_RAW_OCC 5  // workgroups per CU (<= 96 VGPRs, 24 KB LDS each)
#endif
#endif

// ABL: timing ablations (outputs not meaningful): 1 parse only a workgroup's
// first tile (identical rand tiles), 2 one DMA unit per job plane, 3 no
// stores, 4 no jobs (walk, prefix, parse and barriers only)
template <bool SGN, int ABL>
__global__ void __launch_bounds__(NT, TDBG_RAW_OCC) unfilter_stream_raw_kernel(const KParams kp) {
  __shared__ Lds L;
  const uint32_t w = wave_(), l = lane_();
  Walk wk{};
  wk.ntl = work_items(kp);
  const bool chunked = kp.chunks != nullptr;
  wk.base = 0;
  wk.loaded = false;
  uint64_t it = 0;
  uint64_t ok_tiles = 0;
  Desc cur{};
  bool have = false;
  // the first tile this workgroup decodes (declining the others on the way)
  while (walk_next(kp, wk, it, cur)) {
    it++;
    if (takes(kp, cur)) {
      have = true;
      break;
    }
    decline(kp, cur.t);
  }
  if constexpr (PW) {
    // the parser wave (w == NWV) is one tile ahead: tile n + 1's prefix DMA
    // and parse (into the other window-table slot) run while the job waves
    // decode tile n; one barrier per tile publishes the slot and frees the
    // one just used
    const bool parser = w == NWV;
    uint32_t slot = 0;
    if (have && parser) {
      prefix_dma(L, cur, w, l);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      parse<SGN>(L, cur, l, chunked, 0);
    }
    lds_barrier();
    while (have) {
      Desc nxt{};
      bool hn = false;
      while (walk_next(kp, wk, it, nxt)) {
        it++;
        if (takes(kp, nxt)) {
          hn = true;
          break;
        }
        decline(kp, nxt.t);
      }
      if (parser) {
        if (hn) {
          prefix_dma(L, nxt, w, l);  // PF: only this wave reads it, and its last parse is done
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          parse<SGN>(L, nxt, l, chunked, slot ^ 1);
        }
      } else {
        const bool ok = __builtin_amdgcn_readfirstlane(L.hd[slot][0]) != 0;
        const uint32_t wsh = __builtin_amdgcn_readfirstlane(L.hd[slot][1]);
        if (ok) {
          if (ABL != 4) tile_jobs<SGN, ABL>(L, cur, w, l, wsh, slot);
          ok_tiles++;
          if (threadIdx.x == 0 && kp.status && !chunked) kp.status[cur.t] = TDBG_OK;
        } else {
          decline(kp, cur.t);
        }
      }
      lds_barrier();
      slot ^= 1;
      cur = nxt;
      have = hn;
    }
    have = false;  // (the two-barrier loop below is not taken)
  }
  if (have) prefix_dma(L, cur, w, l);
  bool pf_waited = false;
  while (have) {
    // the next tile to prefetch
    Desc nxt{};
    bool hn = false;
    while (walk_next(kp, wk, it, nxt)) {
      it++;
      if (takes(kp, nxt)) {
        hn = true;
        break;
      }
      decline(kp, nxt.t);
    }
    if (ABL != 1 || ok_tiles == 0) {
      if (!pf_waited) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      lds_barrier();  // B1: the prefix has landed; the last tile's jobs are done with TAB
      if (w == 0) parse<SGN>(L, cur, l, chunked, 0);
      lds_barrier();  // B2: window table and verdict
    }
    const bool ok = __builtin_amdgcn_readfirstlane(L.hd[0][0]) != 0;
    const uint32_t wsh = __builtin_amdgcn_readfirstlane(L.hd[0][1]);
    // PF is free (only wave 0 read it, before B2): the next tile's prefix
    if (hn && ABL != 1) prefix_dma(L, nxt, w, l);
    pf_waited = false;
    if (ok) {
      if (ABL != 4) tile_jobs<SGN, ABL>(L, cur, w, l, wsh, 0);
      pf_waited = true;  // the first job's wait covered the prefix (older)
      ok_tiles++;
      if (threadIdx.x == 0 && kp.status && !chunked) kp.status[cur.t] = TDBG_OK;
    } else {
      decline(kp, cur.t);
    }
    cur = nxt;
    have = hn;
  }
  if (kp.stats && threadIdx.x == 0 && ok_tiles && chunked) {
    atomicAdd((unsigned long long*)&kp.stats[TDBG_STAT_STREAM_CHUNKS], (unsigned long long)ok_tiles);
  } else if (kp.stats && threadIdx.x == 0 && ok_tiles) {
    atomicAdd((unsigned long long*)&kp.stats[TDBG_STAT_FUSED_TILES], (unsigned long long)ok_tiles);
    atomicAdd((unsigned long long*)&kp.stats[TDBG_STAT_FUSED_BYTES], (unsigned long long)(ok_tiles * OUTB));
    atomicAdd((unsigned long long*)&kp.stats[TDBG_STAT_STREAM_TILES], (unsigned long long)ok_tiles);
    atomicAdd((unsigned long long*)&kp.stats[TDBG_STAT_STREAM_RAW_TILES], (unsigned long long)ok_tiles);
  }
}

}  // namespace sraw
}  // namespace tdbg

extern "C" uint32_t tdbg_stream_raw_grid(int cus) {
  static const int g = tdbg_hook("TDBG_RAW_GRID") ? atoi(tdbg_hook("TDBG_RAW_GRID")) : 0;  // experiments
  return g > 0 ? (uint32_t)g : (uint32_t)cus * TDBG_RAW_OCC;
}

extern "C" hipError_t tdbg_launch_stream_raw(const tdbg::KParams* kp, uint32_t grid, int sgn, hipStream_t s) {
  using namespace tdbg::sraw;
  static const int abl = tdbg_hook("TDBG_RAW_ABL") ? atoi(tdbg_hook("TDBG_RAW_ABL")) : 0;
  auto k = sgn ? (abl == 1   ? unfilter_stream_raw_kernel<true, 1>
                  : abl == 2 ? unfilter_stream_raw_kernel<true, 2>
                  : abl == 3 ? unfilter_stream_raw_kernel<true, 3>
                  : abl == 4 ? unfilter_stream_raw_kernel<true, 4>
                             : unfilter_stream_raw_kernel<true, 0>)
               : unfilter_stream_raw_kernel<false, 0>;
  TDBG_LAUNCH(k, dim3(grid), dim3(NT), s, *kp);
  return hipGetLastError();
}
