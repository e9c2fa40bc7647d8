// tdbg_forward_small.hip -- forward ("filter") direction of the scan
// configs' pipelines on 8-byte values, one 64 KiB tile = one
// chunk (WriterBase::filter_tile -> FilterPipeline::run_forward,
// writer_base.cc:870-915, filter_pipeline.cc:208-369), gfx950:
//
//   MODE 0  C3a [DOUBLE_DELTA] (dd_compressor.cc:211-312, 406-450)
//   MODE 1  C3b [RLE], 8-byte cells (rle_compressor.cc:51-101)
//   MODE 2  C4  [POSITIVE_DELTA(1024), BIT_WIDTH_REDUCTION(256)] on uint64
//           (positive_delta_filter.cc:140-245, bit_width_reduction_filter.cc:
//           110-280, 406-447)
//
// The general forward kernel (tdbg_forward.hip) runs these through a global
// scratch slot one byte at a time.  Here a 256-thread workgroup owns a
// tile: thread T holds values 32T..32T+31 (and the two before) in
// registers, one workgroup reduction decides the tile's shape (DD: the bit
// size; RLE: the run heads), the compressed stream is built in LDS next to
// the tile header and the compression frame, and the whole filtered tile
// leaves with lane-consecutive 16-B stores.
//
// Filtered tile (one chunk): [u64 1] [u32 65536][u32 cl][u32 16] (chunk
// header, filter_pipeline.cc:332-363) [u32 0][u32 1][u32 65536][u32 cl]
// (compression frame: 0 metadata parts, 1 data part,
// compression_filter.cc:240-301) then the compressed part of cl bytes:
//   DD:  [u8 bitsize][u64 8192][u64 x0][u64 x1] + ceil(8190 (bitsize+1) / 64)
//        u64 words of codes (a sign bit, then bitsize magnitude bits, MSB
//        first from bit 63 of each little-endian word)
//   RLE: nr records [u64 value][u8 len >> 8][u8 len & 255]
// C4's chunk has no compression frame: [u32 65536][u32 dn][u32 4108], md =
// BWR md [u32 65536][u32 256] + 256 x [u64 min][u8 bits][u32 256] then PD md
// [u32 64] + 64 x [u64 first][u32 1024] (each filter prepends its md,
// filter_buffer.cc), data = the BWR-compressed deltas.  Thread T's 32 values
// are exactly BWR window T, and PD window p is threads 4p..4p+3.
//
// Tiles of any other shape (sizes, alignments, capacity), and those whose
// result this kernel does not build (DD: values that could overflow the
// checked arithmetic, |v| >= 2^61, or bit sizes above 30; RLE: more than
// RMAX runs; C4: a decreasing value, the reference's error, or data beyond
// the LDS image) are queued (KParams::fbq) for the general forward kernel,
// which runs on the queue right after, so every status and byte stays the
// oracle's (tests/test_gpu_forward.py).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/tiledb_amd.h"
#include "tdbg_desc.h"
#include "tdbg_device.h"

namespace tdbg {
namespace fsm {

constexpr int NT = 256;
constexpr int NWV = NT / 64;
constexpr uint32_t NV = 8192;   // 8-byte values per tile
constexpr uint32_t TB = NV * 8; // tile bytes
constexpr uint32_t HDR = 36;    // tile + chunk header + compression frame
// DD: the image starts at LDS byte 3, so DD-output byte 25 (image byte 61,
// the first code word) is LDS byte 64: dword-aligned words
constexpr uint32_t IB_DD = 3;
constexpr uint32_t WD0 = (IB_DD + HDR + 25) / 4;  // LDS dword of code word 0's first half
constexpr uint32_t CBMAX = 31;
constexpr uint32_t WORDS_MAX = ((NV - 2) * CBMAX + 63) / 64;
// RLE: the image starts at LDS byte 4 (records at 40 + 10 r: 2-byte aligned)
constexpr uint32_t IB_RLE = 4;
constexpr uint32_t RMAX = 2048;  // runs per tile taken here (20 KB of records)
constexpr uint32_t BDW = WD0 + 2 * WORDS_MAX + 8;  // image dwords (+ the store loop's read-ahead)
static_assert(IB_RLE + HDR + 10 * RMAX + 32 <= 4 * BDW, "RLE image fits");
// C4: image at LDS byte 0; md 4,108 B; data from 4,128 (dword-aligned)
constexpr uint32_t ML_C4 = 8 + 256 * 13 + 4 + 64 * 12;
constexpr uint32_t D0_C4 = 20 + ML_C4;
constexpr uint32_t DMAX_C4 = 4 * BDW - D0_C4 - 32;  // data bytes taken here
static_assert(ML_C4 == 4108 && D0_C4 % 4 == 0, "C4 layout");
static_assert(WD0 % 4 == 0, "16-B zeroing of the code words");

struct Lds {
  uint32_t B[BDW];
  uint16_t H[RMAX + 2];  // RLE: run head positions, H[nr] = 8192
  uint64_t red[NWV];
  uint32_t cnt[NWV];
};

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const v4u g_cu4;
typedef __attribute__((address_space(1))) v4u g_u4;

__device__ __forceinline__ void lds_u8(Lds& L, uint32_t o, uint32_t v) { ((uint8_t*)L.B)[o] = (uint8_t)v; }
__device__ __forceinline__ void lds_u32b(Lds& L, uint32_t o, uint32_t v) {
#pragma unroll
  for (int i = 0; i < 4; i++) lds_u8(L, o + i, v >> (8 * i));
}

template <int CTRL>
__device__ __forceinline__ uint32_t dpp_(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, false);
}
// maximum over the wave (every lane of a 16-lane row first, then the rows)
__device__ __forceinline__ uint64_t wave_max64(uint64_t v) {
  auto step = [&](uint64_t o) { v = o > v ? o : v; };
  step(((uint64_t)dpp_<0xB1>((uint32_t)(v >> 32)) << 32) | dpp_<0xB1>((uint32_t)v));
  step(((uint64_t)dpp_<0x4E>((uint32_t)(v >> 32)) << 32) | dpp_<0x4E>((uint32_t)v));
  step(((uint64_t)dpp_<0x141>((uint32_t)(v >> 32)) << 32) | dpp_<0x141>((uint32_t)v));
  step(((uint64_t)dpp_<0x140>((uint32_t)(v >> 32)) << 32) | dpp_<0x140>((uint32_t)v));
  uint64_t m = 0;
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const uint64_t x = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(v >> 32), 16 * r) << 32) |
                       (uint32_t)__builtin_amdgcn_readlane((uint32_t)v, 16 * r);
    m = x > m ? x : m;
  }
  return m;
}

// The DoubleDelta codes of thread T's positions 32T..32T+31 in four runs of
// 8 (S[2 + i] = low dword of position 32T + i, S[0], S[1] = the two before;
// |dd| < 2^30, so the wrapped 32-bit double delta is exact), at
// compile-time code width CB: a run's 8 codes are packed MSB first at
// compile-time bit positions into 8 run dwords, then shifted to the run's
// stream offset with one v_alignbit per 32-bit chunk.  Stream chunk c is
// LDS dword WD0 + (c ^ 1) (the high half of a little-endian u64 word comes
// first).  Chunks wholly inside a run are plain writes; the first and the
// last one or two, shared with the neighbouring runs, are OR-ed into the
// zeroed region.  Thread 0's first run starts at position 0, which has no
// code, nor has 1: two zero codes at stream bit -2 CB, chunks below 0 not
// written.
template <int CB>
__device__ __forceinline__ void dd_emit(Lds& L, const uint32_t (&S)[34], uint32_t T) {
  constexpr uint32_t BS = CB - 1;
  constexpr int JF = (8 * CB) / 32 - 1;   // chunks 1..JF lie inside a run for any start bit
  constexpr int JX = (8 * CB + 30) / 32;  // the last chunk a run can reach
#pragma unroll
  for (int r = 0; r < 4; r++) {
    uint32_t code[8];
    uint32_t dprev = S[8 * r + 1] - S[8 * r];
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const uint32_t d = S[8 * r + i + 2] - S[8 * r + i + 1];
      const int32_t dd = (int32_t)(d - dprev);
      dprev = d;
      const uint32_t a = (uint32_t)(dd < 0 ? -dd : dd);
      code[i] = (((uint32_t)dd >> 31) << BS) | a;
    }
    if (r == 0) {
      code[0] = T == 0 ? 0u : code[0];
      code[1] = T == 0 ? 0u : code[1];
    }
    uint32_t R[8];
#pragma unroll
    for (int j = 0; j < 8; j++) R[j] = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const int off = j * CB, w0 = off >> 5, sh = off & 31;
      if (sh + CB <= 32) {
        R[w0] |= code[j] << (32 - sh - CB);
      } else {
        R[w0] |= code[j] >> (sh + CB - 32);
        R[w0 + 1] |= code[j] << (64 - sh - CB);
      }
    }
    const int32_t B0 = (32 * (int32_t)T + 8 * r - 2) * CB;  // stream bit of the run's first code
    const int32_t c0 = B0 >> 5;
    const uint32_t nb0 = (uint32_t)B0 & 31u;
    const int32_t base = (int32_t)WD0 + (c0 & ~1);
    const uint32_t par = (uint32_t)c0 & 1u;
    // dword of chunk c0 + j = base + ((j + par) ^ 1)
    uint32_t* const pe = L.B + (base + 1 - (int32_t)par);
    uint32_t* const po = L.B + (base - 1 + 3 * (int32_t)par);
    const int32_t jmax = (int32_t)((8 * CB - 1 + nb0) >> 5);
#pragma unroll
    for (int j = 0; j <= JX; j++) {
      const uint32_t hi = j == 0 ? 0u : R[j - 1], lo = j == 8 ? 0u : R[j];
      const uint32_t ch = __builtin_amdgcn_alignbit(hi, lo, nb0);
      uint32_t* const dst = (j & 1 ? po : pe) + j;
      const bool inside = r != 0 || c0 + j >= 0;
      if (j >= 1 && j <= JF) {
        if (inside) *dst = ch;
      } else if (j <= jmax && inside) {
        atomicOr(dst, ch);
      }
    }
  }
}

// image bytes [S0, S0 + total) of LDS to out, lane-consecutive 16-B units
// (two aligned ds_read_b128 per lane, shifted by the image's start within
// its 16-B unit); the partial last unit byte by byte
__device__ __forceinline__ void store_image(const Lds& L, uint32_t S0, uint32_t total, uint8_t* out, uint32_t T) {
  const uint32_t s16 = S0 & 15, k0 = S0 >> 4, rr = s16 & 3, qd = s16 >> 2;
  const uint32_t nu = (total + 15) >> 4;
  for (uint32_t u = T; u < nu; u += NT) {
    const v4u A = *(const v4u*)(L.B + 4 * (k0 + u)), Bq = *(const v4u*)(L.B + 4 * (k0 + u + 1));
    const uint32_t W8[8] = {A.x, A.y, A.z, A.w, Bq.x, Bq.y, Bq.z, Bq.w};
    v4u y;
    switch (qd) {  // (uniform)
#define TDBG_SH(q)                                                                                   \
  case q:                                                                                            \
    y = v4u{__builtin_amdgcn_alignbyte(W8[q + 1], W8[q], rr), __builtin_amdgcn_alignbyte(W8[q + 2], W8[q + 1], rr), \
            __builtin_amdgcn_alignbyte(W8[q + 3], W8[q + 2], rr), __builtin_amdgcn_alignbyte(W8[q + 4], W8[q + 3], rr)}; \
    break;
      TDBG_SH(0) TDBG_SH(1) TDBG_SH(2) default: TDBG_SH(3)
#undef TDBG_SH
    }
    if (16 * u + 16 <= total) {
      __builtin_nontemporal_store(y, (g_u4*)(out + 16 * u));
    } else {
      const uint32_t yy[4] = {y.x, y.y, y.z, y.w};
      for (uint32_t b = 0; 16 * u + b < total; b++) out[16 * u + b] = (uint8_t)(yy[b >> 2] >> (8 * (b & 3)));
    }
  }
}

// tile header [u64 1][u32 65536][u32 cl][u32 16] and the compression frame
// [u32 0][u32 1][u32 65536][u32 cl] at image offset 0 (LDS byte ib)
__device__ __forceinline__ void write_headers(Lds& L, uint32_t ib, uint32_t cl) {
  lds_u32b(L, ib, 1);
  lds_u32b(L, ib + 4, 0);
  lds_u32b(L, ib + 8, TB);
  lds_u32b(L, ib + 12, cl);
  lds_u32b(L, ib + 16, 16);
  lds_u32b(L, ib + 20, 0);
  lds_u32b(L, ib + 24, 1);
  lds_u32b(L, ib + 28, TB);
  lds_u32b(L, ib + 32, cl);
}

// (C4's 32 deltas and their window packing need more than 128 VGPRs: three
// workgroups per CU there, four for C3a / C3b)
template <int MODE, bool SGN>
__global__ void __launch_bounds__(NT, MODE == 2 ? 3 : 4) filter_small_kernel(const KParams kp) {
  __shared__ Lds L;
  uint64_t taken = 0;
  // A grid of at least one workgroup per tile (a multiple of 8): one tile per
  // workgroup, dealt so that each XCD (workgroups go round-robin over the 8)
  // takes a contiguous eighth of the tiles; a smaller grid walks the tiles.
  const uint32_t G = gridDim.x;
  const bool np = G >= kp.ntiles && (G & 7) == 0;
  const uint32_t bid = np ? (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3) : blockIdx.x;
  for (uint64_t j = bid; j < kp.ntiles; j += G) {
    // thread index opaque to the optimizer (per-thread index math is
    // tile-invariant; hoisting it pins registers)
    uint32_t T = threadIdx.x;
    asm volatile("" : "+v"(T));
    const uint32_t l = T & 63, w = __builtin_amdgcn_readfirstlane(T >> 6);
    const uint64_t t = j;
    uint8_t* out = kp.out[t];
    const uint64_t cap = kp.out_size[t];
    const bool shape = kp.in_size[t] == TB && (((uintptr_t)kp.in[t]) & 15) == 0 && (((uintptr_t)out) & 15) == 0 &&
                       cap >= 64;
    bool ok = shape;
    __syncthreads();  // B0: the last tile's image is stored (LDS free)
    if (shape) {      // (uniform)
      const g_cu4* src = (const g_cu4*)kp.in[t];
      v4u U[16];
#pragma unroll
      for (int i = 0; i < 16; i++) U[i] = src[16 * T + i];
      const v4u P = T ? src[16 * T - 1] : v4u{0u, 0u, 0u, 0u};  // positions 32T - 2, 32T - 1
      // v[k + 2] = position 32T + k, v[0], v[1] the two before
      uint32_t lo[34], hi[34];
      lo[0] = P.x;
      hi[0] = P.y;
      lo[1] = P.z;
      hi[1] = P.w;
#pragma unroll
      for (int i = 0; i < 16; i++) {
        lo[2 + 2 * i] = U[i].x;
        hi[2 + 2 * i] = U[i].y;
        lo[3 + 2 * i] = U[i].z;
        hi[3 + 2 * i] = U[i].w;
      }
      auto val = [&](int k) -> uint64_t { return ((uint64_t)hi[k] << 32) | lo[k]; };
      if (MODE == 0) {
        // ---- zero the code words (codes are OR-ed in) ----
        for (uint32_t d = WD0 + 4 * T; d < BDW - 4; d += 4 * NT) *(v4u*)(L.B + d) = v4u{0u, 0u, 0u, 0u};
        // ---- bit size (compute_bitsize, dd_compressor.cc:265-311): the
        // first delta and every double delta, in 64 bits; values outside
        // [-2^61, 2^61) (signed) or [0, 2^61) are left to the general kernel
        // (its checked arithmetic decides their status) ----
        uint64_t m = 0;
        bool inr = true;
        uint64_t dprev = val(1) - val(0);
#pragma unroll
        for (int k = 2; k < 34; k++) {
          const uint64_t v = val(k);
          inr = inr && (SGN ? ((v + (1ull << 61)) >> 62) == 0 : (v >> 61) == 0);
          const uint64_t d = v - val(k - 1);
          const int64_t dd = (int64_t)(d - dprev);
          dprev = d;
          uint64_t a = dd < 0 ? 0ull - (uint64_t)dd : (uint64_t)dd;
          if (k < 4) {  // thread 0: position 0 has no delta, position 1 counts its first delta
            const int64_t sd = (int64_t)d;
            const uint64_t ad = sd < 0 ? 0ull - (uint64_t)sd : (uint64_t)sd;
            a = T != 0 ? a : k == 3 ? ad : 0ull;
          }
          m = a > m ? a : m;
        }
        if (!inr) m = ~0ull;
        m = wave_max64(m);
        if (l == 0) L.red[w] = m;
        __syncthreads();  // B1
        m = 0;
#pragma unroll
        for (int v = 0; v < NWV; v++) m = L.red[v] > m ? L.red[v] : m;
        const uint32_t bitsize = m ? 64 - __builtin_clzll(m) : 1;  // do { ++b; m >>= 1; } while (m)
        ok = m < (1ull << 30);  // bit size <= 30: codes of <= 31 bits
        const uint32_t cb = bitsize + 1;
        const uint32_t words = ((NV - 2) * cb + 63) / 64;
        const uint32_t cl = 25 + 8 * words;
        if (ok) {
          if (T == 0) {
            write_headers(L, IB_DD, cl);
            lds_u8(L, IB_DD + HDR, bitsize);
            lds_u32b(L, IB_DD + HDR + 1, NV);
            lds_u32b(L, IB_DD + HDR + 5, 0);
            // x0, x1 at image 45, 53 = LDS bytes 48, 56 (dword-aligned)
            L.B[(IB_DD + HDR + 9) / 4] = lo[2];
            L.B[(IB_DD + HDR + 9) / 4 + 1] = hi[2];
            L.B[(IB_DD + HDR + 17) / 4] = lo[3];
            L.B[(IB_DD + HDR + 17) / 4 + 1] = hi[3];
          }
          switch (__builtin_amdgcn_readfirstlane(cb)) {
#define TDBG_FCB(c) \
  case c: dd_emit<c>(L, lo, T); break;
            TDBG_FCB(2) TDBG_FCB(3) TDBG_FCB(4) TDBG_FCB(5) TDBG_FCB(6) TDBG_FCB(7) TDBG_FCB(8) TDBG_FCB(9)
            TDBG_FCB(10) TDBG_FCB(11) TDBG_FCB(12) TDBG_FCB(13) TDBG_FCB(14) TDBG_FCB(15) TDBG_FCB(16)
            TDBG_FCB(17) TDBG_FCB(18) TDBG_FCB(19) TDBG_FCB(20) TDBG_FCB(21) TDBG_FCB(22) TDBG_FCB(23)
            TDBG_FCB(24) TDBG_FCB(25) TDBG_FCB(26) TDBG_FCB(27) TDBG_FCB(28) TDBG_FCB(29) TDBG_FCB(30)
            TDBG_FCB(31)
#undef TDBG_FCB
            default:
              break;
          }
        }
        __syncthreads();  // B2: the image is complete
        const uint32_t total = HDR + cl;
        ok = ok && total <= cap;
        if (ok) store_image(L, IB_DD, total, out, T);
        if (ok && T == 0) {
          if (kp.status) kp.status[t] = TDBG_OK;
          if (kp.need) kp.need[t] = 0;
          if (kp.out_len) kp.out_len[t] = total;
        }
      } else if (MODE == 2) {
        // ---- PD: deltas within windows of 128 values (threads 4p..4p+3),
        // 0 at a window start; a decreasing value is the reference's error
        // (TDBG_E_PD_DECREASING), left to the general kernel ----
        const bool wstart = (T & 3) == 0;
        const uint32_t flo = lo[2], fhi = hi[2];  // the window's first value (wstart)
        bool dec = false;
#pragma unroll
        for (int k = 33; k >= 2; k--) {
          const uint64_t cur = val(k), prev = val(k - 1);
          uint64_t dl = cur - prev;
          if (k == 2) dl = wstart ? 0ull : dl;
          dec = dec || ((k != 2 || !wstart) && cur < prev);
          lo[k] = (uint32_t)dl;
          hi[k] = (uint32_t)(dl >> 32);
        }
        // ---- BWR window = this thread's 32 deltas: compute_bits_required
        // (bit_width_reduction_filter.cc:406-447), unsigned ----
        uint64_t mn = val(2), mx = val(2);
#pragma unroll
        for (int k = 3; k < 34; k++) {
          const uint64_t v = val(k);
          mn = v < mn ? v : mn;
          mx = v > mx ? v : mx;
        }
        const uint64_t range = mx - mn;
        uint32_t bits = 64;
        uint64_t minv = 0;
        if (range != ~0ull) {
          const uint64_t ro = range + 1;
          const uint32_t nbits = 64 - __builtin_clzll(ro);
          bits = nbits <= 8 ? 8 : nbits <= 16 ? 16 : nbits <= 32 ? 32 : 64;
          minv = mn;
        }
        const uint32_t cbw = bits >> 3;            // bytes per element (8: raw)
        const uint32_t csz = 32 * cbw;             // the window's compressed bytes
        const uint32_t inc = wave_incscan_u32(csz);
        if (l == 63) L.cnt[w] = inc;
        const uint64_t decw = __builtin_amdgcn_ballot_w64(dec);  // (every lane active)
        if (l == 0) L.red[w] = decw ? 1u : 0u;
        __syncthreads();  // B1
        uint32_t off = inc - csz, dn = 0;
        bool anydec = false;
#pragma unroll
        for (int v = 0; v < NWV; v++) {
          const uint32_t c = L.cnt[v];
          off += (uint32_t)v < w ? c : 0u;
          dn += c;
          anydec = anydec || L.red[v] != 0;
        }
        ok = !anydec && dn <= DMAX_C4;
        if (ok) {
          if (T == 0) {
            L.B[0] = 1;
            L.B[1] = 0;
            L.B[2] = TB;
            L.B[3] = dn;
            L.B[4] = ML_C4;
            L.B[5] = TB;   // BWR md: orig, windows
            L.B[6] = 256;
            L.B[(20 + 8 + 256 * 13) / 4] = 64;  // PD md: windows
          }
          // BWR md entry [u64 min][u8 bits][u32 256] (13 B, unaligned)
          const uint32_t eo = 28 + 13 * T;
          lds_u32b(L, eo, (uint32_t)minv);
          lds_u32b(L, eo + 4, (uint32_t)(minv >> 32));
          lds_u8(L, eo + 8, bits);
          lds_u32b(L, eo + 9, 256);
          if (wstart) {  // PD md entry [u64 first][u32 1024]
            const uint32_t po = (20 + 8 + 256 * 13 + 4 + 12 * (T >> 2)) / 4;
            L.B[po] = flo;
            L.B[po + 1] = fhi;
            L.B[po + 2] = 1024;
          }
          // the window's data at D0 + off (a multiple of 32): the deltas
          // minus the window minimum in cbw bytes, or raw
          uint32_t* dst = L.B + (D0_C4 + off) / 4;
          if (cbw == 1) {
#pragma unroll
            for (int q = 0; q < 8; q++)
              dst[q] = ((lo[4 * q + 2] - (uint32_t)minv) & 0xffu) | (((lo[4 * q + 3] - (uint32_t)minv) & 0xffu) << 8) |
                       (((lo[4 * q + 4] - (uint32_t)minv) & 0xffu) << 16) | ((lo[4 * q + 5] - (uint32_t)minv) << 24);
          } else if (cbw == 2) {
#pragma unroll
            for (int q = 0; q < 16; q++)
              dst[q] = ((lo[2 * q + 2] - (uint32_t)minv) & 0xffffu) | ((lo[2 * q + 3] - (uint32_t)minv) << 16);
          } else if (cbw == 4) {
#pragma unroll
            for (int q = 0; q < 32; q++) dst[q] = lo[q + 2] - (uint32_t)minv;
          } else {
#pragma unroll
            for (int q = 0; q < 32; q++) {
              dst[2 * q] = lo[q + 2];
              dst[2 * q + 1] = hi[q + 2];
            }
          }
        }
        __syncthreads();  // B2: the image is complete
        const uint32_t total = 20 + ML_C4 + dn;
        ok = ok && total <= cap;
        if (ok) store_image(L, 0, total, out, T);
        if (ok && T == 0) {
          if (kp.status) kp.status[t] = TDBG_OK;
          if (kp.need) kp.need[t] = 0;
          if (kp.out_len) kp.out_len[t] = total;
        }
      } else {
        // ---- RLE (rle_compressor.cc:51-101): a run head wherever a value
        // differs from the one before (runs of one tile's 8192 values never
        // reach the 65,535 split) ----
        uint32_t hm = 0;
#pragma unroll
        for (int k = 0; k < 32; k++) {
          const bool head = lo[k + 2] != lo[k + 1] || hi[k + 2] != hi[k + 1] || (k == 0 && T == 0);
          hm |= head ? 1u << k : 0u;
        }
        const uint32_t cnt = (uint32_t)__builtin_popcount(hm);
        const uint32_t inc = wave_incscan_u32(cnt);
        if (l == 63) L.cnt[w] = inc;
        __syncthreads();  // B1
        uint32_t r0 = inc - cnt, nr = 0;
#pragma unroll
        for (int v = 0; v < NWV; v++) {
          const uint32_t c = L.cnt[v];
          r0 += (uint32_t)v < w ? c : 0u;
          nr += c;
        }
        ok = nr <= RMAX;
        if (ok) {
          uint32_t r = r0;
          for (uint32_t mm = hm; mm; mm &= mm - 1, r++) L.H[r] = (uint16_t)(32 * T + __builtin_ctz(mm));
          if (T == 0) L.H[nr] = (uint16_t)NV;
        }
        __syncthreads();  // B2: run heads
        const uint32_t cl = 10 * nr;
        if (ok) {
          if (T == 0) write_headers(L, IB_RLE, cl);
          uint32_t r = r0;
          for (uint32_t mm = hm; mm; mm &= mm - 1, r++) {
            const uint32_t k = (uint32_t)__builtin_ctz(mm);
            const uint32_t len = (uint32_t)L.H[r + 1] - (uint32_t)L.H[r];
            // the head's value: position 32T + k (readlane-free: a uniform
            // select over the thread's 32 values)
            uint32_t vlo = 0, vhi = 0;
#pragma unroll
            for (int q = 0; q < 32; q++) {
              vlo = (uint32_t)q == k ? lo[q + 2] : vlo;
              vhi = (uint32_t)q == k ? hi[q + 2] : vhi;
            }
            uint16_t* rec = (uint16_t*)((uint8_t*)L.B + IB_RLE + HDR + 10 * r);
            rec[0] = (uint16_t)vlo;
            rec[1] = (uint16_t)(vlo >> 16);
            rec[2] = (uint16_t)vhi;
            rec[3] = (uint16_t)(vhi >> 16);
            rec[4] = (uint16_t)(((len & 0xffu) << 8) | (len >> 8));  // big-endian length
          }
        }
        __syncthreads();  // B3: the image is complete
        const uint32_t total = HDR + cl;
        ok = ok && total <= cap;
        if (ok) store_image(L, IB_RLE, total, out, T);
        if (ok && T == 0) {
          if (kp.status) kp.status[t] = TDBG_OK;
          if (kp.need) kp.need[t] = 0;
          if (kp.out_len) kp.out_len[t] = total;
        }
      }
    }
    if (ok) taken++;
    if (!ok && T == 0) {
      // the general forward kernel takes this tile (and reports its status)
      const uint32_t k = atomicAdd(kp.fbq, 1u);
      if (k < kp.fbq_cap) kp.fbq[1 + k] = (uint32_t)t;
      else if (kp.status) kp.status[t] = TDBG_E_INTERNAL;
    }
  }
  if (kp.stats && threadIdx.x == 0 && taken)
    atomicAdd((unsigned long long*)&kp.stats[TDBG_STAT_STRIDE * (1 + (blockIdx.x & 63)) + TDBG_STAT_FWD_STREAM_TILES],
              (unsigned long long)taken);  // (one slot per 64 workgroups: tdbg_host.cpp read_stats sums them)
}

}  // namespace fsm
}  // namespace tdbg

// mode 0 [DOUBLE_DELTA] on 8-byte values (sgn: the DD type is signed),
// mode 1 [RLE] with 8-byte cells, mode 2 [POSITIVE_DELTA(1024), BWR(256)] on
// uint64
extern "C" hipError_t tdbg_launch_filter_small(const tdbg::KParams* kp, uint32_t grid, int mode, int sgn,
                                               hipStream_t s) {
  using namespace tdbg::fsm;
  if (mode == 0 && sgn) hipLaunchKernelGGL((filter_small_kernel<0, true>), dim3(grid), dim3(NT), 0, s, *kp);
  else if (mode == 0) hipLaunchKernelGGL((filter_small_kernel<0, false>), dim3(grid), dim3(NT), 0, s, *kp);
  else if (mode == 1) hipLaunchKernelGGL((filter_small_kernel<1, false>), dim3(grid), dim3(NT), 0, s, *kp);
  else hipLaunchKernelGGL((filter_small_kernel<2, false>), dim3(grid), dim3(NT), 0, s, *kp);
  return hipGetLastError();
}
