// tdbg_forward_stream.hip -- forward ("filter") direction of the headline
// pipeline [BYTESHUFFLE, DOUBLE_DELTA, BIT_WIDTH_REDUCTION] on 4-byte
// integers, one 64 KiB tile = one chunk (the write path WriterBase::
// filter_tile -> FilterPipeline::run_forward, writer_base.cc:870-915,
// filter_pipeline.cc:208-369), LDS-resident, gfx950.
//
// The general forward kernel (tdbg_forward.hip) runs every filter through a
// global scratch slot with byte-granular accesses.  Here one 512-thread
// workgroup owns a tile and the chunk never leaves the CU until its filtered
// image is stored:
//
//   * Byteshuffle (byteshuffle_filter.cc:60-89): thread T loads the 16-B
//     units 8T..8T+7 (values 32T..32T+31) and two units before them; a 4x4
//     byte transpose of a unit gives the unit's dword in each of the four
//     byte planes, so the thread holds positions 8T-2..8T+7 of every plane
//     of the shuffled stream s (int32, 16,384 values) in registers.
//   * DoubleDelta (dd_compressor.cc:211-312): the bit size is the bit length
//     of max(|d1|, |dd_i|) over the tile (one workgroup max); codes (sign,
//     then bitsize magnitude bits, MSB first in little-endian u64 words) are
//     OR-ed into the DD output in LDS at their bit offsets, or the values are
//     stored raw (bitsize >= 31).  The compression filter's metadata part
//     (the byteshuffle header: two int32) becomes the 17-byte DD part before
//     it (compression_filter.cc:240-301).
//   * BWR (bit_width_reduction_filter.cc:110-280, 406-447): 8 lanes per
//     256-B window read its 64 elements once into registers; min / max give
//     the window's width; an exclusive workgroup scan of the compressed
//     sizes places every window; the compressed bytes are written in place
//     below the DD output (a window's output never reaches past its own
//     input), next to the metadata and tile header, so the whole filtered
//     tile is one contiguous LDS image.
//   * The image leaves with lane-consecutive 16-B stores.
//
// The LDS image: DD-output byte x at LDS byte DELTA + x (DELTA = 2 mod 4, so
// the DD words -- DD-output byte 34 + 8q -- are dword aligned); compressed
// data byte x at X0 + x (X0 = DELTA - 2); tile header and metadata right
// below X0.  ~71 KB: two workgroups per CU.
//
// Tiles of any other shape (size, alignment, capacity) are queued (KParams::
// fbq) for the general forward kernel, which runs on the queue right after,
// so every status and byte stays the oracle's (tests/test_gpu_forward.py).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "../../include/tiledb_amd.h"
#include "tdbg_desc.h"
#include "tdbg_device.h"

namespace tdbg {
namespace fws {

constexpr uint32_t NV = 16384;              // int32 values per tile
constexpr uint32_t TB = NV * 4;             // tile bytes
constexpr uint32_t NWMAX = 257;             // BWR windows over <= 65,562 DD-output bytes
constexpr uint32_t MLMAX = 8 + 9 * NWMAX + 24;
constexpr uint32_t DELTA = 2370;            // >= 22 + MLMAX, = 2 mod 4
constexpr uint32_t X0 = DELTA - 2;          // compressed data byte 0
constexpr uint32_t DOUT_MAX = 17 + 9 + TB;  // DD output bytes (raw)
constexpr uint32_t BDW = (DELTA + DOUT_MAX + 320 + 15) / 16 * 4;  // image dwords (+ reads past the last window)
constexpr uint32_t WD0 = (DELTA + 34) / 4;  // LDS dword of DD word 0
static_assert(DELTA % 4 == 2 && X0 >= 20 + MLMAX, "LDS image layout");
constexpr uint32_t GRID_CAP = 1u << 22;

// NT threads per workgroup: 512 (persistent grid, two workgroups per CU at
// 128 VGPRs) or 1024 (one workgroup per tile, two per CU at 64 VGPRs); a
// thread owns UPT = 4096 / NT of the tile's 16-B units
template <int NT>
struct Cfg {
  static constexpr int NWV = NT / 64;
  static constexpr uint32_t UPT = 4096 / NT;                 // units (runs of UPT values per plane) per thread
  static constexpr uint32_t WPP = NT / 8;                    // BWR windows per pass (8 lanes each)
  static constexpr uint32_t PASSES = (NWMAX + WPP - 1) / WPP;  // BWR window passes
};

template <int NT>
struct Lds {
  uint32_t B[BDW];
  uint32_t wcs[NWMAX + 7];   // window compressed bytes, then (after the scan) its data offset
  uint32_t wbits[NWMAX + 7]; // the window's bits field
  int32_t wmin[NWMAX + 7];
  uint64_t red[4 * Cfg<NT>::NWV];
  uint32_t scan[Cfg<NT>::NWV];
  uint64_t clk[8];  // diagnostics: phase clocks (TDBG_PROF)
};

// Diagnostics (KParams::prof, TDBG_PROF=1): per-workgroup shader-clock
// cycles per phase: 0 loads + transposes (after B0), 1 bit size + B1, 2 DD
// output + B2, 3 BWR window pass + B3, 4 scan + headers + B4/B5, 5 in-place
// compression + B6, 6 image store
struct Clock {
  uint64_t* out;
  uint64_t* acc;
  uint64_t t;
  __device__ __forceinline__ void init(uint64_t* o, uint64_t* a) {
    out = o;
    acc = a;
    if (!out) return;
    t = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0)
      for (int k = 0; k < 8; k++) acc[k] = 0;
  }
  __device__ __forceinline__ void mark(int k) {
    if (!out) return;
    const uint64_t n = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) acc[k] += n - t;
    t = n;
  }
  __device__ __forceinline__ void flush() {
    if (!out || threadIdx.x != 0) return;
    for (int k = 0; k < 8; k++) out[blockIdx.x * TDBG_PROF_PHASES + k] = acc[k];
  }
};

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const v4u g_cu4;
typedef __attribute__((address_space(1))) v4u g_u4;

__device__ __forceinline__ void tr4(uint32_t p0, uint32_t p1, uint32_t p2, uint32_t p3, uint32_t (&w)[4]) {
  // w[d] byte k = p_k byte d
  const uint32_t a = __builtin_amdgcn_perm(p1, p0, 0x05010400u);
  const uint32_t b = __builtin_amdgcn_perm(p3, p2, 0x05010400u);
  const uint32_t c = __builtin_amdgcn_perm(p1, p0, 0x07030602u);
  const uint32_t d = __builtin_amdgcn_perm(p3, p2, 0x07030602u);
  w[0] = __builtin_amdgcn_perm(b, a, 0x05040100u);
  w[1] = __builtin_amdgcn_perm(b, a, 0x07060302u);
  w[2] = __builtin_amdgcn_perm(d, c, 0x05040100u);
  w[3] = __builtin_amdgcn_perm(d, c, 0x07060302u);
}

template <class LDS>
__device__ __forceinline__ void lds_byte(LDS& L, uint32_t o, uint32_t v) { ((uint8_t*)L.B)[o] = (uint8_t)v; }
template <class LDS>
__device__ __forceinline__ void lds_u32b(LDS& L, uint32_t o, uint32_t v) {
#pragma unroll
  for (int i = 0; i < 4; i++) lds_byte(L, o + i, v >> (8 * i));
}


// Reductions over a 16-lane DPP row (the lanes of one BWR window, or a
// wave's row): quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror
// -- every lane ends with the row's result, VALU only.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, false);
}
template <bool SGN>
__device__ __forceinline__ void half_minmax(uint32_t& mn, uint32_t& mx) {  // over 8 lanes
  auto step = [&](uint32_t a, uint32_t b) {
    if (SGN) {
      mn = (int32_t)a < (int32_t)mn ? a : mn;
      mx = (int32_t)b > (int32_t)mx ? b : mx;
    } else {
      mn = a < mn ? a : mn;
      mx = b > mx ? b : mx;
    }
  };
  step(dpp_<0xB1>(mn), dpp_<0xB1>(mx));
  step(dpp_<0x4E>(mn), dpp_<0x4E>(mx));
  step(dpp_<0x141>(mn), dpp_<0x141>(mx));
}
__device__ __forceinline__ uint64_t row_max64(uint64_t v) {
  auto step = [&](uint64_t o) { v = o > v ? o : v; };
  step(((uint64_t)dpp_<0xB1>((uint32_t)(v >> 32)) << 32) | dpp_<0xB1>((uint32_t)v));
  step(((uint64_t)dpp_<0x4E>((uint32_t)(v >> 32)) << 32) | dpp_<0x4E>((uint32_t)v));
  step(((uint64_t)dpp_<0x141>((uint32_t)(v >> 32)) << 32) | dpp_<0x141>((uint32_t)v));
  step(((uint64_t)dpp_<0x140>((uint32_t)(v >> 32)) << 32) | dpp_<0x140>((uint32_t)v));
  return v;
}

// DoubleDelta codes of thread T's four runs (plane k: positions 8T..8T+7,
// i.e. S[2..9][k]) at compile-time code width CB = bitsize + 1
// (dd_compressor.cc:243-257, 406-450: a sign bit, then bitsize magnitude bits, MSB
// first from bit 63 of little-endian u64 words).  A run's 8 codes are one
// contiguous bit range: they are packed at compile-time bit positions into 8
// run dwords R (MSB first), then shifted to the run's stream bit offset with
// one v_alignbit per output chunk.  Chunk c of the stream (32 bits, stream
// order) is LDS dword WD0 + (c ^ 1) (the high half of a u64 word comes
// first).  Chunks wholly inside the run are plain writes; the first and the
// last one or two are shared with the neighbouring runs and OR-ed (the
// region was zeroed before B1).  Thread 0's plane-0 run has codes from
// position 2 only: it is packed with two zero codes in front at stream bit
// -2 CB and its chunks below 0 are not written.
template <int CB, int NT>
__device__ __forceinline__ void dd_emit(Lds<NT>& L, const uint32_t (&S)[Cfg<NT>::UPT + 2][4], uint32_t T) {
  constexpr int UPT = (int)Cfg<NT>::UPT;
  constexpr uint32_t BS = CB - 1;            // bitsize
  constexpr int JF = (UPT * CB) / 32 - 1;    // chunks 1..JF lie inside the run for any start bit
  constexpr int JX = (UPT * CB + 30) / 32;   // the last chunk a run can reach
#pragma unroll
  for (int k = 0; k < 4; k++) {
    uint32_t code[UPT];
    uint32_t dprev = S[1][k] - S[0][k];
#pragma unroll
    for (int i = 2; i < UPT + 2; i++) {
      // (coded: |dd| < 2^30, so the wrapped 32-bit value is exact)
      const uint32_t d = S[i][k] - S[i - 1][k];
      const int32_t dd = (int32_t)(d - dprev);
      dprev = d;
      const uint32_t a = (uint32_t)(dd < 0 ? -dd : dd);
      code[i - 2] = (((uint32_t)dd >> 31) << BS) | a;
    }
    const bool t0 = k == 0 && T == 0;
    if (k == 0) {
      code[0] = t0 ? 0u : code[0];
      code[1] = t0 ? 0u : code[1];
    }
    uint32_t R[UPT];
#pragma unroll
    for (int j = 0; j < UPT; j++) R[j] = 0;
#pragma unroll
    for (int j = 0; j < UPT; j++) {
      const int off = j * CB, w0 = off >> 5, sh = off & 31;
      if (sh + CB <= 32) {
        R[w0] |= code[j] << (32 - sh - CB);
      } else {
        R[w0] |= code[j] >> (sh + CB - 32);
        R[w0 + 1] |= code[j] << (64 - sh - CB);
      }
    }
    // stream bit of the run's first code (code index 4096 k + UPT T - 2)
    const int32_t B0 = ((int32_t)(4096 * k) + UPT * (int32_t)T - 2) * CB;
    const int32_t c0 = B0 >> 5;
    const uint32_t nb0 = (uint32_t)B0 & 31u;
    const int32_t base = (int32_t)WD0 + (c0 & ~1);
    const uint32_t par = (uint32_t)c0 & 1u;
    // dword of chunk c0 + j: base + ((j + par) ^ 1), i.e. (even j) base + 1 - par + j,
    // (odd j) base - 1 + 3 par + j
    uint32_t* const pe = L.B + (base + 1 - (int32_t)par);
    uint32_t* const po = L.B + (base - 1 + 3 * (int32_t)par);
    const int32_t jmax = (int32_t)((UPT * CB - 1 + nb0) >> 5);
#pragma unroll
    for (int j = 0; j <= JX; j++) {
      const uint32_t hi = j == 0 ? 0u : R[j - 1], lo = j >= UPT ? 0u : R[j];
      const uint32_t ch = __builtin_amdgcn_alignbit(hi, lo, nb0);
      uint32_t* const dst = (j & 1 ? po : pe) + j;
      const bool inside = k != 0 || c0 + j >= 0;  // (thread 0, plane 0: no chunks below 0)
      if (j >= 1 && j <= JF) {
        if (inside) *dst = ch;
      } else if (j <= jmax && inside) {
        atomicOr(dst, ch);
      }
    }
  }
}

// The tile loop: NT = 512 walks tiles blockIdx.x, + gridDim.x, ... (the next
// tile's units loaded behind this one's stores); NT = 1024 takes the one work
// item (b & 7) * ceil(cnt / 8) + (b >> 3) of [base, base + cnt): each XCD
// (workgroups are dealt round-robin over the 8) works through a contiguous
// eighth of the launch (placement assumption for speed only).
template <bool SGN, int NT>
__device__ __forceinline__ void filter_c5_body(const KParams& kp, uint32_t base, uint32_t cnt) {
  constexpr bool PERSIST = NT == 512;
  constexpr int NWV = Cfg<NT>::NWV;
  constexpr uint32_t UPT = Cfg<NT>::UPT, WPP = Cfg<NT>::WPP, PASSES = Cfg<NT>::PASSES;
  __shared__ Lds<NT> L;
  Clock pc;
  // (phase clocks of the first 512 workgroups: the profile buffer's rows)
  pc.init(PERSIST || blockIdx.x < 512 ? kp.prof : nullptr, L.clk);
  auto shape_of = [&](uint64_t jj) {
    const uint8_t* ii = kp.in[jj];
    return kp.in_size[jj] == TB && (((uintptr_t)ii) & 15) == 0 && (((uintptr_t)kp.out[jj]) & 15) == 0 &&
           kp.out_size[jj] >= 64;
  };
  v4u U[UPT + 2];
  auto load_units = [&](uint64_t jj, uint32_t T) {
    // units UPT T..UPT T + UPT - 1 and the two before (wrapping into the last
    // plane's end for T = 0)
    const g_cu4* src = (const g_cu4*)kp.in[jj];
#pragma unroll
    for (uint32_t i = 0; i < UPT + 2; i++) U[i] = src[(UPT * T + i - 2) & 4095u];
  };
  bool pre = false;  // U holds this tile's units already (loaded at the end of the last iteration)
  uint64_t j0 = blockIdx.x, jstep = gridDim.x;
  if (!PERSIST) {
    const uint32_t n8 = (cnt + 7) >> 3;
    const uint32_t jj = (blockIdx.x & 7) * n8 + (blockIdx.x >> 3);
    if (jj >= cnt) return;
    j0 = (uint64_t)base + jj;
    jstep = ~0ull >> 1;  // (one tile)
  }
  for (uint64_t j = j0; j < kp.ntiles; j += jstep) {
    // thread index opaque to the optimizer: the unrolled per-thread index
    // math is tile-invariant, and hoisting it out of the tile loop pins (and
    // spills) dozens of registers
    uint32_t T = threadIdx.x;
    asm volatile("" : "+v"(T));
    const uint32_t l = T & 63, w = __builtin_amdgcn_readfirstlane(T >> 6);
    const uint64_t t = j;
    uint8_t* out = kp.out[t];
    const uint64_t cap = kp.out_size[t];
    // this kernel's tile shape; anything else goes to the general kernel
    const bool shape = shape_of(t);
    bool ok = shape;
    __syncthreads();  // B0: the last tile's image is stored (LDS free)
    if (shape) {
      // (issued here, their latency overlaps the zeroing below, unless the
      // last iteration already issued them right after its image stores:
      // then they also overlap B0.  A prefetch issued before the last tile's
      // image stores measured slower -- the stores waited behind the loads.)
      if (!pre) load_units(t, T);
      // ---- zero the DD word region (codes are OR-ed in) ----
      static_assert(BDW % 4 == 0, "16-B zeroing");
      for (uint32_t d = (WD0 & ~3u) + 4 * T; d < BDW; d += 4 * NT) *(v4u*)(L.B + d) = v4u{0u, 0u, 0u, 0u};
      // S[i][k]: position UPT T + i - 2 of plane k (for T = 0 and i < 2: plane k-1's end)
      uint32_t S[UPT + 2][4];
#pragma unroll
      for (uint32_t i = 0; i < UPT + 2; i++) tr4(U[i].x, U[i].y, U[i].z, U[i].w, S[i]);
      if (T == 0) {
#pragma unroll
        for (int i = 0; i < 2; i++) {
          S[i][3] = S[i][2];
          S[i][2] = S[i][1];
          S[i][1] = S[i][0];
          S[i][0] = 0;  // (positions -2, -1 do not exist)
        }
      }
      pc.mark(0);
      // ---- DoubleDelta bit size: max(|d1|, |dd_i|), i >= 2 ----
      // (in f64, which holds every int32 / uint32 value and their first and
      // second differences, |dd| < 2^34, exactly: one conversion, two
      // subtractions and a max with an |.| modifier per value instead of
      // 64-bit integer arithmetic)
      double mxd = 0.0;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        auto f = [&](uint32_t v) { return SGN ? (double)(int32_t)v : (double)v; };
        double x2 = f(S[0][k]), x1 = f(S[1][k]);
#pragma unroll
        for (uint32_t i = 2; i < UPT + 2; i++) {
          const uint32_t P = 4096 * k + UPT * T + i - 2;
          const double x = f(S[i][k]);
          const double d = x - x1, dp = x1 - x2;
          double a = __builtin_fabs(d - dp);
          // (only positions 0 and 1 -- thread 0, plane 0 -- differ: no dd
          // there, and d1 counts for position 1; a compile-time guard keeps
          // the selects off every other value)
          if (k == 0 && i < 4) a = P >= 2 ? a : P == 1 ? __builtin_fabs(d) : 0.0;
          mxd = __builtin_fmax(mxd, a);
          x2 = x1;
          x1 = x;
        }
      }
      uint64_t mx = (uint64_t)mxd;
      mx = row_max64(mx);
      // the wave's maximum from its four rows (readlane: scalar), one LDS
      // entry per wave
      {
        auto rl = [&](int k) -> uint64_t {
          return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(mx >> 32), k) << 32) |
                 (uint32_t)__builtin_amdgcn_readlane((uint32_t)mx, k);
        };
        const uint64_t a = rl(0), b = rl(16), c = rl(32), d = rl(48);
        const uint64_t ab = a > b ? a : b, cd = c > d ? c : d;
        mx = ab > cd ? ab : cd;
      }
      if (l == 0) L.red[w] = mx;
      __syncthreads();  // B1
      mx = 0;
#pragma unroll
      for (int v = 0; v < NWV; v++) mx = L.red[v] > mx ? L.red[v] : mx;
      // (the 64-bit extensions of the bit-size pass are recomputed below, not
      // kept live across the barrier: 40 values would take 80 registers)
#pragma unroll
      for (uint32_t i = 0; i < UPT + 2; i++)
#pragma unroll
        for (int k = 0; k < 4; k++) asm volatile("" : "+v"(S[i][k]));
      const uint32_t bitsize = mx ? 64 - __builtin_clzll(mx) : 1;  // do { ++b; m >>= 1; } while (m)
      pc.mark(1);
      const bool raw = bitsize >= 31;
      const uint32_t cb = bitsize + 1;
      const uint32_t words = raw ? 0u : ((NV - 2) * cb + 63) / 64;
      const uint32_t cl1 = raw ? 9 + TB : 17 + 8 * words;
      const uint32_t Ld = 17 + cl1;  // BWR input bytes
      // ---- the DD output ----
      if (T == 0) {
        // md part (the byteshuffle header [1][65536] as two int32):
        // [bitsize 0][u64 2][1][65536]; data part header [bitsize][u64 16384]
        lds_byte(L, DELTA, 0);
        lds_u32b(L, DELTA + 1, 2);
        lds_u32b(L, DELTA + 5, 0);
        lds_u32b(L, DELTA + 9, 1);
        lds_u32b(L, DELTA + 13, TB);
        lds_byte(L, DELTA + 17, bitsize);
        lds_u32b(L, DELTA + 18, NV);
        lds_u32b(L, DELTA + 22, 0);
      }
      // s0, s1 (x0, x1; or the first raw values) at DD-output 26 = dword 599
      if (raw) {
#pragma unroll
        for (int k = 0; k < 4; k++)
#pragma unroll
          for (uint32_t i = 2; i < UPT + 2; i++) L.B[(DELTA + 26) / 4 + 4096 * k + UPT * T + i - 2] = S[i][k];
      } else {
        if (T == 0) {
          L.B[(DELTA + 26) / 4] = S[2][0];
          L.B[(DELTA + 30) / 4] = S[3][0];
        }
        // one instantiation per code width (uniform)
        switch (__builtin_amdgcn_readfirstlane(cb)) {
#define TDBG_FCB(c) \
  case c: dd_emit<c, NT>(L, S, T); break;
          TDBG_FCB(2) TDBG_FCB(3) TDBG_FCB(4) TDBG_FCB(5) TDBG_FCB(6) TDBG_FCB(7) TDBG_FCB(8) TDBG_FCB(9)
          TDBG_FCB(10) TDBG_FCB(11) TDBG_FCB(12) TDBG_FCB(13) TDBG_FCB(14) TDBG_FCB(15) TDBG_FCB(16)
          TDBG_FCB(17) TDBG_FCB(18) TDBG_FCB(19) TDBG_FCB(20) TDBG_FCB(21) TDBG_FCB(22) TDBG_FCB(23)
          TDBG_FCB(24) TDBG_FCB(25) TDBG_FCB(26) TDBG_FCB(27) TDBG_FCB(28) TDBG_FCB(29) TDBG_FCB(30)
          TDBG_FCB(31)
#undef TDBG_FCB
          default:
            break;  // (cb = bitsize + 1 is 2..31 when not raw)
        }
      }
      __syncthreads();  // B2: DD output complete
      pc.mark(2);
      // ---- BWR windows: 8 lanes each (32 bytes a lane), 64 per pass; elements
      // into registers ----
      const uint32_t nw = (Ld + 255) / 256;
      const uint32_t g = T >> 3, li = T & 7;
      // (NT = 1024: the elements are read again for the compression, one pass
      // at a time, instead of held in registers across B3-B5 -- 64 VGPRs)
      constexpr bool REREAD = !PERSIST;
      constexpr uint32_t EP = REREAD ? 1 : PASSES;
      uint32_t E[EP][8];
      // DD-output bytes [256 wi + 32 li, +32) = LDS dwords from 592 + 64 wi + 8 li, shifted by 2
      // (windows 2, 3 mod 4 read their second half first: every
      // ds_read_b128 lane group then covers 64 distinct banks)
      auto load_win = [&](uint32_t wi, uint32_t (&e8)[8]) {
        const uint32_t d0 = (DELTA - 2) / 4 + 64 * wi + 8 * li;
        const uint32_t hs = 4 * ((wi >> 1) & 1);
        const v4u qa = *(const v4u*)(L.B + d0 + hs), qb = *(const v4u*)(L.B + d0 + 4 - hs);
        const uint32_t q8 = L.B[d0 + 8];
        const bool sw = hs != 0;
        const v4u q0 = sw ? qb : qa, q1 = sw ? qa : qb;
        const uint32_t Q[9] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, q8};
#pragma unroll
        for (int e = 0; e < 8; e++) e8[e] = __builtin_amdgcn_alignbyte(Q[e + 1], Q[e], 2);
      };
#pragma unroll
      for (uint32_t p = 0; p < PASSES; p++) {
        const uint32_t wi = WPP * p + g;
        const uint32_t ep = REREAD ? 0 : p;
#pragma unroll
        for (int e = 0; e < 8; e++) E[ep][e] = 0;
        if (WPP * p < nw) {  // (uniform)
          if (wi < nw) {  // (uniform over the window's 8 lanes)
            load_win(wi, E[ep]);
            const uint32_t nb = Ld - 256 * wi < 256 ? Ld - 256 * wi : 256;
            const uint32_t ne = nb >> 2;
            auto mm = [&](uint32_t v, uint32_t& mn, uint32_t& mx) {
              if (SGN) {
                mn = (int32_t)v < (int32_t)mn ? v : mn;
                mx = (int32_t)v > (int32_t)mx ? v : mx;
              } else {
                mn = v < mn ? v : mn;
                mx = v > mx ? v : mx;
              }
            };
            uint32_t mn32 = E[ep][0], mx32 = E[ep][0];
            if (ne == 64) {  // every window but the last: all 8 elements count
#pragma unroll
              for (int e = 1; e < 8; e++) mm(E[ep][e], mn32, mx32);
            } else {
              mn32 = SGN ? 0x7fffffffu : 0xffffffffu;
              mx32 = SGN ? 0x80000000u : 0u;
#pragma unroll
              for (int e = 0; e < 8; e++)
                if (8 * li + e < ne) mm(E[ep][e], mn32, mx32);
            }
            half_minmax<SGN>(mn32, mx32);
            if (li == 0) {
              // compute_bits_required (bit_width_reduction_filter.cc:406-447),
              // in 32 bits: range = max - min < 2^32 is exact as a u32
              // difference; signed: bits 32 when range > INT32_MAX or
              // range + 1 > INT32_MAX, i.e. range >= 2^31 - 1
              uint32_t bits = 32;
              int32_t minv = 0;
              if (ne > 0) {
                const uint32_t range = mx32 - mn32;
                if (SGN ? range < 0x7fffffffu : range != 0xffffffffu) {
                  const uint32_t ro = range + 1;
                  bits = ro <= (SGN ? 127u : 255u) ? 8 : ro <= (SGN ? 32767u : 65535u) ? 16 : 32;
                  minv = (int32_t)mn32;
                }
              }
              const bool wraw = bits >= 32 || (nb & 3) != 0;
              L.wcs[wi] = wraw ? nb : ne * (bits >> 3);
              L.wbits[wi] = bits;
              L.wmin[wi] = minv;
            }
          }
        }
      }
      __syncthreads();  // B3: window table
      pc.mark(3);
      // exclusive scan of the compressed sizes (thread = window)
      const uint32_t cs = T < nw ? L.wcs[T] : 0u;
      const uint32_t inc = wave_incscan_u32(cs);
      if (l == 63) L.scan[w] = inc;
      __syncthreads();  // B4
      uint32_t pre = 0, fl = 0;
#pragma unroll
      for (int v = 0; v < NWV; v++) {
        const uint32_t x = L.scan[v];
        pre += (uint32_t)v < w ? x : 0u;
        fl += x;
      }
      const uint32_t ml = 8 + 9 * nw + 24;
      if (T < nw) {
        L.wcs[T] = pre + inc - cs;  // (read only after B5)
        // md entry [i32 minv][u8 bits][u32 nb] at image MD + 8 + 9 T, one
        // thread per window
        const uint32_t nb = Ld - 256 * T < 256 ? Ld - 256 * T : 256;
        const uint32_t eo = X0 - ml + 8 + 9 * T;
        lds_u32b(L, eo, (uint32_t)L.wmin[T]);
        lds_byte(L, eo + 4, L.wbits[T]);
        lds_u32b(L, eo + 5, nb);
      }
      const uint32_t S0 = X0 - ml - 20;
      const uint32_t total = 20 + ml + fl;
      ok = total <= cap;
      if (T == 0) {
        // tile header [u64 1][u32 65536][u32 fl][u32 ml], BWR md head
        // [u32 Ld][u32 nw], compression frame [1][1][8][17][65536][cl1]
        lds_u32b(L, S0, 1);
        lds_u32b(L, S0 + 4, 0);
        lds_u32b(L, S0 + 8, TB);
        lds_u32b(L, S0 + 12, fl);
        lds_u32b(L, S0 + 16, ml);
        lds_u32b(L, S0 + 20, Ld);
        lds_u32b(L, S0 + 24, nw);
        const uint32_t fo = S0 + 28 + 9 * nw;
        lds_u32b(L, fo, 1);
        lds_u32b(L, fo + 4, 1);
        lds_u32b(L, fo + 8, 8);
        lds_u32b(L, fo + 12, 17);
        lds_u32b(L, fo + 16, TB);
        lds_u32b(L, fo + 20, cl1);
      }
      __syncthreads();  // B5: offsets; every element is in registers
      pc.mark(4);
      // ---- compressed windows, in place below the DD output ----
      // (REREAD: pass p reads its windows' elements, a barrier, then writes:
      // a window's output [off, off + cs) lies below 256 (wi + 1), so a pass's
      // writes never reach a later pass's inputs, and inside a pass every read
      // is done before any write)
#pragma unroll
      for (uint32_t p = 0; p < PASSES; p++) {
        const uint32_t wi = WPP * p + g;
        const uint32_t ep = REREAD ? 0 : p;
        if (REREAD) {
          if (WPP * p >= nw) break;  // (uniform)
          if (wi < nw) load_win(wi, E[ep]);
          __syncthreads();
        }
        if (WPP * p < nw && wi < nw) {
          const uint32_t off = L.wcs[wi], bits = L.wbits[wi];
          const uint32_t nbw = Ld - 256 * wi < 256 ? Ld - 256 * wi : 256;
          const uint32_t kind = (bits >= 32 || (nbw & 3) != 0) ? 2u : bits == 8 ? 0u : 1u;
          const uint32_t mnv = (uint32_t)L.wmin[wi];
          const uint32_t a = X0 + off;  // 4-aligned: every earlier window's size is a multiple of 4
          uint32_t r[8];
#pragma unroll
          for (int e = 0; e < 8; e++) r[e] = E[ep][e] - mnv;
          if (kind == 0) {
            uint32_t x0 = 0, x1 = 0;
#pragma unroll
            for (int e = 0; e < 4; e++) {
              x0 |= (r[e] & 0xffu) << (8 * e);
              x1 |= (r[4 + e] & 0xffu) << (8 * e);
            }
            *(uint2*)(L.B + (a >> 2) + 2 * li) = make_uint2(x0, x1);
          } else if (kind == 1) {
            *(v4u*)(L.B + (a >> 2) + 4 * li) =
                v4u{(r[0] & 0xffffu) | (r[1] << 16), (r[2] & 0xffffu) | (r[3] << 16), (r[4] & 0xffffu) | (r[5] << 16),
                    (r[6] & 0xffffu) | (r[7] << 16)};
          } else {
            *(v4u*)(L.B + (a >> 2) + 8 * li) = v4u{E[ep][0], E[ep][1], E[ep][2], E[ep][3]};
            *(v4u*)(L.B + (a >> 2) + 8 * li + 4) = v4u{E[ep][4], E[ep][5], E[ep][6], E[ep][7]};
          }
        }
      }
      __syncthreads();  // B6: the filtered image is complete in LDS
      pc.mark(5);
      if (ok) {
        // ---- store: image bytes [S0, S0 + total) to out, 16-B lane units ----
        // (two aligned ds_read_b128 per lane -- lane-consecutive, conflict-free --
        // shifted by the image's start within its 16-B unit)
        const uint32_t s16 = S0 & 15, k0 = S0 >> 4, r = s16 & 3, qd = s16 >> 2;
        const uint32_t nu = (total + 15) >> 4;
        for (uint32_t u = T; u < nu; u += NT) {
          const v4u A = *(const v4u*)(L.B + 4 * (k0 + u)), Bq = *(const v4u*)(L.B + 4 * (k0 + u + 1));
          const uint32_t W8[8] = {A.x, A.y, A.z, A.w, Bq.x, Bq.y, Bq.z, Bq.w};
          v4u y;
          switch (qd) {  // (uniform)
#define TDBG_SH(q)                                                                                   \
  case q:                                                                                            \
    y = v4u{__builtin_amdgcn_alignbyte(W8[q + 1], W8[q], r), __builtin_amdgcn_alignbyte(W8[q + 2], W8[q + 1], r), \
            __builtin_amdgcn_alignbyte(W8[q + 3], W8[q + 2], r), __builtin_amdgcn_alignbyte(W8[q + 4], W8[q + 3], r)}; \
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
        if (T == 0) {
          if (kp.stats) atomicAdd((unsigned long long*)&kp.stats[TDBG_STAT_FWD_STREAM_TILES], 1ull);
          if (kp.status) kp.status[t] = TDBG_OK;
          if (kp.need) kp.need[t] = 0;
          if (kp.out_len) kp.out_len[t] = total;
        }
      }
    }
    // the next tile's units, behind this tile's stores
    pre = false;
    if (PERSIST && j + gridDim.x < kp.ntiles && shape_of(j + gridDim.x)) {
      uint32_t Tn = threadIdx.x;
      asm volatile("" : "+v"(Tn));
      load_units(j + gridDim.x, Tn);
      pre = true;
    }
    pc.mark(6);
    if (!ok && T == 0) {
      // the general forward kernel takes this tile (and reports OUT_FULL etc.)
      const uint32_t k = atomicAdd(kp.fbq, 1u);
      if (k < kp.fbq_cap) kp.fbq[1 + k] = (uint32_t)t;
      else if (kp.status) kp.status[t] = TDBG_E_INTERNAL;
    }
  }
  pc.flush();
}

template <bool SGN>
__global__ void __launch_bounds__(512, 4) filter_stream_c5_kernel(const KParams kp) {
  filter_c5_body<SGN, 512>(kp, 0, 0);
}

template <bool SGN>
__global__ void __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(8, 8)))
filter_c5tile_kernel(const KParams kp, uint32_t base, uint32_t cnt) {
  filter_c5_body<SGN, 1024>(kp, base, cnt);
}

}  // namespace fws
}  // namespace tdbg

// sgn: the DD and BWR stages' integer type (INT32 / UINT32) is signed
// tile: one 1024-thread workgroup per tile (grid = the tiles, launches of at
// most GRID_CAP), else the persistent 512-thread kernel on `grid` workgroups
extern "C" hipError_t tdbg_launch_filter_c5(const tdbg::KParams* kp, uint32_t grid, int sgn, int tile, hipStream_t s) {
  using namespace tdbg::fws;
  if (!tile) {
    if (sgn) hipLaunchKernelGGL((filter_stream_c5_kernel<true>), dim3(grid), dim3(512), 0, s, *kp);
    else hipLaunchKernelGGL((filter_stream_c5_kernel<false>), dim3(grid), dim3(512), 0, s, *kp);
    return hipGetLastError();
  }
  for (uint64_t b = 0; b < kp->ntiles; b += GRID_CAP) {
    const uint32_t cnt = (uint32_t)(kp->ntiles - b < GRID_CAP ? kp->ntiles - b : GRID_CAP);
    const uint32_t g = 8 * ((cnt + 7) / 8);
    if (sgn) hipLaunchKernelGGL((filter_c5tile_kernel<true>), dim3(g), dim3(1024), 0, s, *kp, (uint32_t)b, cnt);
    else hipLaunchKernelGGL((filter_c5tile_kernel<false>), dim3(g), dim3(1024), 0, s, *kp, (uint32_t)b, cnt);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}
