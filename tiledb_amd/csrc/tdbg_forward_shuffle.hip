// tdbg_forward_shuffle.hip -- forward ("filter") direction of the shuffle
// configs on 4-byte values, one 64 KiB tile = one chunk (WriterBase::
// filter_tile -> FilterPipeline::run_forward, writer_base.cc:870-915,
// filter_pipeline.cc:208-369), gfx950, no LDS staging:
//
//   MODE 0  C1  [BYTESHUFFLE] (byteshuffle_filter.cc:60-89)
//   MODE 1  C2  [BITSHUFFLE, BWR] with BWR a pass-through (FLOAT32,
//           bit_width_reduction_filter.cc:166-176), or [BITSHUFFLE] alone
//   MODE 2  C2i [BITSHUFFLE, BWR(256)] on INT32 / UINT32
//           (bitshuffle_filter.cc:63-126, bit_width_reduction_filter.cc:
//           110-280, 406-447)
//
// A 512-thread workgroup takes a tile; wave b owns the 8,192-B bitshuffle
// block b (2,048 elements) and lane t' its elements 32t'..32t'+31 (eight
// 16-B loads).  Bitshuffle (kiyo-masui bshuf_trans_bit_elem, TileDB's
// 8,192-B blocking): per byte plane p, two 4x4 byte transposes gather byte
// p of each group of 8 elements into a 64-bit matrix, transpose8x8 turns it
// into the group's 8 bit rows (row 8p + k: bit k of byte p), and two more
// 4x4 transposes assemble, per row, the dword of the lane's four groups --
// so row r of block b is exactly the wave's 64 dwords, written by one store
// instruction (256 consecutive bytes).  That row is also BWR window
// 32 b + r (256-B windows over the shuffled part): C2i reduces it through
// the wave's LDS area (min / max -> width), the 256 window sizes go through one
// workgroup scan, and each window is written compressed where the scan put
// it (8-bit: a quad's four bytes as one dword, 16-bit: a pair's halves).
// Byteshuffle (C1): the lane's 32 elements give, per plane, 32 bytes of
// that plane at plane offset 32 t' (eight dword stores per plane: the
// data starts at tile byte 28).
//
// Filtered tile: [u64 1][u32 65536][u32 dn][u32 ml] then md then data.
//   C1, C2: md = [u32 1][u32 65536] (the shuffle's part table), data = the
//           shuffled 65,536 B (ml = 8, dn = 65,536);
//   C2i:    md = BWR md [u32 65536][u32 256] + 256 x [i32 min][u8 bits]
//           [u32 256] then the bitshuffle md (each filter prepends its md),
//           data = the compressed windows.
// Tiles of any other shape (sizes, alignment, capacity) are queued
// (KParams::fbq) for the general forward kernel, which runs on the queue
// right after (tests/test_gpu_forward.py).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/tiledb_amd.h"
#include "tdbg_desc.h"
#include "tdbg_device.h"

namespace tdbg {
namespace fsh {

constexpr int NT = 512;
constexpr int NWV = NT / 64;
constexpr uint32_t NV = 16384;   // 4-byte values per tile
constexpr uint32_t TB = NV * 4;  // tile bytes
constexpr uint32_t NW = 256;     // BWR windows (C2i)
constexpr uint32_t ML_BWR = 8 + 9 * NW;
constexpr uint32_t ML_C2I = ML_BWR + 8;
constexpr uint32_t D0_C2I = 20 + ML_C2I;  // data offset (a multiple of 4)
static_assert(D0_C2I % 4 == 0, "C2i data dword-aligned");

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const v4u g_cu4;
typedef __attribute__((address_space(1))) v4u g_u4;
typedef __attribute__((address_space(1))) uint32_t g_u32;

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

template <int CTRL>
__device__ __forceinline__ uint32_t dpp_(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, false);
}

// min and max of a 32-bit value over the wave (signed or unsigned), scalar
template <bool SGN>
__device__ __forceinline__ void wave_minmax32(uint32_t v, uint32_t& mn, uint32_t& mx) {
  uint32_t a = v, b = v;
  auto step = [&](uint32_t x, uint32_t y) {
    if (SGN) {
      a = (int32_t)x < (int32_t)a ? x : a;
      b = (int32_t)y > (int32_t)b ? y : b;
    } else {
      a = x < a ? x : a;
      b = y > b ? y : b;
    }
  };
  step(dpp_<0xB1>(a), dpp_<0xB1>(b));
  step(dpp_<0x4E>(a), dpp_<0x4E>(b));
  step(dpp_<0x141>(a), dpp_<0x141>(b));
  step(dpp_<0x140>(a), dpp_<0x140>(b));
  uint32_t m0 = __builtin_amdgcn_readlane(a, 0), x0 = __builtin_amdgcn_readlane(b, 0);
#pragma unroll
  for (int r = 1; r < 4; r++) {
    const uint32_t m = __builtin_amdgcn_readlane(a, 16 * r), x = __builtin_amdgcn_readlane(b, 16 * r);
    if (SGN) {
      m0 = (int32_t)m < (int32_t)m0 ? m : m0;
      x0 = (int32_t)x > (int32_t)x0 ? x : x0;
    } else {
      m0 = m < m0 ? m : m0;
      x0 = x > x0 ? x : x0;
    }
  }
  mn = m0;
  mx = x0;
}

// compute_bits_required (bit_width_reduction_filter.cc:406-447) for a full
// window of 4-byte elements, in 32 bits: range = max - min is exact as a
// u32 difference; signed: 32 when range > INT32_MAX or range + 1 >
// INT32_MAX.  Returns the width (8 / 16 / 32) and the window offset.
template <bool SGN>
__device__ __forceinline__ uint32_t window_bits(uint32_t mn, uint32_t mx, uint32_t& minv) {
  const uint32_t range = mx - mn;
  minv = 0;
  if (SGN ? range < 0x7fffffffu : range != 0xffffffffu) {
    const uint32_t ro = range + 1;
    minv = mn;
    return ro <= (SGN ? 127u : 255u) ? 8 : ro <= (SGN ? 32767u : 65535u) ? 16 : 32;
  }
  return 32;
}

__device__ __forceinline__ void st32(uint8_t* base, uint32_t off, uint32_t v) {
  *(g_u32*)(base + off) = v;
}
__device__ __forceinline__ void st8(uint8_t* base, uint32_t off, uint32_t v) { base[off] = (uint8_t)v; }

template <int MODE, bool SGN>
__global__ void __launch_bounds__(NT, 2) filter_shuffle4_kernel(const KParams kp) {
  __shared__ uint32_t wsz[NWV];  // C2i: compressed bytes of each wave's 32 windows
  __shared__ uint32_t red[MODE == 2 ? NWV : 1][8][64];  // C2i: a wave's 8 rows being reduced
  uint64_t taken = 0;
  // A grid of at least one workgroup per tile (a multiple of 8): one tile per
  // workgroup, dealt so that each XCD (workgroups go round-robin over the 8)
  // takes a contiguous eighth of the tiles; a smaller grid walks the tiles.
  const uint32_t G = gridDim.x;
  const bool np = G >= kp.ntiles && (G & 7) == 0;
  const uint32_t bid = np ? (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3) : blockIdx.x;
  for (uint64_t j = bid; j < kp.ntiles; j += G) {
    uint32_t T = threadIdx.x;
    asm volatile("" : "+v"(T));
    const uint32_t l = T & 63, w = __builtin_amdgcn_readfirstlane(T >> 6);
    const uint64_t t = j;
    uint8_t* out = kp.out[t];
    const uint64_t cap = kp.out_size[t];
    const bool shape = kp.in_size[t] == TB && (((uintptr_t)kp.in[t]) & 15) == 0 && (((uintptr_t)out) & 15) == 0 &&
                       cap >= 28;
    bool ok = shape;
    uint32_t total = 28 + TB;  // C1, C2 (C2i: set below)
    if (MODE == 2) __syncthreads();  // B0: wsz of the last tile read
    if (shape) {  // (uniform)
      // the lane's 32 elements: 128 B at block w, offset 128 l
      const g_cu4* src = (const g_cu4*)(kp.in[t] + 8192u * w + 128u * l);
      uint32_t d[32];
#pragma unroll
      for (int i = 0; i < 8; i++) {
        const v4u u = src[i];
        d[4 * i] = u.x;
        d[4 * i + 1] = u.y;
        d[4 * i + 2] = u.z;
        d[4 * i + 3] = u.w;
      }
      if (MODE == 0) {
        // ---- byteshuffle: plane p, bytes [32 (256 w + l), +32) = byte p of
        // elements 32 (64 w + l) .. +31 ----
        ok = total <= cap;
        if (ok) {
          uint32_t P[4][8];  // [plane][dword]: 4 elements' byte p
#pragma unroll
          for (int q = 0; q < 8; q++) {
            uint32_t x[4];
            tr4(d[4 * q], d[4 * q + 1], d[4 * q + 2], d[4 * q + 3], x);
#pragma unroll
            for (int p = 0; p < 4; p++) P[p][q] = x[p];
          }
#pragma unroll
          for (int p = 0; p < 4; p++) {
            uint8_t* o = out + 28 + 16384u * p + 32u * (64u * w + l);
            // (4-byte aligned: dword stores)
#pragma unroll
            for (int q = 0; q < 8; q++) st32(o, 4 * q, P[p][q]);
          }
        }
      } else {
        // ---- bitshuffle: the lane's dword of each of the 32 rows ----
        uint32_t R[32];
#pragma unroll
        for (int p = 0; p < 4; p++) {
          uint64_t y[4];
#pragma unroll
          for (int g = 0; g < 4; g++) {
            uint32_t lo[4], hi[4];
            tr4(d[8 * g], d[8 * g + 1], d[8 * g + 2], d[8 * g + 3], lo);
            tr4(d[8 * g + 4], d[8 * g + 5], d[8 * g + 6], d[8 * g + 7], hi);
            // byte m = byte p of element 8 g + m -> byte k = bit k of those
            y[g] = transpose8x8(((uint64_t)hi[p] << 32) | lo[p]);
          }
          uint32_t a[4], b[4];
          tr4((uint32_t)y[0], (uint32_t)y[1], (uint32_t)y[2], (uint32_t)y[3], a);
          tr4((uint32_t)(y[0] >> 32), (uint32_t)(y[1] >> 32), (uint32_t)(y[2] >> 32), (uint32_t)(y[3] >> 32), b);
#pragma unroll
          for (int k = 0; k < 4; k++) {
            R[8 * p + k] = a[k];
            R[8 * p + 4 + k] = b[k];
          }
        }
        if (MODE == 1) {
          ok = total <= cap;
          if (ok) {
            uint8_t* o = out + 28 + 8192u * w + 4u * l;
#pragma unroll
            for (int r = 0; r < 32; r++) st32(o, 256 * r, R[r]);
          }
        } else {
          // ---- C2i: BWR window 32 w + r = row r of this wave's block.  Its
          // min / max: the wave's rows go through its LDS area 8 at a time
          // (lane l then reduces 8 dwords of row l / 8, and 3 DPP steps
          // finish the row in its 8 lanes) instead of 32 full-wave DPP
          // reductions; round q's lane 8 i holds row 8 q + i's width and
          // offset ----
          uint32_t rb[4], rm[4];
          uint32_t wtot = 0;
#pragma unroll
          for (int q = 0; q < 4; q++) {
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int i = 0; i < 8; i++) red[w][i][l] = R[8 * q + i];
            __builtin_amdgcn_wave_barrier();  // (one wave: its LDS operations complete in order)
            const uint32_t row = l >> 3, seg = l & 7;
            const v4u a = *(const v4u*)&red[w][row][8 * seg], b = *(const v4u*)&red[w][row][8 * seg + 4];
            const uint32_t x[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
            uint32_t mn = x[0], mx = x[0];
#pragma unroll
            for (int i = 1; i < 8; i++) {
              if (SGN) {
                mn = (int32_t)x[i] < (int32_t)mn ? x[i] : mn;
                mx = (int32_t)x[i] > (int32_t)mx ? x[i] : mx;
              } else {
                mn = x[i] < mn ? x[i] : mn;
                mx = x[i] > mx ? x[i] : mx;
              }
            }
            auto comb = [&](uint32_t m2, uint32_t x2) {
              if (SGN) {
                mn = (int32_t)m2 < (int32_t)mn ? m2 : mn;
                mx = (int32_t)x2 > (int32_t)mx ? x2 : mx;
              } else {
                mn = m2 < mn ? m2 : mn;
                mx = x2 > mx ? x2 : mx;
              }
            };
            comb(dpp_<0xB1>(mn), dpp_<0xB1>(mx));    // lanes i ^ 1
            comb(dpp_<0x4E>(mn), dpp_<0x4E>(mx));    // lanes i ^ 2
            comb(dpp_<0x141>(mn), dpp_<0x141>(mx));  // row half mirror: lanes 7 - i of the 8
            uint32_t mv;
            rb[q] = window_bits<SGN>(mn, mx, mv);
            rm[q] = mv;
#pragma unroll
            for (int i = 0; i < 8; i++) {
              const uint32_t bits = __builtin_amdgcn_readlane(rb[q], 8 * i);
              wtot += bits == 8 ? 64u : bits == 16 ? 128u : 256u;
            }
          }
          if (l == 0) wsz[w] = wtot;
          __syncthreads();  // B1: every wave's total
          uint32_t pre = 0, dn = 0;
#pragma unroll
          for (int v = 0; v < NWV; v++) {
            const uint32_t x = wsz[v];
            pre += (uint32_t)v < w ? x : 0u;
            dn += x;
          }
          total = D0_C2I + dn;
          ok = total <= cap;
          if (ok) {
            if (T == 0) {
              st32(out, 0, 1);
              st32(out, 4, 0);
              st32(out, 8, TB);
              st32(out, 12, dn);
              st32(out, 16, ML_C2I);
              st32(out, 20, TB);  // BWR md: orig, windows
              st32(out, 24, NW);
              st32(out, 20 + ML_BWR, 1);  // bitshuffle md: one part of 65,536 B
              st32(out, 24 + ML_BWR, TB);
            }
            if ((l & 7) == 0) {  // windows 32 w + 8 q + l / 8: md entries [i32 min][u8 bits][u32 256] (9 B)
#pragma unroll
              for (int q = 0; q < 4; q++) {
                const uint32_t eo = 28 + 9 * (32 * w + 8 * q + (l >> 3));
#pragma unroll
                for (int i = 0; i < 4; i++) st8(out, eo + i, rm[q] >> (8 * i));
                st8(out, eo + 4, rb[q]);
                st8(out, eo + 5, 0);
                st8(out, eo + 6, 1);
                st8(out, eo + 7, 0);
                st8(out, eo + 8, 0);
              }
            }
            // the windows' data, in order (offsets: multiples of 4)
            uint32_t off = D0_C2I + pre;
#pragma unroll
            for (int r = 0; r < 32; r++) {
              const uint32_t bits = __builtin_amdgcn_readlane(rb[r >> 3], 8 * (r & 7));
              const uint32_t rel = R[r] - __builtin_amdgcn_readlane(rm[r >> 3], 8 * (r & 7));
              if (bits == 32) {
                st32(out, off + 4 * l, R[r]);
                off += 256;
              } else if (bits == 16) {
                const uint32_t nb = dpp_<0xB1>(rel);  // the pair's other lane
                if ((l & 1) == 0) st32(out, off + 2 * l, (rel & 0xffffu) | (nb << 16));
                off += 128;
              } else {
                const uint32_t q1 = dpp_<0xB1>(rel), q2 = dpp_<0x4E>(rel), q3 = dpp_<0x1B>(rel);
                if ((l & 3) == 0)
                  st32(out, off + l, (rel & 0xffu) | ((q1 & 0xffu) << 8) | ((q2 & 0xffu) << 16) | (q3 << 24));
                off += 64;
              }
            }
          }
        }
      }
      if (ok && T == 0) {
        if (kp.status) kp.status[t] = TDBG_OK;
        if (kp.need) kp.need[t] = 0;
        if (kp.out_len) kp.out_len[t] = total;
      }
      if (MODE != 2 && ok && T == 0) {
        // C1, C2: headers [u64 1][u32 65536][u32 65536][u32 8][u32 1][u32 65536]
        st32(out, 0, 1);
        st32(out, 4, 0);
        st32(out, 8, TB);
        st32(out, 12, TB);
        st32(out, 16, 8);
        st32(out, 20, 1);
        st32(out, 24, TB);
      }
    }
    if (ok) taken++;
    if (!ok && T == 0) {
      const uint32_t k = atomicAdd(kp.fbq, 1u);
      if (k < kp.fbq_cap) kp.fbq[1 + k] = (uint32_t)t;
      else if (kp.status) kp.status[t] = TDBG_E_INTERNAL;
    }
  }
  if (kp.stats && threadIdx.x == 0 && taken)
    atomicAdd((unsigned long long*)&kp.stats[TDBG_STAT_STRIDE * (1 + (blockIdx.x & 63)) + TDBG_STAT_FWD_STREAM_TILES],
              (unsigned long long)taken);  // (one slot per 64 workgroups: tdbg_host.cpp read_stats sums them)
}

}  // namespace fsh
}  // namespace tdbg

// mode 0 [BYTESHUFFLE], 1 [BITSHUFFLE] (+ pass-through BWR), 2 [BITSHUFFLE,
// BWR(256)] on 4-byte integers (sgn: signed)
extern "C" hipError_t tdbg_launch_filter_shuffle4(const tdbg::KParams* kp, uint32_t grid, int mode, int sgn,
                                                  hipStream_t s) {
  using namespace tdbg::fsh;
  if (mode == 0) hipLaunchKernelGGL((filter_shuffle4_kernel<0, false>), dim3(grid), dim3(NT), 0, s, *kp);
  else if (mode == 1) hipLaunchKernelGGL((filter_shuffle4_kernel<1, false>), dim3(grid), dim3(NT), 0, s, *kp);
  else if (sgn) hipLaunchKernelGGL((filter_shuffle4_kernel<2, true>), dim3(grid), dim3(NT), 0, s, *kp);
  else hipLaunchKernelGGL((filter_shuffle4_kernel<2, false>), dim3(grid), dim3(NT), 0, s, *kp);
  return hipGetLastError();
}
