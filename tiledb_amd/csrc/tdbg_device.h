// tdbg_device.h -- device helpers for the gfx950 unfilter kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/tiledb_amd.h"
#include "tdbg_rules.h"

#define GEN_NT 256  // threads per workgroup, general interpreter (4 wave64)
#define DD_EPT 8    // double-delta elements per thread per round

namespace tdbg {

// ---- byte access at arbitrary alignment ----------------------------------
// Loads k (1..8) little-endian bytes at p.  Only dwords that contain a
// requested byte are touched, so a read never crosses into a page that holds
// none of the requested bytes (safe at the end of a global allocation).
__device__ __forceinline__ uint64_t ldn(const uint8_t* p, uint32_t k) {
  const uintptr_t a = (uintptr_t)p;
  const uint32_t* q = (const uint32_t*)(a & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(a & 3);
  const uint32_t nd = (sh + k + 3) >> 2;
  const uint32_t d0 = q[0];
  const uint32_t d1 = nd > 1 ? q[1] : 0u;
  const uint32_t d2 = nd > 2 ? q[2] : 0u;
  const uint32_t lo = __builtin_amdgcn_alignbyte(d1, d0, sh);
  const uint32_t hi = __builtin_amdgcn_alignbyte(d2, d1, sh);
  uint64_t v = ((uint64_t)hi << 32) | lo;
  if (k < 8) v &= (1ull << (8 * k)) - 1;
  return v;
}

__device__ __forceinline__ void stn(uint8_t* p, uint64_t v, uint32_t k) {
  const uintptr_t a = (uintptr_t)p;
  if (k == 8 && (a & 7) == 0) { *(uint64_t*)p = v; return; }
  if (k == 4 && (a & 3) == 0) { *(uint32_t*)p = (uint32_t)v; return; }
  if (k == 2 && (a & 1) == 0) { *(uint16_t*)p = (uint16_t)v; return; }
  for (uint32_t i = 0; i < k; i++) p[i] = (uint8_t)(v >> (8 * i));
}

__host__ __device__ __forceinline__ uint64_t wmask(uint32_t w) {
  return w >= 8 ? ~0ull : ((1ull << (8 * w)) - 1);
}
__host__ __device__ __forceinline__ int64_t sext64(uint64_t v, uint32_t w) {
  if (w >= 8) return (int64_t)v;
  const uint32_t s = 64 - 8 * w;
  return (int64_t)(v << s) >> s;
}

// 8x8 bit-matrix transpose: bit (8i+j) <-> bit (8j+i) (Hacker's Delight).
__host__ __device__ __forceinline__ uint64_t transpose8x8(uint64_t x) {
  uint64_t t;
  t = (x ^ (x >> 7)) & 0x00AA00AA00AA00AAull;
  x = x ^ t ^ (t << 7);
  t = (x ^ (x >> 14)) & 0x0000CCCC0000CCCCull;
  x = x ^ t ^ (t << 14);
  t = (x ^ (x >> 28)) & 0x00000000F0F0F0F0ull;
  x = x ^ t ^ (t << 28);
  return x;
}

// ---- wave64 / block scans --------------------------------------------------
// Wave scans run on DPP lane moves (VALU, no LDS round trip): row_shr:1,2,4,8
// scan each 16-lane row, row_bcast:15 / row_bcast:31 carry rows 0->1, 2->3
// and 0-1 -> 2-3.  Lanes with no source read 0 (old = 0, bound_ctrl).
enum : int {
  DPP_ROW_SHR1 = 0x111, DPP_ROW_SHR2 = 0x112, DPP_ROW_SHR4 = 0x114, DPP_ROW_SHR8 = 0x118,
  DPP_ROW_BCAST15 = 0x142, DPP_ROW_BCAST31 = 0x143
};
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ uint32_t dpp0(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWS, 0xf, true);
}
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ uint64_t dpp0(uint64_t v) {
  return (uint64_t)dpp0<CTRL, ROWS>((uint32_t)v) | ((uint64_t)dpp0<CTRL, ROWS>((uint32_t)(v >> 32)) << 32);
}
// the six steps; the bcast steps write only the rows named (0xa: rows 1, 3;
// 0xc: rows 2, 3), every other lane reads 0
template <class T, class F>
__device__ __forceinline__ void wave_scan_steps(T& x, F&& comb) {
  comb(dpp0<DPP_ROW_SHR1>(x), 1);
  comb(dpp0<DPP_ROW_SHR2>(x), 2);
  comb(dpp0<DPP_ROW_SHR4>(x), 4);
  comb(dpp0<DPP_ROW_SHR8>(x), 8);
  comb(dpp0<DPP_ROW_BCAST15, 0xa>(x), 15);
  comb(dpp0<DPP_ROW_BCAST31, 0xc>(x), 31);
}

__device__ __forceinline__ uint64_t wave_incscan_u64(uint64_t x) {
  wave_scan_steps(x, [&](uint64_t y, int) { x += y; });
  return x;
}
__device__ __forceinline__ uint32_t wave_incscan_u32(uint32_t x) {
  wave_scan_steps(x, [&](uint32_t y, int) { x += y; });
  return x;
}

// Inclusive prefix XOR of one u64 per thread over the workgroup (XOR
// filter); total = XOR of all; red >= NT/64 entries of LDS.
template <int NT = GEN_NT>
__device__ __forceinline__ uint64_t block_incscan_xor(uint64_t x, uint64_t& total, uint64_t* red) {
  const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t y = __shfl_up(x, d, 64);
    if (lane >= (uint32_t)d) x ^= y;
  }
  if (lane == 63) red[wid] = x;
  __syncthreads();
  uint64_t pre = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < NT / 64; i++) {
    const uint64_t s = red[i];
    if ((uint32_t)i < wid) pre ^= s;
    tot ^= s;
  }
  __syncthreads();
  total = tot;
  return pre ^ x;
}

// Exclusive block scan of one u64 per thread; red >= NT/64 entries of LDS.
template <int NT = GEN_NT>
__device__ __forceinline__ uint64_t block_exscan_u64(uint64_t v, uint64_t& total,
                                                     uint64_t* red) {
  const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint64_t inc = wave_incscan_u64(v);
  if (lane == 63) red[wid] = inc;
  __syncthreads();
  uint64_t pre = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < NT / 64; i++) {
    const uint64_t s = red[i];
    if ((uint32_t)i < wid) pre += s;
    tot += s;
  }
  __syncthreads();
  total = tot;
  return pre + inc - v;
}

template <int NT = GEN_NT>
__device__ __forceinline__ uint64_t block_min_u64(uint64_t v, uint64_t* red) {
  const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const uint64_t y = __shfl_xor(v, d, 64);
    v = y < v ? y : v;
  }
  if (lane == 0) red[wid] = v;
  __syncthreads();
  uint64_t m = ~0ull;
#pragma unroll
  for (int i = 0; i < NT / 64; i++) m = red[i] < m ? red[i] : m;
  __syncthreads();
  return m;
}

// Code of value i (j = i - 2) at bit s = j*(b+1) of the MSB-first u64 word
// stream: sign bit then b magnitude bits (dd_compressor.cc:356-404).
__device__ __forceinline__ uint64_t dd_code(const uint8_t* bs, uint64_t s, uint32_t b) {
  const uint64_t wi = s >> 6;
  const uint32_t r = (uint32_t)(s & 63);
  uint64_t hi = ldn(bs + 8 * wi, 8) << r;
  if (r + b + 1 > 64) hi |= ldn(bs + 8 * (wi + 1), 8) >> (64 - r);
  const uint64_t code = hi >> (63 - b);
  const uint64_t mag = b ? (code & ((1ull << b) - 1)) : 0;
  return ((code >> b) & 1) ? (0 - mag) : mag;
}

// ---- double-delta second-order tuple scan ----------------------------------
// For a run of n elements with first differences e: E = sum e,
// X = sum_m sum_{k<=m} e_k.  Concatenating A then B (n_B elements):
// E = E_A + E_B, X = X_A + X_B + n_B * E_A.
struct DDAgg { uint64_t E, X; };
struct DDCarry { uint64_t E, X; };

__device__ __forceinline__ DDAgg dd_local(const uint64_t (&e)[DD_EPT]) {
  DDAgg a = {0, 0};
#pragma unroll
  for (int k = 0; k < DD_EPT; k++) { a.E += e[k]; a.X += a.E; }
  return a;
}

// Exclusive scan of DDAgg over the block (each thread = DD_EPT elements).
// Writes the whole-round aggregate to `total`.
template <int NT = GEN_NT>
__device__ __forceinline__ DDAgg block_ddscan2(DDAgg a, DDAgg& total, uint64_t* red) {
  const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  DDAgg inc = a;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t oE = __shfl_up(inc.E, d, 64);
    const uint64_t oX = __shfl_up(inc.X, d, 64);
    if (lane >= (uint32_t)d) {
      inc.X = oX + inc.X + (uint64_t)d * DD_EPT * oE;
      inc.E = oE + inc.E;
    }
  }
  DDAgg ex;
  ex.E = __shfl_up(inc.E, 1, 64);
  ex.X = __shfl_up(inc.X, 1, 64);
  if (lane == 0) { ex.E = 0; ex.X = 0; }
  if (lane == 63) { red[2 * wid] = inc.E; red[2 * wid + 1] = inc.X; }
  __syncthreads();
  DDAgg P = {0, 0}, T = {0, 0};
#pragma unroll
  for (int i = 0; i < NT / 64; i++) {
    const uint64_t wE = red[2 * i], wX = red[2 * i + 1];
    if ((uint32_t)i < wid) { P.X = P.X + wX + 64ull * DD_EPT * P.E; P.E += wE; }
    T.X = T.X + wX + 64ull * DD_EPT * T.E;
    T.E += wE;
  }
  __syncthreads();
  DDAgg r;
  r.E = P.E + ex.E;
  r.X = P.X + ex.X + (uint64_t)lane * DD_EPT * P.E;
  total = T;
  return r;
}

}  // namespace tdbg
