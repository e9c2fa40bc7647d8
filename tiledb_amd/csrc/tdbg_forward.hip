// tdbg_forward.hip -- forward ("filter") direction on gfx950: the write path
// WriterBase::filter_tile -> FilterPipeline::run_forward
// (writer_base.cc:870-915, filter_pipeline.cc:208-369,382-426) with every
// filter's run_forward: byteshuffle, bitshuffle, bit-width reduction,
// positive delta, the compression filter with DoubleDelta / RLE / Delta,
// XOR and float scaling.
//
// Work decomposition: a persistent grid of 256-thread workgroups, one tile
// at a time per workgroup; the tile's chunks (WriterTile::compute_chunk_size,
// tile.cc:87-100) run in order so each chunk's output offset is known when it
// is written: [u64 nchunks] then per chunk [u32 orig][u32 filtered][u32 md]
// [md][data] (filter_pipeline.cc:332-363).  Within a chunk the filters run in
// pipeline order, every filter block-parallel, intermediates in the
// workgroup's global scratch slot (L2/MALL resident).
//
// FilterBuffer model (filter_buffer.cc): after every forward filter the data
// is ONE buffer (each filter concatenates its output parts); the metadata is
// a list of parts, newest first, kept back to back at the END of a metadata
// buffer so a prepend is a pointer move.  A compression filter compresses
// every metadata part and the data part (compression_filter.cc:240-301) and
// replaces the metadata with its frame header.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/tiledb_amd.h"
#include "tdbg_desc.h"
#include "tdbg_device.h"

namespace tdbg {

constexpr int FNT_F = 256;
constexpr uint32_t FWD_MAXMD = 48;

struct FwdShared {
  uint64_t red[FNT_F / 64 * 2 + 8];
  uint32_t md_len[FWD_MAXMD];  // metadata parts, newest (front) first
  uint32_t md_n, md_start;     // parts occupy md[md_start, md_cap)
  uint32_t flag[4];
  uint64_t bcast[4];
};

struct FwdSlot {
  uint8_t* buf[2];
  uint8_t* md[2];
  uint64_t* tab;
  uint64_t buf_cap, md_cap, tab_cap;  // bytes; tab_cap in bytes
};

// ---- block helpers ---------------------------------------------------------
__device__ __forceinline__ uint64_t blk_max_u64(uint64_t v, uint64_t* red) {
  const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const uint64_t y = __shfl_xor(v, d, 64);
    v = y > v ? y : v;
  }
  if (lane == 0) red[wid] = v;
  __syncthreads();
  uint64_t m = 0;
#pragma unroll
  for (int i = 0; i < FNT_F / 64; i++) m = red[i] > m ? red[i] : m;
  __syncthreads();
  return m;
}

__device__ __forceinline__ bool blk_any(bool p) { return __syncthreads_or(p ? 1 : 0) != 0; }

__device__ __forceinline__ void blk_copy(uint8_t* dst, const uint8_t* src, uint64_t n) {
  if (((((uintptr_t)dst) | ((uintptr_t)src)) & 3) == 0) {
    const uint64_t nd = n >> 2;
    for (uint64_t i = threadIdx.x; i < nd; i += FNT_F) ((uint32_t*)dst)[i] = ((const uint32_t*)src)[i];
    for (uint64_t i = (nd << 2) + threadIdx.x; i < n; i += FNT_F) dst[i] = src[i];
  } else {
    for (uint64_t i = threadIdx.x; i < n; i += FNT_F) dst[i] = src[i];
  }
}

// wave-level min / max of 64 lanes (signed or unsigned 64-bit)
template <bool SGN>
__device__ __forceinline__ void wave_minmax(uint64_t& mn, uint64_t& mx) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const uint64_t a = __shfl_xor(mn, d, 64), b = __shfl_xor(mx, d, 64);
    if (SGN) {
      mn = (int64_t)a < (int64_t)mn ? a : mn;
      mx = (int64_t)b > (int64_t)mx ? b : mx;
    } else {
      mn = a < mn ? a : mn;
      mx = b > mx ? b : mx;
    }
  }
}

// ---- byteshuffle forward (blosc2 shuffle; byteshuffle_filter.cc:60-89) ------
__device__ void f_byteshuffle_fwd(uint8_t* out, const uint8_t* in, uint64_t n, uint32_t ts) {
  if (ts <= 1) { blk_copy(out, in, n); return; }
  const uint64_t N = n / ts;
  for (uint64_t i = threadIdx.x; i < N; i += FNT_F) {
    const uint64_t v = ldn(in + i * ts, ts);
    for (uint32_t j = 0; j < ts; j++) out[j * N + i] = (uint8_t)(v >> (8 * j));
  }
  for (uint64_t i = N * ts + threadIdx.x; i < n; i += FNT_F) out[i] = in[i];
}

// ---- bitshuffle forward of one part (bitshuffle_filter.cc:128-166) --------
__device__ void f_bitshuffle_part_fwd(uint8_t* out, const uint8_t* in, uint64_t n, uint32_t ts) {
  if (n % ts != 0 || n % 8 != 0) { blk_copy(out, in, n); return; }
  for (uint64_t b0 = 0; b0 < n; b0 += 8192) {
    const uint64_t nb = n - b0 < 8192 ? n - b0 : 8192;
    const uint64_t ne = nb / ts, n8 = ne - ne % 8, rowb = n8 / 8;
    const uint8_t* s = in + b0;
    uint8_t* d = out + b0;
    const uint64_t items = rowb * ts;
    for (uint64_t it = threadIdx.x; it < items; it += FNT_F) {
      const uint64_t q = it / ts;
      const uint32_t b = (uint32_t)(it % ts);
      uint64_t x = 0;
      for (uint32_t m = 0; m < 8; m++) x |= (uint64_t)s[(8 * q + m) * ts + b] << (8 * m);
      const uint64_t y = transpose8x8(x);
      for (uint32_t k = 0; k < 8; k++) d[(8ull * b + k) * rowb + q] = (uint8_t)(y >> (8 * k));
    }
    for (uint64_t i = n8 * ts + threadIdx.x; i < nb; i += FNT_F) d[i] = s[i];
  }
}

// ---- XOR forward (xor_filter.cc:149-177): out[j] = in[j] ^ in[j-1] --------
__device__ void f_xor_fwd(uint8_t* out, const uint8_t* in, uint64_t n, uint32_t ts) {
  const uint64_t ne = n / ts;
  for (uint64_t j = threadIdx.x; j < ne; j += FNT_F) {
    const uint64_t v = ldn(in + j * ts, ts);
    const uint64_t p = j ? ldn(in + (j - 1) * ts, ts) : 0;
    stn(out + j * ts, v ^ p, ts);
  }
  for (uint64_t i = ne * ts + threadIdx.x; i < n; i += FNT_F) out[i] = 0;  // as the oracle
}

// ---- float scaling forward (float_scaling_filter.cc:60-99) ----------------
__device__ void f_fscale_fwd(uint8_t* out, const uint8_t* in, uint64_t ne, uint32_t ts, uint32_t bw,
                             double sc, double of) {
  for (uint64_t j = threadIdx.x; j < ne; j += FNT_F) {
    int64_t q;
    if (ts == 4) {
      const float x = __uint_as_float((uint32_t)ldn(in + 4 * j, 4));
      q = (int64_t)roundf(__fdiv_rn(__fsub_rn(x, (float)of), (float)sc));
    } else {
      const double x = __longlong_as_double((long long)ldn(in + 8 * j, 8));
      q = (int64_t)round(__ddiv_rn(__dsub_rn(x, of), sc));
    }
    stn(out + bw * j, (uint64_t)q, bw);
  }
}

// ---- BWR forward (bit_width_reduction_filter.cc:110-280, 406-447) ---------
// md [u32 orig][u32 nwin] + nwin x [T offset][u8 bits][u32 nbytes]; one data
// buffer.  tab[2k] = compressed bytes of window k (then its output offset),
// tab[2k+1] = bits | offset << 8 is recomputed, not stored.
template <int W, bool SGN>
__device__ int64_t f_bwr_fwd(uint8_t* out, const uint8_t* in, uint32_t ps, uint32_t ws, uint32_t nw,
                             uint8_t* md, uint64_t* tab, FwdShared& sh) {
  const uint32_t E = W + 5;
  if (threadIdx.x == 0) {
    stn(md, ps, 4);
    stn(md + 4, nw, 4);
  }
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t mw = wmask(W);
  // pass 1: per window (one wave each) min / max -> bits, offset; md entry
  for (uint32_t k = wave; k < nw; k += FNT_F / 64) {
    const uint32_t nb = ws < ps - k * ws ? ws : ps - k * ws;
    const uint32_t ne = nb / W;
    const uint8_t* wp = in + (uint64_t)k * ws;
    uint64_t mn = SGN ? (uint64_t)INT64_MAX : ~0ull, mx = SGN ? (uint64_t)INT64_MIN : 0ull;
    for (uint32_t j = lane; j < ne; j += 64) {
      uint64_t v = ldn(wp + (uint64_t)j * W, W);
      if (SGN) v = (uint64_t)sext64(v, W);
      if (SGN) {
        mn = (int64_t)v < (int64_t)mn ? v : mn;
        mx = (int64_t)v > (int64_t)mx ? v : mx;
      } else {
        mn = v < mn ? v : mn;
        mx = v > mx ? v : mx;
      }
    }
    wave_minmax<SGN>(mn, mx);
    uint32_t bits = 8 * W;
    uint64_t minv = 0;
    if (ne > 0) {
      if (SGN) {
        const int64_t smn = (int64_t)mn, smx = (int64_t)mx;
        bool ovf = false;
        int64_t range = 0;
        if (W < 8) {
          range = smx - smn;
          const int64_t lim = (int64_t)(mw >> 1);
          ovf = range > lim || range + 1 > lim;
        } else {
          ovf = __builtin_sub_overflow(smx, smn, &range) || range == INT64_MAX;
        }
        if (!ovf) {
          const int64_t ro = range + 1;
          bits = ro <= 127 ? 8 : ro <= 32767 ? 16 : ro <= 2147483647LL ? 32 : 64;
          minv = mn;
        }
      } else {
        const uint64_t range = mx - mn;
        if (range != mw) {
          const uint64_t ro = range + 1;
          const uint32_t nbits = 64 - __clzll(ro);
          bits = nbits <= 8 ? 8 : nbits <= 16 ? 16 : nbits <= 32 ? 32 : 64;
          minv = mn;
        }
      }
    }
    const bool raw = bits >= 8u * W || nb % W != 0;
    if (lane == 0) {
      uint8_t* e = md + 8 + (uint64_t)k * E;
      stn(e, minv, W);
      e[W] = (uint8_t)bits;
      stn(e + W + 1, nb, 4);
      tab[2 * k] = raw ? nb : (uint64_t)ne * (bits / 8);
      tab[2 * k + 1] = (minv & mw) | ((uint64_t)0);  // offset (bits from md)
    }
  }
  __syncthreads();
  // pass 2: exclusive scan of compressed sizes -> output offsets
  uint64_t carry = 0;
  for (uint32_t b = 0; b < nw; b += FNT_F) {
    const uint32_t k = b + threadIdx.x;
    const uint64_t c = k < nw ? tab[2 * k] : 0;
    uint64_t tot;
    const uint64_t ex = carry + block_exscan_u64<FNT_F>(c, tot, sh.red);
    if (k < nw) tab[2 * k] = ex;
    carry += tot;
  }
  __syncthreads();
  // pass 3: per window (one wave each) write the data
  for (uint32_t k = wave; k < nw; k += FNT_F / 64) {
    const uint32_t nb = ws < ps - k * ws ? ws : ps - k * ws;
    const uint32_t ne = nb / W;
    const uint8_t* wp = in + (uint64_t)k * ws;
    const uint32_t bits = md[8 + (uint64_t)k * E + W];
    const uint64_t minv = tab[2 * k + 1];
    uint8_t* op = out + tab[2 * k];
    if (bits >= 8u * W || nb % W != 0) {
      for (uint32_t j = lane; j < nb; j += 64) op[j] = wp[j];
    } else {
      const uint32_t cb = bits / 8;
      for (uint32_t j = lane; j < ne; j += 64) {
        const uint64_t rel = (ldn(wp + (uint64_t)j * W, W) - minv) & mw;
        stn(op + (uint64_t)j * cb, rel, cb);
      }
    }
  }
  __syncthreads();
  return (int64_t)carry;
}

// ---- positive delta forward (positive_delta_filter.cc:140-245) -------------
// md [u32 nwin] + nwin x [T first][u32 nbytes]; deltas, d[0] = 0.
template <int W, bool SGN>
__device__ int f_pd_fwd(uint8_t* out, const uint8_t* in, uint32_t ps, uint32_t ws, uint32_t nw, uint8_t* md,
                        FwdShared& sh) {
  const uint32_t E = W + 4;
  if (threadIdx.x == 0) stn(md, nw, 4);
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t mw = wmask(W);
  bool bad = false;
  for (uint32_t k = wave; k < nw; k += FNT_F / 64) {
    const uint32_t nb = ws < ps - k * ws ? ws : ps - k * ws;
    const uint8_t* wp = in + (uint64_t)k * ws;
    uint8_t* op = out + (uint64_t)k * ws;
    if (lane == 0) {
      // value<T>() reads past a short last window (:217): zero-filled here
      const uint32_t avail = nb < W ? nb : W;
      uint64_t first = 0;
      for (uint32_t b = 0; b < avail; b++) first |= (uint64_t)wp[b] << (8 * b);
      uint8_t* e = md + 4 + (uint64_t)k * E;
      stn(e, first, W);
      stn(e + W, nb, 4);
    }
    if (nb % W != 0) {
      for (uint32_t j = lane; j < nb; j += 64) op[j] = wp[j];
    } else {
      const uint32_t ne = nb / W;
      for (uint32_t j = lane; j < ne; j += 64) {
        const uint64_t cur = ldn(wp + (uint64_t)j * W, W);
        const uint64_t prev = j ? ldn(wp + (uint64_t)(j - 1) * W, W) : cur;
        const bool lt = SGN ? (sext64(cur, W) < sext64(prev, W)) : (cur < prev);
        bad |= lt;
        stn(op + (uint64_t)j * W, (cur - prev) & mw, W);
      }
    }
  }
  return blk_any(bad) ? TDBG_E_PD_DECREASING : TDBG_OK;
}

// ---- DoubleDelta::compress<T> of one part (dd_compressor.cc:211-312) -------
// [u8 bitsize][u64 num] + raw part, or [T x0][T x1] + (num-2) codes of
// (1 + bitsize) bits, MSB-first in little-endian u64 words.  Returns the
// status; *clen = compressed bytes.  Checked deltas as in the reference's
// compute_bitsize (arithmetic.h; tdb_oracle.c dd_delta).
__device__ __forceinline__ bool dd_delta_chk(uint64_t cur, uint64_t prev, uint32_t w, bool sgn,
                                             int64_t* d) {
  if (sgn || w < 8) {
    if (w < 8) {
      const int64_t a = sgn ? sext64(cur, w) : (int64_t)cur;
      const int64_t b = sgn ? sext64(prev, w) : (int64_t)prev;
      *d = a - b;
      return true;
    }
    return !__builtin_sub_overflow((int64_t)cur, (int64_t)prev, d);
  }
  if (cur >= prev) {
    const uint64_t r = cur - prev;
    if (r > (uint64_t)INT64_MAX) return false;
    *d = (int64_t)r;
    return true;
  }
  const uint64_t r = prev - cur;
  if (r > (uint64_t)INT64_MAX) {
    if (r == (uint64_t)INT64_MAX + 1) { *d = INT64_MIN; return true; }
    return false;
  }
  *d = -(int64_t)r;
  return true;
}

__device__ __forceinline__ uint64_t uabs64_(int64_t v) { return v < 0 ? 0 - (uint64_t)v : (uint64_t)v; }

__device__ int64_t f_dd_fwd(uint8_t* out, uint64_t cap, const uint8_t* in, uint64_t n, uint32_t w,
                            bool sgn, FwdShared& sh) {
  if (w == 0) return -TDBG_E_DD_TYPE;
  const uint64_t num = n / w;
  if (num == 0) return -TDBG_E_ARG;  // iassert(num > 0) dd_compressor.cc:216
  uint32_t bitsize = 0;
  bool ovf_any = false;
  if (num > 2) {
    uint64_t mx = 0;
    bool ovf = false;
    for (uint64_t i = 1 + threadIdx.x; i < num; i += FNT_F) {
      int64_t d, dp = 0, dd;
      ovf |= !dd_delta_chk(ldn(in + i * w, w), ldn(in + (i - 1) * w, w), w, sgn, &d);
      if (i == 1) {
        const uint64_t a = uabs64_(d);
        mx = a > mx ? a : mx;
      } else {
        ovf |= !dd_delta_chk(ldn(in + (i - 1) * w, w), ldn(in + (i - 2) * w, w), w, sgn, &dp);
        ovf |= __builtin_sub_overflow(d, dp, &dd);
        const uint64_t a = uabs64_(dd);
        mx = a > mx ? a : mx;
      }
    }
    ovf_any = blk_any(ovf);
    mx = blk_max_u64(mx, sh.red);
    bitsize = 64 - (mx ? __clzll(mx) : 63);  // do { ++b; m >>= 1; } while (m)
  }
  const bool raw = bitsize >= 8 * w - 1;
  const uint32_t cb = bitsize + 1;
  const uint64_t words = (!raw && num > 2) ? ((num - 2) * cb + 63) / 64 : 0;
  const uint64_t total = raw ? 9 + n : 9 + w * (num < 2 ? num : 2) + 8 * words;
  int64_t res = (int64_t)total;
  if (ovf_any) res = -TDBG_E_DD_OVERFLOW;
  else if (total > cap) res = -TDBG_E_OUT_FULL;
  if (res >= 0) {
    if (threadIdx.x == 0) {
      out[0] = (uint8_t)bitsize;
      stn(out + 1, num, 8);
    }
    if (raw) {
      blk_copy(out + 9, in, n);
    } else {
      if (threadIdx.x == 0) {
        stn(out + 9, ldn(in, w), w);
        if (num > 1) stn(out + 9 + w, ldn(in + w, w), w);
      }
      // word-owner packing: word wi holds bits [64 wi, 64 wi + 64) of the
      // code stream; code j (value i = j + 2) occupies bits [j cb, j cb + cb)
      uint8_t* bs = out + 9 + 2 * w;
      const uint64_t ncode = num - 2;
      for (uint64_t wi = threadIdx.x; wi < words; wi += FNT_F) {
        uint64_t word = 0;
        const uint64_t lo = (64 * wi) / cb, hi = (64 * wi + 63) / cb;
        for (uint64_t j = lo; j <= hi && j < ncode; j++) {
          const uint64_t i = j + 2;
          const uint64_t a = ldn(in + i * w, w), b = ldn(in + (i - 1) * w, w), c = ldn(in + (i - 2) * w, w);
          const int64_t x0 = sgn ? sext64(a, w) : (int64_t)a, x1 = sgn ? sext64(b, w) : (int64_t)b,
                        x2 = sgn ? sext64(c, w) : (int64_t)c;
          const int64_t curd = (int64_t)((uint64_t)x0 - (uint64_t)x1);
          const int64_t prevd = (int64_t)((uint64_t)x1 - (uint64_t)x2);
          const int64_t dd = (int64_t)((uint64_t)curd - (uint64_t)prevd);
          const uint64_t code = ((uint64_t)(dd < 0 ? 1 : 0) << bitsize) | uabs64_(dd);
          const int64_t p = (int64_t)(j * cb) - (int64_t)(64 * wi);  // code start within the word
          const int64_t shl = 64 - p - (int64_t)cb;
          word |= shl >= 0 ? (shl < 64 ? code << shl : 0ull) : code >> (-shl);
        }
        stn(bs + 8 * wi, word, 8);
      }
    }
  }
  __syncthreads();
  return res;
}

// ---- Delta::compress<T> of one part (delta_compressor.cc:224-249) ----------
__device__ int64_t f_delta_fwd(uint8_t* out, uint64_t cap, const uint8_t* in, uint64_t n, uint32_t w) {
  if (w == 0) return -TDBG_E_DELTA_TYPE;
  const uint64_t num = n / w, nv = num ? num : 1;
  const uint64_t total = 8 + nv * w;
  if (total > cap) return -TDBG_E_OUT_FULL;
  if (threadIdx.x == 0) {
    stn(out, num, 8);
    stn(out + 8, num ? ldn(in, w) : 0, w);
  }
  const uint64_t m = wmask(w);
  for (uint64_t i = 1 + threadIdx.x; i < num; i += FNT_F)
    stn(out + 8 + i * w, (ldn(in + i * w, w) - ldn(in + (i - 1) * w, w)) & m, w);
  __syncthreads();
  return (int64_t)total;
}

// ---- RLE::compress (rle_compressor.cc:51-101) -------------------------------
// runs of equal cs-byte values, split at 65535: record [value][len>>8][len&255].
// heads: i == 0, a value change, or (i - run start) % 65535 == 0; tab holds
// the head positions, then each head writes its record.
__device__ bool cells_eq(const uint8_t* a, const uint8_t* b, uint64_t cs) {
  if (cs <= 8) return ldn(a, (uint32_t)cs) == ldn(b, (uint32_t)cs);
  for (uint64_t k = 0; k < cs; k++)
    if (a[k] != b[k]) return false;
  return true;
}

__device__ int64_t f_rle_fwd(uint8_t* out, uint64_t cap, const uint8_t* in, uint64_t n, uint64_t cs,
                             uint64_t* tab, uint64_t tab_cap, FwdShared& sh, uint64_t* need) {
  const uint64_t nv = n / cs;
  if (nv == 0) return 0;
  if (n % cs) return -TDBG_E_RLE_FORMAT;
  if ((nv + 1) * 8 > tab_cap) { *need = (nv + 1) * 8 + 256; return -TDBG_E_SCRATCH; }
  // pass 1: run starts (value changes) -> the start of each element's run
  // (running max over the block), heads at start + 65535 k
  uint64_t carry_start = 0, carry_heads = 0;
  for (uint64_t b = 0; b < nv; b += FNT_F) {
    const uint64_t i = b + threadIdx.x;
    const bool valid = i < nv;
    const bool chg = valid && (i == 0 || !cells_eq(in + i * cs, in + (i - 1) * cs, cs));
    // inclusive max-scan of change positions
    uint64_t st = chg ? i : 0;
    {
      const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(st, d, 64);
        if (lane >= (uint32_t)d) st = y > st ? y : st;
      }
      if (lane == 63) sh.red[wid] = st;
      __syncthreads();
      uint64_t pre = carry_start;
      for (uint32_t k = 0; k < wid; k++) pre = sh.red[k] > pre ? sh.red[k] : pre;
      uint64_t tot = carry_start;
#pragma unroll
      for (int k = 0; k < FNT_F / 64; k++) tot = sh.red[k] > tot ? sh.red[k] : tot;
      __syncthreads();
      st = pre > st ? pre : st;
      carry_start = tot;
    }
    const bool head = valid && (chg || (i - st) % 65535 == 0);
    uint64_t tot;
    const uint64_t r = carry_heads + block_exscan_u64<FNT_F>(head ? 1 : 0, tot, sh.red);
    if (head) tab[r] = i;
    carry_heads += tot;
  }
  const uint64_t nr = carry_heads;
  const uint64_t rs = cs + 2;
  const bool fits = nr * rs <= cap;
  if (threadIdx.x == 0) tab[nr] = nv;
  __syncthreads();
  for (uint64_t r = threadIdx.x; fits && r < nr; r += FNT_F) {
    const uint64_t i = tab[r], len = tab[r + 1] - i;
    uint8_t* o = out + r * rs;
    for (uint64_t k = 0; k < cs; k++) o[k] = in[i * cs + k];
    o[cs] = (uint8_t)(len >> 8);
    o[cs + 1] = (uint8_t)(len & 255);
  }
  __syncthreads();
  return fits ? (int64_t)(nr * rs) : -TDBG_E_OUT_FULL;
}

// ---- one chunk through the forward pipeline --------------------------------
// Data: one buffer (cur, cn).  Metadata: parts sh.md_len[0..md_n) back to
// back at md[mb][md_start, md_cap).
//
// Control flow note: every decision below is workgroup-uniform and the
// per-filter helpers contain barriers, so there is no early return or
// continue between barriers: each stage first sizes its output (a status on
// failure), then runs only if the status is OK.  (An earlier version with a
// `continue` inside the stage switch was miscompiled: the stage output
// pointer update was lost.)
struct StageOut {
  int rc;
  uint64_t on;     // output data bytes
  uint32_t hlen;   // metadata header bytes this stage prepends (0: none)
  bool replace_md; // compression: the metadata becomes one header part
  uint32_t fh;
};

__device__ StageOut fwd_stage(const tdbg_plan& P, uint32_t k, const uint8_t* cur, uint64_t cn,
                              uint8_t* out, FwdSlot& sl, FwdShared& sh, int mb, uint32_t mstart,
                              uint64_t* need) {
  const tdbg_stage& s = P.s[k];
  StageOut r{TDBG_OK, cn, 0, false, 0};
  const uint32_t nparts_in = cn ? 1u : 0u;
  uint8_t* mdb = sl.md[mb];
  // ---- sizing and checks (uniform, no memory writes) ----
  uint32_t ws = 0, nw = 0;
  if (s.kind == TDBG_K_BYTESHUFFLE || s.kind == TDBG_K_XOR) {
    r.hlen = 4 + 4 * nparts_in;
  } else if (s.kind == TDBG_K_FSCALE) {
    r.on = cn / s.dts * s.w;
    r.hlen = 4 + 4 * nparts_in;
  } else if (s.kind == TDBG_K_BITSHUFFLE) {
    r.hlen = 4 + 4 * ((cn - cn % 8 ? 1u : 0u) + (cn % 8 ? 1u : 0u));
  } else if (s.kind == TDBG_K_BWR || s.kind == TDBG_K_PD) {
    const bool bwr = s.kind == TDBG_K_BWR;
    if (cn > 0xffffffffull) {
      r.rc = TDBG_E_UNSUPPORTED;
    } else if (!nparts_in) {
      r.hlen = bwr ? 8 : 4;
      r.on = 0;
    } else {
      const uint32_t ps = (uint32_t)cn;
      ws = (ps < s.window ? ps : s.window) / s.w * s.w;
      if (ws == 0) {
        r.rc = TDBG_E_ARG;  // division by zero in the reference
      } else {
        nw = ps / ws + (ps % ws ? 1 : 0);
        r.hlen = bwr ? 8 + nw * (s.w + 5) : 4 + nw * (s.w + 4);
        if (bwr && (uint64_t)nw * 16 > sl.tab_cap) {
          *need = (uint64_t)nw * 16 + 256;
          r.rc = TDBG_E_SCRATCH;
        }
      }
    }
  } else if (s.kind == TDBG_K_DD || s.kind == TDBG_K_DELTA || s.kind == TDBG_K_RLE) {
    r.replace_md = true;
    r.fh = 8 + 8 * (sh.md_n + nparts_in);
    if (r.fh > sl.md_cap) {
      *need = r.fh + 64;
      r.rc = TDBG_E_SCRATCH;
    }
  } else if (s.kind != TDBG_K_PASS) {
    r.rc = TDBG_E_UNSUPPORTED;
  }
  if (r.rc == TDBG_OK && r.hlen > mstart) {
    *need = sl.md_cap + r.hlen;
    r.rc = TDBG_E_SCRATCH;
  }
  if (r.rc == TDBG_OK && !r.replace_md && s.kind != TDBG_K_PASS && (cn > sl.buf_cap || r.on > sl.buf_cap)) {
    *need = cn > r.on ? cn : r.on;
    r.rc = TDBG_E_SCRATCH;
  }
  if (r.rc != TDBG_OK || s.kind == TDBG_K_PASS) return r;
  // ---- run ----
  uint8_t* h = mdb + mstart - r.hlen;
  switch (s.kind) {
    case TDBG_K_BYTESHUFFLE:
    case TDBG_K_XOR:
    case TDBG_K_FSCALE:
      if (threadIdx.x == 0) {
        stn(h, nparts_in, 4);
        if (nparts_in) stn(h + 4, r.on, 4);
      }
      if (s.kind == TDBG_K_BYTESHUFFLE) f_byteshuffle_fwd(out, cur, cn, s.w);
      else if (s.kind == TDBG_K_XOR) f_xor_fwd(out, cur, cn, s.w);
      else f_fscale_fwd(out, cur, cn / s.dts, s.dts, s.w, P.fs_scale[k], P.fs_offset[k]);
      break;
    case TDBG_K_BITSHUFFLE: {
      const uint64_t rem = cn % 8, p1 = cn - rem;
      if (threadIdx.x == 0) {
        stn(h, (p1 ? 1u : 0u) + (rem ? 1u : 0u), 4);
        uint32_t q = 4;
        if (p1) { stn(h + q, p1, 4); q += 4; }
        if (rem) stn(h + q, rem, 4);
      }
      if (p1) f_bitshuffle_part_fwd(out, cur, p1, s.w);
      for (uint64_t i = p1 + threadIdx.x; i < cn; i += FNT_F) out[i] = cur[i];
      break;
    }
    case TDBG_K_BWR: {
      if (!nparts_in) {
        if (threadIdx.x == 0) { stn(h, 0, 4); stn(h + 4, 0, 4); }
        break;
      }
      const uint32_t ps = (uint32_t)cn;
      int64_t v;
      switch (s.w | (s.sgn << 4)) {
        case 2: v = f_bwr_fwd<2, false>(out, cur, ps, ws, nw, h, sl.tab, sh); break;
        case 4: v = f_bwr_fwd<4, false>(out, cur, ps, ws, nw, h, sl.tab, sh); break;
        case 8: v = f_bwr_fwd<8, false>(out, cur, ps, ws, nw, h, sl.tab, sh); break;
        case 18: v = f_bwr_fwd<2, true>(out, cur, ps, ws, nw, h, sl.tab, sh); break;
        case 20: v = f_bwr_fwd<4, true>(out, cur, ps, ws, nw, h, sl.tab, sh); break;
        case 24: v = f_bwr_fwd<8, true>(out, cur, ps, ws, nw, h, sl.tab, sh); break;
        default: v = -TDBG_E_UNSUPPORTED;
      }
      if (v < 0) r.rc = (int)-v;
      else r.on = (uint64_t)v;
      break;
    }
    case TDBG_K_PD: {
      if (!nparts_in) {
        if (threadIdx.x == 0) stn(h, 0, 4);
        break;
      }
      const uint32_t ps = (uint32_t)cn;
      int v;
      switch (s.w | (s.sgn << 4)) {
        case 1: v = f_pd_fwd<1, false>(out, cur, ps, ws, nw, h, sh); break;
        case 2: v = f_pd_fwd<2, false>(out, cur, ps, ws, nw, h, sh); break;
        case 4: v = f_pd_fwd<4, false>(out, cur, ps, ws, nw, h, sh); break;
        case 8: v = f_pd_fwd<8, false>(out, cur, ps, ws, nw, h, sh); break;
        case 17: v = f_pd_fwd<1, true>(out, cur, ps, ws, nw, h, sh); break;
        case 18: v = f_pd_fwd<2, true>(out, cur, ps, ws, nw, h, sh); break;
        case 20: v = f_pd_fwd<4, true>(out, cur, ps, ws, nw, h, sh); break;
        case 24: v = f_pd_fwd<8, true>(out, cur, ps, ws, nw, h, sh); break;
        default: v = TDBG_E_UNSUPPORTED;
      }
      r.rc = v;
      break;
    }
    default: {  // DD / DELTA / RLE (compression_filter.cc:240-301)
      const uint32_t nmd = sh.md_n;
      const uint32_t np = nmd + nparts_in;
      uint8_t* hdr = sl.md[mb ^ 1] + sl.md_cap - r.fh;
      if (threadIdx.x == 0) {
        stn(hdr, nmd, 4);
        stn(hdr + 4, nparts_in, 4);
      }
      uint64_t o = 0, mo = mstart;
      for (uint32_t i = 0; i < np; i++) {
        if (r.rc == TDBG_OK) {
          const bool is_md = i < nmd;
          const uint8_t* src = is_md ? mdb + mo : cur;
          const uint64_t sn = is_md ? sh.md_len[i] : cn;
          const uint64_t room = sl.buf_cap > o ? sl.buf_cap - o : 0;
          int64_t v;
          if (s.kind == TDBG_K_RLE) v = f_rle_fwd(out + o, room, src, sn, s.cs, sl.tab, sl.tab_cap, sh, need);
          else if (s.kind == TDBG_K_DELTA) v = f_delta_fwd(out + o, room, src, sn, s.w);
          else v = f_dd_fwd(out + o, room, src, sn, s.w, s.sgn != 0, sh);
          if (v == -TDBG_E_OUT_FULL) {  // the scratch buffer, not the caller's output
            *need = sl.buf_cap + sn * 3 + 64;
            v = -TDBG_E_SCRATCH;
          }
          if (v < 0) {
            r.rc = (int)-v;
          } else {
            if (threadIdx.x == 0) {
              stn(hdr + 8 + 8 * i, sn, 4);
              stn(hdr + 12 + 8 * i, (uint64_t)v, 4);
            }
            if (is_md) mo += sn;
            o += (uint64_t)v;
          }
        }
      }
      r.on = o;
      break;
    }
  }
  __syncthreads();
  return r;
}

// Returns the status; on success the chunk's data is (*data, *dn) and its
// metadata md[*mbuf][sh.md_start, md_cap).
__device__ int fwd_chunk(const tdbg_plan& P, const uint8_t* chunk, uint64_t n, FwdSlot& sl, FwdShared& sh,
                         const uint8_t** data, uint64_t* dn, int* mbuf, uint64_t* need) {
  const uint8_t* cur = chunk;
  uint64_t cn = n;
  int cb_ = -1;  // scratch buffer holding cur (-1: the tile)
  int mb = 0;
  int rc = TDBG_OK;
  if (threadIdx.x == 0) {
    sh.md_n = 0;
    sh.md_start = (uint32_t)sl.md_cap;
  }
  __syncthreads();
  for (uint32_t k = 0; k < P.nstages; k++) {
    if (rc == TDBG_OK) {
      const int ob = cb_ == 0 ? 1 : 0;
      const uint32_t mstart = sh.md_start;
      const StageOut r = fwd_stage(P, k, cur, cn, sl.buf[ob], sl, sh, mb, mstart, need);
      rc = r.rc;
      if (rc == TDBG_OK && P.s[k].kind != TDBG_K_PASS) {
        if (threadIdx.x == 0) {
          if (r.replace_md) {  // the frame header replaces the metadata
            sh.md_n = 1;
            sh.md_len[0] = r.fh;
            sh.md_start = (uint32_t)(sl.md_cap - r.fh);
          } else if (sh.md_n < FWD_MAXMD) {  // prepend (filter_buffer.cc:472-506)
            for (uint32_t q = sh.md_n; q > 0; q--) sh.md_len[q] = sh.md_len[q - 1];
            sh.md_len[0] = r.hlen;
            sh.md_n++;
            sh.md_start = mstart - r.hlen;
          } else {
            sh.flag[0] = 1;
          }
        }
        if (r.replace_md) mb ^= 1;
        cur = sl.buf[ob];
        cn = r.on;
        cb_ = ob;
      }
      __syncthreads();
      if (rc == TDBG_OK && sh.flag[0]) rc = TDBG_E_UNSUPPORTED;
    }
  }
  *data = cur;
  *dn = cn;
  *mbuf = mb;
  return rc;
}

__device__ uint32_t fwd_chunk_size(uint64_t tile, uint64_t cell, uint32_t max_chunk) {
  // WriterTile::compute_chunk_size (tile.cc:87-100)
  const uint64_t mc = max_chunk ? max_chunk : 65536;
  uint64_t c = mc < tile ? mc : tile;
  c = c / cell * cell;
  if (c < cell) c = cell;
  return (uint32_t)c;
}

__global__ void __launch_bounds__(FNT_F) filter_tiles_kernel(const KParams kp) {
  __shared__ FwdShared sh;
  FwdSlot sl;
  uint8_t* base = kp.scratch + (uint64_t)blockIdx.x * kp.slot_bytes;
  sl.buf_cap = kp.slot_cap;
  sl.md_cap = kp.md_cap;
  sl.tab_cap = kp.tab_cap;
  sl.buf[0] = base;
  sl.buf[1] = base + kp.slot_cap;
  sl.md[0] = base + 2ull * kp.slot_cap;
  sl.md[1] = sl.md[0] + kp.md_cap;
  sl.tab = (uint64_t*)(sl.md[1] + kp.md_cap);
  uint64_t ntl = kp.ntiles;
  if (kp.ntiles_dev) {  // the LDS-resident forward kernel's queue (tdbg_forward_stream.hip)
    const uint64_t c = (uint32_t)__builtin_amdgcn_readfirstlane(*kp.ntiles_dev);
    ntl = c < ntl ? c : ntl;
  }
  for (uint64_t j = blockIdx.x; j < ntl; j += gridDim.x) {
    const uint64_t t = kp.tile_list ? kp.tile_list[j] : j;
    const uint8_t* in = kp.in[t];
    const uint64_t size = kp.in_size[t];
    uint8_t* out = kp.out[t];
    const uint64_t cap = kp.out_size[t];
    const uint32_t chunk = fwd_chunk_size(size, kp.cell_size ? kp.cell_size : 1, kp.max_chunk);
    uint64_t nchunks = 1, last = chunk;
    if (size != chunk) {
      nchunks = size / chunk;
      last = size % chunk;
      if (last) nchunks++;
      else last = chunk;
    }
    int rc = TDBG_OK;
    uint64_t need = 0;
    uint64_t o = 8;
    if (cap < 8) rc = TDBG_E_OUT_FULL;
    if (threadIdx.x == 0) sh.flag[0] = 0;
    for (uint64_t c = 0; c < nchunks && rc == TDBG_OK; c++) {
      const uint64_t n = c == nchunks - 1 ? last : chunk;
      const uint8_t* dptr;
      uint64_t dn;
      int mb;
      rc = fwd_chunk(kp.plan, in + c * (uint64_t)chunk, n, sl, sh, &dptr, &dn, &mb, &need);
      const uint64_t ms = sl.md_cap - sh.md_start;
      if (rc == TDBG_OK && o + 12 + ms + dn > cap) rc = TDBG_E_OUT_FULL;
      if (rc == TDBG_OK) {
        if (threadIdx.x == 0) {
          stn(out + o, n, 4);
          stn(out + o + 4, dn, 4);
          stn(out + o + 8, ms, 4);
        }
        blk_copy(out + o + 12, sl.md[mb] + sh.md_start, ms);
        blk_copy(out + o + 12 + ms, dptr, dn);
        o += 12 + ms + dn;
      }
      __syncthreads();
    }
    if (rc == TDBG_OK && threadIdx.x == 0) stn(out, nchunks, 8);
    __syncthreads();
    if (threadIdx.x == 0) {
      if (kp.status) kp.status[t] = rc;
      if (kp.need) kp.need[t] = need;
      if (kp.out_len) kp.out_len[t] = rc == TDBG_OK ? o : 0;
    }
  }
}

}  // namespace tdbg

extern "C" hipError_t tdbg_launch_filter(const tdbg::KParams* kp, uint32_t grid, hipStream_t stream) {
  hipLaunchKernelGGL(tdbg::filter_tiles_kernel, dim3(grid), dim3(tdbg::FNT_F), 0, stream, *kp);
  return hipGetLastError();
}
