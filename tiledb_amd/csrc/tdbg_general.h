// tdbg_general.h -- general unfilter interpreter (any combination of the six
// filters, any chunk size), templated on the workgroup size so both the
// general kernel (256 threads) and the fused fast kernels (512 threads) can
// run it; intermediates live in a per-workgroup global scratch slot.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/tiledb_amd.h"
#include "tdbg_desc.h"
#include "tdbg_device.h"

namespace tdbg {

struct Slot {
  uint8_t* buf[2];
  uint8_t* md[2];
  uint8_t* tab;
  uint32_t slot_cap, md_cap, tab_cap;
};

template <int NT>
struct Shared {
  uint64_t red[NT / 64 * 2 + 4];
  uint32_t parts[2 * 64 + 4];
  uint64_t bcast[4];
};

// ---------------------------------------------------------------------------
// stage: plain copy (pass-through into a fixed allocation, empty pipeline)
// ---------------------------------------------------------------------------
template <int NT>
__device__ void g_copy(uint8_t* dst, const uint8_t* src, uint64_t n) {
  const uint32_t tid = threadIdx.x;
  if ((((uintptr_t)dst) & 3) == 0) {
    for (uint64_t i = (uint64_t)tid * 4; i < n; i += NT * 4) {
      uint32_t k = n - i < 4 ? (uint32_t)(n - i) : 4u;
      stn(dst + i, ldn(src + i, k), k);
    }
  } else {
    for (uint64_t i = tid; i < n; i += NT) dst[i] = src[i];
  }
}

template <int NT>
__device__ void g_zero(uint8_t* dst, uint64_t n) {
  for (uint64_t i = threadIdx.x; i < n; i += NT) dst[i] = 0;
}

// ---------------------------------------------------------------------------
// byteshuffle^-1 of one part (blosc2 unshuffle semantics)
// ---------------------------------------------------------------------------
template <int NT>
__device__ void g_unshuffle_part(uint8_t* dst, const uint8_t* src, uint64_t n,
                                 uint32_t ts) {
  if (ts <= 1) { g_copy<NT>(dst, src, n); return; }
  const uint64_t N = n / ts;
  for (uint64_t i = threadIdx.x; i < N; i += NT) {
    uint64_t v = 0;
    for (uint32_t j = 0; j < ts; j++) v |= (uint64_t)src[j * N + i] << (8 * j);
    stn(dst + i * ts, v, ts);
  }
  const uint64_t done = N * ts;
  for (uint64_t i = done + threadIdx.x; i < n; i += NT) dst[i] = src[i];
}

// ---------------------------------------------------------------------------
// bitshuffle^-1 of one part: independent 8192-B blocks, each the
// kiyo-masui bit transpose of its first (n - n%8) elements + copied tail
// (bitshuffle_filter.cc:128-166).
// ---------------------------------------------------------------------------
template <int NT>
__device__ void g_bitunshuffle_part(uint8_t* dst, const uint8_t* src,
                                    uint64_t n, uint32_t ts) {
  if (n % ts != 0 || n % 8 != 0) { g_copy<NT>(dst, src, n); return; }
  for (uint64_t b0 = 0; b0 < n; b0 += 8192) {
    const uint64_t nb = n - b0 < 8192 ? n - b0 : 8192;
    const uint64_t ne = nb / ts, n8 = ne - ne % 8, rowb = n8 / 8;
    const uint8_t* s = src + b0;
    uint8_t* d = dst + b0;
    const uint64_t items = rowb * ts;
    for (uint64_t it = threadIdx.x; it < items; it += NT) {
      const uint64_t q = it / ts;
      const uint32_t b = (uint32_t)(it % ts);
      uint64_t x = 0;
      for (uint32_t k = 0; k < 8; k++) x |= (uint64_t)s[(8ull * b + k) * rowb + q] << (8 * k);
      const uint64_t y = transpose8x8(x);
      for (uint32_t r = 0; r < 8; r++) d[(8 * q + r) * ts + b] = (uint8_t)(y >> (8 * r));
    }
    for (uint64_t i = n8 * ts + threadIdx.x; i < nb; i += NT) d[i] = s[i];
  }
}

// ---------------------------------------------------------------------------
// XOR^-1 of one part (XORFilter::unxor_part, xor_filter.cc:260-286):
// out[j] = in[0] ^ ... ^ in[j] over the part's n/ts whole elements, one
// block prefix-XOR per NT elements with a running carry.  The n % ts tail
// bytes are not written (the reference does not write them either).
// ---------------------------------------------------------------------------
template <int NT>
__device__ void g_unxor_part(uint8_t* dst, const uint8_t* src, uint64_t n, uint32_t ts,
                             Shared<NT>& sh) {
  const uint64_t ne = n / ts;
  uint64_t carry = 0;
  for (uint64_t b = 0; b < ne; b += NT) {
    const uint64_t j = b + threadIdx.x;
    const uint64_t v = j < ne ? ldn(src + j * ts, ts) : 0;
    uint64_t tot;
    const uint64_t x = block_incscan_xor<NT>(v, tot, sh.red) ^ carry;
    if (j < ne) stn(dst + j * ts, x, ts);
    carry ^= tot;
  }
}

// ---------------------------------------------------------------------------
// BWR^-1 (bit_width_reduction_filter.cc:352-404)
// md: [u32 orig][u32 nwin] nwin x [T offset][u8 bits][u32 nbytes]
// ---------------------------------------------------------------------------
struct StageIO {
  const uint8_t* in;
  uint64_t in_n;
  const uint8_t* md;
  uint64_t md_n;
  uint64_t md_used;
  uint8_t* out;
  uint64_t cap;   // fixed allocation size, or scratch capacity
  bool fixed;
  uint64_t out_n; // resulting FilterBuffer::size()
  uint64_t need;  // scratch requirement on TDBG_E_SCRATCH
};

template <int NT>
__device__ int g_bwr(StageIO& io, const tdbg_stage& s, Slot& sl, Shared<NT>& sh) {
  const uint32_t tid = threadIdx.x;
  if (io.md_n < 4) return TDBG_E_MD_READ;
  const uint32_t orig = (uint32_t)ldn(io.md, 4);
  if (io.md_n < 8) return TDBG_E_MD_READ;
  const uint32_t nw = (uint32_t)ldn(io.md + 4, 4);
  uint64_t cap_out;
  if (io.fixed) {
    if (orig > io.cap) return TDBG_E_OUT_FULL;
    cap_out = io.cap;
  } else {
    if (orig > io.cap) { io.need = orig; return TDBG_E_SCRATCH; }
    cap_out = orig;
  }
  const uint32_t E = s.dts + 5;
  const uint32_t w = s.w;
  if ((uint64_t)nw * 8 > sl.tab_cap) {
    // Only windows whose entries exist in md can be decoded; a table larger
    // than scratch is either a huge chunk or corrupt md.
    const uint64_t have = io.md_n >= 8 ? (io.md_n - 8) / E : 0;
    if (have * 8 > sl.tab_cap) { io.need = have * 8 + 64; return TDBG_E_SCRATCH; }
  }
  uint32_t* tab = (uint32_t*)sl.tab;
  uint64_t cin = 0, cout = 0;
  uint64_t first_fail = ~0ull;
  for (uint64_t base = 0; base < nw; base += NT) {
    const uint64_t wi = base + tid;
    const bool valid = wi < nw;
    const bool md_ok = valid && (8 + (wi + 1) * E <= io.md_n);
    uint32_t bits = 0, nb = 0;
    if (md_ok) {
      const uint8_t* e = io.md + 8 + wi * E;
      bits = e[s.dts];
      nb = (uint32_t)ldn(e + s.dts + 1, 4);
    }
    const bool raw = bits >= 8u * w || (nb % w) != 0;
    const uint32_t cb = bits / 8;
    const uint64_t comp = md_ok ? (raw ? nb : (uint64_t)(nb / w) * cb) : 0;
    uint64_t tin, tout;
    const uint64_t in_ex = cin + block_exscan_u64<NT>(comp, tin, sh.red);
    const uint64_t out_ex = cout + block_exscan_u64<NT>(md_ok ? nb : 0, tout, sh.red);
    uint64_t key = ~0ull;
    if (valid) {
      uint32_t code = 0;
      if (!md_ok) code = TDBG_E_MD_READ;
      else if (!raw && bits != 8 && bits != 16 && bits != 32 && bits != 64) code = TDBG_E_BWR_BITS;
      else if (raw) code = copy_fail(io.in_n, in_ex, cap_out, out_ex, nb);
      else code = elem_fail(io.in_n, in_ex, cb, cap_out, out_ex, s.dts, nb / w);
      if (code) key = (wi << 8) | code;
      if (md_ok && wi * 2 + 1 < sl.tab_cap / 4) {
        tab[wi * 2] = (uint32_t)in_ex;
        tab[wi * 2 + 1] = (uint32_t)out_ex;
      }
    }
    const uint64_t f = block_min_u64<NT>(key, sh.red);
    cin += tin;
    cout += tout;
    if (f != ~0ull) { first_fail = f; break; }
  }
  if (first_fail != ~0ull) return (int)(first_fail & 0xff);
  __syncthreads();  // table visible to every wave
  // decode: one wave per window
  const uint32_t lane = tid & 63, wave = tid >> 6;
  for (uint64_t wi = wave; wi < nw; wi += NT / 64) {
    const uint8_t* e = io.md + 8 + wi * E;
    const uint64_t off = ldn(e, s.dts);
    const uint32_t bits = e[s.dts];
    const uint32_t nb = (uint32_t)ldn(e + s.dts + 1, 4);
    const uint32_t ip = tab[wi * 2], op = tab[wi * 2 + 1];
    const bool raw = bits >= 8u * w || (nb % w) != 0;
    if (raw) {
      for (uint32_t j = lane; j < nb; j += 64) io.out[op + j] = io.in[ip + j];
    } else {
      const uint32_t cb = bits / 8, ne = nb / w;
      for (uint32_t j = lane; j < ne; j += 64) {
        uint64_t v = ldn(io.in + ip + (uint64_t)j * cb, cb);
        if (s.sgn) v = (uint64_t)sext64(v, cb);
        v = (v + off) & wmask(w);
        stn(io.out + op + (uint64_t)j * s.dts, v, s.dts);
      }
    }
  }
  io.out_n = io.fixed ? io.cap : cout;
  io.md_used = 8 + (uint64_t)nw * E;
  return TDBG_OK;
}

// ---------------------------------------------------------------------------
// FLOAT_SCALE^-1 (FloatScalingFilter::run_reverse<T, W>,
// float_scaling_filter.cc:164-197): T(scale * double(T(w)) + offset), the
// multiply and the add rounded separately (no FMA contraction, as the
// reference's x86-64 build).  One output prepend per part: a fixed allocation
// takes only the first (filter_buffer.cc:508-545); several parts into a
// growable buffer are not modelled (TDBG_E_UNSUPPORTED, as the oracle).
// ---------------------------------------------------------------------------
template <int NT>
__device__ int g_fscale(StageIO& io, const tdbg_stage& s, double sc, double of) {
  // hipcc contracts a * b + c into an FMA by default (-ffp-contract=fast),
  // even through __dmul_rn/__dadd_rn once inlined; the reference rounds the
  // product and the sum separately (an empty asm on the product pins that)
  if (io.md_n < 4) return TDBG_E_MD_READ;
  const uint32_t np = (uint32_t)ldn(io.md, 4);
  const uint32_t ts = s.dts, bw = s.w;
  uint64_t ip = 0, op = 0;
  for (uint32_t i = 0; i < np; i++) {
    if (4 + 4 * ((uint64_t)i + 1) > io.md_n) return TDBG_E_MD_READ;
    const uint32_t ps = (uint32_t)ldn(io.md + 4 + 4 * i, 4);
    if (ip + ps > io.in_n) return TDBG_E_DATA_READ;
    if (i > 0) return io.fixed ? TDBG_E_OUT_FULL : TDBG_E_UNSUPPORTED;
    const uint64_t ne = ps / bw, on = ne * ts;
    if (on > io.cap) {
      if (io.fixed) return TDBG_E_OUT_FULL;
      io.need = on;
      return TDBG_E_SCRATCH;
    }
    const uint8_t* src = io.in + ip;
    for (uint64_t j = threadIdx.x; j < ne; j += NT) {
      const int64_t q = sext64(ldn(src + j * bw, bw), bw);
      if (ts == 4) {
        const float e = __ll2float_rn(q);
        double prod = sc * (double)e;
        asm volatile("" : "+v"(prod));  // keeps the product rounded: no v_fma_f64
        const float y = __double2float_rn(prod + of);
        stn(io.out + 4 * j, (uint64_t)__float_as_uint(y), 4);
      } else {
        double prod = sc * __ll2double_rn(q);
        asm volatile("" : "+v"(prod));
        const double y = prod + of;
        stn(io.out + 8 * j, (uint64_t)__double_as_longlong(y), 8);
      }
    }
    op = on;
    ip += ps;
  }
  io.md_used = 4 + 4 * (uint64_t)np;
  io.out_n = io.fixed ? io.cap : op;
  return TDBG_OK;
}

// ---------------------------------------------------------------------------
// PD^-1 (positive_delta_filter.cc:324-375)
// md: [u32 nwin] nwin x [T first][u32 nbytes]
// ---------------------------------------------------------------------------
template <int NT>
__device__ int g_pd(StageIO& io, const tdbg_stage& s, Slot& sl, Shared<NT>& sh) {
  const uint32_t tid = threadIdx.x;
  if (io.md_n < 4) return TDBG_E_MD_READ;
  const uint32_t nw = (uint32_t)ldn(io.md, 4);
  uint64_t cap_out;
  if (io.fixed) {
    if (io.in_n > io.cap) return TDBG_E_OUT_FULL;
    cap_out = io.cap;
  } else {
    if (io.in_n > io.cap) { io.need = io.in_n; return TDBG_E_SCRATCH; }
    cap_out = io.in_n;
  }
  const uint32_t E = s.dts + 4;
  const uint32_t w = s.w;
  {
    const uint64_t have = io.md_n >= 4 ? (io.md_n - 4) / E : 0;
    const uint64_t use = have < nw ? have : nw;
    if (use * 4 > sl.tab_cap) { io.need = use * 4 + 64; return TDBG_E_SCRATCH; }
  }
  uint32_t* tab = (uint32_t*)sl.tab;
  uint64_t cin = 0;
  uint64_t first_fail = ~0ull;
  for (uint64_t base = 0; base < nw; base += NT) {
    const uint64_t wi = base + tid;
    const bool valid = wi < nw;
    const bool md_ok = valid && (4 + (wi + 1) * E <= io.md_n);
    uint32_t nb = 0;
    if (md_ok) nb = (uint32_t)ldn(io.md + 4 + wi * E + s.dts, 4);
    uint64_t tot;
    const uint64_t ex = cin + block_exscan_u64<NT>(md_ok ? nb : 0, tot, sh.red);
    uint64_t key = ~0ull;
    if (valid) {
      uint32_t code = 0;
      if (!md_ok) code = TDBG_E_MD_READ;
      else if (nb % w) code = copy_fail(io.in_n, ex, cap_out, ex, nb);
      else code = elem_fail(io.in_n, ex, w, cap_out, ex, s.dts, nb / w);
      if (code) key = (wi << 8) | code;
      if (md_ok) tab[wi] = (uint32_t)ex;
    }
    const uint64_t f = block_min_u64<NT>(key, sh.red);
    cin += tot;
    if (f != ~0ull) { first_fail = f; break; }
  }
  if (first_fail != ~0ull) return (int)(first_fail & 0xff);
  __syncthreads();
  const uint32_t lane = tid & 63, wave = tid >> 6;
  for (uint64_t wi = wave; wi < nw; wi += NT / 64) {
    const uint8_t* e = io.md + 4 + wi * E;
    const uint64_t first = ldn(e, s.dts);
    const uint32_t nb = (uint32_t)ldn(e + s.dts, 4);
    const uint32_t p0 = tab[wi];
    if (nb % w) {
      for (uint32_t j = lane; j < nb; j += 64) io.out[p0 + j] = io.in[p0 + j];
      continue;
    }
    const uint32_t ne = nb / w;
    uint64_t prev = first;
    for (uint32_t j0 = 0; j0 < ne; j0 += 64) {
      const uint32_t j = j0 + lane;
      const uint64_t d = j < ne ? ldn(io.in + p0 + (uint64_t)j * w, w) : 0;
      const uint64_t inc = wave_incscan_u64(d);
      const uint64_t v = prev + inc;
      if (j < ne) stn(io.out + p0 + (uint64_t)j * s.dts, v & wmask(w), s.dts);
      prev = __shfl(v, 63, 64);
    }
  }
  io.out_n = io.fixed ? io.cap : cin;
  io.md_used = 4 + (uint64_t)nw * E;
  return TDBG_OK;
}

// ---------------------------------------------------------------------------
// DoubleDelta::decompress<T> of one part (dd_compressor.cc:314-404),
// block-parallel: codes at fixed bit offsets, then x_i from one tuple scan.
// Returns status; *nvals = values written.
// ---------------------------------------------------------------------------
// zero_rest: bytes of the part past the decoded values are zeroed in scratch
// and left untouched in the tile's fixed allocation (as the oracle models
// the reference's growable vs preallocated buffers).
template <int NT>
__device__ int g_dd_part(const uint8_t* src, uint64_t cn, uint8_t* dst,
                         uint64_t un, uint32_t w, bool zero_rest, Shared<NT>& sh) {
  if (w == 0) return TDBG_E_DD_TYPE;
  if (cn < 9) return TDBG_E_DATA_READ;
  const uint32_t b = src[0];
  const uint64_t num = ldn(src + 1, 8);
  if (b >= 8 * w - 1) {  // raw fallback (:327-331)
    const uint64_t k = cn - 9;
    if (k > un) return TDBG_E_OUT_FULL;
    g_copy<NT>(dst, src + 9, k);
    if (zero_rest) g_zero<NT>(dst + k, un - k);
    return TDBG_OK;
  }
  int rc = dd_check(cn, un, w, b, num);
  if (rc) return rc;
  // bytes past the decoded values are unspecified in the reference (realloc'd
  // memory); zeroed in scratch for determinism, as the oracle does
  {
    const uint64_t nv = num == 0 ? 2 : num;
    if (zero_rest && nv * w < un) g_zero<NT>(dst + nv * w, un - nv * w);
  }
  const uint64_t x0 = ldn(src + 9, w);
  if (num == 1) {
    if (threadIdx.x == 0) stn(dst, x0, w);
    return TDBG_OK;
  }
  const uint64_t x1 = ldn(src + 9 + w, w);
  if (num <= 2) {
    if (threadIdx.x == 0) { stn(dst, x0, w); stn(dst + w, x1, w); }
    return TDBG_OK;
  }
  const uint8_t* bs = src + 9 + 2 * w;
  const uint64_t dinit = x1 - x0;
  const uint64_t xinit = x0 - dinit;
  DDCarry carry = {0, 0};
  const uint64_t per_round = (uint64_t)NT * DD_EPT;
  for (uint64_t r0 = 0; r0 < num; r0 += per_round) {
    const uint64_t i0 = r0 + (uint64_t)threadIdx.x * DD_EPT;
    uint64_t e[DD_EPT];
#pragma unroll
    for (int k = 0; k < DD_EPT; k++) {
      const uint64_t i = i0 + k;
      e[k] = (i >= 2 && i < num) ? dd_code(bs, (i - 2) * (b + 1), b) : 0;
    }
    DDAgg a = dd_local(e);
    DDAgg tot;
    DDAgg pre = block_ddscan2<NT>(a, tot, sh.red);  // exclusive, within round
    // combine with carry of earlier rounds
    const uint64_t E = carry.E + pre.E;
    const uint64_t X = carry.X + pre.X + ((uint64_t)threadIdx.x * DD_EPT) * carry.E;
    uint64_t d = dinit + E;
    uint64_t x = xinit + i0 * dinit + X;
#pragma unroll
    for (int k = 0; k < DD_EPT; k++) {
      const uint64_t i = i0 + k;
      d += e[k];
      x += d;
      if (i < num) stn(dst + i * w, x, w);
    }
    // round total -> carry
    carry.X = carry.X + tot.X + per_round * carry.E;
    carry.E = carry.E + tot.E;
  }
  return TDBG_OK;
}

// ---------------------------------------------------------------------------
// RLE::decompress (rle_compressor.cc:103-141) of one part.
// ---------------------------------------------------------------------------
template <int NT>
__device__ int g_rle_part(const uint8_t* src, uint64_t cn, uint8_t* dst,
                          uint64_t un, uint64_t cs, bool zero_rest, Slot& sl, Shared<NT>& sh,
                          uint64_t* need) {
  const uint64_t rs = cs + 2;
  const uint64_t nr = cn / rs;
  if (nr == 0) { if (zero_rest) g_zero<NT>(dst, un); return TDBG_OK; }
  if (cn % rs) return TDBG_E_RLE_FORMAT;
  if ((nr + 1) * 8 > sl.tab_cap) { *need = (nr + 1) * 8 + 64; return TDBG_E_SCRATCH; }
  uint64_t* start = (uint64_t*)sl.tab;
  uint64_t c = 0;
  for (uint64_t base = 0; base < nr; base += NT) {
    const uint64_t r = base + threadIdx.x;
    uint64_t len = 0;
    if (r < nr) len = ((uint64_t)src[r * rs + cs] << 8) | src[r * rs + cs + 1];
    uint64_t tot;
    const uint64_t ex = c + block_exscan_u64<NT>(len, tot, sh.red);
    if (r < nr) start[r] = ex;
    c += tot;
  }
  if (threadIdx.x == 0) start[nr] = c;
  const uint64_t total = c;
  __syncthreads();
  if (total * cs > un) return TDBG_E_OUT_FULL;
  if (zero_rest) g_zero<NT>(dst + total * cs, un - total * cs);
  // contiguous cell range per thread: one binary search, then walk forward
  const uint64_t c0 = total * threadIdx.x / NT, c1 = total * (threadIdx.x + 1) / NT;
  if (c0 < c1) {
    uint64_t lo = 0, hi = nr;  // largest r with start[r] <= c0
    while (hi - lo > 1) {
      const uint64_t mid = (lo + hi) / 2;
      if (start[mid] <= c0) lo = mid; else hi = mid;
    }
    uint64_t r = lo;
    uint64_t rend = start[r + 1];
    for (uint64_t cc = c0; cc < c1; cc++) {
      while (cc >= rend) { r++; rend = start[r + 1]; }
      const uint8_t* v = src + r * rs;
      if (cs <= 8) stn(dst + cc * cs, ldn(v, (uint32_t)cs), (uint32_t)cs);
      else for (uint64_t k = 0; k < cs; k++) dst[cc * cs + k] = v[k];
    }
  }
  return TDBG_OK;
}

// ---------------------------------------------------------------------------
// Delta::decompress<T> of one part (delta_compressor.cc:251-273):
// [u64 num][T x0][T d1..], x[i] = (T)(x[i-1] + d[i]), x0 written even when
// num == 0.  Status as the reference's first failing call: the read of value
// i (DATA_READ) comes before its write (OUT_FULL).  One block scan per NT
// values with a running carry; bytes past the values are zeroed (unspecified
// in the reference, zeroed by the oracle too).
// ---------------------------------------------------------------------------
template <int NT>
__device__ int g_delta_part(const uint8_t* src, uint64_t cn, uint8_t* dst, uint64_t un,
                            uint32_t w, Shared<NT>& sh) {
  if (w == 0) return TDBG_E_DELTA_TYPE;  // delta_compressor.cc:210-213
  if (cn < 8) return TDBG_E_DATA_READ;
  const uint64_t num = ldn(src, 8);
  const uint64_t nv = num ? num : 1;
  const uint64_t kr = (cn - 8) / w, kw = un / w;  // values readable / writable
  if (nv > kr || nv > kw) return kr <= kw ? TDBG_E_DATA_READ : TDBG_E_OUT_FULL;
  const uint64_t m = wmask(w);
  uint64_t carry = 0;
  for (uint64_t b = 0; b < nv; b += NT) {
    const uint64_t i = b + threadIdx.x;
    const uint64_t d = i < nv ? ldn(src + 8 + i * w, w) : 0;
    uint64_t tot;
    const uint64_t x = carry + block_exscan_u64<NT>(d, tot, sh.red) + d;
    if (i < nv) stn(dst + i * w, x & m, w);
    carry += tot;
  }
  if (nv * w < un) g_zero<NT>(dst + nv * w, un - nv * w);
  return TDBG_OK;
}

// ---------------------------------------------------------------------------
// CompressionFilter::run_reverse (compression_filter.cc:303-347) for DD/RLE
// md: [u32 n_md][u32 n_data] (u32 orig, u32 comp) x (n_md + n_data)
// ---------------------------------------------------------------------------
template <int NT>
__device__ int g_compression(StageIO& io, const tdbg_stage& s, Slot& sl,
                             Shared<NT>& sh, int md_dst, uint64_t* md_out_n) {
  if (io.md_n < 4) return TDBG_E_MD_READ;
  const uint32_t nmd = (uint32_t)ldn(io.md, 4);
  if (io.md_n < 8) return TDBG_E_MD_READ;
  const uint32_t nd = (uint32_t)ldn(io.md + 4, 4);
  const uint64_t np = (uint64_t)nmd + nd;
  const uint64_t have = (io.md_n - 8) / 8;
  // scratch requirements over the pairs that exist
  uint64_t need_md = 0, need_data = 0;
  for (uint64_t i = 0; i < np && i < have; i++) {
    const uint32_t un = (uint32_t)ldn(io.md + 8 + 8 * i, 4);
    if (i < nmd) need_md += un; else need_data += un;
  }
  if (need_md > sl.md_cap) { io.need = need_md; return TDBG_E_SCRATCH; }
  if (!io.fixed && need_data > io.cap) { io.need = need_data; return TDBG_E_SCRATCH; }
  uint8_t* mdo = sl.md[md_dst];
  uint64_t ip = 0, op = 0, mo = 0;
  for (uint64_t i = 0; i < np; i++) {
    if (i >= have) return TDBG_E_MD_READ;
    const uint32_t un = (uint32_t)ldn(io.md + 8 + 8 * i, 4);
    const uint32_t cn = (uint32_t)ldn(io.md + 12 + 8 * i, 4);
    const bool is_md = i < nmd;
    uint8_t* dst;
    if (is_md) {
      dst = mdo + mo;
    } else {
      if (io.fixed && op + un > io.cap) return TDBG_E_OUT_FULL;
      dst = io.out + op;
    }
    if (ip + cn > io.in_n) return TDBG_E_DATA_READ;
    int rc;
    const bool zero_rest = is_md || !io.fixed;
    if (s.kind == TDBG_K_DD) rc = g_dd_part<NT>(io.in + ip, cn, dst, un, s.w, zero_rest, sh);
    else if (s.kind == TDBG_K_DELTA) rc = g_delta_part<NT>(io.in + ip, cn, dst, un, s.w, sh);
    else rc = g_rle_part<NT>(io.in + ip, cn, dst, un, s.cs, zero_rest, sl, sh, &io.need);
    __syncthreads();
    if (rc) return rc;
    if (is_md) mo += un; else op += un;
    ip += cn;
  }
  *md_out_n = mo;
  io.out_n = io.fixed ? io.cap : op;
  return TDBG_OK;
}

// ---------------------------------------------------------------------------
// FilterPipeline::run_reverse for one chunk (filter_pipeline.cc:449-514)
// ---------------------------------------------------------------------------
template <int NT>
__device__ __attribute__((noinline)) int g_chunk(const tdbg_plan& P, const uint8_t* md, uint64_t mdn,
                       const uint8_t* data, uint64_t dn, uint8_t* out,
                       uint64_t orig, Slot& sl, Shared<NT>& sh, uint64_t* need) {
  if (P.nstages == 0) {
    if (dn > orig) return TDBG_E_OUT_FULL;
    g_copy<NT>(out, data, dn);
    return TDBG_OK;
  }
  const uint8_t* cin = data;
  uint64_t cin_n = dn;
  int cin_buf = -1;
  const uint8_t* mdp = md;
  uint64_t md_n = mdn;
  int md_buf = -1;
  for (int k = (int)P.nstages - 1; k >= 0; k--) {
    const tdbg_stage& s = P.s[k];
    StageIO io;
    io.in = cin;
    io.in_n = cin_n;
    io.md = mdp;
    io.md_n = md_n;
    io.md_used = 0;
    io.need = 0;
    const int ob = cin_buf == 0 ? 1 : 0;
    if (k == 0) { io.out = out; io.cap = orig; io.fixed = true; }
    else { io.out = sl.buf[ob]; io.cap = sl.slot_cap; io.fixed = false; }
    io.out_n = 0;
    int rc = TDBG_OK;
    int out_buf = ob;
    switch (s.kind) {
      case TDBG_K_PASS:
        if (io.fixed) {
          if (cin_n > io.cap) rc = TDBG_E_OUT_FULL;
          else g_copy<NT>(io.out, cin, cin_n);
        } else {
          io.out = (uint8_t*)cin;
          io.out_n = cin_n;
          out_buf = cin_buf;
        }
        break;
      case TDBG_K_BYTESHUFFLE:
      case TDBG_K_BITSHUFFLE:
      case TDBG_K_XOR: {  // same md / part walk (xor_filter.cc:220-256)
        if (md_n < 4) { rc = TDBG_E_MD_READ; break; }
        const uint32_t np = (uint32_t)ldn(mdp, 4);
        if (io.fixed) { if (cin_n > io.cap) { rc = TDBG_E_OUT_FULL; break; } }
        else if (cin_n > io.cap) { io.need = cin_n; rc = TDBG_E_SCRATCH; break; }
        uint64_t ip = 0;
        for (uint64_t i = 0; i < np; i++) {
          if (4 + 4 * (i + 1) > md_n) { rc = TDBG_E_MD_READ; break; }
          const uint32_t ps = (uint32_t)ldn(mdp + 4 + 4 * i, 4);
          if (ip + ps > cin_n) { rc = TDBG_E_DATA_READ; break; }
          if (s.kind == TDBG_K_BYTESHUFFLE) g_unshuffle_part<NT>(io.out + ip, cin + ip, ps, s.w);
          else if (s.kind == TDBG_K_XOR) g_unxor_part<NT>(io.out + ip, cin + ip, ps, s.w, sh);
          else g_bitunshuffle_part<NT>(io.out + ip, cin + ip, ps, s.w);
          ip += ps;
        }
        io.md_used = 4 + 4 * (uint64_t)np;
        io.out_n = io.fixed ? io.cap : ip;
        break;
      }
      case TDBG_K_BWR:
        rc = g_bwr<NT>(io, s, sl, sh);
        break;
      case TDBG_K_PD:
        rc = g_pd<NT>(io, s, sl, sh);
        break;
      case TDBG_K_FSCALE:
        rc = g_fscale<NT>(io, s, P.fs_scale[k], P.fs_offset[k]);
        break;
      case TDBG_K_DD:
      case TDBG_K_DELTA:
      case TDBG_K_RLE: {
        const int md_dst = md_buf == 0 ? 1 : 0;
        uint64_t mo = 0;
        rc = g_compression<NT>(io, s, sl, sh, md_dst, &mo);
        if (rc == TDBG_OK) {
          __syncthreads();
          mdp = sl.md[md_dst];
          md_n = mo;
          md_buf = md_dst;
          io.md_used = 0;
        }
        break;
      }
      default:
        rc = TDBG_E_UNSUPPORTED;
    }
    __syncthreads();
    if (rc) {
      if (rc == TDBG_E_SCRATCH) *need = io.need;
      return rc;
    }
    if (s.kind != TDBG_K_DD && s.kind != TDBG_K_DELTA && s.kind != TDBG_K_RLE &&
        s.kind != TDBG_K_PASS) {
      mdp += io.md_used;
      md_n -= io.md_used;
    }
    cin = io.out;
    cin_n = io.out_n;
    cin_buf = out_buf;
  }
  return TDBG_OK;
}

// ---------------------------------------------------------------------------
// Tile::load_chunk_data (tile.cc:280-313) + run_reverse over every chunk.
// ---------------------------------------------------------------------------
template <int NT>
__device__ int g_tile(const KParams& kp, const uint8_t* in, uint64_t fs,
                      uint8_t* out, uint64_t os, Slot& sl, Shared<NT>& sh,
                      uint64_t* need) {
  uint64_t expected = os;
  if (kp.flags & TDBG_TILE_OFFSETS) {
    if (os < 8) return TDBG_E_TILE_SIZE;
    expected = os - 8;
  }
  if (fs < 8) return TDBG_E_TILE_FORMAT;
  const uint64_t nch = ldn(in, 8);
  uint64_t o = 8, total = 0;
  for (uint64_t i = 0; i < nch; i++) {
    if (o + 12 > fs) return TDBG_E_TILE_FORMAT;
    const uint64_t orig = ldn(in + o, 4), fl = ldn(in + o + 4, 4), ml = ldn(in + o + 8, 4);
    o += 12;
    if (ml > fs - o) return TDBG_E_TILE_FORMAT;
    o += ml;
    if (fl > fs - o) return TDBG_E_TILE_FORMAT;
    o += fl;
    total += orig;
  }
  if (total != expected) return TDBG_E_TILE_SIZE;
  o = 8;
  uint64_t coff = 0;
  for (uint64_t i = 0; i < nch; i++) {
    const uint64_t orig = ldn(in + o, 4), fl = ldn(in + o + 4, 4), ml = ldn(in + o + 8, 4);
    o += 12;
    const int rc = g_chunk<NT>(kp.plan, in + o, ml, in + o + ml, fl, out + coff, orig, sl, sh, need);
    if (rc) return rc;
    o += ml + fl;
    coff += orig;
  }
  return TDBG_OK;
}

}  // namespace tdbg
