// tdbg_fast.hip -- fused LDS unfilter kernel for gfx950 (MI355X).
//
// One persistent grid of 512-thread workgroups, two per CU.  Per chunk
// (<= 64.5 KiB after every stage), the chunk metadata and filtered data are
// staged once into LDS with aligned 16-B loads; every intermediate filter
// runs in place in LDS (each thread gathers its 192-B output slice into
// registers, workgroup barrier, writes it back), and the last filter
// (filter 0 of the pipeline, filter_pipeline.cc:483-492) streams its output
// to HBM with coalesced 16-B stores.  HBM traffic is therefore the filtered
// bytes in + the unfiltered bytes out.
//
// Any chunk that does not fit these assumptions (oversized stages, multi-part
// buffers, non-uniform windows, malformed metadata ...) is re-run through the
// general interpreter (tdbg_general.h), which reproduces the reference's
// exact error precedence.  The fast path writes HBM only after its final
// stage validated, so a fallback never leaves partial output behind.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/tiledb_amd.h"
#include "tdbg_desc.h"
#include "tdbg_launch.h"
#include "tdbg_device.h"

#include <type_traits>

namespace tdbg {

constexpr int FNT = 512;             // threads per workgroup
constexpr uint32_t XCAP = 66048;     // in-place data buffer (64.5 KiB)
constexpr uint32_t MDCAP = 4608;     // chunk metadata / decompressed metadata
constexpr uint32_t TABN = 512;       // per-window table entries (uint4)
constexpr uint32_t RUNCAP = TABN * 4 - 1;  // RLE run starts (uint32)
constexpr int SP = 128;              // slice bytes per thread for the scan stages
constexpr int SPD = SP / 4;          // (PD, DD): outputs up to FNT * SP = 64 KiB

struct FastLds {
  uint8_t X[XCAP];
  uint8_t MD[MDCAP];
  uint4 TAB[TABN];
  uint64_t red[4 * FNT / 64 + 8];
  uint32_t flag[4];
  uint32_t pairs[3 * 16];  // compression part table: un, cn, input offset
  uint64_t scan2[2][FNT / 64];  // one-barrier stage scans, ping-pong by stage position
  uint32_t scanf[2][FNT / 64];
};

struct View {
  uint32_t base, n;  // bytes [base, base+n) of L.X
  // 1: base == 0 and dword D of the view lies at dword swz_dw(D) of L.X
  // (written by DD for a following 4-byte byteshuffle only)
  uint32_t swz;
};

// Bank swizzle of a DD output slice (32 dwords per thread): the thread's 16-B
// units rotate by (slice & 7), so a wave's slice stores and the byteshuffle's
// plane reads are both conflict-free.  An involution within each 256-dword
// block.
__device__ __forceinline__ uint32_t swz_dw(uint32_t d) { return d ^ (((d >> 5) & 7u) << 2); }
// the same map on 16-B units: unit U at physical unit U ^ ((U >> 3) & 7)
__device__ __forceinline__ uint32_t swz_u(uint32_t u) { return u ^ ((u >> 3) & 7u); }

// Thread index, opaque to the optimizer: the per-thread index math of the
// unrolled stage loops is tile-invariant, and hoisting it out of the
// persistent tile loop would pin (and spill) dozens of registers for the
// whole kernel.  An empty asm on a copy keeps it inside the loop.
__device__ __forceinline__ uint32_t tid_() {
  uint32_t t = threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}

// ---------------------------------------------------------------------------
// LDS byte access at arbitrary offsets (aligned dword reads + alignbyte)
// ---------------------------------------------------------------------------
// Branch-free: both dwords (one ds_read2_b32) and alignbyte, so reads batch.
__device__ __forceinline__ uint32_t lds32(const uint8_t* X, uint32_t off) {
  const uint32_t a = off & ~3u, sh = off & 3u;
  const uint32_t lo = *(const uint32_t*)(X + a);
  const uint32_t hi = *(const uint32_t*)(X + a + 4);
  return __builtin_amdgcn_alignbyte(hi, lo, sh);
}
// the two dwords covering bytes [off, off + 4)
__device__ __forceinline__ uint2 lds_pair(const uint8_t* X, uint32_t off) {
  const uint32_t a = off & ~3u;
  return make_uint2(*(const uint32_t*)(X + a), *(const uint32_t*)(X + a + 4));
}
__device__ __forceinline__ uint64_t lds64(const uint8_t* X, uint32_t off) {
  return (uint64_t)lds32(X, off) | ((uint64_t)lds32(X, off + 4) << 32);
}
// k in 1..8 little-endian bytes
__device__ __forceinline__ uint64_t ldsn(const uint8_t* X, uint32_t off, uint32_t k) {
  if (k <= 4) {
    const uint32_t v = lds32(X, off);
    return k == 4 ? v : (v & ((1u << (8 * k)) - 1));
  }
  const uint64_t v = lds64(X, off);
  return k == 8 ? v : (v & ((1ull << (8 * k)) - 1));
}

// Wave snapshot of 256 bytes of LDS: lane k holds bytes [4k, 4k + 4) of the
// window.  Header fields at uniform offsets are then read with v_readlane
// (scalar, no LDS round trip), so a parse is one LDS latency instead of a
// chain of dependent ones.
__device__ __forceinline__ uint32_t snap_take(const uint8_t* A, uint32_t base) {
  return lds32(A, base + 4 * (tid_() & 63));
}
// o uniform, o + 4 <= 256
__device__ __forceinline__ uint32_t snap32(uint32_t s, uint32_t o) {
  const uint32_t d0 = __builtin_amdgcn_readlane(s, o >> 2);
  if ((o & 3) == 0) return d0;
  const uint32_t d1 = __builtin_amdgcn_readlane(s, (o >> 2) + 1);
  return __builtin_amdgcn_alignbyte(d1, d0, o & 3);
}
__device__ __forceinline__ uint32_t snap8(uint32_t s, uint32_t o) {
  return (__builtin_amdgcn_readlane(s, o >> 2) >> (8 * (o & 3))) & 0xffu;
}
// k in 1..8 bytes, o + 8 <= 256
__device__ __forceinline__ uint64_t snapn(uint32_t s, uint32_t o, uint32_t k) {
  const uint64_t v = (uint64_t)snap32(s, o) | ((uint64_t)snap32(s, o + 4) << 32);
  return k >= 8 ? v : (v & ((1ull << (8 * k)) - 1));
}

// explicit global (address space 1) accesses: global_load/store, not flat
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const v4u g_cu4;
typedef __attribute__((address_space(1))) v4u g_u4;
typedef __attribute__((address_space(1))) const uint32_t g_cu32;
typedef __attribute__((address_space(1))) uint8_t g_u8;

__device__ __forceinline__ uint64_t gldn(const uint8_t* p, uint32_t k) {
  const uintptr_t a = (uintptr_t)p;
  const g_cu32* q = (const g_cu32*)(a & ~(uintptr_t)3);
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

__device__ __forceinline__ bool block_any(bool p) { return __syncthreads_or(p ? 1 : 0) != 0; }

// ---------------------------------------------------------------------------
// global <-> LDS movement
// ---------------------------------------------------------------------------
// Copies global bytes [g, g+n) into X using aligned 16-B loads of the
// enclosing window; returns the view base (g & 15).  All loads of a thread
// are issued before its LDS stores.
__device__ __forceinline__ bool load_to_lds(uint8_t* X, uint32_t cap, const uint8_t* g,
                                            uint32_t n, uint32_t* base) {
  const uintptr_t a0 = (uintptr_t)g & ~(uintptr_t)15;
  const uintptr_t a1 = ((uintptr_t)g + n + 15) & ~(uintptr_t)15;
  const uint32_t cnt = (uint32_t)((a1 - a0) >> 4);
  *base = (uint32_t)((uintptr_t)g - a0);
  if (cnt * 16 > cap) return false;
  // n == 0 at a 16-B aligned g: no unit to load.  (The clamp below would
  // otherwise read unit cnt - 1 = 2^32 - 1, 64 GiB past g: an empty md or
  // data section at an aligned address -- reachable once tiles sit back to
  // back at arbitrary offsets -- faulted the GPU.)
  if (cnt == 0) return true;
  const g_cu4* src = (const g_cu4*)a0;
  constexpr int LU = (XCAP / 16 + FNT - 1) / FNT;
  // Issue every load first (clamped to a valid unit: no divergent control
  // flow around the loads, so they stay in registers), then the LDS stores.
  const uint32_t t = tid_();
  v4u v[LU];
#pragma unroll
  for (int k = 0; k < LU; k++) {
    const uint32_t u = t + k * FNT;
    v[k] = src[u < cnt ? u : cnt - 1];
  }
#pragma unroll
  for (int k = 0; k < LU; k++) {
    const uint32_t u = t + k * FNT;
    if (u < cnt) *(v4u*)(X + 16 * u) = v[k];
  }
  return true;
}

// store 16 bytes (unit u) of the final output; handles the partial last unit
// and unaligned chunk destinations.
__device__ __forceinline__ void store_unit(uint8_t* gout, uint32_t n, uint32_t off, uint4 v) {
  if (off + 16 <= n && (((uintptr_t)(gout + off)) & 15) == 0) {
    v4u x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, (g_u4*)(gout + off));
    return;
  }
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int d = 0; d < 4; d++)
#pragma unroll
    for (int b = 0; b < 4; b++) {
      const uint32_t o = off + 4 * d + b;
      if (o < n) ((g_u8*)gout)[o] = (uint8_t)(w[d] >> (8 * b));
    }
}

// ---------------------------------------------------------------------------
// stage drivers
// ---------------------------------------------------------------------------
// UB-byte units, computed by fn(u, w[UB/4]).  final: streamed to gout;
// otherwise gathered per thread slice, barrier, written to X[0, n).
// Units [0, nfast) may use ffast, a branch-free variant that is safe for
// any unit index below nfast: those are computed in rounds of RU units with
// clamped indices (every LDS read of a round issued back to back, no
// per-unit control flow); the remaining units use fany.
template <int UB, class FF, class FA>
__device__ __forceinline__ void drive2(FastLds& L, uint32_t n, uint32_t nfast, bool final, uint8_t* gout,
                                       FF ffast, FA fany, bool swz_out = false) {
  constexpr int UD = UB / 4;
  constexpr int RU = UB == 16 ? 3 : 1;
  const uint32_t t = tid_();
  if (final) {
    const uint32_t nu = (n + UB - 1) / UB;
    uint32_t done = 0;
    if ((((uintptr_t)gout) & 15) == 0 && nfast > 0) {  // uniform
      for (uint32_t u0 = 0; u0 < nfast; u0 += RU * FNT) {
        uint32_t w[RU][UD];
#pragma unroll
        for (int r = 0; r < RU; r++) {
          const uint32_t u = u0 + r * FNT + t;
          ffast(u < nfast ? u : nfast - 1, w[r]);
        }
        // materialize every unit here: otherwise the compiler sinks a unit's
        // LDS reads into its (predicated) store block and serializes them
#pragma unroll
        for (int r = 0; r < RU; r++)
#pragma unroll
          for (int q = 0; q < UD; q++) asm volatile("" : "+v"(w[r][q]));
#pragma unroll
        for (int r = 0; r < RU; r++) {
          const uint32_t u = u0 + r * FNT + t;
          if (u < nfast) {
#pragma unroll
            for (int q = 0; q < UD / 4; q++) {
              v4u x = {w[r][4 * q], w[r][4 * q + 1], w[r][4 * q + 2], w[r][4 * q + 3]};
              __builtin_nontemporal_store(x, (g_u4*)(gout + u * UB + 16 * q));
            }
          }
        }
      }
      done = nfast;
    }
    for (uint32_t u = done + t; u < nu; u += FNT) {
      uint32_t w[UD];
      fany(u, w);
#pragma unroll
      for (int q = 0; q < UD / 4; q++)
        store_unit(gout, n, u * UB + 16 * q, make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]));
    }
    return;
  }
  // in place: every unit of the stage is computed into registers (unit
  // u = tid + k*FNT, lane-consecutive, so LDS reads and writes are
  // conflict-free), barrier, then written back to X[0, n)
  constexpr int NU = (XCAP + UB * FNT - 1) / (UB * FNT);
  constexpr int RI = UB == 16 ? 4 : 1;  // units per straight-line batch
  uint32_t r[NU * UD];
#pragma unroll
  for (int k0 = 0; k0 < NU; k0 += RI) {
    const int kend = k0 + RI < NU ? k0 + RI : NU;
    if ((uint32_t)kend * FNT <= nfast) {
      // every unit of the batch takes the fast form (uniform): no per-unit
      // control flow, so the batch's LDS reads issue together
#pragma unroll
      for (int k = k0; k < kend; k++) ffast(t + k * FNT, *(uint32_t(*)[UD])(r + k * UD));
    } else {
#pragma unroll
      for (int k = k0; k < kend; k++) {
        const uint32_t u = t + k * FNT;
        if (u < nfast) ffast(u, *(uint32_t(*)[UD])(r + k * UD));
        else if (u * UB < n) fany(u, *(uint32_t(*)[UD])(r + k * UD));
      }
    }
    __builtin_amdgcn_sched_barrier(0);  // bound the loads in flight
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NU; k++) {
    const uint32_t u = t + k * FNT;
#pragma unroll
    for (int q = 0; q < UD / 4; q++) {
      const uint32_t o = u * UB + 16 * q;
      if (o < n)
        *(uint4*)(L.X + (swz_out ? 16 * swz_u(o >> 4) : o)) =
            make_uint4(r[k * UD + 4 * q], r[k * UD + 4 * q + 1], r[k * UD + 4 * q + 2], r[k * UD + 4 * q + 3]);
    }
  }
  __syncthreads();
}

template <int UB, class F>
__device__ __forceinline__ void drive(FastLds& L, uint32_t n, bool final, uint8_t* gout, F fn,
                                      bool swz_out = false) {
  drive2<UB>(L, n, 0, final, gout, fn, fn, swz_out);
}

// Copy a view to the final output (pass-through / raw stages as filter 0).
__device__ void final_copy(FastLds& L, View v, uint8_t* gout) {
  if (v.swz) {  // base 0, 16-B units swizzled
    for (uint32_t u = tid_(); u * 16 < v.n; u += FNT)
      store_unit(gout, v.n, 16 * u, *(const uint4*)(L.X + 16 * swz_u(u)));
    return;
  }
  for (uint32_t u = tid_(); u * 16 < v.n; u += FNT) {
    const uint32_t o = v.base + 16 * u;
    uint4 x;
    if ((o & 15) == 0) x = *(const uint4*)(L.X + o);
    else x = make_uint4(lds32(L.X, o), lds32(L.X, o + 4), lds32(L.X, o + 8), lds32(L.X, o + 12));
    store_unit(gout, v.n, 16 * u, x);
  }
}

// A thread's 128-B slice [128 t, 128 t + 128) of the view into registers:
// swizzled views with conflict-free 16-B reads, others dword-wise.
__device__ __forceinline__ void slice_load(const FastLds& L, const View& v, uint32_t (&r)[SPD]) {
  const uint32_t t = tid_(), s0 = t * SP;
  if (v.swz) {
#pragma unroll
    for (int q = 0; q < SP / 16; q++) {
      const uint4 x = *(const uint4*)(L.X + 16 * swz_u(8 * t + q));
      r[4 * q] = x.x; r[4 * q + 1] = x.y; r[4 * q + 2] = x.z; r[4 * q + 3] = x.w;
    }
  } else {
#pragma unroll
    for (int k = 0; k < SPD; k++) r[k] = (s0 + 4 * k < v.n) ? lds32(L.X, v.base + s0 + 4 * k) : 0u;
  }
}

// Move a view to X[0, n) in place (slices gathered to registers first).
__device__ void settle(FastLds& L, View& v) {
  if (v.base == 0) return;
  const uint32_t b = v.base;
  drive<16>(L, v.n, false, nullptr, [&](uint32_t u, uint32_t (&w)[4]) {
#pragma unroll
    for (int d = 0; d < 4; d++) w[d] = lds32(L.X, b + 16 * u + 4 * d);
  });
  v.base = 0;
}

// ---------------------------------------------------------------------------
// byteshuffle^-1 (blosc2 unshuffle; byteshuffle_filter.cc:111-166)
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t unshuf_byte(const uint8_t* X, uint32_t base, uint32_t n,
                                                uint32_t N, uint32_t TS, uint32_t p) {
  if (p >= n) return 0;
  if (p < N * TS) return X[base + (p % TS) * N + p / TS];
  return X[base + p];
}

template <int TS>
__device__ __forceinline__ bool f_byteshuffle(FastLds& L, View& cur, uint32_t& mo, uint32_t& mn, bool final,
                              uint8_t* gout, uint32_t cap) {
  if (mn < 8) return false;
  const uint32_t np = lds32(L.MD, mo), ps = lds32(L.MD, mo + 4);
  if (np != 1 || ps != cur.n) return false;
  if (final && ps > cap) return false;
  mo += 8;
  mn -= 8;
  const uint32_t n = ps, N = n / TS, base = cur.base;
  const uint8_t* X = L.X;
  if (TS == 1) {
    if (final) final_copy(L, cur, gout);
    else __syncthreads();  // md reads done before a later stage rewrites MD
    return true;
  }
  const uint32_t full = (N * TS) & ~15u;  // bytes covered by whole vector units
  auto slow = [&](uint32_t u, uint32_t* w) {
#pragma unroll
    for (int d = 0; d < 4; d++) {
      uint32_t v = 0;
#pragma unroll
      for (int b = 0; b < 4; b++) v |= unshuf_byte(X, base, n, N, TS, 16 * u + 4 * d + b) << (8 * b);
      w[d] = v;
    }
  };
  if (TS == 4 && (cur.swz || ((base & 3) == 0 && (N & 3) == 0))) {
    // planes start on dword boundaries: one dword per plane per unit
    const uint32_t swz = cur.swz, q = N >> 2;
    auto unit = [&](const uint32_t (&p)[4], uint32_t (&w)[4]) {
      const uint32_t a = __builtin_amdgcn_perm(p[1], p[0], 0x05010400u);
      const uint32_t b = __builtin_amdgcn_perm(p[3], p[2], 0x05010400u);
      const uint32_t c = __builtin_amdgcn_perm(p[1], p[0], 0x07030602u);
      const uint32_t d = __builtin_amdgcn_perm(p[3], p[2], 0x07030602u);
      w[0] = __builtin_amdgcn_perm(b, a, 0x05040100u);
      w[1] = __builtin_amdgcn_perm(b, a, 0x07060302u);
      w[2] = __builtin_amdgcn_perm(d, c, 0x05040100u);
      w[3] = __builtin_amdgcn_perm(d, c, 0x07060302u);
    };
    auto fast = [&](uint32_t u, uint32_t (&w)[4]) {
      uint32_t p[4];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint32_t d = k * q + u;
        p[k] = *(const uint32_t*)(X + base + 4 * (swz ? swz_dw(d) : d));
      }
      unit(p, w);
    };
    auto slowu = [&](uint32_t u, uint32_t (&w)[4]) {
      if (16 * u + 16 <= full) fast(u, w);
      else slow(u, w);
    };
    if (base == 0 && N == 16384) {
      // a 64 KiB chunk: plane k starts at byte 16384 k (a multiple of the
      // swizzle block), so one address + immediate offsets reads all planes
      auto fast64 = [&](uint32_t u, uint32_t (&w)[4]) {
        const uint32_t* P = (const uint32_t*)(X + 4 * (swz ? swz_dw(u) : u));
        const uint32_t p[4] = {P[0], P[4096], P[8192], P[12288]};
        unit(p, w);
      };
      drive2<16>(L, n, full / 16, final, gout, fast64, slowu);
    } else {
      // (swz implies n = 4N with N % 4 == 0: every unit is a fast unit)
      drive2<16>(L, n, full / 16, final, gout, fast, slowu);
    }
  } else if (TS == 4) {
    auto fast = [&](uint32_t u, uint32_t (&w)[4]) {
      const uint32_t i = 4 * u;
      // the four plane reads issued together, aligned afterwards
      const uint32_t o0 = base + i, o1 = o0 + N, o2 = o1 + N, o3 = o2 + N;
      const uint2 r0 = lds_pair(X, o0), r1 = lds_pair(X, o1), r2 = lds_pair(X, o2), r3 = lds_pair(X, o3);
      const uint32_t p0 = __builtin_amdgcn_alignbyte(r0.y, r0.x, o0 & 3);
      const uint32_t p1 = __builtin_amdgcn_alignbyte(r1.y, r1.x, o1 & 3);
      const uint32_t p2 = __builtin_amdgcn_alignbyte(r2.y, r2.x, o2 & 3);
      const uint32_t p3 = __builtin_amdgcn_alignbyte(r3.y, r3.x, o3 & 3);
      const uint32_t a = __builtin_amdgcn_perm(p1, p0, 0x05010400u);
      const uint32_t b = __builtin_amdgcn_perm(p3, p2, 0x05010400u);
      const uint32_t c = __builtin_amdgcn_perm(p1, p0, 0x07030602u);
      const uint32_t d = __builtin_amdgcn_perm(p3, p2, 0x07030602u);
      w[0] = __builtin_amdgcn_perm(b, a, 0x05040100u);
      w[1] = __builtin_amdgcn_perm(b, a, 0x07060302u);
      w[2] = __builtin_amdgcn_perm(d, c, 0x05040100u);
      w[3] = __builtin_amdgcn_perm(d, c, 0x07060302u);
    };
    drive2<16>(L, n, full / 16, final, gout, fast, [&](uint32_t u, uint32_t (&w)[4]) {
      if (16 * u + 16 <= full) fast(u, w);
      else slow(u, w);
    });
  } else if (TS == 2) {
    auto fast = [&](uint32_t u, uint32_t (&w)[4]) {
      const uint32_t i = 8 * u;
      const uint64_t p0 = lds64(X, base + i), p1 = lds64(X, base + N + i);
      const uint32_t a0 = (uint32_t)p0, a1 = (uint32_t)(p0 >> 32);
      const uint32_t b0 = (uint32_t)p1, b1 = (uint32_t)(p1 >> 32);
      w[0] = __builtin_amdgcn_perm(b0, a0, 0x05010400u);
      w[1] = __builtin_amdgcn_perm(b0, a0, 0x07030602u);
      w[2] = __builtin_amdgcn_perm(b1, a1, 0x05010400u);
      w[3] = __builtin_amdgcn_perm(b1, a1, 0x07030602u);
    };
    drive2<16>(L, n, full / 16, final, gout, fast, [&](uint32_t u, uint32_t (&w)[4]) {
      if (16 * u + 16 <= full) fast(u, w);
      else slow(u, w);
    });
  } else {  // TS == 8: 32-B units = 4 elements
    const uint32_t full32 = (N * TS) & ~31u;
    auto fast = [&](uint32_t u, uint32_t (&w)[8]) {
      const uint32_t i = 4 * u;
      uint32_t p[8];
#pragma unroll
      for (int j = 0; j < 8; j++) p[j] = lds32(X, base + j * N + i);
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const uint32_t q0 = p[4 * h], q1 = p[4 * h + 1], q2 = p[4 * h + 2], q3 = p[4 * h + 3];
        const uint32_t a = __builtin_amdgcn_perm(q1, q0, 0x05010400u);
        const uint32_t b = __builtin_amdgcn_perm(q3, q2, 0x05010400u);
        const uint32_t c = __builtin_amdgcn_perm(q1, q0, 0x07030602u);
        const uint32_t d = __builtin_amdgcn_perm(q3, q2, 0x07030602u);
        w[0 + h] = __builtin_amdgcn_perm(b, a, 0x05040100u);  // element 0 low/high
        w[2 + h] = __builtin_amdgcn_perm(b, a, 0x07060302u);  // element 1
        w[4 + h] = __builtin_amdgcn_perm(d, c, 0x05040100u);  // element 2
        w[6 + h] = __builtin_amdgcn_perm(d, c, 0x07060302u);  // element 3
      }
    };
    drive2<32>(L, n, full32 / 32, final, gout, fast, [&](uint32_t u, uint32_t (&w)[8]) {
      if (32 * u + 32 <= full32) {
        fast(u, w);
      } else {
        slow(2 * u, w);
        slow(2 * u + 1, w + 4);
      }
    });
  }
  cur.base = 0;
  cur.n = n;
  cur.swz = 0;
  return true;
}

// ---------------------------------------------------------------------------
// bitshuffle^-1 (8192-B blocks; bitshuffle_filter.cc:168-212)
// ---------------------------------------------------------------------------
template <int TS>
__device__ __forceinline__ bool f_bitshuffle(FastLds& L, View& cur, uint32_t& mo, uint32_t& mn, bool final,
                             uint8_t* gout, uint32_t cap) {
  if (mn < 8) return false;
  const uint32_t np = lds32(L.MD, mo), ps = lds32(L.MD, mo + 4);
  if (np != 1 || ps != cur.n) return false;
  if (final && ps > cap) return false;
  mo += 8;
  mn -= 8;
  const uint32_t n = ps, base = cur.base;
  if (n % TS != 0 || n % 8 != 0) {  // part copied, not shuffled
    if (final) final_copy(L, cur, gout);
    else __syncthreads();  // md reads done before a later stage rewrites MD
    return true;
  }
  const uint8_t* X = L.X;
  if (TS == 4 && final && n % 8192 == 0) {
    // Whole 8192-B blocks of 4-byte elements (C2 / C2i): a block is 32 bit
    // rows of 256 B (row 8b + k = bit k of byte b of every element), and
    // thread t' of the block's wave owns groups 4t'..4t'+3 (elements
    // 32t'..32t'+31): one dword per row holds its four groups' bytes.  Per
    // byte plane b, two 4x4 byte transposes of the 8 row dwords give each
    // group's 64-bit bit matrix, transpose8x8 turns it into the 8 elements'
    // byte b, and two more 4x4 transposes per group assemble the elements.
    // 32 LDS reads per thread instead of 128 byte reads.  The 128 output
    // bytes go back in place, swizzled, behind a barrier, and leave with
    // lane-consecutive 16-B stores (whole lines: the direct lane-strided
    // stores cost 1.4x the output bytes in HBM writes).
    const uint32_t t = tid_(), blk = t >> 6, tq = t & 63;
    const bool act = blk < n / 8192;  // n <= XCAP: at most 8 blocks, one per wave
    auto tr4 = [](uint32_t p0, uint32_t p1, uint32_t p2, uint32_t p3, uint32_t (&w)[4]) {
      const uint32_t a = __builtin_amdgcn_perm(p1, p0, 0x05010400u);
      const uint32_t b = __builtin_amdgcn_perm(p3, p2, 0x05010400u);
      const uint32_t c = __builtin_amdgcn_perm(p1, p0, 0x07030602u);
      const uint32_t d = __builtin_amdgcn_perm(p3, p2, 0x07030602u);
      w[0] = __builtin_amdgcn_perm(b, a, 0x05040100u);
      w[1] = __builtin_amdgcn_perm(b, a, 0x07060302u);
      w[2] = __builtin_amdgcn_perm(d, c, 0x05040100u);
      w[3] = __builtin_amdgcn_perm(d, c, 0x07060302u);
    };
    uint32_t E[4][8];  // group j: output dwords 0..7
    auto body = [&](auto AL) {
      const uint32_t rb = base + 8192 * blk + 4 * tq;
      uint64_t y[4][4];  // [group j][plane b]
#pragma unroll
      for (int b = 0; b < 4; b++) {
        uint32_t D[8];
#pragma unroll
        for (int k = 0; k < 8; k++) {
          const uint32_t a = rb + (8 * b + k) * 256;
          D[k] = decltype(AL)::value ? *(const uint32_t*)(X + a) : lds32(X, a);
        }
        uint32_t lo[4], hi[4];
        tr4(D[0], D[1], D[2], D[3], lo);
        tr4(D[4], D[5], D[6], D[7], hi);
#pragma unroll
        for (int j = 0; j < 4; j++) y[j][b] = transpose8x8(((uint64_t)hi[j] << 32) | lo[j]);
      }
#pragma unroll
      for (int j = 0; j < 4; j++) {
        uint32_t e0[4], e1[4];
        tr4((uint32_t)y[j][0], (uint32_t)y[j][1], (uint32_t)y[j][2], (uint32_t)y[j][3], e0);
        tr4((uint32_t)(y[j][0] >> 32), (uint32_t)(y[j][1] >> 32), (uint32_t)(y[j][2] >> 32),
            (uint32_t)(y[j][3] >> 32), e1);
#pragma unroll
        for (int m = 0; m < 4; m++) {
          E[j][m] = e0[m];
          E[j][4 + m] = e1[m];
        }
      }
    };
    if (act) {
      if ((base & 3) == 0) body(std::true_type{});  // (uniform) rows dword-aligned
      else body(std::false_type{});
    }
    __syncthreads();  // every row read before the elements overwrite them
    if (act) {
      // thread bytes [8192 blk + 128 t', +128) = units U0 + i, U0 = 512 blk + 8 t'
      const uint32_t u0 = 512 * blk + 8 * tq;
#pragma unroll
      for (int i = 0; i < 8; i++)
        *(uint4*)(L.X + 16 * (u0 + (i ^ (tq & 7)))) =
            make_uint4(E[i >> 1][4 * (i & 1)], E[i >> 1][4 * (i & 1) + 1], E[i >> 1][4 * (i & 1) + 2],
                       E[i >> 1][4 * (i & 1) + 3]);
    }
    __syncthreads();
    cur.base = 0;
    cur.n = n;
    cur.swz = 1;
    final_copy(L, cur, gout);
    return true;
  }
  constexpr int UB = 8 * TS < 16 ? 16 : 8 * TS;  // unit = whole 8-element groups
  constexpr int GPU_ = UB / (8 * TS);             // groups per unit
  drive<UB>(L, n, final, gout, [&](uint32_t u, uint32_t (&w)[UB / 4]) {
#pragma unroll
    for (int gq = 0; gq < GPU_; gq++) {
      const uint32_t o = u * UB + gq * 8 * TS;  // byte offset of the group
      const uint32_t blk = o >> 13, b0 = blk << 13;
      const uint32_t nb = n - b0 < 8192 ? n - b0 : 8192;
      const uint32_t ne = nb / TS, n8 = ne & ~7u, rowb = n8 >> 3;
      const uint32_t q = (o - b0) / (8 * TS);
      uint32_t out[2 * TS];
#pragma unroll
      for (int d = 0; d < 2 * TS; d++) out[d] = 0;
      if (q < rowb) {
#pragma unroll
        for (int b = 0; b < TS; b++) {
          uint64_t x = 0;
#pragma unroll
          for (int k = 0; k < 8; k++)
            x |= (uint64_t)X[base + b0 + (8 * b + k) * rowb + q] << (8 * k);
          const uint64_t y = transpose8x8(x);
          // element m, byte b -> byte m*TS + b of the group
#pragma unroll
          for (int m = 0; m < 8; m++) {
            const uint32_t pos = m * TS + b;
            const uint32_t byte = (uint32_t)(y >> (8 * m)) & 0xffu;
            out[pos >> 2] |= byte << (8 * (pos & 3));
          }
        }
      } else {
#pragma unroll
        for (int d = 0; d < 2 * TS; d++) out[d] = lds32(X, base + o + 4 * d);
      }
#pragma unroll
      for (int d = 0; d < 2 * TS; d++) w[gq * 2 * TS + d] = out[d];
    }
  });
  cur.base = 0;
  cur.n = n;
  return true;
}

// ---------------------------------------------------------------------------
// BWR^-1 (bit_width_reduction_filter.cc:352-404)
// TAB[w] = {in_off, bits | raw << 8, offset lo, offset hi}
// ---------------------------------------------------------------------------
template <int W, bool SGN>
__device__ __forceinline__ uint64_t bwr_elem(const uint8_t* X, uint32_t base, uint4 e, uint32_t j) {
  const uint32_t cb = (e.y & 0xffu) >> 3;
  uint64_t v = ldsn(X, base + e.x + j * cb, cb);
  if (SGN) v = (uint64_t)sext64(v, cb);
  return v + (((uint64_t)e.w << 32) | e.z);
}

// SZ: the next stage reads a swizzled view (1: slice stages PD / XOR,
// 2: a 4-byte byteshuffle, which needs whole 16-B plane units)
template <int W, bool SGN, int SZ, class M>
__device__ __forceinline__ bool f_bwr(FastLds& L, View& cur, uint32_t& mo, uint32_t& mn, bool final,
                      uint8_t* gout, uint32_t cap, uint32_t dts, uint32_t pos, M&& mark) {
  const uint32_t tid = tid_();
  if (mn < 8) return false;
  const uint32_t orig = lds32(L.MD, mo), nw = lds32(L.MD, mo + 4);
  const uint32_t E = dts + 5;
  if (nw == 0 || nw > TABN || 8 + nw * E > mn) return false;
  if (final ? orig > cap : orig > XCAP) return false;
  const uint32_t ws0 = lds32(L.MD, mo + 8 + dts + 1);
  bool bad = ws0 == 0 || ws0 % W != 0;
  // One pass over the windows (thread w owns window w): its entry, a DPP
  // wave scan of (compressed bytes, bytes) packed in a u64 (both sums
  // < 2^32) with the 'bad' / 'not raw' flags alongside, and its table entry
  // with the wave-local input offset -- all before the stage's single
  // barrier.  Readers add the exclusive prefix of the window's wave.  Every
  // window raw <=> the stage is the identity on the first orig bytes.
  uint32_t comp = 0, nb = 0;
  uint4 ent = make_uint4(0, 0, 0, 0);
  if (tid < nw) {
    const uint32_t eo = mo + 8 + tid * E;
    const uint64_t off = ldsn(L.MD, eo, dts);
    const uint32_t bits = L.MD[eo + dts];
    nb = lds32(L.MD, eo + dts + 1);
    const bool raw = bits >= 8u * W || (nb % W) != 0;
    comp = raw ? nb : (nb / W) * (bits >> 3);
    if (!raw && bits != 8 && bits != 16 && bits != 32) bad = true;
    if (tid + 1 < nw ? nb != ws0 : (nb == 0 || nb > ws0)) bad = true;
    if (nb > XCAP) bad = true;  // keeps the packed sums below 2^32
    ent = make_uint4(0, bits | (raw ? 0x100u : 0u), (uint32_t)off, (uint32_t)(off >> 32));
  }
  const uint32_t lane = tid & 63, wid = tid >> 6;
  const uint64_t packed = ((uint64_t)comp << 32) | nb;
  const uint64_t inc = wave_incscan_u64(packed);
  const bool badw = __ballot(bad) != 0;
  const bool cmpw = __ballot(tid < nw && !(ent.y & 0x100u)) != 0;
  if (tid < nw) {
    ent.x = (uint32_t)((inc - packed) >> 32);
    L.TAB[tid] = ent;
  }
  if (lane == 63) L.scan2[pos & 1][wid] = inc;
  if (lane == 0) L.scanf[pos & 1][wid] = (badw ? 1u : 0u) | (cmpw ? 2u : 0u);
  __syncthreads();
  static_assert(FNT / 64 == 8, "wave prefixes below assume 8 waves");
  uint64_t tot = 0;
  uint32_t fl = 0;
  // exclusive input-offset prefix of each wave, as separate values (an
  // array indexed by the window's wave would be demoted to scratch)
  uint32_t P0, P1, P2, P3, P4, P5, P6, P7;
#define TDBG_WPRE(i)                                              \
  P##i = __builtin_amdgcn_readfirstlane((uint32_t)(tot >> 32));   \
  tot += L.scan2[pos & 1][i];                                     \
  fl |= L.scanf[pos & 1][i];
  TDBG_WPRE(0) TDBG_WPRE(1) TDBG_WPRE(2) TDBG_WPRE(3) TDBG_WPRE(4) TDBG_WPRE(5) TDBG_WPRE(6) TDBG_WPRE(7)
#undef TDBG_WPRE
  const uint64_t tin = tot >> 32, tout = tot & 0xffffffffu;
  if ((fl & 1u) || tin > cur.n || tout != orig) return false;
  mo += 8 + nw * E;
  mn -= 8 + nw * E;
  if (!(fl & 2u)) {
    cur.n = orig;
    if (final) final_copy(L, cur, gout);
    return true;
  }
  // the input offset of window w: its wave-local offset + its wave's prefix
  auto wpre = [&](uint32_t w) -> uint32_t {
    const uint32_t i = w >> 6;
    const uint32_t a0 = (i & 1) ? P1 : P0, a1 = (i & 1) ? P3 : P2;
    const uint32_t a2 = (i & 1) ? P5 : P4, a3 = (i & 1) ? P7 : P6;
    const uint32_t b0 = (i & 2) ? a1 : a0, b1 = (i & 2) ? a3 : a2;
    return (i & 4) ? b1 : b0;
  };
  auto tab = [&](uint32_t w) -> uint4 {
    uint4 e = L.TAB[w];
    e.x += wpre(w);
    return e;
  };
  // Power-of-two windows of >= 128 B: the units one call of the fast unit
  // function covers (u = t + k FNT, t < 512) all lie in windows of one wave
  // (w >> 6 = u >> (log2 ws0 + 2) >= 9 bits), so the prefix is picked with
  // scalar selects.  (Clamped units of a final round may differ; their
  // results are discarded.)
  auto tab_u = [&](uint32_t w) -> uint4 {
    uint4 e = L.TAB[w];
    e.x += wpre(__builtin_amdgcn_readfirstlane(w));
    return e;
  };
  mark(6);  // TEMP diagnostics
  const bool so = !final && (SZ == 1 || (SZ == 2 && orig % 16 == 0));
  const uint8_t* X = L.X;
  const uint32_t base = cur.base;
  const bool pow2 = (ws0 & (ws0 - 1)) == 0;
  const uint32_t wsh = pow2 ? __builtin_ctz(ws0) : 0;
  auto win = [&](uint32_t o) -> uint32_t {
    const uint32_t w = pow2 ? (o >> wsh) : (o / ws0);
    return w < nw ? w : nw - 1;
  };
  const bool wuni = pow2 && wsh >= 7;
  if (W == 4 && ws0 % 16 == 0) {
    // 32-bit values: compressed widths are 8 or 16 bits (32 is raw), so a
    // 16-B output unit = 4 elements from <= 8 source bytes (q0, q1) with
    // 32-bit bit-field extracts; raw units take the 16 bytes as they are.
    auto fn16w4g = [&](uint32_t u, uint32_t (&wv)[4], auto&& tabf) {
      const uint32_t o = 16 * u, w = win(o);
      const uint4 e = tabf(w);
      const uint32_t ob = o - w * ws0;
      const bool raw = (e.y & 0x100u) != 0;
      const uint32_t bits = e.y & 0xf8u;  // 8 * compressed bytes
      const uint32_t src = base + e.x + (raw ? ob : (ob >> 2) * (bits >> 3));
      const uint32_t a = src & ~3u, sh = src & 3u;
      uint32_t d[5];
#pragma unroll
      for (int k = 0; k < 5; k++) d[k] = *(const uint32_t*)(X + a + 4 * k);
      uint32_t q[4];
#pragma unroll
      for (int k = 0; k < 4; k++) q[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
      const uint64_t Q = ((uint64_t)q[1] << 32) | q[0];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint32_t lo = k == 0 ? q[0] : (uint32_t)(Q >> (k * bits));
        const uint32_t v = SGN ? (uint32_t)__builtin_amdgcn_sbfe((int32_t)lo, 0, bits)
                               : __builtin_amdgcn_ubfe(lo, 0, bits);
        wv[k] = raw ? q[k] : v + e.z;
      }
    };
    auto fn16w4 = [&](uint32_t u, uint32_t (&wv)[4]) { fn16w4g(u, wv, tab); };
    // power-of-two windows >= 128 B: shifts instead of multiplies, the scalar
    // prefix pick, and the two compressed widths (8 / 16 bits) as plain
    // bit-field extracts of q0 / q1
    auto fn16w4u = [&](uint32_t u, uint32_t (&wv)[4]) {
      const uint32_t o = 16 * u;
      uint32_t w = o >> wsh;
      w = w < nw ? w : nw - 1;
      const uint4 e = tab_u(w);
      const uint32_t ob = o - (w << wsh);
      const bool raw = (e.y & 0x100u) != 0;
      const uint32_t bits = e.y & 0xf8u;  // 8 or 16 unless raw
      const uint32_t src = base + e.x + (raw ? ob : ((ob >> 2) << (bits >> 4)));
      const uint32_t a = src & ~3u, sh = src & 3u;
      uint32_t d[5];
#pragma unroll
      for (int k = 0; k < 5; k++) d[k] = *(const uint32_t*)(X + a + 4 * k);
      uint32_t q[4];
#pragma unroll
      for (int k = 0; k < 4; k++) q[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
      const bool w16 = bits > 8;
      const uint32_t hi = w16 ? q[1] : q[0];
      const uint32_t f[4][2] = {{q[0], 0u}, {q[0], bits}, {hi, w16 ? 0u : 16u}, {hi, w16 ? 16u : 24u}};
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint32_t v = SGN ? (uint32_t)__builtin_amdgcn_sbfe((int32_t)f[k][0], f[k][1], bits)
                               : __builtin_amdgcn_ubfe(f[k][0], f[k][1], bits);
        wv[k] = raw ? q[k] : v + e.z;
      }
    };
    auto part4 = [&](uint32_t u, uint32_t (&wv)[4]) {
      // partial last unit: element-wise (the window may hold fewer bytes)
#pragma unroll
      for (uint32_t k = 0; k < 4; k++) {
        const uint32_t o = 16 * u + 4 * k;
        const uint32_t w = win(o);
        const uint4 e = tab(w);
        const uint32_t ob = o - w * ws0;
        uint64_t v = 0;
        if (o < orig) {
          if (e.y & 0x100u) v = ldsn(X, base + e.x + ob, 4);
          else v = bwr_elem<W, SGN>(X, base, e, ob / 4);
        }
        wv[k] = (uint32_t)v;
      }
    };
    if (wuni) drive2<16>(L, orig, orig / 16, final, gout, fn16w4u, part4, so);
    else drive2<16>(L, orig, orig / 16, final, gout, fn16w4, part4, so);
  } else if ((W == 4 || W == 8) && ws0 % 16 == 0) {
    // Every 16-B output unit lies in one window: one TAB read per unit, the
    // unit's source bytes read as one aligned span, elements extracted in
    // registers.  Compressed elements of a unit span at most 8 bytes.
    constexpr uint32_t NE = 16 / W;
    auto fn16 = [&](uint32_t u, uint32_t (&wv)[4]) {
      const uint32_t o = 16 * u, w = win(o);
      const uint4 e = tab(w);
      const uint32_t ob = o - w * ws0;
      const bool raw = (e.y & 0x100u) != 0;
      const uint32_t cb = (e.y & 0xffu) >> 3;
      const uint32_t src = base + e.x + (raw ? ob : (ob / W) * cb);
      const uint32_t a = src & ~3u, sh = src & 3u;
      uint32_t d[5];
#pragma unroll
      for (int k = 0; k < 5; k++) d[k] = *(const uint32_t*)(X + a + 4 * k);
      uint32_t q[4];
#pragma unroll
      for (int k = 0; k < 4; k++) q[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
      if (raw) {
#pragma unroll
        for (int k = 0; k < 4; k++) wv[k] = q[k];
        return;
      }
      const uint64_t Q = (uint64_t)q[0] | ((uint64_t)q[1] << 32);
      const uint64_t off = ((uint64_t)e.w << 32) | e.z;
      const uint32_t bitsz = 8 * cb;
#pragma unroll
      for (uint32_t k = 0; k < NE; k++) {
        uint64_t v = Q >> (bitsz * k);
        v = bitsz >= 64 ? v : (v & ((1ull << bitsz) - 1));
        if (SGN) v = (uint64_t)sext64(v, cb);
        v += off;
        if (W == 4) {
          wv[k] = (uint32_t)v;
        } else {
          wv[2 * k] = (uint32_t)v;
          wv[2 * k + 1] = (uint32_t)(v >> 32);
        }
      }
    };
    drive2<16>(L, orig, orig / 16, final, gout, fn16, [&](uint32_t u, uint32_t (&wv)[4]) {
      // partial last unit: element-wise (the window may hold fewer bytes)
#pragma unroll
      for (uint32_t k = 0; k < NE; k++) {
        const uint32_t o = 16 * u + W * k;
        const uint32_t w = win(o);
        const uint4 e = tab(w);
        const uint32_t ob = o - w * ws0;
        uint64_t v = 0;
        if (o < orig) {
          if (e.y & 0x100u) v = ldsn(X, base + e.x + ob, W);
          else v = bwr_elem<W, SGN>(X, base, e, ob / W);
        }
        if (W == 4) {
          wv[k] = (uint32_t)v;
        } else {
          wv[2 * k] = (uint32_t)v;
          wv[2 * k + 1] = (uint32_t)(v >> 32);
        }
      }
    }, so);
  } else if (W == 8) {
    auto fn = [&](uint32_t u, uint32_t (&wv)[4]) {
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const uint32_t o = 16 * u + 8 * h;
        const uint32_t w = win(o);
        const uint4 e = tab(w);
        const uint32_t ob = o - w * ws0;
        uint64_t v;
        if (e.y & 0x100u) v = lds64(X, base + e.x + ob);
        else v = bwr_elem<W, SGN>(X, base, e, ob >> 3);
        wv[2 * h] = (uint32_t)v;
        wv[2 * h + 1] = (uint32_t)(v >> 32);
      }
    };
    drive2<16>(L, orig, orig / 16, final, gout, fn, fn, so);
  } else if (W == 4) {
    auto fn = [&](uint32_t u, uint32_t (&wv)[4]) {
      uint32_t w = win(16 * u);
      uint4 e = tab(w);
#pragma unroll
      for (int d = 0; d < 4; d++) {
        const uint32_t o = 16 * u + 4 * d;
        const uint32_t w2 = win(o);
        if (w2 != w) { w = w2; e = tab(w); }
        const uint32_t ob = o - w * ws0;
        if (e.y & 0x100u) wv[d] = lds32(X, base + e.x + ob);
        else wv[d] = (uint32_t)bwr_elem<W, SGN>(X, base, e, ob >> 2);
      }
    };
    drive2<16>(L, orig, orig / 16, final, gout, fn, fn, so);
  } else {  // W == 2: two elements per dword, windows may end mid-dword
    drive<16>(L, orig, final, gout, [&](uint32_t u, uint32_t (&wv)[4]) {
#pragma unroll
      for (int d = 0; d < 4; d++) {
        uint32_t v = 0;
#pragma unroll
        for (int h = 0; h < 2; h++) {
          const uint32_t o = 16 * u + 4 * d + 2 * h;
          const uint32_t w = win(o);
          const uint4 e = tab(w);
          const uint32_t ob = o - w * ws0;
          uint32_t x;
          if (e.y & 0x100u) x = lds32(X, base + e.x + ob) & 0xffffu;
          else x = (uint32_t)bwr_elem<W, SGN>(X, base, e, ob >> 1) & 0xffffu;
          v |= x << (16 * h);
        }
        wv[d] = v;
      }
    }, so);
  }
  cur.base = 0;
  cur.n = orig;
  cur.swz = so ? 1u : 0u;
  return true;
}

// ---------------------------------------------------------------------------
// scans with a per-thread element count
// ---------------------------------------------------------------------------
// Segmented sum (positive delta windows): aggregate (has_head, sum after the
// last head).  Exclusive scan; returns the carry into this thread's slice.
__device__ __forceinline__ uint64_t block_segscan(bool has, uint64_t sum, uint64_t* red) {
  const uint32_t lane = tid_() & 63, wid = tid_() >> 6;
  // (has head, sum since the last head) inclusive over the wave with DPP
  // moves (a lane with no source reads (0, 0), the identity)
  uint32_t ih = has;
  uint64_t is = sum;
  auto comb = [&](uint32_t oh, uint64_t os) {
    if (!ih) { is = os + is; ih = oh; }
  };
  comb(dpp0<DPP_ROW_SHR1>(ih), dpp0<DPP_ROW_SHR1>(is));
  comb(dpp0<DPP_ROW_SHR2>(ih), dpp0<DPP_ROW_SHR2>(is));
  comb(dpp0<DPP_ROW_SHR4>(ih), dpp0<DPP_ROW_SHR4>(is));
  comb(dpp0<DPP_ROW_SHR8>(ih), dpp0<DPP_ROW_SHR8>(is));
  comb(dpp0<DPP_ROW_BCAST15, 0xa>(ih), dpp0<DPP_ROW_BCAST15, 0xa>(is));
  comb(dpp0<DPP_ROW_BCAST31, 0xc>(ih), dpp0<DPP_ROW_BCAST31, 0xc>(is));
  // exclusive = the inclusive value of lane - 1
  uint32_t eh = __shfl_up(ih, 1, 64);
  uint64_t es = __shfl_up(is, 1, 64);
  if (lane == 0) { eh = 0; es = 0; }
  if (lane == 63) { red[2 * wid] = ih; red[2 * wid + 1] = is; }
  __syncthreads();
  uint64_t ps = 0;
  for (uint32_t i = 0; i < wid; i++) {
    if (red[2 * i]) ps = red[2 * i + 1];
    else ps += red[2 * i + 1];
  }
  __syncthreads();
  return eh ? es : ps + es;
}

// packed element access in a slice register file (static indices only)
template <int W, int N>
__device__ __forceinline__ uint64_t rget(const uint32_t (&r)[N], int k) {
  if (W == 8) return (uint64_t)r[2 * k] | ((uint64_t)r[2 * k + 1] << 32);
  if (W == 4) return r[k];
  if (W == 2) return (r[k >> 1] >> (16 * (k & 1))) & 0xffffu;
  return (r[k >> 2] >> (8 * (k & 3))) & 0xffu;
}
template <int W, int N>
__device__ __forceinline__ void rset(uint32_t (&r)[N], int k, uint64_t v) {
  if (W == 8) { r[2 * k] = (uint32_t)v; r[2 * k + 1] = (uint32_t)(v >> 32); return; }
  if (W == 4) { r[k] = (uint32_t)v; return; }
  if (W == 2) {
    const int s = 16 * (k & 1);
    r[k >> 1] = (r[k >> 1] & ~(0xffffu << s)) | (((uint32_t)v & 0xffffu) << s);
    return;
  }
  const int s = 8 * (k & 3);
  r[k >> 2] = (r[k >> 2] & ~(0xffu << s)) | (((uint32_t)v & 0xffu) << s);
}

// write a slice register file to X[0, n) (after the barrier the caller issues)
template <int N>
__device__ __forceinline__ void slice_store(FastLds& L, const uint32_t (&r)[N], uint32_t n, bool swz = false) {
  const uint32_t t = tid_(), s0 = t * (4 * N);
#pragma unroll
  for (int k = 0; k < N / 4; k++) {
    const uint32_t o = s0 + 16 * k;
    if (o < n)
      *(uint4*)(L.X + (swz ? 16 * swz_u(o >> 4) : o)) = make_uint4(r[4 * k], r[4 * k + 1], r[4 * k + 2], r[4 * k + 3]);
  }
}

// ---------------------------------------------------------------------------
// PD^-1 (positive_delta_filter.cc:324-375): segmented prefix sums
// TAB[w] = {first lo, first hi, nb, raw}
// ---------------------------------------------------------------------------
template <int W, int SZ>
__device__ __forceinline__ bool f_pd(FastLds& L, View& cur, uint32_t& mo, uint32_t& mn, bool final,
                     uint8_t* gout, uint32_t cap, uint32_t dts) {
  const uint32_t tid = tid_();
  if (mn < 4) return false;
  const uint32_t nw = lds32(L.MD, mo);
  const uint32_t E = dts + 4;
  const uint32_t n = cur.n;
  if (nw == 0 || nw > TABN || 4 + nw * E > mn) return false;
  if ((final && n > cap) || n > (uint32_t)(FNT * SP)) return false;
  const uint32_t ws0 = lds32(L.MD, mo + 4 + dts);
  bool bad = ws0 == 0 || ws0 % W != 0 || ws0 / W < (uint32_t)(SP / W);
  uint32_t nb = 0;
  if (tid < nw) {
    const uint32_t eo = mo + 4 + tid * E;
    const uint64_t first = ldsn(L.MD, eo, dts);
    nb = lds32(L.MD, eo + dts);
    if (tid + 1 < nw ? nb != ws0 : (nb == 0 || nb > ws0)) bad = true;
    L.TAB[tid] = make_uint4((uint32_t)first, (uint32_t)(first >> 32), nb, (nb % W) ? 1u : 0u);
  }
  uint64_t tot;
  block_exscan_u64<FNT>(nb, tot, L.red);
  bad = bad || tot != n;
  if (block_any(bad)) return false;
  mo += 4 + nw * E;
  mn -= 4 + nw * E;
  constexpr int EP = SP / W;  // elements per thread slice
  const uint32_t s0 = tid * SP;
  const uint32_t e0 = s0 / W;     // first element of the slice
  const uint32_t epw = ws0 / W;   // elements per (full) window
  const uint32_t nel = n / W;     // whole elements (a raw tail window may leave bytes)
  // pass 1: the slice's input bytes as dwords (raw-window bytes pass through
  // untouched), deltas, and the segment aggregate (has head, sum after it)
  uint32_t r[SPD];
  slice_load(L, cur, r);
  // A slice holds at most EP <= epw elements, so it spans at most two
  // windows: w0 (continued from the previous slice unless rem0 == 0) and,
  // from element kh on, w0 + 1.
  const uint32_t w0 = e0 / epw;
  const uint32_t rem0 = e0 - w0 * epw;
  const uint32_t kh = rem0 == 0 ? 0u : epw - rem0;  // slice index of the head
  bool has = false;
  uint64_t sum = 0;
#pragma unroll
  for (int k = 0; k < EP; k++) {
    if (e0 + k < nel) {
      if ((uint32_t)k == kh) { has = true; sum = 0; }
      sum += rget<W>(r, k);
    }
  }
  const uint64_t carry = block_segscan(has, sum, L.red);
  if (e0 < nel) {
    const uint32_t wa = w0 < nw ? w0 : nw - 1;
    const uint4 ta = L.TAB[wa];
    const uint4 tb = L.TAB[wa + 1 < nw ? wa + 1 : wa];
    const uint64_t fa = ((uint64_t)ta.y << 32) | ta.x, fb = ((uint64_t)tb.y << 32) | tb.x;
    uint64_t run = rem0 == 0 ? fa : fa + carry;
#pragma unroll
    for (int k = 0; k < EP; k++) {
      const bool second = rem0 != 0 && (uint32_t)k >= kh;
      const bool raw = second ? tb.w != 0 : ta.w != 0;
      if (e0 + k < nel && !raw) {
        if (rem0 != 0 && (uint32_t)k == kh) run = fb;
        run += rget<W>(r, k);
        rset<W>(r, k, run);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  __syncthreads();
  // swizzled for a slice / byteshuffle consumer (SZ as f_bwr) or the final copy
  const bool so = final || SZ == 1 || (SZ == 2 && n % 16 == 0);
  slice_store(L, r, n, so);
  __syncthreads();
  cur.base = 0;
  cur.n = n;
  cur.swz = so ? 1u : 0u;
  if (final) {
    final_copy(L, cur, gout);
  }
  return true;
}

// ---------------------------------------------------------------------------
// serial codecs for tiny metadata parts (thread 0)
// ---------------------------------------------------------------------------
// DoubleDelta::decompress of one part (dd_compressor.cc:314-360); false on
// any anomaly.  rd(o) returns source byte o, wr(o, v) stores output byte o.
template <class R, class Wr>
__device__ __forceinline__ bool dd_serial_g(R&& rd8, uint32_t cn, Wr&& wr8, uint32_t un, uint32_t W) {
  if (cn < 9) return false;
  const uint32_t b = rd8(0);
  uint64_t num = 0;
  for (int i = 0; i < 8; i++) num |= (uint64_t)rd8(1 + i) << (8 * i);
  if (b >= 8 * W - 1) {
    if (cn - 9 != un) return false;
    for (uint32_t i = 0; i < un; i++) wr8(i, rd8(9 + i));
    return true;
  }
  if (num * W != un || num == 0) return false;
  auto rd = [&](uint32_t off, uint32_t k) {
    uint64_t v = 0;
    for (uint32_t i = 0; i < k; i++) v |= (uint64_t)rd8(off + i) << (8 * i);
    return v;
  };
  if (cn < 9 + W) return false;
  uint64_t x0 = rd(9, W);
  for (uint32_t i = 0; i < W; i++) wr8(i, (uint8_t)(x0 >> (8 * i)));
  if (num == 1) return true;
  if (cn < 9 + 2 * W) return false;
  uint64_t x1 = rd(9 + W, W);
  for (uint32_t i = 0; i < W; i++) wr8(W + i, (uint8_t)(x1 >> (8 * i)));
  if (num == 2) return true;
  const uint64_t words = ((num - 2) * (b + 1) + 63) / 64;
  if (9 + 2 * W + 8 * words > cn) return false;
  const uint32_t bs = 9 + 2 * W;
  uint64_t d = x1 - x0, x = x1;
  for (uint64_t i = 2; i < num; i++) {
    const uint64_t s = (i - 2) * (b + 1);
    const uint64_t wi = s >> 6;
    const uint32_t r = (uint32_t)(s & 63);
    uint64_t hi = rd(bs + 8 * wi, 8) << r;
    if (r + b + 1 > 64) hi |= rd(bs + 8 * (wi + 1), 8) >> (64 - r);
    const uint64_t code = hi >> (63 - b);
    const uint64_t mag = b ? (code & ((1ull << b) - 1)) : 0;
    const uint64_t e = ((code >> b) & 1) ? (0 - mag) : mag;
    d += e;
    x += d;
    for (uint32_t k = 0; k < W; k++) wr8(i * W + k, (uint8_t)(x >> (8 * k)));
  }
  return true;
}

__device__ bool dd_serial(const uint8_t* src, uint32_t cn, uint8_t* dst, uint32_t un, uint32_t W) {
  return dd_serial_g([&](uint32_t o) -> uint32_t { return src[o]; }, cn,
                     [&](uint32_t o, uint8_t v) { dst[o] = v; }, un, W);
}

__device__ bool rle_serial(const uint8_t* src, uint32_t cn, uint8_t* dst, uint32_t un, uint32_t cs) {
  const uint32_t rs = cs + 2;
  if (cn % rs) return false;
  uint32_t o = 0;
  for (uint32_t r = 0; r < cn / rs; r++) {
    const uint32_t len = ((uint32_t)src[r * rs + cs] << 8) | src[r * rs + cs + 1];
    if (o + (uint64_t)len * cs > un) return false;
    for (uint32_t j = 0; j < len; j++)
      for (uint32_t k = 0; k < cs; k++) dst[o + j * cs + k] = src[r * rs + k];
    o += len * cs;
  }
  return o == un;
}

// ---------------------------------------------------------------------------
// DD data part (block-parallel, in place)
// ---------------------------------------------------------------------------
// Double-delta tuple (E, X) exclusive scan in the value width's arithmetic
// (U = uint32_t for W <= 4: everything is modulo 2^(8W) anyway); cnt
// elements per thread.
// (callers issue a barrier before anything else writes `red`: the scan's
// own trailing barrier is left out)
template <class U>
__device__ __forceinline__ void block_ddscan_u(U& E, U& Xs, uint32_t cnt, U* red) {
  const uint32_t lane = tid_() & 63, wid = tid_() >> 6;
  U iE = E, iX = Xs;
  // DPP steps: the received segment precedes this lane's own segment of
  // `len` lanes (row_shr:d: d lanes; bcast15 into rows 1, 3: lane%32 - 15;
  // bcast31 into rows 2, 3: lane - 31); a lane with no source reads (0, 0)
  auto comb = [&](U oE, U oX, uint32_t len) {
    iX = oX + iX + (U)len * (U)cnt * oE;
    iE = oE + iE;
  };
  comb(dpp0<DPP_ROW_SHR1>(iE), dpp0<DPP_ROW_SHR1>(iX), 1);
  comb(dpp0<DPP_ROW_SHR2>(iE), dpp0<DPP_ROW_SHR2>(iX), 2);
  comb(dpp0<DPP_ROW_SHR4>(iE), dpp0<DPP_ROW_SHR4>(iX), 4);
  comb(dpp0<DPP_ROW_SHR8>(iE), dpp0<DPP_ROW_SHR8>(iX), 8);
  comb(dpp0<DPP_ROW_BCAST15, 0xa>(iE), dpp0<DPP_ROW_BCAST15, 0xa>(iX), (lane & 31) - 15);
  comb(dpp0<DPP_ROW_BCAST31, 0xc>(iE), dpp0<DPP_ROW_BCAST31, 0xc>(iX), lane - 31);
  // exclusive from inclusive: iX = eX + X_own + cnt * eE (own = 1 lane)
  const U eE = iE - E, eX = iX - Xs - (U)cnt * eE;
  if (lane == 63) { red[2 * wid] = iE; red[2 * wid + 1] = iX; }
  __syncthreads();
  U PE = 0, PX = 0;
#pragma unroll
  for (int i = 0; i < FNT / 64; i++) {
    if ((uint32_t)i < wid) {
      PX = PX + red[2 * i + 1] + (U)64 * (U)cnt * PE;
      PE += red[2 * i];
    }
  }
  E = PE + eE;
  Xs = PX + eX + (U)lane * (U)cnt * PE;
}

// LDS byte offset of MSB-first 32-bit chunk c of the u64 word stream at bs
// (word c/2 little-endian: its high dword is chunk 2k, its low dword 2k+1)
__device__ __forceinline__ uint32_t dd_chunk_off(uint32_t bs, uint32_t c) {
  return bs + 8 * (c >> 1) + ((c & 1) ? 0u : 4u);
}

// DoubleDelta data part, block-parallel, in place: x_i from the tuple scan of
// the codes.  Arithmetic is modulo 2^(8W) (32-bit lanes for W <= 4), which is
// exactly the reference's (T)(dd + 2*x[i-1] - x[i-2]) (dd_compressor.cc:355).
// Each thread owns EP = SP / W consecutive values: it decodes their codes
// once into registers (independent chunk reads in groups of DG), scans the
// (E, X) tuple over the workgroup, then emits x from the registers.
template <int W, bool ALIGNED, class M>
__device__ __forceinline__ void dd_decode_part_t(FastLds& L, uint32_t src, uint32_t b, uint32_t num,
                                                 M&& mark) {
  typedef typename std::conditional<(W == 8), uint64_t, uint32_t>::type U;
  constexpr int EP = SP / W;   // 32 (W = 4) or 16 (W = 8) values per thread
  constexpr int DG = 4;        // codes per group of in-flight LDS reads
  constexpr int NC = W == 8 ? 3 : 2;  // chunks per code window
  const uint8_t* X = L.X;
  const U x0 = (U)ldsn(X, src + 9, W), x1 = (U)ldsn(X, src + 9 + W, W);
  const uint32_t bs = src + 9 + 2 * W;
  const U dinit = x1 - x0, xinit = x0 - dinit;
  const uint32_t cb = b + 1;
  const uint32_t i0 = tid_() * EP;
  const uint32_t lim = XCAP - 8;  // clamp for the (masked) reads of absent codes
  U e[EP];
#pragma unroll
  for (int g = 0; g < EP; g += DG) {
    uint32_t ch[DG][NC];
#pragma unroll
    for (int q = 0; q < DG; q++) {
      const uint32_t i = i0 + g + q;
      const uint32_t s = (i >= 2 ? i - 2 : 0) * cb;
      const uint32_t c = s >> 5;
#pragma unroll
      for (int h = 0; h < NC; h++) {
        uint32_t off = dd_chunk_off(bs, c + h);
        off = off < lim ? off : 0;
        ch[q][h] = ALIGNED ? *(const uint32_t*)(X + off) : lds32(X, off);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < DG; q++) {
      const uint32_t i = i0 + g + q;
      const uint32_t r = ((i >= 2 ? i - 2 : 0) * cb) & 31;
      U v;
      if (W == 8) {
        uint64_t top = (((uint64_t)ch[q][0] << 32) | ch[q][1]) << r;
        top |= r ? (uint64_t)ch[q][NC - 1] >> (32 - r) : 0ull;
        const uint64_t code = top >> (63 - b);
        const uint64_t mag = code & ((1ull << b) - 1);
        v = (U)(((code >> b) & 1) ? 0 - mag : mag);
      } else {
        const uint32_t top = r ? __builtin_amdgcn_alignbit(ch[q][0], ch[q][1], 32 - r) : ch[q][0];
        const uint32_t code = top >> (31 - b);
        const uint32_t mag = code & ((1u << b) - 1);
        v = (U)(((code >> b) & 1) ? 0u - mag : mag);
      }
      e[g + q] = (i >= 2 && i < num) ? v : (U)0;
    }
  }
  // per-thread aggregates, workgroup tuple scan
  U E = 0, Xs = 0;
#pragma unroll
  for (int k = 0; k < EP; k++) {
    E += e[k];
    Xs += E;
  }
  block_ddscan_u<U>(E, Xs, EP, (U*)L.red);
  mark(7);  // diagnostics: code reads + scan
  U d = dinit + E;
  U x = xinit + (U)i0 * dinit + Xs;
#pragma unroll
  for (int k = 0; k < EP; k++) {  // x in place of the codes (register pressure)
    d += e[k];
    x += d;
    e[k] = x;
  }
  __syncthreads();  // every code read before the values overwrite them
  {
    const uint32_t s0 = tid_() * SP, n = num * W;
#pragma unroll
    for (int q = 0; q < SP / 16; q++) {
      const uint32_t o = s0 + 16 * q;
      uint4 v;
      if (W == 8) {
        const uint64_t a = (uint64_t)e[2 * q], c = (uint64_t)e[2 * q + 1];
        v = make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)c, (uint32_t)(c >> 32));
      } else {
        v = make_uint4((uint32_t)e[4 * q], (uint32_t)e[4 * q + 1], (uint32_t)e[4 * q + 2],
                       (uint32_t)e[4 * q + 3]);
      }
      if (o < n) *(uint4*)(L.X + o) = v;
    }
  }
  __syncthreads();
}

// DoubleDelta data part for 32-bit values (codes <= 31 bits), in place.
//  1. The bitstream's u64 words are rewritten into Y = X[16, 16 + 8*nw) in
//     REVERSED word order (Y word j = stream word nw-1-j; one aligned 16-B
//     unit per lane, gathered to registers, barrier, written back).
//     MSB-first 32-bit chunk c of the stream then sits at Y dword K - c
//     (K = 2*nw - 1), so chunks c and c+1 are the dword pair at K - c - 1
//     whose little-endian 64-bit value is chunk_c:chunk_c+1 -- one
//     ds_read2_b32 and one 64-bit shift extract any code.  (The last
//     chunk's pair starts at Y dword -1: X[12, 16), hence the 16-B offset.)
//  2. Each thread decodes its 32 consecutive codes into registers, the
//     (E, X) tuple is scanned over the workgroup, x is emitted from the
//     registers and stored back over X after a barrier.
template <class M>
__device__ __forceinline__ void dd_decode_part32(FastLds& L, uint32_t src, uint32_t b, uint32_t num,
                                                 M&& mark) {
  typedef uint32_t U;
  constexpr int EP = SP / 4;  // 32 values per thread
  constexpr int NU = (XCAP + 16 * FNT - 1) / (16 * FNT);
  const uint8_t* X = L.X;
  const U x0 = lds32(X, src + 9), x1 = lds32(X, src + 13);
  const uint32_t bs = src + 17;
  const uint32_t cb = b + 1;
  const uint32_t nw = (uint32_t)(((uint64_t)(num - 2) * cb + 63) >> 6);  // words holding codes
  const uint32_t t = tid_();
  {
    // 1. reversed-word copy of the stream to X[0, 8 nw)
    const uint32_t nu = (nw + 1) >> 1;
    uint32_t r[NU][4];
#pragma unroll
    for (int k = 0; k < NU; k++) {
      const uint32_t u = t + k * FNT;
      // Y words 2u, 2u+1 = stream words nw-1-2u, nw-2-2u: the 16 stream
      // bytes starting at word nw-2-2u (clamped at the stream start; a
      // missing word is never read by a code)
      const int32_t w = (int32_t)nw - 2 - 2 * (int32_t)u;
      const uint32_t o = bs + 8 * (uint32_t)(w < 0 ? 0 : w);
      const uint32_t a = o & ~3u, sh = o & 3u;
      uint32_t d[5];
#pragma unroll
      for (int q = 0; q < 5; q++) d[q] = *(const uint32_t*)(X + (a + 4 * q < XCAP ? a + 4 * q : 0));
      __builtin_amdgcn_sched_barrier(0);
      uint32_t v[4];
#pragma unroll
      for (int q = 0; q < 4; q++) v[q] = __builtin_amdgcn_alignbyte(d[q + 1], d[q], sh);
      // (word nw-2-2u, word nw-1-2u) -> (Y word 2u, Y word 2u+1) swapped
      r[k][0] = v[2]; r[k][1] = v[3]; r[k][2] = v[0]; r[k][3] = v[1];
      if (w < 0) { r[k][0] = v[0]; r[k][1] = v[1]; }  // odd nw: Y word 2u = stream word 0
      (void)nu;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NU; k++) {
      const uint32_t u = t + k * FNT;
      if (u < nu) *(uint4*)(L.X + 16 + 16 * u) = make_uint4(r[k][0], r[k][1], r[k][2], r[k][3]);
    }
    __syncthreads();
  }
  // 2. codes -> registers
  const int32_t K1 = 2 * (int32_t)nw - 2;  // Y dword of chunk c+1 is K1 - c ... pair base
  const uint32_t i0 = t * EP;
  const uint32_t mb = b ? (1u << b) - 1 : 0u;
  const uint32_t tsh = 64 - cb;
  U e[EP];
#pragma unroll
  for (int g = 0; g < EP; g += 8) {
    uint64_t V[8];
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const uint32_t i = i0 + g + q;
      const uint32_t sb = (i >= 2 ? i - 2 : 0) * cb;
      int32_t di = K1 - (int32_t)(sb >> 5);
      di = di < -4 ? -4 : di;  // absent codes (i >= num) stay inside X
      // two dwords, 4-B aligned only (ds_read2_b32, never an unaligned b64)
      const uint32_t* Y32 = (const uint32_t*)(X + 16);
      V[q] = ((uint64_t)Y32[di + 1] << 32) | Y32[di];
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const uint32_t i = i0 + g + q;
      const uint32_t sb = (i >= 2 ? i - 2 : 0) * cb;
      // V = chunk_c:chunk_c+1, the code at bit r = sb & 31 of chunk c
      const uint32_t code = (uint32_t)(V[q] >> (tsh - (sb & 31)));
      const uint32_t mag = code & mb;
      const uint32_t neg = (uint32_t)__builtin_amdgcn_sbfe((int32_t)code, b, 1);  // 0 or ~0
      const U v = (mag ^ neg) - neg;
      e[g + q] = (i >= 2 && i < num) ? v : 0u;
    }
  }
  U E = 0, Xs = 0;
#pragma unroll
  for (int k = 0; k < EP; k++) {
    E += e[k];
    Xs += E;
  }
  block_ddscan_u<U>(E, Xs, EP, (U*)L.red);
  mark(7);  // diagnostics: realign + code reads + scan
  const U dinit = x1 - x0, xinit = x0 - dinit;
  U d = dinit + E;
  U x = xinit + (U)i0 * dinit + Xs;
#pragma unroll
  for (int k = 0; k < EP; k++) {
    d += e[k];
    x += d;
    e[k] = x;
  }
  __syncthreads();  // every code read before the values overwrite the stream
  {
    const uint32_t s0 = t * SP, n = num * 4;
#pragma unroll
    for (int q = 0; q < SP / 16; q++) {
      const uint32_t o = s0 + 16 * q;
      if (o < n) *(uint4*)(L.X + o) = make_uint4(e[4 * q], e[4 * q + 1], e[4 * q + 2], e[4 * q + 3]);
    }
  }
  __syncthreads();
}

// DoubleDelta data part for 32-bit values, code width CB = bitsize + 1 known
// at compile time.  Thread t owns codes [32t, 32t + 32): exactly the 32-bit
// MSB-first stream chunks [t CB, t CB + CB), so every code's chunk index and
// bit offset inside the thread's chunk window are constants.  The window is
// read straight from the BWR / load output (CB + 3 aligned dwords, byte-
// realigned with one alignbyte each; chunk 2k of the stream is the HIGH dword
// of little-endian word k, so chunk k of the window is stream dword
// (p + k) ^ 1 with p = t CB & 1).  No realignment pass, no per-code LDS read.
//
// Codes past the last value (j >= num - 2) decode whatever bits follow the
// stream; they only reach the aggregates carried into later threads, whose
// values all lie past num and are never stored.
template <int CB>
__device__ __forceinline__ void dd32_codes_cb(const uint8_t* X, uint32_t bs, uint32_t t, uint32_t (&e)[32]) {
  constexpr int ND = CB + 3;
  const uint32_t c0 = t * CB;
  const uint32_t sb = bs + 8 * (c0 >> 1);
  const uint32_t a = sb & ~3u, sh = sb & 3u;
  // all-ones when the window starts at an odd chunk; opaque, so the select
  // below stays a bit-select (a visible p ? M[..] : M[..] becomes a dynamic
  // index into a scratch copy of M)
  uint32_t pm = (c0 & 1) ? ~0u : 0u;
  asm volatile("" : "+v"(pm));
  uint32_t A[ND];
#pragma unroll
  for (int k = 0; k < ND; k++) A[k] = *(const uint32_t*)(X + a + 4 * k);
  uint32_t M[CB + 2];
#pragma unroll
  for (int k = 0; k < CB + 2; k++) M[k] = __builtin_amdgcn_alignbyte(A[k + 1], A[k], sh);
  uint32_t C[CB];
#pragma unroll
  for (int k = 0; k < CB; k++) C[k] = (M[(k + 1) ^ 1] & pm) | (M[k ^ 1] & ~pm);
#pragma unroll
  for (int q = 0; q < 32; q++) {
    constexpr int B = CB - 1;
    const int P = q * CB, k = P >> 5, r = P & 31;
    // sign = top bit of the code, bit 31 - r of chunk k
    const uint32_t sg = (uint32_t)__builtin_amdgcn_sbfe((int32_t)C[k], 31 - r, 1);
    uint32_t mag;
    if (r + CB <= 32) {
      mag = B ? __builtin_amdgcn_ubfe(C[k], 32 - r - CB, B) : 0u;
    } else {
      const uint32_t z = __builtin_amdgcn_alignbit(C[k], C[k + 1], 64 - r - CB);
      mag = z & ((1u << B) - 1);
    }
    e[q] = (mag ^ sg) - sg;
  }
}

// reads of the thread windows stay inside L.X for every thread of the block
__device__ __forceinline__ bool dd32_fast_ok(uint32_t bs, uint32_t cb) {
  return cb >= 2 && cb <= 32 && bs + 8 * (((FNT - 1) * cb) >> 1) + 4 * (cb + 3) + 4 <= XCAP;
}

template <bool SWZ, class M>
__device__ __forceinline__ bool dd_decode_part32_cb(FastLds& L, uint32_t src, uint32_t b, uint32_t num,
                                                    M&& mark) {
  typedef uint32_t U;
  const uint8_t* X = L.X;
  const U x0 = lds32(X, src + 9), x1 = lds32(X, src + 13);
  const uint32_t bs = src + 17;
  const uint32_t t = tid_();
  U e[32];
  switch (b + 1) {
#define TDBG_DDCB(n) \
    case n: dd32_codes_cb<n>(X, bs, t, e); break;
    TDBG_DDCB(2) TDBG_DDCB(3) TDBG_DDCB(4) TDBG_DDCB(5) TDBG_DDCB(6) TDBG_DDCB(7) TDBG_DDCB(8)
    TDBG_DDCB(9) TDBG_DDCB(10) TDBG_DDCB(11) TDBG_DDCB(12) TDBG_DDCB(13) TDBG_DDCB(14) TDBG_DDCB(15)
    TDBG_DDCB(16) TDBG_DDCB(17) TDBG_DDCB(18) TDBG_DDCB(19) TDBG_DDCB(20) TDBG_DDCB(21) TDBG_DDCB(22)
    TDBG_DDCB(23) TDBG_DDCB(24) TDBG_DDCB(25) TDBG_DDCB(26) TDBG_DDCB(27) TDBG_DDCB(28) TDBG_DDCB(29)
    TDBG_DDCB(30) TDBG_DDCB(31)
    default: dd32_codes_cb<32>(X, bs, t, e); break;
#undef TDBG_DDCB
  }
  U E = 0, Xs = 0;
#pragma unroll
  for (int k = 0; k < 32; k++) {
    E += e[k];
    Xs += E;
  }
  block_ddscan_u<U>(E, Xs, 32, (U*)L.red);
  mark(7);  // diagnostics: code reads + scan
  // state after codes [0, 32t): d_{32t+1}, x_{32t+1}
  const U d1 = x1 - x0;
  U d = d1 + E;
  U x = x1 + (U)(32 * t) * d1 + Xs;
  U v[32];
  v[0] = x - d;
  v[1] = x;
#pragma unroll
  for (int k = 2; k < 32; k++) {
    d += e[k - 2];
    x += d;
    v[k] = x;
  }
  __syncthreads();  // every stream read before the values overwrite it
  // swizzled layout for a following 4-byte byteshuffle (its planes then
  // start on 16-B unit boundaries: num % 4 == 0)
  const bool swz = SWZ && (num & 3) == 0;
  {
    const uint32_t s0 = t * SP, n = num * 4, rot = swz ? (t & 7) : 0u;
#pragma unroll
    for (int q = 0; q < SP / 16; q++) {
      const uint32_t o = s0 + 16 * q;
      if (o < n)
        *(uint4*)(L.X + s0 + 16 * (q ^ rot)) = make_uint4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
    }
  }
  __syncthreads();
  return swz;
}

// returns true when the output was written in the swz_dw layout
template <int W, bool SWZ, class M>
__device__ __forceinline__ bool dd_decode_part(FastLds& L, uint32_t src, uint32_t b, uint64_t num,
                                               M&& mark) {
  if (W == 4 && dd32_fast_ok(src + 17, b + 1)) return dd_decode_part32_cb<SWZ>(L, src, b, (uint32_t)num, mark);
  if (W == 4) dd_decode_part32(L, src, b, (uint32_t)num, mark);
  else if (((src + 9 + 2 * W) & 3) == 0) dd_decode_part_t<W, true>(L, src, b, (uint32_t)num, mark);
  else dd_decode_part_t<W, false>(L, src, b, (uint32_t)num, mark);
  return false;
}

// ---------------------------------------------------------------------------
// compression filter (DD / RLE) -- compression_filter.cc:303-347,413-486
// ---------------------------------------------------------------------------

// Reads the compression md header (compression_filter.cc:323-347) into
// L.pairs; returns false unless it is one data part plus <= 15 md parts that
// fit.  On return (uniform): nmd, data part (src, cn, un), md total.
__device__ bool comp_header(FastLds& L, View cur, uint32_t mo, uint32_t mn, uint32_t& nmd,
                            uint32_t& dsrc, uint32_t& dcn, uint32_t& dun, uint32_t& md_total) {
  if (mn < 8) return false;
  nmd = lds32(L.MD, mo);
  const uint32_t nd = lds32(L.MD, mo + 4);
  if (nd != 1 || nmd > 15 || 8 + 8 * (nmd + 1) > mn) return false;
  uint32_t p = 0;
  md_total = 0;
  for (uint32_t i = 0; i <= nmd; i++) {
    const uint32_t un = lds32(L.MD, mo + 8 + 8 * i), cn = lds32(L.MD, mo + 12 + 8 * i);
    if (tid_() == 0) {
      L.pairs[3 * i] = un;
      L.pairs[3 * i + 1] = cn;
      L.pairs[3 * i + 2] = p;
    }
    if (i < nmd) md_total += un;
    dsrc = cur.base + p;
    dcn = cn;
    dun = un;
    p += cn;
  }
  return p <= cur.n && md_total <= MDCAP;
}

template <int W, bool SWZ, class M>
__device__ __forceinline__ bool f_dd(FastLds& L, View& cur, uint32_t& mo, uint32_t& mn, bool final,
                     uint8_t* gout, uint32_t cap, M&& mark) {
  // compression md header (compression_filter.cc:323-347) from a wave
  // snapshot of MD; part table: (un, cn) pairs, md parts first
  if (mn < 8) return false;
  const uint32_t sm = snap_take(L.MD, mo);
  const uint32_t sx = snap_take(L.X, cur.base);
  const uint32_t nmd = snap32(sm, 0), nd = snap32(sm, 4);
  if (nd != 1 || nmd > 15 || 8 + 8 * (nmd + 1) > mn) return false;
  uint32_t p = 0, mdt = 0, src = 0, c = 0, u = 0;
  for (uint32_t i = 0; i <= nmd; i++) {
    const uint32_t un = snap32(sm, 8 + 8 * i), cn = snap32(sm, 12 + 8 * i);
    if (i < nmd) mdt += un;
    src = p;
    c = cn;
    u = un;
    p += cn;
  }
  if (p > cur.n || mdt > MDCAP) return false;
  if (c < 9) return false;
  const bool in_snap = src + 9 + 8 <= 256;  // md parts and the data header in the snapshot
  const uint32_t b = in_snap ? snap8(sx, src) : L.X[cur.base + src];
  const uint64_t num = in_snap ? snapn(sx, src + 1, 8) : ldsn(L.X, cur.base + src + 1, 8);
  const bool raw = b >= 8u * W - 1;
  if (final && u > cap) return false;
  if (raw) {
    if (c - 9 != u) return false;
  } else {
    // b >= 1 and every word holding a code present: the reference's reads
    // and writes all succeed (a sign bit ending a word forces the next word's
    // read, which b >= 1 needs anyway; dd_compressor.cc:356-404)
    if (num < 3 || num * W != u || u > (uint32_t)(FNT * SP) || b == 0) return false;
    const uint64_t words = ((num - 2) * (uint64_t)(b + 1) + 63) >> 6;
    if (9 + 2 * W + 8 * words > c) return false;
  }
  // metadata parts, serially, into MD[0, mdt).  When that range lies below
  // the compression header and the parts are in the snapshot (the usual
  // case), every wave decodes them from its registers and its lane 0 writes
  // them (identical bytes from every wave; no barrier).  Otherwise thread 0
  // decodes from LDS between two barriers.
  if (mo >= mdt && in_snap) {
    const uint32_t lane = tid_() & 63;
    const bool l0 = lane == 0;
    bool ok = true;
    uint32_t o = 0, ip = 0;
    for (uint32_t i = 0; i < nmd && ok; i++) {
      const uint32_t un = snap32(sm, 8 + 8 * i), cn = snap32(sm, 12 + 8 * i);
      const uint32_t pb = cn >= 9 ? snap8(sx, ip) : 0u;
      const uint64_t pn = cn >= 9 ? snapn(sx, ip + 1, 8) : 0ull;
      // a raw part or one of <= 2 values is its bytes after the 9-byte
      // header (dd_compressor.cc:327-347): lane-parallel copy
      const bool plain = cn >= 9 && un <= 64 &&
                         ((pb >= 8u * W - 1 && cn - 9 == un) ||
                          (pn >= 1 && pn <= 2 && pn * W == un && cn >= 9 + un));
      if (plain) {
        if (lane < un) L.MD[o + lane] = L.X[cur.base + ip + 9 + lane];
      } else {
        ok = dd_serial_g([&](uint32_t q) -> uint32_t { return snap8(sx, ip + q); }, cn,
                         [&](uint32_t q, uint8_t v) { if (l0) L.MD[o + q] = v; }, un, W);
      }
      o += un;
      ip += cn;
    }
    if (!ok) return false;
  } else {
    __syncthreads();  // every thread has read the header
    if (tid_() == 0) {
      bool ok = true;
      uint32_t o = 0, ip = 0;
      for (uint32_t i = 0; i < nmd; i++) {
        const uint32_t un = lds32(L.MD, mo + 8 + 8 * i), cn = lds32(L.MD, mo + 12 + 8 * i);
        ok = ok && dd_serial(L.X + cur.base + ip, cn, L.MD + o, un, W);
        o += un;
        ip += cn;
      }
      L.flag[0] = ok ? 0u : 1u;
    }
    __syncthreads();
    if (L.flag[0]) return false;
  }
  mo = 0;
  mn = mdt;
  if (raw) {
    cur.base = cur.base + src + 9;
    cur.n = u;
    if (final) final_copy(L, cur, gout);
    return true;
  }
  mark(4);  // diagnostics: DD header + metadata parts
  const bool swz = dd_decode_part<W, SWZ>(L, cur.base + src, b, num, mark);
  cur.base = 0;
  cur.n = u;
  cur.swz = swz ? 1u : 0u;
  if (final) final_copy(L, cur, gout);
  return true;
}

__device__ __forceinline__ bool f_rle(FastLds& L, View& cur, uint32_t& mo, uint32_t& mn, bool final,
                      uint8_t* gout, uint32_t cap, uint32_t cs) {
  uint32_t nmd, src, c, u, mdt;
  if (cs != 1 && cs != 2 && cs != 4 && cs != 8) return false;
  if (!comp_header(L, cur, mo, mn, nmd, src, c, u, mdt)) return false;
  const uint32_t rs = cs + 2, nr = c / rs;
  if (c % rs || nr == 0 || nr > RUNCAP || u > XCAP || (final && u > cap)) return false;
  uint32_t* start = (uint32_t*)L.TAB;
  // run starts (cells)
  uint64_t acc = 0;
  for (uint32_t r0 = 0; r0 < nr; r0 += FNT) {
    const uint32_t r = r0 + tid_();
    uint32_t len = 0;
    if (r < nr) len = ((uint32_t)L.X[src + r * rs + cs] << 8) | L.X[src + r * rs + cs + 1];
    uint64_t t;
    const uint64_t ex = acc + block_exscan_u64<FNT>(len, t, L.red);
    if (r < nr) start[r] = (uint32_t)ex;
    acc += t;
  }
  if (tid_() == 0) start[nr] = (uint32_t)acc;
  if (block_any(acc * cs != u)) return false;
  // metadata parts (thread 0)
  if (tid_() == 0) {
    bool ok = true;
    uint32_t o = 0;
    for (uint32_t i = 0; i < nmd; i++) {
      const uint32_t un = L.pairs[3 * i], cn = L.pairs[3 * i + 1], ip = L.pairs[3 * i + 2];
      ok = ok && rle_serial(L.X + cur.base + ip, cn, L.MD + o, un, cs);
      o += un;
    }
    L.flag[0] = ok ? 0u : 1u;
  }
  __syncthreads();
  if (L.flag[0]) return false;
  mo = 0;
  mn = mdt;
  const uint8_t* X = L.X;
  const uint32_t cpu = 16 / cs;  // cells per 16-B unit
  drive<16>(L, u, final, gout, [&](uint32_t uu, uint32_t (&w)[4]) {
    const uint32_t c0 = uu * cpu;
    uint32_t lo = 0, hi = nr;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (start[mid] <= c0) lo = mid; else hi = mid;
    }
    uint32_t r = lo, rend = start[r + 1];
    uint64_t v = ldsn(X, src + r * rs, cs);
    uint32_t buf[4] = {0, 0, 0, 0};
    for (uint32_t k = 0; k < cpu; k++) {
      const uint32_t cc = c0 + k;
      if (cc >= acc) break;
      while (cc >= rend) { r++; rend = start[r + 1]; v = ldsn(X, src + r * rs, cs); }
      const uint32_t bo = k * cs;
      if (cs == 8) { buf[bo >> 2] = (uint32_t)v; buf[(bo >> 2) + 1] = (uint32_t)(v >> 32); }
      else buf[bo >> 2] |= (uint32_t)v << (8 * (bo & 3));
    }
#pragma unroll
    for (int d = 0; d < 4; d++) w[d] = buf[d];
  });
  cur.base = 0;
  cur.n = u;
  return true;
}

// ---------------------------------------------------------------------------
// workgroup scans for the slice stages below: inclusive over the block in
// thread order (DPP within the wave, wave totals through red + one barrier;
// callers barrier before `red` is written again); returns the exclusive
// prefix of this thread.  Op: 0 = add, 1 = xor.
// ---------------------------------------------------------------------------
template <int OP, class U>
__device__ __forceinline__ U block_exscan_op(U v, U* red) {
  const uint32_t lane = tid_() & 63, wid = tid_() >> 6;
  U inc = v;
  wave_scan_steps(inc, [&](U y, int) { inc = OP ? (U)(inc ^ y) : (U)(inc + y); });
  if (lane == 63) red[wid] = inc;
  __syncthreads();
  U pre = 0;
#pragma unroll
  for (int i = 0; i < FNT / 64; i++)
    if ((uint32_t)i < wid) pre = OP ? (U)(pre ^ red[i]) : (U)(pre + red[i]);
  return OP ? (U)(pre ^ inc ^ v) : (U)(pre + inc - v);
}

// ---------------------------------------------------------------------------
// XOR^-1 (XORFilter::unxor_part, xor_filter.cc:260-286) for 4- / 8-byte
// elements: a prefix XOR over the part.  One part covering the view, whole
// elements only (a tail the reference leaves unwritten declines).  Each
// thread XOR-scans its 128-B slice in registers; the block scan carries.
// ---------------------------------------------------------------------------
template <int W, int SZ>
__device__ __forceinline__ bool f_xor(FastLds& L, View& cur, uint32_t& mo, uint32_t& mn, bool final,
                                      uint8_t* gout, uint32_t cap) {
  typedef typename std::conditional<(W == 8), uint64_t, uint32_t>::type U;
  if (mn < 8) return false;
  const uint32_t np = lds32(L.MD, mo), ps = lds32(L.MD, mo + 4);
  if (np != 1 || ps != cur.n || ps % W != 0 || ps > (uint32_t)(FNT * SP)) return false;
  if (final && ps > cap) return false;
  mo += 8;
  mn -= 8;
  const uint32_t n = ps, base = cur.base, t = tid_();
  const uint32_t s0 = t * SP;
  constexpr int EP = SP / W;
  uint32_t r[SPD];
  slice_load(L, cur, r);
  (void)base;
  (void)s0;
  U acc = 0;
#pragma unroll
  for (int e = 0; e < EP; e++) {
    acc ^= (U)rget<W>(r, e);
    rset<W>(r, e, acc);
  }
  const U ex = block_exscan_op<1, U>(acc, (U*)L.red);
#pragma unroll
  for (int e = 0; e < EP; e++) rset<W>(r, e, (U)rget<W>(r, e) ^ ex);
  __syncthreads();  // every slice read before the stores
  const bool so = final || SZ == 1 || (SZ == 2 && n % 16 == 0);
  slice_store(L, r, n, so);
  __syncthreads();
  cur.base = 0;
  cur.n = n;
  cur.swz = so ? 1u : 0u;
  if (final) final_copy(L, cur, gout);
  return true;
}

// Delta::decompress of a small metadata part (thread 0; delta_compressor.cc:
// 251-273, bytes past the values zeroed as tdbg_general.h); false on anomaly
__device__ bool delta_serial(const uint8_t* src, uint32_t cn, uint8_t* dst, uint32_t un, uint32_t W) {
  if (cn < 8) return false;
  uint64_t num = 0;
  for (int i = 0; i < 8; i++) num |= (uint64_t)src[i] << (8 * i);
  const uint64_t nv = num ? num : 1;
  if (nv > (cn - 8) / W || nv > un / W) return false;
  const uint64_t m = wmask(W);
  uint64_t x = 0;
  for (uint64_t i = 0; i < nv; i++) {
    uint64_t d = 0;
    for (uint32_t b = 0; b < W; b++) d |= (uint64_t)src[8 + i * W + b] << (8 * b);
    x = (x + d) & m;
    for (uint32_t b = 0; b < W; b++) dst[i * W + b] = (uint8_t)(x >> (8 * b));
  }
  for (uint64_t i = nv * W; i < un; i++) dst[i] = 0;
  return true;
}

// ---------------------------------------------------------------------------
// CompressionFilter + Delta::decompress<T> (compression_filter.cc:303-347,
// delta_compressor.cc:251-273) for 4- / 8-byte values: the data part
// [u64 num][T x0][T d1 ..] is an inclusive prefix sum (mod 2^8W).  Fused for
// one data part whose values fill it exactly (un == num W, num >= 1); each
// thread sums its slice of values in registers, the block scan carries.
// ---------------------------------------------------------------------------
template <int W, bool SWZ>
__device__ __forceinline__ bool f_delta(FastLds& L, View& cur, uint32_t& mo, uint32_t& mn, bool final,
                                        uint8_t* gout, uint32_t cap) {
  typedef typename std::conditional<(W == 8), uint64_t, uint32_t>::type U;
  uint32_t nmd, src, c, u, mdt;
  if (!comp_header(L, cur, mo, mn, nmd, src, c, u, mdt)) return false;
  if (c < 8 || (final && u > cap) || u > (uint32_t)(FNT * SP)) return false;
  const uint64_t num = ldsn(L.X, src, 8);
  if (num == 0 || num * W != u || 8 + num * W > c) return false;
  // aligned window reads of every thread stay inside L.X
  if (src + 8 + (uint32_t)(FNT * SP) + 8 > XCAP) return false;
  if (tid_() == 0) {
    bool ok = true;
    uint32_t o = 0;
    for (uint32_t i = 0; i < nmd; i++) {
      const uint32_t un = L.pairs[3 * i], cn = L.pairs[3 * i + 1], ip = L.pairs[3 * i + 2];
      ok = ok && delta_serial(L.X + cur.base + ip, cn, L.MD + o, un, W);
      o += un;
    }
    L.flag[0] = ok ? 0u : 1u;
  }
  __syncthreads();
  if (L.flag[0]) return false;
  mo = 0;
  mn = mdt;
  // thread t: values [t EP, t EP + EP) = bytes [t SP, t SP + SP) of the part
  constexpr int EP = SP / W;
  const uint32_t t = tid_();
  const uint32_t sb = src + 8 + t * SP;
  const uint32_t a = sb & ~3u, sh = sb & 3u;
  uint32_t A[SPD + 1];
#pragma unroll
  for (int k = 0; k <= SPD; k++) A[k] = *(const uint32_t*)(L.X + a + 4 * k);
  uint32_t r[SPD];
#pragma unroll
  for (int k = 0; k < SPD; k++) r[k] = __builtin_amdgcn_alignbyte(A[k + 1], A[k], sh);
  U acc = 0;
#pragma unroll
  for (int e = 0; e < EP; e++) {
    acc += (U)rget<W>(r, e);
    rset<W>(r, e, acc);
  }
  const U ex = block_exscan_op<0, U>(acc, (U*)L.red);
#pragma unroll
  for (int e = 0; e < EP; e++) rset<W>(r, e, (U)rget<W>(r, e) + ex);
  __syncthreads();  // every part read before the values overwrite it
  const uint32_t n = u;
  const bool swz = SWZ && W == 4 && ((n >> 2) & 3) == 0;
  {
    const uint32_t s0 = t * SP, rot = swz ? (t & 7) : 0u;
#pragma unroll
    for (int q = 0; q < SP / 16; q++) {
      const uint32_t o = s0 + 16 * q;
      if (o < n) *(uint4*)(L.X + s0 + 16 * (q ^ rot)) = make_uint4(r[4 * q], r[4 * q + 1], r[4 * q + 2], r[4 * q + 3]);
    }
  }
  __syncthreads();
  cur.base = 0;
  cur.n = n;
  cur.swz = swz ? 1u : 0u;
  if (final) final_copy(L, cur, gout);
  return true;
}

// ---------------------------------------------------------------------------
// FLOAT_SCALE^-1 (FloatScalingFilter::run_reverse<T, W>,
// float_scaling_filter.cc:164-197): element-wise T(scale * double(W int) +
// offset), product and sum rounded separately as tdbg_general.h.  One part;
// output units of 16 B gathered in registers (in place) or streamed.
// ---------------------------------------------------------------------------
template <int BW, int TS>
__device__ __forceinline__ uint32_t fscale_one(int64_t q, double sc, double of, uint32_t& hi) {
  if (TS == 4) {
    const float e = __ll2float_rn(q);
    double prod = sc * (double)e;
    asm volatile("" : "+v"(prod));  // keeps the product rounded: no v_fma_f64
    hi = 0;
    return __float_as_uint(__double2float_rn(prod + of));
  } else {
    double prod = sc * __ll2double_rn(q);
    asm volatile("" : "+v"(prod));
    const uint64_t y = (uint64_t)__double_as_longlong(prod + of);
    hi = (uint32_t)(y >> 32);
    return (uint32_t)y;
  }
}

template <int BW, int TS>
__device__ __forceinline__ bool f_fscale(FastLds& L, View& cur, uint32_t& mo, uint32_t& mn, bool final,
                                         uint8_t* gout, uint32_t cap, double sc, double of) {
  if (mn < 8) return false;
  const uint32_t np = lds32(L.MD, mo), ps = lds32(L.MD, mo + 4);
  if (np != 1 || ps > cur.n) return false;
  const uint32_t ne = ps / BW, on = ne * TS;
  if (final ? on > cap : on > XCAP) return false;
  mo += 8;
  mn -= 8;
  const uint8_t* X = L.X;
  const uint32_t base = cur.base;
  constexpr int EPU = 16 / TS;  // values per 16-B output unit
  auto elem = [&](uint32_t j) -> int64_t {
    return sext64(ldsn(X, base + j * BW, BW), BW);
  };
  auto unit = [&](uint32_t u, uint32_t (&w)[4]) {
#pragma unroll
    for (int k = 0; k < EPU; k++) {
      uint32_t hi;
      const uint32_t lo = fscale_one<BW, TS>(elem(EPU * u + k), sc, of, hi);
      if (TS == 4) w[k] = lo;
      else { w[2 * k] = lo; w[2 * k + 1] = hi; }
    }
  };
  auto part = [&](uint32_t u, uint32_t (&w)[4]) {
#pragma unroll
    for (int k = 0; k < 4; k++) w[k] = 0;
#pragma unroll
    for (int k = 0; k < EPU; k++) {
      const uint32_t j = EPU * u + k;
      if (j < ne) {
        uint32_t hi;
        const uint32_t lo = fscale_one<BW, TS>(elem(j), sc, of, hi);
        if (TS == 4) w[k] = lo;
        else { w[2 * k] = lo; w[2 * k + 1] = hi; }
      }
    }
  };
  drive2<16>(L, on, on / 16, final, gout, unit, part);
  cur.base = 0;
  cur.n = on;
  cur.swz = 0;
  return true;
}

// ---------------------------------------------------------------------------
// compile-time pipeline specs
// ---------------------------------------------------------------------------
// Stage code: kind | W << 4 | signed << 8 (0 = no stage).  A spec lists the
// stages in pipeline order (filter 0 first); the fused kernel for a spec
// inlines exactly those stages, so register allocation and LDS address-space
// inference see one small straight-line program.
#define SC(kind, w, sg) ((kind) | ((w) << 4) | ((sg) << 8))

template <int CODE, int POS, int NEXT, class M>
__device__ __forceinline__ bool run_stage(FastLds& L, View& cur, uint32_t& mo, uint32_t& mn,
                                          bool final, uint8_t* gout, uint32_t cap,
                                          const tdbg_plan& P, M&& mark) {
  const tdbg_stage& s = P.s[POS];
  constexpr int K = CODE & 15, W = (CODE >> 4) & 15, SG = (CODE >> 8) & 1;
  // the next stage reads a swizzled view: slice stages (PD, XOR), or a
  // 4-byte byteshuffle (whole plane units)
  constexpr bool NEXT_SLICE = (NEXT & 15) == TDBG_K_PD || (NEXT & 15) == TDBG_K_XOR;
  constexpr bool NEXT_B4 = NEXT == SC(TDBG_K_BYTESHUFFLE, 4, 0);
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (K == TDBG_K_PASS) {
    if (final) {
      if (cur.n > cap) return false;
      final_copy(L, cur, gout);
    }
    return true;
  } else if constexpr (K == TDBG_K_BYTESHUFFLE) {
    return f_byteshuffle<W>(L, cur, mo, mn, final, gout, cap);
  } else if constexpr (K == TDBG_K_BITSHUFFLE) {
    return f_bitshuffle<W>(L, cur, mo, mn, final, gout, cap);
  } else if constexpr (K == TDBG_K_BWR) {
    return f_bwr<W, SG != 0, NEXT_SLICE ? 1 : NEXT_B4 ? 2 : 0>(L, cur, mo, mn, final, gout, cap, s.dts, POS, mark);
  } else if constexpr (K == TDBG_K_PD) {
    return f_pd<W, NEXT_SLICE ? 1 : NEXT_B4 ? 2 : 0>(L, cur, mo, mn, final, gout, cap, s.dts);
  } else if constexpr (K == TDBG_K_DD) {
    // the next stage (the one run after this) is a 4-byte byteshuffle
    constexpr bool SWZ = NEXT == SC(TDBG_K_BYTESHUFFLE, 4, 0);
    return f_dd<W, SWZ>(L, cur, mo, mn, final, gout, cap, mark);
  } else if constexpr (K == TDBG_K_RLE) {
    return f_rle(L, cur, mo, mn, final, gout, cap, (uint32_t)s.cs);
  } else if constexpr (K == TDBG_K_XOR) {
    return f_xor<W, NEXT_SLICE ? 1 : NEXT_B4 ? 2 : 0>(L, cur, mo, mn, final, gout, cap);
  } else if constexpr (K == TDBG_K_DELTA) {
    constexpr bool SWZ = NEXT == SC(TDBG_K_BYTESHUFFLE, 4, 0);
    return f_delta<W, SWZ>(L, cur, mo, mn, final, gout, cap);
  } else if constexpr (K == TDBG_K_FSCALE) {
    // W = byte width of the stored integers, SG: the float type is 8 bytes
    return f_fscale<W, SG ? 8 : 4>(L, cur, mo, mn, final, gout, cap, P.fs_scale[POS], P.fs_offset[POS]);
  } else {
    return false;
  }
}

// Runs the pipeline on a chunk already staged in LDS (data view `cur`,
// metadata at L.MD[mo, mo+mn)).  `hook` runs right before the final stage,
// which only reads LDS and streams to HBM: the caller issues the next tile's
// loads there.  Returns true when gout holds the unfiltered chunk; false =
// the general interpreter must redo the tile (nothing was written to gout).
// Diagnostics: per-workgroup accumulated shader-clock cycles per phase
// (0 wait for the tile, 1 headers, 2-4 intermediate stages in run order,
// 5 final stage, 6 loop tail), enabled by KParams::prof.
struct PhaseClock {
  uint64_t* out;
  uint64_t t, acc[TDBG_PROF_PHASES];
  __device__ __forceinline__ void init(uint64_t* o) {
    out = o;
    if (!out) return;
    t = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < TDBG_PROF_PHASES; k++) acc[k] = 0;
  }
  __device__ __forceinline__ void mark(int k) {
    if (!out) return;
    const uint64_t n = __builtin_amdgcn_s_memtime();
    acc[k] += n - t;
    t = n;
  }
  __device__ __forceinline__ void flush() {
    if (!out || tid_() != 0) return;
    // slots 8..15 belong to the streaming kernel (tdbg_stream.hip), which runs first
    for (int k = 0; k < TDBG_PROF_PHASES / 2; k++) out[blockIdx.x * TDBG_PROF_PHASES + k] = acc[k];
  }
};

template <int S0, int S1, int S2, int S3, class H, class M>
__device__ __forceinline__ bool f_resident(const tdbg_plan& P, View cur, uint32_t mo, uint32_t mn,
                                           uint8_t* gout, uint32_t orig, FastLds& L,
                                           uint32_t dbg_stop, H&& hook, M&& mark) {
  if (dbg_stop == 1) return true;  // timing ablation: load only
  // reverse order: the last filter runs first (filter_pipeline.cc:470-513)
  if constexpr (S3 != 0) {
    if (dbg_stop > 1 && dbg_stop - 1 < 1) return true;
    if (!run_stage<S3, 3, S2>(L, cur, mo, mn, false, gout, orig, P, mark)) return false;
    if (cur.n > XCAP) return false;
    mark(2);
  }
  if constexpr (S2 != 0) {
    if (dbg_stop > 1 && dbg_stop - 1 < (S3 != 0 ? 2u : 1u)) return true;
    if (!run_stage<S2, 2, (S1 != 0 ? S1 : S0)>(L, cur, mo, mn, false, gout, orig, P, mark)) return false;
    if (cur.n > XCAP) return false;
    mark(S3 != 0 ? 3 : 2);
  }
  if constexpr (S1 != 0) {
    if (dbg_stop > 1 && dbg_stop - 1 < (S3 != 0 ? 3u : S2 != 0 ? 2u : 1u)) return true;
    if (!run_stage<S1, 1, S0>(L, cur, mo, mn, false, gout, orig, P, mark)) return false;
    if (cur.n > XCAP) return false;
    mark(S3 != 0 ? 4 : S2 != 0 ? 3 : 2);
  }
  if (dbg_stop > 1) return true;
  hook();
  const bool ok = run_stage<S0, 0, 0>(L, cur, mo, mn, true, gout, orig, P, mark);
  mark(5);
  return ok;
}

template <int S0, int S1, int S2, int S3>
__device__ __forceinline__ bool f_chunk(const tdbg_plan& P, const uint8_t* gmd, uint32_t ml,
                                        const uint8_t* gdata, uint32_t fl, uint8_t* gout,
                                        uint32_t orig, FastLds& L, uint32_t dbg_stop) {
  if (ml > MDCAP - 16) return false;
  uint32_t dbase, mbase;
  const bool ok_d = load_to_lds(L.X, XCAP, gdata, fl, &dbase);
  const bool ok_m = load_to_lds(L.MD, MDCAP, gmd, ml, &mbase);
  if (!ok_d || !ok_m) return false;
  __syncthreads();
  return f_resident<S0, S1, S2, S3>(P, View{dbase, fl}, mbase, ml, gout, orig, L, dbg_stop,
                                    [] {}, [](int) {});
}

// Whole-tile prefetch: the filtered tile image (tile header, chunk header,
// metadata, data) is one contiguous range whose size the host knows, so its
// loads can be issued a tile ahead into registers and committed to LDS later.
constexpr int PLU = (XCAP / 16 + FNT - 1) / FNT;
constexpr uint32_t PCAP = PLU * FNT * 16;  // bytes of tile image the registers hold
// The prefetch keeps PLU*4 VGPRs live through the final stage; specs whose
// final stage is a scan (PD, DD) or that decode 8-byte DD would spill.
constexpr bool pf_enabled(int s0, int s1, int s2, int s3) {
  return (s0 & 15) != TDBG_K_PD && (s0 & 15) != TDBG_K_DD &&
         s1 != (TDBG_K_DD | 8 << 4) && s2 != (TDBG_K_DD | 8 << 4) && s3 != (TDBG_K_DD | 8 << 4);
}

struct Pref {
  v4u v[PLU];
  uint32_t h;  // lane k of every wave: dword k of the image's first 64 bytes
  uint32_t cnt, base;
  bool ok;
};

__device__ __forceinline__ void pf_issue(Pref& pf, const uint8_t* g, uint64_t n) {
  const uintptr_t a0 = (uintptr_t)g & ~(uintptr_t)15;
  const uintptr_t a1 = ((uintptr_t)g + n + 15) & ~(uintptr_t)15;
  pf.cnt = (uint32_t)((a1 - a0) >> 4);
  pf.base = (uint32_t)((uintptr_t)g - a0);
  pf.ok = n >= 20 && n <= PCAP && (uint64_t)pf.cnt * 16 <= PCAP;
  if (!pf.ok) return;
  const g_cu4* src = (const g_cu4*)a0;
  const uint32_t t = tid_();
  const uint32_t hd = (t & 63) < 4 * pf.cnt ? (t & 63) : 4 * pf.cnt - 1;
  pf.h = ((const g_cu32*)a0)[hd];
#pragma unroll
  for (int k = 0; k < PLU; k++) {
    const uint32_t u = t + k * FNT;
    pf.v[k] = src[u < pf.cnt ? u : pf.cnt - 1];
  }
}

// The registers are consumed: tell the compiler, so they are not kept live
// through code that does not use them (the loads were issued long ago).
__device__ __forceinline__ void pf_kill(Pref& pf) {
#pragma unroll
  for (int k = 0; k < PLU; k++) pf.v[k] = v4u{0u, 0u, 0u, 0u};
}

// Commit: metadata bytes [m, m + ml) of the image go to L.MD and
// data bytes [m + ml, m + ml + fl) to L.X, each shifted by a whole number of
// 16-B units (so md starts at MD[m & 15], data at X[(m + ml) & 15]).
__device__ __forceinline__ void pf_commit_split(const Pref& pf, FastLds& L, uint32_t m, uint32_t ml) {
  const uint32_t t = tid_();
  const uint32_t m0 = m & ~15u, d = m + ml, d0 = d & ~15u;
#pragma unroll
  for (int k = 0; k < PLU; k++) {
    const uint32_t u = t + k * FNT, o = 16 * u;
    if (u < pf.cnt) {
      if (o + 16 > m && o < d) *(v4u*)(L.MD + (o - m0)) = pf.v[k];
      if (o + 16 > d) *(v4u*)(L.X + (o - d0)) = pf.v[k];
    }
  }
}

// A tile's batch entry.  Loaded a tile ahead with vector loads (an opaque
// zero offset keeps them off the scalar unit: scalar loads share lgkmcnt with
// every LDS access, so the first LDS wait after them would stall on HBM).
struct TileDesc {
  uint64_t t, fs, os;
  const uint8_t* in;
  uint8_t* out;
};

__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ TileDesc desc_load(const KParams& kp, const uint32_t* tl, uint64_t j) {
  uint32_t z = 0;
  asm volatile("" : "+v"(z));
  TileDesc d;
  d.t = tl ? tl[j + z] : j + z;
  d.fs = kp.in_size[d.t + z];
  d.os = kp.out_size[d.t + z];
  d.in = kp.in[d.t + z];
  d.out = kp.out[d.t + z];
  return d;
}

__device__ __forceinline__ TileDesc desc_uniform(const TileDesc& d) {
  TileDesc u;
  u.t = uni64(d.t);
  u.fs = uni64(d.fs);
  u.os = uni64(d.os);
  u.in = (const uint8_t*)uni64((uint64_t)d.in);
  u.out = (uint8_t*)uni64((uint64_t)d.out);
  return u;
}

template <int S0, int S1, int S2, int S3>
__global__ void __launch_bounds__(FNT, 4)
unfilter_fused_kernel(const KParams kp) {
  __shared__ FastLds L;
  const uint64_t G = gridDim.x;
  PhaseClock pc;
  pc.init(kp.prof);
  Pref pf;
  pf.ok = false;
  pf.cnt = 0;
  pf.base = 0;
  constexpr bool PF = pf_enabled(S0, S1, S2, S3);
  if (kp.chunks) {
    // chunk-parallel launch (TDBG_CHUNK_PARALLEL): work items are the
    // records of the device chunk directory (tdbg_chunkdir.hip); a chunk the
    // fused path declines sends its whole tile to the general interpreter
    // (first decline wins the status, queues the tile, and takes it out of
    // the fused counters the directory pass added it to)
    // (after the streaming kernels' chunk-mode launch: only the chunks they
    // queued, kp.tile_list[0 .. *kp.ntiles_dev))
    uint32_t nck = __builtin_amdgcn_readfirstlane(*kp.nchunks);
    const uint32_t* cl = nullptr;
    if (kp.ntiles_dev) {
      const uint32_t q = __builtin_amdgcn_readfirstlane(*kp.ntiles_dev);
      nck = q < kp.ntiles ? q : (uint32_t)kp.ntiles;
      cl = kp.tile_list;
    }
    for (uint32_t j = blockIdx.x; j < nck; j += (uint32_t)G) {
      const ChunkRec* rp = kp.chunks + (cl ? __builtin_amdgcn_readfirstlane(cl[j]) : j);
      const uint32_t tile = __builtin_amdgcn_readfirstlane(rp->tile);
      const uint32_t ml = __builtin_amdgcn_readfirstlane(rp->ml);
      const uint32_t fl = __builtin_amdgcn_readfirstlane(rp->fl);
      const uint32_t orig = __builtin_amdgcn_readfirstlane(rp->orig);
      const uint64_t in_off = uni64(rp->in_off), out_off = uni64(rp->out_off);
      const int32_t st0 = (int32_t)__builtin_amdgcn_readfirstlane((uint32_t)kp.status[tile]);
      bool ok = true;
      if (st0 == TDBG_OK) {
        const uint8_t* in = (const uint8_t*)uni64((uint64_t)kp.in[tile]) + in_off;
        uint8_t* out = (uint8_t*)uni64((uint64_t)kp.out[tile]) + out_off;
        ok = f_chunk<S0, S1, S2, S3>(kp.plan, in, ml, in + ml, fl, out, orig, L, kp.dbg_stop);
      }
      __syncthreads();  // LDS reads of this chunk done before the next load
      if (!ok && tid_() == 0) {
        if (atomicCAS(&kp.status[tile], (int32_t)TDBG_OK, (int32_t)TDBG_E_FALLBACK) == TDBG_OK) {
          if (kp.fbq) {
            const uint32_t k = atomicAdd(kp.fbq, 1u);
            if (k < kp.fbq_cap) kp.fbq[1 + k] = tile;
          }
          if (kp.stats) {
            atomicAdd((unsigned long long*)&kp.stats[TDBG_STAT_FUSED_TILES], ~0ull);
            atomicAdd((unsigned long long*)&kp.stats[TDBG_STAT_FUSED_BYTES],
                      (unsigned long long)(0 - kp.out_size[tile]));
          }
        }
      }
    }
    pc.flush();
    return;
  }
  // tiles: all ntiles, or a host-given list (the sync entry's retry)
  uint64_t ntl = kp.ntiles;
  if (kp.ntiles_dev) {  // the streaming kernel's queue (tdbg_stream.hip)
    const uint64_t c = (uint32_t)__builtin_amdgcn_readfirstlane(*kp.ntiles_dev);
    ntl = c < ntl ? c : ntl;
  }
  const uint32_t* tl = kp.tile_list;
  uint64_t ok_tiles = 0, ok_bytes = 0;
  TileDesc dn{};
  if (blockIdx.x < ntl) {
    dn = desc_uniform(desc_load(kp, tl, blockIdx.x));
    if (PF) pf_issue(pf, dn.in, dn.fs);
  }
  for (uint64_t j = blockIdx.x; j < ntl; j += G) {
    const TileDesc d = dn;
    const uint64_t t = d.t;
    const uint8_t* in = d.in;
    const uint64_t fs = d.fs;
    uint8_t* out = d.out;
    const uint64_t os = d.os;
    const uint64_t jn = j + G;
    TileDesc dl{};
    if (jn < ntl) dl = desc_load(kp, tl, jn);  // consumed by the hook
    bool hooked = false;
    auto hook = [&]() {
      hooked = true;
      if (jn < ntl) {
        dn = desc_uniform(dl);
        if (PF) pf_issue(pf, dn.in, dn.fs);
      } else {
        pf.ok = false;
        pf_kill(pf);
      }
    };
    int rc = TDBG_OK;
    // Tile::load_chunk_data (tile.cc:280-313)
    uint64_t expected = os;
    if (kp.flags & TDBG_TILE_OFFSETS) {
      if (os < 8) rc = TDBG_E_TILE_SIZE;
      expected = os - 8;
    }
    bool handled = false;
    if (rc == TDBG_OK && pf.ok) {
      // the whole tile is in registers; every wave reads the tile and chunk
      // headers from its own copy of the first dwords (no LDS, no barrier),
      // then metadata goes to L.MD and data to L.X (stages rewrite X in place)
      const uint32_t b = pf.base;
      const uint64_t nch = (uint64_t)snap32(pf.h, b) | ((uint64_t)snap32(pf.h, b + 4) << 32);
      pc.mark(0);
      if (nch == 1) {
        handled = true;
        const uint32_t orig = snap32(pf.h, b + 8), fl = snap32(pf.h, b + 12), ml = snap32(pf.h, b + 16);
        if (ml > fs - 20 || fl > fs - 20 - ml) rc = TDBG_E_TILE_FORMAT;
        else if (orig != expected) rc = TDBG_E_TILE_SIZE;
        else if (ml + 32 > MDCAP || fl + 32 > XCAP) rc = TDBG_E_FALLBACK;
        else {
          const uint32_t m = b + 20;
          pf_commit_split(pf, L, m, ml);
          pf_kill(pf);
          __syncthreads();
          pc.mark(1);
          const bool done = f_resident<S0, S1, S2, S3>(kp.plan, View{(m + ml) & 15u, fl}, m & 15u,
                                                       ml, out, orig, L, kp.dbg_stop, hook,
                                                       [&](int k) { pc.mark(k); });
          if (!done) rc = TDBG_E_FALLBACK;
        }
      }
    }
    if (!handled && rc == TDBG_OK) {
      pf_kill(pf);
      uint64_t nch = 0;
      if (fs < 8) rc = TDBG_E_TILE_FORMAT;
      else {
        nch = gldn(in, 8);
        uint64_t o = 8, total = 0;
        for (uint64_t i = 0; i < nch; i++) {
          if (o + 12 > fs) { rc = TDBG_E_TILE_FORMAT; break; }
          const uint64_t orig = gldn(in + o, 4), fl = gldn(in + o + 4, 4), ml = gldn(in + o + 8, 4);
          o += 12;
          if (ml > fs - o) { rc = TDBG_E_TILE_FORMAT; break; }
          o += ml;
          if (fl > fs - o) { rc = TDBG_E_TILE_FORMAT; break; }
          o += fl;
          total += orig;
        }
        if (rc == TDBG_OK && total != expected) rc = TDBG_E_TILE_SIZE;
      }
      if (rc == TDBG_OK) {
        uint64_t o = 8, coff = 0;
        for (uint64_t i = 0; i < nch; i++) {
          const uint32_t orig = (uint32_t)gldn(in + o, 4), fl = (uint32_t)gldn(in + o + 4, 4),
                         ml = (uint32_t)gldn(in + o + 8, 4);
          o += 12;
          const bool done = f_chunk<S0, S1, S2, S3>(kp.plan, in + o, ml, in + o + ml, fl,
                                                    out + coff, orig, L, kp.dbg_stop);
          __syncthreads();
          if (!done) {  // the general fixup launch redoes the whole tile
            rc = TDBG_E_FALLBACK;
            break;
          }
          o += ml + fl;
          coff += orig;
        }
      }
    }
    if (!hooked) hook();
    __syncthreads();  // LDS reads of this tile done before the next commit
    if (rc == TDBG_OK) {
      ok_tiles++;
      ok_bytes += os;
    }
    if (tid_() == 0) {
      if (kp.status) kp.status[t] = rc;
      if (rc == TDBG_E_FALLBACK && kp.fbq) {
        // bounded: the count was zeroed for this launch and each tile is
        // queued at most once, so k < fbq_cap always holds
        const uint32_t k = atomicAdd(kp.fbq, 1u);
        if (k < kp.fbq_cap) kp.fbq[1 + k] = (uint32_t)t;
      }
    }
    pc.mark(6);
  }
  if (kp.stats && tid_() == 0 && ok_tiles) {
    atomicAdd((unsigned long long*)&kp.stats[TDBG_STAT_FUSED_TILES], (unsigned long long)ok_tiles);
    atomicAdd((unsigned long long*)&kp.stats[TDBG_STAT_FUSED_BYTES], (unsigned long long)ok_bytes);
  }
  pc.flush();
}

}  // namespace tdbg

// ---------------------------------------------------------------------------
// spec table: the instantiated fused kernels
// ---------------------------------------------------------------------------
#define K_PASS TDBG_K_PASS
#define K_BYTE TDBG_K_BYTESHUFFLE
#define K_BIT TDBG_K_BITSHUFFLE
#define K_BWR TDBG_K_BWR
#define K_PD TDBG_K_PD
#define K_DD TDBG_K_DD
#define K_RLE TDBG_K_RLE
#define K_XOR TDBG_K_XOR
#define K_DELTA TDBG_K_DELTA
#define K_FSCALE TDBG_K_FSCALE
#define SPECS(X)                                                        \
  /* C1: [BYTESHUFFLE] int32 / int64 / int16 */                          \
  X(1, SC(K_BYTE, 4, 0), 0, 0, 0)                                        \
  X(2, SC(K_BYTE, 8, 0), 0, 0, 0)                                        \
  X(3, SC(K_BYTE, 2, 0), 0, 0, 0)                                        \
  /* C2: [BITSHUFFLE, BWR (pass-through on float)] */                    \
  X(4, SC(K_BIT, 4, 0), SC(K_PASS, 0, 0), 0, 0)                          \
  X(5, SC(K_BIT, 8, 0), SC(K_PASS, 0, 0), 0, 0)                          \
  X(6, SC(K_BIT, 4, 0), 0, 0, 0)                                         \
  X(7, SC(K_BIT, 8, 0), 0, 0, 0)                                         \
  /* C2i: [BITSHUFFLE, BWR] int32 / int64 */                             \
  X(8, SC(K_BIT, 4, 0), SC(K_BWR, 4, 1), 0, 0)                           \
  X(9, SC(K_BIT, 4, 0), SC(K_BWR, 4, 0), 0, 0)                           \
  X(10, SC(K_BIT, 8, 0), SC(K_BWR, 8, 1), 0, 0)                          \
  X(11, SC(K_BIT, 8, 0), SC(K_BWR, 8, 0), 0, 0)                          \
  /* C3a / C3b: [DOUBLE_DELTA] / [RLE] on 64-bit coords */              \
  X(12, SC(K_DD, 8, 0), 0, 0, 0)                                         \
  X(13, SC(K_DD, 4, 0), 0, 0, 0)                                         \
  X(14, SC(K_RLE, 0, 0), 0, 0, 0)                                        \
  /* C4: [POSITIVE_DELTA, BWR] offsets */                                \
  X(15, SC(K_PD, 8, 0), SC(K_BWR, 8, 0), 0, 0)                           \
  X(16, SC(K_PD, 8, 0), SC(K_BWR, 8, 1), 0, 0)                           \
  X(17, SC(K_PD, 4, 0), SC(K_BWR, 4, 0), 0, 0)                           \
  X(18, SC(K_PD, 4, 0), SC(K_BWR, 4, 1), 0, 0)                           \
  /* C5: [BYTESHUFFLE, DOUBLE_DELTA, BWR] */                             \
  X(19, SC(K_BYTE, 4, 0), SC(K_DD, 4, 0), SC(K_BWR, 4, 1), 0)            \
  X(20, SC(K_BYTE, 4, 0), SC(K_DD, 4, 0), SC(K_BWR, 4, 0), 0)            \
  X(21, SC(K_BYTE, 8, 0), SC(K_DD, 8, 0), SC(K_BWR, 8, 1), 0)            \
  X(22, SC(K_BYTE, 8, 0), SC(K_DD, 8, 0), SC(K_BWR, 8, 0), 0)            \
  /* DD / RLE followed by BWR, BWR alone */                              \
  X(23, SC(K_DD, 8, 0), SC(K_BWR, 8, 1), 0, 0)                           \
  X(24, SC(K_DD, 8, 0), SC(K_BWR, 8, 0), 0, 0)                           \
  X(25, SC(K_BWR, 4, 1), 0, 0, 0)                                        \
  X(26, SC(K_BWR, 8, 0), 0, 0, 0)                                        \
  X(27, SC(K_BWR, 8, 1), 0, 0, 0)                                        \
  /* XOR / DELTA / FLOAT_SCALE pipelines */                              \
  X(28, SC(K_XOR, 4, 0), SC(K_BWR, 4, 1), 0, 0)                          \
  X(29, SC(K_XOR, 8, 0), SC(K_BWR, 8, 1), 0, 0)                          \
  X(30, SC(K_XOR, 4, 0), 0, 0, 0)                                        \
  X(31, SC(K_XOR, 8, 0), 0, 0, 0)                                        \
  X(32, SC(K_BYTE, 4, 0), SC(K_DELTA, 4, 0), SC(K_BWR, 4, 1), 0)         \
  X(33, SC(K_DELTA, 4, 0), 0, 0, 0)                                      \
  X(34, SC(K_DELTA, 8, 0), 0, 0, 0)                                      \
  X(35, SC(K_FSCALE, 4, 1), SC(K_BWR, 4, 1), 0, 0)                       \
  X(36, SC(K_FSCALE, 4, 0), 0, 0, 0)                                     \
  X(37, SC(K_FSCALE, 8, 1), SC(K_BWR, 8, 1), 0, 0)

// The spec table is compiled as TDBG_NPART translation units (the build
// passes -DTDBG_PART=k): part k instantiates the kernels whose id % NPART == k,
// so the heavy kernel instantiations compile in parallel.
#ifndef TDBG_PART
#define TDBG_PART 0
#define TDBG_NPART 1
#endif

#if TDBG_PART == 0
static uint32_t stage_code(const tdbg_stage& s) {
  switch (s.kind) {
    case TDBG_K_PASS: return SC(TDBG_K_PASS, 0, 0);
    case TDBG_K_RLE: return SC(TDBG_K_RLE, 0, 0);
    case TDBG_K_BWR: return SC(TDBG_K_BWR, s.w, s.sgn ? 1 : 0);
    case TDBG_K_PD: case TDBG_K_DD: case TDBG_K_BYTESHUFFLE: case TDBG_K_BITSHUFFLE:
    case TDBG_K_XOR: case TDBG_K_DELTA:
      return SC(s.kind, s.w, 0);
    case TDBG_K_FSCALE:  // w = stored byte width, sign field = 8-byte float type
      return SC(TDBG_K_FSCALE, s.w, s.dts == 8 ? 1 : 0);
    default: return 0xffffffffu;
  }
}

extern "C" uint32_t tdbg_fast_select(const tdbg_plan* plan) {
  if (plan->nstages == 0 || plan->nstages > 4) return TDBG_FAST_NONE;
  uint32_t c[4] = {0, 0, 0, 0};
  for (uint32_t i = 0; i < plan->nstages; i++) c[i] = stage_code(plan->s[i]);
#define MATCH(id, a, b, cc, d) \
  if (c[0] == (uint32_t)(a) && c[1] == (uint32_t)(b) && c[2] == (uint32_t)(cc) && c[3] == (uint32_t)(d)) return id;
  SPECS(MATCH)
#undef MATCH
  return TDBG_FAST_NONE;
}

extern "C" uint32_t tdbg_fast_grid(uint32_t fast, int cus) {
  (void)fast;
  return (uint32_t)cus * 2;  // two ~80 KB workgroups per CU
}

#endif  // TDBG_PART == 0

namespace {
template <int ID, int A, int B, int C, int D>
hipError_t launch_spec(const tdbg::KParams* kp, uint32_t grid, hipStream_t stream) {
  if constexpr (ID % TDBG_NPART == TDBG_PART) {
    TDBG_LAUNCH((tdbg::unfilter_fused_kernel<A, B, C, D>), dim3(grid), dim3(tdbg::FNT), stream,
                       *kp);
    return hipGetLastError();
  } else {
    return hipErrorInvalidValue;
  }
}
}  // namespace

#define TDBG_CAT2(a, b) a##b
#define TDBG_CAT(a, b) TDBG_CAT2(a, b)
extern "C" hipError_t TDBG_CAT(tdbg_launch_fast_part, TDBG_PART)(const tdbg::KParams* kp, uint32_t grid,
                                                                 hipStream_t stream) {
  switch (kp->plan.fast) {
#define LAUNCH(id, a, b, cc, d) \
    case id:                    \
      return launch_spec<id, a, b, cc, d>(kp, grid, stream);
    SPECS(LAUNCH)
#undef LAUNCH
    default:
      return hipErrorInvalidValue;
  }
}
