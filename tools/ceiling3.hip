// HBM ceilings, round 5 (design study, not product):
//   hipcc --offload-arch=gfx950 -O3 -o tools/ceiling3 tools/ceiling3.hip
//   tools/ceiling3 [filter]
// Replaces ceiling2's persistent grid-stride probes (one float4 in flight per
// lane).  Here every kernel is NON-persistent: a workgroup owns one
// contiguous chunk of 256 * U 16-B units, each thread issues its U loads
// before its U stores (U loads in flight per lane), at 100,000 x 64 KiB
// (the metric's C5 output size) unless a line says otherwise.
//   W*: write-only, store cache policy plain / nt / sc1 / sc0 sc1 / nt sc1
//   R*: read-only (xor-reduce; one dword per workgroup written)
//   C*: 1:1 copy
//   X : blockIdx remapped so each XCD (blocks dealt round-robin over 8)
//       owns one contiguous eighth of the buffer
//   T*: C5-rand-shaped tiles: one workgroup per tile, 68,003-B images at
//       odd offsets (aligned cover read), 64 KiB written
// Every line: bytes moved / time (HIP events around 10 launches), frac of
// 8 TB/s.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e = (x);                                                               \
    if (e != hipSuccess) {                                                            \
      printf("err %s line %d\n", hipGetErrorString(e), __LINE__);                     \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

template <int POL>
__device__ __forceinline__ void st16(v4u* p, v4u v) {
  if constexpr (POL == 0) asm volatile("global_store_dwordx4 %0, %1, off" ::"v"(p), "v"(v) : "memory");
  else if constexpr (POL == 1) asm volatile("global_store_dwordx4 %0, %1, off nt" ::"v"(p), "v"(v) : "memory");
  else if constexpr (POL == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
  else if constexpr (POL == 3) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
  else asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" ::"v"(p), "v"(v) : "memory");
}

template <bool NTL>
__device__ __forceinline__ v4u ld16(const v4u* p) {
  if constexpr (NTL) return __builtin_nontemporal_load(p);
  else return *p;
}

__device__ __forceinline__ uint32_t chunk_id(bool xcd) {
  if (!xcd) return blockIdx.x;
  const uint32_t n = gridDim.x;  // a multiple of 8
  return (blockIdx.x & 7) * (n >> 3) + (blockIdx.x >> 3);
}

template <int U, int POL, bool XCD, int NTH>
__global__ void __launch_bounds__(NTH) k_write(v4u* __restrict__ out) {
  const uint64_t base = (uint64_t)chunk_id(XCD) * NTH * U + threadIdx.x;
#pragma unroll
  for (int k = 0; k < U; k++) st16<POL>(out + base + (uint64_t)NTH * k, v4u{(uint32_t)k, 1u, 2u, (uint32_t)base});
}

template <int U, bool NTL, bool XCD, int NTH>
__global__ void __launch_bounds__(NTH) k_read(const v4u* __restrict__ in, uint32_t* sink) {
  const uint64_t base = (uint64_t)chunk_id(XCD) * NTH * U + threadIdx.x;
  v4u r[U];
#pragma unroll
  for (int k = 0; k < U; k++) r[k] = ld16<NTL>(in + base + (uint64_t)NTH * k);
  uint32_t x = 0;
#pragma unroll
  for (int k = 0; k < U; k++) x ^= r[k].x ^ r[k].y ^ r[k].z ^ r[k].w;
  if (x == 0x12345678u) sink[blockIdx.x & 1023] = x;
}

template <int U, int POL, bool NTL, bool XCD, int NTH>
__global__ void __launch_bounds__(NTH) k_copy(const v4u* __restrict__ in, v4u* __restrict__ out) {
  const uint64_t base = (uint64_t)chunk_id(XCD) * NTH * U + threadIdx.x;
  v4u r[U];
#pragma unroll
  for (int k = 0; k < U; k++) r[k] = ld16<NTL>(in + base + (uint64_t)NTH * k);
#pragma unroll
  for (int k = 0; k < U; k++) st16<POL>(out + base + (uint64_t)NTH * k, r[k]);
}

// one workgroup per C5-rand-shaped tile: the aligned cover of a 68,003-B image
// at an odd offset read with NTH threads (units interleaved over the
// workgroup), 64 KiB written (each thread's xor of its loads + k)
template <int POL, bool NTL, bool XCD, int NTH>
__global__ void __launch_bounds__(NTH) k_tile(const uint8_t* __restrict__ in, uint64_t stride,
                                              uint8_t* __restrict__ out) {
  constexpr uint32_t RB = 68003;
  constexpr uint32_t RU = (RB + 31) / 16;
  constexpr uint32_t PER = (RU + NTH - 1) / NTH;
  constexpr uint32_t WPER = 4096 / NTH;
  const uint32_t t = chunk_id(XCD);
  const v4u* s = (const v4u*)(((uint64_t)in + (uint64_t)t * stride) & ~15ull);
  v4u r[PER];
#pragma unroll
  for (uint32_t k = 0; k < PER; k++) {
    const uint32_t u = threadIdx.x + NTH * k;
    r[k] = u < RU ? ld16<NTL>(s + u) : v4u{0, 0, 0, 0};
  }
  v4u acc = {0, 0, 0, 0};
#pragma unroll
  for (uint32_t k = 0; k < PER; k++) acc ^= r[k];
  v4u* d = (v4u*)(out + (uint64_t)t * 65536);
#pragma unroll
  for (uint32_t k = 0; k < WPER; k++) st16<POL>(d + threadIdx.x + NTH * k, acc + k);
}

// persistent grid: workgroup b walks tiles b, b + G, ... or (XCD) the
// contiguous eighth of the tiles of its XCD (b & 7), G / 8 workgroups each
template <uint32_t RB, int POL, bool XCD, int NTH>
__global__ void __launch_bounds__(NTH) k_tileP(const uint8_t* __restrict__ in, uint64_t stride,
                                               uint8_t* __restrict__ out, uint32_t nt) {
  constexpr uint32_t RU = (RB + 31) / 16;
  constexpr uint32_t PER = (RU + NTH - 1) / NTH;
  constexpr uint32_t WPER = 4096 / NTH;
  uint32_t t, hi, step;
  if (XCD) {
    const uint32_t x = blockIdx.x & 7;
    t = (uint32_t)((uint64_t)nt * x / 8) + (blockIdx.x >> 3);
    hi = (uint32_t)((uint64_t)nt * (x + 1) / 8);
    step = gridDim.x >> 3;
  } else {
    t = blockIdx.x;
    hi = nt;
    step = gridDim.x;
  }
  for (; t < hi; t += step) {
    const v4u* s = (const v4u*)(((uint64_t)in + (uint64_t)t * stride) & ~15ull);
    v4u r[PER];
#pragma unroll
    for (uint32_t k = 0; k < PER; k++) {
      const uint32_t u = threadIdx.x + NTH * k;
      r[k] = u < RU ? s[u] : v4u{0, 0, 0, 0};
    }
    v4u acc = {0, 0, 0, 0};
#pragma unroll
    for (uint32_t k = 0; k < PER; k++) acc ^= r[k];
    v4u* d = (v4u*)(out + (uint64_t)t * 65536);
#pragma unroll
    for (uint32_t k = 0; k < WPER; k++) st16<POL>(d + threadIdx.x + NTH * k, acc + k);
  }
}

// non-persistent tile of RB image bytes (stride RB + 3)
template <uint32_t RB, int POL, bool XCD, int NTH>
__global__ void __launch_bounds__(NTH) k_tileN(const uint8_t* __restrict__ in, uint64_t stride,
                                               uint8_t* __restrict__ out) {
  constexpr uint32_t RU = (RB + 31) / 16;
  constexpr uint32_t PER = (RU + NTH - 1) / NTH;
  constexpr uint32_t WPER = 4096 / NTH;
  const uint32_t t = chunk_id(XCD);
  const v4u* s = (const v4u*)(((uint64_t)in + (uint64_t)t * stride) & ~15ull);
  v4u r[PER];
#pragma unroll
  for (uint32_t k = 0; k < PER; k++) {
    const uint32_t u = threadIdx.x + NTH * k;
    r[k] = u < RU ? s[u] : v4u{0, 0, 0, 0};
  }
  v4u acc = {0, 0, 0, 0};
#pragma unroll
  for (uint32_t k = 0; k < PER; k++) acc ^= r[k];
  v4u* d = (v4u*)(out + (uint64_t)t * 65536);
#pragma unroll
  for (uint32_t k = 0; k < WPER; k++) st16<POL>(d + threadIdx.x + NTH * k, acc + k);
}

int main(int argc, char** argv) {
  const char* filt = argc > 1 ? argv[1] : "";
  const uint64_t nt = 100000;
  const uint64_t obytes = nt * 65536;          // 6.55 GB
  const uint64_t istride = 68003;
  const uint64_t ibytes = nt * istride + 65536;  // 6.8 GB
  uint8_t *in, *out;
  uint32_t* sink;
  CK(hipMalloc(&in, ibytes));
  CK(hipMalloc(&out, obytes));
  CK(hipMalloc(&sink, 1 << 20));
  CK(hipMemset(in, 1, ibytes));
  CK(hipMemset(out, 0, obytes));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto timeit = [&](const char* name, double bytes, auto&& launch) {
    if (filt[0] && !strstr(name, filt)) return;
    for (int i = 0; i < 3; i++) launch();
    CK(hipDeviceSynchronize());
    const int reps = 10;
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < reps; i++) launch();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    CK(hipGetLastError());
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= reps;
    printf("%-34s %9.1f us  %7.0f GB/s  frac %.3f\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e9,
           bytes / (ms * 1e-3) / 8e12);
    fflush(stdout);
  };
  const uint64_t n4 = obytes / 16;
  v4u* O = (v4u*)out;
  const v4u* I = (const v4u*)in;
  const char* pol[5] = {"plain", "nt", "sc1", "sc0sc1", "ntsc1"};
  char nm[96];
#define W(U, P, X, NTH)                                                                         \
  snprintf(nm, sizeof nm, "W u%d %s%s b%d", U, pol[P], X ? " X" : "", NTH);                     \
  timeit(nm, (double)obytes, [&] { k_write<U, P, X, NTH><<<n4 / (U * NTH), NTH>>>(O); });
#define R(U, NL, X, NTH)                                                                        \
  snprintf(nm, sizeof nm, "R u%d %s%s b%d", U, NL ? "nt" : "plain", X ? " X" : "", NTH);        \
  timeit(nm, (double)obytes, [&] { k_read<U, NL, X, NTH><<<n4 / (U * NTH), NTH>>>(I, sink); });
#define C(U, P, NL, X, NTH)                                                                                 \
  snprintf(nm, sizeof nm, "C u%d st-%s ld-%s%s b%d", U, pol[P], NL ? "nt" : "plain", X ? " X" : "", NTH);   \
  timeit(nm, 2.0 * obytes, [&] { k_copy<U, P, NL, X, NTH><<<n4 / (U * NTH), NTH>>>(I, O); });
#define T(P, NL, X, NTH)                                                                                      \
  snprintf(nm, sizeof nm, "T r68w64 st-%s ld-%s%s b%d", pol[P], NL ? "nt" : "plain", X ? " X" : "", NTH);    \
  timeit(nm, (68003.0 + 65536) * nt, [&] { k_tile<P, NL, X, NTH><<<nt, NTH>>>(in + 3, istride, out); });

  // write-only
  W(4, 0, false, 256) W(4, 1, false, 256) W(4, 2, false, 256) W(4, 3, false, 256) W(4, 4, false, 256)
  W(16, 0, false, 256) W(16, 1, false, 256) W(16, 2, false, 256) W(16, 3, false, 256) W(16, 4, false, 256)
  W(16, 0, true, 256) W(16, 1, true, 256) W(16, 2, true, 256)
  W(4, 0, false, 1024) W(4, 1, false, 1024) W(4, 2, false, 1024)
  // read-only
  R(4, false, false, 256) R(4, true, false, 256) R(8, false, false, 256) R(16, false, false, 256)
  R(16, true, false, 256) R(16, false, true, 256) R(4, false, false, 1024)
  // copy
  C(4, 0, false, false, 256) C(4, 1, false, false, 256) C(4, 2, false, false, 256) C(4, 3, false, false, 256)
  C(8, 0, false, false, 256) C(8, 1, false, false, 256) C(8, 2, false, false, 256)
  C(16, 0, false, false, 256) C(16, 1, false, false, 256) C(16, 2, false, false, 256)
  C(16, 1, true, false, 256) C(16, 2, true, false, 256)
  C(8, 0, false, true, 256) C(8, 1, false, true, 256) C(8, 2, false, true, 256)
  C(4, 0, false, false, 1024) C(4, 1, false, false, 1024) C(4, 2, false, false, 1024)
  // C5-rand-shaped tiles
  T(0, false, false, 256) T(1, false, false, 256) T(2, false, false, 256) T(3, false, false, 256)
  T(1, true, false, 256) T(2, true, false, 256) T(1, false, true, 256) T(2, false, true, 256)
  T(0, false, false, 512) T(1, false, false, 512) T(2, false, false, 512)
  T(0, false, false, 1024) T(1, false, false, 1024) T(2, false, false, 1024)
  // second set: XCD walk for persistent grids, active-shaped tiles
  int cus = 256;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
#define TP(RB, P, X, NTH, G)                                                                               \
  snprintf(nm, sizeof nm, "P r%dw64 st-%s%s b%d g%d", RB / 1000, pol[P], X ? " X" : "", NTH, G);            \
  timeit(nm, (RB + 65536.0) * nt,                                                                          \
         [&] { k_tileP<RB, P, X, NTH><<<G * cus, NTH>>>(in + 3, RB + 3, out, (uint32_t)nt); });
#define TN(RB, P, X, NTH)                                                                                  \
  snprintf(nm, sizeof nm, "N r%dw64 st-%s%s b%d", RB / 1000, pol[P], X ? " X" : "", NTH);                   \
  timeit(nm, (RB + 65536.0) * nt, [&] { k_tileN<RB, P, X, NTH><<<nt, NTH>>>(in + 3, RB + 3, out); });
  TP(68000, 1, false, 256, 4) TP(68000, 1, true, 256, 4) TP(68000, 0, true, 256, 4)
  TP(68000, 1, false, 256, 5) TP(68000, 1, true, 256, 5) TP(68000, 1, true, 256, 8)
  TP(68000, 1, false, 512, 2) TP(68000, 1, true, 512, 2) TP(68000, 0, true, 512, 2) TP(68000, 1, true, 512, 4)
  TP(68000, 1, true, 1024, 1) TP(68000, 0, true, 1024, 1) TP(68000, 1, true, 1024, 2)
  TN(68000, 1, true, 512) TN(68000, 0, true, 512) TN(68000, 1, true, 1024) TN(68000, 0, true, 1024)
  TN(68000, 2, true, 1024)
  TN(43700, 1, false, 256) TN(43700, 1, true, 256) TN(43700, 1, true, 1024) TP(43700, 1, true, 256, 5)
  TN(20000, 1, false, 256) TN(20000, 1, true, 256) TN(20000, 0, true, 256) TN(20000, 1, true, 512)
  TN(20000, 1, true, 1024) TP(20000, 1, false, 256, 4) TP(20000, 1, true, 256, 4) TP(20000, 0, true, 256, 4)
  TP(20000, 1, true, 512, 2)
  W(4, 0, true, 256) W(4, 1, true, 256) R(4, true, true, 256) C(4, 0, false, true, 256) C(4, 1, false, true, 256)
  C(4, 0, true, true, 256) C(2, 0, false, true, 256) C(2, 1, false, true, 256)
  return 0;
}
