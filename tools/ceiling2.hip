// HBM ceilings, round 4 (design study, not product):
//   hipcc --offload-arch=gfx950 -O3 -o tools/ceiling2 tools/ceiling2.hip
// Measures, at 12,500 and 100,000 tiles of 64 KiB (the C5 shard and the
// whole C5 config on one GPU):
//   copyF4  : the guide's float4 grid-stride copy (MI355X_MICROARCH.md: 6.29 TB/s)
//   copyT   : tile-shaped copy, one 256-thread workgroup per 64 KiB tile
//             (persistent grid), 16 dwordx4 loads then 16 stores per thread
//   readF4  : read-only (xor-reduce, one dword written per workgroup)
//   writeF4 : write-only
//   r20w64  : per tile, 20 KB read + 64 KiB written (C5 'active' ratio)
//   r68w64  : per tile, 68 KB read at an odd byte offset + 64 KiB written (C5 'rand')
// Every line: bytes moved / time, frac of 8 TB/s.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e = (x);                                                               \
    if (e != hipSuccess) {                                                            \
      printf("err %s line %d\n", hipGetErrorString(e), __LINE__);                     \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ void __launch_bounds__(256) k_copyf4(const v4u* __restrict__ in, v4u* __restrict__ out, uint64_t n) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    v4u a = in[i], b = in[i + stride], c = in[i + 2 * stride], d = in[i + 3 * stride];
    if (NT) {
      __builtin_nontemporal_store(a, out + i);
      __builtin_nontemporal_store(b, out + i + stride);
      __builtin_nontemporal_store(c, out + i + 2 * stride);
      __builtin_nontemporal_store(d, out + i + 3 * stride);
    } else {
      out[i] = a;
      out[i + stride] = b;
      out[i + 2 * stride] = c;
      out[i + 3 * stride] = d;
    }
  }
  for (; i < n; i += stride) out[i] = in[i];
}

__global__ void __launch_bounds__(256) k_readf4(const v4u* __restrict__ in, uint32_t* out, uint64_t n) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  uint32_t x = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    const v4u v = in[i];
    x ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (x == 0x12345678u) out[blockIdx.x] = x;
}

template <bool NT>
__global__ void __launch_bounds__(256) k_writef4(v4u* __restrict__ out, uint64_t n) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    const v4u v = {(uint32_t)i, 1u, 2u, 3u};
    if (NT) __builtin_nontemporal_store(v, out + i);
    else out[i] = v;
  }
}

// one workgroup per tile: read RB bytes (16-B units from an arbitrary byte
// offset: the unit-aligned cover is read), write 64 KiB
template <uint32_t RB, bool NT>
__global__ void __launch_bounds__(256) k_tile(const uint8_t* in, uint64_t stride, uint8_t* out, int nt) {
  constexpr uint32_t RU = (RB + 31) / 16;  // units read (cover of an unaligned image)
  constexpr uint32_t PER = (RU + 255) / 256;
  for (int t = blockIdx.x; t < nt; t += gridDim.x) {
    const v4u* s = (const v4u*)(((uint64_t)in + (uint64_t)t * stride) & ~15ull);
    v4u acc = {0, 0, 0, 0};
    v4u r[PER];
#pragma unroll
    for (uint32_t k = 0; k < PER; k++) {
      const uint32_t u = threadIdx.x + 256 * k;
      r[k] = u < RU ? __builtin_nontemporal_load(s + u) : v4u{0, 0, 0, 0};
    }
#pragma unroll
    for (uint32_t k = 0; k < PER; k++) acc ^= r[k];
    v4u* d = (v4u*)(out + (size_t)t * 65536);
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const v4u v = acc + (uint32_t)k;
      if (NT) __builtin_nontemporal_store(v, d + threadIdx.x + 256 * k);
      else d[threadIdx.x + 256 * k] = v;
    }
  }
}

// software-pipelined tile copy: the next tile's loads are issued before the
// current tile's stores (two register sets)
template <uint32_t RB>
__global__ void __launch_bounds__(256) k_tpipe(const uint8_t* in, uint64_t stride, uint8_t* out, int nt) {
  constexpr uint32_t RU = (RB + 31) / 16;
  constexpr uint32_t PER = (RU + 255) / 256;
  v4u r[PER];
  auto ld = [&](int t) {
    const v4u* s = (const v4u*)(((uint64_t)in + (uint64_t)t * stride) & ~15ull);
#pragma unroll
    for (uint32_t k = 0; k < PER; k++) {
      const uint32_t u = threadIdx.x + 256 * k;
      r[k] = u < RU ? __builtin_nontemporal_load(s + u) : v4u{0, 0, 0, 0};
    }
  };
  int t = blockIdx.x;
  if (t < nt) ld(t);
  for (; t < nt; t += gridDim.x) {
    v4u acc = {0, 0, 0, 0};
#pragma unroll
    for (uint32_t k = 0; k < PER; k++) acc ^= r[k];
    if (t + (int)gridDim.x < nt) ld(t + gridDim.x);
    v4u* d = (v4u*)(out + (size_t)t * 65536);
#pragma unroll
    for (int k = 0; k < 16; k++) __builtin_nontemporal_store(acc + (uint32_t)k, d + threadIdx.x + 256 * k);
  }
}

// quarter tiles per wave, no workgroup sync: wave w of the grid's waves
// streams quarter-tiles q = wave id, + nwaves, ...; each quarter reads RB/4
// and writes 16 KiB, loads of the next quarter issued before the stores
template <uint32_t RB>
__global__ void __launch_bounds__(256) k_qwave(const uint8_t* in, uint64_t stride, uint8_t* out, int nt) {
  constexpr uint32_t RU = (RB / 4 + 31) / 16;
  constexpr uint32_t PER = (RU + 63) / 64;
  const uint32_t l = threadIdx.x & 63;
  const int nw = gridDim.x * 4;
  const int nq = nt * 4;
  v4u r[PER];
  auto ld = [&](int q) {
    const v4u* s = (const v4u*)(((uint64_t)in + (uint64_t)(q >> 2) * stride + (RB / 4) * (q & 3)) & ~15ull);
#pragma unroll
    for (uint32_t k = 0; k < PER; k++) {
      const uint32_t u = l + 64 * k;
      r[k] = u < RU ? __builtin_nontemporal_load(s + u) : v4u{0, 0, 0, 0};
    }
  };
  int q = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q < nq) ld(q);
  for (; q < nq; q += nw) {
    v4u acc = {0, 0, 0, 0};
#pragma unroll
    for (uint32_t k = 0; k < PER; k++) acc ^= r[k];
    if (q + nw < nq) ld(q + nw);
    v4u* d = (v4u*)(out + (size_t)q * 16384);
#pragma unroll
    for (int k = 0; k < 16; k++) __builtin_nontemporal_store(acc + (uint32_t)k, d + l + 64 * k);
  }
}

int main() {
  int cus = 256;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const uint64_t maxt = 100000;
  const uint64_t istride = 68000 + 67;  // images at odd byte offsets, up to 68 KB each
  uint8_t *in, *out;
  uint32_t* sink;
  CK(hipMalloc(&in, istride * maxt + 4096));
  CK(hipMalloc(&out, 65536ull * maxt));
  CK(hipMalloc(&sink, 1 << 20));
  CK(hipMemset(in, 1, istride * maxt + 4096));
  CK(hipMemset(out, 0, 65536ull * maxt));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto timeit = [&](const char* name, double bytes, auto&& launch) {
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
    printf("%-30s %9.1f us  %7.0f GB/s  frac %.3f\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e9,
           bytes / (ms * 1e-3) / 8e12);
    fflush(stdout);
  };
  char nm[96];
  for (uint64_t nt : {12500ull, 100000ull}) {
    const uint64_t n4 = nt * 65536 / 16;
    for (int g : {4, 8, 16}) {
      const int grid = g * cus;
      snprintf(nm, sizeof nm, "copyF4   t%llu g%d", (unsigned long long)nt, g);
      timeit(nm, 2.0 * nt * 65536, [&] { k_copyf4<false><<<grid, 256>>>((const v4u*)in, (v4u*)out, n4); });
      snprintf(nm, sizeof nm, "copyF4nt t%llu g%d", (unsigned long long)nt, g);
      timeit(nm, 2.0 * nt * 65536, [&] { k_copyf4<true><<<grid, 256>>>((const v4u*)in, (v4u*)out, n4); });
      snprintf(nm, sizeof nm, "readF4   t%llu g%d", (unsigned long long)nt, g);
      timeit(nm, 1.0 * nt * 65536, [&] { k_readf4<<<grid, 256>>>((const v4u*)in, sink, n4); });
      snprintf(nm, sizeof nm, "writeF4  t%llu g%d", (unsigned long long)nt, g);
      timeit(nm, 1.0 * nt * 65536, [&] { k_writef4<false><<<grid, 256>>>((v4u*)out, n4); });
      snprintf(nm, sizeof nm, "writeF4nt t%llu g%d", (unsigned long long)nt, g);
      timeit(nm, 1.0 * nt * 65536, [&] { k_writef4<true><<<grid, 256>>>((v4u*)out, n4); });
    }
    for (int g : {2, 4, 6, 8}) {
      const int grid = g * cus;
      snprintf(nm, sizeof nm, "copyT    t%llu g%d", (unsigned long long)nt, g);
      timeit(nm, 2.0 * nt * 65536, [&] { k_tile<65536 - 32, false><<<grid, 256>>>(in, 65536, out, (int)nt); });
      snprintf(nm, sizeof nm, "copyTnt  t%llu g%d", (unsigned long long)nt, g);
      timeit(nm, 2.0 * nt * 65536, [&] { k_tile<65536 - 32, true><<<grid, 256>>>(in, 65536, out, (int)nt); });
      snprintf(nm, sizeof nm, "r20w64nt t%llu g%d", (unsigned long long)nt, g);
      timeit(nm, (20000.0 + 65536) * nt, [&] { k_tile<20000, true><<<grid, 256>>>(in + 3, 20000 + 67, out, (int)nt); });
      snprintf(nm, sizeof nm, "r68w64nt t%llu g%d", (unsigned long long)nt, g);
      timeit(nm, (68000.0 + 65536) * nt, [&] { k_tile<68000, true><<<grid, 256>>>(in + 3, istride, out, (int)nt); });
      if (g <= 4) {
        snprintf(nm, sizeof nm, "pipe r20w64 t%llu g%d", (unsigned long long)nt, g);
        timeit(nm, (20000.0 + 65536) * nt, [&] { k_tpipe<20000><<<grid, 256>>>(in + 3, 20000 + 67, out, (int)nt); });
        snprintf(nm, sizeof nm, "pipe r68w64 t%llu g%d", (unsigned long long)nt, g);
        timeit(nm, (68000.0 + 65536) * nt, [&] { k_tpipe<68000><<<grid, 256>>>(in + 3, istride, out, (int)nt); });
      }
      snprintf(nm, sizeof nm, "qwave r20w64 t%llu g%d", (unsigned long long)nt, g);
      timeit(nm, (20000.0 + 65536) * nt, [&] { k_qwave<20000><<<grid, 256>>>(in + 3, 20000 + 67, out, (int)nt); });
      snprintf(nm, sizeof nm, "qwave r68w64 t%llu g%d", (unsigned long long)nt, g);
      timeit(nm, (68000.0 + 65536) * nt, [&] { k_qwave<68000><<<grid, 256>>>(in + 3, istride, out, (int)nt); });
    }
  }
  return 0;
}
