// Design study (not part of the product): how much serial per-tile work the
// register-prefetch / LDS-staged tile structure tolerates before HBM
// throughput drops, plus read-only / write-only / copy ceilings.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/micro_phase tools/micro_phase.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr uint32_t TOUT = 65536, TIN = 65536 + 64 * 6 + 16, TSTRIDE = TIN;
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
constexpr int PLU = (TIN / 16 + 511) / 512;

__device__ __forceinline__ void unshuf_store(const uint8_t* X, uint8_t* gout, uint32_t nth, uint32_t tid) {
  for (uint32_t u = tid; u < TOUT / 16; u += nth) {
    uint32_t a = *(const uint32_t*)(X + 4 * u), b = *(const uint32_t*)(X + 16384 + 4 * u),
             c = *(const uint32_t*)(X + 32768 + 4 * u), dd = *(const uint32_t*)(X + 49152 + 4 * u);
    v4u o;
    for (int e = 0; e < 4; e++) {
      uint32_t lo = __builtin_amdgcn_perm(b, a, ((e + 4) << 8) | e);
      uint32_t hi = __builtin_amdgcn_perm(dd, c, ((e + 4) << 8) | e);
      o[e] = (lo & 0xffff) | (hi << 16);
    }
    ((v4u*)gout)[u] = o;
  }
}

// dependent LDS chain of k reads (a stand-in for serial metadata parsing)
__device__ __forceinline__ uint32_t chain(const uint8_t* X, int k, uint32_t seed) {
  uint32_t v = seed & 0xfc;
  for (int i = 0; i < k; i++) v = (*(const volatile uint32_t*)(X + 4096 + (v & 0x3fc))) & 0x3fc;
  return v;
}

// EARLY: prefetch issued right after commit (before the serial part);
// otherwise right before the final stage.  NB: barriers between phases.
template <bool EARLY, int NBAR>
__global__ void __launch_bounds__(512, 4) k_phase(const uint8_t* in, uint8_t* out, int nt, int k, uint32_t* sink) {
  __shared__ __attribute__((aligned(16))) uint8_t X[66048 + 12000];
  v4u v[PLU];
  auto issue = [&](int t) {
    const v4u* s = (const v4u*)(in + (size_t)t * TSTRIDE);
#pragma unroll
    for (int q = 0; q < PLU; q++) {
      uint32_t u = threadIdx.x + q * 512;
      v[q] = s[u < TIN / 16 ? u : TIN / 16 - 1];
    }
  };
  uint32_t acc = 0;
  if (blockIdx.x < nt) issue(blockIdx.x);
  for (int t = blockIdx.x; t < nt; t += gridDim.x) {
#pragma unroll
    for (int q = 0; q < PLU; q++) {
      uint32_t u = threadIdx.x + q * 512;
      if (u < TIN / 16) *(v4u*)(X + 16 * u) = v[q];
    }
    __syncthreads();
    const bool more = t + (int)gridDim.x < nt;
    if (EARLY && more) issue(t + gridDim.x);
    acc += chain(X, k, threadIdx.x);
    for (int b = 0; b < NBAR; b++) {
      __syncthreads();
      acc += X[4096 + (acc & 1023)];
    }
    if (!EARLY && more) issue(t + gridDim.x);
    unshuf_store(X + 64, out + (size_t)t * TOUT, 512, threadIdx.x);
    __syncthreads();
  }
  if (acc == 0xdeadbeef) sink[0] = acc;
}

// read-only ceiling
__global__ void __launch_bounds__(512) k_read(const uint8_t* in, int nt, uint32_t* sink) {
  uint32_t acc = 0;
  for (int t = blockIdx.x; t < nt; t += gridDim.x) {
    const v4u* s = (const v4u*)(in + (size_t)t * TSTRIDE);
    v4u r[8];
#pragma unroll
    for (int q = 0; q < 8; q++) r[q] = s[threadIdx.x + q * 512];
#pragma unroll
    for (int q = 0; q < 8; q++) acc ^= r[q].x ^ r[q].y ^ r[q].z ^ r[q].w;
  }
  if (acc == 0xdeadbeef) sink[0] = acc;
}

// write-only ceiling
__global__ void __launch_bounds__(512) k_write(uint8_t* out, int nt) {
  for (int t = blockIdx.x; t < nt; t += gridDim.x) {
    v4u* d = (v4u*)(out + (size_t)t * TOUT);
#pragma unroll
    for (int q = 0; q < 8; q++) d[threadIdx.x + q * 512] = v4u{(uint32_t)t, (uint32_t)q, 1u, 2u};
  }
}

// copy, optional nontemporal load / store
template <bool NTL, bool NTS>
__global__ void __launch_bounds__(512) k_copy(const uint8_t* in, uint8_t* out, int nt) {
  for (int t = blockIdx.x; t < nt; t += gridDim.x) {
    const v4u* s = (const v4u*)(in + (size_t)t * TSTRIDE);
    v4u* d = (v4u*)(out + (size_t)t * TOUT);
    v4u r[8];
#pragma unroll
    for (int q = 0; q < 8; q++) r[q] = NTL ? __builtin_nontemporal_load(s + threadIdx.x + q * 512) : s[threadIdx.x + q * 512];
#pragma unroll
    for (int q = 0; q < 8; q++) {
      if (NTS) __builtin_nontemporal_store(r[q], d + threadIdx.x + q * 512);
      else d[threadIdx.x + q * 512] = r[q];
    }
  }
}

template <class F>
float timeit(F launch, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 3; i++) launch();
  hipEventRecord(a);
  for (int i = 0; i < reps; i++) launch();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

int main() {
  const int nt = 12500;
  uint8_t *in, *out;
  uint32_t* sink;
  CK(hipMalloc(&in, (size_t)nt * TSTRIDE));
  CK(hipMalloc(&out, (size_t)nt * TOUT));
  CK(hipMalloc(&sink, 64));
  std::vector<uint8_t> h((size_t)nt * TSTRIDE);
  for (size_t i = 0; i < h.size(); i++) h[i] = (uint8_t)(i * 2654435761u >> 13);
  CK(hipMemcpy(in, h.data(), h.size(), hipMemcpyHostToDevice));
  int cus;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const double rw = (double)nt * (TIN + TOUT);
  auto rep = [&](const char* name, float ms, double bytes) {
    printf("%-40s %8.4f ms  %7.1f GB/s\n", name, ms, bytes / ms / 1e6);
    fflush(stdout);
  };
  char nm[96];
  for (int g : {cus, cus * 2, cus * 4, cus * 8}) {
    snprintf(nm, sizeof nm, "read-only grid=%d", g);
    rep(nm, timeit([&] { hipLaunchKernelGGL(k_read, dim3(g), dim3(512), 0, 0, in, nt, sink); }, 20), (double)nt * TIN);
    snprintf(nm, sizeof nm, "write-only grid=%d", g);
    rep(nm, timeit([&] { hipLaunchKernelGGL(k_write, dim3(g), dim3(512), 0, 0, out, nt); }, 20), (double)nt * TOUT);
  }
  for (int g : {cus * 2, cus * 8}) {
    snprintf(nm, sizeof nm, "copy grid=%d", g);
    rep(nm, timeit([&] { hipLaunchKernelGGL((k_copy<false, false>), dim3(g), dim3(512), 0, 0, in, out, nt); }, 20), rw);
    snprintf(nm, sizeof nm, "copy ntload grid=%d", g);
    rep(nm, timeit([&] { hipLaunchKernelGGL((k_copy<true, false>), dim3(g), dim3(512), 0, 0, in, out, nt); }, 20), rw);
    snprintf(nm, sizeof nm, "copy ntstore grid=%d", g);
    rep(nm, timeit([&] { hipLaunchKernelGGL((k_copy<false, true>), dim3(g), dim3(512), 0, 0, in, out, nt); }, 20), rw);
    snprintf(nm, sizeof nm, "copy nt both grid=%d", g);
    rep(nm, timeit([&] { hipLaunchKernelGGL((k_copy<true, true>), dim3(g), dim3(512), 0, 0, in, out, nt); }, 20), rw);
  }
  for (int k : {0, 10, 30, 60}) {
    for (int nb : {0, 4}) {
      snprintf(nm, sizeof nm, "phase late  chain=%d bars=%d", k, nb);
      if (nb == 0) rep(nm, timeit([&] { hipLaunchKernelGGL((k_phase<false, 0>), dim3(cus * 2), dim3(512), 0, 0, in, out, nt, k, sink); }, 20), rw);
      else rep(nm, timeit([&] { hipLaunchKernelGGL((k_phase<false, 4>), dim3(cus * 2), dim3(512), 0, 0, in, out, nt, k, sink); }, 20), rw);
      snprintf(nm, sizeof nm, "phase early chain=%d bars=%d", k, nb);
      if (nb == 0) rep(nm, timeit([&] { hipLaunchKernelGGL((k_phase<true, 0>), dim3(cus * 2), dim3(512), 0, 0, in, out, nt, k, sink); }, 20), rw);
      else rep(nm, timeit([&] { hipLaunchKernelGGL((k_phase<true, 4>), dim3(cus * 2), dim3(512), 0, 0, in, out, nt, k, sink); }, 20), rw);
    }
  }
  CK(hipDeviceSynchronize());
  printf("done\n");
  return 0;
}
