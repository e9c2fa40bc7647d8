// Design study (not part of the product): LDS-free streaming inverse
// byteshuffle straight from HBM, for tiles whose earlier stages are views
// (plane bases at arbitrary byte offsets).  Checks correctness on the host.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/micro_view tools/micro_view.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr uint32_t TOUT = 65536, N = TOUT / 4, TSTR = 67936, PB = 2391;  // plane base offset in tile
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const uint32_t g_cu32;
typedef __attribute__((address_space(1))) const v4u g_cu4;
typedef __attribute__((address_space(1))) v4u g_u4;

__device__ __forceinline__ v4u mix(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  const uint32_t x = __builtin_amdgcn_perm(b, a, 0x05010400u), y = __builtin_amdgcn_perm(d, c, 0x05010400u);
  const uint32_t z = __builtin_amdgcn_perm(b, a, 0x07030602u), w = __builtin_amdgcn_perm(d, c, 0x07030602u);
  return v4u{__builtin_amdgcn_perm(y, x, 0x05040100u), __builtin_amdgcn_perm(y, x, 0x07060302u),
             __builtin_amdgcn_perm(w, z, 0x05040100u), __builtin_amdgcn_perm(w, z, 0x07060302u)};
}

// V1: wave units of UNITS x 1 KiB output; per lane per step 4 unaligned dword loads + one 16-B store
template <int STEPS, bool NT>
__global__ void __launch_bounds__(256) v1(const uint8_t* in, uint8_t* out, int nt) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t nunits = nt * (TOUT / (STEPS * 1024));
  const uint32_t gw = blockIdx.x * 4 + (threadIdx.x >> 6), nw = gridDim.x * 4;
  for (uint32_t u = gw; u < nunits; u += nw) {
    const uint32_t t = u / (TOUT / (STEPS * 1024)), s0 = (u % (TOUT / (STEPS * 1024))) * STEPS * 64;
    const uint8_t* p = in + (size_t)t * TSTR + PB;
    uint8_t* o = out + (size_t)t * TOUT;
    uint32_t r[STEPS][4];
#pragma unroll
    for (int s = 0; s < STEPS; s++) {
      const uint32_t i = 4 * (s0 + s * 64 + lane);
#pragma unroll
      for (int j = 0; j < 4; j++) r[s][j] = *(g_cu32*)(p + j * N + i);
    }
#pragma unroll
    for (int s = 0; s < STEPS; s++) {
      const v4u x = mix(r[s][0], r[s][1], r[s][2], r[s][3]);
      g_u4* d = (g_u4*)(o + 16 * (s0 + s * 64 + lane));
      if (NT) __builtin_nontemporal_store(x, d); else *d = x;
    }
  }
}

// V2: per lane 16 elements: 4 unaligned dwordx4 plane loads, 4 stores at 64-B lane stride
template <int STEPS, bool NT>
__global__ void __launch_bounds__(256) v2(const uint8_t* in, uint8_t* out, int nt) {
  const uint32_t lane = threadIdx.x & 63;
  constexpr uint32_t UB = STEPS * 4096;  // output bytes per wave unit
  const uint32_t per = TOUT / UB, nunits = nt * per;
  const uint32_t gw = blockIdx.x * 4 + (threadIdx.x >> 6), nw = gridDim.x * 4;
  for (uint32_t u = gw; u < nunits; u += nw) {
    const uint32_t t = u / per, e0 = (u % per) * (UB / 4);
    const uint8_t* p = in + (size_t)t * TSTR + PB;
    uint8_t* o = out + (size_t)t * TOUT;
    v4u r[STEPS][4];
#pragma unroll
    for (int s = 0; s < STEPS; s++) {
      const uint32_t i = e0 + 16 * (s * 64 + lane);
#pragma unroll
      for (int j = 0; j < 4; j++) r[s][j] = *(g_cu4*)(p + j * N + i);
    }
#pragma unroll
    for (int s = 0; s < STEPS; s++)
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const v4u x = mix(r[s][0][q], r[s][1][q], r[s][2][q], r[s][3][q]);
        g_u4* d = (g_u4*)(o + 4 * (e0 + 16 * (s * 64 + lane)) + 16 * q);
        if (NT) __builtin_nontemporal_store(x, d); else *d = x;
      }
  }
}

template <class F>
float timeit(F launch, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int i = 0; i < 3; i++) launch();
  (void)hipEventRecord(a);
  for (int i = 0; i < reps; i++) launch();
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

int main() {
  const int nt = 12500;
  uint8_t *in, *out;
  CK(hipMalloc(&in, (size_t)nt * TSTR));
  CK(hipMalloc(&out, (size_t)nt * TOUT));
  std::vector<uint8_t> h((size_t)nt * TSTR), ho((size_t)nt * TOUT);
  for (size_t i = 0; i < h.size(); i++) h[i] = (uint8_t)((i * 2654435761u) >> 13);
  CK(hipMemcpy(in, h.data(), h.size(), hipMemcpyHostToDevice));
  int cus;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const double bytes = (double)nt * (TSTR + TOUT);
  auto check = [&](const char* name) {
    (void)hipMemset(out, 0, (size_t)nt * TOUT);
    return name;
  };
  auto verify = [&]() {
    (void)hipMemcpy(ho.data(), out, ho.size(), hipMemcpyDeviceToHost);
    for (int t = 0; t < nt; t += 97)
      for (uint32_t i = 0; i < N; i++)
        for (int j = 0; j < 4; j++)
          if (ho[(size_t)t * TOUT + 4 * i + j] != h[(size_t)t * TSTR + PB + j * N + i]) return false;
    return true;
  };
  auto rep = [&](const char* name, float ms, bool ok) {
    printf("%-34s %8.4f ms  %7.1f GB/s  %s\n", name, ms, bytes / ms / 1e6, ok ? "ok" : "MISMATCH");
    fflush(stdout);
  };
  char nm[80];
  for (int wpc : {8, 16, 32}) {
    const int g = cus * wpc / 4;
#define RUN(K, label)                                                                              \
  check(label);                                                                                    \
  {                                                                                                \
    float ms = timeit([&] { hipLaunchKernelGGL(K, dim3(g), dim3(256), 0, 0, in, out, nt); }, 20); \
    snprintf(nm, sizeof nm, "%s waves/cu=%d", label, wpc);                                         \
    rep(nm, ms, verify());                                                                         \
  }
    RUN((v1<4, false>), "v1 steps4");
    RUN((v1<4, true>), "v1 steps4 nt");
    RUN((v1<8, true>), "v1 steps8 nt");
    RUN((v1<16, true>), "v1 steps16 nt");
    RUN((v2<1, true>), "v2 steps1 nt");
    RUN((v2<2, true>), "v2 steps2 nt");
    RUN((v2<2, false>), "v2 steps2");
  }
  printf("done\n");
  return 0;
}
