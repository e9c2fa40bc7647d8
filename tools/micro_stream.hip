// Streaming-structure microbenchmarks for the unfilter kernel design
// (design study, not part of the product).  Build:
//   hipcc --offload-arch=gfx950 -O3 -o tools/micro_stream tools/micro_stream.hip
// Each variant moves NT tiles of TIN bytes (input) to TOUT bytes (output,
// 4-byte byteshuffle inverse) and reports GB/s of (in + out) bytes.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr uint32_t TOUT = 65536, TIN = 65536 + 64, TSTRIDE = 65536 + 64;
typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t pick(uint32_t a, uint32_t b, uint32_t c, uint32_t d, int k) {
  // byte k of each of a,b,c,d -> one u32
  uint32_t ab = __builtin_amdgcn_perm(b, a, 0x0c0c0400u + (k | (k + 4) << 8) * 0 + ((k + 4) << 8 | k));
  uint32_t cd = __builtin_amdgcn_perm(d, c, ((k + 4) << 8 | k));
  return ab | cd << 16;
}

// M1: plain global->global copy, tile-structured, each WG grid-strides tiles.
__global__ void __launch_bounds__(512) m1_copy(const uint8_t* in, uint8_t* out, int nt) {
  for (int t = blockIdx.x; t < nt; t += gridDim.x) {
    const v4u* s = (const v4u*)(in + (size_t)t * TSTRIDE + 64);
    v4u* d = (v4u*)(out + (size_t)t * TOUT);
    v4u r[8];
#pragma unroll
    for (int k = 0; k < 8; k++) r[k] = __builtin_nontemporal_load(s + threadIdx.x + k * 512);
#pragma unroll
    for (int k = 0; k < 8; k++) d[threadIdx.x + k * 512] = r[k];
  }
}

// M4: global->global inverse byteshuffle (4 planes of 16 KiB), no LDS.
__global__ void __launch_bounds__(512) m4_unshuffle(const uint8_t* in, uint8_t* out, int nt) {
  for (int t = blockIdx.x; t < nt; t += gridDim.x) {
    const uint32_t* s = (const uint32_t*)(in + (size_t)t * TSTRIDE + 64);
    v4u* d = (v4u*)(out + (size_t)t * TOUT);
    uint32_t p[8][4];
#pragma unroll
    for (int k = 0; k < 8; k++)
#pragma unroll
      for (int q = 0; q < 4; q++) p[k][q] = s[q * 4096 + threadIdx.x + k * 512];
#pragma unroll
    for (int k = 0; k < 8; k++) {
      v4u o;
      for (int e = 0; e < 4; e++) {
        uint32_t lo = __builtin_amdgcn_perm(p[k][1], p[k][0], 0x0c0c0400u | (e << 8 | e) * 0 | ((e + 4) << 8) | e);
        uint32_t hi = __builtin_amdgcn_perm(p[k][3], p[k][2], ((e + 4) << 8) | e);
        o[e] = (lo & 0xffff) | (hi << 16);
      }
      d[threadIdx.x + k * 512] = o;
    }
  }
}

// LDS->global inverse byteshuffle of one 64 KiB tile by NT threads
template <int NTH>
__device__ __forceinline__ void lds_unshuffle_store(const uint8_t* X, uint8_t* gout) {
  for (uint32_t u = threadIdx.x; u < TOUT / 16; u += NTH) {
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

// M2: the current structure: 512 threads, 2 WG/CU, register prefetch of the
// next tile issued before the LDS->HBM stage.
constexpr int PLU = (TIN / 16 + 511) / 512;
__global__ void __launch_bounds__(512, 4) m2_regpf(const uint8_t* in, uint8_t* out, int nt) {
  __shared__ __attribute__((aligned(16))) uint8_t X[66048 + 14000];
  v4u v[PLU];
  auto issue = [&](int t) {
    const v4u* s = (const v4u*)(in + (size_t)t * TSTRIDE);
#pragma unroll
    for (int k = 0; k < PLU; k++) {
      uint32_t u = threadIdx.x + k * 512;
      v[k] = s[u < TIN / 16 ? u : TIN / 16 - 1];
    }
  };
  if (blockIdx.x < nt) issue(blockIdx.x);
  for (int t = blockIdx.x; t < nt; t += gridDim.x) {
#pragma unroll
    for (int k = 0; k < PLU; k++) {
      uint32_t u = threadIdx.x + k * 512;
      if (u < TIN / 16) *(v4u*)(X + 16 * u) = v[k];
    }
    __syncthreads();
    if (t + (int)gridDim.x < nt) issue(t + gridDim.x);
    lds_unshuffle_store<512>(X + 64, out + (size_t)t * TOUT);
    __syncthreads();
  }
}

// M3: one WG per CU, NTH threads, double-buffered global_load_lds ring.
template <int NTH>
__global__ void __launch_bounds__(NTH, 1) m3_glds(const uint8_t* in, uint8_t* out, int nt) {
  __shared__ __attribute__((aligned(16))) uint8_t X[2][66048];
  constexpr int NI = (TIN / 16 + NTH - 1) / NTH;
  auto issue = [&](int t, int b) {
    const uint8_t* s = in + (size_t)t * TSTRIDE;
    const uint32_t w = threadIdx.x / 64, l = threadIdx.x % 64;
#pragma unroll
    for (int k = 0; k < NI; k++) {
      uint32_t u0 = (w + k * (NTH / 64)) * 64;      // wave's first unit
      uint32_t u = u0 + l;
      if (u0 < TIN / 16) {
        uint32_t uc = u < TIN / 16 ? u : TIN / 16 - 1;
        __builtin_amdgcn_global_load_lds((const void*)(s + 16 * uc), (__attribute__((address_space(3))) void*)(X[b] + 16 * u0), 16, 0, 0);
      }
    }
  };
  int b = 0;
  if (blockIdx.x < nt) issue(blockIdx.x, 0);
  for (int t = blockIdx.x; t < nt; t += gridDim.x, b ^= 1) {
    if (t + (int)gridDim.x < nt) {
      issue(t + gridDim.x, b ^ 1);
      __builtin_amdgcn_s_waitcnt(0x3f70 | (NI & 0xf) | ((NI >> 4) << 14));  // vmcnt(NI): the older tile landed
    } else {
      __builtin_amdgcn_s_waitcnt(0x3f70);  // vmcnt(0)
    }
    __builtin_amdgcn_s_barrier();
    lds_unshuffle_store<NTH>(X[b] + 64, out + (size_t)t * TOUT);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
  }
}

template <class K>
float timeit(K k, int grid, int block, const uint8_t* in, uint8_t* out, int nt, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  for (int i = 0; i < 3; i++) hipLaunchKernelGGL(k, dim3(grid), dim3(block), 0, 0, in, out, nt);
  hipEventRecord(a);
  for (int i = 0; i < reps; i++) hipLaunchKernelGGL(k, dim3(grid), dim3(block), 0, 0, in, out, nt);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

int main() {
  const int nt = 12500;
  uint8_t *in, *out;
  CK(hipMalloc(&in, (size_t)nt * TSTRIDE));
  CK(hipMalloc(&out, (size_t)nt * TOUT));
  std::vector<uint8_t> h((size_t)nt * TSTRIDE);
  for (size_t i = 0; i < h.size(); i++) h[i] = (uint8_t)(i * 2654435761u >> 13);
  CK(hipMemcpy(in, h.data(), h.size(), hipMemcpyHostToDevice));
  int cus; hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const double bytes = (double)nt * (TIN + TOUT);
  auto rep = [&](const char* name, float ms) { printf("%-34s %8.4f ms  %7.1f GB/s\n", name, ms, bytes / ms / 1e6); };
  for (int g : {cus * 2, cus * 4, cus * 8, 8192}) {
    char nm[64]; snprintf(nm, 64, "m1_copy grid=%d", g); rep(nm, timeit(m1_copy, g, 512, in, out, nt, 20));
  }
  for (int g : {cus * 2, cus * 4, cus * 8}) {
    char nm[64]; snprintf(nm, 64, "m4_unshuffle grid=%d", g); rep(nm, timeit(m4_unshuffle, g, 512, in, out, nt, 20));
  }
  rep("m2_regpf grid=2cu", timeit(m2_regpf, cus * 2, 512, in, out, nt, 20));
  rep("m3_glds<1024> grid=cu", timeit(m3_glds<1024>, cus, 1024, in, out, nt, 20));
  rep("m3_glds<512> grid=cu", timeit(m3_glds<512>, cus, 512, in, out, nt, 20));
  rep("m3_glds<256> grid=cu", timeit(m3_glds<256>, cus, 256, in, out, nt, 20));
  CK(hipDeviceSynchronize());
  return 0;
}
