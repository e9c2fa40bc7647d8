// Memory-pattern study for a window-aligned raw-DoubleDelta kernel (design
// study, not product):
//   hipcc --offload-arch=gfx950 -O3 -o tools/micro_raw tools/micro_raw.hip
// C5 'rand' shape: tiles of 68,003 filtered bytes at odd byte offsets, 64 KiB
// output each.  A work unit is a quarter tile (16 steps of 64 output units);
// a wave takes units wave_id, + nwaves, ...  Step s of plane k loads one
// dword per lane at img + 2400 + 16384 k + 256 s + 4 l (unaligned: every
// lane on one BWR window), the byteshuffle transpose makes one 16-B output
// unit per lane, and the step's 1 KB store starts SHIFT units before the
// step's first unit (SHIFT = 6: the window-aligned ownership of the real
// kernel; 0: line-aligned).  D = steps of loads in flight per wave.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                \
  do {                                                                       \
    hipError_t e = (x);                                                      \
    if (e != hipSuccess) {                                                   \
      printf("err %s line %d\n", hipGetErrorString(e), __LINE__);            \
      exit(1);                                                               \
    }                                                                        \
  } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef uint32_t u32a1 __attribute__((aligned(1)));

__device__ __forceinline__ v4u tr4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  const uint32_t t0 = __builtin_amdgcn_perm(b, a, 0x05010400u), t1 = __builtin_amdgcn_perm(b, a, 0x07030602u);
  const uint32_t t2 = __builtin_amdgcn_perm(d, c, 0x05010400u), t3 = __builtin_amdgcn_perm(d, c, 0x07030602u);
  return v4u{__builtin_amdgcn_perm(t2, t0, 0x05040100u), __builtin_amdgcn_perm(t2, t0, 0x07060302u),
             __builtin_amdgcn_perm(t3, t1, 0x05040100u), __builtin_amdgcn_perm(t3, t1, 0x07060302u)};
}

template <int D, int SHIFT, bool NT>
__global__ void __launch_bounds__(256) k_steps(const uint8_t* in, uint64_t stride, uint8_t* out, int nt) {
  const uint32_t l = threadIdx.x & 63;
  const int nw = gridDim.x * 4;
  const int nu = nt * 4;
  for (int u = blockIdx.x * 4 + (threadIdx.x >> 6); u < nu; u += nw) {
    const uint8_t* img = in + (uint64_t)(u >> 2) * stride + 2400 + 4096 * (u & 3);
    uint8_t* o = out + (uint64_t)(u >> 2) * 65536 + 16384 * (u & 3);
    uint32_t v[D][4];
#pragma unroll
    for (int p = 0; p < D; p++)
#pragma unroll
      for (int k = 0; k < 4; k++) v[p][k] = *(const u32a1*)(img + 16384 * k + 256 * p + 4 * l);
#pragma unroll
    for (int s = 0; s < 16; s++) {
      uint32_t x[4];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint32_t nb = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v[s % D][k], 0x130, 0xf, 0xf, false);
        x[k] = __builtin_amdgcn_perm(nb, v[s % D][k], 0x05040302u);
      }
      if (s + D < 16) {
#pragma unroll
        for (int k = 0; k < 4; k++) v[s % D][k] = *(const u32a1*)(img + 16384 * k + 256 * (s + D) + 4 * l);
      }
      const v4u y = tr4(x[0], x[1], x[2], x[3]);
      const int j = 64 * s - SHIFT + (int)l;
      if (j >= 0) {
        v4u* dst = (v4u*)(o + 16 * j);
        if (NT) __builtin_nontemporal_store(y, dst);
        else *dst = y;
      }
    }
  }
}

// Register-staged variant (qwave-like): a unit = UO output bytes of one tile
// (UO/16 output units); per plane the wave loads UO/4 bytes with unaligned
// 16-B loads (lane m: plane dwords 4m..4m+3 of each 1 KB piece), all issued
// before the previous unit's stores (two register sets).  ST = 0: lane m
// stores its 4 units (64 contiguous bytes) directly (64-B lane stride);
// ST = 1: through a wave-private LDS area so every store instruction writes
// 1 KB of consecutive units.
typedef v4u v4a1 __attribute__((aligned(1)));
template <int UO, int ST, bool NT, bool LNT = false>
__global__ void __launch_bounds__(256) k_regs(const uint8_t* in, uint64_t stride, uint8_t* out, int nt) {
  constexpr int R = UO / 4 / 1024;  // 1 KB load pieces per plane
  constexpr int UPT = 65536 / UO;   // units per tile
  __shared__ v4u S[4][256];
  const uint32_t l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nw = gridDim.x * 4;
  const int nu = nt * UPT;
  v4u r[2][4][R];
  auto ld = [&](int u, int b) {
    const uint8_t* img = in + (uint64_t)(u / UPT) * stride + 2400 + (UO / 4) * (u % UPT);
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
      for (int q = 0; q < R; q++) {
        const v4a1* src = (const v4a1*)(img + 16384 * k + 1024 * q + 16 * l);
        r[b][k][q] = LNT ? __builtin_nontemporal_load(src) : *src;
      }
  };
  auto body = [&](int u, int b) {
    uint8_t* o = out + (uint64_t)(u / UPT) * 65536 + UO * (u % UPT);
#pragma unroll
    for (int q = 0; q < R; q++) {
      v4u y[4];
#pragma unroll
      for (int i = 0; i < 4; i++) y[i] = tr4(r[b][0][q][i], r[b][1][q][i], r[b][2][q][i], r[b][3][q][i]);
      if (ST == 0) {
#pragma unroll
        for (int i = 0; i < 4; i++) {
          v4u* dst = (v4u*)(o + 4096 * q + 64 * l + 16 * i);
          if (NT) __builtin_nontemporal_store(y[i], dst);
          else *dst = y[i];
        }
      } else {
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int i = 0; i < 4; i++) S[w][(4 * l + i) ^ ((l >> 3) & 3)] = y[i];  // (swizzle: fewer conflicts)
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const uint32_t un = 64 * i + l;
          const v4u z = S[w][un ^ ((un >> 5) & 3)];
          v4u* dst = (v4u*)(o + 4096 * q + 16 * un);
          if (NT) __builtin_nontemporal_store(z, dst);
          else *dst = z;
        }
      }
    }
  };
  int u = blockIdx.x * 4 + (int)w;
  if (u < nu) ld(u, 0);
  for (; u < nu; u += 2 * nw) {
    if (u + nw < nu) ld(u + nw, 1);
    body(u, 0);
    if (u + nw >= nu) break;
    if (u + 2 * nw < nu) ld(u + 2 * nw, 0);
    body(u + nw, 1);
  }
}

// ceiling2's qwave r68w64 (aligned nt loads of a quarter image, then 16 x 1 KB stores)
__global__ void __launch_bounds__(256) k_qwave(const uint8_t* in, uint64_t stride, uint8_t* out, int nt) {
  constexpr uint32_t RB = 68000;
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
  const uint64_t istride = 68003;  // odd: unaligned images
  uint8_t *in, *out;
  CK(hipMalloc(&in, 68016ull * maxt + 65536));  // the largest stride any variant uses
  CK(hipMalloc(&out, 65536ull * maxt + 4096));
  CK(hipMemset(in, 1, 68016ull * maxt + 65536));
  CK(hipMemset(out, 0, 65536ull * maxt + 4096));
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
    printf("%-34s %9.1f us  %7.0f GB/s  frac %.3f\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e9,
           bytes / (ms * 1e-3) / 8e12);
    fflush(stdout);
  };
  char nm[96];
  for (uint64_t nt : {12500ull, 100000ull}) {
    const double bytes = (68000.0 + 65536) * nt;
    for (int g : {4, 6, 8}) {
      const int grid = g * cus;
#define RUN(D, SH, NTS)                                                                          \
  snprintf(nm, sizeof nm, "steps D%d sh%d %s t%llu g%d", D, SH, NTS ? "nt" : "pl", (unsigned long long)nt, g); \
  timeit(nm, bytes, [&] { k_steps<D, SH, NTS><<<grid, 256>>>(in + 1, istride, out, (int)nt); });
      RUN(4, 0, true)
#define RUNR(UO, ST, NTS, LN, OFF)                                                                          \
  snprintf(nm, sizeof nm, "regs u%d st%d %s%s off%d t%llu g%d", UO, ST, NTS ? "nt" : "pl", LN ? "+ldnt" : "", OFF, (unsigned long long)nt, g); \
  timeit(nm, bytes, [&] { k_regs<UO, ST, NTS, LN><<<grid, 256>>>(in + OFF, OFF ? istride : 68016, out, (int)nt); });
      RUNR(4096, 1, true, false, 1) RUNR(4096, 1, true, true, 1) RUNR(4096, 1, true, true, 0)
      RUNR(16384, 1, true, true, 1) RUNR(16384, 1, true, true, 0)
      snprintf(nm, sizeof nm, "qwave r68w64 t%llu g%d", (unsigned long long)nt, g);
      timeit(nm, bytes, [&] { k_qwave<<<grid, 256>>>(in + 3, istride, out, (int)nt); });
    }
  }
  return 0;
}
