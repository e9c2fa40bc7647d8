// HBM ceilings for the unfilter kernels' access shape (design study, not product).
//   hipcc --offload-arch=gfx950 -O3 -o tools/ceiling tools/ceiling.hip
// Tiles: NT tiles, each writes 64 KiB of output; inputs are tile images of
// IN bytes packed back to back at odd byte offsets (as the C5 tiles are).
// Kernels (256-thread workgroups, persistent grid of G workgroups per CU):
//   W  : write-only (16 dwordx4 stores per thread per tile, 4 KiB per store instruction)
//   WN : same, nontemporal stores
//   D  : LDS-DMA of the IN-byte image (16-B units), then W's stores of data read from LDS
//   DN : same, nontemporal stores
//   C  : plain global->register->global copy of IN-byte images (IN = 65536 only)
// Each prints GB/s of (IN + 65536) bytes per tile.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e = (x);                                                               \
    if (e != hipSuccess) {                                                            \
      printf("err %s line %d\n", hipGetErrorString(e), __LINE__);                     \
      return 1;                                                                       \
    }                                                                                 \
  } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) v4u g_u4;

template <bool NT>
__global__ void __launch_bounds__(256) k_write(uint8_t* out, int nt, uint32_t salt) {
  for (int t = blockIdx.x; t < nt; t += gridDim.x) {
    g_u4* d = (g_u4*)(out + (size_t)t * 65536);
#pragma unroll
    for (int k = 0; k < 16; k++) {
      v4u v = {t ^ salt, (uint32_t)k, threadIdx.x, salt};
      if (NT) __builtin_nontemporal_store(v, d + threadIdx.x + 256 * k);
      else d[threadIdx.x + 256 * k] = v;
    }
  }
}

constexpr uint32_t CAP = 24576;

__device__ __forceinline__ void dma_unit(uint32_t* lds_base_words, uint64_t src, uint32_t dst_lds) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(dst_lds)
      : "memory");
}

// image of `in_bytes` at in + t * stride (stride odd), staged by LDS-DMA one
// tile ahead; the output is 16 dwordx4 per thread built from LDS words
template <bool NT>
__global__ void __launch_bounds__(256) k_dma(const uint8_t* in, uint64_t stride, uint32_t in_bytes, uint8_t* out,
                                             int nt) {
  __shared__ uint32_t C[2][CAP / 4 + 16];
  const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63;
  auto issue = [&](int t, int buf) {
    const uint64_t a0 = (uint64_t)(in + (uint64_t)t * stride) & ~15ull;
    const uint64_t a1 = ((uint64_t)(in + (uint64_t)t * stride) + in_bytes + 15) & ~15ull;
    const uint32_t n16 = (uint32_t)((a1 - a0) >> 4);
    for (uint32_t r = 0; r * 256 < n16; r++) {
      const uint32_t ub = r * 256 + 64 * w;
      if (ub + l < n16) {
        const uint32_t dst =
            (uint32_t)(uintptr_t)((__attribute__((address_space(3))) uint8_t*)C[buf] + 16 * ub);
        dma_unit(nullptr, a0 + 16ull * (ub + l), __builtin_amdgcn_readfirstlane(dst));
      }
    }
  };
  int buf = 0;
  if ((int)blockIdx.x < nt) issue(blockIdx.x, 0);
  for (int t = blockIdx.x; t < nt; t += gridDim.x) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t + (int)gridDim.x < nt) issue(t + gridDim.x, buf ^ 1);
    g_u4* d = (g_u4*)(out + (size_t)t * 65536);
    const uint32_t nw = in_bytes / 4;
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const uint32_t i = (threadIdx.x + 256 * k) % nw;
      const uint32_t x = C[buf][i];
      v4u v = {x, x + 1, x + 2, x + 3};
      if (NT) __builtin_nontemporal_store(v, d + threadIdx.x + 256 * k);
      else d[threadIdx.x + 256 * k] = v;
    }
    buf ^= 1;
  }
}

template <bool NT>
__global__ void __launch_bounds__(256) k_copy(const uint8_t* in, uint8_t* out, int nt) {
  for (int t = blockIdx.x; t < nt; t += gridDim.x) {
    const g_u4* s = (const g_u4*)(in + (size_t)t * 65536);
    g_u4* d = (g_u4*)(out + (size_t)t * 65536);
    v4u r[16];
#pragma unroll
    for (int k = 0; k < 16; k++) r[k] = __builtin_nontemporal_load(s + threadIdx.x + 256 * k);
#pragma unroll
    for (int k = 0; k < 16; k++) {
      if (NT) __builtin_nontemporal_store(r[k], d + threadIdx.x + 256 * k);
      else d[threadIdx.x + 256 * k] = r[k];
    }
  }
}

int main(int argc, char** argv) {
  const int nt = 12500;
  int cus = 256;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  uint8_t *in, *out;
  const uint64_t stride = 65536 + 67;  // odd: images at arbitrary byte offsets
  CK(hipMalloc(&in, stride * nt + 4096));
  CK(hipMalloc(&out, 65536ull * nt));
  CK(hipMemset(in, 1, stride * nt + 4096));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto timeit = [&](const char* name, double bytes_per_tile, auto&& launch) -> int {
    for (int i = 0; i < 3; i++) launch();
    CK(hipDeviceSynchronize());
    const int reps = 20;
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < reps; i++) launch();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= reps;
    printf("%-28s %8.1f us  %7.0f GB/s  frac %.3f\n", name, ms * 1e3, bytes_per_tile * nt / (ms * 1e-3) / 1e9,
           bytes_per_tile * nt / (ms * 1e-3) / 8e12);
    return 0;
  };
  char nm[64];
  for (int g : {2, 4, 8}) {
    const int grid = g * cus;
    snprintf(nm, sizeof nm, "W  g%d", g);
    timeit(nm, 65536, [&] { k_write<false><<<grid, 256>>>(out, nt, 7); });
    snprintf(nm, sizeof nm, "WN g%d", g);
    timeit(nm, 65536, [&] { k_write<true><<<grid, 256>>>(out, nt, 7); });
    snprintf(nm, sizeof nm, "C  g%d", g);
    timeit(nm, 2 * 65536, [&] { k_copy<false><<<grid, 256>>>(in, out, nt); });
    snprintf(nm, sizeof nm, "CN g%d", g);
    timeit(nm, 2 * 65536, [&] { k_copy<true><<<grid, 256>>>(in, out, nt); });
  }
  for (uint32_t ib : {20000u, 24000u}) {
    for (int g : {2, 3}) {
      const int grid = g * cus;
      snprintf(nm, sizeof nm, "D  in%u g%d", ib, g);
      timeit(nm, 65536 + ib, [&] { k_dma<false><<<grid, 256>>>(in, stride, ib, out, nt); });
      snprintf(nm, sizeof nm, "DN in%u g%d", ib, g);
      timeit(nm, 65536 + ib, [&] { k_dma<true><<<grid, 256>>>(in, stride, ib, out, nt); });
    }
  }
  return 0;
}
