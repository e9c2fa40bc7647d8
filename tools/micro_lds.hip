// Design study (not part of the product): does gfx950 serve ds_read_b32 /
// ds_read_b64 at byte-unaligned LDS addresses, with which data, at what cost?
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/micro_lds tools/micro_lds.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

// correctness: LDS filled with byte i = i & 0xff ^ (i >> 8); thread t reads
// 4 (or 8) bytes at byte offset t (any alignment)
__global__ void k_check(uint32_t* out32, uint64_t* out64) {
  __shared__ uint8_t X[8192];
  for (int i = threadIdx.x; i < 8192; i += blockDim.x) X[i] = (uint8_t)((i & 0xff) ^ (i >> 8));
  __syncthreads();
  const uint32_t o = threadIdx.x;
  uint32_t off = o;
  asm volatile("" : "+v"(off));
  out32[o] = *(const uint32_t*)(X + off);
  out64[o] = *(const uint64_t*)(X + off);
}

// throughput: each lane reads `iters` times at base + lane * stride + shift
template <int W>
__global__ void k_rate(uint32_t* sink, uint32_t shift, uint32_t stride, int iters) {
  __shared__ uint8_t X[65536];
  for (int i = threadIdx.x; i < 65536 / 4; i += blockDim.x) ((uint32_t*)X)[i] = i * 2654435761u;
  __syncthreads();
  uint32_t acc = 0;
  uint32_t a = (threadIdx.x * stride + shift) & 0x7fff;
  for (int it = 0; it < iters; it++) {
    uint32_t aa = (a + it * 64) & 0x7fff;
    asm volatile("" : "+v"(aa));
    if (W == 4) acc += *(const uint32_t*)(X + aa);
    else if (W == 8) { uint64_t v = *(const uint64_t*)(X + aa); acc += (uint32_t)v ^ (uint32_t)(v >> 32); }
    else { uint4 v = *(const uint4*)(X + aa); acc += v.x ^ v.y ^ v.z ^ v.w; }
  }
  if (acc == 0x12345678) sink[0] = acc;
}

int main() {
  uint32_t *d32, *sink;
  uint64_t* d64;
  CK(hipMalloc(&d32, 4 * 256));
  CK(hipMalloc(&d64, 8 * 256));
  CK(hipMalloc(&sink, 64));
  hipLaunchKernelGGL(k_check, dim3(1), dim3(256), 0, 0, d32, d64);
  CK(hipDeviceSynchronize());
  std::vector<uint32_t> h32(256);
  std::vector<uint64_t> h64(256);
  CK(hipMemcpy(h32.data(), d32, 4 * 256, hipMemcpyDeviceToHost));
  CK(hipMemcpy(h64.data(), d64, 8 * 256, hipMemcpyDeviceToHost));
  int bad32 = 0, bad64 = 0;
  for (int o = 0; o < 256; o++) {
    uint32_t e32 = 0;
    uint64_t e64 = 0;
    for (int b = 0; b < 8; b++) {
      const int i = o + b;
      const uint64_t v = (uint8_t)((i & 0xff) ^ (i >> 8));
      if (b < 4) e32 |= (uint32_t)v << (8 * b);
      e64 |= v << (8 * b);
    }
    if (h32[o] != e32) { if (bad32 < 4) printf("b32 off %d got %08x want %08x\n", o, h32[o], e32); bad32++; }
    if (h64[o] != e64) { if (bad64 < 4) printf("b64 off %d got %016llx want %016llx\n", o, (unsigned long long)h64[o], (unsigned long long)e64); bad64++; }
  }
  printf("unaligned ds_read_b32: %d/256 wrong; ds_read_b64: %d/256 wrong\n", bad32, bad64);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int iters = 4096;
  struct Cfg { int w; uint32_t shift, stride; const char* name; } cfgs[] = {
      {4, 0, 4, "b32 aligned, stride 4"}, {4, 2, 4, "b32 +2, stride 4"}, {4, 1, 4, "b32 +1, stride 4"},
      {4, 2, 116, "b32 +2, stride 116"}, {4, 0, 116, "b32 aligned, stride 116"},
      {8, 0, 8, "b64 aligned, stride 8"}, {8, 4, 8, "b64 +4, stride 8"}, {8, 2, 8, "b64 +2, stride 8"},
      {16, 0, 16, "b128 aligned, stride 16"}, {16, 2, 16, "b128 +2, stride 16"}};
  for (auto& c : cfgs) {
    for (int rep = 0; rep < 2; rep++) {
      CK(hipEventRecord(e0));
      if (c.w == 4) hipLaunchKernelGGL(k_rate<4>, dim3(1024), dim3(512), 0, 0, sink, c.shift, c.stride, iters);
      else if (c.w == 8) hipLaunchKernelGGL(k_rate<8>, dim3(1024), dim3(512), 0, 0, sink, c.shift, c.stride, iters);
      else hipLaunchKernelGGL(k_rate<16>, dim3(1024), dim3(512), 0, 0, sink, c.shift, c.stride, iters);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double bytes = 1024.0 * 512 * iters * c.w;
      if (rep) printf("%-26s %8.3f ms  %7.1f TB/s (LDS, all CUs)\n", c.name, ms, bytes / ms / 1e9);
    }
  }
  return 0;
}
