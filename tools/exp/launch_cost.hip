#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
struct P { uint32_t* q; uint32_t* out; uint32_t pad[60]; };
__global__ void __launch_bounds__(256) k_empty(P p) { if (p.q[0] == 0) return; p.out[threadIdx.x] = 1; }
__device__ __attribute__((noinline)) void heavy(P p, int n) {
  uint32_t a[300];
  for (int i = 0; i < 300; i++) a[i] = p.out[(i * 7 + threadIdx.x) % 4096];
  for (int j = 0; j < n; j++) for (int i = 0; i < 300; i++) a[(i * 13 + j) % 300] += a[i] * 3 + j;
  uint32_t s = 0; for (int i = 0; i < 300; i++) s += a[(i * p.q[1]) % 300];
  p.out[threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k_scratch(P p) { if (p.q[0] == 0) return; heavy(p, p.q[0]); }
int main() {
  P p{}; hipMalloc(&p.q, 64); hipMemset(p.q, 0, 64); hipMalloc(&p.out, 1 << 20);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  const int grids[] = {1, 32, 256, 1024};
  for (int kind = 0; kind < 2; kind++)
    for (int g : grids) {
      for (int w = 0; w < 50; w++) kind ? k_scratch<<<g, 256>>>(p) : k_empty<<<g, 256>>>(p);
      hipEventRecord(a);
      for (int w = 0; w < 1000; w++) kind ? k_scratch<<<g, 256>>>(p) : k_empty<<<g, 256>>>(p);
      hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b);
      printf("%s grid %4d: %.2f us per launch (back to back)\n", kind ? "scratch" : "empty  ", g, ms);
    }
  return 0;
}
