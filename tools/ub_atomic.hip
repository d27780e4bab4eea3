// Microbenchmark: fp32 atomic-add throughput into L2 for a flash-attention style dQ
// accumulation (vit_small_200: B*H = 192 heads, N = 626 -> 10 tiles of 64 queries,
// head dim 64).  Every (key tile, head) workgroup adds a 64 x 64 fp32 partial into
// each of the head's 10 query tiles: 10 workgroups contend per query tile.
//   atomic  : global atomic add (no return), one wave-instruction = 64 consecutive floats
//   store   : the same bytes as plain stores into private slots (no contention)
//   rmw     : plain load + add + store into the shared target (racy; bandwidth bound)
// Build: hipcc --offload-arch=gfx950 -O3 tools/ub_atomic.hip -o tools/ub_atomic.bin
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %d at %d\n", e_, __LINE__); return 1; } } while (0)

constexpr int QT = 10, KT = 10, BH = 192, HD = 64, TILE = 64 * HD;

template <int MODE>
__global__ __launch_bounds__(256) void dq_accumulate(float* __restrict__ dq, float* __restrict__ slots, float v) {
  const int kt = blockIdx.x, bh = blockIdx.y;
  for (int q = 0; q < QT; ++q) {
    const int qt = (q + kt) % QT;  // staggered start, as key tiles would reach query tiles
    float* dst = dq + ((size_t)bh * QT + qt) * TILE;
#pragma unroll
    for (int i = 0; i < TILE / 256; ++i) {
      const int e = i * 256 + threadIdx.x;
      const float x = v * (float)(e + q);
      if (MODE == 0) atomicAdd(dst + e, x);
      else if (MODE == 1) slots[(((size_t)bh * KT + kt) * QT + qt) * TILE + e] = x;
      else dst[e] += x;
    }
  }
}

int main() {
  float *dq, *slots;
  const size_t n = (size_t)BH * QT * TILE;
  CHECK(hipMalloc(&dq, n * sizeof(float)));
  CHECK(hipMalloc(&slots, n * KT * sizeof(float)));
  CHECK(hipMemset(dq, 0, n * sizeof(float)));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  const dim3 grid(KT, BH);
  const char* names[3] = {"atomic", "store", "rmw"};
  for (int mode = 0; mode < 3; ++mode) {
    for (int w = 0; w < 3; ++w) {
      if (mode == 0) hipLaunchKernelGGL(dq_accumulate<0>, grid, dim3(256), 0, 0, dq, slots, 1e-3f);
      if (mode == 1) hipLaunchKernelGGL(dq_accumulate<1>, grid, dim3(256), 0, 0, dq, slots, 1e-3f);
      if (mode == 2) hipLaunchKernelGGL(dq_accumulate<2>, grid, dim3(256), 0, 0, dq, slots, 1e-3f);
    }
    CHECK(hipDeviceSynchronize());
    const int reps = 20;
    CHECK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) {
      if (mode == 0) hipLaunchKernelGGL(dq_accumulate<0>, grid, dim3(256), 0, 0, dq, slots, 1e-3f);
      if (mode == 1) hipLaunchKernelGGL(dq_accumulate<1>, grid, dim3(256), 0, 0, dq, slots, 1e-3f);
      if (mode == 2) hipLaunchKernelGGL(dq_accumulate<2>, grid, dim3(256), 0, 0, dq, slots, 1e-3f);
    }
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, a, b));
    const double us = 1e3 * ms / reps;
    const double adds = (double)BH * KT * QT * TILE;
    printf("%-7s %8.1f us per launch  (%.1f G adds/s, %.2f TB/s of fp32 payload)\n", names[mode], us, adds / us * 1e-3,
           adds * 4 / us * 1e-6);
  }
  CHECK(hipFree(dq));
  CHECK(hipFree(slots));
  return 0;
}
