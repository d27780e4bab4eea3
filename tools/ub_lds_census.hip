// Residency census: how many workgroups of a given LDS size (and block size) run
// at once on MI355X.  Every workgroup stamps s_memrealtime at entry, touches its
// LDS, then spins ~5 us (bounded, s_sleep) so that a workgroup that had to wait
// for a slot starts visibly later.  Prints, per LDS size, how many of the grid's
// workgroups started within 2 us of the first one.
//   hipcc --offload-arch=gfx950 -O2 tools/ub_lds_census.hip -o /tmp/ub_lds_census && /tmp/ub_lds_census
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

__global__ void census(unsigned long long* stamp, int spin_ticks) {
  extern __shared__ float lds[];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  lds[threadIdx.x] = (float)threadIdx.x;
  __syncthreads();
  if (threadIdx.x == 0) stamp[blockIdx.x] = t0;
  // wait ~spin_ticks of the 100 MHz counter; every wave reaches the exit
  for (int i = 0; i < 100000; ++i) {
    if (__builtin_amdgcn_s_memrealtime() - t0 > (unsigned long long)spin_ticks) break;
    __builtin_amdgcn_s_sleep(2);
  }
  if (lds[threadIdx.x] < 0.f) stamp[0] = 0;  // keep the LDS live
}

// STATIC LDS of SZ bytes (the short attention backward: 384 threads, 79,872 B)
template <int SZ>
__global__ __launch_bounds__(384) void census_static(unsigned long long* stamp, int spin_ticks) {
  __shared__ __attribute__((aligned(16))) char lds[SZ];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  reinterpret_cast<float*>(lds)[threadIdx.x] = (float)threadIdx.x;
  __syncthreads();
  if (threadIdx.x == 0) stamp[blockIdx.x] = t0;
  for (int i = 0; i < 100000; ++i) {
    if (__builtin_amdgcn_s_memrealtime() - t0 > (unsigned long long)spin_ticks) break;
    __builtin_amdgcn_s_sleep(2);
  }
  if (reinterpret_cast<float*>(lds)[threadIdx.x] < 0.f) stamp[0] = 0;
}

// DYNAMIC LDS with the attention kernel's launch bounds (384)
__global__ __launch_bounds__(384) void census_dyn384(unsigned long long* stamp, int spin_ticks) {
  extern __shared__ float ldsd[];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  ldsd[threadIdx.x] = (float)threadIdx.x;
  __syncthreads();
  if (threadIdx.x == 0) stamp[blockIdx.x] = t0;
  for (int i = 0; i < 100000; ++i) {
    if (__builtin_amdgcn_s_memrealtime() - t0 > (unsigned long long)spin_ticks) break;
    __builtin_amdgcn_s_sleep(2);
  }
  if (ldsd[threadIdx.x] < 0.f) stamp[0] = 0;
}

static void run_dyn384(unsigned long long* d, int grid, int bytes) {
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&census_dyn384), hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024);
  std::vector<unsigned long long> h(grid);
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(census_dyn384, dim3(grid), dim3(384), bytes, 0, d, 500);
    if (hipDeviceSynchronize() != hipSuccess) return;
  }
  (void)hipMemcpy(h.data(), d, grid * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  const unsigned long long t0 = *std::min_element(h.begin(), h.end());
  int early = 0;
  for (auto v : h) early += (v - t0) < 200;
  printf("DYNAMIC LDS %6d B, 384 threads, launch_bounds(384): %4d of %d resident at once (%.2f per CU)\n", bytes,
         early, grid, early / 256.0);
}

template <int SZ>
static int run_static(unsigned long long* d, int grid, int nt) {
  std::vector<unsigned long long> h(grid);
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL((census_static<SZ>), dim3(grid), dim3(nt), 0, 0, d, 500);
    if (hipDeviceSynchronize() != hipSuccess) return -1;
  }
  (void)hipMemcpy(h.data(), d, grid * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  const unsigned long long t0 = *std::min_element(h.begin(), h.end());
  int early = 0;
  for (auto v : h) early += (v - t0) < 200;
  printf("STATIC LDS %6d B, %d threads: %4d of %d workgroups resident at once (%.2f per CU)\n", SZ, nt, early, grid,
         early / 256.0);
  return early;
}

int main() {
  const int grid = 512;
  unsigned long long* d;
  (void)hipMalloc(&d, grid * sizeof(unsigned long long));
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&census), hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024);
  const int threads[] = {256, 384};
  const int kib[] = {40, 60, 64, 65, 72, 76, 78, 80};
  for (int nt : threads)
    for (int k : kib) {
      std::vector<unsigned long long> h(grid);
      for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(census, dim3(grid), dim3(nt), k * 1024, 0, d, 500);
        if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed (%d KiB)\n", k); return 1; }
      }
      (void)hipMemcpy(h.data(), d, grid * sizeof(unsigned long long), hipMemcpyDeviceToHost);
      const unsigned long long t0 = *std::min_element(h.begin(), h.end());
      int early = 0;
      for (auto v : h) early += (v - t0) < 200;  // started within 2 us
      printf("block %d threads, LDS %2d KiB: %3d of %d workgroups resident at once (%.2f per CU)\n", nt, k, early,
             grid, early / 256.0);
    }
  const int g2 = 2048;
  unsigned long long* d2;
  (void)hipMalloc(&d2, g2 * sizeof(unsigned long long));
  run_static<79872>(d2, g2, 384);
  run_dyn384(d2, g2, 61440);
  run_dyn384(d2, g2, 79872);
  run_dyn384(d2, g2, 81920);
  (void)hipFree(d2);
  (void)hipFree(d);
  return 0;
}
