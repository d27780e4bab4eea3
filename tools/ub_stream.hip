// Microbenchmark: how fast can one workgroup per CU stream a shared weight
// panel (every workgroup reads the same [R][K] bf16 matrix)?
//   mode 0: LDS-DMA ring (buffer_load ... lds), S stages of 64-deep K tiles, counted vmcnt
//   mode 1: plain global_load_dwordx4 into registers, 8 loads in flight per lane
//   mode 2: LDS-DMA ring, each workgroup reads its OWN copy (no sharing)
// Build: hipcc --offload-arch=gfx950 -O3 -I ddim_cold_amd/csrc tools/ub_stream.hip -o /tmp/ub_stream
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "gemm_common.h"

using namespace dc;

template <int R, int S>
__global__ __launch_bounds__(256) void dma_stream(const bf16* w, int K, float* sink, size_t per_wg_elems) {
  using OB = DmaOperand<R, false>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  OB ob;
  ob.init(w + per_wg_elems * blockIdx.x, K, R, 0, wave, lane);
  const int nk = K / 64;
  float acc = 0.f;
  for (int s = 0; s < S - 1; ++s)
    if (s < nk) ob.issue(smem + s * OB::BYTES, s, wave);
  for (int kt = 0; kt < nk; ++kt) {
    vm_wait_rem<OB::PER_WAVE>(min(S - 2, nk - 1 - kt));
    raw_barrier();
    if (kt + S - 1 < nk) ob.issue(smem + ((kt + S - 1) % S) * OB::BYTES, kt + S - 1, wave);
    acc += *reinterpret_cast<const float*>(smem + (kt % S) * OB::BYTES + threadIdx.x * 4);
  }
  if (acc == 12345.f) sink[blockIdx.x] = acc;
}

template <int R>
__global__ __launch_bounds__(256) void reg_stream(const bf16* w, int K, float* sink) {
  // R rows x K cols bf16; 256 threads x 16 B per load
  const int total = R * K / 8;  // 16-B chunks
  const u32x4* p = reinterpret_cast<const u32x4*>(w);
  uint32_t acc = 0;
  int c = threadIdx.x;
  for (; c + 7 * 256 < total; c += 8 * 256) {
    u32x4 v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = p[c + i * 256];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc ^= v[i][0] ^ v[i][3];
  }
  for (; c < total; c += 256) acc ^= p[c][1];
  if (acc == 0x12345u) sink[blockIdx.x] = (float)acc;
}

int main() {
  const int R = 384, K = 384;
  const int nwg_list[] = {65, 130, 256};
  bf16* w;
  float* sink;
  const size_t elems = (size_t)R * K;
  hipMalloc(&w, elems * 2 * 256);
  hipMemset(w, 0, elems * 2 * 256);
  hipMalloc(&sink, 4096);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  constexpr int S = 3;
  const int lds = S * R * 128;
  hipFuncSetAttribute(reinterpret_cast<const void*>(&dma_stream<384, S>), hipFuncAttributeMaxDynamicSharedMemorySize,
                      lds);
  for (int mode = 0; mode < 3; ++mode)
    for (int nwg : nwg_list) {
      auto launch = [&] {
        if (mode == 0) hipLaunchKernelGGL((dma_stream<384, S>), dim3(nwg), dim3(256), lds, 0, w, K, sink, (size_t)0);
        if (mode == 1) hipLaunchKernelGGL(reg_stream<384>, dim3(nwg), dim3(256), 0, 0, w, K, sink);
        if (mode == 2) hipLaunchKernelGGL((dma_stream<384, S>), dim3(nwg), dim3(256), lds, 0, w, K, sink, elems);
      };
      for (int i = 0; i < 5; ++i) launch();
      hipDeviceSynchronize();
      hipEventRecord(e0);
      const int reps = 50;
      for (int i = 0; i < reps; ++i) launch();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double us = ms * 1e3 / reps;
      const double gbs_per_wg = elems * 2 / (us * 1e-6) / 1e9;
      printf("mode %d (%s) nwg %3d: %7.2f us/launch  %6.1f GB/s per WG  %7.1f GB/s total\n", mode,
             mode == 0 ? "dma shared " : mode == 1 ? "reg shared " : "dma private", nwg, us, gbs_per_wg,
             gbs_per_wg * nwg);
    }
  return 0;
}
