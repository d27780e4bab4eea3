// Microbenchmark: per-workgroup streaming rate of the operand loaders.
//
// A: every workgroup streams the SAME [R][K] bf16 panel (weights shared by all
//    workgroups, L2-resident), 295 KB (R = K = 384):
//      dma<S>  : LDS-DMA ring (buffer_load ... lds), S stages of 64-deep K tiles
//      reg<IN> : global_load_dwordx4 into registers, IN loads in flight per lane
// B: the 64x64-tile GEMM operand pattern: each workgroup streams its own A panel
//    (64 rows) and a shared B panel (64 rows), K = 384, LDS-DMA ring of S stages.
// Build: hipcc --offload-arch=gfx950 -O3 -I ddim_cold_amd/csrc tools/ub_stream.hip -o tools/ub_stream.bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include "gemm_common.h"

using namespace dc;

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %d at %d\n", e_, __LINE__); return 1; } } while (0)

template <int R, int S>
__global__ __launch_bounds__(256) void dma_stream(const bf16* w, int K, float* sink) {
  using OB = DmaOperand<R, false>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  OB ob;
  ob.init(w, K, R, 0, wave, lane);
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

template <int IN>
__global__ __launch_bounds__(256) void reg_stream(const bf16* w, int total16, float* sink) {
  const u32x4* p = reinterpret_cast<const u32x4*>(w);
  uint32_t acc = 0;
  int c = threadIdx.x;
  for (; c + (IN - 1) * 256 < total16; c += IN * 256) {
    u32x4 v[IN];
#pragma unroll
    for (int i = 0; i < IN; ++i) v[i] = p[c + i * 256];
#pragma unroll
    for (int i = 0; i < IN; ++i) acc ^= v[i][0] ^ v[i][3];
  }
  for (; c < total16; c += 256) acc ^= p[c][1];
  if (acc == 0x12345u) sink[blockIdx.x] = (float)acc;
}

// GEMM operand pattern: A panel per workgroup (rows 64*bid), B panel shared
template <int S>
__global__ __launch_bounds__(256) void gemm_pattern(const bf16* a, const bf16* b, int M, int K, float* sink) {
  using OA = DmaOperand<64, false>;
  constexpr int STAGE = 2 * OA::BYTES;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  OA oa, ob;
  oa.init(a, K, M, (blockIdx.x % (M / 64)) * 64, wave, lane);
  ob.init(b, K, 384, (blockIdx.x / (M / 64)) * 64, wave, lane);
  const int nk = K / 64;
  float acc = 0.f;
  for (int s = 0; s < S - 1; ++s)
    if (s < nk) {
      oa.issue(smem + s * STAGE, s, wave);
      ob.issue(smem + s * STAGE + OA::BYTES, s, wave);
    }
  for (int kt = 0; kt < nk; ++kt) {
    vm_wait_rem<2 * OA::PER_WAVE>(min(S - 2, nk - 1 - kt));
    raw_barrier();
    if (kt + S - 1 < nk) {
      oa.issue(smem + ((kt + S - 1) % S) * STAGE, kt + S - 1, wave);
      ob.issue(smem + ((kt + S - 1) % S) * STAGE + OA::BYTES, kt + S - 1, wave);
    }
    acc += *reinterpret_cast<const float*>(smem + (kt % S) * STAGE + threadIdx.x * 4);
  }
  if (acc == 12345.f) sink[blockIdx.x] = acc;
}

// explicit instantiations (hipcc drops host stubs of templates first used in lambdas)
template __global__ void dma_stream<384, 2>(const bf16*, int, float*);
template __global__ void dma_stream<384, 3>(const bf16*, int, float*);
template __global__ void reg_stream<1>(const bf16*, int, float*);
template __global__ void reg_stream<4>(const bf16*, int, float*);
template __global__ void reg_stream<8>(const bf16*, int, float*);
template __global__ void reg_stream<16>(const bf16*, int, float*);
template __global__ void reg_stream<32>(const bf16*, int, float*);
template __global__ void gemm_pattern<2>(const bf16*, const bf16*, int, int, float*);
template __global__ void gemm_pattern<3>(const bf16*, const bf16*, int, int, float*);
template __global__ void gemm_pattern<4>(const bf16*, const bf16*, int, int, float*);
template __global__ void gemm_pattern<6>(const bf16*, const bf16*, int, int, float*);

template <typename F>
static double time_us(F launch, int reps = 200) {
  for (int i = 0; i < 5; ++i) launch();
  (void)hipDeviceSynchronize();
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  for (int i = 0; i < reps; ++i) launch();
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms * 1e3 / reps;
}

template <int S>
static int run_dma(const bf16* w, float* sink, int nwg) {
  const int lds = S * 384 * 128;
  CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&dma_stream<384, S>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  const double us = time_us([&] { hipLaunchKernelGGL((dma_stream<384, S>), dim3(nwg), dim3(256), lds, 0, w, 384, sink); });
  printf("A dma S=%d  nwg %3d: %7.2f us  %6.1f GB/s per WG\n", S, nwg, us, 384 * 384 * 2 / (us * 1e3));
  return 0;
}

template <int IN>
static void run_reg(const bf16* w, float* sink, int nwg) {
  const double us = time_us([&] { hipLaunchKernelGGL(reg_stream<IN>, dim3(nwg), dim3(256), 0, 0, w, 384 * 384 / 8, sink); });
  printf("A reg IN=%2d nwg %3d: %7.2f us  %6.1f GB/s per WG\n", IN, nwg, us, 384 * 384 * 2 / (us * 1e3));
}

template <int S>
static int run_gemm(const bf16* a, const bf16* b, float* sink, int M) {
  const int lds = S * 2 * 64 * 128;
  CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_pattern<S>), hipFuncAttributeMaxDynamicSharedMemorySize,
                            lds));
  const int nwg = (M / 64) * 6;
  const double us = time_us([&] { hipLaunchKernelGGL(gemm_pattern<S>, dim3(nwg), dim3(256), lds, 0, a, b, M, 384, sink); });
  printf("B gemm-pattern S=%d M=%d (%d WGs, 96 KB each): %7.2f us\n", S, M, nwg, us);
  return 0;
}

int main() {
  bf16 *w, *a;
  float* sink;
  CHECK(hipMalloc(&w, 384 * 384 * 2));
  CHECK(hipMemset(w, 0, 384 * 384 * 2));
  CHECK(hipMalloc(&a, 8192 * 384 * 2));
  CHECK(hipMemset(a, 0, 8192 * 384 * 2));
  CHECK(hipMalloc(&sink, 65536));
  const double empty = time_us([&] { hipLaunchKernelGGL(reg_stream<1>, dim3(1), dim3(256), 0, 0, w, 0, sink); });
  printf("empty launch: %.2f us\n", empty);
  for (int nwg : {65, 130, 256}) {
    run_dma<2>(w, sink, nwg);
    run_dma<3>(w, sink, nwg);
    run_reg<4>(w, sink, nwg);
    run_reg<8>(w, sink, nwg);
    run_reg<16>(w, sink, nwg);
    run_reg<32>(w, sink, nwg);
  }
  for (int M : {2048, 4096, 8192}) {
    run_gemm<2>(a, w, sink, M);
    run_gemm<3>(a, w, sink, M);
    run_gemm<4>(a, w, sink, M);
    run_gemm<6>(a, w, sink, M);
  }
  return 0;
}
