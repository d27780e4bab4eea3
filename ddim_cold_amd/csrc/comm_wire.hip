// Gradient wire-format conversion for the native RCCL reducer (comm.cpp).
//
// bf16 wire: the fp32 gradient range is packed to bf16 (round-to-nearest-even)
// on the communication stream, all-reduced by RCCL as ncclBfloat16, and
// unpacked back into the fp32 arena.  Both passes are pure streams over HBM:
// 8 elements (32 B in, 16 B out) per lane, grid capped at 4 waves per CU
// (256 CUs) with a grid-stride loop, so a bucket of a few MB is one short
// kernel that leaves most CUs to the backward it overlaps.
#include "common.h"
#include "kernels.h"

namespace dc {

namespace {
constexpr int kThreads = 256;
constexpr int kMaxBlocks = 256;  // one 4-wave workgroup per CU: the overlapped backward keeps the rest

inline int grid_for(int64_t n8) {
  int64_t b = (n8 + kThreads - 1) / kThreads;
  return (int)(b < 1 ? 1 : (b > kMaxBlocks ? kMaxBlocks : b));
}
}  // namespace

__global__ __launch_bounds__(kThreads) void wire_pack_kernel(const float* __restrict__ src, bf16* __restrict__ dst,
                                                             int64_t n) {
  const int64_t n8 = n / 8;
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n8; i += stride) {
    const float4 a = reinterpret_cast<const float4*>(src)[2 * i];
    const float4 b = reinterpret_cast<const float4*>(src)[2 * i + 1];
    bf16x8 o;
    o[0] = f2bf(a.x); o[1] = f2bf(a.y); o[2] = f2bf(a.z); o[3] = f2bf(a.w);
    o[4] = f2bf(b.x); o[5] = f2bf(b.y); o[6] = f2bf(b.z); o[7] = f2bf(b.w);
    reinterpret_cast<bf16x8*>(dst)[i] = o;
  }
  // tail (n not a multiple of 8): one thread of block 0
  if (blockIdx.x == 0 && threadIdx.x == 0)
    for (int64_t j = n8 * 8; j < n; ++j) dst[j] = f2bf(src[j]);
}

__global__ __launch_bounds__(kThreads) void wire_unpack_kernel(const bf16* __restrict__ src, float* __restrict__ dst,
                                                               int64_t n) {
  const int64_t n8 = n / 8;
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n8; i += stride) {
    const bf16x8 v = reinterpret_cast<const bf16x8*>(src)[i];
    reinterpret_cast<float4*>(dst)[2 * i] = make_float4(bf2f(v[0]), bf2f(v[1]), bf2f(v[2]), bf2f(v[3]));
    reinterpret_cast<float4*>(dst)[2 * i + 1] = make_float4(bf2f(v[4]), bf2f(v[5]), bf2f(v[6]), bf2f(v[7]));
  }
  if (blockIdx.x == 0 && threadIdx.x == 0)
    for (int64_t j = n8 * 8; j < n; ++j) dst[j] = bf2f(src[j]);
}

}  // namespace dc

using namespace dc;

void wire_pack_launch(const float* src, void* dst, int64_t n, hipStream_t stream) {
  if (n <= 0) return;
  wire_pack_kernel<<<grid_for(n / 8), kThreads, 0, stream>>>(src, reinterpret_cast<bf16*>(dst), n);
}

void wire_unpack_launch(const void* src, float* dst, int64_t n, hipStream_t stream) {
  if (n <= 0) return;
  wire_unpack_kernel<<<grid_for(n / 8), kThreads, 0, stream>>>(reinterpret_cast<const bf16*>(src), dst, n);
}
