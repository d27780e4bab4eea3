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

// Bucket hand-off signal of the event-split data-parallel step (engine.py,
// comm_signal="flag"): one lane adds 1 to flags[k] with a system-scope release,
// i.e. after every earlier write of this queue's kernels is visible device-wide;
// the comm stream waits for the counter with a stream wait-value packet.  A plain
// kernel node, unlike an event-record node, keeps the compute graph one
// uninterrupted chain.  Vector-memory atomic (lane-indexed address).
__global__ __launch_bounds__(64) void flag_bump_kernel(unsigned int* __restrict__ flags, int k) {
  const unsigned int lane = threadIdx.x;
  if (lane == 0) __hip_atomic_fetch_add(flags + k + lane, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Comm-stream side of the hand-off: one lane polls flags[k] (system-scope acquire)
// until it reaches `expected` (wrap-safe), sleeping between polls.  Bounded: after
// `ticks` of s_memrealtime (100 MHz; 2e8 = 2 s by default) it gives up and raises
// err[0], so a hand-off that never comes cannot wedge the GPU; the host checks err
// (FlagSignal.check).
__global__ __launch_bounds__(64) void flag_wait_kernel(const unsigned int* __restrict__ flags, int k,
                                                       unsigned int expected, unsigned int* __restrict__ err,
                                                       unsigned long long ticks) {
  const unsigned int lane = threadIdx.x;
  if (lane != 0) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (true) {
    const unsigned int v = __hip_atomic_load(flags + k + lane, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
    if (static_cast<int>(v - expected) >= 0) break;
    if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) {
      __hip_atomic_store(err + lane, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

}  // namespace dc

using namespace dc;

void flag_wait_launch(const void* flags, int k, unsigned int expected, void* err, hipStream_t stream,
                      int64_t timeout_us) {
  const unsigned long long ticks = timeout_us > 0 ? (unsigned long long)timeout_us * 100ull : 200000000ull;
  flag_wait_kernel<<<1, 64, 0, stream>>>(reinterpret_cast<const unsigned int*>(flags), k, expected,
                                         reinterpret_cast<unsigned int*>(err), ticks);
}

void flag_bump_launch(void* flags, int k, hipStream_t stream) {
  flag_bump_kernel<<<1, 64, 0, stream>>>(reinterpret_cast<unsigned int*>(flags), k);
}

void wire_pack_launch(const float* src, void* dst, int64_t n, hipStream_t stream) {
  if (n <= 0) return;
  wire_pack_kernel<<<grid_for(n / 8), kThreads, 0, stream>>>(src, reinterpret_cast<bf16*>(dst), n);
}

void wire_unpack_launch(const void* src, float* dst, int64_t n, hipStream_t stream) {
  if (n <= 0) return;
  wire_unpack_kernel<<<grid_for(n / 8), kThreads, 0, stream>>>(reinterpret_cast<const bf16*>(src), dst, n);
}
