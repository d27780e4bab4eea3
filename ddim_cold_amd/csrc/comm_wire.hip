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
// (FlagSignal.check).  Fail-fast: once err is raised (by this or any earlier wait)
// every later wait returns at once, so a broken hand-off layout costs ONE timeout,
// not one per bucket per step, before the host sees the error and drops it.
__global__ __launch_bounds__(64) void flag_wait_kernel(const unsigned int* __restrict__ flags, int k,
                                                       unsigned int expected, unsigned int* __restrict__ err,
                                                       unsigned long long ticks) {
  const unsigned int lane = threadIdx.x;
  if (lane != 0) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (true) {
    const unsigned int v = __hip_atomic_load(flags + k + lane, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
    if (static_cast<int>(v - expected) >= 0) break;
    if (__hip_atomic_load(err + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) break;
    if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) {
      __hip_atomic_store(err + lane, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

// In-process loopback all-reduce between TWO endpoints on ONE device: stands in for
// RCCL when one process drives two data-parallel engines (parallel/comm.py
// LoopbackPair), so each engine's comm-stream work depends on the OTHER engine's
// compute replay -- the cross-rank dependency a 1-rank group never creates.
// Workgroup b of endpoint e owns chunk b of the buffer and pairs only with
// workgroup b of the peer's launch (no grid-wide barrier; both launches are
// kPairBlocks workgroups, co-resident on a 256-CU device):
//   1. c = arrive[e][b] + 1 (its own counter: graph replays need no host value)
//   2. copy the chunk into stage[e]; publish arrive[e][b] = c (agent release)
//   3. wait for arrive[1-e][b] >= c; chunk = stage[0] + stage[1] (the same order on
//      both endpoints: bit-identical replicas)
//   4. publish done[e][b] = c; wait for done[1-e][b] >= c (the peer has read
//      stage[e], so the next collective may overwrite it)
// Waits are bounded (err[0] raised, later waits return at once), so a hand-off
// that never comes cannot wedge the GPU.
constexpr int kPairBlocks = 64;

__device__ __forceinline__ bool pair_wait(const unsigned int* f, unsigned int c, unsigned int* err,
                                          unsigned long long ticks, unsigned int lane) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (true) {
    const unsigned int v = __hip_atomic_load(f + lane, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    if (static_cast<int>(v - c) >= 0) return true;
    if (__hip_atomic_load(err + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return false;
    if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) {
      __hip_atomic_store(err + lane, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

__global__ __launch_bounds__(256) void pair_allreduce_kernel(float* __restrict__ buf, int64_t n,
                                                             float* __restrict__ stage, int64_t stage_n,
                                                             unsigned int* __restrict__ flags, int e,
                                                             unsigned int* __restrict__ err, unsigned long long ticks) {
  __shared__ unsigned int sh_c;
  __shared__ int sh_ok;
  const int b = blockIdx.x;
  const unsigned int lane = threadIdx.x;
  unsigned int* arrive = flags;                  // [2][kPairBlocks]
  unsigned int* done = flags + 2 * kPairBlocks;  // [2][kPairBlocks]
  const int64_t chunk = (n + kPairBlocks - 1) / kPairBlocks;
  const int64_t lo = b * chunk, hi = lo + chunk < n ? lo + chunk : n;
  if (lane == 0) {
    sh_c = __hip_atomic_load(arrive + e * kPairBlocks + b + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    sh_ok = 1;
  }
  __syncthreads();
  const unsigned int c = sh_c;
  float* mine = stage + (int64_t)e * stage_n;
  for (int64_t i = lo + lane; i < hi; i += 256) mine[i] = buf[i];
  __threadfence();
  __syncthreads();
  if (lane == 0) {
    __hip_atomic_store(arrive + e * kPairBlocks + b + lane, c, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    sh_ok = pair_wait(arrive + (1 - e) * kPairBlocks + b, c, err, ticks, lane) ? 1 : 0;
  }
  __syncthreads();
  if (sh_ok) {
    const float* s0 = stage;
    const float* s1 = stage + stage_n;
    for (int64_t i = lo + lane; i < hi; i += 256) buf[i] = s0[i] + s1[i];
  }
  __threadfence();
  __syncthreads();
  if (lane == 0) {
    __hip_atomic_store(done + e * kPairBlocks + b + lane, c, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    pair_wait(done + (1 - e) * kPairBlocks + b, c, err, ticks, lane);
  }
}

}  // namespace dc

using namespace dc;

int pair_allreduce_flags() { return 4 * kPairBlocks; }

void pair_allreduce_launch(float* buf, int64_t n, float* stage, int64_t stage_n, void* flags, int e, void* err,
                           int64_t timeout_us, hipStream_t stream) {
  const unsigned long long ticks = timeout_us > 0 ? (unsigned long long)timeout_us * 100ull : 200000000ull;
  pair_allreduce_kernel<<<kPairBlocks, 256, 0, stream>>>(buf, n, stage, stage_n, reinterpret_cast<unsigned int*>(flags),
                                                         e, reinterpret_cast<unsigned int*>(err), ticks);
}

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
