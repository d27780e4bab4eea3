// bf16 matrix transposes for the input-gradient GEMMs (engine.TransposedShadows):
// dX = dY W runs on the forward's k-contiguous LDS-DMA path when W^T is stored
// ([in][out]) -- 31.7 -> 25.5 us for vit_small_200's QKV input gradient
// (tools/ub_dgrad_layout.py) against the transposed-operand path's ds_read_b64_tr_b16
// fragments.  After every optimizer step one launch re-transposes the bf16 shadows of
// the weights: 64 x 64 tiles through LDS, 16-byte loads and stores on both sides.
#include "common.h"
#include "kernels.h"
#include <stdexcept>

namespace dc {

struct TrJob {
  const bf16* src;  // [R][C]
  bf16* dst;        // [C][R]
  int R, C;
};
struct TrTable {
  TrJob j[TRANSPOSE_MAX];
  int start[TRANSPOSE_MAX + 1];
  int n;
};

__global__ __launch_bounds__(256) void transpose_bf16_kernel(TrTable tb) {
  __shared__ uint16_t tile[64][64 + 8];  // +16 B per row: the column gathers spread over banks
  const int bid = blockIdx.x;
  int lo = 0, hi = tb.n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (bid >= tb.start[mid]) lo = mid;
    else hi = mid - 1;
  }
  const TrJob& jb = tb.j[lo];
  const int tiles_c = (jb.C + 63) / 64;
  const int local = bid - tb.start[lo];
  const int r0 = (local / tiles_c) * 64, c0 = (local % tiles_c) * 64;
  const uint16_t* src = reinterpret_cast<const uint16_t*>(jb.src);
  uint16_t* dst = reinterpret_cast<uint16_t*>(jb.dst);
  // load: 64 rows x 8 chunks of 8 elements (R % 8 == C % 8 == 0: host check)
  u32x4 v[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int ch = threadIdx.x + 256 * i, r = ch >> 3, c = (ch & 7) * 8;
    v[i] = (r0 + r < jb.R && c0 + c < jb.C)
               ? *reinterpret_cast<const u32x4*>(src + (size_t)(r0 + r) * jb.C + c0 + c)
               : u32x4{0u, 0u, 0u, 0u};
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int ch = threadIdx.x + 256 * i, r = ch >> 3, c = (ch & 7) * 8;
    *reinterpret_cast<u32x4*>(&tile[r][c]) = v[i];
  }
  __syncthreads();
  // store: output row c0 + dc holds tile column dc, 8 chunks of 8 elements
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int ch = threadIdx.x + 256 * i, dc = ch >> 3, rr = (ch & 7) * 8;
    if (c0 + dc >= jb.C || r0 + rr >= jb.R) continue;
    u32x4 w;
#pragma unroll
    for (int e = 0; e < 4; ++e)
      w[e] = (uint32_t)tile[rr + 2 * e][dc] | ((uint32_t)tile[rr + 2 * e + 1][dc] << 16);
    *reinterpret_cast<u32x4*>(dst + (size_t)(c0 + dc) * jb.R + r0 + rr) = w;
  }
}

}  // namespace dc

using namespace dc;

void transpose_bf16_launch(const void* const* srcs, void* const* dsts, const int* R, const int* C, int n,
                           hipStream_t stream) {
  if (n < 1 || n > TRANSPOSE_MAX) throw std::runtime_error("transpose_bf16: 1..TRANSPOSE_MAX matrices per launch");
  TrTable tb{};
  tb.n = n;
  int tiles = 0;
  for (int i = 0; i < n; ++i) {
    if (R[i] % 8 || C[i] % 8) throw std::runtime_error("transpose_bf16: rows and columns must be multiples of 8");
    tb.j[i] = TrJob{reinterpret_cast<const bf16*>(srcs[i]), reinterpret_cast<bf16*>(dsts[i]), R[i], C[i]};
    tb.start[i] = tiles;
    tiles += ((R[i] + 63) / 64) * ((C[i] + 63) / 64);
  }
  for (int i = n; i <= TRANSPOSE_MAX; ++i) tb.start[i] = tiles;
  static_assert(sizeof(TrTable) <= 4000, "kernel argument block");
  hipLaunchKernelGGL(transpose_bf16_kernel, dim3(tiles), dim3(256), 0, stream, tb);
}
