// Input-gradient GEMM with the LayerNorm backward in its epilogue (gfx950).
//
//   dl = dy W             (dy [M][K] bf16, W [K][D] bf16 = nn.Linear weight [out][in])
//   LayerNorm backward of dl at the LN input x (bf16 copy), saved mean / rstd:
//     x_hat = (x - mu) rstd,  dxh = dl gamma,
//     g_out = rstd (dxh - mean(dxh) - x_hat mean(dxh x_hat)) + g_res     (fp32)
//     gy    = bf16(g_out * dropout mask * drop-path scale)                (next dgrad's A)
//     y_out = bf16(x_hat gamma + beta)                                    (re-emitted LN output)
//     dgamma += sum_rows dl x_hat, dbeta += sum_rows dl                   (replica workspace)
//   -- the same outputs as linear_dgrad followed by ln_bwd_kernel (layernorm.hip), which
//   this replaces in the backward of every pre-norm block (ViT.py:124-137, :182) and of
//   the final norm.
//
// Why fused: the row statistics need whole rows, so the workgroup owns FULL rows (BM x D,
// D = 64 NCH) and streams all of W through its LDS ring; 4 waves each own D/4 columns.
//   * ViT-tiny (M = 2,080): one launch instead of two per LayerNorm (15 per step), the
//     dl round trip (bf16 write + read) gone -- latency-bound small kernels.
//   * vit_small_200 (M = 20,032): the LN backward is HBM-bound (16 B/element); the fused
//     kernel drops the 4 B/element of dl and one launch.
// Operand tiles go global -> LDS with the LDS-DMA ring of the main GEMM family
// (gemm_common.h DmaOperand: A k-contiguous, W as NCH transposed 64-column images read
// with ds_read_b64_tr_b16).  The accumulators are in the SWAPPED layout (mfma(B, A) =
// C^T): lane (g, li) holds row li of a 16-row fragment, columns 4g..4g+3 of a 16-column
// fragment -- 16-B vector epilogue accesses, row sums across the 4 g-lanes by
// permlane16/32 swaps, column sums (dgamma / dbeta) by a 16-lane reduce-scatter
// butterfly (45 exchanges for 48 values instead of 192).
#include "common.h"
#include "kernels.h"
#include "gemm_common.h"
#include <stdexcept>

namespace dc {

namespace {

__device__ __forceinline__ float psum16(float v) {  // v + the lane 16 apart
  const uint32_t u = __float_as_uint(v);
  const auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float psum32(float v) {  // v + the lane 32 apart
  const uint32_t u = __float_as_uint(v);
  const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// one reduce-scatter step over lanes BIT apart: the lane keeps the half of v selected by
// its BIT and adds the partner's copy of that half
template <int H, int BIT>
__device__ __forceinline__ void rs_step(const float (&v)[2 * H], float (&o)[H], int li) {
  const bool up = (li & BIT) != 0;
#pragma unroll
  for (int k = 0; k < H; ++k) {
    const float send = up ? v[k] : v[k + H];
    const float keep = up ? v[k + H] : v[k];
    o[k] = keep + __shfl_xor(send, BIT, 64);
  }
}

}  // namespace

template <int BM, int NCH, int S>
__global__ __launch_bounds__(256) void gemm_lnbwd_kernel(LnBwdParams p) {
  constexpr int D = NCH * 64;
  constexpr int FM = BM / 16;   // 16-row fragments (every wave covers all BM rows)
  constexpr int FN = NCH;       // 16-column fragments per wave (D / 4 columns)
  constexpr int WC = 16 * FN;   // columns per wave
  constexpr int V = 8 * FN;     // dgamma || dbeta partials per lane
  static_assert(FN % 2 == 0, "D must be a multiple of 128");
  using OA = DmaOperand<BM, false, 4>;
  using OB = DmaOperand<64, true, 4>;
  constexpr int STAGE = OA::BYTES + NCH * OB::BYTES;
  constexpr int LPT = OA::PER_WAVE + NCH * OB::PER_WAVE;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ float2 rred[4][BM];  // per-wave row partials {sum dxh, sum dxh x_hat}

  const int nwg = (p.M + BM - 1) / BM;
  const int m0 = xcd_remap(blockIdx.x, nwg) * BM;
  const int nk = (p.K + BK - 1) / BK;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, li = lane & 15;
  const int cw = wave * WC;  // first column of the wave

  OA oa;
  OB ob[NCH];
  const bf16* xin = reinterpret_cast<const bf16*>(p.x);
  bf16* gy_out = reinterpret_cast<bf16*>(p.gy);
  bf16* y_out = reinterpret_cast<bf16*>(p.y_out);
  oa.init(reinterpret_cast<const bf16*>(p.dy), p.K, p.M, m0, wave, lane);
#pragma unroll
  for (int c = 0; c < NCH; ++c) ob[c].init(reinterpret_cast<const bf16*>(p.w), D, p.K, 64 * c, wave, lane);

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (s < nk) {
      oa.issue(smem + s * STAGE, s, wave);
#pragma unroll
      for (int c = 0; c < NCH; ++c) ob[c].issue(smem + s * STAGE + OA::BYTES + c * OB::BYTES, s, wave);
    }
  // epilogue operands behind the first tiles: row statistics, gamma of the lane's columns
  float mu[FM], rs[FM];
  int rowc[FM];  // clamped row (loads); rows >= M are masked at the stores
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int r = m0 + i * 16 + li;
    rowc[i] = r < p.M ? r : p.M - 1;
    mu[i] = p.mean[rowc[i]];
    rs[i] = p.rstd[rowc[i]];
  }
  f32x4 gm[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) gm[j] = *reinterpret_cast<const f32x4*>(p.gamma + cw + 16 * j + 4 * g);
  const int64_t rng0 = p.rng[0], rng1 = p.rng[1];

  for (int kt = 0; kt < nk; ++kt) {
    const int rem = min(S - 2, nk - 1 - kt);
    vm_wait_rem<LPT>(rem);
    raw_barrier();
    if (kt + S - 1 < nk) {
      const int st = (kt + S - 1) % S;
      oa.issue(smem + st * STAGE, kt + S - 1, wave);
#pragma unroll
      for (int c = 0; c < NCH; ++c) ob[c].issue(smem + st * STAGE + OA::BYTES + c * OB::BYTES, kt + S - 1, wave);
    }
    const char* la = smem + (kt % S) * STAGE;
    const char* lb = la + OA::BYTES;
    TrFrag tb[2][FN];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int j = 0; j < FN; ++j) tb[s][j] = frag_t_half(lb, cw + j * 16, s, lane);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 af[FM], bfr[FN];
      if (s == 0) {
        constexpr int LATER0 = 2 * FN;
        constexpr int LATER = LATER0 < 16 ? LATER0 : 15;
#pragma unroll
        for (int j = 0; j < FN; ++j) bfr[j] = frag_t_fence_n<LATER>(tb[0][j]);
      } else {
#pragma unroll
        for (int j = 0; j < FN; ++j) bfr[j] = frag_t_fence_n<0>(tb[1][j]);
      }
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = frag_k_perm(la, i * 16 + li, s, g);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma16(bfr[j], af[i], acc[i][j]);
    }
  }

  // ---- epilogue, pass 1: x_hat, dxh, row partials, dgamma / dbeta lane partials
  bf16x4 xv[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
      xv[i][j] = *reinterpret_cast<const bf16x4*>(xin + (size_t)rowc[i] * D + cw + 16 * j + 4 * g);
  float cp[V];  // [dgamma: FN x 4 | dbeta: FN x 4]
#pragma unroll
  for (int k = 0; k < V; ++k) cp[k] = 0.f;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const bool live = m0 + i * 16 + li < p.M;
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float dv = live ? acc[i][j][r] : 0.f;
        const float xh = (bf2f(xv[i][j][r]) - mu[i]) * rs[i];
        const float dxh = dv * gm[j][r];
        s1 += dxh;
        s2 += dxh * xh;
        cp[4 * j + r] += dv * xh;
        cp[4 * FN + 4 * j + r] += dv;
      }
    s1 = psum32(psum16(s1));
    s2 = psum32(psum16(s2));
    if (g == 0) rred[wave][i * 16 + li] = make_float2(s1, s2);
  }
  __syncthreads();
  float c1[FM], c2[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float2 t = rred[w][i * 16 + li];
      a += t.x;
      b += t.y;
    }
    c1[i] = a * (1.0f / D);
    c2[i] = b * (1.0f / D);
  }

  // ---- pass 2: g_out, y_out, gy
  const uint32_t salt_drop = p.thr_drop ? site_salt_v((uint64_t)rng0, (uint64_t)rng1, p.site_drop) : 0u;
  const uint32_t salt_dp = p.thr_dp ? site_salt_v((uint64_t)rng0, (uint64_t)rng1, p.site_dp) : 0u;
  f32x4 bt[FN];
  if (p.y_out) {
#pragma unroll
    for (int j = 0; j < FN; ++j) bt[j] = *reinterpret_cast<const f32x4*>(p.beta + cw + 16 * j + 4 * g);
  }
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int row = m0 + i * 16 + li;
    f32x4 res[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j)
      res[j] = p.g_res ? *reinterpret_cast<const f32x4*>(p.g_res + (size_t)rowc[i] * D + cw + 16 * j + 4 * g)
                       : f32x4{0.f, 0.f, 0.f, 0.f};
    if (row >= p.M) continue;
    float dpsc = 1.f;
    if (p.gy && p.thr_dp) dpsc = dropout_keep(salt_dp, (uint32_t)(row / p.tokens), p.thr_dp) ? p.sc_dp : 0.f;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int col = cw + 16 * j + 4 * g;
      const size_t off = (size_t)row * D + col;
      f32x4 o;
      float xh[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        xh[r] = (bf2f(xv[i][j][r]) - mu[i]) * rs[i];
        const float dxh = acc[i][j][r] * gm[j][r];
        o[r] = (dxh - c1[i] - xh[r] * c2[i]) * rs[i] + res[j][r];
      }
      *reinterpret_cast<f32x4*>(p.g_out + off) = o;
      if (p.y_out) {
        bf16x4 yv;
#pragma unroll
        for (int r = 0; r < 4; ++r) yv[r] = f2bf(xh[r] * gm[j][r] + bt[j][r]);
        *reinterpret_cast<bf16x4*>(y_out + off) = yv;
      }
      if (p.gy) {
        bool k[4] = {true, true, true, true};
        if (p.thr_drop) dropout_keep4(salt_drop, (uint32_t)off, p.thr_drop, k);
        bf16x4 hv;
#pragma unroll
        for (int r = 0; r < 4; ++r) hv[r] = f2bf(k[r] ? o[r] * dpsc * (p.thr_drop ? p.sc_drop : 1.f) : 0.f);
        *reinterpret_cast<bf16x4*>(gy_out + off) = hv;
      }
    }
  }

  // ---- dgamma || dbeta: reduce-scatter over the 16 lanes of a column group, then one
  // atomic per column per workgroup into replica blockIdx % LN_REPLICAS
  float* rep = p.ws + (size_t)(blockIdx.x % p.replicas) * 2 * D;
  float h1[V / 2], h2[V / 4], h3[V / 8], h4[V / 16];
  rs_step<V / 2, 8>(cp, h1, li);
  rs_step<V / 4, 4>(h1, h2, li);
  rs_step<V / 8, 2>(h2, h3, li);
  rs_step<V / 16, 1>(h3, h4, li);
  // lane li holds partial indices [li * V/16, (li+1) * V/16) of cp, summed over the 16 lanes
#pragma unroll
  for (int k = 0; k < V / 16; ++k) {
    const int idx = li * (V / 16) + k;
    const int q = idx / (4 * FN), jr = idx % (4 * FN);
    const int col = cw + 16 * (jr >> 2) + 4 * g + (jr & 3);
    atomicAdd(rep + q * D + col, h4[k]);
  }
}

// explicit instantiations (hipcc drops the host stubs of kernel templates referenced
// only through a static initializer's lambda)
template __global__ void gemm_lnbwd_kernel<64, 6, 2>(LnBwdParams);
template __global__ void gemm_lnbwd_kernel<32, 6, 3>(LnBwdParams);
template __global__ void gemm_lnbwd_kernel<64, 4, 3>(LnBwdParams);
template __global__ void gemm_lnbwd_kernel<32, 4, 3>(LnBwdParams);

template <int BM, int NCH, int S>
static void launch_lnbwd(const LnBwdParams& p, hipStream_t stream) {
  constexpr int stage = BM * 128 + NCH * 64 * 128;
  static_assert(S * stage <= 160 * 1024, "LDS ring exceeds 160 KiB");
  const int nwg = (p.M + BM - 1) / BM;
  static const bool attr = [] {  // dynamic LDS above 64 KiB: opt in once per instantiation
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_lnbwd_kernel<BM, NCH, S>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, S * stage);
    return true;
  }();
  (void)attr;
  hipLaunchKernelGGL((gemm_lnbwd_kernel<BM, NCH, S>), dim3(nwg), dim3(256), S * stage, stream, p);
}

}  // namespace dc

using namespace dc;

bool gemm_lnbwd_supported(int D, int K) { return (D == 256 || D == 384) && K % 64 == 0 && K >= 64; }

void gemm_lnbwd_launch(LnBwdParams p, int D, double p_drop, double p_dp, hipStream_t stream) {
  if (!gemm_lnbwd_supported(D, p.K)) throw std::invalid_argument("gemm_lnbwd: unsupported D / K");
  p.thr_drop = drop_threshold_host(p_drop);
  p.thr_dp = drop_threshold_host(p_dp);
  p.sc_drop = p_drop > 0 ? 1.f / (1.f - (float)p_drop) : 1.f;
  p.sc_dp = p_dp > 0 ? 1.f / (1.f - (float)p_dp) : 1.f;
  // large M: 64-row tiles (2-stage ring: 6 x 8 KiB of W per stage), small M: 32-row
  // tiles, 3 stages -- either way the grid is about one round of the 256 CUs or more
  const bool big = p.M >= 8192;
  if (D == 384) {
    if (big) launch_lnbwd<64, 6, 2>(p, stream);
    else launch_lnbwd<32, 6, 3>(p, stream);
  } else {
    if (big) launch_lnbwd<64, 4, 3>(p, stream);
    else launch_lnbwd<32, 4, 3>(p, stream);
  }
}
