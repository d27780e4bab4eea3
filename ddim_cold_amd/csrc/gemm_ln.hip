// Row-panel GEMM with a fused residual + LayerNorm epilogue (gfx950).
//
//   x_out = res + DropPath(Dropout(A W^T + bias))        (fp32 residual stream)
//   ln    = LayerNorm(x_out) * gamma + beta               (bf16, next GEMM's A)
//   mean, rstd per row                                    (saved for backward)
//
// This is the pre-norm transformer seam `x += branch(...); h = LN(x)`
// (ViT.py:133-137 with the next LayerNorm, VIT:124/128/182) as ONE launch: the
// proj GEMM carries LN2 and the fc2 GEMM carries the next block's LN1 (or the
// final norm), removing every stand-alone LayerNorm-forward kernel after the
// embedding and one HBM round trip of the residual stream per seam.
//
// LayerNorm needs whole rows, so a workgroup owns a BM-row panel and ALL D
// output columns (4 waves x D/4 columns).  The weight panel (D x K, k
// contiguous) streams through an LDS-DMA ring shared by the 4 waves (every
// workgroup reads the same weights: L2-resident after the first touch); the
// row statistics are reduced lane-group -> wave (shuffles) -> workgroup (LDS),
// two-pass (mean, then centred variance) like nn.LayerNorm.
#include "common.h"
#include "kernels.h"
#include "gemm_common.h"
#include <cstdlib>

namespace dc {

struct GemmLnParams {
  const bf16* A;
  const bf16* W;
  int M, K;
  const float* bias;
  const float* res;
  float* x_out;
  const float* gamma;
  const float* beta;
  bf16* ln_out;
  float* mean;
  float* rstd;
  float eps;
  int tokens;
  const int64_t* rng;
  int site_drop;
  uint32_t thr_drop;
  float scale_drop;
  int site_dp;
  uint32_t thr_dp;
  float scale_dp;
  int debug;  // profiling aid: 1 = skip the epilogue, 2 = skip the main loop
};

template <int BM, int D, int S>
__global__ __launch_bounds__(256) void gemm_resid_ln_kernel(GemmLnParams p) {
  constexpr int TN = D / 4, FM = BM / 16, FN = TN / 16;
  using OA = DmaOperand<BM, false>;
  using OB = DmaOperand<D, false>;
  static_assert(OA::PER_WAVE >= 1 && OB::PER_WAVE >= 1, "panel too small for the 4-wave DMA split");
  constexpr int STAGE = OA::BYTES + OB::BYTES;
  constexpr int LPT = OA::PER_WAVE + OB::PER_WAVE;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ float red[4][BM];

  const int m0 = xcd_remap(blockIdx.x, gridDim.x) * BM;
  const int nk = p.K / BK;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, li = lane & 15;

  OA oa;
  OB ob;
  oa.init(p.A, p.K, p.M, m0, wave, lane);
  ob.init(p.W, p.K, D, 0, wave, lane);

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (s < nk) {
      oa.issue(smem + s * STAGE, s, wave);
      ob.issue(smem + s * STAGE + OA::BYTES, s, wave);
    }
  for (int kt = 0; kt < (p.debug == 2 ? 0 : nk); ++kt) {
    vm_wait_rem<LPT>(min(S - 2, nk - 1 - kt));
    raw_barrier();
    if (kt + S - 1 < nk) {
      const int st = (kt + S - 1) % S;
      oa.issue(smem + st * STAGE, kt + S - 1, wave);
      ob.issue(smem + st * STAGE + OA::BYTES, kt + S - 1, wave);
    }
    const char* la = smem + (kt % S) * STAGE;
    const char* lb = la + OA::BYTES;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = frag_k(la, i * 16 + li, s, g);
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = frag_k(lb, wave * TN + j * 16 + li, s, g);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    }
  }

  if (p.debug == 1) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) t += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    if (t == 1234.5f) p.x_out[0] = t;
    return;
  }
  // ---- epilogue phase 1: every global load (bias / gamma / beta per column, residual per element)
  float bcol[FN], gcol[FN], becol[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = wave * TN + j * 16 + li;
    bcol[j] = p.bias[n];
    gcol[j] = p.gamma[n];
    becol[j] = p.beta[n];
  }
  float xv[FM][FN][4];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = min(m0 + i * 16 + 4 * g + r, p.M - 1);
#pragma unroll
      for (int j = 0; j < FN; ++j) xv[i][j][r] = p.res[(size_t)m * D + wave * TN + j * 16 + li];
    }
  const uint32_t salt_drop = p.thr_drop ? site_salt(p.rng, p.site_drop) : 0u;
  const uint32_t salt_dp = p.thr_dp ? site_salt(p.rng, p.site_dp) : 0u;

  // ---- phase 2: residual update (+ row sums)
  float rsum[FM][4];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + i * 16 + 4 * g + r;
      const bool keep_row = p.thr_dp ? dropout_keep(salt_dp, (uint32_t)(m / p.tokens), p.thr_dp) : true;
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = wave * TN + j * 16 + li;
        float v = acc[i][j][r] + bcol[j];
        if (p.thr_drop) v = dropout_keep(salt_drop, (uint32_t)(m * D + n), p.thr_drop) ? v * p.scale_drop : 0.f;
        if (p.thr_dp) v = keep_row ? v * p.scale_dp : 0.f;
        const float x = xv[i][j][r] + v;
        xv[i][j][r] = x;
        s += x;
        if (m < p.M) p.x_out[(size_t)m * D + n] = x;
      }
      rsum[i][r] = s;
    }
  // ---- row mean: 16-lane group (columns li) -> LDS across the 4 waves
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float s = rsum[i][r];
      s += __shfl_xor(s, 1, 64);
      s += __shfl_xor(s, 2, 64);
      s += __shfl_xor(s, 4, 64);
      s += __shfl_xor(s, 8, 64);
      if (li == 0) red[wave][i * 16 + 4 * g + r] = s;
    }
  __syncthreads();
  float mu[FM][4];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = i * 16 + 4 * g + r;
      mu[i][r] = (red[0][row] + red[1][row] + red[2][row] + red[3][row]) * (1.0f / D);
    }
  __syncthreads();
  // ---- centred variance
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float q = 0.f;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const float d = xv[i][j][r] - mu[i][r];
        q += d * d;
      }
      q += __shfl_xor(q, 1, 64);
      q += __shfl_xor(q, 2, 64);
      q += __shfl_xor(q, 4, 64);
      q += __shfl_xor(q, 8, 64);
      if (li == 0) red[wave][i * 16 + 4 * g + r] = q;
    }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = i * 16 + 4 * g + r;
      const int m = m0 + row;
      const float var = (red[0][row] + red[1][row] + red[2][row] + red[3][row]) * (1.0f / D);
      const float rs = rsqrtf(var + p.eps);
      if (m < p.M) {
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int n = wave * TN + j * 16 + li;
          p.ln_out[(size_t)m * D + n] = f2bf((xv[i][j][r] - mu[i][r]) * rs * gcol[j] + becol[j]);
        }
        if (wave == 0 && li == 0) {
          p.mean[m] = mu[i][r];
          p.rstd[m] = rs;
        }
      }
    }
}

template <int BM, int D, int S>
static void launch_ln(const GemmLnParams& p, hipStream_t stream) {
  constexpr int lds = S * (BM * 128 + D * 128);
  static_assert(lds + 4 * BM * 4 <= 160 * 1024, "LDS budget");
  static bool attr = [] {  // > 64 KiB of dynamic LDS must be opted into per kernel
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_resid_ln_kernel<BM, D, S>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, lds) == hipSuccess;
  }();
  (void)attr;
  hipLaunchKernelGGL((gemm_resid_ln_kernel<BM, D, S>), dim3((p.M + BM - 1) / BM), dim3(256), lds, stream, p);
}

#define DC_INST_LN(BM, D, S) template __global__ void gemm_resid_ln_kernel<BM, D, S>(GemmLnParams);
DC_INST_LN(32, 256, 4)
DC_INST_LN(32, 384, 3)
DC_INST_LN(32, 512, 2)
DC_INST_LN(64, 256, 3)
DC_INST_LN(64, 384, 2)
DC_INST_LN(64, 512, 2)

}  // namespace dc

using namespace dc;

bool gemm_resid_ln_supported(int D, int K) { return (D == 256 || D == 384 || D == 512) && K % 64 == 0; }

void gemm_resid_ln(const GemmLnArgs& a, hipStream_t stream) {
  GemmLnParams p{};
  p.A = reinterpret_cast<const bf16*>(a.A);
  p.W = reinterpret_cast<const bf16*>(a.W);
  p.M = a.M; p.K = a.K;
  p.bias = a.bias; p.res = a.res; p.x_out = a.x_out;
  p.gamma = a.gamma; p.beta = a.beta;
  p.ln_out = reinterpret_cast<bf16*>(a.ln_out);
  p.mean = a.mean; p.rstd = a.rstd; p.eps = a.eps;
  p.tokens = a.tokens; p.rng = a.rng;
  p.site_drop = a.site_drop;
  p.thr_drop = drop_threshold_host(a.p_drop);
  p.scale_drop = a.p_drop > 0 ? 1.f / (1.f - (float)a.p_drop) : 1.f;
  p.site_dp = a.site_dp;
  p.thr_dp = drop_threshold_host(a.p_dp);
  p.scale_dp = a.p_dp > 0 ? 1.f / (1.f - (float)a.p_dp) : 1.f;
  static const int dbg = [] {
    const char* e = getenv("DDIM_COLD_LN_GEMM_DEBUG");
    return e ? atoi(e) : 0;
  }();
  p.debug = dbg;
  if (!gemm_resid_ln_supported(a.D, a.K)) throw std::runtime_error("gemm_resid_ln: unsupported D / K");
  const bool wide = a.bm == 64;
  switch (a.D) {
    case 256: wide ? launch_ln<64, 256, 3>(p, stream) : launch_ln<32, 256, 4>(p, stream); break;
    case 384: wide ? launch_ln<64, 384, 2>(p, stream) : launch_ln<32, 384, 3>(p, stream); break;
    default: wide ? launch_ln<64, 512, 2>(p, stream) : launch_ln<32, 512, 2>(p, stream); break;
  }
}
