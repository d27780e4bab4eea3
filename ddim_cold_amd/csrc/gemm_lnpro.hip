// LayerNorm backward as the PROLOGUE of the input-gradient GEMM that consumes its
// output (gfx950).
//
//   LN backward of dl (bf16 [M][D]) at the LN input x (bf16 copy), saved mean / rstd:
//     x_hat = (x - mu) rstd,  dxh = dl gamma,
//     g_out = rstd (dxh - mean(dxh) - x_hat mean(dxh x_hat)) + g_res     (fp32)
//     gy    = bf16(g_out * dropout mask * drop-path scale)
//     y_out = bf16(x_hat gamma + beta)                                    (re-emitted LN output)
//     dgamma += sum_rows dl x_hat, dbeta += sum_rows dl                   (replica workspace)
//   then C = gy W with the consumer's epilogue (bf16: the attention-output gradient of
//   the proj input gradient; DGELU: the fc2 input gradient through GELU' and dropout) --
//   the same outputs as ln_bwd_kernel (layernorm.hip) followed by the dgrad GEMM.  In
//   the pre-norm backward every LayerNorm except block 0's norm1 feeds such a GEMM with
//   K = D (ViT.py:124-137, mlp_ratio 1): the final norm and norm1 of block i feed block
//   i-1's fc2 input gradient, norm2 feeds the proj input gradient.
//
// Why the consumer side: the LayerNorm needs whole rows, and the consumer's reduction
// dimension IS the row (K = D), so a workgroup with BM rows already reads whole rows of
// its A operand.  It computes them (LN backward of its BM rows) into an LDS-resident A
// panel instead of DMA-ing gy, then streams only W through the LDS-DMA ring.  The
// producer side (gemm_lnbwd.hip: full-row output tiles of the previous GEMM) streams the
// whole weight through every workgroup and measured slower; here the row panel is
// recomputed by each of the N/BN column workgroups (D/64 = 6: ~2 us of loads and VALU),
// the workgroups of column 0 write g_out / gy / y_out and the dgamma / dbeta partials,
// and one launch (~6 us on ViT-tiny) per LayerNorm disappears.
//
// Layout: 32 x 64 output tiles, 4 waves (2 x 2 of 16 x 32), swapped accumulators
// (mfma(B, A) = C^T) for the vector epilogues of gemm_epi.h.  The A panel is D/64
// images of [32 rows][64 k] in the DMA swizzle (chunk' = chunk ^ ((row >> 1) & 7)),
// read with frag_k_perm like a DMA'd A stage.
#include "common.h"
#include "kernels.h"
#include "gemm_common.h"
#include "gemm_epi.h"
#include <stdexcept>

namespace dc {

template <int D, int EPI, int S>
__global__ __launch_bounds__(256) void gemm_lnpro_kernel(GemmParams p, LnProParams q) {
  constexpr int BM = 32, BN = 64, WN = 2, TM = 16, TN = 32, FM = TM / 16, FN = TN / 16;
  constexpr int KT = D / 64;
  constexpr int APANEL = KT * BM * 128;
  using OB = DmaOperand<BN, true, 4>;
  constexpr int LPT = OB::PER_WAVE;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* apanel = smem;
  char* ring = smem + APANEL;

  const int tiles_n = (p.N + BN - 1) / BN;
  const int tiles_m = (p.M + BM - 1) / BM;
  const int bid = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int tm = bid / tiles_n, tn = bid - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int g = lane >> 4, li = lane & 15;

#ifdef DDIM_COLD_GEMM_STAMPS
  uint32_t st_t0 = 0, st_t1 = 0, st_t2 = 0;
  if (p.stamps) st_t0 = stamp_now();
#endif
  // W stages first: they land while the LayerNorm prologue runs
  OB ob;
  ob.init(p.B, p.ldb, p.K, n0, wave, lane);
#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (s < KT) ob.issue(ring + s * OB::BYTES, s, wave);
  VecEpi<EPI, FM, FN, false, true> ep;
  ep.prefetch(p, m0 + wm * TM, n0 + wn * TN, g, li);

  // ---------------------------------------------------------------- LayerNorm backward
  // 16 threads per row, two passes of 16 rows; thread (rr, sub) owns the 16-B chunks
  // ch = sub + 16 v (v < D / 128) of its row: chunk ch is chunk ch & 7 of k-tile ch >> 3
  {
    constexpr int NV = D / 128;  // chunks per thread per row
    const int sub = threadIdx.x & 15, rr = threadIdx.x >> 4;
    const bool col0 = tn == 0;  // this workgroup writes the LayerNorm outputs
    const uint64_t rng0 = (uint64_t)q.rng[0], rng1 = (uint64_t)q.rng[1];
    // gamma / beta through LDS: loaded from global per chunk, the compiler hoisted all
    // of them (and the residual rows) to the top -- 343 VGPRs
    __shared__ __attribute__((aligned(16))) float lgam[D], lbet[D];
    __shared__ __attribute__((aligned(16))) float lred[4][2 * D];  // dgamma || dbeta per wave
    // staged behind the first pass's row loads (one memory round trip for both)
    auto stage_gamma = [&]() {
      for (int i = threadIdx.x; i < D / 4; i += 256) {
        reinterpret_cast<f32x4*>(lgam)[i] = reinterpret_cast<const f32x4*>(q.gamma)[i];
        reinterpret_cast<f32x4*>(lbet)[i] =
            q.beta ? reinterpret_cast<const f32x4*>(q.beta)[i] : f32x4{0.f, 0.f, 0.f, 0.f};
      }
      __syncthreads();
    };
    const uint32_t salt_drop = q.thr_drop ? site_salt_v(rng0, rng1, q.site_drop) : 0u;
    const uint32_t salt_dp = q.thr_dp ? site_salt_v(rng0, rng1, q.site_dp) : 0u;
    auto unpack = [](const u32x4& w, float (&f)[8]) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        f[2 * k] = __uint_as_float(w[k] << 16);
        f[2 * k + 1] = __uint_as_float(w[k] & 0xFFFF0000u);
      }
    };
    float dgacc[NV][8], dbacc[NV][8];  // dgamma / dbeta partials of this thread's columns
#pragma unroll
    for (int v = 0; v < NV; ++v)
#pragma unroll
      for (int k = 0; k < 8; ++k) dgacc[v][k] = dbacc[v][k] = 0.f;
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      const int r = rr + 16 * pass;
      const int m = m0 + r;
      const bool live = m < p.M;
      const int mc = live ? m : p.M - 1;
      const bf16* dlr = reinterpret_cast<const bf16*>(q.dl) + (size_t)mc * D;
      const bf16* xr = reinterpret_cast<const bf16*>(q.x) + (size_t)mc * D;
      // residual gradient rows: unconditional (g_out's own rows when there is none; the
      // value is dropped) -- a load under `g_res ?` became a phi that waited on the spot
      const float* grr = (q.g_res ? q.g_res : q.g_out) + (size_t)mc * D;
      const float mu = q.mean[mc], rs = q.rstd[mc];
      u32x4 dlv[NV], xv[NV];
      f32x4 gres[NV][2];
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const int c = 8 * (sub + 16 * v);
        dlv[v] = *reinterpret_cast<const u32x4*>(dlr + c);
        xv[v] = *reinterpret_cast<const u32x4*>(xr + c);
        gres[v][0] = *reinterpret_cast<const f32x4*>(grr + c);
        gres[v][1] = *reinterpret_cast<const f32x4*>(grr + c + 4);
      }
      if (pass == 0) stage_gamma();
      // pass A: row sums of dxh and dxh x_hat (16 lanes), column partials
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const int c = 8 * (sub + 16 * v);
        const f32x4 ga = *reinterpret_cast<const f32x4*>(lgam + c);
        const f32x4 gb = *reinterpret_cast<const f32x4*>(lgam + c + 4);
        float dl[8], xx[8];
        unpack(dlv[v], dl);
        unpack(xv[v], xx);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float gm = k < 4 ? ga[k] : gb[k - 4];
          const float xh = (xx[k] - mu) * rs;
          const float dx = live ? dl[k] : 0.f;
          s1 += dx * gm;
          s2 += dx * gm * xh;
          dgacc[v][k] += dx * xh;
          dbacc[v][k] += dx;
        }
      }
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        s1 += __shfl_xor(s1, o, 64);
        s2 += __shfl_xor(s2, o, 64);
      }
      const float c1 = s1 * (1.0f / D), c2 = s2 * (1.0f / D);
      float dpsc = 1.f;
      if (q.thr_dp) dpsc = dropout_keep(salt_dp, (uint32_t)(mc / q.tokens), q.thr_dp) ? q.sc_dp : 0.f;
      // pass B: g_out, gy (LDS panel; column-0 workgroups also global), y_out
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const int ch = sub + 16 * v, c = 8 * ch;
        const f32x4 ga = *reinterpret_cast<const f32x4*>(lgam + c);
        const f32x4 gb = *reinterpret_cast<const f32x4*>(lgam + c + 4);
        float dl[8], xx[8], o[8], xh[8];
        unpack(dlv[v], dl);
        unpack(xv[v], xx);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float gm = k < 4 ? ga[k] : gb[k - 4];
          xh[k] = (xx[k] - mu) * rs;
          const float res = q.g_res ? (k < 4 ? gres[v][0][k] : gres[v][1][k - 4]) : 0.f;
          o[k] = (dl[k] * gm - c1 - xh[k] * c2) * rs + res;
        }
        bf16x8 h;
#pragma unroll
        for (int k = 0; k < 8; k += 2) {
          float a = o[k] * dpsc, b2 = o[k + 1] * dpsc;
          if (q.thr_drop) {
            const uint32_t hh = drop_hash(salt_drop, (uint32_t)(((size_t)mc * D + c + k) >> 1));
            a = (hh & 0xFFFFu) >= q.thr_drop ? a * q.sc_drop : 0.f;
            b2 = (hh >> 16) >= q.thr_drop ? b2 * q.sc_drop : 0.f;
          }
          h[k] = f2bf(live ? a : 0.f);
          h[k + 1] = f2bf(live ? b2 : 0.f);
        }
        *reinterpret_cast<bf16x8*>(apanel + (ch >> 3) * (BM * 128) + r * 128 + 16 * ((ch & 7) ^ swz(r))) = h;
        if (col0 && live) {
          float* go = q.g_out + (size_t)m * D + c;
          *reinterpret_cast<f32x4*>(go) = f32x4{o[0], o[1], o[2], o[3]};
          *reinterpret_cast<f32x4*>(go + 4) = f32x4{o[4], o[5], o[6], o[7]};
          *reinterpret_cast<bf16x8*>(reinterpret_cast<bf16*>(q.gy) + (size_t)m * D + c) = h;
          if (q.y_out) {
            const f32x4 ba = *reinterpret_cast<const f32x4*>(lbet + c);
            const f32x4 bb = *reinterpret_cast<const f32x4*>(lbet + c + 4);
            bf16x8 y;
#pragma unroll
            for (int k = 0; k < 8; ++k) y[k] = f2bf(xh[k] * (k < 4 ? ga[k] : gb[k - 4]) + (k < 4 ? ba[k] : bb[k - 4]));
            *reinterpret_cast<bf16x8*>(reinterpret_cast<bf16*>(q.y_out) + (size_t)m * D + c) = y;
          }
        }
      }
    }
    // dgamma / dbeta of the column-0 workgroups: the wave's 4 rows x 2 passes summed
    // (lanes 16 apart), the 4 waves through LDS, then ONE atomic per column per workgroup
    // into replica blockIdx % replicas (one per column per wave: the waves' atomics on
    // the same addresses serialised, ~8 us of the column-0 workgroups)
    if (col0) {
#pragma unroll
      for (int v = 0; v < NV; ++v)
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          float a = dgacc[v][k], b2 = dbacc[v][k];
          a += __shfl_xor(a, 16, 64);
          a += __shfl_xor(a, 32, 64);
          b2 += __shfl_xor(b2, 16, 64);
          b2 += __shfl_xor(b2, 32, 64);
          if (lane < 16) {
            const int c = 8 * (sub + 16 * v) + k;
            lred[wave][c] = a;
            lred[wave][D + c] = b2;
          }
        }
      __syncthreads();
      float* rep = q.ws + (size_t)(blockIdx.x % q.replicas) * 2 * D;
      for (int c = threadIdx.x; c < 2 * D; c += 256)
        atomicAdd(rep + c, (lred[0][c] + lred[1][c]) + (lred[2][c] + lred[3][c]));
    }
  }
  __syncthreads();  // the A panel is complete
#ifdef DDIM_COLD_GEMM_STAMPS
  if (p.stamps) st_t1 = stamp_now();
#endif

  // ---------------------------------------------------------------- main loop (W only)
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int kt = 0; kt < KT; ++kt) {
    const int rem = min(S - 2, KT - 1 - kt);
    vm_wait_rem<LPT>(rem);
    raw_barrier();
    if (kt + S - 1 < KT) ob.issue(ring + ((kt + S - 1) % S) * OB::BYTES, kt + S - 1, wave);
    const char* la = apanel + kt * (BM * 128);
    const char* lb = ring + (kt % S) * OB::BYTES;
    TrFrag tb[2][FN];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int j = 0; j < FN; ++j) tb[s][j] = frag_t_half(lb, wn * TN + j * 16, s, lane);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = s == 0 ? frag_t_fence_n<2 * FN>(tb[0][j]) : frag_t_fence_n<0>(tb[1][j]);
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = frag_k_perm(la, wm * TM + i * 16 + li, s, g);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma16(bfr[j], af[i], acc[i][j]);
    }
  }
#ifdef DDIM_COLD_GEMM_STAMPS
  if (p.stamps) st_t2 = stamp_now();
#endif
  ep.finish(p, acc, li);
#ifdef DDIM_COLD_GEMM_STAMPS
  if (p.stamps) {  // same layout as gemm_dma_body: start, prologue done, main loop done, end
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t* o = p.stamps + (size_t)blockIdx.x * GEMM_STAMP_WORDS;
      o[0] = st_t0; o[1] = st_t1; o[2] = st_t2; o[3] = stamp_now();
      o[4] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
      o[5] = __builtin_amdgcn_s_getreg((31 << 11) | 20);
    }
  }
#endif
}

template <int D, int EPI>
static void launch_lnpro(const GemmParams& p, const LnProParams& q, hipStream_t stream) {
  constexpr int S = 3;
  constexpr int lds = (D / 64) * 32 * 128 + S * 64 * 128;
  const int tiles = ((p.M + 31) / 32) * ((p.N + 63) / 64);
  hipLaunchKernelGGL((gemm_lnpro_kernel<D, EPI, S>), dim3(tiles), dim3(256), lds, stream, p, q);
}

template __global__ void gemm_lnpro_kernel<384, EPI_BF16, 3>(GemmParams, LnProParams);
template __global__ void gemm_lnpro_kernel<384, EPI_DGELU, 3>(GemmParams, LnProParams);
template __global__ void gemm_lnpro_kernel<256, EPI_BF16, 3>(GemmParams, LnProParams);
template __global__ void gemm_lnpro_kernel<256, EPI_DGELU, 3>(GemmParams, LnProParams);

}  // namespace dc

using namespace dc;

bool gemm_lnpro_supported(int D, int K, int N) { return (D == 384 || D == 256) && K == D && N % 64 == 0; }

void gemm_lnpro_launch(const GemmArgs& a, int epi, LnProParams q, double p_drop, double p_dp, hipStream_t stream) {
  if (!gemm_lnpro_supported(a.K, a.K, a.N)) throw std::invalid_argument("gemm_lnpro: unsupported shape");
  q.thr_drop = drop_threshold_host(p_drop);
  q.thr_dp = drop_threshold_host(p_dp);
  q.sc_drop = p_drop > 0 ? 1.f / (1.f - (float)p_drop) : 1.f;
  q.sc_dp = p_dp > 0 ? 1.f / (1.f - (float)p_dp) : 1.f;
  GemmParams p = gemm_params_from_args(a);
  if (epi == EPI_BF16) {
    if (a.K == 384) launch_lnpro<384, EPI_BF16>(p, q, stream);
    else launch_lnpro<256, EPI_BF16>(p, q, stream);
  } else if (epi == EPI_DGELU) {
    if (a.K == 384) launch_lnpro<384, EPI_DGELU>(p, q, stream);
    else launch_lnpro<256, EPI_DGELU>(p, q, stream);
  } else {
    throw std::invalid_argument("gemm_lnpro: epilogue must be bf16 or DGELU");
  }
}
