// GEMM parameter block and the fused epilogue family (bias, LayerNorm fold
// consumer/producer, QKV head-major scatter, residual + dropout + drop-path,
// GELU, head / unpatchify / loss / DDIM update, patch embedding, gradient
// accumulate), shared by every GEMM kernel of gemm.hip.
//
// ``PUB`` (VecEpi, off in every current kernel): the epilogue's hand-off outputs
// (bf16 residual copy, LayerNorm statistics, GELU output) are stored
// write-through (sc1) and the statistics it consumes are loaded sc1, for a
// consumer workgroup of the SAME launch on another XCD (MI355X_MICROARCH.md,
// inter-workgroup visibility).
#pragma once
#include "common.h"
#include "kernels.h"

namespace dc {

struct GemmParams {
  const bf16* A;
  const bf16* B;
  int M, N, K;
  int lda, ldb;
  void* C;
  int ldc;
  const float* bias;
  // epilogue extras
  const float* res;      // residual stream in (RESID)
  void* C2;              // second output (GELU: h)
  const bf16* aux;       // saved pre-activation u (DGELU)
  const int64_t* rng;    // {seed, step}
  int site_drop;
  uint32_t thr_drop;
  float scale_drop;
  int site_dp;
  uint32_t thr_dp;
  float scale_dp;
  int tokens;            // tokens per sample (N = P+1), or patches per sample (EMBED)
  int batch;
  int heads, hd;         // QKV scatter
  int chans, img_h, img_w, patch;  // HEAD
  const float* pos;      // EMBED
  const float* temb;
  const int64_t* tsteps;
  int emb_dim;
  int ktiles_per_split;
  const float* coef;     // HEAD mode 1: {sqrt a_t, sqrt(1-a_t), sqrt a_tk, sqrt(1-a_tk)} (device);
                         //   mode 4: one such row per sample ([batch][4])
  long long split_stride;  // EPI_F32: elements between the K-split output slices
  int head_mode;         // HEAD: 0 image, 1 fused DDIM step (res = x_t in, C = x_next, C2 = x0), 2 clamp,
                         //   3 training loss (res = target image, C2 = token-layout grad, loss_parts),
                         //   4 DDIM step with per-sample coefficients (img2img: a sample that has
                         //     not reached its start step has the row {0, 1, 0, 1}: x_next = x_t)
  float loss_beta;       // HEAD mode 3: smooth-L1 beta and 1/numel
  float loss_inv_n;
  float* loss_parts;     // HEAD mode 3: one loss partial per workgroup (gridDim.x entries)
  // LayerNorm fold (GemmArgs): consumer side
  const float* ln_st;
  const float* ln_c;
  float ln_eps;
  float* ln_mean;
  float* ln_rstd;
  // producer side
  float* st_out;
  bf16* xb_out;
  // sampler steps: HEAD modes 1/2 also store the new image in the patch-row layout
  // (bf16 [B*P][C*p*p], the next step's patch-embedding A operand: no patchify
  // launch); EMBED with cls_src also writes the cls rows (cls + pos[0] + temb[t])
  bf16* patch_out;
  const float* cls_src;
  int acc_store;  // EPI_ACC: the target is known to be zero -- store, don't read-add
  float* sq_parts;  // EPI_ACC: sum of squares of this workgroup's final outputs -> sq_parts[sq_slot]
  int sq_slot;
  uint32_t tok_magic;  // floor(2^32 / tokens) (divmagic: row -> sample without a division)
  float ln_invd;       // 1 / K (LayerNorm fold consumer: D = K)
  uint32_t* stamps;    // phase profiling (gemm_set_stamps): per workgroup GEMM_STAMP_WORDS words
};

// the kernel parameter block of a host GemmArgs (gemm.hip base_params)
GemmParams gemm_params_from_args(const GemmArgs& a);

// Phase stamps of the LDS-DMA GEMM (tools/ub_gemm_stamps.py): s_memrealtime (100 MHz)
// at workgroup start, first operand stage ready, main loop done, epilogue done, plus
// the HW_ID / XCC_ID registers (which CU ran it).  Thread 0 stores them with vector
// stores.  Compiled only with -DDDIM_COLD_GEMM_STAMPS (DDIM_COLD_HIPFLAGS at build
// time): even untaken, the stamp branches cost the ViT-tiny step 1.5-2 % in a same-box
// A/B (profiles/stamps_cost_r5.txt) -- they changed the main loop's code.
constexpr int GEMM_STAMP_WORDS = 6;

static __device__ const int64_t kEpiNoRng[2] = {0, 0};  // rng words of GEMMs without dropout
__device__ __forceinline__ uint32_t stamp_now() { return (uint32_t)__builtin_amdgcn_s_memrealtime(); }


// Epilogue in two phases: (1) every global load the epilogue needs (bias per
// column, residual / saved pre-activation / pos+time embedding per element) is
// issued for the whole fragment tile, (2) compute + store.  Interleaving them
// per element serialises the tile on memory latency (the loads may alias the
// stores through GemmParams, so the compiler cannot hoist them).
// The epilogue is "load everything, then compute + store": interleaving per-element
// loads (bias / residual / saved pre-activation / embeddings, which may alias the
// stores through GemmParams) with stores serialises the tile on memory latency.
// Every output index is separable, idx = rowoff(m) + coloff(n), so the integer
// divisions (token -> sample, column -> head / pixel) are done once per row and
// once per column of the lane's fragment, not per element.
struct RowInfo {
  long long off;  // row part of the destination index (-1: skip row)
  int b;          // sample index (drop-path) / helper
};

template <int EPI>
__device__ __forceinline__ RowInfo epi_row(const GemmParams& p, int m) {
  RowInfo ri;
  ri.b = 0;
  if (EPI == EPI_QKV) {
    const int b = m / p.tokens, tok = m - b * p.tokens;
    ri.off = ((long long)b * p.heads * p.tokens + tok) * p.hd;
  } else if (EPI == EPI_RESID) {
    ri.off = (long long)m * p.N;
    ri.b = m / p.tokens;
  } else if (EPI == EPI_GELU || EPI == EPI_DGELU) {
    ri.off = (long long)m * p.N;
  } else if (EPI == EPI_HEAD) {
    const int b = m / p.tokens, tok = m - b * p.tokens;
    ri.b = b;  // sample (head mode 4: per-sample DDIM coefficients)
    if (tok == 0) {
      ri.off = -1;
    } else {
      const int P = p.patch, Wp = p.img_w / P;
      const int patch = tok - 1, hp = patch / Wp, wp = patch - hp * Wp;
      ri.off = (long long)b * p.chans * p.img_h * p.img_w + (long long)hp * P * p.img_w + wp * P;
    }
  } else if (EPI == EPI_EMBED) {
    const int Pn = p.tokens;
    const int b = m / Pn, patch = m - b * Pn;
    ri.off = ((long long)b * (Pn + 1) + patch + 1) * p.emb_dim;
    ri.b = b;
  } else {
    ri.off = (long long)m * p.ldc;
  }
  return ri;
}

template <int EPI>
__device__ __forceinline__ long long epi_col(const GemmParams& p, int n) {
  if (EPI == EPI_QKV) {
    const int D = p.heads * p.hd;
    const int s = n / D, rem = n - s * D;
    const int h = rem / p.hd, d = rem - h * p.hd;
    return (long long)s * p.batch * p.heads * p.tokens * p.hd + (long long)h * p.tokens * p.hd + d;
  }
  if (EPI == EPI_HEAD) {
    const int P = p.patch;
    const int c = n % p.chans, ab = n / p.chans, a = ab / P, bb = ab - a * P;
    return (long long)c * p.img_h * p.img_w + (long long)a * p.img_w + bb;
  }
  return n;
}

// ---- LayerNorm fold.  LN(x) W^T + b = rstd * (x (gamma o W)^T - mean * c) + (b + W beta)
// with c[n] = sum_k bf16(gamma_k W[n][k]) (ln_fold_prep in layernorm.hip), so the
// GEMM consuming a LayerNorm reads the raw residual stream (its bf16 copy) and
// the LayerNorm launch disappears.  The row statistics {sum x, sum x^2} come from
// the epilogue of the GEMM that PRODUCED x (residual / patch-embed epilogue:
// per-row partial sums over its columns, fp32 atomics).
template <int EPI>
struct FoldEpi {
  static constexpr bool CONSUMER =
      EPI == EPI_QKV || EPI == EPI_GELU || EPI == EPI_BF16 || EPI == EPI_F32 || EPI == EPI_HEAD ||
      EPI == EPI_HEADR || EPI == EPI_HEADL;
  static constexpr bool PRODUCER = EPI == EPI_RESID || EPI == EPI_EMBED;
};

// Row statistics layout: st[row][NP][2], NP = D / 32 slots; slot s holds
// {sum, sum^2} of the row's columns 32s..32s+31, written exactly once by the
// wave of the producing epilogue that owns those columns (no atomics, no
// zeroing: deterministic).  Consumers add the slots in a fixed butterfly order.
constexpr int LN_SLOT = 32;
constexpr int LN_MAX_SLOTS = 16;

// (mean, rstd) of a row from its {sum, sum^2} over D = K columns (1/K from the
// host; var + eps >= eps > 0, so the bare v_rsq needs no denormal fix-up)
__device__ __forceinline__ float2 ln_row_stats(const GemmParams& p, float2 st) {
  const float mu = st.x * p.ln_invd;
  const float var = fmaxf(st.y * p.ln_invd - mu * mu, 0.f);
  return make_float2(mu, __builtin_amdgcn_rsqf(var + p.ln_eps));
}

// m / d for 0 <= m < 2^31 with magic = floor(2^32 / d): the high product is q or
// q - 1, one compare fixes it (vs ~15 instructions of a division by a runtime d)
__device__ __forceinline__ int divmagic(int m, int d, uint32_t magic) {
  int q = (int)__umulhi((uint32_t)m, magic);
  if (m - q * d >= d) ++q;
  return q;
}

// Vector-epilogue destination index, 32-bit (the host checks every output has
// < 2^31 elements): row part and column part, separable as in epi_row / epi_col.
struct RowInfo32 {
  int off;  // -1: skip row
  int b;    // sample (drop-path / embeddings)
};
template <int EPI>
__device__ __forceinline__ RowInfo32 epi_row32(const GemmParams& p, int m) {
  RowInfo32 ri;
  ri.b = 0;
  if (EPI == EPI_QKV) {
    const int b = divmagic(m, p.tokens, p.tok_magic), tok = m - b * p.tokens;
    ri.off = (b * p.heads * p.tokens + tok) * p.hd;
  } else if (EPI == EPI_RESID) {
    ri.off = m * p.N;
    ri.b = p.thr_dp ? divmagic(m, p.tokens, p.tok_magic) : 0;  // drop-path sample (training only)
  } else if (EPI == EPI_GELU || EPI == EPI_DGELU) {
    ri.off = m * p.N;
  } else if (EPI == EPI_HEADL) {
    // gradient in the token layout (row m, cls rows included: zero); the target's
    // patch row is m - b - 1 (b = -1 marks a cls row)
    const int b = divmagic(m, p.tokens, p.tok_magic);
    ri.off = m * p.N;
    ri.b = m - b * p.tokens == 0 ? -1 : b;
  } else if (EPI == EPI_HEADR) {
    // token row m of sample b -> patch row b*P + tok - 1 = m - b - 1 (cls rows skipped)
    const int b = divmagic(m, p.tokens, p.tok_magic), tok = m - b * p.tokens;
    ri.off = tok == 0 ? -1 : (m - b - 1) * p.N;
    ri.b = b;
  } else if (EPI == EPI_EMBED) {
    const int b = divmagic(m, p.tokens, p.tok_magic);  // tokens = patches per sample here
    ri.off = (m + b + 1) * p.emb_dim;                  // (b * (P + 1) + patch + 1) * D
    ri.b = b;
  } else {
    ri.off = m * p.ldc;
  }
  return ri;
}

__device__ __forceinline__ float2 f2add(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
template <int MASK>
__device__ __forceinline__ float2 f2xor(float2 a) {
  return make_float2(__shfl_xor(a.x, MASK), __shfl_xor(a.y, MASK));
}

// destination token row of a producer epilogue row (statistics index)
template <int EPI>
__device__ __forceinline__ int fold_token_row(const GemmParams& p, int m) {
  if (EPI == EPI_EMBED) {
    const int b = m / p.tokens;
    return m + b + 1;  // b*(P+1) + patch + 1
  }
  return m;
}

// returns the stored fp32 value of the residual / embedding epilogues (LayerNorm statistics)
template <int EPI>
__device__ __forceinline__ float epilogue(const GemmParams& p, long long idx, int rb, float v, float pre,
                                          uint32_t salt_drop, uint32_t salt_dp, const f32x4& cf) {
  if (EPI == EPI_BF16) {
    reinterpret_cast<bf16*>(p.C)[idx + blockIdx.z * p.split_stride] = f2bf(v);
  } else if (EPI == EPI_F32) {
    reinterpret_cast<float*>(p.C)[idx + blockIdx.z * p.split_stride] = v;
  } else if (EPI == EPI_ATOMIC) {
    atomicAdd(reinterpret_cast<float*>(p.C) + idx, v);
  } else if (EPI == EPI_ACC) {
    reinterpret_cast<float*>(p.C)[idx] = pre + v;  // pre = old C (loaded in phase 1)
  } else if (EPI == EPI_QKV) {
    reinterpret_cast<bf16*>(p.C)[idx] = f2bf(v);
  } else if (EPI == EPI_RESID) {
    if (p.thr_drop) v = dropout_keep(salt_drop, (uint32_t)idx, p.thr_drop) ? v * p.scale_drop : 0.f;
    if (p.thr_dp) v = dropout_keep(salt_dp, (uint32_t)rb, p.thr_dp) ? v * p.scale_dp : 0.f;
    reinterpret_cast<float*>(p.C)[idx] = pre + v;
    return pre + v;
  } else if (EPI == EPI_GELU) {
    reinterpret_cast<bf16*>(p.C)[idx] = f2bf(v);
    float h = gelu_f(v);
    if (p.thr_drop) h = dropout_keep(salt_drop, (uint32_t)idx, p.thr_drop) ? h * p.scale_drop : 0.f;
    reinterpret_cast<bf16*>(p.C2)[idx] = f2bf(h);
  } else if (EPI == EPI_DGELU) {
    if (p.thr_drop) v = dropout_keep(salt_drop, (uint32_t)idx, p.thr_drop) ? v * p.scale_drop : 0.f;
    reinterpret_cast<bf16*>(p.C)[idx] = f2bf(v * gelu_grad_f(pre));
  } else if (EPI == EPI_HEAD) {
    if (p.head_mode == 0) {
      reinterpret_cast<float*>(p.C)[idx] = v;
    } else if (p.head_mode == 3) {
      // smooth-L1 vs the target pixel (`pre`), multi_gpu_trainer.py:124: the image
      // is never written; returns the element's loss / numel (the gradient is
      // stored by the caller in the token layout)
      const float d = v - pre, ad = fabsf(d), b = p.loss_beta;
      return (ad < b ? 0.5f * d * d / b : ad - 0.5f * b) * p.loss_inv_n;
    } else {
      // the sampler's x0-hat clamp (ViT.py:229, ViT_draft2drawing.py:280), and for
      // modes 1 / 4 the whole DDIM update (ViT.py:230-234) with x_t preloaded in `pre`
      const float x0 = fminf(fmaxf(v, -1.f), 1.f);
      if (p.head_mode == 2) {
        reinterpret_cast<float*>(p.C)[idx] = x0;
        return x0;
      } else {
        const float eps = (pre - cf[0] * x0) / cf[1];
        const float xn = cf[2] * x0 + cf[3] * eps;
        reinterpret_cast<float*>(p.C)[idx] = xn;
        reinterpret_cast<float*>(p.C2)[idx] = x0;
        return xn;
      }
    }
  } else if (EPI == EPI_EMBED) {
    v += pre;
    if (p.thr_drop) v = dropout_keep(salt_drop, (uint32_t)idx, p.thr_drop) ? v * p.scale_drop : 0.f;
    reinterpret_cast<float*>(p.C)[idx] = v;
    return v;
  }
  return 0.f;
}

// scalar whole-tile epilogue (HEAD: output columns are not contiguous in memory):
// acc[FM][FN] fragment tiles at (mb + i*16 + 4g + r, nb + j*16 + li)
template <int EPI, int FM, int FN>
__device__ __forceinline__ void run_epilogue_scalar(const GemmParams& p, const f32x4 (&acc)[FM][FN], int mb, int nb,
                                             int g, int li) {
  constexpr bool ELEM = EPI == EPI_RESID || EPI == EPI_DGELU || EPI == EPI_EMBED || EPI == EPI_ACC;
  const bool head_ps = EPI == EPI_HEAD && p.head_mode == 4;  // per-sample coefficient rows
  const bool head_ddim = EPI == EPI_HEAD && (p.head_mode == 1 || head_ps);
  const bool head_loss = EPI == EPI_HEAD && p.head_mode == 3;
  RowInfo rows[FM][4];
  long long cols[FN];
  bool colok[FN];
  float colb[FN];
  const bool has_bias = (EPI != EPI_ATOMIC) && (EPI != EPI_ACC) && p.bias != nullptr;
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = nb + j * 16 + li;
    colok[j] = n < p.N;
    cols[j] = epi_col<EPI>(p, n);
    colb[j] = (has_bias && colok[j]) ? p.bias[n] : 0.f;
  }
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = mb + i * 16 + 4 * g + r;
      rows[i][r] = epi_row<EPI>(p, m < p.M ? m : p.M - 1);
      if (m >= p.M) rows[i][r].off = -1;
    }
  // LayerNorm fold, consumer side: per-row statistics and per-column c
  constexpr bool FC = FoldEpi<EPI>::CONSUMER, FP = FoldEpi<EPI>::PRODUCER;
  const bool fold = FC && p.ln_st != nullptr;
  // slot li of each of the lane's rows (the 16 lanes of a row group hold all <= 16 slots)
  const int np_in = p.K / LN_SLOT;
  float2 lnst[FM][4];
  float colc[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) colc[j] = (fold && colok[j]) ? p.ln_c[nb + j * 16 + li] : 0.f;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = mb + i * 16 + 4 * g + r;
      lnst[i][r] = (fold && m < p.M && li < np_in)
                       ? *reinterpret_cast<const float2*>(p.ln_st + 2 * ((size_t)m * np_in + li))
                       : make_float2(0.f, 0.f);
    }
  // phase 1: element loads
  float pre[FM][FN][4];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = 0.f;
        if ((head_ddim || head_loss) && rows[i][r].off >= 0 && colok[j]) v = p.res[rows[i][r].off + cols[j]];
        if (ELEM && rows[i][r].off >= 0 && colok[j]) {
          const int n = nb + j * 16 + li;
          if (EPI == EPI_RESID) v = p.res[rows[i][r].off + n];
          if (EPI == EPI_ACC && !p.acc_store) v = reinterpret_cast<const float*>(p.C)[rows[i][r].off + n];
          if (EPI == EPI_DGELU) v = bf2f(p.aux[rows[i][r].off + n]);
          if (EPI == EPI_EMBED) {
            const int m = mb + i * 16 + 4 * g + r;
            const int patch = m - rows[i][r].b * p.tokens;
            v = p.pos[(size_t)(patch + 1) * p.emb_dim + n] + p.temb[(size_t)p.tsteps[rows[i][r].b] * p.emb_dim + n];
          }
        }
        pre[i][j][r] = v;
      }
  // phase 2: compute + store
  uint32_t salt_drop = 0, salt_dp = 0;
  if (p.thr_drop) salt_drop = site_salt(p.rng, p.site_drop);
  if (p.thr_dp) salt_dp = site_salt(p.rng, p.site_dp);
  f32x4 cf = f32x4{0.f, 1.f, 0.f, 0.f};
  if (head_ddim && !head_ps) cf = f32x4{p.coef[0], p.coef[1], p.coef[2], p.coef[3]};
  float2 ms[FM][4];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (fold) {  // sum the slots across the 16 lanes (fixed butterfly order: identical on every lane)
        float2 t = lnst[i][r];
        t = f2add(t, f2xor<1>(t));
        t = f2add(t, f2xor<2>(t));
        t = f2add(t, f2xor<4>(t));
        t = f2add(t, f2xor<8>(t));
        lnst[i][r] = t;
      }
      ms[i][r] = fold ? ln_row_stats(p, lnst[i][r]) : make_float2(0.f, 1.f);
      const int m = mb + i * 16 + 4 * g + r;
      // every row's (mean, rstd) for the LayerNorm backward, also rows the epilogue skips
      if (fold && p.ln_mean != nullptr && nb == 0 && li == 0 && m < p.M) {
        p.ln_mean[m] = ms[i][r].x;
        p.ln_rstd[m] = ms[i][r].y;
      }
    }
  const bool prod = FP && p.st_out != nullptr;
  float lsum = 0.f;  // HEAD mode 3: this lane's loss contributions
  float2 part[FM][4][(FN + 1) / 2];  // producer (debug path): per-slot partials of the lane's rows
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int sl = 0; sl < (FN + 1) / 2; ++sl) part[i][r][sl] = make_float2(0.f, 0.f);
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (rows[i][r].off >= 0 && colok[j]) {
          const float a = fold ? (acc[i][j][r] - ms[i][r].x * colc[j]) * ms[i][r].y : acc[i][j][r];
          const float* cs = p.coef + 4 * rows[i][r].b;  // mode 4: this row's sample
          const f32x4 cfr = head_ps ? f32x4{cs[0], cs[1], cs[2], cs[3]} : cf;
          const float o = epilogue<EPI>(p, rows[i][r].off + cols[j], rows[i][r].b, a + colb[j], pre[i][j][r],
                                        salt_drop, salt_dp, cfr);
          if (prod) {
            part[i][r][j / 2] = f2add(part[i][r][j / 2], make_float2(o, o * o));
            p.xb_out[rows[i][r].off + cols[j]] = f2bf(o);
          }
          if (EPI == EPI_HEAD && p.patch_out != nullptr && (p.head_mode == 1 || p.head_mode == 2 || head_ps)) {
            // the new image pixel (c, a, b) of patch row (sample, token - 1), conv-im2col order
            const int m = mb + i * 16 + 4 * g + r, n = nb + j * 16 + li;
            const int c = n % p.chans, ab = n / p.chans;
            p.patch_out[(size_t)(m - m / p.tokens - 1) * p.N + c * p.patch * p.patch + ab] = f2bf(o);
          }
          if (head_loss) {  // gradient of the mean smooth-L1, straight into the token layout
            const int m = mb + i * 16 + 4 * g + r, n = nb + j * 16 + li;
            const float d = (a + colb[j] - pre[i][j][r]) / p.loss_beta;
            reinterpret_cast<bf16*>(p.C2)[(size_t)m * p.N + n] = f2bf(fminf(fmaxf(d, -1.f), 1.f) * p.loss_inv_n);
            lsum += o;
          }
        } else if (head_loss && colok[j] && mb + i * 16 + 4 * g + r < p.M) {  // cls rows: zero gradient
          reinterpret_cast<bf16*>(p.C2)[(size_t)(mb + i * 16 + 4 * g + r) * p.N + nb + j * 16 + li] = f2bf(0.f);
        }
  if (prod) {
    const int np_out = p.N / LN_SLOT;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int sl = 0; sl < (FN + 1) / 2; ++sl) {
          float2 t = part[i][r][sl];
          t = f2add(t, f2xor<1>(t));
          t = f2add(t, f2xor<2>(t));
          t = f2add(t, f2xor<4>(t));
          t = f2add(t, f2xor<8>(t));
          const int m = mb + i * 16 + 4 * g + r;
          if (li == 0 && m < p.M)
            *reinterpret_cast<float2*>(p.st_out + 2 * ((size_t)fold_token_row<EPI>(p, m) * np_out + nb / LN_SLOT +
                                                       sl)) = t;
        }
  }
  if (head_loss) {  // one deterministic partial per workgroup (summed by the step tail)
    __shared__ float lred[4];
    lsum = wave_sum(lsum);
    if ((threadIdx.x & 63) == 0) lred[threadIdx.x >> 6] = lsum;
    __syncthreads();
    if (threadIdx.x == 0) p.loss_parts[blockIdx.x] = (lred[0] + lred[1]) + (lred[2] + lred[3]);
  }
}


// ---- 4x4 transpose inside each quad of lanes (DPP quad_perm, no LDS):
// in:  a[r] = element (row r, column x) of a 4x4 block, x = lane's quad position
// out: o[c] = element (row x, column c)
__device__ __forceinline__ float sel4(const f32x4& a, int i) {
  return i == 0 ? a[0] : i == 1 ? a[1] : i == 2 ? a[2] : a[3];
}
template <int CTRL>
__device__ __forceinline__ float dpp_f(float x) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ f32x4 quad_transpose(const f32x4& a, int x) {
  const float r0 = sel4(a, x);
  const float r1 = dpp_f<0x93>(sel4(a, (x + 1) & 3));  // from quad lane (x-1)&3: (row x, col (x-1)&3)
  const float r2 = dpp_f<0x4E>(sel4(a, (x + 2) & 3));  // (row x, col (x-2)&3)
  const float r3 = dpp_f<0x39>(sel4(a, (x + 3) & 3));  // (row x, col (x-3)&3)
  f32x4 o;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int d = (x - c) & 3;
    o[c] = d == 0 ? r0 : d == 1 ? r1 : d == 2 ? r2 : r3;
  }
  return o;
}

__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ void st4(float* p, const f32x4& v) { *reinterpret_cast<f32x4*>(p) = v; }
__device__ __forceinline__ void st4bf(bf16* p, const f32x4& v) {
  bf16x4 b;
  b[0] = f2bf(v[0]); b[1] = f2bf(v[1]); b[2] = f2bf(v[2]); b[3] = f2bf(v[3]);
  *reinterpret_cast<bf16x4*>(p) = b;
}
// {sum, sum of squares} of 4 consecutive outputs (LayerNorm statistics
// producer).  Explicit fma so every kernel that produces statistics rounds
// identically, whatever the compiler's contraction choice in its context.
__device__ __forceinline__ float2 stat4(const f32x4& v) {
  return make_float2((v[0] + v[1]) + (v[2] + v[3]),
                     __builtin_fmaf(v[0], v[0], v[1] * v[1]) + __builtin_fmaf(v[2], v[2], v[3] * v[3]));
}

// bf16x4 store, write-through (sc1) when the bytes are handed to another workgroup of the launch
template <bool PUB>
__device__ __forceinline__ void st4bf_pub(bf16* p, const f32x4& v) {
  if (!PUB) {
    st4bf(p, v);
  } else {
    bf16x4 b;
    b[0] = f2bf(v[0]); b[1] = f2bf(v[1]); b[2] = f2bf(v[2]); b[3] = f2bf(v[3]);
    st8_sc1(p, __builtin_bit_cast(uint64_t, b));
  }
}
template <bool PUB>
__device__ __forceinline__ void st2f_pub(float* p, float2 v) {
  if (!PUB) *reinterpret_cast<float2*>(p) = v;
  else st8_sc1(p, __builtin_bit_cast(uint64_t, v));
}
template <bool PUB>
__device__ __forceinline__ float2 ld2f_pub(const float* p) {
  if (!PUB) return *reinterpret_cast<const float2*>(p);
  return __builtin_bit_cast(float2, ld8_sc1(p));
}
__device__ __forceinline__ f32x4 ld4bf(const bf16* p) {
  const bf16x4 b = *reinterpret_cast<const bf16x4*>(p);
  return f32x4{bf2f(b[0]), bf2f(b[1]), bf2f(b[2]), bf2f(b[3])};
}

// Vector epilogue: each lane owns 4 CONSECUTIVE columns of one row, so every
// load/store of the epilogue is one 8-/16-byte vector access instead of four
// 2-/4-byte scalar ones.  Requires N % 4 == 0 and output columns contiguous in
// groups of 4 (all epilogues except HEAD).  Two accumulator layouts:
//   SW (swapped MFMA operands, the LDS-DMA GEMMs): mfma(B, A) computes C^T, whose
//     natural layout already is lane = row (li), 4 registers = 4 columns (4g..4g+3)
//     -- no data movement at all;
//   !SW (mfma(A, B), the register-staged fallback GEMM): lane = column, 4 registers
//     = 4 rows, transposed inside lane quads (quad_transpose: ~27 vector
//     instructions per fragment) to lane = row 4g+x, columns 4q..4q+3.
// The lanes that share a row are li>>2 = 0..3 (!SW) or g = 0..3 (SW); the LayerNorm
// statistics reduce over them (lane xor 4, 8 or xor 16, 32).
//
// Split in two so the epilogue's global loads (bias, residual, saved
// pre-activation, embeddings, accumulate target) can be issued BEFORE the main
// loop (`prefetch`) and land while the MFMAs run: at these sizes a GEMM is a
// chain of ~3 dependent memory round trips and this removes one of them.
template <int EPI, int FM, int FN, bool PUB = false, bool SW = false>
struct VecEpi {
  static constexpr bool PRE = EPI == EPI_RESID || EPI == EPI_DGELU || EPI == EPI_EMBED || EPI == EPI_ACC ||
                              EPI == EPI_HEADR || EPI == EPI_HEADL;
  static constexpr bool FC = FoldEpi<EPI>::CONSUMER, FP = FoldEpi<EPI>::PRODUCER;
  RowInfo32 rows[FM];
  f32x4 hcf[FM];    // HEADR: the row's DDIM coefficients {sqrt a_t, sqrt(1-a_t), sqrt a_tk, sqrt(1-a_tk)}
  int cols[FN];
  bool colok[FN];
  f32x4 colb[FN];
  f32x4 pre[FM][FN];
  int rowm[FM];     // GEMM row of the lane's fragment row (-1: out of range)
  float2 lnst[FM][LN_MAX_SLOTS / 4];  // fold consumer: statistics slots u, u+4, .. of the row (u: sharer index)
  f32x4 lnc[FN];    // fold consumer: c of the lane's 4 columns
  bool first_col;   // lane holds column 0 (writes the row's mean / rstd)
  int colbase;      // first column of the wave's tile
  int cls_i;        // EMBED with cls_src: fragment row that is a sample's first patch (-1: none)
  int cls_b;        //   and its sample (kept as a scalar: indexing rowm[cls_i] would put the
                    //   epilogue's arrays in scratch memory)
  f32x4 clsv[FN];   //   cls + pos[0] + temb[t] of that sample's cls row, the lane's columns
  float sqacc;      // ACC with sq_parts: this lane's sum of squares of the stored values
  int64_t rng0, rng1;  // the step's {seed, step}, loaded by prefetch (dropout salts)

  // lane -> (row within the 16-row fragment, first of its 4 columns within the 16-column fragment)
  static __device__ __forceinline__ int rsub(int g, int li) { return SW ? li : 4 * g + (li & 3); }
  static __device__ __forceinline__ int csub(int g, int li) { return SW ? 4 * g : 4 * (li >> 2); }
  // index 0..3 of the lane among the 4 lanes holding the same row
  static __device__ __forceinline__ int sharer(int g, int li) { return SW ? g : li >> 2; }
  // butterfly step K (0, 1) of a sum across the row's 4 lanes: t + partner.  SW:
  // the partners are 16 / 32 lanes apart, exchanged by v_permlane16/32_swap (the
  // two swap results ARE {own, partner} in some order: their sum is t + partner,
  // no address math or LDS crossbar as in __shfl_xor)
  template <int K>
  static __device__ __forceinline__ float psum(float v) {
    const uint32_t u = __float_as_uint(v);
    if (K == 0) {
      const auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);
      return __uint_as_float(r[0]) + __uint_as_float(r[1]);
    }
    const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
  template <int K>
  static __device__ __forceinline__ float2 rowsum(float2 a) {
    if (SW) return make_float2(psum<K>(a.x), psum<K>(a.y));
    return f2add(a, f2xor<4 << K>(a));
  }

  __device__ __forceinline__ void prefetch(const GemmParams& p, int mb, int nb, int g, int li) {
    const int q = sharer(g, li), cs = csub(g, li), rs = rsub(g, li);
    // uniform pointer select + constant-address-space loads -> scalar loads: a vector
    // load under the dropout condition was waited for on the spot (vmcnt(0): the
    // operand stages issued before it too -- tools/ub_gemm_stamps.py, first stage of
    // the vit_small_200 GELU GEMM 2.7 us vs 1.8 without dropout)
    const int64_t* rp = (p.thr_drop || p.thr_dp) ? p.rng : kEpiNoRng;
    const auto* rs4 = (const __attribute__((address_space(4))) int64_t*)(uintptr_t)rp;
    rng0 = rs4[0];
    rng1 = rs4[1];
    const bool fold = FC && p.ln_st != nullptr;
    first_col = nb == 0 && q == 0;
    colbase = nb;
    const bool has_bias = (EPI != EPI_ATOMIC) && (EPI != EPI_ACC) && p.bias != nullptr;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = nb + j * 16 + cs;
      colok[j] = n < p.N;
      // QKV head-major scatter: a 16-column fragment lies inside one head when
      // hd % 16 == 0, so its (wave-uniform, scalar) base column is mapped once
      if (EPI == EPI_QKV && (p.hd & 15) == 0) cols[j] = (int)epi_col<EPI>(p, nb + j * 16) + cs;
      else cols[j] = (int)epi_col<EPI>(p, n);
      colb[j] = (has_bias && colok[j]) ? ld4(p.bias + n) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    int rowsafe[FM];  // the row offset with m clamped (RESID / DGELU operand loads)
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int m = mb + i * 16 + rs;
      rows[i] = epi_row32<EPI>(p, m < p.M ? m : p.M - 1);
      rowsafe[i] = rows[i].off;
      if (m >= p.M) rows[i].off = -1;
      rowm[i] = m < p.M ? m : -1;
      const int np_in = p.K / LN_SLOT;
#pragma unroll
      for (int k = 0; k < LN_MAX_SLOTS / 4; ++k) {
        const int sl = q + 4 * k;
        lnst[i][k] = (fold && m < p.M && sl < np_in) ? ld2f_pub<PUB>(p.ln_st + 2 * ((size_t)m * np_in + sl))
                                                     : make_float2(0.f, 0.f);
      }
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = nb + j * 16 + cs;
      lnc[j] = (fold && colok[j]) ? ld4(p.ln_c + n) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if (EPI == EPI_HEADR) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
        hcf[i] = p.head_mode == 4 ? ld4(p.coef + 4 * rows[i].b)
                 : p.head_mode == 1 ? ld4(p.coef) : f32x4{0.f, 1.f, 0.f, 1.f};
    }
    cls_i = -1;
    cls_b = 0;
    if (EPI == EPI_EMBED && p.cls_src != nullptr) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
        if (rowm[i] >= 0 && rowm[i] % p.tokens == 0) {
          cls_i = i;
          cls_b = rowm[i] / p.tokens;
        }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = nb + j * 16 + cs;
        clsv[j] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (cls_i >= 0 && colok[j])
          clsv[j] = ld4(p.cls_src + n) + ld4(p.pos + n) + ld4(p.temb + (size_t)p.tsteps[cls_b] * p.emb_dim + n);
      }
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
        if (EPI == EPI_RESID || EPI == EPI_DGELU) {
          // unconditional loads at a clamped row / column (finish skips those lanes): a
          // load under a condition became a phi copy that waited for it right here --
          // and, vmcnt being in order, for the operand DMA issued before it
          const int n = nb + j * 16 + cs;
          const int ns = colok[j] ? n : p.N - 4;
          if (EPI == EPI_RESID) v = ld4(p.res + rowsafe[i] + ns);
          else v = ld4bf(p.aux + rowsafe[i] + ns);
        } else if (PRE && rows[i].off >= 0 && colok[j]) {
          const int n = nb + j * 16 + cs;
          if (EPI == EPI_HEADR && p.head_mode != 2) v = ld4(p.res + rows[i].off + n);  // x_t
          if (EPI == EPI_HEADL && rows[i].b >= 0)  // target patch row (m - b - 1)
            v = ld4(p.res + (rows[i].off - (rows[i].b + 1) * p.N) + n);
          if (EPI == EPI_ACC && !p.acc_store) v = ld4(reinterpret_cast<const float*>(p.C) + rows[i].off + n);
          if (EPI == EPI_EMBED) {
            const int m = mb + i * 16 + rs;
            const int patch = m - rows[i].b * p.tokens;
            v = ld4(p.pos + (size_t)(patch + 1) * p.emb_dim + n) +
                ld4(p.temb + (size_t)p.tsteps[rows[i].b] * p.emb_dim + n);
          }
        }
        pre[i][j] = v;
      }
  }

  __device__ __forceinline__ void finish(const GemmParams& p, const f32x4 (&acc_in)[FM][FN], int li) {
    // every prefetched operand (and the rng words) has long landed: one explicit
    // vmcnt(0) here, BEFORE the first store.  Without it the compiler (operands loaded
    // under conditions, stores under conditions: a path-merged count) waited vmcnt(0)
    // at each fragment's first use, i.e. for all the epilogue stores issued so far,
    // and the salts were loaded here and waited for twice.  (gfx9 encoding: vmcnt 0,
    // expcnt 7, lgkmcnt 15.)
    __builtin_amdgcn_s_waitcnt(0x0F70);
    const int x = li & 3;
    const int g = (threadIdx.x & 63) >> 4;
    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = SW ? acc_in[i][j] : quad_transpose(acc_in[i][j], x);
    uint32_t salt_drop = 0, salt_dp = 0;
    if (p.thr_drop) salt_drop = site_salt_v((uint64_t)rng0, (uint64_t)rng1, p.site_drop);
    if (p.thr_dp) salt_dp = site_salt_v((uint64_t)rng0, (uint64_t)rng1, p.site_dp);
    const bool fold = FC && p.ln_st != nullptr;
    const bool prod = FP && p.st_out != nullptr;
    float lsum = 0.f;  // HEADL: this lane's loss contributions
    sqacc = 0.f;
    float2 ms[FM];
    constexpr int SL = FN / 2;  // 32-column statistics slots per wave
    float2 part[FM][SL];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      if (fold) {  // the row's slots: lane-local, then across the 4 lanes of the row (fixed order)
        float2 t = lnst[i][0];
#pragma unroll
        for (int k = 1; k < LN_MAX_SLOTS / 4; ++k) t = f2add(t, lnst[i][k]);
        t = rowsum<1>(rowsum<0>(t));
        ms[i] = ln_row_stats(p, t);
      } else {
        ms[i] = make_float2(0.f, 1.f);
      }
#pragma unroll
      for (int sl = 0; sl < SL; ++sl) part[i][sl] = make_float2(0.f, 0.f);
      if (fold && p.ln_mean != nullptr && first_col && rowm[i] >= 0) {
        p.ln_mean[rowm[i]] = ms[i].x;
        p.ln_rstd[rowm[i]] = ms[i].y;
      }
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      if (rows[i].off < 0) continue;
      const bool keep_row =
          (EPI == EPI_RESID && p.thr_dp) ? dropout_keep(salt_dp, (uint32_t)rows[i].b, p.thr_dp) : true;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        if (!colok[j]) continue;
        const int idx = rows[i].off + cols[j];
        f32x4 v = fold ? (acc[i][j] - ms[i].x * lnc[j]) * ms[i].y + colb[j] : acc[i][j] + colb[j];
        if (EPI == EPI_BF16) {
          st4bf(reinterpret_cast<bf16*>(p.C) + idx + blockIdx.z * p.split_stride, v);
        } else if (EPI == EPI_QKV) {
          st4bf(reinterpret_cast<bf16*>(p.C) + idx, v);
        } else if (EPI == EPI_F32) {
          st4(reinterpret_cast<float*>(p.C) + idx + blockIdx.z * p.split_stride, v);
        } else if (EPI == EPI_ATOMIC) {
#pragma unroll
          for (int c = 0; c < 4; ++c) atomicAdd(reinterpret_cast<float*>(p.C) + idx + c, v[c]);
        } else if (EPI == EPI_ACC) {
          const f32x4 o = pre[i][j] + v;
          st4(reinterpret_cast<float*>(p.C) + idx, o);
          if (p.sq_parts) sqacc += (o.x * o.x + o.y * o.y) + (o.z * o.z + o.w * o.w);
        } else if (EPI == EPI_RESID) {
          bool kp[4] = {true, true, true, true};
          if (p.thr_drop) dropout_keep4(salt_drop, (uint32_t)idx, p.thr_drop, kp);
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            float e = v[c];
            if (p.thr_drop) e = kp[c] ? e * p.scale_drop : 0.f;
            if (p.thr_dp) e = keep_row ? e * p.scale_dp : 0.f;
            v[c] = pre[i][j][c] + e;
          }
          st4(reinterpret_cast<float*>(p.C) + idx, v);
          if (prod) {
            part[i][j / 2] = f2add(part[i][j / 2], stat4(v));
            st4bf_pub<PUB>(p.xb_out + idx, v);
          }
        } else if (EPI == EPI_GELU) {
          st4bf(reinterpret_cast<bf16*>(p.C) + idx, v);
          f32x4 h;
          bool kp[4] = {true, true, true, true};
          if (p.thr_drop) dropout_keep4(salt_drop, (uint32_t)idx, p.thr_drop, kp);
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            float e = gelu_f(v[c]);
            if (p.thr_drop) e = kp[c] ? e * p.scale_drop : 0.f;
            h[c] = e;
          }
          st4bf_pub<PUB>(reinterpret_cast<bf16*>(p.C2) + idx, h);
        } else if (EPI == EPI_DGELU) {
          bool kp[4] = {true, true, true, true};
          if (p.thr_drop) dropout_keep4(salt_drop, (uint32_t)idx, p.thr_drop, kp);
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            float e = v[c];
            if (p.thr_drop) e = kp[c] ? e * p.scale_drop : 0.f;
            v[c] = e * gelu_grad_f(pre[i][j][c]);
          }
          st4bf(reinterpret_cast<bf16*>(p.C) + idx, v);
        } else if (EPI == EPI_HEADL) {
          // smooth-L1 vs the target (multi_gpu_trainer.py:124) and its gradient in the
          // token layout the head backward reads; cls rows get a zero gradient
          f32x4 gr = f32x4{0.f, 0.f, 0.f, 0.f};
          if (rows[i].b >= 0) {
            const float bt = p.loss_beta;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              const float d = v[c] - pre[i][j][c], ad = fabsf(d);
              lsum += (ad < bt ? 0.5f * d * d / bt : ad - 0.5f * bt) * p.loss_inv_n;
              gr[c] = fminf(fmaxf(d / bt, -1.f), 1.f) * p.loss_inv_n;
            }
          }
          st4bf(reinterpret_cast<bf16*>(p.C) + idx, gr);
        } else if (EPI == EPI_HEADR) {
          // ViT.py:229-234 on the patch rows: x0-hat clamp, then (modes 1 / 4) the DDIM
          // update with x_t preloaded in `pre`; the new x_t also as the next step's
          // bf16 patch rows (same index: the embedding weight is column-permuted)
          f32x4 x0;
#pragma unroll
          for (int c = 0; c < 4; ++c) x0[c] = fminf(fmaxf(v[c], -1.f), 1.f);
          f32x4 xn = x0;
          if (p.head_mode != 2) {
            const f32x4 cf = hcf[i];
#pragma unroll
            for (int c = 0; c < 4; ++c) xn[c] = cf[2] * x0[c] + cf[3] * ((pre[i][j][c] - cf[0] * x0[c]) / cf[1]);
            st4(reinterpret_cast<float*>(p.C2) + idx, x0);
          }
          st4(reinterpret_cast<float*>(p.C) + idx, xn);
          if (p.patch_out != nullptr) st4bf(p.patch_out + idx, xn);
        } else if (EPI == EPI_EMBED) {
          v += pre[i][j];
          if (p.thr_drop) {
            bool kp[4];
            dropout_keep4(salt_drop, (uint32_t)idx, p.thr_drop, kp);
#pragma unroll
            for (int c = 0; c < 4; ++c) v[c] = kp[c] ? v[c] * p.scale_drop : 0.f;
          }
          st4(reinterpret_cast<float*>(p.C) + idx, v);
          if (prod) {
            part[i][j / 2] = f2add(part[i][j / 2], stat4(v));
            st4bf_pub<PUB>(p.xb_out + idx, v);
          }
        }
      }
    }
    if (EPI == EPI_EMBED && p.cls_src != nullptr) {
      // the cls row of a sample whose first patch row this lane holds (the same
      // lanes of the row group, so the statistics reduce like the patch rows')
      const int b = cls_b;
      const long long crow = (long long)b * (p.tokens + 1) * p.emb_dim;
      float2 cpart[SL];
#pragma unroll
      for (int sl = 0; sl < SL; ++sl) cpart[sl] = make_float2(0.f, 0.f);
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        if (cls_i < 0 || !colok[j]) continue;
        const long long idx = crow + colbase + j * 16 + csub(g, li);
        f32x4 v = clsv[j];
        if (p.thr_drop) {
          bool kp[4];
          dropout_keep4(salt_drop, (uint32_t)idx, p.thr_drop, kp);
#pragma unroll
          for (int c = 0; c < 4; ++c) v[c] = kp[c] ? v[c] * p.scale_drop : 0.f;
        }
        st4(reinterpret_cast<float*>(p.C) + idx, v);
        if (prod) {
          cpart[j / 2] = f2add(cpart[j / 2], stat4(v));
          st4bf_pub<PUB>(p.xb_out + idx, v);
        }
      }
      if (prod) {
        const int np_out = p.N / LN_SLOT;
#pragma unroll
        for (int sl = 0; sl < SL; ++sl) {
          float2 t = cpart[sl];
          t = rowsum<1>(rowsum<0>(t));
          if (sharer(g, li) == 0 && cls_i >= 0)
            st2f_pub<PUB>(p.st_out + 2 * ((size_t)b * (p.tokens + 1) * np_out + colbase / LN_SLOT + sl), t);
        }
      }
    }
    if (EPI == EPI_HEADL) {  // one deterministic loss partial per workgroup
      __shared__ float lred[4];
      lsum = wave_sum(lsum);
      if ((threadIdx.x & 63) == 0) lred[threadIdx.x >> 6] = lsum;
      __syncthreads();
      if (threadIdx.x == 0) p.loss_parts[blockIdx.x] = (lred[0] + lred[1]) + (lred[2] + lred[3]);
    }
    if (prod) {
      // the 4 lanes of a row hold 32 consecutive columns per slot (fragments j,
      // j+1): reduce, one float2 store per (row, slot)
      const int np_out = p.N / LN_SLOT;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int sl = 0; sl < SL; ++sl) {
          float2 t = part[i][sl];
          t = rowsum<1>(rowsum<0>(t));
          if (sharer(g, li) == 0 && rowm[i] >= 0)
            st2f_pub<PUB>(p.st_out + 2 * ((size_t)fold_token_row<EPI>(p, rowm[i]) * np_out + colbase / LN_SLOT + sl),
                          t);
        }
    }
  }
};

template <int EPI, int FM, int FN>
__device__ __forceinline__ void run_epilogue_vec(const GemmParams& p, const f32x4 (&acc)[FM][FN], int mb, int nb,
                                                 int g, int li) {
  VecEpi<EPI, FM, FN> ep;
  ep.prefetch(p, mb, nb, g, li);
  ep.finish(p, acc, li);
}

// epilogues that take the quad-transposed vector path
template <int EPI>
struct UsesVecEpi {
  // HEAD: columns not contiguous.  ATOMIC: in the accumulator layout one atomic
  // instruction covers 4 rows x 64 B; after the quad transpose it would touch 16
  // rows (4x the cache lines per instruction) - measured 10% slower per step.
  static constexpr bool value = EPI != EPI_HEAD && EPI != EPI_ATOMIC;
};

template <int EPI, int FM, int FN>
__device__ __forceinline__ void run_epilogue(const GemmParams& p, const f32x4 (&acc)[FM][FN], int mb, int nb,
                                             int g, int li) {
  if (!UsesVecEpi<EPI>::value) run_epilogue_scalar<EPI, FM, FN>(p, acc, mb, nb, g, li);
  else run_epilogue_vec<EPI, FM, FN>(p, acc, mb, nb, g, li);
}


}  // namespace dc
