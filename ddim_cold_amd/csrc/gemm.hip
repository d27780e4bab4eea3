// bf16 MFMA GEMM family for gfx950 with fused epilogues.
//
//   C[m][n] = sum_k A(m,k) * B(n,k)
//
// Operand layouts (template flags):
//   AT=false: A stored [M][K] (k contiguous)   AT=true: A stored [K][M]
//   BT=false: B stored [N][K] (k contiguous)   BT=true: B stored [K][N]
// which covers every linear of the ViT:
//   forward   y = x W^T        : AT=0, BT=0  (W is nn.Linear [out,in])
//   dgrad    dx = dy W         : AT=0, BT=1
//   wgrad    dW = dy^T x       : AT=1, BT=1  (split-K over tokens, fp32 atomics)
//
// Tile: BM x BN x 64, 256 threads = 4 waves (WM x WN), v_mfma_f32_16x16x32_bf16.
// LDS images (double-buffered, register-staged so the next tile's global loads
// are in flight during the current tile's MFMAs):
//   k-contiguous operand: [rows][64] bf16, 16-B chunk XOR swizzle
//       chunk' = chunk ^ ((row>>1)&7)  -> ds_read_b128 / ds_read_b64 conflict-free
//   transposed operand:   [64 k-rows][R+16] bf16 (row pad 32 B), read with
//       ds_read_b64_tr_b16 (the hardware transposing LDS read) -> conflict-free.
// When either operand is transposed both operands use the permuted k order
// (lane group g, element j) -> k = j<4 ? 4g+j : 16+4g+(j-4), which is what two
// tr reads naturally deliver; MFMA sums over k so any common permutation is exact.
//
// Grid: one workgroup per output tile (XCD-aware bijective remap of the linear
// block id so tiles that share an A panel share an L2), z = split-K slice.
// Reference semantics covered: nn.Linear / Conv2d-as-GEMM in ViT.py:79-103,150,183.
#include "common.h"
#include "kernels.h"
#include "gemm_common.h"
#include <cstdlib>
#include <algorithm>
#include <type_traits>

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
  const float* coef;     // HEAD mode 1: {sqrt a_t, sqrt(1-a_t), sqrt a_tk, sqrt(1-a_tk)} (device)
  long long split_stride;  // EPI_F32: elements between the K-split output slices
  int head_mode;         // HEAD: 0 image, 1 fused DDIM step (res = x_t in, C = x_next, C2 = x0), 2 clamp,
                         //   3 training loss (res = target image, C2 = token-layout grad, loss_parts)
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
  int debug;  // profiling aid (DDIM_COLD_GEMM_DEBUG): 1 = skip the epilogue, 2 = skip the main loop,
              // 3 = scalar (untransposed) epilogue
};


constexpr int WG_MAX = 6;
struct WgradGroup {
  GemmParams p[WG_MAX];
  int tile_start[WG_MAX + 1];
  int n;
};

static bool getenv_flag(const char* name) {
  const char* e = getenv(name);
  return e && e[0] == '1';
}

static bool dma_disabled() {
  static const bool off = [] {
    const char* e = getenv("DDIM_COLD_GEMM_NO_DMA");
    return e && e[0] == '1';
  }();
  return off;
}

template <int R, bool T>
struct Stage {
  static constexpr int CHUNKS = R * 8;
  static constexpr int PER_T = CHUNKS / 256;
  static constexpr int STRIDE_T = 2 * R + 32;  // bytes per k-row of a transposed image
  static constexpr int BYTES = T ? (BK * STRIDE_T) : (R * 128);
  u32x4 regs[PER_T];

  __device__ __forceinline__ void load(const bf16* __restrict__ base, int ld, int row0, int rows_total,
                                       int k0, int K) {
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      const int c = threadIdx.x + i * 256;
      u32x4 v = {0u, 0u, 0u, 0u};
      if (!T) {
        const int r = c >> 3, kc = c & 7;
        const int gr = row0 + r, gk = k0 + kc * 8;
        if (gr < rows_total && gk < K) v = *reinterpret_cast<const u32x4*>(base + (size_t)gr * ld + gk);
      } else {
        const int r = c / (R / 8), cc = c % (R / 8);
        const int gk = k0 + r, gc = row0 + cc * 8;
        if (gk < K && gc < rows_total) v = *reinterpret_cast<const u32x4*>(base + (size_t)gk * ld + gc);
      }
      regs[i] = v;
    }
  }
  __device__ __forceinline__ void store(char* lds) const {
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      const int c = threadIdx.x + i * 256;
      int off;
      if (!T) {
        const int r = c >> 3, kc = c & 7;
        off = r * 128 + 16 * (kc ^ swz(r));
      } else {
        const int r = c / (R / 8), cc = c % (R / 8);
        off = r * STRIDE_T + cc * 16;
      }
      *reinterpret_cast<u32x4*>(lds + off) = regs[i];
    }
  }
};

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
      EPI == EPI_QKV || EPI == EPI_GELU || EPI == EPI_BF16 || EPI == EPI_F32 || EPI == EPI_HEAD;
  static constexpr bool PRODUCER = EPI == EPI_RESID || EPI == EPI_EMBED;
};

// Row statistics layout: st[row][NP][2], NP = D / 32 slots; slot s holds
// {sum, sum^2} of the row's columns 32s..32s+31, written exactly once by the
// wave of the producing epilogue that owns those columns (no atomics, no
// zeroing: deterministic).  Consumers add the slots in a fixed butterfly order.
constexpr int LN_SLOT = 32;
constexpr int LN_MAX_SLOTS = 16;

// (mean, rstd) of a row from its {sum, sum^2} over D = K columns
__device__ __forceinline__ float2 ln_row_stats(const GemmParams& p, float2 st) {
  const float invd = 1.0f / (float)p.K;
  const float mu = st.x * invd;
  const float var = fmaxf(st.y * invd - mu * mu, 0.f);
  return make_float2(mu, rsqrtf(var + p.ln_eps));
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
      // mode 1 the whole DDIM update (ViT.py:230-234) with x_t preloaded in `pre`
      const float x0 = fminf(fmaxf(v, -1.f), 1.f);
      if (p.head_mode == 2) {
        reinterpret_cast<float*>(p.C)[idx] = x0;
      } else {
        const float eps = (pre - cf[0] * x0) / cf[1];
        reinterpret_cast<float*>(p.C)[idx] = cf[2] * x0 + cf[3] * eps;
        reinterpret_cast<float*>(p.C2)[idx] = x0;
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
  const bool head_ddim = EPI == EPI_HEAD && p.head_mode == 1;
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
          if (EPI == EPI_ACC) v = reinterpret_cast<const float*>(p.C)[rows[i][r].off + n];
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
  if (head_ddim) cf = f32x4{p.coef[0], p.coef[1], p.coef[2], p.coef[3]};
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
          const float o = epilogue<EPI>(p, rows[i][r].off + cols[j], rows[i][r].b, a + colb[j], pre[i][j][r],
                                        salt_drop, salt_dp, cf);
          if (prod) {
            part[i][r][j / 2] = f2add(part[i][r][j / 2], make_float2(o, o * o));
            p.xb_out[rows[i][r].off + cols[j]] = f2bf(o);
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
__device__ __forceinline__ f32x4 ld4bf(const bf16* p) {
  const bf16x4 b = *reinterpret_cast<const bf16x4*>(p);
  return f32x4{bf2f(b[0]), bf2f(b[1]), bf2f(b[2]), bf2f(b[3])};
}

// Vector epilogue: the MFMA accumulator layout (lane = column, 4 registers =
// 4 rows) is transposed inside lane quads so each lane owns 4 CONSECUTIVE
// columns of one row; every load/store of the epilogue is then one 8-/16-byte
// vector access instead of four 2-/4-byte scalar ones.  Requires N % 4 == 0 and
// output columns contiguous in groups of 4 (all epilogues except HEAD).
//
// Split in two so the epilogue's global loads (bias, residual, saved
// pre-activation, embeddings, accumulate target) can be issued BEFORE the main
// loop (`prefetch`) and land while the MFMAs run: at these sizes a GEMM is a
// chain of ~3 dependent memory round trips and this removes one of them.
template <int EPI, int FM, int FN>
struct VecEpi {
  static constexpr bool PRE = EPI == EPI_RESID || EPI == EPI_DGELU || EPI == EPI_EMBED || EPI == EPI_ACC;
  static constexpr bool FC = FoldEpi<EPI>::CONSUMER, FP = FoldEpi<EPI>::PRODUCER;
  RowInfo rows[FM];
  long long cols[FN];
  bool colok[FN];
  f32x4 colb[FN];
  f32x4 pre[FM][FN];
  int rowm[FM];     // GEMM row of the lane's fragment row (-1: out of range)
  float2 lnst[FM][LN_MAX_SLOTS / 4];  // fold consumer: statistics slots q, q+4, .. of the row
  f32x4 lnc[FN];    // fold consumer: c of the lane's 4 columns
  bool first_col;   // lane holds column 0 (writes the row's mean / rstd)
  int colbase;      // first column of the wave's tile

  __device__ __forceinline__ void prefetch(const GemmParams& p, int mb, int nb, int g, int li) {
    const int x = li & 3, q = li >> 2;
    const bool fold = FC && p.ln_st != nullptr;
    first_col = nb == 0 && q == 0;
    colbase = nb;
    const bool has_bias = (EPI != EPI_ATOMIC) && (EPI != EPI_ACC) && p.bias != nullptr;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = nb + j * 16 + 4 * q;
      colok[j] = n < p.N;
      cols[j] = epi_col<EPI>(p, n);
      colb[j] = (has_bias && colok[j]) ? ld4(p.bias + n) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int m = mb + i * 16 + 4 * g + x;
      rows[i] = epi_row<EPI>(p, m < p.M ? m : p.M - 1);
      if (m >= p.M) rows[i].off = -1;
      rowm[i] = m < p.M ? m : -1;
      const int np_in = p.K / LN_SLOT;
#pragma unroll
      for (int k = 0; k < LN_MAX_SLOTS / 4; ++k) {
        const int sl = q + 4 * k;
        lnst[i][k] = (fold && m < p.M && sl < np_in)
                         ? *reinterpret_cast<const float2*>(p.ln_st + 2 * ((size_t)m * np_in + sl))
                         : make_float2(0.f, 0.f);
      }
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = nb + j * 16 + 4 * q;
      lnc[j] = (fold && colok[j]) ? ld4(p.ln_c + n) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
        if (PRE && rows[i].off >= 0 && colok[j]) {
          const int n = nb + j * 16 + 4 * q;
          if (EPI == EPI_RESID) v = ld4(p.res + rows[i].off + n);
          if (EPI == EPI_DGELU) v = ld4bf(p.aux + rows[i].off + n);
          if (EPI == EPI_ACC) v = ld4(reinterpret_cast<const float*>(p.C) + rows[i].off + n);
          if (EPI == EPI_EMBED) {
            const int m = mb + i * 16 + 4 * g + x;
            const int patch = m - rows[i].b * p.tokens;
            v = ld4(p.pos + (size_t)(patch + 1) * p.emb_dim + n) +
                ld4(p.temb + (size_t)p.tsteps[rows[i].b] * p.emb_dim + n);
          }
        }
        pre[i][j] = v;
      }
  }

  __device__ __forceinline__ void finish(const GemmParams& p, const f32x4 (&acc_in)[FM][FN], int li) {
    const int x = li & 3;
    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = quad_transpose(acc_in[i][j], x);
    uint32_t salt_drop = 0, salt_dp = 0;
    if (p.thr_drop) salt_drop = site_salt(p.rng, p.site_drop);
    if (p.thr_dp) salt_dp = site_salt(p.rng, p.site_dp);
    const bool fold = FC && p.ln_st != nullptr;
    const bool prod = FP && p.st_out != nullptr;
    float2 ms[FM];
    constexpr int SL = FN / 2;  // 32-column statistics slots per wave
    float2 part[FM][SL];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      if (fold) {  // the row's slots: lane-local, then across the 4 lanes of the row (fixed order)
        float2 t = lnst[i][0];
#pragma unroll
        for (int k = 1; k < LN_MAX_SLOTS / 4; ++k) t = f2add(t, lnst[i][k]);
        t = f2add(t, f2xor<4>(t));
        t = f2add(t, f2xor<8>(t));
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
        const long long idx = rows[i].off + cols[j];
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
          st4(reinterpret_cast<float*>(p.C) + idx, pre[i][j] + v);
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
            part[i][j / 2] = f2add(part[i][j / 2], make_float2((v[0] + v[1]) + (v[2] + v[3]),
                                                               (v[0] * v[0] + v[1] * v[1]) + (v[2] * v[2] + v[3] * v[3])));
            st4bf(p.xb_out + idx, v);
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
          st4bf(reinterpret_cast<bf16*>(p.C2) + idx, h);
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
            part[i][j / 2] = f2add(part[i][j / 2], make_float2((v[0] + v[1]) + (v[2] + v[3]),
                                                               (v[0] * v[0] + v[1] * v[1]) + (v[2] * v[2] + v[3] * v[3])));
            st4bf(p.xb_out + idx, v);
          }
        }
      }
    }
    if (prod) {
      // the 4 lanes of a row (q = 0..3: lanes x, x+4, x+8, x+12 of the 16-lane
      // group) hold 32 consecutive columns per slot: reduce, one float2 store per
      // (row, slot)
      const int np_out = p.N / LN_SLOT;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int sl = 0; sl < SL; ++sl) {
          float2 t = part[i][sl];
          t = f2add(t, f2xor<4>(t));
          t = f2add(t, f2xor<8>(t));
          if ((li >> 2) == 0 && rowm[i] >= 0)
            *reinterpret_cast<float2*>(p.st_out + 2 * ((size_t)fold_token_row<EPI>(p, rowm[i]) * np_out +
                                                       colbase / LN_SLOT + sl)) = t;
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
  if (!UsesVecEpi<EPI>::value || p.debug == 3) run_epilogue_scalar<EPI, FM, FN>(p, acc, mb, nb, g, li);
  else run_epilogue_vec<EPI, FM, FN>(p, acc, mb, nb, g, li);
}

template <int BM, int BN, int WM, int WN, bool AT, bool BT, int EPI>
__global__ __launch_bounds__(256) void gemm_kernel(GemmParams p) {
  static_assert(WM * WN == 4, "4 waves");
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16;
  constexpr bool PERM = AT || BT;
  using SA = Stage<BM, AT>;
  using SB = Stage<BN, BT>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int STAGE_BYTES = SA::BYTES + SB::BYTES;

  const int tiles_n = (p.N + BN - 1) / BN;
  const int tiles_m = (p.M + BM - 1) / BM;
  const int nwg = tiles_m * tiles_n;
  int bid = blockIdx.x;
  {  // bijective XCD-aware remap: blocks b, b+8 share an XCD -> give each XCD a contiguous tile range
    const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7, idx = bid >> 3;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
  }
  const int tm = bid / tiles_n, tn = bid - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  const int total_kt = (p.K + BK - 1) / BK;
  const int kt0 = blockIdx.z * p.ktiles_per_split;
  const int kt1 = min(total_kt, kt0 + p.ktiles_per_split);

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int g = lane >> 4, li = lane & 15;

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fused bias-gradient row sums of A (wgrad): one extra MFMA vs an all-ones fragment
  const bool do_db = (EPI == EPI_ATOMIC) && AT && (p.bias != nullptr) && (tn == 0) && (wn == 0);
  f32x4 dbacc[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) dbacc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = f2bf(1.f);

  SA sa;
  SB sb;
  if (kt0 < kt1) {
    sa.load(p.A, p.lda, m0, p.M, kt0 * BK, p.K);
    sb.load(p.B, p.ldb, n0, p.N, kt0 * BK, p.K);
    sa.store(smem);
    sb.store(smem + SA::BYTES);
  }
  __syncthreads();

  int cur = 0;
  for (int kt = kt0; kt < kt1; ++kt) {
    const bool more = kt + 1 < kt1;
    if (more) {
      sa.load(p.A, p.lda, m0, p.M, (kt + 1) * BK, p.K);
      sb.load(p.B, p.ldb, n0, p.N, (kt + 1) * BK, p.K);
    }
    const char* la = smem + cur * STAGE_BYTES;
    const char* lb = la + SA::BYTES;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int r = wm * TM + i * 16;
        if (AT) af[i] = frag_t<SA::STRIDE_T>(la, r, s, lane);
        else if (PERM) af[i] = frag_k_perm(la, r + li, s, g);
        else af[i] = frag_k(la, r + li, s, g);
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int r = wn * TN + j * 16;
        if (BT) bfr[j] = frag_t<SB::STRIDE_T>(lb, r, s, lane);
        else if (PERM) bfr[j] = frag_k_perm(lb, r + li, s, g);
        else bfr[j] = frag_k(lb, r + li, s, g);
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
      if (EPI == EPI_ATOMIC && AT && do_db) {
#pragma unroll
        for (int i = 0; i < FM; ++i) dbacc[i] = mfma16(af[i], ones, dbacc[i]);
      }
    }
    if (more) {
      sa.store(smem + (cur ^ 1) * STAGE_BYTES);
      sb.store(smem + (cur ^ 1) * STAGE_BYTES + SA::BYTES);
    }
    __syncthreads();
    cur ^= 1;
  }

  if (EPI == EPI_ATOMIC && AT && do_db && li == 0) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * TM + i * 16 + 4 * g + r;
        if (m < p.M) atomicAdd(const_cast<float*>(p.bias) + m, dbacc[i][r]);
      }
  }

  run_epilogue<EPI, FM, FN>(p, acc, m0 + wm * TM, n0 + wn * TN, g, li);
}


// ============================================================================ LDS-DMA ring variant
// Operand tiles go global -> LDS with bounds-checked `buffer_load_dwordx4 ... lds`
// (no VGPR staging; rows past the end of a tensor read as zero, so ragged M / K
// tails need no masking), up to S-1 K-tiles in flight behind counted
// `s_waitcnt vmcnt(N)` and ONE raw s_barrier per K-tile (a __syncthreads would
// emit vmcnt(0) and drain the ring).  LDS images (128-B rows, 1-KiB DMA pieces
// = 8 rows each, swizzle applied on the per-lane SOURCE address):
//   k-contiguous operand  [rows][64 k]  chunk' = chunk ^ ((row>>1)&7)
//   transposed operand    [64 k][64]    chunk' = chunk ^ (row & 6)   (tr-read conflict-free)
template <int BM, int BN, int WM, int WN, bool AT, bool BT, int EPI, int S>
__device__ __forceinline__ void gemm_dma_body(const GemmParams& p, int tm, int tn) {
  static_assert(WM * WN == 4, "4 waves");
  static_assert(!AT || BM == 64, "transposed A needs BM == 64");
  static_assert(!BT || BN == 64, "transposed B needs BN == 64");
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16;
  constexpr bool PERM = AT || BT;
  using OA = DmaOperand<BM, AT>;
  using OB = DmaOperand<BN, BT>;
  constexpr int STAGE = OA::BYTES + OB::BYTES;
  constexpr int LPT = OA::PER_WAVE + OB::PER_WAVE;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int m0 = tm * BM, n0 = tn * BN;
  const int total_kt = (p.K + BK - 1) / BK;
  const int kt0 = blockIdx.z * p.ktiles_per_split;
  const int nk = min(total_kt, kt0 + p.ktiles_per_split) - kt0;
  if (nk <= 0) return;  // empty split slice (grouped launches); no barrier reached

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int g = lane >> 4, li = lane & 15;

  OA oa;
  OB ob;
  // stored A: non-T [M][lda] (rows M) ; T [K][lda] (rows K).  Same for B with N.
  oa.init(p.A, p.lda, AT ? p.K : p.M, m0, wave, lane);
  ob.init(p.B, p.ldb, BT ? p.K : p.N, n0, wave, lane);

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // fused bias gradient (wgrad): row sums of A via one extra MFMA against an
  // all-ones fragment per k-step, in the waves of the first column tile only
  constexpr bool WG = (EPI == EPI_ATOMIC || EPI == EPI_ACC) && AT;
  const bool do_db = WG && (p.bias != nullptr) && (tn == 0) && (wn == 0);
  f32x4 dbacc[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) dbacc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = f2bf(1.f);

#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (s < nk) {
      oa.issue(smem + s * STAGE, kt0 + s, wave);
      ob.issue(smem + s * STAGE + OA::BYTES, kt0 + s, wave);
    }
  // epilogue operands in flight behind the first operand tiles (see VecEpi)
  constexpr bool VEC = UsesVecEpi<EPI>::value;
  VecEpi<EPI, FM, FN> ep;
  if (VEC && p.debug != 3) ep.prefetch(p, m0 + wm * TM, n0 + wn * TN, g, li);

  // main loop; the bias-gradient MFMA variant is a separate instantiation so the
  // loop carries no per-k-step branch (one made hipcc shuffle the accumulators
  // between AGPRs and VGPRs every iteration)
  auto mainloop = [&](auto db_tag) {
    constexpr bool DB = decltype(db_tag)::value;
    for (int kt = 0; kt < (p.debug == 2 ? 0 : nk); ++kt) {
      const int rem = min(S - 2, nk - 1 - kt);
      vm_wait_rem<LPT>(rem);
      raw_barrier();
      if (kt + S - 1 < nk) {
        const int st = (kt + S - 1) % S;
        oa.issue(smem + st * STAGE, kt0 + kt + S - 1, wave);
        ob.issue(smem + st * STAGE + OA::BYTES, kt0 + kt + S - 1, wave);
      }
      const char* la = smem + (kt % S) * STAGE;
      const char* lb = la + OA::BYTES;
      // transposed operands: the reads of BOTH 32-deep k-steps are issued up
      // front (inline asm, see frag_t_swz_issue); k-step 0 waits only for its own
      TrFrag ta[2][FM], tb[2][FN];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
#pragma unroll
        for (int i = 0; i < FM; ++i)
          if (AT) ta[s][i] = frag_t_swz_issue(la, wm * TM + i * 16, s, lane);
#pragma unroll
        for (int j = 0; j < FN; ++j)
          if (BT) tb[s][j] = frag_t_swz_issue(lb, wn * TN + j * 16, s, lane);
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 af[FM], bfr[FN];
        if (AT || BT) {
          if (s == 0) {
            // reads issued after k-step 0's: 2 per transposed fragment
            constexpr int LATER = 2 * ((AT ? FM : 0) + (BT ? FN : 0));
            static_assert(LATER < 16, "lgkmcnt is 4 bits");
#pragma unroll
            for (int i = 0; i < FM; ++i)
              if (AT) af[i] = frag_t_fence_n<LATER>(ta[0][i]);
#pragma unroll
            for (int j = 0; j < FN; ++j)
              if (BT) bfr[j] = frag_t_fence_n<LATER>(tb[0][j]);
          } else {
#pragma unroll
            for (int i = 0; i < FM; ++i)
              if (AT) af[i] = frag_t_fence_n<0>(ta[1][i]);
#pragma unroll
            for (int j = 0; j < FN; ++j)
              if (BT) bfr[j] = frag_t_fence_n<0>(tb[1][j]);
          }
        }
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int r = wm * TM + i * 16;
          if (AT) continue;
          if (PERM) af[i] = frag_k_perm(la, r + li, s, g);
          else af[i] = frag_k(la, r + li, s, g);
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int r = wn * TN + j * 16;
          if (BT) continue;
          if (PERM) bfr[j] = frag_k_perm(lb, r + li, s, g);
          else bfr[j] = frag_k(lb, r + li, s, g);
        }
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
        if (DB) {
#pragma unroll
          for (int i = 0; i < FM; ++i) dbacc[i] = mfma16(af[i], ones, dbacc[i]);
        }
      }
    }
  };
  if (WG && do_db) mainloop(std::true_type{});
  else mainloop(std::false_type{});

  if (p.debug == 1) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) t += acc[i][j][0] + acc[i][j][3];
    if (t == 1234.5f) reinterpret_cast<float*>(p.C)[0] = t;
    return;
  }
  if (WG && do_db && li == 0) {
    float* db = const_cast<float*>(p.bias);
    float old[FM][4];
#pragma unroll
    for (int i = 0; i < FM; ++i)  // all loads first (see the epilogue note)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * TM + i * 16 + 4 * g + r;
        old[i][r] = (EPI == EPI_ACC && m < p.M) ? db[m] : 0.f;
      }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * TM + i * 16 + 4 * g + r;
        if (m < p.M) {
          if (EPI == EPI_ATOMIC) atomicAdd(db + m, dbacc[i][r]);
          else db[m] = old[i][r] + dbacc[i][r];
        }
      }
  }

  if (VEC && p.debug != 3) ep.finish(p, acc, li);
  else run_epilogue_scalar<EPI, FM, FN>(p, acc, m0 + wm * TM, n0 + wn * TN, g, li);
}

template <int BM, int BN, int WM, int WN, bool AT, bool BT, int EPI, int S>
__global__ __launch_bounds__(256) void gemm_dma_kernel(GemmParams p) {
  const int tiles_n = (p.N + BN - 1) / BN;
  const int tiles_m = (p.M + BM - 1) / BM;
  const int bid = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int tm = bid / tiles_n;
  gemm_dma_body<BM, BN, WM, WN, AT, BT, EPI, S>(p, tm, bid - tm * tiles_n);
}

// Grouped weight-gradient GEMM: up to WG_MAX independent dW = dy^T x problems
// (the four linears of a transformer block, plus the head / patch embedding)
// in ONE launch.  Tiles of all problems share the grid (XCD-aware), blockIdx.z
// is the token (K) split of every problem.
template <int EPI, int S>
__global__ __launch_bounds__(256) void gemm_wgrad_group_kernel(WgradGroup gp) {
  const int bid = xcd_remap(blockIdx.x, gp.tile_start[gp.n]);
  int i = 0;
#pragma unroll
  for (int j = 1; j < WG_MAX; ++j)
    if (j < gp.n && bid >= gp.tile_start[j]) i = j;
  const GemmParams& p = gp.p[i];
  const int tiles_n = (p.N + 63) / 64;
  const int local = bid - gp.tile_start[i];
  const int tm = local / tiles_n;
  gemm_dma_body<64, 64, 2, 2, true, true, EPI, S>(p, tm, local - tm * tiles_n);
}

// Grouped weight gradient, 8 waves: the two halves of the workgroup (waves 0-3
// and 4-7) reduce the two halves of the token range of the SAME 64x64 output
// tile through their own LDS-DMA rings (2 x 64 KiB), then half 1 hands its
// accumulators to half 0 through LDS and half 0 writes the tile with a plain
// read-add-write epilogue.  Twice the operand bytes in flight per CU (what the
// 2-way atomic split bought) without fp32 atomics.  Measured slower than the
// 2-way atomic split (18.1 vs 15.0 us per block group): opt-in only.
template <int S>
__global__ __launch_bounds__(512) void gemm_wgrad_group8_kernel(WgradGroup gp) {
  constexpr int BMN = 64, FM = 2, FN = 2;
  using OP = DmaOperand<64, true>;
  constexpr int STAGE = 2 * OP::BYTES;
  constexpr int LPT = 2 * OP::PER_WAVE;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int bid = xcd_remap(blockIdx.x, gp.tile_start[gp.n]);
  int pi = 0;
#pragma unroll
  for (int j = 1; j < WG_MAX; ++j)
    if (j < gp.n && bid >= gp.tile_start[j]) pi = j;
  const GemmParams& p = gp.p[pi];
  const int tiles_n = (p.N + 63) / 64;
  const int local = bid - gp.tile_start[pi];
  const int tm = local / tiles_n, tn = local - tm * tiles_n;
  const int m0 = tm * BMN, n0 = tn * BMN;

  const int half = __builtin_amdgcn_readfirstlane(threadIdx.x >> 8);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane((threadIdx.x >> 6) & 3);
  const int wm = wave >> 1, wn = wave & 1;
  const int g = lane >> 4, li = lane & 15;
  char* ring = smem + half * S * STAGE;

  const int total_kt = (p.K + BK - 1) / BK;
  const int h0 = (total_kt + 1) / 2;
  const int kt0 = half ? h0 : 0;
  const int nk = half ? total_kt - h0 : h0;
  const int niter = h0;  // both halves run the same number of barriers

  OP oa, ob;
  oa.init(p.A, p.lda, p.K, m0, wave, lane);
  ob.init(p.B, p.ldb, p.K, n0, wave, lane);

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool do_db = (p.bias != nullptr) && (tn == 0) && (wn == 0);
  f32x4 dbacc[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) dbacc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = f2bf(1.f);

#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (s < nk) {
      oa.issue(ring + s * STAGE, kt0 + s, wave);
      ob.issue(ring + s * STAGE + OP::BYTES, kt0 + s, wave);
    }
  for (int kt = 0; kt < niter; ++kt) {
    const bool active = kt < nk;
    if (active) vm_wait_rem<LPT>(min(S - 2, nk - 1 - kt));
    raw_barrier();
    if (!active) continue;
    if (kt + S - 1 < nk) {
      const int st = (kt + S - 1) % S;
      oa.issue(ring + st * STAGE, kt0 + kt + S - 1, wave);
      ob.issue(ring + st * STAGE + OP::BYTES, kt0 + kt + S - 1, wave);
    }
    const char* la = ring + (kt % S) * STAGE;
    const char* lb = la + OP::BYTES;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = frag_t_swz(la, wm * 32 + i * 16, s, lane);
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = frag_t_swz(lb, wn * 32 + j * 16, s, lane);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
      if (do_db) {
#pragma unroll
        for (int i = 0; i < FM; ++i) dbacc[i] = mfma16(af[i], ones, dbacc[i]);
      }
    }
  }
  // hand half 1's partial tile to half 0 through LDS (rings are done)
  __syncthreads();
  f32x4* xch = reinterpret_cast<f32x4*>(smem);  // [FM*FN + FM][256 lanes]
  const int t = threadIdx.x & 255;
  if (half == 1) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) xch[(i * FN + j) * 256 + t] = acc[i][j];
#pragma unroll
    for (int i = 0; i < FM; ++i) xch[(FM * FN + i) * 256 + t] = dbacc[i];
  }
  __syncthreads();
  if (half == 1) return;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] += xch[(i * FN + j) * 256 + t];
#pragma unroll
  for (int i = 0; i < FM; ++i) dbacc[i] += xch[(FM * FN + i) * 256 + t];

  if (do_db && li == 0) {
    float* db = const_cast<float*>(p.bias);
    float old[FM][4];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 32 + i * 16 + 4 * g + r;
        old[i][r] = m < p.M ? db[m] : 0.f;
      }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 32 + i * 16 + 4 * g + r;
        if (m < p.M) db[m] = old[i][r] + dbacc[i][r];
      }
  }
  run_epilogue_vec<EPI_ACC, FM, FN>(p, acc, m0 + wm * 32, n0 + wn * 32, g, li);
}
template __global__ void gemm_wgrad_group8_kernel<4>(WgradGroup);

template <int BM, int BN, int WM, int WN, bool AT, bool BT, int EPI>
static void launch_dma(GemmParams p, int splits, hipStream_t stream) {
  const int total_kt = (p.K + BK - 1) / BK;
  p.ktiles_per_split = (total_kt + splits - 1) / splits;
  splits = (total_kt + p.ktiles_per_split - 1) / p.ktiles_per_split;
  const int tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  // keep every workgroup of the grid co-resident (one round): a 4-stage ring
  // allows 160 KiB / (4 x stage) workgroups per CU, a 3-stage ring 4/3 of that
  constexpr int stage = BM * 128 + BN * 128;
  constexpr int per_cu4 = (160 * 1024) / (4 * stage);
  static const bool force_s4 = getenv_flag("DDIM_COLD_GEMM_S4");
  if (tiles * splits > 256 * per_cu4 && p.ktiles_per_split <= 8 && !force_s4)
    hipLaunchKernelGGL((gemm_dma_kernel<BM, BN, WM, WN, AT, BT, EPI, 3>), dim3(tiles, 1, splits), dim3(256),
                       3 * stage, stream, p);
  else
    hipLaunchKernelGGL((gemm_dma_kernel<BM, BN, WM, WN, AT, BT, EPI, 4>), dim3(tiles, 1, splits), dim3(256),
                       4 * stage, stream, p);
}

template <int BM, int BN, int WM, int WN, bool AT, bool BT, int EPI>
static void launch_cfg(GemmParams p, int splits, hipStream_t stream) {
  using SA = Stage<BM, AT>;
  using SB = Stage<BN, BT>;
  const int lds = 2 * (SA::BYTES + SB::BYTES);
  const int total_kt = (p.K + BK - 1) / BK;
  p.ktiles_per_split = (total_kt + splits - 1) / splits;
  splits = (total_kt + p.ktiles_per_split - 1) / p.ktiles_per_split;
  const int tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  dim3 grid(tiles, 1, splits);
  hipLaunchKernelGGL((gemm_kernel<BM, BN, WM, WN, AT, BT, EPI>), grid, dim3(256), lds, stream, p);
}

// (tag dispatch instead of `if constexpr`: hipcc 7.2 silently drops the host
// stub of a kernel template first referenced inside an if-constexpr branch)
// tile configs: 0 = 32x64, 1 = 64x64, 2 = 128x64, 3 = 128x128 (4 waves, 2x2)
template <bool AT, bool BT, int EPI>
struct DmaTiles {
  static void launch(GemmParams p, int splits, hipStream_t stream, int cfg) {
    switch (cfg) {
      case 0: launch_dma<32, 64, 2, 2, AT, BT, EPI>(p, splits, stream); break;
      case 1: launch_dma<64, 64, 2, 2, AT, BT, EPI>(p, splits, stream); break;
      case 2: launch_dma<128, 64, 2, 2, AT, BT, EPI>(p, splits, stream); break;
      default: launch_dma<128, 128, 2, 2, AT, BT, EPI>(p, splits, stream); break;
    }
  }
};
template <int EPI>
struct DmaTiles<false, true, EPI> {  // transposed B (dgrad): BN = 64
  static void launch(GemmParams p, int splits, hipStream_t stream, int cfg) {
    switch (cfg) {
      case 0: launch_dma<32, 64, 2, 2, false, true, EPI>(p, splits, stream); break;
      case 1: launch_dma<64, 64, 2, 2, false, true, EPI>(p, splits, stream); break;
      default: launch_dma<128, 64, 2, 2, false, true, EPI>(p, splits, stream); break;
    }
  }
};
template <bool BT, int EPI>
struct DmaTiles<true, BT, EPI> {  // transposed A (wgrad): 64x64
  static void launch(GemmParams p, int splits, hipStream_t stream, int) {
    launch_dma<64, 64, 2, 2, true, BT, EPI>(p, splits, stream);
  }
};

// Tile choice: 64x64 when that alone gives ~1 workgroup per CU, else 32x64.
// A cost model "operand bytes per CU" (one CU ingests ~80 GB/s of operand tiles,
// tools/ub_stream.hip) that picks 128x64 / 128x128 for the big shapes measured
// SLOWER everywhere (qkv 2080x1152x384: 11.9 us at 128x128 vs 7.5 at 64x64;
// train step -10%): more, smaller workgroups hide latency better than fewer
// bytes help.  It stays available as DDIM_COLD_GEMM_TILE_MODEL=1, and
// DDIM_COLD_GEMM_TILE=0..3 forces a tile.  The LDS-DMA ring needs K % 64 == 0
// for k-contiguous operands (transposed operands get zero rows past K from the
// buffer bounds check).
static int pick_tiles(int M, int N, int K, int splits, bool at, bool bt) {
  static const int forced = [] {
    const char* e = getenv("DDIM_COLD_GEMM_TILE");
    return e ? atoi(e) : -1;
  }();
  static const bool model = getenv_flag("DDIM_COLD_GEMM_TILE_MODEL");
  if (at) return 1;
  if (forced >= 0) return bt && forced > 2 ? 2 : forced;
  if (!model) return ((M + 63) / 64) * ((N + 63) / 64) * splits >= 240 ? 1 : 0;
  const int nk = ((K + 63) / 64 + splits - 1) / splits;
  const int bms[4] = {32, 64, 128, 128}, bns[4] = {64, 64, 64, 128};
  const int ncfg = bt ? 3 : 4;
  int best = 0;
  long long best_cost = -1, best_tiles = 0;
  for (int c = 0; c < ncfg; ++c) {
    const long long tiles = (long long)((M + bms[c] - 1) / bms[c]) * ((N + bns[c] - 1) / bns[c]) * splits;
    const long long per_cu = (tiles + 255) / 256;
    const long long cost = per_cu * (bms[c] + bns[c]) * 128LL * nk;
    if (best_cost < 0 || cost < best_cost || (cost == best_cost && tiles > best_tiles)) {
      best = c;
      best_cost = cost;
      best_tiles = tiles;
    }
  }
  return best;
}

template <bool AT, bool BT, int EPI>
static void launch_auto(GemmParams p, int splits, hipStream_t stream) {
  const bool dma_ok = (AT || BT || p.K % 64 == 0) && (AT || p.K % 64 == 0) && !dma_disabled();
  if (dma_ok) {
    DmaTiles<AT, BT, EPI>::launch(p, splits, stream, pick_tiles(p.M, p.N, p.K, splits, AT, BT));
    return;
  }
  const int tiles64 = ((p.M + 63) / 64) * ((p.N + 63) / 64);
  const bool big = tiles64 * splits >= 240 || AT;
  if (big) launch_cfg<64, 64, 2, 2, AT, BT, EPI>(p, splits, stream);
  else launch_cfg<32, 64, 2, 2, AT, BT, EPI>(p, splits, stream);
}

// Explicit instantiations: hipcc 7.2 intermittently fails to emit host launch
// stubs for implicitly instantiated kernel templates (undefined
// __device_stub__ at dlopen); build.py also checks the .so for that.
#define DC_INST_DMAT(BM, BN, AT, BT, EPI)                                               \
  template __global__ void gemm_dma_kernel<BM, BN, 2, 2, AT, BT, EPI, 4>(GemmParams); \
  template __global__ void gemm_dma_kernel<BM, BN, 2, 2, AT, BT, EPI, 3>(GemmParams);
#define DC_INST_DMA(BM, AT, BT, EPI) DC_INST_DMAT(BM, 64, AT, BT, EPI)
#define DC_INST_DMA2(AT, BT, EPI) \
  DC_INST_DMA(64, AT, BT, EPI) DC_INST_DMA(32, AT, BT, EPI) DC_INST_DMA(128, AT, BT, EPI)
#define DC_INST_DMA3(EPI) DC_INST_DMA2(false, false, EPI) DC_INST_DMAT(128, 128, false, false, EPI)
DC_INST_DMA3(EPI_BF16)
DC_INST_DMA3(EPI_F32)
DC_INST_DMA3(EPI_QKV)
DC_INST_DMA3(EPI_RESID)
DC_INST_DMA3(EPI_GELU)
DC_INST_DMA3(EPI_HEAD)
DC_INST_DMA3(EPI_EMBED)
DC_INST_DMA2(false, true, EPI_BF16)
DC_INST_DMA2(false, true, EPI_F32)
DC_INST_DMA2(false, true, EPI_DGELU)
DC_INST_DMA(64, true, true, EPI_ATOMIC)
template __global__ void gemm_wgrad_group_kernel<EPI_ATOMIC, 4>(WgradGroup);
template __global__ void gemm_wgrad_group_kernel<EPI_ACC, 4>(WgradGroup);
template __global__ void gemm_wgrad_group_kernel<EPI_ATOMIC, 6>(WgradGroup);
template __global__ void gemm_wgrad_group_kernel<EPI_ACC, 6>(WgradGroup);
template __global__ void gemm_wgrad_group_kernel<EPI_ATOMIC, 8>(WgradGroup);
template __global__ void gemm_wgrad_group_kernel<EPI_ACC, 8>(WgradGroup);

}  // namespace dc

// ============================================================================ host API
using namespace dc;

static GemmParams base_params(const GemmArgs& a) {
  GemmParams p{};
  static const int dbg = [] {
    const char* e = getenv("DDIM_COLD_GEMM_DEBUG");
    return e ? atoi(e) : 0;
  }();
  p.debug = dbg;
  p.A = reinterpret_cast<const bf16*>(a.A);
  p.B = reinterpret_cast<const bf16*>(a.B);
  p.M = a.M; p.N = a.N; p.K = a.K;
  p.lda = a.lda; p.ldb = a.ldb;
  p.C = a.C; p.ldc = a.ldc;
  p.bias = a.bias;
  p.res = a.res; p.C2 = a.C2;
  p.aux = reinterpret_cast<const bf16*>(a.aux);
  p.rng = a.rng;
  p.site_drop = a.site_drop;
  p.thr_drop = drop_threshold_host(a.p_drop);
  p.scale_drop = a.p_drop > 0 ? 1.f / (1.f - (float)a.p_drop) : 1.f;
  p.site_dp = a.site_dp;
  p.thr_dp = drop_threshold_host(a.p_dp);
  p.scale_dp = a.p_dp > 0 ? 1.f / (1.f - (float)a.p_dp) : 1.f;
  p.tokens = a.tokens; p.batch = a.batch; p.heads = a.heads; p.hd = a.hd;
  p.chans = a.chans; p.img_h = a.img_h; p.img_w = a.img_w; p.patch = a.patch;
  p.pos = a.pos; p.temb = a.temb; p.tsteps = a.tsteps; p.emb_dim = a.emb_dim;
  p.coef = a.coef; p.head_mode = a.head_mode;
  p.loss_beta = a.loss_beta; p.loss_inv_n = a.loss_inv_n; p.loss_parts = a.loss_parts;
  p.split_stride = a.split_stride;
  p.ln_st = a.ln_st; p.ln_c = a.ln_c; p.ln_eps = a.ln_eps; p.ln_mean = a.ln_mean; p.ln_rstd = a.ln_rstd;
  p.st_out = a.st_out; p.xb_out = reinterpret_cast<bf16*>(a.xb_out);
  return p;
}

static void check_vec(const GemmParams& p, int epi) {
  // the vector epilogue stores 4 consecutive output columns per lane
  if (epi != EPI_HEAD && (p.N % 4 != 0 || (epi == EPI_QKV && p.hd % 4 != 0) || (epi == EPI_EMBED && p.emb_dim % 4 != 0)))
    throw std::runtime_error("gemm: output width must be a multiple of 4");
}

void gemm_nt(const GemmArgs& a, int epi, hipStream_t stream) {
  GemmParams p = base_params(a);
  check_vec(p, epi);
  switch (epi) {
    case EPI_BF16: launch_auto<false, false, EPI_BF16>(p, 1, stream); break;
    case EPI_F32: launch_auto<false, false, EPI_F32>(p, 1, stream); break;
    case EPI_QKV: launch_auto<false, false, EPI_QKV>(p, 1, stream); break;
    case EPI_RESID: launch_auto<false, false, EPI_RESID>(p, 1, stream); break;
    case EPI_GELU: launch_auto<false, false, EPI_GELU>(p, 1, stream); break;
    case EPI_HEAD: launch_auto<false, false, EPI_HEAD>(p, 1, stream); break;
    case EPI_EMBED: launch_auto<false, false, EPI_EMBED>(p, 1, stream); break;
    default: throw std::runtime_error("gemm_nt: unsupported epilogue");
  }
}

int gemm_nt_grid(int M, int N, int K) {
  // mirrors launch_auto<false, false, *> (one split)
  const bool dma_ok = K % 64 == 0 && !dma_disabled();
  int bm = 64, bn = 64;
  if (dma_ok) {
    const int cfg = pick_tiles(M, N, K, 1, false, false);
    const int bms[4] = {32, 64, 128, 128}, bns[4] = {64, 64, 64, 128};
    bm = bms[cfg < 0 ? 0 : (cfg > 3 ? 3 : cfg)];
    bn = bns[cfg < 0 ? 0 : (cfg > 3 ? 3 : cfg)];
  } else if (((M + 63) / 64) * ((N + 63) / 64) < 240) {
    bm = 32;
  }
  return ((M + bm - 1) / bm) * ((N + bn - 1) / bn);
}

void gemm_dgrad(const GemmArgs& a, int epi, hipStream_t stream) {
  GemmParams p = base_params(a);
  check_vec(p, epi);
  switch (epi) {
    case EPI_BF16:
    case EPI_F32: {
      // K split: slice z writes its partial product to C + z * split_stride
      // (every slice non-empty; the consumer sums the slices)
      const int kt = (p.K + 63) / 64;
      const int splits = std::max(1, std::min(a.splits, kt));
      if (splits != a.splits && a.splits > 1) throw std::runtime_error("gemm_dgrad: more K slices than k-tiles");
      if (splits > 1 && (p.bias || (kt + splits - 1) / splits * (splits - 1) >= kt))
        throw std::runtime_error("gemm_dgrad: K split needs no bias and a non-empty last slice");
      if (epi == EPI_BF16) launch_auto<false, true, EPI_BF16>(p, splits, stream);
      else launch_auto<false, true, EPI_F32>(p, splits, stream);
    } break;
    case EPI_DGELU: launch_auto<false, true, EPI_DGELU>(p, 1, stream); break;
    default: throw std::runtime_error("gemm_dgrad: unsupported epilogue");
  }
}

void gemm_wgrad(const GemmArgs& a, int splits, hipStream_t stream) {
  GemmParams p = base_params(a);
  check_vec(p, EPI_ATOMIC);
  launch_auto<true, true, EPI_ATOMIC>(p, splits, stream);
}

void gemm_wgrad_group(const GemmArgs* probs, int n, int splits, hipStream_t stream) {
  if (n < 1 || n > WG_MAX) throw std::runtime_error("gemm_wgrad_group: 1..6 problems per launch");
  WgradGroup gp{};
  gp.n = n;
  int tiles = 0;
  for (int i = 0; i < n; ++i) {
    gp.p[i] = base_params(probs[i]);
    check_vec(gp.p[i], EPI_ATOMIC);
    const int kt = (gp.p[i].K + BK - 1) / BK;
    gp.p[i].ktiles_per_split = (kt + std::max(splits, 1) - 1) / std::max(splits, 1);
    gp.tile_start[i] = tiles;
    tiles += ((gp.p[i].M + 63) / 64) * ((gp.p[i].N + 63) / 64);
  }
  for (int i = n; i <= WG_MAX; ++i) gp.tile_start[i] = tiles;
  constexpr int lds = 4 * (64 * 128 + 64 * 128);
  if (splits == 0) {  // 8-wave two-half kernel (no atomics)
    static bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_wgrad_group8_kernel<4>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 2 * lds) == hipSuccess;
    (void)attr;
    hipLaunchKernelGGL(gemm_wgrad_group8_kernel<4>, dim3(tiles), dim3(512), 2 * lds, stream, gp);
    return;
  }
  // LDS-DMA ring depth (DDIM_COLD_WGRAD_S = 4 / 6 / 8): the token-reduction loop
  // is bound by operand bytes in flight per CU
  static const int ring = [] {
    const char* e = getenv("DDIM_COLD_WGRAD_S");
    const int v = e ? atoi(e) : 4;
    return v >= 8 ? 8 : v >= 6 ? 6 : 4;
  }();
  const int slds = ring * (64 * 128 + 64 * 128);
  auto go = [&](auto kern) {
    static_assert(true, "");
    if (slds > 65536)
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, slds);
    hipLaunchKernelGGL(kern, dim3(tiles, 1, std::max(splits, 1)), dim3(256), slds, stream, gp);
  };
  if (splits == 1) {
    if (ring == 8) go(gemm_wgrad_group_kernel<EPI_ACC, 8>);
    else if (ring == 6) go(gemm_wgrad_group_kernel<EPI_ACC, 6>);
    else go(gemm_wgrad_group_kernel<EPI_ACC, 4>);
  } else {
    if (ring == 8) go(gemm_wgrad_group_kernel<EPI_ATOMIC, 8>);
    else if (ring == 6) go(gemm_wgrad_group_kernel<EPI_ATOMIC, 6>);
    else go(gemm_wgrad_group_kernel<EPI_ATOMIC, 4>);
  }
}
