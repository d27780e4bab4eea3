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
};

constexpr int BK = 64;

__device__ __forceinline__ int swz(int r) { return (r >> 1) & 7; }

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

// fragment of a k-contiguous image, standard k order
__device__ __forceinline__ bf16x8 frag_k(const char* lds, int r, int s, int g) {
  const int chunk = 4 * s + g;
  return *reinterpret_cast<const bf16x8*>(lds + r * 128 + 16 * (chunk ^ swz(r)));
}
// fragment of a k-contiguous image, permuted k order
__device__ __forceinline__ bf16x8 frag_k_perm(const char* lds, int r, int s, int g) {
  const int ca = 4 * s + (g >> 1), cb = ca + 2;
  const int sub = 8 * (g & 1);
  const u32x2 lo = *reinterpret_cast<const u32x2*>(lds + r * 128 + 16 * (ca ^ swz(r)) + sub);
  const u32x2 hi = *reinterpret_cast<const u32x2*>(lds + r * 128 + 16 * (cb ^ swz(r)) + sub);
  u32x4 v = {lo[0], lo[1], hi[0], hi[1]};
  return __builtin_bit_cast(bf16x8, v);
}
template <int EPI>
__device__ __forceinline__ void epilogue(const GemmParams& p, int m, int n, float v, uint32_t salt_drop,
                                         uint32_t salt_dp) {
  if (EPI == EPI_BF16) {
    if (p.bias) v += p.bias[n];
    reinterpret_cast<bf16*>(p.C)[(size_t)m * p.ldc + n] = f2bf(v);
  } else if (EPI == EPI_F32) {
    if (p.bias) v += p.bias[n];
    reinterpret_cast<float*>(p.C)[(size_t)m * p.ldc + n] = v;
  } else if (EPI == EPI_ATOMIC) {
    atomicAdd(reinterpret_cast<float*>(p.C) + (size_t)m * p.ldc + n, v);
  } else if (EPI == EPI_QKV) {
    if (p.bias) v += p.bias[n];
    const int D = p.heads * p.hd;
    const int s = n / D, rem = n - s * D;
    const int h = rem / p.hd, d = rem - h * p.hd;
    const int b = m / p.tokens, tok = m - b * p.tokens;
    const size_t idx = ((((size_t)s * p.batch + b) * p.heads + h) * p.tokens + tok) * p.hd + d;
    reinterpret_cast<bf16*>(p.C)[idx] = f2bf(v);
  } else if (EPI == EPI_RESID) {
    if (p.bias) v += p.bias[n];
    const size_t idx = (size_t)m * p.N + n;
    if (p.thr_drop) v = dropout_keep(salt_drop, (uint32_t)idx, p.thr_drop) ? v * p.scale_drop : 0.f;
    if (p.thr_dp) {
      const int b = m / p.tokens;
      v = dropout_keep(salt_dp, (uint32_t)b, p.thr_dp) ? v * p.scale_dp : 0.f;
    }
    reinterpret_cast<float*>(p.C)[idx] = p.res[idx] + v;
  } else if (EPI == EPI_GELU) {
    if (p.bias) v += p.bias[n];
    const size_t idx = (size_t)m * p.N + n;
    reinterpret_cast<bf16*>(p.C)[idx] = f2bf(v);
    float h = gelu_f(v);
    if (p.thr_drop) h = dropout_keep(salt_drop, (uint32_t)idx, p.thr_drop) ? h * p.scale_drop : 0.f;
    reinterpret_cast<bf16*>(p.C2)[idx] = f2bf(h);
  } else if (EPI == EPI_DGELU) {
    const size_t idx = (size_t)m * p.N + n;
    if (p.thr_drop) v = dropout_keep(salt_drop, (uint32_t)idx, p.thr_drop) ? v * p.scale_drop : 0.f;
    v *= gelu_grad_f(bf2f(p.aux[idx]));
    reinterpret_cast<bf16*>(p.C)[idx] = f2bf(v);
  } else if (EPI == EPI_HEAD) {
    const int b = m / p.tokens, tok = m - b * p.tokens;
    if (tok == 0) return;
    if (p.bias) v += p.bias[n];
    const int P = p.patch;
    const int Wp = p.img_w / P;
    const int patch = tok - 1, hp = patch / Wp, wp = patch - hp * Wp;
    const int c = n % p.chans, ab = n / p.chans, a = ab / P, bb = ab - a * P;
    reinterpret_cast<float*>(p.C)[(((size_t)b * p.chans + c) * p.img_h + hp * P + a) * p.img_w + wp * P + bb] = v;
  } else if (EPI == EPI_EMBED) {
    // m = b*P + patch ; token row = b*(P+1) + 1 + patch
    const int Pn = p.tokens;  // patches per sample
    const int b = m / Pn, patch = m - b * Pn;
    const int tok = patch + 1;
    const size_t row = (size_t)b * (Pn + 1) + tok;
    v += p.bias[n] + p.pos[(size_t)tok * p.emb_dim + n] + p.temb[(size_t)p.tsteps[b] * p.emb_dim + n];
    const size_t idx = row * p.emb_dim + n;
    if (p.thr_drop) v = dropout_keep(salt_drop, (uint32_t)idx, p.thr_drop) ? v * p.scale_drop : 0.f;
    reinterpret_cast<float*>(p.C)[idx] = v;
  }
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

  // fused bias-gradient column sum (wgrad with AT: A image is [k][BM])
  const bool do_db = (EPI == EPI_ATOMIC) && AT && (p.bias != nullptr) && (tn == 0);
  float db_acc = 0.f;

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
    if (AT && do_db && threadIdx.x < BM) {
      const char* col = la + threadIdx.x * 2;
      float s = 0.f;
#pragma unroll 8
      for (int r = 0; r < BK; ++r) s += bf2f(*reinterpret_cast<const bf16*>(col + r * SA::STRIDE_T));
      db_acc += s;
    }
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
    }
    if (more) {
      sa.store(smem + (cur ^ 1) * STAGE_BYTES);
      sb.store(smem + (cur ^ 1) * STAGE_BYTES + SA::BYTES);
    }
    __syncthreads();
    cur ^= 1;
  }

  if (do_db && threadIdx.x < BM && m0 + (int)threadIdx.x < p.M) atomicAdd(const_cast<float*>(p.bias) + m0 + threadIdx.x, db_acc);

  uint32_t salt_drop = 0, salt_dp = 0;
  if (p.thr_drop) salt_drop = site_salt(p.rng, p.site_drop);
  if (p.thr_dp) salt_dp = site_salt(p.rng, p.site_dp);
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * TM + i * 16 + 4 * g + r;
        const int n = n0 + wn * TN + j * 16 + li;
        if (m < p.M && n < p.N) epilogue<EPI>(p, m, n, acc[i][j][r], salt_drop, salt_dp);
      }
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

// tile choice: 64x64 when it yields >= ~1 wave of workgroups per CU, else 32x64
template <bool AT, bool BT, int EPI>
static void launch_auto(GemmParams p, int splits, hipStream_t stream) {
  const int tiles64 = ((p.M + 63) / 64) * ((p.N + 63) / 64);
  if (tiles64 * splits >= 240) launch_cfg<64, 64, 2, 2, AT, BT, EPI>(p, splits, stream);
  else launch_cfg<32, 64, 2, 2, AT, BT, EPI>(p, splits, stream);
}

}  // namespace dc

// ============================================================================ host API
using namespace dc;

static GemmParams base_params(const GemmArgs& a) {
  GemmParams p{};
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
  return p;
}

void gemm_nt(const GemmArgs& a, int epi, hipStream_t stream) {
  GemmParams p = base_params(a);
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

void gemm_dgrad(const GemmArgs& a, int epi, hipStream_t stream) {
  GemmParams p = base_params(a);
  switch (epi) {
    case EPI_BF16: launch_auto<false, true, EPI_BF16>(p, 1, stream); break;
    case EPI_F32: launch_auto<false, true, EPI_F32>(p, 1, stream); break;
    case EPI_DGELU: launch_auto<false, true, EPI_DGELU>(p, 1, stream); break;
    default: throw std::runtime_error("gemm_dgrad: unsupported epilogue");
  }
}

void gemm_wgrad(const GemmArgs& a, int splits, hipStream_t stream) {
  GemmParams p = base_params(a);
  launch_auto<true, true, EPI_ATOMIC>(p, splits, stream);
}
