// Fused transformer MLP block for gfx950: fc1 -> GELU -> (dropout) -> fc2 ->
// (dropout, drop-path) + residual, in ONE launch (ViT.py:74-90 Mlp inside
// Block.forward ViT.py:132-138, with the preceding LayerNorm norm2 folded in).
//
//   x_out = x1 + DropPath(Dropout(fc2(Dropout(GELU(LN2(x1) W1^T + b1))) ))
//
// Why: at the sampler / training shapes (M = 2,080..4,160 token rows, D = H = 384)
// the two GEMMs of the unfused path are latency-bound launches (~10 us each for
// 1.2 GFLOP: six 64-deep k-tiles per 64x64 tile, 1.5 rounds of workgroups) and
// the hidden activation round-trips through memory between them.  Here a
// workgroup owns a panel of BM token rows for the WHOLE block:
//
//   * the panel's LayerNorm input (bf16 residual copy, BM x D) is DMA'd into LDS
//     once; fc1's hidden rows (BM x H, bf16) never leave LDS; fc2 reads them as
//     its A operand;
//   * the weights are ONE stream of 128-row x 64-deep tiles (fc1: H/128 column
//     chunks x D/64 k-tiles, then fc2: D/128 chunks x H/64) through an S-slot
//     LDS-DMA ring (`buffer_load ... lds`, swizzle on the source address, counted
//     vmcnt waits, one raw s_barrier per tile): S-1 tiles (up to 112 KiB) in
//     flight per CU, which is what bounds these low-intensity shapes (per-CU
//     L2 -> LDS ingest, MI355X_MICROARCH.md "ldsdma-fill");
//   * 4 waves; every wave covers all BM rows and 32 of the chunk's 128 columns
//     (v_mfma_f32_16x16x32_bf16), so one wave owns whole 32-column LayerNorm
//     statistics slots of the output rows;
//   * chunk epilogues: fc1 -> LayerNorm fold (rstd*(acc - mean*c) + b'), GELU,
//     dropout, bf16 into the LDS hidden image (+ u / h to memory when training);
//     fc2 -> bias, dropout, drop-path, residual (its fp32 rows DMA'd into the
//     dead A-image region at the chunk's first tile), fp32 + bf16 outputs and the
//     next LayerNorm's {sum, sum^2} slots.
//
// Same math, rounding points and dropout indices as linear_gelu_fwd +
// linear_residual_fwd (gemm.hip EPI_GELU / EPI_RESID with the LayerNorm fold);
// the output sums run in a different order (tests compare at fp32 tolerance).
#include "common.h"
#include "gemm_common.h"
#include "kernels.h"

namespace dc {

namespace {
constexpr int CW = 128;            // weight rows (output columns) per chunk
constexpr int WT = CW * 128;       // bytes of one ring slot: 128 rows x 64 k bf16
constexpr int WPIECES = WT / 4096; // 1-KiB DMA pieces per wave per weight tile (4)
__host__ __device__ constexpr int kib(int b) { return (b + 1023) / 1024 * 1024; }
__host__ __device__ inline int mlp_cst_bytes(int D, int H) { return kib(4 * H) * 2 + kib(4 * D); }
__host__ __device__ inline int mlp_st_bytes(int BM, int D) { return kib(BM * (D / 32) * 8); }
__host__ __device__ inline int mlp_lds_bytes(int BM, int S, int D, int H) {
  return mlp_cst_bytes(D, H) + mlp_st_bytes(BM, D) + BM * 2 * (D + H) + S * WT;
}
}  // namespace

template <int BM, int S, bool TRAIN>
__global__ __launch_bounds__(256) void mlp_fused_kernel(MlpArgs a) {
  constexpr int FM = BM / 16;  // row fragments per wave (every wave: all BM rows)
  constexpr int FN = 2;        // 2 x 16 columns per wave
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int D = a.D, H = a.H;
  const int KT1 = D / 64, KT2 = H / 64;
  const int NC1 = H / CW, NC2 = D / CW;
  const int T1 = NC1 * KT1, T = T1 + NC2 * KT2;
  const int np = D / 32;  // LayerNorm statistics slots per row
  // LDS: every operand and constant arrives by LDS-DMA, so the kernel issues no
  // global load the compiler would wait on (that wait would drain the ring)
  const float* cst = reinterpret_cast<const float*>(smem);  // c1[H] | b1[H] | b2[D]
  char* stimg = smem + mlp_cst_bytes(D, H);                   // [BM][np][2] f32 LN statistics
  char* aimg = stimg + mlp_st_bytes(BM, D);                   // KT1 x [BM][64] bf16; phase 2: residual [BM][128] f32
  char* himg = aimg + KT1 * BM * 128;                         // KT2 x [BM][64] bf16 hidden (post-GELU)
  char* ring = himg + KT2 * BM * 128;                         // S x [128][64] bf16 weight tiles
  const int m0 = blockIdx.x * BM;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, li = lane & 15;

  // ---- DMA issue helpers (swizzle on the per-lane source address; rows past the
  // tensor end read as zero through the buffer bounds check)
  const auto rs_w1 = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.w1), (short)0, H * D * 2, 0x00020000);
  const auto rs_w2 = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.w2), (short)0, D * H * 2, 0x00020000);
  // Tile t of the stream -> (chunk c, k-tile kt).  Each workgroup walks the chunks
  // and the k-tiles of a chunk in an order rotated by its block id, so the
  // workgroups running together fetch different weight tiles instead of all
  // hitting the same L2 lines at once; every output column still sums its k-tiles
  // in one fixed (rotated) order: deterministic.
  const int rot = blockIdx.x;
  auto tile_of = [&](int t, int& c, int& kt, int& q) {
    const bool p1 = t < T1;
    const int t2 = p1 ? t : t - T1;
    const int kt_n = p1 ? KT1 : KT2, nc = p1 ? NC1 : NC2;
    const int cq = t2 / kt_n;
    q = t2 - cq * kt_n;
    c = (cq + rot) % nc;
    kt = (q + rot) % kt_n;
  };
  auto issue_w = [&](int t, int slot) {
    const bool p1 = t < T1;
    int c, kt, q;
    tile_of(t, c, kt, q);
    const int ld = p1 ? D : H;
    char* dst = ring + slot * WT;
#pragma unroll
    for (int j = 0; j < WPIECES; ++j) {
      const int piece = wave * WPIECES + j;
      const int r = piece * 8 + (lane >> 3), lc = (lane & 7) ^ swz(r);
      const int voff = ((c * CW + r) * ld + 8 * lc) * 2 + kt * 128;
      if (p1)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_w1, (DC_LDS void*)(dst + piece * 1024), 16, voff, 0, 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_w2, (DC_LDS void*)(dst + piece * 1024), 16, voff, 0, 0, 0);
    }
  };
  // constants and the panel's LayerNorm statistics: flat copies in 1-KiB pieces
  // (bytes past each array's end read as zero), dealt to the waves
  {
    auto flat = [&](const void* src, int nbytes, char* dst, int& pc) {
      const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(src), (short)0, nbytes, 0x00020000);
      for (int q = 0; q * 1024 < nbytes; ++q, ++pc)
        if ((pc & 3) == wave)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (DC_LDS void*)(dst + q * 1024), 16, q * 1024 + lane * 16, 0,
                                                   0, 0);
    };
    int pc = 0;
    char* cb = smem;
    flat(a.c1, H * 4, cb, pc);
    flat(a.b1, H * 4, cb + kib(4 * H), pc);
    flat(a.b2, D * 4, cb + 2 * kib(4 * H), pc);
    const int rows = min(BM, a.M - m0);
    flat(a.st_in + (size_t)m0 * np * 2, rows * np * 8, stimg, pc);
  }
  // A panel: KT1 k-tiles of BM rows (BM/8 pieces per k-tile, pieces dealt to waves)
  {
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.xb), (short)0, a.M * D * 2, 0x00020000);
    for (int kt = 0; kt < KT1; ++kt)
      for (int piece = wave; piece < BM / 8; piece += 4) {
        const int r = piece * 8 + (lane >> 3), lc = (lane & 7) ^ swz(r);
        const int voff = ((m0 + r) * D + 8 * lc) * 2 + kt * 128;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (DC_LDS void*)(aimg + kt * BM * 128 + piece * 1024), 16, voff,
                                                 0, 0, 0);
      }
  }
  for (int s = 0; s < S - 1; ++s)
    if (s < T) issue_w(s, s);

  float2 ms[FM][4];  // (mean, rstd) of the lane's rows, from the statistics image at tile 0
  uint32_t salt1 = 0, salt2 = 0, saltd = 0;
  if (a.thr_f1) salt1 = site_salt(a.rng, a.site_f1);
  if (a.thr_f2) salt2 = site_salt(a.rng, a.site_f2);
  if (a.thr_dp) saltd = site_salt(a.rng, a.site_dp);

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  int res_tile = -1;  // tile at whose start the current residual chunk was issued

  for (int t = 0; t < T; ++t) {
    vm_wait_rem<WPIECES>(min(S - 2, T - 1 - t));
    raw_barrier();
    if (t == 0) {
      // slot li of each of the lane's rows, summed over the 16 lanes in the fold
      // consumer epilogue's fixed butterfly order (gemm_epi.h)
      const float* st = reinterpret_cast<const float*>(stimg);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int rr = i * 16 + 4 * g + r, m = m0 + rr;
          float2 u = (m < a.M && li < np) ? *reinterpret_cast<const float2*>(st + 2 * (rr * np + li))
                                          : make_float2(0.f, 0.f);
          u.x += __shfl_xor(u.x, 1); u.y += __shfl_xor(u.y, 1);
          u.x += __shfl_xor(u.x, 2); u.y += __shfl_xor(u.y, 2);
          u.x += __shfl_xor(u.x, 4); u.y += __shfl_xor(u.y, 4);
          u.x += __shfl_xor(u.x, 8); u.y += __shfl_xor(u.y, 8);
          const float invd = 1.0f / (float)D;
          const float mu = u.x * invd;
          const float var = fmaxf(u.y * invd - mu * mu, 0.f);
          ms[i][r] = make_float2(mu, rsqrtf(var + a.eps));
          if (TRAIN && a.mean_out != nullptr && wave == 0 && li == 0 && m < a.M) {
            a.mean_out[m] = ms[i][r].x;
            a.rstd_out[m] = ms[i][r].y;
          }
        }
    }
    const bool p1 = t < T1;
    const int kt_n = p1 ? KT1 : KT2;
    int c, kt, q;
    tile_of(t, c, kt, q);
    if (!p1 && q == 0) {
      // fc2 chunk c: its residual rows x1[m0.., c*128..+127] (fp32) into the A-image
      // region (dead after fc1): BM/2 pieces of two 512-B rows
      const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.x1), (short)0, a.M * D * 4,
                                                        0x00020000);
      for (int piece = wave; piece < BM / 2; piece += 4) {
        const int r = 2 * piece + (lane >> 5);
        const int voff = ((m0 + r) * D + c * CW + (lane & 31) * 4) * 4;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (DC_LDS void*)(aimg + piece * 1024), 16, voff, 0, 0, 0);
      }
      res_tile = t;
    }
    if (t + S - 1 < T) issue_w(t + S - 1, (t + S - 1) % S);

    const char* la = p1 ? aimg + kt * BM * 128 : himg + kt * BM * 128;
    const char* lb = ring + (t % S) * WT;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = frag_k(la, i * 16 + li, s, g);
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = frag_k(lb, wave * 32 + j * 16 + li, s, g);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    }
    if (q != kt_n - 1) continue;

    // ------------------------------------------------------------ chunk epilogue
    if (p1) {
      // fc1 columns n = c*128 + 32*wave + 16j + li of the hidden layer
      float cc[FN], cb[FN];
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = c * CW + wave * 32 + j * 16 + li;
        cc[j] = cst[n];
        cb[j] = cst[kib(4 * H) / 4 + n];
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int rr = i * 16 + 4 * g + r, m = m0 + rr;
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            const int n = c * CW + wave * 32 + j * 16 + li;
            const float v = (acc[i][j][r] - ms[i][r].x * cc[j]) * ms[i][r].y + cb[j];
            float h = gelu_f(v);
            const size_t idx = (size_t)m * H + n;
            if (a.thr_f1) h = dropout_keep(salt1, (uint32_t)idx, a.thr_f1) ? h * a.sc_f1 : 0.f;
            const bf16 hb = f2bf(h);
            const int hk = n >> 6, hc = n & 63;
            *reinterpret_cast<bf16*>(himg + hk * BM * 128 + rr * 128 + 16 * ((hc >> 3) ^ swz(rr)) + 2 * (hc & 7)) = hb;
            if (TRAIN && m < a.M) {
              reinterpret_cast<bf16*>(a.u_out)[idx] = f2bf(v);
              reinterpret_cast<bf16*>(a.h_out)[idx] = hb;
            }
          }
        }
      // the hidden image is complete before the first fc2 tile's barrier
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    } else {
      // the residual chunk (issued at tile res_tile, before that tile's weight
      // pieces): wait until at most the weight pieces issued after it are pending
      const int after = min(t - res_tile + 1, max(0, T - (res_tile + S - 1)));
      vm_wait_rem<WPIECES>(after);
      raw_barrier();  // every wave's residual pieces are in LDS (no vmcnt(0) drain)
      const float* res = reinterpret_cast<const float*>(aimg);
      float cb[FN];
#pragma unroll
      for (int j = 0; j < FN; ++j) cb[j] = cst[2 * kib(4 * H) / 4 + c * CW + wave * 32 + j * 16 + li];
      const int np_out = D / 32;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int rr = i * 16 + 4 * g + r, m = m0 + rr;
          const int b = m / a.tokens;
          float2 part = make_float2(0.f, 0.f);
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            const int col = wave * 32 + j * 16 + li, n = c * CW + col;
            float v = acc[i][j][r] + cb[j];
            const size_t idx = (size_t)m * D + n;
            if (a.thr_f2) v = dropout_keep(salt2, (uint32_t)idx, a.thr_f2) ? v * a.sc_f2 : 0.f;
            if (a.thr_dp) v = dropout_keep(saltd, (uint32_t)b, a.thr_dp) ? v * a.sc_dp : 0.f;
            const float o = res[rr * CW + col] + v;
            if (m < a.M) {
              a.x_out[idx] = o;
              reinterpret_cast<bf16*>(a.xb_out)[idx] = f2bf(o);
            }
            part.x += o;
            part.y += o * o;
          }
          // the row's {sum, sum^2} over this wave's 32 columns = statistics slot
          part.x += __shfl_xor(part.x, 1); part.y += __shfl_xor(part.y, 1);
          part.x += __shfl_xor(part.x, 2); part.y += __shfl_xor(part.y, 2);
          part.x += __shfl_xor(part.x, 4); part.y += __shfl_xor(part.y, 4);
          part.x += __shfl_xor(part.x, 8); part.y += __shfl_xor(part.y, 8);
          if (li == 0 && m < a.M)
            *reinterpret_cast<float2*>(a.st_out + 2 * ((size_t)m * np_out + c * 4 + wave)) = part;
        }
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
}

#define DC_INST_MLP(BM, S)                                                   \
  template __global__ void mlp_fused_kernel<BM, S, true>(MlpArgs);          \
  template __global__ void mlp_fused_kernel<BM, S, false>(MlpArgs);
DC_INST_MLP(16, 4) DC_INST_MLP(16, 6) DC_INST_MLP(16, 8)
DC_INST_MLP(32, 4) DC_INST_MLP(32, 6) DC_INST_MLP(32, 8)
DC_INST_MLP(64, 3)

template <int BM, int S>
static void launch_mlp_t(const MlpArgs& a, bool train, hipStream_t stream) {
  const int lds = mlp_lds_bytes(BM, S, a.D, a.H);
  static const bool attr = [] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&mlp_fused_kernel<BM, S, true>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&mlp_fused_kernel<BM, S, false>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    return true;
  }();
  (void)attr;
  const dim3 grid((a.M + BM - 1) / BM);
  if (train) hipLaunchKernelGGL((mlp_fused_kernel<BM, S, true>), grid, dim3(256), lds, stream, a);
  else hipLaunchKernelGGL((mlp_fused_kernel<BM, S, false>), grid, dim3(256), lds, stream, a);
}

}  // namespace dc

using namespace dc;

bool mlp_fused_supported(int D, int H) {
  return D % CW == 0 && H % CW == 0 && D >= 256 && H >= 128 && D <= 512 && H <= 512;
}

// row-panel height: the smallest panel whose grid still fits one round on the
// 256 CUs (weights are re-read per panel; a second round would double the time),
// then the deepest ring the LDS leaves room for
int mlp_fused_bm(int M) {
  if ((M + 15) / 16 <= 256) return 16;
  if ((M + 31) / 32 <= 256) return 32;
  return 64;
}

void mlp_fused_launch(const MlpArgs& a, hipStream_t stream) {
  if (!mlp_fused_supported(a.D, a.H)) throw std::runtime_error("mlp_fused: unsupported D / H");
  const bool train = a.u_out != nullptr;
  const int bm = a.bm > 0 ? a.bm : mlp_fused_bm(a.M);
  const int budget = 160 * 1024;
  auto fits = [&](int bm_, int s) { return mlp_lds_bytes(bm_, s, a.D, a.H) <= budget; };
  if (bm == 16) {
    if (fits(16, 8)) launch_mlp_t<16, 8>(a, train, stream);
    else if (fits(16, 6)) launch_mlp_t<16, 6>(a, train, stream);
    else launch_mlp_t<16, 4>(a, train, stream);
  } else if (bm == 32) {
    if (fits(32, 8)) launch_mlp_t<32, 8>(a, train, stream);
    else if (fits(32, 6)) launch_mlp_t<32, 6>(a, train, stream);
    else launch_mlp_t<32, 4>(a, train, stream);
  } else {
    if (!fits(64, 3)) throw std::runtime_error("mlp_fused: D + H too large for a 64-row panel");
    launch_mlp_t<64, 3>(a, train, stream);
  }
}
