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
#include "gemm_epi.h"
#include "embed_parts.h"
#include <cstdlib>
#include <algorithm>
#include <type_traits>
#include <atomic>
#include <stdexcept>

namespace dc {

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
__device__ __forceinline__ void gemm_dma_body(const GemmParams& p, int tm, int tn, int kz) {
  constexpr int NW = WM * WN;
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
  // HEADL reduces its loss partials over 4 waves (VecEpi::finish)
  static_assert(NW == 4 || EPI != EPI_HEADL, "HEADL: 4 waves");
  static_assert(!AT || BM == 64 || BM == 128, "transposed A: BM 64 or 128 (two half images)");
  static_assert(!BT || BN == 64 || BN == 128, "transposed B: BN 64 or 128 (two half images)");
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16;
  constexpr bool PERM = AT || BT;
  using OA = typename DmaOp<BM, AT, NW>::type;
  using OB = typename DmaOp<BN, BT, NW>::type;
  constexpr int STAGE = OA::BYTES + OB::BYTES;
  constexpr int LPT = OA::PER_WAVE + OB::PER_WAVE;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int m0 = tm * BM, n0 = tn * BN;
  const int total_kt = (p.K + BK - 1) / BK;
  const int kt0 = kz * p.ktiles_per_split;
  const int nk = min(total_kt, kt0 + p.ktiles_per_split) - kt0;
  if (nk <= 0) return;  // empty split slice (grouped launches); no barrier reached

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int g = lane >> 4, li = lane & 15;
#ifdef DDIM_COLD_GEMM_STAMPS
  uint32_t st_t0 = 0, st_t1 = 0, st_t2 = 0;
  if (p.stamps) st_t0 = stamp_now();
#endif

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
  // epilogue operands in flight behind the first operand tiles (see VecEpi).  The
  // vector epilogues take the SWAPPED accumulator layout: mfma(B, A) = C^T puts 4
  // consecutive output columns of one row in each lane, no quad transpose.
  constexpr bool VEC = UsesVecEpi<EPI>::value;
  VecEpi<EPI, FM, FN, false, VEC> ep;
  if (VEC) ep.prefetch(p, m0 + wm * TM, n0 + wn * TN, g, li);

  // main loop; the bias-gradient MFMA variant is a separate instantiation so the
  // loop carries no per-k-step branch (one made hipcc shuffle the accumulators
  // between AGPRs and VGPRs every iteration)
  auto mainloop = [&](auto db_tag) {
    constexpr bool DB = decltype(db_tag)::value;
    for (int kt = 0; kt < nk; ++kt) {
      const int rem = min(S - 2, nk - 1 - kt);
      vm_wait_rem<LPT>(rem);
      raw_barrier();
#ifdef DDIM_COLD_GEMM_STAMPS
      if (p.stamps && kt == 0) st_t1 = stamp_now();
#endif
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
          if (AT) ta[s][i] = frag_t_half(la, wm * TM + i * 16, s, lane);
#pragma unroll
        for (int j = 0; j < FN; ++j)
          if (BT) tb[s][j] = frag_t_half(lb, wn * TN + j * 16, s, lane);
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 af[FM], bfr[FN];
        if (AT || BT) {
          if (s == 0) {
            // reads issued after k-step 0's: 2 per transposed fragment
            // (clamped to the 4-bit lgkmcnt field: waiting for fewer is correct, just stricter)
            constexpr int LATER0 = 2 * ((AT ? FM : 0) + (BT ? FN : 0));
            constexpr int LATER = LATER0 < 16 ? LATER0 : 15;
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
          for (int j = 0; j < FN; ++j) acc[i][j] = VEC ? mfma16(bfr[j], af[i], acc[i][j]) : mfma16(af[i], bfr[j], acc[i][j]);
        if (DB) {
#pragma unroll
          for (int i = 0; i < FM; ++i) dbacc[i] = mfma16(af[i], ones, dbacc[i]);
        }
      }
    }
  };
  if (WG && do_db) mainloop(std::true_type{});
  else mainloop(std::false_type{});
#ifdef DDIM_COLD_GEMM_STAMPS
  if (p.stamps) st_t2 = stamp_now();
#endif

  float dbsq = 0.f;  // ACC with sq_parts: this lane's bias-gradient squares
  if (WG && do_db && li == 0) {
    float* db = const_cast<float*>(p.bias);
    float old[FM][4];
#pragma unroll
    for (int i = 0; i < FM; ++i)  // all loads first (see the epilogue note)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * TM + i * 16 + 4 * g + r;
        old[i][r] = (EPI == EPI_ACC && m < p.M && !p.acc_store) ? db[m] : 0.f;
      }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * TM + i * 16 + 4 * g + r;
        if (m < p.M) {
          if (EPI == EPI_ATOMIC) {
            atomicAdd(db + m, dbacc[i][r]);
          } else {
            const float o = old[i][r] + dbacc[i][r];
            db[m] = o;
            dbsq += o * o;
          }
        }
      }
  }

  if (VEC) ep.finish(p, acc, li);
  else run_epilogue_scalar<EPI, FM, FN>(p, acc, m0 + wm * TM, n0 + wn * TN, g, li);
#ifdef DDIM_COLD_GEMM_STAMPS
  if (p.stamps) {
    __syncthreads();  // the last wave's epilogue
    if (threadIdx.x == 0) {
      const uint32_t t3 = stamp_now();
      uint32_t* o = p.stamps + (size_t)((blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * GEMM_STAMP_WORDS;
      o[0] = st_t0; o[1] = st_t1; o[2] = st_t2; o[3] = t3;
      o[4] = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
      o[5] = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
    }
  }
#endif
  if constexpr (EPI == EPI_ACC && VEC) {
    if (p.sq_parts) {  // the workgroup's grad-norm partial (fixed reduction order)
      __shared__ float sred[WM * WN];
      const float s = wave_sum(ep.sqacc + dbsq);
      if (lane == 0) sred[wave] = s;
      __syncthreads();
      if (threadIdx.x == 0) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < WM * WN; ++w) t += sred[w];
        p.sq_parts[p.sq_slot] = t;
      }
    }
  }
}

template <int BM, int BN, int WM, int WN, bool AT, bool BT, int EPI, int S>
__global__ __launch_bounds__(64 * WM * WN) void gemm_dma_kernel(GemmParams p) {
  const int tiles_n = (p.N + BN - 1) / BN;
  const int tiles_m = (p.M + BM - 1) / BM;
  const int bid = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int tm = bid / tiles_n;
  gemm_dma_body<BM, BN, WM, WN, AT, BT, EPI, S>(p, tm, bid - tm * tiles_n, blockIdx.z);
}

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
  constexpr int threads = 64 * WM * WN;
  if constexpr (3 * stage > 160 * 1024) {  // 256x192: 2-stage ring (explicitly instantiated below)
    hipLaunchKernelGGL((gemm_dma_kernel<BM, BN, WM, WN, AT, BT, EPI, 2>), dim3(tiles, 1, splits), dim3(threads),
                       2 * stage, stream, p);
  } else {
    if ((tiles * splits > 256 * per_cu4 && p.ktiles_per_split <= 8) || 4 * stage > 160 * 1024)
      hipLaunchKernelGGL((gemm_dma_kernel<BM, BN, WM, WN, AT, BT, EPI, 3>), dim3(tiles, 1, splits), dim3(threads),
                         3 * stage, stream, p);
    else
      hipLaunchKernelGGL((gemm_dma_kernel<BM, BN, WM, WN, AT, BT, EPI, 4>), dim3(tiles, 1, splits), dim3(threads),
                         4 * stage, stream, p);
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

// (tag dispatch instead of `if constexpr`: hipcc 7.2 silently drops the host
// stub of a kernel template first referenced inside an if-constexpr branch)
// tile configs: 0 = 32x64, 1 = 64x64, 2 = 128x64, 3 = 128x128 (4 waves, 2x2);
// 4 = 256x128, 5 = 128x128 (8 waves, 4x2: 512-thread workgroups, for M >= BIG_M)
constexpr int CFG_W8_256 = 4, CFG_W8_128 = 5, CFG_W8_192 = 6;
template <int EPI>
struct Wide8 {  // epilogues with no 4-wave workgroup reduction (HEAD / HEADL sum loss partials over 4 waves)
  static constexpr bool value = EPI == EPI_BF16 || EPI == EPI_F32 || EPI == EPI_QKV || EPI == EPI_RESID ||
                                EPI == EPI_GELU || EPI == EPI_EMBED || EPI == EPI_DGELU;
};
template <bool AT, bool BT, int EPI, bool OK = EPI != EPI_DGELU>
struct Big256 {
  static void go(GemmParams p, int splits, hipStream_t stream) { launch_dma<256, 128, 4, 2, AT, BT, EPI>(p, splits, stream); }
};
template <bool AT, bool BT, int EPI>
struct Big256<AT, BT, EPI, false> {
  static void go(GemmParams, int, hipStream_t) {}
};
template <bool AT, bool BT, int EPI, bool OK = !BT && (EPI == EPI_BF16 || EPI == EPI_QKV || EPI == EPI_GELU)>
struct Big192 {  // 256x192 tiles, 2-stage ring (57 KiB per stage): N = 1152 in 6 column tiles
  static void go(GemmParams p, int splits, hipStream_t stream) { launch_dma<256, 192, 4, 2, AT, BT, EPI>(p, splits, stream); }
};
template <bool AT, bool BT, int EPI>
struct Big192<AT, BT, EPI, false> {  // not built for this epilogue: the 256-row config
  static void go(GemmParams p, int splits, hipStream_t stream) {
    if (EPI != EPI_DGELU) Big256<AT, BT, EPI>::go(p, splits, stream);
    else launch_dma<128, 128, 4, 2, AT, BT, EPI>(p, splits, stream);
  }
};
template <bool AT, bool BT, int EPI, bool OK = Wide8<EPI>::value>
struct Launch8 {
  static void go(GemmParams p, int splits, hipStream_t stream, int cfg) {
    if (cfg == CFG_W8_192) { Big192<AT, BT, EPI>::go(p, splits, stream); return; }
    // DGELU at 256x128 spills (88 B/lane of scratch): its 256-row config is the 128-row one
    if (cfg == CFG_W8_256 && EPI != EPI_DGELU) Big256<AT, BT, EPI>::go(p, splits, stream);
    else launch_dma<128, 128, 4, 2, AT, BT, EPI>(p, splits, stream);
  }
};
template <bool AT, bool BT, int EPI>
struct Launch8<AT, BT, EPI, false> {
  static void go(GemmParams, int, hipStream_t, int) {
    throw std::runtime_error("gemm: 8-wave tiles are not built for this epilogue");
  }
};
template <bool AT, bool BT, int EPI>
struct DmaTiles {
  static void launch(GemmParams p, int splits, hipStream_t stream, int cfg) {
    switch (cfg) {
      case 0: launch_dma<32, 64, 2, 2, AT, BT, EPI>(p, splits, stream); break;
      case 1: launch_dma<64, 64, 2, 2, AT, BT, EPI>(p, splits, stream); break;
      case 2: launch_dma<128, 64, 2, 2, AT, BT, EPI>(p, splits, stream); break;
      case 3: launch_dma<128, 128, 2, 2, AT, BT, EPI>(p, splits, stream); break;
      default: Launch8<AT, BT, EPI>::go(p, splits, stream, cfg); break;
    }
  }
};
template <int EPI>
struct DmaTiles<false, true, EPI> {  // transposed B (dgrad): BN = 64 (4 waves) or 128 (8 waves)
  static void launch(GemmParams p, int splits, hipStream_t stream, int cfg) {
    switch (cfg) {
      case 0: launch_dma<32, 64, 2, 2, false, true, EPI>(p, splits, stream); break;
      case 1: launch_dma<64, 64, 2, 2, false, true, EPI>(p, splits, stream); break;
      case 2: case 3: launch_dma<128, 64, 2, 2, false, true, EPI>(p, splits, stream); break;
      default: Launch8<false, true, EPI>::go(p, splits, stream, cfg); break;
    }
  }
};
template <bool BT, int EPI>
struct DmaTiles<true, BT, EPI> {  // transposed A (wgrad): 64x64
  static void launch(GemmParams p, int splits, hipStream_t stream, int) {
    launch_dma<64, 64, 2, 2, true, BT, EPI>(p, splits, stream);
  }
};

// Tile choice.  M < BIG_M (ViT-tiny / sampler shapes, M = 2-4k): 64x64 when that
// alone gives ~1 workgroup per CU, else 32x64.  A cost model "operand bytes per CU"
// that picked 128x64 / 128x128 for the big shapes of those sizes measured SLOWER
// everywhere (qkv 2080x1152x384: 11.9 us at 128x128 vs 7.5 at 64x64; train step
// -10%): more, smaller workgroups hide latency better than fewer bytes help, and was
// removed.  M >= BIG_M (vit_small_200: M = 20,032): 8-wave 256x128 tiles (4x the
// MFMA work per operand byte of 64x64, one 144 KiB 3-stage ring per CU), for the
// epilogues that support them (Wide8).  gemm_set_tile_override() forces a config
// (tests and micro-benchmarks).  The LDS-DMA ring needs K % 64 == 0 for
// k-contiguous operands (transposed operands get zero rows past K from the buffer
// bounds check).
constexpr int BIG_M = 16384;
static std::atomic<int> g_tile_override{-1};
static int pick_tiles(int M, int N, int K, int splits, bool at, bool bt, bool wide8, bool qkv = false) {
  if (at) return 1;
  const int forced = g_tile_override.load(std::memory_order_relaxed);
  if (forced >= 0) return bt && forced == 3 ? 2 : forced;
  // 8-wave 256x128 tiles only when they still give about one tile per CU: the
  // oxford_flower sampler's N = 256 GEMMs (M = 16,448: 130 such tiles) run faster on
  // 64x64 / 32x64 tiles (tools/ub_gemm_large.py 16448 .. 256: residual 19.7 vs 15.9 us,
  // GELU 16.0 vs 13.2; vit_small_200 N = 384 at M = 20,032: 237 tiles, 8-wave faster)
  // the QKV projection (N = 3D = 1,152 at vit_small_200): 256x192 tiles, 2-stage ring --
  // 474 workgroups (1.85 rounds of 256 CUs) instead of 711 (2.8 rounds): 489 -> 453 us of
  // QKV per step (profiles/qkv192_r6.txt)
  if (wide8 && M >= BIG_M && ((M + 255) / 256) * ((N + 127) / 128) >= 236)
    return qkv && N % 192 == 0 ? CFG_W8_192 : CFG_W8_256;
  return ((M + 63) / 64) * ((N + 63) / 64) * splits >= 240 ? 1 : 0;
}

template <bool AT, bool BT, int EPI>
static void launch_auto(GemmParams p, int splits, hipStream_t stream) {
  const bool dma_ok = (AT || BT || p.K % 64 == 0) && (AT || p.K % 64 == 0);
  if (dma_ok) {
    // DGELU (input gradient through GELU + dropout, bf16 out) stays on 4-wave tiles at
    // every measured M (M = 20,032: 25.5 vs 26.5 us; 40,064: 42.1 vs 49.9)
    int cfg = pick_tiles(p.M, p.N, p.K, splits, AT, BT, Wide8<EPI>::value && EPI != EPI_DGELU, EPI == EPI_QKV);
    // the GELU epilogue (erf-GELU + dropout per element, two bf16 outputs) is the
    // heaviest in vector instructions: twice the waves of 32x64 tiles pay off on the
    // sampler shape (M=4160: 6.56 vs 7.14 us, tools/gpu_tile_sweep3.sh); the other
    // epilogues keep 64x64 there (QKV 11.45 vs 13.54, residual 6.65 vs 7.02)
    // the patch embedding likewise (sampler M=4,096: 7.83 vs 9.08 us, tools/ub_sampler_ends.py)
    if ((EPI == EPI_GELU || EPI == EPI_EMBED) && cfg == 1 && g_tile_override.load(std::memory_order_relaxed) < 0 &&
        ((p.M + 31) / 32) * ((p.N + 63) / 64) <= 1024)
      cfg = 0;
    DmaTiles<AT, BT, EPI>::launch(p, splits, stream, cfg);
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
// 8-wave tiles (4x2 waves): 256x128 and 128x128
#define DC_INST_W8(AT, BT, EPI)                                                    \
  template __global__ void gemm_dma_kernel<256, 128, 4, 2, AT, BT, EPI, 3>(GemmParams); \
  template __global__ void gemm_dma_kernel<256, 128, 4, 2, AT, BT, EPI, 4>(GemmParams); \
  template __global__ void gemm_dma_kernel<128, 128, 4, 2, AT, BT, EPI, 3>(GemmParams); \
  template __global__ void gemm_dma_kernel<128, 128, 4, 2, AT, BT, EPI, 4>(GemmParams);
#define DC_INST_W192(EPI) template __global__ void gemm_dma_kernel<256, 192, 4, 2, false, false, EPI, 2>(GemmParams);
DC_INST_W192(EPI_BF16) DC_INST_W192(EPI_QKV) DC_INST_W192(EPI_GELU)
DC_INST_DMA3(EPI_BF16) DC_INST_W8(false, false, EPI_BF16)
DC_INST_DMA3(EPI_F32) DC_INST_W8(false, false, EPI_F32)
DC_INST_DMA3(EPI_QKV) DC_INST_W8(false, false, EPI_QKV)
DC_INST_DMA3(EPI_RESID) DC_INST_W8(false, false, EPI_RESID)
DC_INST_DMA3(EPI_GELU) DC_INST_W8(false, false, EPI_GELU)
DC_INST_DMA3(EPI_HEAD)
DC_INST_DMA3(EPI_EMBED) DC_INST_W8(false, false, EPI_EMBED)
DC_INST_DMA3(EPI_HEADR)
DC_INST_DMA3(EPI_HEADL)
DC_INST_DMA2(false, true, EPI_BF16) DC_INST_W8(false, true, EPI_BF16)
DC_INST_DMA2(false, true, EPI_F32) DC_INST_W8(false, true, EPI_F32)
DC_INST_DMA2(false, true, EPI_DGELU)
DC_INST_DMA3(EPI_DGELU)  // the same on the k-contiguous path (transposed weight shadow)
template __global__ void gemm_dma_kernel<128, 128, 4, 2, false, false, EPI_DGELU, 3>(GemmParams);
template __global__ void gemm_dma_kernel<128, 128, 4, 2, false, false, EPI_DGELU, 4>(GemmParams);
template __global__ void gemm_dma_kernel<128, 128, 4, 2, false, true, EPI_DGELU, 3>(GemmParams);
template __global__ void gemm_dma_kernel<128, 128, 4, 2, false, true, EPI_DGELU, 4>(GemmParams);
DC_INST_DMA(64, true, true, EPI_ATOMIC)

// Whole-backward weight gradient: every dW += dy^T x of a training step (all
// blocks, head, patch embedding; up to WM_MAX problems) in ONE launch after the
// backward.  Per-block launches of ~400 workgroups are latency-bound (~15 us
// for 3.7 GFLOP); one launch of ~1,500 workgroups keeps every CU streaming
// operand tiles.  Problems are compact descriptors (the kernel-argument block
// must stay under 4 KiB); one token split, so the epilogue is a plain
// read-add-write (EPI_ACC: deterministic, no fp32 atomics).
constexpr int WM_MAX = WGRAD_MULTI_MAX;
constexpr int BIG_WG_K = 16384;  // tokens: 128 x 128 weight-gradient tiles from here
// their LDS ring: 4 x 32 KiB, one workgroup per CU.  A 2-stage ring (two workgroups per CU,
// to soften the last-wave tail of ~5.1 tile rounds) took the vit_small_200 weight
// gradients 638 -> 1,183 us (and 48 problems per launch did not merge its two launches)
constexpr int BIG_WG_STAGES = 4;
// the ring plus the kernel's static LDS (ticket flag, wave sums) within one CU's 160 KiB: a
// 5-stage ring (163,952 B with the statics) is refused at launch (invalid allocation)
static_assert(BIG_WG_STAGES * 2 * 128 * 128 + 256 <= 160 * 1024, "weight-gradient ring exceeds the LDS of one CU");
struct WgDesc {
  const bf16* A;
  const bf16* B;
  float* C;
  float* bias;
  int M, N, K, lda, ldb, ldc;
};
struct WgradMulti {
  WgDesc d[WM_MAX];
  int tile_start[WM_MAX + 1];
  int n;
  int store;  // every target is zero: plain stores (no read-add)
  WgradSq sq;  // sq.parts != nullptr: grad-norm partials (kernels.h)
  // embedding gradients + LayerNorm finalize as extra workgroups (embed_parts.h parts A,
  // B, D; single-process step): nA / nB / nD workgroups after the grad-norm tail, each
  // writing its grad-norm partial to slot tiles + sq.tail + (its index among them)
  EmbedGrad emb;
  ReplicaFinal rf;
  int nA, nB, nD;
  // K-split tail (wide tiles): the first `whole` tiles run whole; the R = tiles - whole
  // last ones in `split` K pieces each, written to ws (per piece: T x T partial + T bias
  // partial), the last piece of a tile to finish (ticket in cnt[tile - whole]) sums the
  // pieces in piece order into the target (deterministic) and writes the tile's partial
  int whole, split;
  float* ws;
  int* cnt;
};
// tail workgroup j of the fused grad-norm: squares of the arena ranges no tile or
// embedding workgroup writes, then zero the unused partial slots (from zfrom on)
template <int NT>
__device__ __forceinline__ void wgrad_sq_tail(const WgradSq& sq, int tiles, int j, int zfrom) {
  float s = 0.f;
  const int64_t stride = (int64_t)sq.tail * NT;
  for (int r = 0; r < sq.nr; ++r)
    for (int64_t i = sq.lo[r] + (int64_t)j * NT + threadIdx.x; i < sq.hi[r]; i += stride) {
      const float v = sq.base[i];
      s += v * v;
    }
  __shared__ float red[NT / 64];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) t += red[w];
    sq.parts[tiles + j] = t;
  }
  for (int i = zfrom + j * NT + threadIdx.x; i < sq.nparts; i += sq.tail * NT) sq.parts[i] = 0.f;
}
// T x TN output tiles of WM x WN waves: 64 x 64 / 4 waves (ViT-tiny, sampler-sized
// token counts), 128 x 128 / 8 waves when the reduction runs over >= BIG_WG_K tokens
// (vit_small_200: 20,032; half the operand bytes per MFMA, ~5 tiles per CU)
template <int T, int S, int TN = T, int WM = 2, int WN = 2>
__global__ __launch_bounds__(64 * WM * WN) void gemm_wgrad_multi_kernel(WgradMulti gm) {
  const int tiles = gm.tile_start[gm.n];
  // the grad-norm tail workgroups first, so their strided sweeps over the untiled arena
  // ranges overlap the tiles instead of trailing them (within noise: profiles/tail_first_r5.txt)
  // block order: the grad-norm tail and the embedding parts first (their strided sweeps
  // and latency-bound column sums overlap the tiles instead of trailing them:
  // profiles/tail_first_r5.txt; embedding parts last measured 1 % slower per ViT-tiny
  // step on one box: profiles/embed_in_wgrad_r6.txt), then the tiles
  constexpr int NT = 64 * WM * WN;
  const int ne = gm.nA + gm.nB + gm.nD;
  const int tail = (int)gridDim.x - tiles - (tiles - gm.whole) * (gm.split - 1) - ne;
  if ((int)blockIdx.x < tail) {
    wgrad_sq_tail<NT>(gm.sq, tiles, blockIdx.x, tiles + tail + ne);
    return;
  }
  if ((int)blockIdx.x < tail + ne) {
    // embedding parts: their scratch is the LDS operand ring (unused by them)
    extern __shared__ __attribute__((aligned(16))) char smem_emb[];
    const int k = (int)blockIdx.x - tail;
    float* sqp = gm.sq.parts ? gm.sq.parts + tiles + tail + k : nullptr;
    if (k < gm.nA) emb_part_a<NT>(gm.emb, k, sqp, reinterpret_cast<float*>(smem_emb));
    else if (k < gm.nA + gm.nB) emb_part_b<NT>(gm.emb, k - gm.nA, smem_emb, sqp);
    else emb_part_d<NT>(gm.rf, k - gm.nA - gm.nB, smem_emb, sqp);
    return;
  }
  const int u = (int)blockIdx.x - tail - ne;
  const int R = tiles - gm.whole;
  int bid, piece = 0;
  if (u < gm.whole) {
    bid = xcd_remap(u, gm.whole);
  } else {  // K piece of a split tile; the pieces with one K range share an XCD
    const int j = xcd_remap(u - gm.whole, R * gm.split);
    piece = j / R;
    bid = gm.whole + (j - piece * R);
  }
  int lo = 0, hi = gm.n - 1;  // problem owning tile `bid`: binary search over tile_start
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (bid >= gm.tile_start[mid]) lo = mid;
    else hi = mid - 1;
  }
  const WgDesc& d = gm.d[lo];
  GemmParams p{};
  p.A = d.A; p.B = d.B; p.C = d.C; p.bias = d.bias;
  p.M = d.M; p.N = d.N; p.K = d.K; p.lda = d.lda; p.ldb = d.ldb; p.ldc = d.ldc;
  p.acc_store = gm.store;
  p.sq_parts = gm.sq.parts;
  p.sq_slot = bid;
  const int nkt = (d.K + BK - 1) / BK;
  p.ktiles_per_split = nkt;
  const int tiles_n = (d.N + TN - 1) / TN;
  const int local = bid - gm.tile_start[lo];
  const int tm = local / tiles_n, tn = local - tm * tiles_n;
  if (u < gm.whole) {
    gemm_dma_body<T, TN, WM, WN, true, true, EPI_ACC, S>(p, tm, tn, 0);
    return;
  }
  // split tile: this piece's partial product (plain stores) into its workspace slot, the
  // target pointers rebased so the epilogue's (row, column) land at (0, 0) of the slot
  constexpr int PS = T * TN + T;  // floats per piece slot: tile + bias partial
  float* slot = gm.ws + (size_t)((bid - gm.whole) * gm.split + piece) * PS;
  const int m0 = tm * T, n0 = tn * TN;
  p.C = slot - ((ptrdiff_t)m0 * TN + n0);
  p.ldc = TN;
  p.bias = d.bias ? slot + T * TN - m0 : nullptr;
  p.acc_store = 1;
  p.sq_parts = nullptr;
  p.ktiles_per_split = (nkt + gm.split - 1) / gm.split;
  if (piece * p.ktiles_per_split < nkt) {
    gemm_dma_body<T, TN, WM, WN, true, true, EPI_ACC, S>(p, tm, tn, piece);
  } else {  // a piece past the last k-tile (short reductions): a zero partial
    for (int i = threadIdx.x; i < PS; i += NT) slot[i] = 0.f;
  }
  // publish (every storing wave drained, then one release), take a ticket; the last
  // piece of the tile sums all of them (cdna_hip_programming.md G16 ticket recipe)
  __shared__ int s_last;
  __shared__ float s_red[NT / 64];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int prev = __hip_atomic_fetch_add(gm.cnt + (bid - gm.whole), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev == gm.split - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      gm.cnt[bid - gm.whole] = 0;  // every piece has taken its ticket: ready for the next launch
    }
    s_last = last;
  }
  __syncthreads();
  if (!s_last) return;
  const float* base = gm.ws + (size_t)((bid - gm.whole) * gm.split) * PS;
  const int rows = min(T, d.M - m0), cols = min(TN, d.N - n0);
  float q = 0.f;
  for (int i = threadIdx.x; i < T * TN / 4; i += NT) {  // 4 columns per thread-step
    const int r = (4 * i) / TN, c = 4 * i - r * TN;
    if (r >= rows || c >= cols) continue;
    f32x4 v = *reinterpret_cast<const f32x4*>(base + 4 * i);
    for (int k = 1; k < gm.split; ++k) {
      const f32x4 w = *reinterpret_cast<const f32x4*>(base + (size_t)k * PS + 4 * i);
      v[0] += w[0]; v[1] += w[1]; v[2] += w[2]; v[3] += w[3];
    }
    f32x4* dst = reinterpret_cast<f32x4*>(d.C + (size_t)(m0 + r) * d.ldc + n0 + c);
    if (!gm.store) {
      const f32x4 o = *dst;
      v[0] += o[0]; v[1] += o[1]; v[2] += o[2]; v[3] += o[3];
    }
    *dst = v;
    q += v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
  }
  if (d.bias && tn == 0) {
    for (int r = threadIdx.x; r < rows; r += NT) {
      float v = base[T * TN + r];
      for (int k = 1; k < gm.split; ++k) v += base[(size_t)k * PS + T * TN + r];
      const float o = gm.store ? v : d.bias[m0 + r] + v;
      d.bias[m0 + r] = o;
      q += o * o;
    }
  }
  if (gm.sq.parts) {
    q = wave_sum(q);
    if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = q;
    __syncthreads();
    if (threadIdx.x == 0) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < NT / 64; ++w) t += s_red[w];
      gm.sq.parts[bid] = t;
    }
  }
}
template __global__ void gemm_wgrad_multi_kernel<64, 3>(WgradMulti);
template __global__ void gemm_wgrad_multi_kernel<128, BIG_WG_STAGES, 128, 4, 2>(WgradMulti);

}  // namespace dc

// ============================================================================ host API
using namespace dc;

static std::atomic<uint32_t*> g_stamps{nullptr};
uint32_t* gemm_set_stamps(uint32_t* buf) { return g_stamps.exchange(buf); }

static GemmParams base_params(const GemmArgs& a) {
  GemmParams p{};
  p.stamps = g_stamps.load(std::memory_order_relaxed);
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
  p.patch_out = reinterpret_cast<bf16*>(a.patch_out);
  p.cls_src = a.cls_src;
  p.tok_magic = p.tokens > 1 ? (uint32_t)(0x100000000ull / (uint64_t)p.tokens) : 0xFFFFFFFFu;
  p.ln_invd = p.K > 0 ? 1.0f / (float)p.K : 0.f;
  return p;
}

GemmParams dc::gemm_params_from_args(const GemmArgs& a) {
  GemmParams p = base_params(a);
  return p;
}

static void check_vec(const GemmParams& p, int epi) {
  // the vector epilogue stores 4 consecutive output columns per lane
  if (epi != EPI_HEAD && (p.N % 4 != 0 || (epi == EPI_QKV && p.hd % 4 != 0) || (epi == EPI_EMBED && p.emb_dim % 4 != 0)))
    throw std::runtime_error("gemm: output width must be a multiple of 4");
  // ... and indexes its outputs / operands with 32-bit offsets
  const long long w = std::max({(long long)p.N, (long long)p.ldc, (long long)p.emb_dim});
  if ((long long)(p.M + p.batch + 1) * w * (p.split_stride > 0 ? 2 : 1) >= (1LL << 31) ||
      p.split_stride >= (1LL << 30))
    throw std::runtime_error("gemm: tensors of >= 2^31 elements are not supported by the epilogue's 32-bit indexing");
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
    case EPI_DGELU: launch_auto<false, false, EPI_DGELU>(p, 1, stream); break;  // dgrad through GELU, W^T given
    case EPI_HEADR:
      if (p.K % 64 != 0) throw std::runtime_error("gemm_nt: EPI_HEADR needs the LDS-DMA GEMM");
      launch_auto<false, false, EPI_HEADR>(p, 1, stream);
      break;
    case EPI_HEADL:
      if (p.K % 64 != 0) throw std::runtime_error("gemm_nt: EPI_HEADL needs the LDS-DMA GEMM");
      launch_auto<false, false, EPI_HEADL>(p, 1, stream);
      break;
    default: throw std::runtime_error("gemm_nt: unsupported epilogue");
  }
}

int gemm_nt_grid(int M, int N, int K) {
  // mirrors launch_auto<false, false, EPI> (one split) for the epilogues that size a
  // per-workgroup buffer from it (HEAD / HEADL: never 8-wave tiles)
  const bool dma_ok = K % 64 == 0;
  int bm = 64, bn = 64;
  if (dma_ok) {
    const int cfg = pick_tiles(M, N, K, 1, false, false, false);
    const int bms[6] = {32, 64, 128, 128, 256, 128}, bns[6] = {64, 64, 64, 128, 128, 128};
    bm = bms[cfg < 0 ? 0 : (cfg > 5 ? 5 : cfg)];
    bn = bns[cfg < 0 ? 0 : (cfg > 5 ? 5 : cfg)];
  } else if (((M + 63) / 64) * ((N + 63) / 64) < 240) {
    bm = 32;
  }
  return ((M + bm - 1) / bm) * ((N + bn - 1) / bn);
}

int gemm_set_tile_override(int cfg) {
  if (cfg < -1 || cfg > 6) throw std::runtime_error("gemm_set_tile_override: -1 (auto) or 0..6");
  return g_tile_override.exchange(cfg);
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

int wgrad_embed_workgroups(const WgradEmbed& emb, bool wide) {
  const int NT = wide ? 512 : 256;
  const EmbedGrad& e = emb.e;
  return (e.N * e.D + NT - 1) / NT + e.owners * ((e.D + EMB_BCOLS - 1) / EMB_BCOLS) +
         (emb.rf.ws ? emb.rf.G * ((emb.rf.C + 15) / 16) : 0);
}

// K pieces for the tail tiles of a wide (one workgroup per CU) launch: with W whole rounds
// of 256 tiles and R tiles left, R x s pieces take ceil(R s / 256) / s tile times instead
// of one (profiles/wgrad_split_r6.txt); s = 1 (no split) when nothing is gained
static int cu_count() {  // one wide workgroup per CU (256 on the MI355X)
  static const int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        v <= 0)
      v = 256;
    return v;
  }();
  return n;
}
// workgroup slots of one round: one 128 x 128 (128 KiB ring) or three 64 x 64 (48 KiB)
// weight-gradient workgroups per CU
static int wgrad_slots(int T) { return (T == 128 ? 1 : 3) * cu_count(); }
int wgrad_split_factor(int tiles, int T) {
  const int C = wgrad_slots(T), R = tiles % C;
  // 64 x 64 tiles (three workgroups per CU): splitting ViT-tiny's 12-tile tail in 6 pieces
  // measured slower (0.7107 -> 0.7146 ms/step, profiles/wgrad_split_r6.txt) -- wide tiles only
  if (R == 0 || T != 128) return 1;
  int best = 1;
  double bt = 1.0;
  for (int s = 2; s <= WGRAD_MAX_SPLIT; ++s) {
    const double t = (double)((R * s + C - 1) / C) / s;
    if (t < bt - 1e-9) { bt = t; best = s; }
  }
  return best;
}
int wgrad_multi_tile(int kmax) { return kmax >= BIG_WG_K ? 128 : 64; }
int64_t wgrad_split_ws_floats(int tiles, int T) {
  const int s = wgrad_split_factor(tiles, T);
  return s > 1 ? (int64_t)(tiles % wgrad_slots(T)) * s * (T * T + T) : 0;
}

int gemm_wgrad_multi(const GemmArgs* probs, int n, hipStream_t stream, bool store, const WgradSq* sq,
                     const WgradEmbed* emb, float* split_ws, int* split_cnt) {
  if (n < 1 || n > WM_MAX) throw std::runtime_error("gemm_wgrad_multi: 1..WGRAD_MULTI_MAX problems per launch");
  WgradMulti gm{};
  gm.n = n;
  gm.store = store ? 1 : 0;
  int tiles = 0;
  // ViT-tiny-sized token counts: 64 x 64 tiles, 3-stage ring (48 KiB: three
  // workgroups per CU).  Measured slower there and not used: 128 x 128 tiles (half the
  // operand bytes per output, one 96 KiB workgroup per CU, ~390 workgroups in 1.5
  // rounds: 0.838 vs 0.824 ms/step), 128 x 64 tiles (24 % fewer operand bytes, same
  // 60-61 us launch), a 4-stage ring (0.833).  Long reductions (>= BIG_WG_K tokens,
  // vit_small_200) take 128 x 128 tiles of 8 waves with a 4-stage 128 KiB ring.
  int kmax = 0;
  for (int i = 0; i < n; ++i) kmax = std::max(kmax, probs[i].K);
  const int T = kmax >= BIG_WG_K ? 128 : 64;
  for (int i = 0; i < n; ++i) {
    const GemmArgs& a = probs[i];
    if (a.N % 4 != 0) throw std::runtime_error("gemm_wgrad_multi: output width must be a multiple of 4");
    WgDesc& d = gm.d[i];
    d.A = reinterpret_cast<const bf16*>(a.A); d.B = reinterpret_cast<const bf16*>(a.B);
    d.C = reinterpret_cast<float*>(a.C); d.bias = const_cast<float*>(a.bias);
    d.M = a.M; d.N = a.N; d.K = a.K; d.lda = a.lda; d.ldb = a.ldb; d.ldc = a.ldc;
    gm.tile_start[i] = tiles;
    tiles += ((a.M + T - 1) / T) * ((a.N + T - 1) / T);
  }
  for (int i = n; i <= WM_MAX; ++i) gm.tile_start[i] = tiles;
  int extra = 0;
  if (emb != nullptr) {
    const int NT = T == 128 ? 512 : 256;
    const EmbedGrad& e = emb->e;
    if (e.B > EMB_BMAX || e.pbn != e.B || e.pb0 != 0 || e.D % 4)
      throw std::runtime_error("gemm_wgrad_multi: embedding parts need <= 256 samples (one part-B pass), D % 4 == 0");
    gm.emb = e;
    gm.rf = emb->rf;
    gm.nA = (e.N * e.D + NT - 1) / NT;
    gm.nB = e.owners * ((e.D + EMB_BCOLS - 1) / EMB_BCOLS);
    gm.nD = emb->rf.ws ? emb->rf.G * ((emb->rf.C + 15) / 16) : 0;
    extra += gm.nA + gm.nB + gm.nD;
    if (extra != wgrad_embed_workgroups(*emb, T == 128)) throw std::logic_error("wgrad_embed_workgroups");
  }
  if (sq != nullptr && sq->parts != nullptr) {
    if (sq->tail < 0 || sq->nr < 0 || sq->nr > WSQ_MAX_RANGES || sq->nparts < tiles + sq->tail + extra)
      throw std::runtime_error("gemm_wgrad_multi: grad-norm partial buffer too small (nparts < tiles + tail + "
                               "embedding workgroups) or more than 16 ranges");
    gm.sq = *sq;
    extra += sq->tail;
  }
  static_assert(sizeof(WgradMulti) <= 4000, "kernel argument block");
  gm.whole = tiles;
  gm.split = 1;
  int pieces = 0;
  if (split_ws != nullptr && split_cnt != nullptr) {
    const int s = wgrad_split_factor(tiles, T);
    if (s > 1) {
      const int R = tiles % wgrad_slots(T);
      gm.whole = tiles - R;
      gm.split = s;
      gm.ws = split_ws;
      gm.cnt = split_cnt;
      pieces = R * s - R;  // extra workgroups beyond one per tile
    }
  }
  if (T == 128) {
    constexpr int lds = BIG_WG_STAGES * 2 * 128 * 128;  // stages x (A + B) 128-wide, 64-deep images
    hipLaunchKernelGGL((gemm_wgrad_multi_kernel<128, BIG_WG_STAGES, 128, 4, 2>), dim3(tiles + pieces + extra), dim3(512),
                       lds, stream, gm);
  } else {
    hipLaunchKernelGGL((gemm_wgrad_multi_kernel<64, 3>), dim3(tiles + pieces + extra), dim3(256),
                       3 * (64 * 128 + 64 * 128), stream, gm);
  }
  return tiles;
}

