// LayerNorm forward / backward for the ViT residual stream (nn.LayerNorm,
// eps 1e-5 — ViT.py:124,128,182).  fp32 residual stream in, bf16 normalised
// activations out (the next GEMM's A operand), fp32 mean/rstd saved.
//
// One wave64 per row, the row held in registers (D/128 float2 per lane,
// 512-B coalesced wave accesses), shuffle reductions only — no LDS in the
// forward.  The backward additionally fuses:
//   * the residual-gradient add  g_out = g_res + dLN/dx,
//   * the *next* residual branch's gradient prep  gy = bf16(g_out * dropout
//     mask * drop-path scale)  (masks regenerated from the counter hash),
//   * dgamma/dbeta column partials, deterministic: reduced per workgroup through
//     LDS into a slot of its own (one row of the workspace, plain stores); a later
//     launch (replica_reduce, the embedding backward or the weight-gradient launch)
//     sums the slots in slot order.  No fp32 atomics: two runs are bit-identical.
//     (An in-launch reduction -- write-through slots, an agent-scope ticket, the
//     last of 16 workgroups summing -- measured 5.7 -> 12.5 us per ViT-tiny launch:
//     every workgroup then waits for its stores to drain, and the last arriver's
//     acquire + slot reads trail the launch.)
#include "common.h"
#include "kernels.h"
#include <algorithm>

namespace dc {

constexpr int LN_NW = 8;        // waves (rows) per workgroup of the backward
constexpr int LN_MAX_WG = 512;  // backward workgroups (= dgamma/dbeta slots) at most

template <int VEC, int NW>
__global__ __launch_bounds__(NW * 64) void ln_fwd_kernel(const float* __restrict__ x, const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, bf16* __restrict__ y,
                                                     float* __restrict__ mean, float* __restrict__ rstd, int M,
                                                     float eps) {
  constexpr int D = VEC * 128;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * NW + (threadIdx.x >> 6);
  if (row >= M) return;
  const float2* xr = reinterpret_cast<const float2*>(x + (size_t)row * D);
  float2 v[VEC];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    v[i] = xr[lane + 64 * i];
    s += v[i].x + v[i].y;
  }
  const float mu = wave_sum(s) * (1.0f / D);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    const float a = v[i].x - mu, b = v[i].y - mu;
    q += a * a + b * b;
  }
  const float rs = rsqrtf(wave_sum(q) * (1.0f / D) + eps);
  const float2* g2 = reinterpret_cast<const float2*>(gamma);
  const float2* b2 = reinterpret_cast<const float2*>(beta);
  bf16x2* yr = reinterpret_cast<bf16x2*>(y + (size_t)row * D);
  float2 gv[VEC], bv[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    gv[i] = g2[lane + 64 * i];
    bv[i] = b2[lane + 64 * i];
  }
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    const int c = lane + 64 * i;
    const float2 gg = gv[i], bb = bv[i];
    bf16x2 o;
    o[0] = f2bf((v[i].x - mu) * rs * gg.x + bb.x);
    o[1] = f2bf((v[i].y - mu) * rs * gg.y + bb.y);
    yr[c] = o;
  }
  if (lane == 0) {
    mean[row] = mu;
    rstd[row] = rs;
  }
}

// DYB: dy (and its K-split partials) in bf16 -- the dgrad GEMMs write half the bytes.
// XB: x is the bf16 copy of the LayerNorm input, the operand the folded forward GEMM
// actually normalised (x_hat from it is the forward's own), 2 bytes per element less.
// Rows: groups of NW*RPW rows, workgroup-strided (grid = ln_bwd_workgroups(M), at most
// LN_MAX_WG: the dgamma/dbeta slots a finalize reads stay bounded at large M).
// gp (the last LayerNorm of the backward, whose output gradient feeds the embedding):
// also the patch-row gradient of the patch embedding -- g_out rows 1..N-1 of each
// sample with the embedding dropout (site_emb) applied, bf16, in patch-row order
// (what the embedding backward's part C wrote).
template <int VEC, int RPW, int NW, bool DYB, bool XB>
__global__ __launch_bounds__(NW * 64) void ln_bwd_kernel(const void* __restrict__ dyv, const void* __restrict__ x,
                                                     const float* __restrict__ mean, const float* __restrict__ rstd,
                                                     const float* __restrict__ gamma, const float* __restrict__ beta,
                                                     const float* __restrict__ g_res,
                                                     float* __restrict__ g_out, bf16* __restrict__ gy,
                                                     bf16* __restrict__ y_out, float* __restrict__ slots, int M,
                                                     int tokens, const int64_t* __restrict__ rng, int site_drop,
                                                     uint32_t thr_drop, float sc_drop, int site_dp, uint32_t thr_dp,
                                                     float sc_dp, int dy_parts, bf16* __restrict__ gp, int site_emb,
                                                     uint32_t thr_emb, float sc_emb) {
  constexpr int D = VEC * 128;
  // dynamic LDS ([NW][2D] floats): static LDS limited the residency of the larger
  // non-256-thread workgroups (tools/ub_lds_census.hip)
  extern __shared__ float red_dyn[];
  float (*red)[2 * D] = reinterpret_cast<float (*)[2 * D]>(red_dyn);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float2* g2 = reinterpret_cast<const float2*>(gamma);
  float2 dgam[VEC], dbet[VEC], gm[VEC], bt[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    dgam[i] = make_float2(0.f, 0.f);
    dbet[i] = make_float2(0.f, 0.f);
    gm[i] = g2[lane + 64 * i];
    bt[i] = y_out ? reinterpret_cast<const float2*>(beta)[lane + 64 * i] : make_float2(0.f, 0.f);
  }
  // rng words loaded here, with the rows' loads, and the salts computed after ONE
  // explicit wait for all of them (below): site_salt() here was sunk by the compiler
  // past the row-data wait, one more dependent round trip per wave
  const uint64_t rng0 = (uint64_t)rng[0], rng1 = (uint64_t)rng[1];  // rng: always a valid [2]
  for (int grp = blockIdx.x; grp * NW * RPW < M; grp += gridDim.x) {
    // RPW rows per wave, all rows' loads issued before any use (latency-bound op)
    float2 xv[RPW][VEC], dv[RPW][VEC], rv[RPW][VEC];
    float muv[RPW], rsv[RPW];
    int rows[RPW];
#pragma unroll
    for (int j = 0; j < RPW; ++j) {
      rows[j] = (grp * NW + wave) * RPW + j;
      const int row = rows[j] < M ? rows[j] : M - 1;
      const float2* xr = reinterpret_cast<const float2*>(reinterpret_cast<const float*>(x) + (size_t)row * D);
      const bf16x2* xr16 = reinterpret_cast<const bf16x2*>(reinterpret_cast<const bf16*>(x) + (size_t)row * D);
      // unconditional load (g_out when there is no residual gradient: same shape, the value
      // is dropped below): `g_res ? load : 0` became a phi copy that waited for every load
      // issued before it
      const float2* gr = reinterpret_cast<const float2*>((g_res ? g_res : g_out) + (size_t)row * D);
      auto ldy = [&](int pt, int i) -> float2 {
        const size_t off = (size_t)pt * M * D + (size_t)row * D;
        if (DYB) {
          const bf16x2 e = reinterpret_cast<const bf16x2*>(reinterpret_cast<const bf16*>(dyv) + off)[lane + 64 * i];
          return make_float2(bf2f(e[0]), bf2f(e[1]));
        }
        return reinterpret_cast<const float2*>(reinterpret_cast<const float*>(dyv) + off)[lane + 64 * i];
      };
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        if (XB) {
          const bf16x2 e = xr16[lane + 64 * i];
          xv[j][i] = make_float2(bf2f(e[0]), bf2f(e[1]));
        } else {
          xv[j][i] = xr[lane + 64 * i];
        }
        dv[j][i] = ldy(0, i);
        rv[j][i] = gr[lane + 64 * i];
      }
      for (int pt = 1; pt < dy_parts; ++pt) {  // K-split dgrad partials
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
          const float2 e = ldy(pt, i);
          dv[j][i].x += e.x;
          dv[j][i].y += e.y;
        }
      }
      muv[j] = mean[row];
      rsv[j] = rstd[row];
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): rows + rng words (gfx9: expcnt 7, lgkmcnt 15)
    // unconditional (a few VALU ops): a use only under `if (gy)` let LLVM sink the loads
    // into that block, past the wait
    const uint32_t salt_drop = site_salt_v(rng0, rng1, site_drop);
    const uint32_t salt_dp = site_salt_v(rng0, rng1, site_dp);
    const uint32_t salt_emb = site_salt_v(rng0, rng1, site_emb);
#pragma unroll
    for (int j = 0; j < RPW; ++j) {
      const int row = rows[j];
      if (row >= M) continue;
      const float mu = muv[j], rs = rsv[j];
      float2 xh[VEC], dxh[VEC];
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        const float2 dvv = dv[j][i];
        xh[i] = make_float2((xv[j][i].x - mu) * rs, (xv[j][i].y - mu) * rs);
        dgam[i].x += dvv.x * xh[i].x;
        dgam[i].y += dvv.y * xh[i].y;
        dbet[i].x += dvv.x;
        dbet[i].y += dvv.y;
        dxh[i] = make_float2(dvv.x * gm[i].x, dvv.y * gm[i].y);
        s1 += dxh[i].x + dxh[i].y;
        s2 += dxh[i].x * xh[i].x + dxh[i].y * xh[i].y;
      }
      const float c1 = wave_sum(s1) * (1.0f / D);
      const float c2 = wave_sum(s2) * (1.0f / D);
      float dpsc = 1.f;
      if (gy && thr_dp) dpsc = dropout_keep(salt_dp, (uint32_t)(row / tokens), thr_dp) ? sc_dp : 0.f;
      const int tok = row % tokens;
      bf16* gprow = (gp && tok != 0) ? gp + ((size_t)(row / tokens) * (tokens - 1) + tok - 1) * D : nullptr;
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        const int c = lane + 64 * i;
        const float2 r = g_res ? rv[j][i] : make_float2(0.f, 0.f);
        float2 o = make_float2((dxh[i].x - c1 - xh[i].x * c2) * rs + r.x, (dxh[i].y - c1 - xh[i].y * c2) * rs + r.y);
        reinterpret_cast<float2*>(g_out + (size_t)row * D)[c] = o;
        if (y_out) {
          // the LayerNorm output itself (bf16), for the weight gradient of the GEMM
          // that consumed it with the LayerNorm folded in (no forward LayerNorm launch)
          bf16x2 yv;
          yv[0] = f2bf(xh[i].x * gm[i].x + bt[i].x);
          yv[1] = f2bf(xh[i].y * gm[i].y + bt[i].y);
          reinterpret_cast<bf16x2*>(y_out + (size_t)row * D)[c] = yv;
        }
        if (gy) {
          float a = o.x * dpsc, b = o.y * dpsc;
          if (thr_drop) {
            const uint32_t idx = (uint32_t)((size_t)row * D + 2 * c);
            const uint32_t hh = drop_hash(salt_drop, idx >> 1);  // idx even: one hash for the pair
            a = (hh & 0xFFFFu) >= thr_drop ? a * sc_drop : 0.f;
            b = (hh >> 16) >= thr_drop ? b * sc_drop : 0.f;
          }
          bf16x2 h;
          h[0] = f2bf(a);
          h[1] = f2bf(b);
          reinterpret_cast<bf16x2*>(gy + (size_t)row * D)[c] = h;
        }
        if (gprow) {  // patch-embedding input gradient (embedding dropout, same pair hash)
          float a = o.x, b = o.y;
          if (thr_emb) {
            const uint32_t hh = drop_hash(salt_emb, (uint32_t)((size_t)row * D + 2 * c) >> 1);
            a = (hh & 0xFFFFu) >= thr_emb ? a * sc_emb : 0.f;
            b = (hh >> 16) >= thr_emb ? b * sc_emb : 0.f;
          }
          bf16x2 h;
          h[0] = f2bf(a);
          h[1] = f2bf(b);
          reinterpret_cast<bf16x2*>(gprow)[c] = h;
        }
      }
    }
  }
  // column partials: waves -> LDS -> this workgroup's slot (plain stores, summed in
  // slot order by a later launch: deterministic, no atomics)
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    const int c = 2 * (lane + 64 * i);
    red[wave][c] = dgam[i].x;
    red[wave][c + 1] = dgam[i].y;
    red[wave][D + c] = dbet[i].x;
    red[wave][D + c + 1] = dbet[i].y;
  }
  __syncthreads();
  float* slot = slots + (size_t)blockIdx.x * 2 * D;
  for (int c = threadIdx.x; c < 2 * D; c += NW * 64) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) s += red[w][c];
    slot[c] = s;
  }
}

// dst[g][c] += sum_{r < R} ws[g][r][c] (rows of stride `rows`) in a fixed order
// (common.h slot_colsum16).  One launch finalises many LayerNorms.
__global__ __launch_bounds__(256) void replica_reduce_kernel(const float* __restrict__ ws,
                                                             float* const* __restrict__ dsts, int C, int R, int rows) {
  __shared__ float red[256];
  const int gi = blockIdx.y, c0 = blockIdx.x * 16;
  const float t = slot_colsum16<256>(ws + (size_t)gi * rows * C, C, R, c0, red);
  if (threadIdx.x < 16 && c0 + (int)threadIdx.x < C) dsts[gi][c0 + threadIdx.x] += t;
}

// LayerNorm fold weights (see gemm.hip "LayerNorm fold"): for each GEMM that
// consumes a LayerNorm, wf[n][k] = bf16(gamma_k W[n][k]), c[n] = sum_k wf[n][k]
// (the bf16 values the MFMA multiplies, so the mean term cancels exactly what
// the GEMM accumulated), bf[n] = b[n] + sum_k beta_k W[n][k].  One wave per
// output row, all folded GEMMs of the model in one launch (after each
// optimizer step; once per sampling run).
// training-step tail run by the fold launch's last workgroup: loss from its
// partials (loss_last, EMA), counters
__device__ __forceinline__ void fold_tail(const FoldTable& tb) {
  {
    __shared__ float red[2][4];
    float lv = 0.f, sv = 0.f;
    for (int i = threadIdx.x; i < tb.loss_nparts; i += 256) lv += tb.loss_parts[i];
    for (int i = threadIdx.x; i < tb.sq_n; i += 256) sv += tb.sq[i];
    lv = wave_sum(lv);
    sv = wave_sum(sv);
    if ((threadIdx.x & 63) == 0) {
      red[0][threadIdx.x >> 6] = lv;
      red[1][threadIdx.x >> 6] = sv;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      const float l = red[0][0] + red[0][1] + red[0][2] + red[0][3];
      const float sq = red[1][0] + red[1][1] + red[1][2] + red[1][3];
      if (tb.loss_last) tb.loss_last[0] = l;
      if (tb.loss_ema) tb.loss_ema[0] = tb.loss_ema[0] * tb.ema_decay + l * (1.f - tb.ema_decay);
      if (isfinite(sq)) tb.step[0] += 1;  // a non-finite step was skipped by the optimizer
      tb.step[1] += 1;
      tb.rng[1] += 1;
    }
  }
}

__global__ __launch_bounds__(256) void ln_fold_kernel(FoldTable tb) {
  // the tail workgroup first, so its serial partial sums overlap the fold rows instead of
  // trailing them (measured within noise: profiles/tail_first_r5.txt)
  if (tb.tail && blockIdx.x == 0) {
    fold_tail(tb);
    return;
  }
  const int bx = (int)blockIdx.x - (tb.tail ? 1 : 0);
  // two rows per wave (32 lanes each), every load of the row issued before use
  constexpr int IT = 4;  // float4 per lane: K <= 32 * 4 * IT = 512
  const int hl = threadIdx.x & 31;
  const int r = bx * 8 + (threadIdx.x >> 5);
  const bool live = r < tb.start[tb.n];
  const int rr = live ? r : tb.start[tb.n] - 1;
  int ji = 0;
#pragma unroll
  for (int j = 1; j < FOLD_MAX; ++j)
    if (j < tb.n && rr >= tb.start[j]) ji = j;
  const FoldJob& jb = tb.j[ji];
  const int n = rr - tb.start[ji], K4 = tb.K / 4;
  const float4* w = reinterpret_cast<const float4*>(reinterpret_cast<const float*>(jb.w) + (size_t)n * tb.K);
  const bf16x4* wb = reinterpret_cast<const bf16x4*>(reinterpret_cast<const bf16*>(jb.w) + (size_t)n * tb.K);
  const float4* g = reinterpret_cast<const float4*>(jb.gamma);
  const float4* b = reinterpret_cast<const float4*>(jb.beta);
  bf16x4* o = reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(jb.wf) + (size_t)n * tb.K);
  float4 wv[IT], gv[IT], bv[IT];
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int k = hl + 32 * i;
    const bool ok = k < K4;
    if (tb.w_bf16) {
      const bf16x4 q = ok ? wb[k] : bf16x4{};
      wv[i] = ok ? make_float4(bf2f(q[0]), bf2f(q[1]), bf2f(q[2]), bf2f(q[3])) : make_float4(0.f, 0.f, 0.f, 0.f);
    } else {
      wv[i] = ok ? w[k] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    gv[i] = ok ? g[k] : make_float4(0.f, 0.f, 0.f, 0.f);
    bv[i] = ok ? b[k] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  float cs = 0.f, bs = 0.f;
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int k = hl + 32 * i;
    bf16x4 q;
    q[0] = f2bf(gv[i].x * wv[i].x); q[1] = f2bf(gv[i].y * wv[i].y);
    q[2] = f2bf(gv[i].z * wv[i].z); q[3] = f2bf(gv[i].w * wv[i].w);
    if (live && k < K4) o[k] = q;
    cs += (bf2f(q[0]) + bf2f(q[1])) + (bf2f(q[2]) + bf2f(q[3]));
    bs += (bv[i].x * wv[i].x + bv[i].y * wv[i].y) + (bv[i].z * wv[i].z + bv[i].w * wv[i].w);
  }
#pragma unroll
  for (int m = 16; m > 0; m >>= 1) {
    cs += __shfl_xor(cs, m, 32);
    bs += __shfl_xor(bs, m, 32);
  }
  if (live && hl == 0) {
    jb.c[n] = cs;
    jb.bf[n] = bs + (jb.bias ? jb.bias[n] : 0.f);
  }
}

// bf16 weights (the optimizer's shadow), K % 8 == 0: 16 lanes per row (16 rows per
// workgroup), 16-byte weight loads and stores -- the 32-lane / 8-byte kernel above
// moved half as many bytes per instruction
__global__ __launch_bounds__(256) void ln_fold16_kernel(FoldTable tb) {
  // the tail workgroup first, so its serial partial sums overlap the fold rows instead of
  // trailing them (measured within noise: profiles/tail_first_r5.txt)
  if (tb.tail && blockIdx.x == 0) {
    fold_tail(tb);
    return;
  }
  const int bx = (int)blockIdx.x - (tb.tail ? 1 : 0);
  constexpr int IT = 4;  // 16-B chunks per lane: K <= 16 * 8 * IT = 512
  const int hl = threadIdx.x & 15;
  const int r = bx * 16 + (threadIdx.x >> 4);
  const bool live = r < tb.start[tb.n];
  const int rr = live ? r : tb.start[tb.n] - 1;
  int ji = 0;
#pragma unroll
  for (int j = 1; j < FOLD_MAX; ++j)
    if (j < tb.n && rr >= tb.start[j]) ji = j;
  const FoldJob& jb = tb.j[ji];
  const int n = rr - tb.start[ji], K8 = tb.K / 8;
  const bf16x8* w = reinterpret_cast<const bf16x8*>(reinterpret_cast<const bf16*>(jb.w) + (size_t)n * tb.K);
  const f32x4* g = reinterpret_cast<const f32x4*>(jb.gamma);
  const f32x4* b = reinterpret_cast<const f32x4*>(jb.beta);
  bf16x8* o = reinterpret_cast<bf16x8*>(reinterpret_cast<bf16*>(jb.wf) + (size_t)n * tb.K);
  bf16x8 wv[IT];
  f32x4 g0[IT], g1[IT], b0[IT], b1[IT];
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int k = hl + 16 * i;
    const bool ok = k < K8;
    const f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
    wv[i] = w[ok ? k : 0];  // out-of-range chunks: gamma = beta = 0 below zero their terms
    g0[i] = ok ? g[2 * k] : z;
    g1[i] = ok ? g[2 * k + 1] : z;
    b0[i] = ok ? b[2 * k] : z;
    b1[i] = ok ? b[2 * k + 1] : z;
  }
  float cs = 0.f, bs = 0.f;
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int k = hl + 16 * i;
    const bf16x8 wq = wv[i];
    const float w0 = bf2f(wq[0]), w1 = bf2f(wq[1]), w2 = bf2f(wq[2]), w3 = bf2f(wq[3]);
    const float w4 = bf2f(wq[4]), w5 = bf2f(wq[5]), w6 = bf2f(wq[6]), w7 = bf2f(wq[7]);
    bf16x8 q;
    q[0] = f2bf(g0[i][0] * w0); q[1] = f2bf(g0[i][1] * w1); q[2] = f2bf(g0[i][2] * w2); q[3] = f2bf(g0[i][3] * w3);
    q[4] = f2bf(g1[i][0] * w4); q[5] = f2bf(g1[i][1] * w5); q[6] = f2bf(g1[i][2] * w6); q[7] = f2bf(g1[i][3] * w7);
    cs += ((bf2f(q[0]) + bf2f(q[1])) + (bf2f(q[2]) + bf2f(q[3]))) + ((bf2f(q[4]) + bf2f(q[5])) + (bf2f(q[6]) + bf2f(q[7])));
    bs += ((b0[i][0] * w0 + b0[i][1] * w1) + (b0[i][2] * w2 + b0[i][3] * w3)) +
          ((b1[i][0] * w4 + b1[i][1] * w5) + (b1[i][2] * w6 + b1[i][3] * w7));
    if (live && k < K8) o[k] = q;
  }
#pragma unroll
  for (int m = 8; m > 0; m >>= 1) {
    cs += __shfl_xor(cs, m, 16);
    bs += __shfl_xor(bs, m, 16);
  }
  if (live && hl == 0) {
    jb.c[n] = cs;
    jb.bf[n] = bs + (jb.bias ? jb.bias[n] : 0.f);
  }
}

}  // namespace dc

using namespace dc;

void ln_fold_launch(const FoldTable& tb, hipStream_t stream) {
  if (tb.n <= 0) return;
  if (tb.n > FOLD_MAX || tb.K % 4 || tb.K > 512) throw std::runtime_error("ln_fold: bad table (K % 4, K <= 512)");
  const int rows = tb.start[tb.n];
  if (tb.w_bf16 && tb.K % 8 == 0) {
    hipLaunchKernelGGL(ln_fold16_kernel, dim3((rows + 15) / 16 + (tb.tail ? 1 : 0)), dim3(256), 0, stream, tb);
    return;
  }
  hipLaunchKernelGGL(ln_fold_kernel, dim3((rows + 7) / 8 + (tb.tail ? 1 : 0)), dim3(256), 0, stream, tb);
}

#define LN_DISPATCH(D, ...)                                                   \
  switch ((D) / 128) {                                                        \
    case 1: { constexpr int VEC = 1; __VA_ARGS__; } break;                    \
    case 2: { constexpr int VEC = 2; __VA_ARGS__; } break;                    \
    case 3: { constexpr int VEC = 3; __VA_ARGS__; } break;                    \
    case 4: { constexpr int VEC = 4; __VA_ARGS__; } break;                    \
    case 6: { constexpr int VEC = 6; __VA_ARGS__; } break;                    \
    case 8: { constexpr int VEC = 8; __VA_ARGS__; } break;                    \
    default: throw std::runtime_error("layernorm: D must be 128*{1,2,3,4,6,8}"); \
  }

void layernorm_fwd_launch(const float* x, const float* gamma, const float* beta, void* y_bf16, float* mean,
                          float* rstd, int M, int D, float eps, hipStream_t stream) {
  if (D % 128) throw std::runtime_error("layernorm: D % 128 != 0");
  // 4 waves per workgroup (one row each); measured 2.6 us for 2 or 4, 3.0 for 8
  LN_DISPATCH(D, hipLaunchKernelGGL((ln_fwd_kernel<VEC, 4>), dim3((M + 3) / 4), dim3(4 * 64), 0, stream, x,
                                    gamma, beta, reinterpret_cast<bf16*>(y_bf16), mean, rstd, M, eps))
}

void layernorm_bwd_launch(const void* dy, bool dy_bf16, const void* x, bool x_bf16, const float* mean, const float* rstd,
                          const float* gamma, const float* beta, const float* g_res, float* g_out, void* gy_bf16,
                          void* y_bf16, float* slots, int M,
                          int D, int tokens, const int64_t* rng, int site_drop, double p_drop, int site_dp,
                          double p_dp, int dy_parts, void* gp_bf16, int site_emb, double p_emb, hipStream_t stream) {
  if (D % 128) throw std::runtime_error("layernorm: D % 128 != 0");
  const uint32_t td = drop_threshold_host(p_drop), tp = drop_threshold_host(p_dp), te = drop_threshold_host(p_emb);
  const float sd = p_drop > 0 ? 1.f / (1.f - (float)p_drop) : 1.f;
  const float sp = p_dp > 0 ? 1.f / (1.f - (float)p_dp) : 1.f;
  const float se = p_emb > 0 ? 1.f / (1.f - (float)p_emb) : 1.f;
#define LN_BWD_GO1(R, W, DYB, XB)                                                                             \
  LN_DISPATCH(D, if (W * 2 * D * sizeof(float) > 65536)                                                         \
                  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&ln_bwd_kernel<VEC, R, W, DYB, XB>),           \
                                            hipFuncAttributeMaxDynamicSharedMemorySize, W * 2 * D * sizeof(float));  \
                hipLaunchKernelGGL((ln_bwd_kernel<VEC, R, W, DYB, XB>), dim3(ln_bwd_workgroups(M)), dim3(W * 64), \
                                    W * 2 * D * sizeof(float), stream, dy, x, mean, rstd, gamma, beta, g_res, g_out, \
                                    reinterpret_cast<bf16*>(gy_bf16), reinterpret_cast<bf16*>(y_bf16), slots,   \
                                    M, tokens, rng, site_drop, td,                                              \
                                    sd, site_dp, tp, sp, dy_parts, reinterpret_cast<bf16*>(gp_bf16), site_emb,  \
                                    te, se))
#define LN_BWD_GO(R, W)                      \
  if (dy_bf16 && x_bf16) LN_BWD_GO1(R, W, true, true)  \
  else if (dy_bf16) LN_BWD_GO1(R, W, true, false)      \
  else if (x_bf16) LN_BWD_GO1(R, W, false, true)       \
  else LN_BWD_GO1(R, W, false, false)
  // measured on the ViT-tiny shape (M 2080, D 384, dropout on): 1 row x 8 waves
  // 5.0 us, 2 x 4 5.9, 1 x 4 5.2, 1 x 16 5.1, 2 x 16 7.2
  static_assert(LN_NW == 8, "ln_bwd launch: 8 waves");
  LN_BWD_GO(1, 8)
#undef LN_BWD_GO
#undef LN_BWD_GO1
}

int ln_bwd_workgroups(int M) { return std::max(1, std::min((M + LN_NW - 1) / LN_NW, LN_MAX_WG)); }

void replica_reduce_launch(const float* ws, float* const* dsts_dev, int G, int C, int R, int rows, hipStream_t stream) {
  hipLaunchKernelGGL(replica_reduce_kernel, dim3((C + 15) / 16, G), dim3(256), 0, stream, ws, dsts_dev, C, R, rows);
}
