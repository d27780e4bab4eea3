// Embedding-gradient reductions of one training step (ViT.py:199-206 backward:
// cls_token, pos_embed, time_embed) and the LayerNorm dgamma/dbeta slot finalize, as
// workgroup-level device functions.  Two launches run them:
//
//   * embed_bwd_kernel (embed.hip): parts A, B, C (patch-row gradient), D;
//   * the single-process step's deferred weight-gradient launch (gemm.hip
//     gemm_wgrad_multi_kernel): parts A, B, D as extra workgroups beside the weight-
//     gradient tiles -- the last LayerNorm backward writes part C's patch rows itself
//     (ln_bwd gp_out) -- so the step has no embedding-backward launch.  There each part
//     workgroup also writes the grad-norm partial of exactly the values it wrote.
//
// Deterministic: every output element has ONE writer and a fixed summation order (no
// fp32 atomics).  NT = threads per workgroup (256 or 512); smem = >= emb_smem_bytes(NT).
#pragma once
#include "common.h"
#include "kernels.h"

namespace dc {

constexpr int EMB_BCOLS = 16;   // columns per part-B workgroup
constexpr int EMB_BMAX = 256;   // samples per part-B pass

__host__ __device__ constexpr int emb_smem_bytes(int NT) {
  return (EMB_BMAX * 8 + EMB_BMAX * 4 + 16 + (NT / 4) * EMB_BCOLS * 4 + 64) > (NT + NT / 64) * 4
             ? (EMB_BMAX * 8 + EMB_BMAX * 4 + 16 + (NT / 4) * EMB_BCOLS * 4 + 64)
             : (NT + NT / 64) * 4;
}


// sum of one value per thread over the workgroup, written by thread 0 to *out (fixed order)
template <int NT>
__device__ __forceinline__ void emb_block_sum_to(float v, float* out, float* red) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) s += red[w];
    *out = s;
  }
}

__device__ __forceinline__ float emb_gm(const EmbedGrad& e, uint32_t salt, size_t idx) {
  const float v = e.g[idx];
  if (!e.thr) return v;
  return dropout_keep(salt, (uint32_t)idx, e.thr) ? v * e.dsc : 0.f;
}

// part A, workgroup `unit`: dpos[n][d] += sum_b g[b][n][d] (and dcls for n = 0), one element
// per thread in sample order.  sq: the squares of the written values.
template <int NT>
__device__ __forceinline__ void emb_part_a(const EmbedGrad& e, int unit, float* sq, float* red) {
  const int N = e.N, D = e.D, B = e.B;
  const uint32_t salt = e.thr ? site_salt(e.rng, e.site) : 0u;
  const int el = unit * NT + threadIdx.x;
  float q = 0.f;
  if (el < N * D) {
    const int n = el / D, d = el - n * D;
    float s = 0.f;
    int b = 0;
    for (; b + 8 <= B; b += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = e.g[((size_t)(b + u) * N + n) * D + d];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        s += e.thr ? (dropout_keep(salt, (uint32_t)(((size_t)(b + u) * N + n) * D + d), e.thr) ? v[u] * e.dsc : 0.f)
                   : v[u];
    }
    for (; b < B; ++b) s += emb_gm(e, salt, ((size_t)b * N + n) * D + d);
    const float o = e.dpos[el] + s;
    e.dpos[el] = o;
    q = o * o;
    if (n == 0) {
      const float oc = e.dcls[d] + s;
      e.dcls[d] = oc;
      q += oc * oc;
    }
  }
  if (sq) emb_block_sum_to<NT>(q, sq, red);
}

// part B, workgroup `unit` = (timestep slot j, 16-column block): the j-th distinct timestep
// of the pass's samples in sample order, summed over every (sample with that t, token)
// row -- NT/4 row lanes x 4 float4 column lanes, four rows in flight per lane, then the
// row lanes in lane order; dtemb[t] += that (the row's only writer in the launch).
template <int NT>
__device__ __forceinline__ void emb_part_b(const EmbedGrad& e, int unit, char* smem, float* sq) {
  constexpr int RL = NT / 4;
  const int N = e.N, D = e.D, pbn = e.pbn, pb0 = e.pb0;
  const uint32_t salt = e.thr ? site_salt(e.rng, e.site) : 0u;
  int64_t* ts = reinterpret_cast<int64_t*>(smem);
  int* flg = reinterpret_cast<int*>(smem + EMB_BMAX * 8);          // first-occurrence flags, then the group
  int* own = reinterpret_cast<int*>(smem + EMB_BMAX * 12);
  float4* racc = reinterpret_cast<float4*>(smem + EMB_BMAX * 12 + 16);  // [RL][EMB_BCOLS / 4]
  float* red = reinterpret_cast<float*>(smem + EMB_BMAX * 12 + 16 + RL * EMB_BCOLS * 4);
  const int nd = (D + EMB_BCOLS - 1) / EMB_BCOLS;
  const int j = unit / nd, d0 = (unit - j * nd) * EMB_BCOLS;
  for (int b = threadIdx.x; b < pbn; b += NT) ts[b] = e.t[pb0 + b];
  if (threadIdx.x == 0) own[0] = -1;
  __syncthreads();
  for (int b = threadIdx.x; b < pbn; b += NT) {
    bool first = true;
    for (int b2 = 0; b2 < b; ++b2) first = first && ts[b2] != ts[b];
    flg[b] = first ? 1 : 0;
  }
  __syncthreads();
  for (int b = threadIdx.x; b < pbn; b += NT) {
    int rank = 0;
    for (int b2 = 0; b2 < b; ++b2) rank += flg[b2];
    if (flg[b] && rank == j) own[0] = b;
  }
  __syncthreads();
  const int b0 = own[0];
  if (b0 < 0) {  // fewer than j + 1 distinct timesteps (uniform over the workgroup)
    if (sq && threadIdx.x == 0) *sq = 0.f;
    return;
  }
  const int64_t t0 = ts[b0];
  __syncthreads();
  for (int b = threadIdx.x; b < pbn; b += NT) {  // the group's samples in order
    if (ts[b] != t0) continue;
    int pos = 0;
    for (int b2 = 0; b2 < b; ++b2) pos += ts[b2] == t0 ? 1 : 0;
    flg[pos] = pb0 + b;
  }
  if (threadIdx.x == 0) {
    int cnt = 0;
    for (int b = 0; b < pbn; ++b) cnt += ts[b] == t0 ? 1 : 0;
    own[1] = cnt;
  }
  __syncthreads();
  const int rows = own[1] * N;
  const int cl = threadIdx.x & 3, rl = threadIdx.x >> 2;
  const int d = d0 + 4 * cl;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  auto src = [&](int r) -> size_t {
    const int s = flg[r / N], n = r - (r / N) * N;
    return ((size_t)s * N + n) * D + d;
  };
  auto addrow = [&](size_t idx, float4 v) {
    if (e.thr) {
      bool k[4];
      dropout_keep4(salt, (uint32_t)idx, e.thr, k);
      v.x = k[0] ? v.x * e.dsc : 0.f;
      v.y = k[1] ? v.y * e.dsc : 0.f;
      v.z = k[2] ? v.z * e.dsc : 0.f;
      v.w = k[3] ? v.w * e.dsc : 0.f;
    }
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
  };
  if (d < D) {
    int r = rl;
    for (; r + 3 * RL < rows; r += 4 * RL) {
      size_t ix[4];
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        ix[u] = src(r + RL * u);
        v[u] = *reinterpret_cast<const float4*>(e.g + ix[u]);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) addrow(ix[u], v[u]);
    }
    for (; r < rows; r += RL) {
      const size_t ix = src(r);
      addrow(ix, *reinterpret_cast<const float4*>(e.g + ix));
    }
  }
  racc[rl * (EMB_BCOLS / 4) + cl] = acc;
  __syncthreads();
  float q = 0.f;
  if (rl == 0 && d < D) {
    float4 s4 = racc[cl];
    for (int l = 1; l < RL; ++l) {
      const float4 p = racc[l * (EMB_BCOLS / 4) + cl];
      s4.x += p.x; s4.y += p.y; s4.z += p.z; s4.w += p.w;
    }
    float4* dst = reinterpret_cast<float4*>(e.dtemb + (size_t)t0 * D + d);
    float4 o = *dst;
    o.x += s4.x; o.y += s4.y; o.z += s4.z; o.w += s4.w;
    *dst = o;
    q = o.x * o.x + o.y * o.y + o.z * o.z + o.w * o.w;
  }
  if (sq) emb_block_sum_to<NT>(q, sq, red);
}

// part D, workgroup `unit` = (LayerNorm, 16-column block): dst[c] (+)= the column's slots
// in a fixed order (common.h slot_colsum16).
template <int NT>
__device__ __forceinline__ void emb_part_d(const ReplicaFinal& rf, int unit, char* smem, float* sq) {
  float* red = reinterpret_cast<float*>(smem);  // [NT] + [NT/64]
  const int cb = (rf.C + 15) / 16;
  const int gi = unit / cb, c0 = (unit - gi * cb) * 16;
  const float t = slot_colsum16<NT>(rf.ws + (size_t)gi * rf.rows * rf.C, rf.C, rf.R, c0, red);
  float q = 0.f;
  if (threadIdx.x < 16 && c0 + (int)threadIdx.x < rf.C) {
    float* dst = rf.dsts[gi] + c0 + threadIdx.x;
    const float o = rf.store ? t : *dst + t;
    *dst = o;
    q = o * o;
  }
  if (sq) emb_block_sum_to<NT>(q, sq, red + NT);
}

}  // namespace dc
