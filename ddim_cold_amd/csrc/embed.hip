// Patch-embedding front end, embedding backward, and the smooth-L1 loss.
//
//  * patchify_cls: NCHW fp32 image -> conv-im2col rows [B*P, C*p*p] bf16 (the A
//    operand of the patch-embed MFMA GEMM, whose EPI_EMBED epilogue adds
//    bias + pos_embed + time_embed[t] + dropout and scatters to token rows);
//    the same launch writes the cls rows  x[b,0,:] = Dropout(cls + pos[0] + temb[t_b]).
//    (ViT.py:150-155 PatchEmbed, ViT.py:199-206 prepare_tokens)
//  * embed_bwd: grads of cls/pos/time embeddings + patch-row grad for the conv
//    weight-gradient GEMM (pos_drop mask regenerated).
//  * smooth_l1: mean smooth-L1 (multi_gpu_trainer.py:124) fused with its
//    gradient, written straight into the token layout the head backward GEMMs
//    read (inverse of the head's unpatchify; cls rows zero).
#include "common.h"
#include "kernels.h"
#include "embed_parts.h"
#include <algorithm>

namespace dc {

// pix_src(x, n, f) with the two nearest-neighbour scales of one pixelation factor
// computed once (same float expressions, so the same source index)
struct PixMap {
  float s_in, s_out;
  int ts, n;
  __device__ PixMap(int n_, int f) : n(n_) {
    ts = n_ / f;
    if (ts < 1) ts = 1;
    s_in = (float)ts / (float)n_;
    s_out = (float)n_ / (float)ts;
  }
  __device__ __forceinline__ int operator()(int x) const {
    int s = (int)floorf((float)x * s_in);
    s = s < ts - 1 ? s : ts - 1;
    const int d = (int)floorf((float)s * s_out);
    return d < n - 1 ? d : n - 1;
  }
};

template <int PT>
__device__ __forceinline__ void patch_segments(const float* __restrict__ img, bf16* __restrict__ patches, int B, int C,
                                               int H, int W, int NP, int Wp, uint32_t csalt, uint32_t nsalt,
                                               int patch_blocks, const ColdSrc& cs, int P_rt = 0) {
  constexpr int PMAX = PT ? PT : 32;
  const int P = PT ? PT : P_rt;
  const int PP = P * P, F = C * PP;
  const int nseg = B * NP * C * P;
  for (int u = blockIdx.x * blockDim.x + threadIdx.x; u < nseg; u += patch_blocks * blockDim.x) {
    const int r1 = u / P, i = u - r1 * P;
    const int row = r1 / C, c = r1 - row * C;
    const int b = row / NP, pidx = row - b * NP;
    const int hp = pidx / Wp, wp = pidx - hp * Wp;
    const int y = hp * P + i, x0 = wp * P;
    const size_t o = (((size_t)b * C + c) * H + y) * W + x0;  // image index of element j = 0
    float v[PMAX];
    if (cs.pool) {
      const int src = cs.draw_idx ? cold_draw_idx(csalt, b, cs.pool_n) : (int)cs.idx[b];
      const float* im = cs.pool + ((size_t)src * C + c) * H * W;
      float* tg = cs.target + (cs.target_rows ? (size_t)row * F + (size_t)i * P * C + c : o);
      const int tstride = cs.target_rows ? C : 1;
      if (cs.gauss_T) {
        // Gaussian DDIM batch fused in: x_t = sqrt(a_t) x0 + sqrt(1-a_t) eps straight
        // into the patch row, target = x0 (gauss_batch_kernel's values)
        const int tt = gauss_draw_t(csalt, b, cs.gauss_T);
        float sa, s1a;
        gauss_coef(tt, cs.gauss_T, sa, s1a);
        const float* ir = im + (size_t)y * W + x0;
#pragma unroll
        for (int j = 0; j < PMAX; ++j) {
          if (!PT && j >= P) break;
          const float x0v = ir[j];
          v[j] = sa * x0v + s1a * gauss_eps(nsalt, (uint32_t)(o + j));
          tg[j * tstride] = x0v;
        }
      } else {
        // cold batch fused in: pixelate the pool image straight into the patch row
        // (x_t) and write the target image (x_{t-1}, or x0) -- same values as
        // cold_batch_kernel + the image path, one launch fewer
        const int tt = cold_draw_t(csalt, b, cs.max_t);
        const PixMap m1(W, 1 << tt);
        const float* r1p = im + (size_t)PixMap(H, 1 << tt)(y) * W;
        if (cs.target_x0) {
          const float* ir = im + (size_t)y * W + x0;
#pragma unroll
          for (int j = 0; j < PMAX; ++j) {
            if (!PT && j >= P) break;
            tg[j * tstride] = ir[j];
          }
        } else {
          const PixMap m0(W, 1 << (tt - 1));
          const float* r0p = im + (size_t)PixMap(H, 1 << (tt - 1))(y) * W;
#pragma unroll
          for (int j = 0; j < PMAX; ++j) {
            if (!PT && j >= P) break;
            tg[j * tstride] = r0p[m0(x0 + j)];
          }
        }
#pragma unroll
        for (int j = 0; j < PMAX; ++j) {
          if (!PT && j >= P) break;
          v[j] = r1p[m1(x0 + j)];
        }
      }
      if (cs.x_t) {
#pragma unroll
        for (int j = 0; j < PMAX; ++j) {
          if (!PT && j >= P) break;
          cs.x_t[o + j] = v[j];
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < PMAX; ++j) {
        if (!PT && j >= P) break;
        v[j] = img[o + j];
      }
    }
    bf16* dst = patches + (size_t)row * F + c * PP + i * P;
    if constexpr (PT == 8) {
      bf16x8 w;
#pragma unroll
      for (int j = 0; j < 8; ++j) w[j] = f2bf(v[j]);
      *reinterpret_cast<bf16x8*>(dst) = w;
    } else if constexpr (PT == 4) {
      bf16x4 w;
#pragma unroll
      for (int j = 0; j < 4; ++j) w[j] = f2bf(v[j]);
      *reinterpret_cast<bf16x4*>(dst) = w;
    } else {
      for (int j = 0; j < P; ++j) dst[j] = f2bf(v[j]);
    }
  }
}

// LayerNorm fold (gemm.hip): with `st` (the first LayerNorm's row statistics,
// [B*N][D/32][2] slots) the cls-row blocks write their rows' complete
// {sum, sum^2} into slot 0 (the other slots zero) plus the rows' bf16 copy; the
// patch rows' slots come from the patch-embed GEMM epilogue.
__global__ __launch_bounds__(256) void patchify_cls_kernel(const float* __restrict__ img, const int64_t* __restrict__ t,
                                                           const float* __restrict__ cls, const float* __restrict__ pos,
                                                           const float* __restrict__ temb, bf16* __restrict__ patches,
                                                           float* __restrict__ x, int B, int C, int H, int W, int P,
                                                           int D, const int64_t* __restrict__ rng, int site,
                                                           uint32_t thr, float dsc, float* __restrict__ st,
                                                           bf16* __restrict__ xb, int patch_blocks, ColdSrc cs) {
  const int Hp = H / P, Wp = W / P, NP = Hp * Wp, F = C * P * P, N = NP + 1;
  if (cs.idx_ctr) cs.idx += (cs.idx_ctr[0] % cs.idx_rows) * cs.idx_stride;  // stepped index table row
  const uint32_t csalt = cs.pool ? site_salt(rng, cs.site) : 0u;
  const uint32_t nsalt = cs.gauss_T ? site_salt(rng, cs.noise_site) : 0u;
  if ((int)blockIdx.x >= patch_blocks) {
    // cls row of sample b
    const int b = blockIdx.x - patch_blocks;
    const size_t row = (size_t)b * N;
    const uint32_t salt = thr ? site_salt(rng, site) : 0u;
    int64_t tb;
    if (cs.pool) {  // this block owns sample b's draw: publish (t, pool index) for the model
      tb = cs.gauss_T ? gauss_draw_t(csalt, b, cs.gauss_T) : cold_draw_t(csalt, b, cs.max_t);
      if (threadIdx.x == 0) {
        cs.t_out[b] = tb;
        if (cs.draw_idx) cs.idx[b] = cold_draw_idx(csalt, b, cs.pool_n);
      }
    } else {
      tb = t[b];
    }
    float s = 0.f, q = 0.f;
    for (int d = threadIdx.x; d < D; d += 256) {
      float v = cls[d] + pos[d] + temb[(size_t)tb * D + d];
      const size_t idx = row * D + d;
      if (thr) v = dropout_keep(salt, (uint32_t)idx, thr) ? v * dsc : 0.f;
      x[idx] = v;
      if (st) {
        xb[idx] = f2bf(v);
        s += v;
        q += v * v;
      }
    }
    if (st) {
      __shared__ float red[2][4];
      s = wave_sum(s);
      q = wave_sum(q);
      if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x >> 6] = s;
        red[1][threadIdx.x >> 6] = q;
      }
      __syncthreads();
      const int np = D / 32;
      float* sr = st + 2 * row * np;
      for (int k = threadIdx.x; k < 2 * np; k += 256)
        sr[k] = k == 0 ? (red[0][0] + red[0][1]) + (red[0][2] + red[0][3])
                       : k == 1 ? (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]) : 0.f;
    }
    return;
  }
  // patch rows: one thread per segment (row, c, i) = the P contiguous row elements
  // k = c*P*P + i*P + j (one image row of one patch channel): the index split, the
  // per-sample draw and the pixelation scales are paid once per segment, the P bf16
  // values leave as one vector store.  Image order instead (wp fastest: coalesced image
  // reads / target writes, patch stores F apart) took the vit_small_200 batch 21.2 -> 47.5 us
  switch (P) {
    case 8: patch_segments<8>(img, patches, B, C, H, W, NP, Wp, csalt, nsalt, patch_blocks, cs); break;
    case 4: patch_segments<4>(img, patches, B, C, H, W, NP, Wp, csalt, nsalt, patch_blocks, cs); break;
    default: patch_segments<0>(img, patches, B, C, H, W, NP, Wp, csalt, nsalt, patch_blocks, cs, P); break;
  }
}

// part A: (n,d) -> dpos (+dcls) ; part B: dtemb rows ; part C: patch-row grads (bf16) ;
// part D: LayerNorm dgamma/dbeta finalize.  Parts A, B, D are embed_parts.h (shared with
// the weight-gradient launch); no fp32 atomics anywhere.
__global__ __launch_bounds__(256) void embed_bwd_kernel(EmbedGrad e, bf16* __restrict__ gpatch, int blocksA,
                                                        int blocksB, int blocksC, ReplicaFinal rf) {
  __shared__ __attribute__((aligned(16))) char smem[emb_smem_bytes(256)];
  const int bid = blockIdx.x;
  if (bid < blocksA) {
    emb_part_a<256>(e, bid, nullptr, reinterpret_cast<float*>(smem));
  } else if (bid < blocksA + blocksB) {
    emb_part_b<256>(e, bid - blocksA, smem, nullptr);
  } else if (bid >= blocksA + blocksB + blocksC) {
    emb_part_d<256>(rf, bid - blocksA - blocksB - blocksC, smem, nullptr);
  } else {
    const float* g = e.g;
    const int B = e.B, N = e.N, D = e.D;
    const uint32_t thr = e.thr, salt = thr ? site_salt(e.rng, e.site) : 0u;
    const float dsc = e.dsc;
    // part C: 4 consecutive columns per thread (one 16-B load, two pair hashes, one 8-B
    // store) with 32-bit index math (the launcher checks the size); one element per
    // thread with 64-bit divisions was ~1/3 of this launch at vit_small_200
    const int D4 = D >> 2, NP = N - 1, total4 = B * NP * D4;
    for (int e = (bid - blocksA - blocksB) * 256 + threadIdx.x; e < total4; e += blocksC * 256) {
      const int row = e / D4, d = (e - row * D4) * 4;
      const int b = row / NP, i = row - b * NP;
      const int src = (b * N + 1 + i) * D + d;
      float4 v = *reinterpret_cast<const float4*>(g + src);
      if (thr) {
        bool k[4];
        dropout_keep4(salt, (uint32_t)src, thr, k);
        v.x = k[0] ? v.x * dsc : 0.f;
        v.y = k[1] ? v.y * dsc : 0.f;
        v.z = k[2] ? v.z * dsc : 0.f;
        v.w = k[3] ? v.w * dsc : 0.f;
      }
      bf16x4 o;
      o[0] = f2bf(v.x);
      o[1] = f2bf(v.y);
      o[2] = f2bf(v.z);
      o[3] = f2bf(v.w);
      *reinterpret_cast<bf16x4*>(gpatch + (size_t)e * 4) = o;
    }
  }
}

template <bool LOSS>
__global__ __launch_bounds__(256) void tokgrad_kernel(const float* __restrict__ pred, const float* __restrict__ target,
                                                      float* __restrict__ parts, bf16* __restrict__ dtok, int B, int C,
                                                      int H, int W, int P, float beta, float inv_numel) {
  __shared__ float red[4];
  const int Wp = W / P, NP = (H / P) * Wp, N = NP + 1, F = C * P * P;
  const size_t n_img = (size_t)B * C * H * W;
  const size_t n_cls = (size_t)B * F;
  float acc = 0.f;
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < n_img + n_cls;
       e += (size_t)gridDim.x * blockDim.x) {
    if (e < n_img) {
      const int xw = (int)(e % W);
      size_t r = e / W;
      const int yh = (int)(r % H);
      r /= H;
      const int c = (int)(r % C);
      const int b = (int)(r / C);
      float gv;
      if (LOSS) {
        const float d = pred[e] - target[e];
        const float ad = fabsf(d);
        acc += ad < beta ? 0.5f * d * d / beta : ad - 0.5f * beta;
        gv = fminf(fmaxf(d / beta, -1.f), 1.f) * inv_numel;
      } else {
        gv = pred[e];
      }
      const int hp = yh / P, a = yh - hp * P, wp = xw / P, bb = xw - wp * P;
      const int tok = 1 + hp * Wp + wp;
      const int f = (a * P + bb) * C + c;
      dtok[((size_t)b * N + tok) * F + f] = f2bf(gv);
    } else {
      const size_t e2 = e - n_img;
      const int b = (int)(e2 / F), f = (int)(e2 % F);
      dtok[(size_t)b * N * F + f] = f2bf(0.f);
    }
  }
  if (LOSS) {
    acc = wave_sum(acc);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) parts[blockIdx.x] = (red[0] + red[1] + red[2] + red[3]) * inv_numel;
  }
}

// loss = sum of the per-block partials; optionally also the trainer's loss
// bookkeeping (multi_gpu_trainer.py:125-126: last loss + EMA 0.99/0.01) so the
// training step needs no extra copy / elementwise launches for it
__global__ __launch_bounds__(256) void sum_parts_kernel(const float* __restrict__ parts, int n, float* __restrict__ out,
                                                        float* __restrict__ loss_last, float* __restrict__ loss_ema,
                                                        float decay) {
  __shared__ float red[4];
  float v = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) v += parts[i];
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float l = red[0] + red[1] + red[2] + red[3];
    out[0] = l;
    if (loss_last) loss_last[0] = l;
    if (loss_ema) loss_ema[0] = loss_ema[0] * decay + l * (1.f - decay);
  }
}

static int grid_for(size_t n) {
  size_t g = (n + 255) / 256;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace dc

using namespace dc;

void patchify_cls_launch(const float* img, const int64_t* t, const float* cls, const float* pos, const float* temb,
                         void* patches, float* x, int B, int C, int H, int W, int patch, int D, const int64_t* rng,
                         int site, double p, float* st, void* xb, hipStream_t stream, ColdSrc cs) {
  // one thread per patch-row segment of `patch` elements (patch_segments)
  const size_t n = (size_t)B * (H / patch) * (W / patch) * C * patch;
  if (patch > 32) throw std::invalid_argument("patchify: patch size > 32");
  if (n >= (size_t)INT32_MAX) throw std::invalid_argument("patchify: too many patch-row segments for 32-bit indexing");
  const uint32_t thr = drop_threshold_host(p);
  const float dsc = p > 0 ? 1.f / (1.f - (float)p) : 1.f;
  const int pb = grid_for(n);
  hipLaunchKernelGGL(patchify_cls_kernel, dim3(pb + B), dim3(256), 0, stream, img, t, cls, pos, temb,
                     reinterpret_cast<bf16*>(patches), x, B, C, H, W, patch, D, rng, site, thr, dsc, st,
                     reinterpret_cast<bf16*>(xb), pb, cs);
}

void embed_bwd_launch(const float* g, const int64_t* t, float* dcls, float* dpos, float* dtemb, void* gpatch, int B,
                      int N, int D, const int64_t* rng, int site, double p, hipStream_t stream, ReplicaFinal rf) {
  if (D % 4 != 0) throw std::invalid_argument("embed_bwd: D must be a multiple of 4");
  if ((size_t)B * N * D >= (size_t)INT32_MAX) throw std::invalid_argument("embed_bwd: too many elements for 32-bit indexing");
  EmbedGrad e = embed_grad_args(g, t, dcls, dpos, dtemb, B, N, D, rng, site, p, 0, std::min(B, EMB_BMAX));
  const int blocksA = cdiv(N * D, 256), blocksB = e.pbn * cdiv(D, EMB_BCOLS);
  const int blocksC = grid_for((size_t)B * (N - 1) * D / 4);
  const int blocksD = rf.ws ? rf.G * cdiv(rf.C, 16) : 0;
  hipLaunchKernelGGL(embed_bwd_kernel, dim3(blocksA + blocksB + blocksC + blocksD), dim3(256), 0, stream, e,
                     reinterpret_cast<bf16*>(gpatch), blocksA, blocksB, blocksC, rf);
  // batches beyond EMB_BMAX samples: further part-B passes (stream-ordered: each adds to
  // the rows the previous passes wrote; a sample's t is owned in its own pass)
  for (int pb0 = EMB_BMAX; pb0 < B; pb0 += EMB_BMAX) {
    EmbedGrad ep = e;
    ep.pb0 = pb0;
    ep.pbn = std::min(B - pb0, EMB_BMAX);
    const int nb = ep.pbn * cdiv(D, EMB_BCOLS);
    hipLaunchKernelGGL(embed_bwd_kernel, dim3(nb), dim3(256), 0, stream, ep, reinterpret_cast<bf16*>(gpatch), 0, nb,
                       0, ReplicaFinal());
  }
}

EmbedGrad embed_grad_args(const float* g, const int64_t* t, float* dcls, float* dpos, float* dtemb, int B, int N,
                          int D, const int64_t* rng, int site, double p, int pb0, int pbn) {
  EmbedGrad e;
  e.g = g; e.t = t; e.dcls = dcls; e.dpos = dpos; e.dtemb = dtemb;
  e.B = B; e.N = N; e.D = D;
  e.thr = drop_threshold_host(p);
  e.dsc = p > 0 ? 1.f / (1.f - (float)p) : 1.f;
  e.rng = rng;
  e.site = site;
  e.pb0 = pb0; e.pbn = pbn;
  e.owners = pbn;
  return e;
}

int smooth_l1_launch(const float* pred, const float* target, float* loss, float* partials, void* dtok, int B,
                     int C, int H, int W, int patch, float beta, float* loss_last, float* loss_ema, float ema_decay,
                     bool finish, hipStream_t stream) {
  const size_t n_img = (size_t)B * C * H * W;
  const size_t n = n_img + (size_t)B * C * patch * patch;
  int grid = grid_for(n);
  if (grid > L1_PARTS) grid = L1_PARTS;
  hipLaunchKernelGGL(tokgrad_kernel<true>, dim3(grid), dim3(256), 0, stream, pred, target, partials,
                     reinterpret_cast<bf16*>(dtok), B, C, H, W, patch, beta, 1.0f / (float)n_img);
  if (finish)
    hipLaunchKernelGGL(sum_parts_kernel, dim3(1), dim3(256), 0, stream, partials, grid, loss, loss_last, loss_ema,
                       ema_decay);
  return grid;
}

void img_to_tokgrad_launch(const float* dimg, void* dtok, int B, int C, int H, int W, int patch, hipStream_t stream) {
  const size_t n = (size_t)B * C * H * W + (size_t)B * C * patch * patch;
  hipLaunchKernelGGL(tokgrad_kernel<false>, dim3(grid_for(n)), dim3(256), 0, stream, dimg, nullptr, nullptr,
                     reinterpret_cast<bf16*>(dtok), B, C, H, W, patch, 1.f, 1.f);
}
