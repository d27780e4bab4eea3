// Diffusion-math and on-GPU data kernels.
//
//  * ddim_step: clamp(x0_hat) + eps_hat + DDIM jump in ONE fp32 pass
//        x0 = clamp(f(x_t,t), -1, 1); eps = (x_t - sqrt(a_t) x0)/sqrt(1-a_t)
//        x_{t-k} = sqrt(a_{t-k}) x0 + sqrt(1-a_{t-k}) eps
//    (algebraically the update of ViT.py:229-234).  The 4 coefficients come
//    from a device table so a captured sampler graph has no host scalars.
//  * randn: counter-based normal (Box-Muller over the dropout hash), graph-safe.
//  * q_sample: sqrt(a_t) x0 + sqrt(1-a_t) eps, a_t = 1 - sqrt((t+1)/T)
//    (diffusion_loader.py:50-54), per-sample t.
//  * pixelate_pair / cold_batch: the cold degradation of diffusion_loader.py:79-97
//    (NEAREST down to floor(W/2^t), NEAREST back up) for (t, t-1) in one pass;
//    cold_batch also draws the batch (pool index, t in 1..max_t) on device.
#include "common.h"
#include "kernels.h"

namespace dc {

__global__ __launch_bounds__(256) void ddim_step_kernel(const float* __restrict__ xt, const float* __restrict__ x0r,
                                                        float* __restrict__ xn, float* __restrict__ x0o,
                                                        const float* __restrict__ coef, int64_t n) {
  const float sa = coef[0], s1a = coef[1], sak = coef[2], s1ak = coef[3];
  const float inv = 1.f / s1a;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float x0 = fminf(fmaxf(x0r[i], -1.f), 1.f);
    const float eps = (xt[i] - sa * x0) * inv;
    if (x0o) x0o[i] = x0;
    xn[i] = sak * x0 + s1ak * eps;
  }
}

__device__ __forceinline__ float u01(uint32_t h) { return ((float)(h >> 8) + 0.5f) * (1.0f / 16777216.0f); }

__global__ __launch_bounds__(256) void randn_kernel(float* __restrict__ out, int64_t n, const int64_t* __restrict__ rng,
                                                    int site) {
  const uint32_t salt = site_salt(rng, site);
  const int64_t pairs = (n + 1) / 2;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < pairs; i += (int64_t)gridDim.x * 256) {
    const float a = u01(mix32(((uint32_t)(2 * i) * 0x9E3779B1u) ^ salt));
    const float b = u01(mix32(((uint32_t)(2 * i + 1) * 0x9E3779B1u) ^ salt));
    const float r = sqrtf(-2.f * __logf(a));
    float s, c;
    __sincosf(6.283185307179586f * b, &s, &c);
    out[2 * i] = r * c;
    if (2 * i + 1 < n) out[2 * i + 1] = r * s;
  }
}

__global__ __launch_bounds__(256) void q_sample_kernel(const float* __restrict__ x0, const int64_t* __restrict__ t,
                                                       const float* __restrict__ eps, float* __restrict__ out, int B,
                                                       int64_t per, int T) {
  const int64_t n = (int64_t)B * per;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int b = (int)(i / per);
    const float a = (float)(1.0 - sqrt(((double)t[b] + 1.0) / (double)T));
    out[i] = sqrtf(a) * x0[i] + sqrtf(1.f - a) * eps[i];
  }
}


__global__ __launch_bounds__(256) void pixelate_pair_kernel(const float* __restrict__ img, const int64_t* __restrict__ idx,
                                                            const int64_t* __restrict__ t, float* __restrict__ xt,
                                                            float* __restrict__ xtm1, int B, int C, int H, int W) {
  const int64_t n = (int64_t)B * C * H * W;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    const int x = (int)(e % W);
    int64_t r = e / W;
    const int y = (int)(r % H);
    r /= H;
    const int c = (int)(r % C);
    const int b = (int)(r / C);
    const int64_t src = idx ? idx[b] : b;
    const int tt = (int)t[b];
    const float* im = img + ((size_t)src * C + c) * H * W;
    const int f1 = 1 << tt, f0 = 1 << (tt - 1);
    xt[e] = im[(size_t)pix_src(y, H, f1) * W + pix_src(x, W, f1)];
    xtm1[e] = im[(size_t)pix_src(y, H, f0) * W + pix_src(x, W, f0)];
  }
}

__global__ void cold_draw_kernel(const int64_t* __restrict__ rng, int site, int pool_n, int max_t, int B,
                                 int64_t* __restrict__ idx, int64_t* __restrict__ t, int draw_idx) {
  const uint32_t salt = site_salt(rng, site);
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    if (draw_idx) idx[b] = mix32(((uint32_t)(2 * b) * 0x9E3779B1u) ^ salt) % (uint32_t)pool_n;
    t[b] = 1 + mix32(((uint32_t)(2 * b + 1) * 0x9E3779B1u) ^ salt) % (uint32_t)max_t;
  }
}

// cold_draw + pixelate_pair in ONE launch: every element recomputes its sample's
// (pool index, t) from the counter hash (two mix32, cheaper than a dependent
// launch); the first element of each sample also stores them for the model.
__global__ __launch_bounds__(256) void cold_batch_kernel(const float* __restrict__ pool, int pool_n,
                                                         const int64_t* __restrict__ rng, int site, int max_t,
                                                         int64_t* __restrict__ idx, int64_t* __restrict__ t,
                                                         int draw_idx, float* __restrict__ xt, float* __restrict__ xtm1,
                                                         int B, int C, int H, int W, const int64_t* __restrict__ idx_ctr,
                                                         int idx_rows, int idx_stride) {
  const uint32_t salt = site_salt(rng, site);
  if (idx_ctr) idx += (idx_ctr[0] % idx_rows) * idx_stride;  // stepped index table row
  const int64_t per = (int64_t)C * H * W;
  const int64_t n = (int64_t)B * per;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    const int b = (int)(e / per);
    const int64_t rem = e - (int64_t)b * per;
    const int64_t src = draw_idx ? (int64_t)(mix32(((uint32_t)(2 * b) * 0x9E3779B1u) ^ salt) % (uint32_t)pool_n)
                                 : idx[b];
    const int tt = 1 + (int)(mix32(((uint32_t)(2 * b + 1) * 0x9E3779B1u) ^ salt) % (uint32_t)max_t);
    if (rem == 0) {
      if (draw_idx) idx[b] = src;
      t[b] = tt;
    }
    const int x = (int)(rem % W);
    const int64_t r = rem / W;
    const int y = (int)(r % H);
    const int c = (int)(r / H);
    const float* im = pool + ((size_t)src * C + c) * H * W;
    const int f1 = 1 << tt, f0 = 1 << (tt - 1);
    xt[e] = im[(size_t)pix_src(y, H, f1) * W + pix_src(x, W, f1)];
    xtm1[e] = im[(size_t)pix_src(y, H, f0) * W + pix_src(x, W, f0)];
  }
}

// Gaussian DDIM batch in ONE launch (GaussianBatcher; diffusion_loader.py:24-58):
// pool index + t ~ U{0..T-1} per sample from the data site's hash, eps from the
// noise site, x_t = q_sample(x0, t, eps); the fused patch-embed path derives the
// same values (embed.hip).
__global__ __launch_bounds__(256) void gauss_batch_kernel(const float* __restrict__ pool, int pool_n,
                                                          const int64_t* __restrict__ rng, int site, int noise_site,
                                                          int T, int64_t* __restrict__ idx, int64_t* __restrict__ t,
                                                          int draw_idx, float* __restrict__ xt, float* __restrict__ x0o,
                                                          int B, int per, const int64_t* __restrict__ idx_ctr,
                                                          int idx_rows, int idx_stride) {
  const uint32_t salt = site_salt(rng, site), nsalt = site_salt(rng, noise_site);
  if (idx_ctr) idx += (idx_ctr[0] % idx_rows) * idx_stride;  // stepped index table row
  const int n = B * per;
  for (int e = blockIdx.x * 256 + threadIdx.x; e < n; e += gridDim.x * 256) {
    const int b = e / per, rem = e - b * per;
    const int src = draw_idx ? cold_draw_idx(salt, b, pool_n) : (int)idx[b];
    const int tt = gauss_draw_t(salt, b, T);
    if (rem == 0) {
      if (draw_idx) idx[b] = src;
      t[b] = tt;
    }
    float sa, s1a;
    gauss_coef(tt, T, sa, s1a);
    const float x0 = pool[(size_t)src * per + rem];
    x0o[e] = x0;
    xt[e] = sa * x0 + s1a * gauss_eps(nsalt, (uint32_t)e);
  }
}

static int g_grid(int64_t n) {
  int64_t g = (n + 255) / 256;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace dc

using namespace dc;

void ddim_step_launch(const float* x_t, const float* x0_raw, float* x_next, float* x0_out, const float* coef,
                      int64_t n, hipStream_t stream) {
  hipLaunchKernelGGL(ddim_step_kernel, dim3(g_grid(n)), dim3(256), 0, stream, x_t, x0_raw, x_next, x0_out, coef, n);
}

void randn_launch(float* out, int64_t n, const int64_t* rng, int site, hipStream_t stream) {
  hipLaunchKernelGGL(randn_kernel, dim3(g_grid((n + 1) / 2)), dim3(256), 0, stream, out, n, rng, site);
}

void q_sample_launch(const float* x0, const int64_t* t, const float* eps, float* out, int B, int64_t per,
                     int total_steps, hipStream_t stream) {
  hipLaunchKernelGGL(q_sample_kernel, dim3(g_grid((int64_t)B * per)), dim3(256), 0, stream, x0, t, eps, out, B, per,
                     total_steps);
}

void pixelate_pair_launch(const float* img, const int64_t* idx, const int64_t* t, float* x_t, float* x_tm1, int B,
                          int C, int H, int W, hipStream_t stream) {
  hipLaunchKernelGGL(pixelate_pair_kernel, dim3(g_grid((int64_t)B * C * H * W)), dim3(256), 0, stream, img, idx, t,
                     x_t, x_tm1, B, C, H, W);
}

void gauss_batch_launch(const float* pool, int pool_n, const int64_t* rng, int site, int noise_site, int T,
                        float* x_t, float* x0, int64_t* t, int64_t* idx, bool draw_idx, int B, int C, int H, int W,
                        hipStream_t stream, const int64_t* idx_ctr, int idx_rows, int idx_stride) {
  const int per = C * H * W;
  hipLaunchKernelGGL(gauss_batch_kernel, dim3(g_grid((int64_t)B * per)), dim3(256), 0, stream, pool, pool_n, rng, site,
                     noise_site, T, idx, t, draw_idx ? 1 : 0, x_t, x0, B, per, idx_ctr, idx_rows, idx_stride);
}

void cold_batch_launch(const float* pool, int pool_n, const int64_t* rng, int site, float* x_t, float* x_tm1,
                       int64_t* t, int64_t* idx_ws, int B, int C, int H, int W, int max_t, bool draw_idx,
                       hipStream_t stream, const int64_t* idx_ctr, int idx_rows, int idx_stride) {
  hipLaunchKernelGGL(cold_batch_kernel, dim3(g_grid((int64_t)B * C * H * W)), dim3(256), 0, stream, pool, pool_n, rng,
                     site, max_t, idx_ws, t, draw_idx ? 1 : 0, x_t, x_tm1, B, C, H, W, idx_ctr, idx_rows, idx_stride);
}
