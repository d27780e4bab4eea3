// Fused optimizer for the flat parameter arena (multi_gpu_trainer.py:89-134:
// AdamW(wd=0.05) + clip_grad_norm_(1.0) + CosineAnnealingLR stepped per
// iteration + zero_grad), graph-capturable: every scalar that changes per step
// (Adam step, scheduler step, RNG step) lives in device memory.
//
//   sqnorm  : sum((g*scale)^2) over the grad arena -> nparts per-block partials (no
//             same-address atomics; every consumer block sums the few KiB of partials).
//             The single-process step skips it: the weight-gradient launch writes the
//             same partials from its epilogues (gemm.hip WgradSq).
//   adamw   : clip coef from the norm, cosine LR from the device step, bias
//             corrections, decoupled weight decay, moment updates, fp32 master
//             update, bf16 shadow-weight refresh (what the GEMMs read), and the
//             grad zeroing — one pass over the arena.  A non-finite norm skips
//             the update (GradScaler semantics, multi_gpu_trainer.py:131).
//   advance : bump {adam step (unless skipped), scheduler step} and the RNG step.
#include "common.h"
#include "kernels.h"

namespace dc {

// sum of the nparts partials by one workgroup (every adamw block does this redundantly:
// a few KiB from L2, no atomics, no extra launch)
__device__ __forceinline__ float sum_parts(const float* __restrict__ parts, int nparts) {
  __shared__ float red[4];
  float v = 0.f;
  for (int i = threadIdx.x; i < nparts; i += 256) v += parts[i];
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

// Lazy range [lz_lo, lz_hi) of the arena (16-B aligned, whole vectors): parameters
// whose gradient is identically zero for the whole run (cold diffusion's unused
// time-embedding rows, t > log2 W).  With m = v = 0 forever, AdamW reduces to the
// decoupled weight decay p *= (1 - lr_t wd); the kernels skip the range (no loads,
// no stores) and the first block multiplies the pending factor into lazy_decay[0],
// which TrainEngine.materialize_lazy() applies to the range when it is next read.
// Vector index j of the compacted space -> arena vector index (the range removed).
__device__ __forceinline__ int64_t lazy_map(int64_t j, int64_t lo4, int64_t len4) {
  return j < lo4 ? j : j + len4;
}

__global__ __launch_bounds__(256) void sqnorm_kernel(const float* __restrict__ g, int64_t n, float* out, float scale,
                                                     int64_t lo4, int64_t len4) {
  __shared__ float red[4];
  float acc = 0.f;
  const int64_t n4 = n / 4, nc4 = n4 - len4;
  const float4* g4 = reinterpret_cast<const float4*>(g);
  // four independent 16-byte loads in flight per thread before any use
  const int64_t st = (int64_t)gridDim.x * 256;
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * st < nc4; i += 4 * st) {
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = g4[lazy_map(i + u * st, lo4, len4)];
#pragma unroll
    for (int u = 0; u < 4; ++u) acc += v[u].x * v[u].x + v[u].y * v[u].y + v[u].z * v[u].z + v[u].w * v[u].w;
  }
  for (; i < nc4; i += st) {
    const float4 v = g4[lazy_map(i, lo4, len4)];
    acc += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    acc += g[i] * g[i];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = (red[0] + red[1] + red[2] + red[3]) * scale * scale;
}

__device__ __forceinline__ void adamw_elem(float& p, float g, float& m, float& v, float coef, float decay, float b1,
                                           float b2, float step_size, float inv_sbc2, float eps) {
  const float gi = g * coef;
  p *= decay;
  m = b1 * m + (1.f - b1) * gi;
  v = b2 * v + (1.f - b2) * gi * gi;
  p -= step_size * m / (sqrtf(v) * inv_sbc2 + eps);
}

// hyper = {base_lr, beta1, beta2, eps, weight_decay, max_norm, T_max, eta_min}
// step  = {adam_step, sched_step}
__global__ __launch_bounds__(256) void adamw_kernel(float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                                                    float* __restrict__ v, bf16* __restrict__ pb, int64_t n,
                                                    const float* __restrict__ sqnorm, int nparts,
                                                    const int64_t* __restrict__ step,
                                                    const float* __restrict__ hyper, float grad_scale, bool vec,
                                                    int64_t zero_hi, int64_t lo4, int64_t len4,
                                                    float* __restrict__ lazy_decay) {
  const float sq = sum_parts(sqnorm, nparts);
  const bool skip = !isfinite(sq);
  const float base_lr = hyper[0], b1 = hyper[1], b2 = hyper[2], eps = hyper[3], wd = hyper[4];
  const float max_norm = hyper[5], tmax = hyper[6], eta_min = hyper[7];
  float coef = grad_scale;
  if (max_norm > 0.f) coef *= fminf(1.f, max_norm / (sqrtf(sq) + 1e-6f));
  const double t = (double)(step[0] + 1);
  const float bc1 = (float)(1.0 - pow((double)b1, t));
  const float bc2 = (float)(1.0 - pow((double)b2, t));
  float lr = base_lr;
  if (tmax > 0.f) lr = eta_min + (base_lr - eta_min) * 0.5f * (1.f + cosf(3.14159265358979f * (float)step[1] / tmax));
  const float step_size = lr / bc1;
  const float inv_sbc2 = 1.f / sqrtf(bc2);
  const float decay = 1.f - lr * wd;
  if (len4 > 0 && !skip && blockIdx.x == 0 && threadIdx.x == 0) lazy_decay[0] *= decay;
  // 16-byte vectors (the arenas are allocator-aligned; `vec` is checked on the host),
  // scalar tail.  Same math per element as the scalar path.
  const int64_t nv = vec ? n / 4 : 0;
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < nv - len4; j += stride) {
    const int64_t i = lazy_map(j, lo4, len4);
    float4 gv = reinterpret_cast<float4*>(g)[i];
    if (4 * i < zero_hi) reinterpret_cast<float4*>(g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (skip) continue;
    float4 pv = reinterpret_cast<const float4*>(p)[i];
    float4 mv = reinterpret_cast<const float4*>(m)[i];
    float4 vv = reinterpret_cast<const float4*>(v)[i];
    adamw_elem(pv.x, gv.x, mv.x, vv.x, coef, decay, b1, b2, step_size, inv_sbc2, eps);
    adamw_elem(pv.y, gv.y, mv.y, vv.y, coef, decay, b1, b2, step_size, inv_sbc2, eps);
    adamw_elem(pv.z, gv.z, mv.z, vv.z, coef, decay, b1, b2, step_size, inv_sbc2, eps);
    adamw_elem(pv.w, gv.w, mv.w, vv.w, coef, decay, b1, b2, step_size, inv_sbc2, eps);
    reinterpret_cast<float4*>(m)[i] = mv;
    reinterpret_cast<float4*>(v)[i] = vv;
    reinterpret_cast<float4*>(p)[i] = pv;
    if (pb) {
      bf16x4 o;
      o[0] = f2bf(pv.x); o[1] = f2bf(pv.y); o[2] = f2bf(pv.z); o[3] = f2bf(pv.w);
      reinterpret_cast<bf16x4*>(pb)[i] = o;
    }
  }
  for (int64_t i = nv * 4 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    float gi = g[i];
    if (i < zero_hi) g[i] = 0.f;
    if (skip) continue;
    float pi = p[i], mi = m[i], vi = v[i];
    adamw_elem(pi, gi, mi, vi, coef, decay, b1, b2, step_size, inv_sbc2, eps);
    m[i] = mi;
    v[i] = vi;
    p[i] = pi;
    if (pb) pb[i] = f2bf(pi);
  }
}

__global__ __launch_bounds__(256) void advance_kernel(int64_t* step, int64_t* rng, const float* sqnorm,
                                                      int nparts) {
  const float sq = sqnorm ? sum_parts(sqnorm, nparts) : 0.f;
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    if (sqnorm == nullptr || isfinite(sq)) step[0] += 1;
    step[1] += 1;
    rng[1] += 1;
  }
}

}  // namespace dc

using namespace dc;

static int opt_grid(int64_t n) {
  int64_t g = (n / 4 + 255) / 256;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

static void check_lazy(int64_t n, int64_t lz_lo, int64_t lz_hi) {
  if (lz_hi > lz_lo && (lz_lo < 0 || lz_hi > n / 4 * 4 || lz_lo % 4 || lz_hi % 4))
    throw std::runtime_error("optimizer lazy range must be whole 16-B vectors inside the arena");
}

void sqnorm_launch(const float* g, int64_t n, float* out, int nparts, float scale, hipStream_t stream,
                   int64_t lz_lo, int64_t lz_hi) {
  check_lazy(n, lz_lo, lz_hi);
  const int64_t len4 = lz_hi > lz_lo ? (lz_hi - lz_lo) / 4 : 0;
  hipLaunchKernelGGL(sqnorm_kernel, dim3(nparts), dim3(256), 0, stream, g, n, out, scale, lz_lo / 4, len4);
}

void adamw_launch(float* p, float* g, float* m, float* v, void* p_bf16, int64_t n, const float* sqnorm,
                  int nparts, const int64_t* step, const float* hyper, float grad_scale, hipStream_t stream, int64_t zero_hi,
                  int64_t lz_lo, int64_t lz_hi, float* lazy_decay) {
  if (zero_hi < 0 || zero_hi > n) zero_hi = n;
  zero_hi = (zero_hi + 3) / 4 * 4 <= n ? (zero_hi + 3) / 4 * 4 : n;  // whole 16-B vectors
  auto al = [](const void* q, uintptr_t a) { return (reinterpret_cast<uintptr_t>(q) & (a - 1)) == 0; };
  const bool vec = al(p, 16) && al(g, 16) && al(m, 16) && al(v, 16) && (p_bf16 == nullptr || al(p_bf16, 8));
  check_lazy(n, lz_lo, lz_hi);
  int64_t len4 = lz_hi > lz_lo ? (lz_hi - lz_lo) / 4 : 0;
  if (!vec || lazy_decay == nullptr) len4 = 0;
  hipLaunchKernelGGL(adamw_kernel, dim3(opt_grid(n - 4 * len4)), dim3(256), 0, stream, p, g, m, v,
                     reinterpret_cast<bf16*>(p_bf16), n, sqnorm, nparts, step, hyper, grad_scale, vec, zero_hi, lz_lo / 4,
                     len4, lazy_decay);
}

void advance_counters_launch(int64_t* step, int64_t* rng, const float* sqnorm, int nparts, hipStream_t stream) {
  hipLaunchKernelGGL(advance_kernel, dim3(1), dim3(256), 0, stream, step, rng, sqnorm, nparts);
}
