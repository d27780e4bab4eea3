// Common gfx950 (CDNA4) device helpers for the ddim_cold_amd kernels.
//
// * bf16 storage as __bf16, fp32 math/accumulation.
// * MFMA fragment types for v_mfma_f32_16x16x32_bf16 (wave64: lane l holds
//   A[row l&15][k 8(l>>4)+j] / B[k][col l&15]; C/D col = l&15,
//   row = 4(l>>4)+reg).
// * Counter-based dropout hash — bit-identical to
//   ddim_cold_amd/ops/reference.py (keep_mask / site_salt).  Elementwise sites
//   regenerate their masks in backward from (seed, step, site, idx) (the attention
//   kernels store theirs as bits); (seed, step) are read from device memory so
//   graph replays draw fresh masks every step.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dc {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

#define DC_LDS __attribute__((address_space(3)))

__device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }
__device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }

// bare v_exp_f32.  exp2f() adds a denormal-range fix-up around it (v_cmp +
// 2 v_cndmask + v_ldexp per call: 3 of every 4 vector instructions of the
// softmax in the flash forward's loop, counted in its .s); softmax inputs are
// <= 0 (or <= 8 with the lazy max of the flash kernels) and results below
// 2^-126 are negligible against the row sum, so the fix-up buys nothing here.
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// ds_read_b64_tr_b16: per 16-lane group, lane 4q+p addresses row q cols 4p..4p+3
// of a 4x16 block; lane i receives column i (4 rows) -> elements 0..3.
__device__ __forceinline__ bf16x4 lds_read_tr(const bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((DC_LDS bf16x4*)(p));
}

// MFMA operand fragment from a transposed LDS image [k rows][cols] (row stride
// STRIDE bytes): operand rows c0..c0+15, permuted k order
//   element j of lane group g <-> k = 32s + (j<4 ? 4g+j : 16+4g+(j-4)).
template <int STRIDE>
__device__ __forceinline__ bf16x8 frag_t(const char* lds, int c0, int s, int lane) {
  const int i = lane & 15, g = lane >> 4, q = i >> 2, p = i & 3;
  const int ra = 32 * s + 4 * g + q;
  const char* pa = lds + ra * STRIDE + (c0 + 4 * p) * 2;
  const bf16x4 lo = lds_read_tr(reinterpret_cast<const bf16*>(pa));
  const bf16x4 hi = lds_read_tr(reinterpret_cast<const bf16*>(pa + 16 * STRIDE));
  bf16x8 v;
  v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
  v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
  return v;
}

// ----------------------------------------------------------------------------- RNG
__host__ __device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

// rng = device pointer to int64[2] = {seed, step}
__device__ __forceinline__ uint32_t site_salt_v(uint64_t seed, uint64_t step, int site) {
  const uint32_t s_lo = (uint32_t)seed, s_hi = (uint32_t)(seed >> 32);
  const uint32_t a = mix32((uint32_t)step * 0x9E3779B9u + s_hi);
  const uint32_t b = mix32(s_lo ^ a);
  return mix32(b + (uint32_t)site * 0x85EBCA6Bu);
}
__device__ __forceinline__ uint32_t site_salt(const int64_t* rng, int site) {
  return site_salt_v((uint64_t)rng[0], (uint64_t)rng[1], site);
}

// Dropout masks (counter-based): element i of a site keeps iff the 16-bit half
// (i & 1) of drop_mix((i >> 1) * golden + salt) is >= thr, thr = 2 round(p 2^15)
// (even, so "half >= thr" is "(half >> 1) >= thr / 2": the attention forward tests
// both halves of a hash at once with 16-bit packed ops).  One hash serves an aligned
// pair of elements.
//
// drop_mix: xorshift-multiply rounds with 24-bit multipliers.  v_mul_u32_u24 is full
// rate, v_mul_lo_u32 (lowbias32's 32-bit multiplies, mix32 above) quarter rate, and
// the shifts by 16 fold into one SDWA xor each: 5 vector instructions instead of
// ~13 issue cycles, in the flash-attention forward's VALU-bound softmax loop.  The
// first multiply reads only the low 24 bits (the top byte enters through the first
// xorshift), so this is not a bijection; the dropout statistics are what matter
// (drop rate, pair / neighbour independence at p = 0.1 over 2^25 elements: within
// sampling noise; tests/test_diffusion_data.py::test_drop_mix_statistics).
constexpr uint32_t DROP_MUL1 = 0xED5AD5u, DROP_MUL2 = 0x2C1B3Du;  // 24-bit odd constants
__host__ __device__ __forceinline__ uint32_t drop_mix(uint32_t x) {
  x ^= x >> 16;
  x = (x & 0xFFFFFFu) * DROP_MUL1;
  x ^= x >> 16;
  x = (x & 0xFFFFFFu) * DROP_MUL2;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint32_t drop_hash(uint32_t salt, uint32_t pair) {
  return drop_mix(pair * 0x9E3779B1u + salt);
}

__device__ __forceinline__ bool dropout_keep(uint32_t salt, uint32_t idx, uint32_t thresh) {
  const uint32_t h = drop_hash(salt, idx >> 1);
  return ((idx & 1u) ? (h >> 16) : (h & 0xFFFFu)) >= thresh;
}

// keep flags of the 4 consecutive elements idx..idx+3 (idx even): two hashes
__device__ __forceinline__ void dropout_keep4(uint32_t salt, uint32_t idx, uint32_t thresh, bool (&k)[4]) {
  const uint32_t h0 = drop_hash(salt, idx >> 1), h1 = drop_hash(salt, (idx >> 1) + 1u);
  k[0] = (h0 & 0xFFFFu) >= thresh;
  k[1] = (h0 >> 16) >= thresh;
  k[2] = (h1 & 0xFFFFu) >= thresh;
  k[3] = (h1 >> 16) >= thresh;
}

// dropout_keep4 with the pair hash input precomputed: pg = (idx >> 1) * golden for an even
// idx.  Consecutive tiles of one mask row differ by a constant number of pairs, so callers
// hoist the multiply (v_mul_lo_u32, quarter rate) out of their tile loops and add a
// (constant-folded) offset.  Same flags as dropout_keep4.
constexpr uint32_t DROP_GOLDEN = 0x9E3779B1u;
__device__ __forceinline__ void dropout_keep4_pg(uint32_t salt, uint32_t pg, uint32_t thresh, bool (&k)[4]) {
  const uint32_t h0 = drop_mix(pg + salt), h1 = drop_mix(pg + DROP_GOLDEN + salt);
  k[0] = (h0 & 0xFFFFu) >= thresh;
  k[1] = (h0 >> 16) >= thresh;
  k[2] = (h1 & 0xFFFFu) >= thresh;
  k[3] = (h1 >> 16) >= thresh;
}

// attention-probability masks index (b, h, q, key) as (bh * N + q) * ld + key
// with the row stride padded to 4 (aligned pairs / quads within a row)
__host__ __device__ __forceinline__ int attn_mask_ld(int N) { return (N + 3) & ~3; }

// drop mask of both 16-bit halves of a pair hash: 0xFFFF in each half whose element
// drops ((half >> 1) < thr / 2, i.e. half < thr for the even thr), 0 where it keeps --
// three packed 16-bit ops for two elements; AND-NOT it onto the packed bf16 pair
__device__ __forceinline__ uint32_t drop_mask2(uint32_t h, uint32_t thr_half2) {
  typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
  typedef short i16x2 __attribute__((ext_vector_type(2)));
  const u16x2 d = (__builtin_bit_cast(u16x2, h) >> (unsigned short)1) - __builtin_bit_cast(u16x2, thr_half2);
  return __builtin_bit_cast(uint32_t, __builtin_bit_cast(i16x2, d) >> (short)15);
}

// even threshold 2 round(p 2^15) (see drop_mix)
inline uint32_t drop_threshold_host(double p) {
  double v = p * 32768.0 + 0.5;
  if (v >= 32768.0) return 65536u;  // drop everything
  if (v <= 0.0) return 0u;
  return 2u * (uint32_t)v;
}

// ----------------------------------------------------------------------------- reductions
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned int gu32;

// write-through 8-B store / L1-bypassing 8-B load (agent-scope relaxed atomics:
// global_store_dwordx2 sc1 / global_load_dwordx2 sc1)
__device__ __forceinline__ void st8_sc1(void* p, uint64_t v) {
  __hip_atomic_store((gu64*)p, (unsigned long long)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld8_sc1(const void* p) {
  return __hip_atomic_load((gu64*)const_cast<void*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_f2_sc1(float* p, float a, float b) {
  st8_sc1(p, (uint64_t)__float_as_uint(a) | ((uint64_t)__float_as_uint(b) << 32));
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// Column sums of R slot rows (the LayerNorm dgamma/dbeta finalize), fixed order
// (deterministic): a workgroup of NT threads covers 16 columns c0.. with NT/16 slot lanes,
// lane l summing rows l, l + NT/16, ... (eight loads in flight), then the lanes in lane
// order.  red: >= NT floats of LDS.  Returns the column total in the threads of lane 0
// (column c0 + threadIdx.x), 0 elsewhere.
template <int NT>
__device__ __forceinline__ float slot_colsum16(const float* __restrict__ w, int C, int R, int c0, float* red) {
  constexpr int SL = NT / 16;
  const int cl = threadIdx.x & 15, sl = threadIdx.x >> 4;
  const int c = c0 + cl;
  float s = 0.f;
  if (c < C) {
    int r = sl;
    for (; r + 7 * SL < R; r += 8 * SL) {
      float a[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) a[u] = w[(size_t)(r + u * SL) * C + c];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += a[u];
    }
    for (; r < R; r += SL) s += w[(size_t)r * C + c];
  }
  red[sl * 16 + cl] = s;
  __syncthreads();
  float t = 0.f;
  if (sl == 0) {
    for (int l = 0; l < SL; ++l) t += red[l * 16 + cl];
  }
  return t;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Standard normal CDF Phi(x) = (1 + erf(x / sqrt 2)) / 2 for the exact (erf) GELU of
// nn.GELU (ViT.py:80).  erff() costs ~40 vector instructions per element (range
// split + an exp inside; the GELU GEMM epilogue ran ~31 VALU per MFMA in the PMC
// table).  Abramowitz & Stegun 7.1.28: erf(z) = 1 - t^-16, t = 1 + a1 z + .. + a6 z^6
// (z >= 0, |error| <= 3e-7), i.e. 6 FMAs, 4 squarings and one v_rcp; the lower tail
// 1 - erf(z) = t^-16 comes out directly (no cancellation).  The error is three
// orders of magnitude below the bf16 rounding of the stored activations.
__device__ __forceinline__ float norm_cdf(float x) {
  const float z = fabsf(x) * 0.70710678118654752f;
  float t = fmaf(z, 4.30638e-5f, 2.765672e-4f);
  t = fmaf(z, t, 1.520143e-4f);
  t = fmaf(z, t, 9.2705272e-3f);
  t = fmaf(z, t, 4.22820123e-2f);
  t = fmaf(z, t, 7.05230784e-2f);
  t = fmaf(z, t, 1.0f);
  t = t * t;
  t = t * t;
  t = t * t;
  t = t * t;
  const float tail = 0.5f * __builtin_amdgcn_rcpf(t);  // Phi(-|x|); 0 once t^16 overflows
  return x >= 0.f ? 1.0f - tail : tail;
}
__device__ __forceinline__ float gelu_f(float x) { return x * norm_cdf(x); }
__device__ __forceinline__ float gelu_grad_f(float x) {
  const float pdf = fexp2(-0.72134752044448170f * x * x) * 0.39894228040143268f;  // exp(-x^2/2)/sqrt(2 pi)
  return norm_cdf(x) + x * pdf;
}

inline int cdiv(int a, int b) { return (a + b - 1) / b; }

// Cold-diffusion pixelation (diffusion_loader.py:79-83, NEAREST down to W/f then
// NEAREST back up): source row/column of output pixel y.
// torch 'nearest' index: min(floor(dst * in/out), in-1)
__device__ __forceinline__ int nearest_src(int dst, int in, int out) {
  const float scale = (float)in / (float)out;
  const int s = (int)floorf((float)dst * scale);
  return s < in - 1 ? s : in - 1;
}
__device__ __forceinline__ int pix_src(int y, int H, int f) {
  int ts = H / f;
  if (ts < 1) ts = 1;
  return nearest_src(nearest_src(y, ts, H), H, ts);
}

// Per-sample cold-batch draw (pool index, t in 1..max_t) from the data site's
// counter hash: cold_batch_kernel and the fused cold patchify derive the same pair.
__device__ __forceinline__ int cold_draw_idx(uint32_t salt, int b, int pool_n) {
  return (int)(mix32(((uint32_t)(2 * b) * 0x9E3779B1u) ^ salt) % (uint32_t)pool_n);
}
__device__ __forceinline__ int cold_draw_t(uint32_t salt, int b, int max_t) {
  return 1 + (int)(mix32(((uint32_t)(2 * b + 1) * 0x9E3779B1u) ^ salt) % (uint32_t)max_t);
}

// Gaussian DDIM batch (diffusion_loader.py:24-58): t ~ U{0..T-1} from the same
// hash slot as the cold t; eps = element o of randn_kernel's draw over the
// [B,C,H,W] noise tensor (Box-Muller pair o/2, cos for even o, sin for odd);
// x_t = sqrt(a_t) x0 + sqrt(1-a_t) eps, a_t = 1 - sqrt((t+1)/T) (q_sample_kernel).
__device__ __forceinline__ int gauss_draw_t(uint32_t salt, int b, int T) {
  return (int)(mix32(((uint32_t)(2 * b + 1) * 0x9E3779B1u) ^ salt) % (uint32_t)T);
}
__device__ __forceinline__ float gauss_eps(uint32_t nsalt, uint32_t o) {
  const uint32_t i = o >> 1;
  const float a = ((float)(mix32((2u * i * 0x9E3779B1u) ^ nsalt) >> 8) + 0.5f) * (1.0f / 16777216.0f);
  const float b = ((float)(mix32(((2u * i + 1u) * 0x9E3779B1u) ^ nsalt) >> 8) + 0.5f) * (1.0f / 16777216.0f);
  const float r = sqrtf(-2.f * __logf(a));
  float s, c;
  __sincosf(6.283185307179586f * b, &s, &c);
  return (o & 1u) ? r * s : r * c;
}
__device__ __forceinline__ void gauss_coef(int t, int T, float& sa, float& s1a) {
  const float a = (float)(1.0 - sqrt(((double)t + 1.0) / (double)T));
  sa = sqrtf(a);
  s1a = sqrtf(1.f - a);
}

}  // namespace dc
