// Image-group persistent forward of the transformer blocks for gfx950
// (ViT-tiny shape: D = 384, 12 heads of 32, N <= 80 tokens per image;
// ViT.py:120-138 / ViT_draft2drawing.py:230-231 semantics, LayerNorm folded).
//
// Why: at this model size every op of the block-by-block launch sequence
// (QKV GEMM, attention, proj+residual, fc1+GELU, fc2+residual) is a ~400-
// workgroup launch whose time is dispatch ramp + first-load latency +
// epilogue drain, not arithmetic (profiles/README.md), and each op waits for
// the whole previous op over the whole batch.  But every op of a block is
// ROW-LOCAL (attention: image-local), so the batch splits into independent
// images.  Here one launch runs ALL blocks: a group of G = 6 workgroups owns
// one image (65 token rows, padded to 80 = 5 MFMA row tiles), workgroup j of
// the group owns output columns [64j, 64j + 64) of every 384-wide op and the
// QKV columns of heads 2j, 2j + 1 (so attention of those heads needs no
// hand-off: q/k/v stay in LDS).  Per block a workgroup does
//
//   QKV(fold LN1) -> attention(2 heads) -> publish o
//   gather o      -> proj + residual    -> publish x1 (bf16 copy) + LN2 stats
//   gather x1     -> fc1(fold LN2)+GELU -> publish h
//   gather h      -> fc2 + residual     -> publish x (bf16 copy) + LN stats
//
// and the only synchronisation is a per-image counter among the 6 workgroups
// of the group (4 hand-offs per block), never a grid-wide seam.  The weight
// panel of the next GEMM (64 rows x 384, 48 KiB, LDS-DMA) is always in flight
// before the hand-off wait, so the wait overlaps the weight stream.
//
// Hand-off protocol (MI355X_MICROARCH.md "inter-workgroup visibility", the
// sc1 row; cdna_hip_programming.md Guideline 16): every handed-off byte is
// stored write-through (sc1, 8 B), every storing wave drains with
// `s_waitcnt vmcnt(0)`, a workgroup barrier, then ONE lane adds 1 to the
// image's counter (agent-scope atomic).  The consumer's lane 0 polls the
// counter (relaxed sc1 loads + s_sleep, bounded: a give-up sets `err` instead
// of hanging), a workgroup barrier, then EVERY load of handed-off bytes is an
// sc1 load to registers (gathers: 16-B buffer_load sc1; statistics: 8-B).
// All other loads read bytes no other workgroup writes in this launch
// (weights, this workgroup's own residual columns).  Every buffer is written
// at most once per launch, and the counters are zeroed by the launcher.
//
// Numerics: the GEMMs issue exactly the MFMA sequence of gemm_dma_body (same
// k order), the epilogues are the gemm_epi.h math (VecEpi / attention short
// kernel), so outputs match the per-op launch sequence bit for bit.
#include "common.h"
#include "kernels.h"
#include "gemm_common.h"
#include "gemm_epi.h"
#include <algorithm>

namespace dc {
namespace vg {

constexpr int D = 384, H = 12, HD = 32, G = 6, RP = 80, KT = 6, FM = RP / 16;
constexpr int ROWB = 128;                          // bytes per LDS image row (64 k, bf16)
constexpr int A_BYTES = KT * RP * ROWB;            // 61440: gathered A panel [kt][80 rows][128 B]
constexpr int B_BYTES = KT * 64 * ROWB;            // 49152: one weight chunk [kt][64 rows][128 B]
constexpr int LDS_BYTES = A_BYTES + 2 * B_BYTES + RP * 8;   // 160384: + per-row (mean, rstd)
constexpr int NPK = 96;                            // padded keys (3 x 32)
constexpr int AS = 2 * HD + 32;                    // attention image row stride (bytes)
constexpr int QI = RP * AS;                        // one head's Q image (in the A region)
constexpr int KVI = NPK * AS;                      // one head's K or V image (in weight buffer 0)
static_assert(2 * QI + 2 * KVI <= B_BYTES && 2 * KVI <= A_BYTES && LDS_BYTES <= 160 * 1024, "LDS map");
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

// attention image helpers (attention.hip's short kernel layout, hd 32)
__device__ __forceinline__ bf16x8 frag_row32(const char* lds, int r, int g) {
  return *reinterpret_cast<const bf16x8*>(lds + r * AS + 16 * g);
}
__device__ __forceinline__ bf16x8 pack8(const f32x4& a, const f32x4& b) {
  bf16x8 v;
  v[0] = f2bf(a[0]); v[1] = f2bf(a[1]); v[2] = f2bf(a[2]); v[3] = f2bf(a[3]);
  v[4] = f2bf(b[0]); v[5] = f2bf(b[1]); v[6] = f2bf(b[2]); v[7] = f2bf(b[3]);
  return v;
}
__device__ __forceinline__ bf16x4 pack4(const f32x4& a) {
  bf16x4 v;
  v[0] = f2bf(a[0]); v[1] = f2bf(a[1]); v[2] = f2bf(a[2]); v[3] = f2bf(a[3]);
  return v;
}

struct DevBlock {
  const bf16 *qkv_wf, *proj_w, *fc1_wf, *fc2_w;
  const float *qkv_bf, *qkv_c, *proj_b, *fc1_bf, *fc1_c, *fc2_b;
  const bf16* xb_in;
  const float *st_in, *x_in;
  bf16 *qkv, *o, *x1b, *u, *h, *xb_out;
  float *lse, *x1, *st1, *x_out, *st_out, *m1, *r1, *m2, *r2;
  int site_a, site_p, site_d1, site_f1, site_f2, site_d2;
  uint32_t thr_dp;
  float sc_dp;
};

struct DevArgs {
  DevBlock blk[VG_MAXL];
  int L, B, N, img0;
  const int64_t* rng;
  uint32_t thr_drop, thr_attn;
  float sc_drop, sc_attn, scale, eps;
  unsigned* ctr;
  unsigned* err;
  unsigned long long* stamps;  // optional: [grid][L][16] s_memrealtime stamps (profiling)
};

// profiling stamp (100 MHz realtime counter), lane 0 only, off when stamps == nullptr
__device__ __forceinline__ void stamp(const DevArgs& a, int l, int k) {
  if (a.stamps != nullptr && threadIdx.x == 0)
    a.stamps[((size_t)blockIdx.x * VG_MAXL + l) * 32 + k] = __builtin_amdgcn_s_memrealtime();
}

// ------------------------------------------------------------------ hand-off
__device__ __forceinline__ void wait_count(unsigned* ctr, unsigned target, unsigned* err) {
  if (threadIdx.x == 0 && target > 0) {
    unsigned spins = 0;
    while (__hip_atomic_load((gu32*)ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > (1u << 22)) {  // seconds: give up (garbage out, flagged) instead of hanging
        __hip_atomic_fetch_or((gu32*)err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keep the sc1 loads below the poll
}

__device__ __forceinline__ void publish(unsigned* ctr) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // EVERY storing wave drains its sc1 stores
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add((gu32*)ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------------ operand staging
// the image's token rows of a handed-off [M][D] bf16 tensor -> registers (sc1,
// rows >= N read as zero by the buffer bounds check) -> swizzled A image
struct Gather {
  static constexpr int CPR = D / 8;                // 48 16-B chunks per row
  static constexpr int PER = RP * CPR / 256;       // 15 per thread
  u32x4 v[PER];
  __device__ __forceinline__ void load(const bf16* img_rows, int N) {
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(img_rows), (short)0, N * D * 2, 0x00020000);
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = threadIdx.x + 256 * i;
      const int r = c / CPR, cc = c - r * CPR;
      v[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (r * D + cc * 8) * 2, 0, 16);
    }
  }
  __device__ __forceinline__ void store(char* A) const {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = threadIdx.x + 256 * i;
      const int r = c / CPR, cc = c - r * CPR;
      const int kt = cc >> 3, kc = cc & 7;
      *reinterpret_cast<u32x4*>(A + kt * RP * ROWB + r * ROWB + 16 * (kc ^ swz(r))) = v[i];
    }
  }
};

// a 64-row weight panel (rows r0.., all 384 k) -> weight buffer, LDS-DMA (12 ops per wave)
__device__ __forceinline__ void issue_weights(char* buf, const bf16* W, int wrows, int r0, int wave, int lane) {
  DmaOperand<64, false> op;
  op.init(W, D, wrows, r0, wave, lane);
#pragma unroll
  for (int kt = 0; kt < KT; ++kt) op.issue(buf + kt * 64 * ROWB, kt, wave);
}

// C[80 x 64] = A[80 x 384] W^T, accumulated TRANSPOSED: acc[i] = mfma(W frag,
// A frag) so lane (g, li) holds row 16i + li, columns 16w + 4g .. +3 of the
// wave's 16 -- four consecutive outputs of one row, the vector layout every
// epilogue wants, with no quad transpose (the k order is gemm_dma_body's).
__device__ __forceinline__ void mma64t(const char* A, const char* Bw, f32x4 (&acc)[FM], int wave, int g, int li) {
  // software-pipelined: the fragments of k32-step t+1 are read while step t's MFMAs run
  // (one wave per SIMD: nothing else hides the LDS latency)
  constexpr int STEPS = 2 * KT;
  bf16x8 bf[2], af[2][FM];
  auto load = [&](int t, int slot) {
    const char* la = A + (t >> 1) * RP * ROWB;
    const char* lb = Bw + (t >> 1) * 64 * ROWB;
    bf[slot] = frag_k(lb, 16 * wave + li, t & 1, g);
#pragma unroll
    for (int i = 0; i < FM; ++i) af[slot][i] = frag_k(la, 16 * i + li, t & 1, g);
  };
#pragma unroll
  for (int i = 0; i < FM; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  load(0, 0);
#pragma unroll
  for (int t = 0; t < STEPS; ++t) {
    if (t + 1 < STEPS) load(t + 1, (t + 1) & 1);
#pragma unroll
    for (int i = 0; i < FM; ++i) acc[i] = mfma16(bf[t & 1], af[t & 1][i], acc[i]);
  }
}

// Row LayerNorm statistics of the image's rows from the producer's slots (sc1):
// thread t < N owns row t, sums the 12 {sum, sum^2} slots in VecEpi's order
// ((s_q + s_q+4 + s_q+8) per q, then (q0 + q1) + (q2 + q3)), writes (mean, rstd)
// to `ms` in LDS and optionally to the saved mean / rstd.
struct RowStats {
  float2 s[D / 32];
  __device__ __forceinline__ void load(const float* st, int row0, int N) {
    const int t = threadIdx.x;
#pragma unroll
    for (int k = 0; k < D / 32; ++k)
      s[k] = t < N ? ld2f_pub<true>(st + 2 * ((size_t)(row0 + t) * (D / 32) + k)) : make_float2(0.f, 0.f);
  }
  __device__ __forceinline__ void finish(float2* ms, float eps, int row0, int N, float* mean_out, float* rstd_out) {
    const int t = threadIdx.x;
    if (t >= RP) return;
    float2 q[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      q[k] = s[k];
      q[k] = f2add(q[k], s[k + 4]);
      q[k] = f2add(q[k], s[k + 8]);
      q[k] = f2add(q[k], make_float2(0.f, 0.f));
    }
    const float2 tot = f2add(f2add(q[0], q[1]), f2add(q[2], q[3]));
    const float invd = 1.0f / (float)D;
    const float mu = tot.x * invd;
    const float var = fmaxf(tot.y * invd - mu * mu, 0.f);
    const float2 r = make_float2(mu, rsqrtf(var + eps));
    ms[t] = r;
    if (mean_out != nullptr && t < N) {
      mean_out[row0 + t] = r.x;
      rstd_out[row0 + t] = r.y;
    }
  }
};

// residual epilogue (EPI_RESID math of VecEpi, LayerNorm producer) on the
// transposed accumulators: x_out = res + DropPath(Dropout(acc + bias)) on the
// workgroup's own columns, bf16 copy and the {sum, sum^2} slots published.  A
// 32-column slot spans waves 2k, 2k+1: the odd wave hands its 4-column partials
// to the even one through LDS, which then reduces over the 4 lane groups -- the
// summation order of VecEpi (two 16-column fragments, then lane quads).
// `prefetch` issues the epilogue's global loads; call it BEFORE the next weight
// panel's LDS-DMA: loads complete in issue order, so a load queued behind a
// 48 KiB DMA waits for it.
struct ResidEpi {
  const float* res;
  const float* bias;
  float* xo;
  bf16* xb;
  float* st;
  int site_drop, site_dp;
  uint32_t thr_dp;
  float sc_dp;
  f32x4 colb, pre[FM];

  __device__ __forceinline__ void prefetch(int row0, int N, int n, int li) {
    colb = ld4(bias + n);
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int r = 16 * i + li;
      pre[i] = r < N ? ld4(res + (size_t)(row0 + r) * D + n) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  __device__ __forceinline__ void finish(const DevArgs& a, const f32x4 (&acc)[FM], int row0, int N, int col0, int wave,
                                         int g, int li, char* xch) {
    const int n = col0 + 16 * wave + 4 * g;
    const uint32_t salt_drop = a.thr_drop ? site_salt(a.rng, site_drop) : 0u;
    const uint32_t salt_dp = thr_dp ? site_salt(a.rng, site_dp) : 0u;
    float2 part[FM];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      part[i] = make_float2(0.f, 0.f);
      const int r = 16 * i + li;
      if (r >= N) continue;
      const int m = row0 + r;
      const long long idx = (long long)m * D + n;
      const bool keep_row = thr_dp ? dropout_keep(salt_dp, (uint32_t)(m / N), thr_dp) : true;
      f32x4 v = acc[i] + colb;
      bool kp[4] = {true, true, true, true};
      if (a.thr_drop) dropout_keep4(salt_drop, (uint32_t)idx, a.thr_drop, kp);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        float ev = v[c];
        if (a.thr_drop) ev = kp[c] ? ev * a.sc_drop : 0.f;
        if (thr_dp) ev = keep_row ? ev * sc_dp : 0.f;
        v[c] = pre[i][c] + ev;
      }
      st4(xo + idx, v);
      part[i] = f2add(part[i], stat4(v));
      st4bf_pub<true>(xb + idx, v);
    }
    float2* xp = reinterpret_cast<float2*>(xch) + (wave >> 1) * FM * 64;
    if (wave & 1) {
#pragma unroll
      for (int i = 0; i < FM; ++i) xp[i * 64 + (threadIdx.x & 63)] = part[i];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();  // LDS only: the sc1 stores drain once, in publish()
    if (!(wave & 1)) {
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        float2 t = f2add(part[i], xp[i * 64 + (threadIdx.x & 63)]);
        t = f2add(t, make_float2(__shfl_xor(t.x, 16, 64), __shfl_xor(t.y, 16, 64)));
        t = f2add(t, make_float2(__shfl_xor(t.x, 32, 64), __shfl_xor(t.y, 32, 64)));
        const int r = 16 * i + li;
        if (g == 0 && r < N)
          st2f_pub<true>(st + 2 * ((size_t)(row0 + r) * (D / 32) + (col0 + 32 * (wave >> 1)) / 32), t);
      }
    }
  }
};

// ------------------------------------------------------------------ attention (attn_fwd_short_kernel math)
// NU (1 or 2) independent (head, 16-query group) units of one wave, their
// instruction streams interleaved (one wave per SIMD: the second unit's MFMAs
// and exponentials fill the first one's latency)
struct AttnUnit {
  const char *Qi, *Ki, *Vi;
  int h, qg;
};
template <int NU>
__device__ __forceinline__ void attention_units(const DevArgs& a, const DevBlock& w, const AttnUnit (&un)[NU], int b,
                                                int N, int lane) {
  constexpr int KTK = NPK / 16;
  const int g = lane >> 4, li = lane & 15;
  const float sl2 = a.scale * LOG2E;
  const bool drop = a.thr_attn != 0;
  const uint32_t salt = drop ? site_salt(a.rng, w.site_a) : 0u;
  f32x4 st[NU][KTK];
  float mx[NU], l[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const bf16x8 qf = frag_row32(un[u].Qi, un[u].qg * 16 + li, g);
#pragma unroll
    for (int t = 0; t < KTK; ++t)
      st[u][t] = mfma16(frag_row32(un[u].Ki, 16 * t + li, g), qf, f32x4{0.f, 0.f, 0.f, 0.f});
  }
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    mx[u] = -INFINITY;
#pragma unroll
    for (int t = 0; t < KTK; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = (16 * t + 4 * g + r) < N ? st[u][t][r] * sl2 : -INFINITY;
        st[u][t][r] = v;
        mx[u] = fmaxf(mx[u], v);
      }
    mx[u] = fmaxf(mx[u], __shfl_xor(mx[u], 16, 64));
    mx[u] = fmaxf(mx[u], __shfl_xor(mx[u], 32, 64));
  }
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int q = un[u].qg * 16 + li;
    const uint32_t rowidx = (uint32_t)(((size_t)(b * H + un[u].h) * N + q) * attn_mask_ld(N));
    l[u] = 0.f;
#pragma unroll
    for (int t = 0; t < KTK; ++t) {
      bool kp[4] = {true, true, true, true};
      if (drop) dropout_keep4(salt, rowidx + (uint32_t)(16 * t + 4 * g), a.thr_attn, kp);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float pv = exp2f(st[u][t][r] - mx[u]);
        l[u] += pv;
        if (drop) pv = kp[r] ? pv * a.sc_attn : 0.f;
        st[u][t][r] = pv;
      }
    }
    l[u] += __shfl_xor(l[u], 16, 64);
    l[u] += __shfl_xor(l[u], 32, 64);
  }
  f32x4 o[NU][HD / 16];
#pragma unroll
  for (int u = 0; u < NU; ++u)
#pragma unroll
    for (int d = 0; d < HD / 16; ++d) o[u][d] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s2 = 0; s2 < NPK / 32; ++s2)
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const bf16x8 pb = pack8(st[u][2 * s2], st[u][2 * s2 + 1]);
#pragma unroll
      for (int d = 0; d < HD / 16; ++d) o[u][d] = mfma16(frag_t<AS>(un[u].Vi, 16 * d, s2, lane), pb, o[u][d]);
    }
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int q = un[u].qg * 16 + li;
    if (q < N) {
      const float inv = 1.f / l[u];
      bf16* orow = w.o + ((size_t)b * N + q) * D + un[u].h * HD;
#pragma unroll
      for (int d = 0; d < HD / 16; ++d)
        st8_sc1(orow + 16 * d + 4 * g, __builtin_bit_cast(uint64_t, pack4(o[u][d] * inv)));
      if (g == 0 && w.lse != nullptr) w.lse[((size_t)b * H + un[u].h) * N + q] = (mx[u] + log2f(l[u])) * LN2;
    }
  }
}

// ------------------------------------------------------------------ the kernel
// Per phase the order is: hand-off wait -> every global load of the phase
// (gather, statistics, epilogue operands) -> the NEXT weight panel's LDS-DMA ->
// LDS stores / MFMA -> epilogue -> publish (one vmcnt(0) drain).  Loads return
// in issue order, so nothing the phase needs queues behind a DMA.  Weight
// buffers alternate: per block q -> X, k -> Y, v -> X, proj -> X, fc1 -> Y,
// fc2 -> X, next q -> Y (so X and Y swap every block); the Q/K images of the
// attention live in Y, the V image in the A region.
__global__ __launch_bounds__(256, 1) void vit_group_fwd_kernel(DevArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Aimg = smem;
  char* WX = smem + A_BYTES;
  char* WY = smem + A_BYTES + B_BYTES;
  float2* ms_lds = reinterpret_cast<float2*>(smem + A_BYTES + 2 * B_BYTES);  // [RP] (mean, rstd)
  const int b = a.img0 + blockIdx.x / G, j = blockIdx.x % G;
  const int N = a.N;
  const int row0 = b * N;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, li = lane & 15;
  unsigned* ctr = a.ctr + b * 16;
  const int col0 = 64 * j;
  const int nl = 16 * wave + 4 * g;   // the lane's 4 columns within a 64-wide panel
  const int ncol = col0 + nl;

  issue_weights(WX, a.blk[0].qkv_wf, 3 * D, col0, wave, lane);  // block 0's q panel
  for (int l = 0; l < a.L; ++l) {
    const DevBlock& w = a.blk[l];
    // ============================================================ QKV (fold LN1) + attention
    stamp(a, l, 0);
    wait_count(ctr, 24u * l, a.err);
    stamp(a, l, 1);
    Gather ga;
    ga.load(w.xb_in + (size_t)row0 * D, N);
    RowStats rs;
    rs.load(w.st_in, row0, N);
    f32x4 lnc[3], colb[3];
#pragma unroll
    for (int s3 = 0; s3 < 3; ++s3) {
      lnc[s3] = ld4(w.qkv_c + s3 * D + col0 + nl);
      colb[s3] = ld4(w.qkv_bf + s3 * D + col0 + nl);
    }
    issue_weights(WY, w.qkv_wf, 3 * D, D + col0, wave, lane);  // k panel
    ga.store(Aimg);
    rs.finish(ms_lds, a.eps, row0, N, j == 0 ? w.m1 : nullptr, w.r1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    vm_wait<12>();  // q panel landed (k panel may still fly)
    raw_barrier();
    stamp(a, l, 16);
    const int hh = wave >> 1, d0 = nl & 31;  // the lane's head (of the workgroup's two) and dim
    float2 msr[FM];
#pragma unroll
    for (int i = 0; i < FM; ++i) msr[i] = ms_lds[16 * i + li];
    // fold epilogue of one of q / k / v -> bf16 -> attention image (row r, 4 dims)
    auto emit = [&](const f32x4(&acc)[FM], int s3, char* img) {
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int r = 16 * i + li;
        if (r >= N) continue;
        const f32x4 v = (acc[i] - msr[i].x * lnc[s3]) * msr[i].y + colb[s3];
        *reinterpret_cast<bf16x4*>(img + hh * (s3 == 0 ? QI : KVI) + r * AS + d0 * 2) = pack4(v);
      }
    };
    char* Qimg = WY;             // after the k GEMM
    char* Kimg = WY + 2 * QI;
    char* Vimg = Aimg;           // after the v GEMM
    {
      f32x4 aq[FM], ak[FM];
      mma64t(Aimg, WX, aq, wave, g, li);
      raw_barrier();  // every wave is done with the q panel
      stamp(a, l, 17);
      issue_weights(WX, w.qkv_wf, 3 * D, 2 * D + col0, wave, lane);  // v panel
      vm_wait<12>();
      raw_barrier();
      stamp(a, l, 18);
      mma64t(Aimg, WY, ak, wave, g, li);
      raw_barrier();  // the k panel is free: Q / K images go there
      stamp(a, l, 19);
      emit(aq, 0, Qimg);
      emit(ak, 1, Kimg);
    }
    vm_wait<0>();
    raw_barrier();
    stamp(a, l, 20);
    {
      f32x4 av[FM];
      mma64t(Aimg, WX, av, wave, g, li);
      raw_barrier();  // A region and the v panel free
      stamp(a, l, 21);
      issue_weights(WX, w.proj_w, D, col0, wave, lane);  // proj panel (lands during the attention)
      emit(av, 2, Vimg);
    }
    // zero the padded key rows of K and V (P is 0 there, but 0 * garbage could be NaN)
    for (int c = threadIdx.x; c < 4 * (NPK - N) * (AS / 16); c += 256) {
      const int im = c / ((NPK - N) * (AS / 16)), rem = c - im * ((NPK - N) * (AS / 16));
      const int r = N + rem / (AS / 16), cc = rem % (AS / 16);
      char* base = im < 2 ? Kimg + im * KVI : Vimg + (im - 2) * KVI;
      *reinterpret_cast<u32x4*>(base + r * AS + cc * 16) = u32x4{0u, 0u, 0u, 0u};
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();
    stamp(a, l, 2);
    if (w.qkv != nullptr) {  // saved for the backward: [3][B][H][N][hd], 16-B rows pieces from the images
      for (int c = threadIdx.x; c < 3 * 2 * N * (HD / 8); c += 256) {
        const int r4 = c % (N * (HD / 8)), sh = c / (N * (HD / 8));
        const int s3 = sh >> 1, h2 = sh & 1, r = r4 >> 2, cc = r4 & 3;
        const char* src = (s3 == 0 ? Qimg + h2 * QI : (s3 == 1 ? Kimg : Vimg) + h2 * KVI) + r * AS + cc * 16;
        *reinterpret_cast<u32x4*>(w.qkv + (((size_t)s3 * a.B + b) * H + 2 * j + h2) * N * HD + (size_t)r * HD +
                                  cc * 8) = *reinterpret_cast<const u32x4*>(src);
      }
    }
    {
      // 2 heads x 5 query groups = 10 units: waves take (w, w + 4) interleaved, then w + 8
      auto unit = [&](int u) {
        const int h2 = u / FM, qg = u - h2 * FM;
        return AttnUnit{Qimg + h2 * QI, Kimg + h2 * KVI, Vimg + h2 * KVI, 2 * j + h2, qg};
      };
      auto valid = [&](int u) { return u < 2 * FM && 16 * (u % FM) < N; };
      if (valid(wave) && valid(wave + 4)) {
        const AttnUnit p2[2] = {unit(wave), unit(wave + 4)};
        attention_units<2>(a, w, p2, b, N, lane);
      } else {
        for (int u = wave; u < wave + 8; u += 4)
          if (valid(u)) {
            const AttnUnit p1[1] = {unit(u)};
            attention_units<1>(a, w, p1, b, N, lane);
          }
      }
      if (valid(wave + 8)) {
        const AttnUnit p1[1] = {unit(wave + 8)};
        attention_units<1>(a, w, p1, b, N, lane);
      }
    }
    publish(ctr);
    stamp(a, l, 3);
    // ============================================================ proj + residual (LN2 statistics)
    stamp(a, l, 4);
    {
      ResidEpi e{w.x_in, w.proj_b, w.x1, w.x1b, w.st1, w.site_p, w.site_d1, w.thr_dp, w.sc_dp};
      e.prefetch(row0, N, ncol, li);  // own columns: no hand-off needed
      wait_count(ctr, 24u * l + 6u, a.err);
      stamp(a, l, 5);
      ga.load(w.o + (size_t)row0 * D, N);
      issue_weights(WY, w.fc1_wf, D, col0, wave, lane);  // fc1 panel
      ga.store(Aimg);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      vm_wait<12>();  // proj panel landed
      raw_barrier();
      f32x4 acc[FM];
      mma64t(Aimg, WX, acc, wave, g, li);
      raw_barrier();  // the A region is free for the slot exchange
      stamp(a, l, 6);
      e.finish(a, acc, row0, N, col0, wave, g, li, Aimg);
    }
    publish(ctr);
    stamp(a, l, 7);
    // ============================================================ fc1 (fold LN2) + GELU
    stamp(a, l, 8);
    wait_count(ctr, 24u * l + 12u, a.err);
    stamp(a, l, 9);
    {
      ga.load(w.x1b + (size_t)row0 * D, N);
      rs.load(w.st1, row0, N);
      const f32x4 c1 = ld4(w.fc1_c + ncol), b1 = ld4(w.fc1_bf + ncol);
      issue_weights(WX, w.fc2_w, D, col0, wave, lane);  // fc2 panel
      ga.store(Aimg);
      rs.finish(ms_lds, a.eps, row0, N, j == 0 ? w.m2 : nullptr, w.r2);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      vm_wait<12>();  // fc1 panel landed
      raw_barrier();
      f32x4 acc[FM];
      mma64t(Aimg, WY, acc, wave, g, li);
      stamp(a, l, 10);
      // VecEpi<EPI_GELU> math: u = fold(acc) (bf16, saved), h = Dropout(GELU(u)) (bf16, published)
      const uint32_t salt = a.thr_drop ? site_salt(a.rng, w.site_f1) : 0u;
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int r = 16 * i + li;
        if (r >= N) continue;
        const float2 m2 = ms_lds[r];
        const long long idx = (long long)(row0 + r) * D + ncol;
        const f32x4 v = (acc[i] - m2.x * c1) * m2.y + b1;
        st4bf(w.u + idx, v);
        bool kp[4] = {true, true, true, true};
        if (a.thr_drop) dropout_keep4(salt, (uint32_t)idx, a.thr_drop, kp);
        f32x4 hv;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          float e = gelu_f(v[c]);
          if (a.thr_drop) e = kp[c] ? e * a.sc_drop : 0.f;
          hv[c] = e;
        }
        st4bf_pub<true>(w.h + idx, hv);
      }
    }
    publish(ctr);
    stamp(a, l, 11);
    // ============================================================ fc2 + residual (next LN1 / final LN statistics)
    stamp(a, l, 12);
    {
      ResidEpi e{w.x1, w.fc2_b, w.x_out, w.xb_out, w.st_out, w.site_f2, w.site_d2, w.thr_dp, w.sc_dp};
      e.prefetch(row0, N, ncol, li);
      wait_count(ctr, 24u * l + 18u, a.err);
      stamp(a, l, 13);
      ga.load(w.h + (size_t)row0 * D, N);
      if (l + 1 < a.L) issue_weights(WY, a.blk[l + 1].qkv_wf, 3 * D, col0, wave, lane);  // next q panel
      ga.store(Aimg);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (l + 1 < a.L) vm_wait<12>();
      else vm_wait<0>();
      raw_barrier();
      f32x4 acc[FM];
      mma64t(Aimg, WX, acc, wave, g, li);
      raw_barrier();
      stamp(a, l, 14);
      e.finish(a, acc, row0, N, col0, wave, g, li, Aimg);
    }
    publish(ctr);
    stamp(a, l, 15);
    char* t = WX;  // the next block's q panel is in Y
    WX = WY;
    WY = t;
  }
}

}  // namespace vg
}  // namespace dc

using namespace dc;

bool vit_group_supported(int D, int H, int hd, int N, int L) {
  return D == vg::D && H == vg::H && hd == vg::HD && N >= 2 && N <= vg::RP && L >= 1 && L <= VG_MAXL;
}

void vit_group_fwd_launch(const VgArgs& a, hipStream_t stream) {
  if (!vit_group_supported(a.D, a.H, a.hd, a.N, a.L)) throw std::runtime_error("vit_group_fwd: unsupported shape");
  vg::DevArgs d{};
  for (int l = 0; l < a.L; ++l) {
    const VgBlock& s = a.blk[l];
    vg::DevBlock& t = d.blk[l];
    t.qkv_wf = (const bf16*)s.qkv_wf; t.proj_w = (const bf16*)s.proj_w;
    t.fc1_wf = (const bf16*)s.fc1_wf; t.fc2_w = (const bf16*)s.fc2_w;
    t.qkv_bf = s.qkv_bf; t.qkv_c = s.qkv_c; t.proj_b = s.proj_b; t.fc1_bf = s.fc1_bf; t.fc1_c = s.fc1_c;
    t.fc2_b = s.fc2_b;
    t.xb_in = (const bf16*)s.xb_in; t.st_in = s.st_in; t.x_in = s.x_in;
    t.qkv = (bf16*)s.qkv; t.o = (bf16*)s.o; t.x1b = (bf16*)s.x1b; t.u = (bf16*)s.u; t.h = (bf16*)s.h;
    t.xb_out = (bf16*)s.xb_out;
    t.lse = s.lse; t.x1 = s.x1; t.st1 = s.st1; t.x_out = s.x_out; t.st_out = s.st_out;
    t.m1 = s.m1; t.r1 = s.r1; t.m2 = s.m2; t.r2 = s.r2;
    t.site_a = s.site_a; t.site_p = s.site_p; t.site_d1 = s.site_d1; t.site_f1 = s.site_f1;
    t.site_f2 = s.site_f2; t.site_d2 = s.site_d2;
    t.thr_dp = drop_threshold_host(s.p_dp);
    t.sc_dp = s.p_dp > 0 ? 1.f / (1.f - (float)s.p_dp) : 1.f;
  }
  d.L = a.L; d.B = a.B; d.N = a.N;
  d.rng = a.rng;
  d.thr_drop = drop_threshold_host(a.p_drop);
  d.sc_drop = a.p_drop > 0 ? 1.f / (1.f - (float)a.p_drop) : 1.f;
  d.thr_attn = drop_threshold_host(a.p_attn);
  d.sc_attn = a.p_attn > 0 ? 1.f / (1.f - (float)a.p_attn) : 1.f;
  d.scale = a.scale; d.eps = a.eps;
  d.ctr = a.ctr; d.err = a.err; d.stamps = (unsigned long long*)a.stamps;
  static const bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&vg::vit_group_fwd_kernel),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, vg::LDS_BYTES) == hipSuccess;
  if (!attr) throw std::runtime_error("vit_group_fwd: cannot raise the LDS limit");
  // every workgroup of a launch must be resident (groups spin on each other):
  // one 156 KiB workgroup per CU -> at most CUs / G images per launch
  static const int cus = [] {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return n > 0 ? n : 256;
  }();
  const int per = std::max(1, cus / vg::G);
  if (hipMemsetAsync(a.ctr, 0, (size_t)a.B * 16 * sizeof(unsigned), stream) != hipSuccess)
    throw std::runtime_error("vit_group_fwd: counter reset failed");
  for (int i0 = 0; i0 < a.B; i0 += per) {
    d.img0 = i0;
    const int n = std::min(per, a.B - i0);
    hipLaunchKernelGGL(vg::vit_group_fwd_kernel, dim3(n * vg::G), dim3(256), vg::LDS_BYTES, stream, d);
  }
}
