// Fused multi-head self-attention for gfx950 (ViT.py:105-117 semantics:
// softmax(Q K^T * hd^-0.5) -> Dropout -> @V), forward + backward, any N, hd in {32, 64}.
//
// Forward (flash-style, online softmax, never materialises N x N):
//   workgroup = 4 waves = 64 query rows of one (b, h); each wave owns 16 queries.
//   K/V tiles of 64 keys staged in LDS with a 32-B row pad (conflict-free for
//   ds_read_b128 row reads AND ds_read_b64_tr_b16 transposed reads).
//   Scores are computed SWAPPED, S^T = K Q^T, so each lane holds 16 keys of ONE
//   query: the row max / row sum need only 2 cross-lane shuffles, and the
//   probability tile P^T is already the B operand of O^T += V^T P^T
//   (bf16-packed registers, no LDS round trip).  V^T fragments come from the V
//   tile through the hardware transposing LDS read.  Dropout on P uses the
//   counter hash (regenerated in backward).  Saves LSE per query.
//
// Backward (no atomics, deterministic, recompute P from LSE):
//   kernel 1 (per 64-query block): delta = rowsum(dO*O) (stored), dQ.
//       S^T = K Q^T, dP^T = V dO^T, dS^T = P^T (M*dP^T - delta), dQ^T += K^T dS^T.
//   kernel 2 (per 64-key block, each wave 16 keys held as register fragments):
//       S = Q K^T, dP = dO V^T, dV^T += dO^T (P*M), dK^T += Q^T dS.
//   dQ/dK/dV are written token-major into dqkv [B*N, 3D] (the layout of the
//   qkv Linear's output columns) so the qkv dgrad/wgrad GEMMs consume it directly.
#include "common.h"
#include "kernels.h"
#include "gemm_common.h"  // xcd_remap
#include <cstdlib>
#include <type_traits>

namespace dc {

constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

template <int HD>
struct AC {
  static constexpr int S = 2 * HD + 32;   // LDS row stride in bytes
  static constexpr int TILE = 64 * S;     // one 64-row tile
  static constexpr int KS = HD / 32;      // MFMA k-steps over hd
  static constexpr int DT = HD / 16;      // 16-row tiles over hd
  static constexpr int CPR = HD / 8;      // 16-B chunks per row
};

// Block coordinates of the long-sequence kernels (grid = query / key tiles x B*H):
// consecutive linear block ids are dispatched round-robin over the 8 XCDs, so the
// gridDim.x workgroups of one (b, h) -- which all read the same Q / dO or K / V rows --
// landed on 8 different L2s (each fetching them: dK/dV and dQ pulled 141 / 146 MB past
// L2 for ~80 MB of operands, profiles/pmc_hires_r5.md).  xcd_remap gives each XCD a
// contiguous range of (b, h)s instead.  DC_ATTN_XCD=0 restores the plain mapping (A/B).
#ifndef DC_ATTN_XCD
#define DC_ATTN_XCD 1
#endif
struct Blk {
  int x, y;
};
__device__ __forceinline__ Blk attn_block() {
#if DC_ATTN_XCD
  const int l = xcd_remap(blockIdx.x + gridDim.x * blockIdx.y, gridDim.x * gridDim.y);
  return {l % (int)gridDim.x, l / (int)gridDim.x};
#else
  return {(int)blockIdx.x, (int)blockIdx.y};
#endif
}

// stage rows r0..r0+63 of a [N][HD] bf16 matrix into a padded LDS image
template <int HD>
__device__ __forceinline__ void stage64(char* lds, const bf16* __restrict__ base, int r0, int N) {
  for (int c = threadIdx.x; c < 64 * AC<HD>::CPR; c += 256) {
    const int r = c / AC<HD>::CPR, cc = c % AC<HD>::CPR;
    u32x4 v = {0u, 0u, 0u, 0u};
    if (r0 + r < N) v = *reinterpret_cast<const u32x4*>(base + (size_t)(r0 + r) * HD + cc * 8);
    *reinterpret_cast<u32x4*>(lds + r * AC<HD>::S + cc * 16) = v;
  }
}

// standard-order fragment (row r, k-step s) from a padded row image
template <int HD>
__device__ __forceinline__ bf16x8 frag_row(const char* lds, int r, int s, int g) {
  return *reinterpret_cast<const bf16x8*>(lds + r * AC<HD>::S + (32 * s + 8 * g) * 2);
}

// standard-order fragment straight from global memory (row < N else zero)
template <int HD>
__device__ __forceinline__ bf16x8 frag_glb(const bf16* __restrict__ base, int row, int N, int s, int g) {
  if (row < N) return *reinterpret_cast<const bf16x8*>(base + (size_t)row * HD + 32 * s + 8 * g);
  bf16x8 z;
#pragma unroll
  for (int j = 0; j < 8; ++j) z[j] = f2bf(0.f);
  return z;
}

__device__ __forceinline__ bf16x8 pack8(const f32x4& a, const f32x4& b) {
  bf16x8 v;
  v[0] = f2bf(a[0]); v[1] = f2bf(a[1]); v[2] = f2bf(a[2]); v[3] = f2bf(a[3]);
  v[4] = f2bf(b[0]); v[5] = f2bf(b[1]); v[6] = f2bf(b[2]); v[7] = f2bf(b[3]);
  return v;
}

// ============================================================================ forward
template <int HD>
__global__ __launch_bounds__(256) void attn_fwd_kernel(const bf16* __restrict__ qkv, bf16* __restrict__ out,
                                                       float* __restrict__ lse, int B, int H, int N, float scale,
                                                       const int64_t* __restrict__ rng, int site, uint32_t thr,
                                                       float dsc) {
  using C = AC<HD>;
  __shared__ __attribute__((aligned(16))) char lds[2 * C::TILE];
  char* Kl = lds;
  char* Vl = lds + C::TILE;
  const int bh = blockIdx.y, b = bh / H, h = bh - b * H;
  const size_t mat = (size_t)N * HD;
  const bf16* qb = qkv + (size_t)bh * mat;
  const bf16* kb = qkv + ((size_t)B * H + bh) * mat;
  const bf16* vb = qkv + ((size_t)2 * B * H + bh) * mat;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, li = lane & 15;
  const int q = blockIdx.x * 64 + wave * 16 + li;  // this lane's query (column of S^T)
  const float sl2 = scale * LOG2E;
  const uint32_t salt = thr ? site_salt(rng, site) : 0u;

  bf16x8 qf[C::KS];
#pragma unroll
  for (int s = 0; s < C::KS; ++s) qf[s] = frag_glb<HD>(qb, q, N, s, g);

  f32x4 o[C::DT];
#pragma unroll
  for (int d = 0; d < C::DT; ++d) o[d] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_run = 0.f;

  for (int kv0 = 0; kv0 < N; kv0 += 64) {
    __syncthreads();
    stage64<HD>(Kl, kb, kv0, N);
    stage64<HD>(Vl, vb, kv0, N);
    __syncthreads();
    f32x4 st[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      st[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < C::KS; ++s) st[t] = mfma16(frag_row<HD>(Kl, 16 * t + li, s, g), qf[s], st[t]);
    }
    float mt = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = kv0 + 16 * t + 4 * g + r;
        const float v = key < N ? st[t][r] * sl2 : -INFINITY;
        st[t][r] = v;
        mt = fmaxf(mt, v);
      }
    mt = fmaxf(mt, __shfl_xor(mt, 16, 64));
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
    const float m_new = fmaxf(m_run, mt);
    const float alpha = fexp2(m_run - m_new);
    float ls = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float pv = fexp2(st[t][r] - m_new);
        ls += pv;
        if (thr) {
          const int key = kv0 + 16 * t + 4 * g + r;
          const uint32_t idx = (uint32_t)(((size_t)bh * N + q) * attn_mask_ld(N) + key);
          pv = dropout_keep(salt, idx, thr) ? pv * dsc : 0.f;
        }
        st[t][r] = pv;
      }
    ls += __shfl_xor(ls, 16, 64);
    ls += __shfl_xor(ls, 32, 64);
    l_run = l_run * alpha + ls;
    m_run = m_new;
#pragma unroll
    for (int d = 0; d < C::DT; ++d) o[d] *= alpha;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const bf16x8 pb = pack8(st[2 * s2], st[2 * s2 + 1]);
#pragma unroll
      for (int d = 0; d < C::DT; ++d) o[d] = mfma16(frag_t<C::S>(Vl, 16 * d, s2, lane), pb, o[d]);
    }
  }
  if (q < N) {
    const float inv = 1.f / l_run;
    const int D = H * HD;
    bf16* orow = out + ((size_t)b * N + q) * D + h * HD;
#pragma unroll
    for (int d = 0; d < C::DT; ++d) {
      bf16x4 v;
      v[0] = f2bf(o[d][0] * inv); v[1] = f2bf(o[d][1] * inv);
      v[2] = f2bf(o[d][2] * inv); v[3] = f2bf(o[d][3] * inv);
      *reinterpret_cast<bf16x4*>(orow + 16 * d + 4 * g) = v;
    }
    if (g == 0) lse[(size_t)bh * N + q] = (m_run + log2f(l_run)) * LN2;
  }
}

// ============================================================================ forward, long sequences
// Flash forward v2 (N > 128): 128 queries per workgroup (4 waves x 32 queries =
// two 16-query MFMA column tiles per wave, so every K / V fragment read from
// LDS feeds two MFMAs), KV tiles of 64 keys DOUBLE-BUFFERED: the next tile's
// global loads are issued before the current tile's MFMAs and land in
// registers, then go to the other LDS buffer — one barrier per tile and no
// exposed load latency.  Dropout is a template flag (branch-free softmax).
// The padded-row zeroing happens in store(), not load(): a select on the loaded
// registers right after the loads made the compiler wait for them there (s_waitcnt
// vmcnt(0) before the tile's MFMAs), i.e. the "prefetch" was a blocking load.
template <int HD>
struct KvStage {  // one 64-row K tile + one 64-row V tile, register-staged
  static constexpr int CPR = HD / 8;
  static constexpr int PER = 64 * CPR / 256;  // 16-B chunks per thread per matrix
  u32x4 k[PER], v[PER];
  bool ok[PER];
  __device__ __forceinline__ void load(const bf16* __restrict__ kb, const bf16* __restrict__ vb, int r0, int N) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = threadIdx.x + i * 256;
      const int r = c / CPR, cc = c - r * CPR;
      const int rr = r0 + r < N ? r0 + r : N - 1;
      ok[i] = r0 + r < N;
      k[i] = *reinterpret_cast<const u32x4*>(kb + (size_t)rr * HD + cc * 8);
      v[i] = *reinterpret_cast<const u32x4*>(vb + (size_t)rr * HD + cc * 8);
    }
  }
  __device__ __forceinline__ void store(char* kl, char* vl) const {
    const u32x4 z = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = threadIdx.x + i * 256;
      const int r = c / CPR, cc = c - r * CPR;
      *reinterpret_cast<u32x4*>(kl + r * AC<HD>::S + cc * 16) = ok[i] ? k[i] : z;
      *reinterpret_cast<u32x4*>(vl + r * AC<HD>::S + cc * 16) = ok[i] ? v[i] : z;
    }
  }
};

// One online-softmax update of a 16-query column tile of S^T (lane li = query,
// 16 of the tile's 64 keys per lane in st, RAW scores): turns st into the
// probabilities of the P.V MFMAs (dropout applied) and updates the running
// max / sum and the output accumulators.
//   * scale folded into one FMA per score: p = exp2(s * sl2 - m), m in scaled
//     log2 units (the max is taken on raw scores; sl2 > 0)
//   * key masking only in the tail tile (MASK; full tiles carry none)
//   * lazy rescale: the reference max m moves only when a tile's max exceeds it
//     by more than 8 (log2 units), so p <= 2^8 (exact in fp32, same relative
//     bf16 precision as p <= 1); numerator and denominator use the same m, so
//     the result is the softmax.  After the first tile the (wave-uniform) branch
//     that rescales o is almost never taken: the o *= alpha pass (an AGPR read +
//     mul + write per accumulator element) and the alpha exp leave the loop.
//   * dropout: st keeps the UNdropped probabilities (the row sum l is taken before
//     dropout); dm[t][j] is the packed drop mask (drop_mask2) of the keys 16t+4g+2j,
//     +1, AND-NOT-ed onto the packed bf16 pair by pack8_drop -- no per-element
//     compare / select -- and dbits the tile's 16 drop flags of this lane (bit
//     drop_bit(t, r), keep_store)
template <int DT, bool DROP, bool MASK>
__device__ __forceinline__ void flash_softmax_tile(f32x4 (&st)[4], f32x4 (&o)[DT], float& m_run, float& l_run,
                                                   int kv0, int N, int g, float sl2, uint32_t salt,
                                                   uint32_t rowidx, uint32_t thr2, uint32_t (&dm)[4][2],
                                                   uint32_t& dbits) {
  float mt = -INFINITY;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (MASK && kv0 + 16 * t + 4 * g + r >= N) st[t][r] = -INFINITY;
      mt = fmaxf(mt, st[t][r]);
    }
  mt = fmaxf(mt, __shfl_xor(mt, 16, 64));
  mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
  const float ms = mt * sl2;
  const bool up = ms > m_run + 8.f;  // m_run = -inf on the first tile: always
  if (__any(up)) {
    const float alpha = up ? fexp2(m_run - ms) : 1.f;
    l_run *= alpha;
#pragma unroll
    for (int d = 0; d < DT; ++d) o[d] *= alpha;
    m_run = up ? ms : m_run;
  }
  const float nm = -m_run;
  float ls = 0.f;
  const uint32_t pgs = DROP ? ((rowidx >> 1) + 2u * (uint32_t)g) * DROP_GOLDEN + salt : 0u;  // rowidx even
  uint32_t db = 0u;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    if (DROP) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        dm[t][j] = drop_mask2(drop_mix(pgs + (uint32_t)(8 * t + j) * DROP_GOLDEN), thr2);
        db |= dm[t][j] & ((1u << (2 * t + j)) | (1u << (16 + 2 * t + j)));
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float pv = fexp2(fmaf(st[t][r], sl2, nm));  // the keep scale 1/(1-p) goes into the final 1/l
      ls += pv;
      st[t][r] = pv;
    }
  }
  if (DROP) dbits = (db & 0xFFu) | ((db >> 8) & 0xFF00u);
  ls += __shfl_xor(ls, 16, 64);
  ls += __shfl_xor(ls, 32, 64);
  l_run += ls;
}

// pack8 with the drop masks of flash_softmax_tile applied to the bf16 pairs (keys
// 16ta+4g+{0,1}, {2,3}, then 16tb+4g+...)
__device__ __forceinline__ bf16x8 pack8_drop(const f32x4& a, const f32x4& b, const uint32_t (&ma)[2],
                                             const uint32_t (&mb)[2]) {
  u32x4 w = __builtin_bit_cast(u32x4, pack8(a, b));
  w[0] &= ~ma[0];
  w[1] &= ~ma[1];
  w[2] &= ~mb[0];
  w[3] &= ~mb[1];
  return __builtin_bit_cast(bf16x8, w);
}

// Stored attention-dropout masks of the long-sequence kernels: one 64-bit word per
// (b, h, 64-key tile, query) = four 16-bit groups in the forward's lane layout: group g
// (bits 16 g .. 16 g + 15 of the word, i.e. uint16 [((bh * ntiles + tile) * N + q) * 4 + g])
// holds the DROP flags of keys 16 t + 4 g + r at bit drop_bit(t, r) -- each forward lane
// stores its own 16 flags (no cross-lane assembly; the 64 lanes of a wave-instruction
// write 128 contiguous bytes), the two backward kernels read them instead of re-hashing
// every mask element (dQ: the forward's lane layout; dK/dV: the query tile's words staged
// in LDS, one bit per lane's key at position keep_bitpos(key)).  The order within a group
// is the forward's mask order: the low halves of its 8 pair hashes (r even) in bits 0-7,
// the high halves (r odd) in bits 8-15.
__device__ __forceinline__ constexpr int drop_bit(int t, int r) { return 8 * (r & 1) + 2 * t + (r >> 1); }
__device__ __forceinline__ void keep_store(uint32_t* __restrict__ keep, size_t word, uint32_t dbits, int g,
                                           bool valid) {
  if (valid) reinterpret_cast<uint16_t*>(keep)[word * 4 + g] = (uint16_t)dbits;
}
// bit position of key k (0..63 within its tile) in the tile word (a DROP flag)
__device__ __forceinline__ int keep_bitpos(int k) { return 16 * ((k >> 2) & 3) + drop_bit(k >> 4, k & 3); }
// Short-sequence kernels: one 32-bit word per lane (query, lane group g) with the DROP flag
// of key 16 t + 4 g + r at bit short_drop_bit(t, r) (t < 8): the low / high halves of the
// pair masks of drop_mask2 land in bits 2t + j / 16 + 2t + j, one AND-OR per pair
__device__ __forceinline__ constexpr int short_drop_bit(int t, int r) { return 16 * (r & 1) + 2 * t + (r >> 1); }

template <int HD, bool DROP>
__global__ __launch_bounds__(256) void attn_fwd_flash2_kernel(const bf16* __restrict__ qkv, bf16* __restrict__ out,
                                                              float* __restrict__ lse, int B, int H, int N,
                                                              float scale, const int64_t* __restrict__ rng, int site,
                                                              uint32_t thr, float dsc, uint32_t* __restrict__ keep) {
  using C = AC<HD>;
  __shared__ __attribute__((aligned(16))) char lds[4 * C::TILE];  // [buf][K | V]
  const Blk blk = attn_block();
  const int bh = blk.y, b = bh / H, h = bh - b * H;
  const size_t mat = (size_t)N * HD;
  const bf16* qb = qkv + (size_t)bh * mat;
  const bf16* kb = qkv + ((size_t)B * H + bh) * mat;
  const bf16* vb = qkv + ((size_t)2 * B * H + bh) * mat;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, li = lane & 15;
  const int qbase = blk.x * 128 + wave * 32;
  const float sl2 = scale * LOG2E;
  const uint32_t salt = DROP ? site_salt(rng, site) : 0u;
  const uint32_t thr2 = (thr >> 1) * 0x10001u;  // thr / 2 in both 16-bit halves (drop_mask2)

  KvStage<HD> stg;
  stg.load(kb, vb, 0, N);
  bf16x8 qf[2][C::KS];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int s = 0; s < C::KS; ++s) qf[u][s] = frag_glb<HD>(qb, qbase + 16 * u + li, N, s, g);
  stg.store(lds, lds + C::TILE);
  __syncthreads();

  f32x4 o[2][C::DT];
  float m_run[2], l_run[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    m_run[u] = -INFINITY;
    l_run[u] = 0.f;
#pragma unroll
    for (int d = 0; d < C::DT; ++d) o[u][d] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const int ntiles = (N + 63) / 64;
  const uint32_t rowidx0 = (uint32_t)(((size_t)bh * N + qbase + li) * attn_mask_ld(N));
  const uint32_t rowstep = (uint32_t)(16 * attn_mask_ld(N));  // second query tile u = 1
  auto tile = [&](int it, auto mask_tag) {
    constexpr bool MASK = decltype(mask_tag)::value;
    const int kv0 = it * 64;
    const bool more = it + 1 < ntiles;
    if (more) stg.load(kb, vb, kv0 + 64, N);  // lands during this tile's MFMAs
    const char* Kl = lds + (it & 1) * 2 * C::TILE;
    const char* Vl = Kl + C::TILE;
    f32x4 st[2][4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      st[0][t] = f32x4{0.f, 0.f, 0.f, 0.f};
      st[1][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < C::KS; ++s) {
        const bf16x8 kf = frag_row<HD>(Kl, 16 * t + li, s, g);
        st[0][t] = mfma16(kf, qf[0][s], st[0][t]);
        st[1][t] = mfma16(kf, qf[1][s], st[1][t]);
      }
    }
    uint32_t dm[2][4][2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      uint32_t dbits = 0u;
      flash_softmax_tile<C::DT, DROP, MASK>(st[u], o[u], m_run[u], l_run[u], kv0, N, g, sl2, salt,
                                            rowidx0 + u * rowstep + kv0, thr2, dm[u], dbits);
      if (DROP && keep != nullptr) {
        const int q = qbase + 16 * u + li;
        keep_store(keep, ((size_t)bh * ntiles + it) * N + q, dbits, g, q < N);
      }
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const bf16x8 pb0 = DROP ? pack8_drop(st[0][2 * s2], st[0][2 * s2 + 1], dm[0][2 * s2], dm[0][2 * s2 + 1])
                              : pack8(st[0][2 * s2], st[0][2 * s2 + 1]);
      const bf16x8 pb1 = DROP ? pack8_drop(st[1][2 * s2], st[1][2 * s2 + 1], dm[1][2 * s2], dm[1][2 * s2 + 1])
                              : pack8(st[1][2 * s2], st[1][2 * s2 + 1]);
#pragma unroll
      for (int d = 0; d < C::DT; ++d) {
        const bf16x8 vf = frag_t<C::S>(Vl, 16 * d, s2, lane);
        o[0][d] = mfma16(vf, pb0, o[0][d]);
        o[1][d] = mfma16(vf, pb1, o[1][d]);
      }
    }
    if (more) stg.store(lds + ((it + 1) & 1) * 2 * C::TILE, lds + ((it + 1) & 1) * 2 * C::TILE + C::TILE);
    __syncthreads();
  };
  const int nfull = N / 64;  // tiles with every key valid
  for (int it = 0; it < nfull; ++it) tile(it, std::false_type{});
  if (nfull < ntiles) tile(nfull, std::true_type{});
  const int D = H * HD;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int q = qbase + 16 * u + li;
    if (q < N) {
      const float inv = (DROP ? dsc : 1.f) / l_run[u];  // dropout keep scale folded in
      bf16* orow = out + ((size_t)b * N + q) * D + h * HD;
#pragma unroll
      for (int d = 0; d < C::DT; ++d) {
        bf16x4 v;
        v[0] = f2bf(o[u][d][0] * inv); v[1] = f2bf(o[u][d][1] * inv);
        v[2] = f2bf(o[u][d][2] * inv); v[3] = f2bf(o[u][d][3] * inv);
        *reinterpret_cast<bf16x4*>(orow + 16 * d + 4 * g) = v;
      }
      if (g == 0) lse[(size_t)bh * N + q] = (m_run[u] + log2f(l_run[u])) * LN2;
    }
  }
}
template __global__ void attn_fwd_flash2_kernel<32, true>(const bf16*, bf16*, float*, int, int, int, float,
                                                          const int64_t*, int, uint32_t, float, uint32_t*);
template __global__ void attn_fwd_flash2_kernel<32, false>(const bf16*, bf16*, float*, int, int, int, float,
                                                           const int64_t*, int, uint32_t, float, uint32_t*);
template __global__ void attn_fwd_flash2_kernel<64, true>(const bf16*, bf16*, float*, int, int, int, float,
                                                          const int64_t*, int, uint32_t, float, uint32_t*);
template __global__ void attn_fwd_flash2_kernel<64, false>(const bf16*, bf16*, float*, int, int, int, float,
                                                           const int64_t*, int, uint32_t, float, uint32_t*);

// ============================================================================ forward, medium sequences
// Resident-KV forward (128 < N <= 320, e.g. the 257-token OxfordFlower config):
// one workgroup per (b, h) stages the head's WHOLE K and V once (dynamic LDS,
// padded rows), then each of ceil(N/32) waves runs an online softmax over
// 64-key chunks for its 32 queries with no barrier in the loop.  B*H
// workgroups (one round on 256 CUs for B*H <= 256) instead of ceil(N/64)*B*H
// tiles that re-stage K/V per 64 keys.
template <int HD, bool DROP>
__global__ __launch_bounds__(640) void attn_fwd_resident_kernel(const bf16* __restrict__ qkv, bf16* __restrict__ out,
                                                                float* __restrict__ lse, int B, int H, int N,
                                                                float scale, const int64_t* __restrict__ rng,
                                                                int site, uint32_t thr, float dsc,
                                                                uint32_t* __restrict__ keep) {
  using C = AC<HD>;
  extern __shared__ __attribute__((aligned(16))) char dyn[];
  const int NP = (N + 63) / 64 * 64;  // keys padded to whole 64-key chunks
  char* Kl = dyn;
  char* Vl = dyn + NP * C::S;
  const int bh = blockIdx.x, b = bh / H, h = bh - b * H;
  const size_t mat = (size_t)N * HD;
  const bf16* qb = qkv + (size_t)bh * mat;
  const bf16* kb = qkv + ((size_t)B * H + bh) * mat;
  const bf16* vb = qkv + ((size_t)2 * B * H + bh) * mat;
  const int nt = blockDim.x;
  // stage K and V: 8 chunks of 16 B in flight per thread per batch
  const int total = NP * C::CPR;
  for (int c0 = threadIdx.x; c0 < total; c0 += 8 * nt) {
    u32x4 kv[8], vv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int c = c0 + u * nt;
      const int r = c / C::CPR, cc = c - r * C::CPR;
      const int rr = r < N ? r : N - 1;
      const u32x4 z = {0u, 0u, 0u, 0u};
      const bool ok = c < total && r < N;
      kv[u] = ok ? *reinterpret_cast<const u32x4*>(kb + (size_t)rr * HD + cc * 8) : z;
      vv[u] = ok ? *reinterpret_cast<const u32x4*>(vb + (size_t)rr * HD + cc * 8) : z;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int c = c0 + u * nt;
      if (c < total) {
        const int r = c / C::CPR, cc = c - r * C::CPR;
        *reinterpret_cast<u32x4*>(Kl + r * C::S + cc * 16) = kv[u];
        *reinterpret_cast<u32x4*>(Vl + r * C::S + cc * 16) = vv[u];
      }
    }
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, li = lane & 15;
  const int qbase = wave * 32;
  bf16x8 qf[2][C::KS];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int s = 0; s < C::KS; ++s) qf[u][s] = frag_glb<HD>(qb, qbase + 16 * u + li, N, s, g);
  const uint32_t salt = DROP ? site_salt(rng, site) : 0u;
  const uint32_t thr2 = (thr >> 1) * 0x10001u;  // thr / 2 in both 16-bit halves (drop_mask2)
  const float sl2 = scale * LOG2E;
  __syncthreads();

  f32x4 o[2][C::DT];
  float m_run[2], l_run[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    m_run[u] = -INFINITY;
    l_run[u] = 0.f;
#pragma unroll
    for (int d = 0; d < C::DT; ++d) o[u][d] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const uint32_t rowidx0 = (uint32_t)(((size_t)bh * N + qbase + li) * attn_mask_ld(N));
  const uint32_t rowstep = (uint32_t)(16 * attn_mask_ld(N));
  const int ntiles = (N + 63) / 64;
  auto chunk = [&](int kv0, auto mask_tag) {
    constexpr bool MASK = decltype(mask_tag)::value;
    const char* Kc = Kl + kv0 * C::S;
    const char* Vc = Vl + kv0 * C::S;
    f32x4 st[2][4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      st[0][t] = f32x4{0.f, 0.f, 0.f, 0.f};
      st[1][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < C::KS; ++s) {
        const bf16x8 kf = frag_row<HD>(Kc, 16 * t + li, s, g);
        st[0][t] = mfma16(kf, qf[0][s], st[0][t]);
        st[1][t] = mfma16(kf, qf[1][s], st[1][t]);
      }
    }
    uint32_t dm[2][4][2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      uint32_t dbits = 0u;
      flash_softmax_tile<C::DT, DROP, MASK>(st[u], o[u], m_run[u], l_run[u], kv0, N, g, sl2, salt,
                                            rowidx0 + u * rowstep + kv0, thr2, dm[u], dbits);
      if (DROP && keep != nullptr) {
        const int q = qbase + 16 * u + li;
        keep_store(keep, ((size_t)bh * ntiles + kv0 / 64) * N + q, dbits, g, q < N);
      }
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const bf16x8 pb0 = DROP ? pack8_drop(st[0][2 * s2], st[0][2 * s2 + 1], dm[0][2 * s2], dm[0][2 * s2 + 1])
                              : pack8(st[0][2 * s2], st[0][2 * s2 + 1]);
      const bf16x8 pb1 = DROP ? pack8_drop(st[1][2 * s2], st[1][2 * s2 + 1], dm[1][2 * s2], dm[1][2 * s2 + 1])
                              : pack8(st[1][2 * s2], st[1][2 * s2 + 1]);
#pragma unroll
      for (int d = 0; d < C::DT; ++d) {
        const bf16x8 vf = frag_t<C::S>(Vc, 16 * d, s2, lane);
        o[0][d] = mfma16(vf, pb0, o[0][d]);
        o[1][d] = mfma16(vf, pb1, o[1][d]);
      }
    }
  };
  const int nfull = N / 64 * 64;
  for (int kv0 = 0; kv0 < nfull; kv0 += 64) chunk(kv0, std::false_type{});
  if (nfull < N) chunk(nfull, std::true_type{});
  const int D = H * HD;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int q = qbase + 16 * u + li;
    if (q < N) {
      const float inv = (DROP ? dsc : 1.f) / l_run[u];  // dropout keep scale folded in
      bf16* orow = out + ((size_t)b * N + q) * D + h * HD;
#pragma unroll
      for (int d = 0; d < C::DT; ++d) {
        bf16x4 v;
        v[0] = f2bf(o[u][d][0] * inv); v[1] = f2bf(o[u][d][1] * inv);
        v[2] = f2bf(o[u][d][2] * inv); v[3] = f2bf(o[u][d][3] * inv);
        *reinterpret_cast<bf16x4*>(orow + 16 * d + 4 * g) = v;
      }
      if (g == 0) lse[(size_t)bh * N + q] = (m_run[u] + log2f(l_run[u])) * LN2;
    }
  }
}
template __global__ void attn_fwd_resident_kernel<32, true>(const bf16*, bf16*, float*, int, int, int, float,
                                                            const int64_t*, int, uint32_t, float, uint32_t*);
template __global__ void attn_fwd_resident_kernel<32, false>(const bf16*, bf16*, float*, int, int, int, float,
                                                             const int64_t*, int, uint32_t, float, uint32_t*);
template __global__ void attn_fwd_resident_kernel<64, true>(const bf16*, bf16*, float*, int, int, int, float,
                                                            const int64_t*, int, uint32_t, float, uint32_t*);
template __global__ void attn_fwd_resident_kernel<64, false>(const bf16*, bf16*, float*, int, int, int, float,
                                                             const int64_t*, int, uint32_t, float, uint32_t*);

template <int HD>
static void launch_resident(const bf16* q, bf16* out, float* lse, int B, int H, int N, float scale,
                            const int64_t* rng, int site, uint32_t thr, float dsc, hipStream_t stream,
                            uint32_t* keep) {
  const int waves = (N + 31) / 32;
  const int NP = (N + 63) / 64 * 64;
  const int lds = 2 * NP * AC<HD>::S;
  static bool attr = [] {
    bool ok = true;
    for (const void* f : {reinterpret_cast<const void*>(&attn_fwd_resident_kernel<HD, true>),
                          reinterpret_cast<const void*>(&attn_fwd_resident_kernel<HD, false>)})
      ok = ok && hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
    return ok;
  }();
  (void)attr;
  if (thr)
    hipLaunchKernelGGL((attn_fwd_resident_kernel<HD, true>), dim3(B * H), dim3(64 * waves), lds, stream, q, out, lse,
                       B, H, N, scale, rng, site, thr, dsc, keep);
  else
    hipLaunchKernelGGL((attn_fwd_resident_kernel<HD, false>), dim3(B * H), dim3(64 * waves), lds, stream, q, out, lse,
                       B, H, N, scale, rng, site, thr, dsc, nullptr);
}

// ============================================================================ backward: dQ (+delta)
// U query groups of 16 per wave (64 U queries per workgroup): every K / V fragment a
// wave reads from LDS feeds U MFMAs (S and dP of each group), and every K^T fragment of
// the dQ update U more.  Only U = 1 is built (attn_bwd_launch: U = 2 measured slower,
// it costs occupancy); the two 32-key halves of a tile each run S / dP -> dS -> dQ in
// turn, so only half a tile's dS is live (128 -> 114 VGPRs).
template <int HD, int U, bool KB>
__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(const bf16* __restrict__ dout, const bf16* __restrict__ qkv,
                                                          const bf16* __restrict__ out, const float* __restrict__ lse,
                                                          float* __restrict__ delta, bf16* __restrict__ dqkv, int B,
                                                          int H, int N, float scale, const int64_t* __restrict__ rng,
                                                          int site, uint32_t thr, float dsc,
                                                          const uint32_t* __restrict__ keep) {
  using C = AC<HD>;
  __shared__ __attribute__((aligned(16))) char lds[4 * C::TILE];  // [buf][K | V], double-buffered
  const Blk blk = attn_block();
  const int bh = blk.y, b = bh / H, h = bh - b * H;
  const int D = H * HD;
  const size_t mat = (size_t)N * HD;
  const bf16* qb = qkv + (size_t)bh * mat;
  const bf16* kb = qkv + ((size_t)B * H + bh) * mat;
  const bf16* vb = qkv + ((size_t)2 * B * H + bh) * mat;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, li = lane & 15;
  KvStage<HD> stg;
  stg.load(kb, vb, 0, N);
  const float sl2 = scale * LOG2E;
  const uint32_t salt = thr ? site_salt(rng, site) : 0u;
  const int ntiles = (N + 63) / 64;
  constexpr bool kbits = KB;  // the launcher passes KB only with stored flags and thr > 0

  int q[U];
  bf16x8 qf[U][C::KS], df[U][C::KS];
  float dl[U], nl2[U];
  uint32_t pgq[U];
  const u32x2* kcol[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    q[u] = blk.x * (64 * U) + wave * (16 * U) + 16 * u + li;
    const bool qv = q[u] < N;
    // dO and O rows of this lane's query are token-major [B, N, D] with head offset h*HD
    const bf16* dorow = dout + ((size_t)b * N + (qv ? q[u] : 0)) * D + h * HD;
    const bf16* orow = out + ((size_t)b * N + (qv ? q[u] : 0)) * D + h * HD;
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < C::KS; ++k) {
      qf[u][k] = frag_glb<HD>(qb, q[u], N, k, g);
      bf16x8 dv, ov;
      if (qv) {
        dv = *reinterpret_cast<const bf16x8*>(dorow + 32 * k + 8 * g);
        ov = *reinterpret_cast<const bf16x8*>(orow + 32 * k + 8 * g);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) { dv[j] = f2bf(0.f); ov[j] = f2bf(0.f); }
      }
      df[u][k] = dv;
#pragma unroll
      for (int j = 0; j < 8; ++j) s += bf2f(dv[j]) * bf2f(ov[j]);
    }
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    dl[u] = s;
    if (qv && g == 0) delta[(size_t)bh * N + q[u]] = s;
    nl2[u] = qv ? -lse[(size_t)bh * N + q[u]] * LOG2E : -INFINITY;
    const uint32_t rowidx = (uint32_t)(((size_t)bh * N + q[u]) * attn_mask_ld(N));
    pgq[u] = ((rowidx >> 1) + 2u * (uint32_t)g) * DROP_GOLDEN;  // pair hash base of this lane's row
    // the forward's stored keep words of this lane's query (one per key tile)
    kcol[u] = reinterpret_cast<const u32x2*>(keep) + (size_t)bh * ntiles * N + (qv ? q[u] : 0);
  }

  f32x4 dq[U][C::DT];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int d = 0; d < C::DT; ++d) dq[u][d] = f32x4{0.f, 0.f, 0.f, 0.f};

  u32x2 kwc[U];  // keep words of the tile about to run (prefetched with its K / V)
#pragma unroll
  for (int u = 0; u < U; ++u) kwc[u] = kbits ? kcol[u][0] : u32x2{0u, 0u};
  stg.store(lds, lds + C::TILE);
  __syncthreads();
  // key mask only in the tail tile: a padded key has a zero K row (no dQ
  // contribution) but exp2(0 - lse) can overflow, so it must not reach dS
  // KB (stored drop flags present) is a kernel template parameter: a runtime kbits / rehash
  // branch per element group merged the two paths' multipliers through phi copies
  auto tile = [&](int it, auto mask_tag) {
    constexpr bool MASK = decltype(mask_tag)::value;
    const int kv0 = it * 64;
    const bool more = it + 1 < ntiles;
    // the next tile's keep words and K / V in one batch, issued on every tile (the last
    // one reloads itself, unused): behind an `if (more)` the compiler's path-merged count
    // was vmcnt(0), and a word loaded in the tile that uses it waited right away -- both
    // exposed the prefetch latency
    u32x2 kw[U];
    const int itn = more ? it + 1 : it;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      kw[u] = kwc[u];
      kwc[u] = KB ? kcol[u][(size_t)itn * N] : u32x2{0u, 0u};
    }
    stg.load(kb, vb, itn * 64, N);  // next tile lands during this tile's MFMAs
    const char* Kl = lds + (it & 1) * 2 * C::TILE;
    const char* Vl = Kl + C::TILE;
    // two halves of 32 keys: dS of a half feeds its dQ MFMAs right away (half the
    // live dS registers)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      f32x4 ds[U][2];
#pragma unroll
      for (int th = 0; th < 2; ++th) {
        const int t = 2 * s2 + th;
        f32x4 st[U], dp[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          st[u] = f32x4{0.f, 0.f, 0.f, 0.f};
          dp[u] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int s = 0; s < C::KS; ++s) {
          const bf16x8 kfr = frag_row<HD>(Kl, 16 * t + li, s, g);
          const bf16x8 vfr = frag_row<HD>(Vl, 16 * t + li, s, g);
#pragma unroll
          for (int u = 0; u < U; ++u) {
            st[u] = mfma16(kfr, qf[u][s], st[u]);
            dp[u] = mfma16(vfr, df[u][s], dp[u]);
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          // dropout multipliers (dsc kept, 0 dropped): the stored DROP flag sign-extended
          // into a mask clearing dsc; without stored flags the lane's 4 keys are
          // consecutive elements of one mask row (aligned: the row stride is a multiple of
          // 4), 2 pair hashes instead of 4 single ones
          float fk[4] = {1.f, 1.f, 1.f, 1.f};
          if constexpr (KB) {
            const uint32_t hw = (g < 2 ? kw[u][0] : kw[u][1]) >> (16 * (g & 1));
#pragma unroll
            for (int r = 0; r < 4; ++r)
              fk[r] = __uint_as_float(__float_as_uint(dsc) & ~(uint32_t)__builtin_amdgcn_sbfe((int)hw, drop_bit(t, r), 1));
          } else {
            if (thr) {
              bool kp[4];
              dropout_keep4_pg(salt, pgq[u] + (uint32_t)(kv0 / 2 + 8 * t) * DROP_GOLDEN, thr, kp);
#pragma unroll
              for (int r = 0; r < 4; ++r) fk[r] = kp[r] ? dsc : 0.f;
            }
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int key = kv0 + 16 * t + 4 * g + r;
            float pr = fexp2(fmaf(st[u][r], sl2, nl2[u]));
            if (MASK && key >= N) pr = 0.f;
            // (factoring dsc out of dS -- delta / dsc here, dsc in the final dQ / dK / dV
            // scales -- measured no faster: N=626 p=0.1 stored masks 145.5 vs 146.4 us).
            // One explicit fma: the KB and rehash instantiations must round alike (stored
            // flags == re-hashed masks, bit for bit), not per the compiler's contraction
            const float dd = (KB || thr) ? fmaf(dp[u][r], fk[r], -dl[u]) : dp[u][r] - dl[u];
            ds[u][th][r] = pr * dd;
          }
        }
      }
      bf16x8 sb[U];
#pragma unroll
      for (int u = 0; u < U; ++u) sb[u] = pack8(ds[u][0], ds[u][1]);
#pragma unroll
      for (int d = 0; d < C::DT; ++d) {
        const bf16x8 kt = frag_t<C::S>(Kl, 16 * d, s2, lane);
#pragma unroll
        for (int u = 0; u < U; ++u) dq[u][d] = mfma16(kt, sb[u], dq[u][d]);
      }
    }
    if (more) stg.store(lds + ((it + 1) & 1) * 2 * C::TILE, lds + ((it + 1) & 1) * 2 * C::TILE + C::TILE);
    __syncthreads();
  };
  const int nfull = N / 64;
  for (int it = 0; it < nfull; ++it) tile(it, std::false_type{});
  if (nfull < ntiles) tile(nfull, std::true_type{});
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (q[u] < N) {
      bf16* row = dqkv + ((size_t)b * N + q[u]) * (3 * D) + h * HD;
#pragma unroll
      for (int d = 0; d < C::DT; ++d) {
        bf16x4 v;
        v[0] = f2bf(dq[u][d][0] * scale); v[1] = f2bf(dq[u][d][1] * scale);
        v[2] = f2bf(dq[u][d][2] * scale); v[3] = f2bf(dq[u][d][3] * scale);
        *reinterpret_cast<bf16x4*>(row + 16 * d + 4 * g) = v;
      }
    }
  }
}

// ============================================================================ backward: dK, dV
// U key groups of 16 per wave (64 U keys per workgroup): every Q / dO fragment read
// from LDS feeds the S^T and dP^T MFMAs of U key groups, every dO^T / Q^T fragment the
// dV / dK updates of U groups (see attn_bwd_dq_kernel).  Per 32-query half of a tile:
// S^T / dP^T -> P / dS -> dV / dK, so half a tile's P and dS are live: 186 -> 150
// VGPRs, 2 -> 3 waves per SIMD, N=626 backward 161 -> 146 us (p=0.1, stored masks).
//
// KB: the forward's stored drop flags are read (a kernel-level template parameter: the
// same as a tag on the loop body measured slower, profiles/attn_bwd_kbtag_r5.txt)
template <int HD, int U, bool KB>
__global__ __launch_bounds__(256) void attn_bwd_dkv_kernel(const bf16* __restrict__ dout,
                                                           const bf16* __restrict__ qkv,
                                                           const float* __restrict__ lse,
                                                           const float* __restrict__ delta,
                                                           bf16* __restrict__ dqkv, int B, int H, int N, float scale,
                                                           const int64_t* __restrict__ rng, int site, uint32_t thr,
                                                           float dsc, const uint32_t* __restrict__ keep) {
  using C = AC<HD>;
  __shared__ __attribute__((aligned(16))) char lds[4 * C::TILE];  // [buf][Q | dO], double-buffered
  __shared__ float s_lse[2][64], s_del[2][64];
  // the forward's keep words of the query tile for this workgroup's U 64-key tiles,
  // [buf][key tile][half][query]
  __shared__ __attribute__((aligned(16))) uint32_t s_keep[2][U][2][64];
  const Blk blk = attn_block();
  const int bh = blk.y, b = bh / H, h = bh - b * H;
  const int D = H * HD;
  const size_t mat = (size_t)N * HD;
  const bf16* qb = qkv + (size_t)bh * mat;
  const bf16* kb = qkv + ((size_t)B * H + bh) * mat;
  const bf16* vb = qkv + ((size_t)2 * B * H + bh) * mat;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, li = lane & 15;
  const float sl2 = scale * LOG2E;
  const uint32_t salt = thr ? site_salt(rng, site) : 0u;

  int key[U];  // this lane's keys (columns of S)
  bf16x8 kf[U][C::KS], vf[U][C::KS];
  f32x4 dk[U][C::DT], dv[U][C::DT];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    key[u] = blk.x * (64 * U) + wave * (16 * U) + 16 * u + li;
#pragma unroll
    for (int s = 0; s < C::KS; ++s) {
      kf[u][s] = frag_glb<HD>(kb, key[u], N, s, g);
      vf[u][s] = frag_glb<HD>(vb, key[u], N, s, g);
    }
#pragma unroll
    for (int d = 0; d < C::DT; ++d) {
      dk[u][d] = f32x4{0.f, 0.f, 0.f, 0.f};
      dv[u][d] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }

  // register-staged prefetch of the next query tile: Q rows (head-major), dO rows
  // (token-major, head slice), LSE, delta and the keep words
  constexpr int PER = 64 * C::CPR / 256;
  // raw loads here, padded-row selects in store_tile (see KvStage: a select next to the
  // loads waits for them)
  u32x4 rq[PER], rd[PER];
  bool rok[PER];
  float rl = 0.f, rdl = 0.f;
  bool rlv = false;
  constexpr bool kbits = KB;  // the launcher passes KB only with stored flags and thr > 0
  const int ntiles = (N + 63) / 64;
  u32x2 rk = u32x2{0u, 0u};
  const int kt_mine = blk.x * U + (threadIdx.x >> 6);  // key tile whose word this thread stages
  auto load_tile = [&](int q0) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = threadIdx.x + i * 256;
      const int r = c / C::CPR, cc = c - r * C::CPR;
      const int rr = q0 + r < N ? q0 + r : N - 1;
      rok[i] = q0 + r < N;
      rq[i] = *reinterpret_cast<const u32x4*>(qb + (size_t)rr * HD + cc * 8);
      rd[i] = *reinterpret_cast<const u32x4*>(dout + ((size_t)b * N + rr) * D + h * HD + cc * 8);
    }
    if (threadIdx.x < 64 * U) {
      const int qq = q0 + (threadIdx.x & 63);
      const int qc = qq < N ? qq : N - 1;
      if (threadIdx.x < 64) {
        rl = lse[(size_t)bh * N + qc];
        rdl = delta[(size_t)bh * N + qc];
        rlv = qq < N;
      }
      if (kbits && kt_mine < ntiles) rk = reinterpret_cast<const u32x2*>(keep)[((size_t)bh * ntiles + kt_mine) * N + qc];
    }
  };
  auto store_tile = [&](int buf) {
    char* ql = lds + buf * 2 * C::TILE;
    char* dl = ql + C::TILE;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = threadIdx.x + i * 256;
      const int r = c / C::CPR, cc = c - r * C::CPR;
      const u32x4 z = {0u, 0u, 0u, 0u};
      *reinterpret_cast<u32x4*>(ql + r * C::S + cc * 16) = rok[i] ? rq[i] : z;
      *reinterpret_cast<u32x4*>(dl + r * C::S + cc * 16) = rok[i] ? rd[i] : z;
    }
    if (threadIdx.x < 64) {
      s_lse[buf][threadIdx.x] = rlv ? rl * LOG2E : INFINITY;
      s_del[buf][threadIdx.x] = rlv ? rdl : 0.f;
    }
    if (threadIdx.x < 64 * U) {
      s_keep[buf][threadIdx.x >> 6][0][threadIdx.x & 63] = rk[0];
      s_keep[buf][threadIdx.x >> 6][1][threadIdx.x & 63] = rk[1];
    }
  };
  load_tile(0);
  store_tile(0);
  __syncthreads();
  // (the stored-flag path as a compile-time tag, as in the dQ kernel, measured slower here:
  // 77.0 -> 84.1 us at N = 626, profiles/attn_bwd_kbtag_r5.txt)
  for (int it = 0; it < ntiles; ++it) {
    const int q0 = it * 64;
    const bool more = it + 1 < ntiles;
    if (more) load_tile(q0 + 64);
    const int buf = it & 1;
    const char* Ql = lds + buf * 2 * C::TILE;
    const char* Dl = Ql + C::TILE;
    const float* sl = s_lse[buf];
    const float* sd = s_del[buf];
    // two halves of 32 queries: P / dS of a half feed its dV / dK MFMAs right away
    // (half the live P / dS registers)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
    f32x4 pm[U][2], ds[U][2];
#pragma unroll
    for (int th = 0; th < 2; ++th) {
      const int t = 2 * s2 + th;
      f32x4 st[U], dp[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        st[u] = f32x4{0.f, 0.f, 0.f, 0.f};
        dp[u] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int s = 0; s < C::KS; ++s) {
        const bf16x8 qfr = frag_row<HD>(Ql, 16 * t + li, s, g);
        const bf16x8 dfr = frag_row<HD>(Dl, 16 * t + li, s, g);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          st[u] = mfma16(qfr, kf[u][s], st[u]);
          dp[u] = mfma16(dfr, vf[u][s], dp[u]);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        // dropout multipliers of (query 16t+4g+r, this lane's key u): dsc kept, 0 dropped
        float fk[4] = {1.f, 1.f, 1.f, 1.f};
        if (kbits) {
          // this lane's key within the workgroup's 64 U: word of tile kl >> 6, bit
          // keep_bitpos (half pos >> 5 of the staged 64-bit word); the stored DROP flag,
          // sign-extended to a 0 / all-ones word, clears dsc (bfe + and-not per element,
          // no compare / select pair per product)
          const int kl = wave * (16 * U) + 16 * u + li;
          const int pos = keep_bitpos(kl & 63);
          const u32x4 w = *reinterpret_cast<const u32x4*>(&s_keep[buf][kl >> 6][pos >> 5][16 * t + 4 * g]);
#pragma unroll
          for (int r = 0; r < 4; ++r)
            fk[r] = __uint_as_float(__float_as_uint(dsc) & ~(uint32_t)__builtin_amdgcn_sbfe((int)w[r], pos & 31, 1));
        } else if (thr) {
          bool kp[4];
          // a mask pair is two adjacent keys of one row, held by lanes li and li^1 --
          // each of the two hashes the pair of 2 of the 4 rows and they swap the results
          // (2 hashes per lane, not 4); the golden-constant multiply is hoisted
          const int odd = li & 1;
          const uint32_t ldh = (uint32_t)(attn_mask_ld(N) >> 1);
          const uint32_t pb = ((uint32_t)(bh * N + q0 + 4 * g + 2 * odd) * ldh + (uint32_t)(key[u] >> 1)) * DROP_GOLDEN;
          const uint32_t ldhg = ldh * DROP_GOLDEN;
          uint32_t hw[2];
#pragma unroll
          for (int v = 0; v < 2; ++v) hw[v] = drop_mix(pb + (uint32_t)(16 * t + v) * ldhg + salt);
          const uint32_t p0 = (uint32_t)__shfl_xor((int)hw[0], 1, 64), p1 = (uint32_t)__shfl_xor((int)hw[1], 1, 64);
          const uint32_t hr[4] = {odd ? p0 : hw[0], odd ? p1 : hw[1], odd ? hw[0] : p0, odd ? hw[1] : p1};
#pragma unroll
          for (int r = 0; r < 4; ++r) kp[r] = (odd ? (hr[r] >> 16) : (hr[r] & 0xFFFFu)) >= thr;
#pragma unroll
          for (int r = 0; r < 4; ++r) fk[r] = kp[r] ? dsc : 0.f;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int qr = 16 * t + 4 * g + r;
          const float pr = fexp2(fmaf(st[u][r], sl2, -sl[qr]));  // padded queries: lse = +inf -> 0
          // dropped: pr * 0 = +0 and fma(dp, 0, -delta) = -delta; one explicit fma so the
          // KB and re-hash instantiations round alike (stored flags == re-hashed masks)
          const float pd = (KB || thr) ? pr * fk[r] : pr;
          const float dd = (KB || thr) ? fmaf(dp[u][r], fk[r], -sd[qr]) : dp[u][r] - sd[qr];
          pm[u][th][r] = pd;
          ds[u][th][r] = pr * dd;
        }
      }
    }
    {
      bf16x8 pb[U], sb[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        pb[u] = pack8(pm[u][0], pm[u][1]);
        sb[u] = pack8(ds[u][0], ds[u][1]);
      }
#pragma unroll
      for (int d = 0; d < C::DT; ++d) {
        const bf16x8 dT = frag_t<C::S>(Dl, 16 * d, s2, lane);
        const bf16x8 qT = frag_t<C::S>(Ql, 16 * d, s2, lane);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          dv[u][d] = mfma16(dT, pb[u], dv[u][d]);
          dk[u][d] = mfma16(qT, sb[u], dk[u][d]);
        }
      }
    }
    }
    if (more) store_tile(buf ^ 1);
    __syncthreads();
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (key[u] < N) {
      bf16* row = dqkv + ((size_t)b * N + key[u]) * (3 * D) + h * HD;
#pragma unroll
      for (int d = 0; d < C::DT; ++d) {
        bf16x4 kv, vv;
        kv[0] = f2bf(dk[u][d][0] * scale); kv[1] = f2bf(dk[u][d][1] * scale);
        kv[2] = f2bf(dk[u][d][2] * scale); kv[3] = f2bf(dk[u][d][3] * scale);
        vv[0] = f2bf(dv[u][d][0]); vv[1] = f2bf(dv[u][d][1]);
        vv[2] = f2bf(dv[u][d][2]); vv[3] = f2bf(dv[u][d][3]);
        *reinterpret_cast<bf16x4*>(row + D + 16 * d + 4 * g) = kv;
        *reinterpret_cast<bf16x4*>(row + 2 * D + 16 * d + 4 * g) = vv;
      }
    }
  }
}
#define DC_INST_BWD(HD, U)                                                                                       \
  template __global__ void attn_bwd_dq_kernel<HD, U, true>(const bf16*, const bf16*, const bf16*, const float*,   \
                                                           float*, bf16*, int, int, int, float, const int64_t*,    \
                                                           int, uint32_t, float, const uint32_t*);                 \
  template __global__ void attn_bwd_dq_kernel<HD, U, false>(const bf16*, const bf16*, const bf16*, const float*,  \
                                                            float*, bf16*, int, int, int, float, const int64_t*,   \
                                                            int, uint32_t, float, const uint32_t*);                \
  template __global__ void attn_bwd_dkv_kernel<HD, U, true>(const bf16*, const bf16*, const float*, const float*,  \
                                                            bf16*, int, int, int, float, const int64_t*, int,      \
                                                            uint32_t, float, const uint32_t*);                     \
  template __global__ void attn_bwd_dkv_kernel<HD, U, false>(const bf16*, const bf16*, const float*, const float*, \
                                                             bf16*, int, int, int, float, const int64_t*, int,     \
                                                             uint32_t, float, const uint32_t*);
DC_INST_BWD(32, 1) DC_INST_BWD(64, 1)

// ============================================================================ short sequences (N <= 128)
// One workgroup per (b, h) holding the WHOLE sequence: NP = 32*ceil(N/32) padded
// rows, NP/16 waves (one 16-query / 16-key strip each).  For the ViT-tiny shape
// (N = 65, hd = 32) the flash kernels above pad to 128 queries x 128 keys and
// launch 2 workgroups per head; here one 6-wave workgroup does exact (not
// online) softmax over 96 keys and the backward is ONE kernel:
//   phase A (wave = 16 queries): S^T = K Q^T, dP^T = V dO^T, delta, P and dS
//            (dropout applied) written to LDS as [q][key] images, dQ^T += K^T dS^T;
//   phase B (wave = 16 keys):    dV^T += dO^T P, dK^T += Q^T dS, contracting over
//            all queries through transposing LDS reads of the images.
// Latency rules: every global load of the kernel (all staged images, O rows,
// LSE) is issued before the first wait (row addresses clamped, padded rows
// zeroed by select, no branches), and dropout is a template flag so the
// softmax / dS loops stay branch-free.  Dropout masks are bit-identical to the
// flash kernels (same element index).
template <int HD, int NP>
struct ShortImg {
  static constexpr int NT = NP * 4;        // threads of the workgroup
  static constexpr int CPR = HD / 8;       // 16-B chunks per row
  static constexpr int PER = NP * CPR / NT;  // chunks per thread (= HD / 32)
  static constexpr int RS = 2 * HD + 32;   // padded LDS row stride (bytes)
  u32x4 v[PER];
  // chunk c -> (row, 16-B chunk).  64-B rows (hd 32): an 8-lane ds_write_b128
  // group takes rows r and r+2 (48 dwords apart, disjoint banks mod 32) instead
  // of r and r+1 (2-way conflict at the 96-B stride)
  __device__ __forceinline__ static void rc(int c, int& r, int& cc) {
    if (CPR == 4) {
      const int grp = c >> 3, j = c & 7;
      r = (grp >> 1) * 4 + (grp & 1) + 2 * (j >> 2);
      cc = j & 3;
    } else {
      r = c / CPR;
      cc = c - r * CPR;
    }
  }
  __device__ __forceinline__ void load(const bf16* __restrict__ base, size_t ld, int N) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = threadIdx.x + i * NT;
      int r, cc;
      rc(c, r, cc);
      const int rr = r < N ? r : N - 1;
      const u32x4 x = *reinterpret_cast<const u32x4*>(base + (size_t)rr * ld + cc * 8);
      const u32x4 z = {0u, 0u, 0u, 0u};
      v[i] = r < N ? x : z;
    }
  }
  __device__ __forceinline__ void store(char* img) const {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = threadIdx.x + i * NT;
      int r, cc;
      rc(c, r, cc);
      *reinterpret_cast<u32x4*>(img + r * RS + cc * 16) = v[i];
    }
  }
};

// [query][key] P / dS images of the short backward: 8-B column pieces XOR-ed by
// ((row >> 2) & 3) so the 16 rows of a ds_write_b64 lane group land on distinct
// banks; the transposed reads (4 rows sharing one XOR) stay conflict-free
__device__ __forceinline__ int pimg_off(int row, int byte, int stride) {
  return row * stride + (byte ^ (((row >> 2) & 3) << 3));
}

template <int STRIDE>
__device__ __forceinline__ bf16x8 frag_t_pimg(const char* lds, int c0, int s, int lane) {
  const int i = lane & 15, g = lane >> 4, q = i >> 2, p = i & 3;
  const int ra = 32 * s + 4 * g + q;  // ra + 16 has the same XOR
  const char* pa = lds + pimg_off(ra, (c0 + 4 * p) * 2, STRIDE);
  const bf16x4 lo = lds_read_tr(reinterpret_cast<const bf16*>(pa));
  const bf16x4 hi = lds_read_tr(reinterpret_cast<const bf16*>(pa + 16 * STRIDE));
  bf16x8 v;
  v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
  v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
  return v;
}

__device__ __forceinline__ bf16x4 pack4(const f32x4& a) {
  bf16x4 v;
  v[0] = f2bf(a[0]); v[1] = f2bf(a[1]); v[2] = f2bf(a[2]); v[3] = f2bf(a[3]);
  return v;
}

template <int HD, int NP, bool DROP>
__global__ __launch_bounds__(NP * 4) void attn_fwd_short_kernel(const bf16* __restrict__ qkv, bf16* __restrict__ out,
                                                                float* __restrict__ lse, int B, int H, int N,
                                                                float scale, const int64_t* __restrict__ rng,
                                                                int site, uint32_t thr, float dsc,
                                                                uint32_t* __restrict__ keep_bits) {
  using I = ShortImg<HD, NP>;
  constexpr int RS = I::RS, KS = HD / 32, DT = HD / 16, KT = NP / 16;
  static_assert(KT * 4 <= 32, "one 32-bit keep word per lane");
  // dynamic LDS (2 * NP * RS bytes, see short_lds): with static LDS, 384-thread
  // workgroups were admitted one per CU from ~60 KB on (tools/ub_lds_census.hip)
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* Kl = lds;
  char* Vl = lds + NP * RS;
  const int bh = blockIdx.x, b = bh / H, h = bh - b * H;
  const size_t mat = (size_t)N * HD;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, li = lane & 15;
  const int q = wave * 16 + li;
  I ik, iv;
  ik.load(qkv + ((size_t)B * H + bh) * mat, HD, N);
  iv.load(qkv + ((size_t)2 * B * H + bh) * mat, HD, N);
  bf16x8 qf[KS];
  {
    const bf16* qrow = qkv + (size_t)bh * mat + (size_t)(q < N ? q : N - 1) * HD;
#pragma unroll
    for (int s = 0; s < KS; ++s) qf[s] = *reinterpret_cast<const bf16x8*>(qrow + 32 * s + 8 * g);
  }
  const uint32_t salt = DROP ? site_salt(rng, site) : 0u;
  ik.store(Kl);
  iv.store(Vl);
  __syncthreads();
  if (wave * 16 >= N) return;  // no barrier follows
  const float sl2 = scale * LOG2E;
  f32x4 st[KT];
#pragma unroll
  for (int t = 0; t < KT; ++t) {
    st[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s) st[t] = mfma16(frag_row<HD>(Kl, 16 * t + li, s, g), qf[s], st[t]);
  }
  float mx = -INFINITY;  // raw-score max (sl2 > 0), scaled below
#pragma unroll
  for (int t = 0; t < KT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (16 * t + 16 > N && 16 * t + 4 * g + r >= N) st[t][r] = -INFINITY;  // tail tiles only (uniform test first)
      mx = fmaxf(mx, st[t][r]);
    }
  mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  mx *= sl2;
  const float nmx = -mx;
  float l = 0.f;
  const uint32_t rowidx = (uint32_t)(((size_t)bh * N + q) * attn_mask_ld(N));
  const uint32_t pgs = DROP ? ((rowidx >> 1) + 2u * (uint32_t)g) * DROP_GOLDEN + salt : 0u;
  const uint32_t thr2 = (thr >> 1) * 0x10001u;  // thr / 2 in both 16-bit halves (drop_mask2)
  // dropout as packed 16-bit drop masks AND-NOT-ed onto the bf16 P pairs (as in the flash
  // forward: no per-element compare / select), the drop flags from the same masks
  uint32_t dm[KT][2], db = 0u;
#pragma unroll
  for (int t = 0; t < KT; ++t) {
    if (DROP) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        dm[t][j] = drop_mask2(drop_mix(pgs + (uint32_t)(8 * t + j) * DROP_GOLDEN), thr2);
        db |= dm[t][j] & ((1u << (2 * t + j)) | (1u << (16 + 2 * t + j)));
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float pv = fexp2(fmaf(st[t][r], sl2, nmx));  // keep scale folded into the final 1/l
      l += pv;
      st[t][r] = pv;
    }
  }
  // the drop flags of this lane's (query, 16t + 4g + r) elements for the backward
  // (short_drop_bit layout): one word per lane instead of re-hashing KT*2 pairs
  if (DROP && keep_bits != nullptr) keep_bits[((size_t)bh * NP + q) * 4 + g] = db;
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);
  f32x4 o[DT];
#pragma unroll
  for (int d = 0; d < DT; ++d) o[d] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s2 = 0; s2 < NP / 32; ++s2) {
    const bf16x8 pb = DROP ? pack8_drop(st[2 * s2], st[2 * s2 + 1], dm[2 * s2], dm[2 * s2 + 1])
                           : pack8(st[2 * s2], st[2 * s2 + 1]);
#pragma unroll
    for (int d = 0; d < DT; ++d) o[d] = mfma16(frag_t<RS>(Vl, 16 * d, s2, lane), pb, o[d]);
  }
  if (q < N) {
    const float inv = (DROP ? dsc : 1.f) / l;
    bf16* orow = out + ((size_t)b * N + q) * (H * HD) + h * HD;
#pragma unroll
    for (int d = 0; d < DT; ++d) *reinterpret_cast<bf16x4*>(orow + 16 * d + 4 * g) = pack4(o[d] * inv);
    if (g == 0) lse[(size_t)bh * N + q] = (mx + log2f(l)) * LN2;
  }
}

template <int HD, int NP, bool DROP, bool KB>
__global__ __launch_bounds__(NP * 4) void attn_bwd_short_kernel(const bf16* __restrict__ dout,
                                                                const bf16* __restrict__ qkv,
                                                                const bf16* __restrict__ out,
                                                                const float* __restrict__ lse,
                                                                bf16* __restrict__ dqkv, int B, int H, int N,
                                                                float scale, const int64_t* __restrict__ rng,
                                                                int site, uint32_t thr, float dsc,
                                                                const uint32_t* __restrict__ keep_bits) {
  using I = ShortImg<HD, NP>;
  constexpr int RS = I::RS, PS = 2 * NP + 32, KS = HD / 32, DT = HD / 16, KT = NP / 16;
  // dynamic LDS (4 * NP * RS + 2 * NP * PS bytes, see short_lds): the same image as a
  // static array (79,872 B at NP 96) got ONE 384-thread workgroup per CU instead of two
  // -- 128 of the ViT-tiny step's 384 workgroups then waited for a second round
  // (workgroup-entry timestamps, tools/ub_lds_census.hip)
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* Ql = lds;
  char* Kl = Ql + NP * RS;
  char* Vl = Kl + NP * RS;
  char* Dl = Vl + NP * RS;
  char* Pl = Dl + NP * RS;   // [q][key] dropped probabilities
  char* Sl = Pl + NP * PS;   // [q][key] dS
  const int bh = blockIdx.x, b = bh / H, h = bh - b * H;
  const int D = H * HD;
  const size_t mat = (size_t)N * HD;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, li = lane & 15;
  const int q = wave * 16 + li;
  const bool qv = q < N;
  const int qc = qv ? q : N - 1;
  // ---- every global load up front
  I iq, ik, iv, id;
  iq.load(qkv + (size_t)bh * mat, HD, N);
  ik.load(qkv + ((size_t)B * H + bh) * mat, HD, N);
  iv.load(qkv + ((size_t)2 * B * H + bh) * mat, HD, N);
  id.load(dout + (size_t)b * N * D + h * HD, D, N);
  bf16x8 of[KS];
  {
    const bf16* orow = out + ((size_t)b * N + qc) * D + h * HD;
#pragma unroll
    for (int s = 0; s < KS; ++s) of[s] = *reinterpret_cast<const bf16x8*>(orow + 32 * s + 8 * g);
  }
  const float lse_raw = lse[(size_t)bh * N + qc];
  // the forward's drop flags (short_drop_bit layout) when it stored them (KB: a kernel
  // template parameter, so the flag and re-hash paths are separate instantiations)
  constexpr bool have_bits = DROP && KB;
  const uint32_t kbits = have_bits ? keep_bits[((size_t)bh * NP + q) * 4 + g] : 0u;
  const uint32_t salt = DROP ? site_salt(rng, site) : 0u;
  iq.store(Ql);
  ik.store(Kl);
  iv.store(Vl);
  id.store(Dl);
  __syncthreads();

  // ---- phase A: this wave's 16 queries against all keys
  const float lse2 = qv ? lse_raw * LOG2E : INFINITY;
  const float sl2 = scale * LOG2E;
  bf16x8 qf[KS], df[KS];
  float dl = 0.f;  // delta = rowsum(dO * O) of this lane's query
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    qf[s] = frag_row<HD>(Ql, q, s, g);
    df[s] = frag_row<HD>(Dl, q, s, g);
#pragma unroll
    for (int j = 0; j < 8; ++j) dl += bf2f(df[s][j]) * bf2f(of[s][j]);
  }
  dl += __shfl_xor(dl, 16, 64);
  dl += __shfl_xor(dl, 32, 64);
  const uint32_t rowidx = (uint32_t)(((size_t)bh * N + q) * attn_mask_ld(N));
  f32x4 ds[KT];
#pragma unroll
  for (int t = 0; t < KT; ++t) {
    f32x4 st = f32x4{0.f, 0.f, 0.f, 0.f}, dp = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      st = mfma16(frag_row<HD>(Kl, 16 * t + li, s, g), qf[s], st);
      dp = mfma16(frag_row<HD>(Vl, 16 * t + li, s, g), df[s], dp);
    }
    f32x4 pm;
    // dropout multipliers: dsc kept, 0 dropped (stored DROP flags, short_drop_bit layout,
    // sign-extended into a mask clearing dsc: bfe + and-not per element)
    float fk[4] = {1.f, 1.f, 1.f, 1.f};
    if constexpr (DROP) {
      if constexpr (KB) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          fk[r] = __uint_as_float(__float_as_uint(dsc) &
                                  ~(uint32_t)__builtin_amdgcn_sbfe((int)kbits, short_drop_bit(t, r), 1));
      } else {
        bool kq[4];
        dropout_keep4_pg(salt, ((rowidx >> 1) + 2u * (uint32_t)g + 8u * (uint32_t)t) * DROP_GOLDEN, thr, kq);
#pragma unroll
        for (int r = 0; r < 4; ++r) fk[r] = kq[r] ? dsc : 0.f;
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int key = 16 * t + 4 * g + r;
      float pr = fexp2(fmaf(st[r], sl2, -lse2));
      if (16 * t + 16 > N && key >= N) pr = 0.f;  // tail tiles only (uniform test first)
      // dropped: pr * 0 = +0, fma(dp, 0, -delta) = -delta; one explicit fma so both
      // instantiations round alike (stored flags == re-hashed masks, bit for bit)
      pm[r] = DROP ? pr * fk[r] : pr;
      ds[t][r] = pr * (DROP ? fmaf(dp[r], fk[r], -dl) : dp[r] - dl);
    }
    *reinterpret_cast<bf16x4*>(Pl + pimg_off(q, (16 * t + 4 * g) * 2, PS)) = pack4(pm);
    *reinterpret_cast<bf16x4*>(Sl + pimg_off(q, (16 * t + 4 * g) * 2, PS)) = pack4(ds[t]);
  }
  f32x4 dq[DT];
#pragma unroll
  for (int d = 0; d < DT; ++d) dq[d] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s2 = 0; s2 < NP / 32; ++s2) {
    const bf16x8 sb = pack8(ds[2 * s2], ds[2 * s2 + 1]);
#pragma unroll
    for (int d = 0; d < DT; ++d) dq[d] = mfma16(frag_t<RS>(Kl, 16 * d, s2, lane), sb, dq[d]);
  }
  if (qv) {
    bf16* row = dqkv + ((size_t)b * N + q) * (3 * D) + h * HD;
#pragma unroll
    for (int d = 0; d < DT; ++d) *reinterpret_cast<bf16x4*>(row + 16 * d + 4 * g) = pack4(dq[d] * scale);
  }
  __syncthreads();

  // ---- phase B: this wave's 16 keys against all queries
  const int key = wave * 16 + li;
  f32x4 dk[DT], dv[DT];
#pragma unroll
  for (int d = 0; d < DT; ++d) {
    dk[d] = f32x4{0.f, 0.f, 0.f, 0.f};
    dv[d] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int s = 0; s < NP / 32; ++s) {
    const bf16x8 pb = frag_t_pimg<PS>(Pl, 16 * wave, s, lane);
    const bf16x8 sb = frag_t_pimg<PS>(Sl, 16 * wave, s, lane);
#pragma unroll
    for (int d = 0; d < DT; ++d) {
      dv[d] = mfma16(frag_t<RS>(Dl, 16 * d, s, lane), pb, dv[d]);
      dk[d] = mfma16(frag_t<RS>(Ql, 16 * d, s, lane), sb, dk[d]);
    }
  }
  if (key < N) {
    bf16* row = dqkv + ((size_t)b * N + key) * (3 * D) + h * HD;
#pragma unroll
    for (int d = 0; d < DT; ++d) {
      *reinterpret_cast<bf16x4*>(row + D + 16 * d + 4 * g) = pack4(dk[d] * scale);
      *reinterpret_cast<bf16x4*>(row + 2 * D + 16 * d + 4 * g) = pack4(dv[d]);
    }
  }
}

// LDS bytes of the short kernels' images (dynamic shared memory)
template <int HD, int NP>
struct ShortLds {
  static constexpr int RS = ShortImg<HD, NP>::RS, PS = 2 * NP + 32;
  static constexpr int FWD = 2 * NP * RS;
  static constexpr int BWD = 4 * NP * RS + 2 * NP * PS;
};

template <typename K>
static void allow_lds(K kernel, int bytes) {
  if (bytes > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

template <int HD, int NP, bool DROP>
struct ShortLaunch {
  static void run(bool bwd, const bf16* d, const bf16* q, const bf16* o, float* lse, const float* lse_in,
                  bf16* outp, int B, int H, int N, float scale, const int64_t* rng, int site, uint32_t thr,
                  float dsc, hipStream_t stream, uint32_t* kb) {
    using L = ShortLds<HD, NP>;
    static const bool attr = [] {
      allow_lds(&attn_fwd_short_kernel<HD, NP, DROP>, L::FWD);
      allow_lds(&attn_bwd_short_kernel<HD, NP, DROP, false>, L::BWD);
      allow_lds(&attn_bwd_short_kernel<HD, NP, DROP, DROP>, L::BWD);
      return true;
    }();
    (void)attr;
    if (!bwd)
      hipLaunchKernelGGL((attn_fwd_short_kernel<HD, NP, DROP>), dim3(B * H), dim3(NP * 4), L::FWD, stream, q, outp,
                         lse, B, H, N, scale, rng, site, thr, dsc, kb);
    else if (DROP && kb != nullptr)  // stored drop flags: the KB instantiation
      hipLaunchKernelGGL((attn_bwd_short_kernel<HD, NP, DROP, DROP>), dim3(B * H), dim3(NP * 4), L::BWD, stream, d,
                         q, o, lse_in, outp, B, H, N, scale, rng, site, thr, dsc, kb);
    else
      hipLaunchKernelGGL((attn_bwd_short_kernel<HD, NP, DROP, false>), dim3(B * H), dim3(NP * 4), L::BWD, stream, d,
                         q, o, lse_in, outp, B, H, N, scale, rng, site, thr, dsc, kb);
  }
};

template <int HD, int NP>
static void launch_short(bool bwd, const bf16* d, const bf16* q, const bf16* o, float* lse, const float* lse_in,
                         bf16* outp, int B, int H, int N, float scale, const int64_t* rng, int site, uint32_t thr,
                         float dsc, hipStream_t stream, uint32_t* kb) {
  if (thr)
    ShortLaunch<HD, NP, true>::run(bwd, d, q, o, lse, lse_in, outp, B, H, N, scale, rng, site, thr, dsc, stream, kb);
  else
    ShortLaunch<HD, NP, false>::run(bwd, d, q, o, lse, lse_in, outp, B, H, N, scale, rng, site, thr, dsc, stream, kb);
}

template <int HD>
static void dispatch_short(bool bwd, const bf16* d, const bf16* q, const bf16* o, float* lse, const float* lse_in,
                           bf16* outp, int B, int H, int N, float scale, const int64_t* rng, int site, uint32_t thr,
                           float dsc, hipStream_t stream, uint32_t* kb = nullptr) {
  switch ((N + 31) / 32) {
    case 1: launch_short<HD, 32>(bwd, d, q, o, lse, lse_in, outp, B, H, N, scale, rng, site, thr, dsc, stream, kb); break;
    case 2: launch_short<HD, 64>(bwd, d, q, o, lse, lse_in, outp, B, H, N, scale, rng, site, thr, dsc, stream, kb); break;
    case 3: launch_short<HD, 96>(bwd, d, q, o, lse, lse_in, outp, B, H, N, scale, rng, site, thr, dsc, stream, kb); break;
    default: launch_short<HD, 128>(bwd, d, q, o, lse, lse_in, outp, B, H, N, scale, rng, site, thr, dsc, stream, kb); break;
  }
}

#define DC_INST_SHORT1(HD, NP, DR)                                                                                 \
  template __global__ void attn_fwd_short_kernel<HD, NP, DR>(const bf16*, bf16*, float*, int, int, int, float,    \
                                                             const int64_t*, int, uint32_t, float, uint32_t*);    \
  template __global__ void attn_bwd_short_kernel<HD, NP, DR, false>(const bf16*, const bf16*, const bf16*,        \
                                                                     const float*, bf16*, int, int, int, float,   \
                                                                     const int64_t*, int, uint32_t, float,        \
                                                                     const uint32_t*);
#define DC_INST_SHORT(HD, NP)                                                                                      \
  DC_INST_SHORT1(HD, NP, true) DC_INST_SHORT1(HD, NP, false)                                                       \
  template __global__ void attn_bwd_short_kernel<HD, NP, true, true>(const bf16*, const bf16*, const bf16*,        \
                                                                      const float*, bf16*, int, int, int, float,  \
                                                                      const int64_t*, int, uint32_t, float,       \
                                                                      const uint32_t*);
DC_INST_SHORT(32, 32) DC_INST_SHORT(32, 64) DC_INST_SHORT(32, 96) DC_INST_SHORT(32, 128)
DC_INST_SHORT(64, 32) DC_INST_SHORT(64, 64) DC_INST_SHORT(64, 96) DC_INST_SHORT(64, 128)


constexpr int SHORT_MAX_N = 128;

}  // namespace dc

using namespace dc;

// Long sequences: the flash / resident forwards store one 64-bit keep word per
// (b, h, 64-key tile, query) for the backward (attn_fwd_launch picks them whenever
// it is handed a keep buffer); short ones one 32-bit word per lane.
static bool long_keep_path(int B, int H, int N) { return N >= 384 || (N <= 320 && B * H >= 192); }

int64_t attn_keep_words(int B, int H, int N, int hd) {
  if (hd != 32 && hd != 64) return 0;
  if (N <= SHORT_MAX_N) return (int64_t)B * H * (32 * ((N + 31) / 32)) * 4;
  if (!long_keep_path(B, H, N)) return 0;  // (320, 384) with few heads: v1 forward, masks re-hashed
  return (int64_t)B * H * N * ((N + 63) / 64) * 2;
}

void attn_fwd_launch(const void* qkv, void* o, float* lse, int B, int H, int N, int hd, float scale,
                     const int64_t* rng, int site, double p, hipStream_t stream, uint32_t* keep_bits) {
  const dim3 grid((N + 63) / 64, B * H);
  const uint32_t thr = drop_threshold_host(p);
  const float dsc = p > 0 ? 1.f / (1.f - (float)p) : 1.f;
  const bf16* q = reinterpret_cast<const bf16*>(qkv);
  bf16* out = reinterpret_cast<bf16*>(o);
  if (hd != 32 && hd != 64) throw std::runtime_error("attention: head dim must be 32 or 64");
  if (N <= SHORT_MAX_N) {
    if (hd == 32)
      dispatch_short<32>(false, nullptr, q, nullptr, lse, nullptr, out, B, H, N, scale, rng, site, thr, dsc, stream,
                         keep_bits);
    else
      dispatch_short<64>(false, nullptr, q, nullptr, lse, nullptr, out, B, H, N, scale, rng, site, thr, dsc, stream,
                         keep_bits);
    return;
  }
  uint32_t* kb = thr ? keep_bits : nullptr;
  // one workgroup per head: needs ~a workgroup per CU to pay off.  Measured N=257
  // hd=64: B*H=256 20.1 vs 31.9 us (one 64-query workgroup per tile); B*H=128 equal
  // without dropout, 27 vs 22 with
  if (N <= 320 && B * H >= 192) {
    if (hd == 32) launch_resident<32>(q, out, lse, B, H, N, scale, rng, site, thr, dsc, stream, kb);
    else launch_resident<64>(q, out, lse, B, H, N, scale, rng, site, thr, dsc, stream, kb);
    return;
  }
  // v2 (128 queries per workgroup) has half the workgroups of v1: measured better from
  // ~600 tokens (N=626: 63 vs 71 us without dropout), worse at N=257 with dropout (25 vs 22 us)
  if (N >= 384) {
    const dim3 grid2((N + 127) / 128, B * H);
    if (hd == 32) {
      if (thr) hipLaunchKernelGGL((attn_fwd_flash2_kernel<32, true>), grid2, dim3(256), 0, stream, q, out, lse, B, H, N, scale, rng, site, thr, dsc, kb);
      else hipLaunchKernelGGL((attn_fwd_flash2_kernel<32, false>), grid2, dim3(256), 0, stream, q, out, lse, B, H, N, scale, rng, site, thr, dsc, kb);
    } else {
      if (thr) hipLaunchKernelGGL((attn_fwd_flash2_kernel<64, true>), grid2, dim3(256), 0, stream, q, out, lse, B, H, N, scale, rng, site, thr, dsc, kb);
      else hipLaunchKernelGGL((attn_fwd_flash2_kernel<64, false>), grid2, dim3(256), 0, stream, q, out, lse, B, H, N, scale, rng, site, thr, dsc, kb);
    }
    return;
  }
  if (keep_bits != nullptr && thr)
    throw std::runtime_error("attention: no stored keep masks on this path (attn_keep_words returned 0)");
  if (hd == 32)
    hipLaunchKernelGGL(attn_fwd_kernel<32>, grid, dim3(256), 0, stream, q, out, lse, B, H, N, scale, rng, site, thr, dsc);
  else
    hipLaunchKernelGGL(attn_fwd_kernel<64>, grid, dim3(256), 0, stream, q, out, lse, B, H, N, scale, rng, site, thr, dsc);
}

void attn_bwd_launch(const void* dout, const void* qkv, const void* o, const float* lse, void* dqkv,
                        float* delta, int B, int H, int N, int hd, float scale, const int64_t* rng, int site,
                        double p, hipStream_t stream, const uint32_t* keep_bits) {
  uint32_t* kb = const_cast<uint32_t*>(keep_bits);  // read-only in the backward kernels
  const dim3 grid((N + 63) / 64, B * H);
  const uint32_t thr = drop_threshold_host(p);
  const float dsc = p > 0 ? 1.f / (1.f - (float)p) : 1.f;
  const bf16* d = reinterpret_cast<const bf16*>(dout);
  const bf16* q = reinterpret_cast<const bf16*>(qkv);
  const bf16* oo = reinterpret_cast<const bf16*>(o);
  bf16* dq = reinterpret_cast<bf16*>(dqkv);
  if (N <= SHORT_MAX_N && (hd == 32 || hd == 64)) {
    if (hd == 32) dispatch_short<32>(true, d, q, oo, nullptr, lse, dq, B, H, N, scale, rng, site, thr, dsc, stream, kb);
    else dispatch_short<64>(true, d, q, oo, nullptr, lse, dq, B, H, N, scale, rng, site, thr, dsc, stream, kb);
    return;
  }
  if (hd != 32 && hd != 64) throw std::runtime_error("attention: head dim must be 32 or 64");
  // one 16-row group per wave (U = 1).  Measured slower and not built: U = 2 (every
  // LDS fragment feeding two MFMAs; N=626 p=0.1 stored masks 154.1 vs 146.1 us, N=2,501
  // 448 vs 337: 174 / 236 VGPRs put dQ / dK-dV at 2 waves per SIMD against 4 / 3), and
  // a dK/dV prefetch two query tiles ahead in two register sets (178 VGPRs, 2 waves per
  // SIMD: 180 vs 146 us) -- the kernels need the latency hiding of occupancy more
  const dim3 gridu((N + 63) / 64, B * H);
#define DC_LAUNCH_BWD(HDV, UV)                                                                                        \
  if (thr && keep_bits) {                                                                                             \
    hipLaunchKernelGGL((attn_bwd_dq_kernel<HDV, UV, true>), gridu, dim3(256), 0, stream, d, q, oo, lse, delta, dq, B,  \
                       H, N, scale, rng, site, thr, dsc, keep_bits);                                                 \
    hipLaunchKernelGGL((attn_bwd_dkv_kernel<HDV, UV, true>), gridu, dim3(256), 0, stream, d, q, lse, delta, dq, B, H, \
                       N, scale, rng, site, thr, dsc, keep_bits);                                                    \
  } else {                                                                                                            \
    hipLaunchKernelGGL((attn_bwd_dq_kernel<HDV, UV, false>), gridu, dim3(256), 0, stream, d, q, oo, lse, delta, dq,  \
                       B, H, N, scale, rng, site, thr, dsc, keep_bits);                                              \
    hipLaunchKernelGGL((attn_bwd_dkv_kernel<HDV, UV, false>), gridu, dim3(256), 0, stream, d, q, lse, delta, dq, B,   \
                       H, N, scale, rng, site, thr, dsc, keep_bits);                                                 \
  }
  if (hd == 32) { DC_LAUNCH_BWD(32, 1) }
  else { DC_LAUNCH_BWD(64, 1) }
#undef DC_LAUNCH_BWD
}
