// Shared gfx950 GEMM building blocks (gemm.hip): LDS image
// swizzles + fragment readers, the LDS-DMA operand loader (bounds-checked
// `buffer_load ... lds` with the swizzle applied on the source address),
// counted vmcnt waits, raw barriers and the XCD-aware block remap.
#pragma once
#include "common.h"

namespace dc {

constexpr int BK = 64;

__device__ __forceinline__ int swz(int r) { return (r >> 1) & 7; }

// fragment of a k-contiguous image, standard k order
__device__ __forceinline__ bf16x8 frag_k(const char* lds, int r, int s, int g) {
  const int chunk = 4 * s + g;
  return *reinterpret_cast<const bf16x8*>(lds + r * 128 + 16 * (chunk ^ swz(r)));
}
// fragment of a k-contiguous image, permuted k order
__device__ __forceinline__ bf16x8 frag_k_perm(const char* lds, int r, int s, int g) {
  const int ca = 4 * s + (g >> 1), cb = ca + 2;
  const int sub = 8 * (g & 1);
  const u32x2 lo = *reinterpret_cast<const u32x2*>(lds + r * 128 + 16 * (ca ^ swz(r)) + sub);
  const u32x2 hi = *reinterpret_cast<const u32x2*>(lds + r * 128 + 16 * (cb ^ swz(r)) + sub);
  u32x4 v = {lo[0], lo[1], hi[0], hi[1]};
  return __builtin_bit_cast(bf16x8, v);
}
// wait until at most N vector-memory ops are outstanding (clamped to the
// 6-bit vmcnt field: waiting for fewer is still correct, just stricter)
template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N < 63 ? N : 63) : "memory");
}
template <int LPT>
__device__ __forceinline__ void vm_wait_rem(int rem) {
  switch (rem) {
    case 0: vm_wait<0>(); break;
    case 1: vm_wait<LPT>(); break;
    case 2: vm_wait<2 * LPT>(); break;
    case 3: vm_wait<3 * LPT>(); break;
    case 4: vm_wait<4 * LPT>(); break;
    case 5: vm_wait<5 * LPT>(); break;
    default: vm_wait<6 * LPT>(); break;
  }
}
__device__ __forceinline__ void raw_barrier() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Transposed-image fragment reads for the LDS-DMA GEMMs.  ds_read_b64_tr_b16 is
// issued from inline asm: through the builtin, hipcc (ROCm 7.2) treats the read
// as aliasing every in-flight LDS-DMA and emits s_waitcnt vmcnt(0) before it,
// draining the whole ring each k-step (found in the .s of every transposed-
// operand GEMM).  The asm read is invisible to the compiler's counters, so the
// caller waits explicitly: issue the reads (frag_t_swz_issue), then
// frag_t_fence() on every fragment before its first use.
struct TrFrag {
  bf16x4 lo, hi;
};
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const DC_LDS char*)(p);
}
__device__ __forceinline__ TrFrag frag_t_swz_issue(const char* lds, int c0, int s, int lane) {
  const int i = lane & 15, g = lane >> 4, q = i >> 2, p = i & 3;
  const int ra = 32 * s + 4 * g + q;
  const int chunk = (c0 >> 3) + (p >> 1);
  const int off = ra * 128 + 16 * (chunk ^ (ra & 6)) + 8 * (p & 1);
  TrFrag f;
  const uint32_t a = lds_addr(lds + off);
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(f.lo) : "v"(a));
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:2048" : "=v"(f.hi) : "v"(a));
  return f;
}
// wait for every outstanding LDS read, tied to the fragment so no use of it can
// be scheduled above the wait
__device__ __forceinline__ bf16x8 frag_t_fence(TrFrag& f) {
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(f.lo), "+v"(f.hi));
  bf16x8 v;
  v[0] = f.lo[0]; v[1] = f.lo[1]; v[2] = f.lo[2]; v[3] = f.lo[3];
  v[4] = f.hi[0]; v[5] = f.hi[1]; v[6] = f.hi[2]; v[7] = f.hi[3];
  return v;
}
// counted variant: wait until at most N LDS reads are outstanding (the N issued
// after this fragment's)
template <int N>
__device__ __forceinline__ bf16x8 frag_t_fence_n(TrFrag& f) {
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(f.lo), "+v"(f.hi) : "n"(N));
  bf16x8 v;
  v[0] = f.lo[0]; v[1] = f.lo[1]; v[2] = f.lo[2]; v[3] = f.lo[3];
  v[4] = f.hi[0]; v[5] = f.hi[1]; v[6] = f.hi[2]; v[7] = f.hi[3];
  return v;
}
__device__ __forceinline__ bf16x8 frag_t_swz(const char* lds, int c0, int s, int lane) {
  TrFrag f = frag_t_swz_issue(lds, c0, s, lane);
  return frag_t_fence(f);
}

// NW: waves of the workgroup (4 or 8); each wave issues PER_WAVE 1-KiB pieces per K tile
template <int R, bool T, int NW = 4>
struct DmaOperand {
  static constexpr int BYTES = R * 128;                // one 64-deep K tile
  static constexpr int PER_WAVE = BYTES / (1024 * NW);  // 1-KiB pieces per wave
  static_assert(PER_WAVE >= 1 && PER_WAVE * 1024 * NW == BYTES, "operand tile must split into whole pieces per wave");
  bf16* base;
  int nbytes;
  int voff[PER_WAVE];  // per-lane byte offset of piece j at k-tile 0
  int kstep;           // byte advance per K tile

  __device__ __forceinline__ void init(const bf16* base, int ld, int rows_total_bytes_rows, int row0, int wave,
                                       int lane) {
    // rows_total_bytes_rows: number of rows of the stored matrix (for the OOB range)
    this->base = const_cast<bf16*>(base);
    nbytes = rows_total_bytes_rows * ld * 2;
#pragma unroll
    for (int j = 0; j < PER_WAVE; ++j) {
      const int piece = wave * PER_WAVE + j;
      const int r = piece * 8 + (lane >> 3), pc = lane & 7;
      if (!T) {
        const int lc = pc ^ ((r >> 1) & 7);
        voff[j] = ((row0 + r) * ld + 8 * lc) * 2;
      } else {
        const int lc = pc ^ (r & 6);
        voff[j] = (r * ld + row0 + 8 * lc) * 2;
      }
    }
    kstep = T ? 64 * ld * 2 : 64 * 2;
  }
  __device__ __forceinline__ void issue(char* lds_tile, int kt, int wave) const {
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, nbytes, 0x00020000);
#pragma unroll
    for (int j = 0; j < PER_WAVE; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsrc, (DC_LDS void*)(lds_tile + (wave * PER_WAVE + j) * 1024), 16, voff[j] + kt * kstep, 0, 0, 0);
  }
};

// A transposed operand 128 columns wide is staged as TWO 64-column half images
// (the transposed-read swizzle and the DMA piece map assume 128-B image rows).
template <int NW = 4>
struct DmaOperandT128 {
  static constexpr int BYTES = 2 * 64 * 128;  // one 64-deep K tile, both halves
  static constexpr int PER_WAVE = 2 * DmaOperand<64, true, NW>::PER_WAVE;
  DmaOperand<64, true, NW> h0, h1;
  __device__ __forceinline__ void init(const bf16* base, int ld, int rows_total, int row0, int wave, int lane) {
    h0.init(base, ld, rows_total, row0, wave, lane);
    h1.init(base, ld, rows_total, row0 + 64, wave, lane);
  }
  __device__ __forceinline__ void issue(char* lds_tile, int kt, int wave) const {
    h0.issue(lds_tile, kt, wave);
    h1.issue(lds_tile + 64 * 128, kt, wave);
  }
};
template <int R, bool T, int NW = 4>
struct DmaOp {
  using type = DmaOperand<R, T, NW>;
};
template <int NW>
struct DmaOp<128, true, NW> {
  using type = DmaOperandT128<NW>;
};
// transposed fragment (operand columns c0..c0+15) of a [64 k][64]-per-half image
__device__ __forceinline__ TrFrag frag_t_half(const char* lds, int c0, int s, int lane) {
  return frag_t_swz_issue(lds + (c0 >> 6) * (64 * 128), c0 & 63, s, lane);
}

// bijective XCD-aware remap: consecutive block ids land on different XCDs
// (round robin); give each XCD a contiguous range of tiles instead
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7, idx = bid >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

}  // namespace dc
