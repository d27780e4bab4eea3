// Host-side launch API of the ddim_cold_amd HIP kernels (no torch headers here,
// so the .hip translation units compile fast; bindings.cpp adapts tensors).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdexcept>

enum GemmEpi : int {
  EPI_BF16 = 0,    // C bf16 = acc (+bias)
  EPI_F32 = 1,     // C f32 = acc (+bias)
  EPI_QKV = 2,     // +bias, scatter to head-major [3,B,H,N,hd] bf16
  EPI_RESID = 3,   // C f32 = res + DropPath(Dropout(acc+bias))
  EPI_GELU = 4,    // C = u = acc+bias (bf16) ; C2 = h = Dropout(GELU(u)) (bf16)
  EPI_HEAD = 5,    // +bias, unpatchify token rows into a [B,C,H,W] f32 image
  EPI_EMBED = 6,   // patch rows -> token rows: +bias +pos +temb[t], Dropout, f32
  EPI_DGELU = 7,   // C bf16 = Dropout(acc) * GELU'(aux)
  EPI_ATOMIC = 8,  // C f32 += acc (split-K / gradient accumulate) ; bias -> fused column sum
  EPI_ACC = 9,     // C f32 += acc, one writer per element (no split) ; bias likewise
  EPI_HEADR = 10,  // sampler step on patch rows: +bias, clamp (+DDIM update), f32 [B*P][C*p*p]
                   //   in head-output column order (contiguous: vector epilogue)
  EPI_HEADL = 11,  // training loss on patch rows: smooth-L1 vs a [B*P][C*p*p] target (head order),
                   //   token-layout bf16 gradient, one loss partial per workgroup
};

struct GemmArgs {
  const void* A = nullptr;
  const void* B = nullptr;
  int M = 0, N = 0, K = 0, lda = 0, ldb = 0;
  void* C = nullptr;
  int ldc = 0;
  const float* bias = nullptr;
  const float* res = nullptr;
  void* C2 = nullptr;
  const void* aux = nullptr;
  const int64_t* rng = nullptr;
  int site_drop = 0;
  double p_drop = 0.0;
  int site_dp = 0;
  double p_dp = 0.0;
  int tokens = 1, batch = 1, heads = 1, hd = 1;
  int chans = 1, img_h = 1, img_w = 1, patch = 1;
  const float* pos = nullptr;
  const float* temb = nullptr;
  const int64_t* tsteps = nullptr;
  int emb_dim = 0;
  const float* coef = nullptr;  // EPI_HEAD head_mode 1
  int head_mode = 0;            // EPI_HEAD: 0 image, 1 fused DDIM step, 2 clamp, 3 smooth-L1 loss + grad
  float loss_beta = 1.f;        // EPI_HEAD mode 3
  float loss_inv_n = 1.f;
  float* loss_parts = nullptr;  // EPI_HEAD mode 3: one partial per workgroup (gemm_nt_grid entries)
  // EPI_F32 dgrad split over K: slice z of `splits` writes its partial product to
  // C + z * split_stride (no atomics, no zeroing; the consumer sums the slices)
  int splits = 1;
  long long split_stride = 0;
  // LayerNorm folded into the GEMM (see gemm.hip "LayerNorm fold"):
  // consumer (QKV / GELU / HEAD / BF16 / F32): A = bf16(x), B = bf16(gamma o W),
  //   bias = b + W beta, y = rstd*(acc - mean*ln_c) + bias with (mean, rstd)
  //   from the row statistics ln_st[m][K/32] = {sum x, sum x^2} per 32-column
  //   slot; optional mean/rstd out
  const float* ln_st = nullptr;
  const float* ln_c = nullptr;
  float ln_eps = 1e-5f;
  float* ln_mean = nullptr;
  float* ln_rstd = nullptr;
  // producer (RESID / EMBED): write {sum, sum^2} of every output row's 32-column
  // slots into st_out[row][N/32] (each slot written once: deterministic, no
  // zeroing) and a bf16 copy of the output to xb_out
  float* st_out = nullptr;
  void* xb_out = nullptr;
  // sampler steps (GemmParams::patch_out / cls_src): HEAD modes 1/2 also write the new
  // image as bf16 patch rows; EMBED writes the cls rows itself (no patchify launch)
  void* patch_out = nullptr;
  const float* cls_src = nullptr;
};

void gemm_nt(const GemmArgs& a, int epi, hipStream_t stream);
// workgroups gemm_nt launches for an [M x N x K] problem (one split)
int gemm_nt_grid(int M, int N, int K);
// force a GEMM tile config for every later launch (-1 = automatic choice; 0..5, see
// gemm.hip "tile configs"); returns the previous setting.  Tests / micro-benchmarks.
int gemm_set_tile_override(int cfg);
// phase stamps of every later LDS-DMA GEMM launch (GEMM_STAMP_WORDS words per
// workgroup, gemm_epi.h) into buf; nullptr turns them off.  Returns the previous buffer.
uint32_t* gemm_set_stamps(uint32_t* buf);
void gemm_dgrad(const GemmArgs& a, int epi, hipStream_t stream);
void gemm_wgrad(const GemmArgs& a, int splits, hipStream_t stream);
// every weight gradient of a step (n <= 32 problems) in one launch, unsplit (plain read-add-write)
// store: every target is zero on entry (plain stores instead of read-add-write)
// Grad-norm partials fused into the weight-gradient launch (single process: it is the
// last writer of the gradient arena): every output tile writes the sum of squares of
// its final dW (+ db) values to parts[tile]; `tail` extra workgroups sum the squares
// of the arena ranges [lo, hi) no weight-gradient tile writes (embeddings, LayerNorms:
// final before this launch) into parts[tiles + j], and zero parts[tiles + tail ..
// nparts).  The optimizer then reads the same partial layout sqnorm writes.
constexpr int WSQ_MAX_RANGES = 16;
constexpr int WGRAD_MULTI_MAX = 32;  // problems per gemm_wgrad_multi launch (kernel-argument block)
struct WgradSq {
  float* parts = nullptr;
  int nparts = 0;
  const float* base = nullptr;
  int nr = 0, tail = 0;
  int64_t lo[WSQ_MAX_RANGES], hi[WSQ_MAX_RANGES];
};
// returns the output tiles launched (grad-norm partial slots used before the tail);
// sq->tail = 0: no tail workgroups, no zero fill (all but the last launch of a step).
// emb (optional): the embedding gradients and the LayerNorm slot finalize ride in the
// launch as extra workgroups (embed_parts.h), each writing the grad-norm partial of its
// outputs after the tail's slots.
struct WgradEmbed;  // below
// split_ws / split_cnt: workspace of wgrad_split_ws_floats(tiles, T) floats and zeroed
// tickets -- the tail tiles past the last whole round of workgroup slots (256 CUs x 1
// wide or x 3 64 x 64 workgroups) run as wgrad_split_factor(tiles, T) K pieces each,
// summed in piece order (deterministic)
constexpr int WGRAD_MAX_SPLIT = 6;
int wgrad_split_factor(int tiles, int T);
int wgrad_multi_tile(int kmax);  // output tile edge gemm_wgrad_multi uses for reductions over kmax tokens
int64_t wgrad_split_ws_floats(int tiles, int T);
int gemm_wgrad_multi(const GemmArgs* probs, int n, hipStream_t stream, bool store = false,
                     const WgradSq* sq = nullptr, const WgradEmbed* emb = nullptr, float* split_ws = nullptr,
                     int* split_cnt = nullptr);
int wgrad_embed_workgroups(const WgradEmbed& emb, bool wide);  // extra workgroups (= grad-norm slots) emb takes

// LayerNorm (layernorm.hip)
void layernorm_fwd_launch(const float* x, const float* gamma, const float* beta, void* y_bf16, float* mean,
                          float* rstd, int M, int D, float eps, hipStream_t stream);
// dgamma||dbeta: workgroup w of the backward (ln_bwd_workgroups(M) of them) stores its
// column partial in row w of slots [ln_bwd_workgroups(M)][2D] (plain stores, no
// atomics); replica_reduce_launch (or the embedding backward / weight-gradient
// launch) sums the rows in row order: deterministic.  gp_bf16 (optional): the
// patch-embedding input gradient (g_out rows 1..N-1 per sample, embedding dropout
// p_emb at site_emb, bf16, patch-row order).
void layernorm_bwd_launch(const void* dy, bool dy_bf16, const void* x, bool x_bf16, const float* mean, const float* rstd,
                          const float* gamma, const float* beta, const float* g_res, float* g_out, void* gy_bf16,
                          void* y_bf16, float* slots, int M,
                          int D, int tokens, const int64_t* rng, int site_drop, double p_drop, int site_dp,
                          double p_dp, int dy_parts, void* gp_bf16, int site_emb, double p_emb, hipStream_t stream);
int ln_bwd_workgroups(int M);

// dst[i] = src[i]^T for bf16 matrices [R][C] (transpose.hip; R, C multiples of 8)
constexpr int TRANSPOSE_MAX = 96;
void transpose_bf16_launch(const void* const* srcs, void* const* dsts, const int* R, const int* C, int n,
                           hipStream_t stream);

// LayerNorm fold weights for the GEMMs that consume a LayerNorm (layernorm.hip)
constexpr int FOLD_MAX = 32;  // GEMMs per fold launch (vit_small_200: 25 in one launch)
struct FoldJob {
  const void* w;       // [rows][K] weight: fp32 master, or its bf16 shadow (FoldTable::w_bf16)
  const float* gamma;  // [K]
  const float* beta;   // [K]
  const float* bias;   // [rows] or null
  void* wf;            // [rows][K] bf16 out: gamma o W
  float* c;            // [rows] out: row sums of wf
  float* bf;           // [rows] out: bias + W beta
};
struct FoldTable {
  FoldJob j[FOLD_MAX];
  int start[FOLD_MAX + 1];
  int n;
  int K;
  int w_bf16 = 0;  // weights given as bf16 (the optimizer's shadow copy: half the bytes)
  // optional training-step tail run by one extra workgroup of the same launch
  // (the fold runs right after the optimizer): finish the smooth-L1 loss from its
  // per-block partials (loss_last, EMA) and advance the step / RNG counters
  int tail = 0;
  const float* loss_parts = nullptr;
  int loss_nparts = 0;
  float* loss_last = nullptr;
  float* loss_ema = nullptr;
  float ema_decay = 0.99f;
  int64_t* step = nullptr;
  int64_t* rng = nullptr;
  const float* sq = nullptr;  // sq_n grad-norm partials (non-finite -> optimizer step skipped)
  int sq_n = 0;
};
void ln_fold_launch(const FoldTable& tb, hipStream_t stream);
// ws [G][rows][C]: sums rows 0..R-1 of each workspace
void replica_reduce_launch(const float* ws, float* const* dsts_dev, int G, int C, int R, int rows, hipStream_t stream);

// Attention (attention.hip)
// keep_bits: optional [attn_keep_words] attention-dropout keep flags, written by
// the short-sequence forward and read by its backward instead of re-hashing
// (ignored by the long-sequence kernels, which always regenerate)
int64_t attn_keep_words(int B, int H, int N, int hd);
void attn_fwd_launch(const void* qkv, void* o, float* lse, int B, int H, int N, int hd, float scale,
                     const int64_t* rng, int site, double p, hipStream_t stream, uint32_t* keep_bits = nullptr);
void attn_bwd_launch(const void* dout, const void* qkv, const void* o, const float* lse, void* dqkv,
                     float* delta, int B, int H, int N, int hd, float scale, const int64_t* rng, int site,
                     double p, hipStream_t stream, const uint32_t* keep_bits = nullptr);

// Embedding / head / loss (embed.hip)
// Optional cold-diffusion batch source fused into patchify (pool != nullptr): the
// patch rows are pixelated straight from the pool (cold_batch_kernel's draw), the
// target image and (t, pool index) are written by the same launch; `img` is unused.
struct ColdSrc {
  const float* pool = nullptr;
  int pool_n = 0, site = 0, max_t = 1;
  bool draw_idx = true, target_x0 = false;
  int64_t* idx = nullptr;    // [B] pool indices (written if draw_idx, else read)
  int64_t* t_out = nullptr;  // [B] t (== the `t` the GEMM epilogue reads)
  float* target = nullptr;   // [B,C,H,W] x_{t-1} (or x0)
  float* x_t = nullptr;      // optional [B,C,H,W] x_t image
  // gauss_T > 0: Gaussian DDIM batch instead (t in 0..T-1, x_t = q_sample(x0, t, eps),
  // eps drawn at noise_site, target = x0)
  int gauss_T = 0, noise_site = 0;
  // target written as patch rows [B*P][C*p*p] in the head's output column order
  // ((a*p + b)*C + c), for the vector loss epilogue (EPI_HEADL)
  bool target_rows = false;
  // stepped index table (!draw_idx): the batch reads idx + (idx_ctr[0] % idx_rows) *
  // idx_stride, i.e. row <device step counter> of an epoch's [steps][micro][B]
  // DistributedSampler table -- K-step graphs replay with no host copy per step
  const int64_t* idx_ctr = nullptr;
  int idx_rows = 1, idx_stride = 0;
};
// Gaussian DDIM batch on device in one launch (pool draw, noise, q_sample)
void gauss_batch_launch(const float* pool, int pool_n, const int64_t* rng, int site, int noise_site, int T,
                        float* x_t, float* x0, int64_t* t, int64_t* idx, bool draw_idx, int B, int C, int H, int W,
                        hipStream_t stream, const int64_t* idx_ctr = nullptr, int idx_rows = 1, int idx_stride = 0);
void patchify_cls_launch(const float* img, const int64_t* t, const float* cls, const float* pos,
                         const float* temb, void* patches, float* x, int B, int C, int H, int W, int patch,
                         int D, const int64_t* rng, int site, double p, float* st, void* xb, hipStream_t stream,
                         ColdSrc cs = ColdSrc());
// optional LayerNorm replica finalize carried by the embedding-backward launch
struct ReplicaFinal {
  const float* ws = nullptr;    // [G][rows][C] LayerNorm workspaces: rows 0..R-1 summed in order
  float* const* dsts = nullptr; // [G] device pointers to the [C] grad ranges (+=, or = with store)
  int G = 0, R = 0, C = 0, rows = 0;
  int store = 0;
};
// Embedding-gradient reductions (embed_parts.h): the argument block
struct EmbedGrad {
  const float* g = nullptr;      // [B][N][D] gradient of the embedding output (the last LayerNorm's g_out)
  const int64_t* t = nullptr;    // [B] timesteps
  float* dcls = nullptr;         // [D]
  float* dpos = nullptr;         // [N][D]
  float* dtemb = nullptr;        // [T][D]
  int B = 0, N = 0, D = 0;
  const int64_t* rng = nullptr;  // {seed, step}: the dropout salt is derived on the device
  int site = 0;
  uint32_t thr = 0;              // embedding dropout (pos_drop)
  float dsc = 1.f;
  int pb0 = 0, pbn = 0;          // part-B sample pass
  int owners = 0;                // part-B timestep slots launched (<= distinct timesteps possible)
};
// the embedding parts as extra workgroups of the weight-gradient launch (gemm.hip)
struct WgradEmbed {
  EmbedGrad e;
  ReplicaFinal rf;
};
EmbedGrad embed_grad_args(const float* g, const int64_t* t, float* dcls, float* dpos, float* dtemb, int B, int N,
                          int D, const int64_t* rng, int site, double p, int pb0, int pbn);
void embed_bwd_launch(const float* g, const int64_t* t, float* dcls, float* dpos, float* dtemb, void* gpatch,
                      int B, int N, int D, const int64_t* rng, int site, double p, hipStream_t stream, ReplicaFinal rf = ReplicaFinal());
// returns the number of per-block loss partials written; finish = false leaves
// summing them (loss, loss_last, EMA) to a later kernel (the step tail of ln_fold)
int smooth_l1_launch(const float* pred, const float* target, float* loss, float* partials, void* dtok, int B,
                     int C, int H, int W, int patch, float beta, float* loss_last, float* loss_ema, float ema_decay,
                     bool finish, hipStream_t stream);
constexpr int L1_PARTS = 512;
void img_to_tokgrad_launch(const float* dimg, void* dtok, int B, int C, int H, int W, int patch,
                           hipStream_t stream);

// Optimizer (optim.hip)
// sqnorm writes `nparts` (>= SQ_PARTS, a multiple of 256) per-block partial sums of
// (g*scale)^2 (no atomics); adamw / advance / the fold tail sum the partials
// themselves.  The single-process step instead has the weight-gradient launch write
// them (gemm_wgrad_multi with WgradSq).
constexpr int SQ_PARTS = 1024;
void sqnorm_launch(const float* g, int64_t n, float* partials, int nparts, float scale, hipStream_t stream,
                   int64_t lz_lo = 0, int64_t lz_hi = 0);
// zero_hi: zero the gradient arena only below this element (the part that is
// accumulated into; everything above is overwritten by its producer next step)
void adamw_launch(float* p, float* g, float* m, float* v, void* p_bf16, int64_t n, const float* sqnorm,
                  int nparts, const int64_t* step, const float* hyper, float grad_scale, hipStream_t stream,
                  int64_t zero_hi = -1, int64_t lz_lo = 0, int64_t lz_hi = 0, float* lazy_decay = nullptr);
void advance_counters_launch(int64_t* step, int64_t* rng, const float* sqnorm, int nparts, hipStream_t stream);

// Diffusion / data (diffusion.hip)
void ddim_step_launch(const float* x_t, const float* x0_raw, float* x_next, float* x0_out, const float* coef,
                      int64_t n, hipStream_t stream);
void pixelate_pair_launch(const float* img, const int64_t* idx, const int64_t* t, float* x_t, float* x_tm1,
                          int B, int C, int H, int W, hipStream_t stream);
void randn_launch(float* out, int64_t n, const int64_t* rng, int site, hipStream_t stream);
void q_sample_launch(const float* x0, const int64_t* t, const float* eps, float* out, int B, int64_t per,
                     int total_steps, hipStream_t stream);
void cold_batch_launch(const float* pool, int pool_n, const int64_t* rng, int site, float* x_t, float* x_tm1,
                       int64_t* t, int64_t* idx_ws, int B, int C, int H, int W, int max_t, bool draw_idx,
                       hipStream_t stream, const int64_t* idx_ctr = nullptr, int idx_rows = 1, int idx_stride = 0);

// gradient wire format (comm_wire.hip): fp32 <-> bf16 (RNE), 16-B aligned buffers
void wire_pack_launch(const float* src, void* dst, int64_t n, hipStream_t stream);
void wire_unpack_launch(const void* src, float* dst, int64_t n, hipStream_t stream);
void flag_bump_launch(void* flags, int k, hipStream_t stream);  // flags[k] += 1, system-scope release
void flag_wait_launch(const void* flags, int k, unsigned int expected, void* err, hipStream_t stream,
                      int64_t timeout_us = 0);  // 0: 2 s
// in-process loopback all-reduce of two endpoints on one device (testing the
// cross-engine hand-off): flags = pair_allreduce_flags() zeroed uint32, stage = 2 x stage_n
int pair_allreduce_flags();
void pair_allreduce_launch(float* buf, int64_t n, float* stage, int64_t stage_n, void* flags, int e, void* err,
                           int64_t timeout_us, hipStream_t stream);
