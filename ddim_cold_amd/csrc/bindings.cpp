// TORCH_LIBRARY registrations for the ddim_cold_amd HIP kernels.
//
// Every op validates shapes / dtypes / contiguity / device on the host before
// launching (a mis-shaped launch of a hand-written kernel can fault the GPU),
// allocates its outputs through the PyTorch caching allocator (graph-capture
// safe) and launches on the current HIP stream.  Op contracts are documented
// (and implemented in plain PyTorch) in ddim_cold_amd/ops/reference.py.
#include <torch/library.h>
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <c10/core/DeviceGuard.h>

#include "kernels.h"
#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>

using at::Tensor;

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

#define CHECK_CUDA(x) TORCH_CHECK((x).is_cuda(), #x " must be a GPU tensor")
#define CHECK_CONTIG(x) TORCH_CHECK((x).is_contiguous(), #x " must be contiguous")
#define CHECK_DT(x, dt) TORCH_CHECK((x).scalar_type() == (dt), #x " must be " #dt ", got ", (x).scalar_type())
#define CHECK_IN(x, dt) \
  CHECK_CUDA(x);        \
  CHECK_CONTIG(x);      \
  CHECK_DT(x, dt)

constexpr auto F32 = at::kFloat;
constexpr auto BF16 = at::kBFloat16;
constexpr auto I64 = at::kLong;

void check_rng(const Tensor& rng) {
  CHECK_IN(rng, I64);
  TORCH_CHECK(rng.numel() >= 2, "rng must hold {seed, step}");
}

void check_linear(const Tensor& a, const Tensor& w, int64_t K) {
  TORCH_CHECK(a.dim() == 2 && w.dim() == 2, "linear operands must be 2-D");
  TORCH_CHECK(a.size(1) == K && w.size(1) == K, "linear K mismatch");
  TORCH_CHECK(K % 8 == 0, "K must be a multiple of 8 (16-B vector loads)");
}

GemmArgs nt_args(const Tensor& a, const Tensor& w) {
  GemmArgs g;
  g.A = a.data_ptr();
  g.B = w.data_ptr();
  g.M = (int)a.size(0);
  g.N = (int)w.size(0);
  g.K = (int)a.size(1);
  g.lda = g.K;
  g.ldb = g.K;
  return g;
}

bool ln_fold_width_ok(int64_t D) { return D % 32 == 0 && D / 32 <= 16; }

// LayerNorm fold, consumer side (gemm.hip): A = bf16(x), w = bf16(gamma o W),
// b = bias + W beta; ln_st [M][2] row {sum, sum^2} of x; ln_c [N] row sums of w
void apply_fold(GemmArgs& g, int M, int N, const c10::optional<Tensor>& ln_st, const c10::optional<Tensor>& ln_c,
                double eps, const c10::optional<Tensor>& ln_mean, const c10::optional<Tensor>& ln_rstd) {
  if (!ln_st.has_value() || !ln_st->defined()) return;
  CHECK_IN((*ln_st), F32);
  TORCH_CHECK(ln_c.has_value() && ln_c->defined(), "LayerNorm fold needs ln_c");
  CHECK_IN((*ln_c), F32);
  TORCH_CHECK(ln_fold_width_ok(g.K), "LayerNorm fold: width must be a multiple of 32, <= 512");
  TORCH_CHECK(ln_st->numel() == 2 * (int64_t)M * (g.K / 32) && ln_c->numel() == N, "LayerNorm fold shapes");
  g.ln_st = ln_st->data_ptr<float>();
  g.ln_c = ln_c->data_ptr<float>();
  g.ln_eps = (float)eps;
  if (ln_mean.has_value() && ln_mean->defined()) {
    TORCH_CHECK(ln_rstd.has_value() && ln_rstd->defined(), "ln_mean needs ln_rstd");
    CHECK_IN((*ln_mean), F32); CHECK_IN((*ln_rstd), F32);
    TORCH_CHECK(ln_mean->numel() == M && ln_rstd->numel() == M, "ln_mean / ln_rstd shapes");
    g.ln_mean = ln_mean->data_ptr<float>();
    g.ln_rstd = ln_rstd->data_ptr<float>();
  }
}

// LayerNorm fold, producer side: row statistics (accumulated, zeroed beforehand) + bf16 copy
void apply_prod(GemmArgs& g, int64_t rows, int64_t D, const c10::optional<Tensor>& st_out,
                const c10::optional<Tensor>& xb_out) {
  if (!st_out.has_value() || !st_out->defined()) return;
  CHECK_IN((*st_out), F32);
  TORCH_CHECK(xb_out.has_value() && xb_out->defined(), "row statistics need the bf16 copy output");
  CHECK_IN((*xb_out), BF16);
  TORCH_CHECK(ln_fold_width_ok(D), "LayerNorm fold: width must be a multiple of 32, <= 512");
  TORCH_CHECK(st_out->numel() == 2 * rows * (D / 32) && xb_out->numel() == rows * D, "LayerNorm-fold producer shapes");
  g.st_out = st_out->data_ptr<float>();
  g.xb_out = xb_out->data_ptr();
}

// ln_st: [B*N][D/32][2] row statistics of the tokens (the first LayerNorm's
// input; LayerNorm fold), filled together with the tokens' bf16 copy xb_out.
static std::tuple<Tensor, Tensor> patch_embed_impl(Tensor img, Tensor t, Tensor w_pe, Tensor b_pe, Tensor cls,
                                                   Tensor pos, Tensor temb, Tensor rng, int64_t site, double p,
                                                   int64_t patch, c10::optional<Tensor> ln_st,
                                                   c10::optional<Tensor> xb_out, ColdSrc cs,
                                                   c10::optional<Tensor> patches_in = c10::nullopt) {
  CHECK_IN(img, F32); CHECK_IN(t, I64); CHECK_IN(w_pe, BF16); CHECK_IN(b_pe, F32);
  CHECK_IN(cls, F32); CHECK_IN(pos, F32); CHECK_IN(temb, F32); check_rng(rng);
  const c10::DeviceGuard guard(img.device());
  TORCH_CHECK(img.dim() == 4, "img must be [B,C,H,W]");
  const int B = img.size(0), C = img.size(1), H = img.size(2), W = img.size(3), P = patch;
  TORCH_CHECK(H % P == 0 && W % P == 0, "image size must be divisible by patch");
  const int D = w_pe.size(0), F = C * P * P;
  TORCH_CHECK(w_pe.numel() == (int64_t)D * F, "patch-embed weight shape mismatch");
  TORCH_CHECK(F % 8 == 0, "C*p*p must be a multiple of 8");
  const int NP = (H / P) * (W / P), N = NP + 1;
  TORCH_CHECK(pos.numel() == (int64_t)N * D && cls.numel() == D && b_pe.numel() == D, "embedding shapes");
  TORCH_CHECK(temb.dim() == 2 && temb.size(1) == D, "time embedding shape");
  TORCH_CHECK(t.numel() == B, "t must be [B]");
  auto x = at::empty({B, N, D}, img.options());
  // patches_in: the patch rows are already there (a sampler step's head wrote them);
  // the GEMM epilogue then writes the cls rows and no patchify launch is needed
  const bool have_patches = patches_in.has_value() && patches_in->defined();
  if (have_patches) {
    CHECK_IN((*patches_in), BF16);
    TORCH_CHECK(patches_in->numel() == (int64_t)B * NP * F, "patches_in must be [B*P, C*p*p]");
    TORCH_CHECK(!cs.pool, "patches_in excludes the fused cold batch draw");
  }
  auto patches = have_patches ? *patches_in : at::empty({(int64_t)B * NP, F}, img.options().dtype(BF16));
  float* st = nullptr;
  void* xb = nullptr;
  if (ln_st.has_value() && ln_st->defined()) {
    CHECK_IN((*ln_st), F32);
    TORCH_CHECK(ln_fold_width_ok(D), "LayerNorm fold: width must be a multiple of 32, <= 512");
    TORCH_CHECK(ln_st->numel() == (int64_t)B * N * (D / 32) * 2, "ln_st must be [B*N, D/32, 2]");
    TORCH_CHECK(xb_out.has_value() && xb_out->defined(), "ln_st needs xb_out");
    CHECK_IN((*xb_out), BF16);
    TORCH_CHECK(xb_out->numel() == (int64_t)B * N * D, "xb_out shape");
    st = ln_st->data_ptr<float>();
    xb = xb_out->data_ptr();
  }
  if (!have_patches)
    patchify_cls_launch(img.data_ptr<float>(), t.data_ptr<int64_t>(), cls.data_ptr<float>(), pos.data_ptr<float>(),
                        temb.data_ptr<float>(), patches.data_ptr(), x.data_ptr<float>(), B, C, H, W, P, D,
                        rng.data_ptr<int64_t>(), site, p, st, xb, cur_stream(), cs);
  GemmArgs g;
  g.A = patches.data_ptr();
  g.B = w_pe.data_ptr();
  g.M = B * NP; g.N = D; g.K = F; g.lda = F; g.ldb = F;
  g.C = x.data_ptr(); g.ldc = D;
  g.bias = b_pe.data_ptr<float>();
  g.rng = rng.data_ptr<int64_t>(); g.site_drop = site; g.p_drop = p;
  g.tokens = NP; g.batch = B;
  g.pos = pos.data_ptr<float>(); g.temb = temb.data_ptr<float>(); g.tsteps = t.data_ptr<int64_t>(); g.emb_dim = D;
  g.st_out = st;  // slice 0, indexed by token row
  g.xb_out = xb;
  if (have_patches) g.cls_src = cls.data_ptr<float>();
  gemm_nt(g, EPI_EMBED, cur_stream());
  return {x, patches};
}

std::tuple<Tensor, Tensor> patch_embed_fwd(Tensor img, Tensor t, Tensor w_pe, Tensor b_pe, Tensor cls, Tensor pos,
                                           Tensor temb, Tensor rng, int64_t site, double p, int64_t patch,
                                           c10::optional<Tensor> ln_st, c10::optional<Tensor> xb_out,
                                           c10::optional<Tensor> patches_in) {
  return patch_embed_impl(img, t, w_pe, b_pe, cls, pos, temb, rng, site, p, patch, ln_st, xb_out, ColdSrc(),
                          patches_in);
}

// Pool indices of a batch source that reads them (!draw_idx): a [B] vector, or with
// `ctr` a stepped table [rows][...] read at row ctr[0] % rows, elements off..off+B
// (the trainer's epoch DistributedSampler table indexed by the device step counter).
struct IdxSel {
  int64_t* p;
  const int64_t* ctr;
  int rows, stride;
};
static IdxSel idx_select(const Tensor& idx, const c10::optional<Tensor>& ctr, int64_t off, int B, bool draw_idx,
                         const char* what) {
  if (ctr.has_value() && ctr->defined()) {
    CHECK_IN((*ctr), I64);
    TORCH_CHECK(ctr->device() == idx.device() && ctr->numel() >= 1, what, ": step counter");
    TORCH_CHECK(!draw_idx, what, ": a stepped index table is read, not drawn");
    TORCH_CHECK(idx.dim() >= 2 && idx.size(0) >= 1, what, ": a stepped index table is [rows, ...]");
    const int64_t rows = idx.size(0), stride = idx.numel() / rows;
    TORCH_CHECK(off >= 0 && off + B <= stride && idx.numel() < ((int64_t)1 << 31), what,
                ": batch offset outside the table row");
    return {idx.data_ptr<int64_t>() + off, ctr->data_ptr<int64_t>(), (int)rows, (int)stride};
  }
  TORCH_CHECK(idx.numel() == B && off == 0, what, ": idx shape");
  return {idx.data_ptr<int64_t>(), nullptr, 1, 0};
}

// patch_embed_fwd with the cold-diffusion batch draw fused into the patchify launch
// (cold_batch + patch_embed_fwd in one launch fewer): `img` is the x_t buffer (its
// shape drives the launch; written only if write_xt), `target`, `t` and `idx` are outputs
// (idx is an input when !draw_idx).  Same values as ops.cold_batch followed by
// patch_embed_fwd on its x_t.
std::tuple<Tensor, Tensor> patch_embed_cold_fwd(Tensor pool, int64_t data_site, int64_t max_t, bool draw_idx,
                                                bool target_x0, Tensor img, Tensor target, Tensor t, Tensor idx,
                                                bool write_xt, Tensor w_pe, Tensor b_pe, Tensor cls, Tensor pos,
                                                Tensor temb, Tensor rng, int64_t site, double p, int64_t patch,
                                                c10::optional<Tensor> ln_st, c10::optional<Tensor> xb_out,
                                                int64_t gauss_T, int64_t noise_site, bool target_rows,
                                                c10::optional<Tensor> idx_ctr, int64_t idx_off) {
  CHECK_IN(pool, F32); CHECK_IN(img, F32); CHECK_IN(target, F32); CHECK_IN(t, I64); CHECK_IN(idx, I64);
  const int B = img.size(0), C = img.size(1), H = img.size(2), W = img.size(3);
  TORCH_CHECK(pool.dim() == 4 && pool.size(1) == C && pool.size(2) == H && pool.size(3) == W, "pool shape");
  TORCH_CHECK(target.sizes() == img.sizes() && t.numel() == B, "cold patch-embed shapes");
  const IdxSel is = idx_select(idx, idx_ctr, idx_off, B, draw_idx, "cold patch-embed");
  if (gauss_T > 0) {
    TORCH_CHECK(target_x0, "Gaussian batch: the target is x0");
    TORCH_CHECK(gauss_T <= temb.size(0), "Gaussian batch: T exceeds the time-embedding rows");
    TORCH_CHECK((int64_t)B * C * H * W < ((int64_t)1 << 31), "Gaussian batch: 32-bit noise index");
  } else {
    TORCH_CHECK(max_t >= 1 && (1 << max_t) <= W && (1 << max_t) <= H, "max_t");
  }
  ColdSrc cs;
  cs.gauss_T = gauss_T;
  cs.noise_site = noise_site;
  cs.target_rows = target_rows;
  cs.pool = pool.data_ptr<float>();
  cs.pool_n = pool.size(0);
  cs.site = data_site;
  cs.max_t = max_t;
  cs.draw_idx = draw_idx;
  cs.target_x0 = target_x0;
  cs.idx = is.p;
  cs.idx_ctr = is.ctr;
  cs.idx_rows = is.rows;
  cs.idx_stride = is.stride;
  cs.t_out = t.data_ptr<int64_t>();
  cs.target = target.data_ptr<float>();
  cs.x_t = write_xt ? img.data_ptr<float>() : nullptr;
  return patch_embed_impl(img, t, w_pe, b_pe, cls, pos, temb, rng, site, p, patch, ln_st, xb_out, cs);
}

std::tuple<Tensor, Tensor, Tensor> layernorm_fwd(Tensor x, Tensor gamma, Tensor beta, double eps) {
  CHECK_IN(x, F32); CHECK_IN(gamma, F32); CHECK_IN(beta, F32);
  const c10::DeviceGuard guard(x.device());
  const int D = x.size(-1);
  const int M = x.numel() / D;
  TORCH_CHECK(gamma.numel() == D && beta.numel() == D, "layernorm affine shape");
  auto y = at::empty(x.sizes(), x.options().dtype(BF16));
  auto mean = at::empty({M}, x.options());
  auto rstd = at::empty({M}, x.options());
  layernorm_fwd_launch(x.data_ptr<float>(), gamma.data_ptr<float>(), beta.data_ptr<float>(), y.data_ptr(),
                       mean.data_ptr<float>(), rstd.data_ptr<float>(), M, D, (float)eps, cur_stream());
  return {y, mean, rstd};
}

// y = a w^T (+ b): plain nn.Linear, bf16 or fp32 output
Tensor linear_fwd(Tensor a, Tensor w, c10::optional<Tensor> b, bool out_fp32, c10::optional<Tensor> ln_st, c10::optional<Tensor> ln_c, double ln_eps) {
  CHECK_IN(a, BF16); CHECK_IN(w, BF16);
  const c10::DeviceGuard guard(a.device());
  const int K = a.size(-1);
  auto a2 = a.view({-1, K});
  check_linear(a2, w, K);
  const int M = a2.size(0), Dout = w.size(0);
  auto out = at::empty({M, Dout}, a.options().dtype(out_fp32 ? at::kFloat : at::kBFloat16));
  GemmArgs g = nt_args(a2, w);
  g.C = out.data_ptr(); g.ldc = Dout;
  if (b.has_value() && b->defined()) {
    CHECK_IN((*b), F32);
    TORCH_CHECK(b->numel() == Dout, "bias shape");
    g.bias = b->data_ptr<float>();
  }
  apply_fold(g, M, Dout, ln_st, ln_c, ln_eps, c10::nullopt, c10::nullopt);
  gemm_nt(g, out_fp32 ? EPI_F32 : EPI_BF16, cur_stream());
  return out;
}

Tensor qkv_fwd(Tensor a, Tensor w, Tensor b, int64_t B, int64_t N, int64_t H, c10::optional<Tensor> ln_st, c10::optional<Tensor> ln_c, double ln_eps,
               c10::optional<Tensor> ln_mean, c10::optional<Tensor> ln_rstd) {
  CHECK_IN(a, BF16); CHECK_IN(w, BF16); CHECK_IN(b, F32);
  const c10::DeviceGuard guard(a.device());
  const int D = a.size(1);
  check_linear(a, w, D);
  TORCH_CHECK(w.size(0) == 3 * D && b.numel() == 3 * D && a.size(0) == B * N && D % H == 0, "qkv shapes");
  auto out = at::empty({3, B, H, N, D / H}, a.options());
  GemmArgs g = nt_args(a, w);
  g.C = out.data_ptr(); g.ldc = 3 * D; g.bias = b.data_ptr<float>();
  g.tokens = N; g.batch = B; g.heads = H; g.hd = D / H;
  apply_fold(g, B * N, 3 * D, ln_st, ln_c, ln_eps, ln_mean, ln_rstd);
  gemm_nt(g, EPI_QKV, cur_stream());
  return out;
}

// attention-dropout keep-flag words the short forward stores for the backward
// (0: this shape takes the long-sequence kernels, which regenerate the masks)
int64_t gemm_tile_override_op(int64_t cfg) { return gemm_set_tile_override((int)cfg); }
// GEMM phase stamps (tools/ub_gemm_stamps.py): an int32 buffer, or None to stop
void gemm_stamps_op(c10::optional<Tensor> buf) {
  if (buf.has_value() && buf->defined()) {
    TORCH_CHECK(buf->is_cuda() && buf->scalar_type() == at::kInt && buf->is_contiguous(), "gemm_stamps: int32 cuda");
    gemm_set_stamps(reinterpret_cast<uint32_t*>(buf->data_ptr<int32_t>()));
  } else {
    gemm_set_stamps(nullptr);
  }
}

int64_t attn_keep_words_op(int64_t B, int64_t H, int64_t N, int64_t hd) {
  return attn_keep_words((int)B, (int)H, (int)N, (int)hd);
}

static uint32_t* keep_ptr(const c10::optional<Tensor>& keep, int B, int H, int N, int hd) {
  if (!keep.has_value()) return nullptr;
  CHECK_IN(keep.value(), at::kInt);
  const int64_t need = attn_keep_words(B, H, N, hd);
  TORCH_CHECK(need > 0 && keep->numel() >= need, "attention keep-flag buffer: need ", need, " int32 words");
  return reinterpret_cast<uint32_t*>(keep->data_ptr<int32_t>());
}

std::tuple<Tensor, Tensor> attn_fwd(Tensor qkv, double scale, Tensor rng, int64_t site, double p,
                                    c10::optional<Tensor> keep_out) {
  CHECK_IN(qkv, BF16); check_rng(rng);
  const c10::DeviceGuard guard(qkv.device());
  TORCH_CHECK(qkv.dim() == 5 && qkv.size(0) == 3, "qkv must be [3,B,H,N,hd]");
  const int B = qkv.size(1), H = qkv.size(2), N = qkv.size(3), hd = qkv.size(4);
  TORCH_CHECK(hd == 32 || hd == 64, "head dim must be 32 or 64");
  // dropout mask elements are indexed with 32-bit counters (hoisted pair-hash math)
  TORCH_CHECK(p <= 0 || (int64_t)B * H * N * ((N + 3) & ~3) < ((int64_t)1 << 32),
              "attention dropout: more than 2^32 mask elements");
  auto o = at::empty({B, N, H * hd}, qkv.options());
  auto lse = at::empty({B, H, N}, qkv.options().dtype(F32));
  attn_fwd_launch(qkv.data_ptr(), o.data_ptr(), lse.data_ptr<float>(), B, H, N, hd, (float)scale,
                  rng.data_ptr<int64_t>(), site, p, cur_stream(), keep_ptr(keep_out, B, H, N, hd));
  return {o, lse};
}

Tensor linear_residual_fwd(Tensor a, Tensor w, Tensor b, Tensor x, int64_t N, Tensor rng, int64_t site_drop,
                           double p_drop, int64_t site_dp, double p_dp, c10::optional<Tensor> st_out, c10::optional<Tensor> xb_out) {
  CHECK_IN(a, BF16); CHECK_IN(w, BF16); CHECK_IN(b, F32); CHECK_IN(x, F32); check_rng(rng);
  const c10::DeviceGuard guard(a.device());
  const int K = a.size(-1);
  auto a2 = a.view({-1, K});
  check_linear(a2, w, K);
  const int M = a2.size(0), Dout = w.size(0);
  TORCH_CHECK(x.numel() == (int64_t)M * Dout && b.numel() == Dout && M % N == 0, "residual shapes");
  auto out = at::empty(x.sizes(), x.options());
  GemmArgs g = nt_args(a2, w);
  g.C = out.data_ptr(); g.ldc = Dout; g.bias = b.data_ptr<float>(); g.res = x.data_ptr<float>();
  g.rng = rng.data_ptr<int64_t>(); g.site_drop = site_drop; g.p_drop = p_drop; g.site_dp = site_dp; g.p_dp = p_dp;
  g.tokens = N;
  apply_prod(g, M, Dout, st_out, xb_out);
  gemm_nt(g, EPI_RESID, cur_stream());
  return out;
}

std::tuple<Tensor, Tensor> linear_gelu_fwd(Tensor a, Tensor w, Tensor b, Tensor rng, int64_t site, double p,
                                           c10::optional<Tensor> ln_st, c10::optional<Tensor> ln_c, double ln_eps, c10::optional<Tensor> ln_mean,
                                           c10::optional<Tensor> ln_rstd) {
  CHECK_IN(a, BF16); CHECK_IN(w, BF16); CHECK_IN(b, F32); check_rng(rng);
  const c10::DeviceGuard guard(a.device());
  const int K = a.size(-1);
  auto a2 = a.view({-1, K});
  check_linear(a2, w, K);
  const int M = a2.size(0), Hm = w.size(0);
  TORCH_CHECK(b.numel() == Hm, "bias shape");
  auto u = at::empty({M, Hm}, a.options());
  auto h = at::empty({M, Hm}, a.options());
  GemmArgs g = nt_args(a2, w);
  g.C = u.data_ptr(); g.ldc = Hm; g.C2 = h.data_ptr(); g.bias = b.data_ptr<float>();
  g.rng = rng.data_ptr<int64_t>(); g.site_drop = site; g.p_drop = p;
  apply_fold(g, M, Hm, ln_st, ln_c, ln_eps, ln_mean, ln_rstd);
  gemm_nt(g, EPI_GELU, cur_stream());
  return {u, h};
}

Tensor head_fwd(Tensor a, Tensor w, Tensor b, int64_t B, int64_t C, int64_t H, int64_t W, int64_t patch,
                c10::optional<Tensor> ln_st, c10::optional<Tensor> ln_c, double ln_eps, c10::optional<Tensor> ln_mean, c10::optional<Tensor> ln_rstd) {
  CHECK_IN(a, BF16); CHECK_IN(w, BF16); CHECK_IN(b, F32);
  const c10::DeviceGuard guard(a.device());
  const int K = a.size(-1);
  auto a2 = a.view({-1, K});
  check_linear(a2, w, K);
  const int N = (H / patch) * (W / patch) + 1;
  TORCH_CHECK(a2.size(0) == B * N && w.size(0) == C * patch * patch && b.numel() == w.size(0), "head shapes");
  auto img = at::empty({B, C, H, W}, a.options().dtype(F32));
  GemmArgs g = nt_args(a2, w);
  g.C = img.data_ptr(); g.bias = b.data_ptr<float>();
  g.tokens = N; g.batch = B; g.chans = C; g.img_h = H; g.img_w = W; g.patch = patch;
  apply_fold(g, B * N, w.size(0), ln_st, ln_c, ln_eps, ln_mean, ln_rstd);
  gemm_nt(g, EPI_HEAD, cur_stream());
  return img;
}

// Head GEMM with the sampler step fused into its unpatchify epilogue:
//   mode 1 (DDIM): x0 = clamp(head(a), -1, 1); x <- sqrt(a_tk) x0 + sqrt(1-a_tk) (x - sqrt(a_t) x0)/sqrt(1-a_t)
//                  in place, x0 written to x0_out; coef = device row {sqrt a_t, sqrt 1-a_t, sqrt a_tk, sqrt 1-a_tk}
//   mode 2 (cold): x <- clamp(head(a), -1, 1)
//   mode 4 (img2img): mode 1 with one coefficient row per sample (coef [B][4])
void head_step_(Tensor a, Tensor w, Tensor b, Tensor x, c10::optional<Tensor> x0_out, c10::optional<Tensor> coef,
                int64_t patch, int64_t mode, c10::optional<Tensor> ln_st, c10::optional<Tensor> ln_c, double ln_eps,
                c10::optional<Tensor> patches_out) {
  CHECK_IN(a, BF16); CHECK_IN(w, BF16); CHECK_IN(b, F32); CHECK_IN(x, F32);
  const c10::DeviceGuard guard(a.device());
  TORCH_CHECK(x.dim() == 4, "x must be [B, C, H, W]");
  const int B = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int K = a.size(-1);
  auto a2 = a.view({-1, K});
  check_linear(a2, w, K);
  const int N = (H / patch) * (W / patch) + 1;
  TORCH_CHECK(a2.size(0) == B * N && w.size(0) == C * patch * patch && b.numel() == w.size(0), "head shapes");
  TORCH_CHECK(mode == 1 || mode == 2 || mode == 4, "head_step_: mode 1 (ddim), 2 (clamp) or 4 (per-sample ddim)");
  GemmArgs g = nt_args(a2, w);
  g.C = x.data_ptr(); g.bias = b.data_ptr<float>();
  g.tokens = N; g.batch = B; g.chans = C; g.img_h = H; g.img_w = W; g.patch = patch;
  g.head_mode = (int)mode;
  if (mode == 1 || mode == 4) {
    TORCH_CHECK(x0_out.has_value() && coef.has_value(), "ddim mode needs x0_out and coef");
    CHECK_IN((*x0_out), F32); CHECK_IN((*coef), F32);
    TORCH_CHECK(x0_out->sizes() == x.sizes() && coef->numel() >= (mode == 4 ? 4 * B : 4), "x0_out / coef shapes");
    g.res = x.data_ptr<float>(); g.C2 = x0_out->data_ptr(); g.coef = coef->data_ptr<float>();
  }
  if (patches_out.has_value() && patches_out->defined()) {  // the next step's patch rows
    CHECK_IN((*patches_out), BF16);
    TORCH_CHECK(patches_out->numel() == (int64_t)B * (N - 1) * C * patch * patch, "patches_out must be [B*P, C*p*p]");
    g.patch_out = patches_out->data_ptr();
  }
  apply_fold(g, B * N, w.size(0), ln_st, ln_c, ln_eps, c10::nullopt, c10::nullopt);
  gemm_nt(g, EPI_HEAD, cur_stream());
}

// Sampler step on patch rows (EPI_HEADR): x / x0_out / patches_out are [B*P][F]
// (F = C*p*p in the head's output column order), so every epilogue access is a
// contiguous 16-byte vector (the image-layout head_step_ scatters 4-byte pixels).
void head_step_rows_(Tensor a, Tensor w, Tensor b, Tensor x, c10::optional<Tensor> x0_out,
                     c10::optional<Tensor> coef, int64_t batch, int64_t mode, c10::optional<Tensor> ln_st,
                     c10::optional<Tensor> ln_c, double ln_eps, c10::optional<Tensor> patches_out) {
  CHECK_IN(a, BF16); CHECK_IN(w, BF16); CHECK_IN(b, F32); CHECK_IN(x, F32);
  const c10::DeviceGuard guard(a.device());
  const int K = a.size(-1);
  auto a2 = a.view({-1, K});
  check_linear(a2, w, K);
  const int F = w.size(0), B = batch;
  TORCH_CHECK(B >= 1 && x.dim() == 2 && x.size(1) == F && x.size(0) % B == 0, "x must be [B*P, F]");
  const int NP = x.size(0) / B, N = NP + 1;
  TORCH_CHECK(a2.size(0) == (int64_t)B * N && b.numel() == F && F % 4 == 0, "head rows shapes");
  TORCH_CHECK(mode == 1 || mode == 2 || mode == 4, "head_step_rows_: mode 1 (ddim), 2 (clamp) or 4 (per-sample ddim)");
  GemmArgs g = nt_args(a2, w);
  g.C = x.data_ptr(); g.bias = b.data_ptr<float>();
  g.tokens = N; g.batch = B;
  g.head_mode = (int)mode;
  if (mode == 1 || mode == 4) {
    TORCH_CHECK(x0_out.has_value() && coef.has_value(), "ddim mode needs x0_out and coef");
    CHECK_IN((*x0_out), F32); CHECK_IN((*coef), F32);
    TORCH_CHECK(x0_out->sizes() == x.sizes() && coef->numel() >= (mode == 4 ? 4 * B : 4), "x0_out / coef shapes");
    g.res = x.data_ptr<float>(); g.C2 = x0_out->data_ptr(); g.coef = coef->data_ptr<float>();
  }
  if (patches_out.has_value() && patches_out->defined()) {
    CHECK_IN((*patches_out), BF16);
    TORCH_CHECK(patches_out->sizes() == x.sizes(), "patches_out must be [B*P, F]");
    g.patch_out = patches_out->data_ptr();
  }
  apply_fold(g, B * N, F, ln_st, ln_c, ln_eps, c10::nullopt, c10::nullopt);
  gemm_nt(g, EPI_HEADR, cur_stream());
}

// Head GEMM with the training loss in its epilogue (head_mode 3): the smooth-L1
// of the unpatchified prediction vs `target` (multi_gpu_trainer.py:124) as one
// partial per workgroup, and its gradient written straight into the token
// layout the head backward consumes (cls rows zero).  Returns (partials, dtok).
// target_rows: `target` ([B, C, H, W]-shaped) holds patch rows [B*P][C*p*p] in the
// head's output column order (the fused batch draw writes them): vector epilogue
// (EPI_HEADL) with contiguous target loads instead of scattered pixels.
std::tuple<Tensor, Tensor> head_loss(Tensor a, Tensor w, Tensor b, Tensor target, int64_t patch, double beta,
                                     c10::optional<Tensor> ln_st, c10::optional<Tensor> ln_c, double ln_eps,
                                     c10::optional<Tensor> ln_mean, c10::optional<Tensor> ln_rstd,
                                     bool target_rows) {
  CHECK_IN(a, BF16); CHECK_IN(w, BF16); CHECK_IN(b, F32); CHECK_IN(target, F32);
  const c10::DeviceGuard guard(a.device());
  TORCH_CHECK(target.dim() == 4, "target must be [B, C, H, W]");
  const int B = target.size(0), C = target.size(1), H = target.size(2), W = target.size(3);
  const int K = a.size(-1);
  auto a2 = a.view({-1, K});
  check_linear(a2, w, K);
  const int N = (H / patch) * (W / patch) + 1, F = C * patch * patch;
  TORCH_CHECK(a2.size(0) == (int64_t)B * N && w.size(0) == F && b.numel() == F, "head_loss shapes");
  TORCH_CHECK(beta > 0, "smooth-L1 beta must be > 0");
  const int M = B * N;
  auto dtok = at::empty({M, F}, a.options());
  auto parts = at::empty({gemm_nt_grid(M, F, K)}, a.options().dtype(F32));
  GemmArgs g = nt_args(a2, w);
  g.C = dtok.data_ptr(); g.C2 = dtok.data_ptr(); g.bias = b.data_ptr<float>(); g.res = target.data_ptr<float>();
  g.tokens = N; g.batch = B; g.chans = C; g.img_h = H; g.img_w = W; g.patch = patch;
  g.head_mode = 3;
  g.loss_beta = (float)beta;
  g.loss_inv_n = 1.0f / (float)((int64_t)B * C * H * W);
  g.loss_parts = parts.data_ptr<float>();
  apply_fold(g, M, F, ln_st, ln_c, ln_eps, ln_mean, ln_rstd);
  gemm_nt(g, target_rows ? EPI_HEADL : EPI_HEAD, cur_stream());
  return {parts, dtok};
}

std::tuple<Tensor, Tensor> smooth_l1_fwd_bwd(Tensor pred, Tensor target, int64_t N, int64_t patch, double beta,
                                             c10::optional<Tensor> loss_last, c10::optional<Tensor> loss_ema,
                                             double ema_decay, bool finish) {
  CHECK_IN(pred, F32); CHECK_IN(target, F32);
  float* ll = nullptr;
  float* le = nullptr;
  if (loss_last.has_value() && loss_last->defined()) { CHECK_IN((*loss_last), F32); ll = loss_last->data_ptr<float>(); }
  if (loss_ema.has_value() && loss_ema->defined()) { CHECK_IN((*loss_ema), F32); le = loss_ema->data_ptr<float>(); }
  const c10::DeviceGuard guard(pred.device());
  TORCH_CHECK(pred.sizes() == target.sizes() && pred.dim() == 4, "pred/target shape");
  const int B = pred.size(0), C = pred.size(1), H = pred.size(2), W = pred.size(3);
  TORCH_CHECK(N == (H / patch) * (W / patch) + 1, "token count");
  auto loss = at::empty({1}, pred.options());
  auto parts = at::empty({L1_PARTS}, pred.options());
  auto dtok = at::empty({(int64_t)B * N, C * patch * patch}, pred.options().dtype(BF16));
  const int np = smooth_l1_launch(pred.data_ptr<float>(), target.data_ptr<float>(), loss.data_ptr<float>(),
                                  parts.data_ptr<float>(), dtok.data_ptr(), B, C, H, W, patch, (float)beta, ll, le,
                                  (float)ema_decay, finish, cur_stream());
  // finish = false: the per-block partials (their sum is the loss) instead of the loss
  return {finish ? loss : parts.narrow(0, 0, np), dtok};
}

Tensor img_to_tokgrad(Tensor dimg, int64_t N, int64_t patch) {
  CHECK_IN(dimg, F32);
  const c10::DeviceGuard guard(dimg.device());
  const int B = dimg.size(0), C = dimg.size(1), H = dimg.size(2), W = dimg.size(3);
  TORCH_CHECK(N == (H / patch) * (W / patch) + 1, "token count");
  auto dtok = at::empty({(int64_t)B * N, C * patch * patch}, dimg.options().dtype(BF16));
  img_to_tokgrad_launch(dimg.data_ptr<float>(), dtok.data_ptr(), B, C, H, W, patch, cur_stream());
  return dtok;
}

// splits > 1 (fp32 only): [splits, M, K] partial products over K slices
Tensor linear_dgrad(Tensor dy, Tensor w, bool out_fp32, int64_t splits) {
  CHECK_IN(dy, BF16); CHECK_IN(w, BF16);
  const c10::DeviceGuard guard(dy.device());
  TORCH_CHECK(dy.dim() == 2 && w.dim() == 2 && dy.size(1) == w.size(0), "dgrad shapes");
  const int M = dy.size(0), Nout = w.size(0), K = w.size(1);
  TORCH_CHECK(Nout % 8 == 0 && K % 8 == 0, "dgrad dims must be multiples of 8");
  TORCH_CHECK(splits >= 1 && splits <= 4, "dgrad K split: 1..4");
  auto dx = splits > 1 ? at::empty({splits, M, K}, dy.options().dtype(out_fp32 ? F32 : BF16))
                       : at::empty({M, K}, dy.options().dtype(out_fp32 ? F32 : BF16));
  GemmArgs g;
  g.A = dy.data_ptr(); g.B = w.data_ptr();
  g.M = M; g.N = K; g.K = Nout; g.lda = Nout; g.ldb = K;
  g.C = dx.data_ptr(); g.ldc = K;
  g.splits = (int)splits;
  g.split_stride = (long long)M * K;
  gemm_dgrad(g, out_fp32 ? EPI_F32 : EPI_BF16, cur_stream());
  return dx;
}

Tensor linear_dgrad_gelu(Tensor dy, Tensor w, Tensor u, Tensor rng, int64_t site, double p) {
  CHECK_IN(dy, BF16); CHECK_IN(w, BF16); CHECK_IN(u, BF16); check_rng(rng);
  const c10::DeviceGuard guard(dy.device());
  TORCH_CHECK(dy.dim() == 2 && w.dim() == 2 && dy.size(1) == w.size(0), "dgrad shapes");
  const int M = dy.size(0), Nout = w.size(0), K = w.size(1);
  TORCH_CHECK(u.numel() == (int64_t)M * K, "u shape");
  TORCH_CHECK(Nout % 8 == 0 && K % 8 == 0, "dgrad dims must be multiples of 8");
  auto du = at::empty({M, K}, dy.options());
  GemmArgs g;
  g.A = dy.data_ptr(); g.B = w.data_ptr();
  g.M = M; g.N = K; g.K = Nout; g.lda = Nout; g.ldb = K;
  g.C = du.data_ptr(); g.ldc = K; g.aux = u.data_ptr();
  g.rng = rng.data_ptr<int64_t>(); g.site_drop = site; g.p_drop = p;
  gemm_dgrad(g, EPI_DGELU, cur_stream());
  return du;
}

// the same with the transposed weight wt = W^T [in][out] (k-contiguous operand path)
Tensor linear_dgrad_gelu_t(Tensor dy, Tensor wt, Tensor u, Tensor rng, int64_t site, double p) {
  CHECK_IN(dy, BF16); CHECK_IN(wt, BF16); CHECK_IN(u, BF16); check_rng(rng);
  const c10::DeviceGuard guard(dy.device());
  TORCH_CHECK(dy.dim() == 2 && wt.dim() == 2 && dy.size(1) == wt.size(1), "dgrad shapes (wt = W^T)");
  const int M = dy.size(0), Nout = wt.size(1), K = wt.size(0);
  TORCH_CHECK(u.numel() == (int64_t)M * K, "u shape");
  TORCH_CHECK(Nout % 64 == 0 && K % 8 == 0, "dgrad (transposed weight): K % 64 == 0, N % 8 == 0");
  auto du = at::empty({M, K}, dy.options());
  GemmArgs g;
  g.A = dy.data_ptr(); g.B = wt.data_ptr();
  g.M = M; g.N = K; g.K = Nout; g.lda = Nout; g.ldb = Nout;
  g.C = du.data_ptr(); g.ldc = K; g.aux = u.data_ptr();
  g.rng = rng.data_ptr<int64_t>(); g.site_drop = site; g.p_drop = p;
  gemm_nt(g, EPI_DGELU, cur_stream());
  return du;
}

void linear_wgrad(Tensor dy, Tensor x, Tensor dw, c10::optional<Tensor> db) {
  CHECK_IN(dy, BF16); CHECK_IN(x, BF16); CHECK_IN(dw, F32);
  const c10::DeviceGuard guard(dy.device());
  TORCH_CHECK(dy.dim() == 2 && x.dim() == 2 && dy.size(0) == x.size(0), "wgrad shapes");
  const int M = dy.size(0), Nout = dy.size(1), K = x.size(1);
  TORCH_CHECK(dw.numel() == (int64_t)Nout * K, "dw shape");
  TORCH_CHECK(Nout % 8 == 0 && K % 8 == 0, "wgrad dims must be multiples of 8");
  float* dbp = nullptr;
  if (db.has_value() && db->defined()) {
    CHECK_IN((*db), F32);
    TORCH_CHECK(db->numel() == Nout, "db shape");
    dbp = db->data_ptr<float>();
  }
  GemmArgs g;
  g.A = dy.data_ptr(); g.B = x.data_ptr();
  g.M = Nout; g.N = K; g.K = M; g.lda = Nout; g.ldb = K;
  g.C = dw.data_ptr(); g.ldc = K; g.bias = dbp;
  // split the token reduction so the grid fills the chip; fp32 atomics combine the
  // slices, so keep the split count small (atomic bytes = splits x |dW|, chip-wide
  // atomic rate ~1.3 TB/s)
  const int tiles = ((Nout + 63) / 64) * ((K + 63) / 64);
  const int kt = (M + 63) / 64;
  constexpr int max_splits = 8;
  int splits = (256 + tiles - 1) / tiles;
  if (splits > max_splits) splits = max_splits;
  if (splits > kt) splits = kt;
  if (splits < 1) splits = 1;
  gemm_wgrad(g, splits, cur_stream());
}

// Grouped weight gradients: one launch for all (dy_i, x_i) -> dW_i += dy_i^T x_i
// (db_i += colsum dy_i).  The token reduction is split over fp32 atomics (2-way
// for a full block group, more for small groups); splits == 1 would use a plain
// read-add-write epilogue.
// grad-norm partial buffers: every partial is written (sqnorm: one block each; the
// fused weight-gradient launch: tiles + tail, rest zeroed) and summed by consumers
int check_parts(const Tensor& t, const char* who) {
  TORCH_CHECK(t.numel() >= SQ_PARTS && t.numel() % 256 == 0 && t.numel() < (1 << 24), who,
              ": grad-norm partials must be >= SQ_PARTS floats, a multiple of 256");
  return (int)t.numel();
}

static std::vector<GemmArgs> wgrad_probs(const std::vector<Tensor>& dys, const std::vector<Tensor>& xs,
                                         const std::vector<Tensor>& dws,
                                         const std::vector<c10::optional<Tensor>>& dbs, int* tiles_out,
                                         int* min_kt_out) {
  const size_t n = dys.size();
  TORCH_CHECK(xs.size() == n && dws.size() == n && dbs.size() == n, "wgrad_group: list sizes");
  std::vector<GemmArgs> probs;
  int tiles = 0, min_kt = 1 << 30;
  for (size_t i = 0; i < n; ++i) {
    const Tensor &dy = dys[i], &x = xs[i], &dw = dws[i];
    CHECK_IN(dy, BF16); CHECK_IN(x, BF16); CHECK_IN(dw, F32);
    TORCH_CHECK(dy.device() == dys[0].device() && x.device() == dy.device() && dw.device() == dy.device(),
                "wgrad_group: tensors on different devices");
    TORCH_CHECK(dy.dim() == 2 && x.dim() == 2 && dy.size(0) == x.size(0), "wgrad_group shapes");
    const int M = dy.size(0), Nout = dy.size(1), K = x.size(1);
    TORCH_CHECK(dw.numel() == (int64_t)Nout * K, "wgrad_group: dw shape");
    TORCH_CHECK(Nout % 8 == 0 && K % 8 == 0, "wgrad dims must be multiples of 8");
    GemmArgs g;
    g.A = dy.data_ptr(); g.B = x.data_ptr();
    g.M = Nout; g.N = K; g.K = M; g.lda = Nout; g.ldb = K;
    g.C = dw.data_ptr(); g.ldc = K;
    if (dbs[i].has_value() && dbs[i]->defined()) {
      CHECK_IN((*dbs[i]), F32);
      TORCH_CHECK(dbs[i]->numel() == Nout, "wgrad_group: db shape");
      g.bias = dbs[i]->data_ptr<float>();
    }
    probs.push_back(g);
    tiles += ((Nout + 63) / 64) * ((K + 63) / 64);
    min_kt = std::min(min_kt, (M + 63) / 64);
  }
  if (tiles_out) *tiles_out = tiles;
  if (min_kt_out) *min_kt_out = min_kt;
  return probs;
}

// Tickets of the K-split weight-gradient tail: 4,096 ints per (device, stream), zeroed
// once (the first call is an eager step, outside any graph); each split tile's last piece
// resets its ticket, so every launch on that stream finds them zero (launches on one
// stream run in order; two streams -- e.g. two engines in one process -- get their own).
static int* split_tickets(const c10::Device& dev) {
  static std::mutex mu;
  static std::map<std::pair<int, int64_t>, Tensor> bufs;
  const auto key = std::make_pair((int)dev.index(), (int64_t)c10::hip::getCurrentHIPStream(dev.index()).id());
  std::lock_guard<std::mutex> lk(mu);
  auto it = bufs.find(key);
  if (it == bufs.end())
    it = bufs.emplace(key, at::zeros({4096}, at::TensorOptions().dtype(at::kInt).device(dev))).first;
  return it->second.data_ptr<int>();
}

// Every weight gradient of a training step in ONE launch (gemm_wgrad_multi_kernel)
// sq_parts / arena: also write the grad-norm partials of the whole gradient arena
// (the launches must then be its last writers): the arena ranges outside every dW /
// db target and outside the lazy range [lz_lo, lz_hi) go to the tail workgroups of
// the last launch.  More than 32 problems: consecutive launches of <= 32, each
// writing its tiles' partials after the previous launch's.
void linear_wgrad_multi(std::vector<Tensor> dys, std::vector<Tensor> xs, std::vector<Tensor> dws,
                        std::vector<c10::optional<Tensor>> dbs, bool store, c10::optional<Tensor> sq_parts,
                        c10::optional<Tensor> arena, int64_t lz_lo, int64_t lz_hi, c10::optional<Tensor> emb_g,
                        c10::optional<Tensor> emb_t, c10::optional<Tensor> emb_rng, int64_t emb_site, double emb_p,
                        c10::optional<Tensor> emb_cls, c10::optional<Tensor> emb_pos, c10::optional<Tensor> emb_temb,
                        int64_t emb_owners, c10::optional<Tensor> ln_ws, c10::optional<Tensor> ln_ptrs,
                        std::vector<int64_t> ln_offs, int64_t ln_C, int64_t ln_R, bool ln_store) {
  TORCH_CHECK(!dys.empty() && dys.size() == xs.size() && dys.size() == dws.size() && dys.size() == dbs.size(),
              "wgrad_multi: one dy, x, dw, db per problem");
  const c10::DeviceGuard guard(dys[0].device());
  const bool fused = sq_parts.has_value() && sq_parts->defined();
  // embedding gradients + LayerNorm finalize as extra workgroups (embed_parts.h)
  const bool with_emb = emb_g.has_value() && emb_g->defined();
  WgradEmbed we{};
  std::vector<std::pair<int64_t, int64_t>> covered;  // arena ranges the embedding workgroups write
  if (with_emb) {
    const Tensor& g = *emb_g;
    CHECK_IN(g, F32); CHECK_IN((*emb_t), I64); check_rng(*emb_rng);
    CHECK_IN((*emb_cls), F32); CHECK_IN((*emb_pos), F32); CHECK_IN((*emb_temb), F32);
    TORCH_CHECK(g.dim() == 3, "emb_g must be [B, N, D]");
    const int B = g.size(0), N = g.size(1), D = g.size(2);
    TORCH_CHECK(emb_t->numel() == B && emb_cls->numel() == D && emb_pos->numel() == (int64_t)N * D &&
                    emb_temb->size(-1) == D && D % 4 == 0 && B <= 256 && emb_owners >= 1 && emb_owners <= B,
                "wgrad_multi embedding shapes (B <= 256, D % 4 == 0, 1 <= owners <= B)");
    we.e = embed_grad_args(g.data_ptr<float>(), emb_t->data_ptr<int64_t>(), emb_cls->data_ptr<float>(),
                           emb_pos->data_ptr<float>(), emb_temb->data_ptr<float>(), B, N, D,
                           emb_rng->data_ptr<int64_t>(), (int)emb_site, emb_p, 0, B);
    we.e.owners = (int)emb_owners;
    if (ln_ws.has_value() && ln_ws->defined()) {
      CHECK_IN((*ln_ws), F32); CHECK_IN((*ln_ptrs), I64);
      we.rf.G = ln_ptrs->numel();
      we.rf.C = (int)ln_C;
      TORCH_CHECK(we.rf.G > 0 && ln_C > 0 && ln_ws->numel() % ((int64_t)we.rf.G * ln_C) == 0 &&
                      (int64_t)ln_offs.size() == we.rf.G, "wgrad_multi: LayerNorm workspace / offsets");
      we.rf.rows = (int)(ln_ws->numel() / ((int64_t)we.rf.G * ln_C));
      we.rf.R = (int)ln_R;
      TORCH_CHECK(we.rf.R >= 1 && we.rf.R <= we.rf.rows, "wgrad_multi: ln_R");
      we.rf.ws = ln_ws->data_ptr<float>();
      we.rf.dsts = reinterpret_cast<float* const*>(ln_ptrs->data_ptr<int64_t>());
      we.rf.store = ln_store ? 1 : 0;
    }
  }
  WgradSq sq;
  int np = 0;
  if (fused) {
    TORCH_CHECK(arena.has_value() && arena->defined(), "wgrad_multi: grad-norm partials need the gradient arena");
    CHECK_IN((*sq_parts), F32); CHECK_IN((*arena), F32);
    np = check_parts(*sq_parts, "wgrad_multi");
    const float* base = arena->data_ptr<float>();
    const int64_t n = arena->numel();
    // element intervals of the targets inside the arena
    std::vector<std::pair<int64_t, int64_t>> iv;
    auto add = [&](const Tensor& t) {
      TORCH_CHECK(t.is_contiguous(), "wgrad_multi: grad-norm fusion needs contiguous targets");
      const int64_t off = t.data_ptr<float>() - base;
      TORCH_CHECK(off >= 0 && off + t.numel() <= n, "wgrad_multi: a weight-gradient target lies outside the arena");
      iv.emplace_back(off, off + t.numel());
    };
    for (size_t i = 0; i < dws.size(); ++i) {
      add(dws[i]);
      if (dbs[i].has_value() && dbs[i]->defined()) add(*dbs[i]);
    }
    std::sort(iv.begin(), iv.end());
    for (size_t i = 1; i < iv.size(); ++i)
      TORCH_CHECK(iv[i].first >= iv[i - 1].second,
                  "wgrad_multi: overlapping weight-gradient targets (the partials would count them twice)");
    // ranges the tail skips without a tile writing them: the lazy range (zero forever)
    // and the embedding workgroups' outputs (they write their own partials)
    if (lz_hi > lz_lo) iv.emplace_back(lz_lo, lz_hi);
    if (with_emb) {
      auto cov = [&](const Tensor& t) {
        const int64_t off = t.data_ptr<float>() - base;
        TORCH_CHECK(off >= 0 && off + t.numel() <= n, "wgrad_multi: an embedding gradient lies outside the arena");
        iv.emplace_back(off, off + t.numel());
      };
      cov(*emb_cls); cov(*emb_pos); cov(*emb_temb);
      for (int64_t o : ln_offs) {
        TORCH_CHECK(o >= 0 && o + ln_C <= n, "wgrad_multi: a LayerNorm gradient lies outside the arena");
        iv.emplace_back(o, o + ln_C);
      }
    }
    std::sort(iv.begin(), iv.end());
    sq.base = base;
    int64_t cur = 0, rest = 0;
    auto gap = [&](int64_t lo, int64_t hi) {
      if (hi <= lo) return;
      TORCH_CHECK(sq.nr < WSQ_MAX_RANGES, "wgrad_multi: more than 16 arena ranges outside the weight gradients");
      sq.lo[sq.nr] = lo;
      sq.hi[sq.nr] = hi;
      ++sq.nr;
      rest += hi - lo;
    };
    for (const auto& [lo, hi] : iv) {
      gap(cur, lo);
      cur = std::max(cur, hi);
    }
    gap(cur, n);
    sq.tail = (int)std::min<int64_t>(64, std::max<int64_t>(1, (rest + 256 * 16 - 1) / (256 * 16)));
  }
  const size_t total = dys.size();
  // launches of <= WGRAD_MULTI_MAX problems with balanced tile counts (each launch's
  // K-split tail then fills its last round; 32 + 18 problems left a 0.9-round launch)
  int kmax = 0;
  for (const auto& t : dys) kmax = std::max<int>(kmax, (int)t.size(0));
  const int T = wgrad_multi_tile(kmax);
  std::vector<int64_t> ptiles(total);
  int64_t all_tiles = 0;
  for (size_t i = 0; i < total; ++i) {
    ptiles[i] = ((dys[i].size(1) + T - 1) / T) * ((xs[i].size(1) + T - 1) / T);
    all_tiles += ptiles[i];
  }
  const size_t L = (total + WGRAD_MULTI_MAX - 1) / WGRAD_MULTI_MAX;
  std::vector<size_t> cuts{0};
  int64_t cum = 0;
  for (size_t i = 0; i + 1 < total && cuts.size() < L; ++i) {
    cum += ptiles[i];
    const bool full = i + 1 - cuts.back() == (size_t)WGRAD_MULTI_MAX;
    if (full || cum * (int64_t)L >= all_tiles * (int64_t)cuts.size()) cuts.push_back(i + 1);
  }
  cuts.push_back(total);
  bool ok = true;
  for (size_t c = 0; c + 1 < cuts.size(); ++c) ok = ok && cuts[c + 1] - cuts[c] <= (size_t)WGRAD_MULTI_MAX;
  if (!ok) {  // cannot balance within the problem limit: plain chunks
    cuts.clear();
    for (size_t a = 0; a < total; a += WGRAD_MULTI_MAX) cuts.push_back(a);
    cuts.push_back(total);
  }
  int used = 0;  // partial slots written by earlier launches
  for (size_t ci = 0; ci + 1 < cuts.size(); ++ci) {
    const size_t a = cuts[ci], e = cuts[ci + 1];
    // K-split tail of wide launches: workspace from the caching allocator (the capture's
    // pool inside a graph), tickets in a per-device buffer every last piece resets
    float* sws = nullptr;
    int* scnt = nullptr;
    Tensor ws_t;
    {
      int64_t ct = 0;
      for (size_t i = a; i < e; ++i) ct += ptiles[i];
      const int64_t nf = wgrad_split_ws_floats((int)ct, T);
      if (nf > 0) {
        ws_t = at::empty({nf}, dys[0].options().dtype(F32));
        sws = ws_t.data_ptr<float>();
        scnt = split_tickets(dys[0].device());
      }
    }
    std::vector<Tensor> d(dys.begin() + a, dys.begin() + e), x(xs.begin() + a, xs.begin() + e),
        w(dws.begin() + a, dws.begin() + e);
    std::vector<c10::optional<Tensor>> b(dbs.begin() + a, dbs.begin() + e);
    std::vector<GemmArgs> probs = wgrad_probs(d, x, w, b, nullptr, nullptr);
    if (!fused) {
      gemm_wgrad_multi(probs.data(), (int)probs.size(), cur_stream(), store, nullptr,
                       (with_emb && e == total) ? &we : nullptr, sws, scnt);
      continue;
    }
    WgradSq s = sq;
    s.parts = sq_parts->data_ptr<float>() + used;
    s.nparts = np - used;
    if (e < total) {  // tail ranges, zero fill and embedding workgroups ride in the last launch
      s.nr = 0;
      s.tail = 0;
    }
    used += gemm_wgrad_multi(probs.data(), (int)probs.size(), cur_stream(), store, &s,
                             (with_emb && e == total) ? &we : nullptr, sws, scnt);
  }
  TORCH_CHECK(!with_emb || fused || total <= (size_t)WGRAD_MULTI_MAX, "wgrad_multi: embedding parts need sq fusion "
              "or one launch");
}

// grad-norm partial slots the embedding workgroups of a wgrad_multi launch take
int64_t wgrad_embed_slots(int64_t B, int64_t N, int64_t D, int64_t owners, int64_t n_ln, int64_t ln_C, bool wide) {
  WgradEmbed we{};
  we.e.B = (int)B; we.e.N = (int)N; we.e.D = (int)D; we.e.owners = (int)owners;
  float dummy = 0.f;
  if (n_ln > 0) { we.rf.ws = &dummy; we.rf.G = (int)n_ln; we.rf.C = (int)ln_C; }
  return wgrad_embed_workgroups(we, wide);
}

// fp32 <-> bf16 gradient wire (csrc/comm_wire.hip): one fused 16-B-vector
// kernel each way (the torch-collective bf16 wire path of the train engine)
void wire_pack(Tensor src, Tensor dst) {
  CHECK_IN(src, F32); CHECK_IN(dst, BF16);
  TORCH_CHECK(src.numel() == dst.numel(), "wire_pack: sizes");
  const c10::DeviceGuard guard(src.device());
  wire_pack_launch(src.data_ptr<float>(), dst.data_ptr(), src.numel(), cur_stream());
}
void wire_unpack(Tensor src, Tensor dst) {
  CHECK_IN(src, BF16); CHECK_IN(dst, F32);
  TORCH_CHECK(src.numel() == dst.numel(), "wire_unpack: sizes");
  const c10::DeviceGuard guard(src.device());
  wire_unpack_launch(src.data_ptr(), dst.data_ptr<float>(), src.numel(), cur_stream());
}

std::tuple<Tensor, Tensor> layernorm_bwd(Tensor dy, Tensor x, Tensor mean, Tensor rstd, Tensor gamma,
                                         c10::optional<Tensor> g_res, Tensor dgamma, Tensor dbeta, int64_t N,
                                         Tensor rng, int64_t site_drop, double p_drop, int64_t site_dp, double p_dp,
                                         bool emit_gy, c10::optional<Tensor> ws, c10::optional<Tensor> beta, c10::optional<Tensor> y_out,
                                         c10::optional<Tensor> gp_out, int64_t site_emb, double p_emb) {
  CHECK_CUDA(dy); CHECK_CONTIG(dy);
  TORCH_CHECK(dy.scalar_type() == F32 || dy.scalar_type() == BF16, "dy must be fp32 or bf16");
  CHECK_CUDA(x); CHECK_CONTIG(x);
  TORCH_CHECK(x.scalar_type() == F32 || x.scalar_type() == BF16, "layernorm_bwd: x must be fp32 or bf16");
  CHECK_IN(mean, F32); CHECK_IN(rstd, F32); CHECK_IN(gamma, F32);
  CHECK_IN(dgamma, F32); CHECK_IN(dbeta, F32); check_rng(rng);
  const c10::DeviceGuard guard(x.device());
  const int D = x.size(-1), M = x.numel() / D;
  // dy may be [P, M, D]: P partial products (K-split dgrad) summed on load
  const int parts = x.numel() > 0 ? (int)(dy.numel() / x.numel()) : 1;
  TORCH_CHECK(dy.numel() == (int64_t)parts * x.numel() && mean.numel() == M && rstd.numel() == M &&
                  gamma.numel() == D && dgamma.numel() == D && dbeta.numel() == D && M % N == 0 && parts <= 4,
              "layernorm_bwd shapes");
  const float* gr = nullptr;
  if (g_res.has_value() && g_res->defined()) {
    CHECK_IN((*g_res), F32);
    TORCH_CHECK(g_res->numel() == x.numel(), "g_res shape");
    gr = g_res->data_ptr<float>();
  }
  // workspace [S][2D]: one dgamma||dbeta slot per backward workgroup (overwritten)
  const int S = ln_bwd_workgroups(M);
  const bool own_ws = !(ws.has_value() && ws->defined());
  const auto f32o = x.options().dtype(F32);
  Tensor w = own_ws ? at::empty({S, 2 * D}, f32o) : *ws;
  if (!own_ws) {
    CHECK_IN(w, F32);
    TORCH_CHECK(w.numel() == (int64_t)S * 2 * D, "ln ws must hold ln_ws_rows(M) x 2D floats (", S,
                " rows for M = ", M, ")");
  }
  void* gpp = nullptr;
  if (gp_out.has_value() && gp_out->defined()) {  // the patch-embedding input gradient
    CHECK_IN((*gp_out), BF16);
    TORCH_CHECK(N > 1 && gp_out->numel() == (int64_t)(M / N) * (N - 1) * D, "gp_out must be [B*(N-1), D]");
    gpp = gp_out->data_ptr();
  }
  // y_out: also emit the LayerNorm output bf16 (x_hat gamma + beta) for the weight
  // gradient of the GEMM that consumed it through the LayerNorm fold
  const float* bp = nullptr;
  void* yp = nullptr;
  if (y_out.has_value() && y_out->defined()) {
    TORCH_CHECK(beta.has_value() && beta->defined(), "y_out needs beta");
    CHECK_IN((*beta), F32); CHECK_IN((*y_out), BF16);
    TORCH_CHECK(beta->numel() == D && y_out->numel() == x.numel(), "beta / y_out shapes");
    bp = beta->data_ptr<float>();
    yp = y_out->data_ptr();
  }
  auto g_out = at::empty(x.sizes(), f32o);
  Tensor gy = emit_gy ? at::empty({M, D}, x.options().dtype(BF16)) : at::empty({0}, x.options().dtype(BF16));
  layernorm_bwd_launch(dy.data_ptr(), dy.scalar_type() == BF16, x.data_ptr(), x.scalar_type() == BF16, mean.data_ptr<float>(), rstd.data_ptr<float>(),
                       gamma.data_ptr<float>(), bp, gr, g_out.data_ptr<float>(), emit_gy ? gy.data_ptr() : nullptr,
                       yp, w.data_ptr<float>(), M, D, N, rng.data_ptr<int64_t>(), site_drop, p_drop, site_dp, p_dp,
                       parts, gpp, (int)site_emb, p_emb, cur_stream());
  if (own_ws) {
    auto s = w.sum(0);
    dgamma.add_(s.narrow(0, 0, D));
    dbeta.add_(s.narrow(0, D, D));
  }
  return {g_out, gy};
}

int64_t ln_ws_rows_op(int64_t M) { return ln_bwd_workgroups((int)M); }

// dsts[i] = srcs[i]^T (bf16 [R][C] -> [C][R]), every matrix of the list in launches of
// <= TRANSPOSE_MAX matrices (the input-gradient GEMMs' transposed weight shadows)
void transpose_bf16_(std::vector<Tensor> srcs, std::vector<Tensor> dsts) {
  TORCH_CHECK(!srcs.empty() && srcs.size() == dsts.size(), "transpose_bf16_: one dst per src");
  const c10::DeviceGuard guard(srcs[0].device());
  for (size_t a = 0; a < srcs.size(); a += TRANSPOSE_MAX) {
    const size_t e = std::min(srcs.size(), a + (size_t)TRANSPOSE_MAX);
    std::vector<const void*> sp;
    std::vector<void*> dp;
    std::vector<int> R, C;
    for (size_t i = a; i < e; ++i) {
      CHECK_IN(srcs[i], BF16); CHECK_IN(dsts[i], BF16);
      TORCH_CHECK(srcs[i].dim() == 2 && dsts[i].dim() == 2 && dsts[i].size(0) == srcs[i].size(1) &&
                      dsts[i].size(1) == srcs[i].size(0), "transpose_bf16_: dst must be [C, R] for src [R, C]");
      sp.push_back(srcs[i].data_ptr());
      dp.push_back(dsts[i].data_ptr());
      R.push_back((int)srcs[i].size(0));
      C.push_back((int)srcs[i].size(1));
    }
    transpose_bf16_launch(sp.data(), dp.data(), R.data(), C.data(), (int)sp.size(), cur_stream());
  }
}

// ws [G][rows][C]: rows 0..R-1 of each LayerNorm workspace added into its destination
void replica_reduce_(Tensor ws, Tensor dst_ptrs, int64_t C, int64_t R) {
  CHECK_IN(ws, F32); CHECK_IN(dst_ptrs, I64);
  const c10::DeviceGuard guard(ws.device());
  const int G = dst_ptrs.numel();
  TORCH_CHECK(G > 0 && C > 0 && ws.numel() % ((int64_t)G * C) == 0, "replica ws shape");
  const int rows = (int)(ws.numel() / ((int64_t)G * C));
  TORCH_CHECK(R >= 1 && R <= rows, "replica rows");
  replica_reduce_launch(ws.data_ptr<float>(), reinterpret_cast<float* const*>(dst_ptrs.data_ptr<int64_t>()), G, C,
                        (int)R, rows, cur_stream());
}

Tensor attn_bwd(Tensor dout, Tensor qkv, Tensor o, Tensor lse, double scale, Tensor rng, int64_t site, double p,
                c10::optional<Tensor> keep) {
  CHECK_IN(dout, BF16); CHECK_IN(qkv, BF16); CHECK_IN(o, BF16); CHECK_IN(lse, F32); check_rng(rng);
  const c10::DeviceGuard guard(qkv.device());
  TORCH_CHECK(qkv.dim() == 5 && qkv.size(0) == 3, "qkv must be [3,B,H,N,hd]");
  const int B = qkv.size(1), H = qkv.size(2), N = qkv.size(3), hd = qkv.size(4);
  TORCH_CHECK(hd == 32 || hd == 64, "head dim must be 32 or 64");
  TORCH_CHECK(dout.numel() == (int64_t)B * N * H * hd && o.numel() == dout.numel() &&
                  lse.numel() == (int64_t)B * H * N,
              "attn_bwd shapes");
  TORCH_CHECK(p <= 0 || (int64_t)B * H * N * ((N + 3) & ~3) < ((int64_t)1 << 32),
              "attention dropout: more than 2^32 mask elements");
  auto dqkv = at::empty({(int64_t)B * N, 3 * H * hd}, qkv.options());
  auto delta = at::empty({(int64_t)B * H * N}, lse.options());
  attn_bwd_launch(dout.data_ptr(), qkv.data_ptr(), o.data_ptr(), lse.data_ptr<float>(), dqkv.data_ptr(),
                  delta.data_ptr<float>(), B, H, N, hd, (float)scale, rng.data_ptr<int64_t>(), site, p,
                  cur_stream(), keep_ptr(keep, B, H, N, hd));
  return dqkv;
}

Tensor embed_bwd(Tensor g, Tensor t, Tensor rng, int64_t site, double p, Tensor dcls, Tensor dpos, Tensor dtemb,
                 c10::optional<Tensor> ln_ws, c10::optional<Tensor> ln_ptrs, int64_t ln_C, bool ln_store,
                 int64_t ln_R) {
  CHECK_IN(g, F32); CHECK_IN(t, I64); check_rng(rng); CHECK_IN(dcls, F32); CHECK_IN(dpos, F32); CHECK_IN(dtemb, F32);
  const c10::DeviceGuard guard(g.device());
  TORCH_CHECK(g.dim() == 3, "g must be [B,N,D]");
  const int B = g.size(0), N = g.size(1), D = g.size(2);
  TORCH_CHECK(t.numel() == B && dcls.numel() == D && dpos.numel() == (int64_t)N * D && dtemb.size(-1) == D,
              "embed_bwd shapes");
  auto gpatch = at::empty({(int64_t)B * (N - 1), D}, g.options().dtype(BF16));
  ReplicaFinal rf;
  if (ln_ws.has_value() && ln_ws->defined()) {  // replica_reduce_ folded into this launch
    CHECK_IN((*ln_ws), F32);
    TORCH_CHECK(ln_ptrs.has_value() && ln_ptrs->defined(), "ln_ws needs ln_ptrs");
    CHECK_IN((*ln_ptrs), I64);
    rf.G = ln_ptrs->numel();
    rf.C = ln_C;
    TORCH_CHECK(rf.G > 0 && ln_C > 0 && ln_ws->numel() % ((int64_t)rf.G * ln_C) == 0, "replica ws shape");
    rf.rows = (int)(ln_ws->numel() / ((int64_t)rf.G * ln_C));
    rf.R = (int)ln_R;
    TORCH_CHECK(rf.R >= 1 && rf.R <= rf.rows, "ln_R: replica rows to sum");
    rf.ws = ln_ws->data_ptr<float>();
    rf.dsts = reinterpret_cast<float* const*>(ln_ptrs->data_ptr<int64_t>());
    rf.store = ln_store ? 1 : 0;
  }
  embed_bwd_launch(g.data_ptr<float>(), t.data_ptr<int64_t>(), dcls.data_ptr<float>(), dpos.data_ptr<float>(),
                   dtemb.data_ptr<float>(), gpatch.data_ptr(), B, N, D, rng.data_ptr<int64_t>(), site, p,
                   cur_stream(), rf);
  return gpatch;
}

void sqnorm(Tensor g, Tensor out, double scale, int64_t lz_lo, int64_t lz_hi) {
  CHECK_IN(g, F32); CHECK_IN(out, F32);
  const int np = check_parts(out, "sqnorm");
  const c10::DeviceGuard guard(g.device());
  sqnorm_launch(g.data_ptr<float>(), g.numel(), out.data_ptr<float>(), np, (float)scale, cur_stream(), lz_lo, lz_hi);
}

void adamw_step(Tensor p, Tensor g, Tensor m, Tensor v, c10::optional<Tensor> pbf, Tensor sq, Tensor step,
                Tensor hyper, double grad_scale, int64_t zero_hi, int64_t lz_lo, int64_t lz_hi,
                c10::optional<Tensor> lazy_decay) {
  CHECK_IN(p, F32); CHECK_IN(g, F32); CHECK_IN(m, F32); CHECK_IN(v, F32); CHECK_IN(sq, F32); CHECK_IN(step, I64);
  CHECK_IN(hyper, F32);
  const c10::DeviceGuard guard(p.device());
  const int64_t n = p.numel();
  TORCH_CHECK(g.numel() == n && m.numel() == n && v.numel() == n && hyper.numel() >= 8 && step.numel() >= 2,
              "adamw shapes");
  const int np = check_parts(sq, "adamw");
  void* pb = nullptr;
  if (pbf.has_value() && pbf->defined()) {
    CHECK_IN((*pbf), BF16);
    TORCH_CHECK(pbf->numel() == n, "bf16 shadow size");
    pb = pbf->data_ptr();
  }
  float* ld = nullptr;
  if (lazy_decay.has_value() && lazy_decay->defined() && lz_hi > lz_lo) {
    CHECK_IN((*lazy_decay), F32);
    ld = lazy_decay->data_ptr<float>();
  }
  adamw_launch(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), pb, n,
               sq.data_ptr<float>(), np, step.data_ptr<int64_t>(), hyper.data_ptr<float>(), (float)grad_scale,
               cur_stream(), zero_hi, ld ? lz_lo : 0, ld ? lz_hi : 0, ld);
}

void advance_counters(Tensor step, Tensor rng, c10::optional<Tensor> sq) {
  CHECK_IN(step, I64); check_rng(rng);
  const c10::DeviceGuard guard(step.device());
  const float* s = nullptr;
  int np = 0;
  if (sq.has_value() && sq->defined()) {
    CHECK_IN((*sq), F32);
    np = check_parts(*sq, "advance");
    s = sq->data_ptr<float>();
  }
  advance_counters_launch(step.data_ptr<int64_t>(), rng.data_ptr<int64_t>(), s, np, cur_stream());
}

std::tuple<Tensor, Tensor> ddim_step(Tensor x_t, Tensor x0_raw, Tensor coef) {
  CHECK_IN(x_t, F32); CHECK_IN(x0_raw, F32); CHECK_IN(coef, F32);
  const c10::DeviceGuard guard(x_t.device());
  TORCH_CHECK(x_t.numel() == x0_raw.numel() && coef.numel() >= 4, "ddim_step shapes");
  auto xn = at::empty_like(x_t);
  auto x0 = at::empty_like(x_t);
  ddim_step_launch(x_t.data_ptr<float>(), x0_raw.data_ptr<float>(), xn.data_ptr<float>(), x0.data_ptr<float>(),
                   coef.data_ptr<float>(), x_t.numel(), cur_stream());
  return {xn, x0};
}

void ddim_step_(Tensor x, Tensor x0_raw, Tensor x0_out, Tensor coef) {
  CHECK_IN(x, F32); CHECK_IN(x0_raw, F32); CHECK_IN(x0_out, F32); CHECK_IN(coef, F32);
  const c10::DeviceGuard guard(x.device());
  TORCH_CHECK(x.numel() == x0_raw.numel() && x0_out.numel() == x.numel() && coef.numel() >= 4, "ddim_step_ shapes");
  ddim_step_launch(x.data_ptr<float>(), x0_raw.data_ptr<float>(), x.data_ptr<float>(), x0_out.data_ptr<float>(),
                   coef.data_ptr<float>(), x.numel(), cur_stream());
}

void randn_(Tensor out, Tensor rng, int64_t site) {
  CHECK_IN(out, F32); check_rng(rng);
  const c10::DeviceGuard guard(out.device());
  randn_launch(out.data_ptr<float>(), out.numel(), rng.data_ptr<int64_t>(), site, cur_stream());
}

Tensor q_sample(Tensor x0, Tensor t, Tensor eps, int64_t total_steps) {
  CHECK_IN(x0, F32); CHECK_IN(t, I64); CHECK_IN(eps, F32);
  const c10::DeviceGuard guard(x0.device());
  TORCH_CHECK(x0.sizes() == eps.sizes() && t.numel() == x0.size(0), "q_sample shapes");
  auto out = at::empty_like(x0);
  const int B = x0.size(0);
  q_sample_launch(x0.data_ptr<float>(), t.data_ptr<int64_t>(), eps.data_ptr<float>(), out.data_ptr<float>(), B,
                  x0.numel() / B, total_steps, cur_stream());
  return out;
}

std::tuple<Tensor, Tensor> pixelate_pair(Tensor img, c10::optional<Tensor> idx, Tensor t, int64_t B) {
  CHECK_IN(img, F32); CHECK_IN(t, I64);
  const c10::DeviceGuard guard(img.device());
  TORCH_CHECK(img.dim() == 4 && t.numel() == B, "pixelate shapes");
  const int64_t* ip = nullptr;
  if (idx.has_value() && idx->defined()) {
    CHECK_IN((*idx), I64);
    TORCH_CHECK(idx->numel() == B, "idx shape");
    ip = idx->data_ptr<int64_t>();
  } else {
    TORCH_CHECK(img.size(0) == B, "img batch");
  }
  const int C = img.size(1), H = img.size(2), W = img.size(3);
  auto xt = at::empty({B, C, H, W}, img.options());
  auto xtm1 = at::empty({B, C, H, W}, img.options());
  pixelate_pair_launch(img.data_ptr<float>(), ip, t.data_ptr<int64_t>(), xt.data_ptr<float>(), xtm1.data_ptr<float>(),
                       B, C, H, W, cur_stream());
  return {xt, xtm1};
}

// Gaussian DDIM batch (GaussianBatcher): x_t = q_sample(pool[idx], t, eps), x0 = pool[idx]
void gauss_batch(Tensor pool, Tensor rng, int64_t site, int64_t noise_site, int64_t T, Tensor x_t, Tensor x0,
                 Tensor t, Tensor idx, bool draw_idx, c10::optional<Tensor> idx_ctr, int64_t idx_off) {
  CHECK_IN(pool, F32); check_rng(rng); CHECK_IN(x_t, F32); CHECK_IN(x0, F32); CHECK_IN(t, I64); CHECK_IN(idx, I64);
  const c10::DeviceGuard guard(pool.device());
  TORCH_CHECK(x_t.dim() == 4, "gauss_batch: x_t must be [B,C,H,W]");
  const int B = x_t.size(0), C = x_t.size(1), H = x_t.size(2), W = x_t.size(3);
  TORCH_CHECK(pool.dim() == 4 && pool.size(1) == C && pool.size(2) == H && pool.size(3) == W, "pool shape");
  TORCH_CHECK(x0.sizes() == x_t.sizes() && t.numel() == B, "gauss_batch shapes");
  TORCH_CHECK(T >= 1 && (int64_t)B * C * H * W < ((int64_t)1 << 31), "gauss_batch: T / size");
  const IdxSel is = idx_select(idx, idx_ctr, idx_off, B, draw_idx, "gauss_batch");
  gauss_batch_launch(pool.data_ptr<float>(), pool.size(0), rng.data_ptr<int64_t>(), site, noise_site, T,
                     x_t.data_ptr<float>(), x0.data_ptr<float>(), t.data_ptr<int64_t>(), is.p,
                     draw_idx, B, C, H, W, cur_stream(), is.ctr, is.rows, is.stride);
}

void cold_batch(Tensor pool, Tensor rng, int64_t site, Tensor x_t, Tensor x_tm1, Tensor t, Tensor idx_ws,
                int64_t max_t, bool draw_idx, c10::optional<Tensor> idx_ctr, int64_t idx_off) {
  CHECK_IN(pool, F32); check_rng(rng); CHECK_IN(x_t, F32); CHECK_IN(x_tm1, F32); CHECK_IN(t, I64);
  CHECK_IN(idx_ws, I64);
  const c10::DeviceGuard guard(pool.device());
  const int B = x_t.size(0), C = x_t.size(1), H = x_t.size(2), W = x_t.size(3);
  TORCH_CHECK(pool.dim() == 4 && pool.size(1) == C && pool.size(2) == H && pool.size(3) == W, "pool shape");
  TORCH_CHECK(x_tm1.sizes() == x_t.sizes() && t.numel() == B, "cold_batch shapes");
  TORCH_CHECK(max_t >= 1 && (1 << max_t) <= W, "max_t");
  const IdxSel is = idx_select(idx_ws, idx_ctr, idx_off, B, draw_idx, "cold_batch");
  cold_batch_launch(pool.data_ptr<float>(), pool.size(0), rng.data_ptr<int64_t>(), site, x_t.data_ptr<float>(),
                    x_tm1.data_ptr<float>(), t.data_ptr<int64_t>(), is.p, B, C, H, W, max_t,
                    draw_idx, cur_stream(), is.ctr, is.rows, is.stride);
}


// LayerNorm fold weights for a list of GEMMs consuming a LayerNorm (one launch)
void ln_fold_(std::vector<Tensor> ws, std::vector<Tensor> gammas, std::vector<Tensor> betas,
              std::vector<c10::optional<Tensor>> biases, std::vector<Tensor> wfs, std::vector<Tensor> cs,
              std::vector<Tensor> bfs, c10::optional<Tensor> loss_parts, c10::optional<Tensor> loss_last,
              c10::optional<Tensor> loss_ema, double ema_decay, c10::optional<Tensor> step,
              c10::optional<Tensor> rng, c10::optional<Tensor> sq) {
  const size_t n = ws.size();
  TORCH_CHECK(n > 0 && n <= (size_t)FOLD_MAX, "ln_fold_: 1..", FOLD_MAX, " GEMMs per launch");
  TORCH_CHECK(gammas.size() == n && betas.size() == n && biases.size() == n && wfs.size() == n && cs.size() == n &&
                  bfs.size() == n, "ln_fold_: list lengths");
  const c10::DeviceGuard guard(ws[0].device());
  FoldTable tb{};
  tb.n = (int)n;
  tb.K = ws[0].size(-1);
  TORCH_CHECK(tb.K % 4 == 0, "ln_fold_: K % 4");
  int rows = 0;
  tb.w_bf16 = ws[0].scalar_type() == BF16 ? 1 : 0;
  for (size_t i = 0; i < n; ++i) {
    CHECK_IN(ws[i], (tb.w_bf16 ? BF16 : F32)); CHECK_IN(gammas[i], F32); CHECK_IN(betas[i], F32);
    CHECK_IN(wfs[i], BF16); CHECK_IN(cs[i], F32); CHECK_IN(bfs[i], F32);
    TORCH_CHECK(ws[i].dim() == 2 && ws[i].size(1) == tb.K, "ln_fold_: weights must be [rows, K] with one K");
    const int R = ws[i].size(0);
    TORCH_CHECK(gammas[i].numel() == tb.K && betas[i].numel() == tb.K && wfs[i].numel() == (int64_t)R * tb.K &&
                    cs[i].numel() == R && bfs[i].numel() == R, "ln_fold_: shapes");
    for (const Tensor* t : {&ws[i], &gammas[i], &betas[i]})
      TORCH_CHECK(((uintptr_t)t->data_ptr() & 15) == 0, "ln_fold_: 16-B aligned operands");
    TORCH_CHECK(((uintptr_t)wfs[i].data_ptr() & 7) == 0, "ln_fold_: 8-B aligned output");
    FoldJob& j = tb.j[i];
    j.w = ws[i].data_ptr(); j.gamma = gammas[i].data_ptr<float>(); j.beta = betas[i].data_ptr<float>();
    j.bias = nullptr;
    if (biases[i].has_value() && biases[i]->defined()) {
      CHECK_IN((*biases[i]), F32);
      TORCH_CHECK(biases[i]->numel() == R, "ln_fold_: bias shape");
      j.bias = biases[i]->data_ptr<float>();
    }
    j.wf = wfs[i].data_ptr(); j.c = cs[i].data_ptr<float>(); j.bf = bfs[i].data_ptr<float>();
    tb.start[i] = rows;
    rows += R;
  }
  tb.start[n] = rows;
  if (step.has_value() && step->defined()) {  // training-step tail in the same launch
    CHECK_IN((*step), I64); check_rng(*rng);
    TORCH_CHECK(loss_parts.has_value() && loss_parts->defined() && sq.has_value() && sq->defined(),
                "step tail needs loss_parts and sq");
    CHECK_IN((*loss_parts), F32); CHECK_IN((*sq), F32);
    tb.sq_n = check_parts(*sq, "ln_fold_ tail");
    tb.tail = 1;
    tb.loss_parts = loss_parts->data_ptr<float>();
    tb.loss_nparts = (int)loss_parts->numel();
    if (loss_last.has_value() && loss_last->defined()) { CHECK_IN((*loss_last), F32); tb.loss_last = loss_last->data_ptr<float>(); }
    if (loss_ema.has_value() && loss_ema->defined()) { CHECK_IN((*loss_ema), F32); tb.loss_ema = loss_ema->data_ptr<float>(); }
    tb.ema_decay = (float)ema_decay;
    tb.step = step->data_ptr<int64_t>();
    tb.rng = rng->data_ptr<int64_t>();
    tb.sq = sq->data_ptr<float>();
  }
  ln_fold_launch(tb, cur_stream());
}

}  // namespace

TORCH_LIBRARY(ddim_cold, m) {
  m.def("patch_embed_fwd(Tensor img, Tensor t, Tensor w_pe, Tensor b_pe, Tensor cls, Tensor pos, Tensor temb, "
        "Tensor rng, int site, float p, int patch, Tensor(a!)? ln_st=None, Tensor(b!)? xb_out=None, "
        "Tensor? patches_in=None) -> (Tensor, Tensor)");
  m.def("layernorm_fwd(Tensor x, Tensor gamma, Tensor beta, float eps) -> (Tensor, Tensor, Tensor)");
  m.def("qkv_fwd(Tensor a, Tensor w, Tensor b, int B, int N, int H, Tensor? ln_st=None, Tensor? ln_c=None, "
        "float ln_eps=1e-5, Tensor(a!)? ln_mean=None, Tensor(b!)? ln_rstd=None) -> Tensor");
  m.def("attn_fwd(Tensor qkv, float scale, Tensor rng, int site, float p, Tensor? keep_out=None) -> (Tensor, Tensor)");
  m.def("attn_keep_words(int B, int H, int N, int hd) -> int", &attn_keep_words_op);
  m.def("gemm_tile_override(int cfg) -> int", &gemm_tile_override_op);
  m.def("gemm_stamps(Tensor? buf) -> ()", &gemm_stamps_op);
  m.def("linear_residual_fwd(Tensor a, Tensor w, Tensor b, Tensor x, int N, Tensor rng, int site_drop, "
        "float p_drop, int site_dp, float p_dp, Tensor(a!)? st_out=None, Tensor(b!)? xb_out=None) -> Tensor");
  m.def("linear_gelu_fwd(Tensor a, Tensor w, Tensor b, Tensor rng, int site, float p, Tensor? ln_st=None, "
        "Tensor? ln_c=None, float ln_eps=1e-5, Tensor(a!)? ln_mean=None, Tensor(b!)? ln_rstd=None) -> (Tensor, Tensor)");
  m.def("linear_fwd(Tensor a, Tensor w, Tensor? b, bool out_fp32, Tensor? ln_st=None, Tensor? ln_c=None, "
        "float ln_eps=1e-5) -> Tensor");
  m.def("head_fwd(Tensor a, Tensor w, Tensor b, int B, int C, int H, int W, int patch, Tensor? ln_st=None, "
        "Tensor? ln_c=None, float ln_eps=1e-5, Tensor(a!)? ln_mean=None, Tensor(b!)? ln_rstd=None) -> Tensor");
  m.def("head_step_(Tensor a, Tensor w, Tensor b, Tensor(a!) x, Tensor(b!)? x0_out, Tensor? coef, int patch, "
        "int mode, Tensor? ln_st=None, Tensor? ln_c=None, float ln_eps=1e-5, Tensor(c!)? patches_out=None) -> ()");
  m.def("head_step_rows_(Tensor a, Tensor w, Tensor b, Tensor(a!) x, Tensor(b!)? x0_out, Tensor? coef, int batch, "
        "int mode, Tensor? ln_st=None, Tensor? ln_c=None, float ln_eps=1e-5, Tensor(c!)? patches_out=None) -> ()");
  m.def("head_loss(Tensor a, Tensor w, Tensor b, Tensor target, int patch, float beta, Tensor? ln_st=None, "
        "Tensor? ln_c=None, float ln_eps=1e-5, Tensor(a!)? ln_mean=None, Tensor(b!)? ln_rstd=None, "
        "bool target_rows=False) -> (Tensor, Tensor)");
  m.def("smooth_l1_fwd_bwd(Tensor pred, Tensor target, int N, int patch, float beta, Tensor(a!)? loss_last=None, "
        "Tensor(b!)? loss_ema=None, float ema_decay=0.99, bool finish=True) -> (Tensor, Tensor)");
  m.def("img_to_tokgrad(Tensor dimg, int N, int patch) -> Tensor");
  m.def("linear_dgrad(Tensor dy, Tensor w, bool out_fp32, int splits=1) -> Tensor");
  m.def("linear_dgrad_gelu(Tensor dy, Tensor w, Tensor u, Tensor rng, int site, float p) -> Tensor");
  m.def("linear_dgrad_gelu_t(Tensor dy, Tensor wt, Tensor u, Tensor rng, int site, float p) -> Tensor");
  m.def("linear_wgrad(Tensor dy, Tensor x, Tensor(a!) dw, Tensor(b!)? db) -> ()");
  m.def("wire_pack(Tensor src, Tensor(a!) dst) -> ()");
  m.def("wire_unpack(Tensor src, Tensor(a!) dst) -> ()");
  m.def("linear_wgrad_multi(Tensor[] dys, Tensor[] xs, Tensor(a!)[] dws, Tensor(b!)?[] dbs, bool store=False, "
        "Tensor(c!)? sq_parts=None, Tensor? arena=None, int lz_lo=0, int lz_hi=0, Tensor? emb_g=None, "
        "Tensor? emb_t=None, Tensor? emb_rng=None, int emb_site=0, float emb_p=0.0, Tensor(d!)? emb_cls=None, "
        "Tensor(e!)? emb_pos=None, Tensor(f!)? emb_temb=None, int emb_owners=0, Tensor? ln_ws=None, "
        "Tensor? ln_ptrs=None, int[] ln_offs=[], int ln_C=0, int ln_R=0, bool ln_store=False) -> ()");
  m.def("wgrad_embed_slots(int B, int N, int D, int owners, int n_ln, int ln_C, bool wide) -> int", &wgrad_embed_slots);
  m.def("layernorm_bwd(Tensor dy, Tensor x, Tensor mean, Tensor rstd, Tensor gamma, Tensor? g_res, "
        "Tensor(a!) dgamma, Tensor(b!) dbeta, int N, Tensor rng, int site_drop, float p_drop, int site_dp, "
        "float p_dp, bool emit_gy, Tensor(c!)? ws=None, Tensor? beta=None, Tensor(d!)? y_out=None, "
        "Tensor(e!)? gp_out=None, int site_emb=0, float p_emb=0.0) -> (Tensor, Tensor)");
  m.def("replica_reduce_(Tensor ws, Tensor dst_ptrs, int C, int R) -> ()");
  m.def("ln_ws_rows(int M) -> int", &ln_ws_rows_op);
  m.def("transpose_bf16_(Tensor[] srcs, Tensor(a!)[] dsts) -> ()");
  m.def("ln_fold_(Tensor[] ws, Tensor[] gammas, Tensor[] betas, Tensor?[] biases, Tensor(a!)[] wfs, Tensor(b!)[] cs, "
        "Tensor(c!)[] bfs, Tensor? loss_parts=None, Tensor(d!)? loss_last=None, Tensor(e!)? loss_ema=None, "
        "float ema_decay=0.99, Tensor(f!)? step=None, Tensor(g!)? rng=None, Tensor? sq=None) -> ()");
  m.def("attn_bwd(Tensor dout, Tensor qkv, Tensor o, Tensor lse, float scale, Tensor rng, int site, float p, "
        "Tensor? keep=None) -> Tensor");
  m.def("embed_bwd(Tensor g, Tensor t, Tensor rng, int site, float p, Tensor(a!) dcls, Tensor(b!) dpos, "
        "Tensor(c!) dtemb, Tensor? ln_ws=None, Tensor? ln_ptrs=None, int ln_C=0, bool ln_store=False, int ln_R=0) -> Tensor");
  m.def("sqnorm(Tensor g, Tensor(a!) out, float scale, int lz_lo=0, int lz_hi=0) -> ()");
  m.def("adamw_step(Tensor(a!) p, Tensor(b!) g, Tensor(c!) m, Tensor(d!) v, Tensor(e!)? pbf, Tensor sq, "
        "Tensor step, Tensor hyper, float grad_scale, int zero_hi=-1, int lz_lo=0, int lz_hi=0, "
        "Tensor(f!)? lazy_decay=None) -> ()");
  m.def("advance_counters(Tensor(a!) step, Tensor(b!) rng, Tensor? sq) -> ()");
  m.def("ddim_step(Tensor x_t, Tensor x0_raw, Tensor coef) -> (Tensor, Tensor)");
  m.def("ddim_step_(Tensor(a!) x, Tensor x0_raw, Tensor(b!) x0_out, Tensor coef) -> ()");
  m.def("randn_(Tensor(a!) out, Tensor rng, int site) -> ()");
  m.def("q_sample(Tensor x0, Tensor t, Tensor eps, int total_steps) -> Tensor");
  m.def("pixelate_pair(Tensor img, Tensor? idx, Tensor t, int B) -> (Tensor, Tensor)");
  m.def("cold_batch(Tensor pool, Tensor rng, int site, Tensor(a!) x_t, Tensor(b!) x_tm1, Tensor(c!) t, "
        "Tensor(d!) idx_ws, int max_t, bool draw_idx=True, Tensor? idx_ctr=None, int idx_off=0) -> ()");
  m.def("patch_embed_cold_fwd(Tensor pool, int data_site, int max_t, bool draw_idx, bool target_x0, "
        "Tensor(a!) img, Tensor(b!) target, Tensor(c!) t, Tensor(d!) idx, bool write_xt, Tensor w_pe, Tensor b_pe, "
        "Tensor cls, Tensor pos, Tensor temb, Tensor rng, int site, float p, int patch, Tensor(e!)? ln_st=None, "
        "Tensor(f!)? xb_out=None, int gauss_T=0, int noise_site=0, bool target_rows=False, Tensor? idx_ctr=None, "
        "int idx_off=0) -> (Tensor, Tensor)");
  m.def("gauss_batch(Tensor pool, Tensor rng, int site, int noise_site, int T, Tensor(a!) x_t, Tensor(b!) x0, "
        "Tensor(c!) t, Tensor(d!) idx, bool draw_idx=True, Tensor? idx_ctr=None, int idx_off=0) -> ()");
}

TORCH_LIBRARY_IMPL(ddim_cold, CUDA, m) {
  m.impl("patch_embed_fwd", &patch_embed_fwd);
  m.impl("patch_embed_cold_fwd", &patch_embed_cold_fwd);
  m.impl("layernorm_fwd", &layernorm_fwd);
  m.impl("qkv_fwd", &qkv_fwd);
  m.impl("attn_fwd", &attn_fwd);
  m.impl("linear_residual_fwd", &linear_residual_fwd);
  m.impl("linear_gelu_fwd", &linear_gelu_fwd);
  m.impl("head_fwd", &head_fwd);
  m.impl("smooth_l1_fwd_bwd", &smooth_l1_fwd_bwd);
  m.impl("head_loss", &head_loss);
  m.impl("img_to_tokgrad", &img_to_tokgrad);
  m.impl("linear_dgrad", &linear_dgrad);
  m.impl("linear_dgrad_gelu", &linear_dgrad_gelu);
  m.impl("linear_dgrad_gelu_t", &linear_dgrad_gelu_t);
  m.impl("linear_wgrad", &linear_wgrad);
  m.impl("head_step_", &head_step_);
  m.impl("head_step_rows_", &head_step_rows_);
  m.impl("linear_fwd", &linear_fwd);
  m.impl("linear_wgrad_multi", &linear_wgrad_multi);
  m.impl("wire_pack", &wire_pack);
  m.impl("wire_unpack", &wire_unpack);
  m.impl("layernorm_bwd", &layernorm_bwd);
  m.impl("replica_reduce_", &replica_reduce_);
  m.impl("transpose_bf16_", &transpose_bf16_);
  m.impl("ln_fold_", &ln_fold_);
  m.impl("attn_bwd", &attn_bwd);
  m.impl("embed_bwd", &embed_bwd);
  m.impl("sqnorm", &sqnorm);
  m.impl("adamw_step", &adamw_step);
  m.impl("advance_counters", &advance_counters);
  m.impl("ddim_step", &ddim_step);
  m.impl("ddim_step_", &ddim_step_);
  m.impl("randn_", &randn_);
  m.impl("q_sample", &q_sample);
  m.impl("pixelate_pair", &pixelate_pair);
  m.impl("cold_batch", &cold_batch);
  m.impl("gauss_batch", &gauss_batch);
}
