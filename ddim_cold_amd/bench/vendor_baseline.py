"""Same-node vendor-library comparators: the reference's training step and DDIM
sampler built from stock PyTorch-ROCm ops (hipBLASLt GEMMs via ``nn.Linear``,
MIOpen conv, ATen LayerNorm / GELU / dropout, ``F.scaled_dot_product_attention``,
fused ``torch.optim.AdamW``) and captured WHOLE in one ``torch.cuda.CUDAGraph``
(a hipGraph on ROCm).  Python dispatch and launch gaps are therefore gone from
these numbers too: what remains is the vendor kernels themselves, which is the
comparison the hand-written stack has to win.

* :class:`VendorTrainStep` — `multi_gpu_trainer.py:115-134` as one graph: an
  on-device cold batch draw (pool index + t ~ U{1..log2 W} + NEAREST pixelation
  pair, `diffusion_loader.py:79-97`, in plain torch ops), forward under bf16
  autocast (the patch embedding as one GEMM: :func:`_patch_gemm`),
  ``F.smooth_l1_loss`` (mean as a GEMV; bias gradients as GEMMs: :class:`_AddBias`),
  backward, ``clip_grad_norm_(1.0)``,
  ``AdamW(wd=0.05, fused=True, capturable=True)`` with the per-iteration cosine
  LR computed on the device (``CosineAnnealingLR``'s closed form, eta_min 0).
* :class:`VendorSampler` — the 100-step k=20 DDIM loop of `ViT.py:220-237`
  (bf16 autocast forward, fp32 clamp / eps-hat / update) unrolled into one graph.
* :class:`VendorImg2Img` — the draft->drawing call of `ViT_draft2drawing.py:389-409`
  with the same batching as the fused path (all 9 t_starts in ONE batch on the
  shared k=10 grid, per-sample coefficients, a not-yet-started sample kept by an
  identity row) unrolled into one graph: the batched vendor counterpart of
  :func:`ddim_cold_amd.diffusion.samplers.img2img`, so the ratio measures kernels,
  not batching or dispatch.

``attn="sdpa"`` (default) runs attention through ``F.scaled_dot_product_attention``
(the ROCm flash / memory-efficient kernels); ``attn="explicit"`` through the
reference's materialised softmax (``Attention.forward``).  Everything runs
eagerly on the CPU (``use_graph=False``) for the plumbing tests.
"""
from __future__ import annotations

import math
import time
from typing import Optional

import torch
import torch.nn.functional as F


def vendor_forward(model, x: torch.Tensor, t: torch.Tensor, attn: str = "sdpa", patch: str = "conv") -> torch.Tensor:
    """``model.forward_reference`` with the attention core as
    ``F.scaled_dot_product_attention`` (``attn='sdpa'``); same parameters, same
    dropout / drop-path semantics in train mode (`ViT.py:105-137`, `:199-218`).
    Linear layers go through :func:`_linear` (bias gradient as a GEMM)."""
    if attn == "explicit":
        return model.forward_reference(x, t)
    tr = model.training
    h = _tokens(model, x, t, patch)
    for blk in model.blocks:
        a = blk.attn
        B, N, C = h.shape
        H = a.num_heads
        qkv = _linear(a.qkv, blk.norm1(h)).view(B, N, 3, H, C // H).permute(2, 0, 3, 1, 4)
        p = a.attn_drop.p if tr else 0.0
        y = F.scaled_dot_product_attention(qkv[0], qkv[1], qkv[2], dropout_p=p, scale=a.scale)
        y = y.transpose(1, 2).reshape(B, N, C)
        h = h + blk.drop_path(_drop(_linear(a.proj, y), a.proj_drop.p, tr))
        m = blk.mlp
        z = _linear(m.fc2, _drop(m.act(_linear(m.fc1, blk.norm2(h))), m.drop.p, tr))
        h = h + blk.drop_path(_drop(z, m.drop.p, tr))
    return model.unpatchify(_linear(model.head, model.norm(h))[:, 1:, :])


class _AddBias(torch.autograd.Function):
    """y = x + b (b broadcast over the rows) whose bias gradient is a GEMM, ones^T dy,
    instead of ATen's column reduction.  Captured in one graph with the stock
    reductions (``nn.Linear`` bias gradients, ``F.smooth_l1_loss``'s mean), the step
    read stale or garbage reduction outputs from the second replay on: negative
    "smooth-L1 losses" from replay 2, NaN parameters after ~20 back-to-back replays,
    while the same step run eagerly trained normally (tools/vendor_debug.py; a lone
    1M-element ``x.sum()`` graph does replay correctly, so it is specific to the
    reductions of the step).  With the bias gradients and the loss mean as GEMMs
    the graph-replayed step tracks the eager one (loss 0.03-0.045 over 300 replays,
    every parameter finite)."""

    @staticmethod
    def forward(ctx, x, b):
        ctx.bshape, ctx.bdtype = b.shape, b.dtype
        return x + b.to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        g2 = g.reshape(-1, g.shape[-1]).float()
        ones = torch.ones(1, g2.shape[0], device=g.device, dtype=torch.float32)
        return g, (ones @ g2).reshape(ctx.bshape).to(ctx.bdtype)


def _linear(mod, x, weight=None):
    """``nn.Linear`` forward (same weight / bias, bf16 under autocast) with the bias
    gradient of :class:`_AddBias`."""
    y = F.linear(x, mod.weight if weight is None else weight)
    return _AddBias.apply(y, mod.bias) if mod.bias is not None else y


def _mean(x: torch.Tensor) -> torch.Tensor:
    """Mean as a GEMV (replays correctly inside a captured graph, see :class:`_AddBias`)."""
    flat = x.reshape(1, -1)
    ones = torch.ones(flat.shape[1], 1, device=x.device, dtype=x.dtype)
    return (flat @ ones).reshape(()) * (1.0 / flat.shape[1])


def _drop(x, p, training):
    """Dropout as Bernoulli(1-p) keep mask (fp32 uniform < 1-p) and 1/(1-p) scaling.
    Not ``F.dropout``: its bf16 kernel inside a captured graph (PyTorch 2.10 / ROCm
    7) turned the replayed training step NaN after ~12 replays, with fp32 inputs or
    this form it does not (tools/vendor_debug.py bisection).  Costs the vendor step
    one uniform-draw launch per dropout site over the native fused kernel."""
    if not training or p == 0.0:
        return x
    keep = 1.0 - p
    return x * ((torch.rand(x.shape, device=x.device) < keep).to(x.dtype) * (1.0 / keep))


def _patch_gemm(model, x):
    """The patch embedding's stride-p convolution as im2col rows times the reshaped conv
    weight (one GEMM, same values as ``nn.Conv2d`` up to summation order).  The training
    comparator uses it (``VendorTrainStep(patch="gemm")``): with the MIOpen convolution
    the graph-replayed oxford_flower (p=4) step turned its parameters NaN in some runs and
    not others (tools/vendor_debug.py patch: conv 81 non-finite tensors after 220
    replays in one run, finite in the next; the GEMM form finite and bit-identical with
    and without host syncs between replays)."""
    pe = model.patch_embed
    p = pe.patch_size
    B, C, H, W = x.shape
    rows = x.reshape(B, C, H // p, p, W // p, p).permute(0, 2, 4, 1, 3, 5).reshape(B, -1, C * p * p)
    return _linear(pe.proj, rows, weight=pe.proj.weight.reshape(pe.proj.weight.shape[0], -1))


def _tokens(model, x, t, patch="conv"):
    """``prepare_tokens`` (`ViT.py:199-206`) with the pos_drop through :func:`_drop`."""
    B = x.shape[0]
    tok = model.patch_embed(x) if patch == "conv" else _patch_gemm(model, x)
    tok = torch.cat((model.cls_token.expand(B, -1, -1).to(tok.dtype), tok), dim=1)
    return _drop(tok + model.pos_embed + model.time_embed(t).unsqueeze(1), model.pos_drop.p, model.training)


def cold_batch_torch(pool: torch.Tensor, batch: int, max_t: int):
    """(x_t, x_{t-1}, t) with t ~ U{1..max_t}: x_s[h, w] = img[2^s floor(h / 2^s), 2^s floor(w / 2^s)]
    (NEAREST down to W / 2^s then NEAREST up, `diffusion_loader.py:79-83`), in plain
    torch ops on ``pool``'s device (graph-capturable with the default generator)."""
    dev = pool.device
    P, C, H, W = pool.shape
    idx = torch.randint(0, P, (batch,), device=dev)
    t = torch.randint(1, max_t + 1, (batch,), device=dev)
    img = pool.index_select(0, idx)
    bi = torch.arange(batch, device=dev)[:, None, None]
    ar_h = torch.arange(H, device=dev)[None, :]
    ar_w = torch.arange(W, device=dev)[None, :]

    def pix(s):
        f = (1 << s)[:, None]
        rows = (ar_h // f) * f  # [B, H]
        cols = (ar_w // f) * f  # [B, W]
        return img.permute(0, 2, 3, 1)[bi, rows[:, :, None], cols[:, None, :]].permute(0, 3, 1, 2)

    return pix(t), pix(t - 1), t


class VendorTrainStep:
    """The reference training step from stock PyTorch-ROCm ops, captured whole."""

    def __init__(self, model, pool: torch.Tensor, batch: int, lr: float, t_max: int, attn: str = "sdpa",
                 weight_decay: float = 0.05, clip: float = 1.0, use_graph: bool = True, patch: str = "gemm"):
        self.model = model.train()
        self.patch = patch
        self.pool = pool
        self.batch = batch
        self.attn = attn
        self.clip = clip
        self.max_t = int(math.log2(model.img_size[1]))
        dev = pool.device
        self.dev = dev
        self.cuda = dev.type == "cuda"
        self.params = [p for p in model.parameters() if p.requires_grad]
        self.base_lr = lr
        self.t_max = t_max
        self.lr_t = torch.tensor(lr, dtype=torch.float32, device=dev)
        self.step_t = torch.zeros((), dtype=torch.float32, device=dev)
        kw = dict(lr=self.lr_t, weight_decay=weight_decay)
        self.optimizer_kind = "fused"
        if self.cuda:
            try:
                self.opt = torch.optim.AdamW(self.params, fused=True, capturable=True, **kw)
            except (RuntimeError, ValueError):
                self.opt = torch.optim.AdamW(self.params, foreach=True, capturable=True, **kw)
                self.optimizer_kind = "foreach-capturable"
        else:
            self.opt = torch.optim.AdamW(self.params, lr=lr, weight_decay=weight_decay)
            self.optimizer_kind = "cpu"
        self.loss = torch.zeros((), device=dev)
        self.use_graph = use_graph and self.cuda
        self.graph: Optional[torch.cuda.CUDAGraph] = None

    def _body(self):
        x_t, target, t = cold_batch_torch(self.pool, self.batch, self.max_t)
        with torch.autocast(self.dev.type, dtype=torch.bfloat16, enabled=self.cuda, cache_enabled=False):
            pred = vendor_forward(self.model, x_t, t, self.attn, self.patch)
        loss = _mean(F.smooth_l1_loss(pred.float(), target, reduction="none"))
        loss.backward()
        torch.nn.utils.clip_grad_norm_(self.params, self.clip)
        if self.cuda:
            # CosineAnnealingLR(T_max, eta_min=0) stepped per iteration, on the device
            self.lr_t.copy_(0.5 * self.base_lr * (1 + torch.cos(math.pi * self.step_t / self.t_max)))
        else:
            for g in self.opt.param_groups:
                g["lr"] = 0.5 * self.base_lr * (1 + math.cos(math.pi * float(self.step_t) / self.t_max))
        self.opt.step()
        self.step_t += 1
        self.loss.copy_(loss.detach())

    def _eager(self):
        self.opt.zero_grad(set_to_none=True)
        self._body()

    def capture(self, warm: int = 3):
        s = torch.cuda.Stream(self.dev)
        s.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(s):
            for _ in range(warm):
                self._eager()
        torch.cuda.current_stream(self.dev).wait_stream(s)
        torch.cuda.synchronize(self.dev)
        self.opt.zero_grad(set_to_none=True)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._body()
        self.graph = g

    def steps(self, n: int):
        if self.use_graph:
            if self.graph is None:
                self.capture()
            for _ in range(n):
                self.graph.replay()
        else:
            for _ in range(n):
                self._eager()


class VendorSampler:
    """DDIM k-step sampler (`ViT.py:220-237`) from stock ops, all steps in one graph;
    x_T drawn on the device, result returned on the host in [0, 1]."""

    def __init__(self, model, N: int, k: int, attn: str = "sdpa", use_graph: bool = True):
        T = model.total_steps
        if T % k != 0:
            raise ValueError(f"k={k} must divide total_steps={T}")
        self.model = model.eval()
        self.dev = next(model.parameters()).device
        self.cuda = self.dev.type == "cuda"
        self.N, self.k, self.attn = N, k, attn
        C, (H, W) = model.in_chans, model.img_size
        self.ts = list(range(T - 1, 0, -k))
        self.x_in = torch.empty(N, C, H, W, device=self.dev)
        self.out = torch.empty(N, C, H, W, device=self.dev)
        self.tt = [torch.full((N,), t, dtype=torch.int64, device=self.dev) for t in self.ts]
        self.use_graph = use_graph and self.cuda
        self.graph = None

    @torch.no_grad()
    def _body(self):
        T, k = self.model.total_steps, self.k
        x = self.x_in
        x0 = x
        for i, t in enumerate(self.ts):
            with torch.autocast(self.dev.type, dtype=torch.bfloat16, enabled=self.cuda, cache_enabled=False):
                x0 = vendor_forward(self.model, x, self.tt[i], self.attn)
            x0 = torch.clamp(x0.float(), -1.0, 1.0)
            a_tk = 1 - math.sqrt((t + 1 - k) / T)
            a_t = 1 - math.sqrt((t + 1) / T) + 1e-5
            eps = (x - math.sqrt(a_t) * x0) / math.sqrt(1 - a_t)
            x = math.sqrt(a_tk) * (x / math.sqrt(a_t) + (math.sqrt((1 - a_tk) / a_tk) - math.sqrt((1 - a_t) / a_t)) * eps)
        self.out.copy_((x0 + 1) / 2)

    def capture(self):
        s = torch.cuda.Stream(self.dev)
        s.wait_stream(torch.cuda.current_stream(self.dev))
        self.x_in.normal_()
        with torch.cuda.stream(s):
            self._body()
        torch.cuda.current_stream(self.dev).wait_stream(s)
        torch.cuda.synchronize(self.dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._body()
        self.graph = g

    @torch.no_grad()
    def sample(self, generator=None) -> torch.Tensor:
        if self.use_graph and self.graph is None:
            self.capture()  # (draws a scratch x_T of its own for the warm-up)
        self.x_in.normal_(generator=generator)
        if self.use_graph:
            self.graph.replay()
        else:
            self._body()
        return self.out.cpu()


class VendorImg2Img:
    """Batched draft->drawing DDIM loop from stock ops, all steps in one graph: sample i
    joins the shared descending k-grid at ``starts[i]`` (identity coefficients before
    that, :func:`ddim_cold_amd.diffusion.samplers.starts_table`); per step a bf16
    autocast forward, fp32 clamp, eps-hat and update with per-sample coefficients."""

    def __init__(self, model, starts, k: int = 10, attn: str = "sdpa", use_graph: bool = True):
        from ..diffusion.samplers import starts_table
        self.model = model.eval()
        self.dev = next(model.parameters()).device
        self.cuda = self.dev.type == "cuda"
        self.starts, self.k, self.attn = list(starts), k, attn
        B = len(self.starts)
        C, (H, W) = model.in_chans, model.img_size
        self.ts, coef = starts_table(model.total_steps, self.starts, k)
        self.coef = coef.to(self.dev).view(len(self.ts), B, 4, 1, 1, 1)
        self.tt = [torch.full((B,), t, dtype=torch.int64, device=self.dev) for t in self.ts]
        self.x_in = torch.zeros(B, C, H, W, device=self.dev)
        self.out = torch.empty(B, C, H, W, device=self.dev)
        self.use_graph = use_graph and self.cuda
        self.graph = None

    @torch.no_grad()
    def _body(self):
        x = self.x_in
        x0 = x
        for i in range(len(self.ts)):
            with torch.autocast(self.dev.type, dtype=torch.bfloat16, enabled=self.cuda, cache_enabled=False):
                x0 = vendor_forward(self.model, x, self.tt[i], self.attn)
            x0 = torch.clamp(x0.float(), -1.0, 1.0)
            c = self.coef[i]
            eps = (x - c[:, 0] * x0) / c[:, 1]
            x = c[:, 2] * x0 + c[:, 3] * eps
        self.out.copy_((x0 + 1) / 2)

    def capture(self):
        s = torch.cuda.Stream(self.dev)
        s.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(s):
            self._body()
        torch.cuda.current_stream(self.dev).wait_stream(s)
        torch.cuda.synchronize(self.dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._body()
        self.graph = g

    @torch.no_grad()
    def __call__(self, draft: torch.Tensor, generator=None) -> torch.Tensor:
        """One call as :func:`samplers.img2img` makes it: eps drawn on the host, the
        noised starts formed on the device, the loop, the result on the host in [0, 1]."""
        from ..diffusion.samplers import img2img_noised
        B = len(self.starts)
        C, (H, W) = self.model.in_chans, self.model.img_size
        eps = torch.normal(0.0, 1.0, (B, C, H, W), generator=generator).to(self.dev)
        d = draft.to(self.dev).float()
        d = d.unsqueeze(0) if d.dim() == 3 else d
        self.x_in.copy_(img2img_noised(d.expand(B, -1, -1, -1), eps, self.starts, self.model.total_steps))
        if self.use_graph:
            if self.graph is None:
                self.capture()
            self.graph.replay()
        else:
            self._body()
        return self.out.cpu()


def time_vendor_img2img(model, starts, k: int = 10, reps: int = 5, attn: str = "sdpa") -> float:
    """Seconds per draft->drawing call of the graph-captured batched vendor loop."""
    was = model.training
    try:
        v = VendorImg2Img(model, starts, k, attn=attn)
        g = torch.Generator().manual_seed(0)
        C, (H, W) = model.in_chans, model.img_size
        draft = torch.rand(1, C, H, W, generator=g) * 2 - 1
        v(draft, g)  # capture
        torch.cuda.synchronize(v.dev)
        t0 = time.perf_counter()
        for _ in range(reps):
            v(draft, g)
        torch.cuda.synchronize(v.dev)
        return (time.perf_counter() - t0) / reps
    finally:
        model.train(was)


def time_vendor_train(model, pool, batch: int, lr: float, t_max: int, steps: int = 50, warmup: int = 10,
                      attn: str = "sdpa"):
    """(seconds per step, final loss, optimizer kind) of the graph-captured vendor step."""
    v = VendorTrainStep(model, pool, batch, lr, t_max, attn=attn)
    v.steps(warmup)
    torch.cuda.synchronize(v.dev)
    t0 = time.perf_counter()
    v.steps(steps)
    torch.cuda.synchronize(v.dev)
    dt = (time.perf_counter() - t0) / steps
    return dt, float(v.loss.item()), v.optimizer_kind


def time_vendor_sampler(model, N: int, k: int, reps: int = 5, attn: str = "sdpa") -> float:
    """Seconds per N-image batch of the graph-captured vendor DDIM sampler."""
    was = model.training
    try:
        s = VendorSampler(model, N, k, attn=attn)
        g = torch.Generator(device=s.dev).manual_seed(0)
        s.sample(g)  # capture
        torch.cuda.synchronize(s.dev)
        t0 = time.perf_counter()
        for _ in range(reps):
            s.sample(g)
        torch.cuda.synchronize(s.dev)
        return (time.perf_counter() - t0) / reps
    finally:
        model.train(was)
