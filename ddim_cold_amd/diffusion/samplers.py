"""Samplers: DDIM k-step (+ trajectory), cold de-pixelation, draft->drawing img2img.

Reference behaviour: ``ViT.py:220-256`` (DDIM sampler / sequence),
``ViT_draft2drawing.py:259-309`` (cold sampler / sequence),
``ViT_draft2drawing.py:378-419`` (img2img).

MI355X design: the reference issues one H2D timestep copy, ~150 forward
kernels and ~8 elementwise DDIM kernels per step from Python and syncs with a
D2H copy per recorded step.  Here the *whole* sampling loop is captured once
as a hipGraph (static noise buffer, device-resident timestep and coefficient
tables, the fused ``ddim_step_`` kernel doing clamp + eps-hat + update in one
fp32 pass, trajectory written to a device buffer and copied back once), so a
replay is a single host call.  Graphs are cached per (N, k) and re-captured
if the weights they read were reallocated.

Sampling always runs the denoiser in eval mode (no dropout); the reference's
``ViT.py`` CLI forgot ``model.eval()``.

Every step is ONE forward whose head-GEMM epilogue applies the step (DDIM
update, cold clamp, or img2img's DDIM update with per-sample coefficients) and
hands the next step its bf16 patch rows.  (Splitting a batch into concurrent
chains on separate streams measured slower on MI355X -- ViT-tiny N=64 k=20:
46.9 / 56.2 / 76.2 ms for 1 / 2 / 4 chains -- and was removed.)
"""
from __future__ import annotations

import math
import os
import time
from typing import List, Optional, Sequence

import torch

from .. import ops
from .schedule import cold_steps, ddim_coefficients, ddim_table, img2img_alpha


def _use_fused(model, device) -> bool:
    from ..models.vit import _fused_allowed
    probe = torch.empty(0, device=device)
    return _fused_allowed(probe)


class _Denoiser:
    """x0-prediction f(x, t) in eval mode via the fused program (GPU) or the reference (CPU)."""

    def __init__(self, model, device):
        self.model = model
        self.device = torch.device(device)
        self.fused = _use_fused(model, self.device)
        if self.fused:
            from ..models.program import model_tensors
            self.prog = model.program()
            self.P = model_tensors(model)
            self.rng = torch.zeros(2, dtype=torch.int64, device=self.device)

    def key(self):
        return self.key_of(self.model)

    @staticmethod
    def key_of(model):
        """What a captured loop depends on: the engine whose arenas it reads, or the
        parameters' storage + version (checked per call before any denoiser is built:
        building one costs ~0.25 ms of host time)."""
        eng = getattr(model, "_engine", None)
        if eng is not None:
            return ("engine", id(eng))
        return tuple((p.data_ptr(), p._version) for p in model.parameters())

    def step_(self, x, t, mode: int, x0_out=None, coef=None, patches=None):
        """In-place sampler step on ``x`` with the update fused into the head GEMM
        (mode 1: DDIM with ``coef``, x0-hat into ``x0_out``; mode 2: clamp).
        ``patches = (patches_in, patches_out)``: bf16 patch rows of ``x`` handed from
        one step's head epilogue to the next step's patch embedding (no patchify
        launch per step; ``patches_in`` None on the first step)."""
        if self.fused and FUSED_HEAD:
            hs = (mode, x0_out, coef) if patches is None else (mode, x0_out, coef) + tuple(patches)
            self.prog.forward(self.P, x, t, self.rng, False, save=False, head_step=hs)
            return
        x0_raw = self(x, t)
        if mode == 2:
            torch.clamp(x0_raw, -1.0, 1.0, out=x)
        else:
            ops.ddim_step_(x, x0_raw, x0_out, coef)

    def __call__(self, x, t):
        if self.fused:
            out, _ = self.prog.forward(self.P, x, t, self.rng, False, save=False)
            return out
        was = self.model.training
        self.model.eval()
        try:
            return self.model.forward_reference(x, t)
        finally:
            self.model.train(was)


FUSED_HEAD = True  # module constants: tests switch them to compare the paths
# the head epilogue of each step also writes the new x_t as the next step's bf16
# patch rows, so every step after the first skips the patchify launch
PATCH_CHAIN = True


def _patch_rows(model, N: int, device, den) -> Optional[torch.Tensor]:
    """bf16 [N*P, C*p*p] hand-off buffer for the patch-row chain (None: not used)."""
    if not (PATCH_CHAIN and FUSED_HEAD and den.fused):
        return None
    p = model.patch_size
    H, W = model.img_size
    return torch.empty(N * (H // p) * (W // p), model.in_chans * p * p, dtype=torch.bfloat16, device=device)


# the sampler state as fp32 patch rows in the head's output column order
# (ops.image_to_rows): the head epilogue's x_t / x0 / x_next / bf16 patch-row accesses
# are contiguous 16-byte vectors (ops.head_step_rows_) instead of scattered pixels,
# and the first step needs no patchify launch either (head GEMM at N=64: 12.2 -> 7.0
# us, k=20 N=64 sampler 33.40 -> 32.90 ms per batch; profiles/sampler_rows_ab.txt)
ROWS = True


class _Rows:
    """Patch-row state of one captured sampling loop (GPU fused path only).

    Inside the loop: :meth:`begin` converts the [N, C, H, W] start image once and
    permutes the patch-embedding weight's columns into the head's order (so a
    replay after training uses the current weights); :meth:`step` is one forward
    with the update in the head epilogue; :meth:`image` converts rows back."""

    def __init__(self, model, N: int, device, den):
        p = model.patch_size
        H, W = model.img_size
        C = model.in_chans
        NP, F = (H // p) * (W // p), C * p * p
        self.den, self.p, self.shape = den, p, (N, C, H, W)
        self.x = torch.zeros(N * NP, F, device=device)
        self.x0 = torch.zeros_like(self.x)
        self.pin = torch.empty(N * NP, F, dtype=torch.bfloat16, device=device)
        self.w = torch.empty_like(den.P.pe_w)

    def begin(self, x_img):
        self.w.copy_(ops.embed_weight_rows(self.den.P.pe_w, self.shape[1], self.p))
        self.x.copy_(ops.image_to_rows(x_img, self.p))
        self.pin.copy_(self.x)

    def step(self, t, mode: int, coef=None):
        x0 = None if mode == 2 else self.x0.view(self.shape)
        self.den.step_(self.x.view(self.shape), t, mode, x0, coef, patches=(self.pin, self.pin, self.w))

    def image(self, xr):
        return ops.rows_to_image(xr, *self.shape, self.p)


def _rows_state(model, N: int, device, den) -> Optional[_Rows]:
    if not (ROWS and PATCH_CHAIN and FUSED_HEAD and den.fused and torch.device(device).type == "cuda"):
        return None
    return _Rows(model, N, device, den)


def _chain_patches(pbuf, first: bool):
    """(patches_in, patches_out) of one step: the first step patchifies x itself."""
    if pbuf is None:
        return None
    return (None if first else pbuf, pbuf)


def _unit_host(x: torch.Tensor) -> torch.Tensor:
    """(x + 1) / 2 as a host tensor -- the reference's return convention (ViT.py:236)
    -- with the affine done on the device before the copy: on the host it cost ~3 ms
    per 64-image batch (tools/ub_d2h.py; 9 % of a k=20 sampler call), on the GPU
    ~0.02 ms.  Same fp32 operations, same values."""
    if x.device.type == "cpu":
        return (x + 1) / 2
    return x.add(1.0).div_(2.0).cpu()


def _cache(model) -> dict:
    return model.__dict__.setdefault("_sampler_graphs", {})


class _GraphLoop:
    """Capture ``body()`` (a full sampling loop on static buffers) into one hipGraph.

    The first :meth:`run` executes the body eagerly on a side stream (allocator and
    kernel warm-up; its result is this call's result) and captures the graph;
    every later run is one replay.  Loops are cached per model and shape
    (:func:`_cache`), so a repeated call replays."""

    def __init__(self, body, device):
        self.body = body
        self.device = device
        self.graph = None

    def run(self, use_graph: bool):
        if not use_graph or self.device.type != "cuda":
            self.body()
            return
        if self.graph is None:
            s = torch.cuda.Stream(device=self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(s):
                self.body()  # warm-up (allocator, kernels); also produces this call's result
            torch.cuda.current_stream(self.device).wait_stream(s)
            from ..utils.observe import no_gc
            # (a capture records the body without running it: the warm-up's
            # outputs stay this call's result)
            g = torch.cuda.CUDAGraph()
            with no_gc(), torch.cuda.graph(g, capture_error_mode="thread_local"):
                self.body()
            self.graph = g
            self.replays = 0
            return
        self.graph.replay()
        self.replays += 1


class DDIMSampler:
    def __init__(self, model, device, k: int = 10, use_graph: bool = True):
        self.model = model
        self.device = torch.device(device)
        self.k = k
        self.T = model.total_steps
        self.ts, coef = ddim_table(self.T, k, device=self.device)
        self.coef = coef
        self.use_graph = use_graph and self.device.type == "cuda"
        self.H, self.W = model.img_size
        self.C = model.in_chans

    def _state(self, N: int, record: bool):
        key = ("ddim", N, self.k, record, str(self.device))
        cache = _cache(self.model)
        st = cache.get(key)
        if st is not None and st["key"] == _Denoiser.key_of(self.model):
            return st
        den = _Denoiser(self.model, self.device)
        dev = self.device
        x = torch.zeros(N, self.C, self.H, self.W, device=dev)
        x0 = torch.zeros_like(x)
        tt = torch.tensor(self.ts, dtype=torch.int64, device=dev).unsqueeze(1).expand(-1, N).contiguous()
        traj = torch.zeros(len(self.ts), N, self.C, self.H, self.W, device=dev) if record else None
        coef = self.coef
        pbuf = _patch_rows(self.model, N, dev, den)
        rs = _rows_state(self.model, N, dev, den)

        def loop():
            if rs is not None:
                rs.begin(x)
                for i in range(len(self.ts)):
                    rs.step(tt[i], 1, coef[i])
                    if traj is not None:
                        traj[i].copy_(rs.image(rs.x0))
                x0.copy_(rs.image(rs.x0))  # (x_t itself is not returned)
                return
            for i in range(len(self.ts)):
                # forward + clamp + DDIM update, one head epilogue
                den.step_(x, tt[i], 1, x0, coef[i], patches=_chain_patches(pbuf, i == 0))
                if traj is not None:
                    traj[i].copy_(x0)

        st = {"key": den.key(), "x": x, "x0": x0, "traj": traj, "loop": _GraphLoop(loop, dev)}
        cache[key] = st
        return st

    @torch.no_grad()
    def sample(self, N: int, generator: Optional[torch.Generator] = None, verbose: bool = False,
               noise: Optional[torch.Tensor] = None, device_noise: bool = False) -> torch.Tensor:
        """``device_noise``: draw x_T on the GPU (``generator`` then a device generator)
        instead of on the host as the reference does (ViT.py:224-225) -- same
        distribution, a different stream; saves the host draw + copy (~2.5 ms per
        N=64 batch)."""
        st = self._state(N, False)
        t0 = time.time()
        if noise is not None:
            st["x"].copy_(noise)
        elif device_noise:
            st["x"].normal_(0.0, 1.0, generator=generator)
        else:
            st["x"].copy_(torch.normal(0.0, 1.0, (N, self.C, self.H, self.W), generator=generator))
        st["loop"].run(self.use_graph)
        out = _unit_host(st["x0"])
        if verbose:
            print(f"ddim k={self.k} N={N}: {len(self.ts)} steps in {time.time() - t0:.3f}s")
        return out

    @torch.no_grad()
    def sequence(self, N: int, generator: Optional[torch.Generator] = None,
                 noise: Optional[torch.Tensor] = None) -> List[torch.Tensor]:
        st = self._state(N, True)
        if noise is None:
            noise = torch.normal(0.0, 1.0, (N, self.C, self.H, self.W), generator=generator)
        st["x"].copy_(noise)
        first = _unit_host(noise)
        st["loop"].run(self.use_graph)
        traj = _unit_host(st["traj"])
        return [first] + [traj[i] for i in range(traj.shape[0])]


class ColdSampler:
    """Cold de-pixelation sampler: start from constant-colour images, x <- clamp(f(x, t)) for t = S..1."""

    def __init__(self, model, device, use_graph: bool = True, steps: Optional[int] = None):
        self.model = model
        self.device = torch.device(device)
        self.steps = steps or cold_steps(model.img_size[1])
        self.use_graph = use_graph and self.device.type == "cuda"
        self.H, self.W = model.img_size
        self.C = model.in_chans

    def _state(self, N: int):
        key = ("cold", N, self.steps, str(self.device))
        cache = _cache(self.model)
        st = cache.get(key)
        if st is not None and st["key"] == _Denoiser.key_of(self.model):
            return st
        den = _Denoiser(self.model, self.device)
        dev = self.device
        x = torch.zeros(N, self.C, self.H, self.W, device=dev)
        ts = list(range(self.steps, 0, -1))
        tt = torch.tensor(ts, dtype=torch.int64, device=dev).unsqueeze(1).expand(-1, N).contiguous()
        traj = torch.zeros(len(ts), N, self.C, self.H, self.W, device=dev)
        pbuf = _patch_rows(self.model, N, dev, den)
        rs = _rows_state(self.model, N, dev, den)

        def loop():
            if rs is not None:
                rs.begin(x)
                for i in range(len(ts)):
                    rs.step(tt[i], 2)
                    traj[i].copy_(rs.image(rs.x))
                x.copy_(rs.image(rs.x))
                return
            for i in range(len(ts)):
                # forward + clamp in the head epilogue
                den.step_(x, tt[i], 2, patches=_chain_patches(pbuf, i == 0))
                traj[i].copy_(x)

        st = {"key": den.key(), "x": x, "traj": traj, "loop": _GraphLoop(loop, dev)}
        cache[key] = st
        return st

    def _init(self, N, generator):
        c = torch.normal(0.0, 1.0, (N, self.C), generator=generator)
        return c[:, :, None, None].expand(-1, -1, self.H, self.W).contiguous()

    @torch.no_grad()
    def sample(self, N: int, generator=None) -> torch.Tensor:
        st = self._state(N)
        st["x"].copy_(self._init(N, generator))
        st["loop"].run(self.use_graph)
        return _unit_host(st["x"])

    @torch.no_grad()
    def sequence(self, N: int, generator=None) -> List[torch.Tensor]:
        st = self._state(N)
        init = self._init(N, generator)
        st["x"].copy_(init)
        st["loop"].run(self.use_graph)
        traj = _unit_host(st["traj"])
        return [(init + 1) / 2] + [traj[i] for i in range(traj.shape[0])]


IMG2IMG_GRAPHS = 8  # cached img2img loops (graph + buffers) per model


def starts_table(total_steps: int, starts: Sequence[int], k: int):
    """(descending grid ts, [len(ts), B, 4] per-sample DDIM coefficients) for samples
    joining one k-grid at their own start steps; a sample whose start is below
    step t has the identity row {0, 1, 0, 1} there (x_next = x_t exactly)."""
    top = max(starts)
    if any((top - s) % k for s in starts):
        raise ValueError("all start steps must share one k-grid")
    ts = list(range(top, 0, -k))
    if ts[-1] + 1 - k < 0:
        raise ValueError(f"k={k} incompatible with t_start={top}")
    ident = (0.0, 1.0, 0.0, 1.0)
    rows = [[ddim_coefficients(total_steps, t, k) if s >= t else ident for s in starts] for t in ts]
    return ts, torch.tensor(rows, dtype=torch.float32)


@torch.no_grad()
def ddim_from_starts(model, x: torch.Tensor, starts: Sequence[int], k: int, device=None,
                     use_graph: bool = True) -> torch.Tensor:
    """DDIM (jump ``k``) from per-sample start steps, all samples in ONE batch.

    Sample i joins the shared descending grid at its own ``starts[i]``; all starts
    must lie on one k-grid (``(max - s) % k == 0``).  Every step is ONE forward
    whose head epilogue applies the update with per-sample coefficients
    (:func:`ops.head_step_` mode 4: not-yet-started samples get the identity row),
    and the whole loop is one hipGraph, cached per (B, starts, k): a repeated
    call is one replay (at most ``IMG2IMG_GRAPHS`` such loops stay cached per model,
    least recently used evicted).  Returns the final clamped x0-hat on the device,
    in [-1, 1], as a fresh tensor (not the graph's output buffer, which the next call
    with the same key overwrites).
    """
    device = torch.device(device) if device is not None else x.device
    T = model.total_steps
    B = x.shape[0]
    starts = [int(s) for s in starts]
    key = ("img2img", B, tuple(starts), k, str(device))
    cache = _cache(model)
    st = cache.pop(key, None)
    if st is not None:
        cache[key] = st  # most recently used last
    if st is None or st["key"] != _Denoiser.key_of(model):
        cached = [c for c in cache if isinstance(c, tuple) and c[0] == "img2img"]
        for old in cached[:max(0, len(cached) - IMG2IMG_GRAPHS + 1)]:
            del cache[old]
        den = _Denoiser(model, device)
        ts, coef = starts_table(T, starts, k)
        coef = coef.to(device)
        xs = torch.zeros(B, model.in_chans, *model.img_size, device=device)
        x0 = torch.zeros_like(xs)
        tt = torch.tensor(ts, dtype=torch.int64, device=device).unsqueeze(1).expand(-1, B).contiguous()
        pbuf = _patch_rows(model, B, device, den)
        rs = _rows_state(model, B, device, den)

        def loop():
            if rs is not None:
                rs.begin(xs)
                for i in range(len(ts)):
                    rs.step(tt[i], 4, coef[i])
                x0.copy_(rs.image(rs.x0))
                xs.copy_(rs.image(rs.x))
                return
            for i in range(len(ts)):
                den.step_(xs, tt[i], 4, x0, coef[i], patches=_chain_patches(pbuf, i == 0))

        st = {"key": den.key(), "x": xs, "x0": x0, "loop": _GraphLoop(loop, device)}
        cache[key] = st
    st["x"].copy_(x.to(device).float())
    st["loop"].run(use_graph and device.type == "cuda")
    return st["x0"].clone()


@torch.no_grad()
def img2img(model, draft: torch.Tensor, t_starts: Sequence[int] = tuple(range(1599, 2000, 50)), k: int = 10,
            device=None, generator: Optional[torch.Generator] = None, use_graph: bool = True) -> torch.Tensor:
    """Zero-shot draft->drawing (SDEdit-style) for several noise levels at once.

    For each t_start: x = sqrt(1-a) eps + sqrt(a) draft, a = 1 - sqrt(t_start/T)
    (ViT_draft2drawing.py:395-396, note t_start/T not (t+1)/T), then DDIM with
    jump k down to the grid's last step; returns the final x0-hat per t_start
    as CPU images in [0, 1], shape [len(t_starts), C, H, W].

    All t_starts on one k-grid run as ONE batch, each sample joining the shared
    step grid at its own start (the reference loops them one at a time at batch
    1); the loop is one cached hipGraph (:func:`ddim_from_starts`).
    """
    device = torch.device(device) if device is not None else next(model.parameters()).device
    T = model.total_steps
    starts = list(t_starts)
    B = len(starts)
    C, H, W = model.in_chans, *model.img_size
    if draft.dim() == 3:
        draft = draft.unsqueeze(0)
    draft = draft.to(device).float()
    if draft.shape[0] == 1:
        draft = draft.expand(B, -1, -1, -1)
    top = max(starts)
    if any((top - s) % k for s in starts):
        # different grids: run them one by one
        return torch.cat([img2img(model, draft[i:i + 1], [s], k, device, generator, use_graph)
                          for i, s in enumerate(starts)])
    eps = torch.normal(0.0, 1.0, (B, C, H, W), generator=generator).to(device)
    x = img2img_noised(draft, eps, starts, T)
    x0 = ddim_from_starts(model, x, starts, k, device, use_graph)
    return _unit_host(x0)


def img2img_noised(draft: torch.Tensor, eps: torch.Tensor, starts: Sequence[int], total_steps: int) -> torch.Tensor:
    """x = sqrt(1-a) eps + sqrt(a) draft per start step, a = 1 - sqrt(t_start/T)
    (ViT_draft2drawing.py:395-396)."""
    alpha = torch.tensor([img2img_alpha(s, total_steps) for s in starts], device=draft.device).view(-1, 1, 1, 1)
    return torch.sqrt(1 - alpha) * eps + torch.sqrt(alpha) * draft
