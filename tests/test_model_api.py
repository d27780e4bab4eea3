"""Model API parity and the fused program's logic on CPU."""
import math

import pytest
import torch

from ddim_cold_amd.models import DiffusionVisionTransformer, build_model, positionalencoding1d
from ddim_cold_amd.models.program import ViTProgram, collect
from ddim_cold_amd.ops import reference as ref


def expected_keys(depth):
    keys = [("cls_token", None), ("pos_embed", None), ("patch_embed.proj.weight", None),
            ("patch_embed.proj.bias", None), ("time_embed.weight", None)]
    for i in range(depth):
        for n in ["norm1.weight", "norm1.bias", "attn.qkv.weight", "attn.qkv.bias", "attn.proj.weight",
                  "attn.proj.bias", "norm2.weight", "norm2.bias", "mlp.fc1.weight", "mlp.fc1.bias",
                  "mlp.fc2.weight", "mlp.fc2.bias"]:
            keys.append((f"blocks.{i}.{n}", None))
    keys += [("norm.weight", None), ("norm.bias", None), ("head.weight", None), ("head.bias", None)]
    return [k for k, _ in keys]


def test_state_dict_layout_vit_tiny():
    m = build_model("vit_tiny")
    sd = m.state_dict()
    assert list(sd.keys()) == expected_keys(7)
    assert len(sd) == 93
    assert [n for n, _ in m.named_parameters()] == expected_keys(7)
    D, P, C, p = 384, 64, 3, 8
    assert sd["cls_token"].shape == (1, 1, D)
    assert sd["pos_embed"].shape == (1, P + 1, D)
    assert sd["patch_embed.proj.weight"].shape == (D, C, p, p)
    assert sd["time_embed.weight"].shape == (2000, D)
    assert sd["blocks.0.attn.qkv.weight"].shape == (3 * D, D)
    assert sd["blocks.3.mlp.fc1.weight"].shape == (D, D)  # mlp_ratio 1.0
    assert sd["head.weight"].shape == (C * p * p, D)
    assert sum(v.numel() for v in sd.values()) == 7162176  # SURVEY §0 (verified count)


def test_constructor_defaults_and_attributes():
    m = DiffusionVisionTransformer()
    assert m.embed_dim == m.num_features == 256 and m.patch_size == 8 and m.in_chans == 3
    assert list(m.img_size) == [64, 64] and m.total_steps == 2000
    assert m.patch_embed.num_patches == 64
    assert len(m.blocks) == 3 and m.blocks[0].attn.num_heads == 4
    # stochastic depth decay: linspace(0, 0.1, depth), block 0 -> Identity
    assert isinstance(m.blocks[0].drop_path, torch.nn.Identity)
    assert m.drop_path_probs() == pytest.approx([0.0, 0.05, 0.1])
    assert m.blocks[0].attn.scale == pytest.approx((256 // 4) ** -0.5)


def test_load_reference_layout_state_dict_strict():
    src = build_model("oxford_flower")
    sd = {k: v.clone() for k, v in src.state_dict().items()}
    dst = build_model("oxford_flower")
    dst.load_state_dict(sd, strict=True)
    for k in sd:
        assert torch.equal(dst.state_dict()[k], sd[k])


def test_init_statistics():
    torch.manual_seed(0)
    m = build_model("vit_tiny")
    w = m.blocks[0].attn.qkv.weight
    assert w.abs().max() <= 2.0 and abs(w.std().item() - 0.02) < 0.002
    assert torch.all(m.blocks[0].attn.qkv.bias == 0)
    assert torch.all(m.blocks[0].norm1.weight == 1) and torch.all(m.blocks[0].norm1.bias == 0)


def test_unpatchify_layout():
    """Head feature f=(a*p+b)*C+c of token (hp,wp) -> pixel (c, hp*p+a, wp*p+b)."""
    m = DiffusionVisionTransformer(img_size=[16, 16], patch_size=4, embed_dim=32, depth=1, num_heads=2)
    p, C = 4, 3
    Hp = Wp = 4
    tok = torch.zeros(1, Hp * Wp, p * p * C)
    for hp in range(Hp):
        for wp in range(Wp):
            for a in range(p):
                for b in range(p):
                    for c in range(C):
                        tok[0, hp * Wp + wp, (a * p + b) * C + c] = c * 10000 + (hp * p + a) * 100 + (wp * p + b)
    img = m.unpatchify(tok)
    cc, yy, xx = torch.meshgrid(torch.arange(C), torch.arange(16), torch.arange(16), indexing="ij")
    assert torch.equal(img[0], (cc * 10000 + yy * 100 + xx).float())
    assert torch.equal(m.patchify(img), tok)


def test_forward_shapes_and_attention_api():
    m = DiffusionVisionTransformer(img_size=[32, 32], patch_size=8, embed_dim=64, depth=2, num_heads=4).eval()
    x = torch.randn(3, 3, 32, 32)
    t = torch.randint(0, 2000, (3,))
    assert m(x, t).shape == x.shape
    tok = m.prepare_tokens(x, t)
    assert tok.shape == (3, 17, 64)
    y, attn = m.blocks[0].attn(m.blocks[0].norm1(tok))
    assert y.shape == tok.shape and attn.shape == (3, 4, 17, 17)
    assert torch.allclose(attn.sum(-1), torch.ones(3, 4, 17), atol=1e-5)
    assert m.blocks[0](tok, return_attention=True).shape == (3, 4, 17, 17)
    assert m.get_last_selfattention(x, t).shape == (3, 4, 17, 17)


def test_positional_encoding():
    pe = positionalencoding1d(8, 5)
    assert pe.shape == (5, 8)
    assert torch.allclose(pe[:, 0], torch.sin(torch.arange(5.0)))
    assert torch.allclose(pe[:, 1], torch.cos(torch.arange(5.0)))
    with pytest.raises(ValueError):
        positionalencoding1d(7, 5)
    m = DiffusionVisionTransformer(img_size=[32, 32], patch_size=8, embed_dim=64, depth=1, num_heads=4,
                                   timestep_embedding="sinusoidal")
    assert not m.time_embed.weight.requires_grad
    assert torch.allclose(m.time_embed.weight[3], positionalencoding1d(64, 2000)[3])


@pytest.fixture
def fp32_reference(monkeypatch):
    """Run the reference ops without bf16 rounding: isolates the program's logic."""
    from ddim_cold_amd.models import program
    monkeypatch.setattr(ref, "bf16", lambda x: x.float() if x.dtype == torch.bfloat16 else x)
    monkeypatch.setattr(program, "ACT_DTYPE", torch.float32)


@pytest.mark.parametrize("cfg", [dict(img_size=[32, 32], patch_size=8, embed_dim=128, depth=3, num_heads=4),
                                 dict(img_size=[16, 16], patch_size=4, embed_dim=64, depth=2, num_heads=2)])
def test_program_backward_matches_autograd(fp32_reference, cfg):
    """Hand-written backward (all dropout / drop-path sites active) == autograd of the same forward."""
    torch.manual_seed(0)
    m = DiffusionVisionTransformer(drop_rate=0.1, attn_drop_rate=0.1, drop_path_rate=0.2, **cfg).train()
    prog = ViTProgram.from_model(m)
    named = {n: p.detach().clone().requires_grad_(True) for n, p in m.named_parameters()}
    P = collect(named, prog.cfg.depth, prog.cfg.dim)
    B = 3
    H = cfg["img_size"][0]
    img = torch.randn(B, 3, H, H)
    tgt = torch.randn(B, 3, H, H).clamp(-1, 1)
    t = torch.randint(0, 2000, (B,))
    rng = torch.tensor([12345, 7])
    out, _ = prog.forward(P, img, t, rng, True)
    loss, dtok = ref.smooth_l1_fwd_bwd(out, tgt, prog.cfg.tokens, prog.cfg.patch)
    loss.backward()
    grads = {n: torch.zeros_like(p) for n, p in named.items()}
    G = collect(grads, prog.cfg.depth, prog.cfg.dim)
    Pd = collect({n: p.detach() for n, p in named.items()}, prog.cfg.depth, prog.cfg.dim)
    out2, S = prog.forward(Pd, img, t, rng, True)
    assert torch.equal(out2, out.detach())
    prog.backward(Pd, G, S, dtok, rng, True)
    for n, p in named.items():
        a, b = p.grad, grads[n]
        rel = (a - b).abs().max().item() / (a.abs().max().item() + 1e-12)
        assert rel < 1e-4, (n, rel)


def test_program_eval_matches_plain_model(fp32_reference):
    torch.manual_seed(0)
    m = DiffusionVisionTransformer(img_size=[32, 32], patch_size=8, embed_dim=64, depth=2, num_heads=4).eval()
    prog = ViTProgram.from_model(m)
    P = collect({n: p.detach() for n, p in m.named_parameters()}, 2, 64)
    x = torch.randn(2, 3, 32, 32)
    t = torch.randint(0, 2000, (2,))
    with torch.no_grad():
        a = m.forward_reference(x, t)
        b, _ = prog.forward(P, x, t, torch.tensor([0, 0]), False, save=False)
    assert (a - b).abs().max() < 1e-5


def _folded(m, named):
    from ddim_cold_amd.models.program import LnFold
    c = ViTProgram.from_model(m).cfg
    P = collect(dict(named), c.depth, c.dim)
    fold = LnFold(dict(named), c.depth)
    fold.refresh()
    return fold.attach(P)


@pytest.mark.parametrize("cfg", [dict(img_size=[32, 32], patch_size=8, embed_dim=128, depth=3, num_heads=4),
                                 dict(img_size=[16, 16], patch_size=4, embed_dim=64, depth=2, num_heads=2)])
def test_program_layernorm_fold_matches_autograd(fp32_reference, cfg):
    """LayerNorm fold (forward without LayerNorm launches: statistics from the producing
    epilogue, gamma/beta folded into the consumer GEMM, LayerNorm outputs re-emitted
    by the backward) == autograd of the unfolded forward, all dropout sites active."""
    torch.manual_seed(0)
    m = DiffusionVisionTransformer(drop_rate=0.1, attn_drop_rate=0.1, drop_path_rate=0.2, **cfg).train()
    with torch.no_grad():  # non-trivial LayerNorm affine parameters
        for n, p in m.named_parameters():
            if "norm" in n:
                p.add_(0.3 * torch.randn_like(p))
    prog = ViTProgram.from_model(m)
    named = {n: p.detach().clone().requires_grad_(True) for n, p in m.named_parameters()}
    P = collect(named, prog.cfg.depth, prog.cfg.dim)
    B, H = 3, cfg["img_size"][0]
    img = torch.randn(B, 3, H, H)
    tgt = torch.randn(B, 3, H, H).clamp(-1, 1)
    t = torch.randint(0, 2000, (B,))
    rng = torch.tensor([12345, 7])
    out, _ = prog.forward(P, img, t, rng, True)
    loss, dtok = ref.smooth_l1_fwd_bwd(out, tgt, prog.cfg.tokens, prog.cfg.patch)
    loss.backward()
    Pf = _folded(m, {n: p.detach() for n, p in named.items()})
    assert Pf.folded
    out2, S = prog.forward(Pf, img, t, rng, True)
    assert (out2 - out.detach()).abs().max() < 1e-4
    assert S.lf is None and all(b[1] is None and b[8] is None for b in S.blocks)
    grads = {n: torch.zeros_like(p) for n, p in named.items()}
    G = collect(grads, prog.cfg.depth, prog.cfg.dim)
    prog.backward(Pf, G, S, dtok, rng, True)
    for n, p in named.items():
        a, b = p.grad, grads[n]
        rel = (a - b).abs().max().item() / (a.abs().max().item() + 1e-12)
        assert rel < 1e-3, (n, rel)


def test_layernorm_fold_reference_identity():
    """rstd*(x (gamma o W)^T - mean*c) + (b + W beta) == LayerNorm(x) W^T + b."""
    torch.manual_seed(0)
    x = torch.randn(37, 64) * 3 + 0.5
    w, b = torch.randn(48, 64), torch.randn(48)
    g, be = torch.randn(64), torch.randn(64)
    wf, c, bf = torch.empty(48, 64), torch.empty(48), torch.empty(48)
    ref.ln_fold(w, g, be, b, wf, c, bf)
    st = ref.row_stats(x)
    mean, rstd = torch.empty(37), torch.empty(37)
    y = ref._lin(x, wf, bf, st, c, 1e-5, mean, rstd)
    expect = torch.nn.functional.layer_norm(x, (64,), g, be, 1e-5) @ w.t() + b
    # the fold multiplies bf16-rounded (gamma o W); compare against that rounding
    assert (y - expect).abs().max() < 0.05 * expect.abs().max()
    torch.testing.assert_close(mean, x.mean(-1), rtol=1e-5, atol=1e-5)


def _reference_draw_order_state(seed, order, img=16, p=4, D=32, depth=2, H=4, T=2000):
    """Independent replay of the reference constructors' RNG draws (no model class of
    ours): ViT_draft2drawing.py:186-207 (order 'draft2drawing': pos_embed drawn right
    after it is created, before the blocks) vs ViT.py:169-187 (order 'vit': after head)."""
    import torch.nn as nn
    torch.manual_seed(seed)
    proj = nn.Conv2d(3, D, kernel_size=p, stride=p)          # PatchEmbed (default init draws)
    cls = torch.zeros(1, 1, D)
    temb = nn.Embedding(T, D)                                  # normal_ init draw
    pos = torch.zeros(1, (img // p) ** 2 + 1, D)
    if order == "draft2drawing":
        nn.init.trunc_normal_(pos, std=0.02)
    blocks = []
    for _ in range(depth):                                     # Block: LN, qkv, proj, LN, fc1, fc2
        blocks.append([nn.LayerNorm(D), nn.Linear(D, 3 * D), nn.Linear(D, D), nn.LayerNorm(D),
                       nn.Linear(D, D), nn.Linear(D, D)])
    norm = nn.LayerNorm(D)
    head = nn.Linear(D, 3 * p * p)
    if order == "vit":
        nn.init.trunc_normal_(pos, std=0.02)
    nn.init.trunc_normal_(cls, std=0.02)
    nn.init.trunc_normal_(temb.weight, std=0.02)
    # Module.apply: children first, in registration order; Linear -> trunc_normal_ + zero bias
    for blk in blocks:
        for m in blk:
            if isinstance(m, nn.Linear):
                nn.init.trunc_normal_(m.weight, std=0.02)
                nn.init.zeros_(m.bias)
    nn.init.trunc_normal_(head.weight, std=0.02)
    nn.init.zeros_(head.bias)
    sd = {"cls_token": cls, "pos_embed": pos, "patch_embed.proj.weight": proj.weight,
          "patch_embed.proj.bias": proj.bias, "time_embed.weight": temb.weight}
    names = ["norm1", "attn.qkv", "attn.proj", "norm2", "mlp.fc1", "mlp.fc2"]
    for i, blk in enumerate(blocks):
        for n, m in zip(names, blk):
            sd[f"blocks.{i}.{n}.weight"] = m.weight
            sd[f"blocks.{i}.{n}.bias"] = m.bias
    sd.update({"norm.weight": norm.weight, "norm.bias": norm.bias, "head.weight": head.weight,
               "head.bias": head.bias})
    return {k: v.detach() for k, v in sd.items()}


@pytest.mark.parametrize("order", ["draft2drawing", "vit"])
def test_init_draw_order_matches_reference_classes(order):
    from ddim_cold_amd.models.vit import DiffusionVisionTransformer
    ref = _reference_draw_order_state(11, order)
    torch.manual_seed(11)
    m = DiffusionVisionTransformer(img_size=[16, 16], patch_size=4, embed_dim=32, depth=2, num_heads=4,
                                   init_order=order)
    sd = m.state_dict()
    assert list(sd) == list(ref)
    for k in ref:
        assert torch.equal(sd[k], ref[k]), k


def test_init_order_default_is_trainer_class():
    from ddim_cold_amd.models.vit import DiffusionVisionTransformer
    torch.manual_seed(2)
    a = DiffusionVisionTransformer(img_size=[16, 16], patch_size=4, embed_dim=32, depth=2, num_heads=4)
    torch.manual_seed(2)
    b = DiffusionVisionTransformer(img_size=[16, 16], patch_size=4, embed_dim=32, depth=2, num_heads=4,
                                   init_order="draft2drawing")
    assert all(torch.equal(x, y) for x, y in zip(a.state_dict().values(), b.state_dict().values()))
    with pytest.raises(ValueError):
        DiffusionVisionTransformer(img_size=[16, 16], patch_size=4, embed_dim=32, depth=2, num_heads=4,
                                   init_order="x")
