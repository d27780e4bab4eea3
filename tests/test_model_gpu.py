"""Model-level GPU tests: the fused HIP program vs the same program on reference ops,
and the autograd wrapper vs the plain PyTorch model."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from ddim_cold_amd import ops
from ddim_cold_amd.models import DiffusionVisionTransformer, build_model
from ddim_cold_amd.models.program import ViTProgram, collect, model_tensors
from ddim_cold_amd.ops import reference as ref

DEV = "cuda"


def _rel(a, b):
    return ((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-12)).item()


def _frob(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


# Per-tensor bounds, from tools/grad_error_report.py on MI355X (profiles/README.md,
# round 3): fused program vs the same program on reference ops (identical bf16
# rounding points, so only summation order / transcendental approximations differ):
# worst max-rel 5.6e-3, worst Frobenius 4.9e-3 over the 93 gradient tensors;
# autograd (bf16 MFMA) vs the fp32 model: worst max-rel 8.1e-3, Frobenius 7.0e-3.
# A bf16 rounding is 2^-9 (2e-3) relative, so the bounds below are a few bf16
# ulps and ~3-4x the measured worst case.
PROG_MAXREL, PROG_FROB = 2e-2, 1.5e-2
FP32_MAXREL, FP32_FROB = 3e-2, 2e-2


@pytest.mark.parametrize("name", ["vit_tiny", "oxford_flower"])
def test_program_fwd_bwd_vs_reference_ops(name):
    torch.manual_seed(0)
    m = build_model(name).to(DEV).train()
    prog = ViTProgram.from_model(m)
    P = model_tensors(m)
    B = 8
    img = torch.randn(B, 3, 64, 64, device=DEV).clamp(-1, 1)
    tgt = torch.randn_like(img).clamp(-1, 1)
    t = torch.randint(0, 2000, (B,), device=DEV)
    r = torch.tensor([77, 3], dtype=torch.int64, device=DEV)
    results = []
    for force in (False, True):
        grads = {n: torch.zeros_like(p) for n, p in m.named_parameters()}
        G = collect(grads, prog.cfg.depth, prog.cfg.dim)
        ctx = ops.force_reference() if force else torch.no_grad()
        with ctx, torch.no_grad():
            out, S = prog.forward(P, img, t, r, True)
            loss, dtok = ops.smooth_l1_fwd_bwd(out, tgt, prog.cfg.tokens, prog.cfg.patch)
            prog.backward(P, G, S, dtok, r, True)
        torch.cuda.synchronize()
        results.append((out, loss, grads))
    (o1, l1, g1), (o2, l2, g2) = results
    assert _rel(o1, o2) < PROG_MAXREL
    assert abs(l1.item() - l2.item()) / l2.item() < 1e-2
    for n in g1:
        assert _rel(g1[n], g2[n]) < PROG_MAXREL, (n, _rel(g1[n], g2[n]))
        assert _frob(g1[n], g2[n]) < PROG_FROB, (n, _frob(g1[n], g2[n]))


@pytest.mark.parametrize("name", ["vit_tiny", "oxford_flower"])
@pytest.mark.parametrize("embed_with_block0", [True, False])
@pytest.mark.parametrize("mode", ["bucket", "immediate"])
def test_backward_wgrad_schedules_match(name, embed_with_block0, mode):
    """The deferred weight gradients (default: ONE launch after the backward) ==
    one launch per gradient bucket (data parallel) == each issued immediately;
    same tiles, same unsplit reduction order for the launches (bit-identical
    except the token-split patch gradient of the embedding bucket), and the block
    yields keep their order (L-1 .. 0, -1)."""
    torch.manual_seed(0)
    m = build_model(name).to(DEV).train()
    prog = ViTProgram.from_model(m)
    P = model_tensors(m)
    B = 8
    img = torch.randn(B, 3, 64, 64, device=DEV).clamp(-1, 1)
    tgt = torch.randn_like(img).clamp(-1, 1)
    t = torch.randint(0, 2000, (B,), device=DEV)
    r = torch.tensor([77, 3], dtype=torch.int64, device=DEV)
    with torch.no_grad():
        out, S = prog.forward(P, img, t, r, True)
        _, dtok = ops.smooth_l1_fwd_bwd(out, tgt, prog.cfg.tokens, prog.cfg.patch)
    results = []
    for variant in ("tail", mode):
        grads = {n: torch.zeros_like(p) for n, p in m.named_parameters()}
        G = collect(grads, prog.cfg.depth, prog.cfg.dim)
        kw = dict(embed_with_block0=embed_with_block0)
        if variant == "bucket":
            kw["wgrad_flush"] = {3, 1, 0}
        elif variant == "immediate":
            kw["wgrad"] = ops.linear_wgrad
        with torch.no_grad():
            order = list(prog.backward_iter(P, G, S, dtok, r, True, **kw))
        torch.cuda.synchronize()
        assert order == list(range(prog.cfg.depth - 1, -1, -1)) + [-1]
        results.append(grads)
    g1, g2 = results
    for n in g1:
        assert g1[n].abs().max() > 0 or g2[n].abs().max() == 0, n
        assert _rel(g1[n], g2[n]) < 1e-4, n


def test_autograd_wrapper_matches_plain_model():
    torch.manual_seed(0)
    m = build_model("vit_tiny").to(DEV).eval()  # eval: no dropout -> deterministic comparison
    B = 4
    img = torch.randn(B, 3, 64, 64, device=DEV)
    t = torch.randint(0, 2000, (B,), device=DEV)
    out = m(img, t)
    with torch.no_grad():
        out_ref = m.forward_reference(img, t)
    assert _rel(out, out_ref) < FP32_MAXREL
    loss = out.square().mean()
    loss.backward()
    g_fused = {n: p.grad.clone() for n, p in m.named_parameters()}
    m.zero_grad()
    m.forward_reference(img, t).square().mean().backward()
    for n, p in m.named_parameters():
        assert _rel(g_fused[n], p.grad) < FP32_MAXREL, (n, _rel(g_fused[n], p.grad))
        assert _frob(g_fused[n], p.grad) < FP32_FROB, (n, _frob(g_fused[n], p.grad))


def test_high_res_forward():
    torch.manual_seed(0)
    m = build_model("vit_small_200", depth=2).to(DEV).eval()
    img = torch.randn(2, 3, 200, 200, device=DEV)
    t = torch.randint(0, 2000, (2,), device=DEV)
    with torch.no_grad():
        out = m(img, t)
        out_ref = m.forward_reference(img, t)
    assert out.shape == img.shape
    assert _rel(out, out_ref) < 3e-2
