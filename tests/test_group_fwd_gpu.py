"""Image-group persistent block forward (csrc/vit_group.hip) vs the per-op launch
sequence of the LayerNorm-folded forward: same tensors, bit for bit."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from ddim_cold_amd import build_model, ops
from ddim_cold_amd.models import program as pm
from ddim_cold_amd.models.program import ViTProgram, model_tensors

DEV = "cuda"


def _run(m, group, B, training, save, monkeypatch, seed=5):
    monkeypatch.setattr(pm, "GROUP_FWD", group)
    prog = ViTProgram.from_model(m)
    P = model_tensors(m)
    assert P.folded
    g = torch.Generator(device="cpu").manual_seed(seed)
    img = torch.randn(B, 3, 64, 64, generator=g).clamp(-1, 1).to(DEV)
    t = torch.randint(1, 2000, (B,), generator=g).to(DEV)
    r = torch.tensor([91, 4], dtype=torch.int64, device=DEV)
    with torch.no_grad():
        out, S = prog.forward(P, img, t, r, training, save=save)
    torch.cuda.synchronize()
    if group:
        assert int(prog._vg_err.item()) == 0, "a hand-off wait gave up"
    return out, S


@pytest.mark.parametrize("B,training", [(8, True), (32, True), (3, False), (64, False), (50, True)])
def test_group_forward_bit_exact(B, training, monkeypatch):
    torch.manual_seed(0)
    m = build_model("vit_tiny").to(DEV).train(training)
    assert ops.vit_group_ok(384, 12, 32, m.num_tokens, len(m.blocks))
    o1, S1 = _run(m, True, B, training, True, monkeypatch)
    o2, S2 = _run(m, False, B, training, True, monkeypatch)
    names = ["x0", "l1", "m1", "r1", "qkv", "o", "lse", "x1", "l2", "m2", "r2", "u", "h"]
    for i, (b1, b2) in enumerate(zip(S1.blocks, S2.blocks)):
        for n, a, b in zip(names, b1, b2):
            if a is None and b is None:
                continue
            assert torch.equal(a, b), f"block {i} {n}: max diff {(a.float() - b.float()).abs().max().item()}"
    assert torch.equal(S1.xL, S2.xL)
    assert torch.equal(o1, o2)


def test_group_forward_sampler_step(monkeypatch):
    """The fused DDIM step path (no saved tensors, head_step) through the group forward."""
    from ddim_cold_amd.diffusion.samplers import DDIMSampler
    torch.manual_seed(0)
    m = build_model("vit_tiny").to(DEV).eval()
    outs = []
    for group in (True, False):
        monkeypatch.setattr(pm, "GROUP_FWD", group)
        s = DDIMSampler(m, DEV, k=100, use_graph=False)
        outs.append(s.sample(16, generator=torch.Generator().manual_seed(3)))
    assert torch.equal(outs[0], outs[1])
