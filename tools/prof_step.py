"""Profile target: N fused training fwd+bwd steps (eager launches) of ViT-tiny at B=32."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddim_cold_amd.models import build_model
from ddim_cold_amd.models.program import ViTProgram, collect, model_tensors
from ddim_cold_amd import ops
dev = "cuda"; B = int(os.environ.get("B", 32)); steps = int(os.environ.get("STEPS", 20))
torch.manual_seed(0)
m = build_model(os.environ.get("MODEL", "vit_tiny")).to(dev).train()
H = m.img_size[0]
img = torch.randn(B, 3, H, H, device=dev).clamp(-1, 1); tgt = torch.randn_like(img).clamp(-1, 1)
t = torch.randint(1, 7, (B,), device=dev)
prog = ViTProgram.from_model(m); P = model_tensors(m)
grads = {n: torch.zeros_like(p) for n, p in m.named_parameters()}
G = collect(grads, prog.cfg.depth, prog.cfg.dim)
r = torch.tensor([1, 0], dtype=torch.int64, device=dev)
with torch.no_grad():
    for _ in range(steps):
        out, S = prog.forward(P, img, t, r, True)
        loss, dtok = ops.smooth_l1_fwd_bwd(out, tgt, prog.cfg.tokens, prog.cfg.patch)
        prog.backward(P, G, S, dtok, r, True)
torch.cuda.synchronize()
print("done")
