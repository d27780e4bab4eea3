"""Phase timeline of the image-group persistent forward from in-kernel stamps.

    python tools/vg_stamps.py [B]
"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddim_cold_amd import build_model
from ddim_cold_amd.models.program import ViTProgram, model_tensors

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
dev = "cuda"
m = build_model("vit_tiny").to(dev).train()
prog = ViTProgram.from_model(m)
P = model_tensors(m)
img = torch.randn(B, 3, 64, 64, device=dev).clamp(-1, 1)
t = torch.randint(1, 7, (B,), device=dev)
r = torch.tensor([1, 2], dtype=torch.int64, device=dev)
prog.vg_stamps = torch.zeros(B * 6, 8, 32, dtype=torch.int64, device=dev)
for _ in range(5):
    with torch.no_grad():
        prog.forward(P, img, t, r, True)
torch.cuda.synchronize()
s = prog.vg_stamps.cpu().double() * 10.0 / 1000.0  # 100 MHz ticks -> us
L = len(m.blocks)
t0 = s[:, 0, 0].min()
s = s - t0
names = ["qkv", "proj", "fc1", "fc2"]
print(f"B={B}: kernel span {s[:, L - 1, 15].max():.1f} us (first stamp to last publish)")
print("block phase  wait(us)  work(us)  epi+pub(us)  end(us, median WG)")
for l in range(L):
    for p, n in enumerate(names):
        a, b, c, d = (s[:, l, 4 * p + k] for k in range(4))
        print(f"{l:5d} {n:5s} {(b - a).median():9.2f} {(c - b).median():9.2f} {(d - c).median():11.2f} {d.median():10.1f}")
sub = ["gather", "qGEMM", "waitK", "kGEMM", "emitQK", "vGEMM", "emitV"]
ks = [1, 16, 17, 18, 19, 20, 21, 2]
print("QKV phase detail (median us):", "  ".join(f"{n}={(s[:, :, ks[i + 1]] - s[:, :, ks[i]]).median():.2f}" for i, n in enumerate(sub)))
err = int(prog._vg_err.item())
print("err flag", err)
