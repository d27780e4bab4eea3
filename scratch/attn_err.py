import sys, torch
sys.path.insert(0, ".")
from ddim_cold_amd import ops
from ddim_cold_amd.ops import reference as ref
DEV = "cuda"
B, H, N, hd, p = 48, 4, 300, 64, 0.1
g = torch.Generator(device=DEV).manual_seed(3)
u = torch.randn(hd, device=DEV, generator=g); u = u / u.norm()
a = torch.linspace(0.0, 40.0, N, device=DEV)[torch.randperm(N, device=DEV, generator=g)]
b = torch.linspace(0.0, 8.0, N, device=DEV)
qkv = torch.empty(3, B, H, N, hd, device=DEV)
qkv[0] = a[:, None] * u + 0.05 * torch.randn(B, H, N, hd, device=DEV, generator=g)
qkv[1] = b[:, None] * u + 0.05 * torch.randn(B, H, N, hd, device=DEV, generator=g)
qkv[2] = torch.randn(B, H, N, hd, device=DEV, generator=g)
qkv = qkv.to(torch.bfloat16)
r = torch.tensor([1234, 5], dtype=torch.int64, device=DEV)
scale = hd ** -0.5
torch.manual_seed(0)
o, lse = ops.attn_fwd(qkv, scale, r, 5, p)
do = torch.randn(B, N, H * hd, device=DEV).to(torch.bfloat16)
x = ops.attn_bwd(do, qkv, o, lse, scale, r, 5, p).float()
y = ref.attn_bwd(do, qkv, o, lse, scale, r, 5, p).float()
D = H * hd
for i, nm in enumerate("qkv"):
    e = (x[..., i*D:(i+1)*D] - y[..., i*D:(i+1)*D]).abs()
    t = 3e-2 + 3e-2 * y[..., i*D:(i+1)*D].abs()
    print(nm, "bad", int((e > t).sum()), "max err", float(e.max()), "max|ref|", float(y[..., i*D:(i+1)*D].abs().max()), "mean err", float(e.mean()))
# error against exact math (fp64, no intermediate rounding)
qd, kd, vd = (qkv[i].double() for i in range(3))
dof = do.double().view(B, N, H, hd).transpose(1, 2)
of = o.double().view(B, N, H, hd).transpose(1, 2)
s = (qd @ kd.transpose(-1, -2)) * scale
pr = torch.exp(s - lse.double().unsqueeze(-1))
m = ref.attn_keep_mask(B, H, N, r, 5, p, pr.device, 0).double() / (1.0 - p)
dv = (pr * m).transpose(-1, -2) @ dof
dp = (dof @ vd.transpose(-1, -2)) * m
ds = pr * (dp - (dof * of).sum(-1, keepdim=True))
ex = torch.stack(((ds @ kd) * scale, (ds.transpose(-1, -2) @ qd) * scale, dv), 0).permute(1, 3, 0, 2, 4).reshape(B * N, 3 * D)
for i, nm in enumerate("qkv"):
    e = (x[..., i*D:(i+1)*D].double() - ex[..., i*D:(i+1)*D]).abs()
    print(nm, "vs exact: mean err", float(e.mean()), "max", float(e.max()), "rms", float(e.pow(2).mean().sqrt()))
