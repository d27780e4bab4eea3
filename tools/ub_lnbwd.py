"""LayerNorm backward (rows per wave x waves per workgroup configs, torch.ops.ddim_cold.ln_bwd_config)
on the ViT-tiny (M = 2,080) and vit_small_200 (M = 20,032) training shapes, graph-timed."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from ddim_cold_amd import ops  # noqa: E402
from tools.ubench import t  # noqa: E402

dev = "cuda"
D = 384
r = torch.tensor([1, 2], dtype=torch.int64, device=dev)
for M, N in ((2080, 65), (20032, 626)):
    x = torch.randn(M, D, device=dev)
    g, be = torch.randn(D, device=dev), torch.randn(D, device=dev)
    _, mu, rs = ops.layernorm_fwd(x, g, be)
    dyb = (torch.randn(M, D, device=dev)).to(torch.bfloat16)
    gres = torch.randn(M, D, device=dev)
    ws = torch.zeros(ops.LN_REPLICAS, 2 * D, device=dev)
    yo = torch.empty(M, D, dtype=torch.bfloat16, device=dev)
    dg, db = torch.zeros(D, device=dev), torch.zeros(D, device=dev)
    row = {}
    outs = {}
    for cfg, name in ((1, "1x8"), (2, "2x8"), (3, "1x4"), (4, "2x4")):
        old = torch.ops.ddim_cold.ln_bwd_config(cfg)
        fn = lambda: ops.layernorm_bwd(dyb, x, mu, rs, g, gres, dg, db, N, r, 3, 0.1, 4, 0.1, True, ws,  # noqa: E731
                                       beta=be, y_out=yo)
        row[name] = round(t(fn, reps=50), 2)
        ws.zero_()
        outs[name] = [o.clone() for o in fn() if o is not None]
        torch.ops.ddim_cold.ln_bwd_config(old)
    same = all(torch.equal(a, b) for k in outs for a, b in zip(outs[k], outs["1x8"]))
    print(f"M={M}: us {row}  outputs identical across configs: {same}", flush=True)
