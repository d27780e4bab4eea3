"""GPU check of the fused dgrad + LayerNorm backward (csrc/gemm_lnbwd.hip): NaN / inf
census and mismatch locations against the fp32 oracle for several K / modes."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddim_cold_amd import ops
from ddim_cold_amd.ops import reference as ref
DEV = "cuda"
torch.manual_seed(0)
r = torch.tensor([1234, 5], dtype=torch.int64, device=DEV)
for (M, K, D, N) in [(2080, 192, 384, 65), (2080, 384, 384, 65), (2080, 1152, 384, 65), (20032, 384, 384, 626),
                     (8224, 256, 256, 257)]:
    for mode in ("full", "final", "no_gy"):
        for rep in range(2):
            dy = torch.randn(M, K, device=DEV).to(torch.bfloat16)
            w = (torch.randn(K, D, device=DEV) * 0.05).to(torch.bfloat16)
            x = (torch.randn(M, D, device=DEV) * 2 + 0.5).to(torch.bfloat16)
            g, b = torch.randn(D, device=DEV), torch.randn(D, device=DEV)
            _, mu, rs = ref.layernorm_fwd(x.float(), g, b)
            gres = None if mode == "final" else torch.randn(M, D, device=DEV)
            emit = mode != "no_gy"
            p, pdp = (0.1, 0.2) if emit else (0.0, 0.0)
            ws = torch.zeros(ops.LN_REPLICAS, 2 * D, device=DEV)
            y_out = torch.empty(M, D, dtype=torch.bfloat16, device=DEV)
            go, gy = ops.linear_dgrad_lnbwd(dy, w, x, mu, rs, g, gres, torch.zeros(D, device=DEV),
                                            torch.zeros(D, device=DEV), N, r, 7, p, 8, pdp, emit, ws, beta=b,
                                            y_out=y_out)
            torch.cuda.synchronize()
            dl = dy.float() @ w.float()
            dg2, db2 = torch.zeros(D, device=DEV), torch.zeros(D, device=DEV)
            gor, gyr = ref.layernorm_bwd(dl, x.float(), mu, rs, g, gres, dg2, db2, N, r, 7, p, 8, pdp, emit)
            bad = ~torch.isfinite(go)
            err = (go - gor.view_as(go)).abs()
            tol = 2e-3 * gor.abs().max() + 1e-3 * gor.abs().view_as(go)
            mis = ~(err <= tol)
            line = f"M{M} K{K} D{D} {mode} rep{rep}: g_out nonfinite {int(bad.sum())} mismatches {int(mis.sum())}"
            if emit:
                gbad = ~torch.isfinite(gy.float())
                zmis = (gyr.float() == 0) & (gy.float() != 0)
                line += f" | gy nonfinite {int(gbad.sum())} zero-pattern mismatches {int(zmis.sum())}"
                for (i, j) in zmis.nonzero()[:4].tolist():
                    km = ref.keep_mask(M * D, r, 7, p, DEV)[i * D + j].item()
                    ks = ref.keep_mask(M // N, r, 8, pdp, DEV)[i // N].item()
                    line += (f"\n   row {i} col {j}: ours gy {gy[i, j].item():.6e} g_out {go.view(M, D)[i, j].item():.9e} "
                             f"oracle g_out {gor.view(M, D)[i, j].item():.9e} gyr {gyr[i, j].item():.3e} keep {km} sample {ks}")
            ws_sum = ws.sum(0)
            line += f" | dgamma maxerr {(ws_sum[:D] - dg2).abs().max().item():.2e} (scale {dg2.abs().max().item():.2e})"
            print(line, flush=True)
            if mis.any():
                idx = mis.nonzero()[:8].tolist()
                rows = mis.any(1).nonzero().flatten()
                cols = mis.any(0).nonzero().flatten()
                print("   first", idx, "rows", rows.numel(), "(tiles", sorted(set((rows // 32).tolist()))[:10], ") cols",
                      cols.numel(), "col groups", sorted(set((cols // 16).tolist()))[:24], flush=True)
