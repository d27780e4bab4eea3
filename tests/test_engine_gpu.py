"""TrainEngine on the GPU: graph-captured steps (incl. gradient accumulation) agree with the
eager replay of the same step program."""
import pytest
import torch

from ddim_cold_amd import build_model
from ddim_cold_amd.data.synthetic import ColdBatcher, synthetic_pool
from ddim_cold_amd.train.engine import EngineConfig, TrainEngine


def _run(use_graph, grad_accum, steps=5):
    torch.manual_seed(0)
    model = build_model("vit_tiny").cuda().train()
    eng = TrainEngine(model, EngineConfig(lr=1e-3, t_max=100, seed=3, use_graph=use_graph, graph_warmup=1,
                                          grad_accum=grad_accum, temb_rows=7))
    eng.set_batch_fn(ColdBatcher(synthetic_pool(64, seed=1, device="cuda"), 8, eng.rng))
    losses = []
    for _ in range(steps):
        losses.append(float(eng.train_step()))
    torch.cuda.synchronize()
    return eng.flat_p.clone(), losses, eng


@pytest.mark.gpu
@pytest.mark.parametrize("grad_accum", [1, 2])
def test_graph_step_matches_eager(grad_accum):
    pg, lg, eng = _run(True, grad_accum)
    pe, le, _ = _run(False, grad_accum)
    assert eng._graphs is not None and len(eng._graphs) == 1
    assert all(abs(a - b) <= 1e-4 * abs(b) for a, b in zip(lg, le)), (lg, le)
    # AdamW turns last-bit differences of near-zero grads (fp32 atomics) into <= 2*lr per step
    assert (pg - pe).abs().max().item() <= 2 * 1e-3 * 5
    assert int(eng.rng[1]) == 5 * grad_accum and int(eng.step_ctr[0]) == 5
