"""Diagnose the trainer overlap parity: runs tools/trainer_overlap_gpu.py in several
modes and prints the per-parameter relative errors against the single process.

    python tools/overlap_diag.py > gpurun_out/overlap_diag.txt
"""
import json
import os
import subprocess
import sys
import tempfile

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(d, name, force, layout, env_extra):
    out = os.path.join(d, name + ".pt")
    env = dict(os.environ, PYTHONPATH=ROOT)
    env.pop("DDIM_COLD_FAKE_COMM", None)
    env.update(env_extra)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "trainer_overlap_gpu.py"), out,
                        "1" if force else "0", layout or "-"], capture_output=True, text=True, timeout=300,
                       env=env, cwd=d)
    if r.returncode != 0:
        print(name, "FAILED", r.stderr[-1500:], flush=True)
        return None
    res = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    print(name, res, flush=True)
    return torch.load(out, weights_only=True)


def frob(a, b, name=""):
    a, b = a.double(), b.double()
    if name.endswith("attn.qkv.bias"):  # key bias: zero true gradient (see the GPU test)
        n = a.numel() // 3
        a, b = torch.cat((a[:n], a[2 * n:])), torch.cat((b[:n], b[2 * n:]))
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def main():
    steps = os.environ.get("OVERLAP_STEPS", "60")
    with tempfile.TemporaryDirectory() as d:
        base = {"OVERLAP_STEPS": steps}
        single = run(d, "single", False, None, base)
        modes = [
            ("ov", True, "overlap-2", {}),
            ("inline", True, "inline-1", {}),
            ("fake_ov", True, "overlap-2", {"DDIM_COLD_FAKE_COMM": "1"}),
            ("fake_ov_post", True, "overlap-2", {"DDIM_COLD_FAKE_COMM": "1", "DDIM_COLD_PREISSUE": "0"}),
            ("fake_in", True, "inline-1", {"DDIM_COLD_FAKE_COMM": "1"}),
            ("fake_ov4", True, "overlap-4", {"DDIM_COLD_FAKE_COMM": "1"}),
        ]
        for name, force, layout, env in modes:
            p = run(d, name, force, layout, dict(base, **env))
            if p is None or single is None:
                continue
            rows = sorted(((frob(p[k], single[k], k), k) for k in single), reverse=True)
            print(f"  {name} vs single: " + ", ".join(f"{k} {e:.2e}" for e, k in rows[:8]), flush=True)


if __name__ == "__main__":
    main()
