"""Build the native extension ``ddim_cold_amd/_C.so`` in-tree with hipcc.

Every ``csrc/*.hip`` kernel translation unit is compiled for gfx950 only
(``--offload-arch=gfx950``), plus ``csrc/bindings.cpp`` (TORCH_LIBRARY
registrations), then linked against libtorch.  No hipify step, no CUDA
sources, no multi-arch dispatch.  Objects are cached by content hash under
``build/`` so rebuilds only touch changed files.

Usage::

    python -m ddim_cold_amd.build            # build (incremental)
    python -m ddim_cold_amd.build --force    # rebuild everything
    python -m ddim_cold_amd.build --resource-usage   # print VGPR/LDS/occupancy per kernel
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import re
import subprocess
import sys
import sysconfig

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
BUILD = os.path.join(ROOT, "build", "ddim_cold_amd")
OUT = os.path.join(PKG, "_C.so")
ARCH = os.environ.get("DDIM_COLD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _torch_paths():
    import torch
    import torch.utils.cpp_extension as ce
    inc = ce.include_paths("cuda")
    libdir = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, libdir, abi


def _flags(inc, abi, resource_usage=False):
    py_inc = sysconfig.get_paths()["include"]
    f = [
        "-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}",
        "-DUSE_ROCM=1", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_EXTENSION_NAME=_C",
        "-Wno-unused-result", "-Wno-deprecated-declarations", "-Wno-unused-command-line-argument",
        "-fno-gpu-rdc", "-munsafe-fp-atomics",
    ]
    # per-kernel resource remarks (codegen unchanged): the build checks them for
    # scratch memory, see _check_scratch
    f.append("-Rpass-analysis=kernel-resource-usage")
    # DDIM_COLD_HIPFLAGS: extra hipcc flags (e.g. "-save-temps" to inspect the ISA)
    f += os.environ.get("DDIM_COLD_HIPFLAGS", "").split()
    for d in inc + [py_inc, CSRC, "/opt/rocm/include"]:
        f += ["-I", d]
    return f


# Codegen flag for every kernel unit: -amdgpu-mfma-vgpr-form (MFMA accumulators
# in VGPRs instead of AGPRs).  In the flash attention forward the softmax reads
# every score accumulator and rescales the output accumulators, so the AGPR form
# paid a v_accvgpr_read/write per element per tile (96 per 32 MFMAs in the loop's
# .s) and 204 registers (occupancy 2); the VGPR form has none and 152 registers
# (occupancy 3).  Whole-tree A/B on MI355X (tools/gpu_r3_attn.sh, 2 interleaved
# 1000-step pairs): attention unit only 0.7982/0.8012 ms/step, every unit
# 0.7939/0.7954, neither 0.8079/0.8041; sampler k=20 N=64 38.54 / 37.78 / 38.79 ms.
def _unit_flags(src, flags):
    return flags + (["-mllvm", "-amdgpu-mfma-vgpr-form"] if src.endswith(".hip") else [])


def _hash(path, flags):
    h = hashlib.sha256()
    h.update(" ".join(flags).encode())
    with open(path, "rb") as fh:
        h.update(fh.read())
    for hdr in sorted(os.listdir(CSRC)):
        if hdr.endswith(".h"):
            with open(os.path.join(CSRC, hdr), "rb") as fh:
                h.update(fh.read())
    return h.hexdigest()[:16]


def _compile(src, flags, force):
    name = os.path.splitext(os.path.basename(src))[0]
    key = _hash(src, flags)
    obj = os.path.join(BUILD, f"{name}.{key}.o")
    if os.path.isfile(obj) and os.path.isfile(obj + ".log") and not force:
        with open(obj + ".log") as fh:
            return obj, fh.read()
    cmd = [HIPCC] + flags + ["-c", src, "-o", obj + ".tmp"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr[-8000:]}")
    with open(obj + ".log", "w") as fh:
        fh.write(r.stderr)
    os.replace(obj + ".tmp", obj)
    return obj, r.stderr


def _check_scratch(logs):
    """Fail the build if a GPU kernel uses scratch (private) memory: on gfx950 that
    is a global-memory round trip per access -- a dynamically indexed register
    array once put the patch-embedding epilogue there and cost ~4 us per launch.
    DDIM_COLD_ALLOW_SCRATCH=1 downgrades this to a warning."""
    bad = []
    for log in logs:
        for blk in (log or "").split("Function Name: ")[1:]:
            m = re.search(r"ScratchSize \[bytes/lane\]: (\d+)", blk)
            if m and int(m.group(1)) > 0:
                bad.append(f"{blk.split()[0]} ({m.group(1)} B/lane)")
    if not bad:
        return
    msg = "GPU kernels using scratch memory:\n  " + "\n  ".join(bad)
    if os.environ.get("DDIM_COLD_ALLOW_SCRATCH") == "1":
        print("[ddim_cold_amd.build] warning: " + msg)
    else:
        raise RuntimeError(msg)


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hip", ".cpp")))


def build(force: bool = False, jobs: int | None = None, resource_usage: bool = False, verbose: bool = True) -> str:
    os.makedirs(BUILD, exist_ok=True)
    inc, libdir, abi = _torch_paths()
    flags = _flags(inc, abi, resource_usage)
    srcs = sources()
    jobs = jobs or min(len(srcs), max(1, min(8, (os.cpu_count() or 4))))
    objs, logs = [], []
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = {ex.submit(_compile, s, _unit_flags(s, flags), force): s for s in srcs}
        for fut in cf.as_completed(futs):
            obj, log = fut.result()
            objs.append(obj)
            logs.append(log)
            if verbose and log and resource_usage:
                print(log)
    _check_scratch(logs)
    objs.sort()
    newest = max(os.path.getmtime(o) for o in objs)
    if force or not os.path.isfile(OUT) or os.path.getmtime(OUT) < newest or _stale_link(objs):
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", OUT + ".tmp"] + objs + [
            "-L", libdir, "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
            # RCCL: torch's own librccl.so by path (no SONAME; the loader matches the
            # file PyTorch already loaded, so the process keeps ONE RCCL instance)
            os.path.join(libdir, "librccl.so"),
            f"-Wl,-rpath,{libdir}",
        ]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-8000:]}")
        _check_stubs(OUT + ".tmp")
        os.replace(OUT + ".tmp", OUT)
        with open(OUT + ".objs", "w") as fh:
            fh.write("\n".join(os.path.basename(o) for o in objs))
        if verbose:
            print(f"[ddim_cold_amd.build] linked {OUT} ({len(objs)} objects, arch {ARCH})")
    elif verbose:
        print(f"[ddim_cold_amd.build] up to date: {OUT}")
    return OUT


def _check_stubs(so):
    """Fail the build if any kernel launch stub is undefined (a hipcc template-instantiation bug)."""
    r = subprocess.run(["nm", "-u", so], capture_output=True, text=True)
    bad = [l.split()[-1] for l in r.stdout.splitlines() if "__device_stub__" in l]
    if bad:
        os.remove(so)
        raise RuntimeError("undefined kernel launch stubs (add explicit instantiations):\n  " + "\n  ".join(bad))


def _stale_link(objs):
    rec = OUT + ".objs"
    if not os.path.isfile(rec):
        return True
    with open(rec) as fh:
        return fh.read().split("\n") != [os.path.basename(o) for o in objs]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=None)
    ap.add_argument("--resource-usage", action="store_true")
    a = ap.parse_args(argv)
    build(force=a.force, jobs=a.jobs, resource_usage=a.resource_usage)


if __name__ == "__main__":
    sys.exit(main())
