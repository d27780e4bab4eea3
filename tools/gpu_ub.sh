#!/bin/bash
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 200 python tools/ubench.py > gpurun_out/ub_graph.log 2>&1 || exit $?
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 200 python tools/ubench.py > gpurun_out/ub_graph_devkarg.log 2>&1 || exit $?
DDIM_COLD_GEMM_NO_DMA=1 timeout -k 10 200 python tools/ubench.py > gpurun_out/ub_graph_nodma.log 2>&1 || exit $?
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-sampler > gpurun_out/bench_devkarg.log 2>&1 || exit $?
tail -1 gpurun_out/bench_devkarg.log
