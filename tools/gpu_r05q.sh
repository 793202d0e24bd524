#!/bin/bash
# compile-time lazy activation in k_gemm_s / k_wgrad_tr: kernel tests, whole-step and per-launch
# A/B against the previous library (lib/libedet_base.so = the round-5 tile rules)
set -o pipefail
O=gpurun_out/r05q
mkdir -p $O
L=tensorflow2-machine-vision_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "conv1x1" > $O/pytest_conv1x1.log 2>&1 &&
TAG=r05q_ab VARIANTS="base:EDET_LIB=$L/libedet_base.so new:EDET_LIB=$L/libedet.so" REPS=3 bash tools/ab_bench.sh > $O/ab.log 2>&1 &&
TAG=r05q_abk REPS=1 bash tools/ab_kbench.sh > $O/abk.log 2>&1
