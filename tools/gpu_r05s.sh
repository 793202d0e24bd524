#!/bin/bash
# compile-time input activation in the BiFPN fusion kernels: tests, whole-step and per-launch A/B
set -o pipefail
O=gpurun_out/r05s
mkdir -p $O
L=tensorflow2-machine-vision_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "fuse or maxpool" > $O/pytest_fuse.log 2>&1 &&
TAG=r05s_ab VARIANTS="base:EDET_LIB=$L/libedet_base.so new:EDET_LIB=$L/libedet.so" REPS=3 bash tools/ab_bench.sh > $O/ab.log 2>&1 &&
TAG=r05s_abk REPS=1 KB_ARGS="--filter bifpn" bash tools/ab_kbench.sh > $O/abk.log 2>&1
