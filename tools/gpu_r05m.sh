#!/bin/bash
# K-loop tile rules (round 5): conv1x1 kernel tests, whole-step A/B and per-launch A/B against
# the previous library (lib/libedet_base.so)
set -o pipefail
O=gpurun_out/r05m
mkdir -p $O
L=tensorflow2-machine-vision_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "conv1x1_fwd or conv1x1_dgrad" > $O/pytest_conv1x1.log 2>&1 &&
TAG=r05m_ab VARIANTS="base:EDET_LIB=$L/libedet_base.so new:EDET_LIB=$L/libedet.so" REPS=3 bash tools/ab_bench.sh > $O/ab.log 2>&1 &&
TAG=r05m_abk REPS=1 bash tools/ab_kbench.sh > $O/abk.log 2>&1
