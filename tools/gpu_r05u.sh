#!/bin/bash
# k_gate_bn_reduce: one block per (image, 64-channel slice) owning its outputs for C >= 480 over
# H*W <= 4096: tests, whole-step and per-launch A/B against the previous library
set -o pipefail
O=gpurun_out/r05u
mkdir -p $O
L=tensorflow2-machine-vision_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "gate_bn_reduce or sesum or squeeze_excite" > $O/pytest.log 2>&1 &&
TAG=r05u_ab VARIANTS="base:EDET_LIB=$L/libedet_base.so new:EDET_LIB=$L/libedet.so" REPS=3 bash tools/ab_bench.sh > $O/ab.log 2>&1 &&
TAG=r05u_abk REPS=1 KB_ARGS="--filter gate_bn_reduce" bash tools/ab_kbench.sh > $O/abk.log 2>&1
