#!/bin/bash
# register-blocked depthwise dgrad with compile-time accumulate: tests, whole-step and
# per-launch A/B against the previous library
set -o pipefail
O=gpurun_out/r05at
mkdir -p $O
L=tensorflow2-machine-vision_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "dwconv_dgrad" > $O/pytest.log 2>&1 &&
TAG=r05at_ab VARIANTS="base:EDET_LIB=$L/libedet_base.so new:EDET_LIB=$L/libedet.so" REPS=3 bash tools/ab_bench.sh > $O/ab.log 2>&1 &&
TAG=r05at_abk REPS=1 KB_ARGS="--filter dwconv_dgrad_fold,dwconv_dgrad" bash tools/ab_kbench.sh > $O/abk.log 2>&1
