#!/bin/bash
# BN-backward apply with nontemporal rows over >= 524288 rows: tests, whole-step and
# per-launch A/B against the previous library
set -o pipefail
O=gpurun_out/r05ao
mkdir -p $O
L=tensorflow2-machine-vision_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "lazy or apply" > $O/pytest.log 2>&1 &&
TAG=r05ao_ab VARIANTS="base:EDET_LIB=$L/libedet_base.so new:EDET_LIB=$L/libedet.so" REPS=3 bash tools/ab_bench.sh > $O/ab.log 2>&1 &&
TAG=r05ao_abk REPS=1 KB_ARGS="--filter lazy_bwd_apply" bash tools/ab_kbench.sh > $O/abk.log 2>&1
