#!/bin/bash
# round-2 parity tests on the GPU box (reports under gpurun_out/reports)
export EDET_REPORT_DIR=gpurun_out/reports
timeout -k 10 1100 python -u -m pytest -v --timeout 900 --timeout-method thread \
  tests/test_headline_gpu.py tests/test_dp_gpu.py \
  "tests/test_kernels_gpu.py::test_detection_loss" > gpurun_out/gpu_new.log 2>&1
