#!/bin/bash
# k_dwt chunks spanning images: the fused depthwise backward tests incl. the spanning shapes
set -o pipefail
O=gpurun_out/r05ah
mkdir -p $O
L=tensorflow2-machine-vision_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "dwconv_bwd_fused" > $O/pytest.log 2>&1
