set -u
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest -q -x -m gpu tests/test_anchors_gpu.py tests/test_model_gpu.py -k "detect or test_step" > gpurun_out/t_nms.log 2>&1; echo "nms tests rc=$?"; tail -30 gpurun_out/t_nms.log
