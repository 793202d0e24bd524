set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest -q -x tests/test_kernels_gpu.py tests/test_kernels_large_gpu.py -k "conv1x1" > gpurun_out/gs_test.txt 2>&1 || { tail -40 gpurun_out/gs_test.txt; exit 1; }
timeout -k 10 600 python -m pytest -q -x tests/test_model_gpu.py -k "train_step_parity_fp32 or forward_parity" > gpurun_out/gs_model.txt 2>&1 || { tail -40 gpurun_out/gs_model.txt; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline 0 --kernel-timing 0 > gpurun_out/gs_bench.json 2> gpurun_out/gs_bench.log || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/ktrace -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --cpu-baseline 0 --kernel-timing 0 > gpurun_out/ktrace.log 2>&1
