set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest -q -x tests/test_kernels_gpu.py -k "squeeze or gate_bn" > gpurun_out/se_test.txt 2>&1 || { tail -40 gpurun_out/se_test.txt; exit 1; }
timeout -k 10 600 python -m pytest -q -x tests/test_model_gpu.py -k "train_step_parity_fp32 or bf16_within" > gpurun_out/se_model.txt 2>&1 || { tail -40 gpurun_out/se_model.txt; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline 0 --kernel-timing 0 > gpurun_out/se_bench.json 2> gpurun_out/se_bench.log || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/ktrace -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --cpu-baseline 0 --kernel-timing 0 > gpurun_out/ktrace.log 2>&1
