set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
P=$PWD/tensorflow2-machine-vision_amd
timeout -k 10 300 python -m pytest -q -x tests/test_kernels_gpu.py tests/test_kernels_large_gpu.py -k "dw" > gpurun_out/dw_test.txt 2>&1 || { tail -30 gpurun_out/dw_test.txt; exit 1; }
: > gpurun_out/dw_sweep.txt
for v in lib_p1 lib; do
  echo "== $v" >> gpurun_out/dw_sweep.txt
  EDET_LIB=$P/$v/libedet.so timeout -k 10 120 python scripts/dw_sweep.py fwd >> gpurun_out/dw_sweep.txt 2>&1 || exit 1
  EDET_LIB=$P/$v/libedet.so timeout -k 10 120 python scripts/dw_sweep.py wgrad >> gpurun_out/dw_sweep.txt 2>&1 || exit 1
done
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline 0 --kernel-timing 0 > gpurun_out/dw_bench.json 2> gpurun_out/dw_bench.log || exit 1
