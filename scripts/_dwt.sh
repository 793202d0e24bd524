set -u
cd $GRAFT_REPO_ROOT
P=$PWD/tensorflow2-machine-vision_amd
EDET_LIB=$P/lib_d3/libedet.so timeout -k 10 300 python -m pytest -q -x tests/test_kernels_gpu.py tests/test_kernels_large_gpu.py -k "dw" > gpurun_out/dw_test.txt 2>&1 || { tail -30 gpurun_out/dw_test.txt; exit 1; }
: > gpurun_out/dw_sweep.txt
for v in lib lib_d1 lib_d2 lib_d3 lib_d3t1k lib_d1t1k; do
  echo "== $v" >> gpurun_out/dw_sweep.txt
  EDET_LIB=$P/$v/libedet.so timeout -k 10 120 python scripts/dw_sweep.py fwd >> gpurun_out/dw_sweep.txt 2>&1 || exit 1
done
