set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest -q -x tests/test_kernels_gpu.py -k "dwconv" > gpurun_out/dw_test.txt 2>&1 || { tail -30 gpurun_out/dw_test.txt; exit 1; }
for sh in "32 32 32 672 5 1" "32 128 128 144 3 1" "32 64 64 240 5 1" "32 16 16 1152 5 1" "32 128 128 144 5 2" "32 256 256 32 3 1" "32 256 256 96 3 2"; do
  timeout -k 10 60 python scripts/dw_probe.py $sh >> gpurun_out/dw_probe.txt 2>&1 || exit 1
done
