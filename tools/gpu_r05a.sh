set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r05a; mkdir -p $O
EDET_REPORT_DIR=$O timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_augment_gpu.py tests/test_bench_dp_gpu.py \
  -k "sesum or bwd_lazy or folds_equal or dws or wgrad or dgrad_fold or dwconv or skip_nonfinite or bn_moving or squeeze or conv1x1 or optimizer or augment or blur or warp or resize or identity_chain or bench_two_ranks" > $O/pytest.log 2>&1
rc=$?; tail -5 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
L=tensorflow2-machine-vision_amd/lib
VARIANTS="base:EDET_LIB=$L/libedet_base.so patches:EDET_LIB=$L/libedet.so,EDET_LAZY_DY=0,EDET_SESUM_DGRAD=0 lazy:EDET_LIB=$L/libedet.so,EDET_SESUM_DGRAD=0 new:EDET_LIB=$L/libedet.so" REPS=3 TAG=r05a_ab bash tools/ab_bench.sh
