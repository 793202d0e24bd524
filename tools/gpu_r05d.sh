set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r05f; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py \
  -k "conv1x1 or dwconv_fwd or dws or long_blocks" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
L=tensorflow2-machine-vision_amd/lib
VARIANTS="base:EDET_LIB=$L/libedet_base.so,EDET_ALLOW_MISSING=1 fixed:EDET_LIB=$L/libedet.so" REPS=4 TAG=r05f_ab bash tools/ab_bench.sh &&
OLD=$L/libedet_base.so NEW=$L/libedet.so OLDENV="EDET_ALLOW_MISSING=1" REPS=2 TAG=r05f_abk HEADN=60 bash tools/ab_kbench.sh
