#!/bin/bash
# Round-6 library A/B call: GPU tests of the touched kernels (TESTS_K) on the new library, then
# per-launch (kbench, KB_FILTER) and whole-step (bench.py) A/Bs of lib/libedet_base.so (old)
# against lib/libedet.so (new).  Needs libedet_base.so un-ignored in .gpurunignore for the call.
#   gpurun -- 'TAG=r06w TESTS_K="detection_loss or lazy_backward" KB_FILTER=edet_detection_loss bash tools/gpu_r06_ab.sh'
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r06ab}
O=gpurun_out/$TAG; mkdir -p $O
L=tensorflow2-machine-vision_amd/lib
if [ -n "${TESTS_K:-}" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests -k "$TESTS_K" > $O/pytest.log 2>&1
  rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${KB_FILTER:-}" ]; then
  TAG=$TAG/abk OLD=$L/libedet_base.so NEW=$L/libedet.so OLDENV="EDET_ALLOW_MISSING=1" REPS=2 HEADN=${HEADN:-40} KB_ARGS="--filter $KB_FILTER" \
      bash tools/ab_kbench.sh || exit 1
fi
STEPS=30 TAG=$TAG/ab VARIANTS="old:EDET_LIB=$L/libedet_base.so,EDET_ALLOW_MISSING=1 new:EDET_LIB=$L/libedet.so" REPS=${ABREPS:-3} bash tools/ab_bench.sh
