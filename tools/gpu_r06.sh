#!/bin/bash
# Round-6 launcher: named step lists over the tests / bench / probes of this round.
#   gpurun -- 'TAG=r06a STEPS="newtests bench gemmprobe" bash tools/gpu_r06.sh'
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r06}
O=gpurun_out/$TAG
mkdir -p $O
for step in ${STEPS:-}; do
  echo "[gpu_r06] $step"
  case $step in
    newtests)
      EDET_REPORT_DIR=$O/parity timeout -k 10 1000 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu \
          tests/test_headline_gpu.py tests/test_augment_gpu.py tests/test_kernels_gpu.py \
          -k "${TESTS_K:-bf16_emulated or b64_backbone or getdataset or conv1x1_fwd}" > $O/pytest.log 2>&1
      rc=$?; tail -12 $O/pytest.log; [ $rc -eq 0 ] || exit $rc ;;
    tests)
      EDET_REPORT_DIR=$O/parity timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests \
          -k "${TESTS_K:-}" > $O/pytest_k.log 2>&1
      rc=$?; tail -8 $O/pytest_k.log; [ $rc -eq 0 ] || exit $rc ;;
    bench)
      timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.log
      rc=$?; tail -3 $O/bench.log; cut -c1-400 $O/bench.json; [ $rc -eq 0 ] || exit $rc ;;
    gemmprobe)
      timeout -k 10 300 python scripts/gemm_probe.py ${GP_SHAPES:-8192x192x1152 32768x112x672 32768x80x480 131072x40x240 8192x320x64 32768x64x64 8192x64x64 32768x112x64} \
          > $O/gemm_probe.txt 2>&1
      rc=$?; cat $O/gemm_probe.txt | cut -c1-120; [ $rc -eq 0 ] || exit $rc ;;
    kbench)
      timeout -k 10 400 python scripts/kbench.py --top 400 ${KB_ARGS:-} --out $O/${TAG}_kbench.txt > $O/kbench.log 2>&1
      rc=$?; head -32 $O/${TAG}_kbench.txt 2>/dev/null; tail -3 $O/kbench.log; [ $rc -eq 0 ] || exit $rc ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[gpu_r06] done"
