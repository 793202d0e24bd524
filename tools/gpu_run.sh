#!/bin/bash
# One launcher for the GPU box (replaces the per-experiment tools/gpu_r03*.sh of round 3).
#
#   gpurun --timeout 1200 -- 'TAG=r04a STEPS="suite measure configs" bash tools/gpu_run.sh'
#
# STEPS (run in order, the first failure ends the call):
#   suite    pytest -m gpu (parity reports under $O/parity) + __graft_entry__.smoke()
#   tests    pytest -m gpu -k "$K" only (TESTS_K), no reports
#   bench    bench.py with the default arguments
#   measure  scripts/measure.sh: PMC traffic + MFMA passes, bench, rocprof kernel stats, kbench
#   configs  BASELINE config 2 (B0 backbone 224, B = 64) and config 5 (D4 1024, B = 8) bench lines
#   kbench   scripts/kbench.py per-launch table only (KB_ARGS passed through)
# Results land in gpurun_out/$TAG/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-dev}
STEPS=${STEPS:-suite}
O=gpurun_out/$TAG
mkdir -p $O
for step in $STEPS; do
  echo "[gpu_run] $step"
  case $step in
    suite)
      EDET_REPORT_DIR=$O/parity timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread \
          -m gpu tests > $O/pytest_gpu.log 2>&1
      rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
      rc=$?; tail -2 $O/smoke.log; [ $rc -eq 0 ] || exit $rc ;;
    tests)
      timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
          -k "${TESTS_K:-}" > $O/pytest_k.log 2>&1
      rc=$?; tail -5 $O/pytest_k.log; [ $rc -eq 0 ] || exit $rc ;;
    bench)
      timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.log
      rc=$?; tail -3 $O/bench.log; cut -c1-300 $O/bench.json; [ $rc -eq 0 ] || exit $rc ;;
    measure)
      env -u STEPS TAG=$TAG bash scripts/measure.sh > $O/measure.log 2>&1
      rc=$?; tail -8 $O/measure.log; [ $rc -eq 0 ] || exit $rc ;;
    configs)
      timeout -k 10 400 python bench.py --workload backbone --batch 64 --steps 20 --warmup 5 --cpu-baseline 0 \
          > $O/${TAG}_config2_backbone_b64_bench.json 2> $O/config2.log &&
      timeout -k 10 600 python bench.py --model efficientdet-d4 --batch 8 --steps 10 --warmup 3 --cpu-baseline 0 \
          > $O/${TAG}_config5_d4_b8_1gpu_bench.json 2> $O/config5.log
      rc=$?
      cut -c1-200 $O/${TAG}_config2_backbone_b64_bench.json $O/${TAG}_config5_d4_b8_1gpu_bench.json
      [ $rc -eq 0 ] || exit $rc ;;
    kbench)
      timeout -k 10 400 python scripts/kbench.py --top 400 ${KB_ARGS:-} --out $O/${TAG}_kbench.txt \
          > $O/kbench.log 2>&1
      rc=$?; head -30 $O/${TAG}_kbench.txt 2>/dev/null; tail -3 $O/kbench.log; [ $rc -eq 0 ] || exit $rc ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[gpu_run] done"
