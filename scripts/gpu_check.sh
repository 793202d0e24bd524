#!/bin/bash
# GPU round: build, GPU parity tests, smoke, short bench (+ optional rocprof). Stops at the
# first fault/abort/timeout; ordinary test failures (rc 1) do not stop the later steps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
make -C tensorflow2-machine-vision_amd -j16 > $OUT/build.log 2>&1 || { echo "build failed"; tail -20 $OUT/build.log; exit 10; }
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-700} python -m pytest tests -m gpu -q -rf ${PYTEST_ARGS:-} > $OUT/pytest.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -30 $OUT/pytest.log
  ok $rc || exit $rc
fi
if [ "${SKIP_SMOKE:-0}" != "1" ]; then
  timeout -k 10 300 python __graft_entry__.py smoke > $OUT/smoke.log 2>&1; rc=$?
  echo "smoke rc=$rc"; tail -5 $OUT/smoke.log
  ok $rc || exit $rc
fi
if [ "${SKIP_BENCH:-0}" != "1" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py ${BENCH_ARGS:---steps 10 --warmup 3} > $OUT/bench.json 2> $OUT/bench.log; rc=$?
  echo "bench rc=$rc"; tail -25 $OUT/bench.log; cat $OUT/bench.json
  [ $rc -eq 0 ] || exit $rc
fi
if [ "${PROFILE:-0}" = "1" ]; then
  export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --cpu-baseline 0 --kernel-timing 0 > $OUT/prof.log 2>&1; rc=$?
  echo "rocprof rc=$rc"; tail -5 $OUT/prof.log
fi
