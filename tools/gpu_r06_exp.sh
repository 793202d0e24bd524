#!/bin/bash
# Round-6 experiment call: tests, per-shape GEMM probe, and per-launch (abk:<lib>, old = <lib>,
# new = libedet.so) / whole-step (ab:<lib>,...) A/Bs of hand-built libraries against the
# production one
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r06x}
O=gpurun_out/$TAG
mkdir -p $O
L=tensorflow2-machine-vision_amd/lib
for step in ${STEPS:-}; do
  echo "[exp] $step"
  case $step in
    probe:*)
      lib=${step#probe:}
      EDET_LIB=$L/$lib.so timeout -k 10 300 python scripts/gemm_probe.py ${GP_SHAPES:-} > $O/gemm_probe_$lib.txt 2>&1
      rc=$?; [ $rc -eq 0 ] || { tail -5 $O/gemm_probe_$lib.txt; exit $rc; } ;;
    abk:*)
      lib=${step#abk:}
      TAG=$TAG/abk_$lib OLD=$L/$lib.so NEW=$L/libedet.so OLDENV="EDET_ALLOW_MISSING=1" REPS=${REPS:-2} HEADN=${HEADN:-40} \
          bash tools/ab_kbench.sh || exit 1 ;;
    ab:*)
      libs=${step#ab:}
      V="base:EDET_LIB=$L/libedet.so"
      for l in ${libs//,/ }; do V="$V $l:EDET_LIB=$L/$l.so,EDET_ALLOW_MISSING=1"; done
      STEPS=30 TAG=$TAG/ab VARIANTS="$V" REPS=${ABREPS:-3} bash tools/ab_bench.sh || exit 1 ;;
    tests)
      timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
          -k "${TESTS_K:-}" > $O/pytest.log 2>&1
      rc=$?; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit $rc ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[exp] done"
