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
    limiter)
      EAGER="python bench.py --steps 3 --warmup 1 --graph 0 --cpu-baseline 0 --kernel-timing 0"
      rm -rf $O/pmc_lima $O/pmc_limb
      timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
          SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE --kernel-trace -d $O/pmc_lima -o run \
          --output-format csv -- $EAGER > $O/pmc_lima.log 2>&1 &&
      timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT \
          SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --kernel-trace -d $O/pmc_limb -o run \
          --output-format csv -- $EAGER > $O/pmc_limb.log 2>&1 &&
      python scripts/pmc_limiter.py --a $O/pmc_lima --b $O/pmc_limb --steps 6 --tag $TAG --out $O/pmc_limiter.json \
          > $O/${TAG}_pmc_limiter.txt
      rc=$?; find $O -name "*.db" -delete 2>/dev/null; head -40 $O/${TAG}_pmc_limiter.txt; [ $rc -eq 0 ] || { tail -5 $O/pmc_lima.log $O/pmc_limb.log; exit $rc; } ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[gpu_r06] done"
