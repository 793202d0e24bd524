#!/bin/bash
# r03h: inference SE squeeze in the depthwise epilogue -- its tests, then config 2 with roofline tables.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03h
rm -rf $O && mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py -k "squeeze" tests/test_model_gpu.py > $O/pytest.log 2>&1
rc=$?
tail -5 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --workload backbone --batch 64 --steps 20 --warmup 5 --cpu-baseline 0 \
    > $O/r03h_config2_backbone_b64_bench.json 2> $O/config2.log
rc=$?
tail -16 $O/config2.log
cut -c1-300 $O/r03h_config2_backbone_b64_bench.json
exit $rc
