#!/bin/bash
# r03ai: fusion-forward grid cap 2048 -- fusion tests (incl. a strided grid), model tests, then the
# default bench line of the same tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03ai
rm -rf $O && mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py -k "fuse" tests/test_model_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 > $O/bench.json 2> $O/bench.log || { tail -5 $O/bench.log; exit 1; }
cut -c1-200 $O/bench.json
