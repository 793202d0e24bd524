#!/bin/bash
# r03aj: full GPU suite and smoke on the final round-3 tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03aj
rm -rf $O && mkdir -p $O
timeout -k 10 500 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_all.log 2>&1
rc=$?
tail -2 $O/pytest_all.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
