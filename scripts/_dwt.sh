set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_kernels_large_gpu.py -q -x -k "dwconv" --timeout 200 > $O/t.txt 2>&1; rc=$?; tail -3 $O/t.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/kbench.py --reps 10 --top 400 --filter dwconv --out $O/kb_pk.txt > $O/kb1.log 2>&1 &&
timeout -k 10 300 python scripts/kbench.py --reps 10 --top 400 --filter dwconv --dev 7=1 --out $O/kb_nopk.txt > $O/kb2.log 2>&1
rc=$?
head -4 $O/kb_pk.txt; head -4 $O/kb_nopk.txt
exit $rc
