set -u
cd $GRAFT_REPO_ROOT
TEST_TIMEOUT=700 SKIP_BENCH=1 bash scripts/gpu_check.sh > gpurun_out/check.txt 2>&1 || exit $?
TAG=r02d bash scripts/measure.sh > gpurun_out/measure.txt 2>&1
rc=$?
tail -3 gpurun_out/check.txt; tail -20 gpurun_out/measure.txt | cut -c1-300
timeout -k 10 300 python scripts/kbench.py --reps 10 --top 400 --out gpurun_out/kbench_r02d.txt > gpurun_out/kbench.log 2>&1
exit $rc
