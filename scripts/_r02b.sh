set -u
cd $GRAFT_REPO_ROOT
TEST_TIMEOUT=900 bash scripts/gpu_check.sh > gpurun_out/check.txt 2>&1 || exit $?
timeout -k 10 300 python scripts/kbench.py --reps 10 --top 400 --out gpurun_out/kbench_r02c.txt > gpurun_out/kbench.log 2>&1
