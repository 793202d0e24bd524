set -u
cd $GRAFT_REPO_ROOT
true
timeout -k 10 600 python scripts/d4_gnorm.py 14 > gpurun_out/d4_gnorm.txt 2>&1
