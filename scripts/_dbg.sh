set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u scripts/debug_parity.py efficientdet-d0 512 2 81 f32 grad > gpurun_out/dbg_d0_grad.txt 2>&1 &&
timeout -k 10 300 python -u scripts/debug_parity.py efficientdet-d4 1024 1 81 f32 fwd 1 > gpurun_out/dbg_d4_fwd.txt 2>&1 &&
timeout -k 10 300 python -u scripts/debug_parity.py efficientdet-d0 512 2 81 bf16 fwd 1 > gpurun_out/dbg_d0_bf16_fwd.txt 2>&1
