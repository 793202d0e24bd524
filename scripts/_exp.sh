set -u
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --workload backbone --batch 64 --steps 20 --warmup 5 > gpurun_out/bench_bb.json 2> gpurun_out/bench_bb.log; echo "bb rc=$?"; tail -2 gpurun_out/bench_bb.log
timeout -k 10 400 python bench.py --model efficientdet-d4 --batch 8 --steps 10 --warmup 3 --cpu-baseline 0 --kernel-timing 0 > gpurun_out/bench_d4.json 2> gpurun_out/bench_d4.log; echo "d4 rc=$?"; tail -3 gpurun_out/bench_d4.log
