set -u
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest -q -x -m gpu tests > gpurun_out/t_new.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/t_new.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/bench.json 2> gpurun_out/bench.log; echo "bench rc=$?"; grep "img/s" gpurun_out/bench.log
timeout -k 10 200 python scripts/kbench.py --out gpurun_out/kb_new.txt --top 400 > /dev/null 2>gpurun_out/kb_new.err || exit 1
