set -u
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest -q -x -m gpu tests > gpurun_out/t_new.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/t_new.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --overlap 0 > gpurun_out/bench0.json 2> gpurun_out/bench0.log; echo "bench rc=$?"; grep "img/s" gpurun_out/bench0.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --overlap 1 > gpurun_out/bench1.json 2> gpurun_out/bench1.log; echo "bench rc=$?"; grep "img/s\|roofline" gpurun_out/bench1.log
