set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gputest_r03a.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/gputest_r03a.log; exit 1; }
tail -3 gpurun_out/gputest_r03a.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_r03a_driver.json 2> gpurun_out/bench_r03a_driver.err && tail -c 3000 gpurun_out/bench_r03a_driver.json
