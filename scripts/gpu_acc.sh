# CT accounting check + timing (run via gpurun)
set -o pipefail
mkdir -p gpurun_out/acc
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lb.py -m gpu -k "c5 or ct or lb" -x -v --timeout 300 --timeout-method thread > gpurun_out/acc/tests.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -k "c5" -x -v --timeout 300 --timeout-method thread > gpurun_out/acc/tests_full.log 2>&1 &&
timeout -k 10 300 python -u bench.py --workload c5 --no-cpu > gpurun_out/acc/bench.json 2> gpurun_out/acc/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/acc/kt -o run --output-format csv -- python3 bench.py --workload c5 --steps 3 --warmup 1 --no-cpu > gpurun_out/acc/kt.log 2>&1
