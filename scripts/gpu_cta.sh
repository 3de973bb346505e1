# device CT apply check + timing (run via gpurun)
set -o pipefail
mkdir -p gpurun_out/cta
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_epochs.py tests/test_gpu_lb.py -m gpu -k "ct or c5 or lb" -x -v --timeout 300 --timeout-method thread > gpurun_out/cta/tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --workload c5 --ct-apply --steps 3 --warmup 1 --no-cpu > gpurun_out/cta/bench_ct.json 2> gpurun_out/cta/bench_ct.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/cta/ktct -o run --output-format csv -- python3 bench.py --workload c5 --ct-apply --steps 2 --warmup 1 --no-cpu > gpurun_out/cta/ktct.log 2>&1
