# C5 check (run via gpurun): CT GPU tests, C5 bench, kernel trace, ct-apply bench
set -o pipefail
mkdir -p gpurun_out/c5
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -k "c5" -x -v --timeout 300 --timeout-method thread > gpurun_out/c5/tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --workload c5 --no-cpu > gpurun_out/c5/bench.json 2> gpurun_out/c5/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c5/kt -o run --output-format csv -- python3 bench.py --workload c5 --steps 3 --warmup 1 --no-cpu > gpurun_out/c5/kt.log 2>&1 &&
timeout -k 10 300 python -u bench.py --workload c5 --ct-apply --steps 2 --warmup 1 --no-cpu > gpurun_out/c5/bench_ct.json 2> gpurun_out/c5/bench_ct.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c5/ktct -o run --output-format csv -- python3 bench.py --workload c5 --ct-apply --steps 2 --warmup 1 --no-cpu > gpurun_out/c5/ktct.log 2>&1
