# Round-3 check: -m gpu tests, smoke(), default C2 bench, C5 --ct-apply at 20 steps (run via gpurun)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread --durations=25 > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err &&
timeout -k 10 400 python -u bench.py --workload c5 --ct-apply --no-cpu > gpurun_out/bench_c5ct.json 2> gpurun_out/bench_c5ct.err
