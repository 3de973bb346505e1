# A/B (PIPE) then the GPU test suite, smoke, C2 bench and C5 --ct-apply (run via gpurun)
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu_ab3.sh libcfc.so libcfc_p1.so > gpurun_out/ab.txt 2>&1 &&
timeout -k 10 400 python -u bench.py --workload c5 --ct-apply --no-cpu > gpurun_out/bench_c5ct.json 2> gpurun_out/bench_c5ct.err &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread --durations=15 > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
