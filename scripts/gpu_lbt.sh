set -o pipefail
mkdir -p gpurun_out/lb
timeout -k 10 400 python -u -m pytest tests/test_gpu_lb.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/lb/tests_lb.log 2>&1
