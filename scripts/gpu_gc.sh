# CT GC tests, then the kernel A/B (run via gpurun)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ctgc.py tests/test_gpu_epochs.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gc_tests.log 2>&1 || { tail -40 gpurun_out/gc_tests.log; exit 1; }
tail -3 gpurun_out/gc_tests.log
bash scripts/gpu_ab2.sh libcfc.so libcfc_exp3.so libcfc_exp5.so
