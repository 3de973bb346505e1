# round 3: fixes (IPv6 LB unknown-proto rewrite, CT shard accounting), the CT
# apply rework (A/B against the previous build), C3 bench line (run via gpurun)
set -o pipefail
mkdir -p gpurun_out/r3e
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 500 $T tests/test_gpu_lb.py tests/test_gpu_multirank.py \
    > gpurun_out/r3e/t_lb_mr.log 2>&1 || { tail -30 gpurun_out/r3e/t_lb_mr.log; exit 1; }
tail -2 gpurun_out/r3e/t_lb_mr.log
timeout -k 10 500 $T tests/test_gpu_parity.py -k "ct or conntrack or c5 or gc" \
    > gpurun_out/r3e/t_ct.log 2>&1 || { tail -30 gpurun_out/r3e/t_ct.log; exit 1; }
tail -2 gpurun_out/r3e/t_ct.log
for lib in libcfc_apold.so libcfc.so; do
  CFC_LIB=$lib timeout -k 10 400 python -u bench.py --workload c5 --ct-apply --no-cpu \
      --steps 20 --warmup 3 > gpurun_out/r3e/c5a_$lib.json 2> gpurun_out/r3e/c5a_$lib.err || exit 1
  grep -o '"apply_and_gc_ms_per_step": [0-9.]*' gpurun_out/r3e/c5a_$lib.json | sed "s/^/$lib /"
done
timeout -k 10 400 python -u bench.py --workload c3 > gpurun_out/r3e/c3.json 2> gpurun_out/r3e/c3.err || exit 1
echo done
