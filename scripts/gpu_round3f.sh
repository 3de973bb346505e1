# round 3: device CT apply for batches with a load balancer (run via gpurun)
set -o pipefail
mkdir -p gpurun_out/r3f
export CFC_DEBUG_APPLY=1
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 500 $T tests/test_gpu_lb.py > gpurun_out/r3f/t_lb.log 2>&1
rc=$?
tail -40 gpurun_out/r3f/t_lb.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 $T tests/test_gpu_parity.py -k "golden or ct or conntrack or c5 or gc" \
    > gpurun_out/r3f/t_ct.log 2>&1 || { tail -40 gpurun_out/r3f/t_ct.log; exit 1; }
tail -2 gpurun_out/r3f/t_ct.log

timeout -k 10 400 python -u bench.py --workload c5 --ct-apply --no-cpu --steps 20 --warmup 3 \
    > gpurun_out/r3f/c5a.json 2> gpurun_out/r3f/c5a.err || { tail -5 gpurun_out/r3f/c5a.err; exit 1; }
grep -o '"ct_apply": {[^}]*}' gpurun_out/r3f/c5a.json
echo done
