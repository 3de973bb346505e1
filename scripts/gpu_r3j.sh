# round 3: CT apply / GC kernel changes (LDS-staged create requests, block
# counters, four slots per GC thread): CT tests, C5 --ct-apply bench and its
# kernel trace (run via gpurun)
set -o pipefail
O=gpurun_out/r3k
mkdir -p $O
export TMPDIR=/tmp
T="python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 500 $T tests/test_gpu_lb.py tests/test_gpu_ctgc.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_multirank.py -k "lb or gc or ct or c5 or conntrack" > $O/t.log 2>&1
rc=$?
tail -8 $O/t.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u bench.py --workload c5 --ct-apply --no-cpu > $O/bench_c5ct.json 2> $O/bench_c5ct.err || { tail -20 $O/bench_c5ct.err; exit 1; }
grep -o '"ct_apply": {[^}]*}' $O/bench_c5ct.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py --workload c5 --ct-apply --steps 5 --warmup 2 --no-cpu > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
echo done
