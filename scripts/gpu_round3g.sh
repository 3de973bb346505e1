# Round-3 re-entry check of HEAD: -m gpu tests (all, failures listed), the LB
# tests on the A/B library, smoke(), default C2 bench, A/B of libcfc_nd.so
# (stores not deferred), C5 --ct-apply at 20 steps, C3 bench, C2 kernel trace
set -o pipefail
O=gpurun_out/r3g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread --durations=25 > $O/gpu_tests.log 2>&1
rc=$?
tail -12 $O/gpu_tests.log
[ $rc -le 1 ] || exit 1
CFC_LIB=libcfc_nd.so timeout -k 10 300 python -u -m pytest tests/test_gpu_lb.py -v --timeout 200 --timeout-method thread > $O/lb_nd.log 2>&1
rc=$?
tail -5 $O/lb_nd.log
[ $rc -le 1 ] || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
for r in 1 2; do
  for lib in libcfc_nd.so libcfc.so; do
    CFC_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu > $O/ab_$lib.$r.json 2> $O/ab_$lib.$r.err || exit 1
    grep -o '"kernel_ms_per_launch": [0-9.]*' $O/ab_$lib.$r.json | sed "s/^/$lib r$r /"
  done
done
timeout -k 10 400 python -u bench.py --workload c5 --ct-apply --no-cpu > $O/bench_c5ct.json 2> $O/bench_c5ct.err || { tail -20 $O/bench_c5ct.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload c3 --no-cpu > $O/bench_c3.json 2> $O/bench_c3.err || { tail -20 $O/bench_c3.err; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
echo done
