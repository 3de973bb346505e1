# round 3 check of HEAD: the whole -m gpu suite, smoke(), the default C2
# bench, C5 --ct-apply (20 steps, GC at the reference's cadence), C3, and a
# kernel trace of the default bench (run via gpurun)
set -o pipefail
O=gpurun_out/r3final2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider --durations=15 > $O/gpu_tests.log 2>&1
rc=$?
tail -6 $O/gpu_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
timeout -k 10 400 python -u bench.py --workload c5 --ct-apply --no-cpu > $O/bench_c5ct.json 2> $O/bench_c5ct.err || { tail -20 $O/bench_c5ct.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload c3 --no-cpu > $O/bench_c3.json 2> $O/bench_c3.err || { tail -20 $O/bench_c3.err; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
echo done
