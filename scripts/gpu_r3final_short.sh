# round 3, HEAD: the whole -m gpu suite, smoke(), the default C2 bench (run via gpurun)
set -o pipefail
O=gpurun_out/r3final2
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?
tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
grep -o '"value": [0-9.]*' $O/bench.json | head -1
echo done
