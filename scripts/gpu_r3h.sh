# round 3: full -m gpu suite after the LB CT-apply fixes and the IPv6 kernel
# change, smoke, default bench (run via gpurun)
set -o pipefail
O=gpurun_out/r3h
mkdir -p $O
export TMPDIR=/tmp
T="python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $T tests/test_gpu_lb.py > $O/lb.log 2>&1
rc=$?
tail -8 $O/lb.log
[ $rc -le 1 ] || exit 1
timeout -k 10 700 $T tests -m gpu --durations=15 > $O/gpu_tests.log 2>&1
rc=$?
tail -25 $O/gpu_tests.log
[ $rc -le 1 ] || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
echo done
