# LB CT apply fix check + C5 apply kernel trace (run via gpurun)
set -o pipefail
O=gpurun_out/lbfix
mkdir -p $O
export TMPDIR=/tmp
T="python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $T tests/test_gpu_lb.py tests/test_gpu_parity.py -k "lb or ct or c5" > $O/t.log 2>&1
rc=$?
tail -15 $O/t.log
[ $rc -le 1 ] || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py --workload c5 --ct-apply --steps 5 --warmup 2 --no-cpu > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
python3 scripts/pmc_summary.py $O 2>/dev/null | head -60 || true
echo done
