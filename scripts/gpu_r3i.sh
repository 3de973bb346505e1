# round 3: LB CT apply re-check, then the PMC passes for the roofline (C2
# default bench, C3) and the C5 apply kernels (run via gpurun)
set -o pipefail
O=gpurun_out/r3i
mkdir -p $O
export TMPDIR=/tmp
T="python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $T tests/test_gpu_lb.py tests/test_gpu_ctgc.py tests/test_gpu_parity.py -k "lb or gc" > $O/lb.log 2>&1
rc=$?
tail -8 $O/lb.log
[ $rc -le 1 ] || exit 1
bash scripts/profile.sh $O/c2 --steps 3 --warmup 1 --no-cpu || exit 1
bash scripts/profile.sh $O/c3 --workload c3 --steps 3 --warmup 1 --no-cpu || exit 1
bash scripts/profile_cta.sh $O/cta || exit 1
echo done
