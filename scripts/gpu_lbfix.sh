# LB CT apply fix + IPv6 kernel (lens in LDS, early Bloom words) check, C3
# A/B against libcfc_a.so (round-3 v6 kernel), C5 apply kernel trace (gpurun)
set -o pipefail
O=gpurun_out/lbfix
mkdir -p $O
export TMPDIR=/tmp
T="python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $T tests/test_gpu_lb.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "lb or ct or c5 or c3 or v6 or golden" > $O/t.log 2>&1
rc=$?
tail -15 $O/t.log
[ $rc -le 1 ] || exit 1
for r in 1 2; do
  for lib in libcfc_a.so libcfc.so; do
    CFC_LIB=$lib timeout -k 10 200 python -u bench.py --workload c3 --no-cpu > $O/c3_$lib.$r.json 2> $O/c3_$lib.$r.err || exit 1
    grep -o '"kernels": \[[^]]*\]' $O/c3_$lib.$r.json | grep -o '"kernel": "[a-z_0-9]*", "headers": [0-9]*, "ms_per_launch": [0-9.]*' | sed "s/^/$lib r$r /"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py --workload c5 --ct-apply --steps 5 --warmup 2 --no-cpu > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
echo done
