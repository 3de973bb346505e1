# A/B on the default C2 bench, alternating, 2 rounds: plain build, table
# probes with sc1 (L1 bypass), the directory probe an iteration ahead
# (CFC_DIR_AHEAD); the latter's IPv4 parity tests first (run via gpurun)
set -o pipefail
O=gpurun_out/ab_aux
mkdir -p $O
CFC_LIB=libcfc_da.so timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py -k "golden or c2 or endpoints or wide or empty or counters" > $O/da_tests.log 2>&1
rc=$?
tail -3 $O/da_tests.log
[ $rc -eq 0 ] || exit 1
for r in 1 2; do
  for lib in libcfc.so libcfc_x16.so libcfc_da.so; do
    CFC_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu > $O/$lib.$r.json 2> $O/$lib.$r.err || { tail -5 $O/$lib.$r.err; exit 1; }
    grep -o '"kernel_ms_per_launch": [0-9.]*' $O/$lib.$r.json | sed "s/^/$lib r$r /"
  done
done
echo done
