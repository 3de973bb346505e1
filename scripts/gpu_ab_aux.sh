# A/B of the table probes' cache policy (plain / sc1 / nt: L1 bypass) on the
# default C2 bench, alternating, 2 rounds (run via gpurun)
set -o pipefail
O=gpurun_out/ab_aux
mkdir -p $O
for r in 1 2; do
  for lib in libcfc.so libcfc_x16.so libcfc_x2.so; do
    CFC_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu > $O/$lib.$r.json 2> $O/$lib.$r.err || { tail -5 $O/$lib.$r.err; exit 1; }
    grep -o '"kernel_ms_per_launch": [0-9.]*' $O/$lib.$r.json | sed "s/^/$lib r$r /"
  done
done
for lib in libcfc.so libcfc_x16.so; do
  CFC_LIB=$lib timeout -k 10 300 python -u bench.py --workload c3 --no-cpu > $O/c3_$lib.json 2> $O/c3_$lib.err || { tail -5 $O/c3_$lib.err; exit 1; }
  grep -o '"kernel_ms_per_launch": [0-9.]*' $O/c3_$lib.json | sed "s/^/c3 $lib /"
done
echo done
