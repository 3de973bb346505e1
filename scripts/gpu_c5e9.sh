# C5 lookup-only bench line; C5 --ct-apply with the shipped library and with
# a timing-only build whose scan writes no plain-hit summaries (CFC_EXP=9:
# the floor of a sort-based summary), plus a C5 kernel trace (run via gpurun)
set -o pipefail
O=gpurun_out/c5e9
mkdir -p $O
timeout -k 10 400 python -u bench.py --workload c5 --no-cpu > $O/bench_c5.json 2> $O/bench_c5.err || { tail -5 $O/bench_c5.err; exit 1; }
grep -o '"value": [0-9.]*' $O/bench_c5.json | head -1
for lib in libcfc.so libcfc_e9.so; do
  CFC_LIB=$lib timeout -k 10 300 python -u bench.py --workload c5 --ct-apply --no-cpu --steps 8 --warmup 2 > $O/$lib.json 2> $O/$lib.err || { tail -5 $O/$lib.err; exit 1; }
  grep -o '"apply_ms_per_step": [0-9.]*' $O/$lib.json | sed "s/^/$lib /"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py --workload c5 --steps 5 --warmup 2 --no-cpu > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
echo done
