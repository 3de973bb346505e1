# A/B of the CT apply scan's headers per thread (CFC_SCAN_U 2 / 4 / 8) on the
# C5 --ct-apply bench (run via gpurun)
set -o pipefail
O=gpurun_out/ab_scan
mkdir -p $O
for lib in libcfc_u2.so libcfc.so libcfc_u8.so; do
  CFC_LIB=$lib timeout -k 10 300 python -u bench.py --workload c5 --ct-apply --no-cpu --steps 8 --warmup 2 > $O/$lib.json 2> $O/$lib.err || { tail -5 $O/$lib.err; exit 1; }
  grep -o '"apply_ms_per_step": [0-9.]*' $O/$lib.json | sed "s/^/$lib /"
done
echo done
