# timing-only A/B of CT apply scan variants (run via gpurun)
set -o pipefail
mkdir -p gpurun_out/abct
for lib in libcfc.so libcfc_e11.so libcfc_e12.so; do
  CFC_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/abct/$lib -o run --output-format csv -- python3 bench.py --workload c5 --ct-apply --steps 2 --warmup 1 --no-cpu > gpurun_out/abct/$lib.log 2>&1 || exit 1
done
