# A/B of classify kernel builds (CFC_LIB) on the C2 bench (run via gpurun)
set -o pipefail
mkdir -p gpurun_out/ab
for lib in libcfc.so libcfc_u2w1.so libcfc_u3w1.so libcfc_u2w2.so; do
  CFC_LIB=$lib timeout -k 10 240 python -u bench.py --cpu-sample 500000 > gpurun_out/ab/$lib.json 2> gpurun_out/ab/$lib.err || exit 1
done
