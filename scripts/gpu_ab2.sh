# A/B of libcfc builds (CFC_LIB) on the C2 bench, alternating, 2 rounds (run via gpurun)
# usage: bash scripts/gpu_ab2.sh libA.so libB.so ...
set -o pipefail
mkdir -p gpurun_out/ab
for r in 1 2; do
  for lib in "$@"; do
    CFC_LIB=$lib timeout -k 10 240 python -u bench.py --cpu-sample 200000 > gpurun_out/ab/$lib.$r.json 2> gpurun_out/ab/$lib.$r.err || exit 1
    grep -o '"kernel_ms_per_launch": [0-9.]*' gpurun_out/ab/$lib.$r.json | sed "s/^/$lib r$r /"
  done
done
