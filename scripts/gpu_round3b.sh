set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu_ab3.sh libcfc_p0.so libcfc.so libcfc_p2.so libcfc_e8.so > gpurun_out/ab.txt 2>&1 &&
bash scripts/gpu_round3.sh
