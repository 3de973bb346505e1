#!/bin/bash
# One rocprofv3 PMC pass of instruction-mix counters over a short bench run.
#   scripts/pmc_insts.sh OUTDIR [bench args...]
set -e
OUT=${1:-gpurun_out/insts}
shift || true
ARGS=${@:---steps 3 --warmup 1 --no-cpu}
export TMPDIR=/tmp
mkdir -p "$OUT"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES \
    -d "$OUT/insts" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/insts.log" 2>&1
echo "instruction pass done"
