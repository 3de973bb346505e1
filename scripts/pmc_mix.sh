#!/bin/bash
# Instruction-mix / issue counters of the engine kernels over a short bench
# run (one rocprofv3 PMC pass per group, each under its own time limit).
#   scripts/pmc_mix.sh OUTDIR [bench args...]
set -e
OUT=${1:-gpurun_out/mix}
shift || true
ARGS=${@:---steps 3 --warmup 1 --no-cpu}
export TMPDIR=/tmp
mkdir -p "$OUT"
i=0
for grp in \
    "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
    "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES" ; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $grp -d "$OUT/mix$i" -o run \
        --output-format csv -- python3 bench.py $ARGS > "$OUT/mix$i.log" 2>&1
done
echo "mix passes done"
