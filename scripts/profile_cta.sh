#!/bin/bash
# rocprofv3 PMC passes over the C5 bench with device CT apply (run via gpurun)
set -e
OUT=${1:-gpurun_out/prof_cta}
ARGS="--workload c5 --ct-apply --steps 2 --warmup 1 --no-cpu"
export TMPDIR=/tmp
mkdir -p "$OUT"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_REQ_sum" \
    "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"; do
    i=$((i+1))
    timeout -s KILL 400 rocprofv3 --pmc $grp -d "$OUT/pmc$i" -o run \
        --output-format csv -- python3 bench.py $ARGS > "$OUT/pmc$i.log" 2>&1
done
echo "cta profile passes done"
