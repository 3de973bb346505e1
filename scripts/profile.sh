#!/bin/bash
# rocprofv3 passes over bench.py on the GPU box (run via gpurun).
#   scripts/profile.sh OUTDIR [bench args...]
# One kernel-trace/stats pass, then one PMC pass per counter group (the
# counter groups respect gfx950's per-block slot limits; never combined with
# tracing).  Each pass has its own time limit; the script stops at the first
# failure.
set -e
OUT=${1:-gpurun_out/prof}
shift || true
ARGS=${@:---steps 3 --warmup 1 --no-cpu}
export TMPDIR=/tmp
mkdir -p "$OUT"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run \
    --output-format csv -- python3 bench.py $ARGS > "$OUT/kt.log" 2>&1
i=0
for grp in \
    "FETCH_SIZE" \
    "WRITE_SIZE" \
    "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
    "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE GRBM_COUNT" \
    "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_REQ_sum" ; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $grp -d "$OUT/pmc$i" -o run \
        --output-format csv -- python3 bench.py $ARGS > "$OUT/pmc$i.log" 2>&1
done
echo "profile passes done"
