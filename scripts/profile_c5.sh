#!/bin/bash
# rocprofv3 passes over the C5 (conntrack) bench on the GPU box:
# kernel trace + stats, then one PMC pass per counter group (never combined
# with tracing).  Each pass has its own time limit; stops at the first
# failure.  usage: profile_c5.sh OUTDIR [extra bench args, e.g. --ct-apply]
set -e
OUT=${1:-gpurun_out/prof_c5}
shift || true
ARGS="--workload c5 --steps 3 --warmup 1 --no-cpu $*"
export TMPDIR=/tmp
mkdir -p "$OUT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run \
    --output-format csv -- python3 bench.py $ARGS > "$OUT/kt.log" 2>&1
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_REQ_sum" \
    "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"; do
    i=$((i+1))
    timeout -s KILL 400 rocprofv3 --pmc $grp -d "$OUT/pmc$i" -o run \
        --output-format csv -- python3 bench.py $ARGS > "$OUT/pmc$i.log" 2>&1
done
echo "c5 profile passes done"
