#!/bin/bash
# Round-6 profile passes, counters packed into two runs per configuration
# (gfx950 block limits: 4 TCC counters a run — FETCH_SIZE takes 3, WRITE_SIZE
# 2 — and 8 SQ):
#   scripts/profile_r06b.sh OUT c2|c3|c5ct|c5look|c5seq|c5v6 ...
# per group: kernel trace + stats, then the two counter passes, each under
# its own time limit; the first failure ends the script.
set -o pipefail
OUT=${1:?usage: profile_r06b.sh OUT GROUP...}
shift
export TMPDIR=/tmp
for G in "$@"; do
case $G in
c2)     ARGS="--steps 3 --warmup 1 --no-cpu" ;;
c3)     ARGS="--workload c3 --steps 3 --warmup 1 --no-cpu" ;;
c5ct)   ARGS="--workload c5 --ct-apply --steps 6 --warmup 2 --no-cpu" ;;
c5look) ARGS="--workload c5 --steps 3 --warmup 1 --no-cpu" ;;
c5seq)  ARGS="--workload c5 --ct-apply --stream seq --steps 6 --warmup 2 --no-cpu" ;;
c5v6)   ARGS="--workload c5 --family 6 --ct-apply --steps 6 --warmup 2 --no-cpu" ;;
*) echo "unknown group $G"; exit 2 ;;
esac
D="$OUT/$G"
mkdir -p "$D"
echo "== $G kt"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$D/kt" -o run --output-format csv \
    -- python3 bench.py $ARGS > "$D/kt.log" 2>&1 || { echo "kt failed"; tail -5 "$D/kt.log"; exit 1; }
i=0
for grp in "FETCH_SIZE TCC_REQ_sum SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
    "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    echo "== $G pmc$i"
    timeout -s KILL 400 rocprofv3 --pmc $grp -d "$D/pmc$i" -o run --output-format csv \
        -- python3 bench.py $ARGS > "$D/pmc$i.log" 2>&1 || { echo "pmc$i failed"; tail -5 "$D/pmc$i.log"; exit 1; }
done
echo "profile $G done"
done
