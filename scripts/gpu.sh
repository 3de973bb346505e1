#!/bin/bash
# The one GPU-box runner (run via gpurun).  Steps run in order, each under
# its own time limit; the first failure ends the script (no GPU step after a
# fault, abort or time limit).
#
#   scripts/gpu.sh OUTDIR STEP [STEP ...]
#
# STEP is one of
#   tests                     the whole -m gpu suite
#   tests:ARGS                pytest -m gpu with ARGS (e.g. "tests:tests/test_gpu_lb.py -k v6")
#   smoke                     __graft_entry__.smoke()
#   bench:NAME:ARGS           python bench.py ARGS > OUTDIR/NAME.json
#   kt:NAME:ARGS              rocprofv3 --kernel-trace --stats of bench.py ARGS -> OUTDIR/NAME/kt
#   pmc:NAME:ARGS             the PMC passes (scripts/pmc_groups) of bench.py ARGS -> OUTDIR/NAME/pmcN
#   py:NAME:SCRIPT ARGS       python -u SCRIPT ARGS > OUTDIR/NAME.log (ubench drivers, debug scripts)
#   ab:LIBS:ARGS              A/B of in-tree libcfc builds (comma-separated CFC_LIB names),
#                             alternating, two rounds of bench.py ARGS -> OUTDIR/ab/LIB.R.json
set -o pipefail
OUT=${1:?usage: gpu.sh OUTDIR STEP...}
shift
export TMPDIR=/tmp
mkdir -p "$OUT"
# counter groups, one rocprofv3 pass each (gfx950 per-block slot limits)
PMC_GROUPS=(
    "FETCH_SIZE"
    "WRITE_SIZE"
    "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_REQ_sum"
    "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
)
for step in "$@"; do
    kind=${step%%:*}
    rest=${step#*:}
    [ "$rest" = "$step" ] && rest=""
    name=${rest%%:*}
    args=${rest#*:}
    [ "$args" = "$rest" ] && args=""
    echo "== $step"
    case $kind in
    tests)
        timeout -k 10 900 python -u -m pytest ${rest:-tests} -m gpu -x -v --timeout 300 \
            --timeout-method thread -p no:cacheprovider > "$OUT/tests.log" 2>&1
        rc=$?; tail -3 "$OUT/tests.log" ;;
    smoke)
        timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" \
            > "$OUT/smoke.log" 2>&1
        rc=$?; tail -3 "$OUT/smoke.log" ;;
    bench)
        timeout -k 10 600 python -u bench.py $args > "$OUT/$name.json" 2> "$OUT/$name.err"
        rc=$?; cat "$OUT/$name.json"; [ $rc -eq 0 ] || tail -20 "$OUT/$name.err" ;;
    kt)
        mkdir -p "$OUT/$name"
        timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/$name/kt" -o run \
            --output-format csv -- python3 bench.py $args > "$OUT/$name/kt.log" 2>&1
        rc=$? ;;
    pmc)
        i=0; rc=0
        for grp in "${PMC_GROUPS[@]}"; do
            i=$((i+1))
            mkdir -p "$OUT/$name"
            timeout -s KILL 400 rocprofv3 --pmc $grp -d "$OUT/$name/pmc$i" -o run \
                --output-format csv -- python3 bench.py $args > "$OUT/$name/pmc$i.log" 2>&1
            rc=$?; [ $rc -eq 0 ] || break
        done ;;
    py)
        timeout -k 10 600 python -u $args > "$OUT/$name.log" 2>&1
        rc=$?; tail -5 "$OUT/$name.log" ;;
    ab)
        mkdir -p "$OUT/ab"; rc=0
        for r in 1 2; do
            for lib in ${name//,/ }; do
                CFC_LIB=$lib timeout -k 10 300 python -u bench.py $args \
                    > "$OUT/ab/$lib.$r.json" 2> "$OUT/ab/$lib.$r.err"
                rc=$?; [ $rc -eq 0 ] || break 2
                grep -o '"kernel_ms_per_launch": [0-9.]*' "$OUT/ab/$lib.$r.json" | sed "s/^/$lib r$r /"
            done
        done ;;
    *)
        echo "unknown step $step"; exit 2 ;;
    esac
    if [ $rc -ne 0 ]; then
        echo "step failed ($rc): $step"
        exit 1
    fi
done
echo "all steps done"
