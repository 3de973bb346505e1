# round 6: the sparse-with-deletes test, a 20-step dependency-stream line
# (growth, step spread) and the C5 lookup line on its round-6 PMC record
set -o pipefail
D=gpurun_out/s2e
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_ctorder.py -k sparse -q -m gpu --timeout 180 --timeout-method thread > $D/t.log 2>&1 && echo tests done &&
timeout -k 10 400 python bench.py --workload c5 --ct-apply --stream seq --steps 20 --warmup 3 > $D/bench_c5seq20.json 2> $D/bench_c5seq20.err && echo seq20 done &&
timeout -k 10 300 python bench.py --workload c5 > $D/bench_c5look.json 2> $D/bench_c5look.err && echo c5look done
