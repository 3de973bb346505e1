# round 6: the dependency stream over 20 steps (step spread), and with the
# GC held off so the CT table must grow on the device inside the run
set -o pipefail
D=gpurun_out/s2f
mkdir -p $D
timeout -k 10 300 python bench.py --workload c5 --ct-apply --stream seq --steps 20 --warmup 3 --no-cpu > $D/bench_c5seq20.json 2> $D/bench_c5seq20.err && echo seq20 done &&
timeout -k 10 300 python bench.py --workload c5 --ct-apply --stream seq --steps 8 --warmup 1 --gc-interval 1000000 --no-cpu > $D/bench_c5seq_grow.json 2> $D/bench_c5seq_grow.err && echo grow done
