set -o pipefail
D=gpurun_out/s2d
mkdir -p $D
timeout -k 10 300 python bench.py > $D/bench_c2.json 2> $D/bench_c2.err && echo c2 done &&
timeout -k 10 400 python bench.py --workload c5 --ct-apply > $D/bench_c5ct.json 2> $D/bench_c5ct.err && echo c5ct done &&
timeout -k 10 400 python bench.py --workload c5 --ct-apply --stream seq --steps 10 --warmup 2 > $D/bench_c5seq.json 2> $D/bench_c5seq.err && echo c5seq done &&
timeout -k 10 400 python bench.py --workload c5 --family 6 --ct-apply --steps 8 --warmup 2 > $D/bench_c5v6ct.json 2> $D/bench_c5v6ct.err && echo c5v6 done &&
timeout -k 10 300 python bench.py --workload c3 > $D/bench_c3.json 2> $D/bench_c3.err && echo c3 done &&
timeout -k 10 300 python bench.py --workload c5 > $D/bench_c5look.json 2> $D/bench_c5look.err && echo c5look done &&
bash scripts/profile_r06b.sh $D c5look
