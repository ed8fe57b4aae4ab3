set -e
O=gpurun_out/bench_final; mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
QSMD_BENCH_DIST=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --steps 30 --warmup 3 --no-cpu-baseline > $O/bench_dist.json 2> $O/bench_dist.err
cat $O/bench.json; tail -1 $O/bench_dist.json | cut -c1-300
