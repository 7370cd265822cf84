# Round 6, call BF: the N-rank path rehearsed on the final tree with the pe fold: bench.py --gpus 2
# --dist-backend gloo (a child torch.distributed.run, two ranks sharing the one GPU, gloo all-reduce)
set -e
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 3 > gpurun_out/r06bf_bench_gloo2.json 2> gpurun_out/r06bf_bench_gloo2.err
tail -1 gpurun_out/r06bf_bench_gloo2.json | cut -c1-400
