# Round 4, call S: the N-rank bench path on the one-GPU box -- bench.py --gpus 2 launches two ranks
# (torch.distributed.run child), gloo all-reduces the GPU gradient buffers (RCCL refuses two ranks
# on one device); then the N = 1 line on the same box for comparison
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 2 --no-extra-legs --psnr-steps 0 > gpurun_out/r04s_n2.log 2>&1
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-extra-legs --psnr-steps 0 --no-cpu-baseline > gpurun_out/r04s_n1.log 2>&1
timeout -k 10 500 python -u profiles/psnr_seeds.py --seeds 8 > gpurun_out/r04s_psnr_seeds.log 2>&1
echo done
