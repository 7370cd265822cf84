# Round 6, call BI: strong-scaling emulation on one GPU on the final tree (pe fold): the per-rank
# workload of N = 1, 2, 4, 8 ranks (2^17 / N rays), bench.py's configs[1] otherwise (no all-reduce)
set -e
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/r06bi_strong_emulation.jsonl
for r in 131072 65536 32768 16384; do
  timeout -k 10 240 python bench.py --rays $r --no-cpu-baseline --no-gemm-peak --no-extra-legs --psnr-steps 0 > gpurun_out/r06bi_strong_$r.log 2>&1
  tail -1 gpurun_out/r06bi_strong_$r.log >> gpurun_out/r06bi_strong_emulation.jsonl
done
python - <<'PY'
import json
for l in open("gpurun_out/r06bi_strong_emulation.jsonl"):
    d = json.loads(l)
    print(d["config"]["rays_per_step"], d["ms_per_step"], d["value"])
PY
