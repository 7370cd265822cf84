# Same-box A/B(/C..) of libden builds on the default configs[1] step: ROUNDS rounds, each running every
# build once in the given order (short bench.py runs), one JSON line per run (lib, ms per step,
# per-kernel averages, losses) into gpurun_out/<tag>_ab.jsonl.
# usage: bash profiles/ab.sh TAG ROUNDS LIB_A LIB_B [LIB_C ...]
set -e
set -o pipefail
TAG=$1; ROUNDS=$2; shift 2
mkdir -p gpurun_out
for i in $(seq 1 $ROUNDS); do
  for L in "$@"; do
    DEN_LIB=$L timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-gemm-peak \
      --no-extra-legs --psnr-steps 0 > gpurun_out/${TAG}_run.json 2>> gpurun_out/${TAG}_ab.err
    python - "$L" gpurun_out/${TAG}_run.json >> gpurun_out/${TAG}_ab.jsonl <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
k = {n: v["avg_ms"] for n, v in d["roofline"]["kernels"].items()}
print(json.dumps({"lib": sys.argv[1], "ms_per_step": d["ms_per_step"], "value": d["value"], "kernels_avg_ms": k,
                  "loss": d["loss"]}))
PY
  done
done
