# A/B/A timing of experiment builds of libden (DEN_LIB=...), bench.py configs[1], no CPU leg.
# usage: bash profiles/exp_variants.sh <tag> <variant> [<variant> ...]   (variant "base" = libden.so)
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1; shift
for v in "$@"; do
  if [ "$v" = base ]; then lib=deblur-e-nerf_amd/libden.so; else lib=deblur-e-nerf_amd/libden_$v.so; fi
  DEN_LIB=$lib timeout -k 10 240 python bench.py --steps 12 --warmup 3 --no-cpu-baseline --no-gemm-peak --no-extra-legs > gpurun_out/exp_${tag}_$v.log 2>&1 || exit $?
  python - "$v" gpurun_out/exp_${tag}_$v.log >> gpurun_out/exp_${tag}.txt <<'PY'
import json, sys
for line in open(sys.argv[2]):
    if line.startswith("{"):
        d = json.loads(line); k = d["roofline"]["kernels"]
        print(sys.argv[1], d["ms_per_step"], {n: v["step_ms"] for n, v in k.items()}, d["loss"])
PY
done
