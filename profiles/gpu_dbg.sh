set -e
mkdir -p gpurun_out
timeout -k 10 300 python profiles/dbg_persist.py > gpurun_out/dbg_persist.log 2>&1
