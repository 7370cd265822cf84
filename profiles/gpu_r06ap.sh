# Round 6, call AP: does a second workspace-sized allocation remove the slow-process state?  Each
# policy in both process parities: none none second second none none second second
set -e
set -o pipefail
mkdir -p gpurun_out
for p in none none second second none none second second; do
  timeout -k 10 200 python -u profiles/settle_probe.py $p 6 5 >> gpurun_out/r06ap_settle.jsonl 2>> gpurun_out/r06ap_settle.err
done
