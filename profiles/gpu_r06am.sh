# Round 6, call AM: the slow first steps of a bench process -- settle policies (none / zero / sleep),
# each in its own process, twice in alternating order
set -e
set -o pipefail
mkdir -p gpurun_out
for p in none zero sleep sleep zero none; do
  timeout -k 10 200 python -u profiles/settle_probe.py $p 6 5 >> gpurun_out/r06am_settle.jsonl 2>> gpurun_out/r06am_settle.err
done
