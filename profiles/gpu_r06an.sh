# Round 6, call AN (repeated as AO): four processes in a row, each timing its step on two side-by-side workspaces
# alternately (placement_probe2.py): is the slow-process state tied to the process or to its memory?
set -e
set -o pipefail
mkdir -p gpurun_out
cd profiles
for i in 1 2 3 4; do
  timeout -k 10 300 python -u placement_probe2.py 5 6 | tail -1 >> ../gpurun_out/r06ao_placement.jsonl 2>> ../gpurun_out/r06ao_placement.err
done
