# full GPU suite, then the round's measurement (profiles/gpu_r03f.sh)
bash scratch/gpu_full.sh && grep -q " passed" gpurun_out/full.log && ! grep -q " failed" gpurun_out/full.log && bash profiles/gpu_r03f.sh
