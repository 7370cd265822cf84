"""Debug: per-step loss trajectory of bench.py's configs[1] training from one init, hidden backward
path of the loaded libden vs the sample-major path (bwd_path=1): Adam from a random init is chaotic
in its small terms, so the two trajectories bound how far a backward variant may move the losses."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deblur-e-nerf_amd")]
sys.argv = sys.argv[:1]
import torch
import bench
from deblur_e_nerf import _native as nat

a = bench.parse()
for path in (0, 1):
    torch.manual_seed(0)
    ts, _ = bench.build_step(a, "cuda:0")
    if path:
        ts.desc.bwd_path = 1
        ts.ws = torch.empty(nat.render_workspace_bytes(ts.desc), dtype=torch.uint8, device="cuda:0")
    out = []
    for i in range(15):
        out.append([round(x, 6) for x in ts.step()[:3].tolist()])
    print(f"bwd_path={path}", out[0], out[1], out[4], out[14], flush=True)
    del ts
    torch.cuda.empty_cache()
