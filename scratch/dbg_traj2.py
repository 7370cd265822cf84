"""Debug: along one training trajectory (hidden backward path of the loaded libden), the gradient of
every state against the sample-major path's (bwd_path=1) gradient of the same state, per layer."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deblur-e-nerf_amd"), os.path.join(ROOT, "tests")]
sys.argv = sys.argv[:1] + ["--rays", "65536"]
import torch
import bench
from deblur_e_nerf import _native as nat
from _util import unflat, norm_rel

a = bench.parse()
torch.manual_seed(0)
ts, _ = bench.build_step(a, "cuda:0")
ws0 = ts.ws
d1 = nat._desc(ts.cfg, ts.R, a.samples, True, ts.has_bkgd)
d1.bwd_path = 1
ws1 = torch.empty(nat.render_workspace_bytes(d1), dtype=torch.uint8, device="cuda:0")
d0 = ts.desc
for i in range(15):
    ts.desc, ts.ws = d1, ws1
    ts.forward(); ts.backward(); torch.cuda.synchronize()
    g1 = ts.grad.detach().clone()
    ts.desc, ts.ws = d0, ws0
    loss = ts.step()[:3].tolist()
    g0 = ts.grad.detach().clone()
    gf0, gf1 = unflat(g0.cpu(), ts.rd), unflat(g1.cpu(), ts.rd)
    errs = {k: norm_rel(gf0[k], gf1[k]) for k in gf1}
    k = max(errs, key=errs.get)
    print(f"step {i}: loss {[round(x, 6) for x in loss]} worst {k} {errs[k]:.2e}  sigma.w {errs['mlp.sigma_layer.output_layer.weight']:.2e}"
          f" sigma.b {errs['mlp.sigma_layer.output_layer.bias']:.2e} bott.w {errs['mlp.bottleneck_layer.output_layer.weight']:.2e}",
          flush=True)
