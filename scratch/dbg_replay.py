"""Debug: our ngp step vs the reference's marched samples (kept_*), then with them replayed."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "deblur-e-nerf_amd")]
import numpy as np, torch
import test_deblur_gpu as T
from test_nerfacc_gpu import _Draws
from deblur_e_nerf.external import marching, utils as eutils

for fx in sys.argv[1:]:
    z = np.load(os.path.join(ROOT, "tests/golden", fx + ".npz"))
    kept = [(z[f"kept_ri_{i}"], z[f"kept_t0_{i}"], z[f"kept_t1_{i}"]) for i in range(64) if f"kept_ri_{i}" in z.files]
    for replay in (False, True):
        m = T.build_model(z); m.train()
        jit = [z[f"jitter_{i}"] for i in range(4)]
        marching._uniform = _Draws([z["occ_u"]] + (jit if bool(z["pixbw"]) else [np.concatenate(jit)]))
        real = eutils.ray_marching
        ours = []
        calls = iter(kept)
        N = int(z["N"])

        def rm(rays_o, *a, **k):
            if replay:
                # the reference renders the 4 groups in 4 calls of N rays; we render them as one 4N-ray call
                nr = rays_o.shape[0]
                ris, t0s, t1s = [], [], []
                base = 0
                while base < nr:
                    ri, t0, t1 = next(calls)
                    ris.append(torch.from_numpy(ri).long() + base); t0s.append(torch.from_numpy(t0)); t1s.append(torch.from_numpy(t1))
                    base += N
                dev = rays_o.device
                return (torch.cat(ris).to(dev).int(), torch.cat(t0s).to(dev).reshape(-1, 1).float(),
                        torch.cat(t1s).to(dev).reshape(-1, 1).float())
            r = real(rays_o, *a, **k)
            ours.append(tuple(t.detach().cpu() for t in r))
            return r
        eutils.ray_marching = rm
        loss = m.training_step(T._batch(z), 0)
        loss.backward(); torch.cuda.synchronize()
        eutils.ray_marching = real
        if not replay:
            ri = torch.cat([o[0].long() for o in ours]); n_ours = ri.numel()
            n_ref = sum(len(k[0]) for k in kept)
            print(f"== {fx}: our samples {n_ours} (in {len(ours)} calls), reference {n_ref} (in {len(kept)} calls)")
            if len(ours) == 1 and len(kept) == 4:
                # compare per group
                o_ri, o_t0 = ours[0][0].long(), ours[0][1].reshape(-1)
                for g in range(4):
                    sel = (o_ri >= g * N) & (o_ri < (g + 1) * N)
                    r_ri, r_t0 = torch.from_numpy(kept[g][0]).long(), torch.from_numpy(kept[g][1]).reshape(-1)
                    same = sel.sum().item() == r_ri.numel() and torch.equal(o_ri[sel] - g * N, r_ri) and torch.equal(o_t0[sel], r_t0)
                    print(f"   group {g}: ours {int(sel.sum())} ref {r_ri.numel()} identical {same}")
        rf = m.nerf.radiance_field
        for k in ("mlp_base.1.output_layer.bias", "mlp_base.1.hidden_layers.0.bias"):
            g = rf.get_parameter(k).grad.detach().cpu().double().reshape(-1)
            f64 = torch.from_numpy(z[f"grad:{k}_f64"]).double().reshape(-1)
            print(f"   replay={replay} {k}: err vs f64 {float((g - f64).norm() / f64.norm()):.3e}")
