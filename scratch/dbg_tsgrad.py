"""Debug: where does the render-timestamp gradient of the assembled training_step go wrong."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "deblur-e-nerf_amd")]
import numpy as np, torch
import test_deblur_gpu as T
from test_nerfacc_gpu import _Draws
from deblur_e_nerf.external import marching
from oracle import trajectory as otr, events as oev

def cos(a, b):
    a = a.double().reshape(-1).cpu(); b = torch.as_tensor(b).double().reshape(-1)
    return float(a @ b / (a.norm() * b.norm() + 1e-300)), float(a.norm() / (b.norm() + 1e-300))

for fx in sys.argv[1:] or ["step_nopixbw_rd1"]:
    z = np.load(os.path.join(ROOT, "tests/golden", fx + ".npz"))
    m = T.build_model(z); m.train()
    hook = T._TsHook(m)
    cap = {}
    orig_tr = m.trajectory.forward
    def tr(ts):
        p, r = orig_tr(ts)
        cap.setdefault("ts", []).append(ts.detach().clone())
        i = len(cap["ts"]) - 1
        if p.requires_grad:
            p.register_hook(lambda g, i=i: cap.setdefault(("gp", i), g.detach().clone()))
            r.register_hook(lambda g, i=i: cap.setdefault(("gr", i), g.detach().clone()))
        return p, r
    m.trajectory.forward = tr
    orig_pr = m.nerf.pixel_params_to_ray
    def pr(kinv, pix, P, R):
        o, d = orig_pr(kinv, pix, P, R)
        i = len(cap.get("rays", []))
        cap.setdefault("rays", []).append((kinv.detach(), pix.detach(), P.detach(), R.detach()))
        if o.requires_grad:
            o.register_hook(lambda g, i=i: cap.setdefault(("go", i), g.detach().clone()))
            d.register_hook(lambda g, i=i: cap.setdefault(("gd", i), g.detach().clone()))
        return o, d
    m.nerf.pixel_params_to_ray = pr
    jit = [z[f"jitter_{i}"] for i in range(4)]
    draws = [z["occ_u"]] + (jit if bool(z["pixbw"]) else [np.concatenate(jit)])
    marching._uniform = _Draws(draws)
    loss = m.training_step(T._batch(z), 0)
    loss.backward(); torch.cuda.synchronize()
    print(f"== {fx}: loss {float(loss):.7g} ref {float(z['loss']):.7g}; calls {len(cap['ts'])}")
    groups = hook.per_group()
    for i, g in enumerate(groups):
        c, r = cos(g, z[f"dts_g{i}_f64"])
        print(f"  group {i}: cos {c:.4f} norm ratio {r:.4f}")
    # CPU f64 chain from the captured ray gradients
    tw = m.trajectory
    Tts, P, Q = tw.T_wc_timestamp.cpu(), tw.T_wc_position.cpu().double(), tw.T_wc_orientation_quat.cpu().double()
    for i, ts in enumerate(cap["ts"]):
        if ("go", i) not in cap:
            print("  call", i, "no ray grad captured"); continue
        q = ts.cpu().clone().requires_grad_(True)
        p_r, r_r = otr.linear_trajectory(Tts, P, Q, q)
        kinv, pix, _, _ = cap["rays"][i]
        o_r, d_r = oev.pixel_params_to_ray(kinv.cpu().double(), pix.cpu().double(), p_r, r_r)
        go, gd = cap[("go", i)].cpu().double(), cap[("gd", i)].cpu().double()
        ((o_r * go.reshape(o_r.shape)).sum() + (d_r * gd.reshape(d_r.shape)).sum()).backward()
        # our trajectory-level grads vs oracle pixel-ray backward
        p2 = p_r.detach().requires_grad_(True); r2 = r_r.detach().requires_grad_(True)
        o2, d2 = oev.pixel_params_to_ray(kinv.cpu().double(), pix.cpu().double(), p2, r2)
        ((o2 * go.reshape(o2.shape)).sum() + (d2 * gd.reshape(d2.shape)).sum()).backward()
        print(f"  call {i}: |go| {float(go.norm()):.3e} |gd| {float(gd.norm()):.3e}; "
              f"gp cos/ratio {cos(cap[('gp', i)], p2.grad)}; gr cos/ratio {cos(cap[('gr', i)], r2.grad)}")
        ours = torch.cat([g.reshape(-1) for g in groups]) if len(cap['ts']) == 1 else groups[i]
        print(f"     ts grad: ours vs CPU-chain-from-our-ray-grads cos/ratio {cos(ours, q.grad)}")
        ref = np.concatenate([z[f'dts_g{k}_f64'] for k in range(4)]) if len(cap['ts']) == 1 else z[f'dts_g{i}_f64']
        print(f"     CPU-chain vs reference f64 cos/ratio {cos(q.grad, ref)}")
