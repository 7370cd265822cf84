"""Debug: d loss / d mean C of the pixbw step -- our backward vs an f64 recompute on our forward values."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "deblur-e-nerf_amd")]
import numpy as np, torch
import test_deblur_gpu as T
from test_nerfacc_gpu import _Draws
from deblur_e_nerf.external import marching

for fx in sys.argv[1:]:
    z = np.load(os.path.join(ROOT, "tests/golden", fx + ".npz"))
    m = T.build_model(z); m.train()
    cap = {}
    orig = m.loss.compute
    def comp(ev, diff, sub, c):
        cap["ev"] = {k: v.detach().clone() for k, v in ev.items() if torch.is_tensor(v)}
        cap["diff"] = {k: v.detach().clone() for k, v in diff.items() if torch.is_tensor(v)}
        cap["sub"] = {k: v.detach().clone() for k, v in sub.items() if torch.is_tensor(v)}
        cap["c"] = c.detach().clone()
        out = orig(ev, diff, sub, c)
        for k in ("log_intensity_diff",):
            diff[k].register_hook(lambda g: cap.__setitem__("g_diff", g.detach().clone()))
            sub[k].register_hook(lambda g: cap.__setitem__("g_sub", g.detach().clone()))
        c.register_hook(lambda g: cap.__setitem__("g_c", g.detach().clone()))
        return out
    m.loss.compute = comp
    jit = [z[f"jitter_{i}"] for i in range(4)]
    draws = [z["occ_u"]] + (jit if bool(z["pixbw"]) else [np.concatenate(jit)])
    marching._uniform = _Draws(draws)
    loss = m.training_step(T._batch(z), 0)
    loss.backward(); torch.cuda.synchronize()
    ctp = m.contrast_threshold.parametrizations
    dm = float(ctp.mean_contrast_threshold.original.grad)
    print(f"== {fx}: d_mean ours {dm:.9e} ref f32 {float(z['d_mean_ct_orig']):.9e} f64 {float(z['d_mean_ct_orig_f64']):.9e}")
    print("   ev keys", list(cap["ev"]), "diff", list(cap["diff"]), "sub", list(cap["sub"]))
    # f64 recompute of the loss from our forward values: d/dc (normalisation only) and d/d diff-lid
    from oracle.loss import event_loss
    ev, df, sb = cap["ev"], cap["diff"], cap["sub"]
    c64 = cap["c"].double().cpu().reshape(()).requires_grad_(True)
    lid = ev["log_intensity_diff"].double().cpu()
    dl = df["log_intensity_diff"].double().cpu().requires_grad_(True)
    sl = sb["log_intensity_diff"].double().cpu().requires_grad_(True)
    Ld, Lt = event_loss(lid, ev["end_ts"].double().cpu(), ev["start_ts"].double().cpu(), dl,
                        df["ts_diff"].double().cpu(), df["is_valid"].cpu(), sl, sb["is_valid"].cpu(), c64)
    tot = Ld + float(m.hparams.loss.weight.log_intensity_tv) * Lt
    tot.backward()
    print(f"   loss ours {float(loss):.9e} f64-recompute {float(tot):.9e}")
    print(f"   g_c ours {float(cap['g_c'].sum()):.9e} recompute (normalisation + target) {float(c64.grad):.9e}")
    print(f"   g_diff rel {float((cap['g_diff'].double().cpu() - dl.grad).norm() / dl.grad.norm()):.3e}  "
          f"g_sub rel {float((cap['g_sub'].double().cpu() - sl.grad).norm() / sl.grad.norm()):.3e}")
    print(f"   |diff lid| mean {float(dl.abs().mean()):.3e} |sub lid| mean {float(sl.abs().mean()):.3e}")
