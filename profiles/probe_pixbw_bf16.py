"""r05: the pixel-bandwidth step's BF16 gradient against the f64 oracle, for the layer-major (bwd_path 0)
and sample-major (bwd_path 1) backward and the F32 mode -- is a BF16 gradient error a kernel bug (the
paths disagree) or the conditioning of the event loss (they agree)?"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "deblur-e-nerf_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import torch  # noqa: E402
from _util import norm_rel, unflat  # noqa: E402
from oracle import pixbw as opb  # noqa: E402
from oracle.train import pixbw_flat_grad  # noqa: E402
from deblur_e_nerf.train import PixbwTrainStep, synthetic_pixbw_events  # noqa: E402
from oracle import nerf as onerf  # noqa: E402


def run(mode, bwd_path, speed, rd=1):
    N, S, n_s = 4, 16, 128
    ts = PixbwTrainStep(N, it_sample_size=S, n_samples=n_s, radiance_dim=rd, mode=mode, device="cuda", seed=9)
    ts.cfg["bwd_path"] = bwd_path
    raw = synthetic_pixbw_events(N, it_sample_size=S, seed=13, speed=speed)
    if rd == 3:
        raw["channel"] = torch.randint(0, 3, (N,), generator=torch.Generator().manual_seed(13))
    ts.load_events(**raw)
    prm32 = {"tau_in_it_eff_prod": float(ts.pb.tau_in_it_eff_prod)}
    for pn in opb.PARAM_NAMES:
        prm32[pn] = float(getattr(ts.pb, pn).detach())
    min_ts = float(ts.pb.min_ts)
    p32 = unflat(ts.flat.detach().cpu(), rd)
    bk = ts.bkgd_orig.detach().cpu()
    raw64 = {k: (v.double() if v.is_floating_point() and v.dtype == torch.float32 else v) for k, v in raw.items()}
    g64, l64 = pixbw_flat_grad({k: v.double() for k, v in p32.items()}, bk.double(), raw64, S, n_s, rd, prm32,
                               min_ts, dt_dtype=None)
    ts.forward()
    ts.backward()
    torch.cuda.synchronize()
    g = ts.gbuf.detach().cpu().double()
    per = []
    off = 0
    for n, shp in [(n, tuple(v.shape)) for n, v in p32.items()]:
        k = int(torch.tensor(shp).prod())
        per.append((n, norm_rel(g[off:off + k], g64[off:off + k])))
        off += k
    worst = sorted(per, key=lambda t: -t[1])[:4]
    print(f"{mode} rd={rd} bwd_path={bwd_path} speed={speed}: loss {ts.loss.cpu().tolist()} vs f64 {l64}; "
          f"grad rel {norm_rel(g, g64):.3e}; worst {[(n, round(e, 4)) for n, e in worst]}", flush=True)


if __name__ == "__main__":
    speeds = [float(v) for v in sys.argv[1].split(",")] if len(sys.argv) > 1 else [5.0, 1.0]
    paths = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0, 1]
    for speed in speeds:
        for rd in (1, 3):
            run("f32", 0, speed, rd)
            for bp in paths:
                run("bf16", bp, speed, rd)
