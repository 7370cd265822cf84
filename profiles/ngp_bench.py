"""Throughput of the `ngp` radiance field (den_ngp_fwd / den_ngp_bwd) at the reference's default
configuration (configs/train/synthetic.yaml nerf.ngp: 16 levels of 2^19 entries, 64-wide MLPs):
one forward + backward over N samples, as a render call of the training step runs it (points
in the chair AABB, unit directions).  Prints one JSON line.

    python profiles/ngp_bench.py [--n 524288] [--iters 20]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deblur-e-nerf_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

# configs/train/synthetic.yaml nerf.ngp
POS = dict(otype="HashGrid", n_levels=16, n_features_per_level=2, log2_hashmap_size=19, base_resolution=16,
           per_level_scale=1.4472692012786865, interpolation="Linear")
BASE = dict(n_neurons=64, n_hidden_layers=1, geo_feat_dim=15, weight_norm=False)
HEAD = dict(n_neurons=64, n_hidden_layers=2, weight_norm=False)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 19)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rd", type=int, default=1)
    a = ap.parse_args()
    from deblur_e_nerf.external import ngp
    dev = "cuda"
    torch.manual_seed(0)
    f = ngp.NGPradianceField(
        aabb=[-1.5, -1.5, -1.5, 1.5, 1.5, 1.5], pos_encoding_config=dict(POS),
        mlp_base_config=dict(BASE, hidden_activation=torch.nn.Softplus(beta=100),
                             density_activation=ngp.shifted_trunc_exp),
        mlp_head_config=dict(HEAD, hidden_activation=torch.nn.Softplus(beta=100),
                             radiance_activation=torch.nn.Softplus(beta=1), output_dim=a.rd)).to(dev)
    x = torch.rand(a.n, 3, device=dev) * 3 - 1.5
    d = torch.nn.functional.normalize(torch.randn(a.n, 3, device=dev), dim=-1)
    g_rgb = torch.randn(a.n, a.rd, device=dev)
    g_sig = torch.randn(a.n, 1, device=dev)

    def step():
        rgb, sig = f(x, d)
        ((rgb * g_rgb).sum() + (sig * g_sig).sum()).backward()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / a.iters * 1e3
    # forward alone
    with torch.no_grad():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            f(x, d)
        torch.cuda.synchronize()
    ms_fwd = (time.perf_counter() - t0) / a.iters * 1e3
    table_mb = f.mlp_base[0].params.numel() * 4 / 1e6
    print(json.dumps({"what": "ngp field fwd+bwd (den_ngp_fwd/bwd + dW), synthetic.yaml nerf.ngp config",
                      "samples": a.n, "ms_fwd_bwd": round(ms, 3), "ms_fwd_inference": round(ms_fwd, 3),
                      "msamples_per_s_train": round(a.n / ms / 1e3, 2), "table_mb": round(table_mb, 1)}), flush=True)


if __name__ == "__main__":
    main()
