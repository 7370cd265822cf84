"""Oracle: the ``ngp`` radiance field (NGPradianceField) -- CPU PyTorch restatement (test
infrastructure, see __init__).

Reference semantics followed (file:line under /root/reference):
* input contraction AABB / tanh / unisphere + selector   deblur_e_nerf/external/ngp.py:68-106, 230-238
* position encoding tcnn.Encoding (HashGrid)             deblur_e_nerf/external/ngp.py:166-170 -> oracle/tcnn.py
* mlp_base = MLP(32 -> n_neurons x n_hidden -> 1 + geo)  deblur_e_nerf/external/ngp.py:171-187, mlp.py:26-113
* density = shifted_trunc_exp(out[0]) * selector         deblur_e_nerf/external/ngp.py:45-65, 244-250
* SH degree-4 view encoding                              deblur_e_nerf/external/sh_encoder.py:27-80
* mlp_head = MLP(16 + geo -> n_neurons x n_hidden -> rd) deblur_e_nerf/external/ngp.py:188-205, 256-267
* activations (hidden softplus(100) / relu; radiance     deblur_e_nerf/models/nerf.py:17-29, 105-131
  softplus(1) / sigmoid)
Pinned by tests/golden/ngp_*.npz (the reference NGPradianceField run here with oracle/tcnn.py
as tcnn.Encoding); the grid encoding itself is parity unpinned (oracle/tcnn.py).
"""
import torch

from . import tcnn

# configs/train/synthetic.yaml nerf.ngp (also 07_ziggy_and_fuzz_hdr.yaml)
POS_ENCODING = dict(otype="HashGrid", n_levels=16, n_features_per_level=2, log2_hashmap_size=19, base_resolution=16,
                    per_level_scale=1.4472692012786865, interpolation="Linear")
MLP_BASE = dict(hidden_activation="softplus", density_activation="shifted_trunc_exp", n_neurons=64,
                n_hidden_layers=1, geo_feat_dim=15, weight_norm=False)
MLP_HEAD = dict(hidden_activation="softplus", radiance_activation="softplus", n_neurons=64, n_hidden_layers=2,
                weight_norm=False)


def layer_specs(rd, pos=POS_ENCODING, base=MLP_BASE, head=MLP_HEAD, sh_dims=16):
    """(name, in, out) of the MLP layers in the reference's parameter order (after the encoding's
    ``mlp_base.0.params``)."""
    specs, fin = [], pos["n_levels"] * pos["n_features_per_level"]
    for i in range(base["n_hidden_layers"]):
        specs.append((f"mlp_base.1.hidden_layers.{i}", fin, base["n_neurons"]))
        fin = base["n_neurons"]
    specs.append(("mlp_base.1.output_layer", fin, 1 + base["geo_feat_dim"]))
    fin = sh_dims + base["geo_feat_dim"]
    for i in range(head["n_hidden_layers"]):
        specs.append((f"mlp_head.hidden_layers.{i}", fin, head["n_neurons"]))
        fin = head["n_neurons"]
    specs.append(("mlp_head.output_layer", fin, rd))
    return specs


def build_params(rd, seed, pos=POS_ENCODING, table_scale=1e-4):
    """{name: tensor}: the hash table U(-scale, scale) and nn.Linear default-initialised layers
    (the reference passes hidden_init / output_init / bias_init = None: PyTorch's defaults)."""
    g = torch.Generator().manual_seed(seed)
    p = {"mlp_base.0.params": (torch.rand(tcnn.n_params(pos), generator=g) * 2 - 1) * table_scale}
    for name, fin, fout in layer_specs(rd, pos):
        bound = 1.0 / fin ** 0.5
        p[name + ".weight"] = (torch.rand(fout, fin, generator=g) * 2 - 1) * bound
        p[name + ".bias"] = (torch.rand(fout, generator=g) * 2 - 1) * bound
    return p


def contract(x, aabb, ctype=0):
    """-> x in [0,1]^3 (for the interior) and the selector (ngp.py:230-238)."""
    lo, hi = aabb[:3], aabb[3:]
    x = (x - lo) / (hi - lo)
    if ctype == 2:  # UN_BOUNDED_SPHERE
        x = x * 2 - 1
        mag = x.norm(dim=-1, keepdim=True)
        x = torch.where(mag > 1, (2 - 1 / mag) * (x / mag), x)
        x = x / 4 + 0.5
    elif ctype == 1:  # UN_BOUNDED_TANH
        x = (torch.tanh(x - 0.5) + 1) / 2
    sel = ((x > 0.0) & (x < 1.0)).all(dim=-1)
    return x, sel


def _act(name):
    if name == "softplus":
        return lambda t: torch.nn.functional.softplus(t, beta=100)
    return torch.relu


def _trunc_exp(x):
    class F(torch.autograd.Function):
        @staticmethod
        def forward(ctx, v):
            ctx.save_for_backward(v)
            return torch.exp(v)

        @staticmethod
        def backward(ctx, g):
            (v,) = ctx.saved_tensors
            return g * torch.exp(torch.clamp(v, max=15))
    return F.apply(x)


def field(p, x, d, rd, aabb, ctype=0, pos=POS_ENCODING, base=MLP_BASE, head=MLP_HEAD):
    """NGPradianceField.forward(positions, directions) -> (rgb (n, rd), density (n, 1))."""
    xn, sel = contract(x, aabb, ctype)
    h = tcnn.encode(xn.reshape(-1, 3), p["mlp_base.0.params"], pos)
    act = _act(base["hidden_activation"])
    for i in range(base["n_hidden_layers"]):
        h = act(torch.nn.functional.linear(h, p[f"mlp_base.1.hidden_layers.{i}.weight"],
                                           p[f"mlp_base.1.hidden_layers.{i}.bias"]))
    o = torch.nn.functional.linear(h, p["mlp_base.1.output_layer.weight"], p["mlp_base.1.output_layer.bias"])
    kind = base.get("density_activation", "shifted_trunc_exp")
    if kind == "shifted_trunc_exp":
        density = _trunc_exp(o[:, :1] - 1) * sel[:, None]
    else:  # models/nerf.py:20-29: softplus(beta 1), shifted_softplus = softplus(x - 1)
        density = torch.nn.functional.softplus(o[:, :1] - (1 if kind == "shifted_softplus" else 0), beta=1,
                                               threshold=20) * sel[:, None]
    hh = torch.cat([tcnn.sh_encode_deg4(d.reshape(-1, 3)), o[:, 1:]], dim=-1)
    act = _act(head["hidden_activation"])
    for i in range(head["n_hidden_layers"]):
        hh = act(torch.nn.functional.linear(hh, p[f"mlp_head.hidden_layers.{i}.weight"],
                                            p[f"mlp_head.hidden_layers.{i}.bias"]))
    r = torch.nn.functional.linear(hh, p["mlp_head.output_layer.weight"], p["mlp_head.output_layer.bias"])
    rgb = torch.nn.functional.softplus(r) if head["radiance_activation"] == "softplus" else torch.sigmoid(r)
    return rgb, density
