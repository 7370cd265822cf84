"""Split of the ngp field forward: the grid encoding alone (den_hashgrid_fwd) vs the fused field
(den_ngp_fwd, inference) at the synthetic.yaml config, 2^19 samples (HIP events)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deblur-e-nerf_amd"))
import torch  # noqa: E402

from deblur_e_nerf import _native  # noqa: E402

POS = dict(otype="HashGrid", n_levels=16, n_features_per_level=2, log2_hashmap_size=19, base_resolution=16,
           per_level_scale=1.4472692012786865, interpolation="Linear")


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


n = 1 << 19
desc = _native.ngp_desc(1, POS, "softplus", "softplus", 0, [-1.5] * 3 + [1.5] * 3)
P = _native.ngp_param_count(desc)
flat = (torch.rand(P, device="cuda") - 0.5) * 0.2
x01 = torch.rand(n, 3, device="cuda")
x = x01 * 3 - 1.5
d = torch.nn.functional.normalize(torch.randn(n, 3, device="cuda"), dim=-1)
with torch.no_grad():
    t_enc = timed(lambda: _native.hashgrid(flat[:_native.ngp_table_params(desc)], desc, x01))
    t_fwd = timed(lambda: _native.ngp_field(flat, desc, x, d))
    t_den = timed(lambda: _native.ngp_field(flat, desc, x, d, density_only=True))
print(f"encoding {t_enc:.3f} ms, field fwd {t_fwd:.3f} ms, density-only {t_den:.3f} ms (2^19 samples)")
