"""CPU oracle for the Deblur e-NeRF render + event-measurement hot path.

TEST INFRASTRUCTURE ONLY.  This package is a plain PyTorch-CPU restatement of
the reference algorithm (wengflow/deblur-e-nerf @ 2024-10-22), written from the
reference's semantics and pinned against golden vectors produced by running the
reference's own modules (``tests/golden/make_golden.py``).  Only ``tests/``,
``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py`` may
import it -- and only as the checker / the timed CPU baseline.  The product
package (``deblur-e-nerf_amd/deblur_e_nerf``) never imports it and has no CPU
fallback: its ops raise if the HIP library is missing.

Pinning status ("Oracle"):
* radiance field (encoding, MLP, activations)     -- pinned: mlp_rd{1,3}.npz
* FOH discretisation / pixel-bandwidth model       -- pinned: foh.npz, pixbw_*.npz
* event-model contrast thresholds / loss           -- pinned: ct.npz, loss.npz
* event preparation (contrast threshold, refractory
  delay, diff/subdiff timestamps) and pixel rays   -- pinned: events.npz, rays.npz
* nerfacc 0.3.1 compositing + fixed-count sampler  -- PARITY UNPINNED (nerfacc is a
  third-party CUDA package absent from /root/reference); restated from its
  documented semantics and cross-checked against a float64 brute-force loop.
"""
