"""Train-step throughput of the Deblur e-NeRF render + event-measurement hot path.

Workload (BASELINE.json configs[1]): chair-like synthetic scene, 2^17 rays x 128
samples per step through the 8x256 `mlp` NeRF, pixel-bandwidth model off.  Each
step starts from the raw events (32768: counts, i64 timestamps, normalized
samples, pixels, camera poses at the 4 render timestamps) resident in HBM:
event preparation (contrast threshold, refractory delay, diff/subdiff
timestamps, target) and pixel rays on the device, then 4 render groups (diff
start/end, TV start/end) x 32768 events, Huber diff + 1e-3 L1 TV loss,
backward, all-reduce, Adam.  Strong scaling: the 2^17-ray step
is split over the ranks (reference DDP semantics: per-GPU batch = eff // gpus).

    python bench.py [--gpus N --steps K --warmup W]     (N > 1 via torch.distributed.run)

Prints ONE JSON line (rank 0).  See DESIGN.md "Measurement" for the roofline
accounting.
"""
import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "deblur-e-nerf_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

# algorithmic MACs per sample of the forward MLP: 593,152 (rd=1) / 593,408 (rd=3)
MAC_PER_SAMPLE = {1: 593152, 3: 593408}
PEAK_TFLOPS = {"bf16": 2500.0, "f32": 157.3}  # MI355X dense MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (default: WORLD_SIZE under a torch.distributed launcher, else 1)")
    ap.add_argument("--steps", type=int, default=20)
    # every process's first ~10 steps run slow (76 -> 67 ms under a kernel trace with no idle time
    # between kernels, profiles/r06ax_gaps.jsonl): the default times the steady state
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--rays", type=int, default=131072)
    ap.add_argument("--samples", type=int, default=128)
    ap.add_argument("--rd", type=int, default=1)
    ap.add_argument("--mode", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gemm-peak", action="store_true", help="skip the hipBLASLt reference GEMM (profiling runs)")
    ap.add_argument("--pixbw", action="store_true",
                    help="BASELINE configs[2]: pixel-bandwidth model on (it_sample_size = --it-samples)")
    ap.add_argument("--it-samples", type=int, default=16)
    ap.add_argument("--cpu-rays", type=int, default=2048,
                    help="rays of the bounded pixel-bandwidth-on CPU-baseline sample (--pixbw)")
    ap.add_argument("--psnr-steps", type=int, default=None,
                    help="Adam steps of the converged-PSNR leg (default PSNR_LEG's, which the oracle fixtures "
                         "were trained on; 0: skip)")
    ap.add_argument("--psnr-only", action="store_true", help="run the converged-PSNR leg alone and print it")
    ap.add_argument("--no-extra-legs", action="store_true",
                    help="skip the configs[2] (pixel bandwidth on) and F32-mode legs of the N = 1 line")
    ap.add_argument("--cpu-stub", action="store_true",
                    help="launcher test only: gloo on the CPU, a stub step of the same sharding, no GPU")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="N > 1 collective backend: nccl (= RCCL, one GPU per rank) or gloo (rehearsal of the "
                         "N-rank GPU path with every rank on a shared GPU: rank r on device r mod count)")
    a = ap.parse_args()
    if a.gpus is None:
        a.gpus = int(os.environ.get("WORLD_SIZE", "1"))
    if a.psnr_steps is None:
        a.psnr_steps = PSNR_LEG["steps"]
    return a


def launch_ranks(a):
    """``--gpus N`` (N > 1) started outside a torch.distributed launcher: run N ranks, one process
    per GPU as scripts/run.py:84-100's DDP plugin does, by starting ``torch.distributed.run`` as a
    CHILD process (this process never touches the GPU and is never replaced by another program).
    The ranks inherit stdout, so rank 0's JSON line is this command's output; returns their exit
    code."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    return subprocess.run(cmd, env=env).returncode


class StubStep:
    """``--cpu-stub``: the launcher / sharding / timing contract without a GPU.  Rank r of `world`
    holds R / world rays (as TrainStep does: whole events of 4 rays) and each step does a small
    CPU computation over them plus the step's one gradient all-reduce."""

    def __init__(self, rays, world):
        from deblur_e_nerf.train import allreduce_mean
        self.R = rays // world
        self.S = 1
        self._reduce = allreduce_mean
        self.x = torch.linspace(0, 1, self.R * 4).view(self.R, 4)
        self.gbuf = torch.zeros(1024)
        self.loss = torch.zeros(4)

    def step(self):
        self.gbuf.fill_(float(self.x.sum()) / self.R)
        self._reduce(self.gbuf)
        self.loss[0] = self.gbuf[0]
        return self.loss


BASELINE_METRIC = "train-step rays/sec at 131072 rays \u00d7 128 samples; PSNR vs ref"


def metric_name(a):
    """BASELINE.json's metric string on its own workload, else the workload actually run."""
    if (a.rays, a.samples) == (131072, 128):
        return json.loads(f'"{BASELINE_METRIC}"')
    return f"train-step rays/sec at {a.rays} rays x {a.samples} samples"


def build_step(a, dev, rank=0, world=1, pixbw=None, mode=None):
    from deblur_e_nerf.train import PixbwTrainStep, TrainStep, synthetic_events, synthetic_pixbw_events
    pixbw = a.pixbw if pixbw is None else pixbw
    mode = a.mode if mode is None else mode
    per_event = 4 * a.it_samples if pixbw else 4
    assert a.rays % (per_event * world) == 0
    n_events = a.rays // per_event // world
    if pixbw:
        ts = PixbwTrainStep(n_events, it_sample_size=a.it_samples, n_samples=a.samples, radiance_dim=a.rd,
                            mode=mode, device=dev)
        ts.load_events(**synthetic_pixbw_events(n_events, a.it_samples, rank=rank, world=world))
    else:
        ts = TrainStep(n_events, n_samples=a.samples, radiance_dim=a.rd, mode=mode, device=dev)
        ts.load_events(**synthetic_events(n_events, rank=rank, world=world))
    return ts, per_event


def extra_leg(a, dev, pixbw, mode, steps, warmup=2, rays=None):
    """A second workload in the same run (N = 1): BASELINE configs[2] (pixel bandwidth on,
    it_sample_size 16) or configs[1] in F32 (the reference's arithmetic), timed like the main line.
    ``rays``: a smaller batch where the F32 workspace (~20 KB per sample kept for the backward) would not fit one GPU
    at 2^17 rays x 128 samples (314 GiB): the rate is per ray, the batch only has to fill the chip."""
    if rays is not None:
        a = argparse.Namespace(**dict(vars(a), rays=rays))
    ts, per_event = build_step(a, dev, pixbw=pixbw, mode=mode)
    for _ in range(warmup):
        ts.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        ts.step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    out = {"value": round(a.rays * steps / el, 1), "unit": "rays/s", "ms_per_step": round(el / steps * 1e3, 3),
           "steps": steps, "warmup": warmup, "dtype": mode,
           "workload": f"chair synthetic, pixel-bandwidth {'on (it_sample_size=%d)' % a.it_samples if pixbw else 'off'}, "
                       f"{a.rays} rays x {a.samples} samples, mlp 8x256 rd={a.rd}, "
                       f"{a.rays // per_event} events, event prep+rays+fwd+bwd+Adam",
           "loss": [round(x, 6) for x in ts.loss[:3].tolist()]}
    del ts
    torch.cuda.empty_cache()
    return out


PHASE_REPS = 3
# Algorithmic work of each render-path kernel per sample and STEP; FLOP =
# 2 x MAC, per launch = per step / launches per step.  The forward: 593,152 MAC (rd = 1; rd = 3 adds
# 2 x 128).  BF16 (the layer-major backward):
#   render_head_bwd : compositing adjoint, Lr^T (rd x 128) + the fused Lr weight gradient (rd x 128),
#                     Lg^T (128 x 256, bottleneck part) + the fused Lg weight gradient (128 x 283)
#   hidden_bwd      : 7 launches (L7..L1), each dX (256 x 256) + dW (256 x 256); L5 also the pe columns of
#                     its dW (256 x 63) and L1 dW_0 (256 x 63): the pe fold (den_hidden.hip PEM)
#   hidden_bwd_lb   : 1 launch (Lb), dX (256 x 257) + dW (257 x 256)
#   dwstream        : the weight gradients of L0 (256 x 63) and of L5's pe columns (256 x 63) when they are
#                     not folded (den_render_ray_grad's workspace, -DDEN_NO_PE_FOLD builds)
# F32 (the sample-major parity path):
#   render_bwd      : the whole dX chain, Lr^T, Lg^T, Lb^T (257 x 256), L7^T..L1^T (7 x 256 x 256)
#   dw_gemm         : every layer's weight gradient (the forward's MACs)
def flop_per_sample(rd, mode="bf16"):
    fwd = MAC_PER_SAMPLE[rd]
    if mode == "bf16":
        return {"render_fwd_kernel": 2.0 * fwd,
                "render_head_bwd_kernel": 2.0 * (2 * rd * 128 + 128 * 256 + 128 * 283),
                "hidden_bwd_kernel": 2.0 * (7 * 2 * 256 * 256 + 2 * 256 * 63),
                "hidden_bwd_lb_kernel": 2.0 * 2 * 257 * 256,
                "dwstream_kernel": 2.0 * (256 * 63 * 2)}
    return {"render_fwd_kernel": 2.0 * fwd,
            "render_bwd_kernel": 2.0 * (rd * 128 + 128 * 256 + 257 * 256 + 7 * 256 * 256),
            "dw_gemm_kernel": 2.0 * fwd}


# the kernels behind den_timing's classes on the BF16 layer-major path
BF16_KERNEL_NAMES = {"render_bwd_kernel": "render_head_bwd_kernel", "dw_gemm_kernel": "dwstream_kernel"}

# algorithmic HBM bytes per sample and STEP of each BF16 kernel:
#   hidden_bwd: L7..L1 each read dz_l + a_(l-1) and write dz_(l-1), 256 bf16 each = 1536 B; L5 and L1 also
#     read pe (128 B), and L1 keeps dz_0 on chip (-512 B): 7 x 1536 + 2 x 128 - 512 = 10496 B;
#   hidden_bwd_lb: reads dz_b (257 bf16) + S7, writes dz_7 = 1538 B;
#   render_fwd: the activations + record it stores for the backward, S0..S7 + bottleneck + G + pe +
#     record (4096 + 512 + 256 + 128 + 16 B; ve is recomputed by the head backward, not stored);
#   render_head_bwd: the record + G + bottleneck read, dz_b (256 bottleneck + sigma) written
#     (16 + 256 + 512 + 514 B; dz_g stays on chip);
#   dwstream: dz_0 + dz_5 + pe read = 1152 B
BYTES_PER_SAMPLE = {"hidden_bwd_kernel": 7 * 1536 + 2 * 128 - 512, "hidden_bwd_lb_kernel": 1538, "render_fwd_kernel": 5008,
                    "render_head_bwd_kernel": 1298, "dwstream_kernel": 1152}


def pmc_traffic(kernel, a):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 --pmc pass
    (profiles/pmc_traffic.json, FETCH_SIZE x2 per the gfx950 correction + WRITE_SIZE),
    only when it was taken on this exact workload; else None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            t = json.load(f)
        w = t["workload"]
        if (w["rays"], w["samples"], w["mode"], w["rd"], w.get("pixbw", False)) != (a.rays, a.samples, a.mode, a.rd,
                                                                                   a.pixbw):
            return None
        return t["kernels"][kernel]["hbm_bytes_per_launch"]
    except (OSError, KeyError, ValueError):
        return None


def phase_times(ts, reps=PHASE_REPS):
    """Average duration of each phase, measured with HIP events on the stream
    the kernels are launched on (torch's current stream)."""
    import ctypes
    from deblur_e_nerf import _native as nat
    L = nat.lib()
    st = nat._stream(ts.dev)
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    acc = {"render_fwd": 0.0, "bwd_chain": 0.0, "bwd_dw": 0.0, "other": 0.0}
    for _ in range(reps):
        e = [ev() for _ in range(6)]
        e[0].record()
        ts.prepare()
        ts.bkgd = torch.nn.functional.softplus(ts.bkgd_orig)
        ts.io.bkgd = nat._ptr(ts.bkgd)
        nat._check(L.den_render_fwd(ctypes.byref(ts.desc), ctypes.byref(ts.io), st))
        e[1].record()
        args = (ts.N, ts.rd, 2, 0, int(ts.has_bkgd), ts.min_int, ts.wl[0], ts.wl[1], nat._ptr(ts.rgb),
                nat._ptr(ts.opacity), nat._ptr(ts.channel), nat._ptr(ts.target), nat._ptr(ts.c), nat._ptr(ts.ev_ws))
        nat._check(L.den_event_step_fwd(*args, nat._ptr(ts.loss), st))
        nat._check(L.den_event_step_bwd(*args, nat._ptr(ts.d_rgb), st))
        e[2].record()
        gr = nat.RenderGrad(nat._ptr(ts.d_rgb), None, None, nat._ptr(ts.grad), nat._ptr(ts.grad_bkgd))
        nat._check(L.den_render_bwd_part(ctypes.byref(ts.desc), ctypes.byref(ts.io), ctypes.byref(gr), 1, st))
        e[3].record()
        nat._check(L.den_render_bwd_part(ctypes.byref(ts.desc), ctypes.byref(ts.io), ctypes.byref(gr), 2, st))
        e[4].record()
        ts.allreduce()
        ts.optimizer_step()
        e[5].record()
        torch.cuda.synchronize()
        acc["render_fwd"] += e[0].elapsed_time(e[1])
        acc["other"] += e[1].elapsed_time(e[2]) + e[4].elapsed_time(e[5])
        acc["bwd_chain"] += e[2].elapsed_time(e[3])
        acc["bwd_dw"] += e[3].elapsed_time(e[4])
    return {k: v / reps for k, v in acc.items()}


def measured_gemm_peak(dev, dtype, n=8192, reps=10):
    """Achievable dense-GEMM rate on this box (torch.matmul -> hipBLASLt), TFLOP/s:
    the measured denominator SURVEY.md 8(d) asks for beside the spec peak."""
    a = torch.randn(n, n, device=dev, dtype=dtype)
    b = torch.randn(n, n, device=dev, dtype=dtype)
    for _ in range(3):
        a @ b
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        a @ b
    e1.record()
    torch.cuda.synchronize()
    return round(2.0 * n ** 3 * reps / (e0.elapsed_time(e1) * 1e-3) / 1e12, 1)


def _cpu_info(threads):
    """CPU model (/proc/cpuinfo, as lscpu reports it), cores visible and used, torch version."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return dict(cpu_model=model, cores_visible=len(os.sched_getaffinity(0)), torch=torch.__version__,
                threads=threads)


def cpu_threads():
    """All cores of this process's affinity mask, capped by the
    OMP_NUM_THREADS share the GPU box assigns to one GPU's job."""
    n = len(os.sched_getaffinity(0))
    cap = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(cap))) if cap and cap.isdigit() else n


def _time_median(fn, warmup, reps):
    for _ in range(warmup):
        fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2], ts


def cpu_baseline(rd, threads, legs=((4096, 64, 2, 5), (4096, 128, 1, 3))):
    """The oracle (PyTorch-CPU restatement of the reference path, parity-checked
    against the reference modules) timed on the host cores: one full train step
    (event prep + rays + render fwd + event loss + backward + Adam) per leg.
    Leg 0 is BASELINE configs[0] (chair easy, 4096 rays x 64 samples; median of 5
    after 2 warm-ups); leg 1 is the benchmark's 2^17 x 128
    workload scaled down to 4096 x 128 (median of 3 after 1 warm-up, bounded)."""
    from oracle import nerf as onerf
    from oracle.train import prepare_batch, step_loss
    from deblur_e_nerf.train import synthetic_events
    torch.set_num_threads(threads)
    out = []
    for n_rays, n_samples, warm, reps in legs:
        raw = synthetic_events(n_rays // 4, seed=99)
        p = onerf.build_params(rd, 0)
        params = list(p.values())
        for t in params:
            t.requires_grad_(True)
        bk = torch.tensor([0.5413] * rd, requires_grad=True)
        opt = torch.optim.Adam([{"params": params, "weight_decay": 1e-6}, {"params": [bk]}], lr=0.01)

        def step():
            opt.zero_grad()
            b = prepare_batch(raw)
            total, _, _ = step_loss(p, torch.nn.functional.softplus(bk), b, n_samples)
            total.backward()
            opt.step()

        med, ts = _time_median(step, warm, reps)
        out.append(dict(rays=n_rays, samples=n_samples, rays_per_s=round(n_rays / med, 2),
                        s_per_step_median=round(med, 3), s_per_step_all=[round(t, 3) for t in ts],
                        warmup=warm, reps=reps))
    lead = out[0]
    return dict(value=lead["rays_per_s"], unit="rays/s", cores=threads, kind="port",
                sample=f"oracle (PyTorch CPU) train step, BASELINE configs[0] shape {lead['rays']} rays x "
                       f"{lead['samples']} samples (event prep + rays + render fwd + event loss + backward + Adam), "
                       f"median of {lead['reps']} after {lead['warmup']} warm-ups; second leg "
                       f"{out[1]['rays']} x {out[1]['samples']} (the 2^17 x 128 workload scaled down)",
                legs=out, **_cpu_info(threads))


def _view_rays(n_px, radius=4.03, focal_px=None, direction=(0.62, -0.55, 0.56)):
    """Held-out camera: n_px x n_px pixel rays of a pinhole at `radius` along `direction`,
    looking at the origin (the synthetic chair's AABB centre)."""
    c = torch.tensor(direction)
    c = c / c.norm() * radius
    z = -c / c.norm()
    x = torch.linalg.cross(z, torch.tensor([0.0, 0.0, 1.0]))
    x = x / x.norm()
    y = torch.linalg.cross(z, x)
    f = focal_px or 1.2 * n_px
    j, i = torch.meshgrid(torch.arange(n_px) + 0.5, torch.arange(n_px) + 0.5, indexing="ij")
    d = ((i - n_px / 2) / f)[..., None] * x + ((j - n_px / 2) / f)[..., None] * y + z
    d = d.reshape(-1, 3)
    d = d / d.norm(dim=-1, keepdim=True)
    return c.expand(d.shape[0], 3).contiguous(), d.contiguous()


def psnr_vs_oracle(rd, threads, dev, steps=8, n_events=1024, n_samples=64, view=64, modes=("f32", "bf16")):
    """The second half of BASELINE's metric ("PSNR vs ref"; north_star: rendered PSNR within 0.1 dB
    of the reference).  A teacher scene (a differently seeded MLP, density raised) supervises a
    configs[0]-shaped batch (1024 events = 4096 rays x 64 samples): each event's measured
    log-intensity change is the teacher's.  The HIP TrainStep and the oracle (the reference path
    restated, parity-pinned by tests/) train from the SAME init on that batch for `steps` Adam
    steps; both render a held-out 64x64 view (deblur_e_nerf.py:602-652 eval render), scored against
    the teacher's render with the reference's PSNR (metric.py:68-72, data range 1)."""
    from oracle import nerf as onerf
    from oracle.train import step_loss
    from deblur_e_nerf import _native as nat
    from deblur_e_nerf.loss_metric.metric import psnr
    from deblur_e_nerf.train import TrainStep, synthetic_batch
    torch.set_num_threads(threads)
    teacher = onerf.build_params(rd, 77)
    teacher["mlp.sigma_layer.output_layer.bias"] += 3.0
    ones = torch.ones(rd)
    b = synthetic_batch(n_events, seed=21)
    with torch.no_grad():
        col, _, _, _ = onerf.render_rays(teacher, b["rays_o"], b["rays_d"], b["jitter"], n_samples=n_samples,
                                         bkgd=ones)
        y = torch.log(col[:, 0] + 1e-3).view(4, n_events)
        b["lid"] = (y[1] - y[0]).float().contiguous()
        vo, vd = _view_rays(view)
        vu = torch.full((vo.shape[0],), 0.5)
        target, _, _, _ = onerf.render_rays(teacher, vo, vd, vu, n_samples=n_samples, bkgd=ones)
    out = {}
    oracle_view = None
    for mode in modes:
        ts = TrainStep(n_events, n_samples=n_samples, radiance_dim=rd, mode=mode, device=dev, seed=0)
        ts.load_batch(**b)
        if oracle_view is None:  # the oracle student: the same init, torch.optim.Adam as TrainStep's
            flat0 = ts.flat.detach().cpu()
            names = [n for n, _, _ in onerf.layer_specs(rd)]
            p, off = {}, 0
            for n, fin, fout in onerf.layer_specs(rd):
                p[n + ".weight"] = flat0[off:off + fin * fout].view(fout, fin).clone().requires_grad_(True)
                off += fin * fout
                p[n + ".bias"] = flat0[off:off + fout].clone().requires_grad_(True)
                off += fout
            bk = ts.bkgd_orig.detach().cpu().clone().requires_grad_(True)
            leaves = [p[n + s] for n in names for s in (".weight", ".bias")]
            opt = torch.optim.Adam([{"params": leaves, "weight_decay": ts.wd}, {"params": [bk], "weight_decay": 0.0}],
                                   lr=ts.lr)
            t0 = time.perf_counter()
            for _ in range(steps):
                opt.zero_grad()
                total, _, _ = step_loss(p, torch.nn.functional.softplus(bk), b, n_samples)
                total.backward()
                opt.step()
            oracle_s = time.perf_counter() - t0
            with torch.no_grad():
                oracle_view, _, _, _ = onerf.render_rays(p, vo, vd, vu, n_samples=n_samples,
                                                         bkgd=torch.nn.functional.softplus(bk))
            out["oracle"] = {"psnr_db": round(psnr(oracle_view.to(dev), target.to(dev), 1.0), 3),
                             "train_s": round(oracle_s, 2)}
        for _ in range(steps):
            ts.step()
        with torch.no_grad():
            cfg = dict(ts.cfg)
            hv, _, _ = nat.render(vo.to(dev), vd.to(dev), vu.to(dev),
                                  torch.nn.functional.softplus(ts.bkgd_orig.detach()), ts.flat.detach(), cfg,
                                  ts.packed, n_samples)
        ph = psnr(hv, target.to(dev), 1.0)
        out[mode] = {"psnr_db": round(ph, 3), "delta_db": round(ph - out["oracle"]["psnr_db"], 4),
                     "psnr_vs_oracle_render_db": round(psnr(hv, oracle_view.to(dev), 1.0), 2)}
    return dict(out, steps=steps, setup=f"teacher-scene supervision, {n_events} events = {4 * n_events} rays x "
                                        f"{n_samples} samples, {steps} Adam steps from one init, held-out "
                                        f"{view}x{view} view, PSNR vs the teacher render (data range 1)")


def _teacher_batch(gen, n_events, dev="cpu", motion=0.3, radius=4.03):
    """Events of a camera circling the AABB: per event a pixel direction seen from 4 poses (diff
    start / end, TV start / end inside it) moving by up to `motion` along a random direction.
    Drawn on the CPU generator `gen` (the oracle's converged run, tests/golden/make_psnr_oracle.py,
    replays the same sequence), then moved to `dev`."""
    N = n_events
    v = torch.randn(N, 3, generator=gen)
    c0 = v / v.norm(dim=-1, keepdim=True) * radius
    look = -c0 / c0.norm(dim=-1, keepdim=True) + (torch.rand(N, 3, generator=gen) * 2 - 1) * math.sin(0.3)
    look = look / look.norm(dim=-1, keepdim=True)
    m = torch.randn(N, 3, generator=gen)
    m = m / m.norm(dim=-1, keepdim=True) * motion * torch.rand(N, 1, generator=gen)
    s = torch.rand(2, N, 1, generator=gen).sort(dim=0).values
    o = torch.cat([c0, c0 + m, c0 + s[0] * m, c0 + s[1] * m])
    d = look.repeat(4, 1)
    jit = torch.rand(4 * N, generator=gen)
    end = torch.full((N,), 10 ** 9, dtype=torch.int64)
    start = end.double() - 1e6
    b = dict(rays_o=o.contiguous(), rays_d=d.contiguous(), jitter=jit, end_ts=end, start_ts=start,
             ts_diff=end.double() - start)
    return {k: t.to(dev) for k, t in b.items()}


VIEW_DIRS = ((0.62, -0.55, 0.56), (-0.7, 0.3, 0.4), (0.1, 0.8, -0.5), (-0.4, -0.6, -0.3),
             (0.3, 0.3, 0.9), (-0.8, -0.5, 0.2), (0.7, 0.6, -0.2), (-0.2, 0.4, -0.9))
# the converged-PSNR leg: Adam steps, events per batch, samples per ray, views (count, size), lr cuts
# (x lr_gamma at each milestone fraction of the run), the teacher's density bias and colour-head
# output scale, seeds (teacher init, student init, the first batch sequence)
# (r05: chosen by profiles/psnr_sweep.py -- the sequence-to-sequence std of the converged PSNR,
# profiles/r05a_psnr_sweep.jsonl; 1,500 steps reach the plateau that 3,000 do)
PSNR_LEG = dict(steps=1500, n_events=128, n_samples=64, view=32, n_views=8, milestones=(0.3, 0.6, 0.85), lr_gamma=0.3,
                lr0=0.01, teacher_sigma_bias=3.0, teacher_rgb_scale=1.0, batch_seed=123, teacher_seed=77,
                student_seed=0)


# configs[1]'s 128 samples per ray: HIP BF16 - HIP F32, paired per sequence, on the
# same teacher leg at fewer steps (no oracle fixture exists at 128 samples: the oracle's CPU training
# takes hours; the 64-sample leg above is the one pinned to it)
PSNR_LEG_S128 = dict(PSNR_LEG, n_samples=128, steps=400)
PSNR_S128_SEQUENCES = tuple(range(6))


def psnr_leg(**over):
    """PSNR_LEG with overrides (profiles/psnr_sweep.py, make_psnr_oracle.py --leg)."""
    bad = set(over) - set(PSNR_LEG)
    if bad:
        raise KeyError(f"unknown PSNR leg keys {sorted(bad)}")
    return dict(PSNR_LEG, **over)


def teacher_field(rd, leg=None):
    """The converged leg's teacher: the benchmark architecture with another seeded init, the
    density raised by `teacher_sigma_bias` (an opaque scene) and the colour head's output weights
    x `teacher_rgb_scale` (colour contrast on the surfaces); -> flat f32 parameters (CPU)."""
    from deblur_e_nerf.external import mlp, ngp
    L = leg or PSNR_LEG
    torch.manual_seed(L["teacher_seed"])
    field = mlp.VanillaNeRFRadianceField([-1.5, -1.5, -1.5, 1.5, 1.5, 1.5], radiance_dim=rd,
                                         hidden_activation=torch.nn.Softplus(beta=100),
                                         density_activation=ngp.shifted_trunc_exp,
                                         radiance_activation=torch.nn.Softplus(beta=1), mode="f32")
    with torch.no_grad():
        field.mlp.sigma_layer.output_layer.bias.add_(float(L["teacher_sigma_bias"]))
        field.mlp.rgb_layer.output_layer.weight.mul_(float(L["teacher_rgb_scale"]))
    return field.flat_params.detach().clone()


def psnr_views(view, n_views=4):
    """The converged leg's held-out views: rays (CPU) and their count."""
    rays = [_view_rays(view, direction=v) for v in VIEW_DIRS[:n_views]]
    return torch.cat([r[0] for r in rays]), torch.cat([r[1] for r in rays]), n_views


def lr_at(lr0, it, steps, milestones, gamma=0.3):
    return lr0 * gamma ** sum(it >= int(m * steps) for m in milestones)


def _psnr_host(pred, tgt, rng):
    """metric.py:68-72's PSNR on host tensors (B, C, H, W): 10 log10(range^2 / MSE) per image,
    mean over the batch (the oracle's converged run, which has no device)."""
    mse = ((pred.double() - tgt.double()) ** 2).flatten(1).mean(1)
    return float((10.0 * torch.log10(rng * rng / mse)).mean())


def aligned_psnr(pred, tgt, nv, view, dev=None):
    """The reference's evaluation metric on a batch of views: affine log-intensity correction
    (deblur_e_nerf.py:705-833) of the predictions onto the targets, then PSNR (metric.py:68-72,
    data range [0, max target], mean over views; loss_metric.metric on `dev`, the same formula on
    the host without one) -> (psnr dB, uncorrected psnr dB, gamma, scale)."""
    from deblur_e_nerf.models.deblur_e_nerf import affine_log_intensity_correction
    tgt = tgt[:, 0].reshape(nv, view, view).clamp_min(1e-6).cpu()
    pred = pred[:, 0].reshape(nv, view, view).clamp_min(1e-6).cpu()
    corr, gamma, scale = affine_log_intensity_correction(pred, tgt)
    rng = float(tgt.max())
    if dev is None:
        fn = _psnr_host
    else:
        from deblur_e_nerf.loss_metric.metric import psnr

        def fn(a, b, r):
            return psnr(a.to(dev), b.to(dev), r)
    return fn(corr.float(), tgt[:, None], rng), fn(pred[:, None], tgt[:, None], rng), float(gamma[0]), float(scale[0])


def oracle_fixture_path(seq, device="cpu"):
    """The oracle's converged run on batch sequence `seq`: executed by torch on the build container's
    CPU (tests/golden/psnr_oracle_s<k>.npz), or -- for the seed study's many sequences -- by torch's
    own GPU kernels (tests/golden/psnr_oracle_gpu/, make_psnr_oracle.py --device cuda; never libden)."""
    sub = ("golden",) if device == "cpu" else ("golden", "psnr_oracle_gpu")
    return os.path.join(ROOT, "tests", *sub, f"psnr_oracle_s{seq}.npz")


def _load_oracle_fixture(seq, leg, rd, device="cpu"):
    """The oracle fixture of `seq` when it was trained on exactly this leg, else None."""
    import numpy as np
    path = oracle_fixture_path(seq, device)
    if not os.path.exists(path):
        return None
    fx = np.load(path)
    if str(fx["leg"]) != json.dumps(leg, sort_keys=True) or int(fx["rd"]) != rd:
        return None
    return fx


def _stats(xs):
    if not xs:
        return None
    m = sum(xs) / len(xs)
    sd = math.sqrt(sum((x - m) ** 2 for x in xs) / (len(xs) - 1)) if len(xs) > 1 else float("nan")
    return {"n": len(xs), "mean": round(m, 4), "std": round(sd, 4), "sem": round(sd / math.sqrt(len(xs)), 4)}


def psnr_long(rd, dev, steps=None, modes=("f32", "bf16"), sequences=tuple(range(8)), leg=None):
    """BASELINE's "PSNR vs ref" at convergence (PSNR_LEG): for each batch sequence k, the HIP
    TrainStep in F32 (the reference's arithmetic, pinned to the reference at 1e-4 per step by tests/)
    and in BF16 (the benchmark's mode) train from ONE init on a teacher scene for `steps` Adam steps,
    each on a fresh batch of events (drawn on a CPU generator seeded batch_seed + k) whose measured
    log-intensity changes are the teacher's; the learning rate is cut at the milestones (the
    reference's multi_step_lr); the held-out views are aligned to the teacher's by the reference's
    affine log-intensity correction (deblur_e_nerf.py:705-833) and scored with its PSNR
    (metric.py:68-72).  The reference side: tests/golden/psnr_oracle_s<k>.npz, the ORACLE trained the
    same way on the same batch sequence in the build container (tests/golden/make_psnr_oracle.py), and
    for the sequences without one the same oracle executed by torch on a GPU
    (tests/golden/psnr_oracle_gpu/; where both exist their difference is reported, oracle_gpu_minus_cpu).
    Reported per sequence and as mean / std / standard error over the sequences: each mode's PSNR,
    each mode - the oracle (paired, same sequence) and BF16 - F32."""
    from deblur_e_nerf import _native as nat
    from deblur_e_nerf.loss_metric.metric import psnr
    from deblur_e_nerf.train import TrainStep
    L = dict(leg or PSNR_LEG)
    if steps:
        L["steps"] = steps
    steps, n_events, n_samples, view = L["steps"], L["n_events"], L["n_samples"], L["view"]
    tflat = teacher_field(rd, L).to(dev).contiguous()
    tcfg = dict(mode=nat.mode_id("f32"), rd=rd, aabb=[-1.5, -1.5, -1.5, 1.5, 1.5, 1.5], near=1.43, far=6.63)
    tpacked = nat.PackedWeights("f32", rd, dev)
    tpacked.pack(tflat)
    ones = torch.ones(rd, device=dev)
    vo, vd, nv = psnr_views(view, L["n_views"])
    vo, vd = vo.to(dev), vd.to(dev)
    vu = torch.full((vo.shape[0],), 0.5, device=dev)
    with torch.no_grad():
        target, _, _ = nat.render(vo, vd, vu, ones, tflat, tcfg, tpacked, n_samples)
    rows = []
    for seq in sequences:
        fx_cpu, fx_gpu = _load_oracle_fixture(seq, L, rd, "cpu"), _load_oracle_fixture(seq, L, rd, "cuda")
        fx = fx_cpu if fx_cpu is not None else fx_gpu
        row = {"seq": seq}
        for mode in modes:
            ts = TrainStep(n_events, n_samples=n_samples, radiance_dim=rd, mode=mode, device=dev,
                           seed=L["student_seed"], lr=L["lr0"])
            gen = torch.Generator().manual_seed(L["batch_seed"] + seq)
            t0 = time.perf_counter()
            for it in range(steps):
                ts.lr = lr_at(L["lr0"], it, steps, L["milestones"], L["lr_gamma"])
                b = _teacher_batch(gen, n_events, dev)
                with torch.no_grad():
                    col, _, _ = nat.render(b["rays_o"], b["rays_d"], b["jitter"], ones, tflat, tcfg, tpacked,
                                           n_samples)
                y = torch.log(col[:, 0] + 1e-3).view(4, n_events)
                ts.load_batch(lid=(y[1] - y[0]).float().contiguous(), **b)
                ts.step()
            torch.cuda.synchronize()
            train_s = time.perf_counter() - t0
            with torch.no_grad():
                hv, _, _ = nat.render(vo, vd, vu, torch.nn.functional.softplus(ts.bkgd_orig.detach()),
                                      ts.flat.detach(), dict(ts.cfg), ts.packed, n_samples)
            ps, ps_raw, gamma, scale = aligned_psnr(hv, target, nv, view, dev)
            e = {"psnr_db": round(ps, 4), "psnr_uncorrected_db": round(ps_raw, 3), "gamma": round(gamma, 4),
                 "train_s": round(train_s, 2), "final_loss": [round(x, 6) for x in ts.loss[:3].tolist()]}
            if fx is not None:
                orc = torch.from_numpy(fx["pred"]).reshape(-1, 1).to(dev)
                e["minus_oracle_db"] = round(ps - float(fx["psnr_db"]), 4)
                # the HIP-trained views against the oracle-trained ones (range of the oracle's render)
                e["psnr_vs_oracle_render_db"] = round(psnr(hv[:, 0].reshape(nv, 1, view, view),
                                                           orc.reshape(nv, 1, view, view), float(orc.max())), 2)
            row[mode] = e
            del ts
            torch.cuda.empty_cache()
        if fx is not None:
            row["oracle"] = {"psnr_db": round(float(fx["psnr_db"]), 4),
                             "executed_on": "cpu" if fx_cpu is not None else "gpu (torch)"}
            if fx_cpu is not None:
                row["oracle"]["threads"] = int(fx_cpu["threads"])
            if fx_cpu is not None and fx_gpu is not None:
                row["oracle_gpu_minus_cpu_db"] = round(float(fx_gpu["psnr_db"]) - float(fx_cpu["psnr_db"]), 4)
        if "f32" in row and "bf16" in row:
            row["bf16_minus_f32_db"] = round(row["bf16"]["psnr_db"] - row["f32"]["psnr_db"], 4)
        rows.append(row)
        print(json.dumps({"psnr_seq": row}), file=sys.stderr, flush=True)
    summary = {m: _stats([r[m]["psnr_db"] for r in rows if m in r]) for m in modes}
    summary["oracle"] = _stats([r["oracle"]["psnr_db"] for r in rows if "oracle" in r])
    for m in modes:
        summary[f"{m}_minus_oracle"] = _stats([r[m]["minus_oracle_db"] for r in rows
                                               if "minus_oracle_db" in r.get(m, {})])
    summary["bf16_minus_f32"] = _stats([r["bf16_minus_f32_db"] for r in rows if "bf16_minus_f32_db" in r])
    summary["oracle_gpu_minus_cpu"] = _stats([r["oracle_gpu_minus_cpu_db"] for r in rows
                                              if "oracle_gpu_minus_cpu_db" in r])
    return dict(rows=rows, summary=summary, leg=L,
                setup=f"teacher scene, {steps} Adam steps from one init (lr {L['lr0']} x{L['lr_gamma']} at "
                      f"{list(L['milestones'])} of the run), each on a fresh batch of {n_events} events = "
                      f"{4 * n_events} rays x {n_samples} samples; {nv} held-out {view}x{view} views, affine "
                      f"log-intensity correction, mean PSNR vs the teacher; per batch sequence, HIP F32 / BF16 "
                      f"and the oracle trained identically (tests/golden/psnr_oracle_s<k>.npz, executed on "
                      f"the CPU; tests/golden/psnr_oracle_gpu/ by torch on a GPU)")


def cpu_baseline_pixbw(n_rays, n_samples, rd, S, threads):
    """Bounded CPU sample of the pixel-bandwidth-on step (oracle): median of 3 after 1 warm-up."""
    from oracle import nerf as onerf
    from oracle import pixbw as opb
    from oracle.train import pixbw_step_loss
    from deblur_e_nerf.train import EDS_CALIBRATION, synthetic_pixbw_events
    torch.set_num_threads(threads)
    N = max(1, n_rays // (4 * S))
    raw = synthetic_pixbw_events(N, S, seed=99)
    prm = opb.calib_to_params(EDS_CALIBRATION)
    p = onerf.build_params(rd, 0)
    params = list(p.values())
    for t in params:
        t.requires_grad_(True)
    bk = torch.tensor([0.5413] * rd, requires_grad=True)
    opt = torch.optim.Adam([{"params": params, "weight_decay": 1e-6}, {"params": [bk]}], lr=0.01)

    def step():
        opt.zero_grad()
        total, _, _ = pixbw_step_loss(p, torch.nn.functional.softplus(bk), raw, S, n_samples, prm, 5e7)
        total.backward()
        opt.step()

    med, ts = _time_median(step, 1, 3)
    R = 4 * S * N
    return dict(value=round(R / med, 2), unit="rays/s", cores=threads, kind="port",
                sample=f"oracle (PyTorch CPU) pixel-bandwidth-on train step, {N} events x 4 x S={S} = {R} rays x "
                       f"{n_samples} samples, median of 3 after 1 warm-up, {med:.2f} s/step",
                **_cpu_info(threads))


def timed_steps(ts, a, world, dev, sync):
    """W untimed warm-up steps, then EXACTLY K steps bracketed by a barrier + device sync on both
    sides; the max over ranks of the elapsed time (seconds)."""
    for _ in range(a.warmup):
        ts.step()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        ts.step()
    sync()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    return elapsed


def init_ranks(a, world, local, dist_mod=dist, cuda=torch.cuda):
    """One process per GPU: rank `local` binds device `local` and joins the process group over RCCL
    (backend "nccl", bound to that device); --dist-backend gloo rehearses N ranks on fewer GPUs
    (rank r on device r mod count).  -> (world size, this rank's device).  dist_mod / cuda are
    parameters so tests/test_bench_launcher.py checks the wiring on the CPU."""
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if a.dist_backend == "gloo":
            # rehearsal: RCCL refuses two ranks on one device, gloo all-reduces the GPU buffers
            local = local % cuda.device_count()
            cuda.set_device(local)
            dist_mod.init_process_group("gloo")
        else:
            cuda.set_device(local)
            dist_mod.init_process_group("nccl", device_id=torch.device("cuda", local))
        world = dist_mod.get_world_size()
    return world, torch.device("cuda", local)


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(a))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE {world}")
    if a.cpu_stub:
        if world > 1:
            dist.init_process_group("gloo")
        world = dist.get_world_size() if world > 1 else 1
        dev = torch.device("cpu")
        ts = StubStep(a.rays, world)
        elapsed = timed_steps(ts, a, world, dev, lambda: None)
        if rank == 0:
            print(json.dumps({"metric": metric_name(a), "value": round(a.rays * a.steps / elapsed, 1),
                              "unit": "rays/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
                              "ms_per_step": round(elapsed / a.steps * 1e3, 3), "data": "cpu stub",
                              "config": {"rays_per_step": a.rays, "rays_per_rank": ts.R,
                                         "parallelism": f"ray-dp{world}"}}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return
    world, dev = init_ranks(a, world, local)
    from deblur_e_nerf import _native as nat
    if a.psnr_only:
        print(json.dumps(psnr_long(a.rd, dev, steps=a.psnr_steps or None)), flush=True)
        return

    ts, per_event = build_step(a, dev, rank, world)
    rays_per_rank = ts.R
    elapsed = timed_steps(ts, a, world, dev, torch.cuda.synchronize)
    loss = ts.loss[:3].tolist()
    ms = elapsed / a.steps * 1e3
    rays_per_step = a.rays
    value = rays_per_step * a.steps / elapsed

    nat.timing_enable(True)
    if a.pixbw:  # autograd-chained step: per-kernel timing over whole steps, no phase split
        for _ in range(PHASE_REPS):
            ts.step()
        torch.cuda.synchronize()
        phases = {}
    else:
        phases = phase_times(ts)
    nat.timing_enable(False)
    kt = nat.timing_collect()
    n_local = ts.R * (ts.n_samples if a.pixbw else ts.S)
    fps = flop_per_sample(a.rd, a.mode)
    peak = PEAK_TFLOPS[a.mode]
    kernels = {}
    for k, (tot, cnt) in kt.items():
        if cnt == 0:
            continue
        if a.mode == "bf16":
            k = BF16_KERNEL_NAMES.get(k, k)
        avg = tot / cnt
        e = {"launches_per_step": cnt // PHASE_REPS, "avg_ms": round(avg, 4),
             "step_ms": round(tot / PHASE_REPS, 3)}
        if k in fps:
            f = fps[k] * n_local * PHASE_REPS / cnt  # algorithmic flop per launch
            e.update(flop_per_launch=f, tflops=round(f / (avg * 1e-3) / 1e12, 1),
                     mfma_frac=round(f / (avg * 1e-3) / 1e12 / peak, 4))
        if k in BYTES_PER_SAMPLE and a.mode == "bf16":
            b = BYTES_PER_SAMPLE[k] * n_local * PHASE_REPS / cnt  # algorithmic (design) bytes per launch
            e.update(bytes_per_launch=b, gbs=round(b / (avg * 1e-3) / 1e9, 1),
                     hbm_frac=round(b / (avg * 1e-3) / 1e9 / PEAK_HBM_GBS, 4))
        kernels[k] = e
    # the roofline line is on SURVEY.md 8(d)'s axis (MFMA, algorithmic FLOP) for the kernel that
    # takes most of the step; its HBM-axis figures (the design's streamed bytes) ride along
    dom = max((k for k in kernels if k in fps), key=lambda k: kernels[k]["step_ms"])
    de = kernels[dom]
    roofline = {"bound": "mfma", "achieved": de["tflops"], "peak": peak, "unit": "TFLOP/s",
                "frac": de["mfma_frac"], "traffic": pmc_traffic(dom, a), "traffic_unit": "bytes per launch (PMC)",
                "kernel": dom, "avg_launch_ms": de["avg_ms"], "flop_per_launch": de["flop_per_launch"],
                "timing": "hipEvents on the launch stream (den_timing_*)"}
    if "gbs" in de:
        roofline["hbm"] = {"achieved": de["gbs"], "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": de["hbm_frac"],
                           "bytes_per_launch": de["bytes_per_launch"]}
    step_flop = 3.0 * 2.0 * MAC_PER_SAMPLE[a.rd] * n_local
    roofline["step_mfma_frac"] = round(step_flop / (ms * 1e-3) / 1e12 / peak, 4)
    if rank == 0 and not a.no_gemm_peak:
        gp = measured_gemm_peak(dev, torch.bfloat16 if a.mode == "bf16" else torch.float32)
        roofline["mfma_peak_measured"] = {"tflops": gp, "how": "torch.matmul 8192^3 (hipBLASLt), HIP events",
                                          "step_frac": round(step_flop / (ms * 1e-3) / 1e12 / gp, 4)}
    roofline["kernels"] = kernels
    roofline["phases_ms"] = {k: round(v, 3) for k, v in phases.items()}

    legs = None
    if world == 1 and not a.no_extra_legs and not a.pixbw and a.mode == "bf16":
        del ts
        torch.cuda.empty_cache()
        legs = {}
        for name, pb, mode, k, rays in (("configs2_pixbw_on", True, "bf16", 10, None),
                                        ("configs1_f32_65536_rays", False, "f32", 3, a.rays // 2)):
            try:
                legs[name] = extra_leg(a, dev, pb, mode, k, rays=rays)
            except Exception as e:  # pragma: no cover - reported, not fatal
                legs[name] = {"error": repr(e)}
    cpu = None
    psnr_info = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        try:
            threads = cpu_threads()
            cpu = (cpu_baseline_pixbw(a.cpu_rays, a.samples, a.rd, a.it_samples, threads) if a.pixbw
                   else cpu_baseline(a.rd, threads))
        except Exception as e:  # pragma: no cover - reported, not fatal
            cpu = {"error": repr(e)}
        if not a.pixbw:
            try:  # the oracle leg's second product: ΔPSNR of the HIP-trained render vs the oracle-trained one
                psnr_info = psnr_vs_oracle(a.rd, cpu_threads(), dev)
            except Exception as e:  # pragma: no cover - reported, not fatal
                psnr_info = {"error": repr(e)}
            if a.psnr_steps > 0:
                try:  # converged: HIP BF16 vs HIP F32 after psnr_steps steps on fresh teacher batches
                    psnr_info = dict(psnr_info or {}, converged=psnr_long(a.rd, dev, steps=a.psnr_steps))
                except Exception as e:  # pragma: no cover - reported, not fatal
                    psnr_info = dict(psnr_info or {}, converged={"error": repr(e)})
                try:  # the benchmark's 128 samples per ray: BF16 - F32 (paired, no oracle at this size)
                    s128 = psnr_long(a.rd, dev, leg=PSNR_LEG_S128, sequences=PSNR_S128_SEQUENCES)
                    psnr_info = dict(psnr_info or {}, samples128={"summary": {k: s128["summary"][k] for k in
                                                                              ("f32", "bf16", "bf16_minus_f32")},
                                                                  "rows": s128["rows"], "leg": s128["leg"]})
                except Exception as e:  # pragma: no cover - reported, not fatal
                    psnr_info = dict(psnr_info or {}, samples128={"error": repr(e)})
    if rank == 0:
        out = {
            "metric": metric_name(a),
            "value": round(value, 1), "unit": "rays/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": a.mode, "data": "synthetic (chair-like raw events + camera poses, PyTorch default-init weights)",
            "config": {"workload": f"chair synthetic, pixel-bandwidth {'on (it_sample_size=%d)' % a.it_samples if a.pixbw else 'off'}, "
                                   f"{a.rays} rays x {a.samples} samples, "
                                   f"mlp 8x256 rd={a.rd}, event prep+rays+fwd+bwd+allreduce+Adam",
                       "rays_per_step": a.rays, "rays_per_rank": rays_per_rank, "samples_per_ray": a.samples,
                       "events_per_step": a.rays // per_event,
                       "parallelism": f"ray-dp{world}",
                       "collective": (("rccl" if a.dist_backend == "nccl" else "gloo (shared-GPU rehearsal)")
                                      if world > 1 else None)},
            "loss": [round(x, 6) for x in loss],
            "roofline": roofline,
            "cpu_baseline": cpu,
            "extra_legs": legs,
            "psnr": psnr_info,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
