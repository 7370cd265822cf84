"""Seed study of bench.py's converged-PSNR leg.

The leg trains HIP F32 and HIP BF16 from one init for 1,000 Adam steps on a teacher scene; it is not
at convergence, so one batch sequence's PSNR moves by ~1 dB with the sequence.  This script repeats
the leg over K batch sequences (seed shifts 0..K-1; shift 0 is the bench leg, the one the oracle
fixture was trained on) and reports, per sequence and over all of them, PSNR(BF16) - PSNR(F32):
whether the benchmark's BF16 arithmetic moves the converged PSNR beyond the run's own spread.

    python profiles/psnr_seeds.py [--seeds K] [--steps N]   (GPU; one JSON line, progress on stderr)
"""
import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=8)
    ap.add_argument("--steps", type=int, default=bench.PSNR_LEG["steps"])
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    rows = []
    for k in range(a.seeds):
        r = bench.psnr_long(1, dev, steps=a.steps, modes=(f"f32_s{k}", f"bf16_s{k}"))
        f, b = r[f"f32_s{k}"], r[f"bf16_s{k}"]
        row = {"shift": k, "f32_db": f["psnr_db"], "bf16_db": b["psnr_db"],
               "delta_db": round(b["psnr_db"] - f["psnr_db"], 4)}
        if "delta_vs_oracle_db" in f:
            row.update(f32_vs_oracle_db=f["delta_vs_oracle_db"], bf16_vs_oracle_db=b["delta_vs_oracle_db"])
        rows.append(row)
        print(json.dumps(row), file=sys.stderr, flush=True)

    def stats(xs):
        m = sum(xs) / len(xs)
        sd = math.sqrt(sum((x - m) ** 2 for x in xs) / (len(xs) - 1)) if len(xs) > 1 else float("nan")
        return {"mean": round(m, 4), "std": round(sd, 4), "sem": round(sd / math.sqrt(len(xs)), 4)}

    out = {"steps": a.steps, "sequences": a.seeds, "rows": rows,
           "f32_db": stats([r["f32_db"] for r in rows]), "bf16_db": stats([r["bf16_db"] for r in rows]),
           "delta_bf16_minus_f32_db": stats([r["delta_db"] for r in rows]),
           "setup": "bench.psnr_long per batch sequence (PSNR_LEG: teacher scene, one student init, "
                    "512 events x 64 samples per step, lr x0.3 at 50 %/80 %, 4 held-out 64x64 views, "
                    "affine log-intensity correction)"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
