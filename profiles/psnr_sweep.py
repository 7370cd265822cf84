"""Variance study of bench.py's converged-PSNR leg (make the PSNR acceptance
measurable).  For each leg variant (overrides of bench.PSNR_LEG) it trains the HIP TrainStep from
one init on K batch sequences and reports the sequence-to-sequence mean / std of the PSNR -- the
noise against which "within 0.1 dB of the reference" has to be read.

    python profiles/psnr_sweep.py --seqs 4 --modes f32 --variants '[{"steps": 2000, "n_events": 256}]'
    (GPU; one JSON line per variant on stdout and appended to --out, per-sequence rows on stderr)
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seqs", type=int, default=4)
    ap.add_argument("--modes", default="f32")
    ap.add_argument("--variants", default="[{}]", help="JSON list of PSNR_LEG overrides")
    ap.add_argument("--out", default="gpurun_out/psnr_sweep.jsonl")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    for over in json.loads(a.variants):
        leg = bench.psnr_leg(**over)
        r = bench.psnr_long(1, dev, modes=tuple(a.modes.split(",")), sequences=tuple(range(a.seqs)), leg=leg)
        line = json.dumps({"over": over, "summary": r["summary"],
                           "rows": [{k: (v["psnr_db"] if isinstance(v, dict) and "psnr_db" in v else v)
                                     for k, v in row.items()} for row in r["rows"]],
                           "train_s": [row[m]["train_s"] for row in r["rows"] for m in a.modes.split(",")]})
        print(line, flush=True)
        with open(a.out, "a") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
