"""Summarise profiles/gpu_r05pl.sh: instruction-cache counters per launch of the hot kernels for the
page-aligned product and the default placement, beside each build's timed bench line.
    python profiles/sqc_summary.py gpurun_out r05pl"""
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import short  # noqa: E402


def per_launch(path):
    acc = defaultdict(lambda: defaultdict(list))
    with open(path) as f:
        for row in csv.DictReader(f):
            k = short(row["Kernel_Name"])
            if k:
                acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


def bench(path):
    for line in open(path):
        if line.startswith("{"):
            d = json.loads(line)
            return {"ms_per_step": d["ms_per_step"],
                    "kernel_step_ms": {k: v["step_ms"] for k, v in d["roofline"]["kernels"].items()}}
    return None


def main(out, tag):
    res = {}
    for name in ("al", "un"):
        pl = per_launch(os.path.join(out, f"{tag}_{name}", "run_counter_collection.csv"))
        res[name] = {"counters_per_launch": {k: {c: round(v) for c, v in cs.items()} for k, cs in pl.items()},
                     "icache_miss_rate": {k: round(cs["SQC_ICACHE_MISSES"] / max(1.0, cs["SQC_ICACHE_MISSES"] +
                                                                                 cs["SQC_ICACHE_HITS"]), 5)
                                          for k, cs in pl.items() if "SQC_ICACHE_MISSES" in cs},
                     "bench": bench(os.path.join(out, f"{tag}_t_{name}.log"))}
    res["builds"] = {"al": "product: every hot kernel's code page-aligned (DEN_CODE_ALIGN)",
                     "un": "-DDEN_NO_CODE_ALIGN: the linker's default placement"}
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), f"{tag}_sqc.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({n: {"miss": res[n]["icache_miss_rate"], "bench": res[n]["bench"]} for n in ("al", "un")},
                     indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
