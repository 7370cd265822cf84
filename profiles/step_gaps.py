"""Diagnostic: GPU-side time between the kernels of a training step, from a rocprofv3 --kernel-trace
CSV of `bench.py` (its timed region: the run's longest stretch of back-to-back render steps).  Per step:
wall span from one render_fwd_kernel start to the next, the sum of kernel durations in it, the idle
time (gaps) and the largest gaps with the kernels around them.
usage: python profiles/step_gaps.py <kernel_trace.csv>"""
import csv
import json
import sys


def main():
    rows = []
    with open(sys.argv[1]) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if "render_fwd_kernel" in r[2]]
    steps = []
    for a, b in zip(starts, starts[1:]):
        seg = rows[a:b]
        span = rows[b][0] - seg[0][0]
        busy = sum(e - s for s, e, _ in seg)
        gaps = []
        for (s0, e0, n0), (s1, e1, n1) in zip(seg, seg[1:] + [rows[b]]):
            gaps.append((s1 - e0, n0.split("(")[0][-40:], n1.split("(")[0][-40:]))
        gaps.sort(reverse=True)
        steps.append({"span_ms": span / 1e6, "busy_ms": busy / 1e6, "idle_ms": (span - busy) / 1e6, "kernels": len(seg),
                      "top_gaps_us": [(round(g / 1e3, 1), x, y) for g, x, y in gaps[:6]],
                      "kernel_ms": {}})
        for s, e, n in seg:
            k = n.split("(")[0].split("<")[0].split(" ")[-1]
            steps[-1]["kernel_ms"][k] = round(steps[-1]["kernel_ms"].get(k, 0) + (e - s) / 1e6, 4)
    for s in steps:
        print(json.dumps(s))


if __name__ == "__main__":
    main()
