"""Summarise rocprofv3 output of profiles/gpu_round.sh into committed evidence.

    python profiles/pmc_summary.py gpurun_out <round tag>

* profiles/pmc_traffic.json -- HBM bytes per launch of each render-path kernel
  from the separate `--pmc FETCH_SIZE` and `--pmc WRITE_SIZE` passes, corrected
  as MI355X_MICROARCH.md prescribes for gfx950 (FETCH_SIZE counts half the
  bytes of wide coalesced streaming reads: x2; both counters are in KiB).
  bench.py reads it for `roofline.traffic` when the workload matches.
* profiles/<tag>_kernel_stats.md -- the `--kernel-trace --stats` table.
"""
import csv
import json
import os
import sys
from collections import defaultdict

KERNELS = ("render_fwd_kernel", "render_head_bwd_kernel", "render_bwd_kernel", "hidden_bwd_kernel", "dwstream_kernel",
           "dw_gemm_kernel",
           "dw_reduce_kernel", "pack_kernel", "adam_kernel")


def short(name):
    if "hidden_bwd_kernel<true" in name:  # the Lb launch (den_hidden.hip, LB = true)
        return "hidden_bwd_lb_kernel"
    for k in KERNELS:
        if k in name:
            return k
    return None


def per_launch(path, counter):
    acc = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            k = short(row["Kernel_Name"])
            if k:
                acc[k].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def per_launch_all(path):
    """{kernel: {counter: mean per launch}} of one --pmc pass."""
    acc = defaultdict(lambda: defaultdict(list))
    with open(path) as f:
        for row in csv.DictReader(f):
            k = short(row["Kernel_Name"])
            if k:
                acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


def mfma_summary(out_dir, tag, n_simd=1024, prefix=""):
    """MFMA utilisation and stall breakdown per kernel from the two SQ passes of
    profiles/gpu_r02a.sh.  Calibration: SQ_VALU_MFMA_BUSY_CYCLES = 32 x SQ_INSTS_MFMA for
    v_mfma_f32_32x32x16_bf16 (MI355X_MICROARCH.md), summed over the SIMDs; GRBM_GUI_ACTIVE is the
    sum over the 8 XCDs, so the kernel's clock cycles are GRBM_GUI_ACTIVE / 8; utilisation =
    MFMA busy / (1024 SIMDs x kernel cycles).  SQ_WAVE_CYCLES and the SQ_WAIT_* / SQ_ACTIVE_*
    counters are in the same (quad-cycle) unit, so their ratios are wave-time fractions."""
    a = per_launch_all(os.path.join(out_dir, prefix + "pmc_mfma", "run_counter_collection.csv"))
    b = per_launch_all(os.path.join(out_dir, prefix + "pmc_mfma2", "run_counter_collection.csv"))
    res = {}
    for k in a:
        c = dict(a[k])
        c.update(b.get(k, {}))
        cycles = c["GRBM_GUI_ACTIVE"] / 8.0
        wave = c["SQ_WAVE_CYCLES"]
        res[k] = {"counters_per_launch": {n: round(v) for n, v in sorted(c.items())},
                  "kernel_cycles": round(cycles),
                  "mfma_util": round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (n_simd * cycles), 4),
                  "mfma_busy_per_inst": round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / max(c.get("SQ_INSTS_MFMA", 1), 1), 2),
                  "wave_frac_wait_any": round(c["SQ_WAIT_ANY"] / wave, 4),
                  "wave_frac_wait_inst_any": round(c.get("SQ_WAIT_INST_ANY", 0) / wave, 4),
                  "wave_frac_active_inst_any": round(c.get("SQ_ACTIVE_INST_ANY", 0) / wave, 4),
                  "wave_frac_wait_inst_lds": round(c["SQ_WAIT_INST_LDS"] / wave, 4),
                  "lds_bank_conflict_frac": round(c["SQ_LDS_BANK_CONFLICT"] / max(c.get("SQ_LDS_IDX_ACTIVE", 1), 1), 4),
                  "valu_mfma_coexec_frac": round(c.get("SQ_VALU_MFMA_COEXEC_CYCLES", 0) / max(
                      c["SQ_VALU_MFMA_BUSY_CYCLES"], 1), 4),
                  "valu_insts_per_mfma": round(c.get("SQ_INSTS_VALU", 0) / max(c.get("SQ_INSTS_MFMA", 1), 1), 2)}
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), f"{tag}_pmc_mfma.json"), "w") as f:
        json.dump({"source": f"rocprofv3 --pmc, two SQ passes ({tag}); see pmc_summary.mfma_summary",
                   "command": "bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-gemm-peak", "kernels": res}, f,
                  indent=1)
    return res


def roofline_check(out_dir, tag, prefix="", phase_reps=3):
    """roofline.frac reproduced from the rocprofv3 kernel trace of the SAME process that printed the
    bench line (``<prefix>prof/run_kernel_trace.csv`` + the JSON line in ``<prefix>prof.log``).

    bench.py times the dominant kernel with HIP events during its phase-timing leg (PHASE_REPS
    steps after the timed region); those are the LAST ``launches_per_step x PHASE_REPS`` launches of
    that kernel in the trace.  Their rocprof mean, the mean over every launch (cold first steps
    included -- the r03 discrepancy), and the bench's HIP-event mean are written side by side with
    the fraction each implies, to ``profiles/<tag>_roofline_check.json``."""
    with open(os.path.join(out_dir, prefix + "prof.log")) as f:
        line = [ln for ln in f if ln.startswith("{")][-1]
    b = json.loads(line)
    rf = b["roofline"]
    k = rf["kernel"]
    ke = rf["kernels"][k]
    n_phase = ke["launches_per_step"] * phase_reps
    durs = []
    with open(os.path.join(out_dir, prefix + "prof", "run_kernel_trace.csv")) as f:
        for row in csv.DictReader(f):
            if short(row["Kernel_Name"]) == k:
                durs.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]) - int(row["Start_Timestamp"])))
    durs = [d for _, d in sorted(durs)]
    phase = durs[-n_phase:]
    avg_phase = sum(phase) / len(phase) / 1e6
    avg_all = sum(durs) / len(durs) / 1e6
    flop, peak = ke["flop_per_launch"], rf["peak"]
    frac = lambda ms: round(flop / (ms * 1e-3) / 1e12 / peak, 4)  # noqa: E731
    res = {"source": f"rocprofv3 --kernel-trace of the bench process whose JSON line is in {prefix}prof.log ({tag})",
           "kernel": k, "flop_per_launch": flop, "peak_tflops": peak, "launches_total": len(durs),
           "launches_phase_leg": len(phase),
           "bench_hip_event_avg_ms": ke["avg_ms"], "bench_frac": rf["frac"],
           "rocprof_phase_leg_avg_ms": round(avg_phase, 4), "rocprof_phase_leg_frac": frac(avg_phase),
           "rocprof_all_launches_avg_ms": round(avg_all, 4), "rocprof_all_launches_frac": frac(avg_all),
           "rocprof_phase_leg_durations_ms": [round(d / 1e6, 4) for d in phase],
           "hip_event_vs_rocprof": round(ke["avg_ms"] / avg_phase, 4)}
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), f"{tag}_roofline_check.json"), "w") as f:
        json.dump(res, f, indent=1)
    return res


def main(out_dir, tag, prefix=""):
    here = os.path.dirname(os.path.abspath(__file__))
    fetch = per_launch(os.path.join(out_dir, prefix + "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = per_launch(os.path.join(out_dir, prefix + "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE")
    kern = {}
    for k in sorted(set(fetch) & set(write)):
        rd, wr = 2.0 * fetch[k] * 1024, write[k] * 1024
        kern[k] = {"fetch_size_kib": round(fetch[k], 1), "write_size_kib": round(write[k], 1),
                   "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
                   "hbm_bytes_per_launch": rd + wr}
    res = {"source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes ({tag}); "
                     "FETCH_SIZE x2 (gfx950 wide-read correction), KiB -> bytes",
           "command": f"bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-gemm-peak ({f'profiles/gpu_{prefix[:-1]}.sh' if prefix else 'profiles/gpu_r02a.sh'})",
           "workload": {"rays": 131072, "samples": 128, "mode": "bf16", "rd": 1},
           "kernels": kern}
    with open(os.path.join(here, "pmc_traffic.json"), "w") as f:
        json.dump(res, f, indent=1)
    rows = []
    with open(os.path.join(out_dir, prefix + "prof", "run_kernel_stats.csv")) as f:
        for r in csv.DictReader(f):
            rows.append(r)
    # the traced command (PROF_CMD, set by the gpu script; the r02-r06fin3 scripts ran this default)
    cmd = os.environ.get("PROF_CMD", "python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-gemm-peak")
    lines = [f"# rocprofv3 --kernel-trace --stats ({tag})", "",
             f"Command: `rocprofv3 --kernel-trace --stats --output-format csv -- {cmd}` ("
             + (f"profiles/gpu_{prefix[:-1]}.sh" if prefix else "profiles/gpu_r02a.sh, gpu_r02g.sh")
             + "); W + K train steps + 3 phase-timing reps per kernel.", "",
             "| kernel | calls | avg ms | total % |", "|---|---|---|---|"]
    for r in rows[:20]:
        lines.append(f"| `{r['Name'][:90]}` | {r['Calls']} | {float(r['AverageNs']) / 1e6:.3f} | "
                     f"{float(r['Percentage']):.2f} |")
    lines += ["", "HBM traffic per launch (separate PMC passes, profiles/pmc_traffic.json):", "",
              "| kernel | read GB | write GB | total GB |", "|---|---|---|---|"]
    for k, v in kern.items():
        lines.append(f"| `{k}` | {v['hbm_read_bytes_per_launch'] / 1e9:.2f} | "
                     f"{v['hbm_write_bytes_per_launch'] / 1e9:.2f} | {v['hbm_bytes_per_launch'] / 1e9:.2f} |")
    if os.path.exists(os.path.join(out_dir, prefix + "pmc_mfma", "run_counter_collection.csv")):
        mf = mfma_summary(out_dir, tag, prefix=prefix)
        lines += ["", f"MFMA utilisation and wave-time breakdown (separate SQ passes, profiles/{tag}_pmc_mfma.json):",
                  "", "| kernel | MFMA util | wait (waitcnt/barrier) | issue stall | active | LDS-issue stall | "
                  "LDS bank-conflict share | VALU-MFMA co-exec / MFMA busy | VALU insts / MFMA |",
                  "|---|---|---|---|---|---|---|---|---|"]
        for k, v in mf.items():
            lines.append(f"| `{k}` | {v['mfma_util']:.3f} | {v['wave_frac_wait_any']:.2f} | "
                         f"{v['wave_frac_wait_inst_any']:.2f} | {v['wave_frac_active_inst_any']:.2f} | "
                         f"{v['wave_frac_wait_inst_lds']:.3f} | {v['lds_bank_conflict_frac']:.2f} | "
                         f"{v['valu_mfma_coexec_frac']:.2f} | {v['valu_insts_per_mfma']:.2f} |")
    if os.path.exists(os.path.join(out_dir, prefix + "prof", "run_kernel_trace.csv")):
        rc = roofline_check(out_dir, tag, prefix)
        lines += ["", f"roofline.frac from this trace (profiles/{tag}_roofline_check.json): `{rc['kernel']}`, the "
                  f"bench's phase-timing launches: HIP events {rc['bench_hip_event_avg_ms']:.3f} ms "
                  f"(frac {rc['bench_frac']}), rocprof {rc['rocprof_phase_leg_avg_ms']:.3f} ms "
                  f"(frac {rc['rocprof_phase_leg_frac']}); all {rc['launches_total']} launches incl. cold steps "
                  f"{rc['rocprof_all_launches_avg_ms']:.3f} ms (frac {rc['rocprof_all_launches_frac']})."]
    with open(os.path.join(here, f"{tag}_kernel_stats.md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    print(json.dumps(kern, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "")
