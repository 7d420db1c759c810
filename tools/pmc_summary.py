#!/usr/bin/env python3
"""Summarise one gpu_round.sh pass (rocprofv3 CSV output) into the per-round profile files.

    python tools/pmc_summary.py gpurun_out/<run> profiles/<round> --warmup 3 [--config-json bench.json]

Writes
  <prefix>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (as produced)
  <prefix>_traffic.json       HBM bytes per sr_sweep_kernel launch from the PMC passes, plus the
                              SQ/LDS counters and the kernel-trace duration of the timed launches

HBM traffic follows MI355X_MICROARCH.md (HBM section): FETCH_SIZE and WRITE_SIZE are collected
in separate --pmc passes (FETCH_SIZE uses 3 of the 4 TCC slots, WRITE_SIZE 2); rocprofv3 reports
both in KiB; on gfx950 FETCH_SIZE counts half the bytes of a coalesced streaming read, so the
fetch figure is doubled.  The kernel's loads are dword-per-lane (coalesced 256 B per wave), a
width the guide lists as uncalibrated -- the raw values are kept next to the corrected ones.
bench.py reads <prefix>_traffic.json for its roofline.traffic field when the workload matches.
"""
import argparse
import csv
import json
import os
import shutil
import statistics
import sys

KERNEL = "sr_sweep_kernel"


def per_dispatch(path):
    """{counter: [value per sr_sweep_kernel dispatch in dispatch order]} and the kernel name"""
    rows = [r for r in csv.DictReader(open(path)) if KERNEL in r["Kernel_Name"]]
    out, name = {}, None
    by_disp = {}
    for r in rows:
        name = r["Kernel_Name"]
        key = (int(r["Dispatch_Id"]), r["Counter_Name"])
        by_disp[key] = by_disp.get(key, 0.0) + float(r["Counter_Value"])
    for (d, c), v in sorted(by_disp.items()):
        out.setdefault(c, []).append(v)
    return out, name


def find(d, suffix):
    for root, _, files in os.walk(d):
        for f in files:
            if f.endswith(suffix):
                return os.path.join(root, f)
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("run")
    ap.add_argument("prefix")
    ap.add_argument("--warmup", type=int, default=1, help="untimed launches at the start of each PMC pass")
    ap.add_argument("--trace-timed", type=int, default=20, help="timed launches of the kernel-trace run: its last N "
                    "sr_sweep_kernel launches (bench.py --steps; the warm-up launches come first)")
    ap.add_argument("--tag", default="", help="directory prefix of another workload's passes in the same run "
                    "(e.g. c5_: c5_prof, c5_fetch, c5_write, c5_sq*)")
    ap.add_argument("--bench-json", default="", help="bench line of the workload (default <run>/bench.json)")
    args = ap.parse_args()
    t = args.tag
    D = {"prof": t + "prof" if t else "prof", "fetch": t + "fetch" if t else "pmc_fetch",
         "write": t + "write" if t else "pmc_write", "sq": t + "sq" if t else "pmc_sq"}

    res = {"kernel": None, "source": args.run,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over bench.py; "
                     "KiB -> bytes; FETCH_SIZE doubled (gfx950 correction, MI355X_MICROARCH.md HBM); "
                     "traffic = 2*FETCH + WRITE per sr_sweep_kernel launch, warm-up launches dropped"}
    stats = find(os.path.join(args.run, D["prof"]), "kernel_stats.csv")
    if stats:
        shutil.copy(stats, args.prefix + "_kernel_stats.csv")
    trace = find(os.path.join(args.run, D["prof"]), "kernel_trace.csv")
    if trace:
        durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(trace))
                if KERNEL in r["Kernel_Name"]]
        timed = durs[-args.trace_timed:]
        res["trace"] = {"launches": len(durs), "timed_launches": len(timed),
                        "avg_ns_timed": statistics.mean(timed) if timed else None,
                        "min_ns_timed": min(timed) if timed else None, "max_ns_timed": max(timed) if timed else None,
                        "avg_ns_all": statistics.mean(durs) if durs else None}
        # the bench line printed by the profiled run itself (same command as the bench)
        plog = os.path.join(args.run, D["prof"] + ".log")
        if os.path.exists(plog):
            for ln in open(plog):
                if ln.startswith("{") and '"metric"' in ln:
                    b = json.loads(ln)
                    res["trace"]["profiled_run_bench"] = {"value": b["value"], "ms_per_step": b["ms_per_step"],
                                                          "kernel_ms_hip_events": b["roofline"]["kernel_ms"]}
        if timed:
            with open(args.prefix + "_kernel_stats_timed.csv", "w") as fh:
                fh.write('"Name","Calls","AverageNs","MinNs","MaxNs","StdDev","Note"\n')
                fh.write('"%s",%d,%.1f,%d,%d,%.1f,"the %d timed launches of the profiled bench run (warm-up dropped)"\n'
                         % (KERNEL, len(timed), statistics.mean(timed), min(timed), max(timed),
                            statistics.pstdev(timed), len(timed)))
    fetch = find(os.path.join(args.run, D["fetch"]), "counter_collection.csv")
    write = find(os.path.join(args.run, D["write"]), "counter_collection.csv")
    if fetch and write:
        f, name = per_dispatch(fetch)
        w, _ = per_dispatch(write)
        fk = f["FETCH_SIZE"][args.warmup:]
        wk = w["WRITE_SIZE"][args.warmup:]
        res["kernel"] = name
        fb = statistics.mean(fk) * 1024.0
        wb = statistics.mean(wk) * 1024.0
        res["fetch_bytes_raw"] = fb
        res["fetch_bytes"] = 2.0 * fb
        res["write_bytes"] = wb
        res["traffic_bytes_per_launch"] = 2.0 * fb + wb
        res["launches"] = len(fk)
    # every SQ pass (<sq>, <sq>_b, <sq>_c ...: one --pmc run each), merged per counter
    sqd = {}
    for d in sorted(os.listdir(args.run)):
        if d.startswith(D["sq"]) and os.path.isdir(os.path.join(args.run, d)):
            f = find(os.path.join(args.run, d), "counter_collection.csv")
            if f:
                sv, _ = per_dispatch(f)
                for k, v in sv.items():
                    sqd.setdefault(k, statistics.mean(v[args.warmup:]))
    if sqd:
        res["sq"] = sqd
        q = sqd
        if q.get("SQ_INSTS_LDS"):
            q["lds_bank_conflict_cycles_per_lds_inst"] = q.get("SQ_LDS_BANK_CONFLICT", 0.0) / q["SQ_INSTS_LDS"]
        wc = q.get("SQ_WAVE_CYCLES")
        if wc:   # quad-cycle counters over the waves' lifetime (MI355X_MICROARCH.md, rocprofv3 PMC slots)
            res["limiter"] = {k: q[c] / wc for k, c in (("issue_frac", "SQ_ACTIVE_INST_ANY"),
                                                         ("valu_issue_frac", "SQ_ACTIVE_INST_VALU"),
                                                         ("salu_issue_frac", "SQ_ACTIVE_INST_SCA"),
                                                         ("lds_issue_frac", "SQ_ACTIVE_INST_LDS"),
                                                         ("issue_stall_frac", "SQ_WAIT_INST_ANY"),
                                                         ("parked_frac", "SQ_WAIT_ANY")) if c in q}
            if "lds_bank_conflict_cycles_per_lds_inst" in q:
                res["limiter"]["lds_bank_conflict_cycles_per_lds_inst"] = q["lds_bank_conflict_cycles_per_lds_inst"]
            res["limiter"]["definition"] = ("fractions of SQ_WAVE_CYCLES (per-wave lifetime, quad-cycles): issue = "
                                            "SQ_ACTIVE_INST_ANY, parked = SQ_WAIT_ANY (s_waitcnt / barrier), issue "
                                            "stall = SQ_WAIT_INST_ANY; a wave issues at most one instruction per "
                                            "quad-cycle")
    bench = args.bench_json or os.path.join(args.run, "bench.json")
    if os.path.exists(bench):
        try:
            b = json.loads(open(bench).read().strip().splitlines()[-1])
            res["workload"] = {k: b["config"][k] for k in ("sites", "taxa", "chains_per_gpu", "sweeps_per_step")}
        except Exception:
            pass
    with open(args.prefix + "_traffic.json", "w") as fh:
        json.dump(res, fh, indent=1)
    json.dump(res, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
