"""Summarize a tools/profile_round.sh output directory into profiles/ (committed evidence).

Usage: summarize_profile.py OUTDIR ROUND CONFIG MODE [COMMITTED_LINE_JSON [UNPROFILED_LINE_JSON]]

Writes:
  profiles/<round>_<config>_<mode>_kernel_stats.csv   (rocprofv3 --stats table, verbatim)
  profiles/<round>_<config>_<mode>_summary.json       (per-kernel avg duration, HBM bytes per launch)
  profiles/traffic_<config>_<mode>.json               (read by bench.py for roofline.traffic)
"""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def find(d, pattern):
    hits = glob.glob(os.path.join(d, "**", pattern), recursive=True)
    return hits[0] if hits else None


def counters(d, name):
    f = find(d, "*counter_collection.csv")
    per = {}
    if not f:
        return per
    for row in csv.DictReader(open(f)):
        if row.get("Counter_Name") != name:
            continue
        k = row["Kernel_Name"].split("(")[0]
        per.setdefault(k, []).append(float(row["Counter_Value"]))
    return per


def stream_kernel(kernels):
    """(name, stats) of the step's byte-streaming kernel: the k_windows* launch, or the table scan's k_ts_windows (its
    window pass with the index walk beside it): every algorithmic byte passes through it once; a config without one
    (the Snappy frames) falls back to the kernel with the most time."""
    win = [kv for kv in kernels.items() if kv[0].split("::")[-1].split("<")[0] in ("k_windows", "k_windows_q",
                                                                                   "k_ts_windows")]
    if win:
        return max(win, key=lambda kv: kv[1]["total_ns"])
    return max(kernels.items(), key=lambda kv: kv[1]["total_ns"])


def main(outdir, rnd, config, mode, committed=None, unprofiled=None):
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    tag = f"{rnd}_{config}_{mode}"
    stats = find(os.path.join(outdir, "trace"), "*kernel_stats.csv")
    summary = {"round": rnd, "config": config, "mode": mode, "kernels": {}}
    if stats:
        shutil.copy(stats, os.path.join(prof, f"{tag}_kernel_stats.csv"))
        for row in csv.DictReader(open(stats)):
            name = row["Name"].split("(")[0]
            summary["kernels"][name] = {"calls": int(row["Calls"]), "avg_ns": float(row["AverageNs"]),
                                        "total_ns": float(row["TotalDurationNs"]),
                                        "percent": float(row.get("Percentage", 0) or 0)}
    fetch = counters(os.path.join(outdir, "fetch"), "FETCH_SIZE")
    write = counters(os.path.join(outdir, "write"), "WRITE_SIZE")
    traffic = {}
    for k, vals in fetch.items():
        # FETCH_SIZE is in KiB; gfx950 tallies 128-B streaming requests at 64 B -> x2 (MI355X_MICROARCH.md)
        rd = sum(vals) / len(vals) * 1024 * 2
        wr = (sum(write.get(k, [0])) / max(1, len(write.get(k, [0])))) * 1024
        traffic[k] = {"hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
                      "fetch_size_kib_raw": sum(vals) / len(vals), "launches_sampled": len(vals)}
    summary["traffic"] = traffic
    # the roofline fraction this profile implies: the bench line of the SAME command (--extra-out) gives the
    # algorithmic bytes per launch; the dominant kernel's average duration comes from the kernel trace
    bj = os.path.join(outdir, "bench.json")
    if summary["kernels"] and os.path.exists(bj):
        with open(bj) as f:
            line = json.load(f)
        dom = stream_kernel(summary["kernels"])
        bpl = (line.get("roofline") or {}).get("bytes_per_launch")
        if bpl:
            # `kernel` / `frac`: the byte-streaming kernel of the step (k_windows*: every algorithmic byte goes through
            # it once), never merely the kernel with the most time (round 4 charged a WAL step's bytes to k_wal_parse)
            summary["kernel"] = dom[0]
            summary["dominant_by_time"] = max(summary["kernels"].items(), key=lambda kv: kv[1]["total_ns"])[0]
            summary["avg_us"] = round(dom[1]["avg_ns"] / 1e3, 3)
            summary["bytes_per_launch"] = bpl
            summary["frac"] = round(bpl / dom[1]["avg_ns"] / 8000.0, 4)
            summary["bound"] = (line.get("roofline") or {}).get("bound")
            # every kernel of the pipeline per streaming-kernel call (general path: k_windows + k_blocks, WAL:
            # parse + emit + windows + blocks), for configs whose step is more than one kernel, and the fraction of
            # 8 TB/s the whole pipeline's kernel time implies
            summary["pipeline_us_per_call"] = round(
                sum(k["total_ns"] for k in summary["kernels"].values()) / dom[1]["calls"] / 1e3, 3)
            summary["frac_pipeline"] = round(bpl / (summary["pipeline_us_per_call"] * 1e3) / 8000.0, 4)
            summary["bench_line"] = {"value": line["value"], "ms_per_step": line["ms_per_step"],
                                     "frac": line["roofline"]["frac"], "launch_us": line["roofline"]["launch_us"],
                                     "launches": line["roofline"].get("launches"),
                                     "streams": line["config"].get("streams")}
            # the bench line's quantity, recomputed from the kernel trace of the same run: its HIP events span
            # the timed region's launches (kernel-carried events: the first one's start to the last one's end;
            # otherwise from the end of the first launch to the end of the last), dispatch gaps included
            nl = line["roofline"].get("launches") or 0
            trace = find(os.path.join(outdir, "trace"), "*kernel_trace.csv")
            kps = line["config"].get("kernels_per_step") or 0
            steps = line.get("steps") or 0
            if trace and nl:
                rows = list(csv.DictReader(open(trace)))
                ts = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows
                            if r["Kernel_Name"].split("(")[0] == dom[0])
                clock = line["roofline"].get("clock")
                kernel_events = clock in ("carried", "start") if clock else \
                    "carried by the launches" in line["roofline"].get("timing", "")
                span = None
                if kps > 1 and steps > 1:
                    # a step is kps dependent kernels. The timed steps are the last steps * kps dispatches in host
                    # submission order (Dispatch_Id), the first step's kernels the first kps of them. Kernel-carried
                    # events: the first timed launch's start to the last end, / steps; marker events: the end of the
                    # first step to the last end (every stream joined), / (steps - 1).
                    order = sorted(rows, key=lambda r: int(r["Dispatch_Id"]))
                    timed = order[-steps * kps:]
                    names = [r["Kernel_Name"].split("(")[0] for r in timed]
                    if len(timed) == steps * kps and names.count(dom[0]) == steps:
                        t_last = max(int(r["End_Timestamp"]) for r in timed)
                        if kernel_events:
                            span = (t_last - int(timed[0]["Start_Timestamp"])) / 1e3 / steps
                        else:
                            span = (t_last - max(int(r["End_Timestamp"]) for r in timed[:kps])) / 1e3 / (steps - 1)
                        summary["timed_kernels"] = {n: names.count(n) for n in sorted(set(names))}
                elif kernel_events and len(ts) >= nl:  # first launch's start to the latest end (several streams)
                    span = (max(e for _, e in ts[-nl:]) - ts[-nl][0]) / 1e3 / nl
                elif len(ts) > nl:
                    timed = ts[-(nl + 1):]
                    span = (timed[-1][1] - timed[0][1]) / 1e3 / nl
                if span:
                    summary["trace_launch_us"] = round(span, 3)
                    summary["trace_gap_us"] = round(span - summary["avg_us"], 3)
                    summary["frac_from_trace"] = round(bpl / (span * 1e3) / 8000.0, 4)
                    summary["kernels_per_step"] = kps or 1
                    # against the profiled run's own line (the same process the trace comes from)
                    summary["agreement_profiled_run"] = round(summary["frac_from_trace"] / line["roofline"]["frac"], 4)
            # against the COMMITTED line (the line DESIGN.md quotes; tools/gpu_round.sh commits the profiled run's own
            # line) and, when given, an un-profiled run of the same command taken right after
            for key, path in (("", committed), ("_unprofiled", unprofiled)):
                if not (path and os.path.exists(path) and "trace_launch_us" in summary):
                    continue
                with open(path) as f:
                    cl = json.load(f)
                cr = cl.get("roofline") or {}
                summary["committed_line" if not key else "unprofiled_line"] = {
                    "file": os.path.relpath(path, ROOT), "value": cl["value"], "ms_per_step": cl["ms_per_step"],
                    "launch_us": cr.get("launch_us"), "frac": cr.get("frac")}
                if cr.get("launch_us"):
                    summary["agreement" + key] = round(cr["launch_us"] / summary["trace_launch_us"], 4)
                summary["agreement_wall" + key] = round(cl["ms_per_step"] * 1e3 / summary["trace_launch_us"], 4)
            summary["note"] = ("frac: the dominant kernel's average duration alone (rocprofv3 kernel trace); "
                               "frac_from_trace: the bench line's measure (its timed launches, first to last, per "
                               "launch) on the same trace -- the difference is the dispatch gap between two in-order "
                               "launches. agreement = the committed line's GPU time per launch / the trace's "
                               "(1.0: the trace reproduces the committed line); agreement_wall = its wall time per step / "
                               "the trace's; *_unprofiled: the same against an un-profiled run of the command; "
                               "agreement_profiled_run = frac_from_trace / the profiled run's own line frac")
    with open(os.path.join(prof, f"{tag}_summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    # the streaming kernel's traffic for bench.py, and the whole step's (every kernel's bytes per step)
    dom = stream_kernel(summary["kernels"])[0] if summary["kernels"] else None
    hot = None
    for k in traffic:
        if dom and dom.split("<")[0] in k:
            hot = k
    if hot is None and traffic:
        hot = max(traffic, key=lambda k: traffic[k]["hbm_read_bytes_per_launch"])
    if hot:
        t = traffic[hot]
        calls = {k: v["calls"] for k, v in summary["kernels"].items()}
        per_step = calls.get(dom) or 1
        # every kernel's bytes per step: a kernel's average per launch x its launches per streaming-kernel launch
        # (kernels named in the trace with at least half as many launches; the one-off launches of the set-up, e.g.
        # the WAL bench's seal, are not steps)
        stepk = {k: v for k, v in traffic.items() if k in calls and 2 * calls[k] >= per_step}
        step_rd = sum(v["hbm_read_bytes_per_launch"] * calls[k] / per_step for k, v in stepk.items())
        step_wr = sum(v["hbm_write_bytes_per_launch"] * calls[k] / per_step for k, v in stepk.items())
        bpl = summary.get("bytes_per_launch")
        summary["step_traffic"] = {
            "read_bytes": step_rd, "write_bytes": step_wr, "kernels": sorted(stepk),
            "read_x": round(step_rd / bpl, 4) if bpl else None, "write_x": round(step_wr / bpl, 4) if bpl else None,
            "stream_kernel": hot, "stream_kernel_read_x": round(t["hbm_read_bytes_per_launch"] / bpl, 4) if bpl else None,
            "note": "HBM bytes per step over every kernel of the step (FETCH_SIZE x1024 x2, WRITE_SIZE x1024), and "
                    "their ratio to the algorithmic bytes of one step (bytes_per_launch)"}
        with open(os.path.join(prof, f"{tag}_summary.json"), "w") as f:
            json.dump(summary, f, indent=1)
        with open(os.path.join(prof, f"traffic_{config}_{mode}.json"), "w") as f:
            json.dump({"kernel": hot, "hbm_bytes_per_launch": t["hbm_read_bytes_per_launch"] + t["hbm_write_bytes_per_launch"],
                       "hbm_read_bytes_per_launch": t["hbm_read_bytes_per_launch"],
                       "hbm_write_bytes_per_launch": t["hbm_write_bytes_per_launch"],
                       "step_hbm_read_bytes": step_rd, "step_hbm_write_bytes": step_wr,
                       "source": f"profiles/{tag}_summary.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes; "
                                 "FETCH_SIZE KiB x1024 x2 per the gfx950 correction)"}, f, indent=1)
    if summary.get("bench_line", {}).get("streams", 1) > 1 and "kernel" in summary:
        summary["overlap_note"] = ("launches rotate over several streams and run concurrently (two workgroups per CU, "
                                   "one of each launch): a launch's own duration (avg_us, frac) spans its overlap with "
                                   "its neighbours; the rate of the stream of launches is trace_launch_us")
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:7])
