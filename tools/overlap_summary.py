#!/usr/bin/env python3
"""Kernel concurrency of bench.py's pipelined loop, from a rocprofv3 --kernel-trace CSV.

usage: overlap_summary.py --trace DIR --kernel 'render_kernel<false, false, 1, false>'
                          --skip W --frames K [--bench gpurun_out/x.json] -o profiles/overlap_c3.json

bench.py validates its Q = 16 framebuffers with one frame each (engine.frame_pipeline),
submits W warmup frames, then K timed frames, then single frames for kernel_ms: --skip Q + W.
The render dispatches are taken in dispatch (= submission) order and the K timed ones
are [Q+W, Q+W+K).  Over those:
  span_per_frame_ms   (last end - first start) / K
  union_per_frame_ms  length of the union of the launches' [start, end) intervals / K:
                      time the GPU had at least one render launch running, per frame
  concurrency         sum of launch durations / union length (mean launches running at once)
  max_overlap         most launches running at the same instant
  time_at_overlap     fraction of the union spent with exactly n launches running
  mean_launch_ms      average launch duration in the pipelined loop (each launch's own
                      interval stretches when it shares the GPU with its neighbours)
Frame chains (--extra-kernel, repeatable: C5's compacted bounce render, whose frame is the queued
primary pass plus per-level k_qcount / k_qscan / k_bounce launches): the window runs from the first
timed primary dispatch's start to the start of the first primary dispatch after the timed ones,
and every dispatch of the extra kernels starting inside it joins the union (the frames in flight
at either edge make this approximate to about one frame in `frames`).
With --bench the same run's bench line is read for ms_per_step (value's clock) and the
union per frame is compared with it (reference: RayTracer.swift:166,197-203 time the
whole render).
"""
import argparse
import csv
import glob
import json
import os
import statistics


def rows(trace):
    files = [trace] if os.path.isfile(trace) else glob.glob(os.path.join(trace, "**", "*kernel_trace.csv"),
                                                              recursive=True)
    if not files:
        raise SystemExit(f"no *kernel_trace.csv under {trace}")
    out = []
    for f in files:
        out.extend(csv.DictReader(open(f)))
    return out


def summarize(trace_rows, kernel, skip, frames, extra_kernels=()):
    rk = [r for r in trace_rows if kernel in r["Kernel_Name"]]
    rk.sort(key=lambda r: int(r["Dispatch_Id"]))
    if len(rk) < skip + frames:
        raise SystemExit(f"{len(rk)} dispatches of {kernel!r}, need {skip + frames}")
    sel = rk[skip:skip + frames]
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in sel)
    t0, t1 = iv[0][0], max(e for _, e in iv)
    if extra_kernels:
        tend = int(rk[skip + frames]["Start_Timestamp"]) if len(rk) > skip + frames else None
        for r in trace_rows:
            if any(k in r["Kernel_Name"] for k in extra_kernels) and kernel not in r["Kernel_Name"]:
                s_, e_ = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
                if s_ >= t0 and (tend is None or s_ < tend):
                    iv.append((s_, e_))
        iv.sort()
        t1 = max(e for _, e in iv)
    # sweep: +1 at a start, -1 at an end (ends first at equal times: [start, end) intervals)
    ev = sorted([(s, 1) for s, _ in iv] + [(e, -1) for _, e in iv], key=lambda x: (x[0], x[1]))
    cur, last, union, peak = 0, t0, 0, 0
    at = {}
    for t, dlt in ev:
        if cur > 0:
            union += t - last
            at[cur] = at.get(cur, 0) + (t - last)
        cur += dlt
        peak = max(peak, cur)
        last = t
    durs = [e - s for s, e in iv]
    res = {
        "kernel": kernel, "extra_kernels": list(extra_kernels), "frames": frames, "skipped": skip, "dispatches_seen": len(rk),
        "span_per_frame_ms": round((t1 - t0) / frames / 1e6, 5),
        "union_per_frame_ms": round(union / frames / 1e6, 5),
        "concurrency": round(sum(durs) / union, 3),
        "max_overlap": peak,
        "mean_launch_ms": round(statistics.mean(durs) / 1e6, 5),
        "median_launch_ms": round(statistics.median(durs) / 1e6, 5),
        "time_at_overlap": {str(k): round(v / union, 4) for k, v in sorted(at.items())},
        "idle_fraction_of_span": round(1.0 - union / (t1 - t0), 5),
    }
    # other kernels inside the same window (counter delivery, bounce levels ...)
    others = {}
    for r in trace_rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s >= t0 and e <= t1 and kernel not in r["Kernel_Name"] and not any(k in r["Kernel_Name"] for k in extra_kernels):
            k = r["Kernel_Name"]
            o = others.setdefault(k, [0, 0])
            o[0] += 1
            o[1] += e - s
    res["other_kernels_in_window"] = {k: {"calls": c, "total_ms": round(d / 1e6, 4)} for k, (c, d) in others.items()}
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--extra-kernel", action="append", default=[], help="other kernels of a frame chain")
    ap.add_argument("--skip", type=int, required=True)
    ap.add_argument("--frames", type=int, required=True)
    ap.add_argument("--bench", default=None, help="the same run's bench JSON line (file)")
    ap.add_argument("--lib", default=None, help="the libmyrt.so the trace measured (its sha256 prefix is recorded)")
    ap.add_argument("-o", "--out", required=True)
    a = ap.parse_args()
    res = summarize(rows(a.trace), a.kernel, a.skip, a.frames, tuple(a.extra_kernel))
    if a.lib:
        import hashlib
        with open(a.lib, "rb") as fh:
            res["lib_sha256_16"] = hashlib.sha256(fh.read()).hexdigest()[:16]
    if a.bench and os.path.exists(a.bench):
        line = None
        for ln in open(a.bench):
            ln = ln.strip()
            if ln.startswith("{"):
                line = json.loads(ln)
        if line:
            res["bench_ms_per_step"] = line["ms_per_step"]
            res["bench_value"] = line["value"]
            res["union_vs_ms_per_step"] = round(res["union_per_frame_ms"] / line["ms_per_step"], 4)
    res["what"] = ("bench.py's timed loop under rocprofv3 --kernel-trace: render launches [skip, skip+frames) in "
                   "dispatch order; union = time with at least one render launch running")
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
