#!/usr/bin/env python3
"""Roofline summary of the render megakernel from rocprofv3 passes (one counter group per pass).

usage: pmc_roofline.py --kernel 'render_kernel<false, false, 1, false>' --trace DIR --fetch DIR --write DIR
                       --td DIR --valu DIR [--sq DIR] --lib myraytracer_amd/libmyrt.so -o profiles/roofline_c3.json

Per launch (median over the dispatches of that kernel):
  hbm_bytes_per_launch = FETCH_SIZE x 2 + WRITE_SIZE (KB -> B).  /opt/skills/guides/MI355X_MICROARCH.md,
      "HBM": on gfx950 FETCH_SIZE tallies 128-B requests at 64 B, so it reads half the bytes; both
      counters include Infinity-Cache (MALL) hits, so this is an upper bound on DRAM bytes.
  td_busy  = (TD_TD_BUSY_sum / 256 CUs) / (GRBM_GUI_ACTIVE / 8 XCDs): texture-data (vector-memory
      return) path utilisation - the resource that binds this kernel.
  ta_busy  = TA_BUSY_avr / (GRBM_GUI_ACTIVE / 8).
  The compute roofline, every figure from ONE pass (--valu: GRBM_GUI_ACTIVE, SQ_ACTIVE_INST_VALU,
  SQ_THREAD_CYCLES_VALU, SQ_INSTS_VALU, ... of the same dispatches):
  valu_busy = SQ_ACTIVE_INST_VALU / 256 CUs / (GRBM_GUI_ACTIVE / 8)  (rocprofiler-sdk's VALUBusy),
  valu_lane_util = SQ_THREAD_CYCLES_VALU / (64 x SQ_ACTIVE_INST_VALU),
  lane_throughput_frac = valu_busy x valu_lane_util: the fraction of the VALU lane-cycles the
      kernel's arithmetic used (1.0 = every SIMD issuing full-width every cycle).
  kernel_ms = average duration from the --kernel-trace --stats pass.
lib_sha256_16 ties the summary to the library build it measured (bench.py checks it).

Frame chains (--kernel given more than once; the first names the frame's first kernel): a frame
that runs several launches (C5's compacted bounce render: the queued primary pass, then per level
k_bounce, then k_queue_done; round 5: k_qcount / k_qscan per level too) is summarised per FRAME: frames = dispatches of
the first kernel; every counter is summed over all dispatches of the listed kernels and divided by
the frames; kernel_ms = the listed kernels' total duration per frame; busy / utilisation ratios
divide the chain's summed counters.  `chain` lists each kernel's share.
"""
import argparse
import csv
import glob
import hashlib
import json
import os
import statistics


def _files(path, pattern):
    if os.path.isfile(path):
        return [path]
    return glob.glob(os.path.join(path, "**", pattern), recursive=True)


def counter(path, name, kernel):
    vals = {}
    for f in _files(path, "*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != name or kernel not in r["Kernel_Name"]:
                continue
            key = r.get("Dispatch_Id") or r.get("Correlation_Id") or str(len(vals))
            vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    if not vals:
        raise SystemExit(f"no {name} rows for kernel {kernel!r} under {path}")
    return statistics.median(vals.values()), len(vals)


def counter_total(path, name, kernel):
    """Sum of a counter over every dispatch of `kernel` and the number of dispatches."""
    vals = {}
    for f in _files(path, "*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != name or kernel not in r["Kernel_Name"]:
                continue
            key = r.get("Dispatch_Id") or r.get("Correlation_Id") or str(len(vals))
            vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    if not vals:
        raise SystemExit(f"no {name} rows for kernel {kernel!r} under {path}")
    return sum(vals.values()), len(vals)


def kernel_total_ms(path, kernel):
    for f in _files(path, "*kernel_stats.csv"):
        for r in csv.DictReader(open(f)):
            if kernel in r["Name"]:
                return float(r["TotalDurationNs"]) / 1e6, int(r["Calls"])
    raise SystemExit(f"kernel {kernel!r} not in the kernel stats under {path}")


def chain(a):
    """Per-frame figures of a multi-kernel frame (see the module docstring)."""
    def present(k):
        try:
            kernel_total_ms(a.trace, k)
            return True
        except SystemExit:
            return False
    ks = [a.kernel[0]] + [k for k in a.kernel[1:] if present(k)]   # a config may skip some passes
    _, frames = kernel_total_ms(a.trace, ks[0])
    _, pmc_frames = counter_total(a.fetch, "FETCH_SIZE", ks[0])

    def per_frame(path, name, n):
        return sum(counter_total(path, name, k)[0] for k in ks) / n

    ms = sum(kernel_total_ms(a.trace, k)[0] for k in ks) / frames
    f_kb = per_frame(a.fetch, "FETCH_SIZE", pmc_frames)
    w_kb = per_frame(a.write, "WRITE_SIZE", pmc_frames)
    gui = per_frame(a.td, "GRBM_GUI_ACTIVE", pmc_frames)
    td = per_frame(a.td, "TD_TD_BUSY_sum", pmc_frames)
    ta = per_frame(a.td, "TA_BUSY_avr", pmc_frames)
    res = {"kernel": " + ".join(ks), "frame_chain": True, "kernel_ms": round(ms, 4), "trace_frames": frames,
           "pmc_frames": pmc_frames, "fetch_size_kb_raw": f_kb, "write_size_kb_raw": w_kb,
           "fetch_bytes_corrected": f_kb * 1024 * 2, "write_bytes": w_kb * 1024,
           "hbm_bytes_per_launch": int(f_kb * 1024 * 2 + w_kb * 1024),
           "hbm_GBs": round((f_kb * 2048 + w_kb * 1024) / (ms * 1e-3) / 1e9, 1),
           "td_busy": round((td / 256) / (gui / 8), 4),
           "correction": "FETCH_SIZE x2 (gfx950 64-B tally of 128-B requests); MALL hits included; "
                         "per frame = sums over the chain's dispatches / frames",
           "chain": {k: {"ms_per_frame": round(kernel_total_ms(a.trace, k)[0] / frames, 4),
                         "calls_per_frame": kernel_total_ms(a.trace, k)[1] / frames,
                         "write_kb_per_frame": round(counter_total(a.write, "WRITE_SIZE", k)[0] / pmc_frames, 1)}
                     for k in ks}}
    res["ta_busy"] = round(ta / (gui / 8), 4)
    if a.valu:
        _, vframes = counter_total(a.valu, "GRBM_GUI_ACTIVE", ks[0])
        vgui = per_frame(a.valu, "GRBM_GUI_ACTIVE", vframes)
        thr = per_frame(a.valu, "SQ_THREAD_CYCLES_VALU", vframes)
        act = per_frame(a.valu, "SQ_ACTIVE_INST_VALU", vframes)
        ins = per_frame(a.valu, "SQ_INSTS_VALU", vframes)
        res["valu_lane_util"] = round(thr / (64 * act), 4)
        res["valu_busy"] = round(act / 256 / (vgui / 8), 4)
        res["lane_throughput_frac"] = round(res["valu_busy"] * res["valu_lane_util"], 4)
        res["valu_insts_per_launch"] = int(ins)
        res["valu_pass"] = {"GRBM_GUI_ACTIVE": vgui, "SQ_ACTIVE_INST_VALU": act, "SQ_THREAD_CYCLES_VALU": thr,
                            "SQ_INSTS_VALU": ins,
                            "note": "one rocprofv3 --pmc pass; per frame = sums over the chain's dispatches"}
    return res


def kernel_ms(path, kernel):
    for f in _files(path, "*kernel_stats.csv"):
        for r in csv.DictReader(open(f)):
            if kernel in r["Name"]:
                return float(r["AverageNs"]) / 1e6, int(r["Calls"])
    raise SystemExit(f"kernel {kernel!r} not in the kernel stats under {path}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", required=True, action="append",
                    help="the kernel; repeat for a frame chain (first = the frame's first launch)")
    ap.add_argument("--trace", required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--td", required=True)
    ap.add_argument("--valu", help="one pass holding GRBM_GUI_ACTIVE + SQ_ACTIVE_INST_VALU + SQ_THREAD_CYCLES_VALU")
    ap.add_argument("--sq")
    ap.add_argument("--lib", required=True)
    ap.add_argument("-o", "--out", required=True)
    a = ap.parse_args()
    if len(a.kernel) > 1:
        res = chain(a)
        with open(a.lib, "rb") as fh:
            res["lib_sha256_16"] = hashlib.sha256(fh.read()).hexdigest()[:16]
        with open(a.out, "w") as fh:
            json.dump(res, fh, indent=1)
        print(json.dumps(res))
        return
    a.kernel = a.kernel[0]
    ms, calls = kernel_ms(a.trace, a.kernel)
    f_kb, nf = counter(a.fetch, "FETCH_SIZE", a.kernel)
    w_kb, nw = counter(a.write, "WRITE_SIZE", a.kernel)
    gui, _ = counter(a.td, "GRBM_GUI_ACTIVE", a.kernel)
    td, _ = counter(a.td, "TD_TD_BUSY_sum", a.kernel)
    ta, _ = counter(a.td, "TA_BUSY_avr", a.kernel)
    res = {"kernel": a.kernel, "kernel_ms": round(ms, 4), "trace_calls": calls, "pmc_launches": [nf, nw],
           "fetch_size_kb_raw": f_kb, "write_size_kb_raw": w_kb,
           "fetch_bytes_corrected": f_kb * 1024 * 2, "write_bytes": w_kb * 1024,
           "hbm_bytes_per_launch": int(f_kb * 1024 * 2 + w_kb * 1024),
           "hbm_GBs": round((f_kb * 2048 + w_kb * 1024) / (ms * 1e-3) / 1e9, 1),
           "td_busy": round((td / 256) / (gui / 8), 4), "ta_busy": round(ta / (gui / 8), 4),
           "correction": "FETCH_SIZE x2 (gfx950 64-B tally of 128-B requests); MALL hits included"}
    if a.valu:
        vgui, _ = counter(a.valu, "GRBM_GUI_ACTIVE", a.kernel)
        thr, _ = counter(a.valu, "SQ_THREAD_CYCLES_VALU", a.kernel)
        act, _ = counter(a.valu, "SQ_ACTIVE_INST_VALU", a.kernel)
        ins, _ = counter(a.valu, "SQ_INSTS_VALU", a.kernel)
        res["valu_lane_util"] = round(thr / (64 * act), 4)
        # VALUBusy (rocprofiler-sdk derived counter for gfx950): SQ_ACTIVE_INST_VALU counts
        # quad-cycles per CU summed over its 4 SIMDs -> fraction of cycles the SIMDs issue VALU
        res["valu_busy"] = round(act / 256 / (vgui / 8), 4)
        res["lane_throughput_frac"] = round(res["valu_busy"] * res["valu_lane_util"], 4)
        res["valu_insts_per_launch"] = int(ins)
        res["valu_pass"] = {"GRBM_GUI_ACTIVE": vgui, "SQ_ACTIVE_INST_VALU": act, "SQ_THREAD_CYCLES_VALU": thr,
                            "SQ_INSTS_VALU": ins,
                            "note": "one rocprofv3 --pmc pass: every compute-roofline figure divides counters "
                                    "of the same dispatches"}
    with open(a.lib, "rb") as fh:
        res["lib_sha256_16"] = hashlib.sha256(fh.read()).hexdigest()[:16]
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
