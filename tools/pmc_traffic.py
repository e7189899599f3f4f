#!/usr/bin/env python3
"""HBM traffic per launch of one kernel from rocprofv3 --pmc CSVs (one counter per pass).

usage: pmc_traffic.py --kernel render_kernel<false --fetch DIR_OR_CSV --write DIR_OR_CSV -o out.json

Correction (/opt/skills/guides/MI355X_MICROARCH.md, "HBM"): FETCH_SIZE (KB) counts the
L2's memory-side read requests at 64 B while gfx950 issues 128-B requests, so it reads
half the bytes -> doubled here.  WRITE_SIZE (KB) is taken as is.  Both include
Infinity-Cache (MALL) hits, so this is an upper bound on DRAM bytes.
"""
import argparse, csv, glob, json, os, statistics


def _rows(path):
    files = [path] if os.path.isfile(path) else glob.glob(os.path.join(path, "**", "*counter_collection.csv"),
                                                         recursive=True)
    for f in files:
        yield from csv.DictReader(open(f))


def per_launch(path, counter, kernel):
    vals = {}
    for r in _rows(path):
        if r["Counter_Name"] != counter or kernel not in r["Kernel_Name"]:
            continue
        key = r.get("Dispatch_Id") or r.get("Correlation_Id") or str(len(vals))
        vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])   # summed over XCD/dims
    if not vals:
        raise SystemExit(f"no {counter} rows for kernel matching {kernel!r} in {path}")
    return statistics.median(vals.values()), len(vals)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("-o", "--out", required=True)
    a = ap.parse_args()
    f_kb, nf = per_launch(a.fetch, "FETCH_SIZE", a.kernel)
    w_kb, nw = per_launch(a.write, "WRITE_SIZE", a.kernel)
    fetch = f_kb * 1024 * 2
    write = w_kb * 1024
    res = {"kernel": a.kernel, "launches": [nf, nw], "fetch_size_kb_raw": f_kb, "write_size_kb_raw": w_kb,
           "fetch_bytes_corrected": fetch, "write_bytes": write, "hbm_bytes_per_launch": int(fetch + write),
           "correction": "FETCH_SIZE x2 (gfx950 64-B tally of 128-B requests); MALL hits included"}
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
