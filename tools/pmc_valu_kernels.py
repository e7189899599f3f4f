#!/usr/bin/env python3
"""Per-kernel VALU figures from ONE rocprofv3 --pmc pass (the `_valu` pass of
tools/final_session.sh / prof_session.sh), for frames that run several kernels (the full
trace() passes of C3g / C3r: k_level, k_shade, render_full, ...).

usage: tools/pmc_valu_kernels.py gpurun_out/TAG_c3g_valu [-o profiles/TAG_c3g_valu.txt]

Per kernel (median over its dispatches): VALU busy = SQ_ACTIVE_INST_VALU / 256 CUs /
(GRBM_GUI_ACTIVE / 8 XCDs), lane utilisation = SQ_THREAD_CYCLES_VALU / (64 *
SQ_ACTIVE_INST_VALU), their product, and VALU instructions per dispatch (same definitions as
tools/pmc_roofline.py --valu).
"""
import collections
import csv
import glob
import os
import statistics
import sys


def main():
    path = sys.argv[1]
    out = sys.argv[sys.argv.index("-o") + 1] if "-o" in sys.argv else None
    files = [path] if os.path.isfile(path) else glob.glob(os.path.join(path, "**", "*counter_collection.csv"),
                                                           recursive=True)
    per = collections.defaultdict(lambda: collections.defaultdict(float))   # (kernel, dispatch) -> counter
    for f in files:
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("myrt::dev::", "")
            if "rocclr" in k or "__amd" in k:
                continue
            d = r.get("Dispatch_Id") or r.get("Correlation_Id")
            per[(k, d)][r["Counter_Name"]] += float(r["Counter_Value"])
    rows = collections.defaultdict(list)
    for (k, _), c in per.items():
        if c.get("SQ_ACTIVE_INST_VALU", 0) <= 0 or c.get("GRBM_GUI_ACTIVE", 0) <= 0:
            continue
        busy = c["SQ_ACTIVE_INST_VALU"] / 256 / (c["GRBM_GUI_ACTIVE"] / 8)
        util = c["SQ_THREAD_CYCLES_VALU"] / (64 * c["SQ_ACTIVE_INST_VALU"])
        rows[k].append((busy, util, busy * util, c.get("SQ_INSTS_VALU", 0.0), c["GRBM_GUI_ACTIVE"] / 8))
    lines = ["%-44s %6s %9s %9s %9s %14s %12s" % ("kernel", "disp", "valu_busy", "lane_util", "product",
                                                 "valu_insts", "gui_cycles")]
    for k, v in sorted(rows.items(), key=lambda kv: -sum(x[4] for x in kv[1])):
        med = [statistics.median(x[i] for x in v) for i in range(5)]
        lines.append("%-44s %6d %9.3f %9.3f %9.3f %14.0f %12.0f" % (k[:44], len(v), *med))
    text = "\n".join(lines) + "\n"
    sys.stdout.write(text)
    if out:
        open(out, "w").write(text)


if __name__ == "__main__":
    main()
