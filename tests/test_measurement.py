"""The measurement tooling behind bench.py's line (CPU only): the CPU-baseline core count read
from the cgroup quota, the kernel-overlap summary of a rocprofv3 kernel trace
(tools/overlap_summary.py, roofline.pipelined) and the PMC roofline summary
(tools/pmc_roofline.py: FETCH_SIZE x2 on gfx950, VALU busy / lane utilisation)."""
import csv
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import bench  # noqa: E402
import overlap_summary  # noqa: E402


@pytest.mark.parametrize("raw, cpus", [("1600000 100000", 16), ("150000 100000", 2), ("50000 100000", 1),
                                       ("max 100000", None)])
def test_cgroup_quota(tmp_path, raw, cpus):
    f = tmp_path / "cpu.max"
    f.write_text(raw + "\n")
    got, path, seen = bench.cgroup_cpu_quota(str(f))
    assert got == cpus and path == str(f) and seen == raw


def test_cgroup_quota_missing(tmp_path):
    assert bench.cgroup_cpu_quota(str(tmp_path / "absent"))[0] is None


def _trace_rows(spans, kernel="render_kernel<false, false, 1, false>"):
    rows = []
    for k, (s, e, name) in enumerate(spans):
        rows.append({"Kernel_Name": f"void myrt::dev::{name or kernel}(myrt::RenderParams)",
                     "Dispatch_Id": str(k + 1), "Start_Timestamp": str(s), "End_Timestamp": str(e)})
    return rows


def test_overlap_summary_union_and_concurrency():
    K = "render_kernel<false, false, 1, false>"
    spans = [(0, 1_000_000, None),                      # a validation frame: skipped
             (2_000_000, 12_000_000, None),             # timed frame 1
             (7_000_000, 17_000_000, None),             # timed frame 2, overlaps frame 1 by 5 ms
             (3_000_000, 4_000_000, "k_counters_out"),  # another kernel inside the window
             (20_000_000, 30_000_000, None),            # timed frame 3, after a 3 ms gap
             (40_000_000, 41_000_000, None)]            # a single frame after the timed ones
    res = overlap_summary.summarize(_trace_rows(spans), K, skip=1, frames=3)
    # union [2, 17) + [20, 30) = 25 ms over 3 frames; launches sum to 30 ms
    assert res["union_per_frame_ms"] == pytest.approx(25 / 3, rel=1e-6)
    assert res["span_per_frame_ms"] == pytest.approx(28 / 3, rel=1e-6)
    assert res["concurrency"] == pytest.approx(30 / 25, rel=1e-3)
    assert res["max_overlap"] == 2
    assert res["time_at_overlap"] == {"1": pytest.approx(20 / 25, abs=1e-4), "2": pytest.approx(5 / 25, abs=1e-4)}
    assert res["idle_fraction_of_span"] == pytest.approx(3 / 28, abs=1e-5)
    assert res["other_kernels_in_window"] == {"void myrt::dev::k_counters_out(myrt::RenderParams)":
                                              {"calls": 1, "total_ms": 1.0}}


def test_overlap_summary_frame_chain():
    """C5's frame chain: bounce-level launches inside the timed window join the union."""
    K = "render_kernel<false, false, 1, false>"
    spans = [(0, 1_000_000, None),                      # skipped
             (2_000_000, 6_000_000, None),              # timed frame 1: primary pass
             (6_000_000, 8_000_000, "k_bounce<1>"),     # its bounce level
             (9_000_000, 12_000_000, None),             # timed frame 2
             (12_000_000, 13_000_000, "k_bounce<1>"),
             (20_000_000, 21_000_000, None),            # a single frame after the timed ones
             (21_000_000, 22_000_000, "k_bounce<1>")]   # its level: outside the window
    res = overlap_summary.summarize(_trace_rows(spans, K), K, skip=1, frames=2, extra_kernels=("k_bounce<1>",))
    # union [2, 8) + [9, 13) = 10 ms over 2 frames
    assert res["union_per_frame_ms"] == pytest.approx(5.0, rel=1e-6)
    assert res["other_kernels_in_window"] == {}


def test_overlap_summary_needs_enough_dispatches():
    with pytest.raises(SystemExit):
        overlap_summary.summarize(_trace_rows([(0, 1, None)]), "render_kernel", skip=1, frames=1)


def _write_csv(path, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=list(rows[0]))
        w.writeheader()
        w.writerows(rows)


def test_pmc_roofline_summary(tmp_path):
    K = "render_kernel<false, false, 1, false>"
    name = f"void myrt::dev::{K}(myrt::RenderParams)"
    _write_csv(str(tmp_path / "trace/x/1_kernel_stats.csv"),
               [{"Name": name, "Calls": "45", "AverageNs": "750000.0"},
                {"Name": "k_counters_out", "Calls": "45", "AverageNs": "4000.0"}])

    def pmc(sub, counters):
        rows = []
        for d in (1, 2, 3):                              # three launches; the median is taken
            for c, v in counters.items():
                rows.append({"Dispatch_Id": str(d), "Kernel_Name": name, "Counter_Name": c,
                             "Counter_Value": str(v * (1.0 if d == 2 else (0.5 if d == 1 else 2.0)))})
        _write_csv(str(tmp_path / sub / "x/1_counter_collection.csv"), rows)
    pmc("fetch", {"FETCH_SIZE": 87000.0})
    pmc("write", {"WRITE_SIZE": 11000.0})
    pmc("td", {"GRBM_GUI_ACTIVE": 15_000_000.0, "TD_TD_BUSY_sum": 340_000_000.0, "TA_BUSY_avr": 700_000.0})
    # the compute roofline's own pass: its GRBM_GUI_ACTIVE (not the TD pass's) divides its SQ counters
    pmc("valu", {"GRBM_GUI_ACTIVE": 16_000_000.0, "SQ_ACTIVE_INST_VALU": 318_000_000.0,
                 "SQ_THREAD_CYCLES_VALU": 10_500_000_000.0, "SQ_INSTS_VALU": 300_000_000.0})
    pmc("sq", {"SQ_INSTS_SALU": 1.0})
    lib = tmp_path / "lib.so"
    lib.write_bytes(b"not a library")
    out = tmp_path / "roofline.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_roofline.py"), "--kernel", K,
                    "--trace", str(tmp_path / "trace"), "--fetch", str(tmp_path / "fetch"),
                    "--write", str(tmp_path / "write"), "--td", str(tmp_path / "td"), "--valu", str(tmp_path / "valu"),
                    "--sq", str(tmp_path / "sq"),
                    "--lib", str(lib), "-o", str(out)], check=True, capture_output=True)
    r = json.loads(out.read_text())
    assert r["kernel_ms"] == 0.75 and r["trace_calls"] == 45 and r["pmc_launches"] == [3, 3]
    # gfx950: FETCH_SIZE counts 128-B requests at 64 B -> x2; KB -> bytes
    assert r["hbm_bytes_per_launch"] == int(87000 * 1024 * 2 + 11000 * 1024)
    assert r["hbm_GBs"] == pytest.approx((87000 * 2048 + 11000 * 1024) / 0.75e-3 / 1e9, abs=0.1)
    assert r["td_busy"] == pytest.approx((340e6 / 256) / (15e6 / 8), abs=1e-4)
    assert r["valu_busy"] == pytest.approx(318e6 / 256 / (16e6 / 8), abs=1e-4)
    assert r["valu_lane_util"] == pytest.approx(10.5e9 / (64 * 318e6), abs=1e-4)
    assert r["lane_throughput_frac"] == pytest.approx(r["valu_busy"] * r["valu_lane_util"], abs=1e-4)
    assert r["valu_insts_per_launch"] == 300_000_000
    assert len(r["lib_sha256_16"]) == 16


def test_pmc_roofline_frame_chain(tmp_path):
    """A frame of several launches (C5's compacted bounce render): per-frame sums over the chain."""
    K0, K1 = "render_kernel<false, false, 1, true>", "k_bounce<1>"
    n0, n1 = f"void myrt::dev::{K0}(myrt::RenderParams)", f"void myrt::dev::{K1}(myrt::RenderParams, int)"
    # 2 frames: one primary pass and 4 bounce levels each
    _write_csv(str(tmp_path / "trace/x/1_kernel_stats.csv"),
               [{"Name": n0, "Calls": "2", "TotalDurationNs": "5000000", "AverageNs": "2500000.0"},
                {"Name": n1, "Calls": "8", "TotalDurationNs": "2000000", "AverageNs": "250000.0"}])

    def pmc(sub, counters):
        rows, d = [], 0
        for name, launches, scale in ((n0, 2, 1.0), (n1, 8, 0.1)):
            for _ in range(launches):
                d += 1
                for c, v in counters.items():
                    rows.append({"Dispatch_Id": str(d), "Kernel_Name": name, "Counter_Name": c,
                                 "Counter_Value": str(v * scale)})
        _write_csv(str(tmp_path / sub / "x/1_counter_collection.csv"), rows)
    pmc("fetch", {"FETCH_SIZE": 100000.0})
    pmc("write", {"WRITE_SIZE": 10000.0})
    pmc("td", {"GRBM_GUI_ACTIVE": 10_000_000.0, "TD_TD_BUSY_sum": 200_000_000.0, "TA_BUSY_avr": 500_000.0})
    pmc("valu", {"GRBM_GUI_ACTIVE": 10_000_000.0, "SQ_ACTIVE_INST_VALU": 200_000_000.0,
                 "SQ_THREAD_CYCLES_VALU": 6_400_000_000.0, "SQ_INSTS_VALU": 100_000_000.0})
    lib = tmp_path / "lib.so"
    lib.write_bytes(b"not a library")
    out = tmp_path / "roofline.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_roofline.py"), "--kernel", K0, "--kernel", K1,
                    "--trace", str(tmp_path / "trace"), "--fetch", str(tmp_path / "fetch"),
                    "--write", str(tmp_path / "write"), "--td", str(tmp_path / "td"), "--valu", str(tmp_path / "valu"),
                    "--lib", str(lib), "-o", str(out)], check=True, capture_output=True)
    r = json.loads(out.read_text())
    per_frame = 1.0 + 4 * 0.1                          # one primary pass + four levels at 0.1 each
    assert r["frame_chain"] and r["trace_frames"] == 2 and r["pmc_frames"] == 2
    assert r["kernel_ms"] == pytest.approx(3.5)        # (5 + 2) ms over 2 frames
    assert r["hbm_bytes_per_launch"] == int(per_frame * (100000 * 1024 * 2 + 10000 * 1024))
    assert r["valu_busy"] == pytest.approx(200e6 / 256 / (10e6 / 8), abs=1e-4)   # ratios of the chain's sums
    assert r["valu_lane_util"] == pytest.approx(6.4e9 / (64 * 200e6), abs=1e-4)
    assert r["chain"][K1]["calls_per_frame"] == 4


def test_pmc_valu_kernels_per_kernel_figures(tmp_path):
    """tools/pmc_valu_kernels.py: per-kernel VALU busy / lane utilisation from one pass."""
    rows = []
    for d, (name, act, thr, gui) in enumerate([("void myrt::dev::k_shade<1>(myrt::RenderParams)", 2.56e8, 6.4e9, 8e6),
                                               ("void myrt::dev::k_level<1>(myrt::RenderParams, int)", 1.28e8, 4.096e9, 8e6)]):
        for c, v in (("SQ_ACTIVE_INST_VALU", act), ("SQ_THREAD_CYCLES_VALU", thr), ("GRBM_GUI_ACTIVE", gui),
                     ("SQ_INSTS_VALU", act)):
            rows.append({"Dispatch_Id": str(d + 1), "Kernel_Name": name, "Counter_Name": c, "Counter_Value": str(v)})
    _write_csv(str(tmp_path / "valu/x/1_counter_collection.csv"), rows)
    out = tmp_path / "v.txt"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_valu_kernels.py"), str(tmp_path / "valu"),
                    "-o", str(out)], check=True, capture_output=True)
    lines = {l.split()[0]: l.split() for l in out.read_text().splitlines()[1:]}
    busy = 2.56e8 / 256 / (8e6 / 8)
    assert float(lines["k_shade<1>"][2]) == pytest.approx(busy, abs=1e-3)
    assert float(lines["k_shade<1>"][3]) == pytest.approx(6.4e9 / (64 * 2.56e8), abs=1e-3)
    assert float(lines["k_level<1>"][3]) == pytest.approx(4.096e9 / (64 * 1.28e8), abs=1e-3)


def test_isa_loops_census():
    """tools/isa_loops.py groups instructions by innermost loop header (LLVM loop comments)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import isa_loops
    asm = """_Zkern:
\ts_mov_b32 s0, 0
.LBB0_1:                                ; =>This Loop Header: Depth=1
\tv_add_f32 v0, v0, v1
\tv_readlane_b32 s4, v127, 3
.LBB0_2:                                ;   Parent Loop BB0_1 Depth=1
                                        ; =>  This Inner Loop Header: Depth=2
\tscratch_load_dword v2, off, off offset:8 ; 4-byte Folded Reload
\tv_mul_f32 v2, v2, v2
; %bb.3:                                ;   in Loop: Header=BB0_1 Depth=1
\ts_load_dword s1, s[0:1], 0x0
\tv_writelane_b32 v127, s1, 4
.Lfunc_end0:
""".split("\n")
    rows = isa_loops.census(asm, 1)
    assert rows["BB0_1"]["depth"] == 1 and rows["BB0_1"]["readlane"] == 1 and rows["BB0_1"]["writelane"] == 1
    assert rows["BB0_1"]["s_load"] == 1 and rows["BB0_1"]["valu"] == 3
    assert rows["BB0_2"]["depth"] == 2 and rows["BB0_2"]["scratch_ld"] == 1 and rows["BB0_2"]["valu"] == 1


def test_numa_helpers():
    """bench.py's NUMA fields: cpulist parsing / printing, the node map from
    sysfs, and the per-page node census of a buffer (move_pages with no target nodes)."""
    import numpy as np
    assert bench._cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert bench._ranges({0, 1, 2, 3, 8, 10, 11}) == "0-3,8,10-11"
    nodes = bench.numa_nodes()
    assert all(isinstance(k, int) and v for k, v in nodes.items())
    a = np.zeros(1 << 20, np.uint8)
    a[:] = 1                                          # every page present
    got = bench.pages_by_node(a.ctypes.data, a.nbytes)
    if got is not None:                               # move_pages may be refused in a sandbox
        pg = os.sysconf("SC_PAGE_SIZE")
        assert sum(got.values()) >= a.nbytes // pg
        if nodes:
            assert set(int(k) for k in got) <= set(nodes)
    assert bench.pages_by_node(a.ctypes.data, 0) == {}
