#!/usr/bin/env python3
"""Summarise a tools/gpu_round.sh run (rocprofv3 CSVs) into profiles/<tag>/.

* kernel_stats.csv            — rocprofv3 --kernel-trace --stats summary (copied)
* verify_kernel_trace.json    — per-kernel/grid duration statistics from the trace
* pmc_traffic.json            — HBM bytes per launch from the PMC passes, corrected
                                as /opt/skills/guides/MI355X_MICROARCH.md §HBM says:
                                FETCH_SIZE is reported in KiB and counts exactly 1/2
                                of the bytes of a 16-B/lane streaming read on gfx950
                                (so bytes = 2 x 1024 x FETCH_SIZE); WRITE_SIZE (KiB)
                                is exact for 16-B/lane streaming stores.
usage: python tools/prof_summary.py gpurun_out/r01 profiles/r01
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

import numpy as np

# kernel name -> workload tag, per bench.py's launches (the profiled runs pass --no-extras, so
# each kernel has one workload; the grid depends on the launch geometry and is only reported)
WORKLOADS = {
    "verify_wg_kernel": "config2 verify: 4096 x 64 KiB (268435456 B read)",
    "verify_wave_kernel": "config3/4 verify: 4M x 1472 B datagrams (6065743872 B payload read)",
    "verify_quad_kernel": "config3/4 verify: 4M x 1472 B datagrams (6065743872 B payload read)",
    "fill_kernel": "config2 fill: 4096 x 64 KiB (268435456 B written)",
}
ALGO_BYTES = {"verify_wg_kernel": 268435456, "verify_wave_kernel": 4194304 * 1446, "verify_quad_kernel": 4194304 * 1446,
              "fill_kernel": 268435456}


def _kname(name):
    return name.split("(")[0].split("<")[0].split("::")[-1].strip()


def _grid(r):
    return r.get("Grid_Size") or r.get("Grid_Size_X")


def main(src, dst):
    os.makedirs(dst, exist_ok=True)
    ks = os.path.join(src, "prof_kt", "run_kernel_stats.csv")
    if os.path.exists(ks):
        shutil.copy(ks, os.path.join(dst, "kernel_stats.csv"))
    out = {}
    tr = os.path.join(src, "prof_kt", "run_kernel_trace.csv")
    if os.path.exists(tr):
        by = defaultdict(list)
        for r in csv.DictReader(open(tr)):
            by[(_kname(r["Kernel_Name"]), _grid(r))].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        for k, d in by.items():
            if k[0] not in WORKLOADS:
                continue
            # one grid per kernel: the one launched most often
            if len(d) < max(len(v) for kk, v in by.items() if kk[0] == k[0]):
                continue
            d = np.array(d)
            out[WORKLOADS[k[0]]] = {"kernel": k[0], "grid": int(k[1]), "launches": int(d.size),
                                 "avg_us": round(float(d.mean()) / 1e3, 2), "median_us": round(float(np.median(d)) / 1e3, 2),
                                 "min_us": round(float(d.min()) / 1e3, 2),
                                 "algorithmic_GBps_at_avg": round(ALGO_BYTES[k[0]] / float(d.mean()), 1)}
        json.dump(out, open(os.path.join(dst, "kernel_trace_summary.json"), "w"), indent=1)
    pmc = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE", "TCC_EA0_RDREQ_sum"):
        p = os.path.join(src, "prof_pmc_%s" % ctr, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        by = defaultdict(list)
        for r in csv.DictReader(open(p)):
            by[(_kname(r["Kernel_Name"]), _grid(r))].append(float(r["Counter_Value"]))
        for k, v in by.items():
            if k[0] not in WORKLOADS:
                continue
            if len(v) < max(len(vv) for kk, vv in by.items() if kk[0] == k[0]):
                continue
            e = pmc.setdefault(WORKLOADS[k[0]], {"kernel": k[0], "grid": int(k[1]), "algorithmic_bytes": ALGO_BYTES[k[0]]})
            e[ctr + "_median"] = float(np.median(v))
            e["launches_" + ctr] = len(v)
    for name, e in pmc.items():
        if "FETCH_SIZE_median" in e:
            e["hbm_read_bytes_per_launch"] = int(2 * 1024 * e["FETCH_SIZE_median"])
        if "TCC_EA0_RDREQ_sum_median" in e:
            e["hbm_read_bytes_per_launch_from_rdreq"] = int(128 * e["TCC_EA0_RDREQ_sum_median"])
        if "WRITE_SIZE_median" in e:
            e["hbm_write_bytes_per_launch"] = int(1024 * e["WRITE_SIZE_median"])
        main_bytes = e.get("hbm_write_bytes_per_launch") if e["kernel"] == "fill_kernel" else e.get(
            "hbm_read_bytes_per_launch")
        if main_bytes:
            e["traffic_over_algorithmic"] = round(main_bytes / e["algorithmic_bytes"], 4)
    if pmc:
        v = pmc.get(WORKLOADS["verify_wg_kernel"], {})
        pmc_out = {"workload": "config2", "buffers": 4096, "hbm_bytes_per_launch": v.get("hbm_read_bytes_per_launch"),
                   "correction": "bytes = 2 x 1024 x FETCH_SIZE(KiB) (gfx950 streaming-read halving)",
                   "kernels": pmc}
        json.dump(pmc_out, open(os.path.join(dst, "pmc_traffic.json"), "w"), indent=1)
    print(json.dumps({"trace": out, "pmc": pmc}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
