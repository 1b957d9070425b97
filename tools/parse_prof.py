#!/usr/bin/env python3
"""Summarise a tools/profile.sh run into profiles/<tag>_*.

Reads rocprofv3 CSVs (kernel stats, kernel trace, FETCH_SIZE and WRITE_SIZE counter passes) and
writes:
  profiles/<tag>_kernel_stats.csv   the --stats summary as rocprofv3 wrote it
  profiles/<tag>_pmc.json           per-launch averages for the MSCCL kernel: duration (trace),
                                    FETCH_SIZE, WRITE_SIZE and the HBM traffic they imply
                                    (FETCH_SIZE doubled: on gfx950 it reports half the bytes of a
                                    16-B/lane streaming read, MI355X_MICROARCH.md "HBM"; both in KiB)
  profiles/<tag>_bench.json         the bench JSON line printed under the kernel-trace pass
"""
import csv
import glob
import json
import os
import shutil
import sys


def rows(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def col(row, *names):
    low = {k.lower(): k for k in row}
    for n in names:
        if n.lower() in low:
            return row[low[n.lower()]]
    raise KeyError(names)


def find(d, pattern):
    return sorted(glob.glob(os.path.join(d, "**", pattern), recursive=True))


def is_msccl(name):
    return any(k in name for k in ("mscclKernel", "mscclSmallKernel", "mscclFoldKernel", "mscclPairKernel",
                                   "mscclTwoPhaseKernel", "mscclDirectKernel"))


def counter_avg(d, counter):
    files = find(d, "*counter_collection.csv")
    vals = []
    for f in files:
        for r in rows(f):
            if not is_msccl(col(r, "Kernel_Name", "KernelName", "Kernel-Name")):
                continue
            if col(r, "Counter_Name", "CounterName") != counter:
                continue
            vals.append(float(col(r, "Counter_Value", "CounterValue")))
    return (sum(vals) / len(vals), len(vals)) if vals else (None, 0)


def per_kernel(out):
    """Every interpreter kernel of the run separately (a run timing several configurations
    launches a different kernel instantiation per configuration): calls, average duration from
    the trace, FETCH_SIZE / WRITE_SIZE averages and the traffic they imply."""
    res = {}
    for f in find(os.path.join(out, "kt"), "*kernel_trace.csv"):
        for r in rows(f):
            name = col(r, "Kernel_Name", "KernelName")
            if is_msccl(name):
                d = res.setdefault(name, {"durs": []})
                d["durs"].append(int(col(r, "End_Timestamp", "EndNs")) - int(col(r, "Start_Timestamp", "BeginNs")))
    for sub, counter in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        for f in find(os.path.join(out, sub), "*counter_collection.csv"):
            for r in rows(f):
                name = col(r, "Kernel_Name", "KernelName", "Kernel-Name")
                if is_msccl(name) and col(r, "Counter_Name", "CounterName") == counter:
                    res.setdefault(name, {"durs": []}).setdefault(counter, []).append(
                        float(col(r, "Counter_Value", "CounterValue")))
    out_d = {}
    for name, d in res.items():
        e = {"launches": len(d["durs"]), "avg_ns": sum(d["durs"]) / len(d["durs"]) if d["durs"] else None}
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            v = d.get(counter, [])
            e[counter.lower() + "_kib_avg"] = sum(v) / len(v) if v else None
        if e["fetch_size_kib_avg"] is not None and e["write_size_kib_avg"] is not None:
            e["traffic_bytes_per_launch"] = (2.0 * e["fetch_size_kib_avg"] + e["write_size_kib_avg"]) * 1024.0
        out_d[name] = e
    return out_d


def main():
    out, tag = sys.argv[1], sys.argv[2]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prof = os.path.join(root, "profiles")
    os.makedirs(prof, exist_ok=True)
    res = {"tag": tag}
    # the device sources this profile was taken on (bench.py uses a committed profile's traffic
    # only for the same kernel_src_hash)
    sys.path.insert(0, root)
    import bench
    res["kernel_src"] = bench.kernel_src_hash()
    stats = find(os.path.join(out, "kt"), "*kernel_stats.csv")
    if stats:
        shutil.copy(stats[0], os.path.join(prof, tag + "_kernel_stats.csv"))
        for r in rows(stats[0]):
            if is_msccl(col(r, "Name", "KernelName", "Kernel_Name")):
                res["kernel"] = col(r, "Name", "KernelName", "Kernel_Name")
                res["stats_calls"] = int(col(r, "Calls"))
                res["stats_avg_ns"] = float(col(r, "AverageNs", "Average_Ns", "AvgNs"))
    traces = find(os.path.join(out, "kt"), "*kernel_trace.csv")
    durs = []
    for f in traces:
        for r in rows(f):
            if is_msccl(col(r, "Kernel_Name", "KernelName")):
                durs.append(int(col(r, "End_Timestamp", "EndNs")) - int(col(r, "Start_Timestamp", "BeginNs")))
    if durs:
        res["trace_launches"] = len(durs)
        res["trace_avg_ns"] = sum(durs) / len(durs)
    fetch, nf = counter_avg(os.path.join(out, "fetch"), "FETCH_SIZE")
    write, nw = counter_avg(os.path.join(out, "write"), "WRITE_SIZE")
    res["fetch_size_kib_avg"], res["fetch_launches"] = fetch, nf
    res["write_size_kib_avg"], res["write_launches"] = write, nw
    if fetch is not None and write is not None:
        res["traffic_bytes_per_launch"] = (2.0 * fetch + write) * 1024.0
        res["traffic_note"] = "(2 x FETCH_SIZE + WRITE_SIZE) x 1024 per interpreter-kernel dispatch (gfx950 FETCH_SIZE correction)"
    res["per_kernel"] = per_kernel(out)
    kt = os.path.join(out, "kt.json")
    if os.path.exists(kt):
        try:
            line = [ln for ln in open(kt).read().splitlines() if ln.startswith("{")][-1]
            bench = json.loads(line)
            json.dump(bench, open(os.path.join(prof, tag + "_bench.json"), "w"), indent=1)
            res["bench_kernel_ms"] = bench["roofline"].get("kernel_ms")
            res["bench_algorithmic_bytes_per_launch"] = bench["roofline"].get("algorithmic_bytes_per_launch")
        except (IndexError, ValueError, KeyError):
            pass
    json.dump(res, open(os.path.join(prof, tag + "_pmc.json"), "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
