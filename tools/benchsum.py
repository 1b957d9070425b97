"""Summarise bench.py JSON lines: sweep (device time per launch, busbw, kernel), secondary
schedule lines and the headline roofline.  python tools/benchsum.py a.json [b.json ...]"""
import json
import sys

for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print("== %s: value %s avg %s verified %s" % (f, d["value"], d.get("avg_busbw"), d["verified"]))
    for s in d["sweep"]:
        print("  %10d %10.2f us %9.2f GB/s  %s" % (s["bytes"], s["kernel_ms"] * 1e3, s["busbw"], s["kernel"]))
    for k, v in d.get("schedules", {}).items():
        print("  %s: %s" % (k, {x: v.get(x) for x in ("kernel_ms", "busbw", "kernel", "verified", "memside_frac",
                                                      "payload_frac", "error") if x in v}))
    r = d["roofline"]
    print("  roofline: %s" % {k: r.get(k) for k in ("achieved", "frac", "payload_frac", "traffic_over_algorithmic",
                                                   "kernel")})
