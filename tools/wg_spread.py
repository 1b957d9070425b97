"""Workgroup end times of one traced launch, by XCD and by rank (the per-slot output of
tools/trace_report.py under MSCCL_AMD_TRACE=2: "rank r slot s: start t0 | done t xcc k").
  python tools/wg_spread.py gpurun_out/c3_t2.txt"""
import collections
import re
import sys

import numpy as np


def main():
    rows = []
    for line in open(sys.argv[1]):
        m = re.match(r"rank (\d+) slot\s+(\d+): start ([\d.]+) \| done ([\d.]+) xcc (\d+)", line)
        if m:
            rows.append((int(m.group(1)), int(m.group(2)), float(m.group(3)), float(m.group(4)), int(m.group(5))))
    if not rows:
        print("no traced workgroups")
        return
    start = np.array([r[2] for r in rows])
    end = np.array([r[3] for r in rows])
    print("%d workgroups: start span %.2f us; end min %.1f median %.1f max %.1f us" % (
        len(rows), start.max() - start.min(), end.min(), np.median(end), end.max()))
    for name, key in (("xcc", 4), ("rank", 0)):
        g = collections.defaultdict(list)
        for r in rows:
            g[r[key]].append(r[3])
        print("by %s: %s" % (name, "  ".join("%d: mean %.1f max %.1f" % (k, np.mean(v), np.max(v))
                                              for k, v in sorted(g.items()))))
    late = sorted(rows, key=lambda r: -r[3])[:8]
    print("latest: %s" % ", ".join("r%d s%d x%d %.1f" % (r[0], r[1], r[4], r[3]) for r in late))


if __name__ == "__main__":
    main()
