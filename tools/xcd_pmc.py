#!/usr/bin/env python3
"""Per-XCD sums of one TCC counter over the dispatches of one kernel, from a rocprofv3 JSON
(`rocprofv3 --pmc <counter> --output-format json`): the JSON keeps every (TCC instance, XCC)
value of a dispatch, the CSV only their sum.

  python tools/xcd_pmc.py gpurun_out/<dir>/run_results.json [--kernel mscclSmallKernel]

Prints, per XCC, the counter's mean per dispatch (summed over its 16 TCC instances), and the
odd / even XCD ratio.  Unknown JSON layouts print the keys it found instead of guessing."""
import argparse
import collections
import json
import sys


def walk(o, f):
    stack = [o]
    while stack:
        x = stack.pop()
        if isinstance(x, dict):
            f(x)
            stack.extend(x.values())
        elif isinstance(x, list):
            stack.extend(x)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--kernel", default="mscclSmallKernel")
    a = ap.parse_args()
    root = json.load(open(a.path))
    dims = {}       # instance id -> {dimension name: index}
    names = {}      # kernel id -> name
    counters = {}   # counter id -> name

    order = {}      # counter id -> dimensions of its instances, in the listed order

    def reg(o):
        if "instance_id" in o and isinstance(o.get("dimensions"), list):
            dims[o["instance_id"]] = {d.get("dimension_name"): d.get("index") for d in o["dimensions"] if isinstance(d, dict)}
        if isinstance(o.get("instances"), list) and "id" in o:
            cid = o["id"]["handle"] if isinstance(o["id"], dict) else o["id"]
            order[cid] = [{d.get("dimension_name"): d.get("index") for d in x.get("dimensions", [])}
                          for x in o["instances"] if isinstance(x, dict)]
        if "kernel_id" in o and any(k in o for k in ("kernel_name", "truncated_kernel_name", "formatted_kernel_name")):
            names[o["kernel_id"]] = o.get("kernel_name") or o.get("formatted_kernel_name") or o.get("truncated_kernel_name")
        if "id" in o and "name" in o and ("block" in o or "description" in o):
            cid = o["id"]["handle"] if isinstance(o["id"], dict) else o["id"]
            counters[cid] = o["name"]
    walk(root, reg)

    per = collections.defaultdict(lambda: collections.defaultdict(float))  # dispatch -> xcc -> value
    seen_keys = set()

    def rec(o):
        recs = o.get("records")
        if not isinstance(recs, list) or not recs or not isinstance(recs[0], dict):
            return
        kid, did = None, None

        def find(x):
            nonlocal kid, did
            if "kernel_id" in x and kid is None:
                kid = x["kernel_id"]
            if "dispatch_id" in x and did is None:
                did = x["dispatch_id"]
        walk({k: v for k, v in o.items() if k != "records"}, find)
        if kid is None or a.kernel not in str(names.get(kid, "")):
            return
        for i, r in enumerate(recs):
            seen_keys.update(r.keys())
            iid = r.get("instance_id")
            if isinstance(iid, dict):
                iid = iid.get("handle")
            v = r.get("counter_value", r.get("value"))
            cid = r.get("counter_id")
            if isinstance(cid, dict):
                cid = cid.get("handle")
            # records without an instance id come in the order of the counter's "instances" list
            if iid is not None:
                d = dims.get(iid)
            else:
                d = order[cid][i] if len(order.get(cid, ())) == len(recs) else None
            if d is None or v is None:
                continue
            per[did][d.get("DIMENSION_XCC", 0)] += float(v)
    walk(root, rec)
    if not per:
        print("no %s records matched; instance ids %d, kernels %d, record keys %s" % (
            a.kernel, len(dims), len(names), sorted(seen_keys)))
        return 1
    xccs = sorted({x for v in per.values() for x in v})
    mean = {x: sum(v.get(x, 0.0) for v in per.values()) / len(per) for x in xccs}
    print("%s: %d dispatches; per XCC, mean per dispatch over the 16 TCC instances" % (a.kernel, len(per)))
    for x in xccs:
        print("  XCC %d  %14.1f" % (x, mean[x]))
    odd = [mean[x] for x in xccs if x % 2]
    even = [mean[x] for x in xccs if x % 2 == 0]
    if odd and even and sum(even):
        print("  odd / even XCDs: %.4f" % ((sum(odd) / len(odd)) / (sum(even) / len(even))))
    return 0


if __name__ == "__main__":
    sys.exit(main())
