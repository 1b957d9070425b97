"""Print bench sweeps side by side: python tools/sweep_table.py file.json ..."""
import json, os, sys
cols = []
for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    cols.append((os.path.basename(f).replace(".json", "").replace("0_1073741825_", ""), {r["bytes"]: r for r in d["sweep"]}))
sizes = sorted(set(b for _, c in cols for b in c))
print("%10s " % "bytes" + " ".join("%14s" % n[:14] for n, _ in cols))
for b in sizes:
    print("%10d " % b + " ".join(("%6.1fus %6.1f" % (c[b]["ms"] * 1e3, c[b]["busbw"])) if b in c else "%14s" % "-" for _, c in cols))
