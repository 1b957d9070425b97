"""Repeat the GPU AllToAll parity test's exact sequence (fresh communicators per call, the five
RCCL schedules in test order) and localise any mismatch (diagnostic, GPU).

usage: python tools/diag_a2a_loop.py [reps]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("MSCCL_AMD_TIMEOUT_SEC", "20")
from oracle import loader as L  # noqa: E402
from tests.test_gpu_widening_alltoall import RCCL, run_xml  # noqa: E402

NAMES = ["alltoall-8n-0-9kb.xml", "alltoall-8n-9kb-190kb.xml", "alltoall-8n-190kb-512kb.xml",
         "alltoall-8n-512kb-7mb.xml", "alltoall-8n-7mb-43mb.xml"]


def localise(name, gpu, ins, count, ncpl, n=8, ts=4):
    blk = count * ts
    chunk = blk * n // ncpl
    out = []
    for r in range(n):
        g = gpu[r].view(np.uint8)
        e = np.concatenate([ins[q].view(np.uint8)[r * blk:(r + 1) * blk] for q in range(n)])
        d = np.flatnonzero((g != e).reshape(-1, 16).any(axis=1))
        if len(d) == 0:
            continue
        runs = np.split(d, np.flatnonzero(np.diff(d) != 1) + 1)
        for run in runs[:16]:
            b0, b1 = run[0] * 16, (run[-1] + 1) * 16
            ch = b0 // chunk
            seg = g[b0:b1]
            if (seg == 0).all():
                kind = "zeros"
            else:
                kind = "other (%.0f%% bytes right)" % (100.0 * float((seg == e[b0:b1]).mean()))
                # does it equal some other place of any rank's input? (misplaced data)
                for q in range(n):
                    src = ins[q].view(np.uint8)
                    pos = -1
                    probe = seg[:16].tobytes()
                    idx = src.tobytes().find(probe)
                    if idx >= 0:
                        pos = idx
                        kind += "; first pack found in rank %d input at byte %d (chunk %d +%d)" % (
                            q, pos, pos // chunk, pos % chunk)
                        break
            out.append("  %s rank %d out chunk %d (peer %d, slot %d) bytes [%d,%d) of chunk %d: %d packs, %s" % (
                name, r, ch, b0 // blk, ch % max(1, ncpl // n), b0 - ch * chunk, b1 - ch * chunk, chunk,
                len(run), kind))
    return out


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    bad = 0
    total = 0
    t0 = time.time()
    for rep in range(reps):
        for name in NAMES:
            xml = open(os.path.join(RCCL, name)).read()
            a = L.parse_xml(xml, 0, 8)
            n, dt, ts = 8, 7, 4
            ncpl = a.nchunksperloop
            count = max(ncpl, (a.minBytes // (ts * n) // ncpl + 1) * ncpl)
            ins, gpu, ora = run_xml(xml, n, L.ALLTOALL, count, dt, seed=5 + rep)
            total += 1
            ok = all(np.array_equal(gpu[r].view(np.uint8), ora[r].view(np.uint8)) for r in range(n))
            if not ok:
                bad += 1
                print("rep %d %s: MISMATCH" % (rep, name), flush=True)
                for ln in localise(name, gpu, ins, count, ncpl):
                    print(ln, flush=True)
        print("rep %d done (%d bad of %d, %.0f s)" % (rep, bad, total, time.time() - t0), flush=True)
    print("RESULT: %d of %d calls wrong" % (bad, total), flush=True)


if __name__ == "__main__":
    main()
