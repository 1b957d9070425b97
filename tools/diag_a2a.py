"""Localise AllToAll mismatches on co-resident ranks (diagnostic, GPU).

Runs an RCCL AllToAll schedule K times on 8 co-resident ranks with fresh inputs per launch and a
sentinel-filled output, checks every output byte against the collective's definition, and for
every wrong 16-B pack reports (rank, output chunk, peer, channel, offset inside the chunk) and
what the bad bytes are: the sentinel (never written), zeros, the expected data of an earlier
launch (stale FIFO slot), or something else.

usage: python tools/diag_a2a.py [xml-name] [iters]   (env knobs are read at comm init)
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import msccl_amd as M  # noqa: E402
from oracle import loader as L  # noqa: E402

RCCL = "/opt/rocm/share/rccl/msccl-algorithms"


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "alltoall-8n-7mb-43mb.xml"
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    xml = open(os.path.join(RCCL, name)).read()
    a = L.parse_xml(xml, 0, 8)
    n, ts = 8, 4
    ncpl = a.nchunksperloop
    count = max(ncpl, (a.minBytes // (ts * n) // ncpl + 1) * ncpl)
    path = "/tmp/diag_a2a_%d.xml" % os.getpid()
    open(path, "w").write(xml)
    os.environ["MSCCL_XML_FILES"] = path
    os.environ.setdefault("MSCCL_AMD_TIMEOUT_SEC", "20")
    dev = torch.device("cuda:0")
    comms = M.Comm.init_all([0] * n)
    blk = count * ts                      # bytes of one (rank -> peer) block
    chunk = blk * n // ncpl               # bytes of one MSCCL chunk
    print("%s: count=%d floats, block=%d B, chunk=%d B, ncpl=%d, env FORCE_REMOTE=%s COARSE=%s" % (
        name, count, blk, chunk, ncpl, os.environ.get("MSCCL_AMD_FORCE_REMOTE", "0"),
        os.environ.get("MSCCL_AMD_ARENA_COARSE", "0")), flush=True)
    history = []   # expected outputs of earlier launches
    bad_launches = 0
    stream = torch.cuda.current_stream().cuda_stream
    try:
        for it in range(iters):
            g = torch.Generator(device="cpu").manual_seed(1234 + it)
            ins = [torch.randint(0, 256, (blk * n,), dtype=torch.uint8, generator=g) for _ in range(n)]
            t_in = [x.to(dev) for x in ins]
            t_out = [torch.full((blk * n,), 0xA5, dtype=torch.uint8, device=dev) for _ in range(n)]
            torch.cuda.synchronize()
            with M.group():
                for c, x, y in zip(comms, t_in, t_out):
                    c.all_to_all(x.data_ptr(), y.data_ptr(), count, M.FLOAT32, stream)
            torch.cuda.synchronize()
            errs = [c.async_error() for c in comms]
            got = [t.cpu().numpy() for t in t_out]
            exp = [np.concatenate([ins[q].numpy()[r * blk:(r + 1) * blk] for q in range(n)]) for r in range(n)]
            nbad = 0
            lines = []
            for r in range(n):
                d = got[r] != exp[r]
                if not d.any():
                    continue
                pk = np.flatnonzero(d.reshape(-1, 16).any(axis=1))
                nbad += len(pk)
                # group contiguous packs
                starts = [pk[0]]
                ends = []
                for i in range(1, len(pk)):
                    if pk[i] != pk[i - 1] + 1:
                        ends.append(pk[i - 1])
                        starts.append(pk[i])
                ends.append(pk[-1])
                for s, e in list(zip(starts, ends))[:12]:
                    b0, b1 = s * 16, (e + 1) * 16
                    ch = b0 // chunk
                    g_ = got[r][b0:b1]
                    kind = "other"
                    if (g_ == 0xA5).all():
                        kind = "sentinel(never written)"
                    elif (g_ == 0).all():
                        kind = "zeros"
                    else:
                        for k, h in enumerate(reversed(history)):
                            if np.array_equal(g_, h[r][b0:b1]):
                                kind = "stale: launch it-%d" % (k + 1)
                                break
                        if kind == "other":
                            frac = float((g_ == exp[r][b0:b1]).mean())
                            kind = "other (%.0f%% bytes right)" % (100 * frac)
                    q = b0 // blk
                    lines.append("  rank %d out chunk %d (peer %d, chan-slot %d) bytes [%d,%d) of chunk (%d B, %d packs): %s" % (
                        r, ch, q, ch % (ncpl // n), b0 - ch * chunk, b1 - ch * chunk, b1 - b0, (b1 - b0) // 16, kind))
            if nbad or any(errs):
                bad_launches += 1
                print("launch %d: %d bad packs, async errors %s" % (it, nbad, errs), flush=True)
                for ln in lines[:40]:
                    print(ln, flush=True)
            history.append(exp)
            history = history[-9:]
        print("RESULT %s: %d of %d launches wrong" % (name, bad_launches, iters), flush=True)
    finally:
        for c in comms:
            c.destroy()


if __name__ == "__main__":
    main()
