"""PCIe copy rates behind the host-resident AllReduce (msccl_amd/hostpath.py): pinned H2D alone,
D2H alone, both directions at once on two streams, and the pipelined AllReduce of 2 co-resident
ranks at several chunk sizes (2 x 32 MiB fp32).
  python tools/e2e_probe.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import msccl_amd as M  # noqa: E402
from msccl_amd import hostpath, xmlgen  # noqa: E402


def timed(fn, reps=10):
    import torch
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    import torch
    nbytes = 32 << 20
    cnt = nbytes // 4
    path = "/tmp/e2e_probe_%d.xml" % os.getpid()
    open(path, "w").write(xmlgen.allreduce_pair_oneshot(16, "LL"))
    os.environ["MSCCL_XML_FILES"] = path
    comms = M.Comm.init_all([0, 0])
    hin = [torch.rand(cnt).pin_memory() for _ in range(2)]
    hout = [torch.empty(cnt).pin_memory() for _ in range(2)]
    dev = [torch.empty(cnt, device="cuda:0") for _ in range(2)]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def h2d():
        with torch.cuda.stream(s1):
            for i in range(2):
                dev[i].copy_(hin[i], non_blocking=True)

    def d2h():
        with torch.cuda.stream(s2):
            for i in range(2):
                hout[i].copy_(dev[i], non_blocking=True)

    def both():
        h2d()
        d2h()
    mb = 2 * nbytes / 1e6
    for name, fn in (("H2D 2 x 32 MiB", h2d), ("D2H 2 x 32 MiB", d2h), ("H2D and D2H at once", both)):
        ms = timed(fn)
        print("%-24s %.3f ms  (%.1f GB/s per direction)" % (name, ms, mb / ms), flush=True)
    streams = {}
    for chunk in (32 << 20, 16 << 20, 8 << 20, 4 << 20, 2 << 20, 1 << 20):
        ms = timed(lambda: hostpath.all_reduce_host_staged(comms, hin, hout, dev, M.FLOAT32, M.SUM, chunk, streams))
        print("pipelined AllReduce, %2d MiB chunks: %.3f ms" % (chunk >> 20, ms), flush=True)
    # the pipeline's parts in isolation, 2 MiB chunks: copies only (H2D -> event -> D2H), the
    # collectives only, and H2D chunks alone on one stream
    h = hostpath._hip
    pool = hostpath._Events()
    st = [s.cuda_stream for s in streams[0]]
    csz = 2 << 20
    nch = nbytes // csz

    def copies_only(with_coll=False, with_copies=True, d2h_on=True):
        ev = 0
        for k in range(nch):
            ob = k * csz
            if with_copies:
                for i in range(2):
                    h.memcpy(dev[i].data_ptr() + ob, hin[i].data_ptr() + ob, csz, 1, st[0])
                e = pool.get(h, 0, ev); ev += 1
                h.record(e, st[0]); h.wait(st[1], e, 0)
            if with_coll:
                with M.group():
                    for c, b in zip(comms, dev):
                        c.all_reduce(b.data_ptr() + ob, b.data_ptr() + ob, csz // 4, M.FLOAT32, M.SUM, st[1])
            if with_copies and d2h_on:
                e = pool.get(h, 0, ev); ev += 1
                h.record(e, st[1]); h.wait(st[2], e, 0)
                for i in range(2):
                    h.memcpy(hout[i].data_ptr() + ob, dev[i].data_ptr() + ob, csz, 2, st[2])
    for name, fn in (("chunked copies, no collective", lambda: copies_only()),
                     ("chunked H2D only", lambda: copies_only(d2h_on=False)),
                     ("chunked collectives only", lambda: copies_only(True, False)),
                     ("chunked copies + collectives", lambda: copies_only(True))):
        print("%-32s 2 MiB chunks: %.3f ms" % (name, timed(fn)), flush=True)
    # zero-copy: the collective reads the pinned inputs and writes the pinned outputs itself (their
    # device addresses from hipHostGetDevicePointer), out of place
    if os.environ.get("E2E_ZERO_COPY") == "1":
        import ctypes
        L = M.lib()
        L.hipHostGetDevicePointer.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p, ctypes.c_uint]

        def dptr(t):
            p = ctypes.c_void_p()
            rc = L.hipHostGetDevicePointer(ctypes.byref(p), ctypes.c_void_p(t.data_ptr()), 0)
            if rc != 0 or not p.value:
                raise RuntimeError("hipHostGetDevicePointer: %d" % rc)
            return p.value
        for c in comms:
            c.destroy()
        open(path, "w").write(xmlgen.allreduce_pair_oneshot(16, "LL", inplace=False))
        comms = M.Comm.init_all([0, 0])
        din = [dptr(t) for t in hin]
        dout = [dptr(t) for t in hout]
        print("device addresses equal host addresses:", [d == t.data_ptr() for d, t in zip(din, hin)], flush=True)
        s0 = torch.cuda.current_stream().cuda_stream
        for small in (4096, 1 << 20, cnt):
            for o in hout:
                o.zero_()
            with M.group():
                for c, i, o in zip(comms, din, dout):
                    c.all_reduce(i, o, small, M.FLOAT32, M.SUM, s0)
            torch.cuda.synchronize()
            ok = all(torch.equal(o[:small], hin[0][:small] + hin[1][:small]) for o in hout)
            print("zero-copy %d floats: %s, async errors %s" % (small, "bit-exact" if ok else "MISMATCH",
                                                                [c.async_error() for c in comms]), flush=True)

        def zc():
            with M.group():
                for c, i, o in zip(comms, din, dout):
                    c.all_reduce(i, o, cnt, M.FLOAT32, M.SUM, s0)
        print("zero-copy AllReduce 2 x 32 MiB: %.3f ms" % timed(zc), flush=True)
    t0 = time.perf_counter()
    for _ in range(10):
        hostpath.all_reduce_host_staged(comms, hin, hout, dev, M.FLOAT32, M.SUM, 4 << 20, streams)
    print("host enqueue time per call, 4 MiB chunks: %.3f ms" % ((time.perf_counter() - t0) / 10 * 1e3), flush=True)
    torch.cuda.synchronize()
    for c in comms:
        c.destroy()


if __name__ == "__main__":
    main()
