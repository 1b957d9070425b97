"""AllReduce of host-resident buffers, the path the north star starts and ends in: the user's
pinned host tensors are copied in, reduced and copied out.

all_reduce_host (zero copy).  The collective itself reads the pinned inputs and writes the pinned
outputs over PCIe, through their device addresses (hipHostGetDevicePointer): no device staging
buffer and no copy engine.  The fused exchange reads each input once and writes each output once,
so PCIe carries S in and S out per rank, in both directions at once.  2 co-resident ranks at
32 MiB each: 1.70 ms, bit-exact, against 3.16 ms for the serial copy-in / reduce / copy-out on one
stream.  Copying 2 x 32 MiB in and out concurrently takes 1.38 ms, the floor
(profiles/r05z_e2e_probe.txt).

all_reduce_host_staged.  The buffers move through device buffers in chunks on three HIP streams
per device: H2D, collective, D2H, ordered by events.  Cross-stream waits on the copy engines cost
about 100 us per chunk here, so it only helps with two or three large chunks (16 MiB chunks:
2.03 ms).  It is kept for host memory that has no device address.

A chunk's collective is an ordinary ncclAllReduce of that chunk on every rank, in one group.  An
AllReduce is elementwise, so the chunks together give the whole call's result.  The bits equal
the whole call's whenever the schedule's per-element fold order does not depend on the element's
position: the 2-rank pair exchange, the rank-ordered one-shot, and any schedule on exact-integer
inputs.  A schedule that folds different chunk classes in different orders (the two-phase
all-pairs at n > 2) still gives a valid AllReduce with identical bits on every rank.  Its
association may differ from the unchunked call's.
"""
import ctypes
from typing import List, Optional, Sequence

from . import SUM, Comm, group, lib

_H2D, _D2H = 1, 2            # hipMemcpyHostToDevice, hipMemcpyDeviceToHost
_EVENT_DISABLE_TIMING = 0x2  # hipEventDisableTiming


class _Hip:
    """The HIP runtime calls of the pipeline, resolved through the library's handle (the runtime it
    was linked against, the one torch has loaded): hipMemcpyAsync and events cost a few
    microseconds per call, against tens for a torch slice copy, which left the pipeline host-bound
    (tools/e2e_probe.py)."""

    def __init__(self):
        L = lib()
        self.memcpy = L.hipMemcpyAsync
        self.memcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
        self.create = L.hipEventCreateWithFlags
        self.create.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
        self.record = L.hipEventRecord
        self.record.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        self.wait = L.hipStreamWaitEvent
        self.wait.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint]
        self.destroy = L.hipEventDestroy
        self.destroy.argtypes = [ctypes.c_void_p]
        self.set_device = L.hipSetDevice
        self.set_device.argtypes = [ctypes.c_int]
        self.get_device = L.hipGetDevice
        self.get_device.argtypes = [ctypes.POINTER(ctypes.c_int)]
        self.host_dev_ptr = L.hipHostGetDevicePointer
        self.host_dev_ptr.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p, ctypes.c_uint]

    def check(self, rc: int, what: str) -> None:
        if rc != 0:
            raise RuntimeError("%s failed: hipError %d" % (what, rc))


_hip: Optional[_Hip] = None


class _Events:
    """A pool of timing-free events per device, reused across calls (an event may be re-recorded once
    the waits on its earlier record have been enqueued)."""

    def __init__(self):
        self.pool = {}

    def get(self, h: _Hip, dev: int, i: int) -> int:
        evs = self.pool.setdefault(dev, [])
        while len(evs) <= i:
            e = ctypes.c_void_p()
            h.check(h.create(ctypes.byref(e), _EVENT_DISABLE_TIMING), "hipEventCreateWithFlags")
            evs.append(e.value)
        return evs[i]


def all_reduce_host_staged(comms: Sequence[Comm], host_in: Sequence, host_out: Sequence, dev_bufs: Sequence,
                           dtype: int, op: int = SUM, chunk_bytes: int = 16 << 20,
                           streams: Optional[dict] = None) -> None:
    """host_in[r] (pinned) -> AllReduce over the ranks of `comms` -> host_out[r] (pinned), through
    dev_bufs[r] (a device tensor of the same size on rank r's device).  The copies and collectives
    are enqueued and this returns without waiting: synchronise the devices (or the caller's current
    streams, which wait for the whole call) before reading host_out.  streams: a dict this call
    fills with {device: (h2d, coll, d2h)} torch streams and an event pool; pass the same dict to
    later calls to reuse them."""
    import torch
    h = _hip_rt()
    n = len(comms)
    if not (len(host_in) == len(host_out) == len(dev_bufs) == n):
        raise ValueError("one host input, host output and device buffer per rank")
    numel = host_in[0].numel()
    esize = host_in[0].element_size()
    for t in list(host_in) + list(host_out) + list(dev_bufs):
        if t.numel() != numel or t.element_size() != esize or not t.is_contiguous():
            raise ValueError("every buffer must be contiguous with the same element count and size")
    for t in list(host_in) + list(host_out):
        if not t.is_pinned():
            raise ValueError("host buffers must be pinned (asynchronous copies)")
    if streams is None:
        streams = {}
    devs = [b.device.index for b in dev_bufs]
    udevs = sorted(set(devs))
    for d in udevs:
        if d not in streams:
            with torch.cuda.device(d):
                streams[d] = tuple(torch.cuda.Stream() for _ in range(3))
    pool = streams.setdefault("events", _Events())
    st = {d: tuple(s.cuda_stream for s in streams[d]) for d in udevs}
    cur = {d: torch.cuda.current_stream(d).cuda_stream for d in udevs}
    # chunks of whole 16-B packs (the schedules' chunk arithmetic), the last one ragged
    pe = max(1, 16 // esize)
    step = max(pe, (chunk_bytes // esize) // pe * pe)
    hin = [t.data_ptr() for t in host_in]
    hout = [t.data_ptr() for t in host_out]
    dbuf = [t.data_ptr() for t in dev_bufs]
    saved = ctypes.c_int()
    h.check(h.get_device(ctypes.byref(saved)), "hipGetDevice")
    ev = 0

    def fence(d, src, dst):
        # dst waits for everything enqueued on src so far
        nonlocal ev
        e = pool.get(h, d, ev)
        ev += 1
        h.check(h.record(e, src), "hipEventRecord")
        h.check(h.wait(dst, e, 0), "hipStreamWaitEvent")
    try:
        for d in udevs:
            h.check(h.set_device(d), "hipSetDevice")
            for s in st[d]:
                fence(d, cur[d], s)  # the buffers may still be in use on the caller's stream
        for off in range(0, numel, step):
            cnt = min(step, numel - off)
            nb, ob = cnt * esize, off * esize
            for r in range(n):
                h.check(h.set_device(devs[r]), "hipSetDevice")
                h.check(h.memcpy(dbuf[r] + ob, hin[r] + ob, nb, _H2D, st[devs[r]][0]), "hipMemcpyAsync H2D")
            for d in udevs:
                h.check(h.set_device(d), "hipSetDevice")
                fence(d, st[d][0], st[d][1])
            with group():
                for r, c in enumerate(comms):
                    c.all_reduce(dbuf[r] + ob, dbuf[r] + ob, cnt, dtype, op, st[devs[r]][1])
            for d in udevs:
                h.check(h.set_device(d), "hipSetDevice")
                fence(d, st[d][1], st[d][2])
            for r in range(n):
                h.check(h.set_device(devs[r]), "hipSetDevice")
                h.check(h.memcpy(hout[r] + ob, dbuf[r] + ob, nb, _D2H, st[devs[r]][2]), "hipMemcpyAsync D2H")
        for d in udevs:
            h.check(h.set_device(d), "hipSetDevice")
            for s in st[d]:
                fence(d, s, cur[d])  # the caller's stream sees the whole call
    finally:
        h.set_device(saved.value)


def _hip_rt() -> _Hip:
    global _hip
    if _hip is None:
        _hip = _Hip()
    return _hip


def device_address(t) -> int:
    """The device address of pinned host tensor t (hipHostGetDevicePointer; the host address
    itself on this platform).  Raises if the memory is not mapped for the device."""
    h = _hip_rt()
    if not t.is_pinned():
        raise ValueError("host buffers must be pinned (mapped for the device)")
    p = ctypes.c_void_p()
    rc = h.host_dev_ptr(ctypes.byref(p), ctypes.c_void_p(t.data_ptr()), 0)
    if rc != 0 or not p.value:
        raise RuntimeError("hipHostGetDevicePointer failed: hipError %d" % rc)
    return p.value


def all_reduce_host(comms: Sequence[Comm], host_in: Sequence, host_out: Sequence, dtype: int, op: int = SUM,
                    streams: Optional[Sequence[int]] = None) -> None:
    """Zero-copy AllReduce of pinned host tensors: host_in[r] -> host_out[r] (the same tensor for
    in place) over the ranks of `comms`, one group.  The collective runs on streams[r] (a HIP
    stream handle; default: the current torch stream of rank r's device) and reads / writes the
    host memory itself; synchronise that stream before reading host_out."""
    import torch
    n = len(comms)
    if not (len(host_in) == len(host_out) == n):
        raise ValueError("one host input and output per rank")
    numel = host_in[0].numel()
    for t in list(host_in) + list(host_out):
        if t.numel() != numel or t.element_size() != host_in[0].element_size() or not t.is_contiguous():
            raise ValueError("every buffer must be contiguous with the same element count and size")
    src = [device_address(t) for t in host_in]
    dst = [device_address(t) for t in host_out]
    if streams is None:
        streams = [torch.cuda.current_stream(c.device).cuda_stream for c in comms]
    with group():
        for r, c in enumerate(comms):
            c.all_reduce(src[r], dst[r], numel, dtype, op, streams[r])


def reduce_scatter_host(comms: Sequence[Comm], host_in: Sequence, host_out: Sequence, dtype: int, op: int = SUM,
                        streams: Optional[Sequence[int]] = None) -> None:
    """Zero-copy ReduceScatter of pinned host tensors: host_in[r] holds nranks x recvcount elements,
    host_out[r] recvcount (rank r's reduced block), as all_reduce_host."""
    import torch
    n = len(comms)
    if not (len(host_in) == len(host_out) == n) or any(t.numel() != host_in[0].numel() for t in host_in):
        raise ValueError("one host input and output per rank, inputs of one size")
    recvcount = host_out[0].numel()
    if host_in[0].numel() != recvcount * n or any(t.numel() != recvcount for t in host_out):
        raise ValueError("inputs must hold nranks x recvcount elements, outputs recvcount")
    src = [device_address(t) for t in host_in]
    dst = [device_address(t) for t in host_out]
    if streams is None:
        streams = [torch.cuda.current_stream(c.device).cuda_stream for c in comms]
    with group():
        for r, c in enumerate(comms):
            c.reduce_scatter(src[r], dst[r], recvcount, dtype, op, streams[r])


def all_gather_host(comms: Sequence[Comm], host_in: Sequence, host_out: Sequence, dtype: int,
                    streams: Optional[Sequence[int]] = None) -> None:
    """Zero-copy AllGather of pinned host tensors: host_in[r] holds sendcount elements, host_out[r]
    nranks x sendcount, as all_reduce_host."""
    import torch
    n = len(comms)
    if not (len(host_in) == len(host_out) == n):
        raise ValueError("one host input and output per rank")
    sendcount = host_in[0].numel()
    if any(t.numel() != sendcount for t in host_in) or any(t.numel() != sendcount * n for t in host_out):
        raise ValueError("inputs must hold sendcount elements, outputs nranks x sendcount")
    src = [device_address(t) for t in host_in]
    dst = [device_address(t) for t in host_out]
    if streams is None:
        streams = [torch.cuda.current_stream(c.device).cuda_stream for c in comms]
    with group():
        for r, c in enumerate(comms):
            c.all_gather(src[r], dst[r], sendcount, dtype, streams[r])


def default_chunk_bytes(nbytes: int, chunks: int = 2, floor: int = 1 << 20) -> int:
    """A chunk size for all_reduce_host_staged on nbytes per rank: `chunks` pipeline stages, at least
    `floor` bytes each (each chunk costs ~100 us of cross-stream waits on the copy engines)."""
    return max(floor, (nbytes + chunks - 1) // chunks)


__all__: List[str] = ["all_reduce_host", "reduce_scatter_host", "all_gather_host", "all_reduce_host_staged",
                       "device_address", "default_chunk_bytes"]
