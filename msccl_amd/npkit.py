"""NPKit dump reader and Chrome-trace converter (include/msccl_amd_npkit.h).

The dump is the file set of the reference's NpKit::Dump (src/misc/npkit.cc:64-127); `to_trace`
produces the trace the reference's tools/npkit_trace_generator.py produces from it (same
events, names, timestamps and arguments), so traces from either tool load the same way in
chrome://tracing or Perfetto.

    python -m msccl_amd.npkit --input_dir /tmp --output_dir out/   # writes out/npkit_event_trace.json
"""
import argparse
import json
import os
import re
import struct
from typing import Dict, List

# include/msccl_amd_npkit.h (the reference's npkit_event.h values)
EVENTS = {
    "NPKIT_EVENT_INVALID": 0x0,
    "NPKIT_EVENT_SEND_ENTRY": 0x1, "NPKIT_EVENT_SEND_EXIT": 0x2,
    "NPKIT_EVENT_SEND_FROM_OUTPUT_ENTRY": 0x3, "NPKIT_EVENT_SEND_FROM_OUTPUT_EXIT": 0x4,
    "NPKIT_EVENT_DIRECT_SEND_ENTRY": 0x5, "NPKIT_EVENT_DIRECT_SEND_EXIT": 0x6,
    "NPKIT_EVENT_DIRECT_SEND_FROM_OUTPUT_ENTRY": 0x7, "NPKIT_EVENT_DIRECT_SEND_FROM_OUTPUT_EXIT": 0x8,
    "NPKIT_EVENT_RECV_ENTRY": 0x9, "NPKIT_EVENT_RECV_EXIT": 0xA,
    "NPKIT_EVENT_DIRECT_RECV_ENTRY": 0xB, "NPKIT_EVENT_DIRECT_RECV_EXIT": 0xC,
    "NPKIT_EVENT_REDUCE_ENTRY": 0xD, "NPKIT_EVENT_REDUCE_EXIT": 0xE,
    "NPKIT_EVENT_LOCAL_COPY_ENTRY": 0xF, "NPKIT_EVENT_LOCAL_COPY_EXIT": 0x10,
    "NPKIT_EVENT_COPY_SEND_ENTRY": 0x11, "NPKIT_EVENT_COPY_SEND_EXIT": 0x12,
    "NPKIT_EVENT_DIRECT_COPY_SEND_ENTRY": 0x13, "NPKIT_EVENT_DIRECT_COPY_SEND_EXIT": 0x14,
    "NPKIT_EVENT_RECV_COPY_SEND_ENTRY": 0x15, "NPKIT_EVENT_RECV_COPY_SEND_EXIT": 0x16,
    "NPKIT_EVENT_DIRECT_RECV_COPY_SEND_ENTRY": 0x17, "NPKIT_EVENT_DIRECT_RECV_COPY_SEND_EXIT": 0x18,
    "NPKIT_EVENT_RECV_COPY_DIRECT_SEND_ENTRY": 0x19, "NPKIT_EVENT_RECV_COPY_DIRECT_SEND_EXIT": 0x1A,
    "NPKIT_EVENT_RECV_REDUCE_COPY_ENTRY": 0x1B, "NPKIT_EVENT_RECV_REDUCE_COPY_EXIT": 0x1C,
    "NPKIT_EVENT_RECV_REDUCE_SEND_ENTRY": 0x1D, "NPKIT_EVENT_RECV_REDUCE_SEND_EXIT": 0x1E,
    "NPKIT_EVENT_DIRECT_RECV_REDUCE_SEND_ENTRY": 0x1F, "NPKIT_EVENT_DIRECT_RECV_REDUCE_SEND_EXIT": 0x20,
    "NPKIT_EVENT_RECV_REDUCE_COPY_SEND_ENTRY": 0x21, "NPKIT_EVENT_RECV_REDUCE_COPY_SEND_EXIT": 0x22,
    "NPKIT_EVENT_DIRECT_RECV_REDUCE_COPY_SEND_ENTRY": 0x23, "NPKIT_EVENT_DIRECT_RECV_REDUCE_COPY_SEND_EXIT": 0x24,
    "NPKIT_EVENT_NET_SEND_ENTRY": 0x25, "NPKIT_EVENT_NET_SEND_EXIT": 0x26,
    "NPKIT_EVENT_NET_RECV_ENTRY": 0x27, "NPKIT_EVENT_NET_RECV_EXIT": 0x28,
    "NPKIT_EVENT_DEP_CHECK_ENTRY": 0x29, "NPKIT_EVENT_DEP_CHECK_EXIT": 0x2A,
    "NPKIT_EVENT_TIME_SYNC_GPU": 0x2B, "NPKIT_EVENT_TIME_SYNC_CPU": 0x2C,
}
NAMES = {v: k for k, v in EVENTS.items()}
GPU_BUFFERS, CPU_BUFFERS = 512, 32

# interpreter transfer type (algo.h numbering: s r rcs rrs rrc rrcs cpy re _ cs) -> the primitive's
# event name, <name>_ENTRY / <name>_EXIT (interpreter.h: nkPrim)
TRANSFER_EVENT = {0: "SEND", 1: "RECV", 2: "RECV_COPY_SEND", 3: "RECV_REDUCE_SEND", 4: "RECV_REDUCE_COPY",
                  5: "RECV_REDUCE_COPY_SEND", 6: "LOCAL_COPY", 7: "REDUCE", 9: "COPY_SEND"}


def parse_events(raw: bytes) -> List[dict]:
    """16-byte events: type u8, size u32, rsvd u24, timestamp u64 (npkit_struct.h:8-17)."""
    out = []
    for off in range(0, len(raw) - len(raw) % 16, 16):
        lo, ts = struct.unpack_from("<QQ", raw, off)
        out.append({"id": lo & 0xFF, "size": (lo >> 8) & 0xFFFFFFFF, "rsvd": lo >> 40, "timestamp": ts})
    return out


def read_buffer(dump_dir: str, rank: int, buf: int) -> List[dict]:
    with open(os.path.join(dump_dir, "gpu_events_rank_%d_buf_%d" % (rank, buf)), "rb") as f:
        return parse_events(f.read())


def _number(path: str) -> float:
    with open(path) as f:
        return float(f.read())


def _short_name(event: str) -> str:
    # NPKIT_EVENT_RECV_REDUCE_COPY_ENTRY -> RECV_REDUCE_COPY (one occurrence of each marker word)
    words = event.split("_")
    for w in ("NPKIT", "EVENT", "ENTRY"):
        if w in words:
            words.remove(w)
    return "_".join(words)


def _gpu_trace(events: List[dict], rank: int, buf: int, gpu_scale: float, cpu_scale: float) -> List[dict]:
    """One buffer's events on the host timeline: every launch opens with TIME_SYNC_CPU (host
    time) and TIME_SYNC_GPU (GPU clock at the same instant)."""
    out: List[dict] = []
    cpu_base = gpu_base = None
    seq: Dict[str, int] = {}
    for e in events:
        name = NAMES[e["id"]]
        if name == "NPKIT_EVENT_TIME_SYNC_CPU":
            cpu_base, gpu_base = e["timestamp"] / cpu_scale, None
            continue
        if name == "NPKIT_EVENT_TIME_SYNC_GPU":
            if gpu_base is None:
                gpu_base = e["timestamp"] / gpu_scale
            continue
        if gpu_base is None:
            gpu_base = e["timestamp"] / gpu_scale
        entry = name.endswith("_ENTRY")
        rec = {"ph": "B" if entry else "E", "ts": cpu_base + e["timestamp"] / gpu_scale - gpu_base,
               "pid": rank, "tid": buf + 1}
        if entry:
            k = seq.get(name, 0)
            seq[name] = k + 1
            rec.update({"name": _short_name(name), "cat": "GPU",
                        "args": {"rank": rank, "buf_idx": buf, "seq": k, "rsvd_0": e["rsvd"], "size_0": e["size"]}})
        else:
            dt = rec["ts"] - out[-1]["ts"]
            rec["args"] = {"size": e["size"], "rsvd": e["rsvd"],
                           "bw (GB/s)": e["size"] / dt / 1e3 if dt > 0 else 0.0}
        out.append(rec)
    return out


def _cpu_trace(events: List[dict], rank: int, channel: int, cpu_scale: float) -> List[dict]:
    """CPU (proxy) events, one 'fiber' per concurrently open slot.  The xGMI path writes these
    files empty (include/msccl_amd_npkit.h); kept for dumps that carry them."""
    out: List[dict] = []
    seq: Dict[str, int] = {}
    free: List[bool] = []
    opened: List[float] = []
    fiber_of: Dict[int, int] = {}
    for e in events:
        name = NAMES[e["id"]]
        entry = name.endswith("_ENTRY")
        rec = {"ph": "B" if entry else "E", "ts": e["timestamp"] / cpu_scale, "pid": rank}
        slot = e["rsvd"]
        if entry:
            fid = next((i for i, f in enumerate(free) if f), len(free))
            if fid == len(free):
                free.append(True)
                opened.append(0.0)
            fiber_of[slot] = fid
            opened[fid] = rec["ts"]
            free[fid] = False
            k = seq.get(name, 0)
            seq[name] = k + 1
            rec.update({"name": name, "cat": "CPU",
                        "args": {"rank": rank, "channel": channel, "slot": slot, "seq": k, "size_0": e["size"]}})
        else:
            fid = fiber_of.pop(slot)
            free[fid] = True
            dt = max(0.001, rec["ts"] - opened[fid])
            rec["args"] = {"size": e["size"], "bw (GB/s)": e["size"] / dt / 1e3}
        rec["tid"] = fid + (channel + 1) * 1000
        out.append(rec)
    return out


def to_trace(dump_dir: str) -> dict:
    """Chrome trace of a dump directory: GPU events of every (rank, buffer), CPU events of every
    (rank, channel), sorted by time (stable), displayTimeUnit ns."""
    files = next(os.walk(dump_dir))[2]
    gpu_files = [f for f in files if f.startswith("gpu_events_rank_")]
    cpu_files = [f for f in files if f.startswith("cpu_events_rank_")]
    ranks = list(set(int(re.match(r"gpu_events_rank_(\d+)_", f).group(1)) for f in gpu_files))
    bufs = list(set(int(re.search(r"_buf_(\d+)", f).group(1)) for f in gpu_files))
    channels = list(set(int(re.search(r"_channel_(\d+)", f).group(1)) for f in cpu_files))
    events: List[dict] = []
    for rank in ranks:
        cpu_scale = (_number(os.path.join(dump_dir, "cpu_clock_period_den_rank_%d" % rank)) /
                     _number(os.path.join(dump_dir, "cpu_clock_period_num_rank_%d" % rank)) / 1e6)
        gpu_scale = _number(os.path.join(dump_dir, "gpu_clock_rate_rank_%d" % rank)) * 1e3 / 1e6
        for b in bufs:
            events.extend(_gpu_trace(read_buffer(dump_dir, rank, b), rank, b, gpu_scale, cpu_scale))
        for c in channels:
            with open(os.path.join(dump_dir, "cpu_events_rank_%d_channel_%d" % (rank, c)), "rb") as f:
                events.extend(_cpu_trace(parse_events(f.read()), rank, c, cpu_scale))
    events.sort(key=lambda x: x["ts"])
    return {"traceEvents": events, "displayTimeUnit": "ns"}


def main(argv=None) -> None:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--input_dir", default="/tmp", help="NPKit dump directory")
    ap.add_argument("--output_dir", required=True)
    a = ap.parse_args(argv)
    os.makedirs(a.output_dir, exist_ok=True)
    with open(os.path.join(a.output_dir, "npkit_event_trace.json"), "w") as f:
        json.dump(to_trace(a.input_dir), f)


if __name__ == "__main__":
    main()
