#!/usr/bin/env python3
"""AllReduce bus-bandwidth benchmark for the MI355X MSCCL runtime (nccl-tests all_reduce_perf style).

Metric (BASELINE.json): AllReduce bus-BW GB/s, device-resident, 128 B - 32 MiB sweep, with
busBW = (S / t) * 2(n-1)/n (nccl-tests convention used by the reference README:57).

  python bench.py                      # N=1: config C2 = 2-rank all-pairs LL fp32 AllReduce, both
                                       # ranks co-resident on cuda:0 (one fused launch per step)
  torchrun --nproc-per-node N bench.py --gpus N   # one rank per GPU, all-pairs LL over xGMI
                                       # (fp32; fp16 at N=8 = config C3)

A "step" is one AllReduce of S bytes per rank on every rank.  `value` is the bus bandwidth at
the largest size of the sweep (32 MiB); the whole sweep is in `sweep`.  Inputs are resident in
HBM before the timed region.  rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import msccl_amd as M  # noqa: E402
from msccl_amd import xmlgen  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
XGMI_LINK_GBS = 153.0          # task statement, per link (see DESIGN.md calibration note)
SIZES = [128 << k for k in range(19)]  # 128 B .. 32 MiB


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs, one rank each (default 1: config C2 with 2 ranks co-resident on cuda:0). "
                         "Without torch.distributed.run's WORLD_SIZE, N > 1 starts N rank processes itself")
    ap.add_argument("--steps", type=int, default=100, help="timed steps per size (one hipGraph of K launches; 100 keeps the graph launch under 0.2 us per step)")
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--vranks", type=int, default=2, help="co-resident ranks at --gpus 1 (config C2: 2)")
    ap.add_argument("--proto", default="LL")
    ap.add_argument("--dtype", default=None)
    ap.add_argument("--instances", type=int, default=0, help="all-pairs instances for large sizes (0 = auto)")
    ap.add_argument("--tiers", default=None, help="schedule tiers lo:hi:instances,... (default: see make_xmls)")
    ap.add_argument("--sizes", default=None, help="comma list of bytes (default 128B..32MiB)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--e2e", action="store_true", help="also time H2D + AllReduce + D2H")
    ap.add_argument("--eager", action="store_true",
                    help="launch the K timed steps one by one from Python (default: capture them into one hipGraph "
                         "and time its replay, as the reference's nccl-tests run does with -G 100, README.md:57)")
    ap.add_argument("--extras", default=None,
                    help="also measure C4 (ring Simple bf16 256 MiB) / C5 (RS+AG fp32 64 MiB), e.g. C4,C5 "
                         "(default: both when 8 ranks run one per GPU)")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the secondary schedule lines (msccl-tools two-phase all-pairs, RCCL 8n-32tb)")
    ap.add_argument("--pmc", default="auto", choices=("auto", "off"),
                    help="auto: at N=1 measure the headline launch's HBM traffic with two rocprofv3 PMC "
                         "passes (FETCH_SIZE, WRITE_SIZE) of a headline-only child run")
    ap.add_argument("--no-tuning", action="store_true",
                    help="at --gpus N > 1 skip the tuning keys (run_tuning: lowering caps, Simple FIFO sizes, link rate)")
    ap.add_argument("--quiet", action="store_true")
    return ap.parse_args(argv)


def launch_plan(gpus, env, device_count):
    """How `bench.py --gpus N` runs (the reference's harness is `mpirun -np 8 ... all_reduce_perf
    -g 1`, README.md:57: one process per GPU).  Returns (mode, detail):
      ("rank", W)     started by torch.distributed.run (WORLD_SIZE = W > 1): this process is one rank
      ("local", 1)    N = 1: config C2, its 2 ranks co-resident on cuda:0, one process
      ("spawn", N)    N > 1 without WORLD_SIZE: start N rank processes (torch.distributed.run),
                      relay rank 0's line; this process never touches the GPU
      ("refuse", msg) fewer GPUs than ranks (MSCCL_AMD_BENCH_ONE_GPU=1 rehearses N processes on
                      cuda:0 instead), or --gpus disagreeing with WORLD_SIZE
    `device_count` is torch.cuda.device_count(), which does not initialise the GPU."""
    one_gpu = env.get("MSCCL_AMD_BENCH_ONE_GPU") == "1"
    world = int(env.get("WORLD_SIZE", "1") or "1")
    if world > 1:
        if gpus is not None and gpus != world:
            return "refuse", "--gpus %d but WORLD_SIZE=%d" % (gpus, world)
        if device_count < world and not one_gpu:
            return "refuse", ("%d ranks need %d GPUs, %d visible (MSCCL_AMD_BENCH_ONE_GPU=1 rehearses them "
                              "on one GPU)" % (world, world, device_count))
        return "rank", world
    n = gpus or 1
    if n <= 1:
        return "local", 1
    if device_count < n and not one_gpu:
        return "refuse", ("--gpus %d needs %d GPUs, %d visible (MSCCL_AMD_BENCH_ONE_GPU=1 rehearses %d "
                          "processes on one GPU)" % (n, n, device_count, n))
    return "spawn", n


def spawn_ranks(n: int, argv) -> int:
    """Start n rank processes with torch.distributed.run on 127.0.0.1 and wait for them; their
    stdout (rank 0's JSON line) is this process's.  Returns the launcher's exit code."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)
    return subprocess.call(cmd)


def schedule_bytes(algo: dict, size_per: int, ts: int, proto: int, payload_only: bool = False, fused=(),
                   l2_reuse: bool = True):
    """Algorithmic HBM bytes and wire bytes of one launch for one rank (whole schedule).
    payload_only counts FIFO traffic at its payload size (LL flags / LL128 flag words excluded).
    fused: thread blocks whose s + rrc exchange ran fused (comm info "algoFuse"): the rrc reuses
    the source the s read, one read of B less.
    l2_reuse: the same source chunks sent by several thread blocks of the launch (one block to k
    peers: an all-pairs AllGather, the two-phase AllReduce's reduced chunk) are read from HBM once;
    the other k - 1 reads are served by L2 (PMC: the 8-rank AllGather read 0.775x and the C3 shape
    0.947x of the byte model that counted every read, profiles/r03_extras8_pmc.json)."""
    f = 1.0 if payload_only else {0: 2.0, 1: 4.0 / 3.0}.get(proto, 1.0)  # LL: 8 B data per 16-B line
    hbm = wire = 0
    sent = set()
    for b_i, tb in enumerate(algo["tbs"]):
        first_s = b_i in fused and proto == 0
        for t in tb["transfers"]:
            typ, cnt, nred = t[0], t[5], t[10]
            b = cnt * size_per * ts
            if typ == 0:      # s
                hbm += b + f * b; wire += f * b
                key = (t[1], t[2], cnt)
                if first_s:
                    hbm -= b
                    first_s = False
                elif l2_reuse and key in sent:
                    hbm -= b
                sent.add(key)
            elif typ == 1:    # r
                hbm += f * b + b
            elif typ == 2:    # rcs
                hbm += f * b + b + f * b; wire += f * b
            elif typ == 3:    # rrs
                hbm += f * b + b + f * b; wire += f * b
            elif typ == 4:    # rrc
                hbm += f * b + b + b
            elif typ == 5:    # rrcs
                hbm += f * b + b + b + f * b; wire += f * b
            elif typ == 6:    # cpy
                hbm += 2 * b
            elif typ == 7:    # re
                hbm += (nred + 1) * b + b
    return int(round(hbm)), int(round(wire))


KERNEL_NAMES = {0: "mscclKernel", 1: "mscclSmallKernel", 2: "mscclFoldKernel (lowered)",
                3: "mscclPairKernel", 4: "mscclTwoPhaseKernel (lowered)", 5: "mscclDirectKernel (direct form)"}


def kernel_name(last: dict) -> str:
    """The kernel a communicator's last launch ran (comm info "last", enqueue.cc: launchGroup)."""
    k = last.get("kernel", -1)
    if k == 3 and last.get("ringColl") == 5:
        return "mscclPairKernel (lowered)"
    if k == 1 and last.get("set") == 1:
        return "mscclSmallKernel<exchange set>"
    return KERNEL_NAMES.get(k, "mscclKernel")


def lowered_bytes(last: dict, n: int, nbytes: int):
    """(HBM bytes, wire bytes, payload-only HBM bytes) of one rank's lowered launch (LL lines: 16 B
    per 8-B payload), or None when the launch ran the schedule as written (schedule_bytes then):
      fold (kernel 2): the input read once, lines to and from each of the n - 1 peers, the result;
      lowered pair (kernel 3 on the flat connections): S read, 2 S of lines out, 2 S in, S written;
      two-phase (kernel 4): per (n - 1)/n S of peer-owned data: read, lines out (A), lines in and
        the owner's result lines in (C), written; per S/n owned: read, the peers' lines in (B),
        written, result lines out: (10 (n - 1) + 2) / n S (9 S at 8 ranks, 6 S at 2)."""
    k = last.get("kernel", -1)
    if k == 2:
        return (int(2 * nbytes + 2 * 2.0 * (n - 1) * nbytes), int(2.0 * (n - 1) * nbytes),
                int(2 * nbytes + 2 * (n - 1) * nbytes))
    if k == 3 and last.get("ringColl") == 5:
        return 6 * nbytes, 2 * nbytes, 4 * nbytes
    if k == 4:
        return (int(round((10 * (n - 1) + 2) * nbytes / n)), int(round(4 * (n - 1) * nbytes / n)),
                int(round((6 * (n - 1) + 2) * nbytes / n)))
    return None


PAIR_TIERS = "0:4096:1:p,4096:1073741825:16:p"   # the 2-rank pair one-shot tiers of rounds 2-5


def make_xmls(n: int, proto: str, inst_large: int, tmp: str, tiers_arg=None, remote: bool = False):
    """All-pairs schedules in size tiers, as a user registers several msccl-tools XMLs with
    minBytes/maxBytes (MSCCL_XML_FILES, at most 4): [(lo, hi, instances, path, kind)].  At 2
    ranks the two-phase all-pairs, one instance below 4 KiB and inst_large above.  At more ranks:
    rank-ordered one-shot (4 instances; lowered to the one-hop fold) below 64 KiB, then two-phase
    all-pairs with 4 instances below 4 MiB and inst_large above.  remote (one rank per GPU, peers
    over xGMI): inst_large from 64 KiB on."""
    if tiers_arg:
        # lo:hi:instances[:kind], kind "a" = two-phase all-pairs (default), "o" = one-shot,
        # "O" = rank-ordered one-shot, "p" = 2-rank one-hop exchange (s, rrc), "r" = ring with
        # `instances` channels (for 2 ranks the fused all-pairs exchange s, rrcs, r)
        spec = []
        for t in tiers_arg.split(","):
            f = t.split(":")
            spec.append((int(f[0]), int(f[1]), int(f[2])) + ((f[3],) if len(f) > 3 else ()))
    elif n <= 2:
        # Two ranks: the msccl-tools two-phase all-pairs XML itself (the north star's schedule),
        # one instance below 4 KiB, inst_large above.  The runtime lowers it at upload
        # (msccl_amd/csrc/lower.cc): calls up to 4 KiB run the one-hop fold, larger ones the pair
        # exchange on the flat connections (6 S HBM bytes per rank against the schedule's 7.5 S),
        # with the schedule's values.  Same box, driver form (--steps 20), against the pair
        # one-shot XML (PAIR_TIERS, rounds 2-5): 32 MiB 535.4 -> 546.8 GB/s, sweep average
        # 116.4 -> 120.8 (profiles/r06g_c2_pair.json, r06g_c2_allpairs.json)
        spec = [(0, 4 << 10, 1, "a"), (4 << 10, (1 << 30) + 1, inst_large, "a")]
    else:
        # rank-ordered one-shot (s, r, re, cpy; the same bits on every rank) below 64 KiB: the
        # runtime lowers it to the one-hop fold there (msccl_amd/csrc/lower.cc), which beats the
        # two-phase all-pairs up to that size (8 ranks, fp16, graph replay: 16 KiB 18.8 -> 12.7 us,
        # 64 KiB 23.1 -> 16.0; profiles/r04b_xover.txt); the two-phase schedule takes over above
        # (lowered too up to 128 KiB: profiles/r04t_lat.txt)
        # two instance counts: up to 4 below 4 MiB (8 ranks: 128 KiB 17.9 against 21.1 us with 8,
        # 512 KiB 24.1 against 26.5), inst_large from 4 MiB (32 MiB 538 against 570 us,
        # profiles/r04o_c3_inst.txt)
        # profiles/r04o_c3_inst.txt).  Those counts are set by 8 ranks sharing one GPU's CUs; with
        # one rank per GPU a rank's workgroups have its GPU to themselves and each thread block
        # drives one xGMI link, so the mid tier takes inst_large too (8 thread blocks per link)
        mid = inst_large if remote else min(4, inst_large)
        spec = [(0, 64 << 10, 4, "O"), (64 << 10, 4 << 20, mid), (4 << 20, (1 << 30) + 1, inst_large)]
    tiers = []
    for k, t in enumerate(spec):
        lo, hi, inst = t[:3]
        kind = t[3] if len(t) > 3 else "a"
        if kind in ("o", "O"):
            x = xmlgen.allreduce_oneshot(n, inst, proto, lo, hi, name="oneshot_t%d_i%d" % (k, inst),
                                         ordered=kind == "O")
        elif kind == "p":
            x = xmlgen.allreduce_pair_oneshot(inst, proto, True, lo, hi, name="pair_t%d_i%d" % (k, inst))
        elif kind == "r":
            x = xmlgen.allreduce_ring(n, inst, proto, True, lo, hi, name="ring_t%d_i%d" % (k, inst))
        else:
            x = xmlgen.allreduce_allpairs(n, inst, proto, True, lo, hi, name="allpairs_t%d_i%d" % (k, inst))
        pth = os.path.join(tmp, "bench_ap%d_%s_t%d_i%d_%s_%d.xml" % (n, proto, k, inst, kind, os.getpid()))
        open(pth, "w").write(x)
        tiers.append((lo, hi, inst, pth, kind))
    return tiers


def tier_of(tiers, nbytes):
    for t in tiers:
        if t[0] <= nbytes < t[1]:
            return t
    raise ValueError("no schedule tier for %d bytes" % nbytes)


def cpu_baseline(n: int, nbytes: int, dt: int, seconds: float):
    """Time oracle/cpu_allreduce.c (OpenMP) on a bounded sample: repeated n-rank AllReduces."""
    libp = os.path.join(ROOT, "oracle", "build", "libcpu_allreduce.so")
    if not os.path.exists(libp):
        return None
    lib = ctypes.CDLL(libp)
    ts = M.TYPE_SIZE[dt]
    cnt = nbytes // ts
    bufs = [np.random.default_rng(r).standard_normal(cnt).astype(np.float32 if dt == M.FLOAT32 else np.float16)
            if dt != M.BFLOAT16 else np.zeros(cnt, np.uint16) for r in range(n)]
    ptrs = (ctypes.c_void_p * n)(*[b.ctypes.data for b in bufs])
    chunk = max(1, cnt // (n * n))
    threads = lib.cpu_allreduce_allpairs(ptrs, n, ctypes.c_long(cnt), ctypes.c_long(chunk), dt)
    reps = 0
    t0 = time.perf_counter()
    while True:
        lib.cpu_allreduce_allpairs(ptrs, n, ctypes.c_long(cnt), ctypes.c_long(chunk), dt)
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    t = el / reps
    bus = nbytes / t * 2 * (n - 1) / n / 1e9
    return {"value": round(bus, 3), "unit": "GB/s", "cores": int(threads), "kind": "port",
            "sample": "%d x %d-rank all-pairs-order AllReduce of %d B %s per rank (oracle/cpu_allreduce.c, "
                      "OpenMP, %.1f s)" % (reps, n, nbytes, {7: "fp32", 6: "fp16", 9: "bf16"}[dt], el),
            "ms_per_allreduce": round(t * 1e3, 4)}


def config_id(n: int, proto: str, dtname: str) -> str:
    """The BASELINE.json config an all-pairs AllReduce sweep of n ranks is: C2 (2 ranks, LL, fp32),
    C3 (8 ranks, LL, fp16), or none ("" : a shape of its own)."""
    if proto == "LL" and n == 2 and dtname == "fp32":
        return "C2"
    if proto == "LL" and n == 8 and dtname == "fp16":
        return "C3"
    return ""


SCHEDULE_NAMES = {"a": "msccl-tools two-phase all-pairs XML", "o": "one-shot all-pairs XML",
                  "O": "rank-ordered one-shot all-pairs XML", "p": "pair one-shot XML (s, rrc; not all-pairs)",
                  "r": "ring XML"}


def workload_desc(multi: bool, n: int, proto: str, dtname: str, one_gpu: bool = False, kind: str = "a") -> str:
    """The workload label: the config, the schedule the headline size actually ran (kind: its
    tier's, make_xmls), the placement."""
    cid = config_id(n, proto, dtname)
    sched = SCHEDULE_NAMES[kind]
    if not multi:
        return ("%s%d-rank %s AllReduce through the %s, %s, ranks co-resident on one MI355X "
                "(fused launch, local HBM in place of xGMI)"
                % ((cid + ": ") if cid == "C2" else (cid + " shape: ") if cid else "", n, proto, sched, dtname))
    if one_gpu:
        return ("rehearsal: %d rank processes sharing one MI355X (hipIpc FIFOs, local HBM in place of "
                "xGMI), %s AllReduce through the %s, %s" % (n, proto, sched, dtname))
    return ("%s: %d-rank %s AllReduce through the %s over xGMI, %s, one rank per GPU"
            % (cid or "%d-GPU" % n, n, proto, sched, dtname))


TIER_KINDS = {"a": "allreduce_allpairs (two-phase: s, r, re, s, r; msccl-tools form)",
              "o": "allreduce_oneshot", "O": "allreduce_oneshot (rank-ordered)",
              "p": "allreduce_pair_oneshot (s, rrc per thread block)", "r": "allreduce_ring"}


def pmc_traffic(cfg_key: dict, src_hash: str):
    """HBM bytes per headline launch from the committed rocprofv3 PMC summary of the same
    configuration (tools/profile.sh -> profiles/<tag>_pmc.json) taken on the same device sources
    (its "kernel_src" stamp equals kernel_src_hash()), or (None, None)."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc.json")), reverse=True):
        try:
            pmc = json.load(open(f))
            bench = json.load(open(f.replace("_pmc.json", "_bench.json")))
        except (OSError, ValueError):
            continue
        c = bench.get("config", {})
        if pmc.get("kernel_src") != src_hash:
            continue
        if all(c.get(k, {} if k == "knobs" else None) == v for k, v in cfg_key.items()) and pmc.get("traffic_bytes_per_launch"):
            return round(pmc["traffic_bytes_per_launch"]), os.path.relpath(f, ROOT)
    return None, None


_STREAMS = {}


def bench_stream(dev):
    """One collective stream per device for the whole run: every part of the bench launches on it.
    A stream is a hardware queue; rank processes that share one GPU (the one-GPU rehearsal) and
    each hold several would oversubscribe the GPU's queues, which the command processor then
    time-slices (about 11 ms per slice, profiles/r06h_rehearse_8.json)."""
    import torch
    key = str(dev)
    if key not in _STREAMS:
        _STREAMS[key] = torch.cuda.Stream(dev)
    s = _STREAMS[key]
    s.wait_stream(torch.cuda.current_stream(dev))
    return s


def init_comms(multi: bool, world: int, rank: int, n: int):
    """Communicators for the current MSCCL_XML_FILES: one per process (multi) or n co-resident."""
    if multi:
        import torch.distributed as dist
        obj = [M.get_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        return [M.Comm.init_rank(world, obj[0], rank)]
    return M.Comm.init_all([0] * n)


def run_extra(cfg: str, a, multi: bool, world: int, rank: int, n: int, tmp: str) -> dict:
    """BASELINE.json configs[3] (C4: ring AllReduce, Simple, bf16, 256 MiB per rank) and
    configs[4] (C5: all-pairs ReduceScatter then AllGather, fp32, 64 MiB total)."""
    import torch
    dev = torch.device("cuda", torch.cuda.current_device())
    if cfg == "C4":
        # 32 rings (the reference's MAXCHANNELS) over the xGMI-disjoint Hamiltonian cycles of
        # xmlgen.allreduce_ring: 2 co-resident ranks, 256 MiB bf16: 180 GB/s with 2 rings, 645 with 32
        chans = int(os.environ.get("MSCCL_AMD_BENCH_C4_CHANNELS", "0")) or 32
        xmls = {"ar": xmlgen.allreduce_ring(n, chans, "Simple", True, 0, 1 << 40, name="c4_ring")}
        dt, S = M.BFLOAT16, 256 << 20
    elif cfg == "C5":
        # 2 ranks: 16 instances (RS 126 -> 243, AG 225 -> 373 GB/s against 4); up to 8 ranks: 8
        # (8 co-resident ranks: AG 0.280 against 0.298 ms with 4, RS within noise,
        # profiles/r04r_c4knobs.txt); beyond, as many as keep n (n - 1) x instances thread blocks
        # resident when the ranks share one GPU
        c5i = int(os.environ.get("MSCCL_AMD_BENCH_C5_INSTANCES", "0")) or (
            16 if n <= 2 else 8 if n <= 8 else max(1, 512 // (n * (n - 1))))
        rs_form = os.environ.get("MSCCL_AMD_BENCH_RS_FORM", "chain")   # "scratch": the round-2 form
        xmls = {"rs": xmlgen.reduce_scatter_allpairs(n, c5i, "Simple", False, 0, 1 << 40, name="c5_rs", form=rs_form),
                "ag": xmlgen.allgather_allpairs(n, c5i, "Simple", False, 0, 1 << 40, name="c5_ag")}
        dt, S = M.FLOAT32, 64 << 20
    elif cfg == "FB":
        # ring fallback (enqueue.cc:461-476): 32 MiB + one element matches no all-pairs schedule
        xmls = {"ap": xmlgen.allreduce_allpairs(n, 1, "LL", True, 0, 1 << 40, name="fb_ap")}
        dt, S = M.FLOAT32, (32 << 20) + 4
    else:
        raise ValueError(cfg)
    paths = []
    for k, x in xmls.items():
        pth = os.path.join(tmp, "bench_%s_%s_%d.xml" % (cfg, k, os.getpid()))
        open(pth, "w").write(x)
        paths.append(pth)
    os.environ["MSCCL_XML_FILES"] = ":".join(paths)
    # algorithmic HBM bytes of one launch on this GPU, summed over the ranks it runs (schedule_bytes)
    ranks_here = [rank] if multi else list(range(n))

    def launch_bytes(path, coll_count, mult, ts_):
        tot = 0
        for r in ranks_here:
            al = M.algo_json(path, r, n)
            size_per = coll_count * mult // al["nchunksperloop"]
            tot += schedule_bytes(al, size_per, ts_, al["proto"])[0]
        return tot

    def note(msg):
        if rank == 0 and not a.quiet:
            print("# %s: %s" % (cfg, msg), file=sys.stderr, flush=True)
    note("init %d ranks" % n)
    comms = init_comms(multi, world, rank, n)
    note("init done")
    ts = M.TYPE_SIZE[dt]
    stream = bench_stream(dev)
    nloc = len(comms)
    try:
        ranks = [rank] if multi else list(range(n))
        tdt = {M.BFLOAT16: torch.bfloat16, M.FLOAT32: torch.float32}[dt]

        def pattern(r, cnt):
            j = torch.arange(cnt, device=dev, dtype=torch.int64)
            return ((j * 5 + r * 3 + (j >> 7)) % 9 - 4).to(tdt)

        def agree(good):
            if multi:
                g = torch.tensor([1 if good else 0], dtype=torch.int32)
                torch.distributed.all_reduce(g, op=torch.distributed.ReduceOp.MIN)
                good = bool(g.item())
            return good

        if cfg in ("C4", "FB"):
            cnt = S // ts
            bufs = [torch.zeros((S + 1) // 2, dtype=torch.int16, device=dev) for _ in range(nloc)]

            def step():
                with M.group():
                    for c, b in zip(comms, bufs):
                        c.all_reduce(b.data_ptr(), b.data_ptr(), cnt, dt, M.SUM, stream.cuda_stream)

            def check():
                for r, b in zip(ranks, bufs):
                    b.view(torch.uint8)[:S].view(tdt).copy_(pattern(r, cnt))
                want = sum(pattern(r, cnt).float() for r in range(n)).to(tdt)
                torch.cuda.synchronize()
                step()
                torch.cuda.synchronize()
                return agree(all(torch.equal(b.view(torch.uint8)[:S].view(tdt), want) for b in bufs))
            # the direct form (kernel 5, lower.h: DirectLowering): every rank reads S and writes S
            phases = {"allreduce": (step, S * 2 * (n - 1) / n, launch_bytes(paths[0], cnt, 1, ts), 2 * S * nloc)}
        else:
            rc = S // ts // n
            ins = [torch.empty(S // 4, dtype=torch.float32, device=dev).uniform_(-1, 1) for _ in range(nloc)]
            mids = [torch.empty(rc, dtype=torch.float32, device=dev) for _ in range(nloc)]
            outs = [torch.empty(S // 4, dtype=torch.float32, device=dev) for _ in range(nloc)]

            def rs():
                with M.group():
                    for c, i, m in zip(comms, ins, mids):
                        c.reduce_scatter(i.data_ptr(), m.data_ptr(), rc, dt, M.SUM, stream.cuda_stream)

            def ag():
                with M.group():
                    for c, m, o in zip(comms, mids, outs):
                        c.all_gather(m.data_ptr(), o.data_ptr(), rc, dt, stream.cuda_stream)

            def check():
                for r, i in zip(ranks, ins):
                    i.copy_(pattern(r, S // 4))
                full = sum(pattern(r, S // 4).float() for r in range(n))
                torch.cuda.synchronize()
                rs()
                ag()
                torch.cuda.synchronize()
                good = all(torch.equal(m, full[r * rc:(r + 1) * rc]) for r, m in zip(ranks, mids))
                return agree(good and all(torch.equal(o, full) for o in outs))
            # direct forms: the ReduceScatter reads every rank's block and writes its own ((n + 1) S / n
            # per rank), the AllGather reads its block once and writes it n times (the same)
            phases = {"reduce_scatter": (rs, S * (n - 1) / n, launch_bytes(paths[0], rc, n, ts), (n + 1) * (S // n) * nloc),
                      "all_gather": (ag, S * (n - 1) / n, launch_bytes(paths[1], rc * ts, n, 1), (n + 1) * (S // n) * nloc)}
        res = {}
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for name, (fn, busbytes, algo_bytes, direct_bytes) in phases.items():
            note("%s warmup" % name)
            for _ in range(max(1, a.warmup)):
                fn()
            if multi:
                torch.distributed.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ev0.record(stream)
            k = max(1, min(a.steps, 10))
            for _ in range(k):
                fn()
            ev1.record(stream)
            torch.cuda.synchronize()
            if multi:
                torch.distributed.barrier()
            t = (time.perf_counter() - t0) / k
            ev_ms = ev0.elapsed_time(ev1) / k
            if multi:
                tt = torch.tensor([t, ev_ms], dtype=torch.float64)
                torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
                t, ev_ms = float(tt[0]), float(tt[1])
            if any(c.async_error() != 0 for c in comms):
                raise RuntimeError("kernel reported an error (timeout/abort)")
            last = comms[0].info()["last"]
            if last.get("kernel") == 5:
                algo_bytes = direct_bytes
            res[name] = {"ms": round(t * 1e3, 4), "kernel_ms": round(ev_ms, 4), "kernel": kernel_name(last),
                         "busbw": round(busbytes / t / 1e9, 3), "steps": k,
                         # roofline: algorithmic bytes of the launch on this GPU / its event time,
                         # against the 8 TB/s HBM peak.  Memory-side: FIFO slots and re-read blocks
                         # stay in the L2 / MALL, so the rate can exceed what the HBM array delivers
                         # (a float4 device copy reaches 6.29 TB/s, MI355X_MICROARCH.md)
                         "algorithmic_bytes_per_launch": algo_bytes,
                         "memside_frac": round(algo_bytes / (ev_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4)}
            note("%s %.3f ms, busbw %.1f GB/s" % (name, t * 1e3, busbytes / t / 1e9))
        res["memside_frac_note"] = ("algorithmic bytes / kernel time / 8 TB/s, L2 / MALL hits included: above "
                                    "0.79 (the 6.29 TB/s device-copy rate) it is not an HBM-array fraction")
        res["verified"] = check()
        res["bytes"] = S
        res["dtype"] = {M.BFLOAT16: "bf16", M.FLOAT32: "f32"}[dt]
        res["ranks"] = n
        res["schedule"] = {"C4": "allreduce_ring x%d Simple" % chans if cfg == "C4" else "",
                           "C5": "reduce_scatter_allpairs (%s) + allgather_allpairs x%d Simple" % (rs_form, c5i)
                                 if cfg == "C5" else "",
                           "FB": "ring fallback (no schedule matches)"}[cfg]
        return res
    finally:
        for c in comms:
            c.destroy()


TUNE_SIZES = (64 << 10, 128 << 10, 256 << 10, 512 << 10, 1 << 20)
TUNE_LOWER_CAPS = (128 << 10, 256 << 10, 512 << 10)
TUNE_BUFFSIZES = (256 << 10, 4 << 20)


def run_tuning(a, world: int, rank: int, n: int, tmp: str, dt: int, headline_xmls: str, sweep, xgmi_cal,
               one_gpu: bool) -> dict:
    """bench.py --gpus N (N > 1, one rank per process): the data that sets the defaults tuned on
    co-resident ranks for one rank per GPU, in bounded extra keys of the line:
      lower_max_bytes  the headline's schedules at 64 KiB - 1 MiB with MSCCL_AMD_LOWER_MAX_BYTES
                       = 128 / 256 / 512 KiB and with the default (plan.h: defaultLowerMaxBytes,
                       the link model's crossover): where the lowered one-hop fold stops paying;
      buffsize         (N = 8) C4 / C5 with NCCL_BUFFSIZE = 256 KiB / 4 MiB (the Simple FIFO,
                       4 MiB by default towards other GPUs);
      link             the one-way cuda:0 -> cuda:1 copy rate and the 128 B AllReduce time (an
                       upper bound of the hop latency L the §8b model assumes to be 2 us).
    Every size is timed like the sweep (K steps in one hipGraph, barrier + max over ranks) and
    checked once on exact integers; C4 / C5 as the configs key times them."""
    import torch
    dev = torch.device("cuda", torch.cuda.current_device())
    ts = M.TYPE_SIZE[dt]
    tdt = {M.FLOAT32: torch.float32, M.FLOAT16: torch.float16, M.BFLOAT16: torch.bfloat16}[dt]
    k = max(1, min(a.steps, 20))
    out = {"steps": k, "lower_max_bytes": {}}
    buf = torch.empty(max(TUNE_SIZES) // ts, dtype=tdt, device=dev).uniform_(-1, 1)
    stream = bench_stream(dev)
    stream.wait_stream(torch.cuda.current_stream(dev))

    def maxed(vals):
        tt = torch.tensor(vals, dtype=torch.float64)
        torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
        return [float(v) for v in tt]

    saved = {v: os.environ.get(v) for v in ("MSCCL_AMD_LOWER_MAX_BYTES", "NCCL_BUFFSIZE", "MSCCL_XML_FILES")}
    try:
        os.environ["MSCCL_XML_FILES"] = headline_xmls
        for cap in (None,) + TUNE_LOWER_CAPS:
            if cap is None:
                os.environ.pop("MSCCL_AMD_LOWER_MAX_BYTES", None)
            else:
                os.environ["MSCCL_AMD_LOWER_MAX_BYTES"] = str(cap)
            comm = init_comms(True, world, rank, n)[0]
            rows = {}
            try:
                for nbytes in TUNE_SIZES:
                    cnt = nbytes // ts

                    def step():
                        comm.all_reduce(buf.data_ptr(), buf.data_ptr(), cnt, dt, M.SUM, stream.cuda_stream)
                    for _ in range(max(1, a.warmup)):
                        step()
                    # the sweep's timing: the K steps captured into one hipGraph, replayed once
                    # untimed, then timed (a rank's launches do not wait on its host)
                    torch.cuda.synchronize()
                    graph = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(graph, stream=stream, capture_error_mode="relaxed"):
                        for _ in range(k):
                            step()
                    with torch.cuda.stream(stream):
                        graph.replay()
                    torch.cuda.synchronize()
                    torch.distributed.barrier()
                    t0 = time.perf_counter()
                    with torch.cuda.stream(stream):
                        graph.replay()
                    torch.cuda.synchronize()
                    torch.distributed.barrier()
                    t = maxed([(time.perf_counter() - t0) / k])[0]
                    del graph
                    if comm.async_error() != 0:
                        raise RuntimeError("kernel reported an error at %d bytes" % nbytes)
                    last = comm.info()["last"]
                    j = torch.arange(cnt, device=dev, dtype=torch.int64)
                    buf[:cnt].copy_((((j * 7 + rank * 3 + (j >> 5)) % 9) - 4).to(tdt))
                    want = sum((((j * 7 + r * 3 + (j >> 5)) % 9) - 4).float() for r in range(n)).to(tdt)
                    torch.cuda.synchronize()
                    step()
                    torch.cuda.synchronize()
                    good = maxed([0.0 if torch.equal(buf[:cnt], want) else 1.0])[0] == 0.0
                    rows[str(nbytes)] = {"us": round(t * 1e6, 2), "kernel": kernel_name(last), "verified": good}
            finally:
                comm.destroy()
            out["lower_max_bytes"]["default" if cap is None else str(cap)] = rows
        os.environ.pop("MSCCL_AMD_LOWER_MAX_BYTES", None)
        if world == 8:
            out["buffsize"] = {}
            for bs in TUNE_BUFFSIZES:
                os.environ["NCCL_BUFFSIZE"] = str(bs)
                row = {}
                for cfg in ("C4", "C5"):
                    try:
                        r = run_extra(cfg, a, True, world, rank, n, tmp)
                        row[cfg] = {p: r[p]["kernel_ms"] for p in ("allreduce", "reduce_scatter", "all_gather") if p in r}
                        row[cfg]["verified"] = r["verified"]
                    except Exception as e:  # noqa: BLE001  (reported, the headline stands)
                        row[cfg] = {"error": str(e)[:200]}
                out["buffsize"][str(bs)] = row
    finally:
        for v, x in saved.items():
            if x is None:
                os.environ.pop(v, None)
            else:
                os.environ[v] = x
    out["link"] = {"copy_gbs_0_to_1": xgmi_cal,
                   "copy_note": None if xgmi_cal is not None else
                   ("ranks share one GPU (rehearsal): no link to measure" if one_gpu else "peer copy failed"),
                   "allreduce_%dB_us" % sweep[0]["bytes"]: round(sweep[0]["ms"] * 1e3, 2)}
    out["verified"] = all(r["verified"] for rows in out["lower_max_bytes"].values() for r in rows.values()) and \
        all(c.get("verified", False) for row in out.get("buffsize", {}).values() for c in row.values())
    return out


RCCL_32TB = "/opt/rocm/share/rccl/msccl-algorithms/allreduce-allpairs-8n-ll-32tb.xml"


def secondary_schedules(multi: bool, n: int, nbytes: int):
    """The north star's number is "for the all-pairs XML schedule": next to the headline tier, the
    same AllReduce through (1) the msccl-tools two-phase all-pairs form (xmlgen.allreduce_allpairs,
    the shape of the RCCL-shipped allreduce-allpairs-8n XMLs) at the headline's ranks and size, and
    (2) at N=1 the RCCL-shipped 8n-32tb LL schedule itself on 8 co-resident ranks, fp16 (config C3's
    shape; maxBytes raised from 64 KiB so it admits 32 MiB, as tests/test_gpu_configs.py does).
    At 2 ranks the headline already runs the two-phase all-pairs XML: the line beside it is the
    pair one-shot XML (xmlgen.allreduce_pair_oneshot x16, the headline schedule of rounds 2-5).
    Returns [(name, xml_text, ranks, bytes, dtype)]."""
    if n <= 2:
        out = [("pair_oneshot", xmlgen.allreduce_pair_oneshot(16, "LL", True, 0, 1 << 40, name="sec_pair"),
                n, nbytes, None)]
    else:
        out = [("allpairs_two_phase", xmlgen.allreduce_allpairs(n, 4, "LL", True, 0, 1 << 40,
                                                                 name="sec_allpairs"), n, nbytes, None)]
    if not multi and os.path.exists(RCCL_32TB):
        x = open(RCCL_32TB).read().replace('maxBytes="65536"', 'maxBytes="%d"' % ((32 << 20) + 1))
        out.append(("rccl_allpairs_8n_ll_32tb", x, 8, 32 << 20, M.FLOAT16))
    return out


def run_secondary(name: str, xml_text: str, n: int, nbytes: int, dt: int, a, multi: bool, rank: int,
                  tmp: str) -> dict:
    """One schedule, one size: warmup, K timed AllReduces (HIP events on the collective's stream
    and the host clock, max over ranks), then one step on exact integers that must equal the exact
    sum.  Co-resident ranks at N=1 (n of them on cuda:0), one rank per process otherwise."""
    import torch
    pth = os.path.join(tmp, "bench_sec_%s_%d.xml" % (name, os.getpid()))
    with open(pth, "w") as f:
        f.write(xml_text)
    os.environ["MSCCL_XML_FILES"] = pth
    dev = torch.device("cuda", torch.cuda.current_device())
    comms = init_comms(multi, n if multi else 1, rank, n)
    try:
        ts = M.TYPE_SIZE[dt]
        cnt = nbytes // ts
        tdt = {M.FLOAT32: torch.float32, M.FLOAT16: torch.float16, M.BFLOAT16: torch.bfloat16}[dt]
        ranks = [rank] if multi else list(range(n))
        bufs = [torch.empty(cnt, dtype=tdt, device=dev).uniform_(-1, 1) for _ in ranks]
        stream = bench_stream(dev)
        stream.wait_stream(torch.cuda.current_stream(dev))

        def step():
            with M.group():
                for c, b in zip(comms, bufs):
                    c.all_reduce(b.data_ptr(), b.data_ptr(), cnt, dt, M.SUM, stream.cuda_stream)
        for _ in range(max(1, a.warmup)):
            step()
        k = max(1, a.steps)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if multi:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev0.record(stream)
        for _ in range(k):
            step()
        ev1.record(stream)
        torch.cuda.synchronize()
        if multi:
            torch.distributed.barrier()
        t = (time.perf_counter() - t0) / k
        ev_ms = ev0.elapsed_time(ev1) / k
        if multi:
            tt = torch.tensor([t, ev_ms], dtype=torch.float64)
            torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
            t, ev_ms = float(tt[0]), float(tt[1])
        if any(c.async_error() != 0 for c in comms):
            raise RuntimeError("kernel reported an error (timeout/abort)")
        info = comms[0].info()
        last = info["last"]
        # the launch's algorithmic bytes (the bytes model of what ran: the schedule as written, or
        # its lowered form) and the memory-side / payload fractions of the 8 TB/s peak, as the
        # headline's roofline computes them
        low = lowered_bytes(last, n, nbytes)
        if low is not None:
            hbm, _, payload = low
        else:
            algo = M.algo_json(pth, rank if multi else 0, n)
            fz = set(info.get("algoFuse", [[]])[0]) if last.get("small", 0) == 1 else ()
            size_per = cnt // algo["nchunksperloop"]
            hbm, _ = schedule_bytes(algo, size_per, ts, 0, fused=fz)
            payload, _ = schedule_bytes(algo, size_per, ts, 0, payload_only=True, fused=fz)
        on_gpu = 1 if multi else n
        kern_s = ev_ms / 1e3
        roof = {"algorithmic_bytes": hbm * on_gpu, "payload_bytes": payload * on_gpu,
                "memside_frac": round(hbm * on_gpu / kern_s / 1e9 / HBM_PEAK_GBS, 4),
                "payload_frac": round(payload * on_gpu / kern_s / 1e9 / HBM_PEAK_GBS, 4)}
        j = torch.arange(cnt, device=dev, dtype=torch.int64)
        pat = [((j * 7 + r * 3 + (j >> 5)) % 9 - 4).to(torch.float32) for r in range(n)]
        for r, b in zip(ranks, bufs):
            b.copy_(pat[r].to(tdt))
        want = sum(pat).to(tdt)
        torch.cuda.synchronize()
        step()
        torch.cuda.synchronize()
        good = all(torch.equal(b, want) for b in bufs)
        if multi:
            g = torch.tensor([1 if good else 0], dtype=torch.int32)
            torch.distributed.all_reduce(g, op=torch.distributed.ReduceOp.MIN)
            good = bool(g.item())
        return {"ranks": n, "bytes": nbytes, "dtype": {M.FLOAT32: "f32", M.FLOAT16: "f16", M.BFLOAT16: "bf16"}[dt],
                "ms": round(t * 1e3, 5), "kernel_ms": round(ev_ms, 5),
                "busbw": round(nbytes / t * 2 * (n - 1) / n / 1e9, 3), "verified": good, "steps": k,
                "kernel": kernel_name(last), "lowered": low is not None, **roof}
    finally:
        for c in comms:
            c.destroy()


def kernel_src_hash() -> str:
    """Hash of the device sources: a PMC profile is evidence for the current kernel only if it was
    taken on the same sources (tools/parse_prof.py stamps it)."""
    import hashlib
    h = hashlib.sha1()
    d = os.path.join(ROOT, "msccl_amd", "csrc", "device")
    for f in sorted(os.listdir(d)):
        if f.endswith((".h", ".hip")):
            with open(os.path.join(d, f), "rb") as fh:
                h.update(f.encode() + fh.read())
    return h.hexdigest()[:12]


def live_pmc(a, timeout_s: int = 150):
    """HBM traffic of the headline launch, measured in this run: two rocprofv3 PMC passes
    (FETCH_SIZE, then WRITE_SIZE: they do not fit one TCC pass on gfx950) over a child bench run of
    the headline size only, so every interpreter dispatch in it is a headline launch.  Per the
    MI355X guide's HBM section: traffic = (2 x FETCH_SIZE + WRITE_SIZE) x 1 KiB (gfx950 FETCH_SIZE
    reports half of a 16-B-per-lane streaming read).  Returns (bytes per launch, detail) or (None, why)."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3")
    if prof is None:
        return None, "rocprofv3 not found"
    child = [sys.executable, os.path.abspath(__file__), "--sizes", "33554432", "--steps", "10", "--warmup", "3",
             "--no-cpu", "--quiet", "--no-secondary", "--pmc", "off", "--extras", "", "--eager",
             "--vranks", str(a.vranks), "--proto", a.proto]
    if a.dtype:
        child += ["--dtype", a.dtype]
    if a.instances:
        child += ["--instances", str(a.instances)]
    if a.tiers:
        child += ["--tiers", a.tiers]
    vals = {}
    tmp = tempfile.mkdtemp(prefix="bench_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(tmp, counter)
            cmd = ["timeout", "-s", "KILL", str(timeout_s), prof, "--pmc", counter, "--output-format", "csv",
                   "-d", d, "-o", "run", "--"] + child
            r = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, timeout=timeout_s + 30)
            if r.returncode != 0:
                return None, "rocprofv3 --pmc %s exited %d: %s" % (counter, r.returncode,
                                                                   r.stderr.decode(errors="replace")[-200:])
            v = []
            for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
                with open(f, newline="") as fh:
                    for row in csv.DictReader(fh):
                        if "msccl" in row.get("Kernel_Name", "") and row.get("Counter_Name") == counter:
                            v.append(float(row["Counter_Value"]))
            if not v:
                return None, "no %s rows for the interpreter kernel" % counter
            vals[counter] = (sum(v) / len(v), len(v))
    except (OSError, subprocess.SubprocessError) as e:
        return None, "rocprofv3 pass failed: %s" % e
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    fetch, nf = vals["FETCH_SIZE"]
    write, nw = vals["WRITE_SIZE"]
    return (2.0 * fetch + write) * 1024.0, {"fetch_size_kib": round(fetch, 1), "write_size_kib": round(write, 1),
                                           "launches": [nf, nw]}


def main():
    a = parse()
    import torch
    mode, detail = launch_plan(a.gpus, os.environ, torch.cuda.device_count())
    if mode == "refuse":
        print("bench.py: %s" % detail, file=sys.stderr, flush=True)
        sys.exit(2)
    if mode == "spawn":
        sys.exit(spawn_ranks(detail, sys.argv[1:]))
    # Only the result line goes to stdout: libraries that print there (gloo's connection report,
    # HIP runtime messages) are sent to stderr at the file-descriptor level.
    sys.stdout.flush()
    result_fd = os.dup(1)
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    multi = mode == "rank"
    one_gpu = os.environ.get("MSCCL_AMD_BENCH_ONE_GPU") == "1"
    n = world if multi else a.vranks
    dtname = a.dtype or ("fp16" if (multi and world >= 8) else "fp32")
    dt = M.DTYPE_NAMES[dtname]
    ts = M.TYPE_SIZE[dt]
    proto_id = {"LL": 0, "LL128": 1, "Simple": 2}[a.proto]
    # all-pairs instances of the large tier: 8 up to 8 ranks (8 co-resident ranks, fp16 32 MiB:
    # 2 / 4 / 8 instances 0.60 / 0.62 / 0.52 ms, 16 exceeds the 512 co-resident workgroups,
    # profiles/r04n_c3inst.txt); beyond, as many as keep n (n - 1) thread blocks within 512
    inst = a.instances or (16 if n <= 2 else 8 if n <= 8 else max(1, 512 // (n * (n - 1))))
    sizes = [int(s) for s in a.sizes.split(",")] if a.sizes else SIZES
    tmp = os.environ.get("TMPDIR", "/tmp")
    # peers on other GPUs: one rank per process and GPU (not the one-GPU rehearsal, unless it forces
    # the runtime's cross-GPU paths with MSCCL_AMD_FORCE_REMOTE=1: then the driver's 8-GPU tiers too)
    remote = mode == "rank" and (os.environ.get("MSCCL_AMD_BENCH_ONE_GPU") != "1" or
                                 os.environ.get("MSCCL_AMD_FORCE_REMOTE") == "1")
    tiers = make_xmls(n, a.proto, inst, tmp, a.tiers, remote=remote)
    os.environ["MSCCL_XML_FILES"] = ":".join(t[3] for t in tiers)
    os.environ.setdefault("MSCCL_AMD_TIMEOUT_SEC", "30")

    if multi:
        import torch.distributed as dist
        # MSCCL_AMD_BENCH_ONE_GPU=1 puts every rank on cuda:0: rehearses the multi-process path
        # (bootstrap, hipIpc FIFOs, barriers, max over ranks) on a one-GPU box
        local = 0 if one_gpu else local
        torch.cuda.set_device(local)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        devs = [torch.device("cuda", local)]
        my_ranks = [rank]
    else:
        devs = [torch.device("cuda", 0)] * n
        my_ranks = list(range(n))
    comms = init_comms(multi, world, rank, n)

    def barrier():
        if multi:
            torch.distributed.barrier()

    xgmi_cal = None
    if multi:
        # SURVEY 8(d) calibration: one-way peer copy cuda:0 -> cuda:1 (xGMI), 256 MiB, rank 0
        if rank == 0 and torch.cuda.device_count() > 1 and not one_gpu:
            xgmi_cal = calibrate_xgmi()
        barrier()
    stream = bench_stream(devs[0])
    stream.wait_stream(torch.cuda.current_stream(devs[0]))
    maxb = max(sizes)
    bufs = [torch.empty(maxb // 4 + 64, dtype=torch.float32, device=d).uniform_(-1, 1) for d in devs]
    algos = {t[3]: M.algo_json(t[3], my_ranks[0], n) for t in tiers}
    fused = {t[3]: set(f) for t, f in zip(tiers, comms[0].info().get("algoFuse", []))}

    ptrs = [b.data_ptr() for b in bufs]
    sh = stream.cuda_stream

    def one_step(nbytes):
        cnt = nbytes // ts
        with M.group():
            for c, p in zip(comms, ptrs):
                c.all_reduce(p, p, cnt, dt, M.SUM, sh)

    def pattern(r, cnt, dev):
        # exact small integers (|x| <= 4): every partial sum of up to 8 ranks is exact in every
        # dtype, so any association order must give exactly sum_r pattern(r)
        j = torch.arange(cnt, device=dev, dtype=torch.int64)
        return ((j * 7 + r * 3 + (j >> 5)) % 9 - 4).to(torch.float32)

    def verify(nbytes):
        """One step on exact-integer inputs after the timed steps: the result on every local rank
        must be the exact sum over all ranks (the timed kernel provably did the work)."""
        cnt = nbytes // ts
        tdt = {M.FLOAT32: torch.float32, M.FLOAT16: torch.float16, M.BFLOAT16: torch.bfloat16}[dt]
        for r, b in zip(my_ranks, bufs):
            b.view(tdt)[:cnt].copy_(pattern(r, cnt, b.device).to(tdt))
        want = sum(pattern(r, cnt, bufs[0].device) for r in range(n)).to(tdt)
        torch.cuda.synchronize()   # the refill runs on torch's stream, the collective on `stream`
        one_step(nbytes)
        torch.cuda.synchronize()
        good = all(torch.equal(b.view(tdt)[:cnt], want) for b in bufs)
        if multi:
            g = torch.tensor([1 if good else 0], dtype=torch.int32)
            torch.distributed.all_reduce(g, op=torch.distributed.ReduceOp.MIN)
            good = bool(g.item())
        return good

    results = []
    verified = []
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    # Clock warm-up before the sweep: an idle GPU starts the first timed size at low clocks (the
    # 128 B point once read 27 us instead of 8-9 us).  One process: about 0.3 s of mid-size
    # AllReduces.  Several: every rank must issue the same number of collectives, so a fixed count.
    # A one-size run (a rocprofv3 pass over the headline) warms up with that size, so every
    # interpreter dispatch of the run is a launch of that size.
    wsize = maxb if len(sizes) == 1 else min(maxb, 1 << 20)
    if (wsize // ts) % algos[tier_of(tiers, wsize)[3]]["nchunksperloop"] == 0:
        if multi:
            for _ in range(1000):
                one_step(wsize)
            torch.cuda.synchronize()
        else:
            t_end = time.perf_counter() + 0.3
            while time.perf_counter() < t_end:
                for _ in range(10):
                    one_step(wsize)
                torch.cuda.synchronize()
        barrier()
    for nbytes in sizes:
        cnt = nbytes // ts
        tier = tier_of(tiers, nbytes)
        ncpl = algos[tier[3]]["nchunksperloop"]
        if cnt % ncpl:
            continue
        for _ in range(a.warmup):
            one_step(nbytes)
        graph = None
        if not a.eager:
            # nccl-tests -G style (the reference's run, README.md:57): the K timed steps captured
            # once into a hipGraph; one untimed replay uploads it, the timed one replays the K steps
            torch.cuda.synchronize()
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=stream, capture_error_mode="relaxed"):
                for _ in range(a.steps):
                    one_step(nbytes)
            with torch.cuda.stream(stream):
                graph.replay()
            torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev0.record(stream)
        if graph is not None:
            with torch.cuda.stream(stream):
                graph.replay()
        else:
            for _ in range(a.steps):
                one_step(nbytes)
        ev1.record(stream)
        torch.cuda.synchronize()
        barrier()
        wall = time.perf_counter() - t0
        ev_ms = ev0.elapsed_time(ev1) / a.steps
        t = wall / a.steps
        if multi:
            tt = torch.tensor([t, ev_ms], dtype=torch.float64)
            torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
            t, ev_ms = float(tt[0]), float(tt[1])
        for c in comms:
            if c.async_error() != 0:
                raise RuntimeError("kernel reported an error (timeout/abort) at %d bytes" % nbytes)
        algbw = nbytes / t / 1e9
        bus = algbw * 2 * (n - 1) / n
        algo = algos[tier[3]]
        size_per = cnt // ncpl
        # the fused s + rrc pass runs only in mscclSmallKernel: the discount of one source read
        # applies to sizes whose launches ran there (comm info "last": the kernel of the last launch)
        last = comms[0].info()["last"]
        small = last.get("small", 0) == 1
        fz = fused.get(tier[3], ()) if small else ()
        low = lowered_bytes(last, n, nbytes)   # a lowered launch (msccl_amd/csrc/lower.cc)
        if low is not None:
            hbm, wire, payload = low
        else:
            hbm, wire = schedule_bytes(algo, size_per, ts, proto_id, fused=fz)
            payload, _ = schedule_bytes(algo, size_per, ts, proto_id, payload_only=True, fused=fz)
        ok = verify(nbytes)
        verified.append(ok)
        results.append({"bytes": nbytes, "ms": round(t * 1e3, 5), "kernel_ms": round(ev_ms, 5),
                        "payload_bytes_per_rank": payload, "verified": ok, "small": small,
                        "kernel": kernel_name(last), "lowered": low is not None,
                        "fused": bool(fz), "tier": tier[4],
                         "algbw": round(algbw, 3), "busbw": round(bus, 3),
                         "hbm_bytes_per_rank": hbm, "wire_bytes_per_rank": wire})
        if not a.quiet and rank == 0:
            print("# %10d B  %9.2f us  algbw %8.2f  busbw %8.2f GB/s" % (nbytes, t * 1e6, algbw, bus),
                  file=sys.stderr, flush=True)
    head = results[-1]
    headline_small = head["small"]  # which kernel the headline ran
    # roofline of the dominant (largest) launch
    ranks_on_gpu = 1 if multi else n
    kernel_s = head["kernel_ms"] / 1e3
    achieved = head["hbm_bytes_per_rank"] * ranks_on_gpu / kernel_s / 1e9
    payload_rate = head["payload_bytes_per_rank"] * ranks_on_gpu / kernel_s / 1e9
    roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
            "payload_achieved": round(payload_rate, 2),
            # the same fraction with the protocol's FIFO bytes at payload size (LL: half of each
            # 16-B line is flags), so the LL flag share is visible in one number
            "payload_frac": round(payload_rate / HBM_PEAK_GBS, 4),
            "note": ("achieved counts the protocol's FIFO bytes (LL: 16-B line per 8-B payload); "
                     "payload_achieved counts them at payload size.  The launch's buffers (%d MiB, plus "
                     "FIFO slots) fit the 256 MB MALL, whose hits FETCH_SIZE counts: traffic is "
                     "memory-side bytes, not HBM-array bytes" % (head["bytes"] * ranks_on_gpu >> 20)),
            "kernel": "%s %s Sum %s" % (head["kernel"], dtname, a.proto),
            "algorithmic_bytes_per_launch": head["hbm_bytes_per_rank"] * ranks_on_gpu,
            "kernel_ms": head["kernel_ms"]}
    if multi and not one_gpu and world > 1:
        # the xGMI roofline only where the ranks are on different GPUs (a one-GPU rehearsal's
        # "links" are local HBM: a fraction of the xGMI peak would not be a measurement)
        link = XGMI_LINK_GBS * (n - 1)
        roof["xgmi"] = {"busbw": head["busbw"], "peak": link, "frac": round(head["busbw"] / link, 4),
                        "ll_ceiling": round(link * {0: 0.5, 1: 0.75}.get(proto_id, 1.0), 1),
                        "link_gbs_assumed": XGMI_LINK_GBS, "link_gbs_measured": xgmi_cal}
    workload = workload_desc(multi, n, a.proto, dtname, one_gpu, head["tier"])
    knobs = {k: v for k, v in sorted(os.environ.items()) if k.startswith("MSCCL_AMD_") and k != "MSCCL_AMD_TIMEOUT_SEC"}
    cfg_key = {"workload": workload, "bytes_per_rank": head["bytes"], "instances_large": inst, "knobs": knobs}
    schedule = TIER_KINDS[head["tier"]] + (", s + rrc fused into one pass" if head["fused"] else "") + \
        (", lowered at upload: runs as %s (msccl_amd/csrc/lower.cc)" % head["kernel"] if head["lowered"] else "")
    e2e = None
    if a.e2e and rank == 0 and not multi:
        e2e = measure_e2e(comms, n, maxb, dt, ts, stream, devs[0])
    for c in comms:
        c.destroy()
    comms = []
    secondary = {}
    if not a.no_secondary and head["bytes"] == 32 << 20:
        for name, x, sn, sb, sdt in secondary_schedules(multi, n, head["bytes"]):
            try:
                secondary[name] = run_secondary(name, x, sn, sb, sdt if sdt is not None else dt, a, multi, rank, tmp)
            except Exception as e:  # noqa: BLE001  (reported in the JSON line, the headline stands)
                secondary[name] = {"error": str(e)[:300]}
            if rank == 0 and not a.quiet:
                print("# secondary %s: %s" % (name, secondary[name]), file=sys.stderr, flush=True)
    # HBM traffic of the headline launch: measured now (N=1, rocprofv3 on PATH), else the committed
    # profile of the same configuration, valid only if taken on the same device sources
    src_hash = kernel_src_hash()
    if a.pmc == "auto" and not multi and rank == 0:
        tb, detail = live_pmc(a)
        if tb is not None:
            roof["traffic"] = round(tb)
            roof["traffic_source"] = {"measured": "this run: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over "
                                                  "a headline-only child run", **detail, "kernel_src": src_hash}
        else:
            roof["traffic_source"] = {"measured": None, "why": detail}
    if roof["traffic"] is None:
        tb, src = pmc_traffic(cfg_key, src_hash)
        if tb is not None:
            roof["traffic"], roof["traffic_source"] = tb, {"profile": src, "kernel_src": src_hash}
    if roof["traffic"] is not None:
        roof["traffic_over_algorithmic"] = round(roof["traffic"] / roof["algorithmic_bytes_per_launch"], 4)
    extras = {}
    which = a.extras if a.extras is not None else ("C4,C5" if multi and world == 8 else "")
    for cfg in [w for w in which.split(",") if w]:
        try:
            extras[cfg] = run_extra(cfg, a, multi, world, rank, n, tmp)
        except Exception as e:  # noqa: BLE001  (reported in the JSON line, the headline stands)
            extras[cfg] = {"error": str(e)[:300]}
    tuning = None
    if multi and world > 1 and not a.no_tuning:
        try:
            tuning = run_tuning(a, world, rank, n, tmp, dt, ":".join(t[3] for t in tiers), results, xgmi_cal, one_gpu)
        except Exception as e:  # noqa: BLE001  (reported in the JSON line, the headline stands)
            tuning = {"error": str(e)[:300]}
    cpu = None
    if not a.no_cpu and rank == 0 and not multi:   # the host baseline is quoted at N=1 only
        cpu = cpu_baseline(n, maxb, dt if dt in (6, 7, 9) else 7, a.cpu_seconds)
    out = {
        "metric": "AllReduce bus-BW GB/s (device-resident), 128B-32MB",
        "value": head["busbw"], "unit": "GB/s", "n_gpus": world if multi else 1, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": head["ms"], "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": {"fp32": "f32", "fp16": "f16", "bf16": "bf16"}.get(dtname, dtname),
        "data": "synthetic",
        "config": {"workload": workload,
                   "ranks": n, "devices": 1 if (one_gpu or not multi) else world,
                   "bytes_per_rank": head["bytes"], "schedule": schedule,
                   "instances_large": inst, "proto": a.proto, "sweep_bytes": [sizes[0], sizes[-1]],
                   "tiers": [[t[0], t[1], t[2], {"a": "allpairs", "o": "oneshot", "O": "oneshot-ordered",
                                                 "p": "pair-oneshot", "r": "ring"}[t[4]]] for t in tiers],
                   "launch": "eager" if a.eager else "hipgraph (K steps captured, replayed once)",
                   "knobs": knobs},
        "avg_busbw": round(float(np.mean([r["busbw"] for r in results])), 3),
        "verified": bool(verified) and all(verified),
        "verification": "after each size's timed steps, one step on exact-integer inputs on every rank "
                        "must equal the exact sum over ranks",
        # `value` is the metric as BASELINE.json and nccl-tests define it (bus bandwidth seen by
        # each rank); the whole job moves n_ranks times that
        "aggregate": {"ranks": n, "busbw_sum_gbs": round(head["busbw"] * n, 3),
                      "algbw_sum_gbs": round(head["bytes"] / (head["ms"] / 1e3) / 1e9 * n, 3)},
        "roofline": roof,
        "cpu_baseline": cpu,
        "sweep": [{k: r[k] for k in ("bytes", "ms", "kernel_ms", "busbw", "verified", "kernel")} for r in results],
    }
    if e2e:
        out["e2e"] = e2e
    if secondary:
        out["schedules"] = secondary
    if extras:
        out["configs"] = extras
    if tuning:
        out["tuning"] = tuning
    if rank == 0:
        sys.stdout.flush()
        os.write(result_fd, (json.dumps(out) + "\n").encode())
    for c in comms:
        c.destroy()
    if multi:
        torch.distributed.destroy_process_group()


def calibrate_xgmi(nbytes: int = 256 << 20, reps: int = 5):
    """One-way device-to-device copy GB/s between cuda:0 and cuda:1 (is 153 GB/s
    per link one-way?).  Returns None when the copy fails."""
    import torch
    try:
        src = torch.empty(nbytes, dtype=torch.uint8, device="cuda:0")
        dst = torch.empty(nbytes, dtype=torch.uint8, device="cuda:1")
        dst.copy_(src)
        torch.cuda.synchronize("cuda:0")
        torch.cuda.synchronize("cuda:1")
        t0 = time.perf_counter()
        for _ in range(reps):
            dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize("cuda:0")
        torch.cuda.synchronize("cuda:1")
        gbs = nbytes * reps / (time.perf_counter() - t0) / 1e9
        del src, dst
        return round(gbs, 2)
    except Exception:  # noqa: BLE001  (reported as unmeasured)
        return None


def measure_e2e(comms, n, nbytes, dt, ts, stream, dev):
    """Host-resident end to end: pinned H2D of every rank's input, AllReduce, D2H."""
    import torch
    cnt = nbytes // ts
    host_in = [torch.empty(nbytes // 4, dtype=torch.float32).uniform_(-1, 1).pin_memory() for _ in range(n)]
    host_out = [torch.empty(nbytes // 4, dtype=torch.float32).pin_memory() for _ in range(n)]
    dbufs = [torch.empty(nbytes // 4, dtype=torch.float32, device=dev) for _ in range(n)]
    reps = 10
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        with torch.cuda.stream(stream):   # copies and the collective ordered on one stream
            for i in range(n):
                dbufs[i].copy_(host_in[i], non_blocking=True)
            with M.group():
                for c, b in zip(comms, dbufs):
                    c.all_reduce(b.data_ptr(), b.data_ptr(), cnt, dt, M.SUM, stream.cuda_stream)
            for i in range(n):
                host_out[i].copy_(dbufs[i], non_blocking=True)
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / reps
    algbw = nbytes / t / 1e9
    serial_out = [h.clone() for h in host_out]
    from msccl_amd import hostpath
    res = {"bytes": nbytes, "ms": round(t * 1e3, 4), "algbw": round(algbw, 3),
           "busbw": round(algbw * 2 * (n - 1) / n, 3)}
    # zero copy (msccl_amd/hostpath.py): the collective reads and writes the pinned buffers itself,
    # in place on a pinned copy of the inputs (the tiers' XMLs are in place)
    host_io = [h.clone().pin_memory() for h in host_in]
    hostpath.all_reduce_host(comms, host_io, host_io, dt, M.SUM)
    torch.cuda.synchronize()
    same = all(torch.equal(a, b) for a, b in zip(host_io, serial_out))
    t0 = time.perf_counter()
    for _ in range(reps):
        hostpath.all_reduce_host(comms, host_io, host_io, dt, M.SUM)
    torch.cuda.synchronize()
    tz = (time.perf_counter() - t0) / reps
    res["zero_copy"] = {"ms": round(tz * 1e3, 4), "algbw": round(nbytes / tz / 1e9, 3),
                        "same_bits_as_serial": bool(same)}
    # staged: chunks through H2D / collective / D2H streams
    chunk = hostpath.default_chunk_bytes(nbytes)
    streams = {}
    for o in host_out:
        o.zero_()
    hostpath.all_reduce_host_staged(comms, host_in, host_out, dbufs, dt, M.SUM, chunk, streams)
    torch.cuda.synchronize()
    same = all(torch.equal(a, b) for a, b in zip(host_out, serial_out))
    t0 = time.perf_counter()
    for _ in range(reps):
        hostpath.all_reduce_host_staged(comms, host_in, host_out, dbufs, dt, M.SUM, chunk, streams)
    torch.cuda.synchronize()
    tp = (time.perf_counter() - t0) / reps
    res["staged"] = {"ms": round(tp * 1e3, 4), "algbw": round(nbytes / tp / 1e9, 3), "chunk_bytes": chunk,
                     "same_bits_as_serial": bool(same)}
    return res


if __name__ == "__main__":
    main()
