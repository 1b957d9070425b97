"""GPU parity: the HIP interpreter through the C-ABI vs the CPU oracle, bit-exact.

Ranks are co-resident on cuda:0 (ncclCommInitAll with a repeated device) so one MI355X runs
every rank of the schedule; the kernels, FIFOs, head/tail credits and dependency flags are the
same as over xGMI.  Every comparison is bit-for-bit against oracle/sim.py on the same seeded
inputs (the reference's association order is part of the contract).
"""
import os

import numpy as np
import pytest

from msccl_amd import xmlgen
from oracle import loader as L
from oracle import numerics as N

pytestmark = pytest.mark.gpu
os.environ.setdefault("MSCCL_AMD_TIMEOUT_SEC", "20")


def check(xml, n, coll, count, dt, op=0, inplace=True, seed=1, mode="uniform", iters=1):
    from tests.gpu_harness import run_collective
    gpu, ora, _ = run_collective(xml, n, coll, count, dt, op, inplace, seed, mode, iters)
    for r in range(n):
        g, o = gpu[r].view(np.uint8), np.asarray(ora[r]).view(np.uint8)
        if not np.array_equal(g, o):
            bad = np.nonzero(g != o)[0]
            raise AssertionError("rank %d: %d differing bytes, first at byte %d" % (r, len(bad), bad[0]))


# all-pairs AllReduce: protocol x dtype x size (small reduce path, multi-iteration, maxAllowedCount split)
@pytest.mark.parametrize("proto", ["LL", "LL128", "Simple"])
@pytest.mark.parametrize("dt", [7, 6, 9])
@pytest.mark.parametrize("n,inst,count", [
    (2, 1, 4 * 8),            # 128 B fp32: smallest C2 point, per-element reduce path
    (2, 4, 16 * 1000),        # small path (nelem*count < nthreads)
    (2, 4, 1 << 18),          # multi-iteration, maxAllowedCount = 1
    (2, 16, (1 << 20) + 16 * 64),
    (4, 2, 32 * 4099),        # odd per-chunk size: unaligned 16-B packs, element tails
    (8, 4, 256 * 300),
])
def test_allpairs_allreduce(proto, dt, n, inst, count):
    check(xmlgen.allreduce_allpairs(n, inst, proto), n, L.ALLREDUCE, count, dt)


@pytest.mark.parametrize("proto", ["LL", "LL128", "Simple"])
@pytest.mark.parametrize("n,inst,count,dt", [
    (2, 1, 32, 7),              # 128 B fp32 (the C2 sweep's first point)
    (2, 16, 16 * 4099, 7),      # odd chunk: element tails, per-element reduce path off
    (2, 16, (1 << 20), 6),
    (4, 2, 2 * 3001, 9),
    (8, 1, 8 * 1000, 7),
])
def test_oneshot_allreduce(proto, n, inst, count, dt):
    """xmlgen.allreduce_oneshot (the bench's latency tier) vs the oracle, bit-exact."""
    check(xmlgen.allreduce_oneshot(n, inst, proto), n, L.ALLREDUCE, count, dt)


@pytest.mark.parametrize("proto", ["LL", "LL128", "Simple"])
@pytest.mark.parametrize("n,inst,count,dt", [
    (8, 1, 64, 6),              # 128 B fp16 (the C3 sweep's first point)
    (8, 4, 4 * 5003, 6),
    (4, 16, 16 * 4096, 9),
    (3, 2, 2 * 777, 7),
])
def test_oneshot_ordered_allreduce(proto, n, inst, count, dt):
    """Rank-ordered one-shot vs the oracle, bit-exact, and the same bits on every rank."""
    from tests.gpu_harness import run_collective
    xml = xmlgen.allreduce_oneshot(n, inst, proto, ordered=True)
    check(xml, n, L.ALLREDUCE, count, dt)
    gpu, _, _ = run_collective(xml, n, L.ALLREDUCE, count, dt, 0, True, 5, "uniform", 1)
    for r in range(1, n):
        assert np.array_equal(gpu[0].view(np.uint8), gpu[r].view(np.uint8))


@pytest.mark.parametrize("proto", ["LL", "LL128", "Simple"])
def test_allpairs_out_of_place(proto):
    check(xmlgen.allreduce_allpairs(8, 2, proto, inplace=False), 8, L.ALLREDUCE, 128 * 513, 7, inplace=False)


@pytest.mark.parametrize("proto,dt", [("Simple", 9), ("LL", 7), ("Simple", 6), ("LL128", 9), ("LL128", 8)])
def test_ring_allreduce(proto, dt):
    check(xmlgen.allreduce_ring(8, 4, proto), 8, L.ALLREDUCE, 32 * 20000, dt)


def test_ring_c4_shape_large():
    """C4 shape at reduced size: 8-rank ring, Simple, bf16, multi-chunk (2 interpreter iterations)."""
    check(xmlgen.allreduce_ring(8, 8, "Simple"), 8, L.ALLREDUCE, 64 * (1 << 16) + 64 * 7, 9)


@pytest.mark.parametrize("op", [1, 2, 3])
@pytest.mark.parametrize("dt", [7, 6, 9, 8])
def test_other_ops(op, dt):
    check(xmlgen.allreduce_allpairs(4, 2, "LL"), 4, L.ALLREDUCE, 32 * 777, dt, op=op)


@pytest.mark.parametrize("dt", [0, 1, 2, 3, 4, 5])
def test_integer_types(dt):
    check(xmlgen.allreduce_allpairs(4, 1, "Simple"), 4, L.ALLREDUCE, 16 * 1001, dt, mode="exact")
    check(xmlgen.allreduce_allpairs(2, 2, "LL"), 2, L.ALLREDUCE, 8 * 999, dt, op=2)


@pytest.mark.parametrize("proto,inplace", [("Simple", False), ("LL", True), ("Simple", True), ("LL128", False)])
def test_reduce_scatter(proto, inplace):
    check(xmlgen.reduce_scatter_allpairs(8, 2, proto, inplace=inplace), 8, L.REDUCE_SCATTER, 2 * 50000, 7,
          inplace=inplace)


@pytest.mark.parametrize("proto,inplace", [("Simple", False), ("Simple", True), ("LL", True), ("LL", False),
                                           ("LL128", False)])
@pytest.mark.parametrize("dt,count", [(7, 16 * 50001), (6, 4 * 1000 + 4), (9, 16 << 16), (2, 3 * 7)])
def test_reduce_scatter_two_ranks(proto, inplace, dt, count):
    """The 2-rank ReduceScatter (s of the peer's chunk, rrc of the own one: no scratch)."""
    inst = 4 if count % 4 == 0 else 1
    check(xmlgen.reduce_scatter_allpairs(2, inst, proto, inplace=inplace), 2, L.REDUCE_SCATTER, count, dt,
          inplace=inplace)


@pytest.mark.parametrize("proto,inplace", [("Simple", False), ("LL", True), ("LL", False), ("LL128", True)])
def test_all_gather(proto, inplace):
    check(xmlgen.allgather_allpairs(8, 2, proto, inplace=inplace), 8, L.ALLGATHER, 2 * 33333, 7, inplace=inplace)


def test_repeated_launches_persist_fifo_state():
    """Many launches on the same communicators: step counters, LL flags and workIndex carry over."""
    check(xmlgen.allreduce_allpairs(4, 2, "LL"), 4, L.ALLREDUCE, 32 * 64, 7, mode="exact", iters=40)
    check(xmlgen.allreduce_allpairs(4, 2, "Simple"), 4, L.ALLREDUCE, 32 * 640, 7, mode="exact", iters=25)


def test_rccl_allpairs_schedules(rccl_xmls):
    for f in rccl_xmls:
        base = os.path.basename(f)
        if not base.startswith("allreduce-allpairs-8n"):
            continue
        text = open(f).read()
        a = L.parse_xml(text, 0, 8)
        ncpl = a.nchunksperloop
        lo = -(-a.minBytes // 2 // ncpl) * ncpl          # fp16 elements, multiple of ncpl, >= minBytes
        count = max(ncpl * 16, lo)
        count = min(count, (a.maxBytes - 1) // 2 // ncpl * ncpl)
        assert a.minBytes <= 2 * count < a.maxBytes
        check(text, 8, L.ALLREDUCE, count, 6, inplace=bool(a.inplace))


def test_rccl_ring16_ll(rccl_xmls):
    p = "/opt/rocm/share/rccl/msccl-unit-test-algorithms/all-reduce-ring-ll.xml"
    if not os.path.exists(p):
        pytest.skip("fixture missing")
    text = open(p).read()
    check(text, 16, L.ALLREDUCE, 384 * 4, 7)


@pytest.mark.parametrize("name", ["ap2_ll_f32", "ap4_ll_bf16", "ring8_simple_bf16", "rs8_simple_f32", "ap4_ll128_f16",
                                  "ag8_ll_f32", "ap8_ll_f16_rccl32tb", "ap2_ll_i32_exact"])
def test_golden_vectors_on_gpu(name):
    from tests.golden import make_golden as G
    from tests.gpu_harness import run_collective
    case = [c for c in G.CASES if c[0] == name][0]
    _, xf, n, coll, count, dt, op, inplace, mode = case
    try:
        xml = xf()
    except OSError:
        pytest.skip("source XML missing")
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", name + ".npz"))
    gpu, _, ins = run_collective(xml, n, coll, count, dt, op, inplace, seed=7, mode=mode)
    assert np.array_equal(np.stack(ins), z["inputs"])
    for r in range(n):
        assert np.array_equal(gpu[r].view(np.uint8), z["outputs"][r].view(np.uint8)), r


@pytest.mark.parametrize("split", [1, 2, 8])
@pytest.mark.parametrize("proto", ["LL", "LL128", "Simple"])
def test_workgroup_split_is_value_neutral(split, proto, monkeypatch):
    """Running each XML thread block as `split` workgroups (sub-connections) changes no bit."""
    monkeypatch.setenv("MSCCL_AMD_SPLIT", str(split))
    check(xmlgen.allreduce_allpairs(4, 2, proto), 4, L.ALLREDUCE, 32 * 3001, 9)
    check(xmlgen.allreduce_ring(4, 2, proto), 4, L.ALLREDUCE, 8 * 77, 7, op=2)
    check(xmlgen.reduce_scatter_allpairs(4, 1, proto), 4, L.REDUCE_SCATTER, 4 * 1000 + 4, 6, inplace=False)


@pytest.mark.parametrize("proto,per_chunk,dt", [
    ("LL", 8192 * 3 + 100, 7),        # 3 full LL iterations (merged) + a partial one on the per-element path
    ("LL", 8192 * 5, 9),              # bf16: 2.5 LL iterations
    ("Simple", 524288 * 2 + 1000, 7),  # 2 full Simple iterations (merged) + a partial one
    ("LL128", 144000 * 2 + 60, 7),     # 2 full LL128 iterations (576000-B steps) + a partial one
    ("LL", 8192 * 16, 7),              # 16 iterations: merged steps longer than one FIFO slot
])
def test_merged_iterations_are_value_neutral(proto, per_chunk, dt):
    """Consecutive full interpreter iterations run as one op (RankWork.merge): bit-exact vs the
    oracle, which runs the reference's iteration grid one iteration at a time."""
    x = xmlgen.allreduce_allpairs(2, 1, proto)
    ncpl = 4
    check(x, 2, L.ALLREDUCE, ncpl * per_chunk, dt)


@pytest.mark.parametrize("op", [0, 2])
@pytest.mark.parametrize("dt", [6, 8, 0])
def test_ll128_types_and_ops(op, dt):
    """LL128 (CDNA4 16-B line form): 3 packs per 4 lines, partial units, every element width."""
    for count in (16 * 3 * 7 + 5 * 16, 64 * 1001):
        check(xmlgen.allreduce_allpairs(4, 2, "LL128"), 4, L.ALLREDUCE, count, dt, op=op,
              mode="exact" if dt == 0 else "uniform")


def test_ll_and_ll128_share_a_fifo(tmp_path):
    """An LL and an LL128 schedule on the same connections, alternating launches on the same
    communicators: the flag words of either line format never satisfy the other's wait."""
    import torch
    import msccl_amd as M
    a = tmp_path / "ll.xml"
    b = tmp_path / "ll128.xml"
    a.write_text(xmlgen.allreduce_allpairs(2, 1, "LL", min_bytes=0, max_bytes=1 << 16))
    b.write_text(xmlgen.allreduce_allpairs(2, 1, "LL128", min_bytes=1 << 16, max_bytes=1 << 30))
    os.environ["MSCCL_XML_FILES"] = "%s:%s" % (a, b)
    comms = M.Comm.init_all([0, 0])
    try:
        g = torch.Generator().manual_seed(5)
        for it, count in enumerate([4 * 1000, 4 * 40000] * 4):
            x = [torch.randint(-4, 5, (count,), generator=g).float() for _ in range(2)]
            d = [t.cuda() for t in x]
            with M.group():
                for c, t in zip(comms, d):
                    c.all_reduce(t.data_ptr(), t.data_ptr(), count, M.FLOAT32, M.SUM, 0)
            torch.cuda.synchronize()
            for t in d:
                assert torch.equal(t.cpu(), x[0] + x[1]), it
        assert all(c.async_error() == 0 for c in comms)
    finally:
        for c in comms:
            c.destroy()


@pytest.mark.parametrize("proto,n,count,dt", [
    ("Simple", 2, 2 * (1 << 22) + 2 * 512, 9),   # 4 M bf16 per chunk: 16 Simple iterations
    ("LL", 2, 2 * (1 << 20), 7),                 # 1 M fp32 per chunk: 128 LL iterations
])
def test_large_calls_respect_fifo_depth(proto, n, count, dt, monkeypatch):
    """Both ranks of a ring send before they receive.  Merged calls (iterations, a transfer's
    chunks) stay within kMaxOpSlots FIFO slots per sub-connection, so one workgroup per thread
    block (no split) must not deadlock on a call larger than its FIFO."""
    monkeypatch.setenv("MSCCL_AMD_SPLIT", "1")
    check(xmlgen.allreduce_ring(n, 1, proto), n, L.ALLREDUCE, count, dt, mode="exact")
