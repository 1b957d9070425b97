"""GPU parity of ncclAllToAll and ncclCustomCollective (MSCCL additions, nccl.h.in:286-304):
RCCL-shipped msccl-tools AllToAll schedules (all five 8-rank size tiers) and a custom-collective
schedule, bit-exact against the oracle simulator, plus the AllToAll definition itself."""
import os

import numpy as np
import pytest

import msccl_amd as M
from msccl_amd import xmlgen
from oracle import loader as L
from oracle import numerics as N
from oracle import plan as P
from oracle import sim as S

pytestmark = pytest.mark.gpu
os.environ.setdefault("MSCCL_AMD_TIMEOUT_SEC", "20")
RCCL = "/opt/rocm/share/rccl/msccl-algorithms"


def run_xml(xml, n, coll, count, dt, seed=5):
    import torch
    from tests.gpu_harness import gen_inputs, to_torch, from_torch
    path = "/tmp/msccl_a2a_%d_%d.xml" % (os.getpid(), abs(hash(xml)) % 100000)
    open(path, "w").write(xml)
    os.environ["MSCCL_XML_FILES"] = path
    comms = M.Comm.init_all([0] * n)
    in_n = count * n if coll == L.ALLTOALL else count
    ins = gen_inputs(n, in_n, dt, seed)
    try:
        dev = torch.device("cuda:0")
        t_in = [to_torch(x, dev) for x in ins]
        t_out = [torch.zeros_like(t) for t in t_in]
        s = torch.cuda.current_stream().cuda_stream
        with M.group():
            for c, a, b in zip(comms, t_in, t_out):
                if coll == L.ALLTOALL:
                    c.all_to_all(a.data_ptr(), b.data_ptr(), count, dt, s)
                else:
                    c.custom(a.data_ptr(), b.data_ptr(), count, dt, 0, s)
        torch.cuda.synchronize()
        assert all(c.async_error() == 0 for c in comms)
        gpu = [from_torch(t, N.storage(dt)) for t in t_out]
    finally:
        for c in comms:
            c.destroy()
    algos = [L.parse_xml(xml, r, n) for r in range(n)]
    call = P.Call(coll, count, dt, 0, n, 0, False)
    assert P.select([algos[0]], call) == 0
    plan = P.make_plan([algos[0]], call, 0)
    if coll == L.ALLTOALL:
        o_in = [x.view(np.int8).copy() for x in ins]
        o_out = [np.zeros(in_n * N.type_size(dt), np.int8) for _ in range(n)]
    else:
        o_in = [x.copy() for x in ins]
        o_out = [np.zeros(in_n, N.storage(dt)) for _ in range(n)]
    res, _ = S.run(algos, plan, o_in, o_out, coll, False)
    ora = [np.asarray(r).view(N.storage(dt)) for r in res]
    return ins, gpu, ora


@pytest.mark.parametrize("name", ["alltoall-8n-0-9kb.xml", "alltoall-8n-9kb-190kb.xml",
                                  "alltoall-8n-190kb-512kb.xml", "alltoall-8n-512kb-7mb.xml",
                                  "alltoall-8n-7mb-43mb.xml"])
def test_rccl_alltoall_schedules(name):
    p = os.path.join(RCCL, name)
    if not os.path.exists(p):
        pytest.skip("fixture missing")
    xml = open(p).read()
    a = L.parse_xml(xml, 0, 8)
    n, dt, ts = 8, 7, 4
    ncpl = a.nchunksperloop
    count = max(ncpl, (a.minBytes // (ts * n) // ncpl + 1) * ncpl)   # nBytes = count*ts*n >= minBytes
    assert a.minBytes <= count * ts * n < a.maxBytes, (count, a.minBytes, a.maxBytes)
    ins, gpu, ora = run_xml(xml, n, L.ALLTOALL, count, dt)
    from tests.gpu_harness import describe_mismatch
    chunk = count * n // ncpl   # elements (fp32) of one MSCCL chunk
    for r in range(n):
        assert np.array_equal(gpu[r].view(np.uint8), ora[r].view(np.uint8)), \
            "rank %d (chunks of %d floats, block q = chunks [q*%d, (q+1)*%d)):\n%s" % (
                r, chunk, ncpl // n, ncpl // n, describe_mismatch(gpu[r], ora[r], chunk))
        # the collective's definition: block p of rank r's output is block r of rank p's input
        for q in range(n):
            assert np.array_equal(gpu[r][q * count:(q + 1) * count], ins[q][r * count:(r + 1) * count]), (r, q)


@pytest.mark.parametrize("proto", ["LL", "Simple"])
def test_custom_collective(proto):
    """ncclCustomCollective runs the schedule registered with coll="custom" (algorithm index 0)."""
    xml = xmlgen.allreduce_allpairs(4, 2, proto, inplace=False).replace('coll="allreduce"', 'coll="custom"')
    n, count = 4, 32 * 1000
    ins, gpu, ora = run_xml(xml, n, L.CUSTOM, count, 7)
    for r in range(n):
        assert np.array_equal(gpu[r].view(np.uint8), ora[r].view(np.uint8)), r


@pytest.mark.parametrize("name,inplace", [("allgather_16n_direct_0_3m_ll128.xml", True),
                                          ("allgather_16n_direct_0_3m_ll128_op.xml", False)])
def test_rccl_allgather_16n_ll128(name, inplace):
    """RCCL's 16-rank direct AllGather (LL128), 16 co-resident ranks in one launch."""
    from tests.test_gpu_parity import check
    p = os.path.join(RCCL, name)
    if not os.path.exists(p):
        pytest.skip("fixture missing")
    xml = open(p).read()
    a = L.parse_xml(xml, 0, 16)
    assert a.valid and bool(a.inplace) == inplace
    count = 64 * a.nchunksperloop
    check(xml, 16, L.ALLGATHER, count, 6, inplace=inplace)
