"""Host-resident AllReduce (msccl_amd/hostpath.py): the zero-copy call (the collective reads and
writes pinned host memory) and the staged copy / collective / copy pipeline give the whole
device-resident call's bits and the oracle's, ragged last chunk included; a non-pinned buffer is
refused."""
import os

import numpy as np
import pytest

import msccl_amd as M
from msccl_amd import hostpath, xmlgen
from tests.gpu_harness import gen_inputs

pytestmark = pytest.mark.gpu
os.environ.setdefault("MSCCL_AMD_TIMEOUT_SEC", "20")


def _comms(tmp_path, xml):
    p = tmp_path / "s.xml"
    p.write_text(xml)
    os.environ["MSCCL_XML_FILES"] = str(p)
    return M.Comm.init_all([0, 0])


@pytest.mark.parametrize("count,chunk", [((5 << 20) // 4, 1 << 20), ((3 << 20) // 4 + 7, 1 << 20), (4096, 4 << 20)])
def test_pipelined_host_allreduce_matches_device_call(tmp_path, count, chunk):
    import torch
    comms = _comms(tmp_path, xmlgen.allreduce_pair_oneshot(16, "LL"))
    try:
        ins = gen_inputs(2, count, 7, 13)
        host_in = [torch.from_numpy(x).pin_memory() for x in ins]
        host_out = [torch.zeros(count, dtype=torch.float32).pin_memory() for _ in range(2)]
        dev = [torch.empty(count, dtype=torch.float32, device="cuda:0") for _ in range(2)]
        hostpath.all_reduce_host_staged(comms, host_in, host_out, dev, M.FLOAT32, M.SUM, chunk)
        torch.cuda.synchronize()
        # the whole call, device-resident
        whole = [torch.from_numpy(x).cuda() for x in ins]
        s = torch.cuda.current_stream().cuda_stream
        with M.group():
            for c, b in zip(comms, whole):
                c.all_reduce(b.data_ptr(), b.data_ptr(), count, M.FLOAT32, M.SUM, s)
        torch.cuda.synchronize()
        assert all(c.async_error() == 0 for c in comms)
        for r in range(2):
            got = host_out[r].numpy().view(np.uint32)
            assert np.array_equal(got, whole[r].cpu().numpy().view(np.uint32)), "rank %d" % r
        # the oracle: both ranks hold fn(peer, local), i.e. x0 + x1 in fp32
        want = (ins[0].astype(np.float32) + ins[1].astype(np.float32)).view(np.uint32)
        assert np.array_equal(host_out[0].numpy().view(np.uint32), want)
    finally:
        for c in comms:
            c.destroy()


def test_unpinned_host_buffer_is_refused(tmp_path):
    import torch
    comms = _comms(tmp_path, xmlgen.allreduce_pair_oneshot(1, "LL"))
    try:
        host = [torch.zeros(64) for _ in range(2)]
        dev = [torch.zeros(64, device="cuda:0") for _ in range(2)]
        with pytest.raises(ValueError):
            hostpath.all_reduce_host_staged(comms, host, host, dev, M.FLOAT32)
        with pytest.raises(ValueError):
            hostpath.all_reduce_host(comms, host, host, M.FLOAT32)
    finally:
        for c in comms:
            c.destroy()


@pytest.mark.parametrize("inplace", [False, True])
@pytest.mark.parametrize("count", [4096, (3 << 20) // 4 + 7, (8 << 20) // 4])
def test_zero_copy_host_allreduce(tmp_path, count, inplace):
    """The collective on pinned host memory (its device addresses), out of place with an
    out-of-place pair schedule and in place with an in-place one (a ragged count takes the ring
    fallback): x0 + x1 on both ranks, bit for bit."""
    import torch
    comms = _comms(tmp_path, xmlgen.allreduce_pair_oneshot(16, "LL", inplace=inplace))
    try:
        ins = gen_inputs(2, count, 7, 17)
        host_in = [torch.from_numpy(x).pin_memory() for x in ins]
        host_out = host_in if inplace else [torch.zeros(count, dtype=torch.float32).pin_memory() for _ in range(2)]
        hostpath.all_reduce_host(comms, host_in, host_out, M.FLOAT32, M.SUM)
        torch.cuda.synchronize()
        assert all(c.async_error() == 0 for c in comms)
        want = (ins[0].astype(np.float32) + ins[1].astype(np.float32)).view(np.uint32)
        for r in range(2):
            assert np.array_equal(host_out[r].numpy().view(np.uint32), want), "rank %d" % r
    finally:
        for c in comms:
            c.destroy()


def test_zero_copy_reduce_scatter_and_all_gather(tmp_path):
    """ReduceScatter then AllGather (C5's pair at 4 ranks, Simple) on pinned host memory: the
    oracle's values (exact-integer inputs, so any fold order gives the same bits)."""
    import torch
    n, rc = 4, (1 << 20) // 4
    p1, p2 = tmp_path / "rs.xml", tmp_path / "ag.xml"
    p1.write_text(xmlgen.reduce_scatter_allpairs(n, 2, "Simple", False, 0, 1 << 40, name="rs"))
    p2.write_text(xmlgen.allgather_allpairs(n, 2, "Simple", False, 0, 1 << 40, name="ag"))
    os.environ["MSCCL_XML_FILES"] = "%s:%s" % (p1, p2)
    comms = M.Comm.init_all([0] * n)
    try:
        ins = gen_inputs(n, rc * n, 7, 23, mode="exact")
        hin = [torch.from_numpy(x).pin_memory() for x in ins]
        hmid = [torch.zeros(rc, dtype=torch.float32).pin_memory() for _ in range(n)]
        hout = [torch.zeros(rc * n, dtype=torch.float32).pin_memory() for _ in range(n)]
        hostpath.reduce_scatter_host(comms, hin, hmid, M.FLOAT32, M.SUM)
        torch.cuda.synchronize()
        hostpath.all_gather_host(comms, hmid, hout, M.FLOAT32)
        torch.cuda.synchronize()
        assert all(c.async_error() == 0 for c in comms)
        total = np.sum(np.stack([x.astype(np.float64) for x in ins]), axis=0).astype(np.float32)
        for r in range(n):
            assert np.array_equal(hmid[r].numpy(), total[r * rc:(r + 1) * rc]), "ReduceScatter rank %d" % r
            assert np.array_equal(hout[r].numpy(), total), "AllGather rank %d" % r
    finally:
        for c in comms:
            c.destroy()
