"""Group aggregation under MSCCL_AMD_REFERENCE_SELECTION (src/enqueue.cc:448-460): two ops of one
communicator in a group skip MSCCL and take the ring / tree fallback with the reference's bits;
by default both run the MSCCL schedule."""
import os

import numpy as np
import pytest

import msccl_amd as M
from msccl_amd import xmlgen
from oracle import loader as L
from tests.gpu_harness import CoResident, describe_mismatch, from_torch, gen_inputs, to_torch
from oracle import numerics as N

pytestmark = pytest.mark.gpu
os.environ.setdefault("MSCCL_AMD_TIMEOUT_SEC", "20")


@pytest.mark.parametrize("ref", ["0", "1"])
def test_two_ops_per_comm_in_a_group(tmp_path, monkeypatch, ref):
    import torch
    from oracle import ring as R
    monkeypatch.setenv("MSCCL_AMD_REFERENCE_SELECTION", ref)
    monkeypatch.setenv("NCCL_ALGO", "MSCCL,Ring,Tree")   # MSCCL enabled for AllReduce in both modes
    n, count, dt = 2, 1024, 7
    xml = xmlgen.allreduce_allpairs(n, 1, "LL")
    with CoResident(n, [xml], str(tmp_path)) as cr:
        xa, xb = gen_inputs(n, count, dt, 1), gen_inputs(n, count, dt, 2)
        ta = [to_torch(x, torch.device("cuda:0")) for x in xa]
        tb = [to_torch(x, torch.device("cuda:0")) for x in xb]
        torch.cuda.synchronize()
        with M.group():
            for r, c in enumerate(cr.comms):
                c.all_reduce(ta[r].data_ptr(), ta[r].data_ptr(), count, dt, M.SUM, 0)
                c.all_reduce(tb[r].data_ptr(), tb[r].data_ptr(), count, dt, M.SUM, 0)
        torch.cuda.synchronize()
        assert all(c.async_error() == 0 for c in cr.comms)
        last = [c.info()["last"] for c in cr.comms]
        # the fallback (algo -1) only under the reference's selection; the schedule (algo 0) runs
        # interpreted or lowered to the fold kernel otherwise
        assert all((l["algo"] < 0) == (ref == "1") for l in last), last
        for ins, t in ((xa, ta), (xb, tb)):
            if ref == "1":
                want, _ = R.run(L.ALLREDUCE, count, dt, 0, [x.copy() for x in ins], [None] * n, True)
            else:
                want, _ = cr.oracle(L.ALLREDUCE, count, dt, 0, ins, True)
            for r in range(n):
                got = from_torch(t[r], N.storage(dt))
                assert np.array_equal(got.view(np.uint32), np.asarray(want[r]).view(np.uint32)), \
                    describe_mismatch(got, np.asarray(want[r]))
        # one op per communicator: MSCCL in both modes
        with M.group():
            for r, c in enumerate(cr.comms):
                c.all_reduce(ta[r].data_ptr(), ta[r].data_ptr(), count, dt, M.SUM, 0)
        torch.cuda.synchronize()
        assert all(c.info()["last"]["algo"] == 0 for c in cr.comms)
