"""Capture an NPKit dump of a few 2-rank AllReduce launches (GPU) for the golden fixture:
    MSCCL_AMD_NPKIT=1 NPKIT_DUMP_DIR=<dir> python tools/npkit_capture.py
then tests/golden/make_npkit_golden.py <dir> packs it and runs the reference's generator on it."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import msccl_amd as M  # noqa: E402
from msccl_amd import xmlgen  # noqa: E402


def main():
    import torch
    assert os.environ.get("MSCCL_AMD_NPKIT") == "1" and os.environ.get("NPKIT_DUMP_DIR")
    path = "/tmp/npkit_capture_%d.xml" % os.getpid()
    open(path, "w").write(xmlgen.allreduce_allpairs(2, 1, "LL"))
    os.environ["MSCCL_XML_FILES"] = path
    comms = M.Comm.init_all([0, 0])
    bufs = [torch.ones(1 << 14, device="cuda") for _ in comms]
    for _ in range(4):
        with M.group():
            for c, b in zip(comms, bufs):
                c.all_reduce(b.data_ptr(), b.data_ptr(), 1 << 14, M.FLOAT32, M.SUM, 0)
    torch.cuda.synchronize()
    for c in comms:
        c.destroy()
    print("dumped into", os.environ["NPKIT_DUMP_DIR"])


if __name__ == "__main__":
    main()
