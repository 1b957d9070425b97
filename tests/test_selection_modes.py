"""MSCCL gating by NCCL_ALGO and MSCCL_AMD_REFERENCE_SELECTION (host-only, no GPU).

Reference rules (src/graph/tuning.cc:186-217, src/enqueue.cc:448-460):
  * NCCL_ALGO gates MSCCL for AllReduce only ("Only disable algo for Allreduce since others only
    have one"); MSCCL is off for AllReduce unless NCCL_ALGO lists it;
  * a group with more than one op of a communicator skips MSCCL (tested on the GPU).
This runtime turns MSCCL on by default; MSCCL_AMD_REFERENCE_SELECTION=1 restores the rules."""
import pytest

import msccl_amd as M
from msccl_amd import xmlgen
from oracle import loader as L


@pytest.fixture
def files(tmp_path):
    ar = tmp_path / "ar.xml"
    ar.write_text(xmlgen.allreduce_allpairs(2, 1, "LL"))
    ag = tmp_path / "ag.xml"
    ag.write_text(xmlgen.allgather_allpairs(2, 1, "LL"))
    return str(ar), str(ag)


def _algo(path, coll, count=1024):
    return M.plan_json(path, 0, 2, coll, count, 7, 0, coll == L.ALLREDUCE)["algo"]


@pytest.mark.parametrize("ref,nccl_algo,want", [
    ("0", None, 0), ("0", "MSCCL", 0), ("0", "Ring,Tree", -1), ("0", "^MSCCL", -1), ("0", "^Ring", 0),
    ("1", None, -1), ("1", "MSCCL", 0), ("1", "Ring,MSCCL", 0), ("1", "Ring", -1), ("1", "^Tree", 0),
])
def test_allreduce_gate(files, monkeypatch, ref, nccl_algo, want):
    monkeypatch.setenv("MSCCL_AMD_REFERENCE_SELECTION", ref)
    if nccl_algo is None:
        monkeypatch.delenv("NCCL_ALGO", raising=False)
    else:
        monkeypatch.setenv("NCCL_ALGO", nccl_algo)
    assert _algo(files[0], L.ALLREDUCE) == want


@pytest.mark.parametrize("ref", ["0", "1"])
def test_other_collectives_ignore_nccl_algo(files, monkeypatch, ref):
    monkeypatch.setenv("MSCCL_AMD_REFERENCE_SELECTION", ref)
    monkeypatch.setenv("NCCL_ALGO", "Ring")
    assert _algo(files[1], L.ALLGATHER) == 0
