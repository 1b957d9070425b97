"""Product XML loader (msccl_amd/csrc/xml.cc via the C-ABI) == oracle loader, accept/reject and program."""
import os

import pytest

import msccl_amd as M
from msccl_amd import xmlgen
from oracle import loader as L
from tests.conftest import xml_ngpus
from tests import test_oracle_loader as T


def compare(path, n, ranks=None):
    for r in (ranks if ranks is not None else range(n)):
        rc, prod = M.try_algo_json(path, r, n)
        try:
            o = L.load_xml(path, r, n).to_dict()
            orc = 0
        except L.XmlError as e:
            o, orc = None, e.code
        assert rc == orc, (path, r, rc, orc)
        if o is not None:
            assert prod == o, (path, r)


def test_rccl_fixtures(rccl_xmls):
    for f in rccl_xmls:
        n = xml_ngpus(f)
        compare(f, n, range(n) if n <= 8 else [0, 1, n // 2, n - 1])


GEN = [
    ("ap2", lambda: xmlgen.allreduce_allpairs(2, 4, "LL"), 2),
    ("ap2op", lambda: xmlgen.allreduce_allpairs(2, 2, "Simple", inplace=False), 2),
    ("ap4", lambda: xmlgen.allreduce_allpairs(4, 2, "LL"), 4),
    ("ap8", lambda: xmlgen.allreduce_allpairs(8, 4, "LL"), 8),
    ("ring8", lambda: xmlgen.allreduce_ring(8, 4, "Simple"), 8),
    ("ring4op", lambda: xmlgen.allreduce_ring(4, 2, "LL", inplace=False), 4),
    ("rs8", lambda: xmlgen.reduce_scatter_allpairs(8, 2), 8),
    ("rs4ip", lambda: xmlgen.reduce_scatter_allpairs(4, 1, inplace=True), 4),
    ("ag8", lambda: xmlgen.allgather_allpairs(8, 2), 8),
    ("ag4ip", lambda: xmlgen.allgather_allpairs(4, 1, inplace=True), 4),
]


@pytest.mark.parametrize("name,fn,n", GEN)
def test_generated(tmp_path, name, fn, n):
    p = tmp_path / (name + ".xml")
    p.write_text(fn())
    compare(str(p), n)


def synthetic_cases():
    out = [("ok", T.mk(T.TB_OK)), ("chain", T.mk(T.RE_CHAIN))]
    for i, (text, _code) in enumerate(T.test_rejections.pytestmark[0].args[1]):
        out.append(("rej%d" % i, text))
    return out


def test_synthetic_accept_reject(tmp_path):
    for name, text in synthetic_cases():
        p = tmp_path / (name + ".xml")
        p.write_text(text)
        compare(str(p), 2)


def test_missing_file():
    rc, _ = M.try_algo_json("/nonexistent/x.xml", 0, 2)
    assert rc == 2  # ncclSystemError (xml.cc:881-886)
