"""Oracle XML loader: pinned against the reference loader's own output and its accept/reject rules.

Pins: SURVEY.md Appendix D records what the reference loader (graph/xml.cc + graph/topo.cc,
compiled by the survey session) produced for the RCCL-shipped msccl-tools XMLs; the asserts
below restate those observations.  Accept/reject cases restate topo.cc:759-1193 and
xml.cc:20-211 rule by rule.
"""
import os

import pytest

from oracle import loader as L
from tests.conftest import RCCL_XML_DIR

AP32 = os.path.join(RCCL_XML_DIR, "allreduce-allpairs-8n-ll-32tb.xml")
AP32OP = os.path.join(RCCL_XML_DIR, "allreduce-allpairs-8n-ll-32tb-op.xml")
APSIMPLE = os.path.join(RCCL_XML_DIR, "allreduce-allpairs-8n-simple.xml")


def need(p):
    if not os.path.exists(p):
        pytest.skip("fixture %s missing" % p)


def test_appendix_d_rank0_header():
    need(AP32)
    a = L.load_xml(AP32, 0, 8)
    assert a.valid and a.nBlocks == 32 and a.nchannels == 4 and a.nchunksperloop == 256
    assert a.nScratchChunks == 224 and a.proto == L.PROTO_LL and a.minBytes == 0 and a.maxBytes == 65536


def test_appendix_d_tb0_fused_reduce():
    need(AP32)
    tb0 = L.load_xml(AP32, 0, 8).tbs[0]
    assert len(tb0.transfers) == 1
    t = tb0.transfers[0]
    assert (t.type, t.srcbuf, t.dstbuf, t.dstoff, t.count, t.hasDep) == (L.RE, L.SCRATCH, L.INPUT, 0, 1, 1)
    deps = [(tb0.depBid[t.depPtr + i], tb0.depStep[t.depPtr + i]) for i in range(t.numDeps)]
    assert deps == [(8, 1), (12, 1), (16, 1), (20, 1), (24, 1), (28, 1), (4, 1)]
    assert tb0.redSrcOff[t.redPtr:t.redPtr + t.numReds] == [0, 8, 16, 24, 32, 40, 48]


def test_appendix_d_tb4_program():
    need(AP32)
    tb4 = L.load_xml(AP32, 0, 8).tbs[4]
    tr = tb4.transfers
    assert [(x.type, x.srcbuf, x.srcoff, x.dstbuf, x.dstoff, x.count, x.hasDep) for x in tr] == [
        (L.SEND, L.INPUT, 8, L.SCRATCH, 0, 8, 0),
        (L.RECV, L.INPUT, 0, L.SCRATCH, 0, 8, 1),
        (L.RE, L.SCRATCH, 49, L.INPUT, 1, 1, 1),
        (L.SEND, L.INPUT, 0, L.INPUT, 0, 8, 0),
        (L.RECV, L.INPUT, 8, L.INPUT, 8, 8, 0),
    ]
    assert tb4.redSrcOff == [1, 9, 17, 25, 33, 41, 49]
    assert tr[3].numDeps == 7  # six nops + the send's own dependency on tb0


@pytest.mark.parametrize("rank", [0, 3, 7])
def test_appendix_d_channels_have_7_peers(rank):
    need(AP32)
    a = L.load_xml(AP32, rank, 8)
    for c in range(4):
        sends = [t.send for t in a.tbs if t.chan == c and t.send >= 0]
        recvs = [t.recv for t in a.tbs if t.chan == c and t.recv >= 0]
        assert sorted(sends) == sorted(recvs) == [p for p in range(8) if p != rank]


def test_appendix_d_op_variant_copy_first():
    need(AP32OP)
    a = L.load_xml(AP32OP, 0, 8)
    t = a.tbs[0].transfers[0]
    assert (t.type, t.srcbuf, t.srcoff, t.dstbuf, t.dstoff, t.count, t.hasDep) == (L.CPY, L.INPUT, 0, L.OUTPUT, 0, 8, 1)
    assert a.inplace == 0


def test_appendix_d_simple_variant():
    need(APSIMPLE)
    a = L.load_xml(APSIMPLE, 0, 8)
    assert a.nBlocks == 64 and a.nchannels == 8 and a.nchunksperloop == 512 and a.proto == L.PROTO_SIMPLE


def test_scratch_slots_ascending_peers():
    """Appendix B: rank r's scratch slots hold peers in ascending order, skipping r."""
    need(AP32)
    for r in (0, 3, 7):
        a = L.load_xml(AP32, r, 8)
        peers = [p for p in range(8) if p != r]
        for tb in a.tbs:
            if tb.recv >= 0 and tb.chan == 0:
                assert tb.transfers[1].dstoff == peers.index(tb.recv) * 8


# ----------------------------------------------------------------------------- synthetic rules
HDR = '<algo name="t" proto="LL" nchannels="1" nchunksperloop="2" ngpus="2" coll="allreduce" inplace="1">'


def mk(body0, body1=None, hdr=HDR):
    body1 = body0 if body1 is None else body1
    return (hdr + '\n  <gpu id="0" i_chunks="2" o_chunks="0" s_chunks="1">\n' + body0 + "  </gpu>\n"
            '  <gpu id="1" i_chunks="2" o_chunks="0" s_chunks="1">\n' + body1 + "  </gpu>\n</algo>\n")


TB_OK = ('    <tb id="0" send="1" recv="1" chan="0">\n'
         '      <step s="0" type="s" srcbuf="i" srcoff="0" dstbuf="s" dstoff="0" cnt="1" depid="-1" deps="-1" hasdep="0"/>\n'
         '      <step s="1" type="r" srcbuf="i" srcoff="0" dstbuf="s" dstoff="0" cnt="1" depid="-1" deps="-1" hasdep="0"/>\n'
         "    </tb>\n")


def test_minimal_ok():
    a = L.parse_xml(mk(TB_OK), 0, 2)
    assert a.nBlocks == 1 and len(a.tbs[0].transfers) == 2


@pytest.mark.parametrize("text,code", [
    (mk(TB_OK).replace("  <gpu", "\t<gpu", 1), L.INTERNAL),                     # tab is not whitespace
    (mk(TB_OK).replace('ngpus="2"', 'ngpus="4"'), L.INVALID_USAGE),              # ngpus != nRanks
    (mk(TB_OK).replace('proto="LL"', 'proto="ll"'), L.INVALID_USAGE),            # protocol name
    (mk(TB_OK).replace('coll="allreduce"', 'coll="bcast"'), L.INVALID_USAGE),    # collective name
    (mk(TB_OK).replace('srcbuf="i" srcoff="0" dstbuf="s" dstoff="0" cnt="1" depid="-1" deps="-1" hasdep="0"/>\n      <step s="1"',
                       'srcbuf="x" srcoff="0" dstbuf="s" dstoff="0" cnt="1" depid="-1" deps="-1" hasdep="0"/>\n      <step s="1"'),
     L.INVALID_USAGE),                                                           # buffer name
    (mk(TB_OK.replace('cnt="1" depid="-1" deps="-1" hasdep="0"/>\n      <step s="1"',
                      'cnt="72" depid="-1" deps="-1" hasdep="0"/>\n      <step s="1"')), L.INTERNAL),  # cnt >= 72
    (mk(TB_OK.replace('srcoff="0" dstbuf="s" dstoff="0" cnt="1" depid="-1" deps="-1" hasdep="0"/>\n      <step s="1"',
                      'srcoff="2" dstbuf="s" dstoff="0" cnt="1" depid="-1" deps="-1" hasdep="0"/>\n      <step s="1"')),
     L.INVALID_USAGE),                                                           # src offset bound
    (mk(TB_OK.replace('tb id="0"', 'tb id="1"')), L.INVALID_USAGE),               # tb ids must start at 0
    (mk(TB_OK + TB_OK), L.INVALID_USAGE),                                        # duplicate tb id
    (mk(TB_OK.replace('send="1"', 'send="0"')), L.INVALID_USAGE),                # peer == self
    (mk(TB_OK.replace('send="1"', 'send="-1"')), L.INVALID_USAGE),               # send without sendpeer
    (mk(TB_OK.replace('chan="0"', 'chan="32"')), L.INVALID_USAGE),               # channel out of range
    (mk(TB_OK.replace('hasdep="0"/>\n    </tb>', 'hasdep="2"/>\n    </tb>')), L.INTERNAL),  # hasdep not 0/1
    (mk(TB_OK.replace('<step s="1"', '<step s="256"')), L.INTERNAL),             # step >= 256
    (mk(TB_OK.replace('type="r"', 'type="q"')), L.INTERNAL),                     # unknown type
    (mk(TB_OK).replace('nchannels="1"', "nchannels='1'"), L.INTERNAL),           # value must close with "
    (mk(TB_OK).replace("</algo>", ""), L.INTERNAL),                              # unterminated
    (mk(TB_OK).replace('inplace="1"', 'inplace="1" nthreads="100"'), L.INVALID_USAGE),  # nthreads % 32
    (mk(TB_OK).replace('inplace="1"', 'inplace="1" minBytes="10" maxBytes="5"'), L.INVALID_USAGE),
    (mk(TB_OK).replace('i_chunks="2"', 'i_chunks="3"', 1), L.INVALID_USAGE),     # i_chunks vs nchunksperloop
])
def test_rejections(text, code):
    with pytest.raises(L.XmlError) as ei:
        L.parse_xml(text, 0, 2)
    assert ei.value.code == code


def test_comments_unknown_elements_and_attr_limit():
    extra = " ".join('a%d="1"' % i for i in range(20))
    text = "<!-- header comment -->\n<foo><bar x=\"1\"/></foo>\n" + mk(
        TB_OK.replace('<tb id="0"', "<!-- c --><tb id=\"0\"").replace("</tb>", '<junk z="1"/></tb>'))
    # extra attributes after the real ones: parsed and dropped beyond MAX_ATTR_COUNT (16)
    a = L.parse_xml(text.replace('inplace="1"', 'inplace="1" ' + extra, 1), 0, 2)
    assert a.nBlocks == 1
    # 20 extra attributes first: the real ones fall beyond MAX_ATTR_COUNT and are lost
    with pytest.raises(L.XmlError):
        L.parse_xml(text.replace('name="t" proto', 'name="t" ' + extra + " proto", 1), 0, 2)


def test_strtol_semantics():
    assert L._strtol("0x10") == 16 and L._strtol("010") == 8 and L._strtol("12abc") == 12 and L._strtol("-3") == -3


RE_CHAIN = ('    <tb id="0" send="-1" recv="-1" chan="0">\n'
            '      <step s="0" type="nop" srcbuf="i" srcoff="-1" dstbuf="o" dstoff="-1" cnt="0" depid="1" deps="0" hasdep="0"/>\n'
            '      <step s="1" type="re" srcbuf="s" srcoff="0" dstbuf="i" dstoff="0" cnt="1" depid="1" deps="1" hasdep="0"/>\n'
            '      <step s="2" type="re" srcbuf="i" srcoff="1" dstbuf="i" dstoff="0" cnt="1" depid="-1" deps="-1" hasdep="0"/>\n'
            '      <step s="3" type="re" srcbuf="i" srcoff="1" dstbuf="i" dstoff="0" cnt="1" depid="-1" deps="-1" hasdep="1"/>\n'
            "    </tb>\n"
            '    <tb id="1" send="1" recv="1" chan="0">\n'
            '      <step s="0" type="s" srcbuf="i" srcoff="0" dstbuf="s" dstoff="0" cnt="1" depid="-1" deps="-1" hasdep="1"/>\n'
            '      <step s="1" type="r" srcbuf="i" srcoff="0" dstbuf="s" dstoff="0" cnt="1" depid="-1" deps="-1" hasdep="1"/>\n'
            "    </tb>\n")


def test_nop_packing_and_reduce_fusion():
    a = L.parse_xml(mk(RE_CHAIN), 0, 2)
    tb = a.tbs[0]
    # nop's dependency is packed into the first re; the src buffer changes at s=2 so the chain
    # restarts there and s=3 fuses into it (topo.cc:1043-1053)
    assert len(tb.transfers) == 2
    t0, t1 = tb.transfers
    assert t0.numDeps == 2 and [tb.depBid[i] for i in range(2)] == [1, 1] and t0.numReds == 1
    assert t1.numDeps == 0 and t1.numReds == 2 and t1.hasDep == 1
    assert tb.redSrcOff == [0, 1, 1]


def test_dependency_chain_must_end_on_depid():
    bad = RE_CHAIN.replace('<step s="1" type="re" srcbuf="s" srcoff="0" dstbuf="i" dstoff="0" cnt="1" depid="1" deps="1"',
                           '<step s="1" type="re" srcbuf="s" srcoff="0" dstbuf="i" dstoff="0" cnt="1" depid="-1" deps="-1"')
    with pytest.raises(L.XmlError) as ei:
        L.parse_xml(mk(bad), 0, 2)
    assert ei.value.code == L.INVALID_USAGE


def test_file_list_skips_failures(tmp_path):
    good = tmp_path / "g.xml"
    good.write_text(mk(TB_OK))
    bad = tmp_path / "b.xml"
    bad.write_text("<algo")
    algos = L.load_xml_files(":".join([str(bad), str(good), str(tmp_path / "missing.xml"), str(good)]), 0, 2)
    assert len(algos) == 2
