"""Which exchanges a rank offers to run fused (transport.cc: fusableTbs), from the product loader
on the CPU.  Init fuses an exchange only when both ends offer it (GPU: tests/test_gpu_fused.py)."""
import pytest

import msccl_amd as M
from msccl_amd import xmlgen
from tests.test_gpu_fused import _asymmetric_xml


def _offers(tmp_path, xml, n):
    p = tmp_path / "s.xml"
    p.write_text(xml)
    return [M.fusable_json(str(p), r, n) for r in range(n)]


@pytest.mark.parametrize("inst", [1, 4, 16])
def test_pair_exchange_offers_every_thread_block(tmp_path, inst):
    offers = _offers(tmp_path, xmlgen.allreduce_pair_oneshot(inst, "LL"), 2)
    for r in range(2):
        assert offers[r] == [[k, 0, k, 1 - r] for k in range(inst)]


def test_schedules_without_the_shape_offer_nothing(tmp_path):
    # two-phase all-pairs: s then r (not rrc); one-shot: s then r; ring: rrs / rrcs chains;
    # 2-rank ReduceScatter: s and rrc of different source chunks
    for xml, n in [(xmlgen.allreduce_allpairs(2, 2, "LL"), 2), (xmlgen.allreduce_allpairs(8, 1, "LL"), 8),
                   (xmlgen.allreduce_oneshot(4, 2, "LL"), 4), (xmlgen.allreduce_ring(4, 2, "LL"), 4),
                   (xmlgen.reduce_scatter_allpairs(2, 4, "Simple"), 2)]:
        assert all(o == [] for o in _offers(tmp_path, xml, n))


def test_asymmetric_exchange_is_offered_by_one_end_only(tmp_path):
    offers = _offers(tmp_path, _asymmetric_xml(), 2)
    assert offers[0] == [[0, 0, 0, 1]] and offers[1] == []


def _sendcopy(tmp_path, xml, n):
    p = tmp_path / "sc.xml"
    p.write_text(xml)
    return [M.fusable_json(str(p), r, n, "sendcopy") for r in range(n)]


def _sc_xml(cpy_src, cpy_dst, inplace=False, coll="allreduce"):
    """2 ranks, one tb: s of input chunks [0, 2), a cpy of those chunks to `cpy_dst` = (buf, off),
    then the receive.  cpy_src = (buf, off) of the cpy (the s reads i0)."""
    from msccl_amd.xmlgen import _Tb, _emit
    gpus = {}
    for r in range(2):
        tb = _Tb(0, 1 - r, 1 - r, 0)
        tb.add("s", "i", 0, "o", 0, 2)
        tb.add("cpy", cpy_src[0], cpy_src[1], cpy_dst[0], cpy_dst[1], 2)
        tb.add("r", "i", 0, "o", 2, 2)
        gpus[r] = (4, 4, 4, [tb])
    return _emit("sc", "Simple", 1, 4, 2, coll, inplace, gpus, 0, 1 << 40)


def test_allgather_own_block_copy_send(tmp_path):
    """The out-of-place AllGather's own block: s then cpy of the same chunk, fused."""
    offers = _sendcopy(tmp_path, xmlgen.allgather_allpairs(4, 2, "Simple"), 4)
    assert all(o == [[0, 0], [1, 0]] for o in offers)
    assert all(o == [] for o in _sendcopy(tmp_path, xmlgen.allgather_allpairs(4, 2, "Simple", inplace=True), 4))


@pytest.mark.parametrize("dst,fused", [
    (("o", 0), True),     # another buffer (out of place)
    (("s", 0), True),     # scratch never aliases i / o
    (("i", 0), True),     # a self-copy writes back what it read
    (("i", 2), True),     # disjoint chunks of the same buffer
    (("i", 1), False),    # overlaps the chunks being sent: the pass could send copied values
])
def test_send_copy_needs_disjoint_or_identical_ranges(tmp_path, dst, fused):
    offers = _sendcopy(tmp_path, _sc_xml(("i", 0), dst), 2)
    assert all(o == ([[0, 0]] if fused else []) for o in offers), offers


def test_send_copy_in_place_aliasing(tmp_path):
    # in place AllReduce: i and o are one buffer, so o1 overlaps i0..i1
    assert all(o == [] for o in _sendcopy(tmp_path, _sc_xml(("i", 0), ("o", 1), inplace=True), 2))
    assert all(o == [[0, 0]] for o in _sendcopy(tmp_path, _sc_xml(("i", 0), ("o", 2), inplace=True), 2))
