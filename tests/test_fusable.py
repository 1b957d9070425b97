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
