"""Ring schedules over the full xGMI mesh (xmlgen.hamiltonian_decomposition / ring_cycles).

On a fully connected 8-GPU node the C4 ring AllReduce should use every GPU's 7 links: the
complete directed graph K8* splits into 7 arc-disjoint directed Hamiltonian cycles (Tillson's
theorem holds for every n except 4 and 6), while the rotations i -> i + s with s coprime to 8 give
only 4 ("disjoint directed Hamiltonian cycles on the 8-GPU full mesh")."""
import collections

import pytest

from msccl_amd import xmlgen
from oracle import loader as L


@pytest.mark.parametrize("n", [2, 3, 5, 7, 8, 9, 10, 12, 16])
def test_decomposition_covers_every_arc_once(n):
    cyc = xmlgen.hamiltonian_decomposition(n)
    assert cyc is not None and len(cyc) == n - 1
    arcs = collections.Counter()
    for c in cyc:
        assert sorted(c) == list(range(n))          # a Hamiltonian cycle
        for i in range(n):
            arcs[(c[i], c[(i + 1) % n])] += 1
    assert set(arcs) == {(i, j) for i in range(n) for j in range(n) if i != j}
    assert set(arcs.values()) == {1}


@pytest.mark.parametrize("n", [4, 6])
def test_no_decomposition_falls_back_to_rotations(n):
    assert xmlgen.hamiltonian_decomposition(n) is None
    rings = xmlgen.ring_cycles(n, 4)
    assert all(sorted(r) == list(range(n)) for r in rings)


def test_c4_schedule_uses_all_56_links():
    """The C4 schedule (8 ranks, 32 channels): every directed link carries a ring, and no link
    carries more than ceil(32 / 7) = 5 channels (the stride form: 8 channels on 4 links)."""
    n, ch = 8, 32
    x = xmlgen.allreduce_ring(n, ch, "Simple", True, 0, 1 << 40, name="c4_ring")
    load = collections.Counter()
    for r in range(n):
        a = L.parse_xml(x, r, n)
        assert a.valid
        for tb in a.tbs:
            load[(r, tb.send)] += 1
    assert len(load) == n * (n - 1)
    assert max(load.values()) == 5 and min(load.values()) == 4
    old = collections.Counter()
    for st in [1, 3, 5, 7] * 8:
        for r in range(n):
            old[(r, (r + st) % n)] += 1
    assert len(old) == 32 and max(old.values()) == 8


def test_ring_xml_matches_the_loader_on_every_rank():
    x = xmlgen.allreduce_ring(8, 8, "Simple")
    rings = xmlgen.ring_cycles(8, 8)
    for r in range(8):
        a = L.parse_xml(x, r, 8)
        for c, tb in enumerate(a.tbs):
            pos = rings[c].index(r)
            assert tb.send == rings[c][(pos + 1) % 8] and tb.recv == rings[c][pos - 1]
