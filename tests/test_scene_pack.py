"""CPU: the node array's placement (scene_data.NODE_ORDERS, PTMI_NODE_ORDER)
and stride (64 / 80 B) change where nodes sit, never the tree the kernels
walk: from the root ref, every placement reaches the same boxes, refs
resolved, in the same depth-first order (so the traversal, which follows
refs, visits the same nodes in the same order)."""
import numpy as np
import pytest

from ptmi import scene_data as sd


def _walk(L, node_bytes):
    out, stack = [], [L.root_ref]
    while stack:
        r = stack.pop()
        if r < 0:
            out.append(('leaf', int(r)))
            continue
        assert r % node_bytes == 0
        row = L.nodes[r // node_bytes]
        out.append(tuple(np.asarray(row[:12]).tolist()) + (float(row[14]), float(row[15])))
        refs = row[12:14].view(np.int32)
        stack.extend([int(refs[1]), int(refs[0])])
    return out


@pytest.mark.parametrize('name', ['vol2_final_scene', 'wavefront_comparison', 'cornell_smoke'])
def test_every_placement_walks_the_same_tree(name):
    sa = sd.load_fixture(name)
    base = sd.pack_device(sa)
    want = _walk(base, 80)
    for nb in sd.NODE_STRIDES:
        for order in sd.NODE_ORDERS:
            L = sd.pack_device(sa, nb, True, order)
            assert L.n_inner == base.n_inner == sd.pack_device(sa).nodes.shape[0]
            assert L.nodes.shape[1] * 4 == nb
            assert _walk(L, nb) == want, (nb, order)
            if nb == 64 and order == 'pairs':  # two internal siblings share one 128-B line
                refs = L.nodes[:, 12:14].view(np.int32)
                both = (refs[:, 0] >= 0) & (refs[:, 1] >= 0)
                assert np.array_equal(refs[both, 0] // 128, refs[both, 1] // 128)


def test_unknown_order_and_stride_are_refused():
    sa = sd.load_fixture('cornell_smoke')
    with pytest.raises(ValueError):
        sd.pack_device(sa, 80, True, 'random')
    with pytest.raises(ValueError):
        sd.pack_device(sa, 96)
