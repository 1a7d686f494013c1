"""CPU: the packed node array walks the reference's tree: from the root ref,
following refs (byte offsets of 80-B nodes), the walk reaches every internal
node's two child boxes and every leaf in the reference's depth-first order.
Other strides and placements are refused."""
import numpy as np
import pytest

from ptmi import scene_data as sd


def _walk(L):
    out, stack = [], [L.root_ref]
    while stack:
        r = stack.pop()
        if r < 0:
            out.append(('leaf', int(r)))
            continue
        assert r % sd.NODE_BYTES == 0
        row = L.nodes[r // sd.NODE_BYTES]
        out.append(tuple(np.asarray(row[:12]).tolist()) + (float(row[14]), float(row[15])))
        refs = row[12:14].view(np.int32)
        stack.extend([int(refs[1]), int(refs[0])])
    return out


def _ref_walk(sa):
    """The same walk over the reference's own BVH arrays."""
    b = sa.bvh
    left, right, pidx = b['bvh_left_child'], b['bvh_right_child'], b['bvh_prim_idx']
    out, stack = [], [0]
    while stack:
        i = stack.pop()
        if pidx[i] >= 0:
            out.append('leaf')
            continue
        l, r = int(left[i]), int(right[i])
        out.append(tuple(np.concatenate([np.stack([b['bvh_bbox_min'][l], b['bvh_bbox_min'][r]], 1).ravel(),
                                         np.stack([b['bvh_bbox_max'][l], b['bvh_bbox_max'][r]], 1).ravel()]).tolist()))
        stack.extend([r, l])
    return out


@pytest.mark.parametrize('name', ['vol2_final_scene', 'wavefront_comparison', 'cornell_smoke'])
def test_node_array_walks_the_reference_tree(name):
    sa = sd.load_fixture(name)
    L = sd.pack_device(sa)
    got = _walk(L)
    want = _ref_walk(sa)
    assert len(got) == len(want)
    for g, w in zip(got, want):
        if w == 'leaf':
            assert g[0] == 'leaf'
        else:  # boxes interleaved per component: min.x L,R, min.y L,R, ..., max.z L,R
            assert g[:12] == w


def test_unknown_stride_is_refused():
    sa = sd.load_fixture('cornell_smoke')
    with pytest.raises(ValueError):
        sd.pack_device(sa, 64)
    with pytest.raises(ValueError):
        sd.pack_device(sa, 96)
