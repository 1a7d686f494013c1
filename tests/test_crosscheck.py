"""The compile boundary accepts the reference's own world objects: arrays from
ptmi.scene_compiler.compile_scene + ptmi.bvh.compile_bvh on worlds built by the
reference's scenes.py equal the reference's compile_scene / compile_bvh output
(tests/golden/gen_fixtures.py --crosscheck-ptmi, run where /root/reference exists)."""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def test_reference_worlds_compile_identically():
    with open(os.path.join(HERE, 'golden', 'ptmi_crosscheck.json')) as f:
        d = json.load(f)
    assert set(d['scenes']) == {'wavefront_comparison', 'vol2_final_scene', 'cornell_smoke',
                                'vol2_final_scene_comparison'}
    for name, r in d['scenes'].items():
        assert r['arrays_equal'] and not r['mismatches'] and r['same_primitive_objects'], name
