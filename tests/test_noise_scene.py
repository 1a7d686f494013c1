"""The `marble` edge scene (tests/edge_scenes.py) exercises the megakernel's
wave-cooperative turbulence (perlin_turb3_wave, pt_device.hpp): its Perlin
hits are found from the leaf code's material class, so the scene must put
the noise class (a Lambertian with a noise texture) in its leaf codes. The GPU comparison with the oracle is
tests/test_gpu_edge.py::test_noise_textured_scene."""
import numpy as np

from edge_scenes import edge_scene
from ptmi import scene_data as sd


def test_marble_leaves_carry_the_noise_class():
    sa = edge_scene('marble')[0]
    lay = sd.pack_device(sa)
    refs = lay.nodes[:, 12:14].copy().view(np.int32).ravel()
    leaves = refs[refs < 0]
    cls = (leaves >> 25) & 7
    assert int(np.sum(cls == sd.CLASS_NOISE)) == 5  # the ground and four spheres
    assert [int(np.sum(cls == c)) for c in (sd.CLASS_LAMBERTIAN, sd.CLASS_GLOSSY, sd.CLASS_EMISSIVE)] == [1, 1, 1]
