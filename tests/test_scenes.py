"""Scene inputs: the 07 scene equals allocateScene() (Main.cu:39-67)
value for value, the C++ host scenes equal the Python ones byte for byte,
and the seeded stress scene is pinned by a digest."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from bwrt import scenes

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(REPO, "bwidman-raytracer_amd", "bin", "bwrt_render")
STRESS_DIGEST = "46bf9aa197814263b3bf29079df3a9014a4520536ad71f7d6ca96dc0e73d50ed"


def f32(x):
    return float(np.float32(x))


def test_scene_07_values():
    s = scenes.scene_07()
    assert s.counts == (6, 1, 4, 0)
    cam = s.camera
    assert (cam.position.x, cam.position.y, cam.position.z) == (0, 1, 0)
    assert tuple(cam.angle) == (0, 0) and cam.fov == f32(np.float32(3.1415926535) / 2)
    exp = [((-6, 3, -4), 1, (1, .6, .2), 20, 1, 1.05), ((6, 3, -4), 1, (1, .2, .6), 20, 1, 1.05),
           ((-.5, .2, -3), .2, (.2, .8, .2), 5, 1, 1.05), ((0, .75, -4), .75, (1, 1, 1), 0, .001, 10),
           ((-4, 1, -6), 1, (.2, 0, .8), 0, 1, 1.05), ((4, 2, -8), 2, (1, .1, 0), 0, 1, 1.05)]
    for sp, (p, r, alb, e, rough, ior) in zip(s.spheres, exp):
        assert sp.position.tolist() == [f32(v) for v in p] and sp.radius == f32(r)
        m = sp.mat
        assert m.albedo.tolist() == [f32(v) for v in alb]
        assert (m.emittance, m.roughness, m.refractive_index) == (f32(e), f32(rough), f32(ior))
    pl = s.planes[0]
    assert pl.directions[0].tolist() == [0, 0, 1] and pl.directions[1].tolist() == [1, 0, 0]
    assert pl.mat.albedo.tolist() == [0.5] * 3
    apex = [f32(-1.5), 1.0, f32(-3.5)]
    assert all(t.vertices[2].tolist() == apex for t in s.triangles)
    assert s.triangles[0].vertices[0].tolist() == [-2, 0, -3]


@pytest.mark.parametrize("key", ["07", "01", "04", "04_box"])
def test_cpp_host_scenes_match_python(key, tmp_path):
    if not os.path.exists(CLI):
        pytest.fail("bwrt_render not built (run __graft_entry__.build())")
    out = tmp_path / "scene.bin"
    subprocess.run([CLI, "--scene", key, "--dump-scene", str(out)], check=True)
    s = scenes.SCENES[key]()
    want = bytes(s.camera)
    for arr, n in zip((s.spheres, s.planes, s.triangles, s.quads), s.counts):
        want += C.string_at(arr, C.sizeof(arr._type_) * n)
    assert out.read_bytes() == want


def test_stress_scene_digest():
    s = scenes.stress_scene()
    assert s.counts == (256, 1, 10000, 0)
    assert sum(1 for sp in s.spheres[:256] if sp.mat.emittance > 0) == 8
    d1 = s.digest()
    assert d1 == scenes.stress_scene().digest()  # deterministic
    assert d1 == STRESS_DIGEST
