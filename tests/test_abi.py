"""The C ABI (include/rt_abi.h): libbwrt.so loads, exports every declared
symbol, and its structs are byte-compatible with the reference's world types
(/root/reference/bwidman-raytracer/src/WorldTypes.cuh:4-53).  No compute
calls here (no GPU in the CPU suite)."""
import ctypes as C

import pytest

from bwrt import abi


def test_library_exports_every_declared_symbol(bwrt_lib):
    declared = abi.declared_functions()
    assert len(declared) >= 20
    missing = [f for f in declared if not hasattr(bwrt_lib, f)]
    assert not missing, missing


@pytest.mark.parametrize("struct,size,offsets", [
    (abi.Vec3, 12, {"x": 0, "y": 4, "z": 8}),
    (abi.Material, 24, {"albedo": 0, "emittance": 12, "roughness": 16, "refractive_index": 20}),
    (abi.Sphere, 40, {"position": 0, "radius": 12, "mat": 16}),
    (abi.Plane, 60, {"origin": 0, "directions": 12, "mat": 36}),
    (abi.Triangle, 60, {"vertices": 0, "mat": 36}),
    (abi.Quad, 72, {"vertices": 0, "mat": 48}),
    (abi.Camera, 24, {"position": 0, "angle": 12, "fov": 20}),
    (abi.SceneStruct, 88, {"camera": 0, "spheres": 24, "sphere_count": 32, "planes": 40,
                           "plane_count": 48, "triangles": 56, "triangle_count": 64, "quads": 72,
                           "quad_count": 80}),
])
def test_struct_layout_matches_reference(struct, size, offsets):
    assert C.sizeof(struct) == size
    for name, off in offsets.items():
        assert getattr(struct, name).offset == off


def test_material_defaults(bwrt_lib):
    m = bwrt_lib.rt_material_default()
    assert (m.albedo.x, m.albedo.y, m.albedo.z, m.emittance, m.roughness) == (0, 0, 0, 0, 1)
    assert m.refractive_index == C.c_float(1.05).value  # WorldTypes.cuh:19


def test_error_strings_and_arg_checks(bwrt_lib):
    assert bwrt_lib.rt_error_string(0) == b"ok"
    assert bwrt_lib.rt_error_string(-5) == b"no scene"
    assert bwrt_lib.rt_shard_rows(1080, 3, 8) == 135
    assert bwrt_lib.rt_shard_rows(55, 1, 2) == 27
    assert bwrt_lib.rt_create(0, None) == -1
    assert bwrt_lib.rt_render(None, 16, 16, 1, None) == -1
    assert bwrt_lib.rt_version().decode().count(".") == 2


def test_no_device_fails_loudly_on_cpu(bwrt_lib):
    """Without a GPU a GPU context refuses to exist (the CPU fallback is a
    separate, explicit backend: rt_create_cpu, tests/test_cpu_fallback.py)."""
    if bwrt_lib.rt_device_count() > 0:
        pytest.skip("a GPU is visible")
    ctx = C.c_void_p()
    assert bwrt_lib.rt_create(0, C.byref(ctx)) == -2  # RT_ERR_NO_DEVICE
