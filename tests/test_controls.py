"""Camera controls (Controls.cuh:5-75) through the C ABI, on the CPU.

rt_apply_controls is host code (no GPU): it is compared bit for bit with a
float32 restatement of the reference written here — rotationMatrix3DY(a0) *
rotationMatrix3DX(a1) (Math.cuh:191-225: matrix product by row/column dots),
times (0,0,-1) / (1,0,0) (Math.cuh:144-150), position += / -= moveSpeed * dir
(Math.cuh:12-30) in the reference's key order, moveSpeed = 5*dt,
rotSpeed = 2*dt.  cosf/sinf are the host libm's, as in the reference build.
"""
import ctypes as C

import numpy as np
import pytest

from bwrt import abi
from bwrt.abi import KEYS, CONTROLS_MOVED, CONTROLS_QUIT

f32 = np.float32
_libm = C.CDLL("libm.so.6")
_libm.cosf.restype = C.c_float
_libm.cosf.argtypes = [C.c_float]
_libm.sinf.restype = C.c_float
_libm.sinf.argtypes = [C.c_float]


def dot(a, b):
    return f32(f32(f32(a[0] * b[0]) + f32(a[1] * b[1])) + f32(a[2] * b[2]))


def ref_controls(pos, angle, keys, dt):
    """Controls.cuh:5-75 restated in float32 (returns new pos, angle, moved, quit)."""
    pos = [f32(v) for v in pos]
    angle = [f32(v) for v in angle]
    dt = f32(dt)
    move = f32(f32(5) * dt)
    rot = f32(f32(2) * dt)
    cy, sy = f32(_libm.cosf(angle[0])), f32(_libm.sinf(angle[0]))
    cx, sx = f32(_libm.cosf(angle[1])), f32(_libm.sinf(angle[1]))
    L = [[cy, f32(0), sy], [f32(0), f32(1), f32(0)], [f32(-sy), f32(0), cy]]
    U = [[f32(1), f32(0), f32(0)], [f32(0), cx, f32(-sx)], [f32(0), sx, cx]]
    M = [[dot(L[i], [U[0][j], U[1][j], U[2][j]]) for j in range(3)] for i in range(3)]
    front = [dot(M[i], [f32(0), f32(0), f32(-1)]) for i in range(3)]
    right = [dot(M[i], [f32(1), f32(0), f32(0)]) for i in range(3)]
    moved = False

    def add(v, sign):
        nonlocal pos, moved
        kv = [f32(move * c) for c in v]
        pos = [f32(p + k) if sign > 0 else f32(p - k) for p, k in zip(pos, kv)]
        moved = True

    if keys & KEYS["W"]:
        add(front, +1)
    if keys & KEYS["A"]:
        add(right, -1)
    if keys & KEYS["S"]:
        add(front, -1)
    if keys & KEYS["D"]:
        add(right, +1)
    if keys & KEYS["SPACE"]:
        pos[1] = f32(pos[1] + move); moved = True
    if keys & KEYS["LEFT_SHIFT"]:
        pos[1] = f32(pos[1] - move); moved = True
    if keys & KEYS["LEFT"]:
        angle[0] = f32(angle[0] + rot); moved = True
    if keys & KEYS["RIGHT"]:
        angle[0] = f32(angle[0] - rot); moved = True
    if keys & KEYS["UP"]:
        angle[1] = f32(angle[1] + rot); moved = True
    if keys & KEYS["DOWN"]:
        angle[1] = f32(angle[1] - rot); moved = True
    return pos, angle, moved, bool(keys & KEYS["ESCAPE"])


def test_controls_match_reference_restatement(bwrt_lib):
    rng = np.random.default_rng(7)
    for it in range(3000):
        pos = rng.uniform(-20, 20, 3).astype(np.float32)
        angle = rng.uniform(-7, 7, 2).astype(np.float32)
        dt = np.float32(rng.choice([1 / 60, 1 / 144, 0.25, rng.uniform(0, 0.1)]))
        keys = int(rng.integers(0, 1 << 11)) if it % 3 else (1 << int(rng.integers(0, 11)))
        cam = abi.Camera(abi.Vec3(*map(float, pos)), (C.c_float * 2)(*map(float, angle)), 1.5707964)
        flags = bwrt_lib.rt_apply_controls(C.byref(cam), keys, float(dt))
        p2, a2, moved, quit_ = ref_controls(pos, angle, keys, dt)
        got_p = np.array([cam.position.x, cam.position.y, cam.position.z], np.float32)
        got_a = np.array([cam.angle[0], cam.angle[1]], np.float32)
        assert got_p.tobytes() == np.array(p2, np.float32).tobytes(), (keys, pos, angle, dt)
        assert got_a.tobytes() == np.array(a2, np.float32).tobytes()
        assert bool(flags & CONTROLS_MOVED) == moved
        assert bool(flags & CONTROLS_QUIT) == quit_
        assert np.float32(cam.fov) == np.float32(1.5707964)


def test_controls_no_keys_is_a_no_op(bwrt_lib):
    cam = abi.Camera(abi.Vec3(0.0, 1.0, 0.0), (C.c_float * 2)(0.3, -0.2), 1.5707964)
    before = bytes(cam)
    assert bwrt_lib.rt_apply_controls(C.byref(cam), 0, 0.016) == 0
    assert bytes(cam) == before


def test_controls_forward_moves_along_view(bwrt_lib):
    """Sanity: at angles (0,0) W moves -z by 5*dt, D moves +x, SPACE +y."""
    cam = abi.Camera(abi.Vec3(0.0, 1.0, 0.0), (C.c_float * 2)(0.0, 0.0), 1.5707964)
    assert bwrt_lib.rt_apply_controls(C.byref(cam), KEYS["W"] | KEYS["D"] | KEYS["SPACE"], 0.1) == CONTROLS_MOVED
    assert (cam.position.x, cam.position.y, cam.position.z) == pytest.approx((0.5, 1.5, -0.5), abs=1e-6)


def test_controls_null_camera(bwrt_lib):
    assert bwrt_lib.rt_apply_controls(None, KEYS["W"], 0.1) == abi.RT_ERR_INVALID_ARGUMENT
    assert bwrt_lib.rt_controls(None, KEYS["W"], 0.1) == abi.RT_ERR_INVALID_ARGUMENT
