"""Scene definitions for the benchmark/parity configurations.

* scene_07(): exactly the scene hard-coded in allocateScene()
  (/root/reference/bwidman-raytracer/src/Main.cu:39-67) — configs 3/4.
* scene_01(): the 01_red_circle scene: one emissive
  red unit sphere at distance 3, camera at the origin — config 1.
* scene_04(): the 04_path_tracing stand-in: 07's two
  lights, left-purple and right-red spheres, and the floor plane — config 2.
* scene_04_box(): scene_04 plus the commented-out mirror quads of
  Main.cu:80-84 (exercises quadIntersection, Intersection.cuh:141-173).
* stress_scene(): 10,000 seeded random triangles + 256 spheres (8 emissive)
  + the 07 floor plane — config 5.  Own xorshift32 generator (below).

All values go through float32 exactly as the C++ aggregate initialisers do
(double literal -> float), so the bytes equal the reference's.
"""
from __future__ import annotations

import ctypes as C
import hashlib

import numpy as np

from .abi import Camera, Material, Plane, Quad, SceneStruct, Sphere, Triangle, Vec3

PI = np.float32(3.1415926535)          # Math.cuh:5 (#define PI 3.1415926535f)


def vec(x, y, z) -> Vec3:
    return Vec3(float(x), float(y), float(z))


def material(albedo=(0, 0, 0), emittance=0.0, roughness=1.0, refractive_index=1.05) -> Material:
    """WorldTypes.cuh:15-20 defaults: albedo 0, emittance 0, roughness 1, IOR 1.05."""
    return Material(vec(*albedo), float(emittance), float(roughness), float(refractive_index))


class Scene:
    """Owns the primitive arrays and exposes an rt_scene (SceneStruct)."""

    def __init__(self, camera: Camera, spheres=(), planes=(), triangles=(), quads=(), name=""):
        self.name = name
        self.camera = camera
        self.spheres = (Sphere * max(len(spheres), 1))(*spheres)
        self.planes = (Plane * max(len(planes), 1))(*planes)
        self.triangles = (Triangle * max(len(triangles), 1))(*triangles)
        self.quads = (Quad * max(len(quads), 1))(*quads)
        self.counts = (len(spheres), len(planes), len(triangles), len(quads))
        self.struct = SceneStruct(
            camera,
            C.cast(self.spheres, C.POINTER(Sphere)), len(spheres),
            C.cast(self.planes, C.POINTER(Plane)), len(planes),
            C.cast(self.triangles, C.POINTER(Triangle)), len(triangles),
            C.cast(self.quads, C.POINTER(Quad)), len(quads))

    def ptr(self):
        return C.byref(self.struct)

    def set_camera(self, camera: Camera):
        self.camera = camera
        self.struct.camera = camera

    def digest(self) -> str:
        """SHA-256 over camera + the used bytes of every primitive array."""
        h = hashlib.sha256()
        h.update(bytes(self.camera))
        for arr, n in zip((self.spheres, self.planes, self.triangles, self.quads), self.counts):
            h.update(C.string_at(arr, C.sizeof(arr._type_) * n))
        return h.hexdigest()

    def primitive_bytes(self) -> int:
        return sum(C.sizeof(a._type_) * n for a, n in
                   zip((self.spheres, self.planes, self.triangles, self.quads), self.counts))


def camera_07() -> Camera:
    """Main.cu:39: camera = { {0,1,0}, {0,0}, PI/2 }."""
    return Camera(vec(0, 1, 0), (C.c_float * 2)(0.0, 0.0), float(PI / np.float32(2)))


def _spheres_07():
    return [
        Sphere(vec(-6, 3, -4), 1.0, material((1, 0.6, 0.2), 20)),            # orange light left
        Sphere(vec(6, 3, -4), 1.0, material((1, 0.2, 0.6), 20)),             # purple light right
        Sphere(vec(-0.5, 0.2, -3), 0.2, material((0.2, 0.8, 0.2), 5)),       # green light centre
        Sphere(vec(0, 0.75, -4), 0.75, material((1, 1, 1), 0, 0.001, 10)),   # centre white
        Sphere(vec(-4, 1, -6), 1.0, material((0.2, 0, 0.8), 0, 1)),          # left purple
        Sphere(vec(4, 2, -8), 2.0, material((1, 0.1, 0), 0, 1)),             # right red
    ]


def _floor():
    return Plane(vec(0, 0, 0), (Vec3 * 2)(vec(0, 0, 1), vec(1, 0, 0)), material((0.5, 0.5, 0.5)))


def _pyramid():
    m = material((0.95, 0.9, 0.2))
    return [
        Triangle((Vec3 * 3)(vec(-2, 0, -3), vec(-1, 0, -3), vec(-1.5, 1, -3.5)), m),  # front
        Triangle((Vec3 * 3)(vec(-1, 0, -4), vec(-2, 0, -4), vec(-1.5, 1, -3.5)), m),  # back
        Triangle((Vec3 * 3)(vec(-2, 0, -4), vec(-2, 0, -3), vec(-1.5, 1, -3.5)), m),  # left
        Triangle((Vec3 * 3)(vec(-1, 0, -3), vec(-1, 0, -4), vec(-1.5, 1, -3.5)), m),  # right
    ]


def scene_07() -> Scene:
    """allocateScene(), Main.cu:38-109 (quads commented out there: quadCount = 0)."""
    return Scene(camera_07(), _spheres_07(), [_floor()], _pyramid(), [], name="07_specular_BRDF")


def scene_01() -> Scene:
    cam = Camera(vec(0, 0, 0), (C.c_float * 2)(0.0, 0.0), float(PI / np.float32(2)))
    return Scene(cam, [Sphere(vec(0, 0, -3), 1.0, material((1, 0, 0), 1))], name="01_red_circle")


def scene_04() -> Scene:
    s = _spheres_07()
    return Scene(camera_07(), [s[0], s[1], s[4], s[5]], [_floor()], name="04_path_tracing")


def _mirror_quads():
    """The mirror quads of Main.cu:80-84 (commented out in the reference)."""
    w = 10.0
    m = material((1, 0.8, 0.2), 0, 0.005, 10)
    q = lambda *v: Quad((Vec3 * 4)(*[vec(*p) for p in v]), m)
    return [
        q((w, 0, -w), (w, w, -w), (-w, w, -w), (-w, 0, -w)),                       # front
        q((-w, 0, -w - 1), (-w, w, -w - 1), (w, w, -w - 1), (w, 0, -w - 1)),       # back
        q((-w, 0, -w), (-w, w, -w), (-w, w, -w - 1), (-w, 0, -w - 1)),             # left
        q((w, 0, -w - 1), (w, w, -w - 1), (w, w, -w), (w, 0, -w)),                 # right
        q((w, w, -w), (w, w, -w - 1), (-w, w, -w - 1), (-w, w, -w)),               # top
    ]


def scene_04_box() -> Scene:
    s = _spheres_07()
    return Scene(camera_07(), [s[0], s[1], s[4], s[5]], [_floor()], [], _mirror_quads(),
                 name="04_box_quads")


def empty_scene() -> Scene:
    return Scene(camera_07(), name="empty")


# ---------------------------------------------------------------------------
# Stress scene generator (config 5).  xorshift32 (Marsaglia 13/17/5), seed
# 0x5EED; uniform(a, b) = a + (b - a) * u, u = (x >> 8) * 2**-24, all in
# float32.  The generated bytes are pinned by STRESS_SHA256 (tests).
STRESS_SEED = 0x5EED
STRESS_SHA256 = "46bf9aa197814263b3bf29079df3a9014a4520536ad71f7d6ca96dc0e73d50ed"  # Scene.digest()


class XorShift32:
    def __init__(self, seed: int):
        self.x = seed & 0xFFFFFFFF or 1

    def next(self) -> int:
        x = self.x
        x ^= (x << 13) & 0xFFFFFFFF
        x ^= x >> 17
        x ^= (x << 5) & 0xFFFFFFFF
        self.x = x
        return x

    def uniform(self, a: float, b: float) -> np.float32:
        u = np.float32(self.next() >> 8) * np.float32(2.0 ** -24)
        a32, b32 = np.float32(a), np.float32(b)
        return np.float32(a32 + np.float32(b32 - a32) * u)


def stress_scene(n_triangles=10000, n_spheres=256, n_emissive=8, seed=STRESS_SEED) -> Scene:
    rng = XorShift32(seed)
    tris = []
    for _ in range(n_triangles):
        cx, cy, cz = rng.uniform(-10, 10), rng.uniform(0, 6), rng.uniform(-30, -4)
        size = rng.uniform(0.3, 1.0)
        verts = []
        for _k in range(3):
            dx, dy, dz = rng.uniform(-1, 1), rng.uniform(-1, 1), rng.uniform(-1, 1)
            verts.append(vec(cx + size * dx, cy + size * dy, cz + size * dz))
        alb = (rng.uniform(0.2, 0.95), rng.uniform(0.2, 0.95), rng.uniform(0.2, 0.95))
        rough = rng.uniform(0.01, 1.0) if (rng.next() & 3) == 0 else np.float32(1.0)
        tris.append(Triangle((Vec3 * 3)(*verts), material(alb, 0, rough)))
    sph = []
    for i in range(n_spheres):
        p = vec(rng.uniform(-12, 12), rng.uniform(0.1, 5), rng.uniform(-32, -3))
        r = rng.uniform(0.1, 0.6)
        alb = (rng.uniform(0.2, 1.0), rng.uniform(0.2, 1.0), rng.uniform(0.2, 1.0))
        e = rng.uniform(10, 20) if i < n_emissive else np.float32(0.0)
        rough = rng.uniform(0.001, 1.0)
        ior = rng.uniform(1.05, 10.0)
        sph.append(Sphere(p, float(r), material(alb, e, rough, ior)))
    return Scene(camera_07(), sph, [_floor()], tris, [], name="stress")


SCENES = {
    "07": scene_07,
    "01": scene_01,
    "04": scene_04,
    "04_box": scene_04_box,
    "stress": stress_scene,
    "empty": empty_scene,
}

# BASELINE.json configs: (scene, width, height, spp, max_bounces, gpus)
CONFIGS = {
    "c1": ("01", 256, 256, 1, 1, 0),
    "c2": ("04", 1280, 720, 4, 3, 1),
    "c3": ("07", 1920, 1080, 8, 4, 1),
    "c4": ("07", 3840, 2160, 16, 6, 8),
    "c5": ("stress", 1920, 1080, 32, 8, 8),
}
