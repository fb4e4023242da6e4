"""Seeded scene generators shared by the GPU parity and CPU-fallback tests."""
import numpy as np

from bwrt import scenes


def _random_scene(seed):
    """Seeded random scene with the awkward cases the reference's arithmetic
    meets: rays starting inside spheres (camera inside one), shared triangle
    edges (ties), degenerate (zero-area) triangles, non-planar / non-convex
    quads, planes with non-unit normals, roughness 0 and 1, IOR 1 (no
    Fresnel contrast), emitters of every primitive kind."""
    import ctypes as C
    from bwrt.abi import Camera, Plane, Quad, Sphere, Triangle, Vec3
    rng = np.random.default_rng(seed)
    U = lambda a, b, n=None: rng.uniform(a, b, n)  # noqa: E731
    v = lambda p: Vec3(*map(float, p))  # noqa: E731

    def mat():
        m = scenes.material(tuple(U(0, 1, 3)), float(rng.choice([0, 0, 0, U(1, 20)])),
                            float(rng.choice([0.0, 1.0, U(0, 1), U(0, 0.05)])),
                            float(rng.choice([1.0, 1.05, U(1, 10)])))
        return m
    cam = Camera(v(U(-1, 1, 3) + [0, 1, 0]), (C.c_float * 2)(*map(float, U(-0.6, 0.6, 2))),
                 float(U(0.8, 2.2)))
    sph = [Sphere(v(U(-4, 4, 3) + [0, 1, -6]), float(U(0.2, 2)), mat()) for _ in range(int(rng.integers(0, 6)))]
    if seed % 3 == 0:  # camera inside a sphere
        sph.append(Sphere(v([cam.position.x, cam.position.y, cam.position.z]), 0.5, mat()))
    pln = [Plane(v([0, 0, 0]), (Vec3 * 2)(v([0, 0, float(U(0.5, 3))]), v([float(U(0.5, 3)), 0, 0])), mat())]
    if seed % 2:
        pln.append(Plane(v([0, 0, -12]), (Vec3 * 2)(v(U(-1, 1, 3)), v(U(-1, 1, 3))), mat()))
    tri = []
    for _ in range(int(rng.integers(0, 8))):
        a, b, c = (U(-3, 3, 3) + [0, 1.5, -5] for _ in range(3))
        tri.append(Triangle((Vec3 * 3)(v(a), v(b), v(c)), mat()))
        if rng.random() < 0.5:  # neighbour sharing the edge a-b
            d = U(-3, 3, 3) + [0, 1.5, -5]
            tri.append(Triangle((Vec3 * 3)(v(b), v(a), v(d)), mat()))
    tri.append(Triangle((Vec3 * 3)(v([0, 1, -4]), v([1, 1, -4]), v([2, 1, -4])), mat()))  # zero area
    quads = []
    for _ in range(int(rng.integers(0, 4))):
        pts = [U(-3, 3, 3) + [0, 1.5, -7] for _ in range(4)]
        quads.append(Quad((Vec3 * 4)(*[v(p) for p in pts]), mat()))
    return scenes.Scene(cam, sph, pln, tri, quads, name=f"random{seed}")


def _scaled(scene, k):
    """The same scene with every coordinate (camera, primitives) times k."""
    for arr, n in zip((scene.spheres, scene.planes, scene.triangles, scene.quads), scene.counts):
        for i in range(n):
            p = arr[i]
            for name in ("position", "origin"):
                if hasattr(p, name):
                    q = getattr(p, name)
                    q.x, q.y, q.z = q.x * k, q.y * k, q.z * k
            if hasattr(p, "radius"):
                p.radius = p.radius * k
            for vs in ("vertices",):
                if hasattr(p, vs):
                    for q in getattr(p, vs):
                        q.x, q.y, q.z = q.x * k, q.y * k, q.z * k
    c = scene.camera
    c.position.x, c.position.y, c.position.z = c.position.x * k, c.position.y * k, c.position.z * k
    scene.set_camera(c)
    return scene
