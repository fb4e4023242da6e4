"""Plain-text scene files (twin of host/scene_file.hpp; format documented
there): camera / sphere / plane / triangle / quad, one per line, material
fields after the geometry with the WorldTypes.cuh:15-20 defaults for omitted
ones.  save() writes %.9g floats, which read back bit-exactly."""
from __future__ import annotations

import ctypes as C

import numpy as np

from .abi import Camera, Plane, Quad, Sphere, Triangle, Vec3
from .scenes import Scene, camera_07, material, vec

_GEOM = {"sphere": 4, "plane": 9, "triangle": 9, "quad": 12}


def _mat(vals):
    if not 3 <= len(vals) <= 6:
        raise ValueError("material needs 3..6 numbers")
    m = material(tuple(vals[:3]))
    if len(vals) > 3:
        m.emittance = vals[3]
    if len(vals) > 4:
        m.roughness = vals[4]
    if len(vals) > 5:
        m.refractive_index = vals[5]
    return m


def loads(text: str, name: str = "") -> Scene:
    cam = camera_07()
    sph, pln, tri, quad = [], [], [], []
    for lineno, line in enumerate(text.splitlines(), 1):
        line = line.split("#", 1)[0].split()
        if not line:
            continue
        kind, vals = line[0], [float(np.float32(v)) for v in line[1:]]
        try:
            if kind == "camera" and len(vals) == 6:
                cam = Camera(vec(*vals[:3]), (C.c_float * 2)(vals[3], vals[4]), vals[5])
            elif kind in _GEOM and len(vals) >= _GEOM[kind] + 3:
                g, m = vals[:_GEOM[kind]], _mat(vals[_GEOM[kind]:])
                v = [vec(*g[i:i + 3]) for i in range(0, len(g) - 2, 3)]
                if kind == "sphere":
                    sph.append(Sphere(vec(*g[:3]), g[3], m))
                elif kind == "plane":
                    pln.append(Plane(v[0], (Vec3 * 2)(v[1], v[2]), m))
                elif kind == "triangle":
                    tri.append(Triangle((Vec3 * 3)(*v), m))
                else:
                    quad.append(Quad((Vec3 * 4)(*v), m))
            else:
                raise ValueError(f"cannot parse {kind!r} with {len(vals)} numbers")
        except ValueError as e:
            raise ValueError(f"line {lineno}: {e}") from None
    return Scene(cam, sph, pln, tri, quad, name=name)


def load(path: str) -> Scene:
    with open(path) as f:
        return loads(f.read(), name=path)


def _f(x) -> str:
    return "%.9g" % float(np.float32(x))


def dumps(scene: Scene) -> str:
    out = ["# bwrt scene: camera / sphere / plane / triangle / quad (host/scene_file.hpp)"]
    v = lambda a: " ".join(_f(c) for c in (a.x, a.y, a.z))  # noqa: E731
    m = lambda a: "  " + v(a.albedo) + " " + " ".join(_f(c) for c in (a.emittance, a.roughness, a.refractive_index))  # noqa: E731
    c = scene.camera
    out.append(f"camera {v(c.position)} {_f(c.angle[0])} {_f(c.angle[1])} {_f(c.fov)}")
    ns, npl, nt, nq = scene.counts
    for s in scene.spheres[:ns]:
        out.append(f"sphere {v(s.position)} {_f(s.radius)}{m(s.mat)}")
    for p in scene.planes[:npl]:
        out.append(f"plane {v(p.origin)} {v(p.directions[0])} {v(p.directions[1])}{m(p.mat)}")
    for t in scene.triangles[:nt]:
        out.append("triangle " + " ".join(v(x) for x in t.vertices) + m(t.mat))
    for q in scene.quads[:nq]:
        out.append("quad " + " ".join(v(x) for x in q.vertices) + m(q.mat))
    return "\n".join(out) + "\n"


def save(path: str, scene: Scene) -> None:
    with open(path, "w") as f:
        f.write(dumps(scene))
