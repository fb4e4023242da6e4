#!/usr/bin/env python3
"""Offline study for config 5 (stress scene): what a wider BVH would save per
ray, before building one on the GPU (VERDICT r03 "next" #2).

One binned-SAH build (16 bins, leaves <= 8 primitives, no spatial splits)
over the stress scene's 10,000 triangles and 256 spheres; the same tree
collapsed to 4- and 8-wide nodes (the internal child of largest surface area
opened first, Wald et al. / Ylitie et al. 2017).  Rays: camera rays of the 07
camera at random pixels of 1920x1080, plus one diffuse bounce from each
camera ray's hit (a random direction in the normal's hemisphere), in float64.
Walk: closest-first with a stack, leaves tested when reached, boxes pruned
against the closest hit (the CPU fallback's order; the GPU's threaded walk
speculates past parked leaves and makes about twice the visits).

Per ray it reports node fetches, child-box tests, primitive tests, and node
bytes fetched for the formats a GPU would read: binary fp16 16-byte nodes
(the product's), a compressed 4-wide node of 64 B and an 8-wide node of 80 B
(quantised child boxes, CWBVH).  usage: tools/wide_bvh_study.py [rays]
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "bwidman-raytracer_amd")]
from bwrt import scenes  # noqa: E402


def prims_of(scene):
    tris = []
    for i in range(scene.counts[2]):
        t = scene.triangles[i]
        tris.append([[v.x, v.y, v.z] for v in t.vertices])
    sph = []
    for i in range(scene.counts[0]):
        s = scene.spheres[i]
        sph.append([s.position.x, s.position.y, s.position.z, abs(s.radius)])
    tris, sph = np.array(tris, np.float64), np.array(sph, np.float64)
    lo = np.concatenate([tris.min(1), sph[:, :3] - sph[:, 3:]])
    hi = np.concatenate([tris.max(1), sph[:, :3] + sph[:, 3:]])
    return tris, sph, lo, hi


def area(lo, hi):
    d = np.maximum(hi - lo, 0.0)
    return 2.0 * (d[..., 0] * d[..., 1] + d[..., 1] * d[..., 2] + d[..., 2] * d[..., 0])


class Node:
    __slots__ = ("lo", "hi", "kids", "prims")

    def __init__(self, lo, hi):
        self.lo, self.hi, self.kids, self.prims = lo, hi, [], None


def build(idx, lo, hi, max_leaf=8, bins=16):
    nlo, nhi = lo[idx].min(0), hi[idx].max(0)
    node = Node(nlo, nhi)
    if len(idx) <= max_leaf:
        node.prims = idx
        return node
    c = 0.5 * (lo[idx] + hi[idx])
    best = (np.inf, None, None)
    for a in range(3):
        cmin, cmax = c[:, a].min(), c[:, a].max()
        if cmax - cmin < 1e-12:
            continue
        b = np.minimum(((c[:, a] - cmin) / (cmax - cmin) * bins).astype(int), bins - 1)
        for s in range(1, bins):
            L, R = idx[b < s], idx[b >= s]
            if len(L) == 0 or len(R) == 0:
                continue
            cost = area(lo[L].min(0), hi[L].max(0)) * len(L) + area(lo[R].min(0), hi[R].max(0)) * len(R)
            if cost < best[0]:
                best = (cost, L, R)
    if best[1] is None or best[0] >= area(nlo, nhi) * len(idx) and len(idx) <= 127:
        node.prims = idx
        return node
    node.kids = [build(best[1], lo, hi, max_leaf, bins), build(best[2], lo, hi, max_leaf, bins)]
    return node


def collapse(node, width):
    if node.prims is not None:
        return node
    kids = list(node.kids)
    while len(kids) < width:
        inner = [k for k in kids if k.prims is None]
        if not inner:
            break
        big = max(inner, key=lambda k: area(k.lo, k.hi))
        kids.remove(big)
        kids += big.kids
    w = Node(node.lo, node.hi)
    w.kids = [collapse(k, width) for k in kids]
    return w


def count_nodes(node):
    return 0 if node.prims is not None else 1 + sum(count_nodes(k) for k in node.kids)


def hit_prim(p, o, d, tris, sph, ntri):
    if p < ntri:  # Moller-Trumbore (any exact triangle test does for counting)
        v0, v1, v2 = tris[p]
        e1, e2 = v1 - v0, v2 - v0
        h = np.cross(d, e2)
        a = e1 @ h
        if abs(a) < 1e-12:
            return np.inf
        f = 1.0 / a
        s = o - v0
        u = f * (s @ h)
        if u < 0 or u > 1:
            return np.inf
        q = np.cross(s, e1)
        v = f * (d @ q)
        if v < 0 or u + v > 1:
            return np.inf
        t = f * (e2 @ q)
        return t if t > 1e-4 else np.inf
    c, r = sph[p - ntri, :3], sph[p - ntri, 3]
    xp = o - c
    b = 2 * (xp @ d)
    cc = xp @ xp - r * r
    disc = b * b - 4 * (d @ d) * cc
    if disc < 0:
        return np.inf
    t = (-b - np.sqrt(disc)) / (2 * (d @ d))
    return t if t > 1e-4 else np.inf


def slab(lo, hi, o, inv, tmax):
    t0, t1 = (lo - o) * inv, (hi - o) * inv
    tn = np.maximum(np.minimum(t0, t1).max(-1), 0.0)
    tf = np.maximum(t0, t1).min(-1)
    return tn, (tn <= tf) & (tn <= tmax)


def walk(root, o, d, tris, sph, ntri, st):
    inv = 1.0 / np.where(np.abs(d) < 1e-20, 1e-20, d)
    best, stack = np.inf, [root]
    while stack:
        n = stack.pop()
        st["fetch"] += 1
        kids = n.kids
        klo = np.array([k.lo for k in kids])
        khi = np.array([k.hi for k in kids])
        st["box"] += len(kids)
        tn, ok = slab(klo, khi, o, inv, best)
        order = np.argsort(tn)
        push = []
        for i in order:
            if not ok[i] or tn[i] > best:
                continue
            k = kids[i]
            if k.prims is not None:
                for p in k.prims:
                    st["prim"] += 1
                    best = min(best, hit_prim(int(p), o, d, tris, sph, ntri))
            else:
                push.append((tn[i], k))
        for t, k in sorted(push, key=lambda x: -x[0]):
            if t <= best:
                stack.append(k)
    return best


def main():
    nrays = int(sys.argv[1]) if len(sys.argv) > 1 else 1500
    scene = scenes.stress_scene()
    tris, sph, lo, hi = prims_of(scene)
    ntri = len(tris)
    sys.setrecursionlimit(100000)
    root = build(np.arange(len(lo)), lo, hi)
    trees = {2: root, 4: collapse(root, 4), 8: collapse(root, 8)}
    rng = np.random.default_rng(5)
    cam = np.array([0.0, 1.0, 0.0])
    W, H = 1920, 1080
    rays = []
    for _ in range(nrays):
        x, y = rng.integers(W), rng.integers(H)
        d = np.array([x - W // 2, y - H // 2, -(W // 2)], np.float64)  # FOV pi/2, angles 0 (Main.cu:287-288)
        rays.append((cam, d / np.linalg.norm(d)))
    stats = {}
    for wdt, tree in trees.items():
        st = {"fetch": 0, "box": 0, "prim": 0}
        sec = []
        for o, d in rays:
            t = walk(tree, o, d, tris, sph, ntri, st)
            if wdt == 2 and np.isfinite(t):
                p = o + t * d
                r = rng.normal(size=3)
                r /= np.linalg.norm(r)
                sec.append((p, r))
        if wdt == 2:
            sec_rays = sec
        for o, d in sec_rays:
            walk(tree, o, d, tris, sph, ntri, st)
        n = len(rays) + len(sec_rays)
        stats[wdt] = {k: v / n for k, v in st.items()}
        stats[wdt]["nodes"] = count_nodes(tree)
    node_bytes = {2: 16, 4: 64, 8: 80}
    print(f"stress scene, {len(rays)} camera + {len(sec_rays)} bounce rays; binned SAH, leaves <= 8")
    print("width  nodes  fetches/ray  child-box tests/ray  prim tests/ray  node bytes/ray (node size)")
    for wdt in (2, 4, 8):
        s = stats[wdt]
        print(f"{wdt:5d}  {s['nodes']:5d}  {s['fetch']:11.1f}  {s['box']:19.1f}  {s['prim']:14.1f}  "
              f"{s['fetch'] * node_bytes[wdt]:8.0f} ({node_bytes[wdt]} B)")


if __name__ == "__main__":
    main()
