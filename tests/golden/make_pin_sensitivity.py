"""How much can the reference-held pin detect?  (TEST INFRASTRUCTURE)

The only real-CUDA outputs of the reference are its PNG screenshots, so the
oracle's quirks are pinned against them only
statistically: the 07 image's 16x16 block means after 1024 frames (MAE <=
1.5 LSB, tests/test_gpu_parity.py test_converges_to_reference_png) and the
01 disc's geometry (tests/test_oracle.py).  This script builds the oracle's
compile-time mutants (oracle/oracle.c ORC_MUTANT 1..9, and 10 = the same
source with FMA contraction), each replacing ONE quirk by its "natural"
formula, runs both checks on every mutant, and records:

  mae_vs_png        block-mean MAE vs Renders/07 (1024 frames, 1920x1080,
                    maxBounces 5, the test's alignment)
  png_check_passes  mae_vs_png <= 1.5: the PNG check would NOT reject it
  disc              the 01 disc check (rows, mean edge error, area)
  mean_abs_diff_vs_oracle  mean |RGB difference| against the unmutated
                    oracle at the same frames and seeds (LSB): the
                    mutant's effect size, independent of the PNG
  pixels_differing_vs_oracle / frame_sum_pixels_differing_vs_oracle
                    pixels whose RGBA8 / float frameSum differ from the
                    unmutated oracle's (what the bit-exact tests see)
  png_where_it_differs  a sharper reading of the same PNG: only the 16x16
                    block channels where mutant and oracle differ by more
                    than 2 LSB (beyond the 1024-frame noise), each one's MAE
                    against the PNG there and how often the mutant is closer

-> tests/golden/pin_sensitivity.json (read by tests/test_oracle.py).

  python tests/golden/make_pin_sensitivity.py [--frames 1024]
(about 3 CPU-minutes per mutant on 8 threads; builds into oracle/_mut/)
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
ORACLE = os.path.join(REPO, "oracle")
sys.path[:0] = [os.path.join(REPO, "bwidman-raytracer_amd"), ORACLE]

import oracle as O  # noqa: E402
from bwrt import scenes  # noqa: E402

MUTANTS = {
    0: ("none", "the oracle as shipped (reference semantics)"),
    1: ("A.5 jitter scale", "0.001 * (W / 1000.0) instead of the integer W / 1000 (Main.cu:291)"),
    2: ("A.6 half-pixel offset", "pixelPosition + 0.5 (Main.cu:287 has none)"),
    3: ("A.9 unit polygon normals", "normalised triangle/quad shading normals (Intersection.cuh:114, 136)"),
    4: ("A.10 tangent frame", "helper-axis test not inverted: no zero tangents for n ~ y (Main.cu:152-153)"),
    5: ("A.11 G1 tan^2", "rough^2 * tan^2 instead of rough^2 * tan^4 in G1 (Main.cu:116-119)"),
    6: ("A.11 isnan guard", "no isnan(G) -> 1 in specularWeight (Main.cu:139-140)"),
    7: ("A.12 forward fold", "acc += T e, T *= brdf cos instead of the innermost-first recursion (Main.cu:268)"),
    8: ("A.14/A.15 std::min/max", "NaN-propagating clamps instead of fminf / fmaxf (Math.cuh:245-247, Main.cu:116)"),
    9: ("libm transcendentals", "glibc sinf / cosf / atanf instead of the Cephes sequence (Main.cu:175-182)"),
    10: ("FMA contraction", "the oracle built with -ffp-contract=fast -march=x86-64-v3"),
}
CFLAGS = ["-O3", "-std=c11", "-fPIC", "-fopenmp", "-fno-fast-math", "-w", "-shared"]


def build(k):
    out = os.path.join(ORACLE, "_mut", f"liboracle_m{k}.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    flags = CFLAGS + (["-ffp-contract=fast", "-march=x86-64-v3"] if k == 10 else
                      ["-ffp-contract=off", f"-DORC_MUTANT={k}"])
    subprocess.run(["gcc", *flags, "-o", out, os.path.join(ORACLE, "oracle.c"), "-lm"], check=True)
    return out


def render_blocks(rgba, g):
    top = rgba[::-1, :, :3]
    dx, dy, ph, pw, b = (int(g[k]) for k in ("dx", "dy", "png_h", "png_w", "block"))
    crop = top[dy:dy + ph, dx:dx + pw]
    hh, ww = ph // b * b, pw // b * b
    return crop[:hh, :ww].astype(np.float64).reshape(hh // b, b, ww // b, b, 3).mean((1, 3))


def block_mae(rgba, g):
    return float(np.abs(render_blocks(rgba, g) - g["blocks"]).mean())


def discriminating(mut_blocks, base_blocks, g, thresh=2.0):
    """The PNG's verdict where the mutant's effect exceeds the noise: block
    channels whose means differ by more than `thresh` LSB between mutant and
    oracle, and each one's MAE against the PNG there."""
    sel = np.abs(mut_blocks - base_blocks) > thresh
    n = int(sel.sum())
    if n == 0:
        return {"block_channels": 0}
    png = g["blocks"]
    em, eb = np.abs(mut_blocks - png)[sel], np.abs(base_blocks - png)[sel]
    return {"block_channels": n, "threshold_lsb": thresh, "mutant_mae": round(float(em.mean()), 4),
            "oracle_mae": round(float(eb.mean()), 4), "mutant_closer_frac": round(float((em < eb).mean()), 4)}


def disc_check(g):
    """tests/test_oracle.py test_01_geometry_matches_reference_png's measures"""
    st = O.render_image(scenes.scene_01(), 1280, 720, 1, 1)
    m = (st.rgba[::-1, :, 0] > 100)[:int(g["png_h"]), :int(g["png_w"])]
    first = np.where(m.any(1), m.argmax(1), -1)
    last = np.where(m.any(1), m.shape[1] - 1 - m[:, ::-1].argmax(1), -1)
    rows = g["first"] >= 0
    rows_match = bool(np.array_equal(first >= 0, rows))
    err = np.concatenate([np.abs(first - g["first"])[rows], np.abs(last - g["last"])[rows]])
    area_png = int((g["last"] - g["first"] + 1)[rows].sum())
    area = int((last - first + 1)[rows].sum())
    passes = rows_match and err.mean() < 1.0 and abs(area - area_png) <= 0.005 * area_png
    return {"rows_match": rows_match, "mean_edge_err_px": round(float(err.mean()), 4),
            "area_rel_diff": round((area - area_png) / area_png, 5), "passes": bool(passes)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1024)
    ap.add_argument("--mutants", default=",".join(map(str, MUTANTS)))
    args = ap.parse_args()
    g07 = np.load(os.path.join(HERE, "07_png_blocks16.npz"))
    g01 = np.load(os.path.join(HERE, "01_png_disc.npz"))
    out_path = os.path.join(HERE, "pin_sensitivity.json")
    res = json.load(open(out_path)) if os.path.exists(out_path) else {}
    res.update({"frames": args.frames, "width": 1920, "height": 1080, "max_bounces": 5,
                "png_threshold_lsb": 1.5, "mutants": res.get("mutants", {})})
    base_rgb = None
    for k in [int(x) for x in args.mutants.split(",")]:
        t0 = time.time()
        O.use_library(build(k))
        st = O.OracleState(1920, 1080)
        chunk = 128
        for f in range(0, args.frames, chunk):
            O.render(scenes.scene_07(), st, min(chunk, args.frames - f), 5, first_frame=1 if f == 0 else None)
        rgb = st.rgba[..., :3].astype(np.int16)
        if k == 0:
            base_rgb, base_acc = rgb, st.accum.copy()
            np.save(os.path.join(ORACLE, "_mut", "base_rgb.npy"), rgb)
            np.save(os.path.join(ORACLE, "_mut", "base_acc.npy"), base_acc)
        elif base_rgb is None:
            base_rgb = np.load(os.path.join(ORACLE, "_mut", "base_rgb.npy"))
            base_acc = np.load(os.path.join(ORACLE, "_mut", "base_acc.npy"))
        acc_diff = ~((st.accum == base_acc) | (np.isnan(st.accum) & np.isnan(base_acc)))
        mae = block_mae(st.rgba, g07)
        np.save(os.path.join(ORACLE, "_mut", f"rgba_m{k}.npy"), st.rgba)
        base_rgba = np.load(os.path.join(ORACLE, "_mut", "rgba_m0.npy"))
        disc_blocks = discriminating(render_blocks(st.rgba, g07), render_blocks(base_rgba, g07), g07)
        name, what = MUTANTS[k]
        res["mutants"][str(k)] = {
            "name": name, "change": what, "mae_vs_png": round(mae, 4), "png_check_passes": mae <= 1.5,
            "disc": disc_check(g01),
            "mean_abs_diff_vs_oracle": round(float(np.abs(rgb - base_rgb).mean()), 4),
            "pixels_differing_vs_oracle": int((rgb != base_rgb).any(-1).sum()),
            "frame_sum_pixels_differing_vs_oracle": int(acc_diff.any(-1).sum()),
            "png_where_it_differs": disc_blocks}
        print(f"mutant {k} ({name}): MAE {mae:.3f}, disc {res['mutants'][str(k)]['disc']['passes']}, "
              f"|diff| {res['mutants'][str(k)]['mean_abs_diff_vs_oracle']} ({time.time() - t0:.0f} s)", flush=True)
        with open(out_path, "w") as f:
            json.dump(res, f, indent=1)
    O.use_library(O.LIB_PATH)


if __name__ == "__main__":
    main()
