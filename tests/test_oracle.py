"""Pinning the oracle (oracle/oracle.c) to the reference's own outputs.

The reference has no tests or fixtures; its renders are the only outputs of
the real CUDA program (Renders/*.png).  Fixtures derived from them live in
tests/golden/ (made by tests/golden/make_golden.py in the build container):
  * 01_red_circle.png pins the camera/sphere geometry (exact disc mask);
  * 07_specular_BRDF.png pins the full path tracer statistically (block
    means of a converged image; the oracle reaches block-mean MAE 1.06 LSB at
    1024 frames, oracle_07_1024.json; the GPU test re-derives that number).
The cuRAND XORWOW stream restated here is checked against an independent
pure-Python restatement (the CUDA header is not in the container: the exact
stream is "parity unpinned" against real cuRAND)."""
import json
import os

import numpy as np
import pytest

from bwrt import scenes

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
M32 = 0xFFFFFFFF


def py_xorwow(seed, n):
    s0 = (seed & M32) ^ 0xAAD26B49
    s1 = ((seed >> 32) & M32) ^ 0xF7DCEFDD
    t0, t1 = (1099087573 * s0) & M32, (2591861531 * s1) & M32
    d = (6615241 + t1 + t0) & M32
    v = [(123456789 + t0) & M32, 362436069 ^ t0, (521288629 + t1) & M32, 88675123 ^ t1, (5783321 + t0) & M32]
    out = []
    for _ in range(n):
        t = v[0] ^ (v[0] >> 2)
        v = v[1:] + [(v[4] ^ ((v[4] << 4) & M32)) ^ (t ^ ((t << 1) & M32))]
        d = (d + 362437) & M32
        out.append((v[4] + d) & M32)
    return out


def test_rng_known_answers(oracle):
    kat = json.load(open(os.path.join(GOLDEN, "rng_kat.json")))
    for seed, vals in kat.items():
        assert oracle.curand_stream(int(seed), 16).tolist() == vals
        assert py_xorwow(int(seed), 16) == vals


def test_config1_01_scene_exact(oracle):
    """Config 1 (01 scene, 256x256, 1 spp, 1 bounce): exactly two colours:
    black and tonemap(1,0,0) = (209,0,0), the same in every frame."""
    st = oracle.render_image(scenes.scene_01(), 256, 256, 1, 1)
    cols, counts = np.unique(st.rgba.reshape(-1, 4), axis=0, return_counts=True)
    assert cols.tolist() == [[0, 0, 0, 255], [209, 0, 0, 255]]
    assert counts.tolist() == [59099, 6437]
    oracle.render(scenes.scene_01(), st, 3, 1)   # later frames: same image
    assert np.unique(st.rgba.reshape(-1, 4), axis=0).tolist() == cols.tolist()


def test_01_geometry_matches_reference_png(oracle):
    """Renders/01_red_circle.png (1279x718 crop of the 1280x720 window): the
    disc the oracle renders at 1280x720 covers exactly the PNG's rows, its
    left/right edges agree to < 1 px on average (the PNG was scaled by the
    window system: a few edge pixels are blended), and the areas agree to
    within 0.5 %."""
    g = np.load(os.path.join(GOLDEN, "01_png_disc.npz"))
    st = oracle.render_image(scenes.scene_01(), 1280, 720, 1, 1)
    m = (st.rgba[::-1, :, 0] > 100)[:int(g["png_h"]), :int(g["png_w"])]  # top row first, like the PNG
    first = np.where(m.any(1), m.argmax(1), -1)
    last = np.where(m.any(1), m.shape[1] - 1 - m[:, ::-1].argmax(1), -1)
    rows = g["first"] >= 0
    assert np.array_equal(first >= 0, rows)
    err = np.concatenate([np.abs(first - g["first"])[rows], np.abs(last - g["last"])[rows]])
    assert err.mean() < 1.0, err.mean()
    area_png = int((g["last"] - g["first"] + 1)[rows].sum())
    area = int((last - first + 1)[rows].sum())
    assert abs(area - area_png) <= 0.005 * area_png, (area, area_png)


def test_07_converged_oracle_record():
    """The recorded 1024-frame convergence of the oracle to the real-CUDA 07
    render (tests/golden/make_golden.py --converge): block-mean MAE <= 1.5."""
    rec = json.load(open(os.path.join(GOLDEN, "oracle_07_1024.json")))
    assert rec["frames"] == 1024 and rec["max_bounces"] == 5
    assert rec["block_mean_mae_lsb"] <= 1.5


def test_07_early_convergence_trend(oracle):
    """A cheap live check of the same pinning: 32 frames of the 07 scene at
    1920x1080 already sit within the measured convergence curve
    (MAE ~19 at 32 frames, 6.8 at 128, 1.06 at 1024)."""
    g = np.load(os.path.join(GOLDEN, "07_png_blocks16.npz"))
    st = oracle.render_image(scenes.scene_07(), 1920, 1080, 32, 5)
    top = st.rgba[::-1, :, :3]
    dx, dy, ph, pw, b = (int(g[k]) for k in ("dx", "dy", "png_h", "png_w", "block"))
    crop = top[dy:dy + ph, dx:dx + pw]
    hh, ww = ph // b * b, pw // b * b
    blocks = crop[:hh, :ww].astype(np.float64).reshape(hh // b, b, ww // b, b, 3).mean((1, 3))
    mae = np.abs(blocks - g["blocks"]).mean()
    assert mae < 25, mae
    # and the same blocks are far from a wrong scene (empty -> black)
    assert np.abs(g["blocks"]).mean() > 40


def test_progressive_accumulation_semantics(oracle):
    """accumulatedFrames (Main.cu:301-305): 3+5 frames == 8 frames; frame 1
    resets frameSum while the RNG continues."""
    s = scenes.scene_07()
    a = oracle.OracleState(64, 36)
    oracle.render(s, a, 3, 4, first_frame=1)
    oracle.render(s, a, 5, 4)
    b = oracle.render_image(s, 64, 36, 8, 4)
    assert np.array_equal(a.rgba, b.rgba) and np.array_equal(a.rng, b.rng)
    assert np.array_equal(a.accum, b.accum, equal_nan=True)


def test_shards_equal_full_image(oracle):
    s = scenes.scene_07()
    full = oracle.render_image(s, 80, 45, 2, 4).rgba
    for r in range(3):
        part = oracle.render_image(s, 80, 45, 2, 4, row_offset=r, row_stride=3).rgba
        assert np.array_equal(part, full[r::3])


@pytest.mark.parametrize("key", ["04", "04_box", "empty"])
def test_other_scenes_render(oracle, key):
    st = oracle.render_image(scenes.SCENES[key](), 64, 36, 2, 3)
    assert (st.rgba[..., 3] == 255).all()
    if key == "empty":
        assert (st.rgba[..., :3] == 0).all()
    else:
        assert st.rgba[..., :3].max() > 0


def test_work_profile_counters(oracle):
    """~1.95 closest-hit queries per path on the 07 scene, maxB 4."""
    oracle.render_image(scenes.scene_07(), 480, 270, 2, 4)
    q, p = oracle.last_counters()
    assert p == 480 * 270 * 2
    assert 1.8 < q / p < 2.1


@pytest.mark.parametrize("cfg", ["c2", "c3"])
def test_bench_query_counts(oracle, cfg):
    """bench.py's actual-segment counts (closest-hit queries per full frame,
    counted on the GPU by the diagnostic build) equal the oracle's own count
    of the same frame: the paths are deterministic and bit-exact."""
    import bench
    key, W, H, SPP, MB, _ = scenes.CONFIGS[cfg]
    oracle.render_image(scenes.SCENES[key](), W, H, SPP, MB)
    q, p = oracle.last_counters()
    assert p == W * H * SPP
    assert q == bench.QUERIES_PER_FRAME[cfg]


def _pin_verdicts(rec):
    """Which mutants the reference-held evidence rejects (tests/golden/
    make_pin_sensitivity.py): the 07 block-mean check (MAE > 1.5), the 01 disc
    check, or the sharper reading of the same PNG (in the >= 100 block
    channels where mutant and oracle differ by > 2 LSB, the mutant is >= 0.5
    LSB farther from the PNG)."""
    out = {}
    for k, v in rec["mutants"].items():
        sharp = v.get("png_where_it_differs") or {}
        out[k] = {"png_mae": not v["png_check_passes"], "disc": not v["disc"]["passes"],
                  "png_sharp": sharp.get("block_channels", 0) >= 100 and
                  sharp["mutant_mae"] - sharp["oracle_mae"] >= 0.5}
    return out


def test_pin_sensitivity_record():
    """How much the reference's PNGs can pin (SURVEY Appendix A quirks as
    oracle mutants, 1024 frames): the unmutated oracle reproduces its recorded
    convergence; the half-pixel and integer-jitter quirks are rejected by the
    01 disc, unit polygon normals by the sharper reading of the 07 PNG;
    every other mutant passes every check, and DESIGN.md names each of those
    as pinned by restatement only."""
    rec = json.load(open(os.path.join(GOLDEN, "pin_sensitivity.json")))
    assert rec["frames"] == 1024 and rec["max_bounces"] == 5
    m = rec["mutants"]
    assert set(m) == {str(k) for k in range(11)}
    base = json.load(open(os.path.join(GOLDEN, "oracle_07_1024.json")))["block_mean_mae_lsb"]
    assert abs(m["0"]["mae_vs_png"] - base) < 1e-3 and m["0"]["disc"]["passes"]
    assert m["0"]["pixels_differing_vs_oracle"] == 0
    v = _pin_verdicts(rec)
    rejected = {k for k, r in v.items() if any(r.values())}
    assert rejected == {"1", "2", "3"}, rejected
    assert not any(r["png_mae"] for r in v.values())  # the block-mean check alone rejects none
    design = open(os.path.join(os.path.dirname(GOLDEN), "..", "DESIGN.md")).read()
    section = design[design.index("Pinned by restatement only"):]
    section = section[:section.index("\n\n")]
    for k, r in m.items():
        if k != "0" and k not in rejected:
            assert r["name"] in section, r["name"]
