"""GPU parity: the HIP path (libbwrt.so via the C ABI) against the oracle.

Bar: bit-exact.  Both sides evaluate the reference's float operations in the
reference's order with one IEEE-754 rounding each (no FMA contraction,
correctly rounded div/sqrt, the same transcendental sequence), and the RNG
is integer work, so RGBA8 output, frameSum accumulators and RNG states must
be identical (NaN accumulators compare equal to NaN).
"""
import json
import os

import numpy as np
import pytest

from bwrt import scenes
from scenegen import _random_scene, _scaled

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def same_state(gpu, st_oracle):
    rows, w = st_oracle.rows, st_oracle.width
    rng, acc = gpu.get_state(rows, w)
    assert np.array_equal(rng, st_oracle.rng), "RNG state differs"
    assert np.array_equal(acc, st_oracle.accum, equal_nan=True), \
        f"accum differs at {np.argwhere(~((acc == st_oracle.accum) | (np.isnan(acc) & np.isnan(st_oracle.accum))))[:5]}"


def assert_kernel(r, prefix):
    """The launch policy picked the kernel named `prefix` (rt_last_kernel_name).
    Pins the product library's policy; skipped for an A/B variant library
    (BWRT_LIB set), whose policy may differ while its results may not."""
    if not os.environ.get("BWRT_LIB"):
        assert r.last_kernel_name().startswith(prefix), r.last_kernel_name()


def run_pair(gpu, oracle, scene, w, h, spp, mb, row_offset=0, row_stride=1):
    gpu.set_scene(scene)
    gpu.init_rand(w, h, row_offset, row_stride)  # reseed: RNG streams persist across renders
    img = gpu.render(w, h, spp, mb, first_frame=1, row_offset=row_offset, row_stride=row_stride)
    st = oracle.OracleState(w, h, row_offset, row_stride)
    oracle.render(scene, st, spp, mb, first_frame=1)
    return img, st


def test_config1_01_kat(gpu, oracle):
    img, st = run_pair(gpu, oracle, scenes.scene_01(), 256, 256, 1, 1)
    assert np.array_equal(img, st.rgba)
    cols, counts = np.unique(img.reshape(-1, 4), axis=0, return_counts=True)
    assert cols.tolist() == [[0, 0, 0, 255], [209, 0, 0, 255]]
    assert counts.tolist() == [59099, 6437]
    same_state(gpu, st)


@pytest.mark.parametrize("w,h,spp,mb", [(320, 180, 4, 4), (1280, 720, 2, 5)])
def test_07_small(gpu, oracle, w, h, spp, mb):
    img, st = run_pair(gpu, oracle, scenes.scene_07(), w, h, spp, mb)
    assert np.array_equal(img, st.rgba)
    same_state(gpu, st)


def test_config3_07_full_size(gpu, oracle):
    """BASELINE config 3 exactly: 07 scene, 1920x1080, 8 spp, 4 bounces, through
    the launch policy's kernel for it (the bench's kernel)."""
    img, st = run_pair(gpu, oracle, scenes.scene_07(), 1920, 1080, 8, 4)
    assert_kernel(gpu, "rt_render_sorted_kernel<256,grec>")
    assert np.array_equal(img, st.rgba)
    same_state(gpu, st)


# the per-rank workloads of the headline metric's 2 / 4 / 8-GPU points
# (rank r of G renders rows y = r mod G), plus 6 rows apart, the pair kernel's
# boundary (345,600 pixels <= 256 CUs x RT_SPREAD_PIX 1,400), each through the
# DEFAULT launch policy and the kernel it picks for that shard (global
# records from RT_GREC_MIN_GEN = 1.4 resident generations: 1/2 has 2.26, 1/4
# 1.13)
@pytest.mark.parametrize("stride,offset,kernel", [(2, 1, "rt_render_sorted_kernel<256,grec>"),
                                                  (4, 3, "rt_render_sorted_kernel<256>"),
                                                  (6, 2, "rt_render_pair_kernel<128>"),
                                                  (8, 5, "rt_render_pair_kernel<128>")])
def test_config3_shards(gpu, oracle, stride, offset, kernel):
    """Config 3 (07, 1920x1080, 8 spp, 4 bounces) as one rank's row shard of
    a G-GPU frame: RGBA, frameSum and RNG bit-exact with the oracle on the
    same rows (the global-index seeds make shards exact, Main.cu:377)."""
    img, st = run_pair(gpu, oracle, scenes.scene_07(), 1920, 1080, 8, 4, row_offset=offset, row_stride=stride)
    assert_kernel(gpu, kernel)
    assert img.shape[0] == len(range(offset, 1080, stride))
    assert np.array_equal(img, st.rgba)
    same_state(gpu, st)


def test_config2_04(gpu, oracle):
    img, st = run_pair(gpu, oracle, scenes.scene_04(), 1280, 720, 4, 3)
    assert np.array_equal(img, st.rgba)
    same_state(gpu, st)


def test_quads_04_box(gpu, oracle):
    img, st = run_pair(gpu, oracle, scenes.scene_04_box(), 640, 360, 4, 5)
    assert np.array_equal(img, st.rgba)
    same_state(gpu, st)


def test_stress_scene_small(gpu, oracle):
    img, st = run_pair(gpu, oracle, scenes.stress_scene(), 96, 54, 2, 8)
    assert np.array_equal(img, st.rgba)
    same_state(gpu, st)


@pytest.mark.parametrize("n16,mask", [(None, None), ("0", None), (None, "7"), ("0", "7"), (None, "1")])
def test_stress_c5_rows_bvh(gpu, oracle, monkeypatch, n16, mask):
    """Config-5 geometry (1920x1080 stress scene, 8 bounces) on 8 full-width
    rows (y = 3 mod 135): 10,256 primitives take the BVH path; the oracle is
    the reference's brute-force loop, so this pins the BVH's exact
    key-ordered tie-breaking and conservative culling — with the default
    16-byte fp16 nodes and octant arrays from the scene extents, with 32-byte
    nodes (BWRT_BVH_N16=0) and with other octant masks."""
    if n16 is not None:
        monkeypatch.setenv("BWRT_BVH_N16", n16)
    if mask is not None:
        monkeypatch.setenv("BWRT_BVH_ORDER_MASK", mask)
    img, st = run_pair(gpu, oracle, scenes.stress_scene(), 1920, 1080, 2, 8, row_offset=3, row_stride=135)
    monkeypatch.delenv("BWRT_BVH_N16", raising=False)
    monkeypatch.delenv("BWRT_BVH_ORDER_MASK", raising=False)
    gpu.set_scene(scenes.scene_07())
    assert np.array_equal(img, st.rgba)
    same_state(gpu, st)


def _c5_digests(rgba, acc, rng):
    import hashlib
    return {"rgba": hashlib.sha256(np.ascontiguousarray(rgba).tobytes()).hexdigest(),
            "accum": hashlib.sha256(np.ascontiguousarray(acc).tobytes()).hexdigest(),
            "rng": hashlib.sha256(np.ascontiguousarray(rng).tobytes()).hexdigest()}


def _c5_golden(name):
    g = json.load(open(os.path.join(GOLDEN, "c5_rows_32spp.json")))
    return g, g["samples"][name]


def test_config5_rows_32spp(gpu):
    """Config 5 at its own frame count: 8 full-width rows of the stress scene
    (y = 3 mod 135), 32 spp, 8 bounces, through the default ray-refill
    kernel, whose lanes refill across frame boundaries — RGBA, frameSum and
    RNG state bit-exact with the oracle's brute-force loop (its digests,
    tests/golden/make_c5_golden.py: minutes of oracle time)."""
    g, smp = _c5_golden("rows8")
    W, H, spp, mb = g["width"], g["height"], g["spp"], g["max_bounces"]
    gpu.set_scene(scenes.stress_scene())
    gpu.init_rand(W, H, smp["row_offset"], smp["row_stride"])
    img, acc = gpu.render(W, H, spp, mb, first_frame=1, row_offset=smp["row_offset"], row_stride=smp["row_stride"],
                          want_accum=True)
    rng, _ = gpu.get_state(smp["rows"], W)
    gpu.set_scene(scenes.scene_07())
    got = _c5_digests(img, acc, rng)
    assert got == {k: smp[k] for k in got}, (got, float(img[0, :, :3].mean()), smp["rgba_first_row_mean"])


def test_config5_shard_of_8_32spp(gpu, bwrt_lib):
    """One of config 5's 8 interleaved-row shards (rows 5, 13, 21, ...: the
    8-GPU run's per-rank work, rendered under the small-shard launch policy),
    32 spp, 8 bounces: every 9th row of the GPU shard against the oracle's
    digests, and the whole shard against the product's CPU fallback (itself
    pinned to the same digests, tests/test_cpu_fallback.py)."""
    from bwrt import Renderer
    g, smp = _c5_golden("rows15")
    W, H, spp, mb = g["width"], g["height"], g["spp"], g["max_bounces"]
    s = scenes.stress_scene()
    gpu.set_scene(s)
    gpu.init_rand(W, H, 5, 8)
    img, acc = gpu.render(W, H, spp, mb, first_frame=1, row_offset=5, row_stride=8, want_accum=True)
    rng, _ = gpu.get_state(135, W)
    gpu.set_scene(scenes.scene_07())
    got = _c5_digests(img[::9], acc[::9], rng[:, ::9])
    assert got == {k: smp[k] for k in got}, got
    with Renderer.cpu(0, lib=bwrt_lib) as c:
        c.set_scene(s)
        c.init_rand(W, H, 5, 8)
        cimg, cacc = c.render(W, H, spp, mb, first_frame=1, row_offset=5, row_stride=8, want_accum=True)
        crng, _ = c.get_state(135, W)
    assert np.array_equal(cimg, img)
    assert np.array_equal(crng, rng)
    assert np.array_equal(cacc, acc, equal_nan=True)


def test_cpu_fallback_equals_gpu_config3(gpu, bwrt_lib):
    """The product's scalar C++ CPU fallback (rt_render_cpu, all host cores)
    and the HIP kernel on BASELINE config 3 in full: the same bits."""
    from bwrt import Renderer
    s = scenes.scene_07()
    gpu.set_scene(s)
    gpu.init_rand(1920, 1080)
    img, acc = gpu.render(1920, 1080, 8, 4, first_frame=1, want_accum=True)
    with Renderer.cpu(0, lib=bwrt_lib) as c:
        c.set_scene(s)
        c.init_rand(1920, 1080)
        cimg, cacc = c.render(1920, 1080, 8, 4, first_frame=1, want_accum=True)
        crng, _ = c.get_state(1080, 1920)
    rng, _ = gpu.get_state(1080, 1920)
    assert np.array_equal(cimg, img)
    assert np.array_equal(cacc, acc, equal_nan=True)
    assert np.array_equal(crng, rng)


@pytest.mark.parametrize("batch,refill", [(1, 1), (64, 64), (33, 1), (1, 64), (60, 36)])
def test_stress_bvh_refill_schedules(bwrt_lib, oracle, monkeypatch, batch, refill):
    """The refill kernel's scheduling knobs only decide WHEN a lane tests its
    parked leaves (BWRT_LEAF_BATCH: once that many of 64 lanes are ready) and
    takes its next ray (BWRT_REFILL: once that many of 64 have finished), never
    what it tests: every schedule, from one lane at a time to whole waves,
    is bit-exact with the oracle (8 bounces, the stress scene's BVH)."""
    from bwrt import Renderer
    monkeypatch.setenv("BWRT_LEAF_BATCH", str(batch))
    monkeypatch.setenv("BWRT_REFILL", str(refill))
    r = Renderer(0, lib=bwrt_lib)  # the knobs are read when the context is made
    monkeypatch.delenv("BWRT_LEAF_BATCH")
    monkeypatch.delenv("BWRT_REFILL")
    try:
        img, st = run_pair(r, oracle, scenes.stress_scene(), 96, 54, 2, 8)
        assert np.array_equal(img, st.rgba)
        same_state(r, st)
    finally:
        r.close()


@pytest.mark.parametrize("k,n16,mb", [(3e4, 0, 6), (1e-4, 1, 6), (1.0, 1, 6), (100.0, 1, 1), (1e3, 1, 6), (1e10, 0, 3)])
def test_stress_bvh_scaled(gpu, oracle, monkeypatch, capfd, k, n16, mb):
    """The stress scene scaled by 3e4 (box corners beyond the fp16 range:
    the BVH keeps 32-byte nodes) and by 1e-4 (corners down in the fp16
    subnormal range, rounded out to +-2^-14).  From scale 100 up, secondary
    directions reflected about the un-normalised triangle normals reach 1e16
    and the reference's sphere test overflows to a NaN distance, which it
    accepts: those rays must take the brute-force loop (bvh_safe).  At 1e10
    every test overflows.  Bit-exact in every case."""
    monkeypatch.setenv("BWRT_BVH_STATS", "1")
    s = _scaled(scenes.stress_scene(), k)
    img, st = run_pair(gpu, oracle, s, 96, 54, 2, mb)
    monkeypatch.delenv("BWRT_BVH_STATS")
    assert f"n16 {n16}" in capfd.readouterr().err
    gpu.set_scene(scenes.scene_07())
    assert np.array_equal(img, st.rgba)
    same_state(gpu, st)


def test_stress_brute_force_with_culling(gpu, oracle, monkeypatch):
    """The stress scene through the brute-force loop (BVH disabled): 10,000
    random triangles, many of them skinny, exercise the conservative
    cull-sphere test in front of every exact triangle test."""
    monkeypatch.setenv("BWRT_BVH_MIN", "100000000")
    img, st = run_pair(gpu, oracle, scenes.stress_scene(), 96, 54, 2, 8)
    monkeypatch.delenv("BWRT_BVH_MIN")
    gpu.set_scene(scenes.scene_07())
    assert np.array_equal(img, st.rgba)
    same_state(gpu, st)


@pytest.mark.parametrize("name,w,h,spp,mb", [("07", 320, 180, 4, 5), ("04", 320, 180, 4, 3),
                                              ("04_box", 320, 180, 4, 5), ("01", 256, 256, 1, 1)])
def test_bvh_forced_on_small_scenes(gpu, oracle, monkeypatch, name, w, h, spp, mb):
    """BWRT_BVH_MIN=1 routes even the reference scenes through the BVH: their
    shared pyramid / box edges produce exact distance ties, which the BVH must
    resolve to the same primitive as the reference's interleaved loop."""
    monkeypatch.setenv("BWRT_BVH_MIN", "1")
    scene = {"07": scenes.scene_07, "04": scenes.scene_04, "04_box": scenes.scene_04_box,
             "01": scenes.scene_01}[name]()
    img, st = run_pair(gpu, oracle, scene, w, h, spp, mb)
    monkeypatch.delenv("BWRT_BVH_MIN")
    gpu.set_scene(scenes.scene_07())  # leave the session renderer on the brute-force path
    assert np.array_equal(img, st.rgba)
    same_state(gpu, st)


@pytest.mark.parametrize("name,w,h,spp,mb,scale", [("07", 320, 180, 4, 5, 1.0), ("04_box", 320, 180, 4, 5, 1.0),
                                                    ("stress", 96, 54, 2, 8, 1.0), ("stress", 48, 27, 2, 6, 1e3),
                                                    ("stress", 96, 54, 2, 6, 1e-4)])
def test_bvh_vertex_leaf_records(bwrt_lib, oracle, monkeypatch, name, w, h, spp, mb, scale):
    """The ray-refill kernel's vertex-form leaf records: it forms each
    polygon's plane and inner normals from the vertices with the compile
    step's own float operations — bit-exact with the oracle on the pyramid's
    and the box's shared edges (exact ties; BWRT_BVH_MIN=1 routes them
    through the BVH), the stress scene, and the stress scene scaled so its
    secondary rays overflow (1e3) or its boxes sit in the fp16 subnormal
    range (1e-4)."""
    from bwrt import Renderer
    monkeypatch.setenv("BWRT_BVH_MIN", "1")
    r = Renderer(0, lib=bwrt_lib)
    try:
        scene = {"07": scenes.scene_07, "04_box": scenes.scene_04_box, "stress": scenes.stress_scene}[name]()
        if scale != 1.0:
            scene = _scaled(scene, scale)
        img, st = run_pair(r, oracle, scene, w, h, spp, mb)
        assert_kernel(r, "rt_render_bvh_refill_kernel<64")
        assert np.array_equal(img, st.rgba)
        same_state(r, st)
    finally:
        r.close()


def test_config5_rows_vertex_leaf_records(bwrt_lib):
    """Config 5's 1/8-shard golden rows (32 spp, 8 bounces) on a fresh
    context: the oracle's digests."""
    from bwrt import Renderer
    r = Renderer(0, lib=bwrt_lib)
    try:
        g, smp = _c5_golden("rows15")
        W, H, spp, mb = g["width"], g["height"], g["spp"], g["max_bounces"]
        r.set_scene(scenes.stress_scene())
        r.init_rand(W, H, 5, 8)
        img, acc = r.render(W, H, spp, mb, first_frame=1, row_offset=5, row_stride=8, want_accum=True)
        rng, _ = r.get_state(135, W)
        got = _c5_digests(img[::9], acc[::9], rng[:, ::9])
        assert got == {k: smp[k] for k in got}, got
    finally:
        r.close()


@pytest.mark.parametrize("w,h", [(100, 37), (1, 1), (63, 65)])
def test_ragged_sizes(gpu, oracle, w, h):
    img, st = run_pair(gpu, oracle, scenes.scene_07(), w, h, 3, 4)
    assert np.array_equal(img, st.rgba)
    same_state(gpu, st)


@pytest.mark.parametrize("mb", [0, 1, 12, 32])
def test_bounce_limits(gpu, oracle, mb):
    img, st = run_pair(gpu, oracle, scenes.scene_07(), 160, 90, 2, mb)
    assert np.array_equal(img, st.rgba)
    same_state(gpu, st)


def test_empty_scene(gpu, oracle):
    img, st = run_pair(gpu, oracle, scenes.empty_scene(), 128, 72, 2, 4)
    assert np.array_equal(img, st.rgba)
    assert (img[..., :3] == 0).all() and (img[..., 3] == 255).all()


def test_progressive_continuation(gpu, oracle):
    """3 frames then 5 more (continuing the frame counter) == 8 frames at once
    (Main.cu:467-480), and a reset restarts accumulation but not the RNG."""
    s = scenes.scene_07()
    gpu.set_scene(s)
    w, h = 256, 144
    gpu.init_rand(w, h)
    gpu.render(w, h, 3, 4, first_frame=1)
    assert gpu.frame_counter == 4
    img = gpu.render(w, h, 5, 4)  # first_frame=0: continue at 4
    assert gpu.frame_counter == 9
    st = oracle.OracleState(w, h)
    oracle.render(s, st, 8, 4, first_frame=1)
    assert np.array_equal(img, st.rgba)
    same_state(gpu, st)
    gpu.reset_accumulation()
    img2 = gpu.render(w, h, 2, 4)
    oracle.render(s, st, 2, 4, first_frame=1)
    assert np.array_equal(img2, st.rgba)
    same_state(gpu, st)


def test_drop_in_render_entry_point(gpu, oracle):
    """rt_render(ctx, width, height, samples): context max_bounces (default 5)."""
    s = scenes.scene_07()
    gpu.set_scene(s)
    gpu.set_max_bounces(5)
    gpu.init_rand(192, 108)
    img = gpu.render_simple(192, 108, 4)
    st = oracle.OracleState(192, 108)
    oracle.render(s, st, 4, 5, first_frame=1)
    assert np.array_equal(img, st.rgba)


@pytest.mark.parametrize("stride", [2, 3, 8])
def test_row_shards_match_full_image(gpu, oracle, stride):
    """Pixel-row shards (the multi-GPU partition) are byte-identical to the
    corresponding rows of the full image: the RNG seed is the global index."""
    s = scenes.scene_07()
    gpu.set_scene(s)
    w, h = 320, 180
    gpu.init_rand(w, h)
    full = gpu.render(w, h, 4, 4, first_frame=1)
    for r in range(stride):
        part = gpu.render(w, h, 4, 4, first_frame=1, row_offset=r, row_stride=stride)
        assert np.array_equal(part, full[r::stride])


def test_checkpoint_resume(gpu, oracle):
    s = scenes.scene_07()
    gpu.set_scene(s)
    w, h = 128, 96
    gpu.init_rand(w, h)
    gpu.render(w, h, 3, 4, first_frame=1)
    rng, acc = gpu.get_state(h, w)
    gpu.render(w, h, 2, 4)                    # advance, then roll back
    gpu.set_state(rng, acc, 4)
    img = gpu.render(w, h, 2, 4)
    st = oracle.OracleState(w, h)
    oracle.render(s, st, 5, 4, first_frame=1)
    assert np.array_equal(img, st.rgba)


def test_camera_moved(gpu, oracle):
    """A rotated/moved camera (controls(), Controls.cuh:5-75) resets accumulation."""
    from bwrt.abi import Camera, Vec3
    import ctypes as C
    s = scenes.scene_07()
    gpu.set_scene(s)
    gpu.init_rand(160, 90)
    gpu.render(160, 90, 2, 4, first_frame=1)
    cam = Camera(Vec3(0.3, 1.2, 0.5), (C.c_float * 2)(0.35, -0.2), s.camera.fov)
    gpu.set_camera(cam)
    assert gpu.frame_counter == 1
    img = gpu.render(160, 90, 2, 4)
    s.set_camera(cam)
    # oracle: the same two frames of the original view first (RNG continues)
    st2 = oracle.OracleState(160, 90)
    oracle.render(scenes.scene_07(), st2, 2, 4, first_frame=1)
    oracle.render(s, st2, 2, 4, first_frame=1)
    assert np.array_equal(img, st2.rgba)


def test_controls_drive_the_camera(gpu, oracle):
    """rt_controls (Controls.cuh:5-75): a frame with W + LEFT held moves and
    turns the context camera and restarts accumulation; the next frames
    match the oracle rendering the moved camera from accumulatedFrames = 1
    with the RNG streams continuing."""
    s = scenes.scene_07()
    gpu.set_scene(s)
    gpu.init_rand(160, 90)
    gpu.render(160, 90, 2, 4, first_frame=1)
    assert gpu.frame_counter == 3
    flags = gpu.controls(["W", "LEFT", "UP"], 0.05)
    assert flags == 1 and gpu.frame_counter == 1
    cam = gpu.get_camera()
    assert cam.angle[0] == np.float32(0.1) and cam.angle[1] == np.float32(0.1)
    assert gpu.controls([], 0.05) == 0 and gpu.frame_counter == 1
    img = gpu.render(160, 90, 3, 4)
    st = oracle.OracleState(160, 90)
    oracle.render(scenes.scene_07(), st, 2, 4, first_frame=1)
    s.set_camera(cam)
    oracle.render(s, st, 3, 4, first_frame=1)
    assert np.array_equal(img, st.rgba)
    same_state(gpu, st)


def test_background_color(gpu, oracle):
    """backgroundColor (Main.cu:27) as a runtime setting: misses and the
    depth cut-off return it; bit-exact with the oracle."""
    s = scenes.scene_07()
    gpu.set_background(0.25, 0.5, 1.0)
    try:
        gpu.set_scene(s)
        gpu.init_rand(200, 120)
        img = gpu.render(200, 120, 3, 2, first_frame=1)
    finally:
        gpu.set_background(0.0, 0.0, 0.0)
    st = oracle.OracleState(200, 120)
    oracle.render(s, st, 3, 2, first_frame=1, background=(0.25, 0.5, 1.0))
    assert np.array_equal(img, st.rgba)
    same_state(gpu, st)
    assert img[-1, 0, 2] > 100  # the sky (top row) is now blue


@pytest.mark.parametrize("spp,mb", [(3, 4), (2, 8)])
def test_samples_per_pixel_in_frame_loop(gpu, oracle, spp, mb):
    """samplesPerPixel > 1 (Main.cu:27, 296-299; the launch policy takes the
    one-path-per-lane kernel): n paths from one jittered camera ray per
    frame, the last one kept and scaled by 1/n — bit-exact with the oracle."""
    s = scenes.scene_07() if mb == 4 else scenes.stress_scene()
    gpu.set_scene(s)
    gpu.set_samples_per_pixel(spp)
    try:
        gpu.init_rand(96, 54)
        gpu.render(96, 54, 2, mb, first_frame=1)
        img = gpu.render(96, 54, 1, mb)
    finally:
        gpu.set_samples_per_pixel(1)
        gpu.set_scene(scenes.scene_07())
    st = oracle.OracleState(96, 54)
    oracle.render(s, st, 2, mb, first_frame=1, samples_per_pixel=spp)
    oracle.render(s, st, 1, mb, samples_per_pixel=spp)
    assert np.array_equal(img, st.rgba)
    same_state(gpu, st)


def test_converges_to_reference_png(gpu):
    """Real-CUDA sanity (statistical): 1024 frames of the 07 scene at
    1920x1080, maxBounces 5 (Main.cu:26) vs Renders/07_specular_BRDF.png:
    16x16 block-mean MAE <= 1.5 LSB (fixture tests/golden/07_png_blocks16.npz)."""
    g = np.load(os.path.join(GOLDEN, "07_png_blocks16.npz"))
    gpu.set_scene(scenes.scene_07())
    gpu.init_rand(1920, 1080)
    gpu.render(1920, 1080, 512, 5, first_frame=1)
    img = gpu.render(1920, 1080, 512, 5)
    top = img[::-1, :, :3]
    dx, dy, ph, pw, b = (int(g[k]) for k in ("dx", "dy", "png_h", "png_w", "block"))
    crop = top[dy:dy + ph, dx:dx + pw]
    hh, ww = ph // b * b, pw // b * b
    blocks = crop[:hh, :ww].astype(np.float64).reshape(hh // b, b, ww // b, b, 3).mean((1, 3))
    mae = np.abs(blocks - g["blocks"]).mean()
    ref = os.path.join(GOLDEN, "oracle_07_1024.json")
    if os.path.exists(ref):
        # the GPU is bit-exact with the oracle, so it reproduces the oracle's MAE
        assert abs(mae - json.load(open(ref))["block_mean_mae_lsb"]) < 1e-6
    assert mae <= 1.5, mae


def test_config4_07_4k_max_size(gpu, oracle):
    """BASELINE config 4's per-GPU work at its full size on one GPU: 07 scene,
    3840x2160 (jitter scale 0.003), 16 spp, 6 bounces — bit-exact."""
    img, st = run_pair(gpu, oracle, scenes.scene_07(), 3840, 2160, 16, 6)
    assert np.array_equal(img, st.rgba)
    same_state(gpu, st)


def test_config4_shard_of_8(gpu, oracle):
    """One of the 8 interleaved-row shards of config 4 (rows 5, 13, 21, ...)."""
    img, st = run_pair(gpu, oracle, scenes.scene_07(), 3840, 2160, 16, 6, row_offset=5, row_stride=8)
    assert np.array_equal(img, st.rgba)


@pytest.mark.parametrize("blocks", [None, 3])
def test_deinterleave_kernel(bwrt_lib, monkeypatch, blocks):
    """rt_deinterleave_rows_device (the multi-GPU gather epilogue) on device
    buffers: gathered [shards][rows_per_shard][W] -> image [H][W] — 16 bytes
    per lane when the width is a multiple of 4 and both buffers are 16-byte
    aligned, 4 otherwise (odd widths, a buffer offset by one pixel); with
    the grid capped at 3 blocks (BWRT_DEINT_BLOCKS) the loop strides over
    the rest."""
    import torch
    from bwrt import Renderer
    from bwrt.dist import ShardPlan, deinterleave_reference
    r = _fresh_renderer(bwrt_lib, monkeypatch, BWRT_DEINT_BLOCKS=blocks) if blocks else Renderer(0, lib=bwrt_lib)
    try:
        for h, w, shards, off in [(1080, 1920, 8, 0), (2160, 3840, 8, 0), (1080, 1920, 1, 0), (36, 64, 4, 0),
                                  (36, 64, 4, 1), (55, 33, 2, 0), (7, 5, 3, 0)]:
            plan = ShardPlan(h, shards, 0)
            g = torch.randint(0, 2**31 - 1, (shards * plan.rows_per_shard * w + off,), dtype=torch.int32,
                              device="cuda")[off:]
            out = torch.empty(h * w + off, dtype=torch.int32, device="cuda")[off:]
            # (torch's default stream is the null stream, whose handle 0 means
            # "the context's stream" to the C ABI: the inputs must be ready
            # before a launch on another stream)
            torch.cuda.synchronize()
            r.deinterleave_device(g.data_ptr(), out.data_ptr(), w, h, shards, plan.rows_per_shard,
                                  torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            want = deinterleave_reference(g.cpu().numpy().reshape(shards, plan.rows_per_shard, w, 1), plan, w)
            assert np.array_equal(out.cpu().numpy().reshape(h, w), want[..., 0]), (h, w, shards, off)
    finally:
        r.close()


def test_context_stream_priority(bwrt_lib, monkeypatch):
    """The context's own stream (rt_get_stream) runs at the device's highest
    priority, so a render dispatches ahead of a gather overlapping it
    (bench.py's pipelined N > 1 step); BWRT_STREAM_PRIO=0 gives a normal one."""
    import ctypes as C
    from bwrt import Renderer
    hip = C.CDLL("libamdhip64.so")  # the runtime torch and libbwrt.so share
    least, greatest = C.c_int(), C.c_int()
    assert hip.hipDeviceGetStreamPriorityRange(C.byref(least), C.byref(greatest)) == 0

    def prio(r):
        p = C.c_int()
        assert hip.hipStreamGetPriority(C.c_void_p(r.stream_handle()), C.byref(p)) == 0
        return p.value

    r = Renderer(0, lib=bwrt_lib)
    try:
        assert prio(r) == greatest.value
    finally:
        r.close()
    r = _fresh_renderer(bwrt_lib, monkeypatch, BWRT_STREAM_PRIO=0)
    try:
        assert prio(r) == 0  # the default priority (hipStreamCreateWithFlags)
    finally:
        r.close()


def test_render_device_into_torch_buffer(gpu, oracle):
    """rt_render_device into a torch-allocated device buffer on a torch stream
    (the bench / multi-GPU path) equals the host-buffer render."""
    import torch
    s = scenes.scene_07()
    gpu.set_scene(s)
    w, h = 256, 144
    gpu.init_rand(w, h)
    buf = torch.zeros(h * w, dtype=torch.int32, device="cuda")
    stream = torch.cuda.Stream()
    torch.cuda.synchronize()  # (the zero fill ran on torch's default stream, unordered with `stream`)
    gpu.render_device(gpu.params(w, h, 3, 4, first_frame=1), buf.data_ptr(), stream.cuda_stream)
    stream.synchronize()
    img = buf.cpu().numpy().view(np.uint8).reshape(h, w, 4)
    st = oracle.render_image(s, w, h, 3, 4)
    assert np.array_equal(img, st.rgba)
    assert gpu.last_kernel_ms() > 0


def test_kernel_timing_off_and_on(gpu, oracle):
    """rt_set_kernel_timing: the launch's start / end events ride on the
    kernels' dispatch packets; with timing off rt_last_kernel_ms is -1 (no
    stale value), the render and its ordering event are unchanged (a host
    render on the context's stream after a device render on a torch stream
    continues the state in order), and timing on again gives durations."""
    import torch
    s = scenes.scene_07()
    gpu.set_scene(s)
    w, h, mb = 320, 180, 4
    gpu.init_rand(w, h)
    st = oracle.OracleState(w, h)
    buf = torch.zeros(h * w, dtype=torch.int32, device="cuda")
    stream = torch.cuda.Stream()
    torch.cuda.synchronize()  # (the zero fill ran on torch's default stream, unordered with `stream`)
    try:
        gpu.render(w, h, 1, mb, first_frame=1)
        assert gpu.last_kernel_ms() > 0
        gpu.set_kernel_timing(False)
        assert gpu.last_kernel_ms() == -1.0
        gpu.render_device(gpu.params(w, h, 2, mb, first_frame=2), buf.data_ptr(), stream.cuda_stream)
        assert gpu.last_kernel_ms() == -1.0
        img = gpu.render(w, h, 2, mb, first_frame=4)  # waits for the torch-stream render
        want = oracle.render(s, st, 5, mb, first_frame=1)
        assert np.array_equal(img, want)
        gpu.set_kernel_timing(True)
        gpu.render(w, h, 1, mb, first_frame=6)
        assert gpu.last_kernel_ms() > 0
    finally:
        gpu.set_kernel_timing(True)


def test_state_writes_wait_for_device_render(gpu, oracle):
    """rt_set_scene / rt_init_rand / rt_set_state right after an asynchronous
    rt_render_device on a torch stream must not overwrite the scene or the
    shard state under the running kernel (they wait for that stream), and a
    render on the context's own stream after one on a torch stream continues
    its state in order."""
    import torch
    w, h, spp, mb = 640, 360, 8, 4
    s07, s04 = scenes.scene_07(), scenes.scene_04()
    stream = torch.cuda.Stream()
    buf = torch.zeros(h * w, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()  # (the zero fill ran on torch's default stream, unordered with `stream`)
    seeds = oracle.OracleState(w, h)
    oracle.render(s07, seeds, 0, mb, first_frame=1)  # curand_init states only
    st = oracle.OracleState(w, h)
    oracle.render(s07, st, spp, mb, first_frame=1)
    for _ in range(3):
        # scene swap queued behind the render
        gpu.set_scene(s07)
        gpu.init_rand(w, h)
        gpu.render_device(gpu.params(w, h, spp, mb, first_frame=1), buf.data_ptr(), stream.cuda_stream)
        gpu.set_scene(s04)
        stream.synchronize()
        assert np.array_equal(buf.cpu().numpy().view(np.uint8).reshape(h, w, 4), st.rgba)
        # reseed queued behind the render: the fresh seeds must survive it
        gpu.set_scene(s07)
        gpu.render_device(gpu.params(w, h, spp, mb, first_frame=1), buf.data_ptr(), stream.cuda_stream)
        gpu.init_rand(w, h)
        rng, _ = gpu.get_state(h, w)
        assert np.array_equal(rng, seeds.rng)
        # checkpoint restore queued behind the render
        gpu.render_device(gpu.params(w, h, spp, mb, first_frame=1), buf.data_ptr(), stream.cuda_stream)
        gpu.set_state(seeds.rng, np.zeros((h, w, 3), np.float32), 1)
        rng, _ = gpu.get_state(h, w)
        assert np.array_equal(rng, seeds.rng)
    # a de-interleave on a second, unordered stream between the render and the
    # state writes: the writes wait for the render itself (its event), not for
    # the last stream used, and that stream may be gone by the next write
    g = torch.zeros(h * w, dtype=torch.int32, device="cuda")
    out = torch.empty_like(g)
    torch.cuda.synchronize()
    for _ in range(2):
        gpu.set_scene(s07)
        gpu.init_rand(w, h)
        gpu.render_device(gpu.params(w, h, spp, mb, first_frame=1), buf.data_ptr(), stream.cuda_stream)
        s2 = torch.cuda.Stream()
        gpu.deinterleave_device(g.data_ptr(), out.data_ptr(), w, h, 1, h, s2.cuda_stream)
        gpu.set_scene(s04)
        stream.synchronize()
        assert np.array_equal(buf.cpu().numpy().view(np.uint8).reshape(h, w, 4), st.rgba)
        s2.synchronize()
        del s2
        gpu.set_scene(s07)
        gpu.render_device(gpu.params(w, h, spp, mb, first_frame=1), buf.data_ptr(), stream.cuda_stream)
        gpu.init_rand(w, h)
        rng, _ = gpu.get_state(h, w)
        assert np.array_equal(rng, seeds.rng)
        gpu.synchronize()
    # device render on a torch stream, then a synchronous continuation on
    # the context's stream: frames 1..4 then 5..8 equal one 8-frame render
    gpu.init_rand(w, h)
    gpu.render_device(gpu.params(w, h, 4, mb, first_frame=1), buf.data_ptr(), stream.cuda_stream)
    img = gpu.render(w, h, 4, mb)
    assert np.array_equal(img, st.rgba)
    same_state(gpu, st)


def test_context_stream_renders_defer_their_event(gpu, oracle):
    """Renders on the context's own stream (rt_get_stream, kernel timing off)
    record their end event only when a later call needs it: back-to-back
    renders on that stream, then a render on a torch stream (it must wait
    for them), a state read and a scene upload (they must wait too), then
    the context stream again — every frame continues the state in order."""
    import torch
    s = scenes.scene_07()
    w, h, mb = 320, 180, 4
    gpu.set_scene(s)
    gpu.init_rand(w, h)
    st = oracle.OracleState(w, h)
    buf = torch.zeros(h * w, dtype=torch.int32, device="cuda")
    ctx_stream = torch.cuda.ExternalStream(gpu.stream_handle())
    other = torch.cuda.Stream()
    torch.cuda.synchronize()  # (the zero fill ran on torch's default stream, unordered with these)
    gpu.set_kernel_timing(False)
    try:
        for f in (1, 3):  # frames 1-2, 3-4 on the context stream (handle, then NULL)
            gpu.render_device(gpu.params(w, h, 2, mb, first_frame=f), buf.data_ptr(),
                              ctx_stream.cuda_stream if f == 1 else None)
        gpu.render_device(gpu.params(w, h, 2, mb, first_frame=5), buf.data_ptr(), other.cuda_stream)
        other.synchronize()
        oracle.render(s, st, 6, mb, first_frame=1)
        assert np.array_equal(buf.cpu().numpy().view(np.uint8).reshape(h, w, 4), st.rgba)
        same_state(gpu, st)
        gpu.render_device(gpu.params(w, h, 2, mb, first_frame=7), buf.data_ptr(), None)
        rng, _ = gpu.get_state(h, w)  # waits for the deferred event's render
        oracle.render(s, st, 2, mb, first_frame=7)
        assert np.array_equal(rng, st.rng)
        gpu.render_device(gpu.params(w, h, 2, mb, first_frame=9), buf.data_ptr(), None)
        gpu.set_scene(scenes.scene_04())  # must not swap the scene under the running render
        ctx_stream.synchronize()
        oracle.render(s, st, 2, mb, first_frame=9)
        assert np.array_equal(buf.cpu().numpy().view(np.uint8).reshape(h, w, 4), st.rgba)
    finally:
        gpu.set_kernel_timing(True)
        gpu.set_scene(s)


def test_cli_progressive_loop_with_controls(bwrt_lib, oracle, tmp_path):
    """The C++ host loop (host/bwrt_render.cpp, Main.cu:467-496): 2 frames,
    then W+LEFT held for one frame (controls() restarts accumulation), then 4
    more frames; the PNG (top row first) equals the oracle's image of the
    moved camera from accumulatedFrames = 1 with the RNG streams continuing."""
    import ctypes as C
    import subprocess
    from PIL import Image
    from bwrt.abi import KEYS
    cli = os.path.join(os.path.dirname(GOLDEN), "..", "bwidman-raytracer_amd", "bin", "bwrt_render")
    png = tmp_path / "out.png"
    r = subprocess.run([cli, "--scene", "07", "--width", "160", "--height", "90", "--frames", "6",
                        "--keys", "*1,W+LEFT*1,*9", "--dt", "0.05", "--out", str(png)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    s = scenes.scene_07()
    cam = s.camera
    moved = type(cam).from_buffer_copy(bytes(cam))
    assert bwrt_lib.rt_apply_controls(C.byref(moved), KEYS["W"] | KEYS["LEFT"], 0.05) == 1
    st = oracle.OracleState(160, 90)
    oracle.render(s, st, 2, 5, first_frame=1)
    s2 = scenes.scene_07()
    s2.set_camera(moved)
    oracle.render(s2, st, 4, 5, first_frame=1)
    img = np.asarray(Image.open(png).convert("RGBA"))[::-1]
    assert np.array_equal(img, st.rgba)
    # 4 frames since the reset by the move: accumulatedFrames = 5 (Main.cu:480-491)
    assert "camera" in r.stdout and "Samples: 5" in r.stdout
    # the same loop across 3 contexts (rt_render_multi; one device here)
    png3 = tmp_path / "out3.png"
    r = subprocess.run([cli, "--scene", "07", "--width", "160", "--height", "90", "--frames", "6", "--gpus", "3",
                        "--keys", "*1,W+LEFT*1,*9", "--dt", "0.05", "--out", str(png3)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert np.array_equal(np.asarray(Image.open(png3).convert("RGBA"))[::-1], st.rgba)


def test_repeated_renders_are_identical(gpu, oracle):
    """Race check: the workgroup task queue must give the same bits every
    time, including right after a launch with a different LDS layout (the
    07 scene at 4 bounces vs the 04 scene at 3)."""
    cases = [(scenes.scene_04(), 640, 360, 4, 3), (scenes.scene_07(), 640, 360, 4, 4)]
    want = []
    for s, w, h, spp, mb in cases:
        st = oracle.OracleState(w, h)
        oracle.render(s, st, spp, mb, first_frame=1)
        want.append(st)
    for _ in range(6):
        for (s, w, h, spp, mb), st in zip(cases, want):
            gpu.set_scene(s)
            gpu.init_rand(w, h)
            img = gpu.render(w, h, spp, mb, first_frame=1)
            assert np.array_equal(img, st.rgba)
            same_state(gpu, st)


@pytest.mark.parametrize("n", [2, 3])
def test_render_multi_contexts(bwrt_lib, oracle, n):
    """rt_render_multi (single-process multi-GPU for C++ hosts): n contexts —
    here all on device 0, as a rehearsal of n GPUs — each render rows
    y = i (mod n) concurrently; the gathered frames equal the oracle's, for
    two successive calls (frame counters continue in step)."""
    from bwrt import Renderer, render_multi
    s = scenes.scene_07()
    rs = [Renderer(0, lib=bwrt_lib) for _ in range(n)]
    try:
        for i, r in enumerate(rs):
            r.set_scene(s)
            r.set_max_bounces(4)
            r.init_rand(320, 181, i, n)
        st = oracle.OracleState(320, 181)
        for call in range(2):
            img = render_multi(rs, 320, 181, 2)
            oracle.render(s, st, 2, 4, first_frame=1 if call == 0 else None)
            assert np.array_equal(img, st.rgba), f"call {call}"
        assert all(r.frame_counter == 5 for r in rs)
    finally:
        for r in rs:
            r.close()


@pytest.mark.parametrize("seed", list(range(40)))
def test_random_scenes(gpu, oracle, monkeypatch, seed):
    """Bit-exact on seeded random scenes, through the brute-force loop and
    (odd seeds) through the BVH; every fourth scene is scaled by 1e3 or 1e-3
    (cull-sphere and BVH margins are relative to the scene scale)."""
    if seed % 2:
        monkeypatch.setenv("BWRT_BVH_MIN", "1")
    s = _random_scene(seed)
    if seed % 4 == 2:
        s = _scaled(s, 1e3 if seed % 8 == 2 else 1e-3)
    mb = [0, 1, 2, 4, 6, 9][seed % 6]
    img, st = run_pair(gpu, oracle, s, 80, 45, 3, mb)
    monkeypatch.delenv("BWRT_BVH_MIN", raising=False)
    gpu.set_scene(scenes.scene_07())
    assert np.array_equal(img, st.rgba)
    same_state(gpu, st)


@pytest.mark.parametrize("seed,k", [(3, 1e6), (5, 1e10), (7, 1e-6), (9, 1e-10), (11, 1e15), (13, 1e19)])
@pytest.mark.parametrize("bvh", [False, True])
def test_random_scenes_extreme_scales(gpu, oracle, monkeypatch, seed, k, bvh):
    """Random scenes scaled far beyond any sensible range: overflow in the
    reference's tests turns distances into inf / NaN, which the reference
    accepts in its own way (a NaN distance is accepted, and then every later
    candidate); the brute-force loop's culling and the BVH must step aside
    for such rays (cull_dmax, bvh_safe) — bit-exact through both paths."""
    if bvh:
        monkeypatch.setenv("BWRT_BVH_MIN", "1")
    s = _scaled(_random_scene(seed), k)
    img, st = run_pair(gpu, oracle, s, 64, 36, 2, 4)
    monkeypatch.delenv("BWRT_BVH_MIN", raising=False)
    gpu.set_scene(scenes.scene_07())
    assert np.array_equal(img, st.rgba)
    same_state(gpu, st)


def _fresh_renderer(bwrt_lib, monkeypatch, **env):
    """A renderer created under BWRT_* launch knobs (read at rt_create)."""
    from bwrt import Renderer
    for k, v in env.items():
        monkeypatch.setenv(k, str(v))
    try:
        return Renderer(0, lib=bwrt_lib)
    finally:
        for k in env:
            monkeypatch.delenv(k)


@pytest.mark.parametrize("block", [64, 128, 256])
@pytest.mark.parametrize("w,h,mb", [(160, 90, 4), (100, 37, 6), (160, 90, 2), (120, 70, 3), (64, 40, 0)])
def test_global_records_forced(bwrt_lib, oracle, monkeypatch, block, w, h, mb):
    """The sorted kernel with its recursion records in global memory
    (BWRT_GREC=1; the launch policy picks it for deep paths such as config 4)
    at every workgroup size, including ragged sizes and a row shard.  Levels
    0-1 stay in LDS: at max_bounces 2 no level reaches global memory, at 3
    exactly one does (the boundaries of the split)."""
    r = _fresh_renderer(bwrt_lib, monkeypatch, BWRT_GREC=1, BWRT_BLOCK=block)
    try:
        for off, stride in ((0, 1), (1, 3)):
            img, st = run_pair(r, oracle, scenes.scene_07(), w, h, 3, mb, row_offset=off, row_stride=stride)
            assert np.array_equal(img, st.rgba)
            same_state(r, st)
            # continuation (frames 4-5 in a second launch): the deferred fold
            # of a launch's last frame happens inside that launch
            img = r.render(w, h, 2, mb, first_frame=4, row_offset=off, row_stride=stride)
            oracle.render(scenes.scene_07(), st, 2, mb, first_frame=4)
            assert np.array_equal(img, st.rgba)
            same_state(r, st)
    finally:
        r.close()


@pytest.mark.parametrize("spread", [1, 0])
def test_pair_kernel_forced_on_off(bwrt_lib, oracle, monkeypatch, spread):
    """BWRT_SPREAD=1 forces the pair kernel (128-lane groups for 64 pixels:
    an owner wave and a helper wave that runs the SPEC tasks and half of
    every closest hit); BWRT_SPREAD=0 keeps small frames, which the policy
    gives to the pair kernel, on the sorted kernel (128-lane groups).
    Ragged sizes (the last group part-owned), a one-pixel frame, row shards,
    quads, exact ties, and a scene scaled by 1e10 (rays that fail bvh_safe:
    the whole loop on the owner)."""
    r = _fresh_renderer(bwrt_lib, monkeypatch, BWRT_SPREAD=spread)
    cases = [(scenes.scene_07(), 160, 90, 3, 4, 0, 1), (scenes.scene_04_box(), 96, 61, 2, 4, 1, 3),
             (_random_scene(7), 81, 45, 2, 3, 0, 1), (scenes.scene_07(), 1, 1, 2, 4, 0, 1),
             (_scaled(_random_scene(3), 1e10), 64, 36, 2, 4, 0, 1), (scenes.scene_04_box(), 96, 61, 2, 6, 0, 1)]
    try:
        for scene, w, h, spp, mb, off, stride in cases:
            img, st = run_pair(r, oracle, scene, w, h, spp, mb, row_offset=off, row_stride=stride)
            assert np.array_equal(img, st.rgba)
            same_state(r, st)
            # (max_bounces >= 5: the policy keeps the deep record stack in
            # global memory, which only the sorted kernel has)
            want = "rt_render_pair_kernel<128>" if spread and mb <= 4 else "rt_render_sorted_kernel<128"
            assert_kernel(r, want)
    finally:
        r.close()


def test_pair_kernel_order_feedback(bwrt_lib, oracle, monkeypatch):
    """The pair kernel forced on a multi-generation grid (07 at 1080p, 64
    pixels per group) with launch-order feedback: blockIdx order, then
    reordered twice; every frame equals the oracle."""
    w, h, mb = 1920, 1080, 4
    scene = scenes.scene_07()
    st = oracle.OracleState(w, h)
    oracle.render(scene, st, 1, mb, first_frame=1)
    # (BWRT_GREC=0: a full frame would take global records, which the pair
    # kernel does not have)
    r = _fresh_renderer(bwrt_lib, monkeypatch, BWRT_SPREAD=1, BWRT_ORDER=1, BWRT_ORDER_PERIOD=2, BWRT_GREC=0)
    try:
        r.set_scene(scene)
        for _ in range(3):
            r.init_rand(w, h)
            img = r.render(w, h, 1, mb, first_frame=1)
            assert np.array_equal(img, st.rgba)
            same_state(r, st)
        assert_kernel(r, "rt_render_pair_kernel<128>+order")
    finally:
        r.close()


@pytest.mark.parametrize("name", ["07", "04_box"])
def test_simple_kernel_ab_reference(bwrt_lib, oracle, monkeypatch, name):
    """The one-path-per-lane kernel kept as the A/B reference (BWRT_KERNEL=simple)."""
    r = _fresh_renderer(bwrt_lib, monkeypatch, BWRT_KERNEL="simple")
    scene = {"07": scenes.scene_07, "04_box": scenes.scene_04_box}[name]()
    try:
        img, st = run_pair(r, oracle, scene, 200, 113, 3, 5)
        assert np.array_equal(img, st.rgba)
        same_state(r, st)
    finally:
        r.close()


def test_launch_order_feedback_bvh_refill(bwrt_lib, monkeypatch):
    """Launch-order feedback in the BVH ray-refill kernel (config 5's
    product path): the stress scene at 1920x1080, 2 spp, 8 bounces — a grid
    of 32,400 single-wave groups, several resident generations — rendered
    four times (blockIdx order, then reordered: BVH scenes re-sort their
    order after every launch, so kept orders are covered by
    test_launch_order_feedback only) and once as a continuation; every image, frameSum and RNG state
    equals the product's CPU fallback (itself pinned to the oracle,
    tests/test_cpu_fallback.py; the brute-force oracle would need minutes)."""
    from bwrt import Renderer
    s = scenes.stress_scene()
    with Renderer.cpu(0, lib=bwrt_lib) as c:
        c.set_scene(s)
        c.init_rand(1920, 1080)
        want = c.render(1920, 1080, 2, 8, first_frame=1, want_accum=True)
        want_rng, _ = c.get_state(1080, 1920)
        cont = c.render(1920, 1080, 1, 8, want_accum=True)
        cont_rng, _ = c.get_state(1080, 1920)
    r = _fresh_renderer(bwrt_lib, monkeypatch, BWRT_ORDER=1)
    try:
        r.set_scene(s)
        for _ in range(4):
            r.init_rand(1920, 1080)
            img, acc = r.render(1920, 1080, 2, 8, first_frame=1, want_accum=True)
            rng, _ = r.get_state(1080, 1920)
            assert np.array_equal(img, want[0]) and np.array_equal(acc, want[1], equal_nan=True)
            assert np.array_equal(rng, want_rng)
        img, acc = r.render(1920, 1080, 1, 8, want_accum=True)
        rng, _ = r.get_state(1080, 1920)
        assert np.array_equal(img, cont[0]) and np.array_equal(acc, cont[1], equal_nan=True)
        assert np.array_equal(rng, cont_rng)
    finally:
        r.close()


@pytest.mark.parametrize("scene_name,w,h,spp,mb,grec", [("07", 1920, 1080, 2, 4, 0), ("04", 1600, 1200, 2, 3, 0),
                                                       ("07", 1920, 1080, 2, 6, 1)])
def test_launch_order_feedback(bwrt_lib, oracle, monkeypatch, scene_name, w, h, spp, mb, grec):
    """Launch-order feedback (grids of several resident generations: each
    launch records its tile-groups' durations and the next launch starts the
    most expensive first): the first render runs in blockIdx order, the
    following ones reordered — every one equals the oracle bit for bit, and
    a progressive continuation under the new order does too.  The 07 1080p
    maxBounces-4 case is config 3's product path (the launch policy's
    global-memory records on a multi-generation frame: level 2-3 outside
    LDS, 7 resident groups per CU); the grec case is config 4's (maxBounces
    6: levels 2-5 outside LDS) reordered."""
    scene = scenes.SCENES[scene_name]()
    st = oracle.OracleState(w, h)
    oracle.render(scene, st, spp, mb, first_frame=1)
    r = _fresh_renderer(bwrt_lib, monkeypatch, BWRT_ORDER=1, BWRT_ORDER_PERIOD=2, BWRT_GREC=grec) if grec else \
        _fresh_renderer(bwrt_lib, monkeypatch, BWRT_ORDER=1, BWRT_ORDER_PERIOD=2)
    try:
        r.set_scene(scene)
        # blockIdx order first, then orders re-sorted every 2nd launch (launch 1
        # keeps launch 0's sort, launch 2 sorts again; the product re-sorts
        # every 16th, rt_context.cpp order_period)
        for _ in range(4):
            r.init_rand(w, h)
            img = r.render(w, h, spp, mb, first_frame=1)
            assert np.array_equal(img, st.rgba)
            same_state(r, st)
        oracle.render(scene, st, 1, mb)
        img = r.render(w, h, 1, mb)
        assert np.array_equal(img, st.rgba)
        same_state(r, st)
    finally:
        r.close()
