"""The product's scalar C++ CPU fallback (rt_create_cpu / rt_render_cpu,
bwidman-raytracer_amd/csrc/rt_cpu.cpp over the per-ray functions of
csrc/rt_path.h that the HIP kernels use) against the oracle — CPU only.

Bar: bit-exact (RGBA8, frameSum accumulators, RNG states), as for the GPU.
BASELINE config 1 runs here in full (the reference's "scalar C++ CPU path"
case); configs 2 and 3 on row crops, the quad scene, five seeded random
scenes (odd seeds through the BVH), and config 5's geometry (the 10k-triangle
stress scene through the CPU's scalar BVH walk).
"""
import ctypes as C

import numpy as np
import pytest

from bwrt import abi, scenes
from scenegen import _random_scene, _scaled


@pytest.fixture(scope="module")
def cpu(bwrt_lib):
    from bwrt import Renderer
    r = Renderer.cpu(0, lib=bwrt_lib)
    yield r
    r.close()


def same_state(r, st):
    rng, acc = r.get_state(st.rows, st.width)
    assert np.array_equal(rng, st.rng), "RNG state differs"
    assert np.array_equal(acc, st.accum, equal_nan=True), "accum differs"


def run_pair(r, oracle, scene, w, h, spp, mb, row_offset=0, row_stride=1):
    r.set_scene(scene)
    r.init_rand(w, h, row_offset, row_stride)
    img = r.render(w, h, spp, mb, first_frame=1, row_offset=row_offset, row_stride=row_stride)
    st = oracle.OracleState(w, h, row_offset, row_stride)
    oracle.render(scene, st, spp, mb, first_frame=1)
    return img, st


def test_config1_01_full(cpu, oracle):
    """BASELINE config 1 exactly: 01 scene, 256x256, 1 spp, 1 bounce."""
    img, st = run_pair(cpu, oracle, scenes.scene_01(), 256, 256, 1, 1)
    assert np.array_equal(img, st.rgba)
    cols, counts = np.unique(img.reshape(-1, 4), axis=0, return_counts=True)
    assert cols.tolist() == [[0, 0, 0, 255], [209, 0, 0, 255]]
    assert counts.tolist() == [59099, 6437]
    same_state(cpu, st)


@pytest.mark.parametrize("name,w,h,spp,mb,off,stride", [
    ("04", 1280, 720, 4, 3, 7, 16),    # config 2, 45 rows
    ("07", 1920, 1080, 8, 4, 5, 27),   # config 3, 40 rows
    ("07", 3840, 2160, 2, 6, 11, 240),  # config 4 geometry (jitter 0.003), 9 rows
])
def test_configs_row_crops(cpu, oracle, name, w, h, spp, mb, off, stride):
    img, st = run_pair(cpu, oracle, scenes.SCENES[name](), w, h, spp, mb, off, stride)
    assert np.array_equal(img, st.rgba)
    same_state(cpu, st)


def test_quads_04_box(cpu, oracle):
    img, st = run_pair(cpu, oracle, scenes.scene_04_box(), 320, 180, 4, 5)
    assert np.array_equal(img, st.rgba)
    same_state(cpu, st)


@pytest.mark.parametrize("seed", range(5))
def test_random_scenes(cpu, oracle, monkeypatch, seed):
    """Odd seeds through the BVH (BWRT_BVH_MIN=1, read at rt_set_scene)."""
    if seed % 2:
        monkeypatch.setenv("BWRT_BVH_MIN", "1")
    s = _random_scene(seed)
    if seed == 2:
        s = _scaled(s, 1e3)
    img, st = run_pair(cpu, oracle, s, 80, 45, 3, [0, 1, 2, 4, 6][seed])
    assert np.array_equal(img, st.rgba)
    same_state(cpu, st)


def test_stress_c5_rows_bvh(cpu, oracle):
    """Config-5 geometry: two full-width rows of the stress scene (10,256
    primitives: the CPU's scalar walk of the BVH), 2 spp, 8 bounces; the
    oracle is the reference's brute-force loop."""
    img, st = run_pair(cpu, oracle, scenes.stress_scene(), 1920, 1080, 2, 8, row_offset=400, row_stride=540)
    assert np.array_equal(img, st.rgba)
    same_state(cpu, st)


def test_stress_scaled_overflow(cpu, oracle):
    """The stress scene x1e3: secondary rays overflow the reference's tests,
    so they must take the brute-force loop (bvh_safe) on the CPU too."""
    img, st = run_pair(cpu, oracle, _scaled(scenes.stress_scene(), 1e3), 48, 27, 2, 6)
    assert np.array_equal(img, st.rgba)
    same_state(cpu, st)


@pytest.mark.parametrize("mb", [0, 12, 32])
def test_bounce_limits_and_ragged(cpu, oracle, mb):
    img, st = run_pair(cpu, oracle, scenes.scene_07(), 63, 65, 2, mb)
    assert np.array_equal(img, st.rgba)
    same_state(cpu, st)


def test_progressive_continuation_and_checkpoint(cpu, oracle):
    """3 then 5 frames == 8 at once; reset restarts accumulation, not the RNG;
    a checkpoint restore rolls the state back."""
    s = scenes.scene_07()
    w, h = 128, 72
    cpu.set_scene(s)
    cpu.init_rand(w, h)
    cpu.render(w, h, 3, 4, first_frame=1)
    rng, acc = cpu.get_state(h, w)
    assert cpu.frame_counter == 4
    img = cpu.render(w, h, 5, 4)
    assert cpu.frame_counter == 9
    st = oracle.OracleState(w, h)
    oracle.render(s, st, 8, 4, first_frame=1)
    assert np.array_equal(img, st.rgba)
    same_state(cpu, st)
    cpu.set_state(rng, acc, 4)
    assert np.array_equal(cpu.render(w, h, 5, 4), st.rgba)
    cpu.reset_accumulation()
    img2 = cpu.render(w, h, 2, 4)
    oracle.render(s, st, 2, 4, first_frame=1)
    assert np.array_equal(img2, st.rgba)
    same_state(cpu, st)


def test_thread_count_invariance(bwrt_lib, oracle):
    """1, 3 and all threads give the same bits (pixels are independent)."""
    from bwrt import Renderer
    s = scenes.scene_07()
    st = oracle.render_image(s, 160, 90, 3, 4)
    with Renderer.cpu(1, lib=bwrt_lib) as r:
        assert r.threads == 1 and r.is_cpu
        r.set_scene(s)
        for t in (1, 3, 0):
            r.init_rand(160, 90)
            img = r.render_cpu(160, 90, 3, 4, first_frame=1, threads=t)
            assert np.array_equal(img, st.rgba), t
            assert r.last_kernel_ms() > 0


def test_controls_and_background(cpu, oracle):
    s = scenes.scene_07()
    cpu.set_scene(s)
    cpu.init_rand(96, 54)
    cpu.render(96, 54, 2, 4, first_frame=1)
    assert cpu.controls(["W", "LEFT"], 0.05) == 1 and cpu.frame_counter == 1
    cam = cpu.get_camera()
    cpu.set_background(0.25, 0.5, 1.0)
    try:
        img = cpu.render(96, 54, 2, 4)
    finally:
        cpu.set_background(0.0, 0.0, 0.0)
    st = oracle.OracleState(96, 54)
    oracle.render(scenes.scene_07(), st, 2, 4, first_frame=1)
    s.set_camera(cam)
    oracle.render(s, st, 2, 4, first_frame=1, background=(0.25, 0.5, 1.0))
    assert np.array_equal(img, st.rgba)


def test_drop_in_render_entry_point(cpu, oracle):
    s = scenes.scene_07()
    cpu.set_scene(s)
    cpu.set_max_bounces(5)
    cpu.init_rand(96, 54)
    img = cpu.render_simple(96, 54, 2)
    st = oracle.render_image(s, 96, 54, 2, 5)
    assert np.array_equal(img, st.rgba)


def test_explicit_backend_only(bwrt_lib, cpu):
    """The CPU path is never implicit: rt_create without a device still fails
    (RT_ERR_NO_DEVICE), rt_render_cpu refuses a non-CPU context, and the
    device-memory entry points refuse a CPU context."""
    if bwrt_lib.rt_device_count() == 0:
        ctx = C.c_void_p()
        assert bwrt_lib.rt_create(0, C.byref(ctx)) == abi.RT_ERR_NO_DEVICE
    assert bwrt_lib.rt_render_cpu(None, None, 0, None, None) == abi.RT_ERR_INVALID_ARGUMENT
    p = abi.RenderParams(16, 16, 1, 1, 1, 0, 1)
    cpu.set_scene(scenes.scene_01())
    assert bwrt_lib.rt_render_device(cpu.ctx, C.byref(p), None, None) == abi.RT_ERR_UNSUPPORTED
    assert bwrt_lib.rt_deinterleave_rows_device(cpu.ctx, C.c_void_p(8), C.c_void_p(8), 4, 4, 1, 4,
                                                None) == abi.RT_ERR_UNSUPPORTED
    arr = (C.c_void_p * 1)(cpu.ctx.value)
    assert bwrt_lib.rt_render_multi(arr, 1, 16, 16, 1, None) == abi.RT_ERR_UNSUPPORTED
    assert bwrt_lib.rt_synchronize(cpu.ctx) == 0
    assert bwrt_lib.rt_cpu_threads() >= 1
    assert bwrt_lib.rt_context_threads(cpu.ctx) == bwrt_lib.rt_cpu_threads()


@pytest.mark.parametrize("name", ["rows8", "rows15"])
def test_config5_32spp_digests(cpu, name):
    """Config 5 at its own frame count (stress scene, 32 spp, 8 bounces) on
    the rows of tests/golden/c5_rows_32spp.json: the CPU fallback reproduces
    the oracle's RGBA / frameSum / RNG digests (the oracle itself needs
    minutes for these rows: tests/golden/make_c5_golden.py)."""
    import hashlib
    import json
    import os
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "c5_rows_32spp.json")))
    smp = g["samples"][name]
    W, H = g["width"], g["height"]
    cpu.set_scene(scenes.stress_scene())
    cpu.init_rand(W, H, smp["row_offset"], smp["row_stride"])
    img, acc = cpu.render(W, H, g["spp"], g["max_bounces"], first_frame=1, row_offset=smp["row_offset"],
                          row_stride=smp["row_stride"], want_accum=True)
    rng, _ = cpu.get_state(smp["rows"], W)
    for key, arr in (("rgba", img), ("accum", acc), ("rng", rng)):
        assert hashlib.sha256(arr.tobytes()).hexdigest() == smp[key], key


@pytest.mark.parametrize("spp,mb", [(3, 4), (2, 0)])
def test_samples_per_pixel_in_frame_loop(cpu, oracle, spp, mb):
    """samplesPerPixel > 1 (Main.cu:27, 296-299): n paths from the frame's
    one jittered camera ray, the last one kept and scaled by 1/n, every
    path's RNG draws consumed — bit-exact with the oracle, and a frame
    continuation behaves as in the reference."""
    s = scenes.scene_07()
    cpu.set_scene(s)
    cpu.set_samples_per_pixel(spp)
    try:
        cpu.init_rand(96, 54)
        cpu.render(96, 54, 2, mb, first_frame=1)
        img = cpu.render(96, 54, 1, mb)
    finally:
        cpu.set_samples_per_pixel(1)
    st = oracle.OracleState(96, 54)
    oracle.render(s, st, 2, mb, first_frame=1, samples_per_pixel=spp)
    oracle.render(s, st, 1, mb, samples_per_pixel=spp)
    assert np.array_equal(img, st.rgba)
    same_state(cpu, st)


def test_cli_config1_on_cpu_fallback(bwrt_lib, oracle, tmp_path):
    """BASELINE config 1 through the C++ host (host/bwrt_render.cpp, the
    reference's main loop) on the scalar C++ CPU path: --cpu, 01 scene,
    256x256, 1 spp, 1 bounce — the PNG equals the oracle's KAT image."""
    import os
    import subprocess
    from PIL import Image
    cli = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bwidman-raytracer_amd",
                       "bin", "bwrt_render")
    png = tmp_path / "c1.png"
    r = subprocess.run([cli, "--cpu", "2", "--scene", "01", "--width", "256", "--height", "256", "--frames", "1",
                        "--max-bounces", "1", "--out", str(png)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    # "Samples:" = accumulatedFrames * samplesPerPixel after accumulatedFrames++ (Main.cu:480, 491)
    assert "CPU fallback: 2 threads" in r.stdout and "Samples: 2" in r.stdout
    st = oracle.render_image(scenes.scene_01(), 256, 256, 1, 1)
    assert np.array_equal(np.asarray(Image.open(png).convert("RGBA"))[::-1], st.rgba)
    # samplesPerPixel 2 on the same loop: "Samples:" = (frames + 1) x spp (Main.cu:491)
    r = subprocess.run([cli, "--cpu", "--scene", "07", "--width", "64", "--height", "36", "--frames", "3",
                        "--spp", "2", "--out", str(tmp_path / "s.ppm")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "Samples: 8" in r.stdout


def _denormal_07():
    """Scene 07 with emittance and albedo scaled so the emitted radiance and
    every accumulated frameSum value are f32 denormals."""
    s = scenes.scene_07()
    for i in range(s.counts[0]):
        m = s.spheres[i].mat
        m.emittance = m.emittance * 1e-20
        m.albedo.x, m.albedo.y, m.albedo.z = m.albedo.x * 1e-19, m.albedo.y * 1e-19, m.albedo.z * 1e-19
    return s


def test_caller_ftz_daz_does_not_leak(bwrt_lib, oracle):
    """A caller that set FTZ / DAZ on its thread (torch.set_flush_denormal, a
    -ffast-math library) gets the same frame: the library pins the host float
    state for its scene compile and render threads, and restores the caller's.
    Round 3's library returned flushed frameSum values here."""
    import torch
    from bwrt import Renderer
    s = _denormal_07()
    w, h, spp, mb = 64, 36, 2, 4
    st = oracle.render_image(s, w, h, spp, mb)
    assert ((np.abs(st.accum) < 1.18e-38) & (st.accum != 0)).sum() > 100  # the case is live
    with Renderer.cpu(3, lib=bwrt_lib) as c:
        assert torch.set_flush_denormal(True)
        try:
            c.set_scene(s)
            c.init_rand(w, h)
            img = c.render(w, h, spp, mb, first_frame=1)
            still_ftz = np.array([1e-40], dtype=np.float32) * np.float32(2)
        finally:
            torch.set_flush_denormal(False)
        assert still_ftz[0] == 0.0  # the caller's FTZ / DAZ is back after the calls
        assert np.array_equal(img, st.rgba)
        same_state(c, st)


def test_tuning_knobs_need_the_gate(bwrt_lib, capfd, monkeypatch):
    """BWRT_* knobs change nothing unless BWRT_TUNING=1 (a default context
    always takes the launch policy): BWRT_BVH_STATS's BVH report on the
    stress scene appears only under the gate."""
    from bwrt import Renderer
    monkeypatch.setenv("BWRT_BVH_STATS", "1")
    for gate, expect in (("0", False), ("1", True)):
        monkeypatch.setenv("BWRT_TUNING", gate)
        with Renderer.cpu(1, lib=bwrt_lib) as c:
            c.set_scene(scenes.stress_scene())
        err = capfd.readouterr().err
        assert ("bvh:" in err) == expect, (gate, err)
