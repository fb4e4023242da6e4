"""§8(f) host-side rows: scene files (host/scene_file.hpp + bwrt/scenefile.py)
and image output with the row flip (host/image_io.hpp + bwrt/image.py).
CPU only: the C++ side runs through the CLI's no-GPU paths and a small
harness compiled here with g++."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from bwrt import image, scenefile, scenes

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(REPO, "bwidman-raytracer_amd", "bin", "bwrt_render")
HOST = os.path.join(REPO, "bwidman-raytracer_amd", "host")


def scene_bytes(s):
    out = bytes(s.camera)
    for arr, n in zip((s.spheres, s.planes, s.triangles, s.quads), s.counts):
        out += C.string_at(arr, C.sizeof(arr._type_) * n)
    return out


@pytest.mark.parametrize("key", ["07", "01", "04", "04_box", "stress", "empty"])
def test_python_scene_file_round_trip(key):
    s = scenes.SCENES[key]()
    back = scenefile.loads(scenefile.dumps(s))
    assert back.counts == s.counts
    assert scene_bytes(back) == scene_bytes(s)


@pytest.mark.parametrize("key", ["07", "04_box"])
def test_cpp_saves_what_python_reads(key, tmp_path):
    f = tmp_path / "s.txt"
    subprocess.run([CLI, "--scene", key, "--save-scene", str(f), "--frames", "0"], check=True)
    assert scene_bytes(scenefile.load(str(f))) == scene_bytes(scenes.SCENES[key]())
    assert f.read_text() == scenefile.dumps(scenes.SCENES[key]())  # same text, both writers


def test_cpp_reads_what_python_saves(tmp_path):
    s = scenes.stress_scene()
    f, b = tmp_path / "stress.txt", tmp_path / "stress.bin"
    scenefile.save(str(f), s)
    subprocess.run([CLI, "--scene-file", str(f), "--dump-scene", str(b)], check=True)
    assert b.read_bytes() == scene_bytes(s)


def test_scene_file_defaults_and_errors(tmp_path):
    s = scenefile.loads("camera 1 2 3 0.5 -0.25 1.2\nsphere 0 0 -5 1  1 0 0\n"
                        "# comment\nquad 0 0 0 1 0 0 1 1 0 0 1 0  0.5 0.5 0.5 2 0.3  # trailing\n")
    assert s.counts == (1, 0, 0, 1)
    m = s.spheres[0].mat
    assert (m.emittance, m.roughness, m.refractive_index) == (0.0, 1.0, float(np.float32(1.05)))
    q = s.quads[0].mat
    assert (q.emittance, q.roughness) == (2.0, float(np.float32(0.3)))
    assert s.camera.fov == float(np.float32(1.2))
    with pytest.raises(ValueError, match="line 1"):
        scenefile.loads("sphere 1 2\n")
    bad = tmp_path / "bad.txt"
    bad.write_text("camera 0 1 0 0 0 1.5\ntriangle 0 0 0 1 1 1\n")
    r = subprocess.run([CLI, "--scene-file", str(bad), "--dump-scene", str(tmp_path / "x")],
                       capture_output=True, text=True)
    assert r.returncode == 2 and "line 2" in r.stderr


def _rgba(h=37, w=53):
    rng = np.random.default_rng(3)
    return rng.integers(0, 256, (h, w, 4), dtype=np.uint8)


def test_python_png_flips_rows():
    from PIL import Image
    import io
    a = _rgba()
    img = np.asarray(Image.open(io.BytesIO(image.encode_png(a))).convert("RGBA"))
    assert np.array_equal(img, a[::-1])


HARNESS = r'''
#include <cstdio>
#include <vector>
#include "image_io.hpp"
int main(int argc, char** argv) {
    const int w = 300, h = 257;  // > 65535 bytes of raw data: several stored blocks
    std::vector<uint8_t> px((size_t)w * h * 4);
    for (size_t i = 0; i < px.size(); i++) px[i] = (uint8_t)((i * 2654435761u) >> 13);
    if (!bwrt::write_png(argv[1], w, h, px.data())) return 1;
    if (!bwrt::write_ppm(argv[2], w, h, px.data())) return 1;
    FILE* f = std::fopen(argv[3], "wb");
    std::fwrite(px.data(), 1, px.size(), f);
    std::fclose(f);
    return 0;
}
'''


def test_cpp_png_and_ppm_writers(tmp_path):
    from PIL import Image
    src = tmp_path / "h.cpp"
    src.write_text(HARNESS)
    exe = tmp_path / "h"
    subprocess.run(["g++", "-O1", "-std=c++17", "-I", HOST, "-o", str(exe), str(src)], check=True)
    png, ppm, raw = tmp_path / "a.png", tmp_path / "a.ppm", tmp_path / "a.raw"
    subprocess.run([str(exe), str(png), str(ppm), str(raw)], check=True)
    a = np.frombuffer(raw.read_bytes(), np.uint8).reshape(257, 300, 4)
    assert np.array_equal(np.asarray(Image.open(png).convert("RGBA")), a[::-1])
    assert np.array_equal(np.asarray(Image.open(ppm).convert("RGB")), a[::-1, :, :3])


def test_cli_usage():
    """--help prints the usage and exits 0; an unknown option exits 2 with it."""
    ok = subprocess.run([CLI, "--help"], capture_output=True, text=True, timeout=30)
    assert ok.returncode == 0 and ok.stdout.startswith("usage: bwrt_render")
    bad = subprocess.run([CLI, "--no-such-option"], capture_output=True, text=True, timeout=30)
    assert bad.returncode == 2 and "unknown option --no-such-option" in bad.stderr and "usage:" in bad.stderr
