"""Generate the committed golden fixtures under tests/golden/.

Runs ONLY in the build container (it reads /root/reference, which does not
exist on the GPU box).  Outputs are data (inputs/expected outputs), never
reference source:

  07_png_blocks16.npz   16x16 block means of Renders/07_specular_BRDF.png
                        (the only real-CUDA output of the current kernel),
                        in render coordinates: PNG pixel (px, py) = render
                        pixel (px + DX, py + DY) (top-left origin).
  01_png_disc.npz       per-row [first, last] red pixel of the disc in
                        Renders/01_red_circle.png (1279x718 crop of 1280x720).
  rng_kat.json          first 16 curand() outputs for seeds 0, 1, 1919,
                        2073599 (restated cuRAND XORWOW; self-consistency).
  oracle_07_1024.json   block-mean MAE of the oracle vs the 07 PNG after
                        1024 frames at 1920x1080, maxBounces 5 (Main.cu:26),
                        if --converge is given (≈3 CPU-minutes on 8 threads).

Usage: python tests/golden/make_golden.py [--converge]
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, "bwidman-raytracer_amd"), os.path.join(REPO, "oracle")]

RENDERS = "/root/reference/Renders"
BLOCK = 16
DX, DY = 2, 1   # measured alignment of the 07 PNG (best block-mean MAE over 0..3 x 0..3)


def load_png(name):
    from PIL import Image
    return np.asarray(Image.open(os.path.join(RENDERS, name)).convert("RGB"))


def blocks(img, block=BLOCK):
    h, w = img.shape[0] // block * block, img.shape[1] // block * block
    return img[:h, :w].astype(np.float64).reshape(h // block, block, w // block, block, 3).mean((1, 3))


def png07_blocks():
    png = load_png("07_specular_BRDF.png")
    return png.shape, blocks(png)


def render_blocks(rgba_bottom_up, dx=DX, dy=DY, png_shape=(1077, 1917)):
    """Block means of a 1920x1080 render (row 0 = bottom) on the PNG's grid."""
    top = rgba_bottom_up[::-1, :, :3]
    crop = top[dy:dy + png_shape[0], dx:dx + png_shape[1]]
    return blocks(crop)


def main():
    shape, b = png07_blocks()
    np.savez_compressed(os.path.join(HERE, "07_png_blocks16.npz"), blocks=b.astype(np.float32),
                        dx=DX, dy=DY, png_h=shape[0], png_w=shape[1], block=BLOCK)
    png = load_png("01_red_circle.png")
    red = png[..., 0] >= 100
    first = np.where(red.any(1), red.argmax(1), -1)
    last = np.where(red.any(1), red.shape[1] - 1 - red[:, ::-1].argmax(1), -1)
    np.savez_compressed(os.path.join(HERE, "01_png_disc.npz"), first=first.astype(np.int16),
                        last=last.astype(np.int16), png_h=png.shape[0], png_w=png.shape[1])
    import oracle as O
    kat = {str(s): [int(v) for v in O.curand_stream(s, 16)] for s in (0, 1, 1919, 2073599)}
    with open(os.path.join(HERE, "rng_kat.json"), "w") as f:
        json.dump(kat, f, indent=1)
    if "--converge" in sys.argv:
        from bwrt import scenes
        st = O.OracleState(1920, 1080)
        for _ in range(8):
            O.render(scenes.scene_07(), st, 128, 5)
        mae = float(np.abs(render_blocks(st.rgba) - b).mean())
        with open(os.path.join(HERE, "oracle_07_1024.json"), "w") as f:
            json.dump({"frames": 1024, "max_bounces": 5, "width": 1920, "height": 1080,
                       "dx": DX, "dy": DY, "block": BLOCK, "block_mean_mae_lsb": mae}, f, indent=1)
        print("oracle 1024-frame block MAE vs 07 PNG:", mae)
    print("fixtures written to", HERE)


if __name__ == "__main__":
    main()
