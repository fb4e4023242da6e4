"""Image writers (the reference's display path, Main.cu:317-366 / 382-399,
draws the RGBA8 surface with row 0 at the bottom; files are written top row
first).  PNG via the standard library's zlib; PPM (P6).  Twin of
host/image_io.hpp."""
from __future__ import annotations

import struct
import zlib

import numpy as np


def _chunk(kind: bytes, data: bytes) -> bytes:
    return struct.pack(">I", len(data)) + kind + data + struct.pack(">I", zlib.crc32(kind + data) & 0xFFFFFFFF)


def encode_png(rgba: np.ndarray) -> bytes:
    """rgba: (H, W, 4) uint8, row 0 = bottom of the screen."""
    a = np.ascontiguousarray(np.asarray(rgba, dtype=np.uint8)[::-1])
    h, w = a.shape[:2]
    raw = np.concatenate([np.zeros((h, 1), np.uint8), a.reshape(h, w * 4)], axis=1).tobytes()
    ihdr = struct.pack(">IIBBBBB", w, h, 8, 6, 0, 0, 0)
    return (b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", ihdr) + _chunk(b"IDAT", zlib.compress(raw, 6))
            + _chunk(b"IEND", b""))


def save_png(path: str, rgba: np.ndarray) -> None:
    with open(path, "wb") as f:
        f.write(encode_png(rgba))


def save_ppm(path: str, rgba: np.ndarray) -> None:
    a = np.asarray(rgba, dtype=np.uint8)[::-1, :, :3]
    with open(path, "wb") as f:
        f.write(b"P6\n%d %d\n255\n" % (a.shape[1], a.shape[0]))
        f.write(np.ascontiguousarray(a).tobytes())
