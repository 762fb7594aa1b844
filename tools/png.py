"""Minimal PNG writer (stdlib zlib) for eyeballing films: (3,H,W) float -> 8-bit sRGB-ish."""
import struct
import sys
import zlib

import numpy as np


def write_png(path, film, gamma=2.2):
    f = np.clip(np.asarray(film, np.float32), 0.0, 1.0) ** (1.0 / gamma)
    img = (f.transpose(1, 2, 0) * 255.0 + 0.5).astype(np.uint8)
    h, w, _ = img.shape
    raw = b"".join(b"\x00" + img[y].tobytes() for y in range(h))

    def chunk(tag, data):
        return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)

    with open(path, "wb") as fp:
        fp.write(b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0))
                 + chunk(b"IDAT", zlib.compress(raw, 6)) + chunk(b"IEND", b""))


if __name__ == "__main__":
    write_png(sys.argv[2], np.load(sys.argv[1]))
