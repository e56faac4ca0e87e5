"""Minimal PNG encode/decode (8-bit RGB/RGBA, no interlace) on zlib.

Used by tests and tools to write/read output.png; the product CLI has its own
C++ writer (csrc/host/png.cpp).  Pixel bytes are what parity compares, never
file bytes (stbi_write_png's deflate output is not reproduced).
"""
import struct
import zlib

import numpy as np


def _chunk(tag, data):
    c = struct.pack(">I", len(data)) + tag + data
    return c + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)


def encode(img: np.ndarray, level: int = 6) -> bytes:
    img = np.ascontiguousarray(img, np.uint8)
    h, w, c = img.shape
    ctype = {3: 2, 4: 6}[c]
    raw = np.zeros((h, 1 + w * c), np.uint8)
    raw[:, 1:] = img.reshape(h, w * c)
    return (b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, ctype, 0, 0, 0))
            + _chunk(b"IDAT", zlib.compress(raw.tobytes(), level)) + _chunk(b"IEND", b""))


def write(path, img):
    with open(path, "wb") as f:
        f.write(encode(img))


def _paeth(a, b, c):
    p = a + b - c
    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
    if pa <= pb and pa <= pc:
        return a
    return b if pb <= pc else c


def decode(data: bytes) -> np.ndarray:
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, hdr = 8, b"", None
    while pos < len(data):
        n = struct.unpack(">I", data[pos:pos + 4])[0]
        tag = data[pos + 4:pos + 8]
        body = data[pos + 8:pos + 8 + n]
        if tag == b"IHDR":
            hdr = struct.unpack(">IIBBBBB", body)
        elif tag == b"IDAT":
            idat += body
        pos += 12 + n
    w, h, depth, ctype = hdr[0], hdr[1], hdr[2], hdr[3]
    assert depth == 8 and hdr[6] == 0
    c = {0: 1, 2: 3, 4: 2, 6: 4}[ctype]
    raw = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(h, 1 + w * c)
    out = np.zeros((h, w * c), np.int32)
    for y in range(h):
        f, line = raw[y, 0], raw[y, 1:].astype(np.int32)
        prev = out[y - 1] if y else np.zeros(w * c, np.int32)
        if f == 0:
            out[y] = line
        elif f == 2:
            out[y] = (line + prev) & 255
        else:
            row = np.zeros(w * c, np.int32)
            for i in range(w * c):
                a = row[i - c] if i >= c else 0
                b = prev[i]
                cc = prev[i - c] if i >= c else 0
                if f == 1:
                    row[i] = (line[i] + a) & 255
                elif f == 3:
                    row[i] = (line[i] + ((a + b) >> 1)) & 255
                else:
                    row[i] = (line[i] + _paeth(a, b, cc)) & 255
            out[y] = row
    return out.reshape(h, w, c).astype(np.uint8)


def read(path):
    with open(path, "rb") as f:
        return decode(f.read())
