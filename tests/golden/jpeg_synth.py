"""Minimal baseline JPEG writer for decoder fixtures (test infrastructure only).

PIL only writes 1x1 / 2x1 / 2x2 chroma sampling; stb_image also decodes 1x2 (its vertical
triangle filter) and every other integer ratio (nearest replication), 4-component CMYK / YCCK
(Adobe APP14 transform 0 / 2) and 'R','G','B' component ids.  This writer emits such files
directly from random quantised DCT coefficients (no forward DCT needed: the decoders under test
see an ordinary bitstream), Huffman-coded with the example tables of ITU T.81 Annex K.3.
"""
from __future__ import annotations

import struct

import numpy as np

# T.81 Table K.3 / K.5 (luminance DC / AC) code-length counts and symbol values
DC_BITS = [0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0]
DC_VALS = list(range(12))
AC_BITS = [0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7D]
AC_VALS = [
    0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51, 0x61, 0x07,
    0x22, 0x71, 0x14, 0x32, 0x81, 0x91, 0xA1, 0x08, 0x23, 0x42, 0xB1, 0xC1, 0x15, 0x52, 0xD1, 0xF0,
    0x24, 0x33, 0x62, 0x72, 0x82, 0x09, 0x0A, 0x16, 0x17, 0x18, 0x19, 0x1A, 0x25, 0x26, 0x27, 0x28,
    0x29, 0x2A, 0x34, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3A, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49,
    0x4A, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5A, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69,
    0x6A, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7A, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88, 0x89,
    0x8A, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9A, 0xA2, 0xA3, 0xA4, 0xA5, 0xA6, 0xA7,
    0xA8, 0xA9, 0xAA, 0xB2, 0xB3, 0xB4, 0xB5, 0xB6, 0xB7, 0xB8, 0xB9, 0xBA, 0xC2, 0xC3, 0xC4, 0xC5,
    0xC6, 0xC7, 0xC8, 0xC9, 0xCA, 0xD2, 0xD3, 0xD4, 0xD5, 0xD6, 0xD7, 0xD8, 0xD9, 0xDA, 0xE1, 0xE2,
    0xE3, 0xE4, 0xE5, 0xE6, 0xE7, 0xE8, 0xE9, 0xEA, 0xF1, 0xF2, 0xF3, 0xF4, 0xF5, 0xF6, 0xF7, 0xF8,
    0xF9, 0xFA]
ZIGZAG = [0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6, 7, 14,
          21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53,
          60, 61, 54, 47, 55, 62, 63]


def _codes(bits, vals):
    table, code, k = {}, 0, 0
    for length in range(1, 17):
        for _ in range(bits[length - 1]):
            table[vals[k]] = (code, length)
            code += 1
            k += 1
        code <<= 1
    return table


class _Bits:
    def __init__(self):
        self.out = bytearray()
        self.acc = 0
        self.n = 0

    def put(self, code, length):
        for i in range(length - 1, -1, -1):
            self.acc = (self.acc << 1) | ((code >> i) & 1)
            self.n += 1
            if self.n == 8:
                self.out.append(self.acc)
                if self.acc == 0xFF:
                    self.out.append(0)   # byte stuffing
                self.acc = self.n = 0

    def flush(self):
        while self.n:
            self.put(1, 1)   # pad with ones
        return bytes(self.out)


def _magnitude(v):
    return 0 if v == 0 else int(abs(v)).bit_length()


def _seg(marker, body):
    return struct.pack(">BBH", 0xFF, marker, len(body) + 2) + body


def encode(width, height, sampling, seed=0, adobe=None, jfif=True, ids=None, quant=None, restart=0):
    """A baseline JPEG of random coefficients.  sampling: [(h, v)] per component (1, 3 or 4);
    adobe: None or the APP14 colour transform (0 / 1 / 2); ids: component ids (default 1..n);
    restart: the restart interval in MCUs (DRI), 0 = none."""
    rng = np.random.default_rng(seed)
    n = len(sampling)
    ids = ids or list(range(1, n + 1))
    dc_t, ac_t = _codes(DC_BITS, DC_VALS), _codes(AC_BITS, AC_VALS)
    hmax, vmax = max(h for h, _ in sampling), max(v for _, v in sampling)
    mcux, mcuy = -(-width // (8 * hmax)), -(-height // (8 * vmax))
    q = np.asarray(quant if quant is not None else rng.integers(1, 12, 64), np.int64)
    out = b"\xff\xd8"
    if jfif:
        out += _seg(0xE0, b"JFIF\x00\x01\x01\x00\x00\x01\x00\x01\x00\x00")
    if adobe is not None:
        out += _seg(0xEE, b"Adobe\x00" + struct.pack(">BHHB", 100, 0, 0, adobe))
    out += _seg(0xDB, bytes([0]) + bytes(int(q[ZIGZAG[i]]) for i in range(64)))
    sof = struct.pack(">BHHB", 8, height, width, n) + b"".join(bytes([ids[c], (h << 4) | v, 0]) for c, (h, v) in enumerate(sampling))
    out += _seg(0xC0, sof)
    out += _seg(0xC4, bytes([0x00]) + bytes(DC_BITS) + bytes(DC_VALS))
    out += _seg(0xC4, bytes([0x10]) + bytes(AC_BITS) + bytes(AC_VALS))
    if restart:
        out += _seg(0xDD, struct.pack(">H", restart))
    out += _seg(0xDA, bytes([n]) + b"".join(bytes([ids[c], 0x00]) for c in range(n)) + b"\x00\x3f\x00")
    bits = _Bits()
    pred = [0] * n
    data = bytearray()
    for m in range(mcux * mcuy):
        if restart and m and m % restart == 0:
            data += bits.flush() + bytes([0xFF, 0xD0 + (m // restart - 1) % 8])
            bits = _Bits()
            pred = [0] * n
        for c, (h, v) in enumerate(sampling):
            for _ in range(h * v):
                # a smooth-ish block: DC around mid grey, a few low-frequency ACs
                dc = int(rng.integers(-60, 61)) // int(q[0]) + int(rng.integers(-3, 4))
                diff = dc - pred[c]
                pred[c] = dc
                s = _magnitude(diff)
                bits.put(*dc_t[s])
                if s:
                    bits.put(diff if diff > 0 else diff + (1 << s) - 1, s)
                coefs = np.zeros(64, np.int64)
                for k in rng.choice(np.arange(1, 20), size=int(rng.integers(0, 6)), replace=False):
                    coefs[k] = int(rng.integers(-40, 41)) // max(1, int(q[ZIGZAG[k]]) // 2)
                run = 0
                last = max([k for k in range(1, 64) if coefs[k]] or [0])
                for k in range(1, last + 1):
                    a = int(coefs[k])
                    if a == 0:
                        run += 1
                        continue
                    while run > 15:
                        bits.put(*ac_t[0xF0])
                        run -= 16
                    s = _magnitude(a)
                    bits.put(*ac_t[(run << 4) | s])
                    bits.put(a if a > 0 else a + (1 << s) - 1, s)
                    run = 0
                if last < 63:
                    bits.put(*ac_t[0x00])   # EOB
    data += bits.flush()
    return out + bytes(data) + b"\xff\xd9"
