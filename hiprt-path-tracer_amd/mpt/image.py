"""Image decoding for the scene and envmap loaders, with the semantics of the decoder the
reference compiles (stb_image, thirdparties/stbi/stb_image.h):

* textures: ``Image8Bit::read_image`` (src/Image/Image.cpp:33-61) = ``stbi_load(path, &w, &h,
  &n, output_channels)`` without a vertical flip -- PNG restated here with the standard
  library's zlib and libmpt's scanline filter reversal (``mpt_png_unfilter``, csrc/image.cpp),
  JPEG by libmpt's restatement of stb_image's decoder (``mpt_jpeg_decode``, csrc/jpeg.cpp);
* envmaps and the baked LUTs: ``Image32Bit::read_image_hdr`` (Image.cpp:342-370) =
  ``stbi_loadf`` with ``flipY`` -- Radiance .hdr by ``mpt_hdr_decode`` (csrc/jpeg.cpp); an 8-bit
  file through ``stbi_loadf`` becomes ``pow(v / 255, 2.2)`` (alpha ``v / 255``).
  ``load_envmap`` is ``RendererEnvmap``'s read (RendererEnvmap.cpp:39-48: 4 channels, flipped).

Every decode is pinned byte for byte (float for float) against the reference's own stb_image.h
compiled from its sources (oracle/_ref, tests/golden/images, tests/test_image_decode.py).

What stb_image does and this module restates:
* every PNG colour type (grey, RGB, palette, grey + alpha, RGBA), bit depths 1/2/4/8/16,
  Adam7 interlacing, the tRNS chunk (an alpha channel for palette / grey / RGB images);
* 16-bit samples reduced to 8 bits by keeping the high byte (stbi__convert_16_to_8);
* sub-byte grey samples scaled to 0..255 (stbi__depth_scale_table: x1, x0x55, x0x11, x0x01);
* the conversion to the requested channel count (stbi__convert_format): grey -> RGB
  replicates, RGB -> grey is ``(77 r + 150 g + 29 b) >> 8`` (stbi__compute_y), a missing
  alpha is 255, an unwanted alpha is dropped.

Other formats (TGA, BMP, DDS, ...) raise ``ValueError``: the loader names the texture and
fails loudly rather than rendering a different scene.
"""
from __future__ import annotations

import struct
import zlib

import numpy as np

PNG_SIG = b"\x89PNG\r\n\x1a\n"
_CHANNELS = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}
# Adam7 passes: (x0, y0, dx, dy)
_ADAM7 = [(0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2), (0, 1, 1, 2)]


def _unfilter(raw: bytes, rows: int, row_bytes: int, bpp: int) -> np.ndarray:
    from . import _check, lib
    out = np.empty((rows, row_bytes), np.uint8)
    if rows == 0 or row_bytes == 0:
        return out
    src = np.frombuffer(raw, np.uint8)
    _check(lib().mpt_png_unfilter(src.ctypes.data, len(src), out.ctypes.data, rows, row_bytes, bpp))
    return out


def _samples(rows: np.ndarray, width: int, depth: int, ch: int) -> np.ndarray:
    """Unpacked samples [h, width * ch] (uint8 for depth <= 8 as stored, uint16 for 16)."""
    h = rows.shape[0]
    if depth == 8:
        return rows[:, :width * ch]
    if depth == 16:
        return rows[:, :2 * width * ch].reshape(h, width * ch, 2).astype(np.uint16) @ np.array([256, 1], np.uint16)
    bits = np.unpackbits(rows, axis=1)[:, :width * ch * depth].reshape(h, width * ch, depth)
    return (bits @ (1 << np.arange(depth - 1, -1, -1))).astype(np.uint8)


def decode_png(data: bytes) -> np.ndarray:
    """PNG bytes -> uint8 [h, w, c] in the file's own channels (c = 1, 2, 3 or 4 after palette /
    tRNS expansion), 16-bit samples reduced to their high byte as stb_image does."""
    if data[:8] != PNG_SIG:
        raise ValueError("not a PNG file")
    pos, idat, plte, trns, ihdr = 8, [], None, None, None
    while pos + 8 <= len(data):
        n, kind = struct.unpack(">I4s", data[pos:pos + 8])
        body = data[pos + 8:pos + 8 + n]
        pos += 12 + n
        if kind == b"IHDR":
            ihdr = struct.unpack(">IIBBBBB", body)
        elif kind == b"PLTE":
            plte = np.frombuffer(body, np.uint8).reshape(-1, 3)
        elif kind == b"tRNS":
            trns = body
        elif kind == b"IDAT":
            idat.append(body)
        elif kind == b"IEND":
            break
    if ihdr is None:
        raise ValueError("PNG without IHDR")
    w, h, depth, ctype, comp, filt, interlace = ihdr
    if ctype not in _CHANNELS or comp != 0 or filt != 0 or interlace not in (0, 1):
        raise ValueError(f"unsupported PNG (colour type {ctype}, compression {comp}, filter {filt}, interlace {interlace})")
    if ctype == 3 and plte is None:
        raise ValueError("palette PNG without PLTE")
    ch = _CHANNELS[ctype]
    raw = zlib.decompress(b"".join(idat))
    bpp = max(1, ch * depth // 8)

    def pass_samples(buf, pw, ph):
        rb = (pw * ch * depth + 7) // 8
        rows = _unfilter(buf, ph, rb, bpp)
        return _samples(rows, pw, depth, ch).reshape(ph, pw, ch), ph * (rb + 1)

    if interlace == 0:
        img, _ = pass_samples(raw, w, h)
    else:
        img = np.zeros((h, w, ch), np.uint16 if depth == 16 else np.uint8)
        off = 0
        for x0, y0, dx, dy in _ADAM7:
            pw, ph = (w - x0 + dx - 1) // dx if w > x0 else 0, (h - y0 + dy - 1) // dy if h > y0 else 0
            if pw == 0 or ph == 0:
                continue
            sub, used = pass_samples(raw[off:], pw, ph)
            img[y0::dy, x0::dx] = sub
            off += used
    # transparency key / palette expansion before the depth reduction (stbi__compute_transparency)
    if ctype == 3:
        idx = img[..., 0].astype(np.intp)
        pal = plte
        if trns is not None:
            a = np.full(len(pal), 255, np.uint8)
            t = np.frombuffer(trns, np.uint8)[:len(pal)]
            a[:len(t)] = t
            pal = np.concatenate([pal, a[:, None]], 1)
        return np.ascontiguousarray(pal[np.minimum(idx, len(pal) - 1)])
    if trns is not None and ctype in (0, 2):
        key = np.array(struct.unpack(">" + "H" * (len(trns) // 2), trns), np.uint16)[:ch]
        alpha = np.where(np.all(img.astype(np.uint16) == key, axis=-1), 0, 255 if depth != 16 else 65535)
        img = np.concatenate([img, alpha[..., None].astype(img.dtype)], -1)
    if depth == 16:
        img = (img >> 8).astype(np.uint8)
    elif depth < 8 and ctype == 0:
        img = (img.astype(np.uint16) * {1: 0xFF, 2: 0x55, 4: 0x11}[depth]).astype(np.uint8)
    return np.ascontiguousarray(img.astype(np.uint8))


def convert_channels(img: np.ndarray, n: int) -> np.ndarray:
    """stbi__convert_format: [h, w, c] uint8 -> [h, w, n]."""
    c = img.shape[-1]
    if c == n:
        return img
    f = img.astype(np.uint32)
    if c in (1, 2):
        g, a = f[..., 0], (f[..., 1] if c == 2 else np.full(f.shape[:2], 255, np.uint32))
        rgb = np.stack([g, g, g], -1)
    else:
        rgb = f[..., :3]
        a = f[..., 3] if c == 4 else np.full(f.shape[:2], 255, np.uint32)
        g = (rgb[..., 0] * 77 + rgb[..., 1] * 150 + rgb[..., 2] * 29) >> 8
    out = {1: g[..., None], 2: np.stack([g, a], -1), 3: rgb, 4: np.concatenate([rgb, a[..., None]], -1)}[n]
    return np.ascontiguousarray(out.astype(np.uint8))


def is_jpeg(data: bytes) -> bool:
    return data[:2] == b"\xff\xd8"


def is_hdr(data: bytes) -> bool:
    return data.startswith(b"#?RADIANCE\n") or data.startswith(b"#?RGBE\n")


def decode_jpeg(data: bytes, channels: int = 0) -> np.ndarray:
    """JPEG bytes -> uint8 [h, w, n] (n = channels, or the file's 3 / 1), stbi_load's bytes."""
    import ctypes as C
    from . import _check, lib
    buf = np.frombuffer(data, np.uint8)
    w, h, comp = C.c_int32(), C.c_int32(), C.c_int32()
    _check(lib().mpt_jpeg_decode(buf.ctypes.data, len(buf), channels, None, 0, C.byref(w), C.byref(h), C.byref(comp)))
    n = channels or (3 if comp.value >= 3 else 1)
    out = np.empty((h.value, w.value, n), np.uint8)
    _check(lib().mpt_jpeg_decode(buf.ctypes.data, len(buf), channels, out.ctypes.data, out.size, C.byref(w), C.byref(h),
                                 C.byref(comp)))
    return out


def decode_hdr(data: bytes, channels: int = 0) -> np.ndarray:
    """Radiance .hdr bytes -> float32 [h, w, n] (n = channels or 3), rows as stored."""
    import ctypes as C
    from . import _check, lib
    buf = np.frombuffer(data, np.uint8)
    w, h = C.c_int32(), C.c_int32()
    _check(lib().mpt_hdr_decode(buf.ctypes.data, len(buf), channels, None, 0, C.byref(w), C.byref(h)))
    out = np.empty((h.value, w.value, channels or 3), np.float32)
    _check(lib().mpt_hdr_decode(buf.ctypes.data, len(buf), channels, out.ctypes.data, out.size, C.byref(w), C.byref(h)))
    return out


def _kind(data: bytes) -> str:
    head = data[:4]
    return "DDS" if head == b"DDS " else "TGA/BMP/other"


def read_image(data: bytes, channels: int) -> np.ndarray:
    """Image8Bit::read_image(path, channels, flipY = false) on the file's bytes (stbi_load)."""
    if data[:8] == PNG_SIG:
        return convert_channels(decode_png(data), channels)
    if is_jpeg(data):
        return decode_jpeg(data, channels)
    raise ValueError(f"texture format {_kind(data)} is not supported (PNG and JPEG)")


def read_image_hdr(data: bytes, channels: int, flip_y: bool = True) -> np.ndarray:
    """Image32Bit::read_image_hdr(path, channels, flipY) on the file's bytes (stbi_loadf): float32
    [h, w, channels], the rows flipped when flip_y (stbi_set_flip_vertically_on_load)."""
    if is_hdr(data):
        img = decode_hdr(data, channels)
    elif data[:8] == PNG_SIG or is_jpeg(data):
        # stbi__ldr_to_hdr: colour channels pow(v / 255, 2.2) * 1 in double, alpha v / 255
        ldr = read_image(data, channels).astype(np.float32)
        img = np.empty(ldr.shape, np.float32)
        n = channels if channels & 1 else channels - 1
        img[..., :n] = (np.power((ldr[..., :n] / np.float32(255.0)).astype(np.float64), float(np.float32(2.2)))
                        * float(np.float32(1.0))).astype(np.float32)
        if n < channels:
            img[..., n:] = ldr[..., n:] / np.float32(255.0)
    else:
        raise ValueError(f"image format {_kind(data)} is not supported by read_image_hdr (.hdr, PNG, JPEG)")
    return np.ascontiguousarray(img[::-1]) if flip_y else img


def load_envmap(path) -> np.ndarray:
    """The envmap as RendererEnvmap reads it (RendererEnvmap.cpp:39-48 -> ThreadFunctions::read_envmap,
    ThreadFunctions.cpp:145-151): read_image_hdr(path, 4, flipY = true) -> float32 [h, w, 4], the
    input of mpt.build_envmap.  (.exr envmaps, read by tinyexr in the reference, are not supported.)"""
    path = str(path)
    if path.endswith(".exr"):
        raise ValueError("OpenEXR envmaps are not supported (use .hdr)")
    with open(path, "rb") as f:
        return read_image_hdr(f.read(), 4, True)


def to_rgba8(img: np.ndarray) -> np.ndarray:
    """The texture as the kernels read it (include/mpt.h: RGBA8 per texel): what a 1 / 2 / 4
    channel HIP texture object returns for tex2D<float4>: missing colour channels 0, a
    missing alpha 1 (255); 3-channel images get alpha 255."""
    h, w, c = img.shape
    out = np.zeros((h, w, 4), np.uint8)
    out[..., 3] = 255
    if c == 2:
        out[..., 0], out[..., 1] = img[..., 0], img[..., 1]
    else:
        out[..., :c] = img
    return out


def encode_png(img: np.ndarray, filters=(0, 1, 2, 3, 4), palette=None, interlace=False) -> bytes:
    """Minimal PNG writer (tests and fixtures): uint8 [h, w, c] (c = 1..4) or palette indices
    with `palette` [n, 3] (+ alpha column -> tRNS); row filters cycled from `filters`."""
    img = np.asarray(img)
    h, w = img.shape[:2]
    c = 1 if img.ndim == 2 else img.shape[2]
    if palette is not None:
        ctype, ch = 3, 1
    else:
        ctype, ch = {1: 0, 2: 4, 3: 2, 4: 6}[c], c
    px = img.reshape(h, w, ch).astype(np.uint8)

    def filt(rows):
        out = bytearray()
        prev = np.zeros(rows.shape[1] * ch, np.int32)
        for y in range(rows.shape[0]):
            cur = rows[y].reshape(-1).astype(np.int32)
            f = filters[y % len(filters)]
            a = np.concatenate([np.zeros(ch, np.int32), cur[:-ch]]) if len(cur) else cur
            cc = np.concatenate([np.zeros(ch, np.int32), prev[:-ch]]) if len(cur) else cur
            if f == 0:
                d = cur
            elif f == 1:
                d = cur - a
            elif f == 2:
                d = cur - prev
            elif f == 3:
                d = cur - ((a + prev) >> 1)
            else:
                p = a + prev - cc
                pa, pb, pc = np.abs(p - a), np.abs(p - prev), np.abs(p - cc)
                d = cur - np.where((pa <= pb) & (pa <= pc), a, np.where(pb <= pc, prev, cc))
            out += bytes([f]) + (d & 0xFF).astype(np.uint8).tobytes()
            prev = cur
        return bytes(out)

    if interlace:
        raw = b"".join(filt(px[y0::dy, x0::dx]) for x0, y0, dx, dy in _ADAM7
                       if px[y0::dy, x0::dx].size)
    else:
        raw = filt(px)

    def chunk(k, b):
        return struct.pack(">I", len(b)) + k + b + struct.pack(">I", zlib.crc32(k + b) & 0xFFFFFFFF)

    out = PNG_SIG + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, ctype, 0, 0, 1 if interlace else 0))
    if palette is not None:
        pal = np.asarray(palette, np.uint8)
        out += chunk(b"PLTE", pal[:, :3].tobytes())
        if pal.shape[1] == 4:
            out += chunk(b"tRNS", pal[:, 3].tobytes())
    return out + chunk(b"IDAT", zlib.compress(raw)) + chunk(b"IEND", b"")
