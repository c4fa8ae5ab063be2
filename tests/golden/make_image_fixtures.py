"""Generates tests/golden/images/: decoder inputs and the decodes of the reference's own image
decoder (test infrastructure; run in the build container, where /root/reference exists).

The reference decodes textures with stb_image's stbi_load and envmaps / LUTs with stbi_loadf
(src/Image/Image.cpp:33-61, 342-370).  oracle/Makefile's `ref` target compiles the reference's
unmodified thirdparties/stbi/stb_image.h (where it lies) behind oracle/stbi_ref.c into
oracle/_ref/stbi_decode; this script runs it on
  * synthetic inputs written here (PIL JPEGs: 4:4:4 / 4:2:2 / 4:2:0, progressive, restart
    markers, optimised tables, grey, CMYK, q100, 1-pixel-wide and tiny images; jpeg_synth.py
    baseline files with the sampling ratios PIL cannot write (1x2, 4x1, 3x1, 1x4), 'R','G','B'
    ids, Adobe RGB / CMYK / YCCK / YCbCrK, restart intervals; PNGs of every colour type; Radiance
    .hdr files, RLE, flat and stb's non-RLE-first-scanline fallback), committed as inputs with
    every decode in decodes.npz;
  * the reference's own files (the-white-room's JPEG textures, the README render, the baked
    LUT .hdr files): too large to commit, so the SHA-256 of each decode goes to
    reference_files.json and tests/test_image_decode.py decodes them when /root/reference is
    present.

usage: make -C oracle ref && python tests/golden/make_image_fixtures.py
"""
from __future__ import annotations

import glob
import hashlib
import io
import json
import os
import struct
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
OUT = os.path.join(HERE, "images")
STBI = os.path.join(ROOT, "oracle", "_ref", "stbi_decode")
REF = "/root/reference"
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(ROOT, "hiprt-path-tracer_amd"))

U8_REQS = (0, 1, 2, 3, 4)
F32_REQS = ((1, 1), (3, 0), (4, 1))


def stbi(path, mode, req, flip):
    tmp = os.path.join(OUT, ".tmp.bin")
    r = subprocess.run([STBI, mode, str(req), str(flip), path, tmp], capture_output=True, text=True)
    if r.returncode != 0:
        return None
    raw = open(tmp, "rb").read()
    os.remove(tmp)
    w, h, c = struct.unpack("<3i", raw[:12])
    return np.frombuffer(raw[12:], np.uint8 if mode == "u8" else np.float32).reshape(h, w, req or c)


def _test_image(w, h, seed):
    """A smooth gradient with texture and a few hard edges (exercises every coefficient band)."""
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w].astype(np.float32)
    img = np.stack([128 + 100 * np.sin(x / 5.0 + seed), 128 + 90 * np.cos(y / 4.0), 255 * ((x + y) % 11 < 5)], -1)
    img += rng.normal(0, 12, img.shape)
    return np.clip(img, 0, 255).astype(np.uint8)


def _rgbe(rgb):
    """float [h, w, 3] -> RGBE bytes per pixel (frexp, as Radiance writers do)."""
    m = rgb.max(-1)
    e = np.zeros(m.shape, np.int32)
    mant, e = np.frexp(m)
    scale = np.where(m > 1e-32, mant * 256.0 / np.where(m > 0, m, 1), 0)
    out = np.zeros(rgb.shape[:2] + (4,), np.uint8)
    out[..., :3] = np.clip(rgb * scale[..., None], 0, 255).astype(np.uint8)
    out[..., 3] = np.where(m > 1e-32, e + 128, 0)
    return out


def _hdr(rgbe, rle=True, header="#?RADIANCE"):
    h, w = rgbe.shape[:2]
    body = bytearray()
    for j in range(h):
        row = rgbe[j]
        if not rle:
            body += row.tobytes()
            continue
        body += bytes([2, 2, w >> 8, w & 255])
        for k in range(4):
            ch, i = row[:, k], 0
            while i < w:
                r = 1
                while i + r < w and r < 127 and ch[i + r] == ch[i]:
                    r += 1
                if r >= 3:
                    body += bytes([128 + r, ch[i]])
                    i += r
                else:
                    d = 1
                    while i + d < w and d < 128 and not (i + d + 2 < w and ch[i + d] == ch[i + d + 1] == ch[i + d + 2]):
                        d += 1
                    body += bytes([d]) + ch[i:i + d].tobytes()
                    i += d
    return f"{header}\nFORMAT=32-bit_rle_rgbe\nEXPOSURE=1.0\n\n-Y {h} +X {w}\n".encode() + bytes(body)


def inputs():
    from PIL import Image

    import jpeg_synth
    from mpt import image as mimg
    files = {}
    base = _test_image(45, 37, 1)
    pil = Image.fromarray(base)
    for name, kw in [("q75_444", dict(quality=75, subsampling=0)), ("q75_422", dict(quality=75, subsampling=1)),
                     ("q90_420", dict(quality=90, subsampling=2)), ("prog_420", dict(quality=80, subsampling=2, progressive=True)),
                     ("prog_444_opt", dict(quality=85, subsampling=0, progressive=True, optimize=True)),
                     ("restart_rows", dict(quality=70, subsampling=2, restart_marker_rows=1)),
                     ("restart_blocks_prog", dict(quality=70, subsampling=2, progressive=True, restart_marker_blocks=5)),
                     ("q100_420", dict(quality=100, subsampling=2)), ("q20_420", dict(quality=20, subsampling=2))]:
        b = io.BytesIO()
        pil.save(b, "JPEG", **kw)
        files[f"pil_{name}.jpg"] = b.getvalue()
    for name, im in [("grey", pil.convert("L")), ("cmyk", pil.convert("CMYK")),
                     ("w1_420", Image.fromarray(_test_image(1, 19, 2))), ("tiny_420", Image.fromarray(_test_image(3, 2, 3))),
                     ("w17_422", Image.fromarray(_test_image(17, 9, 4)))]:
        for prog in (False, True):
            b = io.BytesIO()
            im.save(b, "JPEG", quality=80, subsampling=2 if im.mode != "L" else 0, progressive=prog)
            files[f"pil_{name}{'_prog' if prog else ''}.jpg"] = b.getvalue()
    synth = [("v2", [(1, 2), (1, 1), (1, 1)], {}), ("h4", [(4, 1), (1, 1), (1, 1)], {}),
             ("h3", [(3, 1), (1, 1), (1, 1)], {}), ("v4", [(1, 4), (1, 1), (1, 1)], {}),
             ("hv2_restart2", [(2, 2), (1, 1), (1, 1)], dict(restart=2)),
             ("ids_rgb", [(1, 1)] * 3, dict(ids=[ord("R"), ord("G"), ord("B")], jfif=False)),
             ("adobe_rgb", [(1, 1)] * 3, dict(adobe=0, jfif=False)),
             ("adobe_ycc_nojfif", [(2, 1), (1, 1), (1, 1)], dict(adobe=1, jfif=False)),
             ("cmyk", [(2, 2), (1, 1), (1, 1), (2, 2)], dict(adobe=0, jfif=False)),
             ("ycck", [(2, 2), (1, 1), (1, 1), (2, 2)], dict(adobe=2, jfif=False)),
             ("ycbcrk", [(1, 1)] * 4, dict(adobe=1)), ("grey_2x2", [(2, 2)], {})]
    for i, (name, samp, kw) in enumerate(synth):
        files[f"synth_{name}.jpg"] = jpeg_synth.encode(29, 23, samp, seed=10 + i, **kw)
    # PNG: every colour type stb converts (the loader's own decoder is mpt.image.decode_png)
    rgba = np.concatenate([base, (base[..., :1] // 2 + 60)], -1)
    files["rgba8.png"] = mimg.encode_png(rgba)
    files["rgb8_interlaced.png"] = mimg.encode_png(base, interlace=True)
    files["grey8.png"] = mimg.encode_png(base[..., 0])
    files["greya8.png"] = mimg.encode_png(rgba[..., [0, 3]])
    pal = np.array([[255, 0, 0, 255], [0, 255, 0, 128], [0, 0, 255, 0], [250, 250, 250, 255]], np.uint8)
    files["palette_trns.png"] = mimg.encode_png((base[..., 0] // 64).astype(np.uint8), palette=pal)
    # Radiance .hdr
    rng = np.random.default_rng(5)
    sky = np.exp(rng.normal(0, 2, (13, 40, 3))).astype(np.float32)
    sky[2, :5] = 0.0                                   # zero exponents
    sky[4, 10:30] = sky[4, 10]                         # runs
    e = _rgbe(sky)
    files["rle.hdr"] = _hdr(e)
    files["rgbe_header.hdr"] = _hdr(e, header="#?RGBE")
    files["flat_w6.hdr"] = _hdr(_rgbe(sky[:, :6]), rle=False)
    files["flat_w40.hdr"] = _hdr(e, rle=False)        # width >= 8 without RLE: stb's fallback path
    return files


def main():
    if not os.path.exists(STBI):
        sys.exit("build oracle/_ref/stbi_decode first: make -C oracle ref")
    os.makedirs(OUT, exist_ok=True)
    arrays = {}
    for name, data in sorted(inputs().items()):
        path = os.path.join(OUT, name)
        with open(path, "wb") as f:
            f.write(data)
        if name.endswith(".hdr"):
            for req, flip in F32_REQS:
                arrays[f"{name}|f32|{req}|{flip}"] = stbi(path, "f32", req, flip)
        else:
            for req in U8_REQS:
                d = stbi(path, "u8", req, 0)
                if d is None:
                    raise RuntimeError(f"stb_image refused {name}")
                arrays[f"{name}|u8|{req}|0"] = d
            arrays[f"{name}|f32|4|1"] = stbi(path, "f32", 4, 1)   # stbi_loadf of an 8-bit file
    np.savez_compressed(os.path.join(OUT, "decodes.npz"), **arrays)
    ref = {}
    if os.path.isdir(REF):
        jpgs = sorted(glob.glob(f"{REF}/data/GLTFs/the-white-room/*.jpg")) + [f"{REF}/README_data/Features/img/cornell_pbr_reference.jpg"]
        for p in jpgs:
            for req in (1, 3, 4):
                ref[f"{os.path.relpath(p, REF)}|u8|{req}|0"] = hashlib.sha256(stbi(p, "u8", req, 0).tobytes()).hexdigest()
        for p in sorted(glob.glob(f"{REF}/data/BRDFsData/**/*.hdr", recursive=True))[::7]:
            ref[f"{os.path.relpath(p, REF)}|f32|1|1"] = hashlib.sha256(stbi(p, "f32", 1, 1).tobytes()).hexdigest()
    with open(os.path.join(OUT, "reference_files.json"), "w") as f:
        json.dump(ref, f, indent=1, sort_keys=True)
    print(f"{len(arrays)} decodes, {len(ref)} reference-file hashes -> {OUT}")


if __name__ == "__main__":
    main()
