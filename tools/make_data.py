#!/usr/bin/env python3
"""Converts the reference's data assets into the repo's data/ directory.

Runs only where /root/reference exists (this container).  Outputs are DATA
(inputs of the renderer), committed so that the GPU box, which has no
/root/reference, can load them:

* data/luts.npz -- the energy-compensation LUTs the reference ships in
  data/BRDFsData (baked by its own GPUBaker, GPUBakerConstants.h:15-32), decoded
  exactly as Image32Bit::read_image_hdr(path, 1 channel, flipY=true) does
  (Image/Image.cpp:342-370 -> stb_image 'stbi__hdr_convert', thirdparties/stbi/
  stb_image.h:7130-7155: 1 channel = (r+g+b) * 2^(e-136) / 3, rows flipped), and
  stacked in the order CPURenderer::setup_brdfs_data loads them
  (Renderer/CPURenderer.cpp:93-132).  Also the sheen LTC parameter table
  (Device/includes/BSDFs/SheenLTCFittedParameters.h, 32x32 float3 published by
  Zeltner et al. 2022), as numbers.
* data/scenes/*.gltf|.bin -- the shipped test scenes (data/GLTFs).
"""
import os
import re
import shutil
import sys

import numpy as np

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data")


def read_rgbe(path):
    """Radiance .hdr (RGBE, new-style RLE or flat) -> uint8 array (H, W, 4) in file row order."""
    with open(path, "rb") as f:
        data = f.read()
    pos = 0
    # header lines until blank line
    while True:
        end = data.index(b"\n", pos)
        line = data[pos:end]
        pos = end + 1
        if line.strip() == b"":
            break
    end = data.index(b"\n", pos)
    res = data[pos:end].decode().split()
    pos = end + 1
    assert res[0] == "-Y" and res[2] == "+X", res
    h, w = int(res[1]), int(res[3])
    out = np.zeros((h, w, 4), np.uint8)
    buf = np.frombuffer(data, np.uint8)
    for y in range(h):
        if w < 8 or w > 0x7FFF or not (buf[pos] == 2 and buf[pos + 1] == 2 and (buf[pos + 2] & 0x80) == 0):
            # flat scanline
            out[y] = buf[pos:pos + 4 * w].reshape(w, 4)
            pos += 4 * w
            continue
        sw = (int(buf[pos + 2]) << 8) | int(buf[pos + 3])
        assert sw == w
        pos += 4
        for c in range(4):
            x = 0
            while x < w:
                count = int(buf[pos])
                pos += 1
                if count > 128:
                    count -= 128
                    out[y, x:x + count, c] = buf[pos]
                    pos += 1
                else:
                    out[y, x:x + count, c] = buf[pos:pos + count]
                    pos += count
                x += count
    return out


def hdr_to_float(rgbe, channels):
    """stbi__hdr_convert semantics, then vertical flip (flipY=true)."""
    e = rgbe[..., 3].astype(np.int32)
    f1 = np.ldexp(np.float32(1.0), e - 136).astype(np.float32)
    nz = rgbe[..., 3] != 0
    if channels == 1:
        s = (rgbe[..., 0].astype(np.int32) + rgbe[..., 1] + rgbe[..., 2]).astype(np.float32)
        v = (s * f1) / np.float32(3.0)
        v = np.where(nz, v, np.float32(0.0)).astype(np.float32)
    else:
        v = rgbe[..., :3].astype(np.float32) * f1[..., None]
        v = np.where(nz[..., None], v, np.float32(0.0)).astype(np.float32)
        if channels == 4:
            v = np.concatenate([v, np.ones_like(v[..., :1])], axis=-1)
    return np.ascontiguousarray(v[::-1])


def load_lut(path):
    return hdr_to_float(read_rgbe(path), 1)


def main():
    if not os.path.isdir(REF):
        print("no /root/reference here; nothing to do")
        return 0
    os.makedirs(OUT, exist_ok=True)
    b = os.path.join(REF, "data", "BRDFsData")
    conductor = load_lut(os.path.join(b, "GGX", "GGX_Conductor_128x128.hdr"))
    glossy = np.stack([load_lut(os.path.join(b, "GlossyDielectrics", "%dGlossy_Ess_128x64x128.hdr" % i)) for i in range(128)])
    glass = np.stack([load_lut(os.path.join(b, "GGX", "Glass", "%dGGX_Glass_Ess_256x16x128.hdr" % i)) for i in range(128)])
    glass_inv = np.stack([load_lut(os.path.join(b, "GGX", "Glass", "%dinv_GGX_Glass_Ess_256x16x128.hdr" % i)) for i in range(128)])
    thin = np.stack([load_lut(os.path.join(b, "GGX", "Glass", "%dGGX_Thin_Glass_Ess_32x32x96.hdr" % i)) for i in range(96)])
    src = open(os.path.join(REF, "src/Device/includes/BSDFs/SheenLTCFittedParameters.h")).read()
    trip = re.findall(r"make_float3\(\s*([-0-9.eE+]+)f?\s*,\s*([-0-9.eE+]+)f?\s*,\s*([-0-9.eE+]+)f?\s*\)", src)
    sheen = np.array([[float(a), float(b_), float(c)] for a, b_, c in trip], np.float32).reshape(32, 32, 3)
    print("shapes", conductor.shape, glossy.shape, glass.shape, glass_inv.shape, thin.shape, sheen.shape)
    np.savez_compressed(os.path.join(OUT, "luts.npz"), ggx_conductor=conductor, glossy_dielectric=glossy,
                        ggx_glass=glass, ggx_glass_inverse=glass_inv, ggx_thin_glass=thin, sheen_ltc=sheen)
    sd = os.path.join(OUT, "scenes")
    os.makedirs(sd, exist_ok=True)
    for n in ["cornell_pbr", "multi-dispersion", "nested-dielectrics", "nested-dielectrics-complex"]:
        for ext in (".gltf", ".bin"):
            shutil.copyfile(os.path.join(REF, "data", "GLTFs", n + ext), os.path.join(sd, n + ext))
    return 0


if __name__ == "__main__":
    sys.exit(main())
