"""Image decoding pinned to the reference's own decoder (scene / envmap ingestion).

The reference reads textures with stb_image's stbi_load and envmaps / baked LUTs with stbi_loadf
(src/Image/Image.cpp:33-61, 342-370).  tests/golden/make_image_fixtures.py ran the reference's
unmodified stb_image.h (compiled from /root/reference by oracle/Makefile's `ref` target) on the
committed inputs of tests/golden/images/ and stored every decode; mpt.image (PNG in Python +
mpt_png_unfilter, JPEG / .hdr in csrc/jpeg.cpp) must reproduce them byte for byte -- float for
float for stbi_loadf.  The reference's own JPEG textures (the-white-room), its README render and
its LUT .hdr files are checked through SHA-256 of the stb decode when /root/reference exists.
No GPU: the decoders are host code in libmpt.
"""
import hashlib
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
IMG = os.path.join(HERE, "golden", "images")
REF = "/root/reference"


def _decodes():
    with np.load(os.path.join(IMG, "decodes.npz")) as z:
        return {k: z[k] for k in z.files}


DECODES = _decodes()


def _decode(name, mode, req, flip):
    from mpt import image
    data = open(os.path.join(IMG, name), "rb").read()
    if mode == "u8":
        out = image.read_image(data, req) if req else (
            image.decode_jpeg(data) if image.is_jpeg(data) else image.decode_png(data))
        return out
    return image.read_image_hdr(data, req, bool(flip))


@pytest.mark.parametrize("key", sorted(DECODES))
def test_decode_matches_stb_image(key):
    name, mode, req, flip = key.split("|")
    want = DECODES[key]
    got = _decode(name, mode, int(req), int(flip))
    assert got.shape == want.shape, (got.shape, want.shape)
    if mode == "f32":
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), f"{key}: {(got != want).sum()} floats differ"
    else:
        assert np.array_equal(got, want), f"{key}: {(got != want).sum()} bytes differ (max {np.abs(got.astype(int) - want).max()})"


def test_every_input_has_decodes():
    names = {k.split("|")[0] for k in DECODES}
    files = {f for f in os.listdir(IMG) if f.endswith((".jpg", ".png", ".hdr"))}
    assert names == files
    assert any(n.startswith("synth_") for n in names) and any("prog" in n for n in names)


REF_HASHES = json.load(open(os.path.join(IMG, "reference_files.json")))


@pytest.mark.skipif(not os.path.isdir(REF), reason="the reference checkout is not present (build container only)")
@pytest.mark.parametrize("key", sorted(REF_HASHES))
def test_reference_files_decode_like_stb_image(key):
    from mpt import image
    rel, mode, req, flip = key.split("|")
    data = open(os.path.join(REF, rel), "rb").read()
    out = image.read_image(data, int(req)) if mode == "u8" else image.read_image_hdr(data, int(req), bool(int(flip)))
    assert hashlib.sha256(np.ascontiguousarray(out).tobytes()).hexdigest() == REF_HASHES[key]


def test_load_envmap_is_read_image_hdr_4_flipped(tmp_path):
    from mpt import image
    p = tmp_path / "sky.hdr"
    p.write_bytes(open(os.path.join(IMG, "rle.hdr"), "rb").read())
    env = image.load_envmap(p)
    want = DECODES["rle.hdr|f32|4|1"]
    assert env.shape == want.shape and np.array_equal(env, want)
    assert np.all(env[..., 3] == 1.0)
    with pytest.raises(ValueError, match="EXR"):
        image.load_envmap(tmp_path / "sky.exr")


def test_unsupported_and_corrupt_inputs_raise():
    import mpt
    from mpt import image
    with pytest.raises(ValueError, match="not supported"):
        image.read_image(b"DDS " + bytes(100), 4)
    jpg = open(os.path.join(IMG, "pil_q75_444.jpg"), "rb").read()
    with pytest.raises(mpt.MptError, match="jpeg"):
        image.decode_jpeg(jpg[:2] + b"\xff\xc4\x00\x03\x20")   # a DHT naming table class 2
    with pytest.raises(mpt.MptError, match="hdr"):
        image.decode_hdr(b"#?RADIANCE\nFORMAT=32-bit_rle_xyze\n\n-Y 1 +X 1\n\x00\x00\x00\x00")


def _patch_sof(jpg, h, w):
    """The JPEG with its SOF0 frame size replaced (marker FFC0: Lf, P, Y, X)."""
    i = jpg.index(b"\xff\xc0")
    return jpg[:i + 5] + h.to_bytes(2, "big") + w.to_bytes(2, "big") + jpg[i + 9:]


def test_jpeg_header_query_validates_before_allocating():
    """mpt_jpeg_decode's header-only call (out == NULL, what decode_jpeg sizes its array by) runs the
    frame header's checks: an oversized (65535 x 65535 x 3 > 2^31 bytes) or zero frame is an error
    there, not an allocation; a file cut inside the SOF reads zeros and fails the same way."""
    import mpt
    from mpt import image
    jpg = open(os.path.join(IMG, "pil_q75_444.jpg"), "rb").read()
    with pytest.raises(mpt.MptError, match="too large"):
        image.decode_jpeg(_patch_sof(jpg, 65535, 65535))
    with pytest.raises(mpt.MptError, match="height"):
        image.decode_jpeg(_patch_sof(jpg, 0, 64))
    with pytest.raises(mpt.MptError, match="jpeg"):
        image.decode_jpeg(jpg[:jpg.index(b"\xff\xc0") + 6])


def test_jpeg_undefined_tables_are_deterministic():
    """A scan that names Huffman tables no DHT defined decodes from zeroed tables (stb memsets its
    decoder, stb_image.h:4031): the outcome -- here an error -- is the same on every call."""
    import mpt
    from mpt import image
    jpg = bytearray(open(os.path.join(IMG, "pil_q75_444.jpg"), "rb").read())
    i = jpg.index(b"\xff\xda")
    n = jpg[i + 4]
    for c in range(n):
        jpg[i + 6 + 2 * c] = 0x33          # Td = Ta = 3: never defined in this file
    outcomes = []
    for _ in range(3):
        try:
            outcomes.append(image.decode_jpeg(bytes(jpg)).tobytes())
        except mpt.MptError as e:
            outcomes.append(str(e))
    assert outcomes[0] == outcomes[1] == outcomes[2]


@pytest.mark.gpu
def test_every_stb_fixture_on_the_gpu_box():
    """The decode fixtures again inside the GPU run (the driver records that run): every committed
    input decodes byte for byte as the reference's stb_image did (host code of libmpt)."""
    bad = []
    for key in sorted(DECODES):
        name, mode, req, flip = key.split("|")
        got = _decode(name, mode, int(req), int(flip))
        want = DECODES[key]
        same = got.shape == want.shape and (np.array_equal(got.view(np.uint32), want.view(np.uint32)) if mode == "f32"
                                            else np.array_equal(got, want))
        if not same:
            bad.append(key)
    assert not bad and len(DECODES) > 200, bad[:5]
