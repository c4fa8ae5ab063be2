"""glTF ingestion with textures (SceneParser.cpp:22-220,
ThreadFunctions.cpp:30-143), on the synthetic textured room of
mpt.synthetic.write_textured_gltf (the reference's one textured glTF ships without its .bin).

CPU: the PNG decoder against PIL (when importable; the decoder itself needs only zlib and
libmpt's scanline filter reversal) and its own writer over every colour type, filter and
interlacing; stb_image's channel conversions; the texture slot order, indices and channel
counts of SceneParser::get_textures_paths_and_indices / load_scene_texture; constant-emission
folding (CONSTANT_EMISSIVE_TEXTURE); the V flip and the dropped coordinates of untextured
meshes; .gltf (files, '%20' names, data: URIs) and .glb (bufferView images) giving the same
scene.  GPU: the textured room rendered by libmpt equals the CPU oracle bit for bit."""
import io

import numpy as np
import pytest

from mpt import abi, image, scene, synthetic


@pytest.fixture(scope="module")
def room(tmp_path_factory):
    d = tmp_path_factory.mktemp("room")
    return scene.load_gltf(synthetic.write_textured_gltf(str(d)))


@pytest.mark.parametrize("channels", [1, 2, 3, 4])
@pytest.mark.parametrize("interlace", [False, True])
def test_png_roundtrip_every_filter(channels, interlace):
    rng = np.random.default_rng(channels)
    x = rng.integers(0, 256, (23, 29, channels)).astype(np.uint8)
    for filters in ((0,), (1,), (2,), (3,), (4,), (0, 1, 2, 3, 4)):
        y = image.decode_png(image.encode_png(x, filters=filters, interlace=interlace))
        assert np.array_equal(y, x), filters


def test_png_palette_trns():
    rng = np.random.default_rng(1)
    pal = np.concatenate([rng.integers(0, 256, (9, 3)), rng.integers(0, 256, (9, 1))], 1).astype(np.uint8)
    idx = rng.integers(0, 9, (11, 13)).astype(np.uint8)
    assert np.array_equal(image.decode_png(image.encode_png(idx, palette=pal)), pal[idx])
    assert np.array_equal(image.decode_png(image.encode_png(idx, palette=pal[:, :3])), pal[idx, :3])


@pytest.mark.parametrize("mode", ["1", "L", "LA", "RGB", "RGBA", "P", "I;16"])
def test_png_matches_pil(mode):
    PIL = pytest.importorskip("PIL.Image")
    rng = np.random.default_rng(7)
    a = rng.integers(0, 256, (21, 19, 4)).astype(np.uint8)
    if mode == "1":
        im = PIL.fromarray(a[..., 0] > 127).convert("1")
    elif mode == "I;16":
        im = PIL.fromarray((a[..., 0].astype(np.uint16) * 257 + 7).astype(np.uint16))
    elif mode == "P":
        im = PIL.fromarray(a[..., :3]).convert("P")
    else:
        im = PIL.fromarray({"L": a[..., 0], "LA": a[..., :2], "RGB": a[..., :3], "RGBA": a}[mode], mode)
    for interlace in (0, 1):
        b = io.BytesIO()
        im.save(b, "PNG", interlace=interlace)
        got = image.decode_png(b.getvalue())
        ref = PIL.open(io.BytesIO(b.getvalue()))
        if mode == "I;16":
            want = (np.asarray(ref.convert("I")) >> 8).astype(np.uint8)[..., None]
        elif mode == "P":
            want = np.asarray(ref.convert("RGB"))
        else:
            want = np.asarray(ref.convert("L" if mode == "1" else mode)).reshape(got.shape)
        assert np.array_equal(got, want), (mode, interlace)


def test_stb_channel_conversion():
    """stbi__convert_format: RGB -> grey = (77 r + 150 g + 29 b) >> 8, grey -> RGB replicates,
    a missing alpha is 255."""
    px = np.array([[[10, 200, 30], [255, 255, 255], [0, 0, 0]]], np.uint8)
    g = image.convert_channels(px, 1)[..., 0]
    assert g.tolist() == [[(10 * 77 + 200 * 150 + 30 * 29) >> 8, 255, 0]]
    assert image.convert_channels(px, 4)[..., 3].tolist() == [[255, 255, 255]]
    ga = np.array([[[7, 99]]], np.uint8)
    assert image.convert_channels(ga, 4).tolist() == [[[7, 7, 7, 99]]]
    assert image.convert_channels(ga, 1).tolist() == [[[7]]]
    assert image.to_rgba8(np.array([[[5]]], np.uint8)).tolist() == [[[5, 0, 0, 255]]]


def test_unsupported_format_fails_loudly():
    """Formats the loader does not decode (DDS, TGA, ...) and corrupt JPEGs raise; JPEG itself is
    decoded (tests/test_image_decode.py pins it against the reference's stb_image)."""
    import mpt
    with pytest.raises(ValueError, match="DDS"):
        image.read_image(b"DDS " + b"\0" * 16, 4)
    with pytest.raises(mpt.MptError, match="jpeg"):
        image.read_image(b"\xff\xd8\xff\xe0" + b"\0" * 16, 4)


def test_texture_slots_and_indices(room):
    """Per material, slots in the order base colour, emission, roughness-metallic, specular,
    coat, sheen, transmission, normal map; global index = the material's offset + local index."""
    m = room.materials
    slots = ["base_color_texture_index", "emission_texture_index", "roughness_metallic_texture_index",
             "specular_texture_index", "coat_texture_index", "sheen_texture_index",
             "specular_transmission_texture_index", "normal_map_texture_index"]
    got = [[getattr(x, s) for s in slots] for x in m]
    assert got == [[0, -1, 1, -1, -1, -1, -1, 2],
                   [-1] * 8,
                   [-1, 3, -1, 4, 5, -1, -1, -1],
                   [-1, -2, -1, -1, -1, 7, 8, -1],
                   [-1] * 8]
    assert len(room.textures) == 9 and all(t.dtype == np.uint8 and t.shape[2] == 4 for t in room.textures)


def test_texture_channel_counts(room, tmp_path):
    """load_scene_texture's channel counts: roughness-metallic 3 (alpha 255), specular / coat /
    sheen / transmission 1 (stb grey, stored as (y, 0, 0, 255)), base colour / normal / emission 4."""
    import os
    d = tmp_path / "r"
    synthetic.write_textured_gltf(str(d))
    raw = image.decode_png(open(os.path.join(d, "left_specular.png"), "rb").read())
    spec = room.textures[4]
    y = (raw[..., 0].astype(np.uint32) * 77 + raw[..., 1].astype(np.uint32) * 150 + raw[..., 2].astype(np.uint32) * 29) >> 8
    assert np.array_equal(spec[..., 0], y) and not spec[..., 1:3].any() and (spec[..., 3] == 255).all()
    mr = room.textures[1]
    assert np.array_equal(mr[..., :3], image.decode_png(open(os.path.join(d, "floor_mr.png"), "rb").read()))
    assert (mr[..., 3] == 255).all()
    coat = room.textures[5]    # grey + alpha -> 1 channel: the grey value
    la = image.decode_png(open(os.path.join(d, "left_coat.png"), "rb").read())
    assert np.array_equal(coat[..., 0], la[..., 0])


def test_constant_emission_folded(room, tmp_path):
    """A constant emission texture (every stb value within 5 of the first texel) is not kept:
    emission_texture_index = CONSTANT_EMISSIVE_TEXTURE and emission = the texel sampled at uv
    (0, 0) -- the bottom-left one -- / 255 (ThreadFunctions.cpp:84-93, Image.cpp:161-193); the
    folded material is then an NEE light (its triangles join the emissive list), while the
    varying emission texture keeps the default black emission and no NEE entry."""
    import os
    d = tmp_path / "r"
    synthetic.write_textured_gltf(str(d))
    em = image.decode_png(open(os.path.join(d, "right_emission.png"), "rb").read())
    m = room.materials[3]
    assert m.emission_texture_index == scene.CONSTANT_EMISSIVE_TEXTURE
    want = em[-1, 0, :3].astype(np.float32) / np.float32(255.0)
    assert [m.emission.r, m.emission.g, m.emission.b] == [float(x) for x in want]
    left = room.materials[2]
    assert (left.emission.r, left.emission.g, left.emission.b) == (0.0, 0.0, 0.0) and left.emission_texture_index == 3
    tri_mat = room.material_indices[room.emissive]
    assert sorted(set(tri_mat.tolist())) == [3, 4]


def test_texcoords_flipped_and_dropped(room):
    """ASSIMP's glTF2 importer flips V; untextured meshes get zero coordinates."""
    floor = room.texcoords[room.triangle_indices.reshape(-1, 3)[room.material_indices == 0].ravel()]
    assert np.allclose(sorted(set(floor[:, 1].tolist())), [-0.5, 1.0])
    wall = room.triangle_indices.reshape(-1, 3)[room.material_indices == 1].ravel()
    assert not room.texcoords[wall].any()


def test_glb_equals_gltf(room, tmp_path):
    b = scene.load_gltf(synthetic.write_textured_gltf(str(tmp_path / "glb"), glb=True))
    for k in ("vertices", "normals", "texcoords", "triangle_indices", "material_indices", "emissive"):
        assert np.array_equal(getattr(room, k), getattr(b, k)), k
    assert len(b.textures) == len(room.textures)
    assert all(np.array_equal(x, y) for x, y in zip(room.textures, b.textures))
    assert [bytes(m) for m in b.materials] == [bytes(m) for m in room.materials]


@pytest.mark.gpu
@pytest.mark.parametrize("lss", ["mis", "ris"])
def test_gpu_textured_gltf_matches_oracle(room, luts, lss):
    import mpt
    from oracle import oracle as orc
    W, H = 48, 48
    cam = scene.make_camera(room.camera_info, W, H)
    opt = abi.KernelOptions.default()
    opt.direct_light_sampling = abi.LSS_MIS_LIGHT_BSDF if lss == "mis" else abi.LSS_RIS_BSDF_AND_LIGHT
    frames = [scene.make_frame(cam, W, H, options=opt, sample_number=s, random_seed=seed)
              for s, seed in scene.cpu_seed_schedule(3)]
    with mpt.GPURenderer(0) as r:
        r.set_scene(room)
        r.set_luts(luts)
        for f in frames:
            r.render(f)
        r.synchronize_kernel()
        img = [r.framebuffer(k) for k in (abi.FB_COLOR, abi.FB_ALBEDO, abi.FB_NORMALS)]
    ref = orc.Oracle(room, luts).render(frames, aov=True)
    for k in range(3):
        assert np.array_equal(img[k], ref[k]), f"aov {k}: {(img[k] != ref[k]).sum()} values differ"
    assert img[0].mean() > 0
