"""Host-side scene preparation: glTF -> the flat arrays of the reference's ``Scene``.

The reference ingests scenes with ASSIMP (``SceneParser::parse_scene_file``,
src/Scene/SceneParser.cpp:22-220, flags PreTransformVertices | Triangulate) and
produces flat SoA arrays (``Scene``, SceneParser.h:80-131).  ASSIMP is an empty
submodule in the reference snapshot, so this module restates the parts of its glTF2
importer that the reference consumes:

* one output mesh per (material) in material order (PreTransformVertices joins the
  node-transformed primitives sharing a material);
* material parameters read as ``SceneParser::read_material_properties``
  (SceneParser.cpp:366-407) reads them from ASSIMP's glTF2 material keys, then
  ``make_safe`` + ``precompute_properties`` (HostDeviceCommon/Material.h:44-71);
* the emissive triangle list of ``ThreadFunctions::load_scene_parse_emissive_triangles``
  (Threads/ThreadFunctions.cpp:116-143);
* the textures of ``SceneParser::prepare_textures`` / ``get_textures_paths_and_indices`` /
  ``assign_material_texture_indices`` (SceneParser.cpp:278-347, 409-455) and
  ``ThreadFunctions::load_scene_texture`` (ThreadFunctions.cpp:30-97): per material, in the
  order base colour, emission, roughness-metallic, specular, coat, sheen, transmission,
  normal map, each decoded (mpt/image.py: PNG) with the channel count the reference asks
  stb_image for, and a constant emissive texture folded into the material's emission
  (``CONSTANT_EMISSIVE_TEXTURE``);
* the camera of ``SceneParser::parse_camera`` (SceneParser.cpp:222-276) and
  ``Camera::to_hiprt`` / ``get_view_matrix`` (Scene/Camera.cpp:9-45), including the
  reference's '+0.425 rad' vertical-FOV term and its matrix conventions.

ASSIMP's own conversions (glTF yfov -> mHorizontalFOV = yfov * aspect, default
material values, the glTF2 importer's texture types: baseColorTexture -> BASE_COLOR,
metallicRoughnessTexture -> METALNESS and DIFFUSE_ROUGHNESS with one path,
KHR_materials_specular.specularTexture -> SPECULAR, clearcoatTexture -> CLEARCOAT,
sheenColorTexture -> SHEEN, transmissionTexture -> TRANSMISSION, its V flip of texture
coordinates, v -> 1 - v) are assumptions of this restatement; they only
decide which scene is rendered, not the renderer's parity, since the oracle and the
HIP path consume the same arrays.  One deliberate superset: embedded images (data URIs,
bufferViews, .glb) are decoded; the reference hands ASSIMP's '*N' embedded-texture names to
stb_image as file paths, which fails and leaves an empty texture.
"""
import base64
import json
import math
import os
import struct
import warnings

import numpy as np

from . import abi

_COMP = {5120: np.int8, 5121: np.uint8, 5122: np.int16, 5123: np.uint16, 5125: np.uint32, 5126: np.float32}
_NCOMP = {"SCALAR": 1, "VEC2": 2, "VEC3": 3, "VEC4": 4, "MAT4": 16}

DATA_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "data")


class SceneData:
    """Flat arrays + materials, i.e. what ``mpt_upload_scene`` receives."""

    def __init__(self):
        self.triangle_indices = None  # int32 [T*3]
        self.vertices = None          # float32 [V,3]
        self.normals = None           # float32 [V,3]
        self.has_normals = None       # uint8 [V]
        self.texcoords = None         # float32 [V,2]
        self.material_indices = None  # int32 [T]
        self.materials = []           # list[abi.Material]
        self.emissive = None          # int32 [E]
        self.textures = []            # list of uint8 [h, w, 4]
        self.camera_info = None       # dict for make_camera
        self.name = ""

    @property
    def num_triangles(self):
        return len(self.material_indices)

    def finalize(self):
        self.emissive = np.array([i for i, m in enumerate(self.material_indices)
                                  if _is_emissive(self.materials[m])], np.int32)
        return self

    def to_abi(self):
        """Builds an abi.Scene.  The arrays it points to are kept alive by the returned
        struct itself (`_keep`), so every caller that holds the struct -- e.g. a CPU oracle
        that reads the scene in place -- keeps its own copy valid, whatever later calls do."""
        C = abi.C
        s = abi.Scene()
        keep = []
        s._keep = keep
        self._keep = keep

        def ptr(a, t):
            a = np.ascontiguousarray(a)
            keep.append(a)
            return a.ctypes.data_as(C.POINTER(t))

        s.triangle_indices = ptr(self.triangle_indices.astype(np.int32), abi.i32)
        s.num_triangles = self.num_triangles
        s.vertices = ptr(self.vertices.astype(np.float32), abi.f32)
        s.vertex_normals = ptr(self.normals.astype(np.float32), abi.f32)
        s.has_vertex_normals = ptr(self.has_normals.astype(np.uint8), C.c_uint8)
        s.texcoords = ptr(self.texcoords.astype(np.float32), abi.f32)
        s.num_vertices = len(self.vertices)
        s.material_indices = ptr(self.material_indices.astype(np.int32), abi.i32)
        mats = (abi.Material * len(self.materials))(*self.materials)
        keep.append(mats)
        s.materials = C.cast(mats, C.POINTER(abi.Material))
        s.num_materials = len(self.materials)
        s.emissive_triangle_indices = ptr(self.emissive.astype(np.int32) if len(self.emissive) else np.zeros(1, np.int32), abi.i32)
        s.num_emissive_triangles = len(self.emissive)
        s.num_textures = len(self.textures)
        if self.textures:
            texs = [np.ascontiguousarray(t, dtype=np.uint8) for t in self.textures]
            keep.extend(texs)
            arr = (C.POINTER(C.c_uint8) * len(texs))(*[t.ctypes.data_as(C.POINTER(C.c_uint8)) for t in texs])
            keep.append(arr)
            s.texture_data = C.cast(arr, C.POINTER(C.POINTER(C.c_uint8)))
            dims = np.array([[t.shape[1], t.shape[0]] for t in texs], np.int32).ravel()
            s.texture_dims = ptr(dims, abi.i32)
        return s


def _is_emissive(m):
    """SimplifiedRendererMaterial::is_emissive (Material.h:35-41) && !emissive_texture_used."""
    f = np.float32
    e, k = m.emission, f(m.emission_strength)
    nz = lambda v: not (f(v) * k < f(1e-10) and f(v) * k > f(-1e-10))
    return (nz(e.r) or nz(e.g) or nz(e.b) or m.emissive_texture_used) and not m.emissive_texture_used


def _quat_to_mat(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]], np.float64)


def _node_matrix(n):
    if "matrix" in n:
        return np.array(n["matrix"], np.float64).reshape(4, 4).T
    m = np.eye(4)
    t = n.get("translation", [0, 0, 0])
    r = n.get("rotation", [0, 0, 0, 1])
    s = n.get("scale", [1, 1, 1])
    m[:3, :3] = _quat_to_mat(r) @ np.diag(s)
    m[:3, 3] = t
    return m


def _view(g, bins, view_idx, byte_offset, dt, cnt, n):
    """cnt elements of n components of dtype dt from a bufferView (honouring byteStride)."""
    bv = g["bufferViews"][view_idx]
    off = bv.get("byteOffset", 0) + byte_offset
    stride = bv.get("byteStride", 0)
    buf = bins[bv["buffer"]]
    if stride and stride != n * dt.itemsize:
        return np.array(np.ndarray((cnt, n), dt, buf, off, (stride, dt.itemsize)))
    return np.frombuffer(buf, dt, cnt * n, off).reshape(cnt, n).copy()


# glTF 2.0 §3.11 (accessor.normalized): integer components as fractions of their range
_NORM = {np.dtype(np.uint8): 255.0, np.dtype(np.int8): 127.0, np.dtype(np.uint16): 65535.0, np.dtype(np.int16): 32767.0}


def _accessor(g, bins, idx):
    """An accessor as [count, components]: its bufferView data (zeros without one), the sparse
    substitutions applied (glTF 2.0 §3.6.2.3), and, for a normalized integer accessor
    (KHR_mesh_quantization positions / normals / texcoords), the components mapped to [0, 1] or
    [-1, 1] (§3.11: c / 255, max(c / 127, -1), c / 65535, max(c / 32767, -1)) as float32."""
    a = g["accessors"][idx]
    dt = np.dtype(_COMP[a["componentType"]])
    n = _NCOMP[a["type"]]
    cnt = a["count"]
    if "bufferView" in a:
        arr = _view(g, bins, a["bufferView"], a.get("byteOffset", 0), dt, cnt, n)
    else:
        arr = np.zeros((cnt, n), dt)
    sp = a.get("sparse")
    if sp:
        k = sp["count"]
        ii, vv = sp["indices"], sp["values"]
        where = _view(g, bins, ii["bufferView"], ii.get("byteOffset", 0), np.dtype(_COMP[ii["componentType"]]), k, 1).ravel()
        arr[where.astype(np.int64)] = _view(g, bins, vv["bufferView"], vv.get("byteOffset", 0), dt, k, n)
    if a.get("normalized") and dt in _NORM:
        f = arr.astype(np.float32) / np.float32(_NORM[dt])
        return np.maximum(f, np.float32(-1.0)) if dt.kind == "i" else f
    return arr


def _triangles(mode, idx):
    """A primitive's index list as triangles: TRIANGLES as they are, TRIANGLE_STRIP with every
    other triangle's first two vertices swapped (one winding) and TRIANGLE_FAN around its first
    vertex -- what ASSIMP's glTF 2 importer builds before the reference reads the faces
    (SceneParser.cpp:151-165 takes three indices per face; glTF 2.0 §3.7.2.1)."""
    n = len(idx)
    if mode == 4:
        return idx[: n - n % 3].reshape(-1, 3)
    if n < 3:
        return np.zeros((0, 3), np.int64)
    i = np.arange(n - 2)
    if mode == 5:
        odd = (i % 2) == 1
        a = np.where(odd, idx[i + 1], idx[i])
        b = np.where(odd, idx[i], idx[i + 1])
        return np.stack([a, b, idx[i + 2]], 1)
    return np.stack([np.full(n - 2, idx[0]), idx[i + 1], idx[i + 2]], 1)   # mode 6: fan


def _material_from_gltf(gm, tex=None):
    """SceneParser::read_material_properties on ASSIMP's glTF2 material keys.  tex: the
    material's texture indices (assigned before the properties are read, SceneParser.cpp:73-80,
    so a material with an emission texture keeps the default black emission)."""
    m = abi.Material.default()
    for k, v in (tex or {}).items():
        setattr(m, k, v)
    pbr = gm.get("pbrMetallicRoughness", {})
    bc = pbr.get("baseColorFactor", [1.0, 1.0, 1.0, 1.0])
    m.base_color = abi.Color(*bc[:3])
    ext = gm.get("extensions", {})
    if m.emission_texture_index == -1:
        m.emission = abi.Color(*gm.get("emissiveFactor", [0.0, 0.0, 0.0]))
    if "KHR_materials_emissive_strength" in ext:
        m.emission_strength = ext["KHR_materials_emissive_strength"].get("emissiveStrength", 1.0)
    m.metallic = pbr.get("metallicFactor", 1.0)
    m.roughness = pbr.get("roughnessFactor", 1.0)
    if "KHR_materials_anisotropy" in ext:
        m.anisotropy = ext["KHR_materials_anisotropy"].get("anisotropyStrength", 0.0)
    if "KHR_materials_sheen" in ext:
        sh = ext["KHR_materials_sheen"]
        m.sheen_color = abi.Color(*sh.get("sheenColorFactor", [0.0, 0.0, 0.0]))
        m.sheen_roughness = sh.get("sheenRoughnessFactor", 0.0)
        m.sheen = 1.0
    if "KHR_materials_specular" in ext:
        m.specular = ext["KHR_materials_specular"].get("specularFactor", 1.0)
        m.specular_tint = 1.0
        m.specular_color = abi.Color(1.0)
    if "KHR_materials_clearcoat" in ext:
        cc = ext["KHR_materials_clearcoat"]
        m.coat = cc.get("clearcoatFactor", 0.0)
        m.coat_roughness = cc.get("clearcoatRoughnessFactor", 0.0)
    if "KHR_materials_ior" in ext:
        m.ior = ext["KHR_materials_ior"].get("ior", 1.5)
    if "KHR_materials_transmission" in ext:
        m.specular_transmission = ext["KHR_materials_transmission"].get("transmissionFactor", 0.0)
    if "KHR_materials_volume" in ext:
        v = ext["KHR_materials_volume"]
        if "attenuationColor" in v:
            m.absorption_color = abi.Color(*v["attenuationColor"])
        if "attenuationDistance" in v:
            m.absorption_at_distance = v["attenuationDistance"]
    if gm.get("alphaMode", "OPAQUE") != "OPAQUE":
        m.alpha_opacity = bc[3]
    m.make_safe()
    m.precompute_properties()
    return m


# Texture slots in the order SceneParser::get_textures_paths_and_indices reads them
# (SceneParser.cpp:409-455), with the glTF texture that ASSIMP's glTF2 importer files under
# that aiTextureType and the channel count load_scene_texture asks stb_image for
# (ThreadFunctions.cpp:44-83; roughness + metallic share one path -> the packed 3-channel slot).
_TEX_SLOTS = [
    ("base_color_texture_index", lambda gm, e: gm.get("pbrMetallicRoughness", {}).get("baseColorTexture"), 4),
    ("emission_texture_index", lambda gm, e: gm.get("emissiveTexture"), 4),
    ("roughness_metallic_texture_index", lambda gm, e: gm.get("pbrMetallicRoughness", {}).get("metallicRoughnessTexture"), 3),
    ("specular_texture_index", lambda gm, e: e.get("KHR_materials_specular", {}).get("specularTexture"), 1),
    ("coat_texture_index", lambda gm, e: e.get("KHR_materials_clearcoat", {}).get("clearcoatTexture"), 1),
    ("sheen_texture_index", lambda gm, e: e.get("KHR_materials_sheen", {}).get("sheenColorTexture"), 1),
    ("specular_transmission_texture_index", lambda gm, e: e.get("KHR_materials_transmission", {}).get("transmissionTexture"), 1),
    ("normal_map_texture_index", lambda gm, e: gm.get("normalTexture"), 4),
]
CONSTANT_EMISSIVE_TEXTURE = -2   # RendererMaterial::CONSTANT_EMISSIVE_TEXTURE (Material.h:236-237)


def _read_glb(path):
    """Binary glTF: the JSON chunk and the BIN chunk (buffer 0)."""
    with open(path, "rb") as f:
        data = f.read()
    magic, version, length = struct.unpack_from("<4sII", data, 0)
    if magic != b"glTF" or version != 2:
        raise ValueError(f"{path}: not a glTF 2 binary")
    pos, g, binchunk = 12, None, None
    while pos + 8 <= min(length, len(data)):
        n, kind = struct.unpack_from("<I4s", data, pos)
        body = data[pos + 8:pos + 8 + n]
        if kind == b"JSON":
            g = json.loads(body.decode("utf-8"))
        elif kind == b"BIN\x00":
            binchunk = body
        pos += 8 + n
    if g is None:
        raise ValueError(f"{path}: GLB without a JSON chunk")
    return g, binchunk


def _uri_bytes(base, uri):
    if uri.startswith("data:"):
        return base64.b64decode(uri.split(",", 1)[1])
    # SceneParser::normalize_texture_paths (SceneParser.cpp:476-494): '%20' -> ' '
    with open(os.path.join(base, uri.replace("%20", " ")), "rb") as f:
        return f.read()


def _image_bytes(g, bins, base, image_index):
    im = g["images"][image_index]
    if "uri" in im:
        return _uri_bytes(base, im["uri"])
    bv = g["bufferViews"][im["bufferView"]]
    off = bv.get("byteOffset", 0)
    return bytes(bins[bv["buffer"]][off:off + bv["byteLength"]])


def _load_textures(g, bins, base, materials_json):
    """SceneParser::prepare_textures + assign_material_texture_indices + the texture-loading
    threads (ThreadFunctions::load_scene_texture): per material, its textures in slot order
    (global index = the material's offset + its local index), decoded with the slot's channel
    count, an emission texture of constant colour (stb values within 5 of the first texel,
    Image8Bit::is_constant_color(5), Image.cpp:250-271) folded into the material (emission =
    its texel sampled at uv (0, 0), i.e. the bottom-left texel / 255, Image.cpp:161-193) and
    replaced by CONSTANT_EMISSIVE_TEXTURE.  Returns (per-material {slot: index},
    per-material constant emission or None, textures as RGBA8, per-material texture count)."""
    from . import image
    tex_idx, const_em, textures, per_mat = [], [], [], []
    cache = {}
    for gm in materials_json:
        ext = gm.get("extensions", {})
        slots, em = {}, None
        n0 = len(textures)
        for slot, get, channels in _TEX_SLOTS:
            info = get(gm, ext)
            if not info or "index" not in info:
                continue
            src = g["textures"][info["index"]].get("source")
            if src is None:
                continue
            key = (src, channels)
            if key not in cache:
                try:
                    cache[key] = image.read_image(_image_bytes(g, bins, base, src), channels)
                except (OSError, ValueError) as e:
                    raise ValueError(f"texture {g['images'][src].get('uri', src)!r} ({slot}): {e}") from None
            img = cache[key]
            if slot == "emission_texture_index":
                first = img[0, 0].astype(np.int32)
                if np.all(np.abs(img.astype(np.int32) - first) <= 5):
                    slots[slot] = CONSTANT_EMISSIVE_TEXTURE
                    em = img[-1, 0, :3].astype(np.float32) / np.float32(255.0)
                    textures.append(np.array([[[0, 0, 0, 255]]], np.uint8))   # the slot stays, never read
                    continue
            slots[slot] = len(textures)
            textures.append(image.to_rgba8(img))
        tex_idx.append(slots)
        const_em.append(em)
        per_mat.append(len(textures) - n0)
    return tex_idx, const_em, textures, per_mat


def load_gltf(path, aspect_override=None):
    """Loads a .gltf (+ .bin, + textures) or a .glb into SceneData."""
    base = os.path.dirname(path)
    bins = []
    if path.endswith(".glb"):
        g, binchunk = _read_glb(path)
        for k, b in enumerate(g.get("buffers", [])):
            bins.append(binchunk if "uri" not in b and k == 0 else _uri_bytes(base, b["uri"]))
    else:
        with open(path) as f:
            g = json.load(f)
        for b in g.get("buffers", []):
            bins.append(_uri_bytes(base, b["uri"]))

    # world transforms
    world = {}

    def visit(ni, parent):
        n = g["nodes"][ni]
        m = parent @ _node_matrix(n)
        world[ni] = m
        for c in n.get("children", []):
            visit(c, m)

    scene_idx = g.get("scene", 0)
    roots = g["scenes"][scene_idx]["nodes"] if "scenes" in g else list(range(len(g["nodes"])))
    for r in roots:
        visit(r, np.eye(4))

    materials_json = g.get("materials", [])
    n_mat = len(materials_json)
    # instances: (material, positions, normals or None, texcoords or None, indices)
    inst = []
    need_default = False
    for ni, n in enumerate(g["nodes"]):
        if "mesh" not in n or ni not in world:
            continue
        M = world[ni]
        R = M[:3, :3]
        RIT = np.linalg.inv(R).T
        for prim in g["meshes"][n["mesh"]]["primitives"]:
            mode = prim.get("mode", 4)
            if mode not in (4, 5, 6):
                # points / lines have no surface: ASSIMP hands them over as 1- or 2-index faces,
                # which the reference's three-index face loop (SceneParser.cpp:151-165) reads past
                warnings.warn(f"{os.path.basename(path)}: mesh {n['mesh']}: primitive mode {mode} (points / lines) skipped")
                continue
            att = prim["attributes"]
            pos = _accessor(g, bins, att["POSITION"]).astype(np.float64)
            pos = (pos @ R.T + M[:3, 3]).astype(np.float32)
            nrm = None
            if "NORMAL" in att:
                nrm = _accessor(g, bins, att["NORMAL"]).astype(np.float64) @ RIT.T
                nrm /= np.maximum(np.linalg.norm(nrm, axis=1, keepdims=True), 1e-30)
                nrm = nrm.astype(np.float32)
            uv = _accessor(g, bins, att["TEXCOORD_0"]).astype(np.float32) if "TEXCOORD_0" in att else None
            if "indices" in prim:
                idx = _accessor(g, bins, prim["indices"]).astype(np.int64).ravel()
            else:
                idx = np.arange(len(pos), dtype=np.int64)
            mi = prim.get("material")
            if mi is None:
                need_default = True
                mi = n_mat
            inst.append((mi, pos, nrm, uv, _triangles(mode, idx)))

    total_mats = n_mat + (1 if need_default else 0)
    tex_idx, const_em, textures, tex_count = _load_textures(g, bins, base, materials_json)
    mats = [_material_from_gltf(gm, t) for gm, t in zip(materials_json, tex_idx)]
    for m, em in zip(mats, const_em):
        if em is not None:      # Material::set_emission after the texture thread (ThreadFunctions.cpp:87-93)
            m.emission = abi.Color(*[float(x) for x in em])
    if need_default:
        mats.append(_material_from_gltf({}))
        tex_count.append(0)

    sd = SceneData()
    sd.name = os.path.splitext(os.path.basename(path))[0]
    tri, verts, nrms, hasn, uvs, mids = [], [], [], [], [], []
    voff = 0
    # PreTransformVertices: output meshes ordered by material index
    for mi in range(total_mats):
        for (m, pos, nrm, uv, idx) in inst:
            if m != mi:
                continue
            tri.append(idx + voff)
            verts.append(pos)
            nrms.append(nrm if nrm is not None else np.zeros_like(pos))
            hasn.append(np.full(len(pos), 1 if nrm is not None else 0, np.uint8))
            # texcoords only kept when the material has textures (SceneParser.cpp:136-141),
            # V flipped by ASSIMP's glTF2 importer
            if uv is not None and tex_count[mi] > 0:
                uvs.append(np.stack([uv[:, 0], np.float32(1.0) - uv[:, 1]], 1).astype(np.float32))
            else:
                uvs.append(np.zeros((len(pos), 2), np.float32))
            mids.append(np.full(len(idx), mi, np.int32))
            voff += len(pos)
    sd.triangle_indices = np.concatenate(tri).astype(np.int32).ravel()
    sd.vertices = np.concatenate(verts).astype(np.float32)
    sd.normals = np.concatenate(nrms).astype(np.float32)
    sd.has_normals = np.concatenate(hasn)
    sd.texcoords = np.concatenate(uvs)
    sd.material_indices = np.concatenate(mids)
    sd.materials = mats
    sd.textures = textures

    cams = [(ni, n) for ni, n in enumerate(g["nodes"]) if "camera" in n and ni in world]
    if cams:
        ni, n = cams[0]
        cam = g["cameras"][n["camera"]]
        p = cam.get("perspective", {})
        aspect = p.get("aspectRatio", 16.0 / 9.0)
        M = world[ni]
        sd.camera_info = dict(position=M[:3, 3].copy(), lookat=M[:3, :3] @ np.array([0.0, 0.0, -1.0]),
                              up=M[:3, :3] @ np.array([0.0, 1.0, 0.0]),
                              hfov=p.get("yfov", 0.7) * (aspect if aspect != 0 else 1.0),
                              aspect=aspect, znear=p.get("znear", 0.1), zfar=p.get("zfar", 100.0))
    return sd.finalize()


def load_scene(name):
    """Loads a scene shipped in data/scenes (copied from the reference's data/GLTFs)."""
    p = os.path.join(DATA_DIR, "scenes", name + ".gltf")
    return load_gltf(p if os.path.exists(p) else p[:-5] + ".glb")


# ----------------------------------------------------------------------------------
# Camera: SceneParser::parse_camera + Camera::to_hiprt (float32, glm conventions)
# ----------------------------------------------------------------------------------
def _lookat(eye, center, up):
    f = center - eye
    f = f / np.linalg.norm(f)
    s = np.cross(f, up)
    s = s / np.linalg.norm(s)
    u = np.cross(s, f)
    V = np.eye(4)
    V[0, :3], V[1, :3], V[2, :3] = s, u, -f
    V[0, 3], V[1, 3], V[2, 3] = -s @ eye, -u @ eye, f @ eye
    return V


def _perspective(fovy, aspect, n, f):
    t = math.tan(fovy / 2.0)
    P = np.zeros((4, 4))
    P[0, 0] = 1.0 / (aspect * t)
    P[1, 1] = 1.0 / t
    P[2, 2] = -(f + n) / (f - n)
    P[3, 2] = -1.0
    P[2, 3] = -(2.0 * f * n) / (f - n)
    return P


def make_camera(camera_info, width, height, jitter=True):
    """Returns abi.Camera for the scene camera at the given resolution.

    parse_camera: inverse(lookAt(position, lookat, up)) decomposed into translation +
    rotation, vertical_fov = 2 atan(tan(hfov/2) * aspect) + 0.425 with aspect = W/H
    (main.cpp:43), glm::perspective.  to_hiprt stores, row-major, the inverse of the
    (transposed-for-row-major) view matrix and glm's column-major inverse projection
    reinterpreted as row-major (Camera.cpp:9-26, 37-45).
    """
    if camera_info is None:
        camera_info = dict(position=np.zeros(3), lookat=np.array([0.0, 0.0, -1.0]), up=np.array([0.0, 1.0, 0.0]),
                           hfov=40.0 / 180 * math.pi, aspect=1280 / 720, znear=0.1, zfar=100.0)
    aspect = width / height
    eye = np.asarray(camera_info["position"], np.float64)
    V = _lookat(eye, np.asarray(camera_info["lookat"], np.float64), np.asarray(camera_info["up"], np.float64))
    cam_to_world = np.linalg.inv(V)
    vfov = 2.0 * math.atan(math.tan(camera_info["hfov"] * 0.5) * aspect) + 0.425
    P = _perspective(vfov, aspect, camera_info["znear"], camera_info["zfar"])
    # row-major view (world->view) and its inverse
    view = np.linalg.inv(cam_to_world)
    inv_view_rowmajor = np.linalg.inv(view)
    # glm stores P column-major; inverse(P) reinterpreted row-major == inverse(P)^T
    inv_proj_reinterpreted = np.linalg.inv(P).T
    # Camera.cpp:20-21: glm's view_matrix (already the transposed world->view matrix,
    # Camera.cpp:50) times projection_matrix, stored column-major and reinterpreted row-major:
    # (view^T P)^T = P^T view.  With the transposed inverse projection of the camera rays this
    # reprojects a first hit onto its own pixel (Utils.h:426-437, restir_reproject).
    view_proj = P.T @ view
    cam = abi.Camera()
    for i in range(4):
        for j in range(4):
            cam.inverse_view.m[i][j] = float(np.float32(inv_view_rowmajor[i, j]))
            cam.inverse_projection.m[i][j] = float(np.float32(inv_proj_reinterpreted[i, j]))
            cam.view_projection.m[i][j] = float(np.float32(view_proj[i, j]))
    cam.do_jittering = bool(jitter)
    return cam


# ----------------------------------------------------------------------------------
# LUTs
# ----------------------------------------------------------------------------------
def load_luts():
    """The reference's energy-compensation LUTs (see tools/make_data.py)."""
    d = np.load(os.path.join(DATA_DIR, "luts.npz"))
    return {k: np.ascontiguousarray(d[k], np.float32) for k in d.files}


def luts_to_abi(luts):
    C = abi.C
    L = abi.Luts()
    keep = []

    def p(a):
        a = np.ascontiguousarray(a, np.float32)
        keep.append(a)
        return a.ctypes.data_as(C.POINTER(abi.f32))

    L.ggx_conductor_ess = p(luts["ggx_conductor"])
    L.glossy_dielectric_ess = p(luts["glossy_dielectric"])
    L.ggx_glass_ess = p(luts["ggx_glass"])
    L.ggx_glass_inverse_ess = p(luts["ggx_glass_inverse"])
    L.ggx_thin_glass_ess = p(luts["ggx_thin_glass"])
    L.sheen_ltc_params = p(luts["sheen_ltc"])
    L._keep = keep
    return L


# ----------------------------------------------------------------------------------
# Frame / seed schedule
# ----------------------------------------------------------------------------------
def cpu_seed_schedule(nframes, first_sample=0):
    """(sample_number, random_seed) per frame as CPURenderer::render does
    (Renderer/CPURenderer.cpp:90, 271-287): random_seed starts at 42 and after each
    frame becomes m_rng.xorshift32() with m_rng seeded 42."""
    out = []
    seed = 42
    rng = 42
    for f in range(nframes):
        out.append((first_sample + f, seed))
        x = rng
        x ^= (x << 13) & 0xFFFFFFFF
        x ^= x >> 17
        x ^= (x << 5) & 0xFFFFFFFF
        rng = x & 0xFFFFFFFF
        seed = rng
    return out


def _xorshift32(x):
    x ^= (x << 13) & 0xFFFFFFFF
    x ^= x >> 17
    x ^= (x << 5) & 0xFFFFFFFF
    return x & 0xFFFFFFFF


def gpu_seed_schedule(nframes, restir_spatial_passes=None, first_sample=0, fused=True, temporal=True, spatial=True,
                      samples_per_frame=1, presampling=True):
    """Per-sample seeds as the reference's GPU front-end draws them from m_rng (seeded 42,
    GPURenderer.cpp:50): GPURenderer::update once per displayed frame (update_render_data,
    GPURenderer.cpp:980-983; its value is overwritten before any launch), then per sample
    of GPURenderer::render (GPURenderer.cpp:424-486) the camera launch, the ReSTIR DI passes
    (ReSTIRDIRenderPass.cpp:233-264, 298-431) and the path-tracing launch.  ReSTIR draws:
    presampling, initial candidates, then fused: temporal seed + permutation bits
    (configure_temporal_pass_for_fused_spatiotemporal) and the fused kernel's seed
    (configure_spatial_pass_for_fused_spatiotemporal(0)), one per extra spatial pass;
    unfused: temporal seed + permutation bits if the temporal pass runs, one per spatial
    pass.  Returns dicts with sample_number, camera_random_seed, restir_di_seeds (the
    MptFrame layout, include/mpt.h) and random_seed (path tracing)."""
    st = [42]

    def draw():
        st[0] = _xorshift32(st[0])
        return st[0]

    out = []
    for f in range(nframes):
        if f % samples_per_frame == 0:
            draw()                                   # GPURenderer::update
        cam = draw()
        seeds = [0] * 8
        if restir_spatial_passes is not None:
            if presampling:                          # launch_presampling_lights_pass only when enabled
                seeds[0] = draw()
            seeds[1] = draw()
            if fused:
                draw()                               # temporal seed, overwritten before the launch
                seeds[3] = draw()
                seeds[2] = draw()
                for p in range(1, restir_spatial_passes):
                    seeds[4 + p] = draw()
            else:
                if temporal:
                    seeds[2] = draw()
                    seeds[3] = draw()
                if spatial:
                    for p in range(restir_spatial_passes):
                        seeds[4 + p] = draw()
        rs = draw()
        out.append({"sample_number": first_sample + f, "camera_random_seed": cam,
                    "restir_di_seeds": seeds, "random_seed": rs})
    return out


def make_frame(camera, width, height, options=None, settings=None, world=None, flags=None,
               sample_number=0, random_seed=42, band=(1, 0, 1), camera_random_seed=0, restir_di_seeds=None):
    fr = abi.Frame()
    fr.render_settings = settings if settings is not None else parity_settings()
    fr.render_settings.sample_number = sample_number
    # GPURenderer::render clears need_to_reset after the first launch (GPURenderer.cpp:446)
    fr.render_settings.need_to_reset = sample_number == 0
    fr.world_settings = world if world is not None else abi.WorldSettings.default()
    fr.current_camera = camera
    fr.prev_camera = camera
    fr.options = options if options is not None else abi.KernelOptions.default()
    fr.bsdf_flags = flags if flags is not None else abi.BSDFFlags.default()
    fr.random_seed = random_seed
    fr.res_x, fr.res_y = width, height
    fr.band_height, fr.band_index, fr.band_count = band
    fr.camera_random_seed = camera_random_seed
    if restir_di_seeds is not None:
        for i, v in enumerate(list(restir_di_seeds)[:8]):
            fr.restir_di_seeds[i] = v
        # ReSTIRDIRenderPass::configure_temporal_pass_for_fused_spatiotemporal draws the
        # permutation-sampling bits right after the pass seed (ReSTIRDIRenderPass.cpp:416)
        fr.render_settings.restir_di_settings.permutation_sampling_random_bits = abi.C.c_int32(restir_di_seeds[3]).value
    return fr


def parity_settings(nb_bounces=3):
    """Reference defaults with the parity pins of BASELINE.md §2: adaptive sampling
    off, alpha testing off (scenes without alpha textures), freeze_random off."""
    s = abi.RenderSettings.default()
    s.enable_adaptive_sampling = False
    s.enable_pixel_stop_noise_threshold = False
    s.stop_pixel_noise_threshold = 0.0
    s.do_alpha_testing = False
    s.nb_bounces = nb_bounces
    return s


# ----------------------------------------------------------------------------------
# Synthetic assets (SURVEY.md §8d stand-ins for inputs not shipped in the container)
# ----------------------------------------------------------------------------------
def procedural_sky(width=2048, height=1024, seed=7, sun_dir=(0.3, 0.8, 0.5), sun_radiance=2000.0):
    """Seeded HDR sky, RGBA32F [height, width, 4] in the reference's equirectangular
    layout (row 0 = bottom after the loader's vertical flip): a vertical gradient, a
    small bright sun lobe and low-amplitude seeded noise, so the alias table is far
    from uniform (stand-in for the Bistro HDR)."""
    rng = np.random.default_rng(seed)
    v = (np.arange(height) + 0.5) / height           # 0 bottom .. 1 top
    u = (np.arange(width) + 0.5) / width
    theta = (1.0 - v) * math.pi                       # polar angle from +Y
    phi = u * 2.0 * math.pi
    st = np.sin(theta)[:, None]
    d = np.stack([st * np.cos(phi)[None, :], np.repeat(np.cos(theta)[:, None], width, 1),
                  st * np.sin(phi)[None, :]], -1)
    up = np.clip(d[..., 1], -1.0, 1.0)
    horizon = np.array([0.9, 0.85, 0.8])
    zenith = np.array([0.25, 0.45, 0.9])
    ground = np.array([0.18, 0.16, 0.14])
    t = np.clip(up, 0.0, 1.0)[..., None]
    col = np.where(up[..., None] >= 0.0, horizon * (1 - t) + zenith * t, ground)
    s = np.asarray(sun_dir, np.float64)
    s = s / np.linalg.norm(s)
    cosang = np.clip(d @ s, -1.0, 1.0)
    sun = np.exp((cosang - 1.0) * 4000.0) * sun_radiance
    col = col + sun[..., None] * np.array([1.0, 0.95, 0.85])
    col = col * (1.0 + 0.05 * rng.standard_normal((height, width, 1)))
    rgba = np.concatenate([np.maximum(col, 0.0), np.ones((height, width, 1))], -1)
    return np.ascontiguousarray(rgba, np.float32)


def envmap_world(intensity=1.0):
    w = abi.WorldSettings.default()
    w.ambient_light_type = abi.AMBIENT_ENVMAP
    w.envmap_intensity = intensity
    return w
