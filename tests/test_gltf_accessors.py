"""glTF geometry ingestion: the primitive modes and accessor forms the reference
gets from ASSIMP's glTF 2 importer (SceneParser.cpp:25 reads with aiProcess_Triangulate |
aiProcess_PreTransformVertices, then takes three indices per face, SceneParser.cpp:151-165).

* TRIANGLE_STRIP / TRIANGLE_FAN become triangle lists (strip: every other triangle's first two
  vertices swapped so that all keep one winding; fan: around the first vertex);
* points / lines are skipped with a warning (they have no surface);
* sparse accessors substitute their values (also over an accessor without a bufferView = zeros);
* normalized integer accessors (KHR_mesh_quantization) are dequantised per glTF 2.0 §3.11.
CPU only: the scene loader is host code."""
import json
import struct

import numpy as np
import pytest

from mpt import scene


def _write(tmp_path, prims, accessors, blobs, extra_nodes=()):
    """A one-mesh glTF: prims = primitive dicts; accessors reference bufferViews 0..len(blobs)-1."""
    data = b""
    views = []
    for b in blobs:
        while len(data) % 4:
            data += b"\0"
        views.append({"buffer": 0, "byteOffset": len(data), "byteLength": len(b)})
        data += b
    (tmp_path / "m.bin").write_bytes(data)
    g = {"asset": {"version": "2.0"}, "buffers": [{"uri": "m.bin", "byteLength": len(data)}], "bufferViews": views,
         "accessors": accessors, "meshes": [{"primitives": prims}], "materials": [{}],
         "nodes": [{"mesh": 0}, *extra_nodes], "scenes": [{"nodes": list(range(1 + len(extra_nodes)))}], "scene": 0}
    p = tmp_path / "m.gltf"
    p.write_text(json.dumps(g))
    return str(p)


def _f32(a):
    return np.asarray(a, np.float32).tobytes()


POS = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0], [1, 1, 0], [0, 2, 0], [1, 2, 0]], np.float32)


def _tris(sd):
    V = np.asarray(sd.vertices).reshape(-1, 3)
    return V[np.asarray(sd.triangle_indices).reshape(-1, 3)]


def test_strip_and_fan_become_triangle_lists(tmp_path):
    acc = [{"bufferView": 0, "componentType": 5126, "count": 6, "type": "VEC3", "min": [0, 0, 0], "max": [1, 2, 0]},
           {"bufferView": 1, "componentType": 5123, "count": 6, "type": "SCALAR"}]
    idx = np.arange(6, dtype=np.uint16).tobytes()
    strip = scene.load_gltf(_write(tmp_path, [{"attributes": {"POSITION": 0}, "indices": 1, "mode": 5}], acc, [_f32(POS), idx]))
    want = POS[[[0, 1, 2], [2, 1, 3], [2, 3, 4], [4, 3, 5]]]
    assert np.array_equal(_tris(strip), want)
    # one winding: every triangle's geometric normal points the same way
    nz = [np.cross(t[1] - t[0], t[2] - t[0])[2] for t in _tris(strip)]
    assert all(z > 0 for z in nz) or all(z < 0 for z in nz)
    fan = scene.load_gltf(_write(tmp_path, [{"attributes": {"POSITION": 0}, "mode": 6}], acc[:1], [_f32(POS)]))
    assert np.array_equal(_tris(fan), POS[[[0, 1, 2], [0, 2, 3], [0, 3, 4], [0, 4, 5]]])
    assert len(fan.material_indices) == 4


def test_points_and_lines_are_skipped_with_a_warning(tmp_path):
    acc = [{"bufferView": 0, "componentType": 5126, "count": 6, "type": "VEC3"}]
    prims = [{"attributes": {"POSITION": 0}, "mode": 4}, {"attributes": {"POSITION": 0}, "mode": 1}]
    with pytest.warns(UserWarning, match="mode 1"):
        sd = scene.load_gltf(_write(tmp_path, prims, acc, [_f32(POS)]))
    assert sd.num_triangles == 2


def test_sparse_accessor_substitutes_values(tmp_path):
    moved = POS.copy()
    moved[[1, 4]] = [[5, 0, 0], [0, 7, 0]]
    acc = [{"bufferView": 0, "componentType": 5126, "count": 6, "type": "VEC3",
            "sparse": {"count": 2, "indices": {"bufferView": 1, "componentType": 5121},
                       "values": {"bufferView": 2}}},
           # no bufferView: zeros, then the sparse values
           {"componentType": 5126, "count": 6, "type": "VEC3",
            "sparse": {"count": 2, "indices": {"bufferView": 1, "componentType": 5121}, "values": {"bufferView": 2}}}]
    blobs = [_f32(POS), bytes([1, 4]), _f32([[5, 0, 0], [0, 7, 0]])]
    sd = scene.load_gltf(_write(tmp_path, [{"attributes": {"POSITION": 0}}], acc, blobs))
    assert np.array_equal(np.asarray(sd.vertices).reshape(-1, 3), moved)
    sd0 = scene.load_gltf(_write(tmp_path, [{"attributes": {"POSITION": 1}}], acc, blobs))
    z = np.zeros_like(POS)
    z[[1, 4]] = [[5, 0, 0], [0, 7, 0]]
    assert np.array_equal(np.asarray(sd0.vertices).reshape(-1, 3), z)


def test_normalized_integer_accessors_are_dequantised(tmp_path):
    q = np.array([[0, 0, 0], [32767, 0, 0], [0, 32767, 0], [-32768, -16384, 1]], np.int16)
    nq = np.array([[0, 0, 127, 0], [0, 0, 127, 0], [0, 0, 127, 0], [0, -128, 0, 0]], np.int8)   # VEC3 padded to 4 B
    uvq = np.array([[0, 0], [65535, 0], [0, 65535], [32768, 65535]], np.uint16)
    acc = [{"bufferView": 0, "componentType": 5122, "normalized": True, "count": 4, "type": "VEC3"},
           {"bufferView": 1, "componentType": 5120, "normalized": True, "count": 4, "type": "VEC3"},
           {"bufferView": 2, "componentType": 5123, "normalized": True, "count": 4, "type": "VEC2"},
           {"bufferView": 3, "componentType": 5121, "count": 6, "type": "SCALAR"}]
    blobs = [q.tobytes(), nq.tobytes(), uvq.tobytes(), bytes([0, 1, 2, 1, 3, 2])]
    path = _write(tmp_path, [{"attributes": {"POSITION": 0, "NORMAL": 1, "TEXCOORD_0": 2}, "indices": 3}], acc, blobs)
    g = json.load(open(path))
    g["bufferViews"][1]["byteStride"] = 4      # int8 VEC3 normals are 4-byte aligned per element
    g["extensionsUsed"] = ["KHR_mesh_quantization"]
    json.dump(g, open(path, "w"))
    sd = scene.load_gltf(path)
    want = np.maximum(q.astype(np.float32) / np.float32(32767.0), np.float32(-1.0))
    assert np.array_equal(np.asarray(sd.vertices).reshape(-1, 3), want)
    nrm = np.asarray(sd.normals).reshape(-1, 3)
    assert np.allclose(nrm[0], [0, 0, 1]) and np.allclose(nrm[3], [0, -1, 0])   # -128 / 127 clamped to -1
    assert sd.num_triangles == 2
