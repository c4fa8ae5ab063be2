"""Seeded procedural stand-in for the Bistro exterior.

The Bistro glTF is not in the container, so the C3/C4 workloads run on a procedural
city of the same scale: a street grid of buildings whose facades are tessellated into
recessed windows (18 triangles per window cell), roofs, sidewalks, street lamps (the
emissive triangles NEE samples) and trees (smooth-shaded icospheres), ≈2.6 M triangles
for the default seed.  Everything is generated with numpy from ``seed`` (default 1234),
so the scene is identical on every machine without shipping a file.
"""
from __future__ import annotations

import math

import numpy as np

from . import abi
from .scene import SceneData


def _mat(base, rough=0.8, metallic=0.0, specular=0.5, emission=None, strength=1.0):
    m = abi.Material.default()
    m.base_color = abi.Color(*base)
    m.roughness = rough
    m.metallic = metallic
    m.specular = specular
    if emission is not None:
        m.emission = abi.Color(*emission)
        m.emission_strength = strength
    m.make_safe()
    m.precompute_properties()
    return m


class _Builder:
    def __init__(self):
        self.v, self.n, self.hn, self.idx, self.mi = [], [], [], [], []
        self.nv = 0

    def quads(self, p00, p10, p11, p01, mat):
        """Batch of quads (arrays [K,3] of corners, counter-clockwise) -> 2 flat triangles each."""
        k = len(p00)
        if k == 0:
            return
        V = np.stack([p00, p10, p11, p01], 1).reshape(-1, 3)
        base = self.nv + 4 * np.arange(k)[:, None]
        I = np.concatenate([base + np.array([0, 1, 2]), base + np.array([0, 2, 3])], 1).reshape(-1, 3)
        self.v.append(V)
        self.n.append(np.zeros_like(V))
        self.hn.append(np.zeros(len(V), np.uint8))
        self.idx.append(I)
        self.mi.append(np.broadcast_to(np.asarray(mat, np.int32), (k,)).repeat(2) if np.ndim(mat) == 0
                       else np.repeat(np.asarray(mat, np.int32), 2))
        self.nv += len(V)

    def mesh(self, V, N, I, mat):
        self.v.append(V)
        self.n.append(N)
        self.hn.append(np.ones(len(V), np.uint8))
        self.idx.append(I + self.nv)
        self.mi.append(np.full(len(I), mat, np.int32))
        self.nv += len(V)


def _icosphere(sub=2):
    t = (1.0 + 5 ** 0.5) / 2.0
    V = [(-1, t, 0), (1, t, 0), (-1, -t, 0), (1, -t, 0), (0, -1, t), (0, 1, t), (0, -1, -t), (0, 1, -t),
         (t, 0, -1), (t, 0, 1), (-t, 0, -1), (-t, 0, 1)]
    F = [(0, 11, 5), (0, 5, 1), (0, 1, 7), (0, 7, 10), (0, 10, 11), (1, 5, 9), (5, 11, 4), (11, 10, 2), (10, 7, 6),
         (7, 1, 8), (3, 9, 4), (3, 4, 2), (3, 2, 6), (3, 6, 8), (3, 8, 9), (4, 9, 5), (2, 4, 11), (6, 2, 10), (8, 6, 7),
         (9, 8, 1)]
    V = [np.array(v, float) / np.linalg.norm(v) for v in V]
    for _ in range(sub):
        cache, F2 = {}, []

        def mid(a, b):
            key = (min(a, b), max(a, b))
            if key not in cache:
                m = V[a] + V[b]
                V.append(m / np.linalg.norm(m))
                cache[key] = len(V) - 1
            return cache[key]
        for a, b, c in F:
            ab, bc, ca = mid(a, b), mid(b, c), mid(c, a)
            F2 += [(a, ab, ca), (b, bc, ab), (c, ca, bc), (ab, bc, ca)]
        F = F2
    return np.array(V), np.array(F, np.int64)


def _leaf_texture(seed: int, size: int = 64) -> np.ndarray:
    """RGBA8 leaf cluster: green shades, alpha 255 inside ~45 % of the texels (seeded
    discs), 0 elsewhere -- the alpha-tested foliage of the Bistro (do_alpha_testing)."""
    rng = np.random.default_rng(seed)
    yy, xx = np.meshgrid(np.arange(size) + 0.5, np.arange(size) + 0.5, indexing="ij")
    cover = np.zeros((size, size), bool)
    for _ in range(14):
        cx, cy, r = rng.uniform(0, size, 2).tolist() + [rng.uniform(0.08, 0.2) * size]
        cover |= (xx - cx) ** 2 + (yy - cy) ** 2 < r * r
    tex = np.zeros((size, size, 4), np.uint8)
    tex[..., 0] = rng.integers(30, 70, (size, size))
    tex[..., 1] = rng.integers(90, 160, (size, size))
    tex[..., 2] = rng.integers(20, 50, (size, size))
    tex[..., 3] = np.where(cover, 255, 0)
    return tex


def procedural_city(seed: int = 1234, blocks: int = 17, leaf_cards: int = 16) -> SceneData:
    rng = np.random.default_rng(seed)
    B = _Builder()
    mats = [
        _mat((0.08, 0.08, 0.085), rough=0.9, specular=0.3),            # 0 asphalt
        _mat((0.45, 0.44, 0.42), rough=0.85, specular=0.4),            # 1 sidewalk
        _mat((0.62, 0.55, 0.45), rough=0.8),                           # 2 wall beige
        _mat((0.55, 0.25, 0.2), rough=0.8),                            # 3 wall brick
        _mat((0.7, 0.7, 0.72), rough=0.7),                             # 4 wall white
        _mat((0.3, 0.35, 0.4), rough=0.6),                             # 5 wall slate
        _mat((0.05, 0.07, 0.08), rough=0.05, specular=1.0),            # 6 window glass (glossy dark)
        _mat((0.2, 0.2, 0.22), rough=0.9),                             # 7 roof
        _mat((0.12, 0.3, 0.08), rough=0.95, specular=0.2),             # 8 foliage
        _mat((0.8, 0.8, 0.82), rough=0.3, metallic=1.0),               # 9 lamp metal
        _mat((1.0, 0.9, 0.7), emission=(1.0, 0.85, 0.6), strength=40.0),  # 10 lamp light
        _mat((1.0, 1.0, 1.0), rough=0.9, specular=0.3),                # 11 leaf cards (alpha-tested texture 0)
    ]
    mats[11].base_color_texture_index = 0
    blk, street = 40.0, 12.0
    pitch = blk + street
    half = blocks * pitch / 2.0
    # ground: asphalt streets as one big quad grid (coarse) + raised sidewalks per block
    g = np.linspace(-half, half, 33)
    gx, gz = np.meshgrid(g[:-1], g[:-1], indexing="ij")
    gx, gz = gx.ravel(), gz.ravel()
    d = g[1] - g[0]
    z0 = np.zeros_like(gx)
    B.quads(np.stack([gx, z0, gz], 1), np.stack([gx, z0, gz + d], 1), np.stack([gx + d, z0, gz + d], 1),
            np.stack([gx + d, z0, gz], 1), 0)
    bx, bz = np.meshgrid(np.arange(blocks), np.arange(blocks), indexing="ij")
    bx = -half + street / 2 + bx.ravel() * pitch
    bz = -half + street / 2 + bz.ravel() * pitch
    h0 = np.full_like(bx, 0.15)
    # sidewalk tops
    B.quads(np.stack([bx, h0, bz], 1), np.stack([bx, h0, bz + blk], 1), np.stack([bx + blk, h0, bz + blk], 1),
            np.stack([bx + blk, h0, bz], 1), 1)
    # buildings: 2x2 per block with jittered footprints
    lots = []
    for i in range(2):
        for j in range(2):
            w = rng.uniform(12.0, 17.0, len(bx))
            dd = rng.uniform(12.0, 17.0, len(bx))
            x0 = bx + 2.0 + i * 19.0 + rng.uniform(0.0, 17.0 - w + 0.01)
            zz0 = bz + 2.0 + j * 19.0 + rng.uniform(0.0, 17.0 - dd + 0.01)
            h = np.clip(rng.lognormal(math.log(22.0), 0.45, len(bx)), 9.0, 90.0)
            lots.append(np.stack([x0, zz0, w, dd, h], 1))
    lots = np.concatenate(lots, 0)
    wall_mat = rng.integers(2, 6, len(lots))
    # roofs
    x0, zz, w, dd, h = lots.T
    B.quads(np.stack([x0, h, zz], 1), np.stack([x0, h, zz + dd], 1), np.stack([x0 + w, h, zz + dd], 1),
            np.stack([x0 + w, h, zz], 1), wall_mat * 0 + 7)
    # facades: (origin, right, normal) per side; cells of ~3.2 m x 3.5 m with a recessed window
    for side in range(4):
        if side == 0:   # -z facade, right = +x
            O = np.stack([x0, np.zeros_like(x0), zz], 1); R = np.array([1.0, 0, 0]); N = np.array([0, 0, -1.0]); L = w
        elif side == 1:  # +x facade, right = +z
            O = np.stack([x0 + w, np.zeros_like(x0), zz], 1); R = np.array([0, 0, 1.0]); N = np.array([1.0, 0, 0]); L = dd
        elif side == 2:  # +z facade, right = -x
            O = np.stack([x0 + w, np.zeros_like(x0), zz + dd], 1); R = np.array([-1.0, 0, 0]); N = np.array([0, 0, 1.0]); L = w
        else:            # -x facade, right = -z
            O = np.stack([x0, np.zeros_like(x0), zz + dd], 1); R = np.array([0, 0, -1.0]); N = np.array([-1.0, 0, 0]); L = dd
        cols = np.maximum(1, np.round(L / 3.2)).astype(int)
        floors = np.maximum(1, np.round(h / 3.5)).astype(int)
        cw, ch = L / cols, h / floors
        ncell = cols * floors
        bi = np.repeat(np.arange(len(lots)), ncell)
        # cell (c, f) indices per building
        starts = np.concatenate([[0], np.cumsum(ncell)[:-1]])
        k = np.arange(ncell.sum()) - np.repeat(starts, ncell)
        c = k % cols[bi]
        f = k // cols[bi]
        U = np.array([0.0, 1.0, 0.0])
        o = O[bi] + (c * cw[bi])[:, None] * R + (f * ch[bi])[:, None] * U
        cwv, chv = cw[bi][:, None], ch[bi][:, None]
        mx, my = 0.22 * cwv, 0.25 * chv                      # wall margins around the window
        depth = rng.uniform(0.15, 0.4, len(bi))[:, None]
        Ru, Uu = R[None, :], U[None, :]

        def P(a, b, dep=0.0):
            return o + a * Ru + b * Uu - dep * N[None, :]
        wm = wall_mat[bi]
        # wall strips: bottom, top, left, right (outward facing => counter-clockwise seen from N)
        B.quads(P(0, 0), P(cwv, 0), P(cwv, my), P(0, my), wm)
        B.quads(P(0, chv - my), P(cwv, chv - my), P(cwv, chv), P(0, chv), wm)
        B.quads(P(0, my), P(mx, my), P(mx, chv - my), P(0, chv - my), wm)
        B.quads(P(cwv - mx, my), P(cwv, my), P(cwv, chv - my), P(cwv - mx, chv - my), wm)
        # reveals (window recess sides)
        B.quads(P(mx, my), P(mx, my, depth), P(cwv - mx, my, depth), P(cwv - mx, my), wm)
        B.quads(P(mx, chv - my), P(cwv - mx, chv - my), P(cwv - mx, chv - my, depth), P(mx, chv - my, depth), wm)
        B.quads(P(mx, my), P(mx, chv - my), P(mx, chv - my, depth), P(mx, my, depth), wm)
        B.quads(P(cwv - mx, my), P(cwv - mx, my, depth), P(cwv - mx, chv - my, depth), P(cwv - mx, chv - my), wm)
        # glass
        B.quads(P(mx, my, depth), P(cwv - mx, my, depth), P(cwv - mx, chv - my, depth), P(mx, chv - my, depth), 6)
    # street lamps along the streets: post (thin box, 4 quads) + emissive panel facing down
    lx = np.concatenate([bx + 5.0, bx + 25.0, bx - 1.5, bx - 1.5])
    lz = np.concatenate([bz - 1.5, bz - 1.5, bz + 5.0, bz + 25.0])
    keep = rng.random(len(lx)) < 0.6
    lx, lz = lx[keep], lz[keep]
    t = 0.08
    for (ax, az, bxo, bzo) in [(-t, -t, t, -t), (t, -t, t, t), (t, t, -t, t), (-t, t, -t, -t)]:
        y0 = np.zeros_like(lx)
        y1 = np.full_like(lx, 5.0)
        B.quads(np.stack([lx + ax, y0, lz + az], 1), np.stack([lx + bxo, y0, lz + bzo], 1),
                np.stack([lx + bxo, y1, lz + bzo], 1), np.stack([lx + ax, y1, lz + az], 1), 9)
    s = 0.35
    y = np.full_like(lx, 4.95)
    B.quads(np.stack([lx - s, y, lz - s], 1), np.stack([lx + s, y, lz - s], 1), np.stack([lx + s, y, lz + s], 1),
            np.stack([lx - s, y, lz + s], 1), 10)
    # trees: smooth icospheres on the sidewalks
    SV, SF = _icosphere(2)
    tx = np.concatenate([bx + rng.uniform(1, 39, len(bx)), bx + rng.uniform(1, 39, len(bx))])
    tz = np.concatenate([bz + 0.8 + 0 * bx, bz + 39.2 + 0 * bx])
    tr = rng.uniform(1.2, 2.2, len(tx))
    ctr = np.stack([tx, 3.0 + tr, tz], 1)
    V = (SV[None, :, :] * tr[:, None, None] + ctr[:, None, :]).reshape(-1, 3)
    Nn = np.broadcast_to(SV[None], (len(tx),) + SV.shape).reshape(-1, 3)
    F = (SF[None, :, :] + (len(SV) * np.arange(len(tx)))[:, None, None]).reshape(-1, 3)
    B.mesh(V, Nn.copy(), F, 8)
    # alpha-tested leaf cards around each crown (random orientation, uv 0..1 per card)
    first_card_vertex = B.nv
    if leaf_cards > 0:
        nt, k = len(tx), leaf_cards
        dirs = rng.normal(size=(nt, k, 3))
        dirs /= np.linalg.norm(dirs, axis=-1, keepdims=True)
        cc = ctr[:, None, :] + dirs * (tr[:, None, None] * rng.uniform(0.6, 1.2, (nt, k, 1)))
        nrm = rng.normal(size=(nt, k, 3))
        nrm /= np.linalg.norm(nrm, axis=-1, keepdims=True)
        a = np.cross(nrm, np.array([0.0, 1.0, 0.0]))
        a /= np.maximum(np.linalg.norm(a, axis=-1, keepdims=True), 1e-6)
        b = np.cross(nrm, a)
        hs = 0.6
        c4 = [cc - hs * a - hs * b, cc + hs * a - hs * b, cc + hs * a + hs * b, cc - hs * a + hs * b]
        B.quads(*[q.reshape(-1, 3) for q in c4], 11)
    sd = SceneData()
    sd.vertices = np.concatenate(B.v).astype(np.float32)
    sd.normals = np.concatenate(B.n).astype(np.float32)
    sd.has_normals = np.concatenate(B.hn).astype(np.uint8)
    sd.texcoords = np.zeros((len(sd.vertices), 2), np.float32)
    ncard_v = len(sd.vertices) - first_card_vertex
    sd.texcoords[first_card_vertex:] = np.tile(np.array([[0, 0], [1, 0], [1, 1], [0, 1]], np.float32), (ncard_v // 4, 1))
    sd.triangle_indices = np.concatenate(B.idx).astype(np.int32).ravel()
    sd.material_indices = np.concatenate(B.mi).astype(np.int32)
    sd.materials = mats
    sd.textures = [_leaf_texture(seed)]
    sd.name = f"procedural_city_{seed}"
    # street-level camera at an intersection looking down a street, slightly up
    cx = -half + street / 2 + (blocks // 2) * pitch - street / 2
    sd.camera_info = dict(position=np.array([cx, 1.7, half - 8.0]), lookat=np.array([cx + 0.8, 4.0, half - 60.0]),
                          up=np.array([0.0, 1.0, 0.0]), hfov=1.0, aspect=16 / 9, znear=0.1, zfar=1000.0)
    return sd.finalize()


def with_alpha_cards(sd: SceneData, opacity: float = 0.5, tex_size: int = 16, alpha_levels=(0, 100, 255)) -> SceneData:
    """Adds two alpha-tested cards to a scene (for do_alpha_testing, FilterFunction.h:19-48):
    a textured card whose base-colour texture is a checkerboard of alpha levels (RGBA8),
    and an untextured card with material alpha_opacity = ``opacity``.  Both stand
    across the Cornell box's opening, so camera, NEE and envmap rays cross them."""
    out = SceneData()
    lo, hi = sd.vertices.min(0), sd.vertices.max(0)
    c = (lo + hi) / 2
    ext = (hi - lo) / 2
    z1, z2 = hi[2] + 0.2 * ext[2], c[2] + 0.3 * ext[2]
    x0, x1 = lo[0] + 0.1 * ext[0], hi[0] - 0.1 * ext[0]
    y0, y1 = lo[1] + 0.1 * ext[1], hi[1] - 0.1 * ext[1]
    cards_v = np.array([[x0, y0, z1], [c[0], y0, z1], [c[0], y1, z1], [x0, y1, z1],      # textured (left half)
                        [c[0], y0, z2], [x1, y0, z2], [x1, y1, z2], [c[0], y1, z2]],     # opacity card (right half)
                       np.float32)
    cards_uv = np.array([[0, 0], [1, 0], [1, 1], [0, 1]] * 2, np.float32)
    nv = len(sd.vertices)
    cards_i = np.array([[0, 1, 2], [0, 2, 3], [4, 5, 6], [4, 6, 7]], np.int32) + nv
    nm = len(sd.materials)
    tm = abi.Material.from_buffer_copy(_mat((0.8, 0.3, 0.2), rough=0.5))
    tm.base_color_texture_index = len(sd.textures)
    om = abi.Material.from_buffer_copy(_mat((0.2, 0.4, 0.8), rough=0.3))
    om.alpha_opacity = opacity
    rng = np.random.default_rng(5)
    tex = np.zeros((tex_size, tex_size, 4), np.uint8)
    tex[..., :3] = rng.integers(64, 256, (tex_size, tex_size, 3))
    yy, xx = np.meshgrid(np.arange(tex_size), np.arange(tex_size), indexing="ij")
    tex[..., 3] = np.asarray(alpha_levels, np.uint8)[((yy // 4) + (xx // 4)) % len(alpha_levels)]
    out.triangle_indices = np.concatenate([sd.triangle_indices.reshape(-1), cards_i.reshape(-1)]).astype(np.int32)
    out.vertices = np.concatenate([sd.vertices, cards_v]).astype(np.float32)
    out.normals = np.concatenate([sd.normals, np.zeros((8, 3), np.float32)]).astype(np.float32)
    out.has_normals = np.concatenate([sd.has_normals, np.zeros(8, np.uint8)]).astype(np.uint8)
    out.texcoords = np.concatenate([sd.texcoords, cards_uv]).astype(np.float32)
    out.material_indices = np.concatenate([sd.material_indices, np.array([nm, nm, nm + 1, nm + 1], np.int32)])
    out.materials = list(sd.materials) + [tm, om]
    out.textures = list(sd.textures) + [tex]
    out.camera_info = sd.camera_info
    out.name = sd.name + "+alpha_cards"
    return out.finalize()


def _panel_grid(x0, x1, y0, y1, z, n=4, flip=False):
    """n x n grid of quads on the plane z = const facing +z (toward the Cornell camera):
    vertices [(n+1)^2, 3], texcoords in [0, 1]^2, triangles [2 n^2, 3]."""
    xs, ys = np.linspace(x0, x1, n + 1), np.linspace(y0, y1, n + 1)
    yy, xx = np.meshgrid(ys, xs, indexing="ij")
    V = np.stack([xx, yy, np.full_like(xx, z)], -1).reshape(-1, 3)
    uv = np.stack([(xx - x0) / (x1 - x0), (yy - y0) / (y1 - y0)], -1).reshape(-1, 2)
    I = []
    for j in range(n):
        for i in range(n):
            a, b, c, d = j * (n + 1) + i, j * (n + 1) + i + 1, (j + 1) * (n + 1) + i + 1, (j + 1) * (n + 1) + i
            I += [[a, b, c], [a, c, d]] if not flip else [[a, c, b], [a, d, c]]
    return V.astype(np.float32), uv.astype(np.float32), np.array(I, np.int64)


def _tex(rng, size, lo=0, hi=256, channels=(0, 1, 2), alpha=255):
    t = np.zeros((size, size, 4), np.uint8)
    for c in channels:
        t[..., c] = rng.integers(lo, hi, (size, size))
    t[..., 3] = alpha
    return t


def with_textured_panels(sd: SceneData, seed: int = 3) -> SceneData:
    """Adds three textured panels in front of the Cornell box's back wall that drive every
    texture slot of RendererMaterial (Material.h:140-159, read by get_intersection_material,
    Device/includes/Material.h:47-159):
    * panel 0 (flat normals): base colour (sRGB), normal map (Texture.h:209-222),
      roughness-metallic (G roughness, B metallic);
    * panel 1 (smooth, tilted vertex normals): base colour, emission texture (index > 0, so
      emissive_texture_used, Material.h:109), specular, specular tint, specular colour;
    * panel 2 (flat): separate metallic and roughness textures, coat, coat roughness, sheen,
      sheen roughness, sheen colour, anisotropy, anisotropy rotation, Oren-Nayar sigma, and a
      normal map.
    Textures are seeded RGBA8 noise of a few levels (alpha 255)."""
    rng = np.random.default_rng(seed)
    S = 16
    texs = list(sd.textures)
    t0 = len(texs)

    def add(t):
        texs.append(t)
        return len(texs) - 1

    def normal_map():
        n = rng.normal(size=(S, S, 3)) * np.array([0.35, 0.35, 0.0]) + np.array([0.0, 0.0, 1.0])
        n /= np.linalg.norm(n, axis=-1, keepdims=True)
        t = np.zeros((S, S, 4), np.uint8)
        t[..., :3] = np.clip(np.round((n * 0.5 + 0.5) * 255.0), 0, 255).astype(np.uint8)
        t[..., 3] = 255
        return t

    def levels(vals, chans=(0,)):
        t = np.zeros((S, S, 4), np.uint8)
        pick = np.asarray(vals, np.uint8)[rng.integers(0, len(vals), (S, S))]
        for c in chans:
            t[..., c] = pick
        t[..., 3] = 255
        return t

    mats = []
    # panel 0
    m0 = abi.Material.from_buffer_copy(_mat((0.7, 0.7, 0.7), rough=0.5))
    if t0 == 0:
        add(_tex(rng, S, 200, 256))           # texture 0: never an emission texture (index > 0 rule)
    m0.base_color_texture_index = add(_tex(rng, S, 40, 256))
    m0.normal_map_texture_index = add(normal_map())
    rm = np.zeros((S, S, 4), np.uint8)
    rm[..., 1] = rng.choice([40, 120, 220], (S, S))           # roughness
    rm[..., 2] = rng.choice([0, 0, 128, 255], (S, S))         # metallic
    rm[..., 3] = 255
    m0.roughness_metallic_texture_index = add(rm)
    mats.append(m0)
    # panel 1
    m1 = abi.Material.from_buffer_copy(_mat((0.5, 0.6, 0.7), rough=0.35))
    m1.base_color_texture_index = add(_tex(rng, S, 60, 256))
    em = np.zeros((S, S, 4), np.uint8)
    em[..., :3] = np.where(rng.random((S, S, 1)) < 0.3, rng.integers(128, 256, (S, S, 3)), 0)
    em[..., 3] = 255
    m1.emission_texture_index = add(em)
    m1.emissive_texture_used = True
    m1.emission = abi.Color(1.0, 1.0, 1.0)
    m1.emission_strength = 3.0
    m1.specular_texture_index = add(levels([60, 160, 255]))
    m1.specular_tint_texture_index = add(levels([0, 128, 255]))
    m1.specular_color_texture_index = add(_tex(rng, S, 100, 256))
    mats.append(m1)
    # panel 2
    m2 = abi.Material.from_buffer_copy(_mat((0.6, 0.45, 0.3), rough=0.4))
    m2.base_color_texture_index = add(_tex(rng, S, 60, 256))
    m2.metallic_texture_index = add(levels([0, 90, 255]))
    m2.roughness_texture_index = add(levels([30, 110, 200]))
    m2.coat_texture_index = add(levels([0, 160, 255]))
    m2.coat_roughness_texture_index = add(levels([10, 90]))
    m2.sheen_texture_index = add(levels([0, 200]))
    m2.sheen_roughness_texture_index = add(levels([60, 180]))
    m2.sheen_color_texture_index = add(_tex(rng, S, 80, 256))
    m2.anisotropic_texture_index = add(levels([0, 120, 230]))
    m2.anisotropic_rotation_texture_index = add(levels([0, 64, 190]))
    m2.oren_sigma_texture_index = add(levels([20, 90]))
    m2.normal_map_texture_index = add(normal_map())
    mats.append(m2)

    nm = len(sd.materials)
    out = SceneData()
    V, N, HN, UV, I, MI = [sd.vertices], [sd.normals], [sd.has_normals], [sd.texcoords], [sd.triangle_indices.reshape(-1, 3)], \
        [sd.material_indices]
    nv = len(sd.vertices)
    z = -1.0
    for k, (x0, x1) in enumerate([(-0.95, -0.35), (-0.3, 0.3), (0.35, 0.95)]):
        pv, puv, pi = _panel_grid(x0, x1, 1.25, 1.85, z)
        if k == 1:   # smooth, tilted vertex normals
            pn = np.stack([0.25 * (puv[:, 0] - 0.5), 0.2 * (puv[:, 1] - 0.5), np.ones(len(pv))], -1)
            pn /= np.linalg.norm(pn, axis=1, keepdims=True)
            hn = np.ones(len(pv), np.uint8)
        else:
            pn = np.zeros_like(pv)
            hn = np.zeros(len(pv), np.uint8)
        V.append(pv); N.append(pn.astype(np.float32)); HN.append(hn); UV.append(puv)
        I.append(pi + nv); MI.append(np.full(len(pi), nm + k, np.int32))
        nv += len(pv)
    out.vertices = np.concatenate(V).astype(np.float32)
    out.normals = np.concatenate(N).astype(np.float32)
    out.has_normals = np.concatenate(HN).astype(np.uint8)
    out.texcoords = np.concatenate(UV).astype(np.float32)
    out.triangle_indices = np.concatenate(I).astype(np.int32).ravel()
    out.material_indices = np.concatenate(MI).astype(np.int32)
    out.materials = list(sd.materials) + mats
    out.textures = texs
    out.camera_info = sd.camera_info
    out.name = sd.name + "+textured_panels"
    return out.finalize()


def write_textured_gltf(dirpath: str, seed: int = 5, glb: bool = False) -> str:
    """Writes a small textured glTF 2 scene (the ingestion test asset: the reference's one
    textured scene, the-white-room-low.gltf, ships without its geometry) and returns its path.

    A floor and a back wall under an emissive ceiling quad, two panels in front:
    * floor: base colour (RGB PNG in a file whose name has a space, referenced as '%20'),
      metallicRoughnessTexture (RGB), normalTexture (RGBA, Adam7-interlaced);
    * back wall: untextured (its texture coordinates are dropped, SceneParser.cpp:136-141);
    * left panel: an emission texture with texel variation (emissiveFactor 1, strength 2),
      KHR_materials_specular.specularTexture (RGB: stb's grey conversion), clearcoatTexture
      (grey + alpha);
    * right panel: a near-constant emission texture (every texel within 5 of the first: folded
      into the material's emission, Image8Bit::is_constant_color(5)), sheenColorTexture in a
      data: URI, transmissionTexture as a palette PNG with tRNS;
    * ceiling: emissiveFactor 5, no texture.
    glb=True writes one .glb with every image in a bufferView."""
    import base64
    import json
    import os
    import struct

    from . import image
    rng = np.random.default_rng(seed)
    S = 16

    def noise(c, lo=0, hi=256, size=S):
        return rng.integers(lo, hi, (size, size, c)).astype(np.uint8)

    nrm = rng.normal(size=(S, S, 3)) * np.array([0.3, 0.3, 0.0]) + np.array([0.0, 0.0, 1.0])
    nrm /= np.linalg.norm(nrm, axis=-1, keepdims=True)
    nrm_img = np.concatenate([np.clip(np.round((nrm * 0.5 + 0.5) * 255), 0, 255).astype(np.uint8),
                              np.full((S, S, 1), 255, np.uint8)], -1)
    em_const = np.clip(np.array([200, 150, 90], np.int32) + rng.integers(-2, 3, (S, S, 3)), 0, 255).astype(np.uint8)
    em_var = np.where(rng.random((S, S, 1)) < 0.4, noise(3, 100, 256), 0).astype(np.uint8)
    pal = np.concatenate([rng.integers(0, 256, (6, 3)), np.array([[255], [128], [0], [255], [60], [255]])], 1)
    images = {
        "floor base.png": image.encode_png(noise(3, 40, 256)),
        "floor_mr.png": image.encode_png(np.concatenate([noise(1), noise(1, 20, 230), noise(1, 0, 256)], -1)),
        "floor_normal.png": image.encode_png(nrm_img, interlace=True),
        "left_emission.png": image.encode_png(em_var),
        "left_specular.png": image.encode_png(noise(3, 30, 256)),
        "left_coat.png": image.encode_png(noise(2, 0, 256)),
        "right_emission.png": image.encode_png(em_const),
        "right_sheen.png": image.encode_png(noise(3, 0, 256)),
        "right_transmission.png": image.encode_png(rng.integers(0, 6, (S, S)).astype(np.uint8), palette=pal),
    }
    names = list(images)

    # geometry: quads (4 vertices, 2 triangles), positions / normals / uvs
    quads = [
        # (corner, edge u, edge v, normal, material)
        ((-1.0, 0.0, 1.0), (2.0, 0.0, 0.0), (0.0, 0.0, -2.0), (0, 1, 0), 0),     # floor
        ((-1.0, 0.0, -1.0), (2.0, 0.0, 0.0), (0.0, 2.0, 0.0), (0, 0, 1), 1),     # back wall
        ((-0.9, 0.3, -0.4), (0.7, 0.0, 0.2), (0.0, 0.9, 0.0), (-0.275, 0, 0.962), 2),  # left panel
        ((0.2, 0.3, -0.3), (0.7, 0.0, -0.2), (0.0, 0.9, 0.0), (0.275, 0, 0.962), 3),   # right panel
        ((-0.3, 1.99, -0.3), (0.6, 0.0, 0.0), (0.0, 0.0, 0.6), (0, -1, 0), 4),   # ceiling light
    ]
    bin_parts, views, accessors, meshes, nodes = [], [], [], [], []

    def add_view(data: bytes, target=None):
        off = sum(len(b) for b in bin_parts)
        pad = (-off) % 4
        if pad:
            bin_parts.append(b"\0" * pad)
            off += pad
        bin_parts.append(data)
        v = {"buffer": 0, "byteOffset": off, "byteLength": len(data)}
        if target:
            v["target"] = target
        views.append(v)
        return len(views) - 1

    def add_acc(arr, ctype, typ, target):
        arr = np.ascontiguousarray(arr)
        a = {"bufferView": add_view(arr.tobytes(), target), "componentType": ctype, "count": int(arr.shape[0]), "type": typ}
        if typ == "VEC3" and ctype == 5126:
            a["min"], a["max"] = arr.min(0).tolist(), arr.max(0).tolist()
        accessors.append(a)
        return len(accessors) - 1

    for k, (p0, eu, ev, n, mat) in enumerate(quads):
        p0, eu, ev = np.array(p0), np.array(eu), np.array(ev)
        P = np.array([p0, p0 + eu, p0 + eu + ev, p0 + ev], np.float32)
        N = np.tile(np.array(n, np.float64) / np.linalg.norm(n), (4, 1)).astype(np.float32)
        UV = np.array([[0, 1], [1, 1], [1, 0], [0, 0]], np.float32) * np.float32(1.5 if k == 0 else 1.0)
        I = np.array([0, 1, 2, 0, 2, 3], np.uint16)
        prim = {"attributes": {"POSITION": add_acc(P, 5126, "VEC3", 34962), "NORMAL": add_acc(N, 5126, "VEC3", 34962),
                               "TEXCOORD_0": add_acc(UV, 5126, "VEC2", 34962)},
                "indices": add_acc(I, 5123, "SCALAR", 34963), "material": mat}
        meshes.append({"primitives": [prim]})
        nodes.append({"mesh": k})
    nodes.append({"camera": 0, "translation": [0.0, 1.0, 3.2]})

    def tex(name):
        return {"index": names.index(name)}
    materials = [
        {"name": "floor", "pbrMetallicRoughness": {"baseColorTexture": tex("floor base.png"), "metallicRoughnessTexture":
                                                  tex("floor_mr.png"), "roughnessFactor": 0.6, "metallicFactor": 0.5},
         "normalTexture": tex("floor_normal.png")},
        {"name": "wall", "pbrMetallicRoughness": {"baseColorFactor": [0.7, 0.65, 0.6, 1.0], "metallicFactor": 0.0,
                                                 "roughnessFactor": 0.8}},
        {"name": "left", "pbrMetallicRoughness": {"baseColorFactor": [0.5, 0.6, 0.7, 1.0], "metallicFactor": 0.0,
                                                 "roughnessFactor": 0.4},
         "emissiveTexture": tex("left_emission.png"), "emissiveFactor": [1.0, 1.0, 1.0],
         "extensions": {"KHR_materials_emissive_strength": {"emissiveStrength": 2.0},
                        "KHR_materials_specular": {"specularFactor": 0.8, "specularTexture": tex("left_specular.png")},
                        "KHR_materials_clearcoat": {"clearcoatFactor": 0.7, "clearcoatRoughnessFactor": 0.2,
                                                    "clearcoatTexture": tex("left_coat.png")}}},
        {"name": "right", "pbrMetallicRoughness": {"baseColorFactor": [0.8, 0.5, 0.4, 1.0], "metallicFactor": 0.0,
                                                  "roughnessFactor": 0.5},
         "emissiveTexture": tex("right_emission.png"), "emissiveFactor": [1.0, 1.0, 1.0],
         "extensions": {"KHR_materials_sheen": {"sheenColorFactor": [0.9, 0.8, 0.7], "sheenRoughnessFactor": 0.4,
                                                "sheenColorTexture": tex("right_sheen.png")},
                        "KHR_materials_transmission": {"transmissionFactor": 0.3,
                                                       "transmissionTexture": tex("right_transmission.png")}}},
        {"name": "light", "pbrMetallicRoughness": {"baseColorFactor": [1, 1, 1, 1], "metallicFactor": 0.0},
         "emissiveFactor": [1.0, 1.0, 1.0], "extensions": {"KHR_materials_emissive_strength": {"emissiveStrength": 5.0}}},
    ]
    imgs = []
    for nm in names:
        if glb:
            imgs.append({"bufferView": add_view(images[nm]), "mimeType": "image/png"})
        elif nm == "right_sheen.png":
            imgs.append({"uri": "data:image/png;base64," + base64.b64encode(images[nm]).decode()})
        else:
            imgs.append({"uri": nm.replace(" ", "%20")})
    binary = b"".join(bin_parts)
    g = {"asset": {"version": "2.0"}, "scene": 0, "scenes": [{"nodes": list(range(len(nodes)))}], "nodes": nodes,
         "meshes": meshes, "materials": materials, "accessors": accessors, "bufferViews": views,
         "textures": [{"source": i} for i in range(len(names))], "images": imgs,
         "cameras": [{"type": "perspective", "perspective": {"yfov": 0.75, "aspectRatio": 1.0, "znear": 0.05, "zfar": 50.0}}],
         "extensionsUsed": ["KHR_materials_emissive_strength", "KHR_materials_specular", "KHR_materials_clearcoat",
                            "KHR_materials_sheen", "KHR_materials_transmission"]}
    os.makedirs(dirpath, exist_ok=True)
    if glb:
        g["buffers"] = [{"byteLength": len(binary)}]
        js = json.dumps(g).encode()
        js += b" " * ((-len(js)) % 4)
        binary += b"\0" * ((-len(binary)) % 4)
        body = struct.pack("<I4s", len(js), b"JSON") + js + struct.pack("<I4s", len(binary), b"BIN\0") + binary
        path = os.path.join(dirpath, "textured_room.glb")
        with open(path, "wb") as f:
            f.write(struct.pack("<4sII", b"glTF", 2, 12 + len(body)) + body)
        return path
    g["buffers"] = [{"uri": "textured_room.bin", "byteLength": len(binary)}]
    with open(os.path.join(dirpath, "textured_room.bin"), "wb") as f:
        f.write(binary)
    for nm in names:
        if nm != "right_sheen.png":
            with open(os.path.join(dirpath, nm), "wb") as f:
                f.write(images[nm])
    path = os.path.join(dirpath, "textured_room.gltf")
    with open(path, "w") as f:
        json.dump(g, f)
    return path


# ---- texture-realistic variant (VERDICT r03 "What's weak" 7) ------------------------------
def _value_noise(rng, size, cells, octaves=3):
    """Smooth periodic value noise in [0, 1), [size, size] float32 (bilinear upsampled lattices)."""
    out = np.zeros((size, size), np.float32)
    amp, tot = 1.0, 0.0
    for o in range(octaves):
        n = cells << o
        lat = rng.random((n, n)).astype(np.float32)
        t = (np.arange(size, dtype=np.float32) + 0.5) * n / size - 0.5
        i0 = np.floor(t).astype(np.int64)
        f = (t - i0).astype(np.float32)
        i0 %= n
        i1 = (i0 + 1) % n
        rows = lat[i0][:, i0] * (1 - f)[None, :] + lat[i0][:, i1] * f[None, :]
        rows1 = lat[i1][:, i0] * (1 - f)[None, :] + lat[i1][:, i1] * f[None, :]
        out += amp * (rows * (1 - f)[:, None] + rows1 * f[:, None])
        tot += amp
        amp *= 0.5
    return out / tot


def _albedo_texture(rng, size, base, pattern):
    """RGBA8 base-colour texture: a tinted noise field with bricks / planks / tiles / plaster."""
    n = _value_noise(rng, size, 8)
    y, x = np.mgrid[0:size, 0:size].astype(np.float32) / size
    if pattern == 0:     # bricks
        row = np.floor(y * 32)
        mortar = ((y * 32) % 1 < 0.12) | (((x * 16 + 0.5 * (row % 2)) % 1) < 0.06)
        shade = 0.75 + 0.5 * n
        shade = np.where(mortar, 1.35, shade)
    elif pattern == 1:   # planks
        shade = 0.7 + 0.4 * n + 0.2 * np.sin(x * 60.0 + 6.0 * n)
    elif pattern == 2:   # tiles
        grout = ((x * 12) % 1 < 0.05) | ((y * 12) % 1 < 0.05)
        shade = np.where(grout, 0.5, 0.85 + 0.3 * n)
    else:                # plaster
        shade = 0.8 + 0.35 * n
    rgb = np.clip(np.asarray(base, np.float32)[None, None, :] * shade[..., None] * 255.0, 0, 255)
    t = np.empty((size, size, 4), np.uint8)
    t[..., :3] = rgb.astype(np.uint8)
    t[..., 3] = 255
    return t


def _normal_texture(rng, size, strength):
    """RGBA8 tangent-space normal map from the gradient of a noise height field."""
    h = _value_noise(rng, size, 16) * strength
    gx = np.roll(h, -1, 1) - np.roll(h, 1, 1)
    gy = np.roll(h, -1, 0) - np.roll(h, 1, 0)
    n = np.stack([-gx * size / 64.0, -gy * size / 64.0, np.ones_like(h)], -1)
    n /= np.linalg.norm(n, axis=-1, keepdims=True)
    t = np.empty((size, size, 4), np.uint8)
    t[..., :3] = np.clip(np.round((n * 0.5 + 0.5) * 255.0), 0, 255).astype(np.uint8)
    t[..., 3] = 255
    return t


def _rm_texture(rng, size, rough, metal):
    """RGB roughness-metallic texture (G roughness, B metallic, Material.h: the packed slot)."""
    n = _value_noise(rng, size, 8)
    t = np.zeros((size, size, 4), np.uint8)
    t[..., 1] = np.clip((rough + 0.3 * (n - 0.5)) * 255.0, 8, 255).astype(np.uint8)
    t[..., 2] = np.clip(metal * 255.0 * (n > 0.35), 0, 255).astype(np.uint8)
    t[..., 3] = 255
    return t


def procedural_city_textured(seed: int = 1235, tex_scale: float = 3.0) -> SceneData:
    """The C3 city with the texture load of a production exterior (the Bistro's materials are
    textured on most surfaces): 64 materials -- 48 facade materials (24 base-colour textures at
    1024^2 in 4 patterns, 8 normal maps at 1024^2, 8 roughness-metallic textures at 512^2), 8
    roof materials and textured asphalt / sidewalks at 2048^2 -- ~190 MB of RGBA8 textures,
    world-space planar texture coordinates (tex_scale metres per repeat).  Glass, lamps,
    foliage and the alpha-tested leaf cards keep the C3 materials."""
    sd = procedural_city(seed)
    rng = np.random.default_rng(seed + 101)
    V = np.asarray(sd.vertices, np.float32)
    I = np.asarray(sd.triangle_indices).reshape(-1, 3)
    M = np.asarray(sd.material_indices).copy()
    mats = list(sd.materials)
    textures = list(sd.textures)          # texture 0: the leaf cards' alpha texture

    def add_tex(t):
        textures.append(t)
        return len(textures) - 1

    palettes = [(0.62, 0.55, 0.45), (0.55, 0.25, 0.2), (0.7, 0.7, 0.72), (0.3, 0.35, 0.4), (0.5, 0.42, 0.3), (0.68, 0.6, 0.52)]
    albedo = [add_tex(_albedo_texture(rng, 1024, palettes[k % len(palettes)], k % 4)) for k in range(24)]
    normals = [add_tex(_normal_texture(rng, 1024, 2.0 + k)) for k in range(8)]
    rms = [add_tex(_rm_texture(rng, 512, 0.5 + 0.05 * k, 0.6 if k % 4 == 3 else 0.0)) for k in range(8)]

    def textured(base_tex, normal_tex, rm_tex, specular=0.5):
        m = _mat((1.0, 1.0, 1.0), rough=1.0, metallic=1.0, specular=specular)
        m.base_color_texture_index = base_tex
        m.normal_map_texture_index = normal_tex
        m.roughness_metallic_texture_index = rm_tex
        m.make_safe()
        m.precompute_properties()
        return m

    facade0 = len(mats)
    for k in range(48):
        mats.append(textured(albedo[k % 24], normals[(k * 5) % 8], rms[(k * 3) % 8]))
    roof0 = len(mats)
    for k in range(8):
        mats.append(textured(albedo[(3 * k + 1) % 24], normals[k], rms[(k + 2) % 8], specular=0.3))
    asphalt = len(mats)
    mats.append(textured(add_tex(_albedo_texture(rng, 2048, (0.09, 0.09, 0.095), 3)), add_tex(_normal_texture(rng, 2048, 4.0)),
                         rms[0], specular=0.3))
    sidewalk = len(mats)
    mats.append(textured(add_tex(_albedo_texture(rng, 2048, (0.5, 0.49, 0.47), 2)), normals[1], rms[1], specular=0.4))
    # reassign: each building's facade (C3 materials 2-5) one of the 48, roofs (7) one of 8
    tri_bld = rng.integers(0, 1 << 30, len(M))
    fac = np.isin(M, [2, 3, 4, 5])
    # one facade material per original wall material and 12 variants by position (blocks of 64 m)
    cen = V[I].mean(1)
    cell = (np.floor(cen[:, 0] / 64.0).astype(np.int64) * 7 + np.floor(cen[:, 2] / 64.0).astype(np.int64) * 13) % 12
    M[fac] = facade0 + (M[fac] - 2) * 12 + cell[fac]
    roof = M == 7
    M[roof] = roof0 + (tri_bld[roof] % 8) * 0 + (cell[roof] % 8)
    M[M == 0] = asphalt
    M[M == 1] = sidewalk
    # world-space planar texture coordinates by the dominant axis of the triangle's normal
    tn = np.cross(V[I[:, 1]] - V[I[:, 0]], V[I[:, 2]] - V[I[:, 0]])
    ax = np.argmax(np.abs(tn), 1)
    uv = np.asarray(sd.texcoords, np.float32).copy()
    retex = M >= facade0
    for a, (ui, vi) in enumerate([(2, 1), (0, 2), (0, 1)]):
        sel = retex & (ax == a)
        vid = np.unique(I[sel].reshape(-1))
        uv[vid, 0] = V[vid, ui] / tex_scale
        uv[vid, 1] = V[vid, vi] / tex_scale
    sd.texcoords = uv.astype(np.float32)
    sd.material_indices = M.astype(np.int32)
    sd.materials = mats
    sd.textures = textures
    sd.name = f"procedural_city_textured_{seed}"
    return sd.finalize()
