"""Camera matrices (mpt.scene.make_camera vs Camera::to_hiprt, Camera.cpp:9-26).

The reference stores glm's column-major matrices reinterpreted as row-major and multiplies
points on the right (matrix_X_point, Math.h:237-254).  The camera ray of a pixel
(HIPRTCamera.h:27-47) and the temporal reprojection of ReSTIR DI (find_temporal_neighbor_index,
Utils.h:426-437) use those matrices; with the reference's conventions a first hit reprojects
onto its own pixel (static camera), so temporal reuse finds the pixel itself.  A wrong
view_projection (e.g. the transposed product) maps every point to the same pixel and silently
disables temporal reuse -- GPU and oracle would still agree, so this is pinned here."""
import numpy as np
import pytest

from mpt import scene, synthetic


def _mxp(m, p):
    """matrix_X_point: row-major m times (p, 1), divided by w unless w is zero."""
    v = m @ np.array([p[0], p[1], p[2], 1.0])
    return v[:3] / v[3] if v[3] != 0 else v[:3]


def _mat(m):
    return np.array([[m.m[i][j] for j in range(4)] for i in range(4)], np.float64)


@pytest.mark.parametrize("res", [(1920, 1080), (256, 256), (640, 360)])
@pytest.mark.parametrize("which", ["city", "cornell_pbr"])
def test_first_hit_reprojects_onto_its_pixel(res, which):
    W, H = res
    sd = synthetic.procedural_city(1234) if which == "city" else scene.load_scene(which)
    cam = scene.make_camera(sd.camera_info, W, H)
    iv, ip, vp = _mat(cam.inverse_view), _mat(cam.inverse_projection), _mat(cam.view_projection)
    rng = np.random.default_rng(7)
    for _ in range(64):
        x, y = rng.uniform(0, W), rng.uniform(0, H)
        # get_camera_ray (HIPRTCamera.h:27-47)
        o = _mxp(iv, [0.0, 0.0, 0.0])
        pd = _mxp(iv, _mxp(ip, [x / W * 2 - 1, y / H * 2 - 1, -1.0]))
        d = (pd - o) / np.linalg.norm(pd - o)
        p = o + rng.uniform(0.5, 50.0) * d
        # find_temporal_neighbor_index's reprojection (Utils.h:428-437)
        ss = _mxp(vp, p)
        fx = (ss[0] + 1.0) * 0.5 * W - 0.5
        fy = (ss[1] + 1.0) * 0.5 * H - 0.5
        assert abs(fx - (x - 0.5)) < 1e-2 and abs(fy - (y - 0.5)) < 1e-2, (x, y, fx, fy)
