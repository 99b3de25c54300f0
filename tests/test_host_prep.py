"""Host scene preparation (librtscene.so) against the reference's own numbers.

Pins: BVH node/leaf/depth counts measured from the reference src/core/BVH.h (SURVEY §8(c),
tests/golden/bvh_counts.json); the HDR decode against the reference hdrloader built from its
own sources (tests/golden/hdr_ref.json, and live against oracle/_ref when present).
"""
import hashlib
import json
import subprocess
import tempfile
from pathlib import Path

import numpy as np
import pytest

from conftest import REFERENCE, ROOT, have_reference
from rtamd import configs as cf
from rtamd import scene_lib as sl

GOLD = ROOT / "tests" / "golden"


def _raw_scene(name):
    m = cf.load_mesh(name)
    pos, _, idx = m.data()
    s = sl.Scene()
    s.add_triangles(pos[idx].reshape(-1, 9), sl.Material())
    s.build_bvh(8)
    return s


@pytest.mark.parametrize("name,key", [("bunny_4000", "raw_bunny_4000"), ("loong_100000", "raw_loong_100000")])
def test_raw_mesh_bvh_counts_match_reference(name, key):
    g = json.loads((GOLD / "bvh_counts.json").read_text())[key]
    c = _raw_scene(name).counts()
    assert (c["n_triangles"], c["n_nodes"], c["n_leaves"]) == (g["triangles"], g["nodes"], g["leaves"])


@pytest.mark.parametrize("cfg,key", [("C2", "C2_scene"), ("C3", "C3_scene")])
def test_config_scene_bvh_counts_match_reference(cfg, key):
    g = json.loads((GOLD / "bvh_counts.json").read_text())[key]
    c = cf.config_scene(cfg).counts
    assert (c["n_triangles"], c["n_nodes"], c["max_depth"]) == (g["triangles"], g["nodes"], g["max_depth"])


@pytest.mark.parametrize("cfg", ["C2", "C3"])
def test_scene_encoding_regression(cfg):
    g = json.loads((GOLD / "scene_hashes.json").read_text())[cfg]
    sd = cf.config_scene(cfg)
    assert hashlib.sha256(sd.tri_enc.tobytes()).hexdigest() == g["tri_enc"]
    assert hashlib.sha256(sd.node_enc.tobytes()).hexdigest() == g["node_enc"]


def test_bvh_structure_invariants():
    sd = cf.config_scene("C2")
    nd = sd.nodes
    n_tri = sd.counts["n_triangles"]
    covered = np.zeros(n_tri, np.int32)
    tri = sd.tri_enc[:, :3, :]  # positions
    stack = [1]
    while stack:
        i = stack.pop()
        if nd["n"][i] > 0:
            assert nd["n"][i] <= 8
            a, b = nd["index"][i], nd["index"][i] + nd["n"][i]
            covered[a:b] += 1
            pts = tri[a:b].reshape(-1, 3)
            assert np.all(pts >= nd["aa"][i] - 0) and np.all(pts <= nd["bb"][i] + 0)
            continue
        for c in (nd["left"][i], nd["right"][i]):
            assert c > 0
            assert np.all(nd["aa"][c] >= nd["aa"][i]) and np.all(nd["bb"][c] <= nd["bb"][i])
            stack.append(c)
    assert np.all(covered == 1)
    # the dummy node 0 of src/core/Scene.h:189-195
    assert (nd["left"][0], nd["right"][0], nd["n"][0]) == (255, 128, 30)


def test_triangle_encoding_layout():
    sd = cf.config_scene("C2")
    t = sd.tri_enc
    lo, hi = sd.ranges[1]
    post = np.argsort(np.zeros(1))  # placeholder to keep numpy import used
    # every bunny triangle carries jade (texels 6..13, src/core/Triangle.h:31-38)
    jade = cf.MATERIALS["jade"].texels().reshape(8, 3)
    plane = cf.MATERIALS["plane"].texels().reshape(8, 3)
    mats = t[:, 6:14, :]
    is_jade = np.all(mats == jade, axis=(1, 2))
    is_plane = np.all(mats == plane, axis=(1, 2))
    assert is_jade.sum() == hi - lo and is_plane.sum() == 2 and np.all(is_jade | is_plane)
    # flat normals: n1 == n2 == n3 == normalize(cross(p2-p1, p3-p1)) (src/core/Triangle.h:109-114)
    assert np.array_equal(t[:, 3], t[:, 4]) and np.array_equal(t[:, 4], t[:, 5])
    assert len(post) == 1


def test_smooth_normals_unit_and_shared():
    m = cf.load_mesh("loong_100000")
    pos, nrm, idx = m.data()
    ln = np.linalg.norm(nrm, axis=1)
    assert np.allclose(ln, 1.0, atol=1e-5)
    # corners at the same position share one normal (GenSmoothNormals, no angle limit)
    key = {}
    for p, n in zip(map(tuple, pos[:3000]), nrm[:3000]):
        if p in key:
            assert np.array_equal(key[p], n)
        key[p] = n


def test_floor_quad_triangulation():
    m = cf.load_mesh("floor")
    pos, _, idx = m.data()
    tris = pos[idx].reshape(-1, 3, 3)
    assert tris.shape == (2, 3, 3)
    # f 1 2 4 3 -> (v1, v2, v4), (v1, v4, v3)
    assert np.array_equal(tris[0], [[-10, 0, 10], [10, 0, 10], [10, 0, -10]])
    assert np.array_equal(tris[1], [[-10, 0, 10], [10, 0, -10], [-10, 0, -10]])


@pytest.mark.skipif(not have_reference(), reason="reference checkout absent")
@pytest.mark.parametrize("name", ["floor", "bunny_4000", "loong_100000"])
def test_assets_equal_obj_parse(name):
    raw = sl.parse_obj_raw(str(REFERENCE / "resources" / "objects" / f"{name}.obj"), 0)
    asset = cf.load_raw_mesh(name)
    assert np.array_equal(raw.positions, asset.positions)
    assert np.array_equal(raw.pos_index, asset.pos_index)
    assert np.array_equal(raw.face_sizes, asset.face_sizes)


@pytest.mark.skipif(not have_reference(), reason="reference checkout absent")
def test_assimp_parse_mode_differs_only_in_last_ulps():
    path = str(REFERENCE / "resources" / "objects" / "bunny_4000.obj")
    a = sl.parse_obj_raw(path, 0).positions
    b = sl.parse_obj_raw(path, 1).positions
    ulps = np.abs(a.view(np.int32).astype(np.int64) - b.view(np.int32).astype(np.int64))
    assert ulps.max() <= 2


def test_hdr_decode_matches_reference_fixture():
    g = json.loads((GOLD / "hdr_ref.json").read_text())
    img, _ = cf.load_env()
    assert img.shape == (g["height"], g["width"], 3)
    assert hashlib.sha256(img.tobytes()).hexdigest() == g["sha256"]
    flat = img.reshape(-1, 3)
    for i, bits in zip(g["sample_index"], g["sample_bits"]):
        assert [int(b) for b in flat[i].view(np.uint32)] == bits
    assert float(img.max()) == g["max"]


def test_hdr_decode_matches_reference_build_live():
    exe = ROOT / "oracle" / "_ref" / "ref_hdr_dump"
    if not exe.exists():
        pytest.skip("oracle/_ref not built (reference absent)")
    with tempfile.TemporaryDirectory() as td:
        out = Path(td) / "o.bin"
        subprocess.run([str(exe), str(ROOT / "assets" / cf.HDR_ASSET), str(out)], check=True)
        raw = out.read_bytes()
    w, h = np.frombuffer(raw[:8], np.int32)
    ref = np.frombuffer(raw[8:], np.float32).reshape(h, w, 3)
    img, _ = cf.load_env()
    assert np.array_equal(img.view(np.uint32), ref.view(np.uint32))


def test_hdr_cache_properties():
    img, cache = cf.load_env()
    h, w, _ = img.shape
    assert abs(float(cache[..., 2].astype(np.float64).sum()) - 1.0) < 1e-3
    assert cache[..., 0].min() >= 0 and cache[..., 0].max() < 1
    assert cache[..., 1].min() >= 0 and cache[..., 1].max() < 1
    # sample positions are multiples of 1/W and 1/H
    assert np.allclose(cache[..., 0] * w, np.round(cache[..., 0] * w), atol=1e-3)
    # brighter texels are sampled more often: the histogram of sampled x follows the marginal
    xs = np.round(cache[..., 0].ravel() * w).astype(int)
    hist = np.bincount(xs, minlength=w) / xs.size
    marg = cache[..., 2].sum(axis=0)
    assert np.corrcoef(hist, marg)[0, 1] > 0.9  # 512 quantised xi_1 values per column


def test_camera_basis():
    cam = sl.camera(-87.78, -14.0, 30.0, 1920 / 1080)
    f, r, u = cam["front"], cam["right"], cam["up"]
    for v in (f, r, u):
        assert abs(np.linalg.norm(v) - 1) < 1e-6
    assert abs(f @ r) < 1e-6 and abs(f @ u) < 1e-6 and abs(r @ u) < 1e-6
    assert abs(cam["half_h"] - np.tan(np.radians(30))) < 1e-6
    assert abs(cam["half_w"] - cam["half_h"] * 1920 / 1080) < 1e-5


def test_rand_origins_fixture_matches_glibc():
    live = sl.cpu_rand_origins(cf.RAND_SEED, 64)
    assert np.array_equal(live, cf.rand_origins(64))
    assert np.all((live >= 674764.0) & (live < 2 * 674764.0))


def test_material_update_post_bvh():
    s = sl.Scene()
    s.add_mesh(cf.load_mesh("floor"), cf.MATERIALS["plane"], (0, 0, 0), (2.2, -2, 3), (14, 7, 7))
    lo, hi = s.add_mesh(cf.load_mesh("bunny_4000"), cf.MATERIALS["jade"], (0, 0, 0), (2.2, -2.5, 3), (2, 2, 2))
    s.build_bvh(8)
    post = s.post_bvh_index()
    bunny_post = np.sort(post[lo:hi])
    # the bunny's post-BVH indices are not one contiguous range in general; update them one by one
    for i in bunny_post[:10]:
        s.set_material(int(i), 1, cf.MATERIALS["golden"])
    tri, _ = s.encode()
    golden = cf.MATERIALS["golden"].texels().reshape(8, 3)
    assert np.all(np.all(tri[bunny_post[:10], 6:14] == golden, axis=(1, 2)))
    soa = s.export_soa()
    assert len(soa["materials"]) == 3


def test_fast_bvh_build_equals_literal_restatement(monkeypatch):
    """The parallel index-sort SAH build (default) produces byte-identical triangles and nodes
    to the line-by-line restatement of buildBVHwithSAH (src/core/BVH.h:110-241)."""
    import hashlib
    from rtamd import scene_lib as sl

    def build(literal):
        monkeypatch.setenv("RTS_BVH_LITERAL", "1" if literal else "0")
        s = sl.Scene()
        for o in cf.CONFIGS["C3"].objects:
            s.add_mesh(cf.load_mesh(o.mesh), cf.MATERIALS[o.material], o.rotate, o.translate, o.scale, o.smooth)
        s.build_bvh(8)
        tri, nodes = s.encode()
        return hashlib.sha256(tri.tobytes()).hexdigest(), hashlib.sha256(nodes.tobytes()).hexdigest()

    assert build(True) == build(False)
