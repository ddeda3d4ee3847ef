"""Mesh I/O at the boundary (b, f2): readNode / readEle / readPoly against the
reference's own parses (the goldens' coords64 / coords32 / markers / tris / poly_*, produced by
running the reference's readers, tests/golden/gen_golden.py), the Triangle writers round-tripping
through them, and the refined-mesh tool (tools/make_mesh.py)."""
import os
import sys

import numpy as np
import pytest

from conftest import GOLDEN, load_pkg

pf = load_pkg()
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import make_mesh  # noqa: E402

REF = "/root/reference"
FILES = {
    "mesh1": ("code/mesh/mesh.1.node", "code/mesh/mesh.1.ele", "code/mesh/mesh.1.poly"),
    "mesh21": ("resources/mesh2.1.node", "resources/mesh2.1.ele", "resources/mesh2.1.poly"),
    "fine": ("resources/mesh_fine.1.node", "resources/mesh_fine.1.ele", "resources/mesh_fine.1.poly"),
}


def golden(name):
    return np.load(os.path.join(GOLDEN, f"golden_{name}.npz"))


@pytest.mark.parametrize("name", ["mesh1", "mesh21", "fine"])
def test_writer_roundtrip_matches_reference_parse(name, tmp_path):
    """write -> readNode / readEle / readPoly reproduces the reference's parse of the original
    files bit for bit: fp64 (StokesColor.py:54-78) and fp32 (poisson.py:27-56) coordinates,
    markers, 0-based triangles, segments."""
    g = golden(name)
    m = pf.load_mesh(name)
    node, ele, poly = (str(tmp_path / f"m.{e}") for e in ("node", "ele", "poly"))
    pf.writeNode(node, m.coords, m.markers, comment="round trip")
    pf.writeEle(ele, m.triangles)
    pf.writePoly(poly, m.segments, m.segment_markers)
    X, mk = pf.readNode(node)
    assert X.dtype == np.float64 and mk.dtype == np.int32
    np.testing.assert_array_equal(X, g["coords64"])
    np.testing.assert_array_equal(mk, g["markers"])
    X32, mk32 = pf.readNode(node, np.float32)
    assert X32.dtype == np.float32
    np.testing.assert_array_equal(X32, g["coords32"])
    np.testing.assert_array_equal(mk32, g["markers"])
    T = pf.readEle(ele)
    assert T.dtype == np.int32
    np.testing.assert_array_equal(T, g["tris"])
    if "poly_segments" in g.files:
        seg, segm = pf.readPoly(poly)
        np.testing.assert_array_equal(seg, g["poly_segments"])
        np.testing.assert_array_equal(segm, g["poly_markers"])


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkout not present (build container only)")
@pytest.mark.parametrize("name", ["mesh1", "mesh21", "fine"])
def test_readers_on_the_reference_files(name):
    """Our readers on the reference's original Triangle files (read as data) = the reference's parse."""
    g = golden(name)
    node, ele, poly = (os.path.join(REF, p) for p in FILES[name])
    X, mk = pf.readNode(node)
    np.testing.assert_array_equal(X, g["coords64"])
    np.testing.assert_array_equal(mk, g["markers"])
    np.testing.assert_array_equal(pf.readNode(node, np.float32)[0], g["coords32"])
    np.testing.assert_array_equal(pf.readEle(ele), g["tris"])
    if "poly_segments" in g.files:
        seg, segm = pf.readPoly(poly)
        np.testing.assert_array_equal(seg, g["poly_segments"])
        np.testing.assert_array_equal(segm, g["poly_markers"])


@pytest.mark.parametrize("level", [1, 2])
def test_refined_mesh_tool(level, tmp_path):
    """tools/make_mesh.py: the refined mesh as Triangle files reads back exactly as the in-memory
    refinement; the refined boundary segments tile the coarse ones (2^L pieces each, endpoints
    chained, all on the boundary)."""
    node, ele, poly = make_mesh.write_mesh("fine", level, str(tmp_path))
    m = pf.load_mesh("fine", refine=level)
    X, mk = pf.readNode(node)
    np.testing.assert_array_equal(X, m.coords)
    np.testing.assert_array_equal(mk, m.markers)
    np.testing.assert_array_equal(pf.readEle(ele), m.triangles)
    seg, segm = pf.readPoly(poly)
    base = pf.load_mesh("fine")
    assert len(seg) == len(base.segments) * 2 ** level
    k = 2 ** level
    for s in range(len(base.segments)):
        piece = seg[s * k:(s + 1) * k]
        assert piece[0, 0] == base.segments[s, 0] and piece[-1, 1] == base.segments[s, 1]
        assert np.array_equal(piece[1:, 0], piece[:-1, 1])
        assert (segm[s * k:(s + 1) * k] == base.segment_markers[s]).all()
    # every segment node is a boundary node of the refined mesh
    assert (mk[np.unique(seg)] != 0).all()


def test_refined_levels_node_counts():
    """The benchmark meshes' sizes: L5 = 894,208 and L7 = 14,230,528 nodes follow
    from N_L = N + E (edges) per level; checked on L1..L3 against Euler's formula (T_L = 4^L T)."""
    base = pf.load_mesh("fine")
    for level in (1, 2, 3):
        m = pf.load_mesh("fine", refine=level)
        assert m.T == base.T * 4 ** level
        # Euler for a planar triangulation with h holes: N - E + T = 1 - h (+ the outer face)
        E = (3 * m.T + len(base.segments) * 2 ** level) // 2
        E0 = (3 * base.T + len(base.segments)) // 2
        assert m.N - E + m.T == base.N - E0 + base.T
