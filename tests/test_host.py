"""CPU: host-side inputs of the path — orbit camera (camera.cpp), TF gradient model
(gradient.cpp + ImGui packing), NRRD reader pinned by the reference's own NrrdIO, CSV loader."""
import hashlib
import json
import os

import numpy as np
import pytest

import pyoracle
import synth
import vr_amd

GOLD = os.path.join(os.path.dirname(__file__), "golden")


# ---------------------------------------------------------------------------- camera
def quat_mul(p, q):
    w1, x1, y1, z1 = p
    w2, x2, y2, z2 = q
    return np.array([w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2, w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                     w1 * y2 + y1 * w2 + z1 * x2 - x1 * z2, w1 * z2 + z1 * w2 + x1 * y2 - y1 * x2])


def quat_rot(q, v):
    w, x, y, z = q
    R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                  [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                  [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])
    return R @ v


def axis_angle(deg, axis):
    a = np.radians(deg)
    return np.concatenate([[np.cos(a / 2)], np.asarray(axis, float) * np.sin(a / 2)])


def test_default_camera():
    c = vr_amd.OrbitCamera()
    # orientation 180 deg about z: camera at (0, -3, 0) looking along +y (camera.cpp:7-13, 36-40)
    assert c.get_position() == pytest.approx([0, -3, 0], abs=1e-6)
    V = c.get_view().reshape(4, 4).T  # row-major
    o = V @ np.array([0, 0, 0, 1.0])
    assert o[:3] == pytest.approx([0, -3, 0], abs=1e-5)
    # coordinate_conversion Rx(90) * S(-1,1,1) (offscreen_pass.cpp:1159-1162) puts it at eye z = -3
    Rx = np.array([[1, 0, 0], [0, 0, -1], [0, 1, 0.0]])
    assert Rx @ np.diag([-1, 1, 1.0]) @ o[:3] == pytest.approx([0, 0, -3], abs=1e-5)


@pytest.mark.parametrize("deltas", [[(100, 60)], [(-300, -150)], [(10, 0), (0, 20), (-45, 33)]])
def test_camera_rotate_matches_float64_quaternions(deltas):
    c = vr_amd.OrbitCamera()
    q = axis_angle(180, [0, 0, 1])
    for dx, dy in deltas:
        c.rotate(dx, dy)
        q = quat_mul(axis_angle(-dx * 0.25, [0, 0, 1]), q)
        right = quat_rot(q, np.array([1.0, 0, 0]))
        q = quat_mul(axis_angle(dy * 0.25, right), q)
    pos = 3.0 * quat_rot(q, np.array([0, 1.0, 0]))
    assert c.get_position() == pytest.approx(pos, abs=2e-5)
    V = c.get_view().reshape(4, 4).T
    R = np.array([quat_rot(q, e) for e in np.eye(3)])  # rows = rotated basis = R^T
    assert V[:3, :3] == pytest.approx(R, abs=2e-5)
    assert V[:3, 3] == pytest.approx(-R @ pos, abs=2e-5)


def test_camera_zoom_clamps():
    c = vr_amd.OrbitCamera()
    c.zoom(2.5)
    assert c.radius == pytest.approx(0.5)
    c.zoom(5)
    assert c.radius == pytest.approx(0.1)   # clamp [0.1, 10] (camera.cpp:33)
    c.zoom(-50)
    assert c.radius == pytest.approx(10.0)


# ---------------------------------------------------------------------------- gradient
def imgui_pack(rgba):
    sat = lambda v: int(min(max(v, 0.0), 1.0) * 255.0 + 0.5)
    return sat(rgba[0]) | sat(rgba[1]) << 8 | sat(rgba[2]) << 16 | sat(rgba[3]) << 24


def _product_gradient(m):
    """vr_gradient_* (the product's TF producer) with the given markers, built through the
    marker API the UI uses (set the two end markers, add the inner ones)."""
    g = vr_amd.Gradient()
    c, a = m["color_markers"], m["alpha_markers"]
    g.set_color_marker(0, c[0][0], c[0][1])
    g.set_color_marker(1, c[-1][0], c[-1][1])
    for loc, rgb in c[1:-1]:
        i = g.add_color_marker(loc, rgb)
        g.set_color_marker(i, loc, rgb)
    g.set_alpha_marker(0, a[0][0], a[0][1])
    g.set_alpha_marker(1, a[-1][0], a[-1][1])
    for loc, al in a[1:-1]:
        i = g.add_alpha_marker(loc, al)
        g.set_alpha_marker(i, loc, al)
    return g


@pytest.mark.parametrize("name", ["tf1_256", "tf2_256", "tf_color_256", "tf1_7", "tf2_7", "tf_color_7"])
def test_gradient_discretize_matches_golden_texels(name):
    """Row f2: the product's Gradient::discretize equals, texel for texel, the golden vectors
    of tests/golden/tf_golden.json -- an independent float32 restatement of gradient.cpp:64-108
    (accumulated texel-centre locations), sample_markers (:471-485), lerp (:13-16) and ImGui's
    published IM_F32_TO_INT8_SAT packing (tools/make_tf_golden.py).  TF-1 is the default
    Gradient(), TF-2 the demo ramp, both as the benchmark uses them."""
    gold = json.load(open(os.path.join(GOLD, "tf_golden.json")))[name]
    tf = _product_gradient(gold).discretize(gold["count"])
    assert tf.tolist() == gold["texels"]


def test_tf_golden_fixture_is_reproducible():
    import make_tf_golden
    built = json.loads(json.dumps(make_tf_golden.build()))
    assert built == json.load(open(os.path.join(GOLD, "tf_golden.json")))


def test_default_gradient_discretize():
    tf = vr_amd.Gradient().discretize(256)
    assert np.array_equal(tf, synth.tf1())
    # texel centres, black -> white, alpha 1 (gradient.cpp:64-70, 90-108)
    assert all((t >> 24) == 255 for t in tf)
    assert (tf & 0xFF).tolist() == sorted((tf & 0xFF).tolist())
    assert tf[0] & 0xFF == 0 and tf[255] & 0xFF == 255


def test_gradient_markers_semantics():
    g = vr_amd.Gradient()
    assert g.add_alpha_marker(0.5, 0.2) == 1
    assert g.marker_count(True) == 3
    assert g.sample(0.25)[3] == pytest.approx(0.6)
    assert g.sample(0.5)[3] == pytest.approx(0.2)
    # first/last markers cannot be removed (gradient.cpp:506-515)
    assert not g.remove_alpha_marker(0) and not g.remove_alpha_marker(2)
    assert g.remove_alpha_marker(1) and g.marker_count(True) == 2
    # add at location 0 goes after the first marker (add_marker :496-498)
    assert g.add_color_marker(0.0, (1, 0, 0)) == 1
    # ends keep their location when edited (:386-400); an edited inner marker is re-sorted
    assert g.set_color_marker(0, 0.7, (0, 1, 0)) == 0
    assert g.sample(0.0)[:3] == pytest.approx([0, 1, 0])
    i = g.add_color_marker(0.3, (0, 0, 1))
    assert g.set_color_marker(i, 0.9, (0, 0, 1)) == 2  # moved past the 0.0 marker? list: 0,0,0.3->0.9
    assert g.marker_count(False) == 4


def test_tf2_matches_demo_markers():
    import synth
    tf = synth.tf2()
    a = (tf >> 24) & 0xFF
    loc = (np.arange(256) + 0.5) / 256
    want = np.where(loc <= 0.14, 0.0, (loc - 0.14) / 0.86)
    assert np.abs(a - (want * 255 + 0.5).astype(int)).max() <= 1


# ---------------------------------------------------------------------------- NRRD
def nrrd_expect():
    return json.load(open(os.path.join(GOLD, "nrrd", "expect.json")))


NRRD_TYPE_TO_VR = {1: 1, 2: 2, 3: 3, 4: 4, 5: 5, 6: 6, 7: 7, 8: 8, 9: 9, 10: 10}


@pytest.mark.parametrize("fname", sorted(json.load(open(os.path.join(GOLD, "nrrd", "expect.json")))))
def test_nrrd_reader_matches_reference_nrrdio(fname):
    """Our reader vs the reference's NrrdIO (golden, generated by oracle/_ref) on every fixture."""
    exp = nrrd_expect()[fname]
    path = os.path.join(GOLD, "nrrd", fname)
    if exp["rc"] != 0:
        with pytest.raises(RuntimeError):
            vr_amd.load_nrrd(path)
        return
    ds = vr_amd.load_nrrd(path)
    assert list(ds.dims) == exp["dims"]
    assert ds.vmin == exp["vmin"] and ds.vmax == exp["vmax"]
    f32 = ds.data.astype(np.float32)
    assert hashlib.sha256(f32.tobytes()).hexdigest() == exp["sha256_f32"]
    if pyoracle.nrrdio_available():  # live cross-check when the reference build is present
        rc, res = pyoracle.nrrdio_load(path)
        assert rc == 0 and np.array_equal(res["data"], f32)


def test_nrrd_roundtrip_writer(tmp_path):
    rng = np.random.default_rng(0)
    for dt in (np.uint8, np.int16, np.float32, np.float64):
        a = (rng.standard_normal((3, 4, 5)) * 50).astype(dt)
        p = str(tmp_path / f"v_{np.dtype(dt).name}.nhdr")
        vr_amd.write_nrrd_raw(p, a)
        ds = vr_amd.load_nrrd(p)
        assert ds.dims == (5, 4, 3) and ds.data.dtype == dt and np.array_equal(ds.data, a)
        assert ds.vmin == float(a.astype(np.float32).min())
        if pyoracle.nrrdio_available():
            rc, res = pyoracle.nrrdio_load(p)
            assert rc == 0 and np.array_equal(res["data"], a.astype(np.float32))


def test_nrrd_large_raw_parallel_read_and_minmax(tmp_path):
    """Raw payloads >= 64 MiB are read (pread) and reduced by chunks on up to 16 threads.  The
    result must be the sequential one (nrrd_file_parser.cpp:39-40 min/max_element over floats):
    a NaN first element stays, later NaNs never enter, equal values keep the first occurrence
    (0.0 / -0.0), and a truncated payload still fails."""
    n = 24 << 20  # 96 MiB of float32, 24 MiB of uint8 x 4
    rng = np.random.default_rng(11)
    u8 = rng.integers(3, 250, size=(96, 1024, 1024), dtype=np.uint8)
    u8[95, 1023, 1023] = 255
    u8[40, 7, 9] = 1
    p = str(tmp_path / "u8.nhdr")
    vr_amd.write_nrrd_raw(p, u8)
    ds = vr_amd.load_nrrd(p)
    assert np.array_equal(ds.data, u8) and (ds.vmin, ds.vmax) == (1.0, 255.0)

    base = (rng.random(n, dtype=np.float32) + 1.0).reshape(96, 512, 512)
    chunk = n // 16
    cases = []
    a = base.copy().ravel()
    a[[chunk, 3 * chunk, n - 1]] = np.nan  # NaNs at chunk starts and the end
    a[5 * chunk + 3] = 0.25
    a[7 * chunk] = 7.5
    cases.append((a, 0.25, 7.5, None))
    a = base.copy().ravel()
    a[0] = np.nan  # NaN first: both results NaN
    cases.append((a, np.nan, np.nan, None))
    a = base.copy().ravel()
    a[5], a[9 * chunk + 1] = 0.0, -0.0  # first occurrence of the minimum wins
    cases.append((a, 0.0, None, False))
    a = base.copy().ravel()
    a[2 * chunk + 17], a[9 * chunk] = -0.0, 0.0
    cases.append((a, 0.0, None, True))
    for i, (arr, lo, hi, signbit) in enumerate(cases):
        p = str(tmp_path / f"f{i}.nhdr")
        vr_amd.write_nrrd_raw(p, arr.reshape(96, 512, 512))
        ds = vr_amd.load_nrrd(p)
        assert np.array_equal(ds.data.view(np.uint32), arr.reshape(96, 512, 512).view(np.uint32))
        if np.isnan(lo):
            assert np.isnan(ds.vmin) and np.isnan(ds.vmax)
            continue
        assert ds.vmin == lo, i
        if hi is not None:
            assert ds.vmax == hi, i
        if signbit is not None:
            assert bool(np.signbit(np.float32(ds.vmin))) == signbit, i

    # attached header + payload in one file, and a truncated payload
    hdr = b"NRRD0004\ntype: uint8\ndimension: 3\nsizes: 1024 1024 96\nencoding: raw\n\n"
    p = tmp_path / "att.nrrd"
    p.write_bytes(hdr + u8.tobytes())
    ds = vr_amd.load_nrrd(str(p))
    assert np.array_equal(ds.data, u8) and (ds.vmin, ds.vmax) == (1.0, 255.0)
    p.write_bytes(hdr + u8.tobytes()[:-1])
    with pytest.raises(RuntimeError, match="Failed to read file"):
        vr_amd.load_nrrd(str(p))


def test_nrrd_missing_file():
    with pytest.raises(RuntimeError, match="Failed to read file"):
        vr_amd.load_nrrd("/nonexistent/file.nhdr")


# ---------------------------------------------------------------------------- CSV
def test_csv_loader(tmp_path):
    files = []
    for z in range(3):
        p = tmp_path / f"s{z}.csv"
        p.write_text("\n".join(",".join(str(z * 100 + y * 10 + x + 1) for x in range(4)) for y in range(2)) + "\n")
        files.append(str(p))
    ds = vr_amd.load_csv(files)
    assert ds.dims == (4, 2, 3)
    assert ds.data[2, 1, 3] == 214.0
    assert ds.vmin == 0.0 and ds.vmax == 214.0   # min seeded at 0 by Dataset{} (csv_file_parser.cpp:16)
    bad = tmp_path / "bad.csv"
    bad.write_text("1,2,3\n4,5\n")
    with pytest.raises(RuntimeError, match="Inconsistant dimensions"):
        vr_amd.load_csv([str(bad)])


def test_csv_loader_edge_cases(tmp_path):
    """csv_file_parser.cpp:14-50 semantics: a trailing ',' adds no field, an empty field is a
    std::stof error, std::stof reads a numeric prefix, negative values lower the 0-seeded min,
    a slice with another row count is rejected."""
    def w(name, text):
        p = tmp_path / name
        p.write_text(text)
        return str(p)
    ds = vr_amd.load_csv([w("a.csv", "1,2,\n-3,4.5x,\n"), w("b.csv", "  5,6\n7,8\n")])
    assert ds.dims == (2, 2, 2)
    assert ds.data.ravel().tolist() == [1, 2, -3, 4.5, 5, 6, 7, 8]
    assert ds.vmin == -3.0 and ds.vmax == 8.0
    with pytest.raises(RuntimeError):
        vr_amd.load_csv([w("c.csv", "1,,2\n")])
    with pytest.raises(RuntimeError, match="Inconsistant dimensions"):
        vr_amd.load_csv([w("d.csv", "1,2\n3,4\n"), w("e.csv", "1,2\n")])
    with pytest.raises(RuntimeError, match="Inconsistant dimensions"):
        vr_amd.load_csv([w("f.csv", "1,2\n\n3,4\n")])
