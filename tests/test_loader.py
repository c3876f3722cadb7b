"""The NeRF dataset front end (ngp::load_nerf, src/nerf_loader.cu:273-743) on the reference's own
datasets, on the CPU (pyngp.load_nerf_dataset needs no GPU):

* data/nerf/fox -- the reference's transforms.json verbatim: JPG frames, OpenCV lens (k1, k2, p1,
  p2), per-axis focal lengths, principal point cx/w, cy/h, aabb_scale 4, and 17 listed frames
  whose files are absent (skipped by the sharpness/exists filter, nerf_loader.cu:364-387);
* data/nerf/test/dataset -- the reference's BlenderNeRF scene (half resolution, see
  tools/make_real_data.py), aabb_scale 1, opaque RGBA.

Transforms are checked against an independent numpy restatement of nerf_matrix_to_ngp
(nerf_loader.h:100-120); focal lengths, lens parameters and the frame set against the json.
"""
import json
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FOX = os.path.join(ROOT, "data", "nerf", "fox")
TEST = os.path.join(ROOT, "data", "nerf", "test", "dataset")


def natural_key(s):
    return [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", s)]


def nerf_to_ngp(m, scale=0.33, offset=(0.5, 0.5, 0.5)):
    x = np.asarray(m, np.float64)[:3, :4].copy()
    x[:, 1] *= -1
    x[:, 2] *= -1
    x[:, 3] = x[:, 3] * scale + np.asarray(offset)
    return x[[1, 2, 0], :]  # cycle axes xyz <- yzx


@pytest.fixture(scope="module")
def ngp():
    import pyngp
    return pyngp


def test_fox_transforms_opencv_lens_and_missing_frames(ngp):
    meta = json.load(open(os.path.join(FOX, "transforms.json")))
    frames = sorted(meta["frames"], key=lambda f: natural_key(f["file_path"]))
    present = [f for f in frames if os.path.exists(os.path.join(FOX, f["file_path"]))]
    assert len(frames) == 67 and len(present) == 50
    d = ngp.load_nerf_dataset(os.path.join(FOX, "transforms.json"))
    assert d.n_images == 50 and d.aabb_scale == 4
    assert list(d.paths) == [f["file_path"] for f in present]
    for i, f in enumerate(present):
        np.testing.assert_allclose(d.transforms[i], nerf_to_ngp(f["transform_matrix"]), atol=2e-6)
    md = d.metadata[0]
    assert list(md.resolution) == [1080, 1920]
    np.testing.assert_allclose(md.focal_length, [meta["fl_x"], meta["fl_y"]], rtol=1e-6)
    np.testing.assert_allclose(md.principal_point, [meta["cx"] / meta["w"], meta["cy"] / meta["h"]], rtol=1e-6)
    assert md.lens.mode == ngp.LensMode.OpenCV
    np.testing.assert_allclose(md.lens.params[:4], [meta["k1"], meta["k2"], meta["p1"], meta["p2"]], rtol=1e-6)
    # JPG decode (PIL through the Testbed's decoder hook; stb_image in the reference)
    from PIL import Image
    img = d.image(0)
    ref = np.asarray(Image.open(os.path.join(FOX, present[0]["file_path"])).convert("RGBA"))
    np.testing.assert_array_equal(img, ref)


def test_test_dataset_split_and_intrinsics(ngp):
    d = ngp.load_nerf_dataset(os.path.join(TEST, "transforms_train.json"))
    t = ngp.load_nerf_dataset(os.path.join(TEST, "transforms_test.json"))
    assert d.n_images == 45 and t.n_images == 5 and d.aabb_scale == 1
    assert not set(d.paths) & set(t.paths)
    meta = json.load(open(os.path.join(TEST, "transforms_train.json")))
    md = d.metadata[3]
    assert list(md.resolution) == [360, 640]
    np.testing.assert_allclose(md.focal_length, [meta["fl_x"], meta["fl_y"]], rtol=1e-6)
    np.testing.assert_allclose(md.principal_point, [0.5, 0.5], rtol=1e-6)
    assert md.lens.mode == ngp.LensMode.Perspective
    frames = sorted(meta["frames"], key=lambda f: natural_key(f["file_path"]))
    for i in (0, 17, 44):
        np.testing.assert_allclose(d.transforms[i], nerf_to_ngp(frames[i]["transform_matrix"]), atol=2e-6)
    img = d.image(0)
    assert img.shape == (640, 360, 4) and img[..., 3].min() == 255


def test_directory_merges_every_json(ngp):
    """A scene directory loads every *.json in it (src/testbed_nerf.cu:2243-2248)."""
    d = ngp.load_nerf_dataset(TEST)
    assert d.n_images == 45 + 5 + 50  # transforms_all + transforms_test + transforms_train


def test_missing_files_and_empty_sets_raise(ngp, tmp_path):
    with pytest.raises(RuntimeError, match="does not exist"):
        ngp.load_nerf_dataset(str(tmp_path / "nope.json"))
    (tmp_path / "t.json").write_text(json.dumps({"camera_angle_x": 0.7, "frames": [
        {"file_path": "missing.png", "transform_matrix": np.eye(4).tolist()}]}))
    with pytest.raises(RuntimeError, match="Could not find image file"):
        ngp.load_nerf_dataset(str(tmp_path / "t.json"))
    # with a sharpness record, frames whose files are absent are dropped instead
    (tmp_path / "s.json").write_text(json.dumps({"camera_angle_x": 0.7, "frames": [
        {"file_path": "missing.png", "sharpness": 3.0, "transform_matrix": np.eye(4).tolist()}]}))
    with pytest.raises((RuntimeError, ValueError), match="No training images"):
        ngp.load_nerf_dataset(str(tmp_path / "s.json"))


def _write_png16_gray(path, arr):
    """Minimal 16-bit grayscale PNG writer (zlib, filter 0) for the depth fixtures."""
    import struct
    import zlib
    h, w = arr.shape
    raw = b"".join(b"\x00" + arr[y].astype(">u2").tobytes() for y in range(h))

    def chunk(t, data):
        return struct.pack(">I", len(data)) + t + data + struct.pack(">I", zlib.crc32(t + data) & 0xFFFFFFFF)
    with open(path, "wb") as f:
        f.write(b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 16, 0, 0, 0, 0))
                + chunk(b"IDAT", zlib.compress(raw)) + chunk(b"IEND", b""))


def test_depth_images_load_scaled(ngp, tmp_path):
    """Depth supervision inputs (src/nerf_loader.cu:419-437, 486-488, 625-637, 728): a frame's
    depth_path is a 16-bit image of the frame's resolution, scaled by integer_depth_scale and the
    dataset scale; frames without one, a missing file, or enable_depth_loading false give no depth;
    a wrong resolution is an error."""
    from PIL import Image
    w, h = 6, 4
    rgb = np.zeros((h, w, 4), np.uint8)
    rgb[..., 3] = 255
    for k in range(3):
        Image.fromarray(rgb).save(tmp_path / f"img{k}.png")
    dep = (np.arange(w * h).reshape(h, w) * 997 % 60000).astype(np.uint16)
    _write_png16_gray(str(tmp_path / "d0.png"), dep)
    frames = [{"file_path": f"img{k}.png", "transform_matrix": np.eye(4).tolist()} for k in range(3)]
    frames[0]["depth_path"] = "d0.png"
    frames[1]["depth_path"] = "missing.png"
    meta = {"camera_angle_x": 0.7, "integer_depth_scale": 1e-3, "scale": 0.5, "frames": frames}
    (tmp_path / "transforms.json").write_text(json.dumps(meta))
    d = ngp.load_nerf_dataset(str(tmp_path / "transforms.json"))
    np.testing.assert_allclose(d.depth(0), dep.astype(np.float32) * np.float32(1e-3 * 0.5), rtol=1e-6)
    assert d.depth(1) is None and d.depth(2) is None
    meta["enable_depth_loading"] = False
    (tmp_path / "transforms.json").write_text(json.dumps(meta))
    assert ngp.load_nerf_dataset(str(tmp_path / "transforms.json")).depth(0) is None
    meta["enable_depth_loading"] = True
    _write_png16_gray(str(tmp_path / "d0.png"), dep[:, :3])
    (tmp_path / "transforms.json").write_text(json.dumps(meta))
    with pytest.raises(RuntimeError, match="wrong resolution"):
        ngp.load_nerf_dataset(str(tmp_path / "transforms.json"))


def test_depth_settings_carry_over_between_jsons(ngp, tmp_path):
    """A directory load reads every *.json in sorted order; integer_depth_scale and
    enable_depth_loading live outside the reference's per-json loop (src/nerf_loader.cu:300, 419,
    435-437, 486-488), so a value set by the first json applies to the jsons after it."""
    from PIL import Image
    w, h = 6, 4
    rgb = np.zeros((h, w, 4), np.uint8)
    rgb[..., 3] = 255
    for k in range(2):
        Image.fromarray(rgb).save(tmp_path / f"img{k}.png")
    dep = (np.arange(w * h).reshape(h, w) * 131 % 50000).astype(np.uint16)
    _write_png16_gray(str(tmp_path / "d1.png"), dep)
    eye = np.eye(4).tolist()
    first = {"camera_angle_x": 0.7, "integer_depth_scale": 2e-3, "scale": 0.5,
             "frames": [{"file_path": "img0.png", "transform_matrix": eye}]}
    second = {"camera_angle_x": 0.7, "frames": [{"file_path": "img1.png", "transform_matrix": eye, "depth_path": "d1.png"}]}
    (tmp_path / "transforms_a.json").write_text(json.dumps(first))
    (tmp_path / "transforms_b.json").write_text(json.dumps(second))
    d = ngp.load_nerf_dataset(str(tmp_path))
    assert d.n_images == 2 and d.depth(0) is None
    np.testing.assert_allclose(d.depth(1), dep.astype(np.float32) * np.float32(2e-3 * 0.5), rtol=1e-6)
    # enable_depth_loading false in the first json turns depth loading off for the second as well
    first["enable_depth_loading"] = False
    (tmp_path / "transforms_a.json").write_text(json.dumps(first))
    assert ngp.load_nerf_dataset(str(tmp_path)).depth(1) is None


def _sharpness_numpy(rgba8):
    """compute_sharpness (src/nerf_loader.cu:111-151), restated in numpy: per tile of a 128 x 72
    grid, the variance of the 5-point Laplacian of the luma of the linear, premultiplied pixels."""
    c = rgba8.astype(np.float32) / np.float32(255)
    lin = np.where(c[..., :3] <= 0.04045, c[..., :3] / 12.92, ((c[..., :3] + 0.055) / 1.055) ** 2.4).astype(np.float32)
    lin = lin * c[..., 3:4]
    lum = (lin[..., 0] * np.float32(0.2126) + lin[..., 1] * np.float32(0.7152) + lin[..., 2] * np.float32(0.0722)).astype(np.float64)
    H, W = lum.shape
    lap = np.zeros_like(lum)
    lap[1:-1, 1:-1] = 4 * lum[1:-1, 1:-1] - lum[:-2, 1:-1] - lum[2:, 1:-1] - lum[1:-1, :-2] - lum[1:-1, 2:]
    out = np.zeros((72, 128))
    for y in range(72):
        y1, y2 = max(y * H // 72, 1), min((y + 1) * H // 72, H - 2)
        for x in range(128):
            x1, x2 = max(x * W // 128, 1), min((x + 1) * W // 128, W - 2)
            if x2 <= x1 or y2 <= y1:
                continue
            t = lap[y1:y2, x1:x2]
            out[y, x] = (t * t).mean() - t.mean() ** 2
    return out


def test_sharpness_matches_numpy_restatement(ngp):
    """The per-image sharpness of include_sharpness_in_error (compute_sharpness, 128 x 72 tiles of
    the variance of the Laplacian) on a frame of the reference's test dataset."""
    d = ngp.load_nerf_dataset(os.path.join(TEST, "transforms_test.json"))
    s = d.sharpness(0)
    ref = _sharpness_numpy(d.image(0))
    assert s.shape == (72, 128) and ref.max() > 0
    np.testing.assert_allclose(s, ref, rtol=2e-3, atol=1e-6 * ref.max())


def test_rolling_shutter_and_end_transforms(ngp, tmp_path):
    """Rolling shutter / motion blur inputs (src/nerf_loader.cu:204-216, 515-516, 664-699): a global
    3- or 4-element rolling_shutter (D defaults to 0), a per-frame override, and per-frame
    transform_matrix_start / transform_matrix_end (end = start when absent), both converted with
    nerf_matrix_to_ngp."""
    from PIL import Image
    rgb = np.zeros((4, 6, 4), np.uint8)
    rgb[..., 3] = 255
    for k in range(3):
        Image.fromarray(rgb).save(tmp_path / f"img{k}.png")
    rng = np.random.default_rng(0)
    mats = [np.vstack([rng.uniform(-1, 1, (3, 4)), [0, 0, 0, 1]]) for _ in range(4)]
    frames = [{"file_path": "img0.png", "transform_matrix": mats[0].tolist()},
              {"file_path": "img1.png", "transform_matrix_start": mats[1].tolist(), "transform_matrix_end": mats[2].tolist(),
               "rolling_shutter": [0.1, 0.2, 0.3, 0.4]},
              {"file_path": "img2.png", "transform_matrix": mats[3].tolist()}]
    meta = {"camera_angle_x": 0.7, "rolling_shutter": [0.5, 0.25, 0.125], "frames": frames}
    (tmp_path / "transforms.json").write_text(json.dumps(meta))
    d = ngp.load_nerf_dataset(str(tmp_path / "transforms.json"))
    rs = [tuple(d.metadata[i].rolling_shutter) for i in range(3)]
    assert rs[0] == rs[2] == (0.5, 0.25, 0.125, 0.0)
    np.testing.assert_allclose(rs[1], (0.1, 0.2, 0.3, 0.4), rtol=1e-7)
    start, end = d.transforms, d.transforms_end
    for i, (ms, me) in enumerate(((mats[0], mats[0]), (mats[1], mats[2]), (mats[3], mats[3]))):
        np.testing.assert_allclose(start[i], nerf_to_ngp(ms), atol=1e-6)
        np.testing.assert_allclose(end[i], nerf_to_ngp(me), atol=1e-6)
