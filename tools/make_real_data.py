"""Builds data/nerf/{test,fox} from the reference checkout's own datasets (run in the build
container, where /root/reference exists; the outputs are committed and travel to the GPU box).

* data/nerf/test/dataset: the reference's BlenderNeRF scene (data/nerf/test/dataset, 50 RGBA
  720x1280 frames, alpha 255 everywhere, aabb_scale 1) at half resolution (360x640, Lanczos),
  stored as RGB PNG (lossless for an opaque image), intrinsics (fl_x/fl_y/cx/cy/w/h) halved.
  Split for the quality protocol: every 10th frame (0005, 0015, ...) -> transforms_test.json,
  the other 45 -> transforms_train.json.
* data/nerf/test2/images: the reference's second BlenderNeRF scene (data/nerf/test2/images, 300 RGBA 720x1280
  frames, alpha 255 everywhere, aabb_scale 1) at quarter resolution (180x320, Lanczos, RGB PNG), all 300 views,
  intrinsics quartered; transforms_train.json lists every frame as the reference's does.  With
  data/nerf/test/dataset it is one of the two scenes whose CUDA-trained density mosaics the reference ships
  (data/nerf/test.density_slices_256x256x256.png, data/nerf/test2/images.density_slices_256x256x256.png), which
  tests/golden/ref_density_slices/ holds byte for byte.
* data/nerf/test2_half/images: the same scene at half resolution (360x640; `python tools/make_real_data.py test2_half`).
* data/nerf/fox: the reference's transforms.json verbatim and its 50 JPG frames as shipped (17
  listed frames are absent from the reference checkout; the loader skips them exactly as
  nerf_loader.cu:364-387 does for files that do not exist).
"""
import json
import os
import shutil
import sys

from PIL import Image

REF = "/root/reference/data/nerf"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "data", "nerf")


def make_test():
    src = os.path.join(REF, "test", "dataset")
    dst = os.path.join(OUT, "test", "dataset")
    os.makedirs(os.path.join(dst, "train"), exist_ok=True)
    meta = json.load(open(os.path.join(src, "transforms_train.json")))
    for k in ("fl_x", "fl_y", "cx", "cy", "w", "h"):
        meta[k] = meta[k] * 0.5
    frames = sorted(meta["frames"], key=lambda f: f["file_path"])
    for fr in frames:
        name = os.path.basename(fr["file_path"])
        im = Image.open(os.path.join(src, fr["file_path"]))
        w, h = im.size
        im = im.resize((w // 2, h // 2), Image.LANCZOS).convert("RGB")
        im.save(os.path.join(dst, "train", name), "PNG", optimize=True)
    test = [f for i, f in enumerate(frames) if i % 10 == 4]
    train = [f for i, f in enumerate(frames) if i % 10 != 4]
    for name, fr in (("transforms_train.json", train), ("transforms_test.json", test), ("transforms_all.json", frames)):
        m = dict(meta)
        m["frames"] = fr
        json.dump(m, open(os.path.join(dst, name), "w"), indent=1)
    shutil.copy(os.path.join(src, "log.txt"), os.path.join(dst, "log.txt"))


def make_test2(div=4, out="test2"):
    """div 4 -> data/nerf/test2 (180x320); div 2 -> data/nerf/test2_half (360x640, VERDICT r05 item 2: the
    reference trained at 720x1280)."""
    src = os.path.join(REF, "test2", "images")
    dst = os.path.join(OUT, out, "images")
    os.makedirs(os.path.join(dst, "train"), exist_ok=True)
    meta = json.load(open(os.path.join(src, "transforms_train.json")))
    for k in ("fl_x", "fl_y", "cx", "cy", "w", "h"):
        meta[k] = meta[k] / div
    for fr in meta["frames"]:
        name = os.path.basename(fr["file_path"])
        im = Image.open(os.path.join(src, fr["file_path"]))
        w, h = im.size
        if div > 1:
            im = im.resize((w // div, h // div), Image.LANCZOS)
        im = im.convert("RGB")
        im.save(os.path.join(dst, "train", name), "PNG", optimize=True)
    json.dump(meta, open(os.path.join(dst, "transforms_train.json"), "w"), indent=1)
    shutil.copy(os.path.join(src, "log.txt"), os.path.join(dst, "log.txt"))


def copy_reference_slices():
    dst = os.path.join(ROOT, "tests", "golden", "ref_density_slices")
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(REF, "test.density_slices_256x256x256.png"), os.path.join(dst, "test.png"))
    shutil.copy(os.path.join(REF, "test2", "images.density_slices_256x256x256.png"), os.path.join(dst, "test2.png"))


def make_fox():
    src = os.path.join(REF, "fox")
    dst = os.path.join(OUT, "fox")
    os.makedirs(os.path.join(dst, "images"), exist_ok=True)
    shutil.copy(os.path.join(src, "transforms.json"), os.path.join(dst, "transforms.json"))
    for name in sorted(os.listdir(os.path.join(src, "images"))):
        shutil.copy(os.path.join(src, "images", name), os.path.join(dst, "images", name))


if __name__ == "__main__":
    if not os.path.isdir(REF):
        sys.exit("the reference checkout is not here (build container only)")
    which = sys.argv[1:] or ["test", "test2", "fox", "slices"]
    if "test" in which:
        make_test()
    if "test2" in which:
        make_test2()
    if "test2_half" in which:
        make_test2(2, "test2_half")
    if "test2_full" in which:
        make_test2(1, "test2_full")  # 720x1280, the reference's training resolution (82 MB)
    if "fox" in which:
        make_fox()
    if "slices" in which:
        copy_reference_slices()
