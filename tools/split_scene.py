"""Deterministic train / held-out split of a transforms.json (quality protocol, GPU box).

Every k-th frame (after the loader's natural sort by file_path, src/nerf_loader.cu:347-349) is
held out -- the "llffhold" convention of the multi-view literature.  Writes
<out>/transforms_train.json and <out>/transforms_test.json with absolute image paths, all other
top-level keys (camera intrinsics, lens, aabb_scale, scale, offset) copied.

Usage: python tools/split_scene.py data/nerf/fox/transforms.json 8 /tmp/fox_split
"""
import copy
import json
import os
import re
import sys


def natural_key(s):
    return [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", s)]


def main(src, k, out):
    k = int(k)
    with open(src) as f:
        meta = json.load(f)
    base = os.path.dirname(os.path.abspath(src))
    frames = sorted(meta["frames"], key=lambda fr: natural_key(fr.get("file_path", "")))
    for fr in frames:
        p = fr["file_path"].replace("\\", "/")
        fr["file_path"] = p if p.startswith("/") else os.path.normpath(os.path.join(base, p))
        if "depth_path" in fr and not fr["depth_path"].startswith("/"):
            fr["depth_path"] = os.path.normpath(os.path.join(base, fr["depth_path"]))
    os.makedirs(out, exist_ok=True)
    for split, sel in (("train", [f for i, f in enumerate(frames) if i % k != 0]),
                       ("test", [f for i, f in enumerate(frames) if i % k == 0])):
        m = copy.deepcopy(meta)
        m["frames"] = sel
        with open(os.path.join(out, f"transforms_{split}.json"), "w") as f:
            json.dump(m, f, indent=1)
        print(f"{split}: {len(sel)} frames", file=sys.stderr)


if __name__ == "__main__":
    main(*sys.argv[1:4])
