"""Synthetic nerf_synthetic-shaped scene (data generator for tests and bench.py).

nerf_synthetic/lego is not available offline, so the benchmark and the
end-to-end tests use a procedurally built "lego-like" object (boxes + spheres,
opaque, Lambert-shaded) rendered from cameras on the upper hemisphere around
the unit cube, in NGP space.  Same shapes as the real dataset: 800x800 RGBA8
frames with transparent background, camera_angle_x = 0.6911112 rad, camera
radius 4.03 in NeRF units (x0.33 NERF_SCALE, +0.5 offset; nerf_loader.h:29,
src/nerf_loader.cu:403-404).
"""
import numpy as np

LEGO_CAMERA_ANGLE_X = 0.6911112070083618
NERF_SCALE = 0.33


def lego_like_primitives(seed=7):
    rng = np.random.default_rng(seed)
    boxes = []
    # base plate + tracks + body + cabin + arm (roughly a bulldozer silhouette in [0.15, 0.85]^3, y up)
    boxes.append(((0.18, 0.30, 0.25), (0.82, 0.34, 0.75), (0.85, 0.70, 0.10)))
    boxes.append(((0.20, 0.25, 0.22), (0.80, 0.31, 0.32), (0.15, 0.15, 0.15)))
    boxes.append(((0.20, 0.25, 0.68), (0.80, 0.31, 0.78), (0.15, 0.15, 0.15)))
    boxes.append(((0.30, 0.34, 0.33), (0.65, 0.50, 0.67), (0.90, 0.75, 0.10)))
    boxes.append(((0.38, 0.50, 0.38), (0.60, 0.66, 0.62), (0.85, 0.70, 0.15)))
    boxes.append(((0.65, 0.36, 0.30), (0.72, 0.56, 0.36), (0.30, 0.30, 0.30)))
    boxes.append(((0.65, 0.36, 0.64), (0.72, 0.56, 0.70), (0.30, 0.30, 0.30)))
    boxes.append(((0.70, 0.28, 0.28), (0.80, 0.45, 0.72), (0.80, 0.65, 0.12)))
    for _ in range(24):  # studs and greebles
        c = rng.uniform((0.30, 0.50, 0.36), (0.64, 0.66, 0.64))
        s = rng.uniform(0.012, 0.03, 3)
        col = rng.uniform(0.1, 0.95, 3)
        boxes.append((tuple(c - s), tuple(c + s), tuple(col)))
    spheres = [((0.25, 0.30, 0.27), 0.045, (0.2, 0.2, 0.2)), ((0.25, 0.30, 0.73), 0.045, (0.2, 0.2, 0.2)),
               ((0.75, 0.30, 0.27), 0.045, (0.2, 0.2, 0.2)), ((0.75, 0.30, 0.73), 0.045, (0.2, 0.2, 0.2)),
               ((0.49, 0.72, 0.50), 0.06, (0.9, 0.1, 0.1))]
    return boxes, spheres


def look_at(pos, target=(0.5, 0.5, 0.5), up=(0.0, 1.0, 0.0)):
    """Camera-to-world 3x4 in the NGP convention: columns right, down, forward, origin."""
    pos = np.asarray(pos, np.float64)
    f = np.asarray(target, np.float64) - pos
    f /= np.linalg.norm(f)
    r = np.cross(f, up)
    r /= np.linalg.norm(r)
    d = np.cross(f, r)
    return np.stack([r, d, f, pos], axis=1).astype(np.float32)


def hemisphere_cameras(n, seed=0, radius=4.03 * NERF_SCALE, center=(0.5, 0.5, 0.5)):
    rng = np.random.default_rng(seed)
    cams = []
    for i in range(n):
        az = 2 * np.pi * ((i * 0.61803398875) % 1.0)
        el = np.arcsin(rng.uniform(0.05, 0.95))
        p = np.array(center) + radius * np.array([np.cos(el) * np.cos(az), np.sin(el), np.cos(el) * np.sin(az)])
        cams.append(look_at(p, center))
    return np.stack(cams)


def focal_from_angle(width, angle_x=LEGO_CAMERA_ANGLE_X):
    return 0.5 * width / np.tan(0.5 * angle_x)


def render_views(cams, width, height, focal, primitives=None, light=(0.4, 0.8, 0.3), device=None, chunk=None):
    """Analytic ray cast -> uint8 RGBA [n, H, W, 4] (sRGB colours, straight alpha).

    Runs in torch so the 100-view 800x800 set builds in about a second on the GPU
    (and still in seconds on CPU for the small test scenes).
    """
    import torch

    dev = torch.device(device) if device is not None else torch.device("cpu")
    boxes, spheres = primitives if primitives is not None else lego_like_primitives()
    lt = torch.tensor(light, dtype=torch.float32, device=dev)
    lt = lt / lt.norm()
    ys, xs = torch.meshgrid(torch.arange(height, dtype=torch.float32, device=dev),
                            torch.arange(width, dtype=torch.float32, device=dev), indexing="ij")
    dirs_cam = torch.stack([(xs + 0.5 - 0.5 * width) / focal, (ys + 0.5 - 0.5 * height) / focal, torch.ones_like(xs)], -1)
    out = np.zeros((len(cams), height, width, 4), np.uint8)
    bmn = torch.tensor([b[0] for b in boxes], dtype=torch.float32, device=dev)
    bmx = torch.tensor([b[1] for b in boxes], dtype=torch.float32, device=dev)
    bcol = torch.tensor([b[2] for b in boxes], dtype=torch.float32, device=dev)
    for k, cam in enumerate(np.asarray(cams, np.float32)):
        R = torch.from_numpy(cam[:, :3]).to(dev)
        o = torch.from_numpy(cam[:, 3]).to(dev)
        d = dirs_cam @ R.T
        d = d / d.norm(dim=-1, keepdim=True)
        inv = 1.0 / d
        best = torch.full((height, width), float("inf"), device=dev)
        col = torch.zeros((height, width, 3), device=dev)
        nrm = torch.zeros((height, width, 3), device=dev)
        for bi in range(bmn.shape[0]):
            t0 = (bmn[bi] - o) * inv
            t1 = (bmx[bi] - o) * inv
            tmin = torch.minimum(t0, t1)
            tmax = torch.maximum(t0, t1)
            tn, axis = tmin.max(-1)
            tf = tmax.min(-1).values
            hit = (tn <= tf) & (tn > 0) & (tn < best)
            best = torch.where(hit, tn, best)
            col = torch.where(hit[..., None], bcol[bi], col)
            n = torch.zeros_like(nrm).scatter_(-1, axis[..., None], -torch.sign(torch.gather(d, -1, axis[..., None])))
            nrm = torch.where(hit[..., None], n, nrm)
        for (c0, r, c) in spheres:
            c0 = torch.tensor(c0, dtype=torch.float32, device=dev)
            oc = o - c0
            b = (d * oc).sum(-1)
            disc = b * b - (oc @ oc - r * r)
            t = -b - torch.sqrt(torch.clamp(disc, min=0))
            hit = (disc > 0) & (t > 0) & (t < best)
            best = torch.where(hit, t, best)
            col = torch.where(hit[..., None], torch.tensor(c, dtype=torch.float32, device=dev), col)
            n = (o + d * t[..., None] - c0) / r
            nrm = torch.where(hit[..., None], n, nrm)
        mask = torch.isfinite(best)
        shade = 0.35 + 0.65 * torch.clamp((nrm * lt).sum(-1), 0, 1)
        rgb = torch.clamp(col * shade[..., None], 0, 1)
        rgb8 = (rgb * 255 + 0.5).to(torch.uint8) * mask[..., None].to(torch.uint8)
        img = torch.cat([rgb8, (mask.to(torch.uint8) * 255)[..., None]], -1)
        out[k] = img.cpu().numpy()
    return out


def write_png(path, rgba):
    """Minimal RGBA8 PNG writer (zlib) so tests can exercise the transforms.json loader."""
    import struct
    import zlib

    h, w, _ = rgba.shape
    raw = b"".join(b"\x00" + rgba[y].tobytes() for y in range(h))

    def chunk(t, body):
        return struct.pack(">I", len(body)) + t + body + struct.pack(">I", zlib.crc32(t + body) & 0xFFFFFFFF)

    with open(path, "wb") as f:
        f.write(b"\x89PNG\r\n\x1a\n")
        f.write(chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 6, 0, 0, 0)))
        f.write(chunk(b"IDAT", zlib.compress(raw, 6)))
        f.write(chunk(b"IEND", b""))


def ngp_to_nerf_matrix(c2w_ngp, scale=NERF_SCALE, offset=(0.5, 0.5, 0.5)):
    """Inverse of nerf_matrix_to_ngp (nerf_loader.h:95-116): NGP 3x4 -> NeRF/Blender 4x4."""
    m = np.asarray(c2w_ngp, np.float64)
    cyc = m[[2, 0, 1], :].copy()  # undo the xyz <- yzx axis cycle
    cyc[:, 1] *= -1
    cyc[:, 2] *= -1
    cyc[:, 3] = (cyc[:, 3] - np.asarray(offset)) / scale
    out = np.eye(4)
    out[:3] = cyc
    return out


def write_nerf_synthetic_scene(root, n_views, width, height, seed=0, split="train", device=None):
    """Write transforms_<split>.json + PNG frames in the nerf_synthetic layout."""
    import json
    import os

    os.makedirs(os.path.join(root, split), exist_ok=True)
    cams = hemisphere_cameras(n_views, seed)
    focal = focal_from_angle(width)
    imgs = render_views(cams, width, height, focal, device=device)
    frames = []
    for i, (cam, img) in enumerate(zip(cams, imgs)):
        write_png(os.path.join(root, split, f"r_{i}.png"), img)
        frames.append({"file_path": f"./{split}/r_{i}", "rotation": 0.0,
                       "transform_matrix": ngp_to_nerf_matrix(cam).tolist()})
    with open(os.path.join(root, f"transforms_{split}.json"), "w") as f:
        json.dump({"camera_angle_x": LEGO_CAMERA_ANGLE_X, "frames": frames}, f, indent=1)
    return cams, imgs
