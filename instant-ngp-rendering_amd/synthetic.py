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


def render_views(cams, width, height, focal, primitives=None, light=(0.4, 0.8, 0.3)):
    """Analytic ray cast -> uint8 RGBA [n, H, W, 4] (sRGB colours, straight alpha)."""
    boxes, spheres = primitives if primitives is not None else lego_like_primitives()
    light = np.asarray(light, np.float32)
    light /= np.linalg.norm(light)
    ys, xs = np.mgrid[0:height, 0:width].astype(np.float32)
    dirs_cam = np.stack([(xs + 0.5 - 0.5 * width) / focal, (ys + 0.5 - 0.5 * height) / focal, np.ones_like(xs)], -1)
    out = np.zeros((len(cams), height, width, 4), np.uint8)
    for k, cam in enumerate(cams):
        R, o = cam[:, :3], cam[:, 3]
        d = dirs_cam @ R.T
        d /= np.linalg.norm(d, axis=-1, keepdims=True)
        best = np.full((height, width), np.inf, np.float32)
        col = np.zeros((height, width, 3), np.float32)
        nrm = np.zeros((height, width, 3), np.float32)
        for (mn, mx, c) in boxes:
            mn, mx = np.asarray(mn, np.float32), np.asarray(mx, np.float32)
            with np.errstate(divide="ignore", invalid="ignore"):
                t0 = (mn - o) / d
                t1 = (mx - o) / d
            tmin = np.minimum(t0, t1)
            tmax = np.maximum(t0, t1)
            tn = tmin.max(-1)
            tf = tmax.min(-1)
            hit = (tn <= tf) & (tn > 0) & (tn < best)
            if hit.any():
                best[hit] = tn[hit]
                col[hit] = c
                axis = tmin.argmax(-1)
                n = np.zeros((height, width, 3), np.float32)
                np.put_along_axis(n, axis[..., None], -np.sign(np.take_along_axis(d, axis[..., None], -1)), -1)
                nrm[hit] = n[hit]
        for (c0, r, c) in spheres:
            oc = o - np.asarray(c0, np.float32)
            b = (d * oc).sum(-1)
            disc = b * b - (oc @ oc - r * r)
            hit0 = disc > 0
            t = -b - np.sqrt(np.maximum(disc, 0))
            hit = hit0 & (t > 0) & (t < best)
            if hit.any():
                best[hit] = t[hit]
                col[hit] = c
                p = o + d * t[..., None]
                n = (p - np.asarray(c0, np.float32)) / r
                nrm[hit] = n[hit]
        mask = np.isfinite(best)
        shade = 0.35 + 0.65 * np.clip((nrm * light).sum(-1), 0, 1)
        rgb = np.clip(col * shade[..., None], 0, 1)
        out[k, ..., :3] = (rgb * 255 + 0.5).astype(np.uint8) * mask[..., None]
        out[k, ..., 3] = mask.astype(np.uint8) * 255
    return out
