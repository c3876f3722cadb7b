"""Synthetic datasets shared by the end-to-end parity tests (host and device views)."""
import ctypes as C

import numpy as np

import ngp_abi as A
import synthetic as S


def pcg_seed(seed, seq=1):
    """pcg32(seed) state after construction (pcg32.h seed()); returns (state, inc)."""
    M = 0x5851F42D4C957F2D
    mask = (1 << 64) - 1
    inc = ((seq << 1) | 1) & mask
    state = 0
    state = (state * M + inc) & mask
    state = (state + seed) & mask
    state = (state * M + inc) & mask
    return state, inc


def pcg_advance(state, inc, delta=1 << 32):
    M = 0x5851F42D4C957F2D
    mask = (1 << 64) - 1
    cur_mult, cur_plus, acc_mult, acc_plus = M, inc, 1, 0
    delta &= mask
    while delta > 0:
        if delta & 1:
            acc_mult = (acc_mult * cur_mult) & mask
            acc_plus = (acc_plus * cur_mult + cur_plus) & mask
        cur_plus = ((cur_mult + 1) * cur_plus) & mask
        cur_mult = (cur_mult * cur_mult) & mask
        delta //= 2
    return (acc_mult * state + acc_plus) & mask, inc


def make_views(n_images=6, W=24, H=24, seed=0):
    cams = S.hemisphere_cameras(n_images, seed=seed)
    focal = S.focal_from_angle(W)
    imgs = S.render_views(cams, W, H, focal)
    return imgs, cams, focal


def image_structs(imgs, cams, focal, pointers, lens=(0, ()), depth_pointers=None, shutter=None):
    """shutter: optional (cams_end, rolling_shutter[4]) -- TrainingXForm::end and the pixel-time
    coefficients of every image (default: end = start, no rolling shutter)."""
    n = len(imgs)
    arr = (A.Image * n)()
    for i in range(n):
        arr[i].pixels = pointers[i]
        arr[i].width = imgs.shape[2]
        arr[i].height = imgs.shape[1]
        arr[i].focal_length[0] = arr[i].focal_length[1] = float(focal)
        arr[i].principal_point[0] = arr[i].principal_point[1] = 0.5
        xf = np.asarray(cams[i], np.float32).T.reshape(-1)  # column-major 4x3
        xe = np.asarray(shutter[0][i] if shutter else cams[i], np.float32).T.reshape(-1)
        for k in range(12):
            arr[i].xform[k] = float(xf[k])
            arr[i].xform_end[k] = float(xe[k])
        if shutter:
            for k in range(4):
                arr[i].rolling_shutter[k] = float(shutter[1][k])
        arr[i].depth = int(depth_pointers[i]) if depth_pointers is not None and depth_pointers[i] else 0
        arr[i].lens_mode = lens[0]
        for k, val in enumerate(lens[1]):
            arr[i].lens_params[k] = float(val)
    return arr


class HostDataset:
    def __init__(self, imgs, cams, focal, lens=(0, ()), depths=None, shutter=None):
        """depths: optional per-image [H][W] f32 depth targets (None entries: no depth)."""
        self.imgs = [np.ascontiguousarray(im) for im in imgs]
        self.depths = [None if d is None else np.ascontiguousarray(d, np.float32) for d in depths] if depths else None
        dp = [0 if d is None else d.ctypes.data for d in self.depths] if self.depths else None
        self.arr = image_structs(imgs, cams, focal, [im.ctypes.data for im in self.imgs], lens, dp, shutter)
        self.n = len(imgs)

    @property
    def ptr(self):
        return C.cast(self.arr, C.c_void_p)


class DeviceDataset:
    def __init__(self, imgs, cams, focal, lens=(0, ()), depths=None, shutter=None):
        import torch
        self.pix = [torch.from_numpy(np.ascontiguousarray(im)).cuda() for im in imgs]
        self.depths = [None if d is None else torch.from_numpy(np.ascontiguousarray(d, np.float32)).cuda() for d in depths] \
            if depths else None
        dp = [0 if d is None else d.data_ptr() for d in self.depths] if self.depths else None
        arr = image_structs(imgs, cams, focal, [p.data_ptr() for p in self.pix], lens, dp, shutter)
        self.meta = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).cuda()
        self.n = len(imgs)

    @property
    def ptr(self):
        return C.c_void_p(self.meta.data_ptr())


def train_args(images_ptr, n_images, n_rays, target, max_samples, step=0, seed=1337, aabb_scale=1):
    a = A.TrainArgs()
    a.images = images_ptr
    a.n_images = n_images
    a.n_rays = n_rays
    a.target_batch_size = target
    a.max_samples = max_samples
    a.training_step = step
    a.rng_state, a.rng_inc = pcg_seed(seed)
    lo, hi = 0.5 - 0.5 * aabb_scale, 0.5 + 0.5 * aabb_scale
    for k in range(3):
        a.aabb_min[k], a.aabb_max[k] = lo, hi
    a.cone_angle_constant = 0.0 if aabb_scale <= 1 else 1.0 / 256.0
    a.max_cascade = max(0, int(np.log2(aabb_scale)))
    a.loss_type = 4  # Huber (configs/nerf/base.json:2-4)
    a.random_bg_color = 1
    a.snap_to_pixel_centers = 1
    a.train_in_linear_colors = 0
    a.color_space = 0
    a.near_distance = 0.1
    a.optimize_mlp = 1
    a.optimize_encoding = 1
    a.defer_optimizer = 1
    return a


def grid_args(images_ptr, n_images, n_uniform, n_nonuniform, ema_step=0, seed=1337, mark=1, clear=1, aabb_scale=1):
    g = A.GridArgs()
    g.images = images_ptr
    g.n_images = n_images
    lo, hi = 0.5 - 0.5 * aabb_scale, 0.5 + 0.5 * aabb_scale
    for k in range(3):
        g.aabb_min[k], g.aabb_max[k] = lo, hi
    g.max_cascade = max(0, int(np.log2(aabb_scale)))
    g.decay = 0.95
    g.n_uniform_samples = n_uniform
    g.n_nonuniform_samples = n_nonuniform
    g.rng_state, g.rng_inc = pcg_seed(seed)
    g.ema_step = ema_step
    g.mark_untrained = mark
    g.clear_visible = clear
    g.use_inference_params = 0
    g.rank, g.world_size = 0, 1
    return g


def render_args(W, H, cam, focal, spp=0, snap=0, shard=(0, 1, 8), min_transmittance=0.01, aabb_scale=1):
    r = A.RenderArgs()
    r.width, r.height, r.sample_index = W, H, spp
    xf = np.asarray(cam, np.float32).T.reshape(-1)
    for k in range(12):
        r.camera[k] = float(xf[k])
    r.focal_length[0] = r.focal_length[1] = float(focal)
    r.screen_center[0] = r.screen_center[1] = 0.5
    r.near_distance = 0.0
    lo, hi = 0.5 - 0.5 * aabb_scale, 0.5 + 0.5 * aabb_scale
    for k in range(3):
        r.aabb_min[k] = r.train_aabb_min[k] = lo
        r.aabb_max[k] = r.train_aabb_max[k] = hi
    r.cone_angle_constant = 0.0 if aabb_scale <= 1 else 1.0 / 256.0
    r.max_cascade = max(0, int(np.log2(aabb_scale)))
    r.min_transmittance = min_transmittance
    r.snap_to_pixel_centers = snap
    r.use_inference_params = 1
    r.train_in_linear_colors = 0
    r.shard_index, r.shard_count, r.shard_rows = shard
    return r


def sphere_bitfield(radius=0.3, center=(0.5, 0.5, 0.5)):
    """Occupancy bitfield (all 8 mips, Morton order) of a solid sphere, via the oracle's own bitfield pass."""
    n = 128
    ii = np.arange(n ** 3, dtype=np.uint64)

    def inv(x):
        r = np.zeros_like(x)
        for b in range(10):
            r |= ((x >> np.uint64(3 * b)) & np.uint64(1)) << np.uint64(b)
        return r
    x, y, z = inv(ii), inv(ii >> np.uint64(1)), inv(ii >> np.uint64(2))
    p = (np.stack([x, y, z], -1).astype(np.float32) + 0.5) / n
    d = np.linalg.norm(p - np.asarray(center, np.float32), axis=-1)
    grid = np.where(d < radius, 1.0, 0.0).astype(np.float32)
    return grid


def testbed_abi_config(tb):
    """The C-ABI network config of a pyngp Testbed's current network (for the oracle)."""
    cfg = tb.network_config
    enc = cfg["encoding"]
    c = A.default_config(n_levels=int(enc["n_levels"]), F=int(enc["n_features_per_level"]),
                         log2_T=int(enc["log2_hashmap_size"]), base_res=int(enc.get("base_resolution", 16)),
                         n_neurons=int(cfg["network"]["n_neurons"]),
                         density_hidden=int(cfg["network"]["n_hidden_layers"]),
                         rgb_hidden=int(cfg["rgb_network"]["n_hidden_layers"]),
                         aabb_scale=int(tb.nerf.training.dataset.aabb_scale))
    c.per_level_scale = float(tb.per_level_scale)  # exactly as the Testbed resolved it
    return c


def testbed_oracle(tb):
    """CPU oracle holding a Testbed's trained state: fp32 weights, the EMA inference weights the
    renderer reads, the density grid and its bitfield (test infrastructure only)."""
    from oracle_abi import Oracle
    o = Oracle(testbed_abi_config(tb))
    lib = A.load()
    h = C.c_void_p(tb.model_handle)
    tb.sync()

    def fetch(kind):
        p, n = C.c_void_p(), C.c_size_t()
        A.check(lib.ngp_model_buffer(h, kind, C.byref(p), C.byref(n)))
        out = np.zeros(n.value // 4, np.float32)
        hip = C.CDLL("libamdhip64.so")
        hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        assert hip.hipMemcpy(out.ctypes.data_as(C.c_void_p), p, n.value, 2) == 0
        return out
    o.set_params(fetch(A.PARAMS_FP32))
    o.set_inference_params(fetch(A.PARAMS_EMA_FP32))
    o.grid_set(tb.density_grid())
    o.set_bitfield(tb.density_grid_bitfield())  # the occupancy the GPU marches (bitfield parity is tested apart)
    return o


def testbed_render_args(tb, W, H, shard=(0, 1, 8), sample_index=0):
    """ngp_render_args exactly as Testbed::render builds them from the Testbed's camera state."""
    r = A.RenderArgs()
    r.width, r.height, r.sample_index = W, H, sample_index
    cam = np.asarray(tb.camera_matrix, np.float32)  # 3x4, columns right/down/forward/origin (NGP space)
    xf = cam.T.reshape(-1)
    for k in range(12):
        r.camera[k] = float(xf[k])
    zoom = float(tb.zoom)
    res_axis = W if tb.fov_axis == 0 else H
    rf = tb.relative_focal_length
    r.focal_length[0], r.focal_length[1] = rf[0] * res_axis * zoom, rf[1] * res_axis * zoom
    sc = tb.screen_center
    r.screen_center[0], r.screen_center[1] = (0.5 - sc[0]) * zoom + 0.5, (0.5 - sc[1]) * zoom + 0.5
    r.near_distance = float(tb.render_near_distance)
    bb = tb.aabb
    for k in range(3):
        r.aabb_min[k] = r.train_aabb_min[k] = bb.min[k]
        r.aabb_max[k] = r.train_aabb_max[k] = bb.max[k]
    r.cone_angle_constant = float(tb.nerf.cone_angle_constant)
    r.max_cascade = int(tb.nerf.max_cascade)
    r.min_transmittance = float(tb.nerf.render_min_transmittance)
    r.snap_to_pixel_centers = int(tb.snap_to_pixel_centers)
    r.use_inference_params = 1
    r.train_in_linear_colors = int(tb.nerf.training.linear_colors)
    r.shard_index, r.shard_count, r.shard_rows = shard
    if tb.nerf.render_with_lens_distortion:
        lens = tb.nerf.render_lens
        r.lens_mode = int(lens.mode)
        for k, v in enumerate(lens.params):
            r.lens_params[k] = float(v)
    return r


def oracle_frame_rows(o, tb, W, H, blocks, rows=8):
    """Render the 8-row blocks `blocks` of a W x H frame with the oracle; returns {row: rgba}."""
    out = {}
    for b in blocks:
        fr, _ = o.render(testbed_render_args(tb, W, H, shard=(b, H // rows, rows)))
        for y in range(b * rows, min(H, (b + 1) * rows)):
            out[y] = fr[y]
    return out
