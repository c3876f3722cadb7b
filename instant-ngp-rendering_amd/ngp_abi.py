"""ctypes binding of the libngp_hip.so C-ABI (include/ngp_hip.h).

This is the reference-side binding a maintainer would add to drive the MI355X
path from Python without the pyngp extension; the struct layouts mirror
include/ngp_hip.h field for field.  Loading fails loudly when the HIP library
is missing — there is no CPU fallback on the product path.
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libngp_hip.so")


class NetworkConfig(C.Structure):
    _fields_ = [
        ("n_levels", C.c_uint32), ("n_features_per_level", C.c_uint32), ("log2_hashmap_size", C.c_uint32),
        ("base_resolution", C.c_uint32), ("per_level_scale", C.c_float),
        ("n_neurons", C.c_uint32), ("density_hidden_layers", C.c_uint32), ("rgb_hidden_layers", C.c_uint32),
        ("rgb_activation", C.c_int32), ("density_activation", C.c_int32),
        ("learning_rate", C.c_float), ("beta1", C.c_float), ("beta2", C.c_float), ("epsilon", C.c_float),
        ("l2_reg", C.c_float), ("ema_decay", C.c_float),
        ("decay_start", C.c_uint32), ("decay_interval", C.c_uint32), ("decay_base", C.c_float),
        ("n_extra_dims", C.c_uint32),
    ]


class ModelInfo(C.Structure):
    _fields_ = [
        ("n_params", C.c_uint64), ("n_mlp_params", C.c_uint64), ("n_grid_params", C.c_uint64),
        ("n_levels", C.c_uint32), ("n_features_per_level", C.c_uint32), ("encoding_width", C.c_uint32),
        ("padded_encoding_width", C.c_uint32),
        ("level_offset", C.c_uint32 * 32), ("level_size", C.c_uint32 * 32), ("level_resolution", C.c_uint32 * 32),
        ("level_scale", C.c_float * 32),
        ("n_layers", C.c_uint32), ("layer_in", C.c_uint32 * 8), ("layer_out", C.c_uint32 * 8),
        ("layer_param_offset", C.c_uint64 * 8),
    ]


class Image(C.Structure):
    _fields_ = [
        ("pixels", C.c_uint64), ("width", C.c_uint32), ("height", C.c_uint32),
        ("focal_length", C.c_float * 2), ("principal_point", C.c_float * 2), ("xform", C.c_float * 12),
        ("lens_mode", C.c_int32), ("lens_params", C.c_float * 7), ("depth", C.c_uint64),
        ("xform_end", C.c_float * 12), ("rolling_shutter", C.c_float * 4),
    ]


class TrainArgs(C.Structure):
    _fields_ = [
        ("images", C.c_void_p), ("n_images", C.c_uint32), ("n_rays", C.c_uint32), ("n_rays_total", C.c_uint32),
        ("target_batch_size", C.c_uint32), ("max_samples", C.c_uint32), ("training_step", C.c_uint32),
        ("rng_state", C.c_uint64), ("rng_inc", C.c_uint64),
        ("ray_index_offset", C.c_uint32), ("n_rays_global", C.c_uint32),
        ("aabb_min", C.c_float * 3), ("aabb_max", C.c_float * 3), ("cone_angle_constant", C.c_float),
        ("max_cascade", C.c_uint32), ("loss_type", C.c_int32), ("random_bg_color", C.c_int32),
        ("background_color", C.c_float * 3), ("snap_to_pixel_centers", C.c_int32),
        ("train_in_linear_colors", C.c_int32), ("color_space", C.c_int32), ("near_distance", C.c_float),
        ("optimize_mlp", C.c_int32), ("optimize_encoding", C.c_int32), ("defer_optimizer", C.c_int32),
        ("error_map", C.c_void_p), ("error_map_res", C.c_uint32 * 2), ("cdf_x_cond_y", C.c_void_p),
        ("cdf_y", C.c_void_p), ("cdf_img", C.c_void_p), ("cdf_res", C.c_uint32 * 2), ("has_lens", C.c_int32),
        ("exposure", C.c_void_p), ("exposure_gradient", C.c_void_p),
        ("cam_pos_gradient", C.c_void_p), ("cam_rot_gradient", C.c_void_p), ("full_forward", C.c_int32),
        ("depth_supervision_lambda", C.c_float), ("depth_loss_type", C.c_int32),
        ("sharpness_data", C.c_void_p), ("sharpness_res", C.c_uint32 * 2), ("sharpness_grid", C.c_void_p),
        ("sharpness_grid_clear", C.c_int32),
        ("distortion_map", C.c_void_p), ("distortion_res", C.c_uint32 * 2), ("distortion_gradient", C.c_void_p),
        ("distortion_gradient_weight", C.c_void_p),
        ("rank", C.c_uint32), ("world_size", C.c_uint32), ("allreduce_i32", C.c_void_p), ("allreduce_user", C.c_void_p),
        ("deterministic", C.c_int32),
        ("max_level_rand_training", C.c_int32),
        ("extra_dims", C.c_void_p), ("extra_dims_gradient", C.c_void_p),
    ]


class TrainStats(C.Structure):
    _fields_ = [
        ("n_rays", C.c_uint32), ("n_rays_with_samples", C.c_uint32),
        ("measured_batch_size_before_compaction", C.c_uint32), ("measured_batch_size", C.c_uint32),
        ("loss", C.c_float), ("forward_early_stop_violations", C.c_uint32), ("sample_capacity_overflow", C.c_uint32),
    ]


class GridArgs(C.Structure):
    _fields_ = [
        ("images", C.c_void_p), ("n_images", C.c_uint32), ("aabb_min", C.c_float * 3), ("aabb_max", C.c_float * 3),
        ("max_cascade", C.c_uint32), ("decay", C.c_float), ("n_uniform_samples", C.c_uint32),
        ("n_nonuniform_samples", C.c_uint32), ("rng_state", C.c_uint64), ("rng_inc", C.c_uint64),
        ("ema_step", C.c_uint32), ("mark_untrained", C.c_int32), ("clear_visible", C.c_int32),
        ("use_inference_params", C.c_int32), ("rank", C.c_uint32), ("world_size", C.c_uint32),
    ]


class GridQuery(C.Structure):
    """ngp_grid_query: the lattice of get_density_on_grid (src/testbed_nerf.cu:3026-3075)."""
    _fields_ = [
        ("res", C.c_uint32 * 3), ("box_min", C.c_float * 3), ("box_max", C.c_float * 3), ("box_to_local", C.c_float * 9),
        ("aabb_min", C.c_float * 3), ("aabb_max", C.c_float * 3), ("max_cascade", C.c_uint32),
        ("mask_with_grid", C.c_int32), ("use_inference_params", C.c_int32),
    ]


class RenderArgs(C.Structure):
    _fields_ = [
        ("width", C.c_uint32), ("height", C.c_uint32), ("sample_index", C.c_uint32), ("camera", C.c_float * 12),
        ("focal_length", C.c_float * 2), ("screen_center", C.c_float * 2), ("near_distance", C.c_float),
        ("aabb_min", C.c_float * 3), ("aabb_max", C.c_float * 3), ("train_aabb_min", C.c_float * 3),
        ("train_aabb_max", C.c_float * 3), ("cone_angle_constant", C.c_float), ("max_cascade", C.c_uint32),
        ("min_transmittance", C.c_float), ("snap_to_pixel_centers", C.c_int32), ("use_inference_params", C.c_int32),
        ("train_in_linear_colors", C.c_int32), ("shard_index", C.c_uint32), ("shard_count", C.c_uint32),
        ("shard_rows", C.c_uint32), ("lens_mode", C.c_int32), ("lens_params", C.c_float * 7),
        ("camera_end", C.c_float * 12), ("rolling_shutter", C.c_float * 4),
        ("distortion_map", C.c_void_p), ("distortion_res", C.c_uint32 * 2),
        ("render_aabb_to_local", C.c_float * 9), ("render_mode", C.c_int32), ("depth_scale", C.c_float),
        ("gbuffer_hard_edges", C.c_int32), ("aperture_size", C.c_float), ("focus_z", C.c_float),
        ("glow_mode", C.c_int32), ("glow_y_cutoff", C.c_float),
        ("extra_dims", C.c_void_p),
        ("host_frame", C.c_void_p), ("host_frame_complete", C.c_void_p), ("host_background", C.c_float * 4),
        ("host_exposure", C.c_float), ("host_color_space", C.c_int32), ("host_output_srgb", C.c_int32),
    ]


class Tuning(C.Structure):
    """ngp_tuning: launch shapes / march schedule (0 = the measured default; results do not depend on them)."""
    _fields_ = [
        ("render_pipelines", C.c_uint32), ("render_pass_samples", C.c_uint32), ("render_lanes", C.c_uint32),
        ("render_first_steps", C.c_uint32), ("render_max_steps", C.c_uint32), ("render_lag", C.c_uint32),
        ("render_budget_scale", C.c_float), ("render_composite_block", C.c_uint32), ("render_generate_block", C.c_uint32),
        ("encode_dense_records", C.c_uint32), ("mlp_workgroups_per_cu", C.c_uint32), ("debug", C.c_uint32),
        ("encode_streaming", C.c_uint32), ("grid_unsorted", C.c_uint32), ("render_mlp_tile", C.c_uint32),
        ("encode_xcd_regions", C.c_uint32), ("render_skip_unfilled", C.c_uint32), ("render_exit_cap", C.c_uint32),
        ("render_priority", C.c_uint32), ("render_host_frame", C.c_uint32),
        ("train_chunk_lanes", C.c_uint32), ("train_sampler_lanes", C.c_uint32), ("render_mlp_pipeline", C.c_uint32),
    ]


# latent-code rows (include/ngp_hip.h NGP_EXTRA_ROW / NGP_EXTRA_DIMS_MAX)
EXTRA_ROW = 32
EXTRA_DIMS_MAX = 32

# enums (include/ngp_hip.h)
PARAMS_FP32, PARAMS_FP16, PARAMS_EMA_FP32, PARAMS_INFER_FP16, GRADS_FP32, ADAM_M, ADAM_V, GRADS_GRID_FP16, \
    GRADS_GRID_FIXED64 = range(9)
SCRATCH_RAY_NUMSTEPS, SCRATCH_COORDS, SCRATCH_MLP_OUT, SCRATCH_RAY_COMPACTED, SCRATCH_DLOSS, SCRATCH_LOSS, \
    SCRATCH_COMPACT_COORDS, SCRATCH_RAY_EVALUATED, SCRATCH_VIOLATIONS = range(9)

RENDER_SHADE, RENDER_AO, RENDER_NORMALS, RENDER_POSITIONS, RENDER_DEPTH, RENDER_COST, RENDER_SLICE = range(7)

TIMERS = ["train_sampler", "train_encode", "train_mlp_infer", "train_loss", "train_mlp_bwd", "train_encode_bwd",
          "optimizer", "grid_update", "render_encode", "render_mlp", "render_march"]
TIMER = {name: i for i, name in enumerate(TIMERS)}

EXPORTS = {
    "ngp_model_create": (C.c_int, [C.c_int, C.POINTER(NetworkConfig), C.c_uint64, C.POINTER(C.c_void_p)]),
    "ngp_model_destroy": (C.c_int, [C.c_void_p]),
    "ngp_model_set_tuning": (C.c_int, [C.c_void_p, C.POINTER(Tuning)]),
    "ngp_tuning_validate": (C.c_int, [C.POINTER(Tuning)]),
    "ngp_model_get_tuning": (C.c_int, [C.c_void_p, C.POINTER(Tuning)]),
    "ngp_model_get_info": (C.c_int, [C.c_void_p, C.POINTER(ModelInfo)]),
    "ngp_model_buffer": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]),
    "ngp_model_params_updated": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p]),
    "ngp_model_reset_optimizer": (C.c_int, [C.c_void_p, C.c_void_p]),
    "ngp_model_encode": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p, C.c_int, C.c_void_p]),
    "ngp_model_encode_indices": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p,
                                           C.c_void_p]),
    "ngp_model_infer": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p, C.c_int, C.c_void_p]),
    "ngp_model_infer_padded": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p, C.c_uint32, C.c_int,
                                         C.c_int, C.c_void_p]),
    "ngp_model_infer_sh_rows": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32,
                                          C.c_void_p, C.c_int, C.c_void_p]),
    "ngp_model_density": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p, C.c_int, C.c_void_p]),
    "ngp_model_backward": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p,
                                     C.c_void_p, C.c_void_p]),
    "ngp_model_backward_extra": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p,
                                           C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "ngp_model_encode_backward": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p]),
    "ngp_train_step": (C.c_int, [C.c_void_p, C.POINTER(TrainArgs), C.c_void_p]),
    "ngp_optimizer_step": (C.c_int, [C.c_void_p, C.c_uint32, C.c_int, C.c_int, C.c_void_p]),
    "ngp_train_read_stats": (C.c_int, [C.c_void_p, C.POINTER(TrainStats), C.c_void_p]),
    "ngp_allreduce_grads": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "ngp_train_scratch": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]),
    "ngp_train_discard": (C.c_int, [C.c_void_p, C.c_void_p]),
    "ngp_train_violation_parts": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]),
    "ngp_density_grid_update": (C.c_int, [C.c_void_p, C.POINTER(GridArgs), C.c_void_p]),
    "ngp_density_grid_evaluate": (C.c_int, [C.c_void_p, C.POINTER(GridArgs), C.c_void_p]),
    "ngp_density_grid_finish": (C.c_int, [C.c_void_p, C.POINTER(GridArgs), C.c_void_p]),
    "ngp_density_grid_bitfield": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p]),
    "ngp_density_grid_buffers": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p),
                                           C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)]),
    "ngp_density_on_grid": (C.c_int, [C.c_void_p, C.POINTER(GridQuery), C.c_void_p, C.c_void_p]),
    "ngp_error_map_build_cdf": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p,
                                          C.c_void_p, C.c_void_p]),
    "ngp_render": (C.c_int, [C.c_void_p, C.POINTER(RenderArgs), C.c_void_p, C.c_void_p, C.c_void_p]),
    "ngp_accumulate_tonemap": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32,
                                         C.c_int, C.c_float, C.POINTER(C.c_float), C.c_int, C.c_void_p]),
    "ngp_timing_enable": (C.c_int, [C.c_void_p, C.c_int]),
    "ngp_timing_read": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_uint64),
                                  C.POINTER(C.c_uint32), C.c_int]),
    "ngp_last_error": (C.c_char_p, []),
    "ngp_version": (C.c_char_p, []),
}

_lib = None


def load(path=LIB_PATH):
    """Load libngp_hip.so and declare every prototype; raises if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(f"libngp_hip.so not found at {path}: build it with `make -C instant-ngp-rendering_amd`")
    lib = C.CDLL(path)
    for name, (res, args) in EXPORTS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(status):
    if status != 0:
        raise RuntimeError(load().ngp_last_error().decode())


def default_config(n_levels=16, F=2, log2_T=19, base_res=16, per_level_scale=None, n_neurons=64,
                   density_hidden=1, rgb_hidden=2, aabb_scale=1, n_extra_dims=0):
    """Network config with the reference's auto-derived per_level_scale (src/testbed.cu:3709-3713)."""
    import numpy as np
    if per_level_scale is None:
        per_level_scale = float(np.exp(np.float32(np.log(np.float32(2048.0 * aabb_scale / base_res)))
                                       / np.float32(n_levels - 1))) if n_levels > 1 else 1.0
    c = NetworkConfig()
    c.n_levels, c.n_features_per_level, c.log2_hashmap_size, c.base_resolution = n_levels, F, log2_T, base_res
    c.per_level_scale = per_level_scale
    c.n_neurons, c.density_hidden_layers, c.rgb_hidden_layers = n_neurons, density_hidden, rgb_hidden
    c.rgb_activation, c.density_activation = 2, 3  # Logistic (LDR), Exponential
    c.learning_rate, c.beta1, c.beta2, c.epsilon, c.l2_reg = 1e-2, 0.9, 0.99, 1e-15, 1e-6
    c.ema_decay, c.decay_start, c.decay_interval, c.decay_base = 0.95, 20000, 10000, 0.33
    c.n_extra_dims = n_extra_dims
    return c
