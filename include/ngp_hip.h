/*
 * ngp_hip.h — C-ABI of the MI355X-native Instant-NGP NeRF hot path.
 *
 * One shared library, libngp_hip.so (instant-ngp-rendering_amd/), exports these
 * entry points.  Plain pointers and sizes only: no torch, tcnn or C++ types cross
 * this boundary.  Device pointers are hipMalloc'd (or torch-allocated) HBM
 * addresses; `ngp_stream` is a hipStream_t (0 = the null stream).
 *
 * Each entry names the reference interface it replaces (paths are relative to
 * the reference checkout, fnysalehi/instant-ngp-rendering):
 *
 *   ngp_model_create          NerfNetwork<T>::NerfNetwork    include/neural-graphics-primitives/nerf_network.h:81
 *                             + Testbed::reset_network        src/testbed.cu:3624 (hash-grid auto params :3680-3724,
 *                               Trainer/Optimizer creation :3726-3727,3846)
 *   ngp_model_encode          tcnn GridEncoding::inference_mixed_precision (called at nerf_network.h:113-118)
 *   ngp_model_infer           NerfNetwork::inference_mixed_precision_impl   nerf_network.h:105-139
 *   ngp_model_infer_padded    the same, 16-row padded output in the reference's CM / RM layouts
 *   ngp_model_density         NerfNetwork::density                          nerf_network.h:270-279
 *   ngp_train_step            Testbed::train_nerf_step        src/testbed_nerf.cu:2683-2930
 *                             (+ Trainer::optimizer_step      src/testbed_nerf.cu:2502, unless deferred)
 *   ngp_optimizer_step        Trainer::optimizer_step          src/testbed_nerf.cu:2502 (tcnn Ema∘ExponentialDecay∘Adam,
 *                                                              configs/nerf/base.json:5-22)
 *   ngp_train_read_stats      NerfCounters::update_after_training  src/testbed_nerf.cu:2422-2446
 *   ngp_allreduce_grads       (no reference counterpart: multi-GPU training is not supported upstream,
 *                             README.md:250-252) -- the data-parallel gradient reduction of SURVEY 8(e)
 *   ngp_density_grid_update   Testbed::update_density_grid_nerf     src/testbed_nerf.cu:2271-2360
 *                             + update_density_grid_mean_and_bitfield :2362-2379
 *   ngp_render                Testbed::render_nerf / NerfTracer      src/testbed_nerf.cu:1827-1987, 1556-1761
 *   ngp_accumulate_tonemap    CudaRenderBuffer::accumulate + tonemap src/render_buffer.cu:635-691 (kernels :232,:533)
 *
 * Error behaviour mirrors the reference: where the reference throws
 * std::runtime_error (CUDA_CHECK_THROW, invalid arguments), these return a
 * non-zero ngp_status and ngp_last_error() holds the message (thread-local).
 * A handle is thread-compatible, not thread-safe; one handle per device.
 */
#ifndef NGP_HIP_H
#define NGP_HIP_H

/* per-sample / per-image latent-code rows (n_extra_dims > 0): NGP_EXTRA_ROW floats, zero past n_extra_dims */
#define NGP_EXTRA_DIMS_MAX 32
#define NGP_EXTRA_ROW 32

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int ngp_status;
#define NGP_OK 0
#define NGP_ERR_INVALID 1
#define NGP_ERR_HIP 2
#define NGP_ERR_OOM 3
#define NGP_ERR_UNSUPPORTED 4

typedef struct ngp_model ngp_model;
typedef void* ngp_stream; /* hipStream_t */

/* Network + optimizer hyper-parameters (configs/nerf/base.json schema). */
typedef struct ngp_network_config {
	/* "encoding": HashGrid (configs/nerf/base.json:23-29) */
	uint32_t n_levels;
	uint32_t n_features_per_level; /* 1, 2, 4 or 8 */
	uint32_t log2_hashmap_size;
	uint32_t base_resolution;
	float per_level_scale; /* resolved on the host exactly as src/testbed.cu:3710-3713 */
	/* "network" / "rgb_network": FullyFusedMLP (configs/nerf/base.json:30-36,50-56) */
	uint32_t n_neurons;             /* 16, 32 or 64 */
	uint32_t density_hidden_layers; /* n_hidden_layers of "network" (1..3) */
	uint32_t rgb_hidden_layers;     /* n_hidden_layers of "rgb_network" (1..3) */
	/* activations (ENerfActivation, common.h:90-95) */
	int32_t rgb_activation;     /* 0 None, 1 ReLU, 2 Logistic, 3 Exponential */
	int32_t density_activation; /* default Exponential */
	/* "optimizer": Ema(decay) ∘ ExponentialDecay(start, interval, base) ∘ Adam */
	float learning_rate, beta1, beta2, epsilon, l2_reg;
	float ema_decay;
	uint32_t decay_start, decay_interval;
	float decay_base;
	/* NerfNetwork's n_extra_dims (nerf_network.h:81-84, NerfDataset::n_extra_dims(): light directions and the
	 * per-image latent code): the dir encoding's Identity part, appended to the rgb network's input after the
	 * SH (rgb input width next_multiple(32 + n_extra_dims, 16)).  0..NGP_EXTRA_DIMS_MAX (32: light directions
	 * 3 + the 16-wide learnable code of optimize_extra_dims, src/testbed.cu:4046-4053, fit); > 0 needs the
	 * 64-neuron network with one density and two rgb hidden layers and an encoding of <= 32 features
	 * (base.json / lego_L16F2.json).  Latent codes travel in rows of NGP_EXTRA_ROW floats. */
	uint32_t n_extra_dims;
} ngp_network_config;

/* Read-only model geometry. */
typedef struct ngp_model_info {
	uint64_t n_params;      /* total = n_mlp_params + n_grid_params */
	uint64_t n_mlp_params;  /* "matrix" params first (nerf_network.h:356-371 ordering) */
	uint64_t n_grid_params; /* hash-grid table entries x F */
	uint32_t n_levels;
	uint32_t n_features_per_level;
	uint32_t encoding_width;        /* n_levels * F */
	uint32_t padded_encoding_width; /* next multiple of 16 (tcnn alignment, nerf_network.h:82) */
	uint32_t level_offset[32];      /* entries, GridEncoding::level_params_offset */
	uint32_t level_size[32];
	uint32_t level_resolution[32];
	float level_scale[32];
	uint32_t n_layers;             /* density layers followed by rgb layers */
	uint32_t layer_in[8], layer_out[8];
	uint64_t layer_param_offset[8];
} ngp_model_info;

/* Parameter buffers, all with the reference ordering [density MLP | rgb MLP | hash grid]. */
enum {
	NGP_PARAMS_FP32 = 0,      /* fp32 master weights (tcnn Trainer full-precision params) */
	NGP_PARAMS_FP16 = 1,      /* fp16 training copy (network_precision_t) */
	NGP_PARAMS_EMA_FP32 = 2,  /* Ema optimizer's running average */
	NGP_PARAMS_INFER_FP16 = 3,/* fp16 inference params (use_inference_params=true) */
	NGP_GRADS_FP32 = 4,       /* gradient buffer (GradientMode::Overwrite each step); the MLP part
	                             [0, n_mlp_params) is used, hash-grid gradients live in GRID_FP16 */
	NGP_ADAM_M = 5,
	NGP_ADAM_V = 6,
	NGP_GRADS_GRID_FP16 = 7,  /* hash-grid gradients [n_params - n_mlp_params], fp16 as tcnn's GridEncoding
	                             backward keeps them; each backward adds into it (packed half2 atomics) */
	NGP_GRADS_GRID_FIXED64 = 8/* the same in deterministic steps: int64 fixed point, value = v * 2^-40 (allocated on the
	                             first deterministic step; null before) */
};

/* One training image; an array of these lives in device memory (TrainingImageMetadata,
 * include/neural-graphics-primitives/nerf_device.cuh:44-59 + TrainingXForm common.h:179-186). */
typedef struct ngp_image {
	uint64_t pixels;          /* device pointer to RGBA8 (sRGB, straight alpha) rows, width*height texels */
	uint32_t width, height;
	float focal_length[2];    /* pixels */
	float principal_point[2]; /* [0,1] */
	float xform[12];          /* camera-to-world 4x3, column-major (right, up, forward, origin), NGP space */
	int32_t lens_mode;        /* 0 Perspective (others: ELensMode, common.h:188-195) */
	float lens_params[7];
	/* depth supervision target (TrainingImageMetadata::depth, nerf_device.cuh:44-59): device pointer to
	 * width*height f32 depths along the optical axis, already multiplied by integer_depth_scale and the
	 * dataset scale (src/nerf_loader.cu:73-82, 728); 0 = no depth for this image */
	uint64_t depth;
	/* rolling shutter / motion blur (TrainingXForm::end, TrainingImageMetadata::rolling_shutter;
	 * get_xform_given_rolling_shutter common_device.cuh:633-636): the ray's camera is
	 * camera_slerp(xform, xform_end, A + B u + C v + D motionblur_time); all-zero = xform (the
	 * sampler honours it in its general instance: set ngp_train_args.has_lens) */
	float xform_end[12];
	float rolling_shutter[4];
} ngp_image;

typedef struct ngp_train_args {
	const ngp_image* images; /* device array [n_images] */
	uint32_t n_images;
	uint32_t n_rays;             /* rays_per_batch (NerfCounters, adapts on the host) */
	uint32_t n_rays_total;       /* running ray count (unused by the default sampler; kept for parity) */
	uint32_t target_batch_size;  /* 2^18 (testbed.h:1015) */
	uint32_t max_samples;        /* max_inference: samples the sampler may emit */
	uint32_t training_step;      /* m_training_step before the step */
	uint64_t rng_state, rng_inc; /* m_rng (pcg32) state; the caller advances it after the step */
	uint32_t ray_index_offset;   /* data-parallel: this rank's first global ray index */
	uint32_t n_rays_global;      /* data-parallel: rays over all ranks (image_idx denominator); 0 = n_rays */
	float aabb_min[3], aabb_max[3];
	float cone_angle_constant;
	uint32_t max_cascade;
	int32_t loss_type;        /* ELossType */
	int32_t random_bg_color;  /* nerf.training.random_bg_color */
	float background_color[3];/* sRGB, used when random_bg_color == 0 */
	int32_t snap_to_pixel_centers;
	int32_t train_in_linear_colors;
	int32_t color_space;      /* EColorSpace: 0 Linear, 1 SRGB */
	float near_distance;
	int32_t optimize_mlp;      /* m_train_network */
	int32_t optimize_encoding; /* m_train_encoding */
	int32_t defer_optimizer;   /* 1: leave grads for an external all-reduce, then call ngp_optimizer_step */
	/* error map (Nerf::Training::ErrorMap, nerf.h:50-59; compute_loss_kernel_train_nerf
	 * src/testbed_nerf.cu:1028-1054; nerf_random_image_pos_training / image_idx nerf_device.cuh:552-598) */
	float* error_map;           /* device [n_images][res_y][res_x] f32: += each ray's mean loss, bilinear; null = off */
	uint32_t error_map_res[2];  /* x, y */
	const float* cdf_x_cond_y;  /* device [n_images][cdf_res_y][cdf_res_x]: sample_focal_plane_proportional_to_error; null = uniform */
	const float* cdf_y;         /* device [n_images][cdf_res_y] */
	const float* cdf_img;       /* device [n_images] normalised image CDF: sample_image_proportional_to_error; null = uniform */
	uint32_t cdf_res[2];        /* x, y */
	int32_t has_lens;           /* 1 if any image has a non-pinhole lens or a rolling shutter (selects the general sampler kernels) */
	/* per-image exposure (Nerf::Training::cam_exposure, src/testbed_nerf.cu:966-985, 1121-1134) */
	const float* exposure;      /* device [n_images][3] log2 scale of the target colours; null = 0 */
	float* exposure_gradient;   /* device [n_images][3] += dL/dexposure of the kept rays; null = off */
	/* extrinsics (compute_cam_gradient_train_nerf, src/testbed_nerf.cu:1163-1269): device [n_images][3]
	 * += the kept rays' origin gradient (translation) and cross(dir, dir gradient) (rotation, angle-axis),
	 * divided by the pixel pdf; null = off */
	float* cam_pos_gradient;
	float* cam_rot_gradient;
	/* 1: run the network over every emitted sample before the loss, as the reference does
	 * (src/testbed_nerf.cu:2797-2802); 0: the early-terminated chunked forward, which evaluates
	 * each ray only up to its transmittance stop (identical loss/compaction/gradients, see
	 * train_stats.forward_early_stop_violations) */
	int32_t full_forward;
	/* depth supervision (compute_loss_kernel_train_nerf, src/testbed_nerf.cu:1013-1015, 1098-1103):
	 * with lambda > 0, rays of images with depth add lambda * d loss(target depth, composited depth)
	 * to dL/d(density) through the depth suffix; depth_loss_type is an ELossType (default L1) */
	float depth_supervision_lambda;
	int32_t depth_loss_type;
	/* sharpness-weighted error deposits (include_sharpness_in_error, src/testbed_nerf.cu:1036-1044,
	 * 2453-2464): sharpness_data = device [n_images][res_y][res_x] variance of the Laplacian of the
	 * images' luma (compute_sharpness, src/nerf_loader.cu:111-151); sharpness_grid = device
	 * [8 cascades][128^3] f32 running max (Morton order), zeroed when sharpness_grid_clear, else
	 * decayed by 0.95 at the start of the step; null = off */
	const float* sharpness_data;
	uint32_t sharpness_res[2];
	float* sharpness_grid;
	int32_t sharpness_grid_clear;
	/* learned image-plane distortion (Testbed::m_distortion, a TrainableBuffer<2, 2, float>):
	 * distortion_map = device [res_y][res_x][2] f32 added to the camera-space ray direction's xy at the
	 * pixel's uv, bilinear (uv_to_ray common_device.cuh:441-443, Buffer2DView::at_lerp common.h:249-266);
	 * null = off.  distortion_gradient / distortion_gradient_weight = device [res_y][res_x][2] += the
	 * kept rays' image-plane direction gradient / 1 (bilinear; compute_cam_gradient_train_nerf
	 * src/testbed_nerf.cu:1234-1246, deposit_image_gradient common_device.cuh:82-115); null = off */
	const float* distortion_map;
	uint32_t distortion_res[2];
	float* distortion_gradient;
	float* distortion_gradient_weight;
	/* data parallelism: this rank's slice of the global batch.  n_rays / ray_index_offset
	 * are the rank's rays of the n_rays_global of the step; target_batch_size and max_samples are the
	 * GLOBAL values.  The step calls allreduce_i32 (sum of world_size int32 device words, on `stream`)
	 * twice -- after sampling and after the loss composite -- to learn every rank's totals, so the
	 * sampler's max_samples cap, the compaction cap and the rollover (tcnn fill_rollover_and_rescale)
	 * apply to the global ray order exactly as in one process training n_rays_global rays
	 * (src/testbed_nerf.cu:779-781, 997-1003, 2862-2870).  world_size <= 1 or a null callback: one
	 * process (rank must be 0). */
	uint32_t rank, world_size;
	ngp_status (*allreduce_i32)(void* user, int32_t* dev, uint32_t n, ngp_stream stream);
	void* allreduce_user;
	/* 1: hash-grid gradients accumulate as 64-bit fixed point (2^-40 units, NGP_GRADS_GRID_FIXED64) with
	 * integer atomics -- order-independent sums, so a step is bit-reproducible and data-parallel ranks
	 * sum exactly (deterministic mode); the optimizer rounds each sum to fp16 once (the
	 * gradient buffer's precision, so the sparse skip sees the same zeros); 0: packed fp16 atomics as
	 * tcnn's GridEncoding backward */
	int32_t deterministic;
	/* Testbed::m_max_level_rand_training (src/testbed_nerf.cu:724, 949, 2797, 2805; python_api.cu:527):
	 * every training ray draws max_level = 2 u (after its pixel, before motionblur_time -- the same
	 * pcg32 draw in the sampler and the loss pass) and the hash-grid levels l >= max_level * L (+1e-3)
	 * of its samples encode to zero and receive no gradient (tcnn GridEncoding::set_max_level_gpu);
	 * the value rides in the pad float of the sample's coordinate row.  0: all levels. */
	int32_t max_level_rand_training;
	/* n_extra_dims > 0 (per-image latent codes, Nerf::Training::extra_dims_gpu, src/testbed_nerf.cu:706-730, 824):
	 * extra_dims = device fp32 [n_images][NGP_EXTRA_ROW], image i's code in row i (zero past n_extra_dims); every sample of
	 * a ray from image i carries row i (NerfCoordinate::set_with_optional_extra_dims); null = zeros.
	 * extra_dims_gradient (optional, device fp32 [n_images][NGP_EXTRA_ROW]) += sum over the kept rays' compacted samples of
	 * dL/d(code) (compute_extra_dims_gradient_train_nerf, src/testbed_nerf.cu:1271-1306; loss-scaled, as the
	 * reference's gradient before its division by LOSS_SCALE at :2588).  Both 16-byte aligned (float4 rows). */
	const float* extra_dims;
	float* extra_dims_gradient;
} ngp_train_args;

typedef struct ngp_train_stats {
	uint32_t n_rays;
	uint32_t n_rays_with_samples;
	uint32_t measured_batch_size_before_compaction; /* numsteps_counter */
	uint32_t measured_batch_size;                   /* numsteps_counter_compacted */
	float loss;                                     /* sum over rays of mean per-ray loss / n_rays */
	/* rays whose loss composite needed a sample the chunked forward had not evaluated (the
	 * chunk stop and the loss stop disagree); must be 0 -- the Testbed switches to the full
	 * forward for the rest of the run if it is not */
	uint32_t forward_early_stop_violations;
	/* data parallelism: 1 if some rank's share of the step's samples did not fit its buffers (sized about
	 * 2 / world_size of max_samples); the step made no update or deposits -- discard it (ngp_train_discard)
	 * and run it again: the rank's buffers grow to the need */
	uint32_t sample_capacity_overflow;
} ngp_train_stats;

typedef struct ngp_grid_args {
	const ngp_image* images; /* device array, for mark_untrained_density_grid */
	uint32_t n_images;
	float aabb_min[3], aabb_max[3];
	uint32_t max_cascade;
	float decay;                     /* nerf.training.density_grid_decay */
	uint32_t n_uniform_samples;      /* NERF_GRID_N_CELLS * n_cascades (first 256 steps) or /4 */
	uint32_t n_nonuniform_samples;
	uint64_t rng_state, rng_inc;     /* nerf.training.density_grid_rng; advanced by 2^32 twice inside */
	uint32_t ema_step;               /* m_nerf.density_grid_ema_step */
	int32_t mark_untrained;          /* step 0 / image-count change (src/testbed_nerf.cu:2293-2309) */
	int32_t clear_visible;           /* m_training_step == 0 */
	int32_t use_inference_params;    /* reference passes false (:2350) */
	uint32_t rank, world_size;       /* data-parallel: evaluate a 1/world_size slice, caller all-reduces (max) tmp */
} ngp_grid_args;

/* A uniform lattice over a box, evaluated by the density network (Testbed::get_density_on_grid,
 * src/testbed_nerf.cu:3026-3075, which compute_and_save_png_slices writes out, src/testbed.cu:534-559). */
typedef struct ngp_grid_query {
	uint32_t res[3];                 /* lattice points per axis (x fastest in the output) */
	float box_min[3], box_max[3];    /* the lattice's box (m_render_aabb by default) */
	float box_to_local[9];           /* row-major; lattice point p is placed at transpose(M) * p (all-zero = identity) */
	float aabb_min[3], aabb_max[3];  /* m_aabb: the network input warp and the density-grid lookup */
	uint32_t max_cascade;
	int32_t mask_with_grid;          /* 1: -10000 where the density grid at mip_from_pos is below
	                                    NERF_MIN_OPTICAL_THICKNESS (grid_samples_half_to_float, :234-250) */
	int32_t use_inference_params;    /* 1: the EMA parameters, as NerfNetwork::density does */
} ngp_grid_query;

typedef struct ngp_render_args {
	uint32_t width, height;
	uint32_t sample_index;   /* spp index of this frame */
	float camera[12];        /* 4x3 column-major camera-to-world (NGP space) */
	float focal_length[2];   /* pixels */
	float screen_center[2];
	float near_distance;     /* m_render_near_distance */
	float aabb_min[3], aabb_max[3];     /* render aabb (m_render_aabb) */
	float train_aabb_min[3], train_aabb_max[3]; /* m_aabb (network input warp) */
	float cone_angle_constant;
	uint32_t max_cascade;
	float min_transmittance; /* nerf.render_min_transmittance */
	int32_t snap_to_pixel_centers;
	int32_t use_inference_params; /* 1 = EMA params (render default) */
	int32_t train_in_linear_colors;
	/* row sharding for multi-GPU (config C): render rows y with (y / shard_rows) % shard_count == shard_index */
	uint32_t shard_index, shard_count, shard_rows;
	/* Nerf::render_lens when render_with_lens_distortion (src/testbed_nerf.cu:1859): ELensMode + params */
	int32_t lens_mode;
	float lens_params[7];
	/* motion blur / rolling shutter of rendered rays (init_rays_with_payload_kernel_nerf,
	 * src/testbed_nerf.cu:1416): camera_slerp(camera, camera_end, A + B u + C v + D
	 * ld_random_val(sample_index, pixel * 72239731)); all-zero rolling_shutter = camera */
	float camera_end[12];
	float rolling_shutter[4];
	/* the learned distortion map (m_distortion.inference_view(), src/testbed_nerf.cu:1854-1857) when
	 * render_with_lens_distortion: device [res_y][res_x][2] f32; null = off */
	const float* distortion_map;
	uint32_t distortion_res[2];
	/* the crop box's frame (Testbed::m_render_aabb_to_local, NerfDataset::render_aabb_to_local): positions are
	 * tested against aabb_min / aabb_max after this row-major 3x3 map (if_unoccupied_advance_to_next_occupied_voxel,
	 * nerf_device.cuh:461-494; init_rays_with_payload_kernel_nerf, src/testbed_nerf.cu:1465-1475); all zeros =
	 * identity */
	float render_aabb_to_local[9];
	/* Testbed::m_render_mode (ERenderMode, common.h:56-67) as NGP_RENDER_MODE_* below; 0 = Shade */
	int32_t render_mode;
	float depth_scale;          /* Depth mode: 1 / dataset scale (src/testbed_nerf.cu:1905) */
	int32_t gbuffer_hard_edges; /* Nerf::render_gbuffer_hard_edges: Depth / Positions from the max-weight sample */
	/* depth of field (uv_to_ray, common_device.cuh:450-456): aperture_size != 0 jitters the ray origin over a disk
	 * on the lens and aims it at the focus plane at camera-space depth focus_z (the reference passes plane_z =
	 * slice_plane_z + scale); Slice mode renders the density / colour slice at depth focus_z instead of tracing */
	float aperture_size;
	float focus_z;
	/* Nerf::glow_mode / glow_y_cutoff (composite_kernel_nerf's glow, src/testbed_nerf.cu:540-628): bit 0 green grid,
	 * bit 1 green cut line, bit 2 mask to alpha, bit 3 radial distance, bit 4 grid mode; 0 = off */
	int32_t glow_mode;
	float glow_y_cutoff;
	/* n_extra_dims > 0: the latent code every rendered sample carries (Nerf::get_rendering_extra_dims,
	 * src/testbed_nerf.cu:3206-3228): device fp32 [NGP_EXTRA_ROW], zero past n_extra_dims; null = zeros; 16-byte aligned */
	const float* extra_dims;
	/* optional (render(): one spp, Shade mode without glow, unsharded): the frame's tonemapped pixels streamed into
	 * caller-owned page-locked host memory [H][W][4] by the kernels that finish their rays, while the march goes
	 * on -- the value ngp_accumulate_tonemap(frame, accum, out, W, H, 0, host_color_space, host_exposure,
	 * host_background, host_output_srgb) leaves in `out`, bit for bit, without the read-back after the frame
	 * (render_to_cpu's copy, src/python_api.cu:124-202).  *host_frame_complete (host memory) is set to 1 when every
	 * pixel was written, 0 when some rays ran out of march iterations (k_retire) and the caller copies the frame
	 * instead.  null = off. */
	float* host_frame;
	int32_t* host_frame_complete;
	float host_background[4];
	float host_exposure;
	int32_t host_color_space;
	int32_t host_output_srgb;
} ngp_render_args;

/* ngp_render_args.render_mode (the reference's ERenderMode; Distortion and EncodingVis are GUI
 * visualisations of this build's scope and are refused) */
enum {
	NGP_RENDER_MODE_SHADE = 0,
	NGP_RENDER_MODE_AO = 1,
	NGP_RENDER_MODE_NORMALS = 2,
	NGP_RENDER_MODE_POSITIONS = 3,
	NGP_RENDER_MODE_DEPTH = 4,
	NGP_RENDER_MODE_COST = 5,
	NGP_RENDER_MODE_SLICE = 6
};

/* Launch shapes and march schedule of the gfx950 kernels (no reference counterpart).  None of
 * them changes a result -- every ray composites its own samples in order whatever the pass
 * split, and the kernel variants compute the same values -- only the speed.  0 = the measured
 * default.  Per model; ngp_model_create starts from all zeros. */
typedef struct ngp_tuning {
	uint32_t render_pipelines;       /* ray pipelines on their own streams, 1..4; 0: 2 for frames of >= 2^16 rays */
	uint32_t render_pass_samples;    /* a pipeline's sample-slot budget per march pass (<= 2^24); 0: 6 * 2^20 for a volume
	                                    (the last frame >= 12 samples per ray), else 3 * 2^20 */
	uint32_t render_lanes;           /* lane budget from which k_generate picks lanes per ray; 0: 2^22 */
	uint32_t render_first_steps;     /* per-ray sample cap of the first pass (doubling per pass); 0: 8 after a frame of >= 12 samples per ray, else 4 */
	uint32_t render_max_steps;       /* per-ray sample cap of any pass; 0: 32 for a volume, 24 for a surface scene */
	uint32_t render_lag;             /* passes a pipeline runs ahead of its counter read-backs, 2..4; 0: 2 */
	float render_budget_scale;       /* headroom of the per-ray transmittance budget; 0: 1.0; < 0: no budget */
	uint32_t render_composite_block; /* k_composite workgroup size (256, 512, 1024); 0: 512 */
	uint32_t render_generate_block;  /* k_generate workgroup size (256, 512); 0: 512 */
	uint32_t encode_dense_records;   /* render-site corner records of the dense levels: 0 on, 1 off */
	uint32_t mlp_workgroups_per_cu;  /* inference-MLP workgroups per CU; 0: the render MLP's resident count (2 at 64-sample
	                                    steps, 4 at 32), else 8 */
	uint32_t debug;                  /* bit 0: per-frame march statistics on stderr; bit 1: per-step sampler statistics;
	                                    bit 2: the chunked training forward stops rays at transmittance 0.999 (forces
	                                    forward_early_stop_violations: exercises the discard-and-retry path);
	                                    bit 3: data-parallel sample buffers start at an eighth of a rank's even share
	                                    (forces sample_capacity_overflow and the retry with grown buffers);
	                                    bit 4: renders stop marching after 40 lattice steps per ray (the retire path) */
	uint32_t encode_streaming;       /* hash encoder (F = 2 planes): 0 = non-temporal encoding stores (the default), 1 = plain */
	uint32_t grid_unsorted;          /* density-grid update sample order (the same grid either way): 0 = bucketed by
	                                    cell (top 14 Morton bits; coherent gathers), 1 = drawing order, 2 = fully sorted
	                                    by cell (hipCUB radix sort) */
	uint32_t render_mlp_tile;        /* render MLP samples per wave step: 1 = 16, 2 = 32, 4 = 64; 0: 64 with two or more
	                                    ray pipelines, 32 with one */
	uint32_t encode_xcd_regions;     /* four-levels-per-thread hash encoder: 0 = each XCD encodes one contiguous eighth of
	                                    the samples (the default), 1 = XCD x takes every eighth chunk */
	uint32_t render_skip_unfilled;   /* 1 = the render MLP skips 16-sample column tiles of slots no ray filled (marked
	                                    by k_generate), 2 = computes every reserved slot; 0: the default (1) */
	uint32_t render_exit_cap;        /* 1 = a ray reserves at most the lattice points left to its AABB exit in a march
	                                    pass, 2 = the per-ray cap alone; 0: the default (2) */
	uint32_t render_priority;        /* wave issue priority (s_setprio 0..3) of the render kernels sharing the CUs:
	                                    bits 0-1 the encoder, 2-3 the MLP, 4-5 the march kernels; 0: all 0 */
	uint32_t render_host_frame;      /* Testbed::render into host memory: 1 = pixels streamed by the kernels
	                                    (ngp_render_args.host_frame), 2 = tonemap then one read-back; 0: the default */
	uint32_t train_chunk_lanes;      /* lanes per ray of the chunked training forward's k_train_chunk (4, 8, 16, 32 or 64);
	                                    0: 64 for batches of <= 4096 rays, else 16 */
	uint32_t train_sampler_lanes;    /* lanes per ray of the training sampler's two passes (8, 16, 32 or 64); 0: 64 */
	uint32_t render_mlp_pipeline;    /* render MLP load pipeline: 1 = round-5 ring (a tile's SH rows fetched right after its
	                                    row indices), 2 = decoupled (row indices two tiles ahead, encodings one, SH rows
	                                    one), 3 = decoupled with encodings two tiles ahead; 0: the default (2) */
} ngp_tuning;

/* --- lifecycle -------------------------------------------------------------------- */
ngp_status ngp_model_create(int hip_device, const ngp_network_config* cfg, uint64_t seed, ngp_model** out);
ngp_status ngp_model_set_tuning(ngp_model* model, const ngp_tuning* tuning);
/* The checks ngp_model_set_tuning applies, without a model (NGP_ERR_INVALID + ngp_last_error on a bad value). */
ngp_status ngp_tuning_validate(const ngp_tuning* tuning);
ngp_status ngp_model_get_tuning(const ngp_model* model, ngp_tuning* tuning);
ngp_status ngp_model_destroy(ngp_model* model);
ngp_status ngp_model_get_info(const ngp_model* model, ngp_model_info* info);
ngp_status ngp_model_buffer(ngp_model* model, int kind, void** dev_ptr, size_t* bytes);
/* After writing NGP_PARAMS_FP32 (e.g. snapshot load): refresh fp16 / EMA / inference copies. */
ngp_status ngp_model_params_updated(ngp_model* model, int reset_optimizer, ngp_stream stream);
ngp_status ngp_model_reset_optimizer(ngp_model* model, ngp_stream stream);

/* --- network evaluation ------------------------------------------------------------ */
/* pos: n positions in [0,1]^3, `stride` floats apart.  enc_out: [n_levels][n][F] fp16 (level-major). */
ngp_status ngp_model_encode(ngp_model* model, const float* pos, uint32_t stride, uint32_t n,
                            uint16_t* enc_out, int use_inference_params, ngp_stream stream);
/* Debug/parity: corner indices [n][n_levels][8] and trilinear weights [n][n_levels][8]. */
ngp_status ngp_model_encode_indices(ngp_model* model, const float* pos, uint32_t stride, uint32_t n,
                                    uint32_t* idx_out, float* w_out, ngp_stream stream);
/* coords: NerfCoordinate records (pos[3], dt, dir[3], extra...) of `floats_per_coord` floats (n_extra_dims > 0: the
 * sample's latent code at floats 7 .. 7 + n_extra_dims, floats_per_coord >= 7 + n_extra_dims).
 * out: [n][4] fp16 = (rgb raw x3, density raw) (the 16-row padded output of the reference, rows 0-3). */
ngp_status ngp_model_infer(ngp_model* model, const float* coords, uint32_t floats_per_coord, uint32_t n,
                           uint16_t* out, int use_inference_params, ngp_stream stream);
/* The reference's full network output: padded_output_width() = 16 fp16 rows per sample (rows 0-2
 * rgb raw, row 3 density raw -- extract_density, nerf_network.h:32-43, 132-138 -- rows 4-15 the rgb
 * network's remaining outputs), column-major as training reads it (src/testbed_nerf.cu:2801:
 * sample i's 16 rows at out[i * out_stride], out_stride >= 16) or row-major as the renderer reads
 * it (:1720: row r of sample i at out[r * out_stride + i], out_stride >= n). */
ngp_status ngp_model_infer_padded(ngp_model* model, const float* coords, uint32_t floats_per_coord, uint32_t n,
                                  uint16_t* out, uint32_t out_stride, int layout_rm, int use_inference_params,
                                  ngp_stream stream);
/* The renderer's network call (NerfTracer's inference_mixed_precision on the compacted samples,
 * src/testbed_nerf.cu:1720): enc [n_levels][n][F] fp16 (level-major, as ngp_model_encode writes), sh_rows
 * [n_rows][16] fp16 = the degree-4 SH of each ray's warped direction (the dir encoding, computed once per ray),
 * sh_row_of_sample [n] u32 = the row of each sample.  out: [n][4] fp16 as ngp_model_infer.  Timed by
 * NGP_TIMER_RENDER_MLP (the MLP dispatch alone).  Networks without extra dims.  Untuned (ngp_tuning render_mlp_pipeline /
 * render_mlp_tile / mlp_workgroups_per_cu 0) it runs the schedule measured best for the network alone on the GPU
 * (the two-tile-deep ring at 32-sample steps, 4 workgroups per CU), not the renderer's. */
ngp_status ngp_model_infer_sh_rows(ngp_model* model, const uint16_t* enc, const uint16_t* sh_rows,
                                   const uint32_t* sh_row_of_sample, uint32_t n, uint32_t n_rows, uint16_t* out,
                                   int use_inference_params, ngp_stream stream);
/* pos: n positions (stride floats). out: [n] fp16 raw density (row 0 of the density MLP output). */
ngp_status ngp_model_density(ngp_model* model, const float* pos, uint32_t stride, uint32_t n,
                             uint16_t* out, int use_inference_params, ngp_stream stream);
/* Parity entry for the fused MLP backward (NerfNetwork::backward_impl, nerf_network.h:189-268):
 * enc [n_levels][n][F] fp16, dirs [n][3] (warped to [0,1]), dL_dout [n][4] fp16 (loss-scaled),
 * sample_weight [n] fp32 (rollover multiplicity, may be NULL). Accumulates MLP grads into
 * NGP_GRADS_FP32 and writes dL_denc [n_levels][n][F] fp16. */
ngp_status ngp_model_backward(ngp_model* model, const uint16_t* enc, const float* dirs, uint32_t n,
                              const uint16_t* dL_dout, const float* sample_weight, uint16_t* dL_denc,
                              ngp_stream stream);
/* The same with the rgb network's extra inputs (n_extra_dims > 0): extra [n][NGP_EXTRA_ROW] fp32 latent codes of the
 * samples (zero past n_extra_dims); dL_dextra (optional) [n][NGP_EXTRA_ROW] fp32 = dL/d(code) of each sample's own row (the network's
 * input gradient that compute_extra_dims_gradient_train_nerf sums, divided by sample_weight). */
ngp_status ngp_model_backward_extra(ngp_model* model, const uint16_t* enc, const float* dirs, const float* extra, uint32_t n,
                                    const uint16_t* dL_dout, const float* sample_weight, uint16_t* dL_denc,
                                    float* dL_dextra, ngp_stream stream);
/* Parity entry for the hash-grid backward scatter: dL_denc [n_levels][n][F] fp16 -> grads. */
ngp_status ngp_model_encode_backward(ngp_model* model, const float* pos, uint32_t stride, uint32_t n,
                                     const uint16_t* dL_denc, ngp_stream stream);

/* --- training ---------------------------------------------------------------------- */
ngp_status ngp_train_step(ngp_model* model, const ngp_train_args* args, ngp_stream stream);
ngp_status ngp_optimizer_step(ngp_model* model, uint32_t training_step, int optimize_mlp, int optimize_encoding,
                              ngp_stream stream);
ngp_status ngp_train_read_stats(ngp_model* model, ngp_train_stats* stats, ngp_stream stream);
/* Data-parallel training: sum the model's gradients over an RCCL communicator (an ncclComm_t):
 * the fp32 MLP gradients and the fp16 hash-grid gradients, in one group on `stream`.  Call it
 * between ngp_train_step (defer_optimizer = 1) and ngp_optimizer_step on every rank.  After a
 * deterministic step the hash-grid part is the int64 fixed-point buffer (an exact integer sum). */
ngp_status ngp_allreduce_grads(ngp_model* model, void* nccl_comm, ngp_stream stream);
/* Debug/parity: device pointers to the last step's scratch (valid until the next step). */
enum {
	NGP_SCRATCH_RAY_NUMSTEPS = 0, /* [n_rays][2] u32: (numsteps, base) after sampling */
	NGP_SCRATCH_COORDS = 1,       /* [max_samples][8] f32: pos3, dt, dir3, pad */
	NGP_SCRATCH_MLP_OUT = 2,      /* [max_samples][4] f16; the first RAY_EVALUATED samples of each ray */
	NGP_SCRATCH_RAY_COMPACTED = 3,/* [n_rays][2] u32: (compacted numsteps, compacted base) */
	NGP_SCRATCH_DLOSS = 4,        /* [target_batch][4] f16 */
	NGP_SCRATCH_LOSS = 5,         /* [n_rays] f32 */
	NGP_SCRATCH_COMPACT_COORDS = 6,/* [target_batch][8] f32 */
	NGP_SCRATCH_RAY_EVALUATED = 7,/* [n_rays] u32: samples of the ray the forward evaluated (bit 31 set); it
	                                 stops once the transmittance is below the loss's threshold. Null when
	                                 every sample was evaluated (full_forward) */
	NGP_SCRATCH_VIOLATIONS = 8    /* 1 u32: the last step's forward_early_stop_violations.  ngp_optimizer_step
	                                 skips the whole update while it is non-zero (data-parallel callers all-reduce
	                                 it with max first); ngp_train_discard then clears the step for a re-run */
};
ngp_status ngp_train_scratch(ngp_model* model, int kind, void** dev_ptr, size_t* bytes);
/* Drops the last step's gradients (MLP and hash grid) before the step is run again -- after a chunked
 * forward reported forward_early_stop_violations, which made its optimizer step a no-op. */
ngp_status ngp_train_discard(ngp_model* model, ngp_stream stream);
/* Data-parallel: the violation word (NGP_SCRATCH_VIOLATIONS) as two int32 parts on the device, so a caller can
 * max-reduce them over the ranks without a host round trip.  to_parts = 1: parts[0] = early-stop count,
 * parts[1] = 1 when this rank's samples overflowed its capacity; to_parts = 0: the word is rebuilt from the
 * (reduced) parts.  parts: 2 int32 of device memory; stream-ordered. */
ngp_status ngp_train_violation_parts(ngp_model* model, int32_t* parts, int to_parts, ngp_stream stream);

/* --- occupancy grid ------------------------------------------------------------------ */
ngp_status ngp_density_grid_update(ngp_model* model, const ngp_grid_args* args, ngp_stream stream);
/* Split form for data-parallel grids: sample+evaluate into tmp, caller all-reduces tmp (max), then finish. */
ngp_status ngp_density_grid_evaluate(ngp_model* model, const ngp_grid_args* args, ngp_stream stream);
ngp_status ngp_density_grid_finish(ngp_model* model, const ngp_grid_args* args, ngp_stream stream);
/* Recompute mean + bitfield + mips from the current grid (update_density_grid_mean_and_bitfield). */
ngp_status ngp_density_grid_bitfield(ngp_model* model, uint32_t max_cascade, ngp_stream stream);
/* grid: [n_cascades][128^3] f32 (Morton order); bitfield: [8][128^3/8] u8; tmp: evaluation buffer;
 * mean: 1 f32 (device). */
ngp_status ngp_density_grid_buffers(ngp_model* model, float** grid, uint8_t** bitfield, float** tmp, float** mean);
/* Testbed::get_density_on_grid (src/testbed_nerf.cu:3026-3075): out[x + y*res.x + z*res.x*res.y] (device, f32) =
 * the raw density-network output (the fp16 value, widened) at lattice point (x, y, z) / (res - 1) of the box
 * (generate_grid_samples_nerf_uniform, :147-160), evaluated in batches of 2^20 points. */
ngp_status ngp_density_on_grid(ngp_model* model, const ngp_grid_query* query, float* out, ngp_stream stream);

/* --- error map ------------------------------------------------------------------------ */
/* construct_cdf_2d + construct_cdf_1d (src/testbed_nerf.cu:1493-1546): per image, the row-wise
 * conditional CDFs of the error map (MIN_PDF 0.01 mixed in), the row CDF, and cdf_img[i] = the
 * image's unnormalised total (the caller normalises it on the host, src/testbed_nerf.cu:2553-2567).
 * All arrays are device pointers; no model needed. */
ngp_status ngp_error_map_build_cdf(const float* error_map, uint32_t n_images, uint32_t res_x, uint32_t res_y,
                                   float* cdf_x_cond_y, float* cdf_y, float* cdf_img, ngp_stream stream);

/* --- rendering --------------------------------------------------------------------- */
/* frame: [H][W][4] f32 premultiplied RGBA, depth: [H][W] f32 (device, caller-owned);
 * cleared and shaded for the rows this shard owns. */
ngp_status ngp_render(ngp_model* model, const ngp_render_args* args, float* frame, float* depth, ngp_stream stream);
/* accumulate_kernel + tonemap_kernel (render_buffer.cu:232,533): accum = running mean over spp,
 * out = accum composited over background, exposure/tonemap(Identity), colour-space conversion. */
ngp_status ngp_accumulate_tonemap(const float* frame, float* accum, float* out, uint32_t width, uint32_t height,
                                  uint32_t sample_count, int color_space, float exposure,
                                  const float* background_rgba, int output_srgb, ngp_stream stream);

/* --- kernel timers (no reference counterpart: instrumentation for bench.py) ---------- */
/* When enabled, each hot-path launch group is bracketed by HIP events on the stream it
 * runs on; ngp_timing_read() synchronises those events and returns the summed duration,
 * the number of launches and the algorithmic units processed (samples for encode/MLP,
 * rays for sampler/loss/march, parameters for the optimizer).  Training-step units are
 * known only on the device; they are attributed when ngp_train_read_stats() reads them. */
enum {
	NGP_TIMER_TRAIN_SAMPLER = 0,    /* generate_training_samples_nerf (rays)            */
	NGP_TIMER_TRAIN_ENCODE = 1,     /* hash-grid forward over all samples (samples)     */
	NGP_TIMER_TRAIN_MLP_INFER = 2,  /* fused MLP inference over all samples (samples)   */
	NGP_TIMER_TRAIN_LOSS = 3,       /* compute_loss_kernel_train_nerf + compaction (rays)*/
	NGP_TIMER_TRAIN_MLP_BWD = 4,    /* fused MLP fwd+bwd on the compacted batch (samples)*/
	NGP_TIMER_TRAIN_ENCODE_BWD = 5, /* hash-grid backward scatter (samples)             */
	NGP_TIMER_OPTIMIZER = 6,        /* Ema/ExponentialDecay/Adam step (params)          */
	NGP_TIMER_GRID_UPDATE = 7,      /* density-grid evaluate + EMA + bitfield (cells)   */
	NGP_TIMER_RENDER_ENCODE = 8,    /* render: hash-grid forward (samples)              */
	NGP_TIMER_RENDER_MLP = 9,       /* render: fused MLP inference (samples)            */
	NGP_TIMER_RENDER_MARCH = 10,    /* render: init/compact/generate/composite (rays)   */
	NGP_TIMER_COUNT = 11
};
/* mask: bit k enables timer k (-1 = all, 0 = off); events cost a few microseconds of GPU
 * time each, so a timed run enables only the timers it reports. */
ngp_status ngp_timing_enable(ngp_model* model, int mask);
ngp_status ngp_timing_read(ngp_model* model, int timer, double* total_ms, uint64_t* units, uint32_t* launches,
                           int reset);

const char* ngp_last_error(void);
const char* ngp_version(void);

#ifdef __cplusplus
}
#endif

#endif /* NGP_HIP_H */
