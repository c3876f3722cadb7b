// testbed.h — host-side Testbed for the MI355X NeRF path (no device code).
//
// Mirrors the reference Testbed's NeRF surface (include/neural-graphics-primitives/
// testbed.h, src/testbed.cu, src/testbed_nerf.cu): dataset loading, network
// (re)configuration, train()/frame(), render(), snapshots, camera helpers.  All
// GPU work goes through the C-ABI of libngp_hip.so (include/ngp_hip.h).
#pragma once

#include <array>
#include <cstdint>
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "../../include/ngp_hip.h"

namespace ngp {
// Page-locked host buffers for frame read-backs, recycled through a small per-size pool (hipHostMalloc
// costs milliseconds; a frame read-back into pageable memory runs at about a fifth of the DMA rate).
void* pinned_host_alloc(size_t bytes);
void pinned_host_release(void* p, size_t bytes);
}  // namespace ngp
#include "json.h"

namespace ngp {
struct pcg32;

enum class ETestbedMode : int { Nerf, Sdf, Image, Volume, Geometry, None };
enum class EColorSpace : int { Linear, SRGB, VisPosNeg };
enum class ELossType : int { L2, L1, Mape, Smape, Huber, LogL1, RelativeL2 };
enum class ENerfActivation : int { None, ReLU, Logistic, Exponential };
enum class ELensMode : int { Perspective, OpenCV, FTheta, LatLong, OpenCVFisheye, Equirectangular };
enum class ETonemapCurve : int { Identity, ACES, Hable, Reinhard };
// ERenderMode (common.h:56-67); Distortion and EncodingVis are GUI visualisations, refused by render()
enum class ERenderMode : int { AO, Shade, Normals, Positions, Depth, Distortion, Cost, Slice };
using mat3 = std::array<float, 9>;  // row-major
constexpr mat3 MAT3_IDENTITY = {1, 0, 0, 0, 1, 0, 0, 0, 1};

using vec2 = std::array<float, 2>;
using vec3 = std::array<float, 3>;
using vec4 = std::array<float, 4>;
using ivec2 = std::array<int, 2>;

// Column-major 4x3 camera-to-world (right, down, forward, origin) in NGP space.
struct Mat43 {
	float m[12] = {1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0};
	vec3 col(int c) const { return {m[3 * c], m[3 * c + 1], m[3 * c + 2]}; }
	void set_col(int c, const vec3& v) { m[3 * c] = v[0]; m[3 * c + 1] = v[1]; m[3 * c + 2] = v[2]; }
};

struct Lens {
	ELensMode mode = ELensMode::Perspective;
	float params[7] = {};
};

struct TrainingImageMetadata {
	ivec2 resolution = {0, 0};
	vec2 focal_length = {1000.f, 1000.f};
	vec2 principal_point = {0.5f, 0.5f};
	Lens lens;
	vec4 rolling_shutter = {0.f, 0.f, 0.f, 0.f};  // pixel time A + B u + C v + D motionblur_time (nerf_loader.cu:204-216)
	vec3 light_dir = {0.f, 0.f, 0.f};  // NGP space (frames with "driver_parameters", nerf_loader.cu:666-675)
};

struct NerfDataset {
	std::vector<TrainingImageMetadata> metadata;
	std::vector<Mat43> xforms;
	std::vector<Mat43> xforms_end;  // TrainingXForm::end where it differs from start (empty / short: end = start)
	std::vector<std::string> paths;
	std::vector<std::vector<uint8_t>> pixels;  // RGBA8, sRGB, straight alpha (EImageDataType::Byte)
	// per image [h][w] depth targets = 16-bit depth x integer_depth_scale x scale (src/nerf_loader.cu:73-82,
	// 625-637, 728); empty (or missing) = no depth for that image
	std::vector<std::vector<float>> depths;
	vec3 up = {0.f, 1.f, 0.f};
	vec3 offset = {0.5f, 0.5f, 0.5f};
	float scale = 0.33f;
	int aabb_scale = 1;
	// transforms.json "render_aabb" (nerf_loader.cu:453-456; empty = min > max) and its frame
	vec3 render_aabb_min = {1.f, 1.f, 1.f}, render_aabb_max = {0.f, 0.f, 0.f};
	mat3 render_aabb_to_local = MAT3_IDENTITY;
	bool is_hdr = false;
	bool from_mitsuba = false;
	size_t n_images = 0;
	// per-image extra network inputs (nerf_loader.h:82-87): a learnable latent code of n_extra_learnable_dims
	// (transforms.json "n_extra_learnable_dims", or 16 once optimize_extra_dims is set), preceded by the frame's
	// light direction when frames carry "driver_parameters" (nerf_loader.cu:478-480, 666-675)
	uint32_t n_extra_learnable_dims = 0;
	bool has_light_dirs = false;
	uint32_t n_extra_dims() const { return (has_light_dirs ? 3u : 0u) + n_extra_learnable_dims; }
	// nerf_loader.h:95-116
	Mat43 nerf_matrix_to_ngp(const float* nerf_3x4_rowmajor, bool scale_columns = false) const;
	// compute_sharpness (src/nerf_loader.cu:111-151) of image i: [72][128] variance of the Laplacian of
	// the luma of the linear, premultiplied pixels per tile (sharpness_resolution {128, 72}, :156)
	std::vector<float> sharpness(size_t i) const;
	Mat43 ngp_matrix_to_nerf(const Mat43& m, bool scale_columns = false) const;
};

struct NerfCounters {
	uint32_t rays_per_batch = 1 << 12;
	uint32_t n_rays_total = 0;
	uint32_t measured_batch_size = 0;
	uint32_t measured_batch_size_before_compaction = 0;
};

struct NerfTraining {
	NerfDataset dataset;
	int n_images_for_training = 0;
	int n_images_for_training_prev = 0;
	bool random_bg_color = true;
	bool linear_colors = false;
	ELossType loss_type = ELossType::L2;
	bool snap_to_pixel_centers = true;
	float near_distance = 0.1f;
	float density_grid_decay = 0.95f;
	bool optimize_extrinsics = false, optimize_distortion = false, optimize_focal_length = false,
	     optimize_exposure = false, optimize_extra_dims = false;
	int view = 0;
	NerfCounters counters_rgb;
	uint64_t density_grid_rng_state = 0, density_grid_rng_inc = 0;
	// Nerf::Training::ErrorMap and its cadence (nerf.h:50-59, 112-118): the per-image error map
	// is always accumulated; sampling follows it only when asked to
	struct ErrorMap {
		ivec2 resolution = {16, 16};
		ivec2 cdf_resolution = {16, 16};
		bool is_cdf_valid = false;
		std::vector<float> pmf_img_cpu;
	} error_map;
	bool sample_focal_plane_proportional_to_error = false;
	bool sample_image_proportional_to_error = false;
	bool include_sharpness_in_error = false;  // not supported (no per-image sharpness data)
	// depth supervision (nerf.h:99,125): weight of the depth loss and its type
	float depth_supervision_lambda = 0.f;
	ELossType depth_loss_type = ELossType::L1;
	// per-image exposure optimisation (Nerf::Training::cam_exposure, nerf.h:65-79, 87-91)
	struct Adam3 {
		vec3 variable = {0.f, 0.f, 0.f}, m = {0.f, 0.f, 0.f}, v = {0.f, 0.f, 0.f};
		uint32_t iter = 0;
	};
	std::vector<Adam3> cam_exposure;
	float exposure_l2_reg = 0.0f;
	// extrinsics (Nerf::Training::cam_pos_offset / cam_rot_offset, nerf.h:65-67, 88-89): per-image
	// translation offset (AdamOptimizer<vec3>) and angle-axis rotation offset (RotationAdamOptimizer,
	// adam_optimizer.h:222-247) applied to the dataset transforms (update_transforms)
	std::vector<Adam3> cam_pos_offset, cam_rot_offset;
	float extrinsic_l2_reg = 1e-4f, extrinsic_learning_rate = 1e-3f;
	// focal length (cam_focal_length_offset, intrinsic_l2_reg 1e-4): the reference's gradient kernel
	// never writes cam_focal_length_gradient (src/testbed_nerf.cu:1163-1269), so the offset only
	// sees its L2 term -- from 0 it stays 0
	struct Adam2 {
		vec2 variable = {0.f, 0.f}, m = {0.f, 0.f}, v = {0.f, 0.f};
		uint32_t iter = 0;
	} cam_focal_length_offset;
	float intrinsic_l2_reg = 1e-4f;
	// per-image latent codes (Nerf::Training::extra_dims_opt, nerf.h:82-86): one VarAdamOptimizer per image
	// (adam_optimizer.h:25-117: lr 1e-4 until the first step takes the network's, eps 1e-8, beta 0.9 / 0.99)
	struct VarAdam {
		std::vector<float> variable, m, v;
		uint32_t iter = 0;
		float learning_rate = 1e-4f, epsilon = 1e-8f, beta1 = 0.9f, beta2 = 0.99f;
		void step(const std::vector<float>& g);
	};
	std::vector<VarAdam> extra_dims_opt;
	uint32_t n_steps_between_cam_updates = 16;
	uint32_t n_steps_since_cam_update = 0;
	uint32_t n_steps_between_error_map_updates = 128;
	uint32_t n_steps_since_error_map_update = 0;
	uint32_t n_rays_since_error_map_update = 0;
};

struct Nerf {
	NerfTraining training;
	uint32_t max_cascade = 0;
	ENerfActivation rgb_activation = ENerfActivation::Exponential;
	ENerfActivation density_activation = ENerfActivation::Exponential;
	float cone_angle_constant = 1.f / 256.f;
	float render_min_transmittance = 0.01f;
	bool render_with_lens_distortion = false;
	Lens render_lens;  // applied to rendered rays when render_with_lens_distortion (src/testbed_nerf.cu:1859)
	bool render_gbuffer_hard_edges = false;  // nerf.h:174
	float sharpen = 0.f;
	uint32_t density_grid_ema_step = 0;
	bool visualize_cameras = false;
	// composite_kernel_nerf's glow (nerf.h:176-177, src/testbed_nerf.cu:540-628)
	float glow_y_cutoff = 0.f;
	int glow_mode = 0;
	vec3 light_dir = {0.5f, 0.5f, 0.5f};  // nerf.h:155: the rendered light direction of datasets with light dirs
	// Nerf::find_closest_training_view (src/testbed_nerf.cu:3231-3244): the training view whose camera is
	// nearest to pose (distance of the origins + 0.25 x distance of the forward axes); training.view if none
	int find_closest_training_view(const Mat43& pose, const std::function<Mat43(size_t)>& transform) const;
};

class Testbed {
public:
	explicit Testbed(ETestbedMode mode = ETestbedMode::None);
	~Testbed();
	Testbed(const Testbed&) = delete;
	Testbed& operator=(const Testbed&) = delete;

	// --- data (Testbed::load_training_data src/testbed.cu:125, load_nerf src/testbed_nerf.cu:2240) ---
	void load_training_data(const std::string& path);
	void load_file(const std::string& path);
	void create_empty_nerf_dataset(size_t n_images, int aabb_scale = 1, bool is_hdr = false);
	void set_image(int frame_idx, const float* rgba, int width, int height);  // linear premultiplied float RGBA
	void set_image_rgba8(int frame_idx, const uint8_t* rgba, int width, int height);
	void set_camera_extrinsics(int frame_idx, const float* c2w_3x4_rowmajor, bool convert_to_ngp = true);
	// Nerf::Training::set_camera_extrinsics_rolling_shutter (src/testbed_nerf.cu:2012-2030)
	void set_camera_extrinsics_rolling_shutter(int frame_idx, const float* start_3x4_rowmajor, const float* end_3x4_rowmajor,
	                                           const vec4& rolling_shutter, bool convert_to_ngp = true);
	Mat43 get_camera_extrinsics(int frame_idx) const;
	// dataset transform with the extrinsic offsets applied (Nerf::Training::transforms)
	Mat43 training_transform(size_t i) const;
	Mat43 training_transform_end(size_t i) const;  // the end transform with the same offsets
	void set_camera_intrinsics(int frame_idx, float fx, float fy = 0.f, float cx = -0.5f, float cy = -0.5f, float k1 = 0.f, float k2 = 0.f,
	                           float p1 = 0.f, float p2 = 0.f, float k3 = 0.f, float k4 = 0.f, bool is_fisheye = false);
	std::function<bool(const std::string&, std::vector<uint8_t>&, int&, int&)> image_decoder;  // non-PNG fallback

	// --- network (reload_network_from_file src/testbed.cu:274, reset_network :3624) ---
	void reload_network_from_file(const std::string& path = "");
	void reload_network_from_json(const Json& json, const std::string& config_base_path = "");
	void reset_network(bool clear_density_grid = true);
	Json network_config() const { return m_network_config; }
	const ngp_network_config& network_abi_config() const { return m_net_cfg; }  // the resolved C-ABI config

	// --- training (train src/testbed.cu:4020, frame :3380) ---
	void train(uint32_t batch_size);
	bool frame();
	void reset_accumulation() { m_spp = 0; }

	// --- rendering (render_to_cpu src/python_api.cu:124) ---
	// copy_to_host=false leaves the tonemapped frame in HBM (render_frame_buffer()) and returns {}.
	std::vector<float> render(int width, int height, int spp, bool linear, uint32_t shard_index = 0,
	                          uint32_t shard_count = 1, uint32_t shard_rows = 8, bool copy_to_host = true);
	// the same into caller-owned host memory of width * height * 4 floats (null: stay in HBM); with a
	// pinned buffer (pinned_host_alloc) the read-back runs at PCIe DMA rate.  host_dst_pinned: the caller
	// guarantees host_dst is page-locked and device-mapped (pinned_host_alloc), so the render kernels may
	// stream finished pixels into it; pageable memory (a std::vector) takes the read-back after the frame
	void render_into(float* host_dst, int width, int height, int spp, bool linear, uint32_t shard_index = 0,
	                 uint32_t shard_count = 1, uint32_t shard_rows = 8, bool host_dst_pinned = false);
	const float* render_frame_buffer() const { return m_out; }
	void set_camera_to_training_view(int trainview);
	void reset_camera();
	float fov() const;
	void set_fov(float degrees);
	// fov_xy / set_fov_xy (src/testbed.cu:3538-3544): per-axis field of view in degrees
	vec2 fov_xy() const;
	void set_fov_xy(const vec2& degrees);
	// the render crop box as a 4x3 frame (axes scaled by the half extents, centre), NGP or NeRF space
	// (crop_box / set_crop_box / crop_box_corners, src/testbed.cu:618-670)
	Mat43 crop_box(bool nerf_space = true) const;
	void set_crop_box(Mat43 m, bool nerf_space = true);
	std::vector<vec3> crop_box_corners(bool nerf_space = true) const;
	// compute_image_mse (src/testbed_image.cu:455-518): the Image mode's network against its image; a NeRF
	// testbed has no image (the reference divides an empty sum by zero elements: NaN)
	float compute_image_mse(bool quantize_to_byte = false) const;
	int find_closest_training_view() const;
	// extra dims (per-image latent codes, NerfNetwork's n_extra_dims): the dataset's width, the codes of the
	// training views (Nerf::Training::get_extra_dims_cpu, src/testbed_nerf.cu:1797-1812) and the code rendered rays
	// carry -- a training view's (rendering_extra_dims_from_training_view >= 0, the default 0, nerf.h:157) or one set
	// with set_rendering_extra_dims (src/testbed_nerf.cu:3206-3280)
	uint32_t n_extra_dims() const { return nerf.training.dataset.n_extra_dims(); }
	int rendering_extra_dims_from_training_view = 0;
	void set_rendering_extra_dims_from_training_view(int trainview);
	void set_rendering_extra_dims(const std::vector<float>& vals);
	std::vector<float> rendering_extra_dims() const;
	std::vector<float> training_extra_dims(int trainview) const;

	// --- snapshots (save_snapshot src/testbed.cu:4775, load_snapshot :4841) ---
	void save_snapshot(const std::string& path, bool include_optimizer_state = false, bool compress = true);
	void load_snapshot(const std::string& path);
	std::vector<float> error_map_data();  // [n_images][res.y][res.x] accumulated since the last CDF update
	static Json read_snapshot_file(const std::string& path);  // msgpack, zlib-inflated if compressed

	// --- multi-GPU: one Testbed per rank, gradients all-reduced over RCCL/xGMI ---
	void init_distributed(int rank, int world_size, const std::string& nccl_unique_id);
	// Test backend: the same data-parallel path with every collective staged through host memory
	// and a caller-supplied all-reduce (e.g. torch.distributed over gloo), so several processes can
	// share one GPU.  fn(host_ptr, n, dtype 0 f32 / 1 f16, op 0 sum / 1 max) reduces in place.
	using HostAllReduce = std::function<void(void*, size_t, int, int)>;
	void init_distributed_host(int rank, int world_size, HostAllReduce fn);
	static std::string nccl_unique_id();
	// config C: one frame row-sharded over the ranks (8-row blocks, interleaved) and gathered into
	// rank 0's frame buffer over RCCL (the reference's aux-device copy-back, src/testbed.cu:5089-5090).
	// Every rank calls it; rank 0 returns the frame (copy_to_host) and holds it in render_frame_buffer().
	std::vector<float> render_distributed(int width, int height, int spp, bool linear, bool copy_to_host = true);
	int rank() const { return m_rank; }
	// a collective backend is set (RCCL or the host-staged one), world size 1 included
	bool distributed() const { return m_comm != nullptr || (bool)m_host_allreduce; }
	// deterministic hash-grid gradients (ngp_train_args.deterministic): bit-reproducible steps
	bool deterministic = false;
	// m_max_level_rand_training (testbed.h:704; src/testbed_nerf.cu:724, 949, 2797-2805): per-ray random
	// hash-grid max level during training
	bool m_max_level_rand_training = false;
	int world_size() const { return m_world; }

	ngp_model* model() const { return m_model; }
	// launch shapes / march schedule of the kernels (ngp_tuning; kept across network reloads)
	const ngp_tuning& tuning() const { return m_tuning; }
	void set_tuning(const ngp_tuning& t);
	void* stream() const { return m_stream; }
	void sync() const;
	// the learned distortion map's parameters, [res_y][res_x][2] (m_distortion.map->params())
	std::vector<float> distortion_map() const { return m_distortion.params; }
	ivec2 distortion_resolution() const { return {m_distortion.rx, m_distortion.ry}; }
	ngp_train_stats last_stats() const { return m_last_stats; }
	std::vector<float> density_grid() const;
	std::vector<uint8_t> density_grid_bitfield() const;
	// get_density_on_grid (src/testbed_nerf.cu:3026-3075): the raw density output on a res3d lattice over the box
	// (x fastest), -10000 where the density grid is below NERF_MIN_OPTICAL_THICKNESS
	std::vector<float> density_on_grid(const std::array<int, 3>& res3d, const vec3& box_min, const vec3& box_max,
	                                   const mat3& box_to_local) const;
	// compute_and_save_png_slices (src/testbed.cu:534-559): an empty box (min > max) means the render aabb with its
	// rotation; thresh = FLT_MAX means mesh_thresh.  Writes filename + ".density_slices_{x}x{y}x{z}.png" and
	// returns the lattice resolution.
	std::array<int, 3> compute_and_save_png_slices(const std::string& filename, int res, vec3 box_min, vec3 box_max,
	                                               float thresh, float density_range, bool flip_y_and_z_axes);
	float mesh_thresh = 2.5f;  // m_mesh.thresh (testbed.h:660)

	// --- state (public like the reference's pybind-exposed members) ---
	ETestbedMode mode = ETestbedMode::None;
	Nerf nerf;
	bool shall_train = false;
	bool train_encoding = true, train_network = true;
	uint32_t training_batch_size = 1 << 18;
	// evaluate every emitted sample before the loss (the reference's forward) instead of the
	// early-terminated chunked forward; switched on automatically if the chunked forward ever
	// misses a sample the loss needs (ngp_train_stats::forward_early_stop_violations)
	bool train_full_forward = false;
	ngp_tuning m_tuning{};
	uint64_t forward_early_stop_violations = 0;
	uint32_t training_step = 0;
	float loss = 0.0f;  // Ema m_loss_scalar (val) of src/testbed.cu:4106-4108
	vec4 background_color = {0.f, 0.f, 0.f, 1.f};
	bool snap_to_pixel_centers = false;
	bool render_ground_truth = false;
	Mat43 camera;
	vec2 relative_focal_length = {1.f, 1.f};
	uint32_t fov_axis = 1;
	float zoom = 1.f;
	vec2 screen_center = {0.5f, 0.5f};
	float scale = 1.5f;
	float exposure = 0.f;
	EColorSpace color_space = EColorSpace::Linear;
	ETonemapCurve tonemap_curve = ETonemapCurve::Identity;
	float render_near_distance = 0.f;
	uint64_t seed = 1337;
	std::string root_dir;
	std::string data_path;
	std::string network_config_path = "base.json";
	bool training_data_available = false;
	vec3 aabb_min = {0.f, 0.f, 0.f}, aabb_max = {1.f, 1.f, 1.f};
	// m_raw_aabb (testbed.h:926): the dataset's aabb as loaded (src/testbed_nerf.cu:2221)
	vec3 raw_aabb_min = {-10.f, -10.f, -10.f}, raw_aabb_max = {10.f, 10.f, 10.f};
	// m_up_dir (testbed.h:732): the dataset's up direction (src/testbed_nerf.cu:2237); kept in snapshots
	vec3 up_dir = {0.f, 1.f, 0.f};
	// the render crop box (m_render_aabb, m_render_aabb_to_local; src/testbed_nerf.cu:2219-2225) and modes
	vec3 render_aabb_min = {0.f, 0.f, 0.f}, render_aabb_max = {1.f, 1.f, 1.f};
	mat3 render_aabb_to_local = MAT3_IDENTITY;
	ERenderMode render_mode = ERenderMode::Shade;
	float aperture_size = 0.f;  // m_aperture_size (depth of field)
	float slice_plane_z = 0.f;  // m_slice_plane_z: focus / slice plane at camera depth slice_plane_z + scale
	double training_ms = 0.0, training_prep_ms = 0.0, render_ms = 0.0;

private:
	void load_nerf_post();
	void upload_dataset();
	void upload_metadata();
	void update_density_grid(uint32_t n_uniform, uint32_t n_nonuniform);
	void train_nerf(uint32_t batch_size, bool get_loss_scalar);
	std::string find_network_config(const std::string& path) const;
	Json load_network_config(const std::string& path) const;
	void build_model(const Json& config);
	void free_device_dataset();
	void ensure_render_buffers(size_t n_pixels);
	void allreduce_f32(float* dev, size_t n, bool max_op);
	void allreduce_dev(void* dev, size_t n, int dtype, bool max_op);  // RCCL or the host-staged backend
	static ngp_status dp_allreduce_i32(void* user, int32_t* dev, uint32_t n, ngp_stream stream);
	HostAllReduce m_host_allreduce;

	void update_error_map_cdf();

	ngp_model* m_model = nullptr;
	void* m_stream = nullptr;
	// error map (device): data [n_images][res.y][res.x], CDFs at cdf_resolution
	float* m_exp = nullptr;       // [n_images][3] log2 exposure (device)
	float* m_exp_grad = nullptr;  // [n_images][3]
	size_t m_exp_cap = 0;
	ngp_network_config m_net_cfg{};
	void update_cam_exposure();
	void update_cam_extrinsics();
	void update_cam_focal_length();
	float* m_cam_grad = nullptr;  // [2][n_images][3]: translation, rotation gradients (device)
	// learned image-plane distortion (Testbed::m_distortion: TrainableBuffer<2, 2, float> with its own
	// ExponentialDecay(Adam) trainer, src/testbed.cu:3781-3792, configs/nerf/base.json:57-73)
	struct DistortionMap {
		int rx = 32, ry = 32;
		float lr = 1e-4f, beta1 = 0.9f, beta2 = 0.99f, eps = 1e-8f, decay_base = 0.33f;
		uint32_t decay_start = 10000, decay_interval = 5000, decay_end = 25000;
		std::vector<float> params, m, v;  // params start at zero (TrainableBuffer::initialize_params)
		std::vector<uint32_t> steps;      // Adam's per-parameter step counts
		uint32_t optimizer_step = 0;
		bool active = false;  // applied to training rays once optimize_distortion was set (a zero map is the identity)
	} m_distortion;
	// latent codes on the device: [n_images + 1][16] (the last row: the rendered code), their gradient
	// [n_images][16]; rendering_extra_dims set by the caller (host, n_extra_dims values)
	float* m_extra = nullptr;
	float* m_extra_grad = nullptr;
	size_t m_extra_rows = 0;
	std::vector<float> m_rendering_extra_dims;
	std::vector<float> m_extra_host;  // staging of the device table (uploaded synchronously)
	float* m_extra_stage = nullptr;   // pinned 16-float staging of the rendered row (copied asynchronously)
	void reset_extra_dims(pcg32* rng);  // Nerf::reset_extra_dims (src/testbed_nerf.cu:3181-3204; rng: n_extra_dims > 0)
	void upload_extra_dims();           // Nerf::Training::update_extra_dims (src/testbed_nerf.cu:1814-1825)
	const float* rendering_extra_dims_device();  // Nerf::get_rendering_extra_dims (src/testbed_nerf.cu:3206-3228)
	void update_extra_dims_step();      // the per-step latent-code Adam (src/testbed_nerf.cu:2580-2599)
	float* m_dist = nullptr;       // device params [ry][rx][2]
	float* m_dist_grad = nullptr;  // device [2][ry][rx][2]: gradient, gradient weight
	void update_distortion_map();
	size_t m_cam_grad_cap = 0;
	float current_learning_rate() const;
	float* m_err = nullptr;
	float* m_cdf_x = nullptr;
	float* m_cdf_y = nullptr;
	float* m_cdf_img = nullptr;
	size_t m_err_cap = 0, m_cdf_cap = 0, m_cdf_img_cap = 0;
	Json m_network_config;
	uint64_t m_rng_state = 0, m_rng_inc = 0;
	// device dataset
	std::vector<void*> m_dev_pixels;
	std::vector<void*> m_dev_depths;  // per image f32 depth targets (null: none)
	void* m_dev_meta = nullptr;
	float* m_dev_sharpness = nullptr;  // [n_images][72][128] (include_sharpness_in_error)
	float* m_sharp_grid = nullptr;     // [8][128^3] running max (Nerf::Training::sharpness_grid)
	bool m_dataset_dirty = true;
	// render buffers
	float* m_frame = nullptr;
	float* m_depth = nullptr;
	float* m_accum = nullptr;
	float* m_out = nullptr;
	size_t m_render_cap = 0;
	uint32_t m_spp = 0;
	ngp_train_stats m_last_stats{};
	// distributed
	int m_rank = 0, m_world = 1;
	void* m_comm = nullptr;
	void* m_red_buf = nullptr;
	float* m_pack = nullptr;  // owned rows of a sharded frame, packed for the gather
	size_t m_pack_cap = 0;
};

std::string natural_sort_key(const std::string& s);
// get_marching_cubes_res (src/marching_cubes.cu:40-47): res_1d along the box's longest side, each axis rounded up to 16
std::array<int, 3> marching_cubes_res(int res_1d, const vec3& box_min, const vec3& box_max);
// save_density_grid_to_png's mosaic (src/marching_cubes.cu:957-1020): the res.z slices (res.y with swap_y_z) of a
// [z][y][x] grid tiled sqrt(res.z) rows down, y flipped, byte = clamp((v - thresh) * 128 / density_range + 128.5);
// returns the 8-bit gray image and its size; zero_x_voxels / near_zero_lattice get the log line's two counts
std::vector<uint8_t> density_slices_mosaic(const std::vector<float>& density, std::array<int, 3> res3d, float thresh,
                                           bool swap_y_z, float density_range, int* width, int* height,
                                           uint32_t* zero_x_voxels = nullptr, uint32_t* near_zero_lattice = nullptr);
// non-PNG images (JPG, ...): decoder(path, rgba8_out, width, height) -> success
using ImageDecoder = std::function<bool(const std::string&, std::vector<uint8_t>&, int&, int&)>;
NerfDataset load_nerf(const std::string& path, const ImageDecoder& image_decoder = nullptr);

}  // namespace ngp
