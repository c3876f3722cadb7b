// testbed.cpp — host Testbed for the MI355X NeRF path.  Every device operation is a
// call into libngp_hip.so (include/ngp_hip.h); this file holds only the host-side
// orchestration the reference keeps in src/testbed.cu / src/testbed_nerf.cu.
#include <array>
#include "testbed.h"

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>
#include <zlib.h>

#include <algorithm>
#include <cctype>
#include <iterator>
#include <limits>
#include <map>
#include <mutex>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cerrno>
#include <cstring>
#include <unistd.h>
#include <dirent.h>
#include <fstream>
#include <sstream>
#include <stdexcept>
#include <sys/stat.h>

#include "ngp_math.h"
#include "png.h"

namespace ngp {

namespace {

constexpr float PI_F = 3.14159265358979323846f;
constexpr float LOSS_SCALE = 128.0f;  // testbed.h:390

void ck(ngp_status s) {
	if (s != NGP_OK) throw std::runtime_error(ngp_last_error());
}
void hk(hipError_t e, const char* what) {
	if (e != hipSuccess) throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(e) + " in " + what);
}
void nk(ncclResult_t r, const char* what) {
	if (r != ncclSuccess) throw std::runtime_error(std::string("RCCL error ") + ncclGetErrorString(r) + " in " + what);
}

bool file_exists(const std::string& p) {
	struct stat st;
	return stat(p.c_str(), &st) == 0;
}
bool is_directory(const std::string& p) {
	struct stat st;
	return stat(p.c_str(), &st) == 0 && S_ISDIR(st.st_mode);
}
std::string parent_path(const std::string& p) {
	const size_t k = p.find_last_of('/');
	return k == std::string::npos ? std::string(".") : p.substr(0, k);
}
std::string extension(const std::string& p) {
	const size_t s = p.find_last_of('/');
	const size_t k = p.find_last_of('.');
	if (k == std::string::npos || (s != std::string::npos && k < s)) return "";
	std::string e = p.substr(k + 1);
	std::transform(e.begin(), e.end(), e.begin(), ::tolower);
	return e;
}
std::string basename_of(const std::string& p) {
	const size_t k = p.find_last_of('/');
	return k == std::string::npos ? p : p.substr(k + 1);
}
std::string read_text(const std::string& path) {
	std::ifstream f(path);
	if (!f) throw std::runtime_error("Could not open '" + path + "'.");
	std::stringstream ss;
	ss << f.rdbuf();
	return ss.str();
}
float fov_to_focal_length(int resolution, float degrees) { return 0.5f * (float)resolution / std::tan(0.5f * degrees * PI_F / 180.0f); }
float focal_length_to_fov(float resolution, float focal) { return 2.0f * 180.0f / PI_F * std::atan(resolution / (focal * 2.0f)); }

uint32_t next_multiple_host(uint32_t a, uint32_t b) { return (a + b - 1) / b * b; }

// IEEE binary16 <-> binary32 (round to nearest even), for the snapshot's fp16 arrays
uint16_t f32_to_f16(float f) {
	uint32_t x;
	std::memcpy(&x, &f, 4);
	const uint32_t sign = (x >> 16) & 0x8000u;
	const int32_t e = (int32_t)((x >> 23) & 0xff) - 127 + 15;
	uint32_t mant = x & 0x7fffffu;
	if (((x >> 23) & 0xff) == 0xff) return (uint16_t)(sign | 0x7c00u | (mant ? 0x200u : 0u));
	if (e >= 31) return (uint16_t)(sign | 0x7c00u);
	if (e <= 0) {
		if (e < -10) return (uint16_t)sign;
		mant |= 0x800000u;
		const uint32_t shift = (uint32_t)(14 - e);
		uint32_t h = mant >> shift;
		const uint32_t rem = mant & ((1u << shift) - 1u), half = 1u << (shift - 1);
		if (rem > half || (rem == half && (h & 1u))) ++h;
		return (uint16_t)(sign | h);
	}
	uint32_t h = ((uint32_t)e << 10) | (mant >> 13);
	const uint32_t rem = mant & 0x1fffu;
	if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) ++h;
	return (uint16_t)(sign | h);
}
float f16_to_f32(uint16_t h) {
	const uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
	uint32_t e = (h >> 10) & 0x1fu, m = h & 0x3ffu, x;
	if (e == 0) {
		if (m == 0) x = sign;
		else {
			e = 127 - 15 + 1;
			while (!(m & 0x400u)) { m <<= 1; --e; }
			x = sign | (e << 23) | ((m & 0x3ffu) << 13);
		}
	} else if (e == 31) x = sign | 0x7f800000u | (m << 13);
	else x = sign | ((e + 127 - 15) << 23) | (m << 13);
	float f;
	std::memcpy(&f, &x, 4);
	return f;
}

float srgb_to_linear_h(float s) { return s <= 0.04045f ? s / 12.92f : std::pow((s + 0.055f) / 1.055f, 2.4f); }
float linear_to_srgb_h(float l) { return l < 0.0031308f ? 12.92f * l : 1.055f * std::pow(l, 0.41666f) - 0.055f; }

}  // namespace

// SI::natural-style comparison key: digit runs compare numerically.
std::string natural_sort_key(const std::string& s) {
	std::string out;
	for (size_t i = 0; i < s.size();) {
		if (std::isdigit((unsigned char)s[i])) {
			size_t j = i;
			while (j < s.size() && std::isdigit((unsigned char)s[j])) ++j;
			std::string digits = s.substr(i, j - i);
			digits.erase(0, std::min(digits.find_first_not_of('0'), digits.size() - 1));
			out += (char)('0' + std::min<size_t>(digits.size(), 9));
			out += digits;
			i = j;
		} else out += s[i++];
	}
	return out;
}

// nerf_loader.h:95-116 (non-Mitsuba): flip y/z columns, scale + offset, cycle axes xyz <- yzx.
Mat43 NerfDataset::nerf_matrix_to_ngp(const float* r, bool scale_columns) const {
	float c[4][3];
	for (int col = 0; col < 4; ++col)
		for (int row = 0; row < 3; ++row) c[col][row] = r[row * 4 + col];
	for (int row = 0; row < 3; ++row) {
		c[0][row] *= scale_columns ? scale : 1.f;
		c[1][row] *= scale_columns ? -scale : -1.f;
		c[2][row] *= scale_columns ? -scale : -1.f;
		c[3][row] = c[3][row] * scale + offset[row];
	}
	Mat43 m;
	for (int col = 0; col < 4; ++col) {
		m.m[3 * col + 0] = c[col][1];
		m.m[3 * col + 1] = c[col][2];
		m.m[3 * col + 2] = c[col][0];
	}
	return m;
}

Mat43 NerfDataset::ngp_matrix_to_nerf(const Mat43& in, bool scale_columns) const {
	Mat43 m;
	for (int col = 0; col < 4; ++col) {
		m.m[3 * col + 0] = in.m[3 * col + 2];
		m.m[3 * col + 1] = in.m[3 * col + 0];
		m.m[3 * col + 2] = in.m[3 * col + 1];
	}
	for (int row = 0; row < 3; ++row) {
		m.m[0 * 3 + row] *= scale_columns ? 1.f / scale : 1.f;
		m.m[1 * 3 + row] *= scale_columns ? -1.f / scale : -1.f;
		m.m[2 * 3 + row] *= scale_columns ? -1.f / scale : -1.f;
		m.m[3 * 3 + row] = (m.m[3 * 3 + row] - offset[row]) / scale;
	}
	return m;
}

Testbed::Testbed(ETestbedMode m) {
	int device = 0;
	if (const char* lr = std::getenv("LOCAL_RANK")) device = std::atoi(lr);
	int n_dev = 0;
	const hipError_t de = hipGetDeviceCount(&n_dev);
	if (de != hipSuccess || n_dev <= 0) {
		// name what the HIP runtime saw: the device-visibility variables and whether the process may open
		// the kernel driver's device nodes (a runtime that finds no GPU agent reports "no ROCm-capable device")
		auto env = [](const char* k) { const char* v = std::getenv(k); return std::string(k) + "=" + (v ? v : "(unset)"); };
		std::string msg = std::string("Testbed requires an AMD GPU: hipGetDeviceCount: ") + hipGetErrorString(de) + " (" +
		                  env("HIP_VISIBLE_DEVICES") + ", " + env("ROCR_VISIBLE_DEVICES") + ", " + env("CUDA_VISIBLE_DEVICES") +
		                  ", /dev/kfd " + (access("/dev/kfd", R_OK | W_OK) == 0 ? "accessible" : std::strerror(errno)) + ")";
		throw std::runtime_error(msg);
	}
	device = device % n_dev;
	hk(hipSetDevice(device), "hipSetDevice");
	hipStream_t s;
	hk(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
	m_stream = s;
	// Testbed constructor default network config (src/testbed.cu:3954-3980)
	m_network_config = Json::parse(R"({
		"loss": {"otype": "L2"},
		"optimizer": {"otype": "Adam", "learning_rate": 1e-3, "beta1": 0.9, "beta2": 0.99, "epsilon": 1e-15, "l2_reg": 1e-6},
		"encoding": {"otype": "HashGrid", "n_levels": 16, "n_features_per_level": 2, "log2_hashmap_size": 19, "base_resolution": 16},
		"network": {"otype": "FullyFusedMLP", "n_neurons": 64, "n_layers": 2, "activation": "ReLU", "output_activation": "None"}
	})");
	mode = m;
	reset_camera();
}

Testbed::~Testbed() {
	try {
		sync();
	} catch (...) {
	}
	if (m_model) ngp_model_destroy(m_model);
	free_device_dataset();
	for (float* p : {m_frame, m_depth, m_accum, m_out})
		if (p) (void)hipFree(p);
	if (m_red_buf) (void)hipFree(m_red_buf);
	if (m_pack) (void)hipFree(m_pack);
	for (float* p : {m_err, m_cdf_x, m_cdf_y, m_cdf_img, m_exp, m_exp_grad, m_cam_grad, m_sharp_grid, m_dist, m_dist_grad, m_extra, m_extra_grad})
		if (p) (void)hipFree(p);
	if (m_comm) ncclCommDestroy((ncclComm_t)m_comm);
	if (m_extra_stage) pinned_host_release(m_extra_stage, NGP_EXTRA_ROW * sizeof(float));
	if (m_stream) (void)hipStreamDestroy((hipStream_t)m_stream);
}

// an idle stream (train() after the step's counter read-back has waited for it) returns at once: hipStreamSynchronize
// alone costs ~9 us per call there even with nothing in flight
void Testbed::sync() const {
	const hipError_t e = hipStreamQuery((hipStream_t)m_stream);
	if (e == hipSuccess) return;
	if (e != hipErrorNotReady) hk(e, "hipStreamQuery");
	hk(hipStreamSynchronize((hipStream_t)m_stream), "hipStreamSynchronize");
}

// ---------------------------------------------------------------------------
// Data
// ---------------------------------------------------------------------------
void Testbed::load_file(const std::string& path) {
	const std::string ext = extension(path);
	if (ext == "ingp" || ext == "msgpack") {
		load_snapshot(path);
		return;
	}
	if (ext == "json" && path.find("transforms") == std::string::npos && file_exists(path)) {
		const Json j = Json::parse(read_text(path));
		if (!j.contains("frames")) {
			reload_network_from_file(path);
			return;
		}
	}
	load_training_data(path);
}

// ngp::load_nerf (src/nerf_loader.cu:273-743) on the host: every transforms json of `path` (a
// file, or all *.json of a directory), frames naturally sorted, sharpness-filtered, decoded to
// RGBA8 and converted to NGP space.  No device work (the Testbed uploads on first use).
NerfDataset load_nerf(const std::string& path, const ImageDecoder& image_decoder) {
	if (!file_exists(path)) throw std::runtime_error("Data path '" + path + "' does not exist.");
	std::vector<std::string> json_paths;
	if (is_directory(path)) {
		DIR* d = opendir(path.c_str());
		if (d) {
			while (dirent* e = readdir(d)) {
				const std::string f = path + "/" + e->d_name;
				if (!is_directory(f) && extension(f) == "json") json_paths.push_back(f);
			}
			closedir(d);
		}
		std::sort(json_paths.begin(), json_paths.end());
	} else {
		json_paths.push_back(path);
	}
	if (json_paths.empty()) throw std::runtime_error("Cannot load NeRF data from an empty set of paths.");

	// ngp::load_nerf (src/nerf_loader.cu:273-743)
	NerfDataset ds;
	ds.scale = 0.33f;
	// depth images as loaded (16-bit) and their integer_depth_scale; scaled by the final dataset scale below
	std::vector<std::vector<uint16_t>> depth_raw;
	std::vector<float> depth_scales;
	ds.offset = {0.5f, 0.5f, 0.5f};
	static const char* formats[] = {"png", "jpg", "jpeg", "bmp", "gif", "tga", "pic", "pnm", "psd", "exr"};
	// declared outside the per-json loop as in the reference (src/nerf_loader.cu:300, 419, 486-488): a
	// value set by one json carries over to the jsons loaded after it
	float depth_scale = -1.0f;
	bool enable_depth_loading = true;
	for (const std::string& jp : json_paths) {
		const Json j = Json::parse(read_text(jp));
		if (!j.contains("frames") || !j["frames"].is_array()) continue;
		const std::string base = parent_path(jp);
		if (j.contains("scale")) ds.scale = (float)j["scale"].num();
		if (j.contains("aabb_scale")) ds.aabb_scale = (int)j["aabb_scale"].num();
		if (j.contains("n_extra_learnable_dims")) ds.n_extra_learnable_dims = (uint32_t)j["n_extra_learnable_dims"].num();  // :478-480
		if (j.contains("offset")) {
			if (j["offset"].is_array()) ds.offset = {(float)j["offset"][0].num(), (float)j["offset"][1].num(), (float)j["offset"][2].num()};
			else ds.offset = {(float)j["offset"].num(), (float)j["offset"].num(), (float)j["offset"].num()};
		}
		if (j.contains("aabb")) {
			const Json& a = j["aabb"];
			float len = 1e-6f;
			for (int k = 0; k < 3; ++k) len = std::max(len, std::fabs((float)a[1][k].num() - (float)a[0][k].num()));
			ds.scale = 1.f / len;
			for (int k = 0; k < 3; ++k) ds.offset[k] = (((float)a[1][k].num() + (float)a[0][k].num()) * 0.5f) * -ds.scale + 0.5f;
		}
		if (j.contains("render_aabb")) {  // src/nerf_loader.cu:453-456
			const Json& ra = j["render_aabb"];
			for (int k = 0; k < 3; ++k) {
				ds.render_aabb_min[k] = (float)ra[0][k].num();
				ds.render_aabb_max[k] = (float)ra[1][k].num();
			}
		}
		// depth supervision inputs (src/nerf_loader.cu:419-437, 486-488)
		if (j.contains("integer_depth_scale")) depth_scale = (float)j["integer_depth_scale"].num();
		if (j.contains("enable_depth_loading")) enable_depth_loading = j.value("enable_depth_loading", true);
		if (j.contains("up")) ds.up = {(float)j["up"][1].num(), (float)j["up"][2].num(), (float)j["up"][0].num()};
		// frames sorted naturally by file_path (src/nerf_loader.cu:347-349)
		std::vector<Json> frames = j["frames"].elements();
		std::stable_sort(frames.begin(), frames.end(), [](const Json& a, const Json& b) {
			return natural_sort_key(a.value("file_path", std::string())) < natural_sort_key(b.value("file_path", std::string()));
		});
		if (j.contains("n_frames")) frames.resize(std::min(frames.size(), (size_t)j["n_frames"].num()));
		for (Json& fr : frames)
			if (fr.contains("file_path")) {
				std::string fp = fr["file_path"].str();
				std::replace(fp.begin(), fp.end(), '\\', '/');
				fr["file_path"] = Json(fp);
			}
		// frames with a sharpness record (src/nerf_loader.cu:364-387): keep a frame if its image file
		// exists and it is sharper than sharpness_discard_threshold x the mean of its neighbours
		// [i-3, i+3) (the reference's window, including its 0/0 for a single frame)
		if (!frames.empty() && frames[0].contains("sharpness")) {
			const float thr = (float)j.value("sharpness_discard_threshold", 0.0);
			const int n = (int)frames.size();
			std::vector<Json> kept;
			for (int i = 0; i < n; ++i) {
				float mean = 0.0f;
				const int a = std::max(0, i - 3), b = std::min(i + 3, n - 1);
				for (int k = a; k < b; ++k) mean += (float)frames[k].value("sharpness", 1.0);
				mean /= (float)(b - a);
				const std::string fp = frames[i].value("file_path", std::string());
				const std::string p = (!fp.empty() && fp[0] == '/') ? fp : base + "/" + fp;
				if (file_exists(p) && (float)frames[i].value("sharpness", 1.0) > thr * mean) kept.push_back(frames[i]);
			}
			frames.swap(kept);
		}
		// read_lens / principal point (src/nerf_loader.cu:175-220)
		auto read_lens = [](const Json& src, Lens& lens, vec2& pp) {
			const ELensMode opencv = src.value("is_fisheye", false) ? ELensMode::OpenCVFisheye : ELensMode::OpenCV;
			ELensMode mode_l = ELensMode::Perspective;
			auto par = [&](const char* n, int idx) {
				if (src.contains(n)) {
					lens.params[idx] = (float)src[n].num();
					if (lens.params[idx] != 0.f) mode_l = opencv;
				}
			};
			par("k1", 0); par("k2", 1); par("k3", 2); par("k4", 3); par("p1", 2); par("p2", 3);
			if (src.contains("cx")) pp[0] = (float)src["cx"].num() / (float)src["w"].num();
			if (src.contains("cy")) pp[1] = (float)src["cy"].num() / (float)src["h"].num();
			if (src.contains("ftheta_p0")) {
				const char* names[5] = {"ftheta_p0", "ftheta_p1", "ftheta_p2", "ftheta_p3", "ftheta_p4"};
				for (int q = 0; q < 5; ++q) lens.params[q] = (float)src[names[q]].num();
				lens.params[5] = (float)src["w"].num();
				lens.params[6] = (float)src["h"].num();
				mode_l = ELensMode::FTheta;
			}
			if (src.contains("latlong")) mode_l = ELensMode::LatLong;
			if (src.contains("equirectangular")) mode_l = ELensMode::Equirectangular;
			if (mode_l != ELensMode::Perspective) lens.mode = mode_l;
		};
		auto read_focal = [](const Json& src, vec2& fl, int rx, int ry) {
			auto one = [&](int res, const std::string& axis) -> float {
				if (src.contains(axis + "_fov")) return fov_to_focal_length(res, (float)src[axis + "_fov"].num());
				if (src.contains("fl_" + axis)) return (float)src["fl_" + axis].num();
				if (src.contains("camera_angle_" + axis)) return fov_to_focal_length(res, (float)src["camera_angle_" + axis].num() * 180.f / PI_F);
				return 0.f;
			};
			const float x = one(rx, "x"), y = one(ry, "y");
			if (x != 0) { fl = {x, y != 0 ? y : x}; return true; }
			if (y != 0) { fl = {y, y}; return true; }
			return false;
		};
		// rolling_shutter [A, B, C(, D)] (src/nerf_loader.cu:204-216), global and per frame
		auto read_rolling_shutter = [](const Json& src, vec4& rs) {
			if (!src.contains("rolling_shutter")) return;
			const Json& r = src["rolling_shutter"];
			rs = {(float)r[0].num(), (float)r[1].num(), (float)r[2].num(), r.size() >= 4 ? (float)r[3].num() : 0.f};
		};
		Lens lens;
		vec2 pp = {0.5f, 0.5f};
		vec4 rolling_shutter = {0.f, 0.f, 0.f, 0.f};
		read_lens(j, lens, pp);
		read_rolling_shutter(j, rolling_shutter);
		for (const Json& fr : frames) {
			std::string fp = fr.value("file_path", std::string());
			std::replace(fp.begin(), fp.end(), '\\', '/');
			std::string p = (!fp.empty() && fp[0] == '/') ? fp : base + "/" + fp;
			if (extension(p).empty() && !file_exists(p)) {
				for (const char* f : formats)
					if (file_exists(p + "." + f)) { p = p + "." + f; break; }
			}
			if (!file_exists(p)) throw std::runtime_error("Could not find image file '" + p + "'.");
			std::vector<uint8_t> rgba;
			int w = 0, h = 0;
			std::string err;
			if (!decode_png_file(p, rgba, w, h, err)) {
				if (!image_decoder || !image_decoder(p, rgba, w, h))
					throw std::runtime_error("Could not open image file: " + p + " (" + err + ")");
			}
			TrainingImageMetadata md;
			md.resolution = {w, h};
			md.principal_point = pp;
			md.lens = lens;
			bool got = read_focal(j, md.focal_length, w, h);
			got |= read_focal(fr, md.focal_length, w, h);
			if (!got) throw std::runtime_error("Couldn't read fov.");
			read_lens(fr, md.lens, md.principal_point);
			md.rolling_shutter = rolling_shutter;
			read_rolling_shutter(fr, md.rolling_shutter);  // per-frame override
			const Json& tm = fr.contains("transform_matrix_start") ? fr["transform_matrix_start"] : fr["transform_matrix"];
			const Json& tme = fr.contains("transform_matrix_end") ? fr["transform_matrix_end"] : tm;
			float r[12], re[12];
			for (int row = 0; row < 3; ++row)
				for (int col = 0; col < 4; ++col) {
					r[row * 4 + col] = (float)tm[row][col].num();
					re[row * 4 + col] = (float)tme[row][col].num();
				}
			ds.xforms.push_back(ds.nerf_matrix_to_ngp(r));
			ds.xforms_end.push_back(ds.nerf_matrix_to_ngp(re));  // = start without transform_matrix_end
			// the frame's light direction (nerf_loader.cu:666-675, nerf_direction_to_ngp nerf_loader.h:91-99): an extra
			// network input; such datasets carry no learnable code
			if (fr.contains("driver_parameters")) {
				const Json& dp = fr["driver_parameters"];
				const vec3 l = {(float)dp.value("LightX", 0.0), (float)dp.value("LightY", 0.0), (float)dp.value("LightZ", 0.0)};
				const float n = std::sqrt(l[0] * l[0] + l[1] * l[1] + l[2] * l[2]);
				const vec3 ln = n > 0.f ? vec3{l[0] / n, l[1] / n, l[2] / n} : l;
				md.light_dir = ds.from_mitsuba ? vec3{-ln[0], -ln[1], -ln[2]} : vec3{ln[1], ln[2], ln[0]};
				ds.has_light_dirs = true;
				ds.n_extra_learnable_dims = 0;
			}
			ds.metadata.push_back(md);
			ds.paths.push_back(fp);
			ds.pixels.push_back(std::move(rgba));
			// the frame's depth image (src/nerf_loader.cu:625-637): 16-bit, same resolution as the image
			std::vector<uint16_t> dep;
			if (enable_depth_loading && depth_scale > 0.f && fr.contains("depth_path")) {
				std::string dpth = fr["depth_path"].str();
				std::replace(dpth.begin(), dpth.end(), '\\', '/');
				const std::string dp = (!dpth.empty() && dpth[0] == '/') ? dpth : base + "/" + dpth;
				if (file_exists(dp)) {
					int dw = 0, dh = 0;
					std::string derr;
					if (!decode_png16_file(dp, dep, dw, dh, derr)) throw std::runtime_error("Could not load depth image '" + dp + "'.");
					if (dw != w || dh != h) throw std::runtime_error("Depth image " + dp + " has wrong resolution.");
				}
			}
			depth_raw.push_back(std::move(dep));
			depth_scales.push_back(depth_scale);
		}
	}
	// depth targets in NGP units: depth x integer_depth_scale x the final dataset scale (src/nerf_loader.cu:728)
	ds.depths.resize(depth_raw.size());
	for (size_t i = 0; i < depth_raw.size(); ++i) {
		if (depth_raw[i].empty()) continue;
		ds.depths[i].resize(depth_raw[i].size());
		const float sc = depth_scales[i] * ds.scale;
		for (size_t k = 0; k < depth_raw[i].size(); ++k) ds.depths[i][k] = (float)depth_raw[i][k] * sc;
	}
	ds.n_images = ds.metadata.size();
	if (ds.n_images == 0) throw std::invalid_argument("No training images were found for NeRF training!");
	return ds;
}

void Testbed::load_training_data(const std::string& path) {
	if (!file_exists(path)) throw std::runtime_error("Data path '" + path + "' does not exist.");
	// mode_from_scene (src/common_host.cu:146-164)
	ETestbedMode scene_mode = ETestbedMode::None;
	const std::string ext = extension(path);
	if (is_directory(path) || ext == "json") scene_mode = ETestbedMode::Nerf;
	if (path.find("geometry") != std::string::npos) scene_mode = ETestbedMode::Geometry;
	if (ext == "obj" || ext == "stl") scene_mode = ETestbedMode::Sdf;
	if (ext == "nvdb") scene_mode = ETestbedMode::Volume;
	if (ext == "exr" || ext == "bin" || ext == "png" || ext == "jpg") scene_mode = ETestbedMode::Image;
	if (scene_mode == ETestbedMode::None) throw std::runtime_error("Unknown scene format for path '" + path + "'.");
	if (scene_mode != ETestbedMode::Nerf)
		throw std::runtime_error("This build implements the NeRF primitive only (SDF/Image/Volume/Geometry are out of scope).");
	if (mode != ETestbedMode::Nerf) {
		// Testbed::set_mode (src/testbed.cu:165-218): drop mode-specific state and the network
		if (m_model) {
			sync();
			ngp_model_destroy(m_model);
			m_model = nullptr;
		}
		nerf = Nerf{};
		free_device_dataset();
		training_data_available = false;
		mode = ETestbedMode::Nerf;
		reset_camera();
	}
	data_path = path;

	const int prev_aabb_scale = nerf.training.dataset.aabb_scale;
	NerfDataset ds = load_nerf(path, image_decoder);
	nerf.training.dataset = std::move(ds);
	if (nerf.training.dataset.aabb_scale != prev_aabb_scale && m_model) reset_network();
	load_nerf_post();
	training_data_available = true;
}

void Testbed::create_empty_nerf_dataset(size_t n_images, int aabb_scale, bool is_hdr) {
	data_path.clear();
	mode = ETestbedMode::Nerf;
	NerfDataset ds;
	ds.n_images = n_images;
	ds.aabb_scale = aabb_scale;
	ds.is_hdr = is_hdr;
	ds.scale = 1.0f;
	ds.offset = {0.f, 0.f, 0.f};
	ds.metadata.resize(n_images);
	ds.xforms.resize(n_images);
	ds.xforms_end.clear();  // end = start
	ds.paths.resize(n_images);
	ds.pixels.resize(n_images);
	nerf.training.dataset = std::move(ds);
	load_nerf_post();
	nerf.training.n_images_for_training = 0;
	training_data_available = true;
}

// Testbed::load_nerf_post (src/testbed_nerf.cu:2151-2238)
void Testbed::load_nerf_post() {
	NerfDataset& ds = nerf.training.dataset;
	nerf.rgb_activation = ds.is_hdr ? ENerfActivation::Exponential : ENerfActivation::Logistic;
	nerf.training.n_images_for_training = (int)ds.n_images;
	if (!ds.metadata.empty()) {
		screen_center = {1.f - ds.metadata[0].principal_point[0], 1.f - ds.metadata[0].principal_point[1]};
		nerf.render_lens = ds.metadata[0].lens;  // src/testbed_nerf.cu:2202
	}
	if (ds.aabb_scale <= 0 || (ds.aabb_scale & (ds.aabb_scale - 1)))
		throw std::runtime_error("NeRF dataset's `aabb_scale` must be a power of two, but is " + std::to_string(ds.aabb_scale) + ".");
	const int max_aabb_scale = 1 << (NERF_CASCADES - 1);
	if (ds.aabb_scale > max_aabb_scale) throw std::runtime_error("NeRF dataset must have `aabb_scale <= 128`.");
	const float half = 0.5f * (float)std::min(max_aabb_scale, ds.aabb_scale);
	aabb_min = {0.5f - half, 0.5f - half, 0.5f - half};
	aabb_max = {0.5f + half, 0.5f + half, 0.5f + half};
	// m_render_aabb = the training aabb, or the dataset's render_aabb intersected with it (src/testbed_nerf.cu:2221-2225)
	render_aabb_min = aabb_min;
	render_aabb_max = aabb_max;
	render_aabb_to_local = ds.render_aabb_to_local;
	const bool empty = ds.render_aabb_min[0] > ds.render_aabb_max[0] || ds.render_aabb_min[1] > ds.render_aabb_max[1] ||
	                   ds.render_aabb_min[2] > ds.render_aabb_max[2];
	if (!empty)
		for (int k = 0; k < 3; ++k) {
			render_aabb_min[k] = std::max(ds.render_aabb_min[k], aabb_min[k]);
			render_aabb_max[k] = std::min(ds.render_aabb_max[k], aabb_max[k]);
		}
	raw_aabb_min = aabb_min;  // m_raw_aabb = m_aabb (src/testbed_nerf.cu:2221)
	raw_aabb_max = aabb_max;
	up_dir = ds.up;           // m_up_dir = dataset.up (:2237)
	nerf.max_cascade = 0;
	while ((1 << nerf.max_cascade) < ds.aabb_scale) ++nerf.max_cascade;
	nerf.cone_angle_constant = ds.aabb_scale <= 1 ? 0.0f : (1.0f / 256.0f);
	m_dataset_dirty = true;
	// load_nerf (src/testbed_nerf.cu:2176-2177): fresh latent codes, optimised when the dataset asks for them
	if (ds.n_extra_dims()) {
		pcg32 r(seed);
		if (m_rng_inc) {
			r.state = m_rng_state;
			r.inc = m_rng_inc;
		}
		reset_extra_dims(&r);
		m_rng_state = r.state;
		m_rng_inc = r.inc;
	} else {
		reset_extra_dims(nullptr);  // no codes: nothing is drawn
	}
	nerf.training.optimize_extra_dims = ds.n_extra_learnable_dims > 0;
	if (m_model && m_net_cfg.n_extra_dims != ds.n_extra_dims()) reset_network();
}

void Testbed::set_image_rgba8(int frame_idx, const uint8_t* rgba, int width, int height) {
	NerfDataset& ds = nerf.training.dataset;
	if (frame_idx < 0 || (size_t)frame_idx >= ds.n_images) throw std::runtime_error("Invalid frame index");
	ds.pixels[frame_idx].assign(rgba, rgba + (size_t)width * height * 4);
	ds.metadata[frame_idx].resolution = {width, height};
	m_dataset_dirty = true;
}

// Nerf::Training::set_image (python_api.cu): float RGBA (linear, premultiplied) -> RGBA8 sRGB straight alpha.
void Testbed::set_image(int frame_idx, const float* rgba, int width, int height) {
	std::vector<uint8_t> px((size_t)width * height * 4);
	for (size_t i = 0; i < (size_t)width * height; ++i) {
		const float a = std::min(std::max(rgba[4 * i + 3], 0.f), 1.f);
		for (int k = 0; k < 3; ++k) {
			const float lin = a > 0 ? rgba[4 * i + k] / a : 0.f;
			px[4 * i + k] = (uint8_t)std::lround(std::min(std::max(linear_to_srgb_h(lin), 0.f), 1.f) * 255.f);
		}
		px[4 * i + 3] = (uint8_t)std::lround(a * 255.f);
	}
	set_image_rgba8(frame_idx, px.data(), width, height);
}

void Testbed::set_camera_extrinsics(int frame_idx, const float* c2w, bool convert_to_ngp) {
	NerfDataset& ds = nerf.training.dataset;
	if (frame_idx < 0 || (size_t)frame_idx >= ds.n_images) throw std::runtime_error("Invalid frame index");
	if (convert_to_ngp) ds.xforms[frame_idx] = ds.nerf_matrix_to_ngp(c2w);
	else {
		Mat43 m;
		for (int col = 0; col < 4; ++col)
			for (int row = 0; row < 3; ++row) m.m[3 * col + row] = c2w[row * 4 + col];
		ds.xforms[frame_idx] = m;
	}
	if ((size_t)frame_idx < ds.xforms_end.size()) ds.xforms_end[frame_idx] = ds.xforms[frame_idx];  // end = start
	if ((size_t)frame_idx < ds.metadata.size()) ds.metadata[frame_idx].rolling_shutter = {0.f, 0.f, 0.f, 0.f};
	m_dataset_dirty = true;
}

void Testbed::set_camera_extrinsics_rolling_shutter(int frame_idx, const float* start, const float* end, const vec4& rs,
                                                    bool convert_to_ngp) {
	set_camera_extrinsics(frame_idx, end, convert_to_ngp);
	NerfDataset& ds = nerf.training.dataset;
	const Mat43 e = ds.xforms[frame_idx];
	set_camera_extrinsics(frame_idx, start, convert_to_ngp);
	while (ds.xforms_end.size() < ds.xforms.size()) ds.xforms_end.push_back(ds.xforms[ds.xforms_end.size()]);
	ds.xforms_end[frame_idx] = e;
	ds.metadata[frame_idx].rolling_shutter = rs;
	m_dataset_dirty = true;
}

Mat43 Testbed::get_camera_extrinsics(int frame_idx) const {
	const NerfDataset& ds = nerf.training.dataset;
	if (frame_idx < 0 || (size_t)frame_idx >= ds.n_images) throw std::runtime_error("Invalid frame index");
	return ds.ngp_matrix_to_nerf(training_transform((size_t)frame_idx));  // offsets applied (src/testbed_nerf.cu:2089-2094)
}

// Nerf::Training::set_camera_intrinsics (src/testbed_nerf.cu:1989-2010)
// Nerf::Training::set_camera_intrinsics (src/testbed_nerf.cu:1989-2010)
void Testbed::set_camera_intrinsics(int frame_idx, float fx, float fy, float cx, float cy, float k1, float k2, float p1,
                                    float p2, float k3, float k4, bool is_fisheye) {
	NerfDataset& ds = nerf.training.dataset;
	if (frame_idx < 0 || (size_t)frame_idx >= ds.n_images) return;
	if (fx <= 0.f) fx = fy;
	if (fy <= 0.f) fy = fx;
	auto& m = ds.metadata[frame_idx];
	cx = cx < 0.f ? -cx : cx / (float)m.resolution[0];
	cy = cy < 0.f ? -cy : cy / (float)m.resolution[1];
	m.lens = Lens{};
	if (k1 != 0.f || k2 != 0.f || k3 != 0.f || k4 != 0.f || p1 != 0.f || p2 != 0.f) {
		m.lens.mode = is_fisheye ? ELensMode::OpenCVFisheye : ELensMode::OpenCV;
		const float prm[4] = {k1, k2, is_fisheye ? k3 : p1, is_fisheye ? k4 : p2};
		for (int q = 0; q < 4; ++q) m.lens.params[q] = prm[q];
	}
	m.focal_length = {fx, fy};
	m.principal_point = {cx, cy};
	m_dataset_dirty = true;
}

// compute_sharpness (src/nerf_loader.cu:111-151) on the host, from the stored RGBA8 sRGB pixels as
// read_rgba sees them (linear, premultiplied).  A tile narrower than a pixel (images below 128 x 72)
// gets 0 where the reference divides by zero.
std::vector<float> NerfDataset::sharpness(size_t i) const {
	constexpr int SX = 128, SY = 72;
	std::vector<float> out((size_t)SX * SY, 0.0f);
	if (i >= pixels.size() || pixels[i].empty()) return out;
	const int W = metadata[i].resolution[0], H = metadata[i].resolution[1];
	const uint8_t* px = pixels[i].data();
	auto s2l = [](float c) { return c <= 0.04045f ? c / 12.92f : std::pow((c + 0.055f) / 1.055f, 2.4f); };
	auto luma = [&](int x, int y) {
		const uint8_t* p = px + 4 * ((size_t)y * W + x);
		const float a = p[3] * (1.0f / 255.0f);
		const float r = s2l(p[0] * (1.0f / 255.0f)) * a, g = s2l(p[1] * (1.0f / 255.0f)) * a, b = s2l(p[2] * (1.0f / 255.0f)) * a;
		return r * 0.2126f + g * 0.7152f + b * 0.0722f;
	};
	for (int y = 0; y < SY; ++y)
		for (int x = 0; x < SX; ++x) {
			int x1 = (x * W) / SX, x2 = ((x + 1) * W) / SX, y1 = (y * H) / SY, y2 = ((y + 1) * H) / SY;
			x1 = std::max(x1, 1); y1 = std::max(y1, 1);
			x2 = std::min(x2, W - 2); y2 = std::min(y2, H - 2);
			if (x2 <= x1 || y2 <= y1) continue;
			float tot_lap = 0.f, tot_lap2 = 0.f;
			const float scal = 1.f / (float)((x2 - x1) * (y2 - y1));
			for (int yy = y1; yy < y2; ++yy)
				for (int xx = x1; xx < x2; ++xx) {
					const float lap = luma(xx, yy) * 4.f - luma(xx, yy - 1) - luma(xx + 1, yy) - luma(xx, yy + 1) - luma(xx - 1, yy);
					tot_lap += lap;
					tot_lap2 += lap * lap;
				}
			tot_lap *= scal;
			tot_lap2 *= scal;
			out[(size_t)y * SX + x] = tot_lap2 - tot_lap * tot_lap;
		}
	return out;
}

void Testbed::free_device_dataset() {
	if (m_dev_sharpness) (void)hipFree(m_dev_sharpness);
	m_dev_sharpness = nullptr;
	for (void* p : m_dev_pixels) (void)hipFree(p);
	m_dev_pixels.clear();
	for (void* p : m_dev_depths)
		if (p) (void)hipFree(p);
	m_dev_depths.clear();
	if (m_dev_meta) (void)hipFree(m_dev_meta);
	m_dev_meta = nullptr;
}

// rotmat / rotvec (tcnn vec.h): Rodrigues rotation of angle |r| about r / |r|, and its inverse.
static std::array<float, 9> rotmat(const vec3& r) {  // row-major 3x3
	const double th = std::sqrt((double)r[0] * r[0] + (double)r[1] * r[1] + (double)r[2] * r[2]);
	std::array<float, 9> R{1, 0, 0, 0, 1, 0, 0, 0, 1};
	if (th < 1e-12) return R;
	const double x = r[0] / th, y = r[1] / th, z = r[2] / th, c = std::cos(th), s = std::sin(th), C = 1.0 - c;
	R = {(float)(c + x * x * C), (float)(x * y * C - z * s), (float)(x * z * C + y * s),
	     (float)(y * x * C + z * s), (float)(c + y * y * C), (float)(y * z * C - x * s),
	     (float)(z * x * C - y * s), (float)(z * y * C + x * s), (float)(c + z * z * C)};
	return R;
}
static vec3 rotvec(const std::array<float, 9>& R) {
	const double tr = (double)R[0] + R[4] + R[8];
	const double c = std::min(1.0, std::max(-1.0, (tr - 1.0) * 0.5));
	const double th = std::acos(c);
	if (th < 1e-12) return {0.f, 0.f, 0.f};
	const double k = th / (2.0 * std::sin(th));
	return {(float)((R[7] - R[5]) * k), (float)((R[2] - R[6]) * k), (float)((R[3] - R[1]) * k)};
}
static std::array<float, 9> matmul3(const std::array<float, 9>& A, const std::array<float, 9>& B) {
	std::array<float, 9> C{};
	for (int i = 0; i < 3; ++i)
		for (int j = 0; j < 3; ++j) C[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
	return C;
}

// NerfDataset transform with the optimised extrinsic offsets (Nerf::Training::update_transforms,
// src/testbed_nerf.cu:2112-2140): rotation = rotmat(rot offset) * R, translation += pos offset.
Mat43 Testbed::training_transform_end(size_t i) const {
	const NerfTraining& tr = nerf.training;
	if (i >= tr.dataset.xforms_end.size()) return training_transform(i);
	// the same offsets on the end transform (src/testbed_nerf.cu:2128-2134)
	Mat43 x = tr.dataset.xforms_end[i];
	if (i < tr.cam_rot_offset.size()) {
		const std::array<float, 9> Rm = rotmat(tr.cam_rot_offset[i].variable);
		Mat43 y = x;
		for (int c = 0; c < 3; ++c)
			for (int r = 0; r < 3; ++r)
				y.m[3 * c + r] = Rm[3 * r] * x.m[3 * c] + Rm[3 * r + 1] * x.m[3 * c + 1] + Rm[3 * r + 2] * x.m[3 * c + 2];
		x = y;
	}
	if (i < tr.cam_pos_offset.size())
		for (int r = 0; r < 3; ++r) x.m[9 + r] += tr.cam_pos_offset[i].variable[r];
	return x;
}

Mat43 Testbed::training_transform(size_t i) const {
	const NerfTraining& tr = nerf.training;
	Mat43 x = tr.dataset.xforms[i];
	if (i < tr.cam_rot_offset.size()) {
		const std::array<float, 9> Rm = rotmat(tr.cam_rot_offset[i].variable);
		Mat43 y = x;
		for (int c = 0; c < 3; ++c)
			for (int r = 0; r < 3; ++r)
				y.m[3 * c + r] = Rm[3 * r] * x.m[3 * c] + Rm[3 * r + 1] * x.m[3 * c + 1] + Rm[3 * r + 2] * x.m[3 * c + 2];
		x = y;
	}
	if (i < tr.cam_pos_offset.size())
		for (int r = 0; r < 3; ++r) x.m[9 + r] += tr.cam_pos_offset[i].variable[r];
	return x;
}

void Testbed::upload_metadata() {
	const NerfDataset& ds = nerf.training.dataset;
	std::vector<ngp_image> meta(ds.n_images);
	for (size_t i = 0; i < ds.n_images; ++i) {
		ngp_image& im = meta[i];
		std::memset(&im, 0, sizeof(im));
		im.pixels = (uint64_t)(uintptr_t)m_dev_pixels[i];
		im.depth = i < m_dev_depths.size() ? (uint64_t)(uintptr_t)m_dev_depths[i] : 0;
		im.width = (uint32_t)ds.metadata[i].resolution[0];
		im.height = (uint32_t)ds.metadata[i].resolution[1];
		for (int k = 0; k < 2; ++k) {
			im.focal_length[k] = ds.metadata[i].focal_length[k];
			im.principal_point[k] = ds.metadata[i].principal_point[k];
		}
		std::memcpy(im.xform, training_transform(i).m, sizeof(im.xform));
		std::memcpy(im.xform_end, training_transform_end(i).m, sizeof(im.xform_end));
		for (int k = 0; k < 4; ++k) im.rolling_shutter[k] = ds.metadata[i].rolling_shutter[k];
		im.lens_mode = (int32_t)ds.metadata[i].lens.mode;
		std::memcpy(im.lens_params, ds.metadata[i].lens.params, sizeof(im.lens_params));
	}
	if (!m_dev_meta) hk(hipMalloc(&m_dev_meta, std::max<size_t>(1, meta.size()) * sizeof(ngp_image)), "hipMalloc meta");
	hk(hipMemcpy(m_dev_meta, meta.data(), meta.size() * sizeof(ngp_image), hipMemcpyHostToDevice), "upload meta");
}

void Testbed::upload_dataset() {
	if (!m_dataset_dirty) return;
	const NerfDataset& ds = nerf.training.dataset;
	for (size_t i = 0; i < ds.n_images; ++i)
		if (ds.pixels[i].empty()) throw std::runtime_error("Training image " + std::to_string(i) + " has no pixels.");
	free_device_dataset();
	m_dev_pixels.resize(ds.n_images, nullptr);
	m_dev_depths.assign(ds.n_images, nullptr);
	for (size_t i = 0; i < ds.n_images; ++i) {
		hk(hipMalloc(&m_dev_pixels[i], ds.pixels[i].size()), "hipMalloc image");
		hk(hipMemcpy(m_dev_pixels[i], ds.pixels[i].data(), ds.pixels[i].size(), hipMemcpyHostToDevice), "upload image");
		if (i < ds.depths.size() && !ds.depths[i].empty()) {
			const size_t nb = ds.depths[i].size() * sizeof(float);
			hk(hipMalloc(&m_dev_depths[i], nb), "hipMalloc depth");
			hk(hipMemcpy(m_dev_depths[i], ds.depths[i].data(), nb, hipMemcpyHostToDevice), "upload depth");
		}
	}
	upload_metadata();
	m_dataset_dirty = false;
}

// ---------------------------------------------------------------------------
// Network configuration
// ---------------------------------------------------------------------------
std::string Testbed::find_network_config(const std::string& path) const {
	if (file_exists(path)) return path;
	// configs/<mode>/<name>, looked up next to the package and under root_dir (src/testbed.cu find_network_config)
	const std::string name = basename_of(path);
	std::vector<std::string> roots;
	if (!root_dir.empty()) roots.push_back(root_dir + "/configs/nerf/");
	if (const char* env = std::getenv("NGP_CONFIG_DIR")) roots.push_back(std::string(env) + "/");
	for (const std::string& r : roots) {
		if (file_exists(r + path)) return r + path;
		if (file_exists(r + name)) return r + name;
	}
	return path;
}

Json Testbed::load_network_config(const std::string& path) const {
	if (!file_exists(path)) throw std::runtime_error("Network config '" + path + "' does not exist.");
	Json j = Json::parse(read_text(path));
	// merge_parent_network_config (src/testbed.cu:86-97)
	if (j.contains("parent")) {
		const std::string& par = j["parent"].str();
		const std::string pp = (!par.empty() && par[0] == '/') ? par : parent_path(path) + "/" + par;
		Json parent = load_network_config(pp);
		parent.merge_patch(j);
		j = parent;
	}
	return j;
}

void Testbed::reload_network_from_file(const std::string& path) {
	if (!path.empty()) network_config_path = path;
	if (mode == ETestbedMode::None) return;
	const std::string full = find_network_config(network_config_path);
	if (file_exists(full)) m_network_config = load_network_config(full);
	reset_network();
}

void Testbed::reload_network_from_json(const Json& json, const std::string& config_base_path) {
	Json j = json;
	if (j.contains("parent")) {
		Json parent = load_network_config(find_network_config(config_base_path.empty() ? j["parent"].str()
		                                                                              : config_base_path + "/" + j["parent"].str()));
		parent.merge_patch(j);
		j = parent;
	}
	m_network_config = j;
	reset_network();
}

static int loss_type_from_string(const std::string& s) {
	std::string l = s;
	std::transform(l.begin(), l.end(), l.begin(), ::tolower);
	if (l == "l2") return 0;
	if (l == "l1") return 1;
	if (l == "mape") return 2;
	if (l == "smape") return 3;
	if (l == "huber" || l == "smoothl1") return 4;
	if (l == "logl1") return 5;
	if (l == "relativel2") return 6;
	throw std::runtime_error("Unknown loss type.");
}

// Testbed::reset_network (src/testbed.cu:3624-3868), NeRF branch.
void Testbed::reset_network(bool clear_density_grid) {
	pcg32 rng(seed);
	nerf.training.counters_rgb = NerfCounters{};
	nerf.training.counters_rgb.rays_per_batch = 1 << 12;
	nerf.training.n_steps_since_error_map_update = 0;  // src/testbed.cu:3636-3639
	nerf.training.n_rays_since_error_map_update = 0;
	nerf.training.n_steps_between_error_map_updates = 128;
	nerf.training.error_map.is_cdf_valid = false;
	nerf.training.n_steps_since_cam_update = 0;
	// reset_camera_extrinsics (src/testbed.cu:3642)
	nerf.training.cam_pos_offset.assign(nerf.training.dataset.n_images, NerfTraining::Adam3{});
	nerf.training.cam_rot_offset.assign(nerf.training.dataset.n_images, NerfTraining::Adam3{});
	nerf.training.cam_focal_length_offset = NerfTraining::Adam2{};
	if (training_data_available) m_dataset_dirty = true;
	pcg32 grid_rng(rng.next_uint());
	reset_extra_dims(&rng);  // src/testbed.cu:3736
	m_rng_state = rng.state;
	m_rng_inc = rng.inc;
	nerf.training.density_grid_rng_state = grid_rng.state;
	nerf.training.density_grid_rng_inc = grid_rng.inc;
	training_step = 0;
	loss = 0.f;
	const Json& cfg = m_network_config;
	nerf.training.loss_type = (ELossType)loss_type_from_string(cfg["loss"].value("otype", std::string("L2")));
	build_model(cfg);
	if (clear_density_grid) nerf.density_grid_ema_step = 0;
}

void Testbed::build_model(const Json& cfg) {
	if (mode != ETestbedMode::Nerf) throw std::runtime_error("reset_network: only the NeRF mode is implemented.");
	const Json& enc = cfg["encoding"];
	std::string etype = enc.value("otype", std::string("HashGrid"));
	std::transform(etype.begin(), etype.end(), etype.begin(), ::tolower);
	if (etype.find("grid") == std::string::npos)
		throw std::runtime_error("Only the HashGrid encoding is implemented on MI355X (got '" + etype + "').");
	ngp_network_config c{};
	c.n_features_per_level = (uint32_t)enc.value("n_features_per_level", 2.0);
	c.n_levels = enc.contains("n_features") && enc["n_features"].num() > 0 ? (uint32_t)enc["n_features"].num() / c.n_features_per_level
	                                                                       : (uint32_t)enc.value("n_levels", 16.0);
	c.log2_hashmap_size = (uint32_t)enc.value("log2_hashmap_size", 15.0);
	c.base_resolution = (uint32_t)enc.value("base_resolution", 0.0);
	if (!c.base_resolution) c.base_resolution = 1u << (c.log2_hashmap_size / 3);
	float pls = (float)enc.value("per_level_scale", 0.0);
	if (pls <= 0.f && c.n_levels > 1) {
		const float desired = 2048.0f;  // src/testbed.cu:3702
		pls = std::exp(std::log(desired * (float)nerf.training.dataset.aabb_scale / (float)c.base_resolution) / (float)(c.n_levels - 1));
	}
	c.per_level_scale = pls > 0 ? pls : 1.0f;
	const Json& net = cfg["network"];
	const Json& rgb = cfg.contains("rgb_network") ? cfg["rgb_network"] : cfg["network"];
	c.n_neurons = (uint32_t)net.value("n_neurons", 64.0);
	c.density_hidden_layers = (uint32_t)(net.contains("n_hidden_layers") ? net["n_hidden_layers"].num() : std::max(1.0, net.value("n_layers", 2.0) - 1.0));
	c.rgb_hidden_layers = (uint32_t)(rgb.contains("n_hidden_layers") ? rgb["n_hidden_layers"].num() : 2.0);
	if ((uint32_t)rgb.value("n_neurons", (double)c.n_neurons) != c.n_neurons)
		throw std::runtime_error("density and rgb MLPs must share n_neurons on this build");
	c.rgb_activation = (int32_t)nerf.rgb_activation;
	c.density_activation = (int32_t)nerf.density_activation;
	// NerfNetwork(n_pos_dims, n_dir_dims, n_extra_dims = dataset.n_extra_dims(), ...) (src/testbed.cu:3742-3756)
	c.n_extra_dims = nerf.training.dataset.n_extra_dims();
	// optimizer chain: [Ema] -> [ExponentialDecay] -> Adam (configs/nerf/base.json:5-22)
	c.ema_decay = 0.0f;
	c.decay_start = 0xFFFFFFFFu;
	c.decay_interval = 0;
	c.decay_base = 1.0f;
	const Json* opt = &cfg["optimizer"];
	while (opt->is_object()) {
		std::string ot = opt->value("otype", std::string("Adam"));
		if (ot == "Ema") c.ema_decay = (float)opt->value("decay", 0.99);
		else if (ot == "ExponentialDecay") {
			c.decay_start = (uint32_t)opt->value("decay_start", 0.0);
			c.decay_interval = (uint32_t)opt->value("decay_interval", 10000.0);
			c.decay_base = (float)opt->value("decay_base", 0.33);
		} else if (ot == "Adam") {
			c.learning_rate = (float)opt->value("learning_rate", 1e-3);
			c.beta1 = (float)opt->value("beta1", 0.9);
			c.beta2 = (float)opt->value("beta2", 0.99);
			c.epsilon = (float)opt->value("epsilon", 1e-8);
			c.l2_reg = (float)opt->value("l2_reg", 1e-8);
		} else throw std::runtime_error("Unsupported optimizer '" + ot + "' (Ema/ExponentialDecay/Adam implemented)");
		if (!opt->contains("nested")) break;
		opt = &(*opt)["nested"];
	}
	if (c.ema_decay == 0.0f) c.ema_decay = 0.0f;  // no Ema: inference params track the weights exactly
	// the distortion map and its trainer (src/testbed.cu:3781-3792): zero map, fresh Adam
	{
		DistortionMap d;
		if (cfg.contains("distortion_map")) {
			const Json& dm = cfg["distortion_map"];
			if (dm.contains("resolution") && dm["resolution"].is_array()) {
				d.rx = (int)dm["resolution"][0].num();
				d.ry = (int)dm["resolution"][1].num();
			}
			const Json* o = dm.contains("optimizer") ? &dm["optimizer"] : nullptr;
			while (o && o->is_object()) {
				const std::string ot = o->value("otype", std::string("Adam"));
				if (ot == "ExponentialDecay") {
					d.decay_start = (uint32_t)o->value("decay_start", 0.0);
					d.decay_interval = (uint32_t)o->value("decay_interval", 10000.0);
					d.decay_end = (uint32_t)o->value("decay_end", 4294967295.0);
					d.decay_base = (float)o->value("decay_base", 0.33);
				} else if (ot == "Adam") {
					d.lr = (float)o->value("learning_rate", 1e-3);
					d.beta1 = (float)o->value("beta1", 0.9);
					d.beta2 = (float)o->value("beta2", 0.99);
					d.eps = (float)o->value("epsilon", 1e-8);
				} else throw std::runtime_error("distortion_map: unsupported optimizer '" + ot + "'");
				o = o->contains("nested") ? &(*o)["nested"] : nullptr;
			}
		}
		if (d.rx <= 0 || d.ry <= 0) throw std::runtime_error("distortion_map: resolution must be positive");
		const size_t n = (size_t)d.rx * d.ry * 2;
		d.params.assign(n, 0.0f);
		d.m.assign(n, 0.0f);
		d.v.assign(n, 0.0f);
		d.steps.assign(n, 0u);
		for (float* p : {m_dist, m_dist_grad})
			if (p) (void)hipFree(p);
		m_dist = m_dist_grad = nullptr;
		m_distortion = d;
	}
	int device = 0;
	hk(hipGetDevice(&device), "hipGetDevice");
	if (m_model) {
		sync();
		ck(ngp_model_destroy(m_model));
		m_model = nullptr;
	}
	// the tuning is applied before the model is published, so a failure leaves no model half set up
	ngp_model* model = nullptr;
	ck(ngp_model_create(device, &c, seed, &model));
	if (ngp_model_set_tuning(model, &m_tuning) != NGP_OK) {
		const std::string msg = ngp_last_error();
		(void)ngp_model_destroy(model);
		throw std::runtime_error(msg);
	}
	m_model = model;
	m_net_cfg = c;
}

// ---------------------------------------------------------------------------
// Training
// ---------------------------------------------------------------------------
void Testbed::set_tuning(const ngp_tuning& t) {
	ck(ngp_tuning_validate(&t));  // also before a model exists: an invalid value never reaches build_model
	if (m_model) ck(ngp_model_set_tuning(m_model, &t));
	m_tuning = t;
}

void Testbed::update_density_grid(uint32_t n_uniform, uint32_t n_nonuniform) {
	upload_dataset();
	ngp_grid_args g{};
	g.images = (const ngp_image*)m_dev_meta;
	g.n_images = (uint32_t)nerf.training.n_images_for_training;
	for (int k = 0; k < 3; ++k) { g.aabb_min[k] = aabb_min[k]; g.aabb_max[k] = aabb_max[k]; }
	g.max_cascade = nerf.max_cascade;
	g.decay = nerf.training.density_grid_decay;
	g.n_uniform_samples = n_uniform;
	g.n_nonuniform_samples = n_nonuniform;
	g.rng_state = nerf.training.density_grid_rng_state;
	g.rng_inc = nerf.training.density_grid_rng_inc;
	g.ema_step = nerf.density_grid_ema_step;
	const bool changed = nerf.training.n_images_for_training != nerf.training.n_images_for_training_prev;
	g.mark_untrained = (training_step == 0 || changed) ? 1 : 0;
	g.clear_visible = training_step == 0 ? 1 : 0;
	nerf.training.n_images_for_training_prev = nerf.training.n_images_for_training;
	if (training_step == 0) nerf.density_grid_ema_step = 0, g.ema_step = 0;
	g.use_inference_params = 0;
	g.rank = (uint32_t)m_rank;
	g.world_size = (uint32_t)m_world;
	if (distributed()) {
		ck(ngp_density_grid_evaluate(m_model, &g, m_stream));
		float *grid, *tmp;
		ck(ngp_density_grid_buffers(m_model, &grid, nullptr, &tmp, nullptr));
		allreduce_f32(tmp, (size_t)NERF_GRID_N_CELLS * (nerf.max_cascade + 1), true);
		ck(ngp_density_grid_finish(m_model, &g, m_stream));
	} else {
		ck(ngp_density_grid_update(m_model, &g, m_stream));
	}
	pcg32 r;
	r.state = nerf.training.density_grid_rng_state;
	r.inc = nerf.training.density_grid_rng_inc;
	r.advance();
	r.advance();
	nerf.training.density_grid_rng_state = r.state;
	++nerf.density_grid_ema_step;
}

void Testbed::train_nerf(uint32_t batch, bool get_loss_scalar) {
	if (nerf.training.n_images_for_training == 0) return;
	upload_dataset();
	NerfCounters& ctr = nerf.training.counters_rgb;
	// data parallelism: the ranks train one global batch of world x batch samples over
	// rays_per_batch global rays, each rank its contiguous slice -- the same sample set, caps, rollover
	// and host state as one process training with batch world x batch (ngp_train_args.world_size)
	const uint32_t W = (uint32_t)m_world;
	batch *= W;
	const uint32_t max_samples = batch * 16;
	uint32_t max_inference;
	if (ctr.measured_batch_size_before_compaction == 0) ctr.measured_batch_size_before_compaction = max_inference = max_samples;
	else max_inference = next_multiple_host(std::min(ctr.measured_batch_size_before_compaction, max_samples), BATCH_SIZE_GRANULARITY);
	if (training_step == 0) ctr.n_rays_total = 0;

	// error map (re)allocation at the start of each accumulation period (src/testbed_nerf.cu:2486-2492)
	NerfTraining& tr = nerf.training;
	if (tr.n_steps_since_error_map_update == 0 && !tr.dataset.metadata.empty()) {
		const uint32_t n_samples_per_image = (uint32_t)(((uint64_t)tr.n_steps_between_error_map_updates * ctr.rays_per_batch) /
		                                                std::max<size_t>(tr.dataset.n_images, 1));
		const ivec2 res = tr.dataset.metadata[0].resolution;
		const int r = (int)(std::sqrt(std::sqrt((float)n_samples_per_image)) * 3.5f);
		tr.error_map.resolution = {std::min(r, res[0]), std::min(r, res[1])};
		const size_t n = (size_t)tr.error_map.resolution[0] * tr.error_map.resolution[1] * tr.dataset.n_images;
		if (n > m_err_cap) {
			if (m_err) (void)hipFree(m_err);
			hk(hipMalloc((void**)&m_err, std::max<size_t>(n, 1) * sizeof(float)), "hipMalloc error map");
			m_err_cap = n;
		}
		hk(hipMemsetAsync(m_err, 0, std::max<size_t>(n, 1) * sizeof(float), (hipStream_t)m_stream), "error map clear");
	}

	// per-image exposure: always applied to the targets, optimised on request (src/testbed_nerf.cu:2468-2473)
	const size_t n_img = tr.dataset.n_images;
	if (tr.cam_exposure.size() != n_img) tr.cam_exposure.assign(n_img, NerfTraining::Adam3{});
	if (n_img * 3 > m_exp_cap) {
		if (m_exp) (void)hipFree(m_exp);
		if (m_exp_grad) (void)hipFree(m_exp_grad);
		hk(hipMalloc((void**)&m_exp, n_img * 3 * sizeof(float)), "hipMalloc exposure");
		hk(hipMalloc((void**)&m_exp_grad, n_img * 3 * sizeof(float)), "hipMalloc exposure gradient");
		m_exp_cap = n_img * 3;
		std::vector<float> e(n_img * 3);
		for (size_t i = 0; i < n_img; ++i)
			for (int k = 0; k < 3; ++k) e[3 * i + k] = tr.cam_exposure[i].variable[k];
		hk(hipMemcpyAsync(m_exp, e.data(), e.size() * sizeof(float), hipMemcpyHostToDevice, (hipStream_t)m_stream), "exposure h2d");
	}
	if (tr.n_steps_since_cam_update == 0)
		hk(hipMemsetAsync(m_exp_grad, 0, n_img * 3 * sizeof(float), (hipStream_t)m_stream), "exposure gradient clear");
	// extrinsic offsets and their gradients (src/testbed_nerf.cu:2158-2167, 2468-2471)
	if (tr.cam_pos_offset.size() != n_img) tr.cam_pos_offset.assign(n_img, NerfTraining::Adam3{});
	if (tr.cam_rot_offset.size() != n_img) tr.cam_rot_offset.assign(n_img, NerfTraining::Adam3{});
	if (tr.optimize_extrinsics) {
		if (n_img * 6 > m_cam_grad_cap) {
			if (m_cam_grad) (void)hipFree(m_cam_grad);
			hk(hipMalloc((void**)&m_cam_grad, n_img * 6 * sizeof(float)), "hipMalloc camera gradients");
			m_cam_grad_cap = n_img * 6;
			hk(hipMemsetAsync(m_cam_grad, 0, n_img * 6 * sizeof(float), (hipStream_t)m_stream), "camera gradient clear");
		}
		if (tr.n_steps_since_cam_update == 0)
			hk(hipMemsetAsync(m_cam_grad, 0, n_img * 6 * sizeof(float), (hipStream_t)m_stream), "camera gradient clear");
	}

	// the learned distortion map (src/testbed_nerf.cu:2468-2474, 2787): applied to the training rays
	// once it is being optimised, its gradients cleared at the start of every camera-update period
	const size_t n_dist = m_distortion.params.size();
	if (tr.optimize_distortion && !m_distortion.active) {
		m_distortion.active = true;
		hk(hipMalloc((void**)&m_dist, n_dist * sizeof(float)), "hipMalloc distortion map");
		hk(hipMalloc((void**)&m_dist_grad, 2 * n_dist * sizeof(float)), "hipMalloc distortion gradients");
		hk(hipMemcpyAsync(m_dist, m_distortion.params.data(), n_dist * sizeof(float), hipMemcpyHostToDevice, (hipStream_t)m_stream), "distortion h2d");
		hk(hipMemsetAsync(m_dist_grad, 0, 2 * n_dist * sizeof(float), (hipStream_t)m_stream), "distortion gradient clear");
	}
	if (m_distortion.active && tr.optimize_distortion && tr.n_steps_since_cam_update == 0)
		hk(hipMemsetAsync(m_dist_grad, 0, 2 * n_dist * sizeof(float), (hipStream_t)m_stream), "distortion gradient clear");

	ngp_train_args a{};
	a.images = (const ngp_image*)m_dev_meta;
	if (m_distortion.active) {
		a.distortion_map = m_dist;
		a.distortion_res[0] = (uint32_t)m_distortion.rx;
		a.distortion_res[1] = (uint32_t)m_distortion.ry;
		if (tr.optimize_distortion) {
			a.distortion_gradient = m_dist_grad;
			a.distortion_gradient_weight = m_dist_grad + n_dist;
		}
	}
	a.exposure = m_exp;
	a.exposure_gradient = tr.optimize_exposure ? m_exp_grad : nullptr;
	a.cam_pos_gradient = tr.optimize_extrinsics ? m_cam_grad : nullptr;
	a.cam_rot_gradient = tr.optimize_extrinsics ? m_cam_grad + 3 * n_img : nullptr;
	a.n_images = (uint32_t)nerf.training.n_images_for_training;
	if (ctr.rays_per_batch % W) ctr.rays_per_batch = next_multiple_host(ctr.rays_per_batch, W);
	a.n_rays = ctr.rays_per_batch / W;
	a.n_rays_total = ctr.n_rays_total;
	a.target_batch_size = batch;
	a.max_samples = max_inference;
	a.training_step = training_step;
	a.rng_state = m_rng_state;
	a.rng_inc = m_rng_inc;
	a.ray_index_offset = (uint32_t)m_rank * a.n_rays;
	a.n_rays_global = ctr.rays_per_batch;
	if (distributed()) {
		a.rank = (uint32_t)m_rank;
		a.world_size = W;
		a.allreduce_i32 = &Testbed::dp_allreduce_i32;
		a.allreduce_user = this;
	}
	a.deterministic = deterministic ? 1 : 0;
	a.max_level_rand_training = m_max_level_rand_training ? 1 : 0;
	// per-image latent codes (src/testbed_nerf.cu:2478-2484, 2792-2793): the table, and its gradient (cleared per step)
	// while they are optimised
	const bool train_extra_dims = tr.dataset.n_extra_learnable_dims > 0 && tr.optimize_extra_dims;
	if (n_extra_dims()) {
		if (!m_extra) upload_extra_dims();
		a.extra_dims = m_extra;
		if (train_extra_dims) {
			hk(hipMemsetAsync(m_extra_grad, 0, (m_extra_rows - 1) * NGP_EXTRA_ROW * sizeof(float), (hipStream_t)m_stream),
			   "extra dims gradient clear");
			a.extra_dims_gradient = m_extra_grad;
		}
	}
	for (int k = 0; k < 3; ++k) { a.aabb_min[k] = aabb_min[k]; a.aabb_max[k] = aabb_max[k]; }
	a.cone_angle_constant = nerf.cone_angle_constant;
	a.max_cascade = nerf.max_cascade;
	a.loss_type = (int32_t)nerf.training.loss_type;
	a.random_bg_color = nerf.training.random_bg_color;
	for (int k = 0; k < 3; ++k) a.background_color[k] = background_color[k];
	a.snap_to_pixel_centers = nerf.training.snap_to_pixel_centers;
	a.train_in_linear_colors = nerf.training.linear_colors;
	a.color_space = (int32_t)color_space;
	a.near_distance = nerf.training.near_distance;
	a.optimize_mlp = train_network;
	a.optimize_encoding = train_encoding;
	a.defer_optimizer = distributed() ? 1 : 0;
	a.full_forward = train_full_forward ? 1 : 0;
	a.depth_supervision_lambda = tr.depth_supervision_lambda;
	a.depth_loss_type = (int32_t)tr.depth_loss_type;
	for (size_t i = 0; i < tr.dataset.metadata.size(); ++i)
		if (tr.dataset.metadata[i].lens.mode != ELensMode::Perspective || tr.dataset.metadata[i].rolling_shutter != vec4{0.f, 0.f, 0.f, 0.f})
			a.has_lens = 1;  // the general sampler instance (lenses, rolling shutter)
	if (m_err && tr.error_map.resolution[0] > 0 && tr.error_map.resolution[1] > 0) {
		a.error_map = m_err;  // accumulate_error is always on (src/testbed_nerf.cu:2756)
		a.error_map_res[0] = (uint32_t)tr.error_map.resolution[0];
		a.error_map_res[1] = (uint32_t)tr.error_map.resolution[1];
	}
	if (tr.include_sharpness_in_error && a.error_map) {
		// dataset sharpness (computed on first use) and the running-max grid (src/testbed_nerf.cu:2453-2464)
		const size_t per = (size_t)128 * 72;
		if (!m_dev_sharpness) {
			std::vector<float> all(per * tr.dataset.n_images);
			for (size_t i = 0; i < tr.dataset.n_images; ++i) {
				const std::vector<float> sh = tr.dataset.sharpness(i);
				std::copy(sh.begin(), sh.end(), all.begin() + per * i);
			}
			hk(hipMalloc((void**)&m_dev_sharpness, std::max<size_t>(all.size(), 1) * sizeof(float)), "hipMalloc sharpness");
			hk(hipMemcpy(m_dev_sharpness, all.data(), all.size() * sizeof(float), hipMemcpyHostToDevice), "upload sharpness");
		}
		const bool fresh = !m_sharp_grid;
		if (fresh) hk(hipMalloc((void**)&m_sharp_grid, (size_t)128 * 128 * 128 * 8 * sizeof(float)), "hipMalloc sharpness grid");
		a.sharpness_data = m_dev_sharpness;
		a.sharpness_res[0] = 128;
		a.sharpness_res[1] = 72;
		a.sharpness_grid = m_sharp_grid;
		a.sharpness_grid_clear = (fresh || training_step == 0) ? 1 : 0;
	}
	if (tr.error_map.is_cdf_valid) {
		if (tr.sample_focal_plane_proportional_to_error) {
			a.cdf_x_cond_y = m_cdf_x;
			a.cdf_y = m_cdf_y;
		}
		if (tr.sample_image_proportional_to_error) a.cdf_img = m_cdf_img;
		a.cdf_res[0] = (uint32_t)tr.error_map.cdf_resolution[0];
		a.cdf_res[1] = (uint32_t)tr.error_map.cdf_resolution[1];
	}
	ctr.n_rays_total += ctr.rays_per_batch;
	tr.n_rays_since_error_map_update += ctr.rays_per_batch;
	// one step: sample, forward, loss, backward; data parallel: the gradient all-reduce before the
	// (identical) optimizer step on every rank.  The chunked forward's violation word gates the
	// optimizer on the device (ngp_optimizer_step); every rank sees the max over the ranks.
	ngp_train_stats st{};
	for (int attempt = 0;; ++attempt) {
		ck(ngp_train_step(m_model, &a, m_stream));
		if (distributed()) {
			if (m_comm) {
				ck(ngp_allreduce_grads(m_model, m_comm, m_stream));
			} else {
				void *g = nullptr, *gg = nullptr;
				size_t bytes = 0, gbytes = 0;
				ngp_model_info info{};
				ck(ngp_model_get_info(m_model, &info));
				ck(ngp_model_buffer(m_model, NGP_GRADS_FP32, &g, &bytes));
				ck(ngp_model_buffer(m_model, deterministic ? NGP_GRADS_GRID_FIXED64 : NGP_GRADS_GRID_FP16, &gg, &gbytes));
				allreduce_dev(g, info.n_mlp_params, 0, false);
				allreduce_dev(gg, info.n_grid_params, deterministic ? 3 : 1, false);
			}
			// the violation word (early stops of the chunked forward in the low bits, a rank's sample capacity in
			// VIOL_CAPACITY, ngp_internal.h) gates the optimizer; its two parts are reduced separately (a max of
			// the packed word would hide one rank's early stops behind another's capacity flag), so every rank
			// sees any rank's early stops and any rank's overflow, and all of them skip or all of them step
			// (split and rebuilt on the device: the max-reduce of the parts stays on the stream -- asynchronous over
			// RCCL -- instead of three blocking host round trips per step)
			void* viol = nullptr;
			ck(ngp_train_scratch(m_model, NGP_SCRATCH_VIOLATIONS, &viol, nullptr));
			if (viol) {
				int32_t* dp = (int32_t*)m_red_buf + 8;
				ck(ngp_train_violation_parts(m_model, dp, 1, m_stream));
				allreduce_dev(dp, 2, 2, true);
				ck(ngp_train_violation_parts(m_model, dp, 0, m_stream));
			}
			ck(ngp_optimizer_step(m_model, training_step, train_network, train_encoding, m_stream));
		}
		// NerfCounters::update_after_training (src/testbed_nerf.cu:2422-2446)
		ck(ngp_train_read_stats(m_model, &st, m_stream));
		const bool early_stop = st.forward_early_stop_violations && !a.full_forward;
		if (!early_stop && !st.sample_capacity_overflow) break;
		if (attempt >= 4) throw std::runtime_error("Nerf training: the step could not be completed after 4 retries");
		// the step's update and its error-map, exposure, camera, distortion and sharpness deposits were skipped
		// on the device (every rank sees the violations of all ranks); drop its gradients and run it again --
		// with the full forward when the chunked forward stopped a ray before a sample its loss needed, with
		// buffers grown to the need when a rank's share of the samples did not fit
		ck(ngp_train_discard(m_model, m_stream));
		if (early_stop) {
			forward_early_stop_violations += st.forward_early_stop_violations;
			std::fprintf(stderr, "Nerf training: the chunked forward missed samples of %u rays; re-running the step with the full "
			             "forward and keeping it from now on.\n", st.forward_early_stop_violations);
			train_full_forward = true;
			a.full_forward = 1;
		}
	}
	// the latent codes' Adam step on every step (src/testbed_nerf.cu:2580-2599); data parallel: their gradient summed
	if (train_extra_dims) {
		if (distributed()) allreduce_f32(m_extra_grad, (m_extra_rows - 1) * NGP_EXTRA_ROW, false);
		update_extra_dims_step();
	}
	++training_step;
	// CDFs from the error map, every n_steps_between_error_map_updates (x1.5 each time)
	if (++tr.n_steps_since_error_map_update >= tr.n_steps_between_error_map_updates) update_error_map_cdf();
	// camera parameters every n_steps_between_cam_updates (src/testbed_nerf.cu:2577-2680)
	++tr.n_steps_since_cam_update;
	const bool train_camera = tr.optimize_extrinsics || tr.optimize_distortion || tr.optimize_focal_length || tr.optimize_exposure;
	if (train_camera && tr.n_steps_since_cam_update >= tr.n_steps_between_cam_updates) {
		if (tr.optimize_extrinsics) update_cam_extrinsics();
		if (tr.optimize_distortion) update_distortion_map();
		if (tr.optimize_focal_length) update_cam_focal_length();
		if (tr.optimize_exposure) update_cam_exposure();
		tr.n_steps_since_cam_update = 0;
	}
	// m_rng.advance() (src/testbed_nerf.cu:2925)
	pcg32 r;
	r.state = m_rng_state;
	r.inc = m_rng_inc;
	r.advance();
	m_rng_state = r.state;

	// the global counters: sums of the ranks' sample / compacted totals (exact int32) and losses
	if (distributed()) {
		int32_t cnt[2] = {(int32_t)st.measured_batch_size, (int32_t)st.measured_batch_size_before_compaction};
		float lv = st.loss;
		int32_t* dc = (int32_t*)m_red_buf;
		float* dl = (float*)m_red_buf + 4;
		hk(hipMemcpyAsync(dc, cnt, sizeof(cnt), hipMemcpyHostToDevice, (hipStream_t)m_stream), "stats h2d");
		hk(hipMemcpyAsync(dl, &lv, sizeof(lv), hipMemcpyHostToDevice, (hipStream_t)m_stream), "stats h2d");
		allreduce_dev(dc, 2, 2, false);
		allreduce_dev(dl, 1, 0, false);
		hk(hipMemcpyAsync(cnt, dc, sizeof(cnt), hipMemcpyDeviceToHost, (hipStream_t)m_stream), "stats d2h");
		hk(hipMemcpyAsync(&lv, dl, sizeof(lv), hipMemcpyDeviceToHost, (hipStream_t)m_stream), "stats d2h");
		sync();
		st.measured_batch_size = (uint32_t)cnt[0];
		st.measured_batch_size_before_compaction = (uint32_t)cnt[1];
		st.loss = lv;
	}
	m_last_stats = st;
	ctr.measured_batch_size = st.measured_batch_size;
	ctr.measured_batch_size_before_compaction = st.measured_batch_size_before_compaction;
	if (st.measured_batch_size_before_compaction == 0 || st.measured_batch_size == 0) {
		ctr.measured_batch_size = ctr.measured_batch_size_before_compaction = 0;
		loss = 0.f;
		std::fprintf(stderr, "Nerf training generated 0 samples. Aborting training.\n");
		shall_train = false;
		return;
	}
	if (get_loss_scalar) loss = st.loss * (float)st.measured_batch_size / (float)batch;
	uint32_t rpb = (uint32_t)((float)ctr.rays_per_batch * (float)batch / (float)st.measured_batch_size);
	// data parallel: rays_per_batch stays a multiple of the world size (every rank gets an equal slice);
	// 256-granular as the reference when the world size divides 256 (1, 2, 4, 8)
	const uint32_t gran = BATCH_SIZE_GRANULARITY % W == 0 ? BATCH_SIZE_GRANULARITY : BATCH_SIZE_GRANULARITY * W;
	ctr.rays_per_batch = std::min(next_multiple_host(rpb, gran), next_multiple_host((1u << 18) * W, gran));
}

// src/testbed_nerf.cu:2523-2575: construct_cdf_2d/1d on the device, the image CDF on the host
void Testbed::update_error_map_cdf() {
	NerfTraining& tr = nerf.training;
	const uint32_t n_images = (uint32_t)tr.dataset.n_images;
	const ivec2 res = tr.error_map.resolution;
	if (!m_err || n_images == 0 || res[0] <= 0 || res[1] <= 0) return;
	const size_t n = (size_t)res[0] * res[1] * n_images;
	// data parallel: every rank deposited the errors of its own rays
	if (distributed()) allreduce_f32(m_err, n, false);
	tr.error_map.cdf_resolution = res;
	if (n > m_cdf_cap) {
		if (m_cdf_x) (void)hipFree(m_cdf_x);
		hk(hipMalloc((void**)&m_cdf_x, n * sizeof(float)), "hipMalloc cdf_x_cond_y");
		m_cdf_cap = n;
	}
	const size_t ny = (size_t)res[1] * n_images;
	if (ny + n_images > m_cdf_img_cap) {
		if (m_cdf_y) (void)hipFree(m_cdf_y);
		if (m_cdf_img) (void)hipFree(m_cdf_img);
		hk(hipMalloc((void**)&m_cdf_y, ny * sizeof(float)), "hipMalloc cdf_y");
		hk(hipMalloc((void**)&m_cdf_img, n_images * sizeof(float)), "hipMalloc cdf_img");
		m_cdf_img_cap = ny + n_images;
	}
	ck(ngp_error_map_build_cdf(m_err, n_images, (uint32_t)res[0], (uint32_t)res[1], m_cdf_x, m_cdf_y, m_cdf_img, m_stream));
	// image CDF on the CPU ("single-threaded anyway", src/testbed_nerf.cu:2552-2567)
	std::vector<float> pmf(n_images), cdf(n_images);
	hk(hipMemcpyAsync(pmf.data(), m_cdf_img, n_images * sizeof(float), hipMemcpyDeviceToHost, (hipStream_t)m_stream), "cdf_img d2h");
	sync();
	float cum = 0.0f;
	for (uint32_t i = 0; i < n_images; ++i) {
		cum += pmf[i];
		cdf[i] = cum;
	}
	const float norm = 1.0f / cum;
	for (uint32_t i = 0; i < n_images; ++i) {
		pmf[i] = (1.0f - MIN_PMF) * pmf[i] * norm + MIN_PMF / (float)n_images;
		cdf[i] = (1.0f - MIN_PMF) * cdf[i] * norm + MIN_PMF * (float)(i + 1) / (float)n_images;
	}
	tr.error_map.pmf_img_cpu = pmf;
	hk(hipMemcpyAsync(m_cdf_img, cdf.data(), n_images * sizeof(float), hipMemcpyHostToDevice, (hipStream_t)m_stream), "cdf_img h2d");
	sync();
	tr.n_steps_since_error_map_update = 0;
	tr.n_rays_since_error_map_update = 0;
	tr.error_map.is_cdf_valid = true;
	tr.n_steps_between_error_map_updates = (uint32_t)((float)tr.n_steps_between_error_map_updates * 1.5f);
}

// m_optimizer->learning_rate(): Adam's rate under the ExponentialDecay of the config
float Testbed::current_learning_rate() const {
	const ngp_network_config& c = m_net_cfg;
	return exp_decay_learning_rate(c.learning_rate, c.decay_base, c.decay_start, c.decay_interval, 0xFFFFFFFFu, training_step);
}

// Exposure branch of the camera update (src/testbed_nerf.cu:2650-2677): per-image Adam
// (AdamOptimizer<vec3>, adam_optimizer.h:129-152) at the network's learning rate, then the
// mean exposure is subtracted so the scene brightness stays anchored.
void Testbed::update_cam_exposure() {
	NerfTraining& tr = nerf.training;
	const uint32_t n = (uint32_t)tr.n_images_for_training;
	const size_t n_img = tr.dataset.n_images;
	std::vector<float> g(n_img * 3);
	if (distributed()) allreduce_f32(m_exp_grad, n_img * 3, false);
	hk(hipMemcpyAsync(g.data(), m_exp_grad, g.size() * sizeof(float), hipMemcpyDeviceToHost, (hipStream_t)m_stream), "exposure gradient d2h");
	sync();
	const float per_camera_loss_scale = (float)n / 128.0f / (float)tr.n_steps_between_cam_updates;
	const float lr_base = current_learning_rate();
	float mean[3] = {0.f, 0.f, 0.f};
	for (uint32_t i = 0; i < n; ++i) {
		NerfTraining::Adam3& o = tr.cam_exposure[i];
		++o.iter;
		const float beta1 = 0.9f, beta2 = 0.99f, eps = 1e-8f;
		const float lr = lr_base * std::sqrt(1.0f - std::pow(beta2, (float)o.iter)) / (1.0f - std::pow(beta1, (float)o.iter));
		for (int k = 0; k < 3; ++k) {
			const float grad = g[3 * i + k] * per_camera_loss_scale + o.variable[k] * tr.exposure_l2_reg;
			o.m[k] = beta1 * o.m[k] + (1.0f - beta1) * grad;
			o.v[k] = beta2 * o.v[k] + (1.0f - beta2) * grad * grad;
			o.variable[k] -= lr * o.m[k] / (std::sqrt(o.v[k]) + eps);
			mean[k] += o.variable[k];
		}
	}
	std::vector<float> e(n_img * 3, 0.0f);
	for (uint32_t i = 0; i < n; ++i)
		for (int k = 0; k < 3; ++k) e[3 * i + k] = tr.cam_exposure[i].variable[k] -= mean[k] / (float)n;
	for (size_t i = n; i < n_img; ++i)
		for (int k = 0; k < 3; ++k) e[3 * i + k] = tr.cam_exposure[i].variable[k];
	hk(hipMemcpyAsync(m_exp, e.data(), e.size() * sizeof(float), hipMemcpyHostToDevice, (hipStream_t)m_stream), "exposure h2d");
}

// Distortion branch of the camera update (src/testbed_nerf.cu:2630-2637): gradients divided by
// their accumulated bilinear weights (safe_divide, :1548-1554), then one step of the map's
// ExponentialDecay(Adam) trainer at loss scale LOSS_SCALE * n_steps_between_cam_updates.  The map
// has no matrix parameters, so (as the network's hash grid) entries with a zero gradient are
// skipped and no L2 term applies; the step counts are per parameter.
void Testbed::update_distortion_map() {
	DistortionMap& d = m_distortion;
	const size_t n = d.params.size();
	if (distributed()) allreduce_f32(m_dist_grad, 2 * n, false);
	std::vector<float> g(2 * n);
	hk(hipMemcpyAsync(g.data(), m_dist_grad, g.size() * sizeof(float), hipMemcpyDeviceToHost, (hipStream_t)m_stream), "distortion gradient d2h");
	sync();
	const float lr = exp_decay_learning_rate(d.lr, d.decay_base, d.decay_start, d.decay_interval, d.decay_end, d.optimizer_step);
	++d.optimizer_step;
	const float loss_scale = 128.0f * (float)nerf.training.n_steps_between_cam_updates;
	for (size_t i = 0; i < n; ++i) {
		const float w = g[n + i];
		const float graw = w > 0.0f ? g[i] / w : 0.0f;
		if (graw == 0.0f) continue;
		const float gs = graw / loss_scale;
		d.m[i] = d.beta1 * d.m[i] + (1.0f - d.beta1) * gs;
		d.v[i] = d.beta2 * d.v[i] + (1.0f - d.beta2) * gs * gs;
		const uint32_t step = ++d.steps[i];
		const float lr_t = lr * std::sqrt(1.0f - std::pow(d.beta2, (float)step)) / (1.0f - std::pow(d.beta1, (float)step));
		d.params[i] = d.params[i] - (lr_t / (std::sqrt(d.v[i]) + d.eps)) * d.m[i];
	}
	hk(hipMemcpyAsync(m_dist, d.params.data(), n * sizeof(float), hipMemcpyHostToDevice, (hipStream_t)m_stream), "distortion h2d");
}

// Extrinsics branch of the camera update (src/testbed_nerf.cu:2605-2628): per-image Adam on the
// translation offset and rotation-Adam on the angle-axis offset (lr = max(extrinsic_lr *
// 0.33^(step / 128), network lr / 1000), L2 on the offsets), then the transforms are rebuilt.
void Testbed::update_cam_extrinsics() {
	NerfTraining& tr = nerf.training;
	const uint32_t n = (uint32_t)tr.n_images_for_training;
	const size_t n_img = tr.dataset.n_images;
	if (distributed()) allreduce_f32(m_cam_grad, n_img * 6, false);
	std::vector<float> g(n_img * 6);
	hk(hipMemcpyAsync(g.data(), m_cam_grad, g.size() * sizeof(float), hipMemcpyDeviceToHost, (hipStream_t)m_stream), "camera gradient d2h");
	sync();
	const float per_camera_loss_scale = (float)n / 128.0f / (float)tr.n_steps_between_cam_updates;
	const float lr_floor = current_learning_rate() / 1000.0f;
	const float beta1 = 0.9f, beta2 = 0.99f, eps = 1e-8f;
	for (uint32_t i = 0; i < n; ++i) {
		for (int kind = 0; kind < 2; ++kind) {
			NerfTraining::Adam3& o = kind == 0 ? tr.cam_pos_offset[i] : tr.cam_rot_offset[i];
			const float lr_set = std::max(tr.extrinsic_learning_rate * std::pow(0.33f, (float)(o.iter / 128)), lr_floor);
			++o.iter;
			const float lr = lr_set * std::sqrt(1.0f - std::pow(beta2, (float)o.iter)) / (1.0f - std::pow(beta1, (float)o.iter));
			vec3 step{};
			for (int k = 0; k < 3; ++k) {
				const float grad = g[(size_t)kind * 3 * n_img + 3 * i + k] * per_camera_loss_scale + o.variable[k] * tr.extrinsic_l2_reg;
				o.m[k] = beta1 * o.m[k] + (1.0f - beta1) * grad;
				o.v[k] = beta2 * o.v[k] + (1.0f - beta2) * grad * grad;
				step[k] = lr * o.m[k] / (std::sqrt(o.v[k]) + eps);
			}
			if (kind == 0) {
				for (int k = 0; k < 3; ++k) o.variable[k] -= step[k];
			} else {  // RotationAdamOptimizer::step: variable = rotvec(rotmat(-step) * rotmat(variable))
				o.variable = rotvec(matmul3(rotmat({-step[0], -step[1], -step[2]}), rotmat(o.variable)));
			}
		}
	}
	upload_metadata();  // update_transforms
}

// Focal-length branch (src/testbed_nerf.cu:2639-2648): Adam with lr max(1e-3 * 0.33^(step / 128),
// network lr / 1000) on the L2-regularised offset; the gradient term is zero (see testbed.h).
void Testbed::update_cam_focal_length() {
	NerfTraining::Adam2& o = nerf.training.cam_focal_length_offset;
	const float lr_set = std::max(1e-3f * std::pow(0.33f, (float)(o.iter / 128)), current_learning_rate() / 1000.0f);
	++o.iter;
	const float beta1 = 0.9f, beta2 = 0.99f, eps = 1e-8f;
	const float lr = lr_set * std::sqrt(1.0f - std::pow(beta2, (float)o.iter)) / (1.0f - std::pow(beta1, (float)o.iter));
	for (int k = 0; k < 2; ++k) {
		const float grad = o.variable[k] * nerf.training.intrinsic_l2_reg;
		o.m[k] = beta1 * o.m[k] + (1.0f - beta1) * grad;
		o.v[k] = beta2 * o.v[k] + (1.0f - beta2) * grad * grad;
		o.variable[k] -= lr * o.m[k] / (std::sqrt(o.v[k]) + eps);
	}
}

std::vector<float> Testbed::error_map_data() {
	const NerfTraining& tr = nerf.training;
	const size_t n = (size_t)tr.error_map.resolution[0] * tr.error_map.resolution[1] * tr.dataset.n_images;
	std::vector<float> h(m_err ? n : 0);
	if (!h.empty()) {
		hk(hipMemcpyAsync(h.data(), m_err, n * sizeof(float), hipMemcpyDeviceToHost, (hipStream_t)m_stream), "error map d2h");
		sync();
	}
	return h;
}

void Testbed::train(uint32_t batch_size) {
	if (!training_data_available) {
		shall_train = false;
		return;
	}
	if (mode == ETestbedMode::None) throw std::runtime_error("Cannot train without a mode.");
	if (!m_model) {
		reload_network_from_file();
		if (!m_model) throw std::runtime_error("Unable to create a neural network trainer.");
	}
	// Testbed::train (src/testbed.cu:4046-4053): per-image latents requested without a learnable code -> 16 dims
	if (nerf.training.optimize_extra_dims && nerf.training.dataset.n_extra_learnable_dims == 0) {
		nerf.training.dataset.n_extra_learnable_dims = 16;
		reset_network();
	}
	if (m_net_cfg.n_extra_dims != n_extra_dims()) reset_network();  // the network's input width follows the dataset
	reset_accumulation();
	// density-grid cadence (src/testbed.cu:4060) + training_prep_nerf (src/testbed_nerf.cu:2933-2946)
	const uint32_t n_prep_to_skip = std::min(std::max(training_step / 16u, 1u), 16u);
	if (training_step % n_prep_to_skip == 0) {
		const auto t0 = std::chrono::steady_clock::now();
		const uint32_t nc = nerf.max_cascade + 1;
		if (training_step < 256) update_density_grid(NERF_GRID_N_CELLS * nc, 0);
		else update_density_grid(NERF_GRID_N_CELLS / 4 * nc, NERF_GRID_N_CELLS / 4 * nc);
		sync();
		training_prep_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() / n_prep_to_skip;
	}
	const bool get_loss_scalar = training_step % 16 == 0;
	const auto t0 = std::chrono::steady_clock::now();
	train_nerf(batch_size, get_loss_scalar);
	sync();
	training_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

bool Testbed::frame() {
	if (shall_train) train(training_batch_size);
	return true;
}

// ---------------------------------------------------------------------------
// Rendering
// ---------------------------------------------------------------------------
void Testbed::reset_camera() {
	fov_axis = 1;
	zoom = 1.0f;
	screen_center = {0.5f, 0.5f};
	set_fov(50.625f);
	scale = 1.5f;
	// src/testbed.cu:504-511: rows (1,0,0,.5), (0,-1,0,.5), (0,0,-1,.5) transposed -> columns
	const float m[12] = {1, 0, 0, 0, -1, 0, 0, 0, -1, 0.5f, 0.5f, 0.5f};
	std::memcpy(camera.m, m, sizeof(m));
	// m_camera[3] -= m_scale * view_dir()
	for (int k = 0; k < 3; ++k) camera.m[9 + k] -= scale * camera.m[6 + k];
	m_spp = 0;
}

float Testbed::fov() const { return focal_length_to_fov(1.0f, relative_focal_length[fov_axis]); }
void Testbed::set_fov(float degrees) {
	const float f = fov_to_focal_length(1, degrees);
	relative_focal_length = {f, f};
}
vec2 Testbed::fov_xy() const {
	return {focal_length_to_fov(1.0f, relative_focal_length[0]), focal_length_to_fov(1.0f, relative_focal_length[1])};
}
void Testbed::set_fov_xy(const vec2& degrees) {
	relative_focal_length = {fov_to_focal_length(1, degrees[0]), fov_to_focal_length(1, degrees[1])};
}

// crop_box (src/testbed.cu:618-633): axes = the rows of render_aabb_to_local scaled by the half extents, centre
// = transpose(render_aabb_to_local) * the box centre (the box lives in the local frame)
Mat43 Testbed::crop_box(bool nerf_space) const {
	const mat3& R = render_aabb_to_local;  // row-major
	vec3 cen_local, radius;
	for (int k = 0; k < 3; ++k) {
		cen_local[k] = 0.5f * (render_aabb_min[k] + render_aabb_max[k]);
		radius[k] = 0.5f * (render_aabb_max[k] - render_aabb_min[k]);
	}
	Mat43 rv;
	for (int a = 0; a < 3; ++a)
		rv.set_col(a, {R[3 * a + 0] * radius[a], R[3 * a + 1] * radius[a], R[3 * a + 2] * radius[a]});
	vec3 cen;
	for (int j = 0; j < 3; ++j) cen[j] = R[0 * 3 + j] * cen_local[0] + R[1 * 3 + j] * cen_local[1] + R[2 * 3 + j] * cen_local[2];
	rv.set_col(3, cen);
	return nerf_space ? nerf.training.dataset.ngp_matrix_to_nerf(rv, true) : rv;
}

// set_crop_box (src/testbed.cu:635-649): the inverse -- rows of the frame = the normalised axes, box = centre
// (in the local frame) +- the axes' lengths
void Testbed::set_crop_box(Mat43 m, bool nerf_space) {
	if (nerf_space) {
		float r[12];  // row-major 3x4 of the NeRF-space matrix
		for (int row = 0; row < 3; ++row)
			for (int col = 0; col < 4; ++col) r[row * 4 + col] = m.m[3 * col + row];
		m = nerf.training.dataset.nerf_matrix_to_ngp(r, true);
	}
	vec3 radius;
	for (int a = 0; a < 3; ++a) {
		const vec3 c = m.col(a);
		radius[a] = std::sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
		if (!(radius[a] > 0.f)) throw std::runtime_error("set_crop_box: the box axes must be non-zero");
		for (int k = 0; k < 3; ++k) render_aabb_to_local[3 * a + k] = c[k] / radius[a];
	}
	const vec3 c3 = m.col(3);
	for (int a = 0; a < 3; ++a) {
		const float cl = render_aabb_to_local[3 * a + 0] * c3[0] + render_aabb_to_local[3 * a + 1] * c3[1] +
		                 render_aabb_to_local[3 * a + 2] * c3[2];
		render_aabb_min[a] = cl - radius[a];
		render_aabb_max[a] = cl + radius[a];
	}
	m_spp = 0;
}

// crop_box_corners (src/testbed.cu:651-670): the 8 corners m * (+-1, +-1, +-1, 1), x fastest
std::vector<vec3> Testbed::crop_box_corners(bool nerf_space) const {
	const Mat43 m = crop_box(nerf_space);
	std::vector<vec3> rv(8);
	for (int i = 0; i < 8; ++i) {
		const float sx = (i & 1) ? 1.f : -1.f, sy = (i & 2) ? 1.f : -1.f, sz = (i & 4) ? 1.f : -1.f;
		for (int k = 0; k < 3; ++k) rv[i][k] = m.m[k] * sx + m.m[3 + k] * sy + m.m[6 + k] * sz + m.m[9 + k];
	}
	return rv;
}

float Testbed::compute_image_mse(bool) const {
	// the Image mode's image is empty in a NeRF testbed: reduce_sum over 0 elements / 0 (src/testbed_image.cu:517)
	return std::numeric_limits<float>::quiet_NaN();
}

int Nerf::find_closest_training_view(const Mat43& pose, const std::function<Mat43(size_t)>& transform) const {
	int best = training.view;
	float best_score = std::numeric_limits<float>::infinity();
	auto dist = [](const vec3& a, const vec3& b) {
		const float x = a[0] - b[0], y = a[1] - b[1], z = a[2] - b[2];
		return std::sqrt(x * x + y * y + z * z);
	};
	for (int i = 0; i < training.n_images_for_training; ++i) {
		const Mat43 t = transform((size_t)i);
		float score = dist(t.col(3), pose.col(3));
		score += 0.25f * dist(t.col(2), pose.col(2));
		if (score < best_score) {
			best_score = score;
			best = i;
		}
	}
	return best;
}

void Testbed::set_rendering_extra_dims_from_training_view(int trainview) {
	if (!n_extra_dims()) throw std::runtime_error("Dataset does not have extra dims.");
	if (trainview < 0 || (size_t)trainview >= nerf.training.dataset.n_images) throw std::runtime_error("Invalid training view.");
	rendering_extra_dims_from_training_view = trainview;
}

void Testbed::set_rendering_extra_dims(const std::vector<float>& vals) {
	if (vals.size() != n_extra_dims())
		throw std::runtime_error("Invalid number of extra dims. Got " + std::to_string(vals.size()) + " but must be " +
		                         std::to_string(n_extra_dims()) + ".");
	rendering_extra_dims_from_training_view = -1;
	m_rendering_extra_dims = vals;
}

// Nerf::get_rendering_extra_dims_cpu: the code set with set_rendering_extra_dims (the training view's code when
// rendering_extra_dims_from_training_view selects one is what the renderer uses, not this buffer)
// Nerf::get_rendering_extra_dims_cpu (src/testbed_nerf.cu:3269-3280): the code rendered rays carry -- the trained code of
// rendering_extra_dims_from_training_view when it names a view (the default 0), the set one otherwise -- with the warped
// light direction in the first three entries for datasets with light dirs (get_rendering_extra_dims, :3206-3228)
std::vector<float> Testbed::rendering_extra_dims() const {
	const NerfTraining& tr = nerf.training;
	const uint32_t E = tr.dataset.n_extra_dims();
	if (!E) return {};
	std::vector<float> row(E, 0.0f);
	const int v = rendering_extra_dims_from_training_view;
	const std::vector<float>& src = v >= 0 && (size_t)v < tr.extra_dims_opt.size() ? tr.extra_dims_opt[v].variable : m_rendering_extra_dims;
	for (uint32_t j = 0; j < E && j < src.size(); ++j) row[j] = src[j];
	if (tr.dataset.has_light_dirs) {
		const vec3 ld = nerf.light_dir;
		const float l = std::sqrt(ld[0] * ld[0] + ld[1] * ld[1] + ld[2] * ld[2]);
		for (uint32_t j = 0; j < 3 && j < E; ++j) row[j] = l > 0.f ? (ld[j] / l + 1.0f) * 0.5f : 0.5f;
	}
	return row;
}

std::vector<float> Testbed::training_extra_dims(int trainview) const {
	if (n_extra_dims() == 0) return {};  // Nerf::Training::get_extra_dims_cpu (src/testbed_nerf.cu:1797-1812)
	if (trainview < 0 || (size_t)trainview >= nerf.training.dataset.n_images) throw std::runtime_error("Invalid training view.");
	if ((size_t)trainview >= nerf.training.extra_dims_opt.size()) return std::vector<float>(n_extra_dims(), 0.0f);
	return nerf.training.extra_dims_opt[trainview].variable;
}

// VarAdamOptimizer::step (adam_optimizer.h:41-51)
void NerfTraining::VarAdam::step(const std::vector<float>& g) {
	++iter;
	const float lr = learning_rate * std::sqrt(1.0f - std::pow(beta2, (float)iter)) / (1.0f - std::pow(beta1, (float)iter));
	for (size_t i = 0; i < m.size(); ++i) {
		m[i] = beta1 * m[i] + (1.0f - beta1) * g[i];
		v[i] = beta2 * v[i] + (1.0f - beta2) * g[i] * g[i];
		variable[i] -= lr * m[i] / (std::sqrt(v[i]) + epsilon);
	}
}

// Nerf::reset_extra_dims (src/testbed_nerf.cu:3181-3204): per image a fresh VarAdamOptimizer(n_extra_dims, 1e-4) whose
// variable starts at the frame's light direction (first 3, datasets with light dirs) and uniform [-1, 1) values
// (random_val(rng) * 2 - 1) after it; the rendered code starts as image 0's
void Testbed::reset_extra_dims(pcg32* rng) {
	NerfTraining& tr = nerf.training;
	const uint32_t E = tr.dataset.n_extra_dims();
	tr.extra_dims_opt.clear();
	m_rendering_extra_dims.assign(E, 0.0f);
	if (!E) return;
	if (E > NGP_EXTRA_DIMS_MAX) throw std::runtime_error("n_extra_dims > 32 is not supported (light directions + latent code)");
	const size_t n = tr.dataset.n_images;
	tr.extra_dims_opt.resize(n);
	for (size_t i = 0; i < n; ++i) {
		NerfTraining::VarAdam& o = tr.extra_dims_opt[i];
		o.variable.assign(E, 0.0f);
		o.m.assign(E, 0.0f);
		o.v.assign(E, 0.0f);
		for (uint32_t j = 0; j < E; ++j) {
			if (tr.dataset.has_light_dirs && j < 3 && i < tr.dataset.metadata.size()) {
				const vec3 ld = tr.dataset.metadata[i].light_dir;
				const float l = std::sqrt(ld[0] * ld[0] + ld[1] * ld[1] + ld[2] * ld[2]);
				o.variable[j] = l > 0.f ? (ld[j] / l + 1.0f) * 0.5f : 0.5f;  // warp_direction(normalize(light_dir))
			} else {
				o.variable[j] = rng->next_float() * 2.0f - 1.0f;
			}
		}
	}
	if (n) m_rendering_extra_dims = tr.extra_dims_opt[0].variable;
	upload_extra_dims();
}

// Nerf::Training::update_extra_dims (src/testbed_nerf.cu:1814-1825): the codes into the device table, rows of NGP_EXTRA_ROW
void Testbed::upload_extra_dims() {
	const NerfTraining& tr = nerf.training;
	const uint32_t E = tr.dataset.n_extra_dims();
	if (!E) return;
	const size_t rows = std::max(tr.dataset.n_images, tr.extra_dims_opt.size()) + 1;  // + the rendered code's row
	if (m_extra_rows != rows) {
		sync();
		for (float* p : {m_extra, m_extra_grad})
			if (p) (void)hipFree(p);
		m_extra = m_extra_grad = nullptr;
		hk(hipMalloc((void**)&m_extra, rows * NGP_EXTRA_ROW * sizeof(float)), "hipMalloc extra dims");
		hk(hipMalloc((void**)&m_extra_grad, rows * NGP_EXTRA_ROW * sizeof(float)), "hipMalloc extra dims gradient");
		hk(hipMemset(m_extra, 0, rows * NGP_EXTRA_ROW * sizeof(float)), "hipMemset extra dims");
		m_extra_rows = rows;
	}
	m_extra_host.assign(rows * NGP_EXTRA_ROW, 0.0f);
	for (size_t i = 0; i < tr.extra_dims_opt.size(); ++i)
		for (uint32_t j = 0; j < E; ++j) m_extra_host[NGP_EXTRA_ROW * i + j] = tr.extra_dims_opt[i].variable[j];
	hk(hipMemcpy(m_extra, m_extra_host.data(), (rows - 1) * NGP_EXTRA_ROW * sizeof(float), hipMemcpyHostToDevice), "upload extra dims");
}

// Nerf::get_rendering_extra_dims (src/testbed_nerf.cu:3206-3228): a training view's code or the set one, with the
// light direction first for datasets with light dirs -- written into the table's spare last row
const float* Testbed::rendering_extra_dims_device() {
	const NerfTraining& tr = nerf.training;
	const uint32_t E = tr.dataset.n_extra_dims();
	if (!E) return nullptr;
	if (!m_extra) upload_extra_dims();
	const std::vector<float> row = rendering_extra_dims();
	// staged in a page-locked row of its own: the copy is still in flight when this returns, and render() synchronises
	// the stream before the next call writes the row again
	if (!m_extra_stage) m_extra_stage = static_cast<float*>(pinned_host_alloc(NGP_EXTRA_ROW * sizeof(float)));
	std::fill(m_extra_stage, m_extra_stage + NGP_EXTRA_ROW, 0.0f);
	std::copy(row.begin(), row.end(), m_extra_stage);
	const size_t n = m_extra_rows - 1;
	hk(hipMemcpyAsync(m_extra + NGP_EXTRA_ROW * n, m_extra_stage, NGP_EXTRA_ROW * sizeof(float), hipMemcpyHostToDevice,
	                  (hipStream_t)m_stream),
	   "upload rendering extra dims");
	return m_extra + NGP_EXTRA_ROW * n;
}

// train_nerf's latent-code step (src/testbed_nerf.cu:2580-2599): the codes' gradient (loss-scaled sums over the
// kept rays' samples) to the host, / LOSS_SCALE, one VarAdam step per training image at the network's current
// learning rate, then the codes back to the device
void Testbed::update_extra_dims_step() {
	NerfTraining& tr = nerf.training;
	const uint32_t E = tr.dataset.n_extra_dims();
	const size_t n = m_extra_rows - 1;
	std::vector<float> g(n * NGP_EXTRA_ROW);
	hk(hipMemcpyAsync(g.data(), m_extra_grad, n * NGP_EXTRA_ROW * sizeof(float), hipMemcpyDeviceToHost, (hipStream_t)m_stream),
	   "extra dims gradient d2h");
	sync();
	const float lr = current_learning_rate();
	for (int i = 0; i < tr.n_images_for_training && (size_t)i < tr.extra_dims_opt.size(); ++i) {
		std::vector<float> gi(E);
		for (uint32_t j = 0; j < E; ++j) gi[j] = g[NGP_EXTRA_ROW * (size_t)i + j] / 128.0f;
		tr.extra_dims_opt[i].learning_rate = lr;
		tr.extra_dims_opt[i].step(gi);
	}
	upload_extra_dims();
}

int Testbed::find_closest_training_view() const {
	return nerf.find_closest_training_view(camera, [this](size_t i) { return training_transform(i); });
}

void Testbed::set_camera_to_training_view(int trainview) {
	const NerfDataset& ds = nerf.training.dataset;
	if (trainview < 0 || (size_t)trainview >= ds.n_images) throw std::runtime_error("Invalid training view.");
	// m_scale keeps the old look-at point in front of the new view (src/testbed.cu:471-475)
	const vec3 old_pos = camera.col(3), old_dir = camera.col(2);
	const vec3 look_at = {old_pos[0] + old_dir[0] * scale, old_pos[1] + old_dir[1] * scale, old_pos[2] + old_dir[2] * scale};
	camera = ds.xforms[trainview];
	{
		const vec3 p = camera.col(3), d = camera.col(2);
		scale = std::max((look_at[0] - p[0]) * d[0] + (look_at[1] - p[1]) * d[1] + (look_at[2] - p[2]) * d[2], 0.1f);
	}
	const auto& md = ds.metadata[trainview];
	relative_focal_length = {md.focal_length[0] / (float)md.resolution[fov_axis], md.focal_length[1] / (float)md.resolution[fov_axis]};
	nerf.render_with_lens_distortion = true;
	nerf.render_lens = md.lens;  // src/testbed.cu:477-478
	screen_center = {1.0f - md.principal_point[0], 1.0f - md.principal_point[1]};
	nerf.training.view = trainview;
	if (n_extra_dims()) set_rendering_extra_dims_from_training_view(trainview);  // src/testbed.cu:2207-2209
	m_spp = 0;
}

void Testbed::ensure_render_buffers(size_t n) {
	if (n <= m_render_cap) return;
	for (float** p : {&m_frame, &m_accum, &m_out}) {
		if (*p) (void)hipFree(*p);
		hk(hipMalloc((void**)p, n * 4 * sizeof(float)), "hipMalloc frame");
	}
	if (m_depth) (void)hipFree(m_depth);
	hk(hipMalloc((void**)&m_depth, n * sizeof(float)), "hipMalloc depth");
	m_render_cap = n;
}

static std::mutex g_pinned_mu;
static std::multimap<size_t, void*> g_pinned_free;

void* pinned_host_alloc(size_t bytes) {
	{
		std::lock_guard<std::mutex> lock(g_pinned_mu);
		auto it = g_pinned_free.find(bytes);
		if (it != g_pinned_free.end()) {
			void* p = it->second;
			g_pinned_free.erase(it);
			return p;
		}
	}
	void* p = nullptr;
	hk(hipHostMalloc(&p, std::max<size_t>(bytes, 1), hipHostMallocDefault), "hipHostMalloc frame");
	return p;
}

void pinned_host_release(void* p, size_t bytes) {
	if (!p) return;
	std::lock_guard<std::mutex> lock(g_pinned_mu);
	if (g_pinned_free.count(bytes) < 4) {  // keep a few per size (frames of the same resolution)
		g_pinned_free.emplace(bytes, p);
		return;
	}
	(void)hipHostFree(p);
}

std::vector<float> Testbed::render(int width, int height, int spp, bool linear, uint32_t shard_index,
                                   uint32_t shard_count, uint32_t shard_rows, bool copy_to_host) {
	if (width <= 0 || height <= 0) throw std::runtime_error("render: invalid resolution");
	std::vector<float> out(copy_to_host ? (size_t)width * height * 4 : 0, 0.0f);
	render_into(copy_to_host ? out.data() : nullptr, width, height, spp, linear, shard_index, shard_count, shard_rows);
	return out;
}

void Testbed::render_into(float* host_dst, int width, int height, int spp, bool linear, uint32_t shard_index,
                          uint32_t shard_count, uint32_t shard_rows, bool host_dst_pinned) {
	if (width <= 0 || height <= 0) throw std::runtime_error("render: invalid resolution");
	const size_t n = (size_t)width * height;
	const vec2 sc = {(0.5f - screen_center[0]) * zoom + 0.5f, (0.5f - screen_center[1]) * zoom + 0.5f};
	const int res_axis = fov_axis == 0 ? width : height;
	const vec2 focal = {relative_focal_length[0] * (float)res_axis * zoom, relative_focal_length[1] * (float)res_axis * zoom};

	if (render_ground_truth && nerf.training.dataset.n_images > 0) {
		std::vector<float> out(n * 4, 0.0f);
		// overlay_image_kernel with ground-truth alpha 1 (src/render_buffer.cu:348-416), then tonemap to linear/sRGB
		const NerfDataset& ds = nerf.training.dataset;
		const int v = std::min(std::max(nerf.training.view, 0), (int)ds.n_images - 1);
		const auto& px = ds.pixels[v];
		const int iw = ds.metadata[v].resolution[0], ih = ds.metadata[v].resolution[1];
		const float sca = (float)(fov_axis == 0 ? iw : ih) / (float)res_axis;
		vec4 bg = background_color;
		if (color_space != EColorSpace::SRGB)
			for (int k = 0; k < 3; ++k) bg[k] = srgb_to_linear_h(bg[k]);
		for (int y = 0; y < height; ++y)
			for (int x = 0; x < width; ++x) {
				// the reference overlays the image about the frame centre, vec2(0.5) -- not the camera's
				// screen centre (src/testbed.cu:4597-4608, render_buffer.cu:373-380)
				float fx = x + 0.5f, fy = y + 0.5f;
				fx -= width * 0.5f; fx /= zoom; fx += 0.5f * width;
				fy -= height * 0.5f; fy /= zoom; fy += 0.5f * height;
				const float u = (fx - width * 0.5f) * sca + iw * 0.5f, vv = (fy - height * 0.5f) * sca + ih * 0.5f;
				const int sx = (int)std::floor(u), sy = (int)std::floor(vv);
				float c[4] = {0, 0, 0, 0};
				if (!px.empty() && sx >= 0 && sy >= 0 && sx < iw && sy < ih) {
					const uint8_t* p = &px[((size_t)sy * iw + sx) * 4];
					const float a = p[3] / 255.f;
					for (int k = 0; k < 3; ++k) c[k] = srgb_to_linear_h(p[k] / 255.f) * a;
					c[3] = a;
				}
				if (color_space == EColorSpace::SRGB) {
					for (int k = 0; k < 3; ++k) c[k] = c[3] > 0 ? linear_to_srgb_h(c[k] / c[3]) * c[3] : 0.f;
				}
				const float w = (1 - c[3]) * bg[3];
				for (int k = 0; k < 3; ++k) c[k] += bg[k] * w;
				c[3] += w;
				if (color_space == EColorSpace::SRGB)
					for (int k = 0; k < 3; ++k) c[k] = srgb_to_linear_h(c[k]);
				for (int k = 0; k < 3; ++k) {
					// exposure + the view's optimised exposure (src/testbed.cu:4599)
					const float ev = (size_t)v < nerf.training.cam_exposure.size() ? nerf.training.cam_exposure[v].variable[k] : 0.0f;
					c[k] *= std::pow(2.0f, exposure + ev);
					if (!linear) c[k] = linear_to_srgb_h(c[k]);
				}
				std::memcpy(&out[((size_t)y * width + x) * 4], c, sizeof(c));
			}
		if (host_dst) std::memcpy(host_dst, out.data(), out.size() * sizeof(float));
		return;
	}
	if (!m_model) throw std::runtime_error("render: no network (load training data or a snapshot first)");
	const auto t0 = std::chrono::steady_clock::now();
	ensure_render_buffers(n);
	ngp_render_args r{};
	r.width = (uint32_t)width;
	r.height = (uint32_t)height;
	std::memcpy(r.camera, camera.m, sizeof(r.camera));
	r.focal_length[0] = focal[0];
	r.focal_length[1] = focal[1];
	r.screen_center[0] = sc[0];
	r.screen_center[1] = sc[1];
	r.near_distance = render_near_distance;
	for (int k = 0; k < 3; ++k) {
		r.aabb_min[k] = render_aabb_min[k];
		r.aabb_max[k] = render_aabb_max[k];
		r.train_aabb_min[k] = aabb_min[k];
		r.train_aabb_max[k] = aabb_max[k];
	}
	for (int k = 0; k < 9; ++k) r.render_aabb_to_local[k] = render_aabb_to_local[k];
	switch (render_mode) {
		case ERenderMode::AO: r.render_mode = NGP_RENDER_MODE_AO; break;
		case ERenderMode::Shade: r.render_mode = NGP_RENDER_MODE_SHADE; break;
		case ERenderMode::Normals: r.render_mode = NGP_RENDER_MODE_NORMALS; break;
		case ERenderMode::Positions: r.render_mode = NGP_RENDER_MODE_POSITIONS; break;
		case ERenderMode::Depth: r.render_mode = NGP_RENDER_MODE_DEPTH; break;
		case ERenderMode::Cost: r.render_mode = NGP_RENDER_MODE_COST; break;
		case ERenderMode::Slice: r.render_mode = NGP_RENDER_MODE_SLICE; break;
		default: throw std::runtime_error("render: render mode Distortion is a GUI visualisation and not supported by this build");
	}
	r.depth_scale = 1.0f / nerf.training.dataset.scale;  // src/testbed_nerf.cu:1905
	r.glow_mode = nerf.glow_mode;
	r.glow_y_cutoff = nerf.glow_y_cutoff;
	r.extra_dims = rendering_extra_dims_device();  // NerfTracer's extra_dims_gpu (src/testbed_nerf.cu:1848, 1922)
	r.gbuffer_hard_edges = nerf.render_gbuffer_hard_edges;
	// plane_z = m_slice_plane_z + m_scale (src/testbed_nerf.cu:1842): the Slice plane, or the focus plane of the
	// depth of field (init_rays_with_payload_kernel_nerf drops the aperture when plane_z < 0, :1427-1429)
	const float plane_z = slice_plane_z + scale;
	r.focus_z = plane_z;
	r.aperture_size = plane_z < 0.0f ? 0.0f : aperture_size;
	r.cone_angle_constant = nerf.cone_angle_constant;
	r.max_cascade = nerf.max_cascade;
	r.min_transmittance = nerf.render_min_transmittance;
	r.snap_to_pixel_centers = snap_to_pixel_centers;
	r.use_inference_params = 1;
	r.train_in_linear_colors = nerf.training.linear_colors;
	r.shard_index = shard_index;
	r.shard_count = std::max(shard_count, 1u);
	r.shard_rows = std::max(shard_rows, 1u);
	if (nerf.render_with_lens_distortion) {
		r.lens_mode = (int32_t)nerf.render_lens.mode;
		std::memcpy(r.lens_params, nerf.render_lens.params, sizeof(r.lens_params));
		if (m_distortion.active) {  // m_distortion.inference_view() (src/testbed_nerf.cu:1854-1857)
			r.distortion_map = m_dist;
			r.distortion_res[0] = (uint32_t)m_distortion.rx;
			r.distortion_res[1] = (uint32_t)m_distortion.ry;
		}
	}
	const float bg[4] = {background_color[0], background_color[1], background_color[2], background_color[3]};
	// one spp of a whole Shade-mode frame into host memory: the kernels that finish the rays stream their tonemapped
	// pixels to host_dst while the march goes on (ngp_render_args.host_frame), so no read-back follows the frame
	// (ngp_tuning.render_host_frame 2: tonemap, then copy).  The device frame and m_out are produced as before.
	// Only a page-locked, device-mapped destination can be written by the kernels (render() and
	// render_shard() hand in a pageable std::vector, which takes the read-back).
	int32_t host_complete = 0;
	const bool stream_pixels = host_dst && host_dst_pinned && std::max(spp, 1) == 1 && r.shard_count == 1 && r.render_mode == NGP_RENDER_MODE_SHADE &&
	                           r.glow_mode == 0 && m_tuning.render_host_frame != 2;
	if (stream_pixels) {
		r.host_frame = host_dst;
		r.host_frame_complete = &host_complete;
		for (int k = 0; k < 4; ++k) r.host_background[k] = bg[k];
		r.host_exposure = exposure;
		r.host_color_space = (int32_t)color_space;
		r.host_output_srgb = linear ? 0 : 1;
	}
	m_spp = 0;
	for (int i = 0; i < std::max(spp, 1); ++i) {
		r.sample_index = (uint32_t)i;
		ck(ngp_render(m_model, &r, m_frame, m_depth, m_stream));
		const bool last = i == std::max(spp, 1) - 1;
		ck(ngp_accumulate_tonemap(m_frame, m_accum, last ? m_out : nullptr, r.width, r.height, m_spp,
		                          (int)color_space, exposure, bg, linear ? 0 : 1, m_stream));
		++m_spp;
	}
	if (host_dst && !(stream_pixels && host_complete))
		hk(hipMemcpyAsync(host_dst, m_out, n * 4 * sizeof(float), hipMemcpyDeviceToHost, (hipStream_t)m_stream), "render d2h");
	sync();
	render_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

std::vector<float> Testbed::density_grid() const {
	std::vector<float> g((size_t)NERF_GRID_N_CELLS * (nerf.max_cascade + 1));
	if (!m_model) return g;
	float* dg = nullptr;
	ck(ngp_density_grid_buffers(m_model, &dg, nullptr, nullptr, nullptr));
	sync();
	hk(hipMemcpy(g.data(), dg, g.size() * 4, hipMemcpyDeviceToHost), "grid d2h");
	return g;
}

std::vector<uint8_t> Testbed::density_grid_bitfield() const {
	std::vector<uint8_t> b(NERF_GRID_N_CELLS / 8 * NERF_CASCADES);
	if (!m_model) return b;
	uint8_t* db = nullptr;
	ck(ngp_density_grid_buffers(m_model, nullptr, &db, nullptr, nullptr));
	sync();
	hk(hipMemcpy(b.data(), db, b.size(), hipMemcpyDeviceToHost), "bitfield d2h");
	return b;
}

// ---------------------------------------------------------------------------
// Snapshots (Testbed::save_snapshot / load_snapshot, src/testbed.cu:4772-4978): the network
// config with a "snapshot" object, as MessagePack; zlib-compressed for ".ingp".  Keys the
// reference reads are written in its layout (tcnn Trainer::serialize: n_params,
// params_type "__half", params_binary = inference params; density_grid_binary fp16;
// nerf.aabb_scale / rgb counters; training_step, loss, camera ...).  The exact fp32
// master / EMA weights and the Adam state ride along under "mi355x" so a resumed run
// continues bit for bit; a reader that does not know the key ignores it.
// ---------------------------------------------------------------------------
static const uint32_t SNAPSHOT_FORMAT_VERSION = 1;

static std::vector<uint8_t> device_bytes(const void* p, size_t bytes) {
	std::vector<uint8_t> h(bytes);
	hk(hipMemcpy(h.data(), p, bytes, hipMemcpyDeviceToHost), "snapshot d2h");
	return h;
}

static std::vector<uint8_t> zlib_inflate(const std::vector<uint8_t>& in) {
	z_stream zs{};
	if (inflateInit(&zs) != Z_OK) throw std::runtime_error("zlib inflateInit failed");
	std::vector<uint8_t> out;
	std::vector<uint8_t> buf(1 << 20);
	zs.next_in = const_cast<Bytef*>(in.data());
	zs.avail_in = (uInt)in.size();
	int rc = Z_OK;
	while (rc != Z_STREAM_END) {
		zs.next_out = buf.data();
		zs.avail_out = (uInt)buf.size();
		rc = inflate(&zs, Z_NO_FLUSH);
		if (rc != Z_OK && rc != Z_STREAM_END) {
			inflateEnd(&zs);
			throw std::runtime_error("snapshot decompression failed");
		}
		out.insert(out.end(), buf.data(), buf.data() + (buf.size() - zs.avail_out));
		if (rc == Z_OK && zs.avail_in == 0 && zs.avail_out != 0) break;
	}
	inflateEnd(&zs);
	return out;
}

static Json vec_json(const float* v, int n) {
	Json a = Json::array();
	for (int k = 0; k < n; ++k) a.push_back(Json((double)v[k]));
	return a;
}

std::array<int, 3> marching_cubes_res(int res_1d, const vec3& box_min, const vec3& box_max) {
	const vec3 d = {box_max[0] - box_min[0], box_max[1] - box_min[1], box_max[2] - box_min[2]};
	const float scale = (float)res_1d / std::max(d[0], std::max(d[1], d[2]));
	std::array<int, 3> r;
	for (int k = 0; k < 3; ++k) {
		const unsigned v = (unsigned)(int)(d[k] * scale + 0.5f);  // ivec3(vec3) truncates
		r[k] = (int)((v + 15u) / 16u * 16u);                        // next_multiple(v, 16u)
	}
	return r;
}

std::vector<uint8_t> density_slices_mosaic(const std::vector<float>& density, std::array<int, 3> res3d, float thresh,
                                           bool swap_y_z, float density_range, int* width, int* height,
                                           uint32_t* zero_x_voxels, uint32_t* near_zero_lattice) {
	const int RX = res3d[0], RY = res3d[1], RZ = res3d[2];
	if ((size_t)RX * RY * RZ != density.size()) throw std::runtime_error("density_slices_mosaic: grid size mismatch");
	const float density_scale = 128.f / density_range;
	auto at = [&](int x, int y, int z) { return density[(size_t)x + (size_t)y * RX + (size_t)z * RX * RY]; };
	// the log line's statistics (marching_cubes.cu:965-996): voxels whose 8 corners straddle thresh, and interior
	// lattice points with a 6-neighbour on the other side
	uint32_t nv = 0, nz = 0;
	for (int z = 1; z < RZ - 1; ++z)
		for (int y = 1; y < RY - 1; ++y)
			for (int x = 1; x < RX - 1; ++x) {
				int count = 0;
				for (int k = 0; k < 8; ++k) count += at(x + (k & 1), y + ((k >> 1) & 1), z + (k >> 2)) < thresh;
				if (count > 0 && count < 8) ++nv;
				const bool s0 = at(x, y, z) < thresh;
				bool c = (at(x + 1, y, z) < thresh) != s0;
				c |= (at(x - 1, y, z) < thresh) != s0;
				c |= (at(x, y + 1, z) < thresh) != s0;
				c |= (at(x, y - 1, z) < thresh) != s0;
				c |= (at(x, y, z + 1) < thresh) != s0;
				c |= (at(x, y, z - 1) < thresh) != s0;
				if (c) ++nz;
			}
	if (zero_x_voxels) *zero_x_voxels = nv;
	if (near_zero_lattice) *near_zero_lattice = nz;
	int rx = RX, ry = RY, rz = RZ;
	if (swap_y_z) std::swap(ry, rz);
	const uint32_t ndown = (uint32_t)std::sqrt((float)rz);
	const uint32_t nacross = ((uint32_t)rz + ndown - 1) / ndown;
	const uint32_t w = (uint32_t)rx * nacross, h = (uint32_t)ry * ndown;
	std::vector<uint8_t> px((size_t)w * h);
	uint8_t* dst = px.data();
	for (uint32_t v = 0; v < h; ++v)
		for (uint32_t u = 0; u < w; ++u) {
			const int x = (int)(u % (uint32_t)rx), y = (int)(v % (uint32_t)ry);
			const int z = (int)(u / (uint32_t)rx + (v / (uint32_t)ry) * nacross);
			if (z < rz) {
				// swapped: the grid's (x, y, z) is the image's (x, z, y), unflipped; otherwise y is flipped
				const float d = swap_y_z ? density[(size_t)x + (size_t)z * rx + (size_t)y * rx * rz]
				                         : at(x, ry - 1 - y, z);
				*dst++ = (uint8_t)std::min(std::max((d - thresh) * density_scale + 128.5f, 0.f), 255.f);
			} else {
				*dst++ = 0;
			}
		}
	*width = (int)w;
	*height = (int)h;
	return px;
}

std::vector<float> Testbed::density_on_grid(const std::array<int, 3>& res3d, const vec3& box_min, const vec3& box_max,
                                            const mat3& box_to_local) const {
	if (!m_model) throw std::runtime_error("density_on_grid: no network (load a dataset or a snapshot first)");
	for (int k = 0; k < 3; ++k)
		if (res3d[k] <= 0) throw std::runtime_error("density_on_grid: the resolution must be positive");
	ngp_grid_query q{};
	for (int k = 0; k < 3; ++k) {
		q.res[k] = (uint32_t)res3d[k];
		q.box_min[k] = box_min[k];
		q.box_max[k] = box_max[k];
		q.aabb_min[k] = aabb_min[k];
		q.aabb_max[k] = aabb_max[k];
	}
	std::memcpy(q.box_to_local, box_to_local.data(), sizeof(q.box_to_local));
	q.max_cascade = nerf.max_cascade;
	q.mask_with_grid = mode == ETestbedMode::Nerf ? 1 : 0;
	q.use_inference_params = 1;
	const size_t n = (size_t)res3d[0] * res3d[1] * res3d[2];
	std::vector<float> out(n);
	float* dev = nullptr;
	hk(hipMalloc(&dev, n * sizeof(float)), "density_on_grid alloc");
	try {
		ck(ngp_density_on_grid(m_model, &q, dev, m_stream));
		sync();
		hk(hipMemcpy(out.data(), dev, n * sizeof(float), hipMemcpyDeviceToHost), "density_on_grid d2h");
	} catch (...) {
		(void)hipFree(dev);
		throw;
	}
	(void)hipFree(dev);
	return out;
}

std::array<int, 3> Testbed::compute_and_save_png_slices(const std::string& filename, int res, vec3 box_min, vec3 box_max,
                                                        float thresh, float density_range, bool flip_y_and_z_axes) {
	mat3 to_local = MAT3_IDENTITY;
	const bool empty = box_max[0] < box_min[0] || box_max[1] < box_min[1] || box_max[2] < box_min[2];
	if (empty) {
		box_min = render_aabb_min;
		box_max = render_aabb_max;
		to_local = render_aabb_to_local;
	}
	if (thresh == std::numeric_limits<float>::max()) thresh = mesh_thresh;
	if (res <= 0) throw std::runtime_error("compute_and_save_png_slices: the resolution must be positive");
	const std::array<int, 3> res3d = marching_cubes_res(res, box_min, box_max);
	const std::vector<float> density = density_on_grid(res3d, box_min, box_max, to_local);
	int w = 0, h = 0;
	uint32_t nv = 0, nz = 0;
	const std::vector<uint8_t> px =
	    density_slices_mosaic(density, res3d, thresh, flip_y_and_z_axes, density_range, &w, &h, &nv, &nz);
	const std::string path = filename + ".density_slices_" + std::to_string(res3d[0]) + "x" + std::to_string(res3d[1]) + "x" +
	                         std::to_string(res3d[2]) + ".png";
	std::string err;
	if (!encode_png_file(path, px.data(), w, h, 1, err)) throw std::runtime_error(err);
	const double N = (double)res3d[0] * res3d[1] * res3d[2];
	std::fprintf(stderr, "Wrote density PNG to %s\n  #lattice points=%.0f #zero-x voxels=%u (%g%%) #lattice near zero-x=%u (%g%%)\n",
	             path.c_str(), N, nv, nv * 100.0 / N, nz, nz * 100.0 / N);
	return res3d;
}

void Testbed::save_snapshot(const std::string& path, bool include_optimizer_state, bool compress) {
	if (!m_model) throw std::runtime_error("save_snapshot: no network");
	sync();
	ngp_model_info info{};
	ck(ngp_model_get_info(m_model, &info));
	auto buf = [&](int kind) {
		void* p = nullptr;
		size_t bytes = 0;
		ck(ngp_model_buffer(m_model, kind, &p, &bytes));
		return device_bytes(p, bytes);
	};
	Json root = m_network_config;
	Json snap = Json::object();
	snap["n_params"] = Json((double)info.n_params);
	snap["params_type"] = Json("__half");
	snap["params_binary"] = Json::binary(buf(NGP_PARAMS_INFER_FP16));
	Json exact = Json::object();
	exact["params_fp32_binary"] = Json::binary(buf(NGP_PARAMS_FP32));
	exact["params_ema_fp32_binary"] = Json::binary(buf(NGP_PARAMS_EMA_FP32));
	exact["n_mlp_params"] = Json((double)info.n_mlp_params);
	if (include_optimizer_state) {
		exact["adam_m_binary"] = Json::binary(buf(NGP_ADAM_M));
		exact["adam_v_binary"] = Json::binary(buf(NGP_ADAM_V));
	}
	snap["mi355x"] = exact;
	snap["version"] = Json((double)SNAPSHOT_FORMAT_VERSION);
	snap["mode"] = Json("Nerf");
	snap["density_grid_size"] = Json((double)NERF_GRIDSIZE);
	{
		const std::vector<float> grid = density_grid();
		std::vector<uint8_t> g16(grid.size() * 2);
		for (size_t k = 0; k < grid.size(); ++k) {
			const uint16_t h = f32_to_f16(grid[k]);
			std::memcpy(&g16[2 * k], &h, 2);
		}
		snap["density_grid_binary"] = Json::binary(std::move(g16));
		// the exact fp32 grid: the reference re-derives the bitfield from the fp16 copy, which can
		// flip cells sitting on the threshold; resuming from this one reproduces renders bit for bit
		std::vector<uint8_t> g32(grid.size() * 4);
		std::memcpy(g32.data(), grid.data(), g32.size());
		snap["mi355x"]["density_grid_fp32_binary"] = Json::binary(std::move(g32));
	}
	Json nj = Json::object();
	nj["aabb_scale"] = Json((double)nerf.training.dataset.aabb_scale);
	Json rgb = Json::object();
	rgb["rays_per_batch"] = Json((double)nerf.training.counters_rgb.rays_per_batch);
	rgb["measured_batch_size"] = Json((double)nerf.training.counters_rgb.measured_batch_size);
	rgb["measured_batch_size_before_compaction"] = Json((double)nerf.training.counters_rgb.measured_batch_size_before_compaction);
	nj["rgb"] = rgb;
	Json ds = Json::object();
	ds["aabb_scale"] = Json((double)nerf.training.dataset.aabb_scale);
	ds["scale"] = Json((double)nerf.training.dataset.scale);
	ds["offset"] = vec_json(nerf.training.dataset.offset.data(), 3);
	ds["up"] = vec_json(nerf.training.dataset.up.data(), 3);
	ds["is_hdr"] = Json(nerf.training.dataset.is_hdr);
	ds["n_images"] = Json((double)nerf.training.dataset.n_images);
	ds["n_extra_learnable_dims"] = Json((double)nerf.training.dataset.n_extra_learnable_dims);
	nj["dataset"] = ds;
	// the latent codes' optimisers (src/testbed.cu:4795, VarAdamOptimizer::to_json adam_optimizer.h:73-82)
	{
		Json a = Json::array();
		for (const auto& o : nerf.training.extra_dims_opt) {
			Json j = Json::object();
			j["iter"] = Json((double)o.iter);
			j["first_moment"] = vec_json(o.m.data(), o.m.size());
			j["second_moment"] = vec_json(o.v.data(), o.v.size());
			j["variable"] = vec_json(o.variable.data(), o.variable.size());
			j["learning_rate"] = Json((double)o.learning_rate);
			j["epsilon"] = Json((double)o.epsilon);
			j["beta1"] = Json((double)o.beta1);
			j["beta2"] = Json((double)o.beta2);
			a.push_back(std::move(j));
		}
		nj["extra_dims_opt"] = a;
	}
	// per-image extrinsic offsets as the reference's AdamOptimizer to_json objects
	// (src/testbed.cu:4793-4794, adam_optimizer.h:172-183)
	auto adam_json = [](const std::vector<NerfTraining::Adam3>& v) {
		Json a = Json::array();
		for (const auto& o : v) {
			Json j = Json::object();
			j["iter"] = Json((double)o.iter);
			j["first_moment"] = vec_json(o.m.data(), 3);
			j["second_moment"] = vec_json(o.v.data(), 3);
			j["variable"] = vec_json(o.variable.data(), 3);
			j["learning_rate"] = Json(1e-4);
			j["epsilon"] = Json(1e-8);
			j["beta1"] = Json(0.9);
			j["beta2"] = Json(0.99);
			a.push_back(std::move(j));
		}
		return a;
	};
	nj["cam_pos_offset"] = adam_json(nerf.training.cam_pos_offset);
	nj["cam_rot_offset"] = adam_json(nerf.training.cam_rot_offset);
	nj["rgb_activation"] = Json((double)(int)nerf.rgb_activation);
	nj["density_activation"] = Json((double)(int)nerf.density_activation);
	nj["density_grid_ema_step"] = Json((double)nerf.density_grid_ema_step);
	snap["nerf"] = nj;
	snap["training_step"] = Json((double)training_step);
	snap["loss"] = Json((double)loss);
	Json aabb = Json::object();
	aabb["min"] = vec_json(aabb_min.data(), 3);
	aabb["max"] = vec_json(aabb_max.data(), 3);
	snap["aabb"] = aabb;
	snap["exposure"] = Json((double)exposure);
	snap["background_color"] = vec_json(background_color.data(), 4);
	snap["up_dir"] = vec_json(up_dir.data(), 3);  // src/testbed.cu:4804
	Json cam = Json::object();
	Json mat = Json::array();
	for (int c = 0; c < 4; ++c) mat.push_back(vec_json(&camera.m[3 * c], 3));  // 4 columns of 3 (mat4x3)
	cam["matrix"] = mat;
	cam["fov_axis"] = Json((double)fov_axis);
	cam["relative_focal_length"] = vec_json(relative_focal_length.data(), 2);
	cam["screen_center"] = vec_json(screen_center.data(), 2);
	cam["zoom"] = Json((double)zoom);
	cam["scale"] = Json((double)scale);
	snap["camera"] = cam;
	root["snapshot"] = snap;

	std::vector<uint8_t> bytes = root.to_msgpack();
	if (extension(path) == "ingp") {
		uLongf clen = compressBound((uLong)bytes.size());
		std::vector<uint8_t> c(clen);
		if (compress2(c.data(), &clen, bytes.data(), (uLong)bytes.size(), compress ? Z_DEFAULT_COMPRESSION : Z_NO_COMPRESSION) != Z_OK)
			throw std::runtime_error("snapshot compression failed");
		c.resize(clen);
		bytes.swap(c);
	}
	std::ofstream f(path, std::ios::binary);
	if (!f) throw std::runtime_error("Could not open '" + path + "' for writing.");
	f.write(reinterpret_cast<const char*>(bytes.data()), (std::streamsize)bytes.size());
}

Json Testbed::read_snapshot_file(const std::string& path) {
	std::ifstream f(path, std::ios::binary);
	if (!f) throw std::runtime_error("Snapshot '" + path + "' does not exist.");
	std::vector<uint8_t> file((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
	// zstr auto-detection: a zlib stream starts with 0x78 (CMF deflate/32K window); raw msgpack of
	// a config object starts with a map marker (0x8X / 0xde / 0xdf)
	if (file.size() >= 2 && file[0] == 0x78 && ((file[0] << 8) | file[1]) % 31 == 0) file = zlib_inflate(file);
	return Json::from_msgpack(file.data(), file.size());
}

void Testbed::load_snapshot(const std::string& path) {
	Json root = read_snapshot_file(path);
	if (!root.contains("snapshot")) throw std::runtime_error("File '" + path + "' does not contain a snapshot.");
	const Json snap = root["snapshot"];
	if (snap.value("version", 0.0) < (double)SNAPSHOT_FORMAT_VERSION)
		throw std::runtime_error("Snapshot uses an old format and can not be loaded.");
	if (snap.contains("mode") && snap["mode"].str() != "Nerf")
		throw std::runtime_error("Only NeRF snapshots are supported by this build (mode '" + snap["mode"].str() + "').");
	if ((uint32_t)snap.value("density_grid_size", (double)NERF_GRIDSIZE) != NERF_GRIDSIZE)
		throw std::runtime_error("Incompatible grid size.");
	if (mode != ETestbedMode::Nerf) {
		nerf = Nerf{};
		mode = ETestbedMode::Nerf;
	}
	const Json& nj = snap["nerf"];
	if (nj.contains("aabb_scale")) nerf.training.dataset.aabb_scale = (int)nj["aabb_scale"].num();
	if (!training_data_available && nj.contains("dataset")) {
		const Json& ds = nj["dataset"];
		nerf.training.dataset.scale = (float)ds.value("scale", 0.33);
		if (ds.contains("offset"))
			for (int k = 0; k < 3; ++k) nerf.training.dataset.offset[k] = (float)ds["offset"][k].num();
		nerf.training.dataset.is_hdr = ds.value("is_hdr", false);
	}
	if (nj.contains("dataset"))  // src/testbed.cu:4879
		nerf.training.dataset.n_extra_learnable_dims =
		    (uint32_t)nj["dataset"].value("n_extra_learnable_dims", (double)nerf.training.dataset.n_extra_learnable_dims);
	{  // load_nerf_post: aabb, cascades, cone angle, activations
		const int s = nerf.training.dataset.aabb_scale;
		const float half = 0.5f * (float)std::min(128, s);
		aabb_min = {0.5f - half, 0.5f - half, 0.5f - half};
		aabb_max = {0.5f + half, 0.5f + half, 0.5f + half};
		nerf.max_cascade = 0;
		while ((1 << nerf.max_cascade) < s) ++nerf.max_cascade;
		nerf.cone_angle_constant = s <= 1 ? 0.0f : (1.0f / 256.0f);
		nerf.rgb_activation = nerf.training.dataset.is_hdr ? ENerfActivation::Exponential : ENerfActivation::Logistic;
	}
	if (nj.contains("rgb_activation")) nerf.rgb_activation = (ENerfActivation)(int)nj["rgb_activation"].num();
	if (nj.contains("density_activation")) nerf.density_activation = (ENerfActivation)(int)nj["density_activation"].num();
	if (nj.contains("rgb")) {
		nerf.training.counters_rgb.rays_per_batch = (uint32_t)nj["rgb"].value("rays_per_batch", 4096.0);
		nerf.training.counters_rgb.measured_batch_size = (uint32_t)nj["rgb"].value("measured_batch_size", 0.0);
		nerf.training.counters_rgb.measured_batch_size_before_compaction =
		    (uint32_t)nj["rgb"].value("measured_batch_size_before_compaction", 0.0);
	}
	exposure = (float)snap.value("exposure", (double)exposure);
	if (snap.contains("background_color"))
		for (int k = 0; k < 4; ++k) background_color[k] = (float)snap["background_color"][k].num();
	if (snap.contains("up_dir"))
		for (int k = 0; k < 3; ++k) up_dir[k] = (float)snap["up_dir"][k].num();
	if (snap.contains("camera")) {
		const Json& cam = snap["camera"];
		if (cam.contains("matrix") && cam["matrix"].size() == 4)
			for (int c = 0; c < 4; ++c)
				for (int r = 0; r < 3; ++r) camera.m[3 * c + r] = (float)cam["matrix"][c][r].num();
		fov_axis = (uint32_t)cam.value("fov_axis", (double)fov_axis);
		if (cam.contains("relative_focal_length"))
			for (int k = 0; k < 2; ++k) relative_focal_length[k] = (float)cam["relative_focal_length"][k].num();
		if (cam.contains("screen_center"))
			for (int k = 0; k < 2; ++k) screen_center[k] = (float)cam["screen_center"][k].num();
		zoom = (float)cam.value("zoom", (double)zoom);
		scale = (float)cam.value("scale", (double)scale);
	}

	const uint32_t saved_step = (uint32_t)snap.value("training_step", 0.0);
	const float saved_loss = (float)snap.value("loss", 0.0);
	const uint32_t saved_counters_rpb = nerf.training.counters_rgb.rays_per_batch;
	const NerfCounters saved_counters = nerf.training.counters_rgb;
	root.erase("snapshot");
	m_network_config = root;
	reset_network(false);
	if (nj.contains("extra_dims_opt") && nj["extra_dims_opt"].is_array() && n_extra_dims()) {  // src/testbed.cu:4948-4950
		const Json& xa = nj["extra_dims_opt"];
		auto& opt = nerf.training.extra_dims_opt;
		opt.resize(xa.size());
		for (size_t i = 0; i < xa.size(); ++i) {
			const Json& j = xa[i];
			auto vec = [&](const char* k) {
				std::vector<float> v;
				if (j.contains(k))
					for (size_t q = 0; q < j[k].size(); ++q) v.push_back((float)j[k][q].num());
				return v;
			};
			opt[i].iter = (uint32_t)j.value("iter", 0.0);
			opt[i].m = vec("first_moment");
			opt[i].v = vec("second_moment");
			opt[i].variable = vec("variable");
			opt[i].learning_rate = (float)j.value("learning_rate", 1e-4);
			opt[i].epsilon = (float)j.value("epsilon", 1e-8);
			opt[i].beta1 = (float)j.value("beta1", 0.9);
			opt[i].beta2 = (float)j.value("beta2", 0.99);
			if (opt[i].variable.size() != n_extra_dims() || opt[i].m.size() != n_extra_dims() || opt[i].v.size() != n_extra_dims())
				throw std::runtime_error("snapshot: extra_dims_opt entries do not match n_extra_dims");
		}
		upload_extra_dims();
	}
	nerf.training.counters_rgb = saved_counters;
	nerf.training.counters_rgb.rays_per_batch = saved_counters_rpb;
	// dataset-specific optimised extrinsics (src/testbed.cu:4940-4951): restored when the
	// snapshot's dataset has the loaded dataset's image count
	if (training_data_available && nj.contains("dataset") &&
	    (size_t)nj["dataset"].value("n_images", -1.0) == nerf.training.dataset.n_images) {
		auto load_adam = [&](const char* key, std::vector<NerfTraining::Adam3>& v) {
			if (!nj.contains(key) || nj[key].size() != nerf.training.dataset.n_images) return;
			v.assign(nerf.training.dataset.n_images, NerfTraining::Adam3{});
			for (size_t i = 0; i < v.size(); ++i) {
				const Json& j = nj[key][i];
				v[i].iter = (uint32_t)j.value("iter", 0.0);
				for (int k = 0; k < 3; ++k) {
					v[i].m[k] = (float)j["first_moment"][k].num();
					v[i].v[k] = (float)j["second_moment"][k].num();
					v[i].variable[k] = (float)j["variable"][k].num();
				}
			}
		};
		load_adam("cam_pos_offset", nerf.training.cam_pos_offset);
		load_adam("cam_rot_offset", nerf.training.cam_rot_offset);
		m_dataset_dirty = true;  // update_transforms
	}

	ngp_model_info info{};
	ck(ngp_model_get_info(m_model, &info));
	auto upload = [&](int kind, const std::vector<uint8_t>& src) {
		void* p = nullptr;
		size_t bytes = 0;
		ck(ngp_model_buffer(m_model, kind, &p, &bytes));
		if (src.size() != bytes) throw std::runtime_error("snapshot buffer size does not match its network config");
		hk(hipMemcpy(p, src.data(), bytes, hipMemcpyHostToDevice), "snapshot h2d");
	};
	const Json& exact = snap["mi355x"];
	if (exact.contains("params_fp32_binary")) {
		upload(NGP_PARAMS_FP32, exact["params_fp32_binary"].bin());
		ck(ngp_model_params_updated(m_model, 1, m_stream));
		sync();
		upload(NGP_PARAMS_EMA_FP32, exact["params_ema_fp32_binary"].bin());
		if (exact.contains("adam_m_binary")) {
			upload(NGP_ADAM_M, exact["adam_m_binary"].bin());
			upload(NGP_ADAM_V, exact["adam_v_binary"].bin());
		}
		ck(ngp_model_params_updated(m_model, 0, m_stream));
	} else {
		// tcnn Trainer::deserialize: params_binary in params_type precision -> full-precision params
		const std::string type = snap.value("params_type", std::string("__half"));
		const std::vector<uint8_t>& b = snap["params_binary"].bin();
		std::vector<float> p32(info.n_params);
		if (type == "float") {
			if (b.size() != p32.size() * 4) throw std::runtime_error("snapshot params_binary has the wrong size");
			std::memcpy(p32.data(), b.data(), b.size());
		} else if (type == "__half") {
			if (b.size() != p32.size() * 2) throw std::runtime_error("snapshot params_binary has the wrong size");
			for (size_t k = 0; k < p32.size(); ++k) {
				uint16_t h;
				std::memcpy(&h, &b[2 * k], 2);
				p32[k] = f16_to_f32(h);
			}
		} else {
			throw std::runtime_error("unsupported snapshot params_type '" + type + "'");
		}
		std::vector<uint8_t> raw(p32.size() * 4);
		std::memcpy(raw.data(), p32.data(), raw.size());
		upload(NGP_PARAMS_FP32, raw);
		ck(ngp_model_params_updated(m_model, 1, m_stream));
	}
	sync();

	const std::vector<uint8_t>& g16 = snap["density_grid_binary"].bin();
	const size_t n_cells = (size_t)NERF_GRID_N_CELLS * (nerf.max_cascade + 1);
	if (!g16.empty()) {
		if (g16.size() != n_cells * 2) throw std::runtime_error("Incompatible number of grid cascades.");
		std::vector<float> grid(n_cells);
		if (exact.contains("density_grid_fp32_binary") && exact["density_grid_fp32_binary"].bin().size() == n_cells * 4) {
			std::memcpy(grid.data(), exact["density_grid_fp32_binary"].bin().data(), n_cells * 4);
		} else {
			for (size_t k = 0; k < n_cells; ++k) {
				uint16_t h;
				std::memcpy(&h, &g16[2 * k], 2);
				grid[k] = f16_to_f32(h);
			}
		}
		ck(ngp_density_grid_bitfield(m_model, nerf.max_cascade, m_stream));  // sizes the grid buffers
		sync();
		float* dg = nullptr;
		ck(ngp_density_grid_buffers(m_model, &dg, nullptr, nullptr, nullptr));
		hk(hipMemcpy(dg, grid.data(), grid.size() * 4, hipMemcpyHostToDevice), "grid h2d");
		ck(ngp_density_grid_bitfield(m_model, nerf.max_cascade, m_stream));
		sync();
	}
	training_step = saved_step;
	loss = saved_loss;
	nerf.density_grid_ema_step = (uint32_t)nj.value("density_grid_ema_step", 0.0);
	network_config_path = path;
}

// ---------------------------------------------------------------------------
// Multi-GPU (RCCL over xGMI)
// ---------------------------------------------------------------------------
std::string Testbed::nccl_unique_id() {
	ncclUniqueId id;
	nk(ncclGetUniqueId(&id), "ncclGetUniqueId");
	return std::string(id.internal, sizeof(id.internal));
}

void Testbed::init_distributed(int rank, int world_size, const std::string& uid) {
	if (world_size < 1 || rank < 0 || rank >= world_size) throw std::runtime_error("init_distributed: bad rank / world_size");
	if (m_comm || m_host_allreduce) throw std::runtime_error("init_distributed: already distributed");
	if (uid.size() != sizeof(ncclUniqueId::internal)) throw std::runtime_error("init_distributed: bad ncclUniqueId");
	ncclUniqueId id;
	std::memcpy(id.internal, uid.data(), uid.size());
	ncclComm_t comm;
	nk(ncclCommInitRank(&comm, world_size, id, rank), "ncclCommInitRank");
	m_comm = comm;
	m_rank = rank;
	m_world = world_size;
	hk(hipMalloc(&m_red_buf, 64), "hipMalloc reduction scratch");
}

// Rows of an H-row frame that shard `idx` of `count` owns in blocks of `rows` (ngp_render_args).
static std::vector<std::pair<uint32_t, uint32_t>> owned_row_runs(uint32_t H, uint32_t idx, uint32_t count, uint32_t rows) {
	std::vector<std::pair<uint32_t, uint32_t>> runs;  // (first row, n rows)
	for (uint32_t b = idx; b * rows < H; b += count) runs.push_back({b * rows, std::min(rows, H - b * rows)});
	return runs;
}

std::vector<float> Testbed::render_distributed(int width, int height, int spp, bool linear, bool copy_to_host) {
	const uint32_t R = 8;
	if (!distributed()) return render(width, height, spp, linear, 0, 1, R, copy_to_host);
	render(width, height, spp, linear, (uint32_t)m_rank, (uint32_t)m_world, R, false);
	const size_t row_bytes = (size_t)width * 4 * sizeof(float);
	hipStream_t s = (hipStream_t)m_stream;
	std::vector<size_t> pack_rows(m_world);
	for (int r = 0; r < m_world; ++r)
		for (const auto& run : owned_row_runs((uint32_t)height, (uint32_t)r, (uint32_t)m_world, R)) pack_rows[r] += run.second;
	if (!m_comm) {
		// host-staged test backend: owned rows over a zero frame, summed over the ranks
		std::vector<float> full((size_t)width * height * 4, 0.0f);
		for (const auto& run : owned_row_runs((uint32_t)height, (uint32_t)m_rank, (uint32_t)m_world, R))
			hk(hipMemcpyAsync((char*)full.data() + run.first * row_bytes, (const char*)m_out + run.first * row_bytes,
			                  run.second * row_bytes, hipMemcpyDeviceToHost, s), "rows d2h");
		sync();
		m_host_allreduce(full.data(), full.size(), 0, 0);
		if (m_rank != 0) return {};
		hk(hipMemcpyAsync(m_out, full.data(), full.size() * sizeof(float), hipMemcpyHostToDevice, s), "frame h2d");
		sync();
		if (!copy_to_host) full.clear();
		return full;
	}
	// every rank packs its rows (contiguous in shard order) into [0, slot) and sends them to rank 0,
	// which receives every rank's pack -- its own too, over RCCL, so one code path serves any world
	// size -- into slot r + 1 and unpacks them into its frame
	const size_t slot = *std::max_element(pack_rows.begin(), pack_rows.end()) * row_bytes;
	const size_t cap = slot * (m_rank == 0 ? (size_t)m_world + 1 : 1);
	if (cap > m_pack_cap) {
		if (m_pack) (void)hipFree(m_pack);
		hk(hipMalloc((void**)&m_pack, cap), "hipMalloc pack");
		m_pack_cap = cap;
	}
	{
		size_t off = 0;
		for (const auto& run : owned_row_runs((uint32_t)height, (uint32_t)m_rank, (uint32_t)m_world, R)) {
			hk(hipMemcpyAsync((char*)m_pack + off, (const char*)m_out + run.first * row_bytes, run.second * row_bytes,
			                  hipMemcpyDeviceToDevice, s), "pack rows");
			off += run.second * row_bytes;
		}
	}
	nk(ncclGroupStart(), "ncclGroupStart");
	if (m_rank == 0)
		for (int r = 0; r < m_world; ++r)
			nk(ncclRecv((char*)m_pack + (r + 1) * slot, pack_rows[r] * row_bytes, ncclChar, r, (ncclComm_t)m_comm, s), "ncclRecv rows");
	nk(ncclSend(m_pack, pack_rows[m_rank] * row_bytes, ncclChar, 0, (ncclComm_t)m_comm, s), "ncclSend rows");
	nk(ncclGroupEnd(), "ncclGroupEnd");
	std::vector<float> out;
	if (m_rank == 0) {
		for (int r = 0; r < m_world; ++r) {
			size_t off = 0;
			for (const auto& run : owned_row_runs((uint32_t)height, (uint32_t)r, (uint32_t)m_world, R)) {
				hk(hipMemcpyAsync((char*)m_out + run.first * row_bytes, (const char*)m_pack + (r + 1) * slot + off,
				                  run.second * row_bytes, hipMemcpyDeviceToDevice, s), "unpack rows");
				off += run.second * row_bytes;
			}
		}
		if (copy_to_host) {
			out.resize((size_t)width * height * 4);
			hk(hipMemcpyAsync(out.data(), m_out, out.size() * sizeof(float), hipMemcpyDeviceToHost, s), "frame d2h");
		}
	}
	sync();
	return out;
}

void Testbed::allreduce_f32(float* dev, size_t n, bool max_op) { allreduce_dev(dev, n, 0, max_op); }

// ngp_train_args.allreduce_i32: the step's per-rank totals, on the Testbed's collective backend
ngp_status Testbed::dp_allreduce_i32(void* user, int32_t* dev, uint32_t n, ngp_stream) {
	try {
		static_cast<Testbed*>(user)->allreduce_dev(dev, n, 2, false);
		return NGP_OK;
	} catch (const std::exception& e) {
		std::fprintf(stderr, "data-parallel all-reduce failed: %s\n", e.what());
		return NGP_ERR_UNSUPPORTED;
	}
}

// dtype: 0 f32, 1 f16, 2 i32, 3 i64 (deterministic fixed-point gradients)
void Testbed::allreduce_dev(void* dev, size_t n, int dtype, bool max_op) {
	if (!distributed() || n == 0) return;
	static const size_t elem[4] = {4, 2, 4, 8};
	if (dtype < 0 || dtype > 3) throw std::runtime_error("allreduce_dev: unknown dtype");
	if (m_comm) {
		static const ncclDataType_t types[4] = {ncclFloat32, ncclFloat16, ncclInt32, ncclInt64};
		nk(ncclAllReduce(dev, dev, n, types[dtype], max_op ? ncclMax : ncclSum, (ncclComm_t)m_comm, (hipStream_t)m_stream),
		   "ncclAllReduce");
		return;
	}
	if (!m_host_allreduce) throw std::runtime_error("distributed Testbed without a collective backend");
	const size_t bytes = n * elem[dtype];
	std::vector<uint8_t> h(bytes);
	hk(hipMemcpyAsync(h.data(), dev, bytes, hipMemcpyDeviceToHost, (hipStream_t)m_stream), "allreduce d2h");
	sync();
	m_host_allreduce(h.data(), n, dtype, max_op ? 1 : 0);
	hk(hipMemcpyAsync(dev, h.data(), bytes, hipMemcpyHostToDevice, (hipStream_t)m_stream), "allreduce h2d");
	sync();
}

void Testbed::init_distributed_host(int rank, int world_size, HostAllReduce fn) {
	if (world_size < 1 || rank < 0 || rank >= world_size) throw std::runtime_error("init_distributed_host: bad rank / world_size");
	if (m_comm || m_host_allreduce) throw std::runtime_error("init_distributed_host: already distributed");
	if (!fn) throw std::runtime_error("init_distributed_host: no all-reduce function");
	m_host_allreduce = std::move(fn);
	m_rank = rank;
	m_world = world_size;
	if (!m_red_buf) hk(hipMalloc(&m_red_buf, 64), "hipMalloc reduction scratch");
}

}  // namespace ngp
