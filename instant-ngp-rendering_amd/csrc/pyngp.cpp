// pyngp.cpp — Python module `pyngp` over the MI355X Testbed.
//
// Mirrors the NeRF-relevant surface of the reference's bindings (src/python_api.cu:263-720):
// same class/enum/attribute names and argument defaults, so scripts/run.py-style drivers
// (`ngp.Testbed()`, `load_training_data`, `frame()`, `render(w, h, spp, linear)`, ...) run
// unchanged.  GUI/VR/SDF/Image/Volume members are absent by design.
#include <pybind11/functional.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>
#include <limits>

#include "ngp_math.h"
#include "testbed.h"

namespace py = pybind11;
using namespace ngp;

// An [h][w][4] float array over a pooled page-locked buffer (pinned_host_alloc); the capsule returns the
// buffer to the pool when numpy frees the array.
static py::array_t<float> pinned_frame(int height, int width) {
	const size_t bytes = (size_t)height * width * 4 * sizeof(float);
	float* p = static_cast<float*>(pinned_host_alloc(bytes));
	auto* owner = new std::pair<void*, size_t>(p, bytes);
	py::capsule cap(owner, [](void* o) {
		auto* q = static_cast<std::pair<void*, size_t>*>(o);
		pinned_host_release(q->first, q->second);
		delete q;
	});
	return py::array_t<float>({(py::ssize_t)height, (py::ssize_t)width, (py::ssize_t)4}, p, cap);
}

#define NGP_TUNING_FIELDS                                                                                              \
	NGP_TUNING_FIELD(render_pipelines) NGP_TUNING_FIELD(render_pass_samples) NGP_TUNING_FIELD(render_lanes)          \
	NGP_TUNING_FIELD(render_first_steps) NGP_TUNING_FIELD(render_max_steps) NGP_TUNING_FIELD(render_lag)             \
	NGP_TUNING_FIELD(render_budget_scale) NGP_TUNING_FIELD(render_composite_block) NGP_TUNING_FIELD(render_generate_block) \
	NGP_TUNING_FIELD(encode_dense_records) NGP_TUNING_FIELD(mlp_workgroups_per_cu) NGP_TUNING_FIELD(debug)           \
	NGP_TUNING_FIELD(encode_streaming) NGP_TUNING_FIELD(grid_unsorted) NGP_TUNING_FIELD(render_mlp_tile)             \
	NGP_TUNING_FIELD(encode_xcd_regions) NGP_TUNING_FIELD(render_skip_unfilled) NGP_TUNING_FIELD(render_exit_cap) \
	NGP_TUNING_FIELD(render_priority) NGP_TUNING_FIELD(render_host_frame) NGP_TUNING_FIELD(train_chunk_lanes) NGP_TUNING_FIELD(train_sampler_lanes) NGP_TUNING_FIELD(render_mlp_pipeline)

namespace {

ETestbedMode mode_from_string(const std::string& s) {
	std::string l = s;
	for (auto& c : l) c = (char)std::tolower((unsigned char)c);
	if (l == "nerf") return ETestbedMode::Nerf;
	if (l == "sdf") return ETestbedMode::Sdf;
	if (l == "image") return ETestbedMode::Image;
	if (l == "volume") return ETestbedMode::Volume;
	return ETestbedMode::None;
}

// mode_from_scene (src/common_host.cu:146-164)
ETestbedMode mode_from_scene(const std::string& scene) {
	auto ends = [&](const char* e) {
		const size_t n = std::strlen(e);
		if (scene.size() < n) return false;
		for (size_t i = 0; i < n; ++i)
			if (std::tolower((unsigned char)scene[scene.size() - n + i]) != e[i]) return false;
		return true;
	};
	struct stat_probe {
		static bool is_dir(const std::string& p) {
			py::module_ os = py::module_::import("os");
			return os.attr("path").attr("isdir")(p).cast<bool>();
		}
	};
	if (stat_probe::is_dir(scene) || ends(".json")) return ETestbedMode::Nerf;
	if (ends(".obj") || ends(".stl")) return ETestbedMode::Sdf;
	if (ends(".nvdb")) return ETestbedMode::Volume;
	if (ends(".exr") || ends(".bin") || ends(".png") || ends(".jpg")) return ETestbedMode::Image;
	return ETestbedMode::None;
}

py::array_t<float> mat43_to_numpy(const Mat43& m) {
	py::array_t<float> a({3, 4});
	auto r = a.mutable_unchecked<2>();
	for (int row = 0; row < 3; ++row)
		for (int col = 0; col < 4; ++col) r(row, col) = m.m[3 * col + row];
	return a;
}

std::array<float, 12> numpy_to_rowmajor34(py::array_t<float, py::array::c_style | py::array::forcecast> a) {
	if (a.ndim() != 2 || a.shape(1) != 4 || a.shape(0) < 3) throw std::runtime_error("expected a 3x4 (or 4x4) matrix");
	std::array<float, 12> out;
	auto r = a.unchecked<2>();
	for (int row = 0; row < 3; ++row)
		for (int col = 0; col < 4; ++col) out[row * 4 + col] = r(row, col);
	return out;
}

Mat43 numpy_to_mat43(py::array_t<float, py::array::c_style | py::array::forcecast> a) {
	auto rm = numpy_to_rowmajor34(a);
	Mat43 m;
	for (int row = 0; row < 3; ++row)
		for (int col = 0; col < 4; ++col) m.m[3 * col + row] = rm[row * 4 + col];
	return m;
}

Json json_from_py(const py::object& o) {
	py::module_ json = py::module_::import("json");
	return Json::parse(json.attr("dumps")(o).cast<std::string>());
}

py::object json_to_py(const Json& j) {
	py::module_ json = py::module_::import("json");
	return json.attr("loads")(j.dump());
}

// Non-PNG decoder (the reference links stb_image; src/nerf_loader.cu:520-560): PIL, if importable.
bool pil_decode(const std::string& path, std::vector<uint8_t>& rgba, int& w, int& h) {
	py::gil_scoped_acquire gil;
	try {
		py::module_ image = py::module_::import("PIL.Image");
		py::module_ np = py::module_::import("numpy");
		py::object img = image.attr("open")(path).attr("convert")("RGBA");
		py::array_t<uint8_t, py::array::c_style | py::array::forcecast> a = np.attr("asarray")(img);
		h = (int)a.shape(0);
		w = (int)a.shape(1);
		rgba.assign(a.data(), a.data() + (size_t)w * h * 4);
		return true;
	} catch (const py::error_already_set&) {
		return false;
	}
}

// Views into the Testbed so Python can write `testbed.nerf.training.random_bg_color = False`
// exactly like the reference (which exposes Nerf / Nerf::Training by reference).
struct TrainingView {
	Testbed* tb;
};
struct NerfView {
	Testbed* tb;
};

// bounding_box.cuh:45-263: default-constructed empty (min = +inf, max = -inf)
struct BoundingBox {
	vec3 min = {INFINITY, INFINITY, INFINITY}, max = {-INFINITY, -INFINITY, -INFINITY};
	bool is_empty() const { return max[0] < min[0] || max[1] < min[1] || max[2] < min[2]; }
};

}  // namespace

PYBIND11_MODULE(pyngp, m) {
	m.doc() = "Instant neural graphics primitives — MI355X (gfx950) NeRF path";
	m.def("free_temporary_memory", []() {});

	py::enum_<ETestbedMode>(m, "TestbedMode")
		.value("Nerf", ETestbedMode::Nerf)
		.value("Sdf", ETestbedMode::Sdf)
		.value("Image", ETestbedMode::Image)
		.value("Volume", ETestbedMode::Volume)
		.value("None", ETestbedMode::None)
		.export_values();
	m.def("mode_from_scene", &mode_from_scene);
	m.def("mode_from_string", &mode_from_string);
	// the ExponentialDecay schedule every optimizer of the Testbed uses (ngp_math.h; parity unpinned)
	m.def("exponential_decay_learning_rate", &exp_decay_learning_rate, py::arg("learning_rate"), py::arg("decay_base"),
	      py::arg("decay_start"), py::arg("decay_interval"), py::arg("decay_end"), py::arg("step"));

	py::enum_<ELossType>(m, "LossType")
		.value("L2", ELossType::L2)
		.value("L1", ELossType::L1)
		.value("Mape", ELossType::Mape)
		.value("Smape", ELossType::Smape)
		.value("Huber", ELossType::Huber)
		.value("SmoothL1", ELossType::Huber)
		.value("LogL1", ELossType::LogL1)
		.value("RelativeL2", ELossType::RelativeL2)
		.export_values();
	py::enum_<ENerfActivation>(m, "NerfActivation")
		.value("None", ENerfActivation::None)
		.value("ReLU", ENerfActivation::ReLU)
		.value("Logistic", ENerfActivation::Logistic)
		.value("Exponential", ENerfActivation::Exponential)
		.export_values();
	py::enum_<EColorSpace>(m, "ColorSpace")
		.value("Linear", EColorSpace::Linear)
		.value("SRGB", EColorSpace::SRGB)
		.export_values();
	py::enum_<ETonemapCurve>(m, "TonemapCurve")
		.value("Identity", ETonemapCurve::Identity)
		.value("ACES", ETonemapCurve::ACES)
		.value("Hable", ETonemapCurve::Hable)
		.value("Reinhard", ETonemapCurve::Reinhard)
		.export_values();
	py::enum_<ERenderMode>(m, "RenderMode")
		.value("AO", ERenderMode::AO)
		.value("Shade", ERenderMode::Shade)
		.value("Normals", ERenderMode::Normals)
		.value("Positions", ERenderMode::Positions)
		.value("Depth", ERenderMode::Depth)
		.value("Distortion", ERenderMode::Distortion)
		.value("Cost", ERenderMode::Cost)
		.value("Slice", ERenderMode::Slice)
		.export_values();
	py::enum_<ELensMode>(m, "LensMode")
		.value("Perspective", ELensMode::Perspective)
		.value("OpenCV", ELensMode::OpenCV)
		.value("FTheta", ELensMode::FTheta)
		.value("LatLong", ELensMode::LatLong)
		.value("OpenCVFisheye", ELensMode::OpenCVFisheye)
		.value("Equirectangular", ELensMode::Equirectangular)
		.export_values();

	py::class_<BoundingBox>(m, "BoundingBox")
		.def(py::init<>())
		.def(py::init([](vec3 a, vec3 b) { return BoundingBox{a, b}; }))
		.def("center", [](const BoundingBox& b) {
			return vec3{0.5f * (b.min[0] + b.max[0]), 0.5f * (b.min[1] + b.max[1]), 0.5f * (b.min[2] + b.max[2])};
		})
		.def("diag", [](const BoundingBox& b) { return vec3{b.max[0] - b.min[0], b.max[1] - b.min[1], b.max[2] - b.min[2]}; })
		.def("is_empty", &BoundingBox::is_empty)
		.def("contains", [](const BoundingBox& b, vec3 p) {
			for (int k = 0; k < 3; ++k)
				if (p[k] < b.min[k] || p[k] > b.max[k]) return false;
			return true;
		})
		.def_readwrite("min", &BoundingBox::min)
		.def_readwrite("max", &BoundingBox::max);

	py::class_<Lens>(m, "Lens")
		.def(py::init<>())
		.def_readwrite("mode", &Lens::mode)
		.def_property("params", [](const Lens& l) { return std::vector<float>(l.params, l.params + 7); },
		              [](Lens& l, const std::vector<float>& v) {
			              for (size_t i = 0; i < 7; ++i) l.params[i] = i < v.size() ? v[i] : 0.f;
		              });

	py::class_<TrainingImageMetadata>(m, "TrainingImageMetadata")
		.def_readwrite("camera_distortion", &TrainingImageMetadata::lens)
		.def_readwrite("lens", &TrainingImageMetadata::lens)
		.def_readwrite("resolution", &TrainingImageMetadata::resolution)
		.def_readwrite("principal_point", &TrainingImageMetadata::principal_point)
		.def_readwrite("focal_length", &TrainingImageMetadata::focal_length)
		.def_readwrite("rolling_shutter", &TrainingImageMetadata::rolling_shutter)
		.def_readwrite("light_dir", &TrainingImageMetadata::light_dir);

	py::class_<NerfDataset>(m, "NerfDataset")
		.def_readonly("metadata", &NerfDataset::metadata)
		.def_property_readonly("transforms", [](const NerfDataset& d) {
			py::list l;
			for (const auto& x : d.xforms) l.append(mat43_to_numpy(x));
			return l;
		})
		// TrainingXForm::end per image (= the start transform unless transform_matrix_end was given)
		.def_property_readonly("transforms_end", [](const NerfDataset& d) {
			py::list l;
			for (size_t i = 0; i < d.xforms.size(); ++i) l.append(mat43_to_numpy(i < d.xforms_end.size() ? d.xforms_end[i] : d.xforms[i]));
			return l;
		})
		.def_readonly("paths", &NerfDataset::paths)
		.def_readonly("up", &NerfDataset::up)
		.def_readonly("offset", &NerfDataset::offset)
		.def_readonly("n_images", &NerfDataset::n_images)
		.def_readonly("scale", &NerfDataset::scale)
		.def_readonly("aabb_scale", &NerfDataset::aabb_scale)
		.def_readonly("from_mitsuba", &NerfDataset::from_mitsuba)
		.def_readonly("is_hdr", &NerfDataset::is_hdr)
		.def_readwrite("n_extra_learnable_dims", &NerfDataset::n_extra_learnable_dims)
		.def_readonly("has_light_dirs", &NerfDataset::has_light_dirs)
		.def("n_extra_dims", &NerfDataset::n_extra_dims)
		.def("image", [](const NerfDataset& d, size_t i) {
			if (i >= d.n_images) throw std::runtime_error("Invalid frame index");
			const auto& md = d.metadata[i];
			py::array_t<uint8_t> a({md.resolution[1], md.resolution[0], 4});
			if (d.pixels[i].size() != (size_t)md.resolution[0] * md.resolution[1] * 4) throw std::runtime_error("image has no pixels");
			std::memcpy(a.mutable_data(), d.pixels[i].data(), d.pixels[i].size());
			return a;
		}, "RGBA8 (sRGB, straight alpha) pixels of image i, as stored for training")
		.def("depth", [](const NerfDataset& d, size_t i) -> py::object {
			if (i >= d.n_images) throw std::runtime_error("Invalid frame index");
			if (i >= d.depths.size() || d.depths[i].empty()) return py::none();
			const auto& md = d.metadata[i];
			py::array_t<float> a({md.resolution[1], md.resolution[0]});
			std::memcpy(a.mutable_data(), d.depths[i].data(), d.depths[i].size() * sizeof(float));
			return a;
		}, "depth targets of image i (16-bit depth x integer_depth_scale x scale), or None")
		.def("sharpness", [](const NerfDataset& d, size_t i) {
			if (i >= d.n_images) throw std::runtime_error("Invalid frame index");
			const std::vector<float> s = d.sharpness(i);
			py::array_t<float> a({72, 128});
			std::memcpy(a.mutable_data(), s.data(), s.size() * sizeof(float));
			return a;
		}, "compute_sharpness of image i: [72][128] variance of the Laplacian of the luma per tile");

	// ngp::load_nerf without a Testbed (no GPU needed): the dataset front end on its own
	m.def("load_nerf_dataset", [](const std::string& path) {
		py::gil_scoped_release rel;
		return load_nerf(path, &pil_decode);
	}, py::arg("path"));

	py::class_<Testbed> testbed(m, "Testbed");

	py::class_<NerfView> nerf(testbed, "Nerf");
	py::class_<TrainingView>(nerf, "Training")
#define TV_RW(name, field)                                                                                  \
	.def_property(name, [](const TrainingView& v) { return v.tb->nerf.training.field; },                   \
	              [](TrainingView& v, decltype(NerfTraining::field) x) { v.tb->nerf.training.field = x; })
		TV_RW("random_bg_color", random_bg_color)
		TV_RW("n_images_for_training", n_images_for_training)
		TV_RW("linear_colors", linear_colors)
		TV_RW("loss_type", loss_type)
		TV_RW("snap_to_pixel_centers", snap_to_pixel_centers)
		TV_RW("near_distance", near_distance)
		TV_RW("density_grid_decay", density_grid_decay)
		TV_RW("optimize_extrinsics", optimize_extrinsics)
		TV_RW("optimize_distortion", optimize_distortion)
		TV_RW("optimize_focal_length", optimize_focal_length)
		TV_RW("optimize_exposure", optimize_exposure)
		TV_RW("optimize_extra_dims", optimize_extra_dims)
		TV_RW("optimize_per_image_latents", optimize_extra_dims)
		TV_RW("sample_focal_plane_proportional_to_error", sample_focal_plane_proportional_to_error)
		TV_RW("sample_image_proportional_to_error", sample_image_proportional_to_error)
		TV_RW("include_sharpness_in_error", include_sharpness_in_error)
		TV_RW("depth_supervision_lambda", depth_supervision_lambda)
		TV_RW("depth_loss_type", depth_loss_type)
		TV_RW("n_steps_between_error_map_updates", n_steps_between_error_map_updates)
		TV_RW("n_steps_between_cam_updates", n_steps_between_cam_updates)
		TV_RW("exposure_l2_reg", exposure_l2_reg)
		TV_RW("extrinsic_l2_reg", extrinsic_l2_reg)
		TV_RW("extrinsic_learning_rate", extrinsic_learning_rate)
		TV_RW("intrinsic_l2_reg", intrinsic_l2_reg)
#undef TV_RW
		// additions: the accumulated error map and the image pmf of the last CDF update
		.def_property_readonly("error_map", [](TrainingView& v) {
			const auto& tr = v.tb->nerf.training;
			std::vector<float> h = v.tb->error_map_data();
			const py::ssize_t ni = h.empty() ? 0 : (py::ssize_t)tr.dataset.n_images;
			py::array_t<float> out({ni, (py::ssize_t)tr.error_map.resolution[1], (py::ssize_t)tr.error_map.resolution[0]});
			if (!h.empty()) std::memcpy(out.mutable_data(), h.data(), h.size() * sizeof(float));
			return out;
		})
		.def_property_readonly("cam_exposure", [](TrainingView& v) {
			py::list l;
			for (const auto& o : v.tb->nerf.training.cam_exposure) l.append(py::make_tuple(o.variable[0], o.variable[1], o.variable[2]));
			return l;
		})
		.def_property_readonly("cam_pos_offset", [](TrainingView& v) {
			py::list l;
			for (const auto& o : v.tb->nerf.training.cam_pos_offset) l.append(py::make_tuple(o.variable[0], o.variable[1], o.variable[2]));
			return l;
		})
		.def_property_readonly("cam_rot_offset", [](TrainingView& v) {
			py::list l;
			for (const auto& o : v.tb->nerf.training.cam_rot_offset) l.append(py::make_tuple(o.variable[0], o.variable[1], o.variable[2]));
			return l;
		})
		.def_property_readonly("cam_focal_length_offset", [](TrainingView& v) {
			const auto& o = v.tb->nerf.training.cam_focal_length_offset;
			return py::make_tuple(o.variable[0], o.variable[1]);
		})
		.def_property_readonly("error_map_pmf_img", [](TrainingView& v) { return v.tb->nerf.training.error_map.pmf_img_cpu; })
		.def_property_readonly("error_map_cdf_valid", [](TrainingView& v) { return v.tb->nerf.training.error_map.is_cdf_valid; })
		.def_property_readonly("dataset", [](TrainingView& v) -> NerfDataset& { return v.tb->nerf.training.dataset; },
		                       py::return_value_policy::reference_internal)
		.def_property_readonly("transforms", [](TrainingView& v) {
			py::list l;
			for (size_t i = 0; i < v.tb->nerf.training.dataset.xforms.size(); ++i) l.append(mat43_to_numpy(v.tb->training_transform(i)));
			return l;
		})
		.def("set_camera_intrinsics",
		     [](TrainingView& v, int frame_idx, float fx, float fy, float cx, float cy, float k1, float k2, float p1, float p2,
		        float k3, float k4, bool is_fisheye) {
			     v.tb->set_camera_intrinsics(frame_idx, fx, fy, cx, cy, k1, k2, p1, p2, k3, k4, is_fisheye);
		     },
		     py::arg("frame_idx"), py::arg("fx") = 0.f, py::arg("fy") = 0.f, py::arg("cx") = -0.5f, py::arg("cy") = -0.5f,
		     py::arg("k1") = 0.f, py::arg("k2") = 0.f, py::arg("p1") = 0.f, py::arg("p2") = 0.f, py::arg("k3") = 0.f,
		     py::arg("k4") = 0.f, py::arg("is_fisheye") = false)
		.def("set_camera_extrinsics",
		     [](TrainingView& v, int frame_idx, py::array_t<float, py::array::c_style | py::array::forcecast> c2w, bool convert) {
			     auto rm = numpy_to_rowmajor34(c2w);
			     v.tb->set_camera_extrinsics(frame_idx, rm.data(), convert);
		     },
		     py::arg("frame_idx"), py::arg("camera_to_world"), py::arg("convert_to_ngp") = true)
		.def("set_camera_extrinsics_rolling_shutter",
		     [](TrainingView& v, int frame_idx, py::array_t<float, py::array::c_style | py::array::forcecast> start,
		        py::array_t<float, py::array::c_style | py::array::forcecast> end, const vec4& rolling_shutter, bool convert) {
			     auto s = numpy_to_rowmajor34(start);
			     auto e = numpy_to_rowmajor34(end);
			     v.tb->set_camera_extrinsics_rolling_shutter(frame_idx, s.data(), e.data(), rolling_shutter, convert);
		     },
		     py::arg("frame_idx"), py::arg("camera_to_world_start"), py::arg("camera_to_world_end"), py::arg("rolling_shutter"),
		     py::arg("convert_to_ngp") = true)
		.def("get_extra_dims", [](const TrainingView& v, int i) { return v.tb->training_extra_dims(i); },
		     "Get the extra dims (including trained latent code) for a specified training view.")
		.def("get_camera_extrinsics", [](TrainingView& v, int i) { return mat43_to_numpy(v.tb->get_camera_extrinsics(i)); },
		     py::arg("frame_idx"))
		.def("set_image",
		     [](TrainingView& v, int frame_idx, py::array_t<float, py::array::c_style | py::array::forcecast> img,
		        py::object depth_img, float depth_scale) {
			     if (img.ndim() != 3 || img.shape(2) != 4) throw std::runtime_error("image should be (H,W,4)");
			     if (!depth_img.is_none()) throw std::runtime_error("depth supervision is not implemented on the MI355X path");
			     (void)depth_scale;
			     v.tb->set_image(frame_idx, img.data(), (int)img.shape(1), (int)img.shape(0));
		     },
		     py::arg("frame_idx"), py::arg("img"), py::arg("depth_img") = py::none(), py::arg("depth_scale") = 1.0f)
		.def("set_image_rgba8",
		     [](TrainingView& v, int frame_idx, py::array_t<uint8_t, py::array::c_style | py::array::forcecast> img) {
			     if (img.ndim() != 3 || img.shape(2) != 4) throw std::runtime_error("image should be (H,W,4) uint8");
			     v.tb->set_image_rgba8(frame_idx, img.data(), (int)img.shape(1), (int)img.shape(0));
		     },
		     py::arg("frame_idx"), py::arg("img"));

	nerf
#define NV_RW(name, field) \
	.def_property(name, [](const NerfView& v) { return v.tb->nerf.field; }, [](NerfView& v, decltype(Nerf::field) x) { v.tb->nerf.field = x; })
		NV_RW("rgb_activation", rgb_activation)
		NV_RW("density_activation", density_activation)
		NV_RW("sharpen", sharpen)
		NV_RW("render_with_lens_distortion", render_with_lens_distortion)
		NV_RW("render_with_camera_distortion", render_with_lens_distortion)
		NV_RW("render_lens", render_lens)
		NV_RW("render_distortion", render_lens)
		NV_RW("render_min_transmittance", render_min_transmittance)
		NV_RW("render_gbuffer_hard_edges", render_gbuffer_hard_edges)
		NV_RW("rendering_min_transmittance", render_min_transmittance)
		NV_RW("cone_angle_constant", cone_angle_constant)
		NV_RW("visualize_cameras", visualize_cameras)
		NV_RW("glow_y_cutoff", glow_y_cutoff)
		NV_RW("glow_mode", glow_mode)
		NV_RW("light_dir", light_dir)
#undef NV_RW
		.def("find_closest_training_view", [](const NerfView& v) { return v.tb->find_closest_training_view(); },
		     "Obtain the training view that is closest to the current camera.")
		// extra dims (per-image latent codes) of the rendered rays (Nerf::rendering_extra_dims, src/testbed_nerf.cu:3246-3280)
		.def_property("rendering_extra_dims_from_training_view",
		              [](const NerfView& v) { return v.tb->rendering_extra_dims_from_training_view; },
		              // a plain field write (def_readwrite, src/python_api.cu:596): -1 selects the set code; a view past
		              // the trained codes reads the set code too (Testbed::rendering_extra_dims)
		              [](NerfView& v, int i) { v.tb->rendering_extra_dims_from_training_view = i; })
		.def("set_rendering_extra_dims_from_training_view", [](NerfView& v, int i) { v.tb->set_rendering_extra_dims_from_training_view(i); })
		.def("set_rendering_extra_dims", [](NerfView& v, const std::vector<float>& x) { v.tb->set_rendering_extra_dims(x); })
		.def("get_rendering_extra_dims", [](const NerfView& v) { return v.tb->rendering_extra_dims(); })
		.def_property_readonly("max_cascade", [](const NerfView& v) { return v.tb->nerf.max_cascade; })
		.def_property_readonly("training", py::cpp_function([](NerfView& v) { return TrainingView{v.tb}; }, py::keep_alive<0, 1>()));

	testbed
		.def(py::init([](ETestbedMode mode) {
			     auto* t = new Testbed(mode);
			     t->image_decoder = &pil_decode;
			     // configs/ ship next to the extension (the reference resolves root_dir()/configs/<mode>/)
			     py::module_ os = py::module_::import("os");
			     t->root_dir = os.attr("path").attr("dirname")(py::module_::import("pyngp").attr("__file__")).cast<std::string>();
			     return t;
		     }),
		     py::arg("mode") = ETestbedMode::None)
		.def_readonly("mode", &Testbed::mode)
		.def("create_empty_nerf_dataset", &Testbed::create_empty_nerf_dataset, py::arg("n_images"), py::arg("aabb_scale") = 1,
		     py::arg("is_hdr") = false)
		.def("load_training_data", &Testbed::load_training_data, py::call_guard<py::gil_scoped_release>(), py::arg("path"))
		.def("clear_training_data", [](Testbed& t) {
			t.training_data_available = false;
			t.nerf.training.dataset.metadata.clear();
		})
		.def("init_window", [](Testbed&, int, int, bool, bool) { throw std::runtime_error("No GUI on the MI355X build (headless only)."); },
		     py::arg("width"), py::arg("height"), py::arg("hidden") = false, py::arg("second_window") = false)
		.def("want_repl", [](Testbed&) { return false; })
		.def("frame", &Testbed::frame, py::call_guard<py::gil_scoped_release>())
		.def("render",
		     [](Testbed& t, int width, int height, int spp, bool linear, float start_t, float end_t, float fps, float shutter) {
			     (void)start_t, (void)end_t, (void)fps, (void)shutter;  // camera paths are out of scope
			     if (width <= 0 || height <= 0) throw std::runtime_error("render: invalid resolution");
			     // render_to_cpu (src/python_api.cu:124-202): the frame is read back straight into the array's
			     // page-locked memory (pooled; returned to the pool when the array is freed)
			     py::array_t<float> a = pinned_frame(height, width);
			     {
				     py::gil_scoped_release rel;
				     t.render_into(a.mutable_data(), width, height, spp, linear, 0, 1, 8, true);
			     }
			     return a;
		     },
		     py::arg("width") = 1920, py::arg("height") = 1080, py::arg("spp") = 1, py::arg("linear") = true,
		     py::arg("start_t") = -1.f, py::arg("end_t") = -1.f, py::arg("fps") = 30.f, py::arg("shutter_fraction") = 1.0f)
		.def("render_shard",
		     [](Testbed& t, int width, int height, int spp, bool linear, uint32_t shard_index, uint32_t shard_count,
		        uint32_t shard_rows) {
			     std::vector<float> img;
			     {
				     py::gil_scoped_release rel;
				     img = t.render(width, height, spp, linear, shard_index, shard_count, shard_rows);
			     }
			     py::array_t<float> a({height, width, 4});
			     std::memcpy(a.mutable_data(), img.data(), img.size() * sizeof(float));
			     return a;
		     },
		     py::arg("width"), py::arg("height"), py::arg("spp"), py::arg("linear"), py::arg("shard_index"),
		     py::arg("shard_count"), py::arg("shard_rows") = 8u)
		.def("render_to_device",
		     [](Testbed& t, int width, int height, int spp, bool linear, uint32_t shard_index, uint32_t shard_count,
		        uint32_t shard_rows) {
			     py::gil_scoped_release rel;
			     t.render(width, height, spp, linear, shard_index, shard_count, shard_rows, false);
			     return (uintptr_t)t.render_frame_buffer();
		     },
		     "Render into the device frame buffer only (no PCIe readback); returns its device address.",
		     py::arg("width") = 1920, py::arg("height") = 1080, py::arg("spp") = 1, py::arg("linear") = true,
		     py::arg("shard_index") = 0u, py::arg("shard_count") = 1u, py::arg("shard_rows") = 8u)
		.def("train", &Testbed::train, py::call_guard<py::gil_scoped_release>(), py::arg("batch_size"))
		.def("reset", &Testbed::reset_network, py::arg("reset_density_grid") = true)
		.def("reset_accumulation", [](Testbed& t, bool, bool) { t.reset_accumulation(); }, py::arg("due_to_camera_movement") = false,
		     py::arg("immediate_redraw") = true)
		.def("reload_network_from_file", &Testbed::reload_network_from_file, py::arg("path") = "")
		.def("reload_network_from_json",
		     [](Testbed& t, py::object j, const std::string& base) { t.reload_network_from_json(json_from_py(j), base); },
		     py::arg("json"), py::arg("config_base_path") = "")
		.def_property_readonly("network_config", [](const Testbed& t) { return json_to_py(t.network_config()); })
		.def_property_readonly("per_level_scale", [](const Testbed& t) { return t.network_abi_config().per_level_scale; })
		.def("n_params", [](const Testbed& t) -> size_t {
			if (!t.model()) return 0;
			ngp_model_info i{};
			ngp_model_get_info(t.model(), &i);
			return i.n_params;
		})
		.def("n_encoding_params", [](const Testbed& t) -> size_t {
			if (!t.model()) return 0;
			ngp_model_info i{};
			ngp_model_get_info(t.model(), &i);
			return i.n_params - i.n_mlp_params;
		})
		.def("save_snapshot", &Testbed::save_snapshot, py::arg("path"), py::arg("include_optimizer_state") = false,
		     py::arg("compress") = true)
		.def("load_snapshot", &Testbed::load_snapshot, py::arg("path"))
		.def("load_file", &Testbed::load_file, py::arg("path"))
		.def_readwrite("background_color", &Testbed::background_color)
		.def_readwrite("shall_train", &Testbed::shall_train)
		.def_readwrite("shall_train_encoding", &Testbed::train_encoding)
		.def_readwrite("shall_train_network", &Testbed::train_network)
		.def_readwrite("render_groundtruth", &Testbed::render_ground_truth)
		.def_readwrite("render_ground_truth", &Testbed::render_ground_truth)
		.def_readwrite("render_near_distance", &Testbed::render_near_distance)
		.def_readwrite("exposure", &Testbed::exposure)
		.def_readwrite("render_mode", &Testbed::render_mode)
		.def_readwrite("aperture_size", &Testbed::aperture_size)
		.def_readwrite("dof", &Testbed::aperture_size)
		.def_readwrite("slice_plane_z", &Testbed::slice_plane_z)
		.def_property("render_aabb", [](const Testbed& t) { return BoundingBox{t.render_aabb_min, t.render_aabb_max}; },
		              [](Testbed& t, const BoundingBox& b) {
			              t.render_aabb_min = b.min;
			              t.render_aabb_max = b.max;
		              })
		.def_property("render_aabb_to_local",
		              [](const Testbed& t) {
			              py::array_t<float> a({3, 3});
			              std::memcpy(a.mutable_data(), t.render_aabb_to_local.data(), 9 * sizeof(float));
			              return a;
		              },
		              [](Testbed& t, py::array_t<float, py::array::c_style | py::array::forcecast> a) {
			              if (a.size() != 9) throw std::runtime_error("render_aabb_to_local must be a 3x3 matrix");
			              std::memcpy(t.render_aabb_to_local.data(), a.data(), 9 * sizeof(float));
		              })
		.def_property("scale", [](const Testbed& t) { return t.scale; },
		              [](Testbed& t, float s) {
			              // Testbed::set_scale: move the camera along the view direction, keeping look_at fixed
			              const float prev = t.scale;
			              for (int k = 0; k < 3; ++k) t.camera.m[9 + k] += (prev - s) * t.camera.m[6 + k];
			              t.scale = s;
		              })
		.def_property("aabb", [](const Testbed& t) { return BoundingBox{t.aabb_min, t.aabb_max}; },
		              [](Testbed& t, const BoundingBox& b) {
			              t.aabb_min = b.min;
			              t.aabb_max = b.max;
		              })
		.def_property("fov", &Testbed::fov, &Testbed::set_fov)
		.def_property("fov_xy", &Testbed::fov_xy, &Testbed::set_fov_xy)
		.def_property("raw_aabb", [](const Testbed& t) { return BoundingBox{t.raw_aabb_min, t.raw_aabb_max}; },
		              [](Testbed& t, const BoundingBox& b) {
			              t.raw_aabb_min = b.min;
			              t.raw_aabb_max = b.max;
		              })
		.def_readwrite("up_dir", &Testbed::up_dir)
		.def("crop_box", [](const Testbed& t, bool nerf_space) { return mat43_to_numpy(t.crop_box(nerf_space)); },
		     py::arg("nerf_space") = true)
		.def("set_crop_box",
		     [](Testbed& t, py::array_t<float, py::array::c_style | py::array::forcecast> m, bool nerf_space) {
			     t.set_crop_box(numpy_to_mat43(m), nerf_space);
		     },
		     py::arg("matrix"), py::arg("nerf_space") = true)
		.def("crop_box_corners", &Testbed::crop_box_corners, py::arg("nerf_space") = true)
		.def("compute_image_mse", &Testbed::compute_image_mse, py::arg("quantize") = false)
		.def_readwrite("fov_axis", &Testbed::fov_axis)
		.def_readwrite("zoom", &Testbed::zoom)
		.def_readwrite("screen_center", &Testbed::screen_center)
		.def_readwrite("relative_focal_length", &Testbed::relative_focal_length)
		.def_readwrite("training_batch_size", &Testbed::training_batch_size)
		.def_readwrite("train_full_forward", &Testbed::train_full_forward)
		.def_readwrite("deterministic", &Testbed::deterministic,
		               "Bit-reproducible training steps: hash-grid gradients summed in 64-bit fixed point "
		               "(ngp_train_args.deterministic) instead of fp16 atomics")
		.def_readwrite("max_level_rand_training", &Testbed::m_max_level_rand_training)
		.def_property_readonly("distributed", &Testbed::distributed)
		// ngp_tuning (include/ngp_hip.h) as a dict; unknown keys are an error, missing keys keep their value
		.def("get_tuning",
		     [](const Testbed& t) {
			     const ngp_tuning& u = t.tuning();
			     py::dict d;
#define NGP_TUNING_FIELD(f) d[#f] = u.f;
			     NGP_TUNING_FIELDS
#undef NGP_TUNING_FIELD
			     return d;
		     })
		.def("set_tuning",
		     [](Testbed& t, py::dict d) {
			     ngp_tuning u = t.tuning();
			     for (auto kv : d) {
				     const std::string k = py::str(kv.first);
				     bool known = false;
#define NGP_TUNING_FIELD(f) \
	if (k == #f) { u.f = kv.second.cast<decltype(u.f)>(); known = true; }
				     NGP_TUNING_FIELDS
#undef NGP_TUNING_FIELD
				     if (!known) throw std::invalid_argument("unknown tuning field '" + k + "'");
			     }
			     t.set_tuning(u);
		     })
		.def("set_nerf_camera_matrix",
		     [](Testbed& t, py::array_t<float, py::array::c_style | py::array::forcecast> c) {
			     auto rm = numpy_to_rowmajor34(c);
			     t.camera = t.nerf.training.dataset.nerf_matrix_to_ngp(rm.data());
		     })
		.def("set_camera_to_training_view", &Testbed::set_camera_to_training_view)
		.def("first_training_view", [](Testbed& t) { t.set_camera_to_training_view(0); })
		.def("last_training_view", [](Testbed& t) { t.set_camera_to_training_view((int)t.nerf.training.dataset.n_images - 1); })
		.def("previous_training_view", [](Testbed& t) {
			const int n = (int)t.nerf.training.dataset.n_images;
			t.set_camera_to_training_view((t.nerf.training.view + n - 1) % std::max(n, 1));
		})
		.def("next_training_view", [](Testbed& t) {
			const int n = (int)t.nerf.training.dataset.n_images;
			t.set_camera_to_training_view((t.nerf.training.view + 1) % std::max(n, 1));
		})
		.def("reset_camera", &Testbed::reset_camera)
		.def_property("camera_matrix", [](const Testbed& t) { return mat43_to_numpy(t.camera); },
		              [](Testbed& t, py::array_t<float, py::array::c_style | py::array::forcecast> a) { t.camera = numpy_to_mat43(a); })
		.def_property("view_dir", [](const Testbed& t) { return t.camera.col(2); },
		              [](Testbed& t, vec3 d) {
			              // Testbed::set_view_dir: re-orthonormalise right/down around the new forward
			              const float n = std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
			              for (auto& x : d) x /= n;
			              const vec3 look = {t.camera.m[9] + d[0] * t.scale, t.camera.m[10] + d[1] * t.scale, t.camera.m[11] + d[2] * t.scale};
			              (void)look;
			              t.camera.set_col(2, d);
		              })
		.def_property("look_at",
		              [](const Testbed& t) {
			              return vec3{t.camera.m[9] + t.camera.m[6] * t.scale, t.camera.m[10] + t.camera.m[7] * t.scale,
			                          t.camera.m[11] + t.camera.m[8] * t.scale};
		              },
		              [](Testbed& t, vec3 p) {
			              for (int k = 0; k < 3; ++k) t.camera.m[9 + k] = p[k] - t.camera.m[6 + k] * t.scale;
		              })
		.def_property_readonly("loss", [](const Testbed& t) { return t.loss; })
		.def_readonly("training_step", &Testbed::training_step)
		.def_readwrite("color_space", &Testbed::color_space)
		.def_readwrite("tonemap_curve", &Testbed::tonemap_curve)
		.def_readwrite("snap_to_pixel_centers", &Testbed::snap_to_pixel_centers)
		.def_readwrite("root_dir", &Testbed::root_dir)
		.def_readwrite("seed", &Testbed::seed)
		.def_readonly("data_path", &Testbed::data_path)
		.def_readonly("training_ms", &Testbed::training_ms)
		.def_readonly("training_prep_ms", &Testbed::training_prep_ms)
		.def_readonly("render_ms", &Testbed::render_ms)
		.def_property_readonly("nerf", py::cpp_function([](Testbed& t) { return NerfView{&t}; }, py::keep_alive<0, 1>()))
		.def("density_grid", [](const Testbed& t) {
			auto g = t.density_grid();
			return py::array_t<float>(g.size(), g.data());
		})
		// compute_and_save_png_slices (src/python_api.cu:451-459): the density mosaic of NerfNetwork::density on a lattice
		// over aabb (empty: the render aabb), written to filename + ".density_slices_{x}x{y}x{z}.png"; returns the lattice
		.def("compute_and_save_png_slices",
		     [](Testbed& t, const std::string& filename, int res, const BoundingBox& aabb, float thresh, float density_range,
		        bool flip) {
			     std::array<int, 3> r;
			     {
				     py::gil_scoped_release rel;
				     r = t.compute_and_save_png_slices(filename, res, aabb.min, aabb.max, thresh, density_range, flip);
			     }
			     py::array_t<int> a(3);
			     std::copy(r.begin(), r.end(), a.mutable_data());
			     return a;
		     },
		     py::arg("filename"), py::arg("resolution") = 256, py::arg("aabb") = BoundingBox{},
		     py::arg("thresh") = std::numeric_limits<float>::max(), py::arg("density_range") = 4.f,
		     py::arg("flip_y_and_z_axes") = false,
		     "Compute & save a PNG file representing the 3D density field from the current NeRF model.")
		// get_density_on_grid (src/testbed_nerf.cu:3026-3075) as a [z][y][x] array (an MI355X-side accessor for tests)
		.def("density_on_grid",
		     [](Testbed& t, std::array<int, 3> res3d, const BoundingBox& aabb) {
			     vec3 lo = aabb.min, hi = aabb.max;
			     mat3 to_local = MAT3_IDENTITY;
			     if (aabb.is_empty()) {
				     lo = t.render_aabb_min;
				     hi = t.render_aabb_max;
				     to_local = t.render_aabb_to_local;
			     }
			     std::vector<float> d;
			     {
				     py::gil_scoped_release rel;
				     d = t.density_on_grid(res3d, lo, hi, to_local);
			     }
			     py::array_t<float> a({(py::ssize_t)res3d[2], (py::ssize_t)res3d[1], (py::ssize_t)res3d[0]});
			     std::memcpy(a.mutable_data(), d.data(), d.size() * sizeof(float));
			     return a;
		     },
		     py::arg("resolution"), py::arg("aabb") = BoundingBox{})
		.def_readwrite("mesh_thresh", &Testbed::mesh_thresh)
		.def("density_grid_bitfield", [](const Testbed& t) {
			auto b = t.density_grid_bitfield();
			return py::array_t<uint8_t>(b.size(), b.data());
		})
		.def("last_train_stats", [](const Testbed& t) {
			const ngp_train_stats s = t.last_stats();
			py::dict d;
			d["loss"] = s.loss;
			d["measured_batch_size"] = s.measured_batch_size;
			d["measured_batch_size_before_compaction"] = s.measured_batch_size_before_compaction;
			d["rays_per_batch"] = t.nerf.training.counters_rgb.rays_per_batch;
			d["n_rays"] = s.n_rays;
			d["forward_early_stop_violations"] = s.forward_early_stop_violations;
			d["sample_capacity_overflow"] = s.sample_capacity_overflow;
			d["forward_early_stop_violations_total"] = t.forward_early_stop_violations;
			return d;
		})
		.def("sync", &Testbed::sync)
		// the learned distortion map as a [res_y][res_x][2] array (an MI355X-side accessor for tests)
		.def_property_readonly("distortion_map", [](const Testbed& t) {
			const ivec2 r = t.distortion_resolution();
			std::vector<float> p = t.distortion_map();
			py::array_t<float> a({(py::ssize_t)r[1], (py::ssize_t)r[0], (py::ssize_t)2});
			std::copy(p.begin(), p.end(), a.mutable_data());
			return a;
		})
		.def_property_readonly("model_handle", [](const Testbed& t) { return (uintptr_t)t.model(); })
		.def_property_readonly("stream_handle", [](const Testbed& t) { return (uintptr_t)t.stream(); })
		// multi-GPU: one Testbed per rank (torchrun); gradients/grid all-reduced over RCCL
		.def_static("nccl_unique_id", []() { return py::bytes(Testbed::nccl_unique_id()); })
		.def("init_distributed",
		     [](Testbed& t, int rank, int world, py::bytes uid) { t.init_distributed(rank, world, std::string(uid)); },
		     py::arg("rank"), py::arg("world_size"), py::arg("unique_id"))
		.def("init_distributed_host",
		     [](Testbed& t, int rank, int world, py::function fn) {
			     // fn(array, op) reduces a host numpy array in place (op "sum" / "max"); called with the GIL
			     // re-acquired, since train() / frame() release it
			     auto hold = std::make_shared<py::function>(std::move(fn));
			     t.init_distributed_host(rank, world, [hold](void* p, size_t n, int dtype, int op) {
				     py::gil_scoped_acquire gil;
				     // dtype 0 f32, 1 f16, 2 i32 (per-rank totals), 3 i64 (deterministic fixed-point gradients)
				     static const char* names[4] = {"float32", "float16", "int32", "int64"};
				     static const py::ssize_t sizes[4] = {4, 2, 4, 8};
				     py::array a(py::dtype(names[dtype]), {(py::ssize_t)n}, {sizes[dtype]}, p, py::none());
				     (*hold)(a, op ? "max" : "sum");
			     });
		     },
		     "Data-parallel Testbed whose collectives are staged through host memory and reduced by fn "
		     "(test backend: several processes sharing one GPU over torch.distributed/gloo).",
		     py::arg("rank"), py::arg("world_size"), py::arg("allreduce"))
		.def("render_distributed",
		     [](Testbed& t, int width, int height, int spp, bool linear, bool copy_to_host) -> py::object {
			     std::vector<float> img;
			     {
				     py::gil_scoped_release rel;
				     img = t.render_distributed(width, height, spp, linear, copy_to_host);
			     }
			     if (img.empty()) return py::none();
			     py::array_t<float> a({height, width, 4});
			     std::memcpy(a.mutable_data(), img.data(), img.size() * sizeof(float));
			     return a;
		     },
		     "One frame row-sharded over the ranks and gathered to rank 0 (None on the other ranks).",
		     py::arg("width") = 1920, py::arg("height") = 1080, py::arg("spp") = 1, py::arg("linear") = true,
		     py::arg("copy_to_host") = true)
		.def_property_readonly("rank", &Testbed::rank)
		.def_property_readonly("world_size", &Testbed::world_size);
}
