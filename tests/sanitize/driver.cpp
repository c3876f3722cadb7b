// AddressSanitizer / UBSan driver for the host code (test infrastructure, CPU only): the JSON and
// MessagePack parsers, the PNG decoder and the CPU oracle, built with -fsanitize=address,undefined
// by tests/test_sanitizers.py.  Malformed inputs must fail with an exception / false, never touch
// memory out of bounds.
//
// Usage: driver <json files...> -- <png files...>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iterator>
#include <random>
#include <stdexcept>
#include <string>
#include <vector>

#include "json.h"
#include "ngp_hip.h"
#include "png.h"

extern "C" {
void oref_set_threads(int n);
void* oref_model_create(const ngp_network_config* cfg);
void oref_model_destroy(void* m);
uint64_t oref_model_n_params(void* m);
uint64_t oref_model_n_mlp_params(void* m);
void oref_model_set_params(void* m, const float* p);
void oref_model_set_inference_params(void* m, const float* ema);
void oref_encode(void* m, const float* pos, uint32_t stride, uint32_t n, float* enc, int use_inf);
void oref_infer(void* m, const float* coords, uint32_t fpc, uint32_t n, float* out, int use_inf);
int oref_train_step(void* m, const ngp_train_args* a);
void oref_optimizer_step(void* m, uint32_t step, int opt_mlp, int opt_enc);
void oref_density_grid_set(void* m, const float* grid, uint32_t n);
void oref_density_grid_bitfield(void* m, uint32_t max_cascade);
int oref_render(void* m, const ngp_render_args* a, float* frame, float* depth);
const char* oref_last_error(void);
}

static std::vector<uint8_t> read_file(const std::string& p) {
	std::ifstream f(p, std::ios::binary);
	return std::vector<uint8_t>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

static int n_checks = 0;

static void fuzz_json(const std::string& text, std::mt19937& rng) {
	const ngp::Json j = ngp::Json::parse(text);
	const std::string d = j.dump();
	const ngp::Json back = ngp::Json::parse(d);
	if (back.dump() != d) throw std::runtime_error("JSON dump round trip differs");
	const std::vector<uint8_t> mp = j.to_msgpack();
	if (ngp::Json::from_msgpack(mp.data(), mp.size()).dump() != d) throw std::runtime_error("msgpack round trip differs");
	// truncations and byte flips: exceptions are fine, memory errors are not
	for (int k = 0; k < 200; ++k) {
		std::string t = text.substr(0, rng() % (text.size() + 1));
		if (k & 1 && !t.empty()) t[rng() % t.size()] = (char)(rng() & 0xff);
		try { (void)ngp::Json::parse(t); } catch (const std::exception&) {}
		std::vector<uint8_t> m(mp.begin(), mp.begin() + rng() % (mp.size() + 1));
		if (k & 1 && !m.empty()) m[rng() % m.size()] ^= (uint8_t)(1u << (rng() % 8));
		try { (void)ngp::Json::from_msgpack(m.data(), m.size()); } catch (const std::exception&) {}
		++n_checks;
	}
}

static void fuzz_png(const std::vector<uint8_t>& data, std::mt19937& rng) {
	std::vector<uint8_t> rgba;
	int w = 0, h = 0;
	std::string err;
	if (!ngp::decode_png_memory(data.data(), data.size(), rgba, w, h, err)) throw std::runtime_error("PNG decode failed: " + err);
	if (rgba.size() != (size_t)w * h * 4) throw std::runtime_error("PNG size");
	for (int k = 0; k < 40; ++k) {
		std::vector<uint8_t> t(data.begin(), data.begin() + rng() % (data.size() + 1));
		if (k & 1 && t.size() > 8) t[8 + rng() % (t.size() - 8)] ^= (uint8_t)(1u << (rng() % 8));
		(void)ngp::decode_png_memory(t.data(), t.size(), rgba, w, h, err);
		++n_checks;
	}
}

// the oracle on a tiny scene: encode, infer, a training step with Adam, a 16 x 16 render
static void run_oracle() {
	oref_set_threads(1);
	ngp_network_config c{};
	c.n_levels = 4; c.n_features_per_level = 2; c.log2_hashmap_size = 14; c.base_resolution = 16;
	c.per_level_scale = 1.5f; c.n_neurons = 16; c.density_hidden_layers = 1; c.rgb_hidden_layers = 2;
	c.rgb_activation = 2; c.density_activation = 3;
	c.learning_rate = 1e-2f; c.beta1 = 0.9f; c.beta2 = 0.99f; c.epsilon = 1e-15f; c.l2_reg = 1e-6f;
	c.ema_decay = 0.95f; c.decay_start = 20000; c.decay_interval = 10000; c.decay_base = 0.33f;
	void* m = oref_model_create(&c);
	if (!m) throw std::runtime_error("oracle model");
	const size_t n = oref_model_n_params(m), n_mlp = oref_model_n_mlp_params(m);
	std::mt19937 rng(3);
	std::uniform_real_distribution<float> U(-0.3f, 0.3f), P(0.f, 1.f);
	std::vector<float> p(n);
	for (size_t i = 0; i < n; ++i) p[i] = i < n_mlp ? U(rng) : 1e-2f * U(rng);
	oref_model_set_params(m, p.data());
	oref_model_set_inference_params(m, p.data());
	const uint32_t S = 300;
	std::vector<float> coords(8 * S), enc(4 * 2 * S), out(4 * S);
	for (uint32_t i = 0; i < S; ++i)
		for (int k = 0; k < 7; ++k) coords[8 * i + k] = P(rng);
	oref_encode(m, coords.data(), 8, S, enc.data(), 0);
	oref_infer(m, coords.data(), 8, S, out.data(), 1);
	// occupancy: a solid ball
	std::vector<float> grid(128 * 128 * 128, 0.0f);
	for (size_t i = 0; i < grid.size(); i += 3) grid[i] = 1.0f;
	oref_density_grid_set(m, grid.data(), (uint32_t)grid.size());
	oref_density_grid_bitfield(m, 0);
	// two 16 x 16 images looking at the centre
	const uint32_t W = 16, H = 16;
	std::vector<uint32_t> px[2];
	ngp_image im[2];
	std::memset(im, 0, sizeof(im));
	for (int k = 0; k < 2; ++k) {
		px[k].resize(W * H);
		for (auto& t : px[k]) t = rng() | 0xff000000u;
		im[k].pixels = (uint64_t)(uintptr_t)px[k].data();
		im[k].width = W; im[k].height = H;
		im[k].focal_length[0] = im[k].focal_length[1] = 20.0f;
		im[k].principal_point[0] = im[k].principal_point[1] = 0.5f;
		const float z = k ? -1.0f : 1.0f;
		const float xf[12] = {1, 0, 0, 0, z, 0, 0, 0, -z, 0.5f, 0.5f, 0.5f + 1.5f * z};  // columns: right, up, fwd, origin
		std::memcpy(im[k].xform, xf, sizeof(xf));
	}
	ngp_train_args a{};
	a.images = im; a.n_images = 2; a.n_rays = 64; a.target_batch_size = 1 << 12; a.max_samples = 1 << 14;
	a.rng_state = 0x853c49e6748fea9bull; a.rng_inc = 0xda3e39cb94b95bdbull;
	for (int k = 0; k < 3; ++k) { a.aabb_min[k] = 0.f; a.aabb_max[k] = 1.f; }
	a.loss_type = 4; a.random_bg_color = 1; a.snap_to_pixel_centers = 1; a.near_distance = 0.1f;
	a.optimize_mlp = 1; a.optimize_encoding = 1;
	std::vector<float> err(2 * 8 * 8, 0.f), sharp(2 * 4 * 4, 0.5f), sgrid((size_t)8 * 128 * 128 * 128, 0.f), depth(W * H, 1.5f);
	im[0].depth = (uint64_t)(uintptr_t)depth.data();
	a.error_map = err.data(); a.error_map_res[0] = a.error_map_res[1] = 8;
	a.sharpness_data = sharp.data(); a.sharpness_res[0] = a.sharpness_res[1] = 4; a.sharpness_grid = sgrid.data();
	a.sharpness_grid_clear = 1;
	a.depth_supervision_lambda = 0.5f; a.depth_loss_type = 1;
	if (oref_train_step(m, &a) != 0) throw std::runtime_error(std::string("oracle train step: ") + oref_last_error());
	oref_optimizer_step(m, 0, 1, 1);
	ngp_render_args r{};
	r.width = W; r.height = H;
	std::memcpy(r.camera, im[0].xform, sizeof(r.camera));
	r.focal_length[0] = r.focal_length[1] = 20.f;
	r.screen_center[0] = r.screen_center[1] = 0.5f;
	for (int k = 0; k < 3; ++k) { r.aabb_min[k] = r.train_aabb_min[k] = 0.f; r.aabb_max[k] = r.train_aabb_max[k] = 1.f; }
	r.min_transmittance = 0.01f; r.use_inference_params = 1; r.shard_count = 1; r.shard_rows = 8;
	std::vector<float> frame(4 * W * H), dbuf(W * H);
	if (oref_render(m, &r, frame.data(), dbuf.data()) != 0) throw std::runtime_error("oracle render");
	for (float v : frame)
		if (!std::isfinite(v)) throw std::runtime_error("non-finite render");
	oref_model_destroy(m);
	++n_checks;
}

int main(int argc, char** argv) {
	std::vector<std::string> jsons, pngs;
	bool png_part = false;
	for (int i = 1; i < argc; ++i) {
		const std::string s = argv[i];
		if (s == "--") { png_part = true; continue; }
		(png_part ? pngs : jsons).push_back(s);
	}
	std::mt19937 rng(1);
	try {
		for (const auto& p : jsons) {
			const std::vector<uint8_t> b = read_file(p);
			fuzz_json(std::string(b.begin(), b.end()), rng);
		}
		for (const auto& p : pngs) fuzz_png(read_file(p), rng);
		run_oracle();
	} catch (const std::exception& e) {
		fprintf(stderr, "FAILED: %s\n", e.what());
		return 1;
	}
	printf("sanitized host checks ok: %d\n", n_checks);
	return 0;
}
