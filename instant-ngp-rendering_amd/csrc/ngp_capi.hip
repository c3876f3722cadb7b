// ngp_capi.hip — the C-ABI of libngp_hip.so (see include/ngp_hip.h).
//
// Host orchestration only: parameter layout, level tables, buffer ownership
// and the launch sequences of the kernels in hashgrid/mlp/train/density_grid/
// render.hip.  Every entry point converts C++ exceptions into an ngp_status +
// thread-local message, the C-ABI analogue of the reference's
// CUDA_CHECK_THROW -> std::runtime_error -> Python RuntimeError chain.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include <rccl/rccl.h>

#include "ngp_internal.h"

namespace ngp {
void run_grid_evaluate(ngp_model* m, const ngp_grid_args* a, hipStream_t s);
void run_grid_finish(ngp_model* m, const ngp_grid_args* a, hipStream_t s);
void run_density_on_grid(ngp_model* m, const ngp_grid_query* q, float* out, hipStream_t s);
void run_grid_bitfield(ngp_model* m, uint32_t max_cascade, hipStream_t s);
void grid_reserve(ngp_model* m, uint32_t n_cascades, uint32_t n_samples);
void run_render(ngp_model* m, const ngp_render_args* a, float* frame, float* depth_buffer, hipStream_t s);
void run_error_map_cdf(const float* error_map, uint32_t n_images, uint32_t rx, uint32_t ry, float* cdf_x_cond_y,
                       float* cdf_y, float* cdf_img, hipStream_t s);
void run_accumulate_tonemap(const float* frame, float* accum, float* out, uint32_t W, uint32_t H, uint32_t spp,
                            int color_space, float exposure, const float* bg, int output_srgb, hipStream_t s);
}  // namespace ngp

using namespace ngp;

static thread_local std::string g_last_error;

template <class F>
static ngp_status guarded(F&& f) {
	try {
		f();
		return NGP_OK;
	} catch (const std::invalid_argument& e) {
		g_last_error = e.what();
		return NGP_ERR_INVALID;
	} catch (const std::bad_alloc& e) {
		g_last_error = e.what();
		return NGP_ERR_OOM;
	} catch (const std::exception& e) {
		g_last_error = e.what();
		return std::string(e.what()).rfind("HIP error", 0) == 0 ? NGP_ERR_HIP : NGP_ERR_UNSUPPORTED;
	}
}

static void require(bool cond, const char* msg) {
	if (!cond) throw std::invalid_argument(msg);
}

static hipStream_t S(ngp_stream s) { return reinterpret_cast<hipStream_t>(s); }

// ngp_tuning.encode_streaming: 0 = the default (non-temporal encoding stores: -2 % render frame time,
// tools/render_ab.py), 1 = plain stores.  ngp_tuning.encode_xcd_regions: 0 = the default (contiguous XCD regions:
// -1.1 % render frame time in a same-weights A/B), 1 = off.
static void apply_encode_tuning(LevelTable& lt, const ngp_tuning& t) {
	lt.streaming = t.encode_streaming == 0 ? 1u : 0u;
	lt.regions = t.encode_xcd_regions == 0 ? 1u : 0u;
}

static void validate_tuning(const ngp_tuning* t) {
	require(t != nullptr, "null argument");
	require(t->render_pipelines <= RenderScratch::MAX_PIPES, "render_pipelines must be 0..4");
	require(t->render_pass_samples <= (16u << 20), "render_pass_samples must be <= 2^24");
	require(t->render_lag == 0 || (t->render_lag >= 2 && t->render_lag <= 4), "render_lag must be 0 or 2..4");
	require(t->render_composite_block == 0 || t->render_composite_block == 256 || t->render_composite_block == 512 ||
	            t->render_composite_block == 1024,
	        "render_composite_block must be 0, 256, 512 or 1024");
	require(t->render_generate_block == 0 || t->render_generate_block == 256 || t->render_generate_block == 512,
	        "render_generate_block must be 0, 256 or 512");
	require(t->encode_dense_records <= 1, "encode_dense_records must be 0 or 1");
	require(t->mlp_workgroups_per_cu <= 32, "mlp_workgroups_per_cu must be <= 32");
	require(t->encode_streaming <= 1, "encode_streaming must be 0 or 1");
	require(t->grid_unsorted <= 2, "grid_unsorted must be 0, 1 or 2");
	require(t->render_mlp_tile == 0 || t->render_mlp_tile == 1 || t->render_mlp_tile == 2 || t->render_mlp_tile == 4,
	        "render_mlp_tile must be 0, 1, 2 or 4");
	require(t->encode_xcd_regions <= 1, "encode_xcd_regions must be 0 or 1");
	require(t->render_skip_unfilled <= 2, "render_skip_unfilled must be 0, 1 or 2");
	require(t->render_exit_cap <= 2, "render_exit_cap must be 0, 1 or 2");
	require(t->render_priority < 64, "render_priority must be < 64 (three 2-bit priorities)");
	require(t->render_host_frame <= 2, "render_host_frame must be 0, 1 or 2");
	require(t->train_chunk_lanes == 0 || (t->train_chunk_lanes >= 4 && t->train_chunk_lanes <= 64 &&
	                                      (t->train_chunk_lanes & (t->train_chunk_lanes - 1)) == 0),
	        "train_chunk_lanes must be 0 or a power of two in [4, 64]");
	require(t->render_mlp_pipeline <= 3, "render_mlp_pipeline must be 0, 1, 2 or 3");
	require(t->train_sampler_lanes == 0 || (t->train_sampler_lanes >= 8 && t->train_sampler_lanes <= 64 &&
	                                        (t->train_sampler_lanes & (t->train_sampler_lanes - 1)) == 0),
	        "train_sampler_lanes must be 0 or a power of two in [8, 64]");
}

// tcnn GridEncodingTemplated constructor (level table); per_level_scale resolved on the host.
static void build_level_table(ngp_model* m) {
	const ngp_network_config& c = m->cfg;
	LevelTable& lt = m->lt;
	lt.n_levels = c.n_levels;
	lt.F = c.n_features_per_level;
	const float log2_pls = std::log2(c.per_level_scale);
	uint32_t offset = 0;
	for (uint32_t l = 0; l < c.n_levels; ++l) {
		const float scale = std::exp2((float)l * log2_pls) * (float)c.base_resolution - 1.0f;
		const uint32_t res = (uint32_t)std::ceil(scale) + 1;
		const uint32_t max_params = 0xFFFFFFFFu / 2;
		const double dense = (double)res * res * res;
		uint32_t params = dense > (double)max_params ? max_params : res * res * res;
		params = next_multiple(params, 8);
		params = std::min(params, 1u << c.log2_hashmap_size);
		lt.scale[l] = scale;
		lt.res[l] = res;
		lt.offset[l] = offset;
		lt.size[l] = params;
		lt.hashed[l] = dense > (double)params ? 1u : 0u;
		offset += params;
	}
	m->n_grid_params = (uint64_t)offset * lt.F;
	apply_encode_tuning(lt, m->tuning);
}

static void build_layers(ngp_model* m) {
	const ngp_network_config& c = m->cfg;
	const uint32_t W = c.n_neurons;
	std::vector<std::pair<uint32_t, uint32_t>> dims;  // (out, in)
	dims.push_back({W, m->enc_pad});
	for (uint32_t h = 1; h < c.density_hidden_layers; ++h) dims.push_back({W, W});
	dims.push_back({16, W});
	m->n_density_layers = (uint32_t)dims.size();
	// rgb_network_input_width = next_multiple(density out 16 + dir encoding (SH 16 + n_extra_dims Identity), 16)
	// (nerf_network.h:84, 93)
	dims.push_back({W, next_multiple(32u + c.n_extra_dims, 16u)});
	for (uint32_t h = 1; h < c.rgb_hidden_layers; ++h) dims.push_back({W, W});
	dims.push_back({16, W});  // 3 used, padded to 16 (tcnn output alignment)
	require(dims.size() <= MAX_LAYERS, "too many MLP layers");
	m->n_layers = (uint32_t)dims.size();
	uint64_t off = 0;
	for (uint32_t l = 0; l < m->n_layers; ++l) {
		m->layers[l].out = dims[l].first;
		m->layers[l].in = dims[l].second;
		m->layers[l].param_offset = off;
		off += (uint64_t)dims[l].first * dims[l].second;
	}
	m->n_mlp_params = off;
}

static void upload_init_params(ngp_model* m, uint64_t seed) {
	std::vector<float> p(m->n_params);
	pcg32 rng(seed);
	for (uint32_t l = 0; l < m->n_layers; ++l) {
		const Layer& L = m->layers[l];
		const float scale = std::sqrt(6.0f / (float)(L.in + L.out));  // Xavier uniform (tcnn FullyFusedMLP)
		for (uint64_t i = 0; i < (uint64_t)L.in * L.out; ++i) p[L.param_offset + i] = (rng.next_float() * 2.0f - 1.0f) * scale;
	}
	for (uint64_t i = 0; i < m->n_grid_params; ++i) p[m->n_mlp_params + i] = (rng.next_float() * 2.0f - 1.0f) * 1e-4f;
	NGP_HIP_CHECK(hipMemcpy(m->params32.ptr, p.data(), m->n_params * sizeof(float), hipMemcpyHostToDevice));
}

static void refresh_derived(ngp_model* m, bool reset_optimizer, hipStream_t s) {
	launch_params_to_half(m->params32.ptr, m->params16.ptr, m->n_params, s);
	if (reset_optimizer) {
		NGP_HIP_CHECK(hipMemcpyAsync(m->ema32.ptr, m->params32.ptr, m->n_params * sizeof(float), hipMemcpyDeviceToDevice, s));
		NGP_HIP_CHECK(hipMemcpyAsync(m->infer16.ptr, m->params16.ptr, m->n_params * sizeof(__half), hipMemcpyDeviceToDevice, s));
		NGP_HIP_CHECK(hipMemsetAsync(m->adam_m.ptr, 0, m->n_params * sizeof(float), s));
		NGP_HIP_CHECK(hipMemsetAsync(m->adam_v.ptr, 0, m->n_params * sizeof(float), s));
		NGP_HIP_CHECK(hipMemsetAsync(m->adam_steps.ptr, 0, m->n_params * sizeof(uint32_t), s));
		NGP_HIP_CHECK(hipMemsetAsync(m->grads.ptr, 0, m->n_params * sizeof(float), s));
		NGP_HIP_CHECK(hipMemsetAsync(m->grid_grads16.ptr, 0, m->n_grid_params * sizeof(__half), s));
		m->ema_step = 0;
	} else {
		launch_params_to_half(m->ema32.ptr, m->infer16.ptr, m->n_params, s);
	}
	pack_mlp_fragments(m, m->params16.ptr, m->frag_train.ptr, s);
	pack_mlp_fragments(m, m->infer16.ptr, m->frag_infer.ptr, s);
}

extern "C" {

const char* ngp_last_error(void) { return g_last_error.c_str(); }
const char* ngp_version(void) { return "ngp_hip 0.1 (gfx950)"; }

ngp_status ngp_model_create(int hip_device, const ngp_network_config* cfg, uint64_t seed, ngp_model** out) {
	return guarded([&] {
		require(cfg && out, "null argument");
		require(cfg->n_levels >= 1 && cfg->n_levels <= MAX_LEVELS, "n_levels must be in [1, 32]");
		require(cfg->n_features_per_level == 1 || cfg->n_features_per_level == 2 || cfg->n_features_per_level == 4 ||
		            cfg->n_features_per_level == 8,
		        "n_features_per_level must be 1, 2, 4 or 8");
		require(cfg->log2_hashmap_size >= 4 && cfg->log2_hashmap_size <= 30, "log2_hashmap_size out of range");
		require(cfg->per_level_scale > 0.0f, "per_level_scale must be positive");
		require(cfg->n_extra_dims <= NGP_EXTRA_DIMS_MAX, "n_extra_dims must be <= 32 (light directions + a 16-wide latent code fit)");
		NGP_HIP_CHECK(hipSetDevice(hip_device));
		auto* m = new ngp_model();
		try {
			m->device = hip_device;
			m->cfg = *cfg;
			m->enc_width = cfg->n_levels * cfg->n_features_per_level;
			m->enc_pad = next_multiple(m->enc_width, 16);
			{  // the plane layout of the internal encodings (ngp_internal.h EncLayout) where L/4 is a power of two
				const uint32_t G = cfg->n_levels / 4;
				const bool pow2 = cfg->n_levels % 4 == 0 && G && (G & (G - 1)) == 0;
				m->enc_lsh = pow2 ? 2u : 0u;
				m->enc_gsh = m->enc_lsh ? (uint32_t)__builtin_ctz(G) : 0u;
			}
			require(m->enc_pad <= 64, "encoding width (n_levels * F) must be <= 64");
			m->mlp_variant = mlp_variant_for(cfg->n_neurons, cfg->density_hidden_layers, cfg->rgb_hidden_layers, m->enc_pad,
			                                 cfg->n_extra_dims);
			if (m->mlp_variant < 0)
				throw std::invalid_argument(cfg->n_extra_dims ? "n_extra_dims > 0 needs the 64-neuron network with 1 density and 2 rgb hidden "
				                                                "layers and an encoding of <= 32 features"
				                                              : "unsupported MLP shape (n_neurons / hidden layers)");
			if (cfg->n_extra_dims) {
				m->zero_extra.reserve(NGP_EXTRA_ROW);
				NGP_HIP_CHECK(hipMemset(m->zero_extra.ptr, 0, NGP_EXTRA_ROW * sizeof(float)));
			}
			build_level_table(m);
			build_layers(m);
			m->n_params = m->n_mlp_params + m->n_grid_params;
			m->frag_halves = mlp_frag_halves(m);
			m->params32.reserve(m->n_params);
			m->params16.reserve(m->n_params);
			m->ema32.reserve(m->n_params);
			m->infer16.reserve(m->n_params);
			m->grads.reserve(m->n_params);
			m->grid_grads16.reserve(m->n_grid_params);
			m->adam_m.reserve(m->n_params);
			m->adam_v.reserve(m->n_params);
			m->adam_steps.reserve(m->n_params);
			m->frag_train.reserve(m->frag_halves);
			m->frag_infer.reserve(m->frag_halves);
			upload_init_params(m, seed);
			refresh_derived(m, true, 0);
			// empty occupancy state: grid zeros, all bits set as the reference's first update would
			grid_reserve(m, 1, 1);
			m->gs.bitfield.reserve(NERF_GRID_N_CELLS / 8 * NERF_CASCADES);
			m->gs.mean.reserve(1);
			m->gs.sum.reserve(1);
			NGP_HIP_CHECK(hipMemset(m->gs.bitfield.ptr, 0xff, m->gs.bitfield.bytes()));
			++m->gs.version;
			NGP_HIP_CHECK(hipMemset(m->gs.mean.ptr, 0, sizeof(float)));
			NGP_HIP_CHECK(hipDeviceSynchronize());
		} catch (...) {
			delete m;
			throw;
		}
		*out = m;
	});
}

ngp_status ngp_model_destroy(ngp_model* m) {
	return guarded([&] {
		if (!m) return;
		(void)hipSetDevice(m->device);
		(void)hipDeviceSynchronize();
		for (auto* b : {&m->params32, &m->ema32, &m->grads, &m->adam_m, &m->adam_v}) b->release();
		m->grid_grads16.release();
		m->grid_grads64.release();
		if (m->sync_event) (void)hipEventDestroy(m->sync_event);
		if (m->stats_host) (void)hipHostFree(m->stats_host);
		m->params16.release();
		m->infer16.release();
		m->adam_steps.release();
		m->adam_corr.release();
		m->frag_train.release();
		m->frag_infer.release();
		TrainScratch& t = m->ts;
		t.ray_numsteps.release(); t.ray_compacted.release(); t.ray_state.release(); t.ray_loss_state.release(); t.ray_depth.release();
		t.coords.release(); t.enc.release(); t.mlp_out.release(); t.ccoords.release(); t.cenc.release();
		t.cpos4.release(); t.ray_aux.release();
		t.dloss.release(); t.cweight.release(); t.csrc.release(); t.denc.release(); t.loss.release(); t.block_sums.release();
		t.counters.release(); t.scan_a.release(); t.scan_b.release(); t.dp.release();
		t.epos.release(); t.edir.release(); t.eenc.release(); t.eout.release(); t.eidx.release();
		t.ray_T.release(); t.ray_eval.release(); t.ray_ebase.release(); t.dsh.release(); t.dpos.release();
		t.simg.release(); t.eimg.release(); t.cimg.release(); t.dextra.release(); t.api_extra.release(); t.api_extra_idx.release();
		GridState& g = m->gs;
		g.grid.release(); g.tmp.release(); g.bitfield.release(); g.mean.release(); g.sum.release();
		g.positions.release(); g.indices.release(); g.enc.release(); g.out.release();
		g.skeys.release(); g.perm_in.release(); g.perm.release(); g.sort_tmp.release(); g.spos.release();
		g.bucket_hist.release(); g.bucket_base.release();
		m->rs.release();
		m->timers.release();
		m->zero_extra.release();
		delete m;
	});
}

ngp_status ngp_model_set_tuning(ngp_model* m, const ngp_tuning* t) {
	return guarded([&] {
		require(m != nullptr, "null argument");
		validate_tuning(t);
		m->tuning = *t;
		apply_encode_tuning(m->lt, *t);
	});
}

ngp_status ngp_tuning_validate(const ngp_tuning* t) {
	return guarded([&] { validate_tuning(t); });
}

ngp_status ngp_model_get_tuning(const ngp_model* m, ngp_tuning* t) {
	return guarded([&] {
		require(m && t, "null argument");
		*t = m->tuning;
	});
}

ngp_status ngp_model_get_info(const ngp_model* m, ngp_model_info* info) {
	return guarded([&] {
		require(m && info, "null argument");
		std::memset(info, 0, sizeof(*info));
		info->n_params = m->n_params;
		info->n_mlp_params = m->n_mlp_params;
		info->n_grid_params = m->n_grid_params;
		info->n_levels = m->lt.n_levels;
		info->n_features_per_level = m->lt.F;
		info->encoding_width = m->enc_width;
		info->padded_encoding_width = m->enc_pad;
		for (uint32_t l = 0; l < m->lt.n_levels; ++l) {
			info->level_offset[l] = m->lt.offset[l];
			info->level_size[l] = m->lt.size[l];
			info->level_resolution[l] = m->lt.res[l];
			info->level_scale[l] = m->lt.scale[l];
		}
		info->n_layers = m->n_layers;
		for (uint32_t l = 0; l < m->n_layers; ++l) {
			info->layer_in[l] = m->layers[l].in;
			info->layer_out[l] = m->layers[l].out;
			info->layer_param_offset[l] = m->layers[l].param_offset;
		}
	});
}

ngp_status ngp_model_buffer(ngp_model* m, int kind, void** ptr, size_t* bytes) {
	return guarded([&] {
		require(m && ptr, "null argument");
		switch (kind) {
			case NGP_PARAMS_FP32: *ptr = m->params32.ptr; if (bytes) *bytes = m->n_params * 4; break;
			case NGP_PARAMS_FP16: *ptr = m->params16.ptr; if (bytes) *bytes = m->n_params * 2; break;
			case NGP_PARAMS_EMA_FP32: *ptr = m->ema32.ptr; if (bytes) *bytes = m->n_params * 4; break;
			case NGP_PARAMS_INFER_FP16: *ptr = m->infer16.ptr; if (bytes) *bytes = m->n_params * 2; break;
			case NGP_GRADS_FP32: *ptr = m->grads.ptr; if (bytes) *bytes = m->n_params * 4; break;
			case NGP_ADAM_M: *ptr = m->adam_m.ptr; if (bytes) *bytes = m->n_params * 4; break;
			case NGP_ADAM_V: *ptr = m->adam_v.ptr; if (bytes) *bytes = m->n_params * 4; break;
			case NGP_GRADS_GRID_FP16: *ptr = m->grid_grads16.ptr; if (bytes) *bytes = m->n_grid_params * 2; break;
			case NGP_GRADS_GRID_FIXED64: *ptr = m->grid_grads64.ptr; if (bytes) *bytes = m->grid_grads64.ptr ? m->n_grid_params * 8 : 0; break;
			default: throw std::invalid_argument("unknown buffer kind");
		}
	});
}

ngp_status ngp_model_params_updated(ngp_model* m, int reset_optimizer, ngp_stream s) {
	return guarded([&] {
		require(m, "null model");
		refresh_derived(m, reset_optimizer != 0, S(s));
	});
}

ngp_status ngp_model_reset_optimizer(ngp_model* m, ngp_stream s) {
	return guarded([&] {
		require(m, "null model");
		refresh_derived(m, true, S(s));
	});
}

ngp_status ngp_model_encode(ngp_model* m, const float* pos, uint32_t stride, uint32_t n, uint16_t* enc, int use_inf,
                            ngp_stream s) {
	return guarded([&] {
		require(m && (n == 0 || (pos && enc)), "null argument");
		require(stride >= 3, "stride must be >= 3 floats");
		const __half* table = (use_inf ? m->infer16.ptr : m->params16.ptr) + m->n_mlp_params;
		launch_hashgrid_fwd(m->lt, pos, stride, n, table, reinterpret_cast<__half*>(enc), EncLayout{n, 0}, S(s));
	});
}

ngp_status ngp_model_encode_indices(ngp_model* m, const float* pos, uint32_t stride, uint32_t n, uint32_t* idx,
                                    float* w, ngp_stream s) {
	return guarded([&] {
		require(m && (n == 0 || (pos && idx && w)), "null argument");
		launch_hashgrid_indices(m->lt, pos, stride, n, idx, w, S(s));
	});
}

// The latent codes NerfCoordinate records carry after their 7 floats (set_with_optional_extra_dims,
// nerf_device.cuh:177-195) -> rows of NGP_EXTRA_ROW (zero-padded) and row indices i (MlpExtra with one row per sample)
__global__ void k_extra_rows(const float* __restrict__ src, uint32_t stride, uint32_t offset, uint32_t E, uint32_t n,
                             float* __restrict__ rows, uint32_t* __restrict__ idx) {
	const uint32_t i = blockIdx.x * 256u + threadIdx.x;
	if (i >= n) return;
	for (uint32_t k = 0; k < NGP_EXTRA_ROW; ++k) rows[NGP_EXTRA_ROW * (size_t)i + k] = k < E ? src[(size_t)i * stride + offset + k] : 0.0f;
	idx[i] = i;
}

static MlpExtra coord_extras(ngp_model* m, const float* src, uint32_t stride, uint32_t offset, uint32_t n, hipStream_t s) {
	MlpExtra x;
	if (!m->cfg.n_extra_dims || n == 0) return x;
	TrainScratch& ts = m->ts;
	ts.api_extra.reserve(NGP_EXTRA_ROW * (size_t)n);
	ts.api_extra_idx.reserve(n);
	k_extra_rows<<<div_up(n, 256u), 256, 0, s>>>(src, stride, offset, m->cfg.n_extra_dims, n, ts.api_extra.ptr, ts.api_extra_idx.ptr);
	NGP_HIP_CHECK(hipGetLastError());
	x.extra = ts.api_extra.ptr;
	x.sample_img = ts.api_extra_idx.ptr;
	return x;
}

ngp_status ngp_model_infer(ngp_model* m, const float* coords, uint32_t fpc, uint32_t n, uint16_t* out, int use_inf,
                           ngp_stream s) {
	return guarded([&] {
		require(m && (n == 0 || (coords && out)), "null argument");
		require(fpc >= 7 + m->cfg.n_extra_dims, "floats_per_coord must be >= 7 + n_extra_dims (NerfCoordinate + extra dims)");
		if (n == 0) return;
		const __half* table = (use_inf ? m->infer16.ptr : m->params16.ptr) + m->n_mlp_params;
		const __half* frags = use_inf ? m->frag_infer.ptr : m->frag_train.ptr;
		TrainScratch& ts = m->ts;
		ts.enc.reserve((size_t)m->lt.n_levels * n * m->lt.F);
		launch_hashgrid_fwd(m->lt, coords, fpc, n, table, ts.enc.ptr, internal_layout(m, n), S(s));
		launch_mlp_infer(m, frags, ts.enc.ptr, internal_layout(m, n), coords, fpc, n, reinterpret_cast<__half*>(out), S(s),
		                 nullptr, 4, nullptr, 0, 4, nullptr, 0, false, coord_extras(m, coords, fpc, 7, n, S(s)));
	});
}

ngp_status ngp_model_infer_padded(ngp_model* m, const float* coords, uint32_t fpc, uint32_t n, uint16_t* out,
                                  uint32_t out_stride, int layout_rm, int use_inf, ngp_stream s) {
	return guarded([&] {
		require(m && (n == 0 || (coords && out)), "null argument");
		require(fpc >= 7 + m->cfg.n_extra_dims, "floats_per_coord must be >= 7 + n_extra_dims (NerfCoordinate + extra dims)");
		require(layout_rm ? out_stride >= n : out_stride >= 16, "out_stride too small for 16 output rows");
		if (n == 0) return;
		const __half* table = (use_inf ? m->infer16.ptr : m->params16.ptr) + m->n_mlp_params;
		const __half* frags = use_inf ? m->frag_infer.ptr : m->frag_train.ptr;
		TrainScratch& ts = m->ts;
		ts.enc.reserve((size_t)m->lt.n_levels * n * m->lt.F);
		launch_hashgrid_fwd(m->lt, coords, fpc, n, table, ts.enc.ptr, internal_layout(m, n), S(s));
		launch_mlp_infer(m, frags, ts.enc.ptr, internal_layout(m, n), coords, fpc, n, reinterpret_cast<__half*>(out), S(s),
		                 nullptr, 4, nullptr, layout_rm ? 2u : 1u, out_stride, nullptr, 0, false, coord_extras(m, coords, fpc, 7, n, S(s)));
	});
}

// level-major [L][n][F] encodings -> the pipelines' EncLayout (the layout the encoder writes inside the renderer)
__global__ void k_enc_relayout(const uint16_t* __restrict__ src, uint16_t* __restrict__ dst, uint32_t L, uint32_t F, uint32_t n,
                               EncLayout lay) {
	const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
	if (t >= L * n) return;
	const uint32_t lvl = t / n, i = t % n;
	const size_t d = lay.vec(lvl, i) * F;
	for (uint32_t f = 0; f < F; ++f) dst[d + f] = src[(size_t)t * F + f];
}

ngp_status ngp_model_infer_sh_rows(ngp_model* m, const uint16_t* enc, const uint16_t* sh_rows, const uint32_t* sh_row_of_sample,
                                   uint32_t n, uint32_t n_rows, uint16_t* out, int use_inf, ngp_stream s) {
	return guarded([&] {
		require(m && (n == 0 || (enc && sh_rows && sh_row_of_sample && out)), "null argument");
		require(m->cfg.n_extra_dims == 0, "ngp_model_infer_sh_rows: networks with extra dims take ngp_model_infer");
		if (n == 0) return;
		const __half* frags = use_inf ? m->frag_infer.ptr : m->frag_train.ptr;
		TrainScratch& ts = m->ts;
		const EncLayout lay = internal_layout(m, n);
		ts.enc.reserve((size_t)m->lt.n_levels * n * m->lt.F);
		k_enc_relayout<<<div_up(m->lt.n_levels * n, 256u), 256, 0, S(s)>>>(enc, reinterpret_cast<uint16_t*>(ts.enc.ptr), m->lt.n_levels,
		                                                                  m->lt.F, n, lay);
		NGP_HIP_CHECK(hipGetLastError());
		// the renderer's network call: its timer (NGP_TIMER_RENDER_MLP) rides on the MLP dispatch alone
		MlpExtra standalone;
		standalone.standalone = true;
		m->timers.begin_kernel(NGP_TIMER_RENDER_MLP);
		launch_mlp_infer(m, frags, ts.enc.ptr, lay, nullptr, 0, n, reinterpret_cast<__half*>(out), S(s), nullptr, 4,
		                 reinterpret_cast<const __half*>(sh_rows), 0, 4, sh_row_of_sample, n_rows, false, standalone);
		m->timers.end(NGP_TIMER_RENDER_MLP, S(s), n);
	});
}

ngp_status ngp_model_density(ngp_model* m, const float* pos, uint32_t stride, uint32_t n, uint16_t* out, int use_inf,
                             ngp_stream s) {
	return guarded([&] {
		require(m && (n == 0 || (pos && out)), "null argument");
		require(stride >= 3, "stride must be >= 3 floats");
		if (n == 0) return;
		const __half* table = (use_inf ? m->infer16.ptr : m->params16.ptr) + m->n_mlp_params;
		const __half* frags = use_inf ? m->frag_infer.ptr : m->frag_train.ptr;
		GridState& g = m->gs;
		g.enc.reserve((size_t)m->lt.n_levels * n * m->lt.F);
		launch_hashgrid_fwd(m->lt, pos, stride, n, table, g.enc.ptr, internal_layout(m, n), S(s));
		launch_mlp_density(m, frags, g.enc.ptr, internal_layout(m, n), n, reinterpret_cast<__half*>(out), S(s));
	});
}

static void model_backward(ngp_model* m, const uint16_t* enc, const float* dirs, const float* extra, uint32_t n,
                           const uint16_t* dloss, const float* weight, uint16_t* denc, float* dextra, ngp_stream s);

ngp_status ngp_model_backward(ngp_model* m, const uint16_t* enc, const float* dirs, uint32_t n, const uint16_t* dloss,
                              const float* weight, uint16_t* denc, ngp_stream s) {
	return guarded([&] { model_backward(m, enc, dirs, nullptr, n, dloss, weight, denc, nullptr, s); });
}

ngp_status ngp_model_backward_extra(ngp_model* m, const uint16_t* enc, const float* dirs, const float* extra, uint32_t n,
                                    const uint16_t* dloss, const float* weight, uint16_t* denc, float* dextra, ngp_stream s) {
	return guarded([&] {
		require(m && (n == 0 || extra), "null argument");
		require(m->cfg.n_extra_dims > 0, "the model has no extra dims (n_extra_dims = 0)");
		model_backward(m, enc, dirs, extra, n, dloss, weight, denc, dextra, s);
	});
}

static void model_backward(ngp_model* m, const uint16_t* enc, const float* dirs, const float* extra, uint32_t n,
                           const uint16_t* dloss, const float* weight, uint16_t* denc, float* dextra, ngp_stream s) {
	{
		require(m && (n == 0 || (enc && dirs && dloss && denc)), "null argument");
		if (n == 0) return;
		// dirs are passed as [n][3]; the MLP kernel reads NerfCoordinate-like records (dir at offset 4)
		TrainScratch& ts = m->ts;
		ts.ccoords.reserve(8 * (size_t)n);
		std::vector<float> tmp((size_t)n * 8, 0.0f);
		std::vector<float> d((size_t)n * 3);
		NGP_HIP_CHECK(hipMemcpyAsync(d.data(), dirs, d.size() * 4, hipMemcpyDeviceToHost, S(s)));
		NGP_HIP_CHECK(hipStreamSynchronize(S(s)));
		for (size_t i = 0; i < n; ++i)
			for (int k = 0; k < 3; ++k) tmp[8 * i + 4 + k] = d[3 * i + k];
		NGP_HIP_CHECK(hipMemcpyAsync(ts.ccoords.ptr, tmp.data(), tmp.size() * 4, hipMemcpyHostToDevice, S(s)));
		MlpExtra x = extra ? coord_extras(m, extra, NGP_EXTRA_ROW, 0, n, S(s)) : MlpExtra{};
		x.dextra = dextra;
		m->timers.begin_kernel(NGP_TIMER_TRAIN_MLP_BWD);
		launch_mlp_train(m, m->frag_train.ptr, reinterpret_cast<const __half*>(enc), EncLayout{n, 0}, ts.ccoords.ptr, 8, n,
		                 reinterpret_cast<const __half*>(dloss), weight, m->grads.ptr, reinterpret_cast<__half*>(denc),
		                 S(s), nullptr, nullptr, x);
		m->timers.end(NGP_TIMER_TRAIN_MLP_BWD, S(s), n);
		NGP_HIP_CHECK(hipStreamSynchronize(S(s)));
	}
}

ngp_status ngp_model_encode_backward(ngp_model* m, const float* pos, uint32_t stride, uint32_t n, const uint16_t* denc,
                                     ngp_stream s) {
	return guarded([&] {
		require(m && (n == 0 || (pos && denc)), "null argument");
		launch_hashgrid_bwd(m->lt, pos, stride, n, reinterpret_cast<const __half*>(denc), EncLayout{n, 0},
		                    m->grid_grads16.ptr, S(s));
	});
}

ngp_status ngp_train_step(ngp_model* m, const ngp_train_args* a, ngp_stream s) {
	return guarded([&] {
		require(m && a, "null argument");
		require(a->images && a->n_images > 0, "training requires at least one image");
		require(a->n_rays > 0 && a->target_batch_size > 0 && a->max_samples > 0, "empty batch");
		require(m->gs.bitfield.ptr != nullptr, "density grid not initialised");
		// the latent-code rows are read and written as float4s (mlp.hip load_extra8, k_extra_gradient)
		require(((uintptr_t)a->extra_dims % 16) == 0 && ((uintptr_t)a->extra_dims_gradient % 16) == 0,
		        "extra_dims / extra_dims_gradient must be 16-byte aligned");
		run_train_step(m, a, S(s));
	});
}

ngp_status ngp_optimizer_step(ngp_model* m, uint32_t step, int opt_mlp, int opt_enc, ngp_stream s) {
	return guarded([&] {
		require(m, "null model");
		launch_optimizer(m, step, opt_mlp, opt_enc, S(s));
	});
}

ngp_status ngp_allreduce_grads(ngp_model* m, void* comm, ngp_stream s) {
	return guarded([&] {
		require(m && comm, "null argument");
		const ncclComm_t c = (ncclComm_t)comm;
		auto nk = [](ncclResult_t r, const char* what) {
			if (r != ncclSuccess) throw std::runtime_error(std::string("RCCL error ") + ncclGetErrorString(r) + " in " + what);
		};
		// one group: the 41 KB fp32 MLP gradients and the fp16 hash-grid gradients (the buffer the
		// packed atomics write) -- summed, so every rank's optimizer step sees the global gradient
		nk(ncclGroupStart(), "ncclGroupStart");
		nk(ncclAllReduce(m->grads.ptr, m->grads.ptr, m->n_mlp_params, ncclFloat32, ncclSum, c, S(s)), "ncclAllReduce(mlp grads)");
		if (m->ts.fixed)  // deterministic step: exact integer sum of the fixed-point gradients
			nk(ncclAllReduce(m->grid_grads64.ptr, m->grid_grads64.ptr, m->n_grid_params, ncclInt64, ncclSum, c, S(s)),
			   "ncclAllReduce(grid grads, fixed point)");
		else
			nk(ncclAllReduce(m->grid_grads16.ptr, m->grid_grads16.ptr, m->n_grid_params, ncclFloat16, ncclSum, c, S(s)),
			   "ncclAllReduce(grid grads)");
		nk(ncclGroupEnd(), "ncclGroupEnd");
	});
}

ngp_status ngp_train_discard(ngp_model* m, ngp_stream s) {
	return guarded([&] {
		require(m, "null model");
		// the gated optimizer step was a no-op on the device, but its host-side EMA step count moved
		if (m->ts.gated_optimizer_ran && m->ema_step > 0) --m->ema_step;
		m->ts.gated_optimizer_ran = false;
		NGP_HIP_CHECK(hipMemsetAsync(m->grads.ptr, 0, m->n_mlp_params * sizeof(float), S(s)));
		NGP_HIP_CHECK(hipMemsetAsync(m->grid_grads16.ptr, 0, m->n_grid_params * sizeof(__half), S(s)));
		if (m->grid_grads64.ptr) NGP_HIP_CHECK(hipMemsetAsync(m->grid_grads64.ptr, 0, m->n_grid_params * sizeof(long long), S(s)));
		if (m->ts.counters.ptr) NGP_HIP_CHECK(hipMemsetAsync(m->ts.counters.ptr + 9, 0, sizeof(uint32_t), S(s)));
	});
}

// the violation word <-> its two reducible parts (one thread; a data-parallel step's only per-step exchange
// besides the gradients, kept on the stream so an RCCL max-reduce of the parts stays asynchronous)
__global__ void k_violation_parts(uint32_t* word, int32_t* parts, int to_parts) {
	if (to_parts) {
		const uint32_t w = *word;
		parts[0] = (int32_t)(w & (VIOL_CAPACITY - 1u));
		parts[1] = (w & VIOL_CAPACITY) ? 1 : 0;
	} else {
		const uint32_t c = (uint32_t)max(parts[0], 0);
		*word = (parts[1] ? VIOL_CAPACITY : 0u) | min(c, VIOL_CAPACITY - 1u);
	}
}

ngp_status ngp_train_violation_parts(ngp_model* m, int32_t* parts, int to_parts, ngp_stream s) {
	return guarded([&] {
		require(m && parts, "null argument");
		require(m->ts.counters.ptr, "no training step has run");
		k_violation_parts<<<1, 1, 0, S(s)>>>(m->ts.counters.ptr + 9, parts, to_parts);
		NGP_HIP_CHECK(hipGetLastError());
	});
}

ngp_status ngp_train_read_stats(ngp_model* m, ngp_train_stats* st, ngp_stream s) {
	return guarded([&] {
		require(m && st, "null argument");
		std::memset(st, 0, sizeof(*st));
		if (!m->ts.counters.ptr) return;
		// into pinned memory: a pageable destination is staged and copied by the runtime before the
		// call returns, which the step's critical path paid every step
		if (!m->stats_host) NGP_HIP_CHECK(hipHostMalloc((void**)&m->stats_host, 16 * sizeof(uint32_t), hipHostMallocDefault));
		const uint32_t* c = m->stats_host;
		NGP_HIP_CHECK(hipMemcpyAsync(m->stats_host, m->ts.counters.ptr, 16 * sizeof(uint32_t), hipMemcpyDeviceToHost, S(s)));
		wait_stream(m, S(s));
		st->n_rays = m->ts.last_n_rays;
		st->measured_batch_size_before_compaction = c[0];
		st->measured_batch_size = c[1];
		KernelTimers& tm = m->timers;
		if (m->ts.chunked)
			for (int p = 0; p < 3; ++p) m->ts.last_rows[p] = c[12 + p];
		if (tm.train_units_pending) {
			// samples the forward evaluated: all emitted ones, or the chunks' rows
			const uint64_t all = m->ts.chunked ? (uint64_t)c[12] + c[13] + c[14] : std::min(c[0], m->ts.last_max_samples);
			const uint64_t comp = c[5];  // this rank's kept samples (min(total, cap))
			tm.units[NGP_TIMER_TRAIN_ENCODE] += all;
			tm.units[NGP_TIMER_TRAIN_MLP_INFER] += all;
			tm.units[NGP_TIMER_TRAIN_MLP_BWD] += comp;
			tm.units[NGP_TIMER_TRAIN_ENCODE_BWD] += comp;
			tm.train_units_pending = false;
		}
		float loss;
		std::memcpy(&loss, &c[8], 4);
		st->loss = loss;
		st->n_rays_with_samples = 0;
		st->forward_early_stop_violations = c[9] & (VIOL_CAPACITY - 1u);
		st->sample_capacity_overflow = (c[9] & VIOL_CAPACITY) ? 1u : 0u;
		if (c[10]) m->ts.rank_cap_hint = next_multiple(c[10] + c[10] / 4, 4096u);  // this rank's need, with headroom
	});
}

ngp_status ngp_train_scratch(ngp_model* m, int kind, void** ptr, size_t* bytes) {
	return guarded([&] {
		require(m && ptr, "null argument");
		TrainScratch& t = m->ts;
		const size_t R = t.last_n_rays, B = t.last_target, MS = t.last_max_samples;
		switch (kind) {
			case NGP_SCRATCH_RAY_NUMSTEPS: *ptr = t.ray_numsteps.ptr; if (bytes) *bytes = R * 8; break;
			case NGP_SCRATCH_COORDS: *ptr = t.coords.ptr; if (bytes) *bytes = MS * 32; break;
			case NGP_SCRATCH_MLP_OUT: *ptr = t.mlp_out.ptr; if (bytes) *bytes = MS * 8; break;
			case NGP_SCRATCH_RAY_COMPACTED: *ptr = t.ray_compacted.ptr; if (bytes) *bytes = R * 8; break;
			case NGP_SCRATCH_DLOSS: *ptr = t.dloss.ptr; if (bytes) *bytes = B * 8; break;
			case NGP_SCRATCH_LOSS: *ptr = t.loss.ptr; if (bytes) *bytes = R * 4; break;
			case NGP_SCRATCH_COMPACT_COORDS: *ptr = t.ccoords.ptr; if (bytes) *bytes = B * 32; break;
			case NGP_SCRATCH_RAY_EVALUATED:
				*ptr = t.chunked ? t.ray_eval.ptr : nullptr;
				if (bytes) *bytes = t.chunked ? R * 4 : 0;
				break;
			case NGP_SCRATCH_VIOLATIONS: *ptr = t.counters.ptr ? t.counters.ptr + 9 : nullptr; if (bytes) *bytes = 4; break;
			default: throw std::invalid_argument("unknown scratch kind");
		}
	});
}

ngp_status ngp_density_grid_update(ngp_model* m, const ngp_grid_args* a, ngp_stream s) {
	return guarded([&] {
		require(m && a, "null argument");
		require(a->max_cascade < NERF_CASCADES, "max_cascade must be < 8");
		m->timers.begin(NGP_TIMER_GRID_UPDATE, S(s));
		run_grid_evaluate(m, a, S(s));
		run_grid_finish(m, a, S(s));
		m->timers.end(NGP_TIMER_GRID_UPDATE, S(s), (uint64_t)a->n_uniform_samples + a->n_nonuniform_samples);
	});
}

ngp_status ngp_density_grid_evaluate(ngp_model* m, const ngp_grid_args* a, ngp_stream s) {
	return guarded([&] {
		require(m && a, "null argument");
		require(a->max_cascade < NERF_CASCADES, "max_cascade must be < 8");
		run_grid_evaluate(m, a, S(s));
	});
}

ngp_status ngp_density_grid_finish(ngp_model* m, const ngp_grid_args* a, ngp_stream s) {
	return guarded([&] {
		require(m && a, "null argument");
		run_grid_finish(m, a, S(s));
	});
}

ngp_status ngp_density_grid_bitfield(ngp_model* m, uint32_t max_cascade, ngp_stream s) {
	return guarded([&] {
		require(m, "null model");
		require(max_cascade < NERF_CASCADES, "max_cascade must be < 8");
		run_grid_bitfield(m, max_cascade, S(s));
	});
}

ngp_status ngp_density_grid_buffers(ngp_model* m, float** grid, uint8_t** bitfield, float** tmp, float** mean) {
	return guarded([&] {
		require(m, "null model");
		if (grid) *grid = m->gs.grid.ptr;
		if (bitfield) {
			*bitfield = m->gs.bitfield.ptr;
			++m->gs.version;  // the caller may write through it
		}
		if (tmp) *tmp = m->gs.tmp.ptr;
		if (mean) *mean = m->gs.mean.ptr;
	});
}

ngp_status ngp_density_on_grid(ngp_model* m, const ngp_grid_query* q, float* out, ngp_stream s) {
	return guarded([&] {
		require(m && q, "null argument");
		const uint64_t n = (uint64_t)q->res[0] * q->res[1] * q->res[2];
		require(n == 0 || out, "null output");
		require(n < (1ull << 32), "lattice too large (at most 2^32 points)");
		require(q->max_cascade < NERF_CASCADES, "max_cascade must be < 8");
		if (q->mask_with_grid)
			require(m->gs.grid.ptr != nullptr && m->gs.n_cascades > q->max_cascade,
			        "density grid not initialised for max_cascade (mask_with_grid)");
		if (n == 0) return;
		run_density_on_grid(m, q, out, S(s));
	});
}

ngp_status ngp_error_map_build_cdf(const float* error_map, uint32_t n_images, uint32_t res_x, uint32_t res_y,
                                   float* cdf_x_cond_y, float* cdf_y, float* cdf_img, ngp_stream s) {
	return guarded([&] {
		require(n_images == 0 || (error_map && cdf_x_cond_y && cdf_y && cdf_img), "null argument");
		run_error_map_cdf(error_map, n_images, res_x, res_y, cdf_x_cond_y, cdf_y, cdf_img, S(s));
	});
}

ngp_status ngp_render(ngp_model* m, const ngp_render_args* a, float* frame, float* depth, ngp_stream s) {
	return guarded([&] {
		require(m && a && frame && depth, "null argument");
		require(a->width > 0 && a->height > 0, "empty render target");
		require(((uintptr_t)a->extra_dims % 16) == 0, "extra_dims must be 16-byte aligned");
		run_render(m, a, frame, depth, S(s));
	});
}

ngp_status ngp_accumulate_tonemap(const float* frame, float* accum, float* out, uint32_t W, uint32_t H, uint32_t spp,
                                  int color_space, float exposure, const float* bg, int output_srgb, ngp_stream s) {
	return guarded([&] {
		require(frame && accum, "null argument");
		run_accumulate_tonemap(frame, accum, out, W, H, spp, color_space, exposure, bg, output_srgb, S(s));
	});
}

ngp_status ngp_timing_enable(ngp_model* m, int mask) {
	return guarded([&] {
		require(m, "null model");
		m->timers.mask = (uint32_t)mask & ((1u << NGP_TIMER_COUNT) - 1u);
	});
}

ngp_status ngp_timing_read(ngp_model* m, int timer, double* total_ms, uint64_t* units, uint32_t* launches, int reset) {
	return guarded([&] {
		require(m, "null model");
		require(timer >= 0 && timer < NGP_TIMER_COUNT, "unknown timer");
		KernelTimers& t = m->timers;
		t.collect();
		if (total_ms) *total_ms = t.ms[timer];
		if (units) *units = t.units[timer];
		if (launches) *launches = t.launches[timer];
		if (reset) {
			t.ms[timer] = 0.0;
			t.units[timer] = 0;
			t.launches[timer] = 0;
		}
	});
}

}  // extern "C"
