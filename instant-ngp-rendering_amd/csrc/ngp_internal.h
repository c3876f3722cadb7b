// ngp_internal.h — model state and kernel launchers of libngp_hip.so (gfx950).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <hip/hip_ext.h>

#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/ngp_hip.h"
#include "ngp_math.h"

namespace ngp {

#define NGP_HIP_CHECK(expr)                                                                               \
	do {                                                                                                  \
		hipError_t _e = (expr);                                                                           \
		if (_e != hipSuccess) {                                                                           \
			throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) + " at " + #expr); \
		}                                                                                                 \
	} while (0)

// Start/stop events bound to the next launch_timed() dispatch on this thread
// (hipExtLaunchKernelGGL): the timestamps come from the kernel's own dispatch packet, so a
// timed kernel costs no marker packets (each hipEventRecord drains the queue, ~5 us).
struct LaunchEvents {
	hipEvent_t a = nullptr, b = nullptr;
};
inline thread_local LaunchEvents g_launch_events;

template <class K, class... Args>
inline void launch_timed(K kernel, dim3 grid, dim3 block, uint32_t lds, hipStream_t s, Args... args) {
	const LaunchEvents e = g_launch_events;
	g_launch_events = LaunchEvents{};
	if (e.a) hipExtLaunchKernelGGL(kernel, grid, block, lds, s, e.a, e.b, 0u, args...);
	else kernel<<<grid, block, lds, s>>>(args...);
}

// HIP-event timers around launch groups (ngp_timing_enable / ngp_timing_read).  A group
// that is exactly one launch_timed() kernel is opened with begin_kernel(): its events ride
// on that dispatch instead of being recorded around it.
struct KernelTimers {
	struct Pending {
		int slot;
		hipEvent_t a, b;
	};
	uint32_t mask = 0;  // bit k: timer k records events
	bool train_units_pending = false;
	std::vector<hipEvent_t> pool;
	std::vector<Pending> pending;
	hipEvent_t open[NGP_TIMER_COUNT] = {};
	hipEvent_t open_stop[NGP_TIMER_COUNT] = {};  // begin_kernel(): stop event of the bound dispatch
	double ms[NGP_TIMER_COUNT] = {};
	uint64_t units[NGP_TIMER_COUNT] = {};
	uint32_t launches[NGP_TIMER_COUNT] = {};

	hipEvent_t take() {
		if (pool.empty()) {
			// timing-only events: no system-scope fence when they complete (the default one writes back and
			// invalidates the caches around every timed launch -- ~10 us of idle GPU per event pair, measured in
			// profiles/r05_timer_gaps.txt); the host reads them after a stream synchronisation
			hipEvent_t e;
			NGP_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
			return e;
		}
		hipEvent_t e = pool.back();
		pool.pop_back();
		return e;
	}
	bool on(int slot) const { return (mask >> slot) & 1u; }
	void begin(int slot, hipStream_t s) {
		if (!on(slot)) return;
		open[slot] = take();
		NGP_HIP_CHECK(hipEventRecord(open[slot], s));
	}
	void begin_kernel(int slot) {
		if (!on(slot)) return;
		open[slot] = take();
		open_stop[slot] = take();
		g_launch_events = LaunchEvents{open[slot], open_stop[slot]};
	}
	void end(int slot, hipStream_t s, uint64_t u = 0) {
		if (!on(slot) || !open[slot]) return;
		if (open_stop[slot]) {
			if (g_launch_events.a == open[slot]) {  // nothing was launched (n == 0): no sample
				g_launch_events = LaunchEvents{};
				pool.push_back(open[slot]);
				pool.push_back(open_stop[slot]);
			} else {
				pending.push_back({slot, open[slot], open_stop[slot]});
				units[slot] += u;
				++launches[slot];
			}
			open[slot] = open_stop[slot] = nullptr;
			return;
		}
		hipEvent_t e = take();
		NGP_HIP_CHECK(hipEventRecord(e, s));
		pending.push_back({slot, open[slot], e});
		open[slot] = nullptr;
		units[slot] += u;
		++launches[slot];
	}
	// units are counted even while the slot's events are off (the march's roofline needs the
	// render's sample count when only the march timer runs)
	void add_units(int slot, uint64_t u) { units[slot] += u; }
	void collect() {
		for (const Pending& p : pending) {
			NGP_HIP_CHECK(hipEventSynchronize(p.b));
			float t = 0.f;
			NGP_HIP_CHECK(hipEventElapsedTime(&t, p.a, p.b));
			ms[p.slot] += t;
			pool.push_back(p.a);
			pool.push_back(p.b);
		}
		pending.clear();
	}
	void release() {
		for (const Pending& p : pending) {
			(void)hipEventDestroy(p.a);
			(void)hipEventDestroy(p.b);
		}
		for (hipEvent_t e : pool) (void)hipEventDestroy(e);
		pending.clear();
		pool.clear();
	}
};

constexpr uint32_t MAX_LEVELS = 32;
constexpr uint32_t MAX_LAYERS = 8;

// SH row index k_generate gives the render slots a ray reserved but did not fill (ngp_tuning.render_skip_unfilled):
// the render MLP skips 16-sample column tiles made of them (their SH loads fall past the rows: zero)
constexpr uint32_t NO_SH_ROW = 0xFFFFFFFFu;

// Per-level hash-grid geometry, computed once on the host (tcnn GridEncodingTemplated ctor).
struct LevelTable {
	uint32_t n_levels;
	uint32_t F;
	float scale[MAX_LEVELS];
	uint32_t res[MAX_LEVELS];
	uint32_t offset[MAX_LEVELS];  // in entries (each entry = F features)
	uint32_t size[MAX_LEVELS];    // entries
	uint32_t hashed[MAX_LEVELS];
	// optional corner records of the dense levels (render site, F = 2; build_dense_records):
	// record (x, y, z) of level l, at rec[rec_off[l] + x + y res + z res^2] for x, y < res and
	// z <= res, holds the entries of corners (x, y, z), (x+1, y, z), (x, y+1, z), (x+1, y+1, z)
	const uint4* rec = nullptr;
	uint32_t rec_off[MAX_LEVELS];
	// optional per-sample max level (tcnn GridEncoding::set_max_level_gpu; training with
	// max_level_rand_training): sample i's value at max_level[i * ml_stride]; levels at or above
	// max_level * L + 1e-3 encode to zero and get no gradient.  null: all levels.
	const float* max_level = nullptr;
	uint32_t ml_stride = 0;
	// 1: non-temporal encoding stores (ngp_tuning.encode_streaming = 0)
	uint32_t streaming = 0;
	// 1: each XCD encodes a contiguous eighth of the chunks, level group by level group (four levels per
	// thread; ngp_tuning.encode_xcd_regions = 0); 0: XCD x takes every eighth chunk
	uint32_t regions = 0;
	// wave issue priority of the encoder's waves (s_setprio; ngp_tuning.render_priority bits 0-1, render site)
	uint32_t prio = 0;
	__host__ __device__ bool level_cut(uint32_t level, uint32_t i) const {
		if (!max_level) return false;
		// tcnn: max_level = (max_level_gpu[i] * num_grid_features) / N_FEATURES_PER_LEVEL; level >= max_level + 1e-3f
		const float ml = (max_level[(size_t)i * ml_stride] * (float)(n_levels * F)) / (float)F;
		return (float)level >= ml + 1e-3f;
	}
	LevelTable with_max_level(const float* p, uint32_t stride) const {
		LevelTable t = *this;
		t.max_level = p;
		t.ml_stride = stride;
		return t;
	}
};

// Layout of an fp16 encoding buffer (n samples, L levels, F features).
//  * lsh = 0: level-major [L][plane][F], the C-ABI layout.
//  * lsh = 2: [G][plane][4][F] with G = L / 4 = 2^gsh planes; plane p holds levels p, p + G,
//    p + 2G, p + 3G -- the four levels one encoder thread computes (k_hashgrid_fwd, LPT = 4),
//    written with one 16-B store (F = 2), and one MLP lane group's share of a 32-deep K step,
//    read with one 16-B load (k_mlp_infer_rf; k_pack permutes the first layer's K to match).
// The internal pipelines use lsh = 2 when L / 4 is a power of two; gradients w.r.t. the
// encoding (dL/denc) stay level-major.
struct EncLayout {
	uint32_t plane = 0;  // samples per plane (row pitch)
	uint32_t lsh = 0;    // 0 or 2
	uint32_t gsh = 0;    // log2 planes (lsh = 2)
	__host__ __device__ size_t vec(uint32_t level, uint32_t i) const {
		if (lsh == 0) return (size_t)level * plane + i;
		return ((size_t)((level & ((1u << gsh) - 1u)) * plane + i) << 2) | (level >> gsh);
	}
};

// Spherical harmonics of degree 4 of a warped direction in [0, 1]^3 (tcnn
// SphericalHarmonicsEncoding, configs/nerf/base.json:37-49): the rgb network's 16 inputs.
__device__ __forceinline__ void sh_deg4(float dx, float dy, float dz, float (&v)[16]) {
	const float x = dx * 2.0f - 1.0f, y = dy * 2.0f - 1.0f, z = dz * 2.0f - 1.0f;
	const float xy = x * y, xz = x * z, yz = y * z, x2 = x * x, y2 = y * y, z2 = z * z;
	v[0] = 0.28209479177387814f;
	v[1] = -0.48860251190291987f * y;
	v[2] = 0.48860251190291987f * z;
	v[3] = -0.48860251190291987f * x;
	v[4] = 1.0925484305920792f * xy;
	v[5] = -1.0925484305920792f * yz;
	v[6] = 0.94617469575755997f * z2 - 0.31539156525251999f;
	v[7] = -1.0925484305920792f * xz;
	v[8] = 0.54627421529603959f * x2 - 0.54627421529603959f * y2;
	v[9] = 0.59004358992664352f * y * (-3.0f * x2 + y2);
	v[10] = 2.8906114426405538f * xy * z;
	v[11] = 0.45704579946446572f * y * (1.0f - 5.0f * z2);
	v[12] = 0.3731763325901154f * z * (5.0f * z2 - 3.0f);
	v[13] = 0.45704579946446572f * x * (1.0f - 5.0f * z2);
	v[14] = 1.4453057213202769f * z * (x2 - y2);
	v[15] = 0.59004358992664352f * x * (-x2 + 3.0f * y2);
}

struct Layer {
	uint32_t in, out;          // logical widths (in padded to tcnn's 16-alignment)
	uint64_t param_offset;     // into the parameter vector (row-major [out][in])
	uint32_t frag_fwd, frag_bwd; // offsets (in halves) into the packed fragment blob
};

// Growable device buffer.
template <typename T>
struct DevBuf {
	T* ptr = nullptr;
	size_t n = 0;
	void reserve(size_t count) {
		if (count <= n) return;
		if (ptr) NGP_HIP_CHECK(hipFree(ptr));
		ptr = nullptr;
		NGP_HIP_CHECK(hipMalloc((void**)&ptr, std::max<size_t>(count, 1) * sizeof(T)));
		n = count;
	}
	// per-step scratch whose size follows the adaptive ray / sample counts: grow with an eighth of
	// headroom, so a count that creeps upward does not free and reallocate (a hipFree waits for the
	// device) every time it sets a new maximum
	void grow(size_t count) {
		if (count <= n) return;
		reserve((count + count / 8 + 4095) & ~(size_t)4095);
	}
	void release() {
		if (ptr) (void)hipFree(ptr);
		ptr = nullptr;
		n = 0;
	}
	size_t bytes() const { return n * sizeof(T); }
};

// Deterministic hash-grid gradients (ngp_train_args.deterministic): 64-bit fixed point in units of
// 2^-40 -- integer sums are exact and order-independent; |gradient| < 2^23 fits, contributions below
// 2^-41 round to zero (fp16, the default accumulation, flushes below 6e-8).
constexpr float GRAD_FIXED_SCALE = 1099511627776.0f;          // 2^40
constexpr float GRAD_FIXED_INV = 1.0f / 1099511627776.0f;     // 2^-40

// high bit of the step's violation word (counters[9]): a data-parallel rank's share of the samples did not fit
// its buffers (k_dp_caps); the low bits count the chunked forward's early-stop violations
constexpr uint32_t VIOL_CAPACITY = 1u << 20;

struct TrainScratch {
	DevBuf<uint32_t> ray_numsteps;     // [R][2]
	DevBuf<uint32_t> ray_compacted;    // [R][2]
	DevBuf<float> ray_state;           // [R][8] : o, d (unnormalised), pad
	DevBuf<float> ray_loss_state;      // [R][8]
	DevBuf<float> ray_depth;           // [R][2] depth supervision: composited depth, lambda * dloss/ddepth
	DevBuf<float> ray_hit;             // [R][4] sharpness: composited hit point
	DevBuf<float> ray_aux;             // [R][4] per-ray dL/dexposure
	DevBuf<float> coords;              // [max_samples][8]
	DevBuf<__half> enc;                // [L][max_samples][F]
	DevBuf<__half> mlp_out;            // [max_samples][4]
	DevBuf<float> ccoords;             // [B][8] compacted
	DevBuf<float> cpos4;               // [B][4] compacted, for the encoder backward
	DevBuf<__half> cenc;               // [L][B][F]
	DevBuf<__half> dloss;              // [B][4]
	DevBuf<float> cweight;             // [B] rollover multiplicity
	DevBuf<uint32_t> csrc;             // [B] compacted sample -> source sample index
	DevBuf<__half> denc;               // [L][B][F]
	DevBuf<float> loss;                // [R]
	DevBuf<uint32_t> block_sums;       // scan scratch
	DevBuf<uint32_t> counters;         // [16]: 0 numsteps total, 1 compacted total, 4 clamped S, 5 clamped c, 8 loss sum,
	                                   //       12..14 evaluation rows of the forward chunks
	DevBuf<uint32_t> scan_a;           // [2R] sampler counts | bases
	DevBuf<uint32_t> scan_b;           // [2R] compacted counts | bases
	// early-terminated forward (k_train_chunk): evaluation rows of the chunks, per-ray state
	DevBuf<float> epos, edir;          // [MSE][4] pos + warped dt | warped direction
	DevBuf<__half> eenc;               // [L][MSE][F]
	DevBuf<__half> eout;               // [MSE][4]
	DevBuf<uint32_t> eidx;             // [MS] sample -> evaluation row
	DevBuf<float> ray_T;               // [R]
	DevBuf<uint32_t> ray_eval, ray_ebase;  // [R]
	DevBuf<float> dsh;                 // [B][16] dL/d(SH inputs) of the compacted batch (extrinsics)
	DevBuf<float> dpos;                // [B][3] dL/d(warped position) of the compacted batch (extrinsics)
	// n_extra_dims > 0: each sample's image (the row of its latent code) in the sampler's, the evaluation rows'
	// and the compacted batch's order, and dL/d(code) of the compacted samples
	DevBuf<uint32_t> simg, eimg, cimg;
	DevBuf<float> dextra;              // [B][16]
	// deterministic steps: per-image fixed-point gradient sums [n_images][IMG_FIX_STRIDE]: exposure 0-2, camera
	// translation 3-5, rotation 6-8, latent code 9-40 (train.hip img_deposit_fixed)
	DevBuf<unsigned long long> img_fix;
	DevBuf<float> api_extra;           // C-ABI entries: the latent codes of coordinate records, rows of NGP_EXTRA_ROW
	DevBuf<uint32_t> api_extra_idx;
	DevBuf<uint32_t> dp;               // data parallel: [0,3) sample DpCaps, [4,7) compaction DpCaps, then 2 x [world] slots
	bool chunked = false;              // last step ran the chunked forward
	bool fixed = false;                // last step accumulated hash-grid gradients in fixed point (deterministic)
	bool gated_optimizer_ran = false;  // an optimizer step gated by the last step's violation word was enqueued
	uint32_t last_rows[3] = {0, 0, 0}; // evaluation rows of each chunk in the last read-back step
	uint32_t last_n_rays = 0, last_target = 0, last_max_samples = 0;
	// data parallelism: the sample capacity a step that did not fit asked for (grown on the retry)
	uint32_t rank_cap_hint = 0;
};

// s_setprio takes an immediate: the wave's issue priority from a kernel argument (0..3)
__device__ __forceinline__ void set_wave_priority(uint32_t p) {
	if (p == 1) __builtin_amdgcn_s_setprio(1);
	else if (p == 2) __builtin_amdgcn_s_setprio(2);
	else if (p >= 3) __builtin_amdgcn_s_setprio(3);
}

constexpr uint32_t IMG_FIX_STRIDE = 9 + NGP_EXTRA_ROW;

struct GridState {
	DevBuf<float> grid;        // [n_cascades][N]
	DevBuf<float> tmp;         // [n_cascades][N]
	DevBuf<uint8_t> bitfield;  // [8][N/8]
	DevBuf<float> mean;        // [1]
	DevBuf<unsigned long long> sum;  // [1] fixed-point accumulator
	DevBuf<float> positions;   // [n_samples][4]
	DevBuf<uint32_t> indices;  // [n_samples]
	DevBuf<__half> enc;        // [L][n][F]
	DevBuf<__half> out;        // [n]
	// the evaluated samples in cell (Morton) order: sort keys / permutation in and out, the
	// positions gathered in that order, radix-sort scratch
	DevBuf<uint32_t> skeys, perm_in, perm, sort_tmp;
	DevBuf<uint32_t> bucket_hist, bucket_base;  // the bucketed cell sort (GRID_BUCKETS; hist kept zero between updates)
	DevBuf<float> spos;        // [n][4]
	uint32_t n_cascades = 0;
	uint64_t version = 0;  // bumped whenever the bitfield may have changed (render caches derive from it)
};

// One ray pipeline of the tracer: its ray set (alternate 8-row blocks of the frame when two
// pipelines run), payload ping-pong buffers, pass scratch and counters.
struct RenderPipeScratch {
	DevBuf<float> payload[3];   // [n][12]: Payload (render.hip)
	DevBuf<float> rgba[3];      // [n][4]
	DevBuf<float> depth[3];     // [n]
	DevBuf<float> coords;       // [max_samples][4] position + warped dt, then [max_samples] SH row indices
	DevBuf<__half> enc;         // [L][max_samples][F]
	DevBuf<__half> out;         // [max_samples][4]
	DevBuf<uint32_t> counters;  // [16]
	// Normals render mode: d(raw density)/d(warped position) of the pass's samples and its scratch
	DevBuf<__half> nrm_dloss, nrm_denc;
	DevBuf<float> nrm;
	DevBuf<uint32_t> host_counter;  // pinned, fine-grained (hipHostMalloc): per-pass counters
	uint32_t* host_counter_dev = nullptr;  // its device address
	uint32_t pass_tag = 0;          // tags of published passes (monotonic across renders)
	hipEvent_t events[2] = {nullptr, nullptr};  // per-pass counter read-backs
	void release() {
		for (int b = 0; b < 3; ++b) { payload[b].release(); rgba[b].release(); depth[b].release(); }
		coords.release(); enc.release(); out.release(); counters.release();
		nrm_dloss.release(); nrm_denc.release(); nrm.release();
		if (host_counter.ptr) (void)hipHostFree(host_counter.ptr);
		host_counter.ptr = nullptr;
		for (auto& e : events)
			if (e) (void)hipEventDestroy(e);
	}
};

struct RenderScratch {
	static constexpr int MAX_PIPES = 4;
	RenderPipeScratch pipe[MAX_PIPES];
	hipStream_t streams[MAX_PIPES] = {};  // pipelines 1.. run on their own streams ([0] unused: the caller's)
	hipEvent_t fork = nullptr, join[MAX_PIPES] = {};  // caller's stream -> pipeline streams -> caller's stream
	DevBuf<uint4> dense_rec;   // corner records of the dense levels (LevelTable::rec), rebuilt per render
	DevBuf<uint4> shrows;      // [W * H][2]: each ray's 16 fp16 SH inputs, indexed by its pixel (k_render_init)
	DevBuf<uint8_t> df;        // octant distance fields [mip][8][N] (ngp_math.h lattice_step_df)
	DevBuf<uint8_t> df_x, df_xy;  // separable passes: [mip][2][N], [mip][4][N]
	DevBuf<float> slice_coords;   // Slice mode: [pixels][8] NerfCoordinate rows (pos.x NaN: no ray)
	DevBuf<__half> slice_enc, slice_out;
	// streamed host frame (ngp_render_args.host_frame): pixels whose ray never marched (1 per pixel, k_render_init),
	// written to the host by k_host_background on its own stream while the passes run
	DevBuf<uint8_t> hmask;
	hipStream_t host_stream = nullptr;
	hipEvent_t host_ev[MAX_PIPES] = {}, host_join = nullptr;
	uint64_t df_version = ~0ull;
	uint32_t df_max_mip = ~0u;
	size_t cap = 0;
	float last_samples_per_ray = 0.0f;  // network samples per ray of the last full Shade frame (0: none yet)
	uint32_t mlp_tile = 4;              // the render MLP's default wave step (16-sample tiles) for this frame
	// per-pixel undistorted directions of an OpenCV / fisheye lens (render.hip RenderK::lens_xy) and what they hold
	DevBuf<float2> lens_xy;
	std::vector<float> lens_key;
	const float2* lens_xy_filled = nullptr;
	void release() {
		lens_xy.release();
		lens_key.clear();
		lens_xy_filled = nullptr;
		for (auto& p : pipe) p.release();
		dense_rec.release(); shrows.release(); df.release(); df_x.release(); df_xy.release();
		slice_coords.release(); slice_enc.release(); slice_out.release(); hmask.release();
		for (auto& e : host_ev)
			if (e) (void)hipEventDestroy(e), e = nullptr;
		if (host_join) (void)hipEventDestroy(host_join);
		host_join = nullptr;
		if (host_stream) (void)hipStreamDestroy(host_stream);
		host_stream = nullptr;
		if (fork) (void)hipEventDestroy(fork);
		fork = nullptr;
		for (int j = 0; j < MAX_PIPES; ++j) {
			if (join[j]) (void)hipEventDestroy(join[j]);
			if (streams[j]) (void)hipStreamDestroy(streams[j]);
			join[j] = nullptr;
			streams[j] = nullptr;
		}
	}
};

}  // namespace ngp

struct ngp_model {
	int device = 0;
	ngp_network_config cfg{};
	ngp::LevelTable lt{};
	uint32_t enc_width = 0, enc_pad = 0;
	uint32_t enc_lsh = 0, enc_gsh = 0;  // EncLayout of the internal encoding buffers
	uint32_t n_layers = 0, n_density_layers = 0;
	ngp::Layer layers[ngp::MAX_LAYERS];
	uint64_t n_mlp_params = 0, n_grid_params = 0, n_params = 0;
	uint32_t frag_halves = 0;  // packed fragment blob size
	int mlp_variant = -1;
	ngp_tuning tuning{};  // launch shapes / march schedule (ngp_model_set_tuning; 0 = default)

	ngp::DevBuf<float> params32, ema32, grads, adam_m, adam_v;
	ngp::DevBuf<__half> grid_grads16;  // hash-grid gradients (fp16, packed atomics)
	ngp::DevBuf<long long> grid_grads64;  // deterministic mode: hash-grid gradients, 2^-40 fixed point
	ngp::DevBuf<__half> params16, infer16;
	ngp::DevBuf<uint32_t> adam_steps;
	// Adam's bias corrections per step count n: {sqrt(1 - beta2^n), 1 - beta1^n}, entries [0, adam_corr_n)
	// (the optimizer's powf pair was most of its instructions: it ran VALU-bound)
	ngp::DevBuf<float> adam_corr;
	uint32_t adam_corr_n = 0;
	float adam_corr_b1 = 0.0f, adam_corr_b2 = 0.0f;
	ngp::DevBuf<__half> frag_train, frag_infer;  // packed MFMA fragments of params16 / infer16
	mutable ngp::DevBuf<float> mlp_partials;      // [workgroup][n_mlp_params] weight-gradient partials of k_mlp_train
	ngp::DevBuf<float> zero_extra;                // n_extra_dims > 0: one all-zero latent-code row (no codes given)
	uint32_t ema_step = 0;

	ngp::TrainScratch ts;
	ngp::GridState gs;
	ngp::RenderScratch rs;
	ngp_train_stats last_stats{};
	bool stats_pending = false;
	ngp::KernelTimers timers;
	hipEvent_t sync_event = nullptr;  // host read-backs spin on it (ngp::wait_stream)
	uint32_t* stats_host = nullptr;   // pinned (hipHostMalloc): the training counters' read-back
	uint32_t last_n_rays = 0;
};

namespace ngp {

// ---- kernel launchers (defined in the .hip files) --------------------------------------
// hashgrid.hip
// site: 0 training step, 1 render, 2 density grid / API (names the kernel instance in profiles)
// Waits for everything enqueued on s by spinning on an event: the per-pass counter
// read-backs are short, and a blocking wait costs tens of microseconds of wake-up.
inline void wait_stream(ngp_model* m, hipStream_t s) {
	if (!m->sync_event) NGP_HIP_CHECK(hipEventCreateWithFlags(&m->sync_event, hipEventDisableTiming));
	NGP_HIP_CHECK(hipEventRecord(m->sync_event, s));
	hipError_t e;
	while ((e = hipEventQuery(m->sync_event)) == hipErrorNotReady) {
	}
	NGP_HIP_CHECK(e);
}

// n: bound on the samples (the device count *n_dev, when given, is the actual one).  max_chunks
// > 0 caps the 256-sample chunks launched per level; the blocks then loop over the chunks
// up to the device count (for large bounds that are rarely reached).
// Corner records of the dense levels of `table` (F = 2) into rs.dense_rec; returns m->lt with
// rec / rec_off set (rec stays null when no level is dense or F != 2).
LevelTable build_dense_records(ngp_model* m, const __half* table, hipStream_t s);
void launch_hashgrid_fwd(const LevelTable& lt, const float* pos, uint32_t stride, uint32_t n, const __half* table,
                         __half* enc, EncLayout enc_layout, hipStream_t s, const uint32_t* n_dev = nullptr, int site = 2,
                         uint32_t max_chunks = 0);
// grad64 non-null: deterministic fixed-point accumulation into it (grad_table16 unused).
// CUs of the current device (cached)
int cu_count();

// max_chunks > 0: blocks loop over the device count past max_chunks 128-sample chunks.
void launch_hashgrid_bwd(const LevelTable& lt, const float* pos, uint32_t stride, uint32_t n, const __half* denc,
                         EncLayout enc_layout, __half* grad_table16, hipStream_t s, const uint32_t* n_dev = nullptr,
                         long long* grad64 = nullptr, uint32_t max_chunks = 0);
void launch_hashgrid_indices(const LevelTable& lt, const float* pos, uint32_t stride, uint32_t n, uint32_t* idx,
                             float* w, hipStream_t s);
// mlp.hip
int mlp_variant_for(uint32_t width, uint32_t dh, uint32_t rh, uint32_t enc_pad, uint32_t n_extra_dims = 0);
uint32_t mlp_frag_halves(const ngp_model* m);
void pack_mlp_fragments(const ngp_model* m, const __half* params16, __half* frags, hipStream_t s);
// The latent codes of a model with n_extra_dims > 0 (the rgb network's extra inputs): extra = fp32 rows of NGP_EXTRA_ROW
// (zero past n_extra_dims), sample i reads row sample_img[i], or row 0 without sample_img; extra null: zeros.
// dextra (training): [n][16] dL/d(latent code) of each sample's own row.
struct MlpExtra {
	const float* extra = nullptr;
	const uint32_t* sample_img = nullptr;
	float* dextra = nullptr;
	// the network alone on the GPU (ngp_model_infer_sh_rows), not beside the renderer's other ray pipeline: the
	// untuned render-MLP schedule defaults to the standalone optimum (launch_mlp_infer)
	bool standalone = false;
};
// coords: per-sample records of coord_stride floats holding the warped direction at
// dir_offset (NerfCoordinate: 4); sh (optional): [n][16] fp16 SH rows used instead
void launch_mlp_infer(const ngp_model* m, const __half* frags, const __half* enc, EncLayout enc_layout,
                      const float* coords, uint32_t coord_stride, uint32_t n, __half* out, hipStream_t s,
                      const uint32_t* n_dev = nullptr, uint32_t dir_offset = 4, const __half* sh = nullptr,
                      uint32_t out_mode = 0, uint32_t out_stride = 4, const uint32_t* sh_ray = nullptr, uint32_t sh_rows = 0,
                      bool skip_unfilled = false, const MlpExtra& x = MlpExtra{});
// render.hip: the octant distance fields of the bitfield's mips [0, max_mip] into m->rs.df (rebuilt only
// when the bitfield changed); the renderer's march and the training sampler (aabb_scale 1) read them
void build_distance_fields(ngp_model* m, uint32_t max_mip, hipStream_t s);
void launch_mlp_density(const ngp_model* m, const __half* frags, const __half* enc, EncLayout enc_layout, uint32_t n,
                        __half* out, hipStream_t s, const uint32_t* n_dev = nullptr);
// dsh (optional): [n][16] dL/d(SH inputs of the rgb network), of the sample's own row (divided
// by its rollover weight), for the camera gradients.  grads_mlp null: dL/denc only (no weight gradients);
// coords null: the zero direction (for dL/dout with zero rgb rows, where the direction does not matter)
void launch_mlp_train(const ngp_model* m, const __half* frags, const __half* enc, EncLayout enc_layout,
                      const float* coords, uint32_t coord_stride, uint32_t n, const __half* dloss,
                      const float* weight, float* grads_mlp, __half* denc, hipStream_t s,
                      const uint32_t* n_dev = nullptr, float* dsh = nullptr, const MlpExtra& x = MlpExtra{});
// dL/d(warped position) through the grid of the first *n_dev samples (dpos [n][3]), divided by weight
void launch_hashgrid_input_grad(const LevelTable& lt, const float* pos, uint32_t stride, uint32_t n, const __half* denc,
                                EncLayout enc_layout, const __half* table, const float* weight, float* dpos, hipStream_t s,
                                const uint32_t* n_dev);
// layout of the encoding buffers the pipelines keep internally (C-ABI buffers: EncLayout{n, 0})
inline EncLayout internal_layout(const ngp_model* m, uint32_t plane) { return EncLayout{plane, m->enc_lsh, m->enc_gsh}; }
// train.hip
struct SamplerParams;
void launch_optimizer(ngp_model* m, uint32_t step, int opt_mlp, int opt_enc, hipStream_t s);
void run_train_step(ngp_model* m, const ngp_train_args* t, hipStream_t s);
void launch_params_to_half(const float* src, __half* dst, size_t n, hipStream_t s);
// device-side exclusive scan of u32 counts (n <= 2^24), totals written to *total
void launch_exclusive_scan(const uint32_t* in, uint32_t* out, uint32_t n, uint32_t* block_sums, uint32_t* total,
                           hipStream_t s);

inline uint32_t div_up(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }
inline uint32_t next_multiple(uint32_t a, uint32_t b) { return div_up(a, b) * b; }

}  // namespace ngp
