// train.hip — NeRF training-step kernels for gfx950.
//
//  k_sample_count / k_sample_write   generate_training_samples_nerf   src/testbed_nerf.cu:679-838
//  k_loss_composite / k_loss_emit    compute_loss_kernel_train_nerf   src/testbed_nerf.cu:841-1160
//  rollover_weight (gather kernel)   tcnn fill_rollover_and_rescale   src/testbed_nerf.cu:2862-2870
//  k_optimizer                       tcnn Ema∘ExponentialDecay∘Adam   src/testbed_nerf.cu:2502
//
// The reference claims output slots with global atomicAdd (numsteps_counter,
// ray_counter, numsteps_counter_compacted), so its sample order depends on
// scheduling.  Here every compaction is an exclusive prefix sum over the ray
// index (wave prefix via DPP shuffles -> workgroup -> grid), i.e. the same
// rule the reference applies ("claim `numsteps` slots, drop the ray if
// base + numsteps > cap") taken in ray-index order: deterministic, and
// bit-identical to the scalar oracle.
#include <cstring>
#include <type_traits>

#include "ngp_internal.h"

namespace ngp {

// ---------------------------------------------------------------------------
// Exclusive scan (deterministic): 1024 elements per workgroup.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t wave_inclusive_scan(uint32_t v) {
	const int lane = threadIdx.x & 63;
#pragma unroll
	for (int d = 1; d < 64; d <<= 1) {
		const uint32_t u = __shfl_up(v, d, 64);
		if (lane >= d) v += u;
	}
	return v;
}

__global__ void __launch_bounds__(256) k_scan_local(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                    uint32_t n, uint32_t* __restrict__ block_sums) {
	__shared__ uint32_t wsum[4];
	const uint32_t base = blockIdx.x * 1024u + threadIdx.x * 4u;
	uint32_t v[4];
#pragma unroll
	for (int k = 0; k < 4; ++k) v[k] = base + k < n ? in[base + k] : 0u;
	const uint32_t tsum = v[0] + v[1] + v[2] + v[3];
	const uint32_t incl = wave_inclusive_scan(tsum);
	const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
	if (lane == 63) wsum[wave] = incl;
	__syncthreads();
	uint32_t woff = 0;
	for (int w = 0; w < wave; ++w) woff += wsum[w];
	uint32_t run = woff + incl - tsum;
#pragma unroll
	for (int k = 0; k < 4; ++k) {
		if (base + k < n) out[base + k] = run;
		run += v[k];
	}
	if (threadIdx.x == 255) block_sums[blockIdx.x] = woff + incl;
}

__global__ void __launch_bounds__(1024) k_scan_blocks(uint32_t* __restrict__ block_sums, uint32_t n_blocks,
                                                      uint32_t* __restrict__ total) {
	__shared__ uint32_t wsum[16];
	__shared__ uint32_t carry;
	if (threadIdx.x == 0) carry = 0;
	__syncthreads();
	for (uint32_t b0 = 0; b0 < n_blocks; b0 += 1024) {
		const uint32_t i = b0 + threadIdx.x;
		const uint32_t v = i < n_blocks ? block_sums[i] : 0u;
		const uint32_t incl = wave_inclusive_scan(v);
		const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
		if (lane == 63) wsum[wave] = incl;
		__syncthreads();
		uint32_t woff = carry;
		for (int w = 0; w < wave; ++w) woff += wsum[w];
		if (i < n_blocks) block_sums[i] = woff + incl - v;
		__syncthreads();
		if (threadIdx.x == 1023) carry = woff + incl;
		__syncthreads();
	}
	if (threadIdx.x == 0) *total = carry;
}

__global__ void k_scan_add(uint32_t* __restrict__ out, uint32_t n, const uint32_t* __restrict__ block_sums) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i < n) out[i] += block_sums[i / 1024u];
}

// The whole scan in one workgroup (n up to SCAN_ONE_BLOCK_MAX: a training batch's rays): tiles of 16 K
// elements staged through LDS (coalesced loads and stores), 16 consecutive elements per thread, wave
// scans, LDS totals, a carry across tiles -- one launch instead of three launch-latency-bound ones (the
// rays of a volume scene's batch are ~2 k, of a surface scene ~35 k).
constexpr uint32_t SCAN_ONE_BLOCK_MAX = 1u << 17;
__global__ void __launch_bounds__(1024) k_scan_one_block(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                         uint32_t n, uint32_t* __restrict__ total) {
	constexpr uint32_t PER = 16, TILE = 1024 * PER;
	__shared__ uint32_t wsum[16];
	__shared__ uint4 stage[TILE / 4];
	uint32_t* st = reinterpret_cast<uint32_t*>(stage);
	const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
	uint32_t carry = 0;
	// the next tile's elements are loaded into registers while this one is scanned (a surface scene's ~35 k rays
	// are three tiles: one global-load latency instead of three)
	uint32_t nxt[PER];
#pragma unroll
	for (uint32_t k = 0; k < PER; ++k) {
		const uint32_t e = k * 1024u + threadIdx.x;
		nxt[k] = e < n ? in[e] : 0u;
	}
	for (uint32_t t0 = 0; t0 < n; t0 += TILE) {
#pragma unroll
		for (uint32_t k = 0; k < PER; ++k) st[k * 1024u + threadIdx.x] = nxt[k];
		if (t0 + TILE < n) {
#pragma unroll
			for (uint32_t k = 0; k < PER; ++k) {
				const uint32_t e = t0 + TILE + k * 1024u + threadIdx.x;
				nxt[k] = e < n ? in[e] : 0u;
			}
		}
		__syncthreads();
		uint32_t v[PER], tsum = 0;
#pragma unroll
		for (uint32_t q = 0; q < PER / 4; ++q) {
			const uint4 u = stage[threadIdx.x * (PER / 4) + q];
			v[4 * q] = u.x, v[4 * q + 1] = u.y, v[4 * q + 2] = u.z, v[4 * q + 3] = u.w;
		}
#pragma unroll
		for (uint32_t k = 0; k < PER; ++k) tsum += v[k];
		const uint32_t incl = wave_inclusive_scan(tsum);
		if (lane == 63) wsum[w] = incl;
		__syncthreads();
		uint32_t woff = carry, tile_total = 0;
		for (uint32_t q = 0; q < 16; ++q) {
			if (q < w) woff += wsum[q];
			tile_total += wsum[q];
		}
		uint32_t run = woff + incl - tsum;
#pragma unroll
		for (uint32_t q = 0; q < PER / 4; ++q) {
			uint4 u;
			u.x = run, run += v[4 * q];
			u.y = run, run += v[4 * q + 1];
			u.z = run, run += v[4 * q + 2];
			u.w = run, run += v[4 * q + 3];
			stage[threadIdx.x * (PER / 4) + q] = u;
		}
		__syncthreads();
#pragma unroll
		for (uint32_t k = 0; k < PER; ++k) {
			const uint32_t e = k * 1024u + threadIdx.x;
			if (t0 + e < n) out[t0 + e] = st[e];
		}
		carry += tile_total;
		__syncthreads();  // stage and wsum are rewritten by the next tile
	}
	if (threadIdx.x == 0) *total = carry;
}

void launch_exclusive_scan(const uint32_t* in, uint32_t* out, uint32_t n, uint32_t* block_sums, uint32_t* total,
                           hipStream_t s) {
	const uint32_t nb = div_up(n, 1024);
	if (nb == 0) {
		NGP_HIP_CHECK(hipMemsetAsync(total, 0, sizeof(uint32_t), s));
		return;
	}
	if (n <= SCAN_ONE_BLOCK_MAX) {
		k_scan_one_block<<<1, 1024, 0, s>>>(in, out, n, total);
		NGP_HIP_CHECK(hipGetLastError());
		return;
	}
	k_scan_local<<<nb, 256, 0, s>>>(in, out, n, block_sums);
	k_scan_blocks<<<1, 1024, 0, s>>>(block_sums, nb, total);
	k_scan_add<<<div_up(n, 256), 256, 0, s>>>(out, n, block_sums);
	NGP_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------
// Camera rays (uv_to_ray, common_device.cuh:393-460; lenses: ngp_math.h lens_direction).
// ---------------------------------------------------------------------------
__device__ __forceinline__ m43 load_xform(const float* x) {
	m43 m;
	for (int c = 0; c < 4; ++c) m.c[c] = mk3(x[3 * c + 0], x[3 * c + 1], x[3 * c + 2]);
	return m;
}

__device__ __forceinline__ uint32_t read_texel(const ngp_image& im, float u, float v) {
	int px = (int)(u * (float)im.width), py = (int)(v * (float)im.height);
	px = px < 0 ? 0 : (px > (int)im.width - 1 ? (int)im.width - 1 : px);
	py = py < 0 ? 0 : (py > (int)im.height - 1 ? (int)im.height - 1 : py);
	return reinterpret_cast<const uint32_t*>(im.pixels)[(size_t)px + (size_t)py * im.width];
}

// read_rgba (common_device.cuh:774-793), Byte images: sRGB -> linear, premultiplied; mask colour -> -1
__device__ __forceinline__ void texel_rgba(uint32_t t, float* rgba) {
	if (t == 0x00FF00FFu) {
		rgba[0] = rgba[1] = rgba[2] = rgba[3] = -1.0f;
		return;
	}
	const float a = (float)((t >> 24) & 0xffu) * (1.0f / 255.0f);
	rgba[0] = srgb_to_linear((float)(t & 0xffu) * (1.0f / 255.0f)) * a;
	rgba[1] = srgb_to_linear((float)((t >> 8) & 0xffu) * (1.0f / 255.0f)) * a;
	rgba[2] = srgb_to_linear((float)((t >> 16) & 0xffu) * (1.0f / 255.0f)) * a;
	rgba[3] = a;
}

struct SamplerArgs {
	const ngp_image* images;
	uint32_t n_images;
	uint32_t n_rays;
	uint32_t n_rays_global;
	uint32_t ray_offset;
	uint32_t max_samples;
	const uint32_t* max_samples_dev;  // data parallel: this rank's share of the global cap (device); null: max_samples
	pcg32 rng;
	aabb3 aabb;
	Stepping st;
	uint32_t max_mip;
	int snap;
	int max_level_rand;  // max_level_rand_training: a per-ray max level draw (src/testbed_nerf.cu:724)
	ErrorCdf cdf;  // error-map importance sampling (null pointers: uniform)
	const uint8_t* bitfield;
	uint32_t* numsteps;  // [R][2]
	uint32_t* counts;    // [R]
	uint32_t* bases;     // [R]
	float* ray_state;    // [R][8]
	float* coords;       // [max][8]
	uint32_t* simg;      // [max] n_extra_dims > 0: the sample's image (its latent-code row); null otherwise
	const float* dmap;   // learned distortion map [dry][drx][2] (null: off; general instance only)
	uint32_t drx, dry;
	const uint8_t* df;   // octant distance fields of mip 0 (aabb_scale 1 only; null: the jump chain)
	const uint32_t* total;   // the scan's sample total
	uint32_t* total_capped;  // k_sample_write: min(total, cap) for the kernels after the sampler
	uint32_t* clear16;       // k_sample_count: the step's 16 counter words, zeroed (no memset dispatch in front of the step)
};

// Image and pixel of global training ray gi from its pcg32 stream (already advanced to
// the ray): image_idx and nerf_random_image_pos_training (nerf_device.cuh:552-598),
// proportional to the error map when its CDFs are given.
// *pdf = img_pdf * uv_pdf, the importance-sampling density the reference divides the loss by
// (src/testbed_nerf.cu:1010).
// GENERAL: error-map CDFs and non-pinhole lenses may be present (a separate kernel instance,
// so the common pinhole / uniform case keeps its register budget).
template <bool GENERAL>
__device__ __forceinline__ uint32_t training_pixel(const ngp_image* images, uint32_t n_images, uint32_t gi,
                                                  uint32_t n_rays_global, const ErrorCdf& cdf, int snap, pcg32& rng,
                                                  float* uo, float* vo, float* pdf = nullptr, float* uv_pdf_out = nullptr) {
	uint32_t img;
	float img_pdf = 1.0f, uv_pdf = 1.0f;
	if (GENERAL && cdf.img) {
		img = cdf_search(ld_random_val(gi, 0xdeadbeefu), cdf.img, n_images);
		img_pdf = (cdf.img[img] - (img > 0 ? cdf.img[img - 1] : 0.0f)) * (float)n_images;
	} else {
		img = image_idx(gi, n_rays_global, n_images);
	}
	const ngp_image& im = images[img];
	float u = rng.next_float(), v = rng.next_float();
	if (GENERAL && cdf.x_cond_y) sample_cdf_2d(&u, &v, img, cdf, &uv_pdf);
	if (pdf) *pdf = img_pdf * uv_pdf;
	if (uv_pdf_out) *uv_pdf_out = uv_pdf;
	if (snap) {
		int px = (int)(u * (float)im.width), py = (int)(v * (float)im.height);
		px = px < 0 ? 0 : (px > (int)im.width - 1 ? (int)im.width - 1 : px);
		py = py < 0 ? 0 : (py > (int)im.height - 1 ? (int)im.height - 1 : py);
		u = ((float)px + 0.5f) / (float)im.width;
		v = ((float)py + 0.5f) / (float)im.height;
	}
	*uo = u;
	*vo = v;
	return img;
}

// Shared by both passes: image, pixel and ray of global ray gi (testbed_nerf.cu:712-777);
// *n0 = first lattice point (stepping space) = entry + jitter; *max_level = the ray's hash-grid
// max level (2 u with max_level_rand_training, drawn before motionblur_time; else 0 = unused).
template <bool GENERAL>
__device__ __forceinline__ bool training_ray(const SamplerArgs& a, uint32_t gi, v3* o, v3* d, float* n0,
                                             float* max_level = nullptr, uint32_t* img_out = nullptr) {
	pcg32 rng = a.rng;
	rng.advance((int64_t)gi * N_MAX_RANDOM_SAMPLES_PER_RAY);
	float u, v;
	const uint32_t img = training_pixel<GENERAL>(a.images, a.n_images, gi, a.n_rays_global, a.cdf, a.snap, rng, &u, &v);
	if (img_out) *img_out = img;
	const ngp_image im = a.images[img];
	float rgba[4];
	texel_rgba(read_texel(im, u, v), rgba);
	if (rgba[0] < 0.0f) return false;
	const float ml = a.max_level_rand ? rng.next_float() * 2.0f : 0.0f;
	if (max_level) *max_level = ml;
	const float motionblur_time = rng.next_float();
	m43 xf = load_xform(im.xform);
	if (GENERAL && (im.rolling_shutter[0] != 0.0f || im.rolling_shutter[1] != 0.0f || im.rolling_shutter[2] != 0.0f ||
	                im.rolling_shutter[3] != 0.0f))
		xf = xform_given_rolling_shutter(xf, load_xform(im.xform_end), im.rolling_shutter, u, v, motionblur_time);
	v3 dir;
	if (!GENERAL) {
		dir = rot(xf, mk3((u - im.principal_point[0]) * (float)im.width / im.focal_length[0],
		                  (v - im.principal_point[1]) * (float)im.height / im.focal_length[1], 1.0f));
	} else if (lens_direction(u, v, (float)im.width, (float)im.height, im.focal_length[0], im.focal_length[1],
	                          im.principal_point[0], im.principal_point[1], im.lens_mode, im.lens_params, &dir)) {
		if (a.dmap) {
			float ddx, ddy;
			distortion_at_lerp(a.dmap, a.drx, a.dry, u, v, &ddx, &ddy);
			dir.x += ddx;
			dir.y += ddy;
		}
		dir = rot(xf, dir);
	} else {
		dir = xf.c[2];  // no ray through this pixel: the camera axis (src/testbed_nerf.cu:762-764)
	}
	*o = xf.c[3];
	*d = normalize(dir);
	float t0, t1;
	ray_intersect(a.aabb, *o, *d, &t0, &t1);
	t0 = fmaxf(t0, 0.0f);
	*n0 = step_to(a.st, t0) + rng.next_float();
	return true;
}

// Lattice point k of a training ray: inside the AABB? a sample (occupied at mip_from_dt)?
// If it is inside but empty, the reference leaves the cell: advance_to_next_voxel at that
// mip (nerf_device.cuh:444-453) -> `jump` lattice steps (>= 1) to the first point past
// the cell's far face.
struct LatticePoint {
	bool inside, occupied;
	float t, dt;
	v3 pos;
	uint32_t jump;
};
__device__ __forceinline__ LatticePoint training_lattice_point(const SamplerArgs& a, v3 o, v3 d, v3 idir, float n0,
                                                              uint32_t k) {
	LatticePoint p;
	const float n = n0 + (float)k;
	p.t = step_from(a.st, n);
	p.dt = step_from(a.st, n + 1.0f) - p.t;
	p.pos = o + d * p.t;
	p.inside = aabb_contains(a.aabb, p.pos);
	const uint32_t mip = mip_from_dt(p.dt, p.pos, a.max_mip);
	p.occupied = p.inside && density_grid_occupied_at(p.pos, a.bitfield, mip);
	p.jump = 1;
	if (p.inside && !p.occupied) {
		const float n_far = step_to(a.st, p.t + distance_to_next_cell(p.pos, d, idir, mip));
		p.jump = (uint32_t)fminf(ceilf(fmaxf(n_far - n, 0.5f)), 1048576.0f);
	}
	return p;
}

// The sampler runs G lanes per ray (G = 8 ... 64, a power of two; one ray per G-lane group of a wave, groups
// independent: every branch below is group-uniform, ballots are taken over the group's bits only).
template <uint32_t G>
__device__ __forceinline__ unsigned long long group_bits(unsigned long long wave_bits, uint32_t g0) {
	return G == 64 ? wave_bits : (wave_bits >> g0) & ((1ull << G) - 1ull);
}

// generate_training_samples_nerf's walk (testbed_nerf.cu:779-795, 814-830) over G lattice
// points of one ray at a time (one per lane): the reference's chain -- a sample at every
// occupied point it visits, a jump past the cell of every empty one, stop at the first
// visited point outside the AABB -- run as a scalar loop over the batch's ballots (one
// iteration per run of samples or per jump).  Returns the batch's sample lanes (bits relative to
// the group's first lane g0); *cur = the lattice offset (from this batch's first point) of the
// next point to visit; *exited once the ray has left the AABB.
template <uint32_t G>
__device__ __forceinline__ unsigned long long training_walk_batch(const LatticePoint& p, uint32_t g0, uint32_t* cur_io,
                                                                  bool* exited) {
	const unsigned long long occ = group_bits<G>(__ballot(p.occupied), g0), in = group_bits<G>(__ballot(p.inside), g0);
	unsigned long long samp = 0;
	uint32_t cur = *cur_io;
	while (cur < G) {
		if (!((in >> cur) & 1ull)) {
			*exited = true;
			break;
		}
		if ((occ >> cur) & 1ull) {
			const unsigned long long rest = (~occ >> cur) & (G == 64 ? ~0ull : ((1ull << (G - cur)) - 1ull));
			const uint32_t run = rest ? (uint32_t)(__ffsll((long long)rest) - 1) : G - cur;  // occupied points from cur
			samp |= (run >= 64u ? ~0ull : ((1ull << run) - 1ull)) << cur;
			cur += run;
		} else {
			cur += (uint32_t)__shfl((int)p.jump, (int)(g0 + cur), 64);
		}
	}
	*cur_io = cur;
	return samp;
}

// aabb_scale 1 (a.df set): the ray's samples are the occupied lattice points inside the AABB (see
// train_step_df), found G lattice points per round with the empty space between them crossed
// through the octant distance fields -- a surface scene's rays cross most of the volume empty, one
// voxel per jump in the chain walk.  visit(rank, k) for every sample in order (rank < cap); returns
// the ray's sample count, capped.
// kb: the lattice point the walk starts from (0, or the round k_sample_count saw emit the ray's first
// sample: the walk from there is the same); *first (if set) = the start of the first emitting round.
template <uint32_t G, class Visit>
__device__ __forceinline__ uint32_t df_walk(const SamplerArgs& a, v3 o, v3 d, v3 idir, float n0, uint32_t cap, uint32_t r,
                                            uint32_t g0, uint32_t kb, uint32_t* first, Visit visit) {
	const uint32_t oct = ray_octant(d);
	const unsigned long long below = (1ull << r) - 1ull;
	uint32_t j = 0;
	while (true) {  // group-uniform
		uint32_t k = kb + r;
		const int st = train_step_df(&k, n0, a.st, o, d, idir, oct, a.df, a.aabb);
		const unsigned long long m_exit = group_bits<G>(__ballot(st == LATTICE_EXIT), g0);
		const unsigned long long m_occ = group_bits<G>(__ballot(st == LATTICE_OCCUPIED), g0);
		// an all-empty round goes on from the group's last lane's verified skip
		const uint32_t k_next = (uint32_t)__shfl((int)(st == LATTICE_SKIPPED ? k : kb + G), (int)(g0 + G - 1), 64);
		const uint32_t fe = m_exit ? (uint32_t)(__ffsll((long long)m_exit) - 1) : 64u;
		const unsigned long long emit = m_occ & (fe >= 64 ? ~0ull : ((1ull << fe) - 1ull));
		if ((emit >> r) & 1ull) {
			const uint32_t rank = j + __popcll(emit & below);
			if (rank < cap) visit(rank, kb + r);
		}
		if (first && j == 0 && emit) *first = kb;
		j += __popcll(emit);
		if (j >= cap) return cap;
		if (m_exit) return j;
		kb = k_next;
	}
}

// pass 1: count the ray's samples (<= NERF_STEPS), G lanes per ray.  The point the walk reached
// when it emitted its first sample goes to ray_state[8 i + 6] (overwritten by the loss kernel
// later), so pass 2 starts there instead of crossing the empty space before it again.
template <bool GENERAL, uint32_t G>
__global__ void __launch_bounds__(256) k_sample_count(SamplerArgs a) {
	const uint32_t lane = threadIdx.x & 63u, r = lane % G, g0 = lane - r;
	const uint32_t i = blockIdx.x * (256u / G) + threadIdx.x / G;
	// the step's first kernel: every later user of the counters runs after it in stream order
	if (blockIdx.x == 0 && threadIdx.x < 16u) a.clear16[threadIdx.x] = 0u;
	if (i >= a.n_rays) return;  // group-uniform
	v3 o, d;
	float n0;
	uint32_t count = 0, first = 0;
	if (!training_ray<GENERAL>(a, a.ray_offset + i, &o, &d, &n0)) {
	} else if (a.df) {
		const v3 idir = mk3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
		count = df_walk<G>(a, o, d, idir, n0, NERF_STEPS, r, g0, 0u, &first, [](uint32_t, uint32_t) {});
	} else {
		const v3 idir = mk3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
		bool exited = false;
		for (uint32_t kb = 0, cur = 0; !exited; kb += G, cur -= G) {
			if (cur >= G) continue;  // a jump past this whole batch
			const uint32_t cur0 = cur;
			const LatticePoint p = training_lattice_point(a, o, d, idir, n0, kb + r);
			const uint32_t c = __popcll(training_walk_batch<G>(p, g0, &cur, &exited));
			if (count == 0 && c) first = kb | cur0;  // kb is a multiple of G, cur0 < G
			if (count + c >= NERF_STEPS) {
				count = NERF_STEPS;
				break;
			}
			count += c;
		}
	}
	if (r == 0) {
		a.counts[i] = count;
		reinterpret_cast<uint32_t*>(a.ray_state)[8 * (size_t)i + 6] = first;
	}
}

// pass 2: same walk, each sample written at base + (its rank among the ray's samples);
// consecutive lanes write consecutive 32-byte coordinates.
template <bool GENERAL, uint32_t G>
__global__ void __launch_bounds__(256) k_sample_write(SamplerArgs a) {
	const uint32_t lane = threadIdx.x & 63u, r = lane % G, g0 = lane - r;
	const uint32_t i = blockIdx.x * (256u / G) + threadIdx.x / G;
	const uint32_t cap = a.max_samples_dev ? *a.max_samples_dev : a.max_samples;
	if (i == 0 && r == 0) *a.total_capped = min(*a.total, cap);  // (no reader in this launch)
	if (i >= a.n_rays) return;
	const uint32_t n = a.counts[i], base = a.bases[i];
	if (n == 0 || base + n > cap) {
		if (r == 0) {
			a.numsteps[2 * i + 0] = 0;
			a.numsteps[2 * i + 1] = 0;
		}
		return;
	}
	// k_sample_count's resume point, read before lane 0 of the group rewrites the ray's state below
	const uint32_t first = reinterpret_cast<const uint32_t*>(a.ray_state)[8 * (size_t)i + 6];
	v3 o, d;
	float n0, max_level;
	uint32_t img = 0;
	training_ray<GENERAL>(a, a.ray_offset + i, &o, &d, &n0, &max_level, &img);
	if (r == 0) {
		a.numsteps[2 * i + 0] = n;
		a.numsteps[2 * i + 1] = base;
		float* rs = a.ray_state + 8 * (size_t)i;
		rs[0] = o.x; rs[1] = o.y; rs[2] = o.z;
		rs[3] = d.x; rs[4] = d.y; rs[5] = d.z;
	}
	const v3 wdir = warp_direction(d);
	const v3 idir = mk3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
	if (a.df) {
		df_walk<G>(a, o, d, idir, n0, n, r, g0, first, nullptr, [&](uint32_t rank, uint32_t k) {
			// the chain walk's training_lattice_point for lattice point k, bit for bit
			const float nk = n0 + (float)k;
			const float t = step_from(a.st, nk);
			const float dt = step_from(a.st, nk + 1.0f) - t;
			const v3 wp = aabb_relative(a.aabb, o + d * t);
			float4* c = reinterpret_cast<float4*>(a.coords + 8 * (size_t)(base + rank));
			c[0] = make_float4(wp.x, wp.y, wp.z, warp_dt(dt));
			c[1] = make_float4(wdir.x, wdir.y, wdir.z, max_level);
			if (a.simg) a.simg[base + rank] = img;
		});
		return;
	}
	const unsigned long long below = (1ull << r) - 1ull;
	uint32_t j = 0;
	bool exited = false;
	for (uint32_t kb = first & ~(G - 1u), cur = first & (G - 1u); j < n && !exited; kb += G, cur -= G) {
		if (cur >= G) continue;
		const LatticePoint p = training_lattice_point(a, o, d, idir, n0, kb + r);
		const unsigned long long m = training_walk_batch<G>(p, g0, &cur, &exited);
		if ((m >> r) & 1ull) {
			const uint32_t rank = j + __popcll(m & below);
			if (rank < n) {
				const v3 wp = aabb_relative(a.aabb, p.pos);
				float4* c = reinterpret_cast<float4*>(a.coords + 8 * (size_t)(base + rank));
				c[0] = make_float4(wp.x, wp.y, wp.z, warp_dt(p.dt));
				c[1] = make_float4(wdir.x, wdir.y, wdir.z, max_level);  // the pad float carries the max level
				if (a.simg) a.simg[base + rank] = img;
			}
		}
		j += __popcll(m);
	}
}

// ---------------------------------------------------------------------------
// Early-terminated forward.  The reference runs the network over every sample the
// sampler emitted (src/testbed_nerf.cu:2797-2802), but compute_loss_kernel_train_nerf
// reads a ray's samples only up to the one where its transmittance falls below 1e-4
// (:905-916) -- on a converged scene ~85 % of the samples lie behind that point.  Here
// the forward runs over chunks of each ray's samples ([0, 16), [16, 48), [48, n)): after
// a chunk, a ray whose transmittance is below half the loss kernel's threshold stops.
// Every sample the loss kernels read is evaluated, with exactly the same network inputs,
// so the loss, the compaction and the gradients do not change (the margin absorbs the
// different association of the transmittance product).
// ---------------------------------------------------------------------------
constexpr uint32_t TRAIN_CHUNKS = 3;
constexpr uint32_t TRAIN_CHUNK_END[TRAIN_CHUNKS] = {16, 48, NERF_STEPS};
constexpr float TRAIN_CHUNK_STOP_T = 0.5e-4f;
constexpr uint32_t RAY_EVAL_DONE = 0x80000000u;

struct ChunkArgs {
	uint32_t n_rays;
	const uint32_t* numsteps;  // [R][2] samples, first sample (sampler)
	const float* coords;       // [MS][8] sampler rows
	float4* epos;              // [MSE] evaluation rows: pos + warped dt
	float4* edir;              // [MSE] warped direction
	const __half* eout;        // [MSE][4] network outputs of the evaluation rows
	__half* mlp_out;           // [MS][4] outputs scattered back to the sampler layout
	uint32_t* eidx;            // [MS] sample -> evaluation row (the compacted gather reads the encoding there)
	float* ray_T;              // [R] transmittance before the ray's next unevaluated sample
	uint32_t* ray_eval;        // [R] samples evaluated and scattered; | RAY_EVAL_DONE once the ray stopped
	uint32_t* ray_ebase;       // [R] evaluation row of the ray's current chunk
	uint32_t* rows;            // evaluation rows claimed for the next chunk
	uint32_t prev_lo, lo, hi;  // previous chunk [prev_lo, lo); next chunk [lo, hi) (lo == hi: none)
	uint32_t eval_offset;      // evaluation row of the next chunk's first claim
	int first, last;
	int density_act;
	float stop_T;              // transmittance below which a ray stops (TRAIN_CHUNK_STOP_T; ngp_tuning.debug bit 2: 0.999)
	const uint32_t* simg;      // [MS] n_extra_dims > 0: each sample's image, copied with its evaluation row into
	uint32_t* eimg;            // [MSE]; null otherwise
};

// One chunk step: composite the previous chunk's outputs (transmittance only) and scatter
// them to the sampler layout, then claim evaluation rows for the next chunk of every ray
// still marching and gather its network inputs.  The last step only scatters.
//
// G lanes per ray (1024-thread blocks, 1024 / G rays each; the host picks G so a launch has
// ~100k+ lanes whether a batch holds 2k long rays of a volume or 35k short ones of a surface
// scene).  The group composites G samples per round: an inclusive product scan of the
// per-sample factors exp(-sigma dt) gives every lane the transmittance before its sample, and
// the ray stops at the first sample where that is below the margin (the sequential loop's
// stop; the product's association differs, which the 2x margin below the loss kernel's
// threshold absorbs).  Row copies are coalesced within the group; the rows of the next chunk
// are claimed with one atomic per block.
template <uint32_t G>
__global__ void __launch_bounds__(1024) k_train_chunk(ChunkArgs a) {
	constexpr uint32_t RPB = 1024u / G;
	__shared__ uint32_t wtot[16];
	__shared__ uint32_t s_base;
	const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
	const uint32_t r = lane % G, g0 = lane - r;
	const unsigned long long gmask = G == 64 ? ~0ull : (((1ull << G) - 1ull) << g0);
	const uint32_t i = blockIdx.x * RPB + threadIdx.x / G;
	const bool valid = i < a.n_rays;  // group-uniform
	uint32_t n = 0, base = 0;
	if (valid) {
		n = a.numsteps[2 * i];
		base = a.numsteps[2 * i + 1];
	}
	float T = 1.0f;
	bool alive = valid && n > 0;
	uint32_t ev = 0;
	if (!a.first) {
		const uint32_t e = valid ? a.ray_eval[i] : RAY_EVAL_DONE;
		alive = alive && !(e & RAY_EVAL_DONE) && e == a.prev_lo;
	}
	const bool entered = a.first ? valid : alive;  // this step owns the ray's state
	if (!a.first && alive) {
		T = a.ray_T[i];
		const uint32_t ebase = a.ray_ebase[i];
		const uint32_t end = min(n, a.lo);
		uint32_t j = a.prev_lo;
		if (!a.last) {
			while (j < end) {  // group-uniform
				const uint32_t jj = j + r;
				float f = 1.0f;
				if (jj < end) {
					const size_t e = ebase + jj - a.prev_lo;
					const uint2 ob = *reinterpret_cast<const uint2*>(a.eout + 4 * e);
					const float raw = __half2float(reinterpret_cast<const __half*>(&ob)[3]);
					const float dt = unwarp_dt(a.epos[e].w);
					f = __expf(-network_to_density(raw, a.density_act) * dt);  // 1 - alpha
				}
				float incl = f;
#pragma unroll
				for (uint32_t o = 1; o < G; o <<= 1) {
					const float y = __shfl_up(incl, o, G);
					if (r >= o) incl *= y;
				}
				const float prev = __shfl_up(incl, 1, G);
				const float Tb = r == 0 ? T : T * prev;  // transmittance before sample jj
				const unsigned long long below = __ballot(jj < end && Tb < a.stop_T) & gmask;
				if (below) {  // the loss kernel stops at or before the first such sample
					const uint32_t k = (uint32_t)(__ffsll((long long)below) - 1) - g0;
					T = __shfl(Tb, g0 + k, 64);
					j += k;
					break;
				}
				const uint32_t m = min(G, end - j);
				T *= __shfl(incl, g0 + m - 1, 64);
				j += m;
			}
		} else {
			j = end;
		}
		const uint32_t scatter = j - a.prev_lo;
		ev = j;
		// stopped inside the chunk, at its end with T already below the margin, or out of samples
		if (j < end || T < a.stop_T || end == n) alive = false;
		// the chunk's outputs back to the sampler layout (rows [prev_lo, j))
		for (uint32_t k = r; k < scatter; k += G) {
			const uint32_t src = base + a.prev_lo + k, e = ebase + k;
			*reinterpret_cast<uint2*>(a.mlp_out + 4 * (size_t)src) = *reinterpret_cast<const uint2*>(a.eout + 4 * (size_t)e);
			a.eidx[src] = e;
		}
	}
	uint32_t claim = 0;
	if (alive && a.hi > a.lo) claim = min(n, a.hi) - a.lo;
	if (entered && r == 0) {
		if (claim) {
			a.ray_T[i] = T;
			a.ray_eval[i] = a.lo;
		} else {
			a.ray_eval[i] = ev | RAY_EVAL_DONE;
		}
	}
	if (a.hi <= a.lo) return;  // last step: nothing to gather (block-uniform)
	// claim rows for the next chunk: wave scan over the groups' leaders, one atomic per block
	const uint32_t mine = r == 0 ? claim : 0u;
	uint32_t x = mine;
#pragma unroll
	for (uint32_t o = 1; o < 64; o <<= 1) {
		const uint32_t y = __shfl_up(x, o, 64);
		if (lane >= o) x += y;
	}
	if (lane == 63) wtot[w] = x;
	__syncthreads();
	if (threadIdx.x == 0) {
		uint32_t t = 0;
		for (uint32_t k = 0; k < 16; ++k) t += wtot[k];
		s_base = t ? atomicAdd(a.rows, t) : 0u;
	}
	__syncthreads();
	// exclusive offset of the group's leader
	uint32_t off = s_base + __shfl(x - mine, g0, 64);
	for (uint32_t k = 0; k < w; ++k) off += wtot[k];
	if (claim == 0) return;
	const uint32_t e0 = a.eval_offset + off;
	if (r == 0) a.ray_ebase[i] = e0;
	for (uint32_t k = r; k < claim; k += G) {
		const uint32_t src = base + a.lo + k;
		const float4* row = reinterpret_cast<const float4*>(a.coords + 8 * (size_t)src);
		a.epos[e0 + k] = row[0];
		a.edir[e0 + k] = row[1];
		if (a.eimg) a.eimg[e0 + k] = a.simg[src];
	}
}

// ---------------------------------------------------------------------------
// Loss: composite (pass 1), prefix sum, emit compacted samples + dL/dout (pass 2).
// ---------------------------------------------------------------------------
struct LossArgs {
	const ngp_image* images;
	ErrorCdf cdf;
	const float* exposure;     // [n_images][3] log2 exposure (null: 0)
	float* exposure_grad;      // [n_images][3] (null: off)
	unsigned long long* exposure_fix;  // deterministic steps: the exposure deposits in 2^-32 fixed point (null: float atomics)
	float4* ray_aux;           // [R]: the ray's dL/dexposure, deposited by k_loss_emit if the ray is kept
	float* error_map;
	uint32_t error_map_rx, error_map_ry;
	uint32_t n_images;
	uint32_t n_rays;
	uint32_t n_rays_global;
	uint32_t ray_offset;
	pcg32 rng;
	aabb3 aabb;
	int snap;
	int max_level_rand;
	int loss_type;
	int random_bg;
	v3 bg;
	int linear_colors;
	int color_space;
	int rgb_act, density_act;
	float near_distance;
	uint32_t max_compacted;
	const uint32_t* max_compacted_dev;  // data parallel: this rank's share of the global cap (device); null: max_compacted
	uint32_t target_batch;
	const uint32_t* numsteps;
	float* ray_state;        // [R][8]: o, d (sampler), u, v of the pixel (k_loss_composite)
	const float* coords;
	const __half* mlp_out;
	uint32_t n_levels, F;
	uint32_t* ccounts;     // [R] compacted count (pre-cap)
	uint32_t* cbases;      // [R]
	float* loss_state;     // [R][8]: grad xyz, rgb_ray xyz, mean_loss, pad
	uint32_t* compacted;   // [R][2]
	float* loss_out;       // [R]
	uint32_t* csrc;        // [B] compacted -> source sample
	__half* dloss;         // [B][4]
	const float* mean_density;
	const uint32_t* ray_eval;  // [R] samples the chunked forward evaluated (null: all of them)
	uint32_t* violations;      // rays whose composite reached past the evaluated samples (must stay 0)
	const uint32_t* viol_gate; // the step's violations over all ranks: non-zero = no deposits (the step re-runs)
	int store_uv_pdf;          // camera gradients: ray_aux[i].w = the pixel's pdf
	float depth_lambda;        // depth supervision (0: off)
	int depth_loss_type;
	float2* ray_depth;         // [R]: composited depth, lambda * dloss/ddepth (k_loss_composite -> k_loss_emit)
	const float* dmap;         // learned distortion map (depth targets use the distorted direction's length)
	uint32_t drx, dry;
	// sharpness-weighted error deposits (null sharp_data: off)
	const float* sharp_data;   // [n_images][res_y][res_x]
	uint32_t sharp_rx, sharp_ry;
	float* sharp_grid;         // [8][128^3] running max
	float4* ray_hit;           // [R]: composited hit point (k_loss_composite -> k_loss_emit)
	uint32_t max_mip;
};

// Scans over the G lanes of a ray's group (inclusive; G = 64: the whole wave).  Lane r of a group takes the
// same sequence of operations for every G > its rank, so a ray whose samples fit one group gets the same bits
// whatever G is.
template <uint32_t G>
__device__ __forceinline__ float group_scan_add(float v, uint32_t r) {
#pragma unroll
	for (uint32_t off = 1; off < G; off <<= 1) {
		const float t = __shfl_up(v, off, G);
		if (r >= off) v += t;
	}
	return v;
}
template <uint32_t G>
__device__ __forceinline__ float group_scan_mul(float v, uint32_t r) {
#pragma unroll
	for (uint32_t off = 1; off < G; off <<= 1) {
		const float t = __shfl_up(v, off, G);
		if (r >= off) v *= t;
	}
	return v;
}
// the ballot bits of the lane's group, shifted to bit 0
template <uint32_t G>
__device__ __forceinline__ unsigned long long group_ballot(bool p, uint32_t lane) {
	const unsigned long long b = __ballot(p);
	return G == 64 ? b : (b >> (lane & ~(G - 1u))) & ((1ull << G) - 1ull);
}

// The loss kernels' lanes per ray: the average kept samples per ray of the global batch (target_batch /
// n_rays_global, the same on every data-parallel rank and in one process with the whole batch), rounded up to
// the group that holds 1.5x it -- 16 for a surface scene's ~8, 64 for a volume's ~100.
inline uint32_t loss_lanes_per_ray(uint32_t target_batch, uint32_t n_rays_global) {
	const float avg = 1.5f * (float)target_batch / (float)std::max(n_rays_global, 1u);
	return avg <= 8.0f ? 8u : avg <= 16.0f ? 16u : avg <= 32.0f ? 32u : 64u;
}

// One compacted-batch sample as the compositor sees it.
struct LossSample {
	v3 rgb;
	float alpha, dt;
	float raw[4];
};
__device__ __forceinline__ LossSample loss_sample(const LossArgs& a, size_t src) {
	LossSample q;
	const uint2 ob = *reinterpret_cast<const uint2*>(a.mlp_out + 4 * src);
	const __half* o = reinterpret_cast<const __half*>(&ob);
	for (int k = 0; k < 4; ++k) q.raw[k] = __half2float(o[k]);
	q.rgb = mk3(network_to_rgb(q.raw[0], a.rgb_act), network_to_rgb(q.raw[1], a.rgb_act), network_to_rgb(q.raw[2], a.rgb_act));
	q.dt = unwarp_dt(a.coords[8 * src + 3]);
	q.alpha = 1.0f - __expf(-network_to_density(q.raw[3], a.density_act) * q.dt);
	return q;
}

// decay_sharpness_grid_nerf (src/testbed_nerf.cu:278-282)
__global__ void __launch_bounds__(256) k_scale_floats(float* __restrict__ x, size_t n, float f, const uint32_t* __restrict__ gate) {
	if (gate && *gate) return;
	const size_t i = (size_t)blockIdx.x * 256u + threadIdx.x;
	if (i < n) x[i] *= f;
}

// |rays_in_unnormalized[i].d| of the training ray through (u, v): the target depth is the depth
// image's value (along the optical axis) times it (src/testbed_nerf.cu:1013); the camera's
// rotation keeps lengths, so the camera-space direction's length is the one
template <bool GENERAL>
__device__ __forceinline__ float unnormalized_dir_length(const ngp_image& im, float u, float v, const float* dmap, uint32_t drx,
                                                         uint32_t dry) {
	v3 dir = mk3((u - im.principal_point[0]) * (float)im.width / im.focal_length[0],
	             (v - im.principal_point[1]) * (float)im.height / im.focal_length[1], 1.0f);
	if (GENERAL && !lens_direction(u, v, (float)im.width, (float)im.height, im.focal_length[0], im.focal_length[1],
	                               im.principal_point[0], im.principal_point[1], im.lens_mode, im.lens_params, &dir))
		return 1.0f;  // no ray through the pixel: the camera axis (src/testbed_nerf.cu:762-764)
	if (GENERAL && dmap) {
		float ddx, ddy;
		distortion_at_lerp(dmap, drx, dry, u, v, &ddx, &ddy);
		dir.x += ddx;
		dir.y += ddy;
	}
	return length(dir);
}

// compute_loss_kernel_train_nerf (testbed_nerf.cu:841-1160), pass 1: G lanes per ray (loss_lanes_per_ray),
// G samples per iteration.  Transmittance T_j = prod_{i<j}(1 - alpha_i) comes from a
// multiplicative group scan, the colour from an additive one; the ray stops at the first
// sample with T_j < 1e-4 (the reference's sequential test), found with a ballot.
template <bool GENERAL, uint32_t G>
__global__ void __launch_bounds__(256) k_loss_composite(LossArgs a) {
	const uint32_t i = blockIdx.x * (256u / G) + threadIdx.x / G;
	const uint32_t lane = threadIdx.x & 63u, r = threadIdx.x % G;
	if (i >= a.n_rays) return;  // group-uniform
	const uint32_t numsteps = a.numsteps[2 * i + 0], base = a.numsteps[2 * i + 1];
	if (numsteps == 0) {
		if (r == 0) a.ccounts[i] = 0;
		return;
	}
	float T = 1.0f;
	v3 rgb_ray = mk3(0.0f);
	float depth_ray = 0.0f;  // depth supervision: sum of weight x distance from the origin
	v3 hit = mk3(0.0f);       // sharpness: sum of weight x position (the reference's hitpoint)
	const bool depth_on = a.depth_lambda > 0.0f;
	v3 ray_o = mk3(0.0f);
	if (depth_on) ray_o = mk3(a.ray_state[8 * (size_t)i + 0], a.ray_state[8 * (size_t)i + 1], a.ray_state[8 * (size_t)i + 2]);
	uint32_t c = numsteps;
	// the chunked forward evaluated at least every sample before this ray's stop
	const uint32_t evaluated = a.ray_eval ? (a.ray_eval[i] & ~RAY_EVAL_DONE) : numsteps;
	for (uint32_t kb = 0; kb < numsteps; kb += G) {
		const uint32_t j = kb + r;
		const bool active = j < numsteps;
		LossSample q;
		if (active && j < evaluated) q = loss_sample(a, (size_t)base + j);
		else { q.alpha = 0.0f; q.rgb = mk3(0.0f); }
		const float incl = group_scan_mul<G>(1.0f - q.alpha, r);
		float excl = __shfl_up(incl, 1, G);
		if (r == 0) excl = 1.0f;
		const float Tj = T * excl;
		const unsigned long long term = group_ballot<G>(active && Tj < 1e-4f, lane);
		const uint32_t first = term ? (uint32_t)(__ffsll((long long)term) - 1) : 64u;
		const float w = (active && r < first) ? q.alpha * Tj : 0.0f;
		rgb_ray.x += __shfl(group_scan_add<G>(q.rgb.x * w, r), G - 1, G);
		rgb_ray.y += __shfl(group_scan_add<G>(q.rgb.y * w, r), G - 1, G);
		rgb_ray.z += __shfl(group_scan_add<G>(q.rgb.z * w, r), G - 1, G);
		if (a.sharp_data) {
			v3 wp = mk3(0.0f);
			if (w != 0.0f) {
				const size_t src = (size_t)base + j;
				wp = unwarp_position(mk3(a.coords[8 * src], a.coords[8 * src + 1], a.coords[8 * src + 2]), a.aabb) * w;
			}
			hit.x += __shfl(group_scan_add<G>(wp.x, r), G - 1, G);
			hit.y += __shfl(group_scan_add<G>(wp.y, r), G - 1, G);
			hit.z += __shfl(group_scan_add<G>(wp.z, r), G - 1, G);
		}
		if (depth_on) {
			float wd = 0.0f;
			if (w != 0.0f) {
				const size_t src = (size_t)base + j;
				const v3 pos = unwarp_position(mk3(a.coords[8 * src], a.coords[8 * src + 1], a.coords[8 * src + 2]), a.aabb);
				wd = w * length(pos - ray_o);
			}
			depth_ray += __shfl(group_scan_add<G>(wd, r), G - 1, G);
		}
		if (term) {
			c = kb + first;
			break;
		}
		T *= __shfl(incl, G - 1, G);
	}
	// runtime guard of the chunked forward: every sample before the stop must have been evaluated
	if (r == 0 && a.ray_eval && evaluated < c) atomicAdd(a.violations, 1u);

	// Same RNG stream as the sampler -> same pixel and background colour (testbed_nerf.cu:938-955).
	const uint32_t gi = a.ray_offset + i;
	pcg32 rng = a.rng;
	rng.advance((int64_t)gi * N_MAX_RANDOM_SAMPLES_PER_RAY);
	float u, v, pdf, uv_pdf;
	const uint32_t img =
	    training_pixel<GENERAL>(a.images, a.n_images, gi, a.n_rays_global, a.cdf, a.snap, rng, &u, &v, &pdf, &uv_pdf);
	const ngp_image im = a.images[img];
	if (a.max_level_rand) rng.advance(1);  // max_level (testbed_nerf.cu:949)
	rng.advance(1);  // motionblur_time
	v3 bg = a.bg;
	if (a.random_bg) {
		const float r0 = rng.next_float(), r1 = rng.next_float(), r2 = rng.next_float();
		bg = mk3(r0, r1, r2);
	}
	bg = mk3(srgb_to_linear(bg.x), srgb_to_linear(bg.y), srgb_to_linear(bg.z));
	float tex[4];
	texel_rgba(read_texel(im, u, v), tex);
	v3 es = mk3(1.0f);  // exposure_scale = 2^exposure[img]
	if (a.exposure) {
		const float* e = a.exposure + 3 * (size_t)img;
		es = mk3(expf(0.6931471805599453f * e[0]), expf(0.6931471805599453f * e[1]), expf(0.6931471805599453f * e[2]));
	}
	tex[0] *= es.x;
	tex[1] *= es.y;
	tex[2] *= es.z;
	v3 target;
	if (a.linear_colors || a.color_space == 0) {
		target = mk3(tex[0], tex[1], tex[2]) + bg * (1.0f - tex[3]);
		if (!a.linear_colors) {
			target = mk3(linear_to_srgb(target.x), linear_to_srgb(target.y), linear_to_srgb(target.z));
			bg = mk3(linear_to_srgb(bg.x), linear_to_srgb(bg.y), linear_to_srgb(bg.z));
		}
	} else {
		bg = mk3(linear_to_srgb(bg.x), linear_to_srgb(bg.y), linear_to_srgb(bg.z));
		if (tex[3] > 0.0f) {
			const v3 s = mk3(linear_to_srgb(tex[0] / tex[3]), linear_to_srgb(tex[1] / tex[3]), linear_to_srgb(tex[2] / tex[3]));
			target = s * tex[3] + bg * (1.0f - tex[3]);
		} else {
			target = bg;
		}
	}
	if (c == numsteps) rgb_ray = rgb_ray + bg * T;
	if (r != 0) return;
	float lx, ly, lz, gx, gy, gz;
	loss_and_gradient(target.x, rgb_ray.x, a.loss_type, &lx, &gx);
	loss_and_gradient(target.y, rgb_ray.y, a.loss_type, &ly, &gy);
	loss_and_gradient(target.z, rgb_ray.z, a.loss_type, &lz, &gz);
	float* ls = a.loss_state + 8 * (size_t)i;
	const float mean_loss = (lx / pdf + ly / pdf + lz / pdf) / 3.0f;  // lg.loss /= img_pdf * uv_pdf; mean(lg.loss)
	ls[0] = gx; ls[1] = gy; ls[2] = gz;
	ls[3] = rgb_ray.x; ls[4] = rgb_ray.y; ls[5] = rgb_ray.z;
	ls[6] = mean_loss;
	ls[7] = __uint_as_float(img);  // the error deposit (k_loss_emit) reuses the pixel
	if (a.sharp_data) a.ray_hit[i] = make_float4(hit.x, hit.y, hit.z, 0.0f);
	if (depth_on) {
		// target depth and lambda * dloss/ddepth (src/testbed_nerf.cu:1013-1015); 0 for images without depth
		float dlg = 0.0f;
		if (im.depth) {
			int px = (int)(u * (float)im.width), py = (int)(v * (float)im.height);
			px = px < 0 ? 0 : (px > (int)im.width - 1 ? (int)im.width - 1 : px);
			py = py < 0 ? 0 : (py > (int)im.height - 1 ? (int)im.height - 1 : py);
			const float target = unnormalized_dir_length<GENERAL>(im, u, v, a.dmap, a.drx, a.dry) *
			                     reinterpret_cast<const float*>(im.depth)[(size_t)px + (size_t)py * im.width];
			float ld, gd;
			loss_and_gradient(target, depth_ray, a.depth_loss_type, &ld, &gd);
			if (target > 0.0f) dlg = a.depth_lambda * gd;
		}
		a.ray_depth[i] = make_float2(depth_ray, dlg);
	}
	if (a.exposure_grad) {
		// symmetric loss: dL/dtarget = -dL/dprediction (src/testbed_nerf.cu:1121-1134)
		v3 dgt = mk3(-gx / uv_pdf, -gy / uv_pdf, -gz / uv_pdf);
		if (!a.linear_colors)
			dgt = mk3(dgt.x / srgb_to_linear_derivative(target.x), dgt.y / srgb_to_linear_derivative(target.y),
			          dgt.z / srgb_to_linear_derivative(target.z));
		const float ls_scale = 128.0f / (float)a.n_rays_global;  // LOSS_SCALE / n_rays
		a.ray_aux[i] = make_float4(ls_scale * dgt.x * es.x * 0.6931471805599453f, ls_scale * dgt.y * es.y * 0.6931471805599453f,
		                           ls_scale * dgt.z * es.z * 0.6931471805599453f, 0.0f);
	}
	if (a.store_uv_pdf) a.ray_aux[i].w = uv_pdf;
	a.ray_state[8 * (size_t)i + 6] = u;
	a.ray_state[8 * (size_t)i + 7] = v;
	a.ccounts[i] = c;
}

// Deterministic steps (ngp_train_args.deterministic): per-image gradient deposits (exposure, camera extrinsics,
// latent codes) are summed as 64-bit integers in 2^-32 units, so the sums do not depend on the order of the rays'
// atomics; k_img_fix_flush adds each step's sum to the float gradient once and clears it.  A contribution is
// clamped at +-2^62 units (+-1.07e9), far beyond any loss-scaled per-ray gradient.
constexpr double IMG_FIXED_SCALE = 4294967296.0;  // 2^32
__device__ __forceinline__ void img_deposit_fixed(unsigned long long* dst, float v) {
	const double x = fmin(fmax((double)v * IMG_FIXED_SCALE, -4.6e18), 4.6e18);
	atomicAdd(dst, (unsigned long long)(long long)rint(x));
}

__global__ void __launch_bounds__(256) k_img_fix_flush(uint32_t n, uint32_t stride, uint32_t first, uint32_t width,
                                                       unsigned long long* __restrict__ fix, float* __restrict__ dst) {
	const uint32_t i = blockIdx.x * 256u + threadIdx.x;
	if (i >= n * width) return;
	const size_t src = (size_t)(i / width) * stride + first + i % width;
	const long long v = (long long)fix[src];
	fix[src] = 0ull;
	if (v) dst[i] += (float)((double)v * (1.0 / IMG_FIXED_SCALE));
}

// pass 2: recomposite the kept samples of the ray (G lanes, G per iteration) and write
// dL/d(raw network output) with the suffix trick (testbed_nerf.cu:1061-1119) plus the
// compacted-slot -> source-sample map; consecutive lanes write consecutive slots.
template <uint32_t G>
__global__ void __launch_bounds__(256) k_loss_emit(LossArgs a) {
	const uint32_t i = blockIdx.x * (256u / G) + threadIdx.x / G;
	const uint32_t lane = threadIdx.x % G;  // the lane's rank in the ray's group
	if (i >= a.n_rays) return;
	const uint32_t n = a.ccounts[i], cbase = a.cbases[i];
	const uint32_t mc = a.max_compacted_dev ? *a.max_compacted_dev : a.max_compacted;
	const uint32_t cn = n == 0 ? 0 : min(mc - min(mc, cbase), n);
	if (lane == 0) {
		a.compacted[2 * i + 0] = cn;
		a.compacted[2 * i + 1] = cbase;
	}
	if (cn == 0) {
		if (lane == 0) a.loss_out[i] = 0.0f;
		return;
	}
	// a step the chunked forward got wrong makes no deposits: it is discarded and run again (Testbed)
	const bool deposit = !(a.viol_gate && *a.viol_gate);
	if (a.exposure_grad && lane == 0 && deposit) {
		const uint32_t img = __float_as_uint(a.loss_state[8 * (size_t)i + 7]);
		const float4 g = a.ray_aux[i];
		if (a.exposure_fix) {
			img_deposit_fixed(&a.exposure_fix[IMG_FIX_STRIDE * (size_t)img + 0], g.x);
			img_deposit_fixed(&a.exposure_fix[IMG_FIX_STRIDE * (size_t)img + 1], g.y);
			img_deposit_fixed(&a.exposure_fix[IMG_FIX_STRIDE * (size_t)img + 2], g.z);
		} else {
			atomicAdd(&a.exposure_grad[3 * (size_t)img + 0], g.x);
			atomicAdd(&a.exposure_grad[3 * (size_t)img + 1], g.y);
			atomicAdd(&a.exposure_grad[3 * (size_t)img + 2], g.z);
		}
	}
	if (a.error_map && lane == 0 && deposit) {
		// bilinear deposit of the ray's mean loss (src/testbed_nerf.cu:1028-1054; rays without
		// compacted samples returned before it); the corner clamp uses the image
		// resolution, as the reference does
		const float u = a.ray_state[8 * (size_t)i + 6], v = a.ray_state[8 * (size_t)i + 7];
		const uint32_t img = __float_as_uint(a.loss_state[8 * (size_t)i + 7]);
		const ngp_image& im = a.images[img];
		float mean_loss = a.loss_state[8 * (size_t)i + 6];
		if (a.sharp_data) {
			// include_sharpness_in_error (src/testbed_nerf.cu:1039-1047): the pixel's sharpness against the
			// running max over the grid cell of the ray's hit point (float bits order like uints for >= 0)
			const float4 h4 = a.ray_hit[i];
			const v3 hp = mk3(h4.x, h4.y, h4.z);
			if (aabb_contains(a.aabb, hp)) {
				int sx = (int)(u * (float)a.sharp_rx), sy = (int)(v * (float)a.sharp_ry);
				sx = sx < 0 ? 0 : (sx > (int)a.sharp_rx - 1 ? (int)a.sharp_rx - 1 : sx);
				sy = sy < 0 ? 0 : (sy > (int)a.sharp_ry - 1 ? (int)a.sharp_ry - 1 : sy);
				const float sharp = a.sharp_data[((size_t)img * a.sharp_ry + sy) * a.sharp_rx + sx] + 1e-6f;
				const uint32_t mip = mip_from_pos(hp, a.max_mip);
				float* cell = a.sharp_grid + (size_t)mip * NERF_GRID_N_CELLS + cascaded_grid_idx_at(hp, mip);
				const float old = __uint_as_float(atomicMax(reinterpret_cast<uint32_t*>(cell), __float_as_uint(sharp)));
				mean_loss *= fmaxf(sharp / fmaxf(sharp, old), 0.01f);
			}
		}
		const float rx = (float)a.error_map_rx, ry = (float)a.error_map_ry;
		const float px = fminf(fmaxf(u * rx - 0.5f, 0.0f), rx - (1.0f + 1e-4f));
		const float py = fminf(fmaxf(v * ry - 0.5f, 0.0f), ry - (1.0f + 1e-4f));
		const int ix = (int)px, iy = (int)py;
		const float wx = px - (float)ix, wy = py - (float)iy;
		const int cx = min(max(ix, 0), (int)im.width - 2), cy = min(max(iy, 0), (int)im.height - 2);
		float* e = a.error_map + (size_t)img * a.error_map_rx * a.error_map_ry;
		atomicAdd(&e[cy * a.error_map_rx + cx], (1.0f - wx) * (1.0f - wy) * mean_loss);
		atomicAdd(&e[cy * a.error_map_rx + cx + 1], wx * (1.0f - wy) * mean_loss);
		atomicAdd(&e[(cy + 1) * a.error_map_rx + cx], (1.0f - wx) * wy * mean_loss);
		atomicAdd(&e[(cy + 1) * a.error_map_rx + cx + 1], wx * wy * mean_loss);
	}
	const uint32_t base = a.numsteps[2 * i + 1];
	const float* ls = a.loss_state + 8 * (size_t)i;
	const v3 grad = mk3(ls[0], ls[1], ls[2]);
	const v3 rgb_ray = mk3(ls[3], ls[4], ls[5]);
	if (lane == 0) a.loss_out[i] = ls[6] / (float)a.n_rays_global;
	const float loss_scale = 128.0f / (float)a.n_rays_global;  // LOSS_SCALE / n_rays (testbed_nerf.cu:1056)
	const float output_l2_reg = a.rgb_act == ACT_EXP ? 1e-4f : 0.0f;
	const float output_l1_reg_density = *a.mean_density < NERF_MIN_OPTICAL_THICKNESS ? 1e-4f : 0.0f;
	const v3 ray_o = mk3(a.ray_state[8 * (size_t)i + 0], a.ray_state[8 * (size_t)i + 1], a.ray_state[8 * (size_t)i + 2]);

	v3 acc = mk3(0.0f);
	float T = 1.0f;
	// depth supervision: the ray's composited depth and lambda * dloss/ddepth (0: no term)
	const float2 rdep = a.depth_lambda > 0.0f ? a.ray_depth[i] : make_float2(0.0f, 0.0f);
	float dacc = 0.0f;
	for (uint32_t kb = 0; kb < cn; kb += G) {
		const uint32_t j = kb + lane;
		const bool active = j < cn;
		const size_t src = (size_t)base + j, dst = (size_t)cbase + j;
		LossSample q;
		if (active) q = loss_sample(a, src);
		else { q.alpha = 0.0f; q.rgb = mk3(0.0f); q.dt = 0.0f; q.raw[0] = q.raw[1] = q.raw[2] = q.raw[3] = 0.0f; }
		const float incl = group_scan_mul<G>(1.0f - q.alpha, lane);
		float excl = __shfl_up(incl, 1, G);
		if (lane == 0) excl = 1.0f;
		const float Tj = T * excl, Tnext = T * incl;
		const float weight = q.alpha * Tj;
		const v3 pre = mk3(group_scan_add<G>(q.rgb.x * weight, lane), group_scan_add<G>(q.rgb.y * weight, lane),
		                   group_scan_add<G>(q.rgb.z * weight, lane));
		const v3 rgb_ray2 = acc + pre;
		float depth = 0.0f;
		if (active) {
			const float4 c0 = *reinterpret_cast<const float4*>(a.coords + 8 * src);
			depth = length(unwarp_position(mk3(c0.x, c0.y, c0.z), a.aabb) - ray_o);
		}
		// depth supervision: inclusive prefix of weight x depth over the ray's samples (depth_ray2)
		const float dpre = rdep.y != 0.0f ? group_scan_add<G>(weight * depth, lane) : 0.0f;
		if (active) {
			a.csrc[dst] = (uint32_t)src;
			const v3 suffix = rgb_ray - rgb_ray2;
			const v3 dloss_by_drgb = grad * weight;
			const float o0 = q.raw[0], o1 = q.raw[1], o2 = q.raw[2], o3 = q.raw[3];
			__half dl[4];
			dl[0] = __float2half(loss_scale * (dloss_by_drgb.x * network_to_rgb_derivative(o0, a.rgb_act) + fmaxf(0.0f, output_l2_reg * o0)));
			dl[1] = __float2half(loss_scale * (dloss_by_drgb.y * network_to_rgb_derivative(o1, a.rgb_act) + fmaxf(0.0f, output_l2_reg * o1)));
			dl[2] = __float2half(loss_scale * (dloss_by_drgb.z * network_to_rgb_derivative(o2, a.rgb_act) + fmaxf(0.0f, output_l2_reg * o2)));
			const float density_derivative = network_to_density_derivative(o3, a.density_act);
			const float drgb = dot(grad, q.rgb * Tnext - suffix);
			// depth_supervision = lambda dloss/ddepth x (T depth - depth suffix)  (src/testbed_nerf.cu:1098-1103)
			const float dsum = rdep.y != 0.0f ? drgb + rdep.y * (Tnext * depth - (rdep.x - (dacc + dpre))) : drgb;
			const float dloss_by_dmlp = density_derivative * (q.dt * dsum);
			dl[3] = __float2half(loss_scale * dloss_by_dmlp + (o3 < 0.0f ? -output_l1_reg_density : 0.0f) +
			                     (o3 > -10.0f && depth < a.near_distance ? 1e-4f : 0.0f));
			*reinterpret_cast<uint2*>(a.dloss + 4 * dst) = *reinterpret_cast<const uint2*>(dl);
		}
		acc = acc + mk3(__shfl(pre.x, G - 1, G), __shfl(pre.y, G - 1, G), __shfl(pre.z, G - 1, G));
		if (rdep.y != 0.0f) dacc += __shfl(dpre, G - 1, G);
		T *= __shfl(incl, G - 1, G);
	}
}

// ---------------------------------------------------------------------------
// Camera extrinsics gradient: compute_cam_gradient_train_nerf (src/testbed_nerf.cu:1163-1269).
// Per ray, over its compacted samples: the position gradient (dL/d warped position ÷ the
// AABB size) adds to the origin gradient and, times the sample's distance from the origin,
// to the direction gradient, together with dL/d direction through the SH encoding (the
// warp's 0.5 and the SH input's 2x - 1 cancel).  Image translation += origin gradient,
// rotation += cross(dir, dir gradient), each divided by the pixel pdf.
// ---------------------------------------------------------------------------
// dL/d(x, y, z) of the degree-4 SH basis (sh4_slice, mlp.hip) at (x, y, z) = 2 wd - 1
__device__ __forceinline__ v3 sh4_input_grad(const float* wd, const float* dsh) {
	const float x = wd[0] * 2.0f - 1.0f, y = wd[1] * 2.0f - 1.0f, z = wd[2] * 2.0f - 1.0f;
	const float x2 = x * x, y2 = y * y, z2 = z * z;
	float gx = 0.0f, gy = 0.0f, gz = 0.0f;
	gy += dsh[1] * -0.48860251190291987f;
	gz += dsh[2] * 0.48860251190291987f;
	gx += dsh[3] * -0.48860251190291987f;
	gx += dsh[4] * 1.0925484305920792f * y;
	gy += dsh[4] * 1.0925484305920792f * x;
	gy += dsh[5] * -1.0925484305920792f * z;
	gz += dsh[5] * -1.0925484305920792f * y;
	gz += dsh[6] * 2.0f * 0.94617469575755997f * z;
	gx += dsh[7] * -1.0925484305920792f * z;
	gz += dsh[7] * -1.0925484305920792f * x;
	gx += dsh[8] * 2.0f * 0.54627421529603959f * x;
	gy += dsh[8] * -2.0f * 0.54627421529603959f * y;
	gx += dsh[9] * 0.59004358992664352f * (-6.0f * x * y);
	gy += dsh[9] * 0.59004358992664352f * (-3.0f * x2 + 3.0f * y2);
	gx += dsh[10] * 2.8906114426405538f * y * z;
	gy += dsh[10] * 2.8906114426405538f * x * z;
	gz += dsh[10] * 2.8906114426405538f * x * y;
	gy += dsh[11] * 0.45704579946446572f * (1.0f - 5.0f * z2);
	gz += dsh[11] * 0.45704579946446572f * (-10.0f * y * z);
	gz += dsh[12] * 0.3731763325901154f * (15.0f * z2 - 3.0f);
	gx += dsh[13] * 0.45704579946446572f * (1.0f - 5.0f * z2);
	gz += dsh[13] * 0.45704579946446572f * (-10.0f * x * z);
	gx += dsh[14] * 1.4453057213202769f * 2.0f * x * z;
	gy += dsh[14] * 1.4453057213202769f * -2.0f * y * z;
	gz += dsh[14] * 1.4453057213202769f * (x2 - y2);
	gx += dsh[15] * 0.59004358992664352f * (-3.0f * x2 + 3.0f * y2);
	gy += dsh[15] * 0.59004358992664352f * (6.0f * x * y);
	return mk3(gx, gy, gz);
}

struct CamGradArgs {
	uint32_t n_rays;
	aabb3 aabb;
	const uint32_t* compacted;   // [R][2] (count, base) in the compacted batch
	const float* ray_state;      // [R][8] o, d
	const float* loss_state;     // [R][8]: [7] image
	const float4* ray_aux;       // [R]: w = pixel pdf
	const float* ccoords;        // [B][8]
	const float* dpos;           // [B][3]
	const float* dsh;            // [B][16]
	float* cam_pos_gradient;     // [n_images][3] (null: off)
	float* cam_rot_gradient;     // [n_images][3]
	unsigned long long* cam_fix; // deterministic steps: [n_images][IMG_FIX_STRIDE], pos at 3, rot at 6 (null: float atomics)
	const ngp_image* images;     // the images' current transforms (distortion gradient)
	const uint32_t* viol_gate;   // non-zero: the step is discarded and re-run -- no deposits
	float* dgrad;                // distortion map gradient / weight [dry][drx][2] (null: off)
	float* dgrad_w;
	uint32_t drx, dry;
};

// deposit_image_gradient (common_device.cuh:82-115): value into the four texels around res * uv,
// bilinear weights, clamped to the edge; the weights into the weight buffer
__device__ __forceinline__ void deposit_image_gradient(float gx, float gy, float* grad, float* gw, uint32_t rx, uint32_t ry,
                                                       float u, float v) {
	const float fx = (float)rx * u, fy = (float)ry * v;
	const int px = (int)fx, py = (int)fy;
	const float wx = fx - (float)px, wy = fy - (float)py;
#pragma unroll
	for (int k = 0; k < 4; ++k) {
		const float w = (k & 1 ? wx : 1.0f - wx) * (k & 2 ? wy : 1.0f - wy);
		int x = px + (k & 1), y = py + (k >> 1);
		x = x > (int)rx - 1 ? (int)rx - 1 : (x < 0 ? 0 : x);
		y = y > (int)ry - 1 ? (int)ry - 1 : (y < 0 ? 0 : y);
		const size_t o = 2 * ((size_t)x + (size_t)y * rx);
		atomicAdd(&grad[o], gx * w);
		atomicAdd(&gw[o], w);
		atomicAdd(&grad[o + 1], gy * w);
		atomicAdd(&gw[o + 1], w);
	}
}

__global__ void __launch_bounds__(256) k_cam_gradient(CamGradArgs a) {
	const uint32_t i = blockIdx.x * 256u + threadIdx.x;
	if (i >= a.n_rays || (a.viol_gate && *a.viol_gate)) return;
	const uint32_t cn = a.compacted[2 * i], cbase = a.compacted[2 * i + 1];
	if (cn == 0) return;
	const float* rs = a.ray_state + 8 * (size_t)i;
	const v3 o = mk3(rs[0], rs[1], rs[2]), d = mk3(rs[3], rs[4], rs[5]);
	const v3 inv_diag = mk3(1.0f / (a.aabb.max.x - a.aabb.min.x), 1.0f / (a.aabb.max.y - a.aabb.min.y),
	                        1.0f / (a.aabb.max.z - a.aabb.min.z));
	v3 go = mk3(0.0f), gd = mk3(0.0f);
	for (uint32_t j = 0; j < cn; ++j) {
		const size_t s = (size_t)cbase + j;
		const float* c = a.ccoords + 8 * s;
		const v3 pg = mk3(a.dpos[3 * s], a.dpos[3 * s + 1], a.dpos[3 * s + 2]) * inv_diag;
		go = go + pg;
		const v3 pos = unwarp_position(mk3(c[0], c[1], c[2]), a.aabb);
		const float t = length(pos - o);
		gd = gd + pg * t + sh4_input_grad(c + 4, a.dsh + 16 * s);
	}
	const uint32_t img = __float_as_uint(a.loss_state[8 * (size_t)i + 7]);
	const float inv_pdf = 1.0f / a.ray_aux[i].w;
	if (a.dgrad) {
		// the direction gradient's component orthogonal to the direction, rotated back into the
		// camera's frame (inverse(mat3(xform)) * g), its xy splatted at the pixel (divided by the pdf)
		const v3 og = gd - d * dot(gd, d);
		const m43 xf = load_xform(a.images[img].xform);
		const v3 ip = inverse3_mul(xf, og);
		deposit_image_gradient(ip.x / a.ray_aux[i].w, ip.y / a.ray_aux[i].w, a.dgrad, a.dgrad_w, a.drx, a.dry, rs[6], rs[7]);
	}
	if (!a.cam_pos_gradient) return;
	const v3 aa = mk3(d.y * gd.z - d.z * gd.y, d.z * gd.x - d.x * gd.z, d.x * gd.y - d.y * gd.x);
	if (a.cam_fix) {
		unsigned long long* f = a.cam_fix + IMG_FIX_STRIDE * (size_t)img;
		img_deposit_fixed(f + 3, go.x * inv_pdf);
		img_deposit_fixed(f + 4, go.y * inv_pdf);
		img_deposit_fixed(f + 5, go.z * inv_pdf);
		img_deposit_fixed(f + 6, aa.x * inv_pdf);
		img_deposit_fixed(f + 7, aa.y * inv_pdf);
		img_deposit_fixed(f + 8, aa.z * inv_pdf);
		return;
	}
	atomicAdd(&a.cam_pos_gradient[3 * (size_t)img + 0], go.x * inv_pdf);
	atomicAdd(&a.cam_pos_gradient[3 * (size_t)img + 1], go.y * inv_pdf);
	atomicAdd(&a.cam_pos_gradient[3 * (size_t)img + 2], go.z * inv_pdf);
	atomicAdd(&a.cam_rot_gradient[3 * (size_t)img + 0], aa.x * inv_pdf);
	atomicAdd(&a.cam_rot_gradient[3 * (size_t)img + 1], aa.y * inv_pdf);
	atomicAdd(&a.cam_rot_gradient[3 * (size_t)img + 2], aa.z * inv_pdf);
}

// compute_extra_dims_gradient_train_nerf (src/testbed_nerf.cu:1271-1306): the ray's compacted samples' dL/d(latent
// code) summed into its image's gradient (one thread per ray, E float atomics; loss-scaled like the reference's)
__global__ void __launch_bounds__(256) k_extra_gradient(uint32_t n_rays, const uint32_t* __restrict__ compacted,
                                                        const float* __restrict__ loss_state, const float* __restrict__ dextra,
                                                        uint32_t E, float* __restrict__ grad, const uint32_t* __restrict__ viol_gate,
                                                        unsigned long long* __restrict__ fix) {
	const uint32_t i = blockIdx.x * 256u + threadIdx.x;
	if (i >= n_rays || (viol_gate && *viol_gate)) return;
	const uint32_t cn = compacted[2 * i], cbase = compacted[2 * i + 1];
	if (cn == 0) return;
	float g[NGP_EXTRA_ROW];
#pragma unroll
	for (uint32_t k = 0; k < NGP_EXTRA_ROW; ++k) g[k] = 0.0f;
	const uint32_t nq = E > 16 ? NGP_EXTRA_ROW / 4 : 4;  // float4s of a row holding the E components
	for (uint32_t j = 0; j < cn; ++j) {
		const float4* src = reinterpret_cast<const float4*>(dextra + NGP_EXTRA_ROW * ((size_t)cbase + j));
#pragma unroll
		for (uint32_t q = 0; q < NGP_EXTRA_ROW / 4; ++q) {
			if (q >= nq) break;
			const float4 v = src[q];
			g[4 * q] += v.x;
			g[4 * q + 1] += v.y;
			g[4 * q + 2] += v.z;
			g[4 * q + 3] += v.w;
		}
	}
	const uint32_t img = __float_as_uint(loss_state[8 * (size_t)i + 7]);
#pragma unroll
	for (uint32_t k = 0; k < NGP_EXTRA_ROW; ++k) {
		if (k >= E) continue;
		if (fix) img_deposit_fixed(&fix[IMG_FIX_STRIDE * (size_t)img + 9 + k], g[k]);
		else atomicAdd(&grad[NGP_EXTRA_ROW * (size_t)img + k], g[k]);
	}
}

// Rollover multiplicity (tcnn fill_rollover_and_rescale, folded): compacted sample j of
// c < B is repeated floor((B-1-j)/c) more times, each copy scaled by c/B.  Data parallel (dp =
// DpCaps of the compaction): the rank's sample j is global sample base + j of the global batch.
__device__ __forceinline__ float rollover_weight(uint32_t j, uint32_t n, uint32_t target, const uint32_t* __restrict__ dp) {
	const uint32_t c = dp ? dp[1] : n, g = dp ? dp[0] + j : j;
	const uint32_t copies = (target - 1 - g) / c;
	return 1.0f + (float)copies * ((float)c / (float)target);
}

// Sum of per-ray losses by one 256-thread workgroup, in the order of a 1024-thread two-level
// reduction (thread t of 1024 sums v[t], v[t + 1024], ...; then a halving tree), so the result
// does not depend on the launch.
__device__ void block_sum_losses(const float* __restrict__ v, uint32_t n, float* __restrict__ out) {
	__shared__ float part[1024];
	for (uint32_t q = 0; q < 4; ++q) {
		const uint32_t t = threadIdx.x + 256u * q;
		float s = 0.0f;
		for (uint32_t i = t; i < n; i += 1024) s += v[i];
		part[t] = s;
	}
	__syncthreads();
	for (uint32_t d = 512; d > 0; d >>= 1) {
		for (uint32_t t = threadIdx.x; t < d; t += 256u) part[t] += part[t + d];
		__syncthreads();
	}
	if (threadIdx.x == 0) *out = part[0];
}

struct CompactFinish {
	const uint32_t* total;    // compacted samples (the loss kernels' count)
	const uint32_t* cap_dev;  // data parallel: the rank's share of the cap (device); null: target
	uint32_t* n_out;          // min(total, cap): the count the kernels after the gather read
	const uint32_t* dp;       // DpCaps of the compaction (data parallel) or null
	float* weight;            // [B] rollover weight per compacted sample
	const float* loss;        // [R] per-ray losses
	uint32_t n_rays;
	float* loss_sum;
};

// The end of the loss stage in one launch: the compacted count, the gather of the compacted batch
// (coords + per-level features) in compacted order -- one thread per compacted sample, so every level
// plane is written by contiguous lanes -- with each sample's rollover weight, and, in the extra last
// workgroup, the sum of the per-ray losses.
template <uint32_t F>
__global__ void __launch_bounds__(256) k_gather_compacted(CompactFinish cf, const uint32_t* __restrict__ csrc,
                                                          const float* __restrict__ coords, const __half* __restrict__ enc,
                                                          EncLayout src_layout, EncLayout dst_layout, uint32_t n_levels, float* __restrict__ ccoords,
                                                          float4* __restrict__ cpos4, __half* __restrict__ cenc, uint32_t target,
                                                          const uint32_t* __restrict__ eidx, const uint32_t* __restrict__ simg,
                                                          uint32_t* __restrict__ cimg) {
	if (blockIdx.x == gridDim.x - 1) {
		block_sum_losses(cf.loss, cf.n_rays, cf.loss_sum);
		return;
	}
	const uint32_t n = min(*cf.total, cf.cap_dev ? *cf.cap_dev : target);
	const uint32_t dst = blockIdx.x * 256u + threadIdx.x;
	if (dst == 0) *cf.n_out = n;  // (no reader in this launch)
	if (dst >= n) return;
	cf.weight[dst] = rollover_weight(dst, n, target, cf.dp);
	const uint32_t src = csrc[dst];
	if (cimg) cimg[dst] = simg[src];  // n_extra_dims > 0: the sample's image (latent-code row)
	const uint32_t esrc = eidx ? eidx[src] : src;  // row of the sample's encoding
	const float4* ci = reinterpret_cast<const float4*>(coords + 8 * (size_t)src);
	float4* co = reinterpret_cast<float4*>(ccoords + 8 * (size_t)dst);
	const float4 c0 = ci[0];
	co[0] = c0;
	co[1] = ci[1];
	cpos4[dst] = c0;
	using VT = typename std::conditional<F == 1, uint16_t, typename std::conditional<F == 2, uint32_t,
	                                     typename std::conditional<F == 4, uint2, uint4>::type>::type>::type;
	const VT* es = reinterpret_cast<const VT*>(enc);
	VT* ed = reinterpret_cast<VT*>(cenc);
	if (src_layout.lsh == 2 && dst_layout.lsh == 2) {
		// whole planes: four levels' features in one vector
		struct alignas(4 * sizeof(VT)) Plane { VT v[4]; };
		const Plane* ps = reinterpret_cast<const Plane*>(enc);
		Plane* pd = reinterpret_cast<Plane*>(cenc);
		for (uint32_t l = 0; l < n_levels; l += 4)
			pd[(size_t)(l >> 2) * dst_layout.plane + dst] = ps[(size_t)(l >> 2) * src_layout.plane + esrc];
	} else {
		for (uint32_t l = 0; l < n_levels; ++l) ed[dst_layout.vec(l, dst)] = es[src_layout.vec(l, esrc)];
	}
}

// Data parallelism (ngp_train_args.world_size > 1): each rank writes its total into its slot of
// [world] words (the others zero), the caller's all-reduce sums them, and every rank derives the
// same global prefix -- so caps and rollover follow the global ray order of one process.
// extra (optional): one more word summed over the ranks, in slots[world] (the chunked forward's violations)
__global__ void k_dp_publish(const uint32_t* __restrict__ total, int32_t* __restrict__ slots, uint32_t world, uint32_t rank,
                             const uint32_t* __restrict__ extra) {
	for (uint32_t q = threadIdx.x; q < world; q += blockDim.x) slots[q] = q == rank ? (int32_t)*total : 0;
	if (extra && threadIdx.x == 0) slots[world] = (int32_t)*extra;
}
// DpCaps: [0] this rank's first global index, [1] min(global total, cap), [2] this rank's share of
// the cap (cap - base, 0 once the ranks before it filled it).  local_cap: the rank's buffer capacity;
// a share it cannot hold (min(own total, share) > local_cap) flags the step (VIOL_CAPACITY in *viol,
// the need in *need): the Testbed discards it and runs it again with buffers grown to the need.
__global__ void k_dp_caps(const int32_t* __restrict__ slots, uint32_t world, uint32_t rank, uint32_t cap,
                          uint32_t* __restrict__ out, uint32_t local_cap, uint32_t* __restrict__ viol, uint32_t* __restrict__ need) {
	if (threadIdx.x || blockIdx.x) return;
	uint64_t base = 0, total = 0;
	for (uint32_t q = 0; q < world; ++q) {
		const uint64_t v = (uint32_t)slots[q];
		if (q < rank) base += v;
		total += v;
	}
	out[0] = (uint32_t)min<uint64_t>(base, 0xffffffffull);
	out[1] = (uint32_t)min<uint64_t>(total, cap);
	out[2] = base >= cap ? 0u : (uint32_t)(cap - base);
	if (viol) {
		const uint32_t want = min((uint32_t)slots[rank], out[2]);
		if (want > local_cap) {
			*viol |= VIOL_CAPACITY;
			*need = want;
			out[2] = local_cap;  // stay inside the buffers; the step is discarded
		}
	}
}

// ---------------------------------------------------------------------------
// Optimizer: Ema( ExponentialDecay( Adam ) ) in one pass over the parameters.
// ---------------------------------------------------------------------------
struct OptArgs {
	uint64_t n, n_mlp;
	float lr, beta1, beta2, eps, l2_reg, loss_scale;
	float ema_decay, ema_debias_old, ema_debias_new;
	int opt_mlp, opt_enc;
	float* w32;
	__half* w16;
	float* grad;      // MLP gradients (fp32), [0, n_mlp)
	__half* grad16;   // hash-grid gradients (fp16), [n_mlp, n)
	long long* grad64;  // deterministic steps: hash-grid gradients in 2^-40 fixed point (replaces grad16)
	const uint32_t* skip;  // chunked forward violations of the step: non-zero = no update at all
	float* m;
	float* v;
	uint32_t* steps;
	float* ema32;
	__half* ema16;
	const float2* corr;  // Adam bias corrections by step count, [0, corr_n) (k_adam_corr)
	uint32_t corr_n;
};

// {sqrt(1 - beta2^n), 1 - beta1^n} for n in [lo, hi): the expressions adam_update evaluates otherwise,
// so a table entry and the inline evaluation are the same float
__global__ void k_adam_corr(float beta1, float beta2, uint32_t lo, uint32_t hi, float2* __restrict__ corr) {
	const uint32_t n = lo + blockIdx.x * 256u + threadIdx.x;
	if (n >= hi) return;
	corr[n] = make_float2(sqrtf(1.0f - powf(beta2, (float)n)), 1.0f - powf(beta1, (float)n));
}

// One parameter's Adam step (shared by both optimizer kernels, so their arithmetic is identical).
__device__ __forceinline__ bool adam_update(const OptArgs& a, bool is_mlp, float graw, float& w, float& m, float& v,
                                            uint32_t& step) {
	const bool update = is_mlp ? (bool)a.opt_mlp : (a.opt_enc && graw != 0.0f);
	if (!update) return false;
	float g = graw / a.loss_scale;
	if (is_mlp) g += a.l2_reg * w;
	m = a.beta1 * m + (1.0f - a.beta1) * g;
	v = a.beta2 * v + (1.0f - a.beta2) * g * g;
	step = step + 1u;
	float lr;
	if (step < a.corr_n) {
		const float2 c = a.corr[step];
		lr = a.lr * c.x / c.y;
	} else {
		lr = a.lr * sqrtf(1.0f - powf(a.beta2, (float)step)) / (1.0f - powf(a.beta1, (float)step));
	}
	w = w - (lr / (sqrtf(v) + a.eps)) * m;
	return true;
}

__device__ __forceinline__ float ema_update(const OptArgs& a, float e, float w) {
	return (e * a.ema_decay * a.ema_debias_old + w * (1.0f - a.ema_decay)) / a.ema_debias_new;
}

// deterministic hash-grid gradients are the exact sum rounded to fp16 once -- the precision the fp16
// buffer holds, so the sparse skip of zero gradients (a sum below fp16's range is zero) matches
__device__ __forceinline__ float fixed_grad(long long q) { return __half2float(__float2half((float)q * GRAD_FIXED_INV)); }

__device__ __forceinline__ void optimize_one(const OptArgs& a, uint64_t i) {
	const bool is_mlp = i < a.n_mlp;
	float graw;
	if (is_mlp) graw = a.grad[i];
	else if (a.grad64) graw = fixed_grad(a.grad64[i - a.n_mlp]);
	else graw = __half2float(a.grad16[i - a.n_mlp]);
	float w = a.w32[i];
	float m, v;
	uint32_t st;
	const bool is_upd = is_mlp ? (bool)a.opt_mlp : (a.opt_enc && graw != 0.0f);
	if (is_upd) {
		m = a.m[i];
		v = a.v[i];
		st = a.steps[i];
		adam_update(a, is_mlp, graw, w, m, v, st);
		a.m[i] = m;
		a.v[i] = v;
		a.steps[i] = st;
		a.w32[i] = w;
		a.w16[i] = __float2half(w);
	}
	// GradientMode::Overwrite for the next step; a fixed-point sum that rounds to fp16 zero is cleared too (its
	// residue must not carry into the next step's sum)
	if (is_mlp) {
		if (graw != 0.0f) a.grad[i] = 0.0f;
	} else if (a.grad64) {
		if (a.grad64[i - a.n_mlp] != 0) a.grad64[i - a.n_mlp] = 0;
	} else if (graw != 0.0f) {
		a.grad16[i - a.n_mlp] = __float2half(0.0f);
	}
	const float e = ema_update(a, a.ema32[i], w);
	a.ema32[i] = e;
	a.ema16[i] = __float2half(e);
}

__global__ void __launch_bounds__(256) k_optimizer(OptArgs a) {
	const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
	if (i >= a.n) return;
	// a step whose chunked forward missed samples is dropped whole; the caller re-runs it
	// (ngp_train_discard + full_forward) -- every thread reads the same word
	if (a.skip && *a.skip) return;
	optimize_one(a, i);
}

// The same update, 8 consecutive parameters per thread with 16-B loads and stores (the one-per-thread
// kernel moves 2- and 4-B words per lane and reached half of the HBM rate).  Needs n_mlp % 8 == 0, so a
// group lies wholly in the MLP or the grid part; Adam's moments and step counts are read only for groups
// with an update (the grid's sparse skip).
__device__ __forceinline__ void ld8(const float* p, float (&x)[8]) {
	const float4 u = reinterpret_cast<const float4*>(p)[0], v = reinterpret_cast<const float4*>(p)[1];
	x[0] = u.x, x[1] = u.y, x[2] = u.z, x[3] = u.w, x[4] = v.x, x[5] = v.y, x[6] = v.z, x[7] = v.w;
}
__device__ __forceinline__ void st8(float* p, const float (&x)[8]) {
	reinterpret_cast<float4*>(p)[0] = make_float4(x[0], x[1], x[2], x[3]);
	reinterpret_cast<float4*>(p)[1] = make_float4(x[4], x[5], x[6], x[7]);
}
__device__ __forceinline__ void st8h(__half* p, const float (&x)[8]) {
	uint4 u;
	uint32_t* w = reinterpret_cast<uint32_t*>(&u);
#pragma unroll
	for (int k = 0; k < 4; ++k) {
		const __half2 h = __halves2half2(__float2half(x[2 * k]), __float2half(x[2 * k + 1]));
		w[k] = *reinterpret_cast<const uint32_t*>(&h);
	}
	*reinterpret_cast<uint4*>(p) = u;
}

__global__ void __launch_bounds__(256) k_optimizer8(OptArgs a) {
	const uint64_t i0 = ((uint64_t)blockIdx.x * 256u + threadIdx.x) * 8u;
	if (i0 >= a.n) return;
	if (a.skip && *a.skip) return;
	if (i0 + 8 > a.n) {
		for (uint64_t i = i0; i < a.n; ++i) optimize_one(a, i);
		return;
	}
	const bool is_mlp = i0 < a.n_mlp;
	const uint64_t gi = i0 - a.n_mlp;
	float g[8];
	bool q_nz = false;  // fixed point: any raw sum non-zero (one that rounds to fp16 zero is cleared as well)
	if (is_mlp) {
		ld8(a.grad + i0, g);
	} else if (a.grad64) {
		const longlong2* q = reinterpret_cast<const longlong2*>(a.grad64 + gi);
#pragma unroll
		for (int k = 0; k < 4; ++k) {
			const longlong2 t = q[k];
			g[2 * k] = fixed_grad(t.x);
			g[2 * k + 1] = fixed_grad(t.y);
			q_nz |= (t.x | t.y) != 0;
		}
	} else {
		const uint4 u = *reinterpret_cast<const uint4*>(a.grad16 + gi);
		const __half* h = reinterpret_cast<const __half*>(&u);
#pragma unroll
		for (int k = 0; k < 8; ++k) g[k] = __half2float(h[k]);
	}
	float w[8];
	ld8(a.w32 + i0, w);
	uint32_t upd = 0, nz = 0;
#pragma unroll
	for (int k = 0; k < 8; ++k) {
		if (is_mlp ? (bool)a.opt_mlp : (a.opt_enc && g[k] != 0.0f)) upd |= 1u << k;
		if (g[k] != 0.0f) nz |= 1u << k;
	}
	if (upd) {
		float m[8], v[8];
		ld8(a.m + i0, m);
		ld8(a.v + i0, v);
		uint4 s0 = reinterpret_cast<const uint4*>(a.steps + i0)[0], s1 = reinterpret_cast<const uint4*>(a.steps + i0)[1];
		uint32_t st[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
#pragma unroll
		for (int k = 0; k < 8; ++k) adam_update(a, is_mlp, g[k], w[k], m[k], v[k], st[k]);
		st8(a.m + i0, m);
		st8(a.v + i0, v);
		reinterpret_cast<uint4*>(a.steps + i0)[0] = make_uint4(st[0], st[1], st[2], st[3]);
		reinterpret_cast<uint4*>(a.steps + i0)[1] = make_uint4(st[4], st[5], st[6], st[7]);
		st8(a.w32 + i0, w);
		if (upd == 0xffu) {
			st8h(a.w16 + i0, w);
		} else {
			// parameters without an update keep their fp16 copy untouched
			uint4 old = *reinterpret_cast<const uint4*>(a.w16 + i0);
			__half* oh = reinterpret_cast<__half*>(&old);
#pragma unroll
			for (int k = 0; k < 8; ++k)
				if ((upd >> k) & 1u) oh[k] = __float2half(w[k]);
			*reinterpret_cast<uint4*>(a.w16 + i0) = old;
		}
	}
	if (nz || q_nz) {  // GradientMode::Overwrite for the next step (zeros where they already are change nothing)
		if (is_mlp) reinterpret_cast<float4*>(a.grad + i0)[0] = reinterpret_cast<float4*>(a.grad + i0)[1] = make_float4(0.f, 0.f, 0.f, 0.f);
		else if (a.grad64) {
#pragma unroll
			for (int k = 0; k < 4; ++k) reinterpret_cast<longlong2*>(a.grad64 + gi)[k] = make_longlong2(0, 0);
		} else *reinterpret_cast<uint4*>(a.grad16 + gi) = make_uint4(0u, 0u, 0u, 0u);
	}
	float e[8];
	ld8(a.ema32 + i0, e);
#pragma unroll
	for (int k = 0; k < 8; ++k) e[k] = ema_update(a, e[k], w[k]);
	st8(a.ema32 + i0, e);
	st8h(a.ema16 + i0, e);
}

__global__ void k_to_half(const float* __restrict__ src, __half* __restrict__ dst, uint64_t n) {
	const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
	if (i < n) dst[i] = __float2half(src[i]);
}

void launch_params_to_half(const float* src, __half* dst, size_t n, hipStream_t s) {
	if (!n) return;
	k_to_half<<<div_up(n, 256), 256, 0, s>>>(src, dst, n);
	NGP_HIP_CHECK(hipGetLastError());
}

void launch_optimizer(ngp_model* m, uint32_t step, int opt_mlp, int opt_enc, hipStream_t s) {
	const ngp_network_config& c = m->cfg;
	OptArgs a{};
	a.n = m->n_params;
	a.n_mlp = m->n_mlp_params;
	// ExponentialDecay (configs/nerf/base.json:9-14): lr *= base at decay_start + k*interval
	a.lr = exp_decay_learning_rate(c.learning_rate, c.decay_base, c.decay_start, c.decay_interval, 0xFFFFFFFFu, step);
	a.beta1 = c.beta1;
	a.beta2 = c.beta2;
	a.eps = c.epsilon;
	a.l2_reg = c.l2_reg;
	a.loss_scale = 128.0f;
	a.ema_decay = c.ema_decay;
	a.ema_debias_old = 1.0f - powf(c.ema_decay, (float)m->ema_step);
	a.ema_debias_new = 1.0f - powf(c.ema_decay, (float)(m->ema_step + 1));
	a.opt_mlp = opt_mlp;
	a.opt_enc = opt_enc;
	a.w32 = m->params32.ptr;
	a.w16 = m->params16.ptr;
	a.grad = m->grads.ptr;
	a.grad16 = m->grid_grads16.ptr;
	a.grad64 = m->ts.fixed ? m->grid_grads64.ptr : nullptr;
	// the step's violation word gates its update (ngp_train_discard re-runs it): the chunked forward's early
	// stops and, in data-parallel training, VIOL_CAPACITY (a rank's share did not fit its buffers) -- which the
	// full forward can raise too, so the gate does not depend on the forward's mode
	a.skip = m->ts.counters.ptr ? m->ts.counters.ptr + 9 : nullptr;
	if (a.skip) m->ts.gated_optimizer_ran = true;
	a.m = m->adam_m.ptr;
	a.v = m->adam_v.ptr;
	a.steps = m->adam_steps.ptr;
	a.ema32 = m->ema32.ptr;
	a.ema16 = m->infer16.ptr;
	// bias-correction table up to step + 2 (a parameter's count is at most the optimizer steps taken;
	// larger counts, e.g. restored from a snapshot, fall back to the inline evaluation)
	{
		const uint32_t need = std::min<uint32_t>(step, 1u << 20) + 2u;
		if (m->adam_corr_b1 != c.beta1 || m->adam_corr_b2 != c.beta2) m->adam_corr_n = 0;
		if (need > m->adam_corr_n) {
			uint32_t lo = m->adam_corr_n;
			if ((size_t)need * 2 > m->adam_corr.n) {
				m->adam_corr.reserve((size_t)std::max<uint32_t>(need * 2u, 1u << 16) * 2);  // grows: refill all
				lo = 0;
			}
			// 4096 steps ahead (entries past a parameter's count are never read), so the table is
			// extended once per 4096 optimizer steps instead of once per step
			const uint32_t fill = std::min<uint32_t>((need + 4095u) & ~4095u, (uint32_t)(m->adam_corr.n / 2));
			k_adam_corr<<<div_up(fill - lo, 256u), 256, 0, s>>>(c.beta1, c.beta2, lo, fill, reinterpret_cast<float2*>(m->adam_corr.ptr));
			NGP_HIP_CHECK(hipGetLastError());
			m->adam_corr_n = fill;
			m->adam_corr_b1 = c.beta1;
			m->adam_corr_b2 = c.beta2;
		}
	}
	a.corr = reinterpret_cast<const float2*>(m->adam_corr.ptr);
	a.corr_n = m->adam_corr_n;
	m->timers.begin_kernel(NGP_TIMER_OPTIMIZER);
	if (a.n_mlp % 8 == 0) launch_timed(k_optimizer8, div_up(div_up(a.n, 8), 256), 256, 0, s, a);
	else launch_timed(k_optimizer, div_up(a.n, 256), 256, 0, s, a);
	m->timers.end(NGP_TIMER_OPTIMIZER, s, a.n);
	NGP_HIP_CHECK(hipGetLastError());
	++m->ema_step;
	pack_mlp_fragments(m, m->params16.ptr, m->frag_train.ptr, s);
	pack_mlp_fragments(m, m->infer16.ptr, m->frag_infer.ptr, s);
}

// ---------------------------------------------------------------------------
// Host orchestration of one training step (Testbed::train_nerf_step).
// ---------------------------------------------------------------------------
// construct_cdf_2d (src/testbed_nerf.cu:1493-1521): one thread per (image, row)
__global__ void __launch_bounds__(256) k_cdf_2d(uint32_t n_images, uint32_t height, uint32_t width,
                                                const float* __restrict__ data, float* __restrict__ cdf_x_cond_y,
                                                float* __restrict__ cdf_y) {
	const uint32_t t = blockIdx.x * 256u + threadIdx.x;
	if (t >= n_images * height) return;
	const uint32_t img = t / height, y = t % height;
	const size_t off = ((size_t)img * height + y) * width;
	float cum = 0.0f;
	for (uint32_t x = 0; x < width; ++x) {
		cum += data[off + x] + 1e-10f;
		cdf_x_cond_y[off + x] = cum;
	}
	cdf_y[(size_t)img * height + y] = cum;
	const float norm = 1.0f / cum;
	for (uint32_t x = 0; x < width; ++x)
		cdf_x_cond_y[off + x] = (1.0f - MIN_PDF) * cdf_x_cond_y[off + x] * norm + MIN_PDF * (float)(x + 1) / (float)width;
}

// construct_cdf_1d (src/testbed_nerf.cu:1523-1546): one thread per image
__global__ void __launch_bounds__(256) k_cdf_1d(uint32_t n_images, uint32_t height, float* __restrict__ cdf_y,
                                                float* __restrict__ cdf_img) {
	const uint32_t img = blockIdx.x * 256u + threadIdx.x;
	if (img >= n_images) return;
	float* cy = cdf_y + (size_t)img * height;
	float cum = 0.0f;
	for (uint32_t y = 0; y < height; ++y) {
		cum += cy[y];
		cy[y] = cum;
	}
	cdf_img[img] = cum;
	const float norm = 1.0f / cum;
	for (uint32_t y = 0; y < height; ++y) cy[y] = (1.0f - MIN_PDF) * cy[y] * norm + MIN_PDF * (float)(y + 1) / (float)height;
}

void run_error_map_cdf(const float* error_map, uint32_t n_images, uint32_t rx, uint32_t ry, float* cdf_x_cond_y,
                       float* cdf_y, float* cdf_img, hipStream_t s) {
	if (n_images == 0 || rx == 0 || ry == 0) return;
	k_cdf_2d<<<div_up((uint64_t)n_images * ry, 256), 256, 0, s>>>(n_images, ry, rx, error_map, cdf_x_cond_y, cdf_y);
	k_cdf_1d<<<div_up(n_images, 256), 256, 0, s>>>(n_images, ry, cdf_y, cdf_img);
	NGP_HIP_CHECK(hipGetLastError());
}

void run_train_step(ngp_model* m, const ngp_train_args* t, hipStream_t s) {
	TrainScratch& ts = m->ts;
	const uint32_t R = t->n_rays, B = t->target_batch_size, MS_global = t->max_samples;
	const uint32_t L = m->lt.n_levels, F = m->lt.F;
	// data parallelism: caps and rollover over the global ray order (ngp_train_args.world_size)
	const uint32_t world = t->world_size > 1 && t->allreduce_i32 ? t->world_size : 1u;
	if (world > 1 && t->rank >= world) throw std::invalid_argument("rank must be < world_size");
	// the sample buffers of this rank: the global cap in one process; with data parallelism about the rank's
	// share (twice the even split, or the need of a step that did not fit -- k_dp_caps flags it), so per-rank
	// memory does not grow with the world size
	// (ngp_tuning.debug bit 3: an eighth of the even split, forcing the overflow and the retry)
	const uint32_t even = (m->tuning.debug & 8u) ? MS_global / world / 8u : 2u * (MS_global / world);
	const uint32_t MS = world > 1 ? std::min(MS_global, std::max(next_multiple(even, 4096u), ts.rank_cap_hint)) : MS_global;
	{
		// 32-bit byte offsets: the MLP's raw encoding buffers and the encoder's planes
		const uint64_t rows = (uint64_t)MS + 48ull * R;  // the chunked forward's evaluation rows (at most)
		if ((uint64_t)m->enc_pad * 2 * rows >= (1ull << 32) || 32ull * rows >= (1ull << 32))
			throw std::invalid_argument("training: max_samples too large for one rank's 32-bit sample buffers "
			                            "(lower the batch per rank)");
	}
	ts.ray_numsteps.grow(2 * (size_t)R);
	ts.ray_compacted.grow(2 * (size_t)R);
	ts.ray_state.grow(8 * (size_t)R);
	ts.ray_loss_state.grow(8 * (size_t)R);
	ts.loss.grow(R);
	ts.coords.grow(8 * (size_t)MS);
	ts.enc.grow((size_t)L * MS * F);
	ts.mlp_out.grow(4 * (size_t)MS);
	ts.ccoords.reserve(8 * (size_t)B);
	// n_extra_dims > 0: each sample's image picks its latent-code row (NerfCoordinate extra dims, src/testbed_nerf.cu:824)
	const bool xd = m->cfg.n_extra_dims > 0;
	if (xd) {
		ts.simg.grow(MS);
		ts.cimg.reserve(B);
		if (t->extra_dims_gradient) ts.dextra.reserve(NGP_EXTRA_ROW * (size_t)B);
	}
	ts.cpos4.reserve(4 * (size_t)B);
	ts.cenc.reserve((size_t)L * B * F);
	ts.dloss.reserve(4 * (size_t)B);
	ts.cweight.reserve(B);
	ts.csrc.reserve(B);
	ts.denc.reserve((size_t)L * B * F);
	ts.block_sums.grow(div_up(std::max(R, 1u), 1024) + 16);
	ts.counters.reserve(16);
	ts.scan_a.grow(2 * (size_t)R);
	ts.scan_b.grow(2 * (size_t)R);
	DevBuf<uint32_t>& counts = ts.scan_a;
	ts.last_n_rays = R;
	ts.last_target = B;
	ts.last_max_samples = MS;
	ts.gated_optimizer_ran = false;

	uint32_t* dp_samples = nullptr;  // DpCaps of the sampler / the compaction (device)
	uint32_t* dp_compact = nullptr;
	auto dp_exchange = [&](const uint32_t* total, uint32_t* caps, int32_t* slots, uint32_t cap, const uint32_t* extra,
	                       uint32_t local_cap) {
		k_dp_publish<<<1, 64, 0, s>>>(total, slots, world, t->rank, extra);
		NGP_HIP_CHECK(hipGetLastError());
		if (t->allreduce_i32(t->allreduce_user, slots, world + (extra ? 1u : 0u), s) != NGP_OK)
			throw std::runtime_error("data-parallel training: the all-reduce of the per-rank totals failed");
		const bool sized = local_cap < cap;
		k_dp_caps<<<1, 64, 0, s>>>(slots, world, t->rank, cap, caps, local_cap, sized ? ts.counters.ptr + 9 : nullptr,
		                           sized ? ts.counters.ptr + 10 : nullptr);
		NGP_HIP_CHECK(hipGetLastError());
	};
	if (world > 1) {
		ts.dp.reserve(8 + 2 * (size_t)world + 2);
		dp_samples = ts.dp.ptr;
		dp_compact = ts.dp.ptr + 4;
	}
	// deterministic hash-grid gradients: the fixed-point buffer, zeroed once (the optimizer clears
	// what it consumed, as for the fp16 buffer)
	ts.fixed = t->deterministic != 0;
	if (ts.fixed && ts.img_fix.n < (size_t)IMG_FIX_STRIDE * t->n_images) {
		ts.img_fix.release();
		ts.img_fix.reserve((size_t)IMG_FIX_STRIDE * t->n_images);
		NGP_HIP_CHECK(hipMemsetAsync(ts.img_fix.ptr, 0, ts.img_fix.bytes(), s));
	}
	if (ts.fixed && !m->grid_grads64.ptr) {
		m->grid_grads64.reserve(m->n_grid_params);
		NGP_HIP_CHECK(hipMemsetAsync(m->grid_grads64.ptr, 0, m->n_grid_params * sizeof(long long), s));
	}

	// the step's counters are zeroed by k_sample_count, its first kernel (sa.clear16)

	SamplerArgs sa{};
	sa.images = t->images;
	sa.n_images = t->n_images;
	sa.n_rays = R;
	sa.n_rays_global = t->n_rays_global ? t->n_rays_global : R;
	sa.ray_offset = t->ray_index_offset;
	sa.max_samples = MS;
	sa.max_samples_dev = dp_samples ? dp_samples + 2 : nullptr;
	sa.rng.state = t->rng_state;
	sa.rng.inc = t->rng_inc;
	sa.aabb.min = mk3(t->aabb_min[0], t->aabb_min[1], t->aabb_min[2]);
	sa.aabb.max = mk3(t->aabb_max[0], t->aabb_max[1], t->aabb_max[2]);
	sa.st = make_stepping(t->cone_angle_constant);
	sa.max_mip = t->max_cascade;
	sa.snap = t->snap_to_pixel_centers;
	sa.max_level_rand = t->max_level_rand_training != 0;
	// aabb_scale 1: cross empty space through the octant distance fields (shared with the renderer,
	// rebuilt when the bitfield changed); the chain walk otherwise
	if (t->max_cascade == 0) {
		build_distance_fields(m, 0, s);
		sa.df = m->rs.df.ptr;
	}
	sa.cdf = ErrorCdf{t->cdf_x_cond_y, t->cdf_y, t->cdf_img, t->cdf_res[0], t->cdf_res[1]};
	sa.bitfield = m->gs.bitfield.ptr;
	sa.numsteps = ts.ray_numsteps.ptr;
	sa.counts = counts.ptr;
	sa.bases = counts.ptr + R;
	sa.ray_state = ts.ray_state.ptr;
	sa.coords = ts.coords.ptr;
	sa.simg = xd ? ts.simg.ptr : nullptr;
	sa.clear16 = ts.counters.ptr;
	if (t->distortion_map && t->distortion_res[0] && t->distortion_res[1]) {
		sa.dmap = t->distortion_map;
		sa.drx = t->distortion_res[0];
		sa.dry = t->distortion_res[1];
	}
	KernelTimers& tm = m->timers;
	tm.begin(NGP_TIMER_TRAIN_SAMPLER, s);
	const bool general = t->cdf_img || t->cdf_x_cond_y || t->has_lens || sa.dmap;
	// lanes per ray of the two sampler passes (a wave per ray for the ~2k rays of a volume scene's batch)
	uint32_t sl = m->tuning.train_sampler_lanes;
	if (sl == 0) sl = 64u;
#define NGP_SAMPLER(KERNEL)                                                                                        \
	switch (sl) {                                                                                                  \
		case 8: if (general) KERNEL<true, 8><<<div_up(R, 32), 256, 0, s>>>(sa); else KERNEL<false, 8><<<div_up(R, 32), 256, 0, s>>>(sa); break; \
		case 16: if (general) KERNEL<true, 16><<<div_up(R, 16), 256, 0, s>>>(sa); else KERNEL<false, 16><<<div_up(R, 16), 256, 0, s>>>(sa); break; \
		case 32: if (general) KERNEL<true, 32><<<div_up(R, 8), 256, 0, s>>>(sa); else KERNEL<false, 32><<<div_up(R, 8), 256, 0, s>>>(sa); break; \
		default: if (general) KERNEL<true, 64><<<div_up(R, 4), 256, 0, s>>>(sa); else KERNEL<false, 64><<<div_up(R, 4), 256, 0, s>>>(sa); break; \
	}
	NGP_SAMPLER(k_sample_count)
	launch_exclusive_scan(sa.counts, sa.bases, R, ts.block_sums.ptr, ts.counters.ptr + 0, s);
	// the global sample cap (src/testbed_nerf.cu:779-781 drops rays past max_samples) over all ranks
	if (world > 1) dp_exchange(ts.counters.ptr + 0, dp_samples, reinterpret_cast<int32_t*>(ts.dp.ptr + 8), MS_global, nullptr, MS);
	sa.total = ts.counters.ptr + 0;
	sa.total_capped = ts.counters.ptr + 4;
	NGP_SAMPLER(k_sample_write)
#undef NGP_SAMPLER
	NGP_HIP_CHECK(hipGetLastError());
	tm.end(NGP_TIMER_TRAIN_SAMPLER, s, R);

	// network inference with the training params (NerfNetwork::inference_mixed_precision): over
	// every emitted sample as the reference does (full_forward), or chunk by chunk up to each
	// ray's stop (k_train_chunk) -- the loss kernels read the same outputs either way
	const bool chunk_off = t->full_forward != 0;
	const bool ml_on = sa.max_level_rand != 0;  // hash-grid levels cut per sample (set_max_level_gpu)
	const LevelTable lt_c = ml_on ? m->lt.with_max_level(ts.ccoords.ptr + 7, 8) : m->lt;  // compacted rows
	const __half* table = m->params16.ptr + m->n_mlp_params;
	const __half* enc_rows = ts.enc.ptr;
	EncLayout enc_layout = internal_layout(m, MS);
	const uint32_t* eidx = nullptr;
	ts.chunked = !chunk_off;
	if (chunk_off) {
		tm.begin_kernel(NGP_TIMER_TRAIN_ENCODE);
		launch_hashgrid_fwd(ml_on ? m->lt.with_max_level(ts.coords.ptr + 7, 8) : m->lt, ts.coords.ptr, 8, MS, table, ts.enc.ptr,
		                    enc_layout, s, ts.counters.ptr + 4, 0);
		tm.end(NGP_TIMER_TRAIN_ENCODE, s);
		tm.begin_kernel(NGP_TIMER_TRAIN_MLP_INFER);
		launch_mlp_infer(m, m->frag_train.ptr, ts.enc.ptr, enc_layout, ts.coords.ptr, 8, MS, ts.mlp_out.ptr, s,
		                 ts.counters.ptr + 4, 4, nullptr, 0, 4, nullptr, 0, false, MlpExtra{t->extra_dims, sa.simg, nullptr});
		tm.end(NGP_TIMER_TRAIN_MLP_INFER, s);
	} else {
		// evaluation rows: chunk p of every ray lands in [off[p], off[p] + cap[p])
		const uint32_t cap[TRAIN_CHUNKS] = {std::min(16 * R, MS), std::min(32 * R, MS), MS};
		const uint32_t off[TRAIN_CHUNKS] = {0, cap[0], cap[0] + cap[1]};
		const uint32_t MSE = off[2] + cap[2];
		ts.epos.grow(4 * (size_t)MSE);
		ts.edir.grow(4 * (size_t)MSE);
		ts.eenc.grow((size_t)L * MSE * F);
		ts.eout.grow(4 * (size_t)MSE);
		ts.eidx.grow(MS);
		if (xd) ts.eimg.grow(MSE);
		ts.ray_T.grow(R);
		ts.ray_eval.grow(R);
		ts.ray_ebase.grow(R);
		ChunkArgs c{};
		c.n_rays = R;
		c.numsteps = ts.ray_numsteps.ptr;
		c.coords = ts.coords.ptr;
		c.epos = reinterpret_cast<float4*>(ts.epos.ptr);
		c.edir = reinterpret_cast<float4*>(ts.edir.ptr);
		c.eout = ts.eout.ptr;
		c.mlp_out = ts.mlp_out.ptr;
		c.eidx = ts.eidx.ptr;
		c.ray_T = ts.ray_T.ptr;
		c.ray_eval = ts.ray_eval.ptr;
		c.ray_ebase = ts.ray_ebase.ptr;
		c.density_act = m->cfg.density_activation;
		c.stop_T = (m->tuning.debug & 4u) ? 0.999f : TRAIN_CHUNK_STOP_T;
		c.simg = sa.simg;
		c.eimg = xd ? ts.eimg.ptr : nullptr;
		for (uint32_t p = 0; p <= TRAIN_CHUNKS; ++p) {
			c.first = p == 0;
			c.last = p == TRAIN_CHUNKS;
			c.prev_lo = p >= 2 ? TRAIN_CHUNK_END[p - 2] : 0u;
			c.lo = p == 0 ? 0u : TRAIN_CHUNK_END[p - 1];
			c.hi = p < TRAIN_CHUNKS ? TRAIN_CHUNK_END[p] : c.lo;
			c.rows = ts.counters.ptr + 12 + std::min(p, TRAIN_CHUNKS - 1);
			c.eval_offset = p < TRAIN_CHUNKS ? off[p] : 0u;
			// lanes per ray: 64 for the ~2k long rays of a volume scene's batch, 16 for the 20-60k rays of a surface
			// scene (its rays that pass 16 samples composite and scatter 32 per chunk: 2 rounds instead of 8 at 4
			// lanes; surface step 1037 vs 1073 us, profiles/r05_train_chunk_lanes_ab.txt)
			uint32_t G = m->tuning.train_chunk_lanes;
			if (G == 0) G = R <= 4096 ? 64u : 16u;
			switch (G) {
			case 64: k_train_chunk<64><<<div_up(R, 16), 1024, 0, s>>>(c); break;
			case 32: k_train_chunk<32><<<div_up(R, 32), 1024, 0, s>>>(c); break;
			case 16: k_train_chunk<16><<<div_up(R, 64), 1024, 0, s>>>(c); break;
			case 8: k_train_chunk<8><<<div_up(R, 128), 1024, 0, s>>>(c); break;
			default: k_train_chunk<4><<<div_up(R, 256), 1024, 0, s>>>(c); break;
			}
			NGP_HIP_CHECK(hipGetLastError());
			if (p == TRAIN_CHUNKS) break;
			// launch about as many encoder chunks as the last step's rows needed; blocks loop
			// over the rest if there are more
			const uint32_t lr = ts.last_rows[p];
			const uint32_t max_chunks = lr ? div_up((uint64_t)lr + lr / 4, 256) + 16 : 0u;
			tm.begin_kernel(NGP_TIMER_TRAIN_ENCODE);
			// chunk p's rows start at sample off[p] of every plane
			__half* eenc_p = ts.eenc.ptr + ((size_t)off[p] * F << m->enc_lsh);
			// max_level_rand_training: the max level rides in the direction row's pad float
			const LevelTable lt_p = ml_on ? m->lt.with_max_level(ts.edir.ptr + 4 * (size_t)off[p] + 3, 4) : m->lt;
			launch_hashgrid_fwd(lt_p, ts.epos.ptr + 4 * (size_t)off[p], 4, cap[p], table, eenc_p, internal_layout(m, MSE), s,
			                    c.rows, 0, max_chunks);
			tm.end(NGP_TIMER_TRAIN_ENCODE, s);
			tm.begin_kernel(NGP_TIMER_TRAIN_MLP_INFER);
			launch_mlp_infer(m, m->frag_train.ptr, eenc_p, internal_layout(m, MSE), ts.edir.ptr + 4 * (size_t)off[p], 4,
			                 cap[p], ts.eout.ptr + 4 * (size_t)off[p], s, c.rows, 0, nullptr, 0, 4, nullptr, 0, false,
			                 MlpExtra{t->extra_dims, xd ? ts.eimg.ptr + off[p] : nullptr, nullptr});
			tm.end(NGP_TIMER_TRAIN_MLP_INFER, s);
		}
		enc_rows = ts.eenc.ptr;
		enc_layout = internal_layout(m, MSE);
		eidx = ts.eidx.ptr;
	}

	LossArgs la{};
	la.images = t->images;
	la.n_images = t->n_images;
	la.n_rays = R;
	la.n_rays_global = sa.n_rays_global;
	la.ray_offset = t->ray_index_offset;
	la.rng = sa.rng;
	la.aabb = sa.aabb;
	la.snap = t->snap_to_pixel_centers;
	la.max_level_rand = sa.max_level_rand;
	la.cdf = sa.cdf;
	la.error_map = t->error_map;
	la.exposure = t->exposure;
	la.exposure_grad = t->exposure_gradient;
	la.exposure_fix = ts.fixed && t->exposure_gradient ? ts.img_fix.ptr : nullptr;
	ts.ray_aux.grow(4 * (size_t)R);
	la.ray_aux = reinterpret_cast<float4*>(ts.ray_aux.ptr);
	la.error_map_rx = t->error_map_res[0];
	la.error_map_ry = t->error_map_res[1];
	la.loss_type = t->loss_type;
	la.random_bg = t->random_bg_color;
	la.bg = mk3(t->background_color[0], t->background_color[1], t->background_color[2]);
	la.linear_colors = t->train_in_linear_colors;
	la.color_space = t->color_space;
	la.rgb_act = m->cfg.rgb_activation;
	la.density_act = m->cfg.density_activation;
	la.near_distance = t->near_distance;
	la.max_compacted = B;
	la.target_batch = B;
	la.numsteps = ts.ray_numsteps.ptr;
	la.ray_state = ts.ray_state.ptr;
	la.coords = ts.coords.ptr;
	la.mlp_out = ts.mlp_out.ptr;
	la.n_levels = L;
	la.F = F;
	la.ccounts = ts.scan_b.ptr;
	la.cbases = ts.scan_b.ptr + R;
	la.loss_state = ts.ray_loss_state.ptr;
	la.compacted = ts.ray_compacted.ptr;
	la.loss_out = ts.loss.ptr;
	la.csrc = ts.csrc.ptr;
	la.dloss = ts.dloss.ptr;
	la.mean_density = m->gs.mean.ptr;
	la.ray_eval = ts.chunked ? ts.ray_eval.ptr : nullptr;
	la.violations = ts.counters.ptr + 9;
	// camera gradients: extrinsics and / or the distortion map's (compute_cam_gradient_train_nerf)
	const bool dist_grad = sa.dmap && t->distortion_gradient && t->distortion_gradient_weight;
	const bool cam = (t->cam_pos_gradient && t->cam_rot_gradient) || dist_grad;
	la.store_uv_pdf = cam ? 1 : 0;
	la.dmap = sa.dmap;
	la.drx = sa.drx;
	la.dry = sa.dry;
	la.depth_lambda = t->depth_supervision_lambda > 0.0f ? t->depth_supervision_lambda : 0.0f;
	la.max_mip = t->max_cascade;
	if (t->sharpness_data && t->sharpness_grid && t->error_map) {
		// train_nerf (src/testbed_nerf.cu:2453-2464): clear at step 0, else decay by 0.95
		const size_t n_cells = (size_t)NERF_GRID_N_CELLS * NERF_CASCADES;
		if (t->sharpness_grid_clear) NGP_HIP_CHECK(hipMemsetAsync(t->sharpness_grid, 0, n_cells * sizeof(float), s));
		la.sharp_data = t->sharpness_data;
		la.sharp_rx = t->sharpness_res[0];
		la.sharp_ry = t->sharpness_res[1];
		la.sharp_grid = t->sharpness_grid;
		ts.ray_hit.grow(4 * (size_t)R);
		la.ray_hit = reinterpret_cast<float4*>(ts.ray_hit.ptr);
	}
	la.depth_loss_type = t->depth_loss_type;
	if (la.depth_lambda > 0.0f) {
		ts.ray_depth.grow(2 * (size_t)R);
		la.ray_depth = reinterpret_cast<float2*>(ts.ray_depth.ptr);
	}
	tm.begin(NGP_TIMER_TRAIN_LOSS, s);
	const uint32_t LG = loss_lanes_per_ray(t->target_batch_size, la.n_rays_global);
#define NGP_LOSS(GG)                                                                       \
	do {                                                                                   \
		if (general) k_loss_composite<true, GG><<<div_up(R, 256u / GG), 256, 0, s>>>(la);  \
		else k_loss_composite<false, GG><<<div_up(R, 256u / GG), 256, 0, s>>>(la);         \
	} while (0)
	switch (LG) {
		case 8: NGP_LOSS(8); break;
		case 16: NGP_LOSS(16); break;
		case 32: NGP_LOSS(32); break;
		default: NGP_LOSS(64); break;
	}
#undef NGP_LOSS
	launch_exclusive_scan(la.ccounts, la.cbases, R, ts.block_sums.ptr, ts.counters.ptr + 1, s);
	// the global compaction cap (src/testbed_nerf.cu:997-1003) over all ranks, and the chunked forward's
	// violations summed over the ranks: every rank skips the step's deposits when any rank saw one
	la.viol_gate = la.violations;
	if (world > 1) {
		int32_t* slots = reinterpret_cast<int32_t*>(ts.dp.ptr + 8 + world);
		dp_exchange(ts.counters.ptr + 1, dp_compact, slots, B, la.violations, B);
		la.max_compacted_dev = dp_compact + 2;
		la.viol_gate = reinterpret_cast<const uint32_t*>(slots + world);
	}
	if (la.sharp_grid && !t->sharpness_grid_clear)  // train_nerf's decay by 0.95 (src/testbed_nerf.cu:2453-2464)
		k_scale_floats<<<div_up((size_t)NERF_GRID_N_CELLS * NERF_CASCADES, 256), 256, 0, s>>>(
		    la.sharp_grid, (size_t)NERF_GRID_N_CELLS * NERF_CASCADES, 0.95f, la.viol_gate);
	switch (LG) {
		case 8: k_loss_emit<8><<<div_up(R, 32u), 256, 0, s>>>(la); break;
		case 16: k_loss_emit<16><<<div_up(R, 16u), 256, 0, s>>>(la); break;
		case 32: k_loss_emit<32><<<div_up(R, 8u), 256, 0, s>>>(la); break;
		default: k_loss_emit<64><<<div_up(R, 4u), 256, 0, s>>>(la); break;
	}
	NGP_HIP_CHECK(hipGetLastError());
	const bool train_debug = (m->tuning.debug & 2u) != 0;
	if (train_debug) {
		// samples per ray emitted vs composited before termination, and what a chunked
		// (early-terminated) forward would evaluate under a few chunk schedules
		std::vector<uint32_t> ns(2 * (size_t)R), cc(R);
		NGP_HIP_CHECK(hipMemcpyAsync(ns.data(), ts.ray_numsteps.ptr, ns.size() * 4, hipMemcpyDeviceToHost, s));
		NGP_HIP_CHECK(hipMemcpyAsync(cc.data(), la.ccounts, cc.size() * 4, hipMemcpyDeviceToHost, s));
		NGP_HIP_CHECK(hipStreamSynchronize(s));
		const uint32_t sched[4][4] = {{8, 16, 32, 1024}, {16, 32, 1024, 0}, {16, 48, 1024, 0}, {32, 1024, 0, 0}};
		uint64_t sn = 0, sc = 0, ev[4] = {0, 0, 0, 0}, full = 0;
		for (uint32_t i = 0; i < R; ++i) {
			const uint32_t n = ns[2 * i], c = cc[i];
			sn += n;
			sc += std::min(c, n);
			full += (c >= n);
			for (int q = 0; q < 4; ++q) {
				uint32_t e = 0;
				for (int p = 0; p < 4 && sched[q][p]; ++p) {
					e = std::min(n, sched[q][p]);
					if (c < e || e == n) break;  // terminated inside the evaluated range
				}
				ev[q] += e;
			}
		}
		fprintf(stderr, "[train] rays %u samples %llu composited %llu (%.1f%%) rays-unterminated %llu | chunked eval "
		        "8/16/32/all %llu, 16/32/all %llu, 16/48/all %llu, 32/all %llu\n", R, (unsigned long long)sn,
		        (unsigned long long)sc, 100.0 * sc / std::max<uint64_t>(sn, 1), (unsigned long long)full,
		        (unsigned long long)ev[0], (unsigned long long)ev[1], (unsigned long long)ev[2], (unsigned long long)ev[3]);
	}

	// compacted batch size c = min(total, B), gather, rollover multiplicity, loss sum: one launch
	const CompactFinish cf{ts.counters.ptr + 1, la.max_compacted_dev, ts.counters.ptr + 5, dp_compact, ts.cweight.ptr,
	                       ts.loss.ptr, R, reinterpret_cast<float*>(ts.counters.ptr + 8)};
	const uint32_t gather_blocks = div_up(B, 256) + 1;
#define NGP_GATHER(FF) k_gather_compacted<FF><<<gather_blocks, 256, 0, s>>>(cf, ts.csrc.ptr, ts.coords.ptr, enc_rows, enc_layout, \
		internal_layout(m, B), L, ts.ccoords.ptr, reinterpret_cast<float4*>(ts.cpos4.ptr), ts.cenc.ptr, B, eidx, sa.simg, xd ? ts.cimg.ptr : nullptr)
	switch (F) {
		case 1: NGP_GATHER(1); break;
		case 2: NGP_GATHER(2); break;
		case 4: NGP_GATHER(4); break;
		default: NGP_GATHER(8); break;
	}
#undef NGP_GATHER
	NGP_HIP_CHECK(hipGetLastError());
	tm.end(NGP_TIMER_TRAIN_LOSS, s, R);

	// fused MLP forward+backward, then hash-grid scatter (Trainer::training_step)
	tm.begin_kernel(NGP_TIMER_TRAIN_MLP_BWD);
	if (cam) {
		ts.dsh.reserve(16 * (size_t)B);
		ts.dpos.reserve(3 * (size_t)B);
	}
	const bool xgrad = xd && t->extra_dims_gradient;
	launch_mlp_train(m, m->frag_train.ptr, ts.cenc.ptr, internal_layout(m, B), ts.ccoords.ptr, 8, B, ts.dloss.ptr, ts.cweight.ptr,
	                 m->grads.ptr, ts.denc.ptr, s, ts.counters.ptr + 5, cam ? ts.dsh.ptr : nullptr,
	                 MlpExtra{t->extra_dims, xd ? ts.cimg.ptr : nullptr, xgrad ? ts.dextra.ptr : nullptr});
	if (xgrad) {
		k_extra_gradient<<<div_up(R, 256u), 256, 0, s>>>(R, ts.ray_compacted.ptr, ts.ray_loss_state.ptr, ts.dextra.ptr,
		                                                 m->cfg.n_extra_dims, t->extra_dims_gradient, la.viol_gate,
		                                                 ts.fixed ? ts.img_fix.ptr : nullptr);
		NGP_HIP_CHECK(hipGetLastError());
	}
	tm.end(NGP_TIMER_TRAIN_MLP_BWD, s);
	tm.begin_kernel(NGP_TIMER_TRAIN_ENCODE_BWD);
	// data parallel: launched for about this rank's share of the global batch (blocks loop past it)
	const uint32_t bwd_chunks = world > 1 ? div_up(B / world + B / (4 * world), 128u) + 16 : 0u;
	launch_hashgrid_bwd(lt_c, ts.cpos4.ptr, 4, B, ts.denc.ptr, EncLayout{B, 0}, m->grid_grads16.ptr, s,
	                    ts.counters.ptr + 5, ts.fixed ? m->grid_grads64.ptr : nullptr, bwd_chunks);
	tm.end(NGP_TIMER_TRAIN_ENCODE_BWD, s);
	if (cam) {
		// input gradients of the compacted samples (Trainer::training_step with dL_dinput), then
		// compute_cam_gradient_train_nerf per ray
		launch_hashgrid_input_grad(lt_c, ts.cpos4.ptr, 4, B, ts.denc.ptr, EncLayout{B, 0}, m->params16.ptr + m->n_mlp_params,
		                           ts.cweight.ptr, ts.dpos.ptr, s, ts.counters.ptr + 5);
		CamGradArgs ca{};
		ca.n_rays = R;
		ca.aabb = sa.aabb;
		ca.compacted = ts.ray_compacted.ptr;
		ca.ray_state = ts.ray_state.ptr;
		ca.loss_state = ts.ray_loss_state.ptr;
		ca.ray_aux = reinterpret_cast<const float4*>(ts.ray_aux.ptr);
		ca.ccoords = ts.ccoords.ptr;
		ca.dpos = ts.dpos.ptr;
		ca.dsh = ts.dsh.ptr;
		ca.cam_pos_gradient = t->cam_pos_gradient;
		ca.cam_rot_gradient = t->cam_rot_gradient;
		if (!(t->cam_pos_gradient && t->cam_rot_gradient)) ca.cam_pos_gradient = ca.cam_rot_gradient = nullptr;
		ca.cam_fix = ts.fixed && ca.cam_pos_gradient ? ts.img_fix.ptr : nullptr;
		ca.images = t->images;
		ca.viol_gate = la.viol_gate;
		if (dist_grad) {
			ca.dgrad = t->distortion_gradient;
			ca.dgrad_w = t->distortion_gradient_weight;
			ca.drx = sa.drx;
			ca.dry = sa.dry;
		}
		k_cam_gradient<<<div_up(R, 256), 256, 0, s>>>(ca);
		NGP_HIP_CHECK(hipGetLastError());
	}
	if (ts.fixed) {
		// the step's fixed-point per-image sums into the float gradients, in image order
		const uint32_t NI = t->n_images;
		auto flush = [&](uint32_t first, uint32_t width, float* dst) {
			if (!dst || !width) return;
			k_img_fix_flush<<<div_up(NI * width, 256u), 256, 0, s>>>(NI, IMG_FIX_STRIDE, first, width, ts.img_fix.ptr, dst);
			NGP_HIP_CHECK(hipGetLastError());
		};
		flush(0, 3, t->exposure_gradient);
		if (cam && t->cam_pos_gradient && t->cam_rot_gradient) {
			flush(3, 3, t->cam_pos_gradient);
			flush(6, 3, t->cam_rot_gradient);
		}
		if (xgrad) flush(9, NGP_EXTRA_ROW, t->extra_dims_gradient);  // rows of NGP_EXTRA_ROW, the first E written
	}
	tm.train_units_pending = tm.mask != 0;

	if (!t->defer_optimizer) launch_optimizer(m, t->training_step, t->optimize_mlp, t->optimize_encoding, s);
	m->stats_pending = true;
}

}  // namespace ngp
