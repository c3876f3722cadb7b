// hashgrid.hip — multiresolution hash-grid encoding, forward and backward, gfx950.
//
// Restates tiny-cuda-nn's GridEncodingTemplated (HashGrid, Linear interpolation,
// CoherentPrime hash) as used by NerfNetwork (include/neural-graphics-primitives/
// nerf_network.h:82, configs/nerf/base.json:23-29).  The per-level geometry is
// resolved once on the host (LevelTable) so host, oracle and device agree bit for
// bit on scale/resolution/offset.
//
// MI355X mapping
//  * one thread = one (sample, level); each thread issues its 8 corner gathers
//    back to back (8 independent loads in flight per lane).
//  * XCD-aware block order: when n_levels % 8 == 0 every workgroup of level l is
//    placed on the XCD group b % 8 == l % 8, and the levels an XCD owns run one
//    after the other, so each XCD's private 4 MiB L2 holds one level's table (2 MiB
//    at T=2^19) instead of the whole 24 MiB table.  Placement only changes speed.
//  * output is an EncLayout (ngp_internal.h): level-major [L][n][F] at the C-ABI, planes
//    of four levels [L/4][n][4][F] inside the pipelines -- a wave of 64 consecutive samples
//    writes 64 contiguous 16-B planes (F = 2).
//  * features accumulate in fp32 (tcnn accumulates in fp16) and are rounded once.
#include <cstring>
#include <type_traits>

#include "encode_device.h"
#include "ngp_internal.h"

namespace ngp {

__device__ __forceinline__ void map_block(uint32_t b, uint32_t n_chunks, uint32_t n_levels, uint32_t* level,
                                          uint32_t* chunk) {
	if ((n_levels & 7u) == 0) {
		// workgroups are dispatched round-robin over the 8 XCDs: XCD x runs level x for the
		// first n_chunks of its workgroups, then level x + 8, ... -- one level's table
		// (<= 2 MiB at T=2^19) at a time in each XCD's 4 MiB L2
		const uint32_t x = b & 7u, k = b >> 3;
		*level = x + 8u * (k / n_chunks);
		*chunk = k % n_chunks;
	} else {
		*level = b / n_chunks;
		*chunk = b % n_chunks;
	}
}


// four levels' feature vectors of one sample: one plane of an EncLayout with lsh = 2
template <uint32_t F>
struct alignas(4 * sizeof(typename FeatVec<F>::T)) Plane4 {
	typename FeatVec<F>::T v[4];
};

// SITE names the call site in profiles (0 training, 1 render, 2 density grid / API).  A
// thread encodes LPT levels of one sample (l, l + L/LPT, ...), so the position row is loaded
// once per LPT levels: the encoder is bound by the texture addresser's per-lane work, which
// this cuts by a seventh at LPT = 4 -- more than the XCD-private L2 locality of one level per
// block is worth.  Strided levels keep a mix of coarse and fine tables in flight (four
// consecutive fine levels at once measured ~15 % slower: L2 working set).  With LPT = 4 and
// the plane layout (EncLayout lsh = 2) the four results are one plane: one 16-B store
// (F = 2) instead of four 4-B stores.  Render slots that a ray reserved but did not fill
// carry x = -1 (k_generate): they get zero features, no gathers.
template <uint32_t F, int SITE, bool QUAD, uint32_t LPT>
__global__ void __launch_bounds__(256) k_hashgrid_fwd(uint32_t n, const float* __restrict__ pos, uint32_t stride,
                                                      const __half* __restrict__ table, const LevelTable lt,
                                                      __half* __restrict__ enc, EncLayout lay, uint32_t n_chunks,
                                                      const uint32_t* __restrict__ n_dev) {
	if (SITE == 1) set_wave_priority(lt.prio);
	uint32_t grp, chunk0 = 0;
	const uint32_t groups = lt.n_levels / LPT;
	if (n_dev) n = min(n, *n_dev);
	// n_chunks per level group are launched; they stride over the chunks the count covers
	uint32_t c_begin, c_end = (n + 255u) >> 8, c_step = n_chunks;
	if (LPT == 4 && lt.regions) {
		// XCD regions (n_chunks a multiple of 8): workgroup b runs on XCD b % 8, so XCD x takes the
		// contiguous chunk range [x R, x R + R) of the device count -- its L2 sees the cells of one
		// eighth of the rays instead of every eighth chunk of all of them
		const uint32_t b = blockIdx.x, K = n_chunks >> 3, R = (c_end + 7u) >> 3;
		grp = b / n_chunks;
		const uint32_t x = (b % n_chunks) & 7u, k = (b % n_chunks) >> 3;
		c_begin = x * R + k;
		c_end = min(c_end, x * R + R);
		c_step = K;
	} else {
		map_block(blockIdx.x, n_chunks, groups, &grp, &chunk0);
		c_begin = chunk0;
	}
	using VT = typename FeatVec<F>::T;
	// levels g, g + L/LPT, ... of the sample
	auto level_of = [&](uint32_t q) { return grp + q * groups; };
	for (uint32_t chunk = c_begin; chunk < c_end; chunk += c_step) {
		const uint32_t i = chunk * 256u + threadIdx.x;
		if (i >= n) continue;
		const float px = pos[(size_t)i * stride + 0], py = pos[(size_t)i * stride + 1], pz = pos[(size_t)i * stride + 2];
	VT o[LPT];
		if (SITE == 1 && px < 0.0f) {
#pragma unroll
			for (uint32_t q = 0; q < LPT; ++q) o[q] = VT{};
		} else if (SITE == 0 && lt.max_level) {
			// levels above the sample's max level are zero (tcnn kernel_grid with max_level_gpu)
#pragma unroll
			for (uint32_t q = 0; q < LPT; ++q)
				o[q] = lt.level_cut(level_of(q), i) ? VT{} : encode_one<F, QUAD>(level_of(q), px, py, pz, table, lt);
		} else {
#pragma unroll
			for (uint32_t q = 0; q < LPT; ++q) o[q] = encode_one<F, QUAD>(level_of(q), px, py, pz, table, lt);
		}
		if constexpr (LPT == 4) {
			if (lay.lsh == 2) {
				Plane4<F> pv;
#pragma unroll
				for (uint32_t q = 0; q < 4; ++q) pv.v[q] = o[q];
				if constexpr (F == 2) {
					if (lt.streaming) {
						// the encodings are written once and read once by the MLP: non-temporal stores
						typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
						const u32x4 w = {pv.v[0], pv.v[1], pv.v[2], pv.v[3]};
						__builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(enc) + (size_t)grp * lay.plane + i);
						continue;
					}
				}
				reinterpret_cast<Plane4<F>*>(enc)[(size_t)grp * lay.plane + i] = pv;
				continue;
			}
		}
#pragma unroll
		for (uint32_t q = 0; q < LPT; ++q) reinterpret_cast<VT*>(enc)[lay.vec(level_of(q), i)] = o[q];
	}
}

// Hash-grid gradients are fp16 and accumulated with packed half2 atomics
// (global_atomic_pk_add_f16, no return), as tcnn's GridEncoding backward does with
// atomicAdd(__half2): one memory-side atomic per entry instead of one per feature.
// F = 1 adds (v, 0) or (0, v) to the aligned pair holding the entry.
typedef _Float16 half2_vec __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void atomic_add_half2(__half* p, float a, float b) {
	const half2_vec v = {(_Float16)a, (_Float16)b};
	__builtin_amdgcn_global_atomic_fadd_v2f16((__attribute__((address_space(1))) half2_vec*)p, v);
}
template <uint32_t F>
__device__ __forceinline__ void scatter_add(__half* gtab, uint32_t idx, const float* v) {
	if constexpr (F == 1) {
		if (idx & 1u) atomic_add_half2(gtab + (idx - 1u), 0.0f, v[0]);
		else atomic_add_half2(gtab + idx, v[0], 0.0f);
	} else {
#pragma unroll
		for (uint32_t f = 0; f < F; f += 2) atomic_add_half2(gtab + (size_t)idx * F + f, v[f], v[f + 1]);
	}
}

// Backward scatter.  Two lanes per (sample, level): lane 2s+h adds the four corners
// x + h of sample s, so in every atomic instruction the x and x+1 corners of a sample sit
// in adjacent lanes -- adjacent table entries (hashed: index ^ (x ^ (x+1)); dense: +1),
// nearly always in the same 64-byte line, which the memory-side atomic unit takes as one
// request instead of two.  Lanes of a parity hold consecutive samples of the compacted
// batch, i.e. consecutive points along the same rays, so at coarse levels they often add
// into the same corner: runs of equal indices (lane, lane+2, ...) are summed with a
// segmented shuffle scan and only the last lane of each run issues the atomic.
// Deterministic mode (FIXED): each corner's contribution is rounded to 2^-40 fixed point first,
// the run sums and the memory-side atomics are 64-bit integer adds -- exact, so the result does not
// depend on the order the waves arrive in.
template <uint32_t F>
__device__ __forceinline__ void scatter_add_fixed(long long* gtab, uint32_t idx, const long long* v) {
#pragma unroll
	for (uint32_t f = 0; f < F; ++f)
		if (v[f]) atomicAdd(reinterpret_cast<unsigned long long*>(gtab + (size_t)idx * F + f), (unsigned long long)v[f]);
}
__device__ __forceinline__ long long to_fixed(float v) {
	const float x = fminf(fmaxf(v * GRAD_FIXED_SCALE, -9.2e18f), 9.2e18f);
	return (long long)rintf(x);
}

constexpr uint32_t BWD_SAMPLES_PER_BLOCK = 128;
template <uint32_t F, bool FIXED>
__device__ __forceinline__ void hashgrid_bwd_chunk(uint32_t n, uint32_t level, uint32_t chunk, const float* __restrict__ pos,
                                                   uint32_t stride, const __half* __restrict__ denc, const EncLayout& lay,
                                                   const LevelTable& lt, __half* __restrict__ grad, long long* __restrict__ grad64) {
	const uint32_t i = chunk * BWD_SAMPLES_PER_BLOCK + (threadIdx.x >> 1), h = threadIdx.x & 1u;
	const int lane = threadIdx.x & 63;

	using VT = typename FeatVec<F>::T;
	float g[F];
	bool active = i < n;
	if (active && !lt.level_cut(level, i)) {
		unpack<F>(reinterpret_cast<const VT*>(denc)[lay.vec(level, i)], g);
		bool any = false;
#pragma unroll
		for (uint32_t f = 0; f < F; ++f) any |= g[f] != 0.0f;
		active = any;
	} else {
		active = false;
#pragma unroll
		for (uint32_t f = 0; f < F; ++f) g[f] = 0.0f;
	}
	if (__ballot(active) == 0ull) return;  // wave-uniform

	const float scale = lt.scale[level];
	const uint32_t res = lt.res[level], size = lt.size[level], hashed = lt.hashed[level];
	__half* gtab = FIXED ? nullptr : grad + (size_t)lt.offset[level] * F;
	long long* gtab64 = FIXED ? grad64 + (size_t)lt.offset[level] * F : nullptr;

	float fx = 0.f, fy = 0.f, fz = 0.f;
	uint32_t gx = 0, gy = 0, gz = 0;
	if (active) {
		pos_fract(pos[(size_t)i * stride + 0], scale, &fx, &gx);
		pos_fract(pos[(size_t)i * stride + 1], scale, &fy, &gy);
		pos_fract(pos[(size_t)i * stride + 2], scale, &fz, &gz);
	}
	const float wx = h ? fx : 1.0f - fx;
	// lanes of this lane's parity at or below it
	const unsigned long long parity = (lane & 1) ? 0xAAAAAAAAAAAAAAAAull : 0x5555555555555555ull;
	const unsigned long long at_or_below = (lane == 63 ? ~0ull : ((2ull << lane) - 1ull)) & parity;

#pragma unroll
	for (uint32_t c = 0; c < 4; ++c) {
		float w = wx;
		w *= (c & 1u) ? fy : 1.0f - fy;
		w *= (c & 2u) ? fz : 1.0f - fz;
		const uint32_t idx = active ? grid_index(hashed, size, res, gx + h, gy + (c & 1u), gz + ((c >> 1) & 1u))
		                            : 0xFFFFFFFFu - (uint32_t)lane;  // inactive lanes never merge
		using AccT = typename std::conditional<FIXED, long long, float>::type;
		AccT v[F];
#pragma unroll
		for (uint32_t f = 0; f < F; ++f) {
			if constexpr (FIXED) v[f] = to_fixed(w * g[f]);
			else v[f] = w * g[f];
		}
		const uint32_t prev = __shfl_up(idx, 2, 64);
		const bool head = lane < 2 || prev != idx;
		const unsigned long long heads = __ballot(head);
		if (~heads == 0ull) {
			if (active) {
				if constexpr (FIXED) scatter_add_fixed<F>(gtab64, idx, v);
				else scatter_add<F>(gtab, idx, v);
			}
			continue;
		}
		// run start of this lane = highest head of its parity at or below it
		const int start = 63 - __clzll(heads & at_or_below);
#pragma unroll
		for (int off = 2; off < 64; off <<= 1) {
#pragma unroll
			for (uint32_t f = 0; f < F; ++f) {
				const AccT t = __shfl_up(v[f], off, 64);
				if (lane - off >= start) v[f] += t;
			}
		}
		const bool tail = lane >= 62 || ((heads >> (lane + 2)) & 1ull);
		if (active && tail) {
			if constexpr (FIXED) scatter_add_fixed<F>(gtab64, idx, v);
			else scatter_add<F>(gtab, idx, v);
		}
	}
}

// Blocks loop over chunks (n_chunks launched per level, the device count may need more); levels [0, n_lv)
template <uint32_t F, bool FIXED>
__global__ void __launch_bounds__(256) k_hashgrid_bwd(uint32_t n, const float* __restrict__ pos, uint32_t stride,
                                                      const __half* __restrict__ denc, EncLayout lay,
                                                      const LevelTable lt, __half* __restrict__ grad,
                                                      long long* __restrict__ grad64, uint32_t n_chunks,
                                                      const uint32_t* __restrict__ n_dev, uint32_t n_lv) {
	uint32_t level, chunk;
	map_block(blockIdx.x, n_chunks, n_lv, &level, &chunk);
	if (n_dev) n = min(n, *n_dev);
	for (; chunk * BWD_SAMPLES_PER_BLOCK < n; chunk += n_chunks)  // block-uniform
		hashgrid_bwd_chunk<F, FIXED>(n, level, chunk, pos, stride, denc, lay, lt, grad, grad64);
}


// dL/d(position) through the grid (tcnn GridEncoding backward with input gradients, used by the
// camera gradients): dL/dx_d = sum_l scale_l sum_c dw_c/df_d sum_f dL/denc[l][f] table[c][f].
// One thread per sample, the training-parameter table; divided by the sample's rollover weight
// (the dL/denc carry it) so it is the gradient of the sample's own row.
template <uint32_t F>
__global__ void __launch_bounds__(256) k_hashgrid_input_grad(uint32_t n, const float* __restrict__ pos, uint32_t stride,
                                                             const __half* __restrict__ denc, EncLayout lay,
                                                             const __half* __restrict__ table, const LevelTable lt,
                                                             const float* __restrict__ weight, float* __restrict__ dpos,
                                                             const uint32_t* __restrict__ n_dev) {
	const uint32_t i = blockIdx.x * 256u + threadIdx.x;
	if (n_dev) n = min(n, *n_dev);
	if (i >= n) return;
	using VT = typename FeatVec<F>::T;
	const float px = pos[(size_t)i * stride + 0], py = pos[(size_t)i * stride + 1], pz = pos[(size_t)i * stride + 2];
	float dx = 0.0f, dy = 0.0f, dz = 0.0f;
	for (uint32_t level = 0; level < lt.n_levels; ++level) {
		float g[F];
		unpack<F>(reinterpret_cast<const VT*>(denc)[lay.vec(level, i)], g);
		bool any = false;
#pragma unroll
		for (uint32_t f = 0; f < F; ++f) any |= g[f] != 0.0f;
		if (!any || lt.level_cut(level, i)) continue;
		const float scale = lt.scale[level];
		const uint32_t res = lt.res[level], size = lt.size[level];
		const VT* tab = reinterpret_cast<const VT*>(table + (size_t)lt.offset[level] * F);
		float fx, fy, fz;
		uint32_t gx, gy, gz;
		pos_fract(px, scale, &fx, &gx);
		pos_fract(py, scale, &fy, &gy);
		pos_fract(pz, scale, &fz, &gz);
		VT vals[8];
		if (lt.hashed[level]) gather_corners<F, true>(tab, size, res, gx, gy, gz, vals);
		else gather_corners<F, false>(tab, size, res, gx, gy, gz, vals);
		float lx = 0.0f, ly = 0.0f, lz = 0.0f;
#pragma unroll
		for (uint32_t c = 0; c < 8; ++c) {
			float v[F];
			unpack<F>(vals[c], v);
			float dot = 0.0f;
#pragma unroll
			for (uint32_t f = 0; f < F; ++f) dot = fmaf(g[f], v[f], dot);
			const float wx = (c & 1u) ? fx : 1.0f - fx, wy = (c & 2u) ? fy : 1.0f - fy, wz = (c & 4u) ? fz : 1.0f - fz;
			lx += dot * ((c & 1u) ? 1.0f : -1.0f) * wy * wz;
			ly += dot * ((c & 2u) ? 1.0f : -1.0f) * wx * wz;
			lz += dot * ((c & 4u) ? 1.0f : -1.0f) * wx * wy;
		}
		dx = fmaf(scale, lx, dx);
		dy = fmaf(scale, ly, dy);
		dz = fmaf(scale, lz, dz);
	}
	const float inv = weight ? 1.0f / weight[i] : 1.0f;
	dpos[3 * (size_t)i + 0] = dx * inv;
	dpos[3 * (size_t)i + 1] = dy * inv;
	dpos[3 * (size_t)i + 2] = dz * inv;
}

void launch_hashgrid_input_grad(const LevelTable& lt, const float* pos, uint32_t stride, uint32_t n, const __half* denc,
                                EncLayout enc_plane, const __half* table, const float* weight, float* dpos, hipStream_t s,
                                const uint32_t* n_dev) {
	if (n == 0) return;
	switch (lt.F) {
		case 1: k_hashgrid_input_grad<1><<<div_up(n, 256), 256, 0, s>>>(n, pos, stride, denc, enc_plane, table, lt, weight, dpos, n_dev); break;
		case 2: k_hashgrid_input_grad<2><<<div_up(n, 256), 256, 0, s>>>(n, pos, stride, denc, enc_plane, table, lt, weight, dpos, n_dev); break;
		case 4: k_hashgrid_input_grad<4><<<div_up(n, 256), 256, 0, s>>>(n, pos, stride, denc, enc_plane, table, lt, weight, dpos, n_dev); break;
		case 8: k_hashgrid_input_grad<8><<<div_up(n, 256), 256, 0, s>>>(n, pos, stride, denc, enc_plane, table, lt, weight, dpos, n_dev); break;
		default: throw std::runtime_error("n_features_per_level must be 1, 2, 4 or 8");
	}
	NGP_HIP_CHECK(hipGetLastError());
}

__global__ void __launch_bounds__(256) k_hashgrid_indices(uint32_t n, const float* __restrict__ pos, uint32_t stride,
                                                          const LevelTable lt, uint32_t* __restrict__ idx_out,
                                                          float* __restrict__ w_out) {
	const uint32_t t = blockIdx.x * 256u + threadIdx.x;
	if (t >= n * lt.n_levels) return;
	const uint32_t i = t / lt.n_levels, level = t % lt.n_levels;
	const float scale = lt.scale[level];
	float fx, fy, fz;
	uint32_t gx, gy, gz;
	pos_fract(pos[(size_t)i * stride + 0], scale, &fx, &gx);
	pos_fract(pos[(size_t)i * stride + 1], scale, &fy, &gy);
	pos_fract(pos[(size_t)i * stride + 2], scale, &fz, &gz);
	for (uint32_t c = 0; c < 8; ++c) {
		float w = 1.0f;
		w *= (c & 1u) ? fx : 1.0f - fx;
		w *= (c & 2u) ? fy : 1.0f - fy;
		w *= (c & 4u) ? fz : 1.0f - fz;
		const uint32_t idx = grid_index(lt.hashed[level], lt.size[level], lt.res[level], gx + (c & 1u),
		                                gy + ((c >> 1) & 1u), gz + ((c >> 2) & 1u));
		idx_out[((size_t)i * lt.n_levels + level) * 8 + c] = lt.offset[level] + idx;
		w_out[((size_t)i * lt.n_levels + level) * 8 + c] = w;
	}
}

// Corner records of the dense levels (LevelTable::rec): one thread per record, four table
// entries gathered with the encoder's own corner indexing (same modulo), one 16-B store.
__global__ void __launch_bounds__(256) k_dense_records(const uint32_t* __restrict__ table, const LevelTable lt,
                                                       uint4* __restrict__ rec, uint32_t total) {
	const uint32_t g = blockIdx.x * 256u + threadIdx.x;
	if (g >= total) return;
	uint32_t level = 0;
	for (uint32_t l = 0; l < lt.n_levels; ++l)
		if (!lt.hashed[l] && lt.rec_off[l] <= g) level = l;
	const uint32_t res = lt.res[level], size = lt.size[level], i = g - lt.rec_off[level];
	const uint32_t x = i % res, y = (i / res) % res, z = i / (res * res);
	const uint32_t* tab = table + lt.offset[level];
	rec[g] = make_uint4(tab[corner_index<false>(size, res, x, y, z)], tab[corner_index<false>(size, res, x + 1u, y, z)],
	                    tab[corner_index<false>(size, res, x, y + 1u, z)], tab[corner_index<false>(size, res, x + 1u, y + 1u, z)]);
}

LevelTable build_dense_records(ngp_model* m, const __half* table, hipStream_t s) {
	LevelTable lt = m->lt;
	lt.rec = nullptr;
	if (lt.F != 2 || m->tuning.encode_dense_records == 1) return lt;
	uint32_t total = 0;
	for (uint32_t l = 0; l < lt.n_levels; ++l) {
		lt.rec_off[l] = total;
		if (!lt.hashed[l]) total += lt.res[l] * lt.res[l] * (lt.res[l] + 1u);
	}
	if (total == 0) return lt;
	m->rs.dense_rec.reserve(total);
	k_dense_records<<<div_up(total, 256u), 256, 0, s>>>(reinterpret_cast<const uint32_t*>(table), lt, m->rs.dense_rec.ptr, total);
	NGP_HIP_CHECK(hipGetLastError());
	lt.rec = m->rs.dense_rec.ptr;
	return lt;
}

template <int SITE>
static void launch_fwd_site(const LevelTable& lt, const float* pos, uint32_t stride, uint32_t n, const __half* table,
                            __half* enc, EncLayout enc_plane, hipStream_t s, const uint32_t* n_dev, uint32_t max_chunks) {
	uint32_t n_chunks = div_up(n, 256);
	if (n_dev && max_chunks) n_chunks = std::min(n_chunks, max_chunks);
	// F = 2: 16-B quad gathers, four levels per thread (l, l + L/4, ...) where L % 4 == 0, else one
	// (8-B pair gathers and two levels per thread measured slower)
	if (lt.F == 2) {
		if (lt.n_levels % 4 == 0) {
			if (lt.regions) n_chunks = div_up(n_chunks, 8u) * 8u;  // K = n_chunks / 8 workgroups per XCD and group
			launch_timed(k_hashgrid_fwd<2, SITE, true, 4>, n_chunks * lt.n_levels / 4, 256, 0, s, n, pos, stride, table, lt, enc,
			             enc_plane, n_chunks, n_dev);
		}
		else
			launch_timed(k_hashgrid_fwd<2, SITE, true, 1>, n_chunks * lt.n_levels, 256, 0, s, n, pos, stride, table, lt, enc,
			             enc_plane, n_chunks, n_dev);
		return;
	}
	const uint32_t blocks = n_chunks * lt.n_levels;
	switch (lt.F) {
		case 1: launch_timed(k_hashgrid_fwd<1, SITE, false, 1>, blocks, 256, 0, s, n, pos, stride, table, lt, enc, enc_plane, n_chunks, n_dev); break;
		case 2: launch_timed(k_hashgrid_fwd<2, SITE, false, 1>, blocks, 256, 0, s, n, pos, stride, table, lt, enc, enc_plane, n_chunks, n_dev); break;
		case 4: launch_timed(k_hashgrid_fwd<4, SITE, false, 1>, blocks, 256, 0, s, n, pos, stride, table, lt, enc, enc_plane, n_chunks, n_dev); break;
		case 8: launch_timed(k_hashgrid_fwd<8, SITE, false, 1>, blocks, 256, 0, s, n, pos, stride, table, lt, enc, enc_plane, n_chunks, n_dev); break;
		default: throw std::runtime_error("n_features_per_level must be 1, 2, 4 or 8");
	}
}

void launch_hashgrid_fwd(const LevelTable& lt, const float* pos, uint32_t stride, uint32_t n, const __half* table,
                         __half* enc, EncLayout enc_plane, hipStream_t s, const uint32_t* n_dev, int site,
                         uint32_t max_chunks) {
	if (n == 0) return;
	if (site == 0) launch_fwd_site<0>(lt, pos, stride, n, table, enc, enc_plane, s, n_dev, max_chunks);
	else if (site == 1) launch_fwd_site<1>(lt, pos, stride, n, table, enc, enc_plane, s, n_dev, max_chunks);
	else launch_fwd_site<2>(lt, pos, stride, n, table, enc, enc_plane, s, n_dev, max_chunks);
	NGP_HIP_CHECK(hipGetLastError());
}

template <bool FIXED>
static void launch_bwd(const LevelTable& lt, const float* pos, uint32_t stride, uint32_t n, const __half* denc,
                       EncLayout enc_plane, __half* grad16, long long* grad64, hipStream_t s, const uint32_t* n_dev,
                       uint32_t n_chunks, uint32_t n_lv) {
	const uint32_t blocks = n_chunks * n_lv;
	switch (lt.F) {
		case 1: launch_timed(k_hashgrid_bwd<1, FIXED>, blocks, 256, 0, s, n, pos, stride, denc, enc_plane, lt, grad16, grad64, n_chunks, n_dev, n_lv); break;
		case 2: launch_timed(k_hashgrid_bwd<2, FIXED>, blocks, 256, 0, s, n, pos, stride, denc, enc_plane, lt, grad16, grad64, n_chunks, n_dev, n_lv); break;
		case 4: launch_timed(k_hashgrid_bwd<4, FIXED>, blocks, 256, 0, s, n, pos, stride, denc, enc_plane, lt, grad16, grad64, n_chunks, n_dev, n_lv); break;
		case 8: launch_timed(k_hashgrid_bwd<8, FIXED>, blocks, 256, 0, s, n, pos, stride, denc, enc_plane, lt, grad16, grad64, n_chunks, n_dev, n_lv); break;
		default: throw std::runtime_error("n_features_per_level must be 1, 2, 4 or 8");
	}
}

void launch_hashgrid_bwd(const LevelTable& lt, const float* pos, uint32_t stride, uint32_t n, const __half* denc,
                         EncLayout enc_plane, __half* grad_table, hipStream_t s, const uint32_t* n_dev, long long* grad64,
                         uint32_t max_chunks) {
	if (n == 0) return;
	uint32_t n_chunks = div_up(n, BWD_SAMPLES_PER_BLOCK);
	if (n_dev && max_chunks) n_chunks = std::min(n_chunks, max_chunks);
	if (grad64) launch_bwd<true>(lt, pos, stride, n, denc, enc_plane, nullptr, grad64, s, n_dev, n_chunks, lt.n_levels);
	else launch_bwd<false>(lt, pos, stride, n, denc, enc_plane, grad_table, nullptr, s, n_dev, n_chunks, lt.n_levels);
	NGP_HIP_CHECK(hipGetLastError());
}

void launch_hashgrid_indices(const LevelTable& lt, const float* pos, uint32_t stride, uint32_t n, uint32_t* idx,
                             float* w, hipStream_t s) {
	if (n == 0) return;
	k_hashgrid_indices<<<div_up((uint64_t)n * lt.n_levels, 256), 256, 0, s>>>(n, pos, stride, lt, idx, w);
	NGP_HIP_CHECK(hipGetLastError());
}

}  // namespace ngp
