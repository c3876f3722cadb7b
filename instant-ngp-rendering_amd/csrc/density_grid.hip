// density_grid.hip — occupancy-grid update for gfx950.
//
//  k_mark_untrained     mark_untrained_density_grid               src/testbed_nerf.cu:74-145
//  k_grid_samples       generate_grid_samples_nerf_nonuniform     src/testbed_nerf.cu:185-214
//  k_splat              splat_grid_samples_nerf_max_nearest_neighbor :216-232
//  k_ema                ema_grid_samples_nerf                     :253-276
//  k_grid_sum / mean    reduce_sum(max(v,0)/N) of update_density_grid_mean_and_bitfield :2362-2370
//  k_grid_to_bitfield   grid_to_bitfield                          :284-308
//  k_bitfield_max_pool  bitfield_max_pool                         :310-331
//
// The mean uses an exact fixed-point (2^-24) integer sum so the threshold, and
// therefore every bitfield bit, is independent of summation order (the
// reference's float atomics are not).
#include <hipcub/hipcub.hpp>

#include "ngp_internal.h"

namespace ngp {

__device__ __forceinline__ m43 load_xform_g(const float* x) {
	m43 m;
	for (int c = 0; c < 4; ++c) m.c[c] = mk3(x[3 * c + 0], x[3 * c + 1], x[3 * c + 2]);
	return m;
}

// inverse of the 3x3 rotation/scale part (column-major)
__device__ __forceinline__ void inverse3(const m43& m, v3 out_rows[3]) {
	const v3 a = m.c[0], b = m.c[1], c = m.c[2];
	// columns a,b,c: M = [a b c]; inverse rows are (b x c, c x a, a x b) / det
	const v3 bc = mk3(b.y * c.z - b.z * c.y, b.z * c.x - b.x * c.z, b.x * c.y - b.y * c.x);
	const v3 ca = mk3(c.y * a.z - c.z * a.y, c.z * a.x - c.x * a.z, c.x * a.y - c.y * a.x);
	const v3 ab = mk3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
	const float det = dot(a, bc);
	const float inv = 1.0f / det;
	out_rows[0] = bc * inv;
	out_rows[1] = ca * inv;
	out_rows[2] = ab * inv;
}

__global__ void __launch_bounds__(256) k_mark_untrained(uint32_t n_elements, float* __restrict__ grid,
                                                        const ngp_image* __restrict__ images, uint32_t n_images,
                                                        int clear_visible) {
	const uint32_t i = blockIdx.x * 256u + threadIdx.x;
	if (i >= n_elements) return;
	const uint32_t level = i / NERF_GRID_N_CELLS, pos_idx = i % NERF_GRID_N_CELLS;
	const uint32_t x = morton3D_invert(pos_idx >> 0), y = morton3D_invert(pos_idx >> 1), z = morton3D_invert(pos_idx >> 2);
	const float voxel_size = scalbnf(1.0f / (float)NERF_GRIDSIZE, (int)level);
	const v3 pos = (mk3((float)x, (float)y, (float)z) / (float)NERF_GRIDSIZE - 0.5f) * scalbnf(1.0f, (int)level) + 0.5f;
	const uint32_t min_count = 1;
	uint32_t count = 0;
	for (uint32_t j = 0; j < n_images && count < min_count; ++j) {
		const ngp_image im = images[j];
		if (im.lens_mode == 2 || im.lens_mode == 3 || im.lens_mode == 5) {  // FTheta, LatLong, Equirectangular
			++count;
			continue;
		}
		const m43 xf = load_xform_g(im.xform);
		v3 inv[3];
		inverse3(xf, inv);
		for (uint32_t k = 0; k < 8; ++k) {
			const v3 corner = pos + mk3((k & 1) ? voxel_size : 0.0f, (k & 2) ? voxel_size : 0.0f, (k & 4) ? voxel_size : 0.0f);
			const v3 dir = normalize(corner - xf.c[3]);
			if (dot(dir, xf.c[2]) < 1e-4f) continue;
			// pos_to_uv (common_device.cuh:497-531): camera frame, dir /= dir.z, the lens's distortion
			const v3 rel = corner - xf.c[3];
			const v3 cd = mk3(dot(inv[0], rel), dot(inv[1], rel), dot(inv[2], rel));
			float cx = cd.x / cd.z, cy = cd.y / cd.z;
			float du = 0.0f, dv = 0.0f;
			if (im.lens_mode == LENS_OPENCV) opencv_delta(im.lens_params, cx, cy, &du, &dv);
			else if (im.lens_mode == LENS_OPENCV_FISHEYE) opencv_fisheye_delta(im.lens_params, cx, cy, &du, &dv);
			cx += du;
			cy += dv;
			const float u = cx * im.focal_length[0] / (float)im.width + im.principal_point[0];
			const float v = cy * im.focal_length[1] / (float)im.height + im.principal_point[1];
			// uv_to_ray back-projection check (pos_to_uv is not injective under lens distortion)
			v3 rd;
			lens_direction(u, v, (float)im.width, (float)im.height, im.focal_length[0], im.focal_length[1], im.principal_point[0],
			               im.principal_point[1], im.lens_mode, im.lens_params, &rd);
			rd = normalize(rot(xf, rd));
			if (length(rd - dir) < 1e-3f && u > 0.0f && v > 0.0f && u < 1.0f && v < 1.0f) {
				++count;
				break;
			}
		}
	}
	if (clear_visible || (grid[i] < 0) != (count < min_count)) grid[i] = (count >= min_count) ? 0.0f : -1.0f;
}

__global__ void __launch_bounds__(256) k_grid_samples(uint32_t n_elements, pcg32 rng, uint32_t step, aabb3 aabb,
                                                      const float* __restrict__ grid_in, float* __restrict__ out,
                                                      uint32_t* __restrict__ indices, uint32_t n_cascades,
                                                      float thresh) {
	const uint32_t i = blockIdx.x * 256u + threadIdx.x;
	if (i >= n_elements) return;
	rng.advance((int64_t)i * 4);
	const uint32_t level = (uint32_t)(rng.next_float() * (float)n_cascades) % n_cascades;
	uint32_t idx = 0;
	for (uint32_t j = 0; j < 10; ++j) {
		idx = ((i + step * n_elements) * 56924617u + j * 19349663u + 96925573u) % NERF_GRID_N_CELLS;
		idx += level * NERF_GRID_N_CELLS;
		if (grid_in[idx] > thresh) break;
	}
	const uint32_t pos_idx = idx % NERF_GRID_N_CELLS;
	const uint32_t x = morton3D_invert(pos_idx >> 0), y = morton3D_invert(pos_idx >> 1), z = morton3D_invert(pos_idx >> 2);
	const float r0 = rng.next_float(), r1 = rng.next_float(), r2 = rng.next_float();
	const v3 pos = ((mk3((float)x, (float)y, (float)z) + mk3(r0, r1, r2)) / (float)NERF_GRIDSIZE - 0.5f) *
	                   scalbnf(1.0f, (int)level) + 0.5f;
	const v3 w = aabb_relative(aabb, pos);
	reinterpret_cast<float4*>(out)[i] = make_float4(w.x, w.y, w.z, warp_dt(MIN_CONE_STEPSIZE));
	indices[i] = idx;
}

__global__ void __launch_bounds__(256) k_splat(uint32_t n, const uint32_t* __restrict__ indices,
                                               const __half* __restrict__ out, float* __restrict__ grid_tmp,
                                               int density_act) {
	const uint32_t i = blockIdx.x * 256u + threadIdx.x;
	if (i >= n) return;
	const float mlp = network_to_density(__half2float(out[i]), density_act);
	const float thickness = mlp * MIN_CONE_STEPSIZE;
	atomicMax(reinterpret_cast<uint32_t*>(grid_tmp) + indices[i], __float_as_uint(thickness));
}

__global__ void __launch_bounds__(256) k_ema(uint32_t n, float decay, float* __restrict__ grid,
                                             const float* __restrict__ tmp) {
	const uint32_t i = blockIdx.x * 256u + threadIdx.x;
	if (i >= n) return;
	const float prev = grid[i];
	grid[i] = prev < 0.0f ? prev : fmaxf(prev * decay, tmp[i]);
}

__global__ void __launch_bounds__(256) k_grid_sum(const float* __restrict__ grid, uint32_t n,
                                                  unsigned long long* __restrict__ sum) {
	const uint32_t i0 = blockIdx.x * 1024u + threadIdx.x;
	unsigned long long s = 0;
#pragma unroll
	for (int k = 0; k < 4; ++k) {
		const uint32_t i = i0 + 256u * k;
		if (i < n) {
			const float v = fminf(fmaxf(grid[i], 0.0f), 65536.0f);
			s += (unsigned long long)(v * 16777216.0f);
		}
	}
	for (int d = 32; d > 0; d >>= 1) s += __shfl_down(s, d, 64);
	// one atomic per block (a same-address atomic per wave serialised at ~11 ns each: 100 us per update)
	__shared__ unsigned long long part[4];
	if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
	__syncthreads();
	if (threadIdx.x == 0) atomicAdd(sum, part[0] + part[1] + part[2] + part[3]);
}

__global__ void k_grid_mean(const unsigned long long* __restrict__ sum, float* __restrict__ mean) {
	*mean = (float)((double)*sum / 16777216.0 / (double)NERF_GRID_N_CELLS);
}

__global__ void __launch_bounds__(256) k_grid_to_bitfield(uint32_t n_elements, uint32_t n_nonzero,
                                                          const float* __restrict__ grid, uint8_t* __restrict__ bits,
                                                          const float* __restrict__ mean) {
	const uint32_t i = blockIdx.x * 256u + threadIdx.x;
	if (i >= n_elements) return;
	if (i >= n_nonzero) {
		bits[i] = 0;
		return;
	}
	const float thresh = fminf(NERF_MIN_OPTICAL_THICKNESS, *mean);
	uint8_t b = 0;
#pragma unroll
	for (uint32_t j = 0; j < 8; ++j) b |= grid[i * 8 + j] > thresh ? (uint8_t)(1u << j) : (uint8_t)0;
	bits[i] = b;
}

__global__ void __launch_bounds__(256) k_bitfield_max_pool(uint32_t n, const uint8_t* __restrict__ prev,
                                                           uint8_t* __restrict__ next) {
	const uint32_t i = blockIdx.x * 256u + threadIdx.x;
	if (i >= n) return;
	uint8_t b = 0;
#pragma unroll
	for (uint32_t j = 0; j < 8; ++j) b |= prev[i * 8 + j] > 0 ? (uint8_t)(1u << j) : (uint8_t)0;
	const uint32_t x = morton3D_invert(i >> 0) + NERF_GRIDSIZE / 8;
	const uint32_t y = morton3D_invert(i >> 1) + NERF_GRIDSIZE / 8;
	const uint32_t z = morton3D_invert(i >> 2) + NERF_GRIDSIZE / 8;
	next[morton3D(x, y, z)] |= b;
}

void grid_reserve(ngp_model* m, uint32_t n_cascades, uint32_t n_samples) {
	GridState& g = m->gs;
	if (g.grid.n < (size_t)NERF_GRID_N_CELLS * n_cascades) {
		// keep contents on growth (cascade count changes only when the dataset changes)
		DevBuf<float> old = g.grid;
		g.grid.ptr = nullptr;
		g.grid.n = 0;
		g.grid.reserve((size_t)NERF_GRID_N_CELLS * n_cascades);
		NGP_HIP_CHECK(hipMemset(g.grid.ptr, 0, g.grid.bytes()));
		if (old.ptr) {
			NGP_HIP_CHECK(hipMemcpy(g.grid.ptr, old.ptr, old.bytes(), hipMemcpyDeviceToDevice));
			old.release();
		}
	}
	g.tmp.reserve((size_t)NERF_GRID_N_CELLS * n_cascades);
	g.n_cascades = std::max(g.n_cascades, n_cascades);
	g.positions.reserve(4 * (size_t)std::max(n_samples, 1u));
	g.indices.reserve(std::max(n_samples, 1u));
	g.enc.reserve((size_t)m->lt.n_levels * std::max(n_samples, 1u) * m->lt.F);
	g.out.reserve(std::max(n_samples, 1u));
}

__global__ void k_iota(uint32_t n, uint32_t* __restrict__ v) {
	const uint32_t i = blockIdx.x * 256u + threadIdx.x;
	if (i < n) v[i] = i;
}

// positions of the samples in sorted order (16-B rows) for the encoder
__global__ void k_gather_rows(uint32_t n, const uint32_t* __restrict__ perm, const float4* __restrict__ src,
                              float4* __restrict__ dst) {
	const uint32_t i = blockIdx.x * 256u + threadIdx.x;
	if (i < n) dst[i] = src[perm[i]];
}

// Bucketed cell sort (ngp_tuning.grid_unsorted 0): the samples only need neighbouring lanes in neighbouring cells, not a
// total order, so they are bucketed by the top 14 bits of the cascade-major Morton key (2^21 / 2^14 = 128 cells, an
// 8x4x4 block of the finest cascade per bucket) in three kernels -- ranks from returning atomics, one-block scan, scatter
// -- instead of a full radix sort (~20 launches, ~200 us per update).  The order inside a bucket follows the atomics'
// arrival; the splat is a max per cell, so the grid does not depend on it.
constexpr uint32_t GRID_BUCKET_BITS = 14, GRID_BUCKETS = 1u << GRID_BUCKET_BITS;

__global__ void __launch_bounds__(256) k_bucket_rank(uint32_t n, const uint32_t* __restrict__ keys, uint32_t shift,
                                                     uint32_t* __restrict__ hist, uint32_t* __restrict__ rank) {
	const uint32_t i = blockIdx.x * 256u + threadIdx.x;
	if (i < n) rank[i] = atomicAdd(hist + (keys[i] >> shift), 1u);
}

// exclusive scan of the bucket counts (one block, 16 buckets per thread); leaves the counts zero for the next update
__global__ void __launch_bounds__(1024) k_bucket_scan(uint32_t* __restrict__ hist, uint32_t* __restrict__ base) {
	constexpr uint32_t PER = GRID_BUCKETS / 1024u;
	__shared__ uint32_t wave_sum[16];
	const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
	uint32_t c[PER], sum = 0;
#pragma unroll
	for (uint32_t k = 0; k < PER; ++k) {
		c[k] = hist[t * PER + k];
		hist[t * PER + k] = 0u;
		sum += c[k];
	}
	uint32_t incl = sum;  // inclusive scan over the wave
#pragma unroll
	for (uint32_t off = 1; off < 64; off <<= 1) {
		const uint32_t v = __shfl_up(incl, off, 64);
		if (lane >= off) incl += v;
	}
	if (lane == 63) wave_sum[w] = incl;
	__syncthreads();
	uint32_t prefix = 0;
	for (uint32_t k = 0; k < w; ++k) prefix += wave_sum[k];
	uint32_t run = prefix + incl - sum;
#pragma unroll
	for (uint32_t k = 0; k < PER; ++k) {
		base[t * PER + k] = run;
		run += c[k];
	}
}

__global__ void __launch_bounds__(256) k_bucket_scatter(uint32_t n, const uint32_t* __restrict__ keys, uint32_t shift,
                                                        const uint32_t* __restrict__ base, const uint32_t* __restrict__ rank,
                                                        const float4* __restrict__ pos, uint32_t* __restrict__ skeys,
                                                        float4* __restrict__ spos) {
	const uint32_t i = blockIdx.x * 256u + threadIdx.x;
	if (i >= n) return;
	const uint32_t key = keys[i], dst = base[key >> shift] + rank[i];
	skeys[dst] = key;
	spos[dst] = pos[i];
}

void run_grid_evaluate(ngp_model* m, const ngp_grid_args* a, hipStream_t s) {
	GridState& g = m->gs;
	const uint32_t n_cascades = a->max_cascade + 1;
	const uint32_t n_elements = NERF_GRID_N_CELLS * n_cascades;
	const uint32_t n_total = a->n_uniform_samples + a->n_nonuniform_samples;
	grid_reserve(m, n_cascades, n_total);
	aabb3 aabb;
	aabb.min = mk3(a->aabb_min[0], a->aabb_min[1], a->aabb_min[2]);
	aabb.max = mk3(a->aabb_max[0], a->aabb_max[1], a->aabb_max[2]);

	if (a->mark_untrained) {
		k_mark_untrained<<<div_up(n_elements, 256), 256, 0, s>>>(n_elements, g.grid.ptr, a->images, a->n_images,
		                                                         a->clear_visible);
	}
	NGP_HIP_CHECK(hipMemsetAsync(g.tmp.ptr, 0, sizeof(float) * n_elements, s));
	pcg32 rng;
	rng.state = a->rng_state;
	rng.inc = a->rng_inc;
	if (a->n_uniform_samples)
		k_grid_samples<<<div_up(a->n_uniform_samples, 256), 256, 0, s>>>(a->n_uniform_samples, rng, a->ema_step, aabb,
		                                                                  g.grid.ptr, g.positions.ptr, g.indices.ptr,
		                                                                  n_cascades, -0.01f);
	rng.advance();
	if (a->n_nonuniform_samples)
		k_grid_samples<<<div_up(a->n_nonuniform_samples, 256), 256, 0, s>>>(
		    a->n_nonuniform_samples, rng, a->ema_step, aabb, g.grid.ptr, g.positions.ptr + 4 * (size_t)a->n_uniform_samples,
		    g.indices.ptr + a->n_uniform_samples, n_cascades, NERF_MIN_OPTICAL_THICKNESS);
	NGP_HIP_CHECK(hipGetLastError());

	// Data-parallel: this rank evaluates a contiguous 1/world slice; tmp is max-reduced by the caller.
	const uint32_t world = std::max(a->world_size, 1u);
	const uint32_t per = div_up(n_total, world);
	const uint32_t first = std::min(n_total, a->rank * per);
	const uint32_t cnt = std::min(n_total - first, per);
	const __half* table = (a->use_inference_params ? m->infer16.ptr : m->params16.ptr) + m->n_mlp_params;
	const __half* frags = a->use_inference_params ? m->frag_infer.ptr : m->frag_train.ptr;
	if (cnt) {
		const float* pos = g.positions.ptr + 4 * (size_t)first;
		const uint32_t* idx = g.indices.ptr + first;
		// the samples are drawn in hash order, so the encoder's gathers were incoherent (2.6x the
		// algorithmic fetch, r02); sorted by cell index (cascade-major Morton order) neighbouring lanes
		// share corners.  The splat is a max per cell: the result does not depend on the order.
		const uint32_t bits = 21u + (uint32_t)std::ceil(std::log2((double)n_cascades));
		if (m->tuning.grid_unsorted == 0) {
			g.skeys.reserve(cnt);
			g.perm_in.reserve(cnt);
			g.spos.reserve(4 * (size_t)cnt);
			if (!g.bucket_hist.ptr) {
				g.bucket_hist.reserve(GRID_BUCKETS);
				NGP_HIP_CHECK(hipMemsetAsync(g.bucket_hist.ptr, 0, GRID_BUCKETS * sizeof(uint32_t), s));
			}
			g.bucket_base.reserve(GRID_BUCKETS);
			const uint32_t shift = bits - GRID_BUCKET_BITS;
			k_bucket_rank<<<div_up(cnt, 256), 256, 0, s>>>(cnt, idx, shift, g.bucket_hist.ptr, g.perm_in.ptr);
			k_bucket_scan<<<1, 1024, 0, s>>>(g.bucket_hist.ptr, g.bucket_base.ptr);
			k_bucket_scatter<<<div_up(cnt, 256), 256, 0, s>>>(cnt, idx, shift, g.bucket_base.ptr, g.perm_in.ptr,
			                                                  reinterpret_cast<const float4*>(pos), g.skeys.ptr,
			                                                  reinterpret_cast<float4*>(g.spos.ptr));
			pos = g.spos.ptr;
			idx = g.skeys.ptr;
		} else if (m->tuning.grid_unsorted == 2) {
			g.skeys.reserve(cnt);
			g.perm_in.reserve(cnt);
			g.perm.reserve(cnt);
			g.spos.reserve(4 * (size_t)cnt);
			size_t tmp_bytes = 0;
			NGP_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, idx, g.skeys.ptr, g.perm_in.ptr, g.perm.ptr, (int)cnt,
			                                                 0, (int)bits, s));
			g.sort_tmp.reserve(tmp_bytes / 4 + 1);
			k_iota<<<div_up(cnt, 256), 256, 0, s>>>(cnt, g.perm_in.ptr);
			NGP_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(g.sort_tmp.ptr, tmp_bytes, idx, g.skeys.ptr, g.perm_in.ptr, g.perm.ptr,
			                                                 (int)cnt, 0, (int)bits, s));
			k_gather_rows<<<div_up(cnt, 256), 256, 0, s>>>(cnt, g.perm.ptr, reinterpret_cast<const float4*>(pos),
			                                               reinterpret_cast<float4*>(g.spos.ptr));
			pos = g.spos.ptr;
			idx = g.skeys.ptr;
		}
		launch_hashgrid_fwd(m->lt, pos, 4, cnt, table, g.enc.ptr, internal_layout(m, cnt), s);
		launch_mlp_density(m, frags, g.enc.ptr, internal_layout(m, cnt), cnt, g.out.ptr, s);
		k_splat<<<div_up(cnt, 256), 256, 0, s>>>(cnt, idx, g.out.ptr, g.tmp.ptr, m->cfg.density_activation);
		NGP_HIP_CHECK(hipGetLastError());
	}
}

void run_grid_bitfield(ngp_model* m, uint32_t max_cascade, hipStream_t s) {
	GridState& g = m->gs;
	g.bitfield.reserve(NERF_GRID_N_CELLS / 8 * NERF_CASCADES);
	++g.version;
	g.mean.reserve(1);
	g.sum.reserve(1);
	grid_reserve(m, max_cascade + 1, 1);
	const uint32_t N = NERF_GRID_N_CELLS;
	NGP_HIP_CHECK(hipMemsetAsync(g.sum.ptr, 0, sizeof(unsigned long long), s));
	k_grid_sum<<<div_up(N, 1024), 256, 0, s>>>(g.grid.ptr, N, g.sum.ptr);  // 2048 blocks of 4 x 256 cells
	k_grid_mean<<<1, 1, 0, s>>>(g.sum.ptr, g.mean.ptr);
	k_grid_to_bitfield<<<div_up(N / 8 * NERF_CASCADES, 256), 256, 0, s>>>(N / 8 * NERF_CASCADES, N / 8 * (max_cascade + 1),
	                                                                      g.grid.ptr, g.bitfield.ptr, g.mean.ptr);
	for (uint32_t level = 1; level < NERF_CASCADES; ++level)
		k_bitfield_max_pool<<<div_up(N / 64, 256), 256, 0, s>>>(N / 64, g.bitfield.ptr + (size_t)(level - 1) * N / 8,
		                                                        g.bitfield.ptr + (size_t)level * N / 8);
	NGP_HIP_CHECK(hipGetLastError());
}

// generate_grid_samples_nerf_uniform (src/testbed_nerf.cu:147-160) for lattice points [first, first + n): point
// (x, y, z) / (res - 1) of the box, placed by transpose(box_to_local), warped into the training aabb.
struct LatticeBox {
	uint32_t rx, ry, rz;
	aabb3 box, train;
	float R[9];  // row-major box_to_local
	int rot;
};

__global__ void __launch_bounds__(256) k_lattice_points(uint32_t first, uint32_t n, LatticeBox L, float4* __restrict__ out) {
	const uint32_t j = blockIdx.x * 256u + threadIdx.x;
	if (j >= n) return;
	const uint32_t i = first + j;
	const uint32_t x = i % L.rx, y = (i / L.rx) % L.ry, z = i / (L.rx * L.ry);
	v3 p = mk3((float)x, (float)y, (float)z) / mk3((float)(L.rx - 1), (float)(L.ry - 1), (float)(L.rz - 1));
	p = p * (L.box.max - L.box.min) + L.box.min;
	if (L.rot) {
		// transpose(M) * p: component c is column c of M (row-major M[r][c] = R[3r + c]) dotted with p
		const float* R = L.R;
		p = mk3(R[0] * p.x + R[3] * p.y + R[6] * p.z, R[1] * p.x + R[4] * p.y + R[7] * p.z,
		        R[2] * p.x + R[5] * p.y + R[8] * p.z);
	}
	const v3 w = aabb_relative(L.train, p);
	out[j] = make_float4(w.x, w.y, w.z, warp_dt(MIN_CONE_STEPSIZE));
}

// grid_samples_half_to_float (:234-250): the raw (not activated) density output, -10000 where the cascaded
// density grid at the point's mip_from_pos cell is below NERF_MIN_OPTICAL_THICKNESS (outside the grid: 0).
__global__ void __launch_bounds__(256) k_grid_density_out(uint32_t n, const float4* __restrict__ rows,
                                                          const __half* __restrict__ mlp, aabb3 train,
                                                          const float* __restrict__ grid, uint32_t max_cascade,
                                                          float* __restrict__ dst) {
	const uint32_t i = blockIdx.x * 256u + threadIdx.x;
	if (i >= n) return;
	float v = __half2float(mlp[i]);
	if (grid) {
		const float4 r = rows[i];
		const v3 pos = unwarp_position(mk3(r.x, r.y, r.z), train);
		const uint32_t mip = mip_from_pos(pos, max_cascade);
		const uint32_t idx = cascaded_grid_idx_at(pos, mip);
		const float g = idx == 0xFFFFFFFFu ? 0.0f : grid[idx + (size_t)mip * NERF_GRID_N_CELLS];
		if (g < NERF_MIN_OPTICAL_THICKNESS) v = -10000.0f;
	}
	dst[i] = v;
}

void run_density_on_grid(ngp_model* m, const ngp_grid_query* q, float* out, hipStream_t s) {
	GridState& g = m->gs;
	LatticeBox L;
	L.rx = q->res[0];
	L.ry = q->res[1];
	L.rz = q->res[2];
	L.box.min = mk3(q->box_min[0], q->box_min[1], q->box_min[2]);
	L.box.max = mk3(q->box_max[0], q->box_max[1], q->box_max[2]);
	L.train.min = mk3(q->aabb_min[0], q->aabb_min[1], q->aabb_min[2]);
	L.train.max = mk3(q->aabb_max[0], q->aabb_max[1], q->aabb_max[2]);
	const RenderBox rb = make_render_box(L.box, q->box_to_local);
	for (int k = 0; k < 9; ++k) L.R[k] = rb.R[k];
	L.rot = rb.rot;
	const uint64_t n_total = (uint64_t)L.rx * L.ry * L.rz;
	const uint32_t batch = (uint32_t)std::min<uint64_t>(n_total, 1u << 20);  // the reference's 1M-point batches
	g.positions.reserve(4 * (size_t)batch);
	g.enc.reserve((size_t)m->lt.n_levels * batch * m->lt.F);
	g.out.reserve(batch);
	const __half* table = (q->use_inference_params ? m->infer16.ptr : m->params16.ptr) + m->n_mlp_params;
	const __half* frags = q->use_inference_params ? m->frag_infer.ptr : m->frag_train.ptr;
	const float* grid = q->mask_with_grid ? g.grid.ptr : nullptr;
	for (uint64_t first = 0; first < n_total; first += batch) {
		const uint32_t cnt = (uint32_t)std::min<uint64_t>(n_total - first, batch);
		float4* rows = reinterpret_cast<float4*>(g.positions.ptr);
		k_lattice_points<<<div_up(cnt, 256), 256, 0, s>>>((uint32_t)first, cnt, L, rows);
		launch_hashgrid_fwd(m->lt, g.positions.ptr, 4, cnt, table, g.enc.ptr, internal_layout(m, cnt), s);
		launch_mlp_density(m, frags, g.enc.ptr, internal_layout(m, cnt), cnt, g.out.ptr, s);
		k_grid_density_out<<<div_up(cnt, 256), 256, 0, s>>>(cnt, rows, g.out.ptr, L.train, grid, q->max_cascade, out + first);
		NGP_HIP_CHECK(hipGetLastError());
	}
}

void run_grid_finish(ngp_model* m, const ngp_grid_args* a, hipStream_t s) {
	GridState& g = m->gs;
	const uint32_t n_elements = NERF_GRID_N_CELLS * (a->max_cascade + 1);
	k_ema<<<div_up(n_elements, 256), 256, 0, s>>>(n_elements, a->decay, g.grid.ptr, g.tmp.ptr);
	NGP_HIP_CHECK(hipGetLastError());
	run_grid_bitfield(m, a->max_cascade, s);
}

}  // namespace ngp
