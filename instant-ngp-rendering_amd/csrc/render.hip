// render.hip — NeRF volume renderer (NerfTracer) for gfx950.
//
//  k_render_init    init_rays_with_payload_kernel_nerf + advance_pos_nerf  src/testbed_nerf.cu:1376-1489, 333-381
//  k_generate       generate_next_nerf_network_inputs                       :421-469
//  k_composite      composite_kernel_nerf (Shade mode) + compact_kernel_nerf :471-677, 1351-1374 (block
//                                                                            ballot + prefix, one atomic per block)
//  k_shade          shade_kernel_nerf                                       :1309-1349
//  k_accum_tonemap  accumulate_kernel + tonemap_kernel                      src/render_buffer.cu:232-266, 533-565
//
// Every ray's result depends only on its own sample sequence (the compaction
// only regroups rays), so the image is deterministic per pixel and matches the
// oracle's straight per-ray march whatever order the waves claim slots in.
#include <chrono>
#include <cstring>

#include "ngp_internal.h"

namespace ngp {

struct Payload {
	float o[3];
	float d[3];
	float n;  // next lattice point to test (stepping space)
	float max_weight;
	uint32_t idx;
	uint32_t n_steps;   // samples written this pass; bit 31: the ray left the AABB
	uint32_t base;      // first sample slot of this pass (samples are ray-major)
	float alpha_last;   // alpha of the last composited sample (next pass's sample budget)
};
constexpr uint32_t PAYLOAD_EXITED = 0x80000000u;
static_assert(sizeof(Payload) == 48, "payload layout");

struct RenderK {
	uint32_t prio;  // wave issue priority of the march kernels (ngp_tuning.render_priority bits 4-5)
	uint32_t W, H;
	uint32_t sample_index;
	m43 cam;
	float fx, fy, scx, scy;
	float near_distance;
	RenderBox aabb;    // the crop box (m_render_aabb in the frame of m_render_aabb_to_local)
	aabb3 train_aabb;  // the network's input warp (m_aabb)
	Stepping st;
	uint32_t max_mip;
	float min_transmittance;
	int snap;
	int linear_colors;
	int rgb_act, density_act;
	uint32_t shard_index, shard_count, shard_rows;
	uint32_t n_local;
	int lens_mode;
	float lens_params[7];
	m43 cam_end;        // motion blur / rolling shutter: the pixel's camera slerps toward it
	float rs[4];
	int rs_on;
	const float* dmap;  // learned distortion map [dry][drx][2] (null: off; LENS instance only)
	uint32_t drx, dry;
	uint32_t h_local, tiles_x;  // local rows; 8x8 pixel tiles per row of tiles
	uint32_t pipe_index, pipe_count;  // this pipeline's 8-row blocks of the shard's rows
	const uint8_t* df;  // octant distance fields [mip][octant][cell] (ngp_math.h lattice_step_df)
	int budget;         // per-ray sample budgets (sample_budget); 0: every ray gets n_steps
	float budget_scale;
	uint32_t* dbg;  // ngp_tuning.debug bit 0: [init lattice steps, init alive, generate iterations, samples, samples composited]
	int mode;       // NGP_RENDER_MODE_*
	float depth_scale;
	int hard_edges;
	float aperture, focus_z;  // depth of field (uv_to_ray, common_device.cuh:450-456)
	const float* normals;     // Normals mode: d(raw density)/d(warped position) per sample slot of the pass, [slot][3]
	float* sdt;               // optional [slot] warped dt, written by k_generate beside the row, read by k_composite (volumes)
	int mark_unfilled;        // unfilled slots get SH row NO_SH_ROW (the render MLP skips tiles of them)
	int exit_cap;             // a ray's per-pass budget is capped by the lattice points left to its exit
	int glow_mode;            // Nerf::glow_mode (composite_kernel_nerf's glow; 0 = off)
	float glow_y_cutoff;
	// ngp_render_args.host_frame (device-mapped), with the tonemap's parameters: finished rays' pixels go straight to it
	float4* hframe;
	uint8_t* hmask;  // [W * H]: 1 = the pixel's ray never marched (its background pixel is written by k_host_background)
	float4 hbg;
	float hexposure;
	int hcolor_space, hsrgb;
	// OpenCV / OpenCV-fisheye lenses: the undistorted camera-space direction (x, y, 1) of every pixel, a function of the
	// pixel, its jitter (sample_index / snap) and the intrinsics only -- cached across frames (RenderScratch::lens_key):
	// lens_fill = 1 computes and stores it (iterative_lens_undistortion, 100 Newton steps at most), 0 reads it back
	float2* lens_xy;
	int lens_fill;
};

// tonemap_kernel's per-pixel body (render_buffer.cu:533-565) after the accumulation: background, exposure, sRGB
__device__ __forceinline__ float4 tonemap_pixel(float4 c, int color_space, float exposure, float4 bg, int output_srgb) {
	if (color_space != 1) {
		bg.x = srgb_to_linear(bg.x);
		bg.y = srgb_to_linear(bg.y);
		bg.z = srgb_to_linear(bg.z);
	}
	const float weight = (1.0f - c.w) * bg.w;
	c.x += bg.x * weight;
	c.y += bg.y * weight;
	c.z += bg.z * weight;
	c.w += weight;
	if (color_space == 1) {
		c.x = srgb_to_linear(c.x);
		c.y = srgb_to_linear(c.y);
		c.z = srgb_to_linear(c.z);
	}
	const float e = powf(2.0f, exposure);
	c.x *= e;
	c.y *= e;
	c.z *= e;
	if (output_srgb) {
		c.x = linear_to_srgb(c.x);
		c.y = linear_to_srgb(c.y);
		c.z = linear_to_srgb(c.z);
	}
	return c;
}

// The finished pixel as render() returns it for one spp: shade_kernel_nerf's Shade colour over the cleared frame
// (t + 0 * (1 - t.w) = t), accumulate_kernel's first sample ((0 * 0 + c) / (0 + 1) = c, after linear_to_srgb in an
// sRGB buffer), then tonemap_pixel -- the arithmetic of k_shade + k_accum_tonemap, so the bits agree.  hit: the ray
// composited colour (c.w > 0.001); otherwise the pixel stays cleared.
__device__ __forceinline__ void write_host_pixel(const RenderK& k, uint32_t idx, float4 c, bool hit) {
	float4 t = hit ? c : make_float4(0.f, 0.f, 0.f, 0.f);
	if (hit && !k.linear_colors) {
		t.x = srgb_to_linear(t.x);
		t.y = srgb_to_linear(t.y);
		t.z = srgb_to_linear(t.z);
	}
	if (k.hcolor_space == 1) {
		t.x = linear_to_srgb(t.x);
		t.y = linear_to_srgb(t.y);
		t.z = linear_to_srgb(t.z);
	}
	k.hframe[idx] = tonemap_pixel(t, k.hcolor_space, k.hexposure, k.hbg, k.hsrgb);
}

// square2disk_shirley (random_val.cuh:112-128)
__device__ __forceinline__ void square2disk_shirley(float a, float b, float* x, float* y) {
	float phi, r;
	if (a * a > b * b) {
		r = a;
		phi = (NGP_PI / 4.0f) * (b / a);
	} else {
		r = b;
		phi = (NGP_PI / 2.0f) - (NGP_PI / 4.0f) * (a / b);
	}
	float s, c;
	sincosf(phi, &s, &c);
	*x = r * c;
	*y = r * s;
}

// uv_to_ray's camera-space -> world ray (common_device.cuh:445-459): rotate, depth of field (the
// origin jittered over the lens disk, the ray aimed at the focus plane), near distance.
__device__ __forceinline__ void camera_ray(const RenderK& k, const m43& cam, v3 dir_cam, float u, float v, v3* o, v3* d) {
	v3 dir = rot(cam, dir_cam);
	v3 origin = cam.c[3];
	if (k.aperture != 0.0f) {
		const v3 lookat = origin + dir * k.focus_z;
		const uint32_t px = (uint32_t)(int)(u * (float)k.W), py = (uint32_t)(int)(v * (float)k.H);
		float bx, by, dx, dy;
		ld_random_val_2d(k.sample_index, px * 19349663u + py * 96925573u, &bx, &by);
		square2disk_shirley(bx * 2.0f - 1.0f, by * 2.0f - 1.0f, &dx, &dy);
		origin = origin + cam.c[0] * (k.aperture * dx) + cam.c[1] * (k.aperture * dy);
		dir = (lookat - origin) * (1.0f / k.focus_z);
	}
	*o = origin + dir * k.near_distance;
	*d = dir;
}

__device__ __forceinline__ uint32_t local_to_global_row(const RenderK& k, uint32_t yl) {
	// pipeline-local row -> shard-local row (alternate 8-row blocks) -> frame row
	yl = ((yl >> 3) * k.pipe_count + k.pipe_index) * 8u + (yl & 7u);
	const uint32_t blk = yl / k.shard_rows, within = yl % k.shard_rows;
	return (blk * k.shard_count + k.shard_index) * k.shard_rows + within;
}

template <bool LENS>
__device__ __forceinline__ bool init_ray_body(const RenderK& k, uint32_t x, uint32_t yl, Payload* pp, float4* __restrict__ frame,
                                              float* __restrict__ depth_buffer);

// Stream compaction slot for a 256-thread block: ballot per wave, LDS prefix over the four
// waves, ONE global atomic per block and flag (instead of one per wave).  Returns the
// output index of this thread (valid only where flag is set).  Order within a block is
// deterministic; order between blocks is not (results never depend on it: every ray
// carries its own pixel index).
// Any block size up to 1024 threads: the atomics on one counter address serialise across
// the chip (~10 ns each), so the big render launches use large blocks to issue few of them.
__device__ __forceinline__ void block_append2(bool fa, bool fb, uint32_t* counter_a, uint32_t* counter_b, uint32_t* ia,
                                              uint32_t* ib) {
	__shared__ uint32_t wa[16], wb[16], base[2];
	const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
	const unsigned long long ma = __ballot(fa), mb = __ballot(fb);
	const unsigned long long below = lane == 0 ? 0ull : (~0ull >> (64 - lane));
	if (lane == 0) {
		wa[w] = (uint32_t)__popcll(ma);
		wb[w] = (uint32_t)__popcll(mb);
	}
	__syncthreads();
	if (threadIdx.x == 0) {
		uint32_t ta = 0, tb = 0;
		for (uint32_t k = 0; k < nw; ++k) {
			ta += wa[k];
			tb += wb[k];
		}
		base[0] = ta ? atomicAdd(counter_a, ta) : 0u;
		base[1] = tb ? atomicAdd(counter_b, tb) : 0u;
	}
	__syncthreads();
	uint32_t pa = base[0], pb = base[1];
	for (uint32_t k = 0; k < w; ++k) {
		pa += wa[k];
		pb += wb[k];
	}
	*ia = pa + (uint32_t)__popcll(ma & below);
	*ib = pb + (uint32_t)__popcll(mb & below);
}

// Reserves cnt consecutive slots of *counter for every thread of a 256-thread block: wave
// scans, LDS totals, ONE atomic per block.  Returns this thread's first slot.
__device__ __forceinline__ uint32_t block_reserve(uint32_t cnt, uint32_t* counter) {
	__shared__ uint32_t wsum[16], bbase;
	const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
	uint32_t x = cnt;
#pragma unroll
	for (uint32_t o = 1; o < 64; o <<= 1) {
		const uint32_t y = __shfl_up(x, o, 64);
		if (lane >= o) x += y;
	}
	if (lane == 63) wsum[w] = x;
	__syncthreads();
	if (threadIdx.x == 0) {
		uint32_t t = 0;
		for (uint32_t k = 0; k < nw; ++k) t += wsum[k];
		bbase = t ? atomicAdd(counter, t) : 0u;
	}
	__syncthreads();
	uint32_t b = bbase;
	for (uint32_t k = 0; k < w; ++k) b += wsum[k];
	return b + x - cnt;
}

// Adds v over the whole block to *counter with one atomic (all threads of the block call it).
__device__ __forceinline__ void block_add(uint32_t v, uint32_t* counter) {
	__shared__ uint32_t ws[16];
	const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
	for (uint32_t o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
	if (lane == 0) ws[w] = v;
	__syncthreads();
	if (threadIdx.x == 0) {
		uint32_t t = 0;
		for (uint32_t k = 0; k < nw; ++k) t += ws[k];
		if (t) atomicAdd(counter, t);
	}
}

// The 16 SH(4) inputs of the warped direction d as fp16 pairs (the rgb network's direction rows).
__device__ __forceinline__ void sh_row(v3 d, uint4* lo, uint4* hi) {
	const v3 wdir = warp_direction(d);
	float v[16];
	sh_deg4(wdir.x, wdir.y, wdir.z, v);
	uint32_t u[8];
#pragma unroll
	for (int q = 0; q < 8; ++q) {
		const _Float16 a = (_Float16)v[2 * q], b = (_Float16)v[2 * q + 1];
		u[q] = (uint32_t)__builtin_bit_cast(uint16_t, a) | ((uint32_t)__builtin_bit_cast(uint16_t, b) << 16);
	}
	*lo = make_uint4(u[0], u[1], u[2], u[3]);
	*hi = make_uint4(u[4], u[5], u[6], u[7]);
}

template <bool LENS>
__global__ void __launch_bounds__(256) k_render_init(RenderK k, Payload* __restrict__ payloads, float4* __restrict__ rgba,
                                                     float* __restrict__ depth, float4* __restrict__ frame,
                                                     float* __restrict__ depth_buffer, uint32_t* __restrict__ counters,
                                                     uint4* __restrict__ shrows) {
	// rays are numbered in 8x8 pixel tiles: a wave's 64 rays are a square patch, so at a
	// given step their samples are close in space (hash-grid gathers share cache lines)
	const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
	const uint32_t tile = r >> 6, x = (tile % k.tiles_x) * 8u + (r & 7u), yl = (tile / k.tiles_x) * 8u + ((r >> 3) & 7u);
	Payload p;
	bool alive = false;
	const bool inside = x < k.W && yl < k.h_local;
	if (inside) alive = init_ray_body<LENS>(k, x, yl, &p, frame, depth_buffer);
	// the pixels of rays that never march are written to the host by k_host_background on a side stream, spread
	// over the frame's passes (written here, a frame's background pixels were a burst of PCIe stores that held
	// this launch up)
	if (k.hframe && inside) k.hmask[p.idx] = alive ? 0 : 1;
	uint32_t slot, unused;
	block_append2(alive, false, &counters[0], &counters[3], &slot, &unused);
	if (alive) {
		payloads[slot] = p;
		rgba[slot] = make_float4(0.f, 0.f, 0.f, 0.f);
		depth[slot] = 0.0f;
		// the rgb network's direction inputs: one row of 16 fp16 SH values per ray and frame, indexed
		// by its pixel (the samples of every pass carry that index), instead of once per sample in the
		// MLP or once per ray and pass in k_generate
		uint4 lo, hi;
		sh_row(mk3(p.d[0], p.d[1], p.d[2]), &lo, &hi);
		shrows[2 * (size_t)p.idx] = lo;
		shrows[2 * (size_t)p.idx + 1] = hi;
	}
}

// init_rays_with_payload_kernel_nerf + advance_pos_nerf for pixel x of local row yl
template <bool LENS>
__device__ __forceinline__ bool init_ray_body(const RenderK& k, uint32_t x, uint32_t yl, Payload* pp, float4* __restrict__ frame,
                                              float* __restrict__ depth_buffer) {
	const uint32_t y = local_to_global_row(k, yl);
	const uint32_t idx = x + k.W * y;
	frame[idx] = make_float4(0.f, 0.f, 0.f, 0.f);
	depth_buffer[idx] = MAX_DEPTH;

	float ox, oy;
	ld_random_pixel_offset(k.snap ? 0u : k.sample_index, &ox, &oy);
	const float u = ((float)x + ox) / (float)k.W, v = ((float)y + oy) / (float)k.H;
	v3 dir = mk3((u - k.scx) * (float)k.W / k.fx, (v - k.scy) * (float)k.H / k.fy, 1.0f);
	// get_xform_given_rolling_shutter (src/testbed_nerf.cu:1416)
	const m43 cam = k.rs_on ? xform_given_rolling_shutter(k.cam, k.cam_end, k.rs, u, v, ld_random_val(k.sample_index, idx * 72239731u))
	                        : k.cam;
	if (LENS && k.lens_xy && !k.lens_fill) {
		const float2 c = k.lens_xy[idx];  // the same bits lens_direction returned when the entry was filled
		dir = mk3(c.x, c.y, 1.0f);
	} else if (LENS && !lens_direction(u, v, (float)k.W, (float)k.H, k.fx, k.fy, k.scx, k.scy, k.lens_mode, k.lens_params, &dir)) {
		*pp = Payload{};  // uv_to_ray returned Ray::invalid(): the pixel stays empty
		pp->idx = idx;
		return false;
	} else if (LENS && k.lens_xy) {
		k.lens_xy[idx] = make_float2(dir.x, dir.y);  // (the cached modes always return a ray with z = 1)
	}
	if (LENS && k.dmap) {  // uv_to_ray: dir.xy += distortion.at_lerp(uv) (common_device.cuh:441-443)
		float ddx, ddy;
		distortion_at_lerp(k.dmap, k.drx, k.dry, u, v, &ddx, &ddy);
		dir.x += ddx;
		dir.y += ddy;
	}
	v3 origin;
	camera_ray(k, cam, dir, u, v, &origin, &dir);

	Payload p;
	p.max_weight = 0.0f;
	p.idx = idx;
	p.n_steps = 0;
	p.base = 0;
	p.alpha_last = 0.0f;
	dir = normalize(dir);
	float t0, t1;
	ray_intersect(k.aabb.box, rbox_local(k.aabb, origin), rbox_local(k.aabb, dir), &t0, &t1);
	const float t = fmaxf(t0, 0.0f) + 1e-6f;
	p.o[0] = origin.x; p.o[1] = origin.y; p.o[2] = origin.z;
	p.d[0] = dir.x; p.d[1] = dir.y; p.d[2] = dir.z;
	p.n = 0.0f;
	bool alive = rbox_contains(k.aabb, origin + dir * t);
	if (alive) {
		// advance_pos_nerf: jitter the start and skip empty space
		const v3 idir = mk3(1.0f / dir.x, 1.0f / dir.y, 1.0f / dir.z);
		float n = step_to(k.st, t) + ld_random_val(k.sample_index, idx * 786433u);
		const uint32_t oct = ray_octant(dir);
		int st;
		uint32_t steps = 0;
		do {
			// several cascades (aabb_scale > 1): every mip's distance fetched at once; one cascade: nothing to climb
			st = k.max_mip ? lattice_step_df<true>(&n, k.st, origin, dir, idir, oct, k.df, k.max_mip, k.aabb)
			               : lattice_step_df<false>(&n, k.st, origin, dir, idir, oct, k.df, k.max_mip, k.aabb);
			++steps;
		} while (st == LATTICE_SKIPPED);
		alive = st == LATTICE_OCCUPIED;
		p.n = n;
		if (k.dbg) {
			atomicAdd(&k.dbg[0], steps);
			atomicAdd(&k.dbg[1], alive ? 1u : 0u);
		}
	}
	*pp = p;
	return alive;
}

// Slice render mode (render_nerf, src/testbed_nerf.cu:1842-1845, 1908-1932): no tracing -- every
// pixel's ray is evaluated once, at camera-space depth focus_z (init_rays_with_payload_kernel_nerf's
// plane_z < 0 branch, :1447-1456), with dt = MIN_CONE_STEPSIZE (generate_nerf_network_inputs_at_current
// _position, :397-403); then compute_nerf_rgba with depth 0.01 (:405-423) and shade_kernel_nerf.
template <bool LENS>
__global__ void __launch_bounds__(256) k_slice_init(RenderK k, uint32_t n, float* __restrict__ coords,
                                                    float4* __restrict__ frame, float* __restrict__ depth_buffer) {
	const uint32_t r = blockIdx.x * 256u + threadIdx.x;
	if (r >= n) return;
	const uint32_t x = r % k.W, yl = r / k.W;
	const uint32_t blk = yl / k.shard_rows, within = yl % k.shard_rows;
	const uint32_t y = (blk * k.shard_count + k.shard_index) * k.shard_rows + within;
	const uint32_t idx = x + k.W * y;
	frame[idx] = make_float4(0.f, 0.f, 0.f, 0.f);
	depth_buffer[idx] = MAX_DEPTH;
	float* c = coords + 8 * (size_t)r;
	float ox, oy;
	ld_random_pixel_offset(k.snap ? 0u : k.sample_index, &ox, &oy);
	const float u = ((float)x + ox) / (float)k.W, v = ((float)y + oy) / (float)k.H;
	v3 dir = mk3((u - k.scx) * (float)k.W / k.fx, (v - k.scy) * (float)k.H / k.fy, 1.0f);
	const m43 cam = k.rs_on ? xform_given_rolling_shutter(k.cam, k.cam_end, k.rs, u, v, ld_random_val(k.sample_index, idx * 72239731u))
	                        : k.cam;
	if (LENS && !lens_direction(u, v, (float)k.W, (float)k.H, k.fx, k.fy, k.scx, k.scy, k.lens_mode, k.lens_params, &dir)) {
		c[0] = __int_as_float(0x7fc00000);  // no ray: the pixel stays empty
		return;
	}
	if (LENS && k.dmap) {
		float ddx, ddy;
		distortion_at_lerp(k.dmap, k.drx, k.dry, u, v, &ddx, &ddy);
		dir.x += ddx;
		dir.y += ddy;
	}
	v3 o, d;
	camera_ray(k, cam, dir, u, v, &o, &d);  // (no aperture in Slice mode)
	const v3 pos = o + d * k.focus_z;        // t = -plane_z * |d| along the normalised direction
	const v3 wp = aabb_relative(k.train_aabb, pos), wd = warp_direction(normalize(d));
	c[0] = wp.x; c[1] = wp.y; c[2] = wp.z; c[3] = warp_dt(MIN_CONE_STEPSIZE);
	c[4] = wd.x; c[5] = wd.y; c[6] = wd.z; c[7] = 0.0f;
	depth_buffer[idx] = k.focus_z;
}

__global__ void __launch_bounds__(256) k_slice_shade(RenderK k, uint32_t n, const float* __restrict__ coords,
                                                     const __half* __restrict__ out, float4* __restrict__ frame) {
	const uint32_t r = blockIdx.x * 256u + threadIdx.x;
	if (r >= n || coords[8 * (size_t)r] != coords[8 * (size_t)r]) return;
	const uint32_t x = r % k.W, yl = r / k.W;
	const uint32_t blk = yl / k.shard_rows, within = yl % k.shard_rows;
	const uint32_t y = (blk * k.shard_count + k.shard_index) * k.shard_rows + within;
	const uint32_t idx = x + k.W * y;
	const __half* o = out + 4 * (size_t)r;
	const float density = network_to_density(__half2float(o[3]), k.density_act);
	const float alpha = fminf(fmaxf(1.0f - __expf(-density * 0.01f), 0.0f), 1.0f);
	float4 t = make_float4(network_to_rgb(__half2float(o[0]), k.rgb_act) * alpha, network_to_rgb(__half2float(o[1]), k.rgb_act) * alpha,
	                       network_to_rgb(__half2float(o[2]), k.rgb_act) * alpha, alpha);
	if (!k.linear_colors) {
		t.x = srgb_to_linear(t.x);
		t.y = srgb_to_linear(t.y);
		t.z = srgb_to_linear(t.z);
	}
	const float4 f = frame[idx];
	frame[idx] = make_float4(t.x + f.x * (1.0f - t.w), t.y + f.y * (1.0f - t.w), t.z + f.z * (1.0f - t.w), t.w + f.w * (1.0f - t.w));
}

// Octant distance fields (ngp_math.h lattice_step_df), three separable exact passes of the
// Chebyshev transform restricted to an orthant: D = min over occupied c' of max_k |c'_k - c_k|
// = min_z' max(dz, min_y' max(dy, min_x' dx)).  Rebuilt only when the bitfield changes.
// Pass x: one thread per (mip, x-sign, z, y) line, a sweep toward the line's start.
__global__ void __launch_bounds__(256) k_df_x(const uint8_t* __restrict__ bitfield, uint8_t* __restrict__ fx, uint32_t max_mip) {
	const uint32_t g = blockIdx.x * 256u + threadIdx.x;
	const uint32_t mip = g >> 15;
	if (mip > max_mip) return;
	const uint32_t sneg = (g >> 14) & 1u, y = g & 127u, z = (g >> 7) & 127u;
	const uint8_t* bits = bitfield + (size_t)mip * (NERF_GRID_N_CELLS / 8);
	uint8_t* out = fx + (size_t)(mip * 2u + sneg) * DF_BYTES_PER_FIELD + (z * NERF_GRIDSIZE + y) * NERF_GRIDSIZE;
	uint32_t dist = mip < max_mip ? 0u : 254u;  // beyond the grid: the next mip (occupied) / outside the AABB
	for (uint32_t k = 0; k < NERF_GRIDSIZE; ++k) {
		const uint32_t x = sneg ? k : NERF_GRIDSIZE - 1u - k;  // positive direction looks at x' >= x
		const uint32_t c = morton3D(x, y, z);
		dist = ((bits[c >> 3] >> (c & 7u)) & 1u) ? 0u : min(dist + 1u, 255u);
		out[x] = (uint8_t)dist;
	}
}

// Passes y and z: one thread per cell and sign combination; h = min_k max(k, f(c + s k)),
// stopping once k reaches the best value so far (the loop is as long as the answer).
template <uint32_t AXIS>
__global__ void __launch_bounds__(256) k_df_yz(const uint8_t* __restrict__ fin, uint8_t* __restrict__ fout, uint32_t max_mip) {
	constexpr uint32_t NV_IN = AXIS == 1 ? 2u : 4u;  // sign combinations of the input / output
	const uint32_t g = blockIdx.x * 256u + threadIdx.x;
	const uint32_t cell = g & (DF_BYTES_PER_FIELD - 1u), v = (g >> 21) & (2u * NV_IN - 1u);
	const uint32_t mip = g >> (AXIS == 1 ? 23 : 24);
	if (mip > max_mip) return;
	const uint32_t x = cell & 127u, y = (cell >> 7) & 127u, z = cell >> 14;
	const uint8_t* f = fin + (size_t)(mip * NV_IN + (v & (NV_IN - 1u))) * DF_BYTES_PER_FIELD;
	const bool neg = (v >> (AXIS == 1 ? 1 : 2)) & 1u;
	const int c0 = AXIS == 1 ? (int)y : (int)z;
	const uint32_t stride = AXIS == 1 ? NERF_GRIDSIZE : NERF_GRIDSIZE * NERF_GRIDSIZE;
	uint32_t h = f[cell];
	// k = 1, 2, ... while k < h, eight lattice steps per round: the eight byte loads of a round are independent
	// (one serial load per step made the pass latency-bound: ~300 us per pass on mostly empty grids).  Steps of a
	// round at or past the final h change nothing (max(k, f) >= k >= h), so the result is the step-by-step one.
	const uint32_t lim = neg ? (uint32_t)c0 : NERF_GRIDSIZE - 1u - (uint32_t)c0;  // steps before leaving the grid
	const int sstride = neg ? -(int)stride : (int)stride;
	uint32_t k = 1;
	while (k < h) {
		if (k > lim) {  // the next step leaves the grid: occupied below max_mip (the next mip), outside the AABB at it
			if (mip < max_mip) h = k;
			break;
		}
		const uint32_t kend = min(k + 8u, lim + 1u);
		uint32_t fk[8];
#pragma unroll
		for (uint32_t u = 0; u < 8; ++u) fk[u] = k + u < kend ? f[(uint32_t)((int)cell + (int)(k + u) * sstride)] : 255u;
#pragma unroll
		for (uint32_t u = 0; u < 8; ++u)
			if (k + u < kend) h = min(h, max(k + u, fk[u]));
		k = kend;
	}
	fout[(size_t)(mip * 2u * NV_IN + v) * DF_BYTES_PER_FIELD + cell] = (uint8_t)h;
	(void)x;
}

void build_distance_fields(ngp_model* m, uint32_t max_mip, hipStream_t s) {
	RenderScratch& rs = m->rs;
	if (rs.df_version == m->gs.version && rs.df_max_mip == max_mip) return;
	const size_t nm = max_mip + 1;
	rs.df.reserve(nm * 8 * DF_BYTES_PER_FIELD);
	rs.df_x.reserve(nm * 2 * DF_BYTES_PER_FIELD);
	rs.df_xy.reserve(nm * 4 * DF_BYTES_PER_FIELD);
	k_df_x<<<div_up(nm * 2 * NERF_GRIDSIZE * NERF_GRIDSIZE, 256), 256, 0, s>>>(m->gs.bitfield.ptr, rs.df_x.ptr, max_mip);
	k_df_yz<1><<<div_up(nm * 4 * DF_BYTES_PER_FIELD, 256), 256, 0, s>>>(rs.df_x.ptr, rs.df_xy.ptr, max_mip);
	k_df_yz<2><<<div_up(nm * 8 * DF_BYTES_PER_FIELD, 256), 256, 0, s>>>(rs.df_xy.ptr, rs.df.ptr, max_mip);
	NGP_HIP_CHECK(hipGetLastError());
	rs.df_version = m->gs.version;
	rs.df_max_mip = max_mip;
}

// After MARCH_ITER passes: rays still marching are finished with what they accumulated.
__global__ void __launch_bounds__(256) k_retire(uint32_t n, const Payload* __restrict__ sp, const float4* __restrict__ srgba,
                                                const float* __restrict__ sdepth, Payload* __restrict__ hp,
                                                float4* __restrict__ hrgba, float* __restrict__ hdepth,
                                                uint32_t* __restrict__ counters) {
	const uint32_t i = blockIdx.x * 256u + threadIdx.x;
	bool hit = false;
	if (i < n) hit = srgba[i].w > 0.001f;
	uint32_t oh, unused;
	block_append2(hit, false, &counters[2], &counters[3], &oh, &unused);
	if (hit) {
		hp[oh] = sp[i];
		hrgba[oh] = srgba[i];
		hdepth[oh] = sdepth[i];
	}
}

// The background pixels of a streamed host frame (rays that never marched: k_render_init's mask), on a side
// stream concurrent with the march passes; a modest grid (grid-stride) so it takes few CU slots.
__global__ void __launch_bounds__(256) k_host_background(RenderK k, uint32_t n) {
	const float4 bgpix = make_float4(0.f, 0.f, 0.f, 0.f);
	for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u)
		if (k.hmask[i]) write_host_pixel(k, i, bgpix, false);
}

// Publishes the tracer's counters [0, 8) of the previous pass to pinned host memory, so the
// host learns a pass's sizes by polling instead of enqueueing a copy and an event after
// every pass (each costs a queue drain).  Called by the first 8 threads of the first
// workgroup of the next pass's k_generate (the previous pass's kernels have all finished,
// and the counters it reads are not touched by this launch), or by k_publish after the
// last pass.  Each counter goes out as one 8-byte store (tag << 32 | value): the host
// waits until all eight words carry the pass's tag, so no store ordering -- and no fence --
// is needed.
__device__ __forceinline__ void publish_counters(const uint32_t* counters, unsigned long long* host, uint32_t tag) {
	const uint32_t v = __hip_atomic_load(counters + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	__hip_atomic_store(host + threadIdx.x, ((unsigned long long)tag << 32) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ void k_publish(const uint32_t* __restrict__ counters, unsigned long long* host, uint32_t tag) {
	if (threadIdx.x < 8) publish_counters(counters, host, tag);
}

// Samples a ray gets this pass: up to n_steps, fewer when its transmittance is already low
// -- enough to reach min_transmittance at the opacity of its last sample, with headroom.
// A short estimate only costs the ray another pass; samples past a ray's termination are
// the ones a fixed per-pass count wastes (the reference uses a fixed count, capped at 8).
__device__ __forceinline__ uint32_t sample_budget(const RenderK& k, float T, float alpha_last, uint32_t n_steps) {
	if (!k.budget || T >= 1.0f || alpha_last <= 1e-4f) return n_steps;
	if (T <= k.min_transmittance || alpha_last >= 0.999f) return 1u;
	const float est = __logf(k.min_transmittance / T) / __logf(1.0f - alpha_last);
	const float b = ceilf(est * k.budget_scale) + 1.0f;
	return b >= (float)n_steps ? n_steps : (uint32_t)fmaxf(b, 1.0f);
}

// Lattice points a ray at stepping-space position n can still sample before it leaves the render
// box: floor(n_exit - n) + 1 points at or before the exit, plus one of margin for the rounding of
// n_exit (a bound only: a ray whose budget runs out before its exit simply continues next pass).
__device__ __forceinline__ uint32_t points_to_exit(const RenderK& k, v3 o, v3 d, float n) {
	float t0, t1;
	ray_intersect(k.aabb.box, rbox_local(k.aabb, o), rbox_local(k.aabb, d), &t0, &t1);
	const float left = step_to(k.st, fminf(t1, MAX_DEPTH)) - n;
	return left < 0.0f ? 1u : (left > 1048576.0f ? 1048576u : (uint32_t)left + 2u);
}

// generate_next_nerf_network_inputs (testbed_nerf.cu:421-469): the next samples of every
// alive ray.  Each ray first reserves its budget of sample slots (one atomic per block),
// so the pass's samples are ray-major and packed; the encode and MLP read the total from
// the device.  G lanes cooperate on one ray: each iteration they test G consecutive
// lattice points at once (ballots give the occupied ones in order and the first exit),
// and an all-empty round jumps on from the last lane's verified skip.  G = 1 for the big
// early passes (one lane per ray, flat loop), up to 64 for the last few thousand rays,
// whose long serial marches otherwise dominate the tail passes.  A ray's budget is its
// transmittance budget (sample_budget), capped by the lattice points left to its exit
// (k.exit_cap): the slots a ray reserves but does not fill still cost a 20-B row store,
// the encoder's zero features and, in mixed tiles, the MLP.
// One ray's march of a pass (the body of generate_next_nerf_network_inputs for G lanes per ray): reserves the ray's
// budget of slots (block_reserve: every thread of the workgroup calls this, running = false for idle lanes), writes
// its samples from lattice point *n on (positions + warped dt rows, SH row indices, optional dt array), pads the
// slots it did not fill, and returns the samples written; *n / *exited / *base are the ray's next state.  cap_slots:
// the slot arrays' extent (a reservation past it is cut; the ray continues next pass).
template <uint32_t G>
__device__ __forceinline__ uint32_t march_ray(const RenderK& k, bool valid, v3 o, v3 d, float* n_io, uint32_t row, uint32_t budget,
                                              float4* __restrict__ posdt, uint32_t* __restrict__ sray, float* __restrict__ sdt,
                                              uint32_t* __restrict__ sample_counter, uint32_t cap_slots, uint32_t* base_out,
                                              bool* exited_out) {
	const uint32_t lane = threadIdx.x & 63u;
	const uint32_t r = lane % G, g0 = lane - r;  // rank in the ray's group, first lane of the group
	const unsigned long long gmask = G == 64 ? ~0ull : (((1ull << G) - 1ull) << g0);
	bool running = valid;
	float n = *n_io;
	const v3 idir = mk3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
	uint32_t base = block_reserve(r == 0 ? budget : 0u, sample_counter);
	if (G > 1) base = __shfl(base, g0, 64);
	if (valid && base + budget > cap_slots) budget = base < cap_slots ? cap_slots - base : 0u;
	float4* const out_rows = posdt + base;
	const uint32_t oct = ray_octant(d);
	uint32_t j = 0, iters = 0;
	bool exited = false;
	if (budget == 0) running = false;
	while (__ballot(running) != 0ull) {
		iters += running;
		float nr = n + (float)r;
		int st = LATTICE_EXIT;
		if (running)
			st = lattice_step_df(&nr, k.st, o, d, idir, oct, k.df, k.max_mip, k.aabb);
		const unsigned long long m_exit = __ballot(running && st == LATTICE_EXIT) & gmask;
		const unsigned long long m_occ = __ballot(running && st == LATTICE_OCCUPIED) & gmask;
		const float n_last = __shfl(st == LATTICE_SKIPPED ? nr : n + (float)G, g0 + G - 1, 64);
		if (!running) continue;
		const uint32_t fe = m_exit ? (uint32_t)(__ffsll((long long)m_exit) - 1) : 64u;
		const unsigned long long emit = m_occ & (fe >= 64 ? ~0ull : ((1ull << fe) - 1ull));
		const uint32_t cnt = __popcll(emit), room = budget - j;
		if ((emit >> lane) & 1ull) {
			const uint32_t rank = __popcll(emit & ((1ull << lane) - 1ull));
			if (rank < room) {
				const float pn = n + (float)r;
				const float t = step_from(k.st, pn);
				const float dt = step_from(k.st, pn + 1.0f) - t;
				const v3 wp = aabb_relative(k.train_aabb, o + d * t);
				out_rows[j + rank] = make_float4(wp.x, wp.y, wp.z, warp_dt(dt));
				if (sdt) sdt[(size_t)base + j + rank] = warp_dt(dt);
				sray[(size_t)base + j + rank] = row;
			}
		}
		if (cnt >= room) {
			unsigned long long m = emit;  // the room-th emitted lane carries the last sample
			for (uint32_t t = 1; t < room; ++t) m &= m - 1ull;
			n += (float)((uint32_t)(__ffsll((long long)m) - 1) - g0 + 1u);
			j = budget;
			running = false;
		} else {
			j += cnt;
			if (m_exit) {
				exited = true;
				running = false;
			} else {
				n = n_last;
			}
		}
	}
	if (valid) {
		// reserved slots the ray did not fill (it left the volume) still go through the encoder
		// and the MLP: x = -1 marks them for the encoder to skip (zero features)
		const uint32_t tail_row = k.mark_unfilled ? NO_SH_ROW : row;
		for (uint32_t q = j + r; q < budget; q += G) {
			posdt[(size_t)base + q] = make_float4(-1.0f, -1.0f, -1.0f, 0.0f);
			sray[(size_t)base + q] = tail_row;
		}
	}
	if (k.dbg && valid && r == 0) {
		atomicAdd(&k.dbg[2], iters);
		atomicAdd(&k.dbg[3], j);
		atomicAdd(&k.dbg[5], budget);
	}
	*n_io = n;
	*base_out = base;
	*exited_out = exited;
	return j;
}

// The ray's slot budget of a pass: sample_budget of its transmittance, capped by the points left to its exit.
__device__ __forceinline__ uint32_t ray_budget(const RenderK& k, float T, float alpha_last, uint32_t n_steps, v3 o, v3 d, float n) {
	uint32_t budget = sample_budget(k, T, alpha_last, n_steps);
	if (k.exit_cap) budget = min(budget, points_to_exit(k, o, d, n));
	return budget;
}

template <uint32_t G>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(8))) k_generate(RenderK k, const uint32_t* __restrict__ alive_counter,
                                                  Payload* __restrict__ payloads, const float4* __restrict__ rgba,
                                                  float4* __restrict__ posdt, uint32_t* __restrict__ sray,
                                                  uint32_t target, uint32_t max_steps,
                                                  uint32_t* __restrict__ next_alive_counter,
                                                  uint32_t* __restrict__ sample_counter, uint32_t* __restrict__ steps_out,
                                                  const uint32_t* counters, unsigned long long* host_prev, uint32_t tag_prev) {
	set_wave_priority(k.prio);
	// the previous pass's counters, before this block zeroes next_alive_counter / steps_out
	if (host_prev && blockIdx.x == 0 && threadIdx.x < 8) publish_counters(counters, host_prev, tag_prev);
	__syncthreads();
	// the pass is sized on the device: the host enqueues passes ahead of their read-backs
	const uint32_t n_alive = *alive_counter;
	// samples per ray per pass (the reference caps this at 8): a free schedule parameter, since
	// every ray composites its own samples in order and stops at the same one whatever the chunking
	const uint32_t n_steps = min(max(target / max(n_alive, 1u), 1u), max_steps);
	if (blockIdx.x == 0 && threadIdx.x == 0) {
		*next_alive_counter = 0;  // filled by this pass's k_composite
		*steps_out = n_alive ? n_steps : 0u;
	}
	const uint32_t i = (blockIdx.x * blockDim.x + threadIdx.x) / G;
	const bool valid = i < n_alive;  // group-uniform
	Payload* p = payloads + (valid ? i : 0);
	v3 o = mk3(0.0f), d = mk3(1.0f);
	float n = 0.0f;
	uint32_t row = 0;  // the ray's SH row (its pixel index; written once per frame by k_render_init)
	uint32_t budget = 0;
	if (valid) {
		o = mk3(p->o[0], p->o[1], p->o[2]);
		d = mk3(p->d[0], p->d[1], p->d[2]);
		n = p->n;
		row = p->idx;
		budget = ray_budget(k, 1.0f - rgba[i].w, p->alpha_last, n_steps, o, d, n);
	}
	uint32_t base;
	bool exited;
	const uint32_t j = march_ray<G>(k, valid, o, d, &n, row, budget, posdt, sray, k.sdt, sample_counter, 0xffffffffu, &base, &exited);
	if (valid && (threadIdx.x % G) == 0) {
		p->n_steps = j | (exited ? PAYLOAD_EXITED : 0u);
		p->base = base;
		if (!exited) p->n = n;
	}
}

// samples loaded ahead of their use in k_composite (8 measured no better, same-weights A/B; so did all
// of a tail pass's samples at once, profiles/r03_tail_composite_ab.txt)
constexpr uint32_t COMPOSITE_AHEAD = 4;

// composite_kernel_nerf's glow (testbed_nerf.cu:540-628): grid lines and a cut line below glow_y_cutoff
// added to the sample's colour (or replacing it, grid mode); mask_to_alpha scales the sample's weight
__device__ __forceinline__ void apply_glow(const RenderK& k, v3 pos, v3 cam_pos, v3* rgb, float* weight) {
	const int gm = k.glow_mode;
	const bool green_grid = gm & 1, green_cutline = gm & 2, mask_to_alpha = gm & 4, radial = gm & 8, grid_mode = gm & 16;
	float glow = 0.0f;
	float dist = pos.y;
	if (radial) dist = fminf(length(pos - cam_pos), (4.5f - pos.y) * 0.333f);
	if (grid_mode) {
		glow = 1.0f / fmaxf(1.0f, dist);
	} else {
		float y = k.glow_y_cutoff - dist, mask = 0.0f;
		if (y > 0.0f) {
			y *= 80.0f;
			mask = fminf(1.0f, y);
			if (green_cutline) glow += fmaxf(0.0f, 1.0f - fabsf(1.0f - y)) * 4.0f;
			if (y > 1.0f) y = 1.0f - (y - 1.0f) * 0.05f;
			if (green_grid) glow += fmaxf(0.0f, y / fmaxf(1.0f, dist));
		}
		if (mask_to_alpha) *weight *= mask;
	}
	if (glow > 0.0f) {
		const float PI = 3.141592653589793f;
		float line = 0.0f;
#pragma unroll
		for (int f = 2; f <= 16; f *= 2) {  // the reference's products, left to right: pos * f * pi * 16
			line += fmaxf(0.0f, cosf(pos.y * (float)f * PI * 16.0f) - 0.975f);
			line += fmaxf(0.0f, cosf(pos.x * (float)f * PI * 16.0f) - 0.975f);
			line += fmaxf(0.0f, cosf(pos.z * (float)f * PI * 16.0f) - 0.975f);
		}
		if (grid_mode) {
			glow = glow * line * 15.0f;
			*rgb = mk3(glow * 0.25f, glow, glow * 0.5f);
		} else {
			glow = glow * glow * 0.25f + glow * line * 15.0f;
			*rgb = mk3(rgb->x + glow * 0.25f, rgb->y + glow, rgb->z + glow * 0.5f);
		}
	}
}

// composite_kernel_nerf's per-ray loop over one pass's samples of the ray (its n_steps slots from p.base): updates
// p (max weight, alpha of the last sample), c and local_depth; returns whether the ray goes on -- neither opaque
// (c.w > 1 - min_transmittance) nor out of the volume during the pass.  sdt: the pass's dt array (null: the rows' w).
template <bool MODES>
__device__ __forceinline__ bool composite_ray(const RenderK& k, Payload& p, float4& c, float& local_depth,
                                              const float4* __restrict__ posdt, const float* __restrict__ sdt,
                                              const __half* __restrict__ out) {
	{
		const v3 cam_fwd = k.cam.c[2], cam_pos = k.cam.c[3];
		const uint32_t actual = p.n_steps & ~PAYLOAD_EXITED;
		const size_t sbase = p.base;
		// samples are loaded 4 ahead of their use (the loop is otherwise one dependent
		// global-load latency per sample)
		bool done = false;
		uint32_t used = actual;
		float alpha_last = p.alpha_last;
		// only each sample's dt is read in the loop (4 B: the dt array for volumes, else the row's w); the position of
		// the max-weight sample -- the depth -- is read once after it
		size_t s_max = ~(size_t)0;
		for (uint32_t j0 = 0; j0 < actual && !done; j0 += COMPOSITE_AHEAD) {
			uint2 o2[COMPOSITE_AHEAD];
			float wdt[COMPOSITE_AHEAD];
#pragma unroll
			for (uint32_t u = 0; u < COMPOSITE_AHEAD; ++u) {
				if (j0 + u < actual) {
					const size_t s = sbase + j0 + u;
					o2[u] = *reinterpret_cast<const uint2*>(out + 4 * s);
					wdt[u] = sdt ? sdt[s] : reinterpret_cast<const float*>(posdt)[4 * s + 3];
				}
			}
#pragma unroll
			for (uint32_t u = 0; u < COMPOSITE_AHEAD; ++u) {
				if (done || j0 + u >= actual) continue;
				const __half2 rg = *reinterpret_cast<const __half2*>(&o2[u].x), bs = *reinterpret_cast<const __half2*>(&o2[u].y);
				const float T = 1.0f - c.w;
				const float dt = unwarp_dt(wdt[u]);
				const float alpha = 1.0f - __expf(-network_to_density(__high2float(bs), k.density_act) * dt);
				float weight = alpha * T;
				v3 rgb = mk3(network_to_rgb(__low2float(rg), k.rgb_act), network_to_rgb(__high2float(rg), k.rgb_act),
				             network_to_rgb(__low2float(bs), k.rgb_act));
				if constexpr (MODES) {
					const size_t s = sbase + j0 + u;
					if (k.glow_mode) {
						const float4 crd = posdt[s];
						apply_glow(k, unwarp_position(mk3(crd.x, crd.y, crd.z), k.train_aabb), cam_pos, &rgb, &weight);
					}
					if (k.mode == NGP_RENDER_MODE_NORMALS) {
						// the reference replaces the network input by its gradient (input_gradient, :1715-1717)
						const float* g = k.normals + 3 * s;
						const float dd = -network_to_density_derivative(__high2float(bs), k.density_act);
						rgb = normalize(mk3(g[0] * dd, g[1] * dd, g[2] * dd));
					} else if (k.mode == NGP_RENDER_MODE_POSITIONS || k.mode == NGP_RENDER_MODE_DEPTH) {
						const float4 crd = posdt[s];
						const v3 pos = unwarp_position(mk3(crd.x, crd.y, crd.z), k.train_aabb);
						rgb = k.mode == NGP_RENDER_MODE_POSITIONS ? (pos - 0.5f) * 0.5f + 0.5f
						                                          : mk3(dot(cam_fwd, pos - mk3(p.o[0], p.o[1], p.o[2])) * k.depth_scale);
					} else if (k.mode == NGP_RENDER_MODE_AO) {
						rgb = mk3(alpha);
					}
				}
				alpha_last = alpha;
				if (!MODES || k.mode != NGP_RENDER_MODE_COST) {
					c.x += rgb.x * weight;
					c.y += rgb.y * weight;
					c.z += rgb.z * weight;
				}
				c.w += weight;
				if (weight > p.max_weight) {
					p.max_weight = weight;
					s_max = sbase + j0 + u;
				}
				if (c.w > (1.0f - k.min_transmittance)) {
					const float inv = 1.0f / c.w;
					if (!MODES || k.mode != NGP_RENDER_MODE_COST) {
						c.x *= inv;
						c.y *= inv;
						c.z *= inv;
					} else {
						c.x += (float)(j0 + u);  // the reference's n_steps = j + current_step at the break
					}
					c.w *= inv;
					used = j0 + u + 1;
					done = true;
				}
			}
		}
		if (s_max != ~(size_t)0) {
			const float4 crd = posdt[s_max];
			const v3 pos = unwarp_position(mk3(crd.x, crd.y, crd.z), k.train_aabb);
			local_depth = dot(cam_fwd, pos - cam_pos);
		}
		if (k.dbg) atomicAdd(&k.dbg[4], used);
		// Cost: a ray going on (or leaving the volume) adds all of this pass's samples
		if (MODES && k.mode == NGP_RENDER_MODE_COST && !done) c.x += (float)actual;
		p.alpha_last = alpha_last;
		// finished: opaque enough, or the ray left the volume during this pass
		return !(done || (p.n_steps & PAYLOAD_EXITED));
	}
}

// composite_kernel_nerf (testbed_nerf.cu:471-677) fused with compact_kernel_nerf (:1351-1374):
// each thread composites its ray's samples of this pass in order, then the block appends the
// ray to the next pass's alive buffer, or (finished with colour) to the hit buffer.
// MODES: the render modes other than Shade (:626-638) replace a sample's colour -- AO: its alpha,
// Positions / Depth: its position / camera depth, Normals: the normalised negative density
// gradient; Cost counts the ray's composited samples in c.x (shade_kernel_nerf turns it into a
// grey level, :1327-1330) as payload.n_steps = j + current_step does (:664-667).
template <bool MODES>
__global__ void __launch_bounds__(1024) k_composite(RenderK k, const uint32_t* __restrict__ alive_in,
                                                   const Payload* __restrict__ sp, const float4* __restrict__ srgba,
                                                   const float* __restrict__ sdepth, const float4* __restrict__ posdt,
                                                   const __half* __restrict__ out,
                                                   Payload* __restrict__ dp, float4* __restrict__ drgba,
                                                   float* __restrict__ ddepth, Payload* __restrict__ hp,
                                                   float4* __restrict__ hrgba, float* __restrict__ hdepth,
                                                   uint32_t* __restrict__ alive_counter, uint32_t* __restrict__ hit_counter,
                                                   uint32_t* __restrict__ next_sample_counter,
                                                   uint32_t* __restrict__ filled_counter) {
	set_wave_priority(k.prio);
	if (blockIdx.x == 0 && threadIdx.x == 0) *next_sample_counter = 0;  // the next pass's k_generate reserves from it
	const uint32_t n_alive = *alive_in;
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	Payload p;
	float4 c = make_float4(0.f, 0.f, 0.f, 0.f);
	float local_depth = 0.0f;
	bool alive = false;
	uint32_t filled = 0;
	if (i < n_alive) {
		p = sp[i];
		c = srgba[i];
		local_depth = sdepth[i];
		alive = true;
	}
	if (alive) {
		filled = p.n_steps & ~PAYLOAD_EXITED;
		alive = composite_ray<MODES>(k, p, c, local_depth, posdt, k.sdt, out);
	}
	const bool hit = i < n_alive && !alive && c.w > 0.001f;
	if (!MODES && k.hframe && i < n_alive && !alive) write_host_pixel(k, p.idx, c, hit);
	// samples the rays actually filled this pass (reserved slots past an exit are not counted):
	// the frame's network-evaluated sample count for the roofline
	block_add(filled, filled_counter);
	uint32_t oa, oh;
	block_append2(alive, hit, alive_counter, hit_counter, &oa, &oh);
	if (alive) {
		dp[oa] = p;
		drgba[oa] = c;
		ddepth[oa] = local_depth;
	} else if (hit) {
		hp[oh] = p;
		hrgba[oh] = c;
		hdepth[oh] = local_depth;
	}
}

// Normals mode: dL/dout = d/d(raw density) for the pass's samples (fp16 [n][4])
__global__ void k_density_unit_dloss(const uint32_t* __restrict__ n_dev, uint32_t n, __half* __restrict__ dl) {
	const uint32_t i = blockIdx.x * 256u + threadIdx.x;
	if (i >= n || i >= *n_dev) return;
	const __half z = __float2half(0.0f);
	dl[4 * (size_t)i + 0] = z;
	dl[4 * (size_t)i + 1] = z;
	dl[4 * (size_t)i + 2] = z;
	dl[4 * (size_t)i + 3] = __float2half(1.0f);
}

// shade_kernel_nerf (testbed_nerf.cu:1309-1349) with its render modes
__global__ void __launch_bounds__(256) k_shade(RenderK k, uint32_t n, const Payload* __restrict__ hp, const float4* __restrict__ hrgba,
                                               const float* __restrict__ hdepth, int linear_colors,
                                               float4* __restrict__ frame, float* __restrict__ depth_buffer) {
	const uint32_t i = blockIdx.x * 256u + threadIdx.x;
	if (i >= n) return;
	const uint32_t idx = hp[i].idx;
	float4 t = hrgba[i];
	if (k.mode == NGP_RENDER_MODE_NORMALS) {
		const v3 nn = normalize(mk3(t.x, t.y, t.z));
		t.x = (0.5f * nn.x + 0.5f) * t.w;
		t.y = (0.5f * nn.y + 0.5f) * t.w;
		t.z = (0.5f * nn.z + 0.5f) * t.w;
	} else if (k.mode == NGP_RENDER_MODE_COST) {
		const float col = t.x / 128.0f;
		t = make_float4(col, col, col, 1.0f);
	} else if (k.hard_edges && k.mode == NGP_RENDER_MODE_DEPTH) {
		const float dv = hdepth[i] * k.depth_scale;
		t.x = t.y = t.z = dv;
	} else if (k.hard_edges && k.mode == NGP_RENDER_MODE_POSITIONS) {
		const v3 d = mk3(hp[i].d[0], hp[i].d[1], hp[i].d[2]);
		const v3 pos = k.cam.c[3] + d * (hdepth[i] / dot(d, k.cam.c[2]));
		t.x = (pos.x - 0.5f) * 0.5f + 0.5f;
		t.y = (pos.y - 0.5f) * 0.5f + 0.5f;
		t.z = (pos.z - 0.5f) * 0.5f + 0.5f;
	}
	if (!linear_colors && k.mode == NGP_RENDER_MODE_SHADE) {
		t.x = srgb_to_linear(t.x);
		t.y = srgb_to_linear(t.y);
		t.z = srgb_to_linear(t.z);
	}
	const float4 f = frame[idx];
	frame[idx] = make_float4(t.x + f.x * (1.0f - t.w), t.y + f.y * (1.0f - t.w), t.z + f.z * (1.0f - t.w),
	                         t.w + f.w * (1.0f - t.w));
	if (t.w > 0.2f) depth_buffer[idx] = hdepth[i];
}

__global__ void __launch_bounds__(256) k_accum_tonemap(uint32_t W, uint32_t H, const float4* __restrict__ frame,
                                                       float4* __restrict__ accum, float4* __restrict__ out,
                                                       float sample_count, int color_space, float exposure,
                                                       float4 bg, int output_srgb) {
	const uint32_t i = blockIdx.x * 256u + threadIdx.x;
	if (i >= W * H) return;
	float4 color = frame[i];
	float4 tmp = sample_count == 0.0f ? make_float4(0.f, 0.f, 0.f, 0.f) : accum[i];
	if (color_space == 1) {
		color.x = linear_to_srgb(color.x);
		color.y = linear_to_srgb(color.y);
		color.z = linear_to_srgb(color.z);
	}
	tmp.x = (tmp.x * sample_count + color.x) / (sample_count + 1.0f);
	tmp.y = (tmp.y * sample_count + color.y) / (sample_count + 1.0f);
	tmp.z = (tmp.z * sample_count + color.z) / (sample_count + 1.0f);
	tmp.w = (tmp.w * sample_count + color.w) / (sample_count + 1.0f);
	accum[i] = tmp;
	if (!out) return;
	out[i] = tonemap_pixel(tmp, color_space, exposure, bg, output_srgb);
}

static uint32_t rows_owned(uint32_t H, uint32_t idx, uint32_t count, uint32_t rows) {
	uint32_t n = 0;
	for (uint32_t y = 0; y < H; ++y)
		if ((y / rows) % count == idx) ++n;
	return n;
}

// The march schedule (ngp_tuning; results do not depend on it):
//  * lanes_target: the lane budget that picks lanes-per-ray in k_generate (4M);
//  * pass_sample_target: a pipeline's sample slots per pass (6M volumes, 3M surfaces; <= 16M: the MLP reads the
//    encodings through raw buffers with 32-bit byte offsets, 64 B/sample);
//  * first_pass_steps / max_steps_per_pass: the per-ray cap of the first pass doubles every pass
//    up to the maximum (surfaces 4 -> 24, volumes 8 -> 32).  A ray's slots past its termination are wasted encoder and MLP
//    work: most rays of a surface scene stop within a few samples of their first occupied one,
//    while rays through a volume need many, so short first passes and geometric growth keep the
//    waste and the pass count both low.  Inside the cap each ray's budget also follows its
//    transmittance and the opacity of its last sample (sample_budget).
static uint32_t lanes_target(const ngp_tuning& t) { return t.render_lanes ? t.render_lanes : 4u << 20; }
// A volume's rays (the model's last frame above VOLUME_SAMPLES_PER_RAY network samples per ray) start with 8:
// 13.69 vs 13.82 ms per fire frame; a surface scene's keep 4 (8: 2.19 vs 2.11 ms; profiles/r04_first_steps_ab.txt)
constexpr float VOLUME_SAMPLES_PER_RAY = 12.0f;
// A pipeline's sample slots per pass: 6 M for a volume (the model's last frame >= VOLUME_SAMPLES_PER_RAY samples per
// ray), 3 M for a surface scene -- 13.67 vs 13.81 ms per fire frame against 5 M (7 M 13.69), 2.67 vs 2.73 ms on the
// surface scene (4 M 2.71; profiles/r05_schedule_sweep.txt; round 3 had measured 5 M best for both)
static uint32_t pass_sample_target(const ngp_tuning& t, float last_spr) {
	const uint32_t def = last_spr >= VOLUME_SAMPLES_PER_RAY ? 6u << 20 : 3u << 20;
	return std::min<uint32_t>(t.render_pass_samples ? t.render_pass_samples : def, 16u << 20);
}
static uint32_t first_pass_steps(const ngp_tuning& t, float last_spr) {
	return t.render_first_steps ? t.render_first_steps : (last_spr >= VOLUME_SAMPLES_PER_RAY ? 8u : 4u);
}
// the per-ray cap of any pass: 32 for a volume, 24 for a surface scene (2.63 vs 2.66 ms per frame; 16: 2.69;
// profiles/r05_schedule_sweep.txt)
static uint32_t max_steps_per_pass(const ngp_tuning& t, float last_spr) {
	return t.render_max_steps ? t.render_max_steps : (last_spr >= VOLUME_SAMPLES_PER_RAY ? 32u : 24u);
}

// rows r < h_shard of a shard with (r / 8) % pipe_count == pipe_index
static uint32_t pipe_rows(uint32_t h_shard, uint32_t pipe_index, uint32_t pipe_count) {
	const uint32_t full = h_shard / 8u, rest = h_shard % 8u;
	uint32_t n = (full / pipe_count + (full % pipe_count > pipe_index ? 1u : 0u)) * 8u;
	if (rest && full % pipe_count == pipe_index) n += rest;
	return n;
}

// Ray pipelines per render (ngp_tuning.render_pipelines, 1 .. 4; default 2 for frames of >= 2^16
// rays).  The pipelines take interleaved 8-row blocks of the frame and run their passes on their
// own streams: one pipeline's latency-bound march kernels overlap another's encoder
// (texture-addresser bound) and MLP (matrix cores).  Every ray composites its own samples in
// order, so the image does not depend on the split.  A scene whose rays stop after a few samples
// (surfaces: the lego-shaped scene's frames carry ~4 network samples per ray) has little encoder
// and MLP work to overlap with: there one pipeline measured 2.7 % faster per 1080p frame against two
// (profiles/r04_mlp_tile_ab.txt), a ~45-sample volume 6 % slower, so the default follows the
// samples per ray of the model's last frame.
constexpr float ONE_PIPE_SAMPLES_PER_RAY = VOLUME_SAMPLES_PER_RAY;
static uint32_t render_pipes(const ngp_tuning& t, uint32_t n, uint32_t h_shard, float last_spr) {
	uint32_t p = n >= (1u << 16) && !(last_spr > 0.0f && last_spr < ONE_PIPE_SAMPLES_PER_RAY) ? 2u : 1u;
	if (t.render_pipelines) p = std::min<uint32_t>(t.render_pipelines, RenderScratch::MAX_PIPES);
	return std::max(1u, std::min(p, div_up(h_shard, 8u)));  // every pipeline gets rows
}

// Pinned host-counter words of a pipeline: per-pass unpacked counters in HC_SLOTS slots (the
// read-back lag, ngp_tuning.render_lag, is at most HC_SLOTS passes), a copy-back slot, and the words the
// kernels publish.
constexpr uint32_t HC_SLOTS = 4, HC_COPYBACK = 16 * HC_SLOTS, HC_PUBLISHED = 128, HC_WORDS = HC_PUBLISHED + 16 * HC_SLOTS;

// passes a pipeline runs ahead of its counter read-backs (ngp_tuning.render_lag, 2 .. HC_SLOTS)
static uint32_t render_lag(const ngp_tuning& t) {
	// 2: 13.58 vs 13.66 ms per fire frame against 3, 2.60 vs 2.66 on the surface scene (round 5's schedule; round 3 had
	// measured 3 0.6 % faster; profiles/r05_schedule_sweep.txt)
	return t.render_lag >= 2 ? std::min<uint32_t>(t.render_lag, HC_SLOTS) : 2u;
}

namespace {
// One pipeline's march state (NerfTracer::trace, testbed_nerf.cu:1639-1755, for its rays).
struct PipeRun {
	RenderK k{};
	RenderPipeScratch* ps = nullptr;
	hipStream_t s = nullptr;
	uint32_t n = 0, n_tiled = 0;
	size_t max_samples = 0;
	int cur = 0;
	uint32_t pass = 0, steps_done = 0, n_alive_ub = 0, base_tag = 0;
	bool marching = false;
	float4* posdt = nullptr;
	uint32_t* sray = nullptr;
	uint4* shrows = nullptr;
	Payload* P(int b) const { return reinterpret_cast<Payload*>(ps->payload[b].ptr); }
	float4* C(int b) const { return reinterpret_cast<float4*>(ps->rgba[b].ptr); }
	uint32_t* hc() const { return ps->host_counter.ptr; }
	unsigned long long* pub_dev() const { return reinterpret_cast<unsigned long long*>(ps->host_counter_dev + HC_PUBLISHED); }
};
}  // namespace

// pass p's counters, published (k_generate of pass p + 1, or k_publish) as (tag << 32 | value)
// words with tag base_tag + p + 1; unpacked into hc[16 * (p % 2) ...]
static const uint32_t* wait_slot(PipeRun& pr, uint32_t pass) {
	volatile unsigned long long* w = reinterpret_cast<volatile unsigned long long*>(pr.hc() + HC_PUBLISHED) + 8 * (pass % HC_SLOTS);
	const uint32_t want = pr.base_tag + pass + 1;
	uint32_t* out = pr.hc() + 16 * (pass % HC_SLOTS);
	// no stream queries while spinning (each one enqueues a marker that drains the queue);
	// only after seconds without the tag is the stream asked whether it failed
	const auto t0 = std::chrono::steady_clock::now();
	for (uint32_t q = 0, spin = 1; q < 8; ++spin) {
		const unsigned long long v = w[q];
		if ((uint32_t)(v >> 32) == want) {
			out[q++] = (uint32_t)v;
			continue;
		}
		if ((spin & 65535u) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(5)) {
			const hipError_t e = hipStreamQuery(pr.s);
			if (e != hipSuccess && e != hipErrorNotReady) NGP_HIP_CHECK(e);
			if (e == hipSuccess && (uint32_t)(w[q] >> 32) != want) throw std::runtime_error("render: pass counters were not published");
		}
	}
	return out;
}

void run_render(ngp_model* m, const ngp_render_args* a, float* frame, float* depth_buffer, hipStream_t s) {
	RenderScratch& rs = m->rs;
	RenderK k{};
	k.W = a->width;
	k.H = a->height;
	k.sample_index = a->sample_index;
	for (int c = 0; c < 4; ++c) k.cam.c[c] = mk3(a->camera[3 * c], a->camera[3 * c + 1], a->camera[3 * c + 2]);
	k.fx = a->focal_length[0];
	k.fy = a->focal_length[1];
	k.scx = a->screen_center[0];
	k.scy = a->screen_center[1];
	k.near_distance = a->near_distance;
	{
		aabb3 box;
		box.min = mk3(a->aabb_min[0], a->aabb_min[1], a->aabb_min[2]);
		box.max = mk3(a->aabb_max[0], a->aabb_max[1], a->aabb_max[2]);
		k.aabb = make_render_box(box, a->render_aabb_to_local);
	}
	if (a->render_mode < NGP_RENDER_MODE_SHADE || a->render_mode > NGP_RENDER_MODE_SLICE)
		throw std::invalid_argument("render_mode must be one of NGP_RENDER_MODE_* (Distortion / EncodingVis are not supported)");
	k.mode = a->render_mode;
	k.prio = (m->tuning.render_priority >> 4) & 3u;
	if (a->host_frame) {
		if (a->render_mode != NGP_RENDER_MODE_SHADE || a->glow_mode || a->shard_count > 1 || a->sample_index != 0 ||
		    !a->host_frame_complete)
			throw std::invalid_argument("host_frame needs one spp of a Shade-mode unsharded frame without glow, and host_frame_complete");
		void* dp = nullptr;
		NGP_HIP_CHECK(hipHostGetDevicePointer(&dp, a->host_frame, 0));
		k.hframe = reinterpret_cast<float4*>(dp);
		k.hbg = make_float4(a->host_background[0], a->host_background[1], a->host_background[2], a->host_background[3]);
		k.hexposure = a->host_exposure;
		k.hcolor_space = a->host_color_space;
		k.hsrgb = a->host_output_srgb;
		rs.hmask.reserve((size_t)k.W * k.H);
		k.hmask = rs.hmask.ptr;
		*a->host_frame_complete = 1;
	}
	k.depth_scale = a->depth_scale;
	k.hard_edges = a->gbuffer_hard_edges;
	k.aperture = k.mode == NGP_RENDER_MODE_SLICE ? 0.0f : a->aperture_size;  // init_rays_with_payload_kernel_nerf:1427-1429
	k.glow_mode = a->glow_mode;
	k.glow_y_cutoff = a->glow_y_cutoff;
	k.focus_z = a->focus_z;
	if (k.aperture != 0.0f && !(k.focus_z > 0.0f)) throw std::invalid_argument("depth of field needs focus_z > 0");
	k.train_aabb.min = mk3(a->train_aabb_min[0], a->train_aabb_min[1], a->train_aabb_min[2]);
	k.train_aabb.max = mk3(a->train_aabb_max[0], a->train_aabb_max[1], a->train_aabb_max[2]);
	k.st = make_stepping(a->cone_angle_constant);
	k.max_mip = a->max_cascade;
	k.min_transmittance = a->min_transmittance;
	k.snap = a->snap_to_pixel_centers;
	k.linear_colors = a->train_in_linear_colors;
	k.rgb_act = m->cfg.rgb_activation;
	k.density_act = m->cfg.density_activation;
	k.lens_mode = a->lens_mode;
	for (int q = 0; q < 7; ++q) k.lens_params[q] = a->lens_params[q];
	for (int c = 0; c < 4; ++c) k.cam_end.c[c] = mk3(a->camera_end[3 * c], a->camera_end[3 * c + 1], a->camera_end[3 * c + 2]);
	for (int q = 0; q < 4; ++q) {
		k.rs[q] = a->rolling_shutter[q];
		k.rs_on |= a->rolling_shutter[q] != 0.0f;
	}
	if (a->distortion_map && a->distortion_res[0] && a->distortion_res[1]) {
		k.dmap = a->distortion_map;
		k.drx = a->distortion_res[0];
		k.dry = a->distortion_res[1];
	}
	k.shard_count = std::max(a->shard_count, 1u);
	k.shard_index = a->shard_index % k.shard_count;
	k.shard_rows = std::max(a->shard_rows, 1u);
	k.tiles_x = div_up(k.W, 8u);
	if (k.mode != NGP_RENDER_MODE_SLICE && (k.lens_mode == LENS_OPENCV || k.lens_mode == LENS_OPENCV_FISHEYE)) {
		// the per-pixel undistortion cache (RenderK::lens_xy): valid while every input of lens_direction and the
		// pixel jitter are the ones it was filled with; the shard geometry decides which rows were filled
		const float key[] = {(float)k.W, (float)k.H, k.fx, k.fy, k.scx, k.scy, (float)k.lens_mode, k.lens_params[0],
		                     k.lens_params[1], k.lens_params[2], k.lens_params[3], k.lens_params[4], k.lens_params[5],
		                     k.lens_params[6], (float)(k.snap ? 0u : k.sample_index), (float)k.shard_index,
		                     (float)k.shard_count, (float)k.shard_rows};
		const std::vector<float> kv(key, key + sizeof(key) / sizeof(key[0]));
		rs.lens_xy.reserve((size_t)k.W * k.H);
		k.lens_xy = rs.lens_xy.ptr;
		k.lens_fill = std::memcmp(kv.data(), rs.lens_key.data(), std::min(kv.size(), rs.lens_key.size()) * sizeof(float)) != 0 ||
		              kv.size() != rs.lens_key.size() || rs.lens_xy_filled != rs.lens_xy.ptr;
		rs.lens_key = kv;
		rs.lens_xy_filled = rs.lens_xy.ptr;
	}
	const uint32_t H_shard = rows_owned(k.H, k.shard_index, k.shard_count, k.shard_rows);
	if (k.W * H_shard == 0) return;
	if (!m->gs.bitfield.ptr) throw std::runtime_error("render: density grid bitfield not initialised");
	if (k.mode == NGP_RENDER_MODE_SLICE) {
		const uint32_t n = k.W * H_shard;
		rs.slice_coords.reserve(8 * (size_t)n);
		rs.slice_enc.reserve((size_t)m->lt.n_levels * n * m->lt.F);
		rs.slice_out.reserve(4 * (size_t)n);
		(k.lens_mode != LENS_PERSPECTIVE || k.dmap ? k_slice_init<true> : k_slice_init<false>)<<<div_up(n, 256u), 256, 0, s>>>(
		    k, n, rs.slice_coords.ptr, reinterpret_cast<float4*>(frame), depth_buffer);
		const __half* tab = (a->use_inference_params ? m->infer16.ptr : m->params16.ptr) + m->n_mlp_params;
		const __half* fr = a->use_inference_params ? m->frag_infer.ptr : m->frag_train.ptr;
		launch_hashgrid_fwd(m->lt, rs.slice_coords.ptr, 8, n, tab, rs.slice_enc.ptr, internal_layout(m, n), s);
		launch_mlp_infer(m, fr, rs.slice_enc.ptr, internal_layout(m, n), rs.slice_coords.ptr, 8, n, rs.slice_out.ptr, s, nullptr,
		                 4, nullptr, 0, 4, nullptr, 0, false, MlpExtra{a->extra_dims, nullptr, nullptr});
		k_slice_shade<<<div_up(n, 256u), 256, 0, s>>>(k, n, rs.slice_coords.ptr, rs.slice_out.ptr, reinterpret_cast<float4*>(frame));
		NGP_HIP_CHECK(hipGetLastError());
		return;
	}
	const ngp_tuning& tu = m->tuning;
	const uint32_t n_pipes = render_pipes(tu, k.W * H_shard, H_shard, rs.last_samples_per_ray);
	// render-MLP wave steps (ngp_tuning.render_mlp_tile 0): 64 samples while another pipeline's encoder shares
	// the CUs (194 VGPRs: 2 waves per SIMD leave it room), 32 with one pipeline (110 VGPRs, 4 waves per SIMD)
	rs.mlp_tile = n_pipes > 1 ? 4u : 2u;

	const uint32_t target = pass_sample_target(tu, rs.last_samples_per_ray), cap = max_steps_per_pass(tu, rs.last_samples_per_ray), cap0 = std::min(first_pass_steps(tu, rs.last_samples_per_ray), cap);
	const bool debug = (tu.debug & 1u) != 0;
	// per-ray sample budgets: headroom factor (default 1.0: measured 1 % faster than 1.5), < 0 = off
	k.budget = !(tu.render_budget_scale < 0.0f);
	k.budget_scale = tu.render_budget_scale > 0.0f ? tu.render_budget_scale : 1.0f;
	// per-pass budgets capped by the lattice points left to the ray's exit (ngp_tuning.render_exit_cap: 1 on, 2 off; off
	// by default since round 5's schedule: with read-back lag 2, 13.51 vs 13.58 ms per fire frame, 2.597 vs 2.603 surface)
	k.exit_cap = tu.render_exit_cap == 1 ? 1 : 0;
	// unfilled slots marked for the render MLP to skip (ngp_tuning.render_skip_unfilled: 1 on, 2 off; 0 the
	// default); Normals runs the MLP backward over every slot, so it keeps real rows
	const bool skip_unfilled = tu.render_skip_unfilled != 2 && k.mode != NGP_RENDER_MODE_NORMALS;
	k.mark_unfilled = skip_unfilled ? 1 : 0;

	if (!rs.fork) NGP_HIP_CHECK(hipEventCreateWithFlags(&rs.fork, hipEventDisableTiming));
	for (uint32_t j = 1; j < n_pipes; ++j) {
		if (rs.streams[j]) continue;
		NGP_HIP_CHECK(hipStreamCreateWithFlags(&rs.streams[j], hipStreamNonBlocking));
		NGP_HIP_CHECK(hipEventCreateWithFlags(&rs.join[j], hipEventDisableTiming));
	}
	// one SH row (16 fp16) per pixel of the frame, written by k_render_init for its alive rays
	const uint32_t sh_rows = k.W * k.H;
	rs.shrows.reserve(2 * (size_t)sh_rows);
	PipeRun pipes[RenderScratch::MAX_PIPES];
	for (uint32_t j = 0; j < n_pipes; ++j) {
		PipeRun& pr = pipes[j];
		pr.k = k;
		pr.k.pipe_index = j;
		pr.k.pipe_count = n_pipes;
		pr.k.h_local = pipe_rows(H_shard, j, n_pipes);
		pr.k.n_local = pr.n = k.W * pr.k.h_local;
		pr.n_tiled = k.tiles_x * 8u * div_up(pr.k.h_local, 8u) * 8u;
		pr.ps = &rs.pipe[j];
		pr.s = j == 0 ? s : rs.streams[j];
		RenderPipeScratch& ps = *pr.ps;
		// the most slots one pass can reserve (see `bound` below): small frames stay small
		pr.max_samples = (std::min<size_t>((size_t)pr.n * cap, std::max<size_t>((size_t)pr.n, (size_t)target)) + 256 + 63) & ~(size_t)63;
		for (int b = 0; b < 3; ++b) {
			ps.payload[b].reserve((size_t)pr.n * 12);
			ps.rgba[b].reserve((size_t)pr.n * 4);
			ps.depth[b].reserve(pr.n);
		}
		// [0, 4 max): position + warped dt rows, [4 max, 5 max): the samples' SH rows (pixel indices)
		ps.coords.reserve(6 * pr.max_samples);  // rows [4 max] | SH rows [max] | dt [max]
		ps.enc.reserve((size_t)m->lt.n_levels * pr.max_samples * m->lt.F);
		ps.out.reserve(4 * pr.max_samples);
		ps.counters.reserve(16);  // [0, 8) the pass counters, [8, 16) debug (pipeline 0)
		if (!ps.host_counter.ptr) {
			// [HC_SLOTS][16] unpacked pass counters, [HC_COPYBACK, +8) copy-back slot,
			// [HC_PUBLISHED, +HC_SLOTS * 16) the published words ([slot][8] x (tag << 32 | value));
			// fine-grained (coherent) so the kernel's system-scope stores reach the polling host
			NGP_HIP_CHECK(hipHostMalloc((void**)&ps.host_counter.ptr, HC_WORDS * sizeof(uint32_t), hipHostMallocCoherent | hipHostMallocMapped));
			std::memset(ps.host_counter.ptr, 0, HC_WORDS * sizeof(uint32_t));
			ps.host_counter.n = HC_WORDS;
			NGP_HIP_CHECK(hipHostGetDevicePointer((void**)&ps.host_counter_dev, ps.host_counter.ptr, 0));
		}
		if (!ps.events[0]) {
			for (auto& e : ps.events) NGP_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
		}
		pr.posdt = reinterpret_cast<float4*>(ps.coords.ptr);  // the encoder reads 16-B position rows once per level
		pr.sray = reinterpret_cast<uint32_t*>(ps.coords.ptr + 4 * pr.max_samples);
		// volumes (the last frame >= VOLUME_SAMPLES_PER_RAY samples per ray): each slot's warped dt also goes to its
		// own array, so k_composite fetches 4 B per sample instead of sharing the 16-B row's line -- 13.33 vs
		// 13.66 ms per fire frame; a surface scene's few samples per ray do not repay the extra store (2.12 vs
		// 2.07 ms), profiles/r04_dt_array_ab.txt
		pr.k.sdt = rs.last_samples_per_ray >= VOLUME_SAMPLES_PER_RAY ? ps.coords.ptr + 5 * pr.max_samples : nullptr;
		pr.shrows = rs.shrows.ptr;
		pr.base_tag = ps.pass_tag;
		pr.n_alive_ub = pr.n;
	}

	KernelTimers& tm = m->timers;
	tm.begin(NGP_TIMER_RENDER_MARCH, s);
	uint32_t* dbg = debug ? rs.pipe[0].counters.ptr + 8 : nullptr;
	if (debug) NGP_HIP_CHECK(hipMemsetAsync(dbg, 0, 8 * sizeof(uint32_t), s));
	build_distance_fields(m, k.max_mip, s);
	k.df = rs.df.ptr;
	NGP_HIP_CHECK(hipMemsetAsync(rs.pipe[0].counters.ptr, 0, 8 * sizeof(uint32_t), s));

	// the encoder's table, and corner records of its dense levels (read by every pipeline)
	const __half* table = (a->use_inference_params ? m->infer16.ptr : m->params16.ptr) + m->n_mlp_params;
	const __half* frags = a->use_inference_params ? m->frag_infer.ptr : m->frag_train.ptr;
	LevelTable lt_render = build_dense_records(m, table, s);
	lt_render.prio = tu.render_priority & 3u;
	// joins the pipeline streams back to s, also when a throw leaves this function early (work the
	// caller enqueues on s next shares the frame, dense records and scratch with them)
	struct StreamJoin {
		RenderScratch& rs;
		hipStream_t s;
		uint32_t n = 1;
		void join() {
			for (uint32_t j = 1; j < n; ++j) {
				NGP_HIP_CHECK(hipEventRecord(rs.join[j], rs.streams[j]));
				NGP_HIP_CHECK(hipStreamWaitEvent(s, rs.join[j], 0));
			}
			n = 1;
		}
		~StreamJoin() {
			for (uint32_t j = 1; j < n; ++j) {
				if (hipEventRecord(rs.join[j], rs.streams[j]) == hipSuccess) (void)hipStreamWaitEvent(s, rs.join[j], 0);
				else (void)hipStreamSynchronize(rs.streams[j]);
			}
		}
	} joiner{rs, s};
	if (n_pipes > 1) {
		for (uint32_t j = 1; j < n_pipes; ++j) NGP_HIP_CHECK(hipMemsetAsync(rs.pipe[j].counters.ptr, 0, 8 * sizeof(uint32_t), s));
		NGP_HIP_CHECK(hipEventRecord(rs.fork, s));
		for (uint32_t j = 1; j < n_pipes; ++j) {
			NGP_HIP_CHECK(hipStreamWaitEvent(rs.streams[j], rs.fork, 0));
			joiner.n = j + 1;
		}
	}
	for (uint32_t j = 0; j < n_pipes; ++j) {
		PipeRun& pr = pipes[j];
		pr.k.df = k.df;
		pr.k.dbg = dbg;
		if (pr.n == 0) continue;
		(k.lens_mode != LENS_PERSPECTIVE || k.dmap ? k_render_init<true> : k_render_init<false>)<<<div_up(pr.n_tiled, 256u), 256, 0, pr.s>>>(
		    pr.k, pr.P(0), pr.C(0), pr.ps->depth[0].ptr, reinterpret_cast<float4*>(frame), depth_buffer,
		    pr.ps->counters.ptr, rs.shrows.ptr);
		pr.marching = true;
	}
	tm.end(NGP_TIMER_RENDER_MARCH, s, k.W * H_shard);
	NGP_HIP_CHECK(hipGetLastError());
	if (k.hframe) {
		// the background pixels stream to the host beside the passes, once every pipeline's init has run
		if (!rs.host_stream) {
			NGP_HIP_CHECK(hipStreamCreateWithFlags(&rs.host_stream, hipStreamNonBlocking));
			NGP_HIP_CHECK(hipEventCreateWithFlags(&rs.host_join, hipEventDisableTiming));
		}
		for (uint32_t j = 0; j < n_pipes; ++j) {
			if (!rs.host_ev[j]) NGP_HIP_CHECK(hipEventCreateWithFlags(&rs.host_ev[j], hipEventDisableTiming));
			NGP_HIP_CHECK(hipEventRecord(rs.host_ev[j], pipes[j].s));
			NGP_HIP_CHECK(hipStreamWaitEvent(rs.host_stream, rs.host_ev[j], 0));
		}
		k_host_background<<<128, 256, 0, rs.host_stream>>>(k, k.W * k.H);
		NGP_HIP_CHECK(hipGetLastError());
		NGP_HIP_CHECK(hipEventRecord(rs.host_join, rs.host_stream));
	}

	// NerfTracer::trace (testbed_nerf.cu:1639-1755): generate -> infer -> composite(+compact),
	// alive rays ping-pong between buffers 0/1, finished rays with colour append to buffer 2.
	// Counters (device): [0]/[1] alive rays in/out, [2] finished rays, [3] filled samples,
	// [4]/[5] sample slots, [6]/[7] samples per ray of the pass.  The host does not wait for a
	// pass before enqueuing the next: kernels read the counts from the device, and launches
	// are sized by the latest count read back (lag passes behind; alive counts only shrink).  A
	// pipeline stops once a read-back shows no alive rays (the pass enqueued meanwhile runs
	// empty).  With two pipelines the host alternates between them, so each stream holds up
	// to two enqueued passes while the host waits on the other's read-back.
	// ngp_tuning.debug bit 4: a 40-step march budget (exercises the retire path of rays that run out of it)
	const uint32_t MARCH_ITER = (tu.debug & 16u) ? 40u : 10000u;
	const uint32_t lag = render_lag(tu);
	// workgroup sizes: k_composite 512 (measured 0.5 % faster than 1024, 256 2 % slower), k_generate
	// 512 (256 measured 4.5 % slower)
	const uint32_t comp_block = tu.render_composite_block ? tu.render_composite_block : 512u;
	const uint32_t gen_block = tu.render_generate_block ? tu.render_generate_block : 512u;
	auto enqueue_pass = [&](PipeRun& pr) {
		const hipStream_t ps = pr.s;
		uint32_t* counters = pr.ps->counters.ptr;
		const uint32_t pass = pr.pass;
		const int cur = pr.cur;
		tm.begin(NGP_TIMER_RENDER_MARCH, ps);
		uint32_t* alive_in = counters + pass % 2;
		uint32_t* alive_out = counters + (pass + 1) % 2;
		uint32_t* samples = counters + 4 + pass % 2;  // zeroed by the previous kernel of the chain
		uint32_t* samples_next = counters + 4 + (pass + 1) % 2;
		uint32_t* steps_out = counters + 6 + pass % 2;
		// lanes per ray: enough rays in flight for ~1M lanes, never fewer than one lane per ray
		const uint32_t want = lanes_target(tu) / std::max(pr.n_alive_ub, 1u);
		const uint32_t G = want >= 64 ? 64u : want >= 16 ? 16u : want >= 4 ? 4u : 1u;
		const uint32_t gblocks = std::max(1u, div_up((uint64_t)pr.n_alive_ub * G, gen_block));
		unsigned long long* host_prev = pass > 0 ? pr.pub_dev() + 8 * ((pass - 1) % HC_SLOTS) : nullptr;
		const uint32_t tag_prev = pr.base_tag + pass;  // = tag of pass - 1
		const uint32_t cap_p = pass >= 8 ? cap : std::min(cap, cap0 << pass);
#define NGP_GEN(GG) k_generate<GG><<<gblocks, gen_block, 0, ps>>>(pr.k, alive_in, pr.P(cur), pr.C(cur), pr.posdt, pr.sray, target, cap_p, alive_out, samples, steps_out, counters, host_prev, tag_prev)
		switch (G) {
			case 1: NGP_GEN(1); break;
			case 4: NGP_GEN(4); break;
			case 16: NGP_GEN(16); break;
			default: NGP_GEN(64); break;
		}
#undef NGP_GEN
		tm.end(NGP_TIMER_RENDER_MARCH, ps);
		// sized for the most samples the pass can reserve; the kernels read the actual total
		const uint64_t bound = std::min<uint64_t>((uint64_t)pr.n_alive_ub * cap_p, std::max(target, pr.n_alive_ub));
		const uint32_t n_elements = next_multiple((uint32_t)std::max<uint64_t>(bound, 1), BATCH_SIZE_GRANULARITY);
		tm.begin_kernel(NGP_TIMER_RENDER_ENCODE);
		launch_hashgrid_fwd(lt_render, reinterpret_cast<const float*>(pr.posdt), 4, n_elements, table, pr.ps->enc.ptr,
		                    internal_layout(m, n_elements), ps, samples, 1);
		tm.end(NGP_TIMER_RENDER_ENCODE, ps);  // units: the pass's sample count, added at its read-back
		tm.begin_kernel(NGP_TIMER_RENDER_MLP);
		launch_mlp_infer(m, frags, pr.ps->enc.ptr, internal_layout(m, n_elements), nullptr, 0, n_elements, pr.ps->out.ptr, ps,
		                 samples, 0, reinterpret_cast<const __half*>(pr.shrows), 0, 4, pr.sray, sh_rows, skip_unfilled,
		                 MlpExtra{a->extra_dims, nullptr, nullptr});
		tm.end(NGP_TIMER_RENDER_MLP, ps);
		if (pr.k.mode == NGP_RENDER_MODE_NORMALS) {
			// Normals (NerfTracer::trace, testbed_nerf.cu:1715-1717, network->input_gradient): the gradient of
			// the raw density w.r.t. the warped position of every sample -- the fused MLP backward from
			// dL/dout = (0, 0, 0, 1) without weight gradients (the rgb rows are zero, so the direction does not
			// enter), then the grid's input gradient
			RenderPipeScratch& sc = *pr.ps;
			sc.nrm_dloss.reserve(4 * (size_t)n_elements);
			sc.nrm_denc.reserve((size_t)m->lt.n_levels * n_elements * m->lt.F);
			sc.nrm.reserve(3 * (size_t)n_elements);
			k_density_unit_dloss<<<div_up(n_elements, 256u), 256, 0, ps>>>(samples, n_elements, sc.nrm_dloss.ptr);
			launch_mlp_train(m, frags, pr.ps->enc.ptr, internal_layout(m, n_elements), nullptr, 0, n_elements, sc.nrm_dloss.ptr,
			                 nullptr, nullptr, sc.nrm_denc.ptr, ps, samples, nullptr, MlpExtra{a->extra_dims, nullptr, nullptr});
			launch_hashgrid_input_grad(m->lt, reinterpret_cast<const float*>(pr.posdt), 4, n_elements, sc.nrm_denc.ptr,
			                           EncLayout{n_elements, 0}, table, nullptr, sc.nrm.ptr, ps, samples);
			pr.k.normals = sc.nrm.ptr;
		}
		tm.begin(NGP_TIMER_RENDER_MARCH, ps);
		if (pr.k.mode == NGP_RENDER_MODE_SHADE && !pr.k.glow_mode)
			k_composite<false><<<std::max(1u, div_up(pr.n_alive_ub, comp_block)), comp_block, 0, ps>>>(
			    pr.k, alive_in, pr.P(cur), pr.C(cur), pr.ps->depth[cur].ptr, pr.posdt, pr.ps->out.ptr, pr.P(1 - cur), pr.C(1 - cur),
			    pr.ps->depth[1 - cur].ptr, pr.P(2), pr.C(2), pr.ps->depth[2].ptr, alive_out, counters + 2, samples_next, counters + 3);
		else
			k_composite<true><<<std::max(1u, div_up(pr.n_alive_ub, comp_block)), comp_block, 0, ps>>>(
			    pr.k, alive_in, pr.P(cur), pr.C(cur), pr.ps->depth[cur].ptr, pr.posdt, pr.ps->out.ptr, pr.P(1 - cur), pr.C(1 - cur),
			    pr.ps->depth[1 - cur].ptr, pr.P(2), pr.C(2), pr.ps->depth[2].ptr, alive_out, counters + 2, samples_next, counters + 3);
		tm.end(NGP_TIMER_RENDER_MARCH, ps);
		NGP_HIP_CHECK(hipGetLastError());
		pr.cur = 1 - cur;
		++pr.pass;
		// the read-back of the previous pass bounds the next one
		if (pr.pass >= lag) {
			const uint32_t q = pr.pass - lag;  // its counters: alive out (the input of pass q + 1, a bound on every later one)
			const uint32_t* c = wait_slot(pr, q);
			pr.steps_done += c[6 + q % 2];
			pr.n_alive_ub = std::min(pr.n_alive_ub, c[(q + 1) % 2]);
			if (pr.n_alive_ub == 0 || pr.steps_done >= MARCH_ITER) pr.marching = false;
		}
	};
	for (bool any = true; any;) {
		any = false;
		for (uint32_t j = 0; j < n_pipes; ++j) {
			if (!pipes[j].marching) continue;
			enqueue_pass(pipes[j]);
			any |= pipes[j].marching;
		}
	}

	uint64_t filled_total = 0;
	for (uint32_t j = 0; j < n_pipes; ++j) {
		PipeRun& pr = pipes[j];
		if (pr.pass == 0) continue;  // no rays
		uint32_t* counters = pr.ps->counters.ptr;
		k_publish<<<1, 64, 0, pr.s>>>(counters, pr.pub_dev() + 8 * ((pr.pass - 1) % HC_SLOTS), pr.base_tag + pr.pass);
		NGP_HIP_CHECK(hipGetLastError());
		const uint32_t* last = wait_slot(pr, pr.pass - 1);
		const uint32_t n_alive = last[pr.pass % 2];
		uint32_t n_hit = last[2];
		// [3]: filled samples of the pipeline's rays (the encoder / MLP skip the unfilled slots' work)
		tm.add_units(NGP_TIMER_RENDER_ENCODE, last[3]);
		tm.add_units(NGP_TIMER_RENDER_MLP, last[3]);
		filled_total += last[3];
		if (n_alive > 0) {
			if (a->host_frame) *a->host_frame_complete = 0;  // their pixels were not streamed: the caller copies the frame
			auto wait_copy = [&](void* dst, const void* src, size_t bytes) {
				NGP_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, pr.s));
				NGP_HIP_CHECK(hipEventRecord(pr.ps->events[0], pr.s));
				hipError_t e;
				while ((e = hipEventQuery(pr.ps->events[0])) == hipErrorNotReady) {
				}
				NGP_HIP_CHECK(e);
			};
			// march budget exhausted: still-alive rays are shaded with what they accumulated
			k_retire<<<div_up(n_alive, 256), 256, 0, pr.s>>>(n_alive, pr.P(pr.cur), pr.C(pr.cur), pr.ps->depth[pr.cur].ptr,
			                                                 pr.P(2), pr.C(2), pr.ps->depth[2].ptr, counters);
			// copy-back of the counters -> slot [HC_COPYBACK, +8), then an event
			wait_copy(pr.hc() + HC_COPYBACK, counters, 8 * sizeof(uint32_t));
			n_hit = pr.hc()[HC_COPYBACK + 2];
		}
		pr.ps->pass_tag = pr.base_tag + pr.pass;
		if (n_hit)
			k_shade<<<div_up(n_hit, 256), 256, 0, pr.s>>>(pr.k, n_hit, pr.P(2), pr.C(2), pr.ps->depth[2].ptr, k.linear_colors,
			                                              reinterpret_cast<float4*>(frame), depth_buffer);
		NGP_HIP_CHECK(hipGetLastError());
	}
	joiner.join();
	if (k.hframe) NGP_HIP_CHECK(hipStreamWaitEvent(s, rs.host_join, 0));
	// the next frame's default pipeline count (render_pipes) follows this one's samples per ray
	if (k.mode == NGP_RENDER_MODE_SHADE && k.W * H_shard >= (1u << 16)) rs.last_samples_per_ray = (float)filled_total / (float)(k.W * H_shard);
	if (debug) {
		uint32_t d[8];
		NGP_HIP_CHECK(hipMemcpyAsync(d, dbg, sizeof(d), hipMemcpyDeviceToHost, s));
		wait_stream(m, s);
		const uint32_t n = k.W * H_shard;
		fprintf(stderr,
		        "[render] rays %u pipelines %u init: alive %u lattice steps %.2f/ray | passes %u (pipeline 0) generate iterations %u "
		        "slots %u samples %u composited %u (%.1f%% of slots)\n",
		        n, n_pipes, d[1], (double)d[0] / n, pipes[0].pass, d[2], d[5], d[3], d[4],
		        100.0 * d[4] / std::max(d[5], 1u));
	}
}

void run_accumulate_tonemap(const float* frame, float* accum, float* out, uint32_t W, uint32_t H, uint32_t spp,
                            int color_space, float exposure, const float* bg, int output_srgb, hipStream_t s) {
	const float4 b = bg ? make_float4(bg[0], bg[1], bg[2], bg[3]) : make_float4(0.f, 0.f, 0.f, 1.f);
	k_accum_tonemap<<<div_up((uint64_t)W * H, 256), 256, 0, s>>>(W, H, reinterpret_cast<const float4*>(frame),
	                                                             reinterpret_cast<float4*>(accum),
	                                                             reinterpret_cast<float4*>(out), (float)spp, color_space,
	                                                             exposure, b, output_srgb);
	NGP_HIP_CHECK(hipGetLastError());
}

}  // namespace ngp
