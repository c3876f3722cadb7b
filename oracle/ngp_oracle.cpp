// ngp_oracle.cpp — TEST INFRASTRUCTURE ONLY.
//
// Scalar CPU restatement of the Instant-NGP NeRF hot path of the reference
// (fnysalehi/instant-ngp-rendering).  Only tests/, __graft_entry__.smoke() and
// bench.py's cpu_baseline leg may load this library; the product path
// (libngp_hip.so) never calls it.
//
// Parity status: the reference cannot be compiled here (CUDA sources, no nvcc,
// empty tiny-cuda-nn submodule) and ships no tests or golden vectors, so the
// tcnn-side pieces (hash grid, SH, MLP, Adam/Ema) are restated from the public
// tiny-cuda-nn algorithm -> "parity unpinned" for those.
// The in-tree pieces (sampler, compositing/loss, occupancy grid, tracer) follow
// the cited reference lines; pcg32, Sobol and SH are pinned by published
// known-answer values in tests/test_oracle.py.
//
// Deliberate, documented deviations shared with the HIP path:
//  * sample/ray compaction is by exclusive prefix sum in ray-index order
//    instead of atomicAdd order (same cap rule, deterministic);
//  * hash-grid features and MLP products accumulate in fp32 (tcnn: fp16);
//  * the rollover copies of fill_rollover_and_rescale are folded into a
//    per-sample multiplicity weight (mathematically identical gradient);
//  * the occupancy mean is an exact 2^-24 fixed-point sum.
//
// Built by oracle/Makefile with g++ -O2 -ffp-contract=off (no fast-math).
#include <omp.h>
#include <thread>
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "../include/ngp_hip.h"

namespace oref {

// ---------------------------------------------------------------------------
// fp16 <-> fp32 (IEEE binary16, round to nearest even)
// ---------------------------------------------------------------------------
static float h2f(uint16_t h) {
	const uint32_t s = (uint32_t)(h >> 15) << 31, e = (h >> 10) & 0x1f, m = h & 0x3ff;
	uint32_t b;
	if (e == 0) {
		if (m == 0) b = s;
		else {  // subnormal
			float f = (float)m * (1.0f / 16777216.0f);
			std::memcpy(&b, &f, 4);
			b |= s;
		}
	} else if (e == 31) b = s | 0x7f800000u | (m << 13);
	else b = s | ((e + 112) << 23) | (m << 13);
	float f;
	std::memcpy(&f, &b, 4);
	return f;
}
static uint16_t f2h(float f) {
	uint32_t x;
	std::memcpy(&x, &f, 4);
	const uint32_t sign = (x >> 16) & 0x8000u;
	const uint32_t absx = x & 0x7fffffffu;
	if (absx >= 0x7f800000u) return (uint16_t)(sign | 0x7c00u | (absx > 0x7f800000u ? 0x200u : 0u));
	if (absx >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u);  // overflow -> inf (>= 65520)
	if (absx < 0x38800000u) {  // subnormal half or zero
		float af;
		std::memcpy(&af, &absx, 4);
		const float scaled = af * 16777216.0f;  // 2^24
		uint32_t q = (uint32_t)std::nearbyint(scaled);
		return (uint16_t)(sign | q);
	}
	uint32_t mant = absx & 0x7fffffu;
	uint32_t exp = (absx >> 23) - 112;
	uint32_t r = (exp << 10) | (mant >> 13);
	const uint32_t rem = mant & 0x1fffu;
	if (rem > 0x1000u || (rem == 0x1000u && (r & 1u))) ++r;
	return (uint16_t)(sign | r);
}
static float rh(float f) { return h2f(f2h(f)); }

// ---------------------------------------------------------------------------
// Small vector math (tcnn vec3 semantics, component-wise IEEE float)
// ---------------------------------------------------------------------------
struct V3 {
	float x, y, z;
};
static V3 v(float x, float y, float z) { return {x, y, z}; }
static V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
static V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static V3 operator*(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
static V3 operator+(V3 a, float s) { return {a.x + s, a.y + s, a.z + s}; }
static V3 operator-(V3 a, float s) { return {a.x - s, a.y - s, a.z - s}; }
static V3 operator/(V3 a, V3 b) { return {a.x / b.x, a.y / b.y, a.z / b.z}; }
static float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static float len(V3 a) { return std::sqrt(dot(a, a)); }
static V3 normalize(V3 a) { return a * (1.0f / len(a)); }

struct Box {
	V3 mn, mx;
	bool contains(V3 p) const { return p.x >= mn.x && p.x <= mx.x && p.y >= mn.y && p.y <= mx.y && p.z >= mn.z && p.z <= mx.z; }
	V3 rel(V3 p) const { return (p - mn) / (mx - mn); }
	// bounding_box.cuh:172-219
	void intersect(V3 o, V3 d, float* t0, float* t1) const {
		const float FMAX = 3.402823466e+38f;
		float tmin = (mn.x - o.x) / d.x, tmax = (mx.x - o.x) / d.x;
		if (tmin > tmax) std::swap(tmin, tmax);
		float tymin = (mn.y - o.y) / d.y, tymax = (mx.y - o.y) / d.y;
		if (tymin > tymax) std::swap(tymin, tymax);
		if (tmin > tymax || tymin > tmax) { *t0 = *t1 = FMAX; return; }
		if (tymin > tmin) tmin = tymin;
		if (tymax < tmax) tmax = tymax;
		float tzmin = (mn.z - o.z) / d.z, tzmax = (mx.z - o.z) / d.z;
		if (tzmin > tzmax) std::swap(tzmin, tzmax);
		if (tmin > tzmax || tzmin > tmax) { *t0 = *t1 = FMAX; return; }
		if (tzmin > tmin) tmin = tzmin;
		if (tzmax < tmax) tmax = tzmax;
		*t0 = tmin;
		*t1 = tmax;
	}
};

// The render crop box in its local frame: local = R * world (Testbed::m_render_aabb_to_local,
// nerf_device.cuh:475, src/testbed_nerf.cu:1467-1469); all-zero R = identity.
struct RBox {
	Box b;
	float R[9];
	bool rot = false;
	V3 local(V3 p) const {
		if (!rot) return p;
		return V3{R[0] * p.x + R[1] * p.y + R[2] * p.z, R[3] * p.x + R[4] * p.y + R[5] * p.z, R[6] * p.x + R[7] * p.y + R[8] * p.z};
	}
	bool contains(V3 p) const { return b.contains(local(p)); }
};
static RBox rbox_of(const Box& b, const float* R) {
	RBox r;
	r.b = b;
	bool any = false, ident = true;
	for (int k = 0; k < 9; ++k) {
		r.R[k] = R[k];
		any |= R[k] != 0.0f;
		ident &= R[k] == ((k % 4 == 0) ? 1.0f : 0.0f);
	}
	r.rot = any && !ident;
	return r;
}

// ---------------------------------------------------------------------------
// pcg32 (tcnn/pcg32.h; default_rng_t, random_val.cuh:26)
// ---------------------------------------------------------------------------
struct Pcg {
	uint64_t state = 0x853c49e6748fea9bULL, inc = 0xda3e39cb94b95bdbULL;
	void seed(uint64_t s, uint64_t q = 1) {
		state = 0;
		inc = (q << 1) | 1;
		next();
		state += s;
		next();
	}
	uint32_t next() {
		const uint64_t old = state;
		state = old * 0x5851f42d4c957f2dULL + inc;
		const uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
		const uint32_t rot = (uint32_t)(old >> 59u);
		return (xs >> rot) | (xs << ((-(int32_t)rot) & 31));
	}
	float nextf() {
		uint32_t u = (next() >> 9) | 0x3f800000u;
		float f;
		std::memcpy(&f, &u, 4);
		return f - 1.0f;
	}
	void advance(int64_t delta_ = (1ll << 32)) {
		uint64_t cm = 0x5851f42d4c957f2dULL, cp = inc, am = 1, ap = 0, delta = (uint64_t)delta_;
		while (delta > 0) {
			if (delta & 1) {
				am *= cm;
				ap = ap * cm + cp;
			}
			cp = (cm + 1) * cp;
			cm *= cm;
			delta /= 2;
		}
		state = am * state + ap;
	}
};

// ---------------------------------------------------------------------------
// Sobol / Laine-Karras (random_val.cuh:162-325): only dims 0 and 1.
// ---------------------------------------------------------------------------
static const uint32_t SOBOL_DIM1_FIRST8[8] = {0x80000000u, 0xc0000000u, 0xa0000000u, 0xf0000000u,
                                              0x88000000u, 0xcc000000u, 0xaa000000u, 0xff000000u};
static uint32_t sobol(uint32_t index, uint32_t dim) {
	uint32_t X = 0, dirn = 0x80000000u;
	for (uint32_t bit = 0; bit < 32; ++bit) {
		const uint32_t d = dim == 0 ? (0x80000000u >> bit) : dirn;
		if (bit < 8 && dim == 1 && d != SOBOL_DIM1_FIRST8[bit]) throw std::logic_error("sobol table");
		if ((index >> bit) & 1) X ^= d;
		dirn ^= dirn >> 1;
	}
	return X;
}
static uint32_t rev(uint32_t x) {
	uint32_t r = 0;
	for (int i = 0; i < 32; ++i) r |= ((x >> i) & 1u) << (31 - i);
	return r;
}
static uint32_t lk(uint32_t x, uint32_t seed) {
	x += seed;
	x ^= x * 0x6c50b47cu;
	x ^= x * 0xb82f1e52u;
	x ^= x * 0xc7afe638u;
	x ^= x * 0x8d22f6e6u;
	return x;
}
static uint32_t scramble(uint32_t x, uint32_t seed) { return rev(lk(rev(x), seed)); }
static uint32_t hcomb(uint32_t seed, uint32_t v) { return seed ^ (v + (seed << 6) + (seed >> 2)); }
static float ldval(uint32_t index, uint32_t seed, uint32_t dim) {
	index = scramble(index, seed);
	return (float)scramble(sobol(index, dim), hcomb(seed, dim)) * (float)(1.0 / 4294967296.0);
}
static float fract(float x) { return x - std::floor(x); }
static void pixel_offset(uint32_t spp, float* ox, float* oy) {
	*ox = fract(0.5f - ldval(0, 0xdeadbeefu, 0) + ldval(spp, 0xdeadbeefu, 0));
	*oy = fract(0.5f - ldval(0, 0xdeadbeefu, 1) + ldval(spp, 0xdeadbeefu, 1));
}

// ---------------------------------------------------------------------------
// Morton (tcnn morton3D)
// ---------------------------------------------------------------------------
static uint32_t morton(uint32_t x, uint32_t y, uint32_t z) {
	uint32_t r = 0;
	for (int b = 0; b < 10; ++b) r |= ((x >> b) & 1u) << (3 * b) | ((y >> b) & 1u) << (3 * b + 1) | ((z >> b) & 1u) << (3 * b + 2);
	return r;
}
static uint32_t morton_inv(uint32_t m) {
	uint32_t r = 0;
	for (int b = 0; b < 10; ++b) r |= ((m >> (3 * b)) & 1u) << b;
	return r;
}

// ---------------------------------------------------------------------------
// NeRF constants and stepping (nerf_device.cuh:24-42, 359-494)
// ---------------------------------------------------------------------------
static const uint32_t GRID = 128, CELLS = GRID * GRID * GRID, STEPS = 1024, CASCADES = 8;
static const float SQRT3_ = 1.73205080757f;
static const float MIN_STEP = SQRT3_ / 1024.0f;
static const float MAX_STEP = MIN_STEP * 128.0f * 1024.0f / 128.0f;
static const float MAXD = 16384.0f;

static float sgn(float x) { return x > 0 ? 1.0f : (x < 0 ? -1.0f : 0.0f); }
// Stepping lattice (see ngp_math.h "Stepping lattice"): samples sit at n0 + k in stepping
// space; constants of the log regime resolved once; divisions by constants are
// multiplies by the reciprocal (the reference builds with --use_fast_math).
static const float INV_MIN_STEP = 1.0f / MIN_STEP;
static const float INV_MAX_STEP = 1.0f / MAX_STEP;
struct Stepping {
	float cone, l, inv_l, a, b, at, bt;
};
static Stepping make_stepping(float cone) {
	Stepping s{cone, 0, 0, 0, 0, 0, 0};
	if (cone <= 1e-5f) return s;
	s.l = logf(1.0f + cone);
	s.inv_l = 1.0f / s.l;
	s.a = (logf(MIN_STEP) - logf(s.l)) * s.inv_l;
	s.b = (logf(MAX_STEP) - logf(s.l)) * s.inv_l;
	s.at = expf(s.a * s.l);
	s.bt = expf(s.b * s.l);
	return s;
}
static float lat_to(const Stepping& s, float t) {
	if (s.cone <= 1e-5f) return t * INV_MIN_STEP;
	if (t <= s.at) return (t - s.at) * INV_MIN_STEP + s.a;
	if (t <= s.bt) return logf(t) * s.inv_l;
	return (t - s.bt) * INV_MAX_STEP + s.b;
}
static float lat_from(const Stepping& s, float n) {
	if (s.cone <= 1e-5f) return n * MIN_STEP;
	if (n <= s.a) return (n - s.a) * MIN_STEP + s.at;
	if (n <= s.b) return expf(n * s.l);
	return (n - s.b) * MAX_STEP + s.bt;
}
static float dist_next_cell(V3 pos, V3 d, V3 idir, uint32_t mip) {
	const float res = std::scalbn((float)GRID, -(int)mip), inv_res = std::scalbn(1.0f / (float)GRID, (int)mip);
	const V3 p = (pos - v(0.5f, 0.5f, 0.5f)) * res;
	const float tx = (std::floor(p.x + 0.5f + 0.5f * sgn(d.x)) - p.x) * idir.x;
	const float ty = (std::floor(p.y + 0.5f + 0.5f * sgn(d.y)) - p.y) * idir.y;
	const float tz = (std::floor(p.z + 0.5f + 0.5f * sgn(d.z)) - p.z) * idir.z;
	return std::fmax(std::fmin(std::fmin(tx, ty), tz) * inv_res, 0.0f);
}
static uint32_t mip_pos(V3 p, uint32_t maxc = CASCADES - 1) {
	int e;
	std::frexp(std::max(std::max(std::fabs(p.x - 0.5f), std::fabs(p.y - 0.5f)), std::fabs(p.z - 0.5f)), &e);
	return (uint32_t)std::min(std::max(e + 1, 0), (int)maxc);
}
static uint32_t mip_dt(float dt, V3 p, uint32_t maxc) {
	const uint32_t mip = mip_pos(p, maxc);
	dt *= 2.0f * GRID;
	if (dt < 1.0f) return mip;
	int e;
	std::frexp(dt, &e);
	return (uint32_t)std::min(std::max((int)mip, e), (int)maxc);
}
static uint32_t grid_idx(V3 p, uint32_t mip) {
	const float s = std::scalbn(1.0f, -(int)mip);
	p = p - v(0.5f, 0.5f, 0.5f);
	p = p * s;
	p = p + v(0.5f, 0.5f, 0.5f);
	const int ix = (int)(p.x * (float)GRID), iy = (int)(p.y * (float)GRID), iz = (int)(p.z * (float)GRID);
	if (ix < 0 || ix >= (int)GRID || iy < 0 || iy >= (int)GRID || iz < 0 || iz >= (int)GRID) return 0xFFFFFFFFu;
	return morton((uint32_t)ix, (uint32_t)iy, (uint32_t)iz);
}
static bool occupied(V3 p, const uint8_t* bits, uint32_t mip) {
	const uint32_t i = grid_idx(p, mip);
	if (i == 0xFFFFFFFFu) return false;
	return bits[i / 8 + CELLS / 8 * mip] & (1u << (i % 8));
}
// First occupied lattice point at or after *n (render march, if_unoccupied_advance_to_next_occupied_voxel
// nerf_device.cuh:462-494 on the lattice): the cell at clamp(mip_from_pos, 0, maxm); an empty one is left
// past its far face at the coarsest empty mip (the reference's climb), the jump taken only when the
// lattice point before the landing point is still in the skipped cell (or already outside the box).
template <class B>
static bool next_occupied(float* n_io, const Stepping& st, V3 o, V3 d, V3 idir, const uint8_t* bits, uint32_t maxm, const B& b) {
	float n = *n_io;
	while (true) {
		const float t = lat_from(st, n);
		const V3 pos = o + d * t;
		if (t >= MAXD || !b.contains(pos)) { *n_io = n; return false; }
		uint32_t mip = std::min(mip_pos(pos), maxm);
		if (occupied(pos, bits, mip)) { *n_io = n; return true; }
		while (mip < maxm && !occupied(pos, bits, mip + 1)) ++mip;
		const uint32_t cell = grid_idx(pos, mip);
		const float n_far = lat_to(st, t + dist_next_cell(pos, d, idir, mip));
		float nn = n + std::ceil(std::max(n_far - n, 0.5f));
		if (nn - n > 1.0f) {
			const V3 last = o + d * lat_from(st, nn - 1.0f);
			if (b.contains(last) && grid_idx(last, mip) != cell) nn = n + 1.0f;
		}
		n = nn;
	}
}
static float warp_dt(float dt) { return (dt - MIN_STEP) / (MIN_STEP * 128.0f - MIN_STEP); }
static float unwarp_dt(float w) { return w * (MIN_STEP * 128.0f - MIN_STEP) + MIN_STEP; }

// ---------------------------------------------------------------------------
// Colour, activations, losses (common_device.cuh:34-80, nerf_device.cuh:74-263,600-615)
// ---------------------------------------------------------------------------
static float s2l(float s) { return s <= 0.04045f ? s / 12.92f : std::pow((s + 0.055f) / 1.055f, 2.4f); }
static float l2s(float l) { return l < 0.0031308f ? 12.92f * l : 1.055f * std::pow(l, 0.41666f) - 0.055f; }
static float logistic(float x) { return 1.0f / (1.0f + std::exp(-x)); }
static float to_rgb(float x, int a) {
	switch (a) {
		case 1: return x > 0 ? x : 0;
		case 2: return logistic(x);
		case 3: return std::exp(std::min(std::max(x, -10.0f), 10.0f));
		default: return x;
	}
}
static float to_rgb_d(float x, int a) {
	switch (a) {
		case 1: return x > 0 ? 1.0f : 0.0f;
		case 2: { const float d = logistic(x); return d * (1 - d); }
		case 3: return std::exp(std::min(std::max(x, -10.0f), 10.0f));
		default: return 1.0f;
	}
}
static float to_density(float x, int a) {
	switch (a) {
		case 1: return x > 0 ? x : 0;
		case 2: return logistic(x);
		case 3: return std::exp(x);
		default: return x;
	}
}
static float to_density_d(float x, int a) {
	switch (a) {
		case 1: return x > 0 ? 1.0f : 0.0f;
		case 2: { const float d = logistic(x); return d * (1 - d); }
		case 3: return std::exp(std::min(std::max(x, -15.0f), 15.0f));
		default: return 1.0f;
	}
}
static void lossg(float target, float pred, int type, float* l, float* g) {
	const float d = pred - target;
	switch (type) {
		case 6: { const float den = pred * pred + 1e-2f; *l = d * d / den; *g = 2 * d / den; } break;
		case 1: *l = std::fabs(d); *g = std::copysign(1.0f, d); break;
		case 2: { const float den = std::fabs(pred) + 1e-2f; *l = std::fabs(d) / den; *g = std::copysign(1.0f / den, d); } break;
		case 3: { const float den = 0.5f * (std::fabs(pred) + std::fabs(target)) + 1e-2f; *l = std::fabs(d) / den; *g = std::copysign(1.0f / den, d); } break;
		case 4: {
			const float ad = std::fabs(d), sq = 0.5f / 0.1f * d * d;
			*l = (ad > 0.1f ? ad - 0.05f : sq) / 5.0f;
			*g = (ad > 0.1f ? (d > 0 ? 1.0f : -1.0f) : d / 0.1f) / 5.0f;
		} break;
		case 5: { const float dv = std::fabs(d) + 1.0f; *l = std::log(dv); *g = std::copysign(1.0f / dv, d); } break;
		default: *l = d * d; *g = 2 * d; break;
	}
}

// ---------------------------------------------------------------------------
// Model
// ---------------------------------------------------------------------------
struct Layer {
	uint32_t out, in;
	uint64_t off;
	bool relu_out, relu_in;
};

struct Model {
	ngp_network_config cfg{};
	uint32_t L = 0, F = 0, E = 0, Epad = 0;
	std::vector<float> scale;
	std::vector<uint32_t> res, offset, size, hashed;
	std::vector<Layer> layers;
	uint32_t n_density_layers = 0;
	uint64_t n_mlp = 0, n_grid = 0, n = 0;
	std::vector<float> p32, ema32, grads, m, vv;
	std::vector<uint16_t> p16, inf16;
	std::vector<uint32_t> steps;
	uint32_t ema_step = 0;
	// occupancy
	std::vector<float> grid, tmp;
	std::vector<uint8_t> bits;
	float mean = 0.0f;
	// last training step scratch (ngp_train_scratch mirror)
	std::vector<uint32_t> ray_numsteps, ray_compacted;
	std::vector<float> coords, ccoords, loss;
	std::vector<uint16_t> mlp_out, dloss;
	uint32_t total_samples = 0, total_compacted = 0;
	float loss_sum = 0.0f;
};

// tcnn GridEncodingTemplated ctor; hash-grid auto params in src/testbed.cu:3680-3724
static void build(Model& M) {
	const auto& c = M.cfg;
	M.L = c.n_levels;
	M.F = c.n_features_per_level;
	M.E = M.L * M.F;
	M.Epad = (M.E + 15) / 16 * 16;
	const float lg = std::log2(c.per_level_scale);
	uint32_t off = 0;
	for (uint32_t l = 0; l < M.L; ++l) {
		const float s = std::exp2((float)l * lg) * (float)c.base_resolution - 1.0f;
		const uint32_t r = (uint32_t)std::ceil(s) + 1;
		const double dense = (double)r * r * r;
		uint32_t p = dense > (double)(0xFFFFFFFFu / 2) ? 0xFFFFFFFFu / 2 : r * r * r;
		p = (p + 7) / 8 * 8;
		p = std::min(p, 1u << c.log2_hashmap_size);
		M.scale.push_back(s);
		M.res.push_back(r);
		M.offset.push_back(off);
		M.size.push_back(p);
		M.hashed.push_back(dense > (double)p ? 1u : 0u);
		off += p;
	}
	M.n_grid = (uint64_t)off * M.F;
	const uint32_t W = c.n_neurons;
	auto add = [&](uint32_t out, uint32_t in, bool ro, bool ri) { M.layers.push_back({out, in, 0, ro, ri}); };
	add(W, M.Epad, true, false);
	for (uint32_t h = 1; h < c.density_hidden_layers; ++h) add(W, W, true, true);
	add(16, W, false, true);
	M.n_density_layers = (uint32_t)M.layers.size();
	// rgb input: density out 16 | dir encoding (SH 16, then the n_extra_dims Identity inputs), padded to 16
	// (nerf_network.h:84, 93)
	add(W, (32 + c.n_extra_dims + 15) / 16 * 16, true, false);
	for (uint32_t h = 1; h < c.rgb_hidden_layers; ++h) add(W, W, true, true);
	add(16, W, false, true);
	uint64_t o = 0;
	for (auto& Ly : M.layers) {
		Ly.off = o;
		o += (uint64_t)Ly.out * Ly.in;
	}
	M.n_mlp = o;
	M.n = M.n_mlp + M.n_grid;
	M.p32.assign(M.n, 0.0f);
	M.ema32.assign(M.n, 0.0f);
	M.grads.assign(M.n, 0.0f);
	M.m.assign(M.n, 0.0f);
	M.vv.assign(M.n, 0.0f);
	M.p16.assign(M.n, 0);
	M.inf16.assign(M.n, 0);
	M.steps.assign(M.n, 0);
	M.grid.assign(CELLS, 0.0f);
	M.bits.assign(CELLS / 8 * CASCADES, 0xff);
}

// ---- hash grid (tcnn grid.h: pos_fract, grid_index with CoherentPrime hash) -----------------
static uint32_t hg_index(const Model& M, uint32_t l, uint32_t x, uint32_t y, uint32_t z) {
	uint32_t idx;
	if (M.hashed[l]) idx = (x * 1u) ^ (y * 2654435761u) ^ (z * 805459861u);
	else idx = x + y * M.res[l] + z * M.res[l] * M.res[l];
	return idx % M.size[l];
}
static void hg_corners(const Model& M, uint32_t l, const float* p, uint32_t idx[8], float w[8]) {
	float fr[3];
	uint32_t g[3];
	for (int d = 0; d < 3; ++d) {
		const float q = std::fma(M.scale[l], p[d], 0.5f);
		const float f = std::floor(q);
		g[d] = (uint32_t)(int)f;
		fr[d] = q - f;
	}
	for (uint32_t c = 0; c < 8; ++c) {
		float ww = 1.0f;
		ww *= (c & 1) ? fr[0] : 1.0f - fr[0];
		ww *= (c & 2) ? fr[1] : 1.0f - fr[1];
		ww *= (c & 4) ? fr[2] : 1.0f - fr[2];
		idx[c] = hg_index(M, l, g[0] + (c & 1), g[1] + ((c >> 1) & 1), g[2] + ((c >> 2) & 1));
		w[c] = ww;
	}
}
// tcnn GridEncoding::set_max_level_gpu (kernel_grid / kernel_grid_backward): sample i's levels at or
// above max_level * (L F) / F + 1e-3 are zero and get no gradient; ml = null: all levels
static bool hg_cut(const Model& M, const float* ml, uint32_t ml_stride, uint32_t i, uint32_t l) {
	if (!ml) return false;
	const float mlv = (ml[(size_t)i * ml_stride] * (float)(M.L * M.F)) / (float)M.F;
	return (float)l >= mlv + 1e-3f;
}

// enc: [L][n][F] (fp16-rounded floats)
static void hg_forward(const Model& M, const uint16_t* params, const float* pos, uint32_t stride, uint32_t n, float* enc,
                       const float* ml = nullptr, uint32_t ml_stride = 0) {
	const uint16_t* tab = params + M.n_mlp;
	// samples are independent (the all-core CPU baseline; 1 thread unless oref_set_threads)
#pragma omp parallel for schedule(static)
	for (uint32_t i = 0; i < n; ++i)
		for (uint32_t l = 0; l < M.L; ++l) {
			if (hg_cut(M, ml, ml_stride, i, l)) {
				for (uint32_t f = 0; f < M.F; ++f) enc[((size_t)l * n + i) * M.F + f] = 0.0f;
				continue;
			}
			uint32_t idx[8];
			float w[8];
			hg_corners(M, l, pos + (size_t)i * stride, idx, w);
			for (uint32_t f = 0; f < M.F; ++f) {
				float acc = 0.0f;
				for (int c = 0; c < 8; ++c) acc = std::fma(w[c], h2f(tab[((size_t)M.offset[l] + idx[c]) * M.F + f]), acc);
				enc[((size_t)l * n + i) * M.F + f] = rh(acc);
			}
		}
}
static void hg_backward(Model& M, const float* pos, uint32_t stride, uint32_t n, const float* denc, const float* ml = nullptr,
                        uint32_t ml_stride = 0) {
	float* g = M.grads.data() + M.n_mlp;
	for (uint32_t i = 0; i < n; ++i)
		for (uint32_t l = 0; l < M.L; ++l) {
			bool any = false;
			for (uint32_t f = 0; f < M.F; ++f) any |= denc[((size_t)l * n + i) * M.F + f] != 0.0f;
			if (!any || hg_cut(M, ml, ml_stride, i, l)) continue;
			uint32_t idx[8];
			float w[8];
			hg_corners(M, l, pos + (size_t)i * stride, idx, w);
			for (int c = 0; c < 8; ++c)
				for (uint32_t f = 0; f < M.F; ++f)
					g[((size_t)M.offset[l] + idx[c]) * M.F + f] += w[c] * denc[((size_t)l * n + i) * M.F + f];
		}
}

// dL/d(position) through the grid (tcnn GridEncoding input gradient, linear interpolation):
// dL/dx_d = sum_l scale_l sum_c (c_d ? 1 : -1) prod_{e != d} w_e sum_f dL/denc[l][f] table[c][f]; ÷ weight
static void hg_input_grad(const Model& M, const uint16_t* params, const float* pos, uint32_t stride, uint32_t n,
                          const float* denc, const float* weight, float* dpos, const float* ml = nullptr, uint32_t ml_stride = 0) {
	const uint16_t* tab = params + M.n_mlp;
	for (uint32_t i = 0; i < n; ++i) {
		float g3[3] = {0.0f, 0.0f, 0.0f};
		const float* p = pos + (size_t)i * stride;
		for (uint32_t l = 0; l < M.L; ++l) {
			bool any = false;
			for (uint32_t f = 0; f < M.F; ++f) any |= denc[((size_t)l * n + i) * M.F + f] != 0.0f;
			if (!any || hg_cut(M, ml, ml_stride, i, l)) continue;
			float fr[3];
			uint32_t gc[3];
			for (int d = 0; d < 3; ++d) {
				const float q = std::fma(M.scale[l], p[d], 0.5f);
				const float fl = std::floor(q);
				gc[d] = (uint32_t)(int)fl;
				fr[d] = q - fl;
			}
			float lg[3] = {0.0f, 0.0f, 0.0f};
			for (uint32_t c = 0; c < 8; ++c) {
				const uint32_t idx = hg_index(M, l, gc[0] + (c & 1), gc[1] + ((c >> 1) & 1), gc[2] + ((c >> 2) & 1));
				float dotv = 0.0f;
				for (uint32_t f = 0; f < M.F; ++f)
					dotv += denc[((size_t)l * n + i) * M.F + f] * h2f(tab[((size_t)M.offset[l] + idx) * M.F + f]);
				const float w[3] = {(c & 1) ? fr[0] : 1.0f - fr[0], (c & 2) ? fr[1] : 1.0f - fr[1], (c & 4) ? fr[2] : 1.0f - fr[2]};
				lg[0] += dotv * ((c & 1) ? 1.0f : -1.0f) * w[1] * w[2];
				lg[1] += dotv * ((c & 2) ? 1.0f : -1.0f) * w[0] * w[2];
				lg[2] += dotv * ((c & 4) ? 1.0f : -1.0f) * w[0] * w[1];
			}
			for (int d = 0; d < 3; ++d) g3[d] += M.scale[l] * lg[d];
		}
		const float w = weight ? weight[i] : 1.0f;
		for (int d = 0; d < 3; ++d) dpos[3 * (size_t)i + d] = g3[d] / w;
	}
}

// ---- spherical harmonics degree 4 (tcnn SphericalHarmonicsEncoding) --------------------------
static void sh4(const float* wdir, float* o) {
	const float x = wdir[0] * 2.0f - 1.0f, y = wdir[1] * 2.0f - 1.0f, z = wdir[2] * 2.0f - 1.0f;
	const float xy = x * y, xz = x * z, yz = y * z, x2 = x * x, y2 = y * y, z2 = z * z;
	o[0] = 0.28209479177387814f;
	o[1] = -0.48860251190291987f * y;
	o[2] = 0.48860251190291987f * z;
	o[3] = -0.48860251190291987f * x;
	o[4] = 1.0925484305920792f * xy;
	o[5] = -1.0925484305920792f * yz;
	o[6] = 0.94617469575755997f * z2 - 0.31539156525251999f;
	o[7] = -1.0925484305920792f * xz;
	o[8] = 0.54627421529603959f * x2 - 0.54627421529603959f * y2;
	o[9] = 0.59004358992664352f * y * (-3.0f * x2 + y2);
	o[10] = 2.8906114426405538f * xy * z;
	o[11] = 0.45704579946446572f * y * (1.0f - 5.0f * z2);
	o[12] = 0.3731763325901154f * z * (5.0f * z2 - 3.0f);
	o[13] = 0.45704579946446572f * x * (1.0f - 5.0f * z2);
	o[14] = 1.4453057213202769f * z * (x2 - y2);
	o[15] = 0.59004358992664352f * x * (-x2 + 3.0f * y2);
	for (int k = 0; k < 16; ++k) o[k] = rh(o[k]);
}

// dL/d(x, y, z) of the SH basis above at (x, y, z) = 2 wdir - 1 (the derivative of each formula)
static V3 sh4_input_grad(const float* wdir, const float* g) {
	const float x = wdir[0] * 2.0f - 1.0f, y = wdir[1] * 2.0f - 1.0f, z = wdir[2] * 2.0f - 1.0f;
	const float x2 = x * x, y2 = y * y, z2 = z * z;
	const float a1 = 0.48860251190291987f, a4 = 1.0925484305920792f, a6 = 0.94617469575755997f, a8 = 0.54627421529603959f,
	            a9 = 0.59004358992664352f, a10 = 2.8906114426405538f, a11 = 0.45704579946446572f, a12 = 0.3731763325901154f,
	            a14 = 1.4453057213202769f;
	const float gx = -a1 * g[3] + a4 * y * g[4] - a4 * z * g[7] + 2.0f * a8 * x * g[8] - 6.0f * a9 * x * y * g[9] +
	                 a10 * y * z * g[10] + a11 * (1.0f - 5.0f * z2) * g[13] + 2.0f * a14 * x * z * g[14] +
	                 a9 * (3.0f * y2 - 3.0f * x2) * g[15];
	const float gy = -a1 * g[1] + a4 * x * g[4] - a4 * z * g[5] - 2.0f * a8 * y * g[8] + a9 * (3.0f * y2 - 3.0f * x2) * g[9] +
	                 a10 * x * z * g[10] + a11 * (1.0f - 5.0f * z2) * g[11] - 2.0f * a14 * y * z * g[14] + 6.0f * a9 * x * y * g[15];
	const float gz = a1 * g[2] - a4 * y * g[5] + 2.0f * a6 * z * g[6] - a4 * x * g[7] + a10 * x * y * g[10] -
	                 10.0f * a11 * y * z * g[11] + a12 * (15.0f * z2 - 3.0f) * g[12] - 10.0f * a11 * x * z * g[13] +
	                 a14 * (x2 - y2) * g[14];
	return v(gx, gy, gz);
}

// ---- MLP (NerfNetwork: density MLP -> [density_out | SH] -> rgb MLP), fp16 I/O, fp32 sums ------
struct Acts {
	std::vector<std::vector<float>> a;  // a[l] = input of layer l (fp16-rounded), a[NL] = final output
};
static void layer_fwd(const Model& M, const uint16_t* P, const Layer& Ly, const std::vector<float>& in, std::vector<float>& out,
                      bool round) {
	out.assign(Ly.out, 0.0f);
	const uint16_t* W = P + Ly.off;
	for (uint32_t r = 0; r < Ly.out; ++r) {
		float acc = 0.0f;
		for (uint32_t k = 0; k < Ly.in; ++k) acc += h2f(W[(size_t)r * Ly.in + k]) * in[k];
		if (Ly.relu_out) acc = std::max(acc, 0.0f);
		out[r] = round ? rh(acc) : acc;
	}
}
// code (n_extra_dims > 0): the sample's latent code, n_extra_dims floats (NerfCoordinate's extra dims), rounded to
// fp16 as tcnn's Identity encoding outputs them; null = zeros
static void mlp_forward_one(const Model& M, const uint16_t* P, const float* enc_col /*E*/, const float* wdir, Acts& A,
                            const float* code = nullptr) {
	const uint32_t NL = (uint32_t)M.layers.size();
	A.a.assign(NL + 1, {});
	A.a[0].assign(M.Epad, 0.0f);
	for (uint32_t k = 0; k < M.E; ++k) A.a[0][k] = enc_col[k];
	for (uint32_t l = 0; l < NL; ++l) {
		if (l == M.n_density_layers) {
			// rgb input = [density_out(16) | SH(16) | extra dims | zero padding]
			std::vector<float> x(M.layers[l].in, 0.0f);
			for (int k = 0; k < 16; ++k) x[k] = A.a[l][k];
			float sh[16];
			sh4(wdir, sh);
			for (int k = 0; k < 16; ++k) x[16 + k] = sh[k];
			for (uint32_t k = 0; k < M.cfg.n_extra_dims && code; ++k) x[32 + k] = rh(code[k]);
			A.a[l] = x;
		}
		layer_fwd(M, P, M.layers[l], A.a[l], A.a[l + 1], true);
	}
}
static void gather_enc(const Model& M, const float* enc, uint32_t n, uint32_t i, float* col) {
	for (uint32_t k = 0; k < M.E; ++k) col[k] = enc[((size_t)(k / M.F) * n + i) * M.F + (k % M.F)];
}
// out: [n][4] = rgb raw (3) + density raw (fp16-rounded)
// codes: sample i's latent code at codes + i * code_stride (code_stride 0: one code for all; null: none)
static void mlp_forward(const Model& M, const uint16_t* P, const float* enc, const float* coords, uint32_t cs, uint32_t n,
                        float* out, const float* codes = nullptr, uint32_t code_stride = 0) {
#pragma omp parallel
	{
	std::vector<float> col(M.E);
	Acts A;
#pragma omp for schedule(static)
	for (uint32_t i = 0; i < n; ++i) {
		gather_enc(M, enc, n, i, col.data());
		mlp_forward_one(M, P, col.data(), coords + (size_t)i * cs + 4, A, codes ? codes + (size_t)i * code_stride : nullptr);
		const uint32_t NL = (uint32_t)M.layers.size();
		out[4 * i + 0] = A.a[NL][0];
		out[4 * i + 1] = A.a[NL][1];
		out[4 * i + 2] = A.a[NL][2];
		out[4 * i + 3] = A.a[M.n_density_layers][0];  // density_out row 0 (first rgb-layer input)
	}
	}
}
// NerfNetwork::backward_impl (nerf_network.h:189-268): rgb MLP bwd -> add_density_gradient -> density MLP bwd
// dsh (optional, [n][16]): dL/d(SH inputs) of the sample's own row (÷ its rollover weight), for the
// camera gradients (tcnn's input gradient through the Composite encoding's SH part)
// codes / code_stride: the samples' latent codes (mlp_forward); dextra (optional, [n][NGP_EXTRA_ROW]): dL/d(rgb input rows
// 32..47) of the sample's own row (÷ its rollover weight) -- the extra dims' input gradient
static void mlp_backward(const Model& M, float* grads, const uint16_t* P, const float* enc, const float* coords, uint32_t cs,
                         uint32_t n, const float* dl /*[n][4] fp16 values*/, const float* weight, float* denc,
                         float* dsh = nullptr, const float* codes = nullptr, uint32_t code_stride = 0, float* dextra = nullptr) {
	const uint32_t NL = (uint32_t)M.layers.size();
	std::vector<float> col(M.E);
	Acts A;
	for (uint32_t i = 0; i < n; ++i) {
		gather_enc(M, enc, n, i, col.data());
		mlp_forward_one(M, P, col.data(), coords + (size_t)i * cs + 4, A, codes ? codes + (size_t)i * code_stride : nullptr);
		const float w = weight ? weight[i] : 1.0f;
		std::vector<float> delta(16, 0.0f);
		for (int r = 0; r < 3; ++r) delta[r] = rh(dl[4 * i + r] * w);
		for (int l = (int)NL - 1; l >= 0; --l) {
			const Layer& Ly = M.layers[l];
			const std::vector<float>& in = A.a[l];
			const uint16_t* W = P + Ly.off;
			float* G = grads + Ly.off;
			for (uint32_t r = 0; r < Ly.out; ++r)
				for (uint32_t k = 0; k < Ly.in; ++k) G[(size_t)r * Ly.in + k] += delta[r] * in[k];
			const uint32_t nin = (l == (int)M.n_density_layers) ? 16 : Ly.in;
			std::vector<float> nd(nin, 0.0f);
			for (uint32_t k = 0; k < nin; ++k) {
				float acc = 0.0f;
				for (uint32_t r = 0; r < Ly.out; ++r) acc += h2f(W[(size_t)r * Ly.in + k]) * delta[r];
				if (Ly.relu_in && !(in[k] > 0.0f)) acc = 0.0f;
				if (l == (int)M.n_density_layers && k == 0) acc += h2f(f2h(dl[4 * i + 3])) * w;
				nd[k] = rh(acc);
			}
			if (dsh && l == (int)M.n_density_layers)
				for (uint32_t k = 16; k < 32; ++k) {
					float acc = 0.0f;
					for (uint32_t r = 0; r < Ly.out; ++r) acc += h2f(W[(size_t)r * Ly.in + k]) * delta[r];
					dsh[16 * (size_t)i + (k - 16)] = acc / w;
				}
			if (dextra && l == (int)M.n_density_layers)
				for (uint32_t k = 32; k < 32 + NGP_EXTRA_ROW; ++k) {
					float acc = 0.0f;
					if (k < Ly.in)
						for (uint32_t r = 0; r < Ly.out; ++r) acc += h2f(W[(size_t)r * Ly.in + k]) * delta[r];
					dextra[NGP_EXTRA_ROW * (size_t)i + (k - 32)] = acc / w;
				}
			if (l == 0) {
				for (uint32_t k = 0; k < M.E; ++k) denc[((size_t)(k / M.F) * n + i) * M.F + (k % M.F)] = nd[k];
			}
			delta = nd;
		}
	}
}

// ---- optimizer: Ema(ExponentialDecay(Adam)) (tcnn; configs/nerf/base.json:5-22) --------------
static void optimizer(Model& M, uint32_t step, int opt_mlp, int opt_enc) {
	const auto& c = M.cfg;
	float lr = c.learning_rate;
	if (c.decay_interval > 0 && step >= c.decay_start) lr = c.learning_rate * std::pow(c.decay_base, (float)((step - c.decay_start) / c.decay_interval + 1));
	const float dold = 1.0f - std::pow(c.ema_decay, (float)M.ema_step), dnew = 1.0f - std::pow(c.ema_decay, (float)(M.ema_step + 1));
	for (uint64_t i = 0; i < M.n; ++i) {
		const float graw = M.grads[i];
		float w = M.p32[i];
		const bool mlp = i < M.n_mlp;
		if (mlp ? (bool)opt_mlp : (opt_enc && graw != 0.0f)) {
			float g = graw / 128.0f;
			if (mlp) g += c.l2_reg * w;
			M.m[i] = c.beta1 * M.m[i] + (1.0f - c.beta1) * g;
			M.vv[i] = c.beta2 * M.vv[i] + (1.0f - c.beta2) * g * g;
			const uint32_t s = ++M.steps[i];
			const float l = lr * std::sqrt(1.0f - std::pow(c.beta2, (float)s)) / (1.0f - std::pow(c.beta1, (float)s));
			w = w - (l / (std::sqrt(M.vv[i]) + c.epsilon)) * M.m[i];
			M.p32[i] = w;
			M.p16[i] = f2h(w);
		}
		M.grads[i] = 0.0f;
		const float e = (M.ema32[i] * c.ema_decay * dold + w * (1.0f - c.ema_decay)) / dnew;
		M.ema32[i] = e;
		M.inf16[i] = f2h(e);
	}
	++M.ema_step;
}

// ---- training images ------------------------------------------------------------------------
struct Cam {
	V3 c[4];
};
static Cam cam_of(const float* x) {
	Cam m;
	for (int k = 0; k < 4; ++k) m.c[k] = v(x[3 * k], x[3 * k + 1], x[3 * k + 2]);
	return m;
}
static V3 rot(const Cam& m, V3 d) { return m.c[0] * d.x + m.c[1] * d.y + m.c[2] * d.z; }

// Buffer2DView<const vec2>::at_lerp (include/neural-graphics-primitives/common.h:249-266) of the
// distortion map [ry][rx][2]: px = int(res * uv), weights = fraction, texels clamped to the edge;
// uv_to_ray adds it to the camera-space direction's xy (common_device.cuh:441-443)
static void distortion_lerp(const float* map, uint32_t rx, uint32_t ry, float u, float vv, float* dx, float* dy) {
	const float fx = (float)rx * u, fy = (float)ry * vv;
	const int px = (int)fx, py = (int)fy;
	const float wx = fx - (float)px, wy = fy - (float)py;
	auto at = [&](int x, int y, int c) {
		x = std::min(std::max(x, 0), (int)rx - 1);
		y = std::min(std::max(y, 0), (int)ry - 1);
		return map[2 * ((size_t)y * rx + x) + c];
	};
	for (int c = 0; c < 2; ++c) {
		const float r = (1.0f - wx) * (1.0f - wy) * at(px, py, c) + wx * (1.0f - wy) * at(px + 1, py, c) +
		                (1.0f - wx) * wy * at(px, py + 1, c) + wx * wy * at(px + 1, py + 1, c);
		*(c ? dy : dx) = r;
	}
}

// camera_slerp / get_xform_given_rolling_shutter (common_device.cuh:628-636).  tcnn's
// slerp(mat3, mat3, t) is absent from the mount: restated as glm's quat_cast -> slerp (lerp when
// cos > 1 - FLT_EPSILON) -> normalize -> mat3_cast, translation mixed; t = 0 returns the start
// (parity unpinned beyond that).
static Cam slerp_cam(const Cam& a, const Cam& b, float t) {
	if (t == 0.0f) return a;
	auto to_q = [](const Cam& m, float* q) {  // w, x, y, z
		const float m00 = m.c[0].x, m01 = m.c[0].y, m02 = m.c[0].z, m10 = m.c[1].x, m11 = m.c[1].y, m12 = m.c[1].z;
		const float m20 = m.c[2].x, m21 = m.c[2].y, m22 = m.c[2].z;
		const float f[4] = {m00 + m11 + m22, m00 - m11 - m22, m11 - m00 - m22, m22 - m00 - m11};
		int bi = 0;
		for (int k = 1; k < 4; ++k)
			if (f[k] > f[bi]) bi = k;
		const float bv = std::sqrt(f[bi] + 1.0f) * 0.5f, mu = 0.25f / bv;
		const float a12 = (m12 - m21) * mu, a20 = (m20 - m02) * mu, a01 = (m01 - m10) * mu;
		const float s01 = (m01 + m10) * mu, s20 = (m20 + m02) * mu, s12 = (m12 + m21) * mu;
		const float r[4][4] = {{bv, a12, a20, a01}, {a12, bv, s01, s20}, {a20, s01, bv, s12}, {a01, s20, s12, bv}};
		for (int k = 0; k < 4; ++k) q[k] = r[bi][k];
	};
	float qa[4], qb[4], q[4];
	to_q(a, qa);
	to_q(b, qb);
	float c = qa[0] * qb[0] + qa[1] * qb[1] + qa[2] * qb[2] + qa[3] * qb[3];
	if (c < 0.0f) {
		for (float& x : qb) x = -x;
		c = -c;
	}
	if (c > 1.0f - 1.1920928955078125e-7f) {
		for (int k = 0; k < 4; ++k) q[k] = qa[k] * (1.0f - t) + qb[k] * t;
	} else {
		const float ang = std::acos(c), s0 = std::sin((1.0f - t) * ang), s1 = std::sin(t * ang), inv = 1.0f / std::sin(ang);
		for (int k = 0; k < 4; ++k) q[k] = (s0 * qa[k] + s1 * qb[k]) * inv;
	}
	const float in = 1.0f / std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
	const float w = q[0] * in, x = q[1] * in, y = q[2] * in, z = q[3] * in;
	Cam r;
	r.c[0] = v(1.0f - 2.0f * (y * y + z * z), 2.0f * (x * y + w * z), 2.0f * (x * z - w * y));
	r.c[1] = v(2.0f * (x * y - w * z), 1.0f - 2.0f * (x * x + z * z), 2.0f * (y * z + w * x));
	r.c[2] = v(2.0f * (x * z + w * y), 2.0f * (y * z - w * x), 1.0f - 2.0f * (x * x + y * y));
	r.c[3] = v(a.c[3].x * (1.0f - t) + b.c[3].x * t, a.c[3].y * (1.0f - t) + b.c[3].y * t, a.c[3].z * (1.0f - t) + b.c[3].z * t);
	return r;
}
static bool rs_on(const float* rs) { return rs[0] != 0.0f || rs[1] != 0.0f || rs[2] != 0.0f || rs[3] != 0.0f; }

// inverse(mat3(m)) * g, glm's adjugate / determinant inverse (compute_cam_gradient_train_nerf
// src/testbed_nerf.cu:1242)
static V3 inv3_mul(const Cam& m, V3 g) {
	const float m00 = m.c[0].x, m01 = m.c[0].y, m02 = m.c[0].z, m10 = m.c[1].x, m11 = m.c[1].y, m12 = m.c[1].z;
	const float m20 = m.c[2].x, m21 = m.c[2].y, m22 = m.c[2].z;
	const float id = 1.0f / (m00 * (m11 * m22 - m21 * m12) - m10 * (m01 * m22 - m21 * m02) + m20 * (m01 * m12 - m11 * m02));
	const float i00 = (m11 * m22 - m21 * m12) * id, i10 = -(m10 * m22 - m20 * m12) * id, i20 = (m10 * m21 - m20 * m11) * id;
	const float i01 = -(m01 * m22 - m21 * m02) * id, i11 = (m00 * m22 - m20 * m02) * id, i21 = -(m00 * m21 - m20 * m01) * id;
	const float i02 = (m01 * m12 - m11 * m02) * id, i12 = -(m00 * m12 - m10 * m02) * id, i22 = (m00 * m11 - m10 * m01) * id;
	return v(i00 * g.x + i10 * g.y + i20 * g.z, i01 * g.x + i11 * g.y + i21 * g.z, i02 * g.x + i12 * g.y + i22 * g.z);
}
static uint32_t texel(const ngp_image& im, float u, float vv) {
	const int px = std::min(std::max((int)(u * (float)im.width), 0), (int)im.width - 1);
	const int py = std::min(std::max((int)(vv * (float)im.height), 0), (int)im.height - 1);
	return reinterpret_cast<const uint32_t*>(im.pixels)[(size_t)px + (size_t)py * im.width];
}
static void rgba_of(uint32_t t, float* o) {
	if (t == 0x00FF00FFu) { o[0] = o[1] = o[2] = o[3] = -1.0f; return; }
	const float a = (float)((t >> 24) & 0xff) * (1.0f / 255.0f);
	o[0] = s2l((float)(t & 0xff) * (1.0f / 255.0f)) * a;
	o[1] = s2l((float)((t >> 8) & 0xff) * (1.0f / 255.0f)) * a;
	o[2] = s2l((float)((t >> 16) & 0xff) * (1.0f / 255.0f)) * a;
	o[3] = a;
}
static uint32_t image_index(uint32_t i, uint32_t n_rays, uint32_t n_img) {
	return (uint32_t)((((uint64_t)i) * n_img) / n_rays) % n_img;  // nerf_device.cuh:597
}
// Lens models of uv_to_ray (common_device.cuh:248-460): ELensMode 0 Perspective, 1 OpenCV,
// 2 FTheta, 3 LatLong, 4 OpenCVFisheye, 5 Equirectangular.
static void lens_delta(int mode, const float* k, float u, float v, float* du, float* dv) {
	if (mode == 1) {  // opencv_lens_distortion_delta
		const float u2 = u * u, uv = u * v, v2 = v * v, r2 = u2 + v2;
		const float radial = k[0] * r2 + k[1] * r2 * r2;
		*du = u * radial + 2.0f * k[2] * uv + k[3] * (r2 + 2.0f * u2);
		*dv = v * radial + 2.0f * k[3] * uv + k[2] * (r2 + 2.0f * v2);
		return;
	}
	// opencv_fisheye_lens_distortion_delta
	const float r = std::sqrt(u * u + v * v);
	if (r > 2.220446049250313e-16f) {
		const float th = std::atan(r), t2 = th * th, t4 = t2 * t2, t6 = t4 * t2, t8 = t4 * t4;
		const float thd = th * (1.0f + k[0] * t2 + k[1] * t4 + k[2] * t6 + k[3] * t8);
		*du = u * thd / r - u;
		*dv = v * thd / r - v;
	} else {
		*du = *dv = 0.0f;
	}
}
// iterative_lens_undistortion: Newton, central-difference Jacobian, <= 100 steps
static void undistort(int mode, const float* k, float* u, float* v) {
	const float x0 = *u, y0 = *v;
	float x = x0, y = y0;
	for (int it = 0; it < 100; ++it) {
		const float s0 = std::max(1.1920929e-7f, std::fabs(1e-6f * x)), s1 = std::max(1.1920929e-7f, std::fabs(1e-6f * y));
		float dx, dy, a0, b0, a1, b1, c0, d0, c1, d1;
		lens_delta(mode, k, x, y, &dx, &dy);
		lens_delta(mode, k, x - s0, y, &a0, &b0);
		lens_delta(mode, k, x + s0, y, &a1, &b1);
		lens_delta(mode, k, x, y - s1, &c0, &d0);
		lens_delta(mode, k, x, y + s1, &c1, &d1);
		const float j00 = 1.0f + (a1 - a0) / (2.0f * s0), j10 = (c1 - c0) / (2.0f * s1);
		const float j01 = (b1 - b0) / (2.0f * s0), j11 = 1.0f + (d1 - d0) / (2.0f * s1);
		const float rx = x + dx - x0, ry = y + dy - y0;
		const float inv = 1.0f / (j00 * j11 - j10 * j01);
		const float sx = (j11 * inv) * rx + (-j10 * inv) * ry, sy = (-j01 * inv) * rx + (j00 * inv) * ry;
		x -= sx;
		y -= sy;
		if (sx * sx + sy * sy < 1e-10f) break;
	}
	*u = x;
	*v = y;
}
// camera-space direction of screen position (u, v); false = invalid ray (F-Theta)
static bool lens_dir(float u, float vv, float rx, float ry, float fx, float fy, float cx, float cy, int mode, const float* k,
                     V3* d) {
	const float PI_F = 3.14159265358979323846f;
	if (mode == 2) {
		const float xp = (u - cx) * k[5], yp = (vv - cy) * k[6];
		const float nrm = std::sqrt(xp * xp + yp * yp);
		const float al = k[0] + nrm * (k[1] + nrm * (k[2] + nrm * (k[3] + nrm * k[4])));
		float sa = std::sin(al);
		const float ca = std::cos(al);
		if (ca <= 1.17549435e-38f || nrm == 0.0f) return false;
		sa *= 1.0f / nrm;
		*d = v(sa * xp, sa * yp, ca);
		return true;
	}
	if (mode == 3) {  // latlong_to_dir
		const float th = (vv - 0.5f) * PI_F, ph = (u - 0.5f) * PI_F * 2.0f;
		*d = v(std::sin(ph) * std::cos(th), std::sin(th), std::cos(ph) * std::cos(th));
		return true;
	}
	if (mode == 5) {  // equirectangular_to_dir
		const float ct = (vv - 0.5f) * 2.0f, st = std::sqrt(std::max(1.0f - ct * ct, 0.0f)), ph = (u - 0.5f) * PI_F * 2.0f;
		*d = v(std::sin(ph) * st, ct, std::cos(ph) * st);
		return true;
	}
	float x = (u - cx) * rx / fx, y = (vv - cy) * ry / fy;
	if (mode == 1 || mode == 4) undistort(mode, k, &x, &y);
	*d = v(x, y, 1.0f);
	return true;
}

// binary_search (common.h:207-230): first index with data[i] >= val, clamped to length-1
static uint32_t cdf_search(float val, const float* data, uint32_t length) {
	if (length == 0) return 0;
	uint32_t first = 0, count = length;
	while (count > 0) {
		const uint32_t step = count / 2, it = first + step;
		if (data[it] < val) {
			first = it + 1;
			count -= step + 1;
		} else {
			count = step;
		}
	}
	return std::min(first, length - 1);
}


// image_idx + nerf_random_image_pos_training with the error-map CDFs (nerf_device.cuh:495-598);
// *pdf = img_pdf * uv_pdf (uv_pdf stays 1 on the uniform half of sample_cdf_2d).
static uint32_t pick_pixel(const ngp_train_args& a, uint32_t gi, uint32_t nrg, Pcg& rng, float* u, float* vv, float* pdf,
                           float* uv_pdf_out = nullptr) {
	uint32_t img;
	float img_pdf = 1.0f, uv_pdf = 1.0f;
	if (a.cdf_img) {
		img = cdf_search(ldval(gi, 0xdeadbeefu, 0), a.cdf_img, a.n_images);  // ld_random_val (random_val.cuh:287-291)
		img_pdf = (a.cdf_img[img] - (img > 0 ? a.cdf_img[img - 1] : 0.0f)) * (float)a.n_images;
	} else {
		img = image_index(gi, nrg, a.n_images);
	}
	const ngp_image& im = a.images[img];
	float x = rng.nextf(), y = rng.nextf();
	if (a.cdf_x_cond_y) {
		const uint32_t rx = a.cdf_res[0], ry = a.cdf_res[1];
		if (x < 0.5f) {
			x = x * 2.0f;
		} else {
			const float su = (x - 0.5f) * 2.0f;
			const float* cy = a.cdf_y + (size_t)img * ry;
			const uint32_t yi = cdf_search(y, cy, ry);
			float prev = yi > 0 ? cy[yi - 1] : 0.0f;
			const float pmf_y = cy[yi] - prev;
			const float sv = (y - prev) / pmf_y;
			const float* cx = a.cdf_x_cond_y + ((size_t)img * ry + yi) * rx;
			const uint32_t xi = cdf_search(su, cx, rx);
			prev = xi > 0 ? cx[xi - 1] : 0.0f;
			const float pmf_x = cx[xi] - prev;
			const float sx = (su - prev) / pmf_x;
			uv_pdf = pmf_x * pmf_y * (float)(rx * ry);
			x = ((float)xi + sx) / (float)rx;
			y = ((float)yi + sv) / (float)ry;
		}
	}
	if (a.snap_to_pixel_centers) {  // nerf_device.cuh:570-572
		const int px = std::min(std::max((int)(x * (float)im.width), 0), (int)im.width - 1);
		const int py = std::min(std::max((int)(y * (float)im.height), 0), (int)im.height - 1);
		x = ((float)px + 0.5f) / (float)im.width;
		y = ((float)py + 0.5f) / (float)im.height;
	}
	*u = x;
	*vv = y;
	if (pdf) *pdf = img_pdf * uv_pdf;
	if (uv_pdf_out) *uv_pdf_out = uv_pdf;
	return img;
}

// generate_training_samples_nerf (src/testbed_nerf.cu:679-838), per-ray: origin, direction,
// first lattice point n0 = to_stepping_space(t_entry) + random; t_entry and the random offset
// are returned too (the literal transcription below starts from them).
static bool train_ray(const ngp_train_args& a, uint32_t gi, uint32_t nrg, V3* o, V3* d, float* st, float* t_entry = nullptr,
                      float* jitter = nullptr, float* dlen = nullptr, float* max_level = nullptr, uint32_t* img_out = nullptr) {
	Pcg rng;
	rng.state = a.rng_state;
	rng.inc = a.rng_inc;
	rng.advance((int64_t)gi * 16);
	float u, vv;
	const uint32_t img = pick_pixel(a, gi, nrg, rng, &u, &vv, nullptr);
	if (img_out) *img_out = img;
	const ngp_image& im = a.images[img];
	float rgba[4];
	rgba_of(texel(im, u, vv), rgba);
	if (rgba[0] < 0.0f) return false;
	// max_level_rand_training (src/testbed_nerf.cu:724): drawn before motionblur_time
	const float ml = a.max_level_rand_training ? rng.nextf() * 2.0f : 0.0f;
	if (max_level) *max_level = ml;
	const float mb = rng.nextf();  // motionblur_time
	Cam x = cam_of(im.xform);
	if (rs_on(im.rolling_shutter))
		x = slerp_cam(x, cam_of(im.xform_end),
		              im.rolling_shutter[0] + im.rolling_shutter[1] * u + im.rolling_shutter[2] * vv + im.rolling_shutter[3] * mb);
	V3 dir;
	if (lens_dir(u, vv, (float)im.width, (float)im.height, im.focal_length[0], im.focal_length[1], im.principal_point[0],
	             im.principal_point[1], im.lens_mode, im.lens_params, &dir)) {
		if (a.distortion_map && a.distortion_res[0] && a.distortion_res[1]) {
			float ddx, ddy;
			distortion_lerp(a.distortion_map, a.distortion_res[0], a.distortion_res[1], u, vv, &ddx, &ddy);
			dir.x += ddx;
			dir.y += ddy;
		}
		dir = rot(x, dir);
	} else {
		dir = x.c[2];  // src/testbed_nerf.cu:762-764
	}
	*o = x.c[3];
	if (dlen) *dlen = len(dir);  // |rays_in_unnormalized[i].d| (src/testbed_nerf.cu:1013)
	*d = normalize(dir);
	const Box b{v(a.aabb_min[0], a.aabb_min[1], a.aabb_min[2]), v(a.aabb_max[0], a.aabb_max[1], a.aabb_max[2])};
	float t0, t1;
	b.intersect(*o, *d, &t0, &t1);
	t0 = std::max(t0, 0.0f);
	const float r = rng.nextf();
	*st = lat_to(make_stepping(a.cone_angle_constant), t0) + r;  // n0: first lattice point
	if (t_entry) *t_entry = t0;
	if (jitter) *jitter = r;
	return true;
}

// The reference's sampling walk (testbed_nerf.cu:779-795) on the stepping lattice: at lattice
// point n0 + k, a sample if the cell at mip_from_dt is occupied (next point k + 1), else
// advance_to_next_voxel at that mip (nerf_device.cuh:444-453): jump to the first lattice point
// past the cell's far face; stop at the first visited point outside the AABB or after `cap`
// samples.  visit(j, k, t, dt, pos) for sample j.
template <class Visit>
static uint32_t training_walk(const Stepping& stp, const Box& box, const uint8_t* bits, uint32_t maxc, V3 o, V3 d, float n0,
                              uint32_t cap, Visit visit) {
	const V3 idir = v(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
	uint32_t j = 0;
	for (uint32_t k = 0; j < cap;) {
		const float n = n0 + (float)k;
		const float t = lat_from(stp, n), dt = lat_from(stp, n + 1.0f) - t;
		const V3 pos = o + d * t;
		if (!box.contains(pos)) break;
		const uint32_t mip = mip_dt(dt, pos, maxc);
		if (occupied(pos, bits, mip)) {
			visit(j, k, t, dt, pos);
			++j;
			++k;
		} else {
			const float n_far = lat_to(stp, t + dist_next_cell(pos, d, idir, mip));
			k += (uint32_t)std::fmin(std::ceil(std::fmax(n_far - n, 0.5f)), 1048576.0f);
		}
	}
	return j;
}

// ---- literal transcription of the reference's stepping (nerf_device.cuh:378-453), for the
// parity test of the lattice walk: chained t, no lattice, the reference's own divisions. ----
static float ref_to_stepping_space(float t, float cone) {
	if (cone <= 1e-5f) return t / MIN_STEP;
	const float log1p_c = logf(1.0f + cone);
	const float a = (logf(MIN_STEP) - logf(log1p_c)) / log1p_c, b = (logf(MAX_STEP) - logf(log1p_c)) / log1p_c;
	const float at = expf(a * log1p_c), bt = expf(b * log1p_c);
	if (t <= at) return (t - at) / MIN_STEP + a;
	if (t <= bt) return logf(t) / log1p_c;
	return (t - bt) / MAX_STEP + b;
}
static float ref_from_stepping_space(float n, float cone) {
	if (cone <= 1e-5f) return n * MIN_STEP;
	const float log1p_c = logf(1.0f + cone);
	const float a = (logf(MIN_STEP) - logf(log1p_c)) / log1p_c, b = (logf(MAX_STEP) - logf(log1p_c)) / log1p_c;
	const float at = expf(a * log1p_c), bt = expf(b * log1p_c);
	if (n <= a) return (n - a) * MIN_STEP + at;
	if (n <= b) return expf(n * log1p_c);
	return (n - b) * MAX_STEP + bt;
}
static float ref_advance_n_steps(float t, float cone, float n) {
	return ref_from_stepping_space(ref_to_stepping_space(t, cone) + n, cone);
}
static float ref_calc_dt(float t, float cone) { return ref_advance_n_steps(t, cone, 1.0f) - t; }
static float ref_advance_to_next_voxel(float t, float cone, V3 pos, V3 dir, V3 idir, uint32_t mip) {
	const float t_target = t + dist_next_cell(pos, dir, idir, mip);
	const float ts = ref_to_stepping_space(t, cone), tt = ref_to_stepping_space(t_target, cone);
	return ref_from_stepping_space(ts + std::ceil(std::fmax(tt - ts, 0.5f)), cone);
}

// if_unoccupied_advance_to_next_occupied_voxel<MIP_FROM_DT = false> (nerf_device.cuh:462-494), the
// renderer's form, literally: the cell at clamp(mip_from_pos(pos), min_mip, max_mip); an empty cell climbs to
// the coarsest empty mip and advance_to_next_voxel jumps the chained t past its far face.
// Distance (in cells of that mip) from pos to the nearest face of the cascade-mip cell grid.
static float face_distance(V3 pos, uint32_t mip) {
	const float res = std::scalbn((float)GRID, -(int)mip);
	float best = 1.0f;
	for (float c : {pos.x, pos.y, pos.z}) {
		const float p = (c - 0.5f) * res;
		best = std::min(best, std::fabs(p - std::round(p)));
	}
	return best;
}
// trace (tests): every point the march visits -- its stepping-space position, the face distance at the mip
// it was decided at (the climbed mip for an empty one) and whether it is occupied
struct MarchTrace {
	std::vector<float> n, face;
	std::vector<uint8_t> occ;
};
static float ref_if_unoccupied_advance(float t, float cone, V3 o, V3 d, V3 idir, const uint8_t* bits, uint32_t min_mip,
                                       uint32_t max_mip, const RBox& box, MarchTrace* tr = nullptr) {
	while (true) {
		const V3 pos = o + d * t;
		if (t >= MAXD || !box.contains(pos)) return MAXD;
		uint32_t mip = std::min(std::max(mip_pos(pos), min_mip), max_mip);
		if (!bits || occupied(pos, bits, mip)) {
			if (tr) { tr->n.push_back(ref_to_stepping_space(t, cone)); tr->face.push_back(face_distance(pos, mip)); tr->occ.push_back(1); }
			return t;
		}
		while (mip < max_mip && !occupied(pos, bits, mip + 1)) ++mip;
		if (tr) { tr->n.push_back(ref_to_stepping_space(t, cone)); tr->face.push_back(face_distance(pos, mip)); tr->occ.push_back(0); }
		t = ref_advance_to_next_voxel(t, cone, pos, d, idir, mip);
	}
}

// One ray of NerfTracer::trace, literally: advance_pos_nerf (src/testbed_nerf.cu:333-362) from the
// payload's t = max(t_entry, 0) + 1e-6 (:1465-1475), then generate_next_nerf_network_inputs passes
// (:421-469) of n_steps samples each, t += dt chained through payload.t across passes.  visit(t, dt) per
// sample until it returns false (the composite's stop) or the ray leaves the box; returns the samples.
template <class Visit>
static uint32_t ref_render_ray(float t_start, float jitter, float cone, V3 o, V3 d, const uint8_t* bits, uint32_t max_mip,
                               const RBox& box, uint32_t n_steps, uint32_t cap, Visit visit, MarchTrace* tr = nullptr) {
	const V3 idir = v(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
	// advance_pos_nerf
	float t = ref_advance_n_steps(t_start, cone, jitter);
	t = ref_if_unoccupied_advance(t, cone, o, d, idir, bits, 0, max_mip, box, tr);
	if (t >= MAXD) return 0;
	uint32_t count = 0;
	for (uint32_t pass = 0; count < cap; ++pass) {
		// generate_next_nerf_network_inputs: payload.t -> n_steps samples -> payload.t
		for (uint32_t j = 0; j < n_steps; ++j) {
			t = ref_if_unoccupied_advance(t, cone, o, d, idir, bits, 0, max_mip, box, tr);
			if (t >= MAXD) return count;
			const float dt = ref_calc_dt(t, cone);
			++count;
			if (!visit(t, dt) || count >= cap) return count;
			t += dt;
		}
	}
	return count;
}

// Data parallelism (ngp_train_args.world_size): every rank learns all ranks' totals
// through the caller's all-reduce (sum of [world] slots, its own slot set) and caps its share of
// the global order: out = {first global index of this rank, min(global total, cap)}; returns the
// rank's share of the cap.  One process: {0, min(total, cap)}, cap.
static uint32_t dp_share(const ngp_train_args& a, uint32_t total, uint32_t cap, uint32_t out[2]) {
	const uint32_t world = a.world_size > 1 && a.allreduce_i32 ? a.world_size : 1u;
	if (world == 1) {
		out[0] = 0;
		out[1] = std::min(total, cap);
		return cap;
	}
	std::vector<int32_t> slots(world, 0);
	slots[a.rank] = (int32_t)total;
	if (a.allreduce_i32(a.allreduce_user, slots.data(), world, nullptr) != 0) throw std::runtime_error("all-reduce failed");
	uint64_t base = 0, sum = 0;
	for (uint32_t q = 0; q < world; ++q) {
		if (q < a.rank) base += (uint32_t)slots[q];
		sum += (uint32_t)slots[q];
	}
	out[0] = (uint32_t)base;
	out[1] = (uint32_t)std::min<uint64_t>(sum, cap);
	return base >= cap ? 0u : (uint32_t)(cap - base);
}

static void train_step(Model& M, const ngp_train_args& a) {
	const uint32_t R = a.n_rays, B = a.target_batch_size;
	const uint32_t nrg = a.n_rays_global ? a.n_rays_global : R;
	const Box box{v(a.aabb_min[0], a.aabb_min[1], a.aabb_min[2]), v(a.aabb_max[0], a.aabb_max[1], a.aabb_max[2])};
	const Stepping stp = make_stepping(a.cone_angle_constant);
	// pass 1: count (testbed_nerf.cu:779-799)
	std::vector<uint32_t> cnt(R, 0);
	std::vector<V3> ro(R), rd(R);
	std::vector<float> rst(R), rdl(R, 1.0f), rml(R, 0.0f);
	std::vector<uint32_t> rimg(R, 0);
	for (uint32_t i = 0; i < R; ++i) {
		V3 o, d;
		float t;
		if (!train_ray(a, a.ray_index_offset + i, nrg, &o, &d, &t, nullptr, nullptr, &rdl[i], &rml[i], &rimg[i])) continue;
		ro[i] = o; rd[i] = d; rst[i] = t;
		cnt[i] = training_walk(stp, box, M.bits.data(), a.max_cascade, o, d, t, STEPS,
		                       [](uint32_t, uint32_t, float, float, V3) {});
	}
	// prefix-sum slot claim in ray order; drop if base + n > cap (testbed_nerf.cu:800-803) -- the cap
	// of the global order when data parallel (this rank's share)
	uint32_t total = 0;
	for (uint32_t i = 0; i < R; ++i) total += cnt[i];
	uint32_t sdp[2];
	const uint32_t MS = dp_share(a, total, a.max_samples, sdp);
	M.ray_numsteps.assign(2 * (size_t)R, 0);
	M.coords.assign(8 * (size_t)a.max_samples, 0.0f);
	uint32_t base = 0;
	for (uint32_t i = 0; i < R; ++i) {
		const uint32_t n = cnt[i];
		const uint32_t b = base;
		base += n;
		if (n == 0 || b + n > MS) continue;
		M.ray_numsteps[2 * i] = n;
		M.ray_numsteps[2 * i + 1] = b;
		// pass 2: write coordinates (testbed_nerf.cu:814-830)
		const V3 d = rd[i];
		const V3 wd = v((d.x + 1.0f) * 0.5f, (d.y + 1.0f) * 0.5f, (d.z + 1.0f) * 0.5f);
		training_walk(stp, box, M.bits.data(), a.max_cascade, ro[i], d, rst[i], n,
		              [&](uint32_t j, uint32_t, float, float dt, V3 pos) {
			              const V3 w = box.rel(pos);
			              float* c = &M.coords[8 * (size_t)(b + j)];
			              c[0] = w.x; c[1] = w.y; c[2] = w.z; c[3] = warp_dt(dt);
			              c[4] = wd.x; c[5] = wd.y; c[6] = wd.z; c[7] = rml[i];  // pad: the ray's max level
		              });
	}
	M.total_samples = base;
	const uint32_t S = std::min(base, MS);
	// n_extra_dims > 0: every sample carries its image's latent code (generate_training_samples_nerf, :730, 824:
	// extra_dims_gpu + img * n_extra_dims; here rows of NGP_EXTRA_ROW)
	const uint32_t XD = M.cfg.n_extra_dims;
	std::vector<float> scodes(XD ? NGP_EXTRA_ROW * (size_t)S : 0, 0.0f);
	if (XD && a.extra_dims)
		for (uint32_t i = 0; i < R; ++i)
			for (uint32_t j = 0; j < M.ray_numsteps[2 * i]; ++j)
				for (uint32_t k = 0; k < NGP_EXTRA_ROW; ++k)
					scodes[NGP_EXTRA_ROW * ((size_t)M.ray_numsteps[2 * i + 1] + j) + k] = a.extra_dims[NGP_EXTRA_ROW * (size_t)rimg[i] + k];
	// inference over the emitted samples with the training params (testbed_nerf.cu:2800-2802)
	std::vector<float> enc((size_t)M.L * S * M.F), out(4 * (size_t)S);
	const bool ml_on = a.max_level_rand_training != 0;
	hg_forward(M, M.p16.data(), M.coords.data(), 8, S, enc.data(), ml_on ? M.coords.data() + 7 : nullptr, 8);
	mlp_forward(M, M.p16.data(), enc.data(), M.coords.data(), 8, S, out.data(), XD ? scodes.data() : nullptr, NGP_EXTRA_ROW);
	M.mlp_out.assign(4 * (size_t)a.max_samples, 0);
	for (size_t k = 0; k < out.size(); ++k) M.mlp_out[k] = f2h(out[k]);

	// compute_loss_kernel_train_nerf (testbed_nerf.cu:841-1119)
	const int ract = M.cfg.rgb_activation, dact = M.cfg.density_activation;
	std::vector<uint32_t> cc(R, 0);
	std::vector<float> lstate(8 * (size_t)R, 0.0f), expg(3 * (size_t)R, 0.0f), ray_uv_pdf(R, 1.0f), ray_uv(2 * (size_t)R, 0.0f);
	// depth supervision (src/testbed_nerf.cu:1013-1015): composited depth and lambda * dloss/ddepth per ray
	const bool depth_on = a.depth_supervision_lambda > 0.0f;
	// include_sharpness_in_error (src/testbed_nerf.cu:1036-1044, 2453-2464)
	const bool sharp_on = a.sharpness_data && a.sharpness_grid && a.error_map;
	if (sharp_on) {
		const size_t nc = (size_t)CELLS * CASCADES;
		for (size_t k = 0; k < nc; ++k) a.sharpness_grid[k] = a.sharpness_grid_clear ? 0.0f : a.sharpness_grid[k] * 0.95f;
	}
	std::vector<V3> ray_hit(R, v(0, 0, 0));
	std::vector<float> ray_depth(R, 0.0f), ray_dlg(R, 0.0f);
	for (uint32_t i = 0; i < R; ++i) {
		const uint32_t ns = M.ray_numsteps[2 * i], b0 = M.ray_numsteps[2 * i + 1];
		if (ns == 0) continue;
		float T = 1.0f;
		float rr = 0, rg = 0, rb = 0, dray = 0;
		uint32_t c = 0;
		for (; c < ns; ++c) {
			if (T < 1e-4f) break;
			const float* o = &out[4 * (size_t)(b0 + c)];
			const float dt = unwarp_dt(M.coords[8 * (size_t)(b0 + c) + 3]);
			const float alpha = 1.0f - std::exp(-to_density(o[3], dact) * dt);
			const float w = alpha * T;
			rr += w * to_rgb(o[0], ract);
			rg += w * to_rgb(o[1], ract);
			rb += w * to_rgb(o[2], ract);
			if (sharp_on) {
				const float* cw = &M.coords[8 * (size_t)(b0 + c)];
				ray_hit[i] = ray_hit[i] + (box.mn + v(cw[0] * (box.mx.x - box.mn.x), cw[1] * (box.mx.y - box.mn.y), cw[2] * (box.mx.z - box.mn.z))) * w;
			}
			if (depth_on) {
				const float* cw = &M.coords[8 * (size_t)(b0 + c)];
				const V3 pos = box.mn + v(cw[0] * (box.mx.x - box.mn.x), cw[1] * (box.mx.y - box.mn.y), cw[2] * (box.mx.z - box.mn.z));
				dray += w * len(pos - ro[i]);
			}
			T *= 1.0f - alpha;
		}
		const uint32_t gi = a.ray_index_offset + i;
		Pcg rng;
		rng.state = a.rng_state;
		rng.inc = a.rng_inc;
		rng.advance((int64_t)gi * 16);
		float u, vv, pdf, uv_pdf;
		const uint32_t img = pick_pixel(a, gi, nrg, rng, &u, &vv, &pdf, &uv_pdf);
		ray_uv_pdf[i] = uv_pdf;
		ray_uv[2 * i] = u;
		ray_uv[2 * i + 1] = vv;
		const ngp_image& im = a.images[img];
		if (a.max_level_rand_training) rng.advance(1);  // max_level (src/testbed_nerf.cu:949)
		rng.advance(1);
		V3 bg = v(a.background_color[0], a.background_color[1], a.background_color[2]);
		if (a.random_bg_color) {
			const float x0 = rng.nextf(), x1 = rng.nextf(), x2 = rng.nextf();
			bg = v(x0, x1, x2);
		}
		bg = v(s2l(bg.x), s2l(bg.y), s2l(bg.z));
		float tex[4];
		rgba_of(texel(im, u, vv), tex);
		float es[3] = {1.0f, 1.0f, 1.0f};  // exposure_scale = 2^exposure[img] (src/testbed_nerf.cu:966)
		if (a.exposure)
			for (int k = 0; k < 3; ++k) es[k] = std::exp(0.6931471805599453f * a.exposure[3 * img + k]);
		for (int k = 0; k < 3; ++k) tex[k] *= es[k];
		V3 tgt;
		if (a.train_in_linear_colors || a.color_space == 0) {
			tgt = v(tex[0], tex[1], tex[2]) + bg * (1.0f - tex[3]);
			if (!a.train_in_linear_colors) {
				tgt = v(l2s(tgt.x), l2s(tgt.y), l2s(tgt.z));
				bg = v(l2s(bg.x), l2s(bg.y), l2s(bg.z));
			}
		} else {
			bg = v(l2s(bg.x), l2s(bg.y), l2s(bg.z));
			tgt = tex[3] > 0 ? v(l2s(tex[0] / tex[3]), l2s(tex[1] / tex[3]), l2s(tex[2] / tex[3])) * tex[3] + bg * (1.0f - tex[3]) : bg;
		}
		if (c == ns) { rr += T * bg.x; rg += T * bg.y; rb += T * bg.z; }
		float lx, ly, lz, gx, gy, gz;
		lossg(tgt.x, rr, a.loss_type, &lx, &gx);
		lossg(tgt.y, rg, a.loss_type, &ly, &gy);
		lossg(tgt.z, rb, a.loss_type, &lz, &gz);
		float* ls = &lstate[8 * (size_t)i];
		ls[0] = gx; ls[1] = gy; ls[2] = gz; ls[3] = rr; ls[4] = rg; ls[5] = rb;
		ls[6] = (lx / pdf + ly / pdf + lz / pdf) / 3.0f;  // lg.loss /= img_pdf * uv_pdf (src/testbed_nerf.cu:1010)
		ls[7] = (float)img;
		if (depth_on && im.depth) {
			const int px = std::min(std::max((int)(u * (float)im.width), 0), (int)im.width - 1);
			const int py = std::min(std::max((int)(vv * (float)im.height), 0), (int)im.height - 1);
			const float target = rdl[i] * reinterpret_cast<const float*>(im.depth)[(size_t)px + (size_t)py * im.width];
			float ld, gd;
			lossg(target, dray, a.depth_loss_type, &ld, &gd);
			ray_depth[i] = dray;
			ray_dlg[i] = target > 0.0f ? a.depth_supervision_lambda * gd : 0.0f;
		}
		if (a.exposure_gradient) {  // src/testbed_nerf.cu:1121-1134, deposited below for kept rays
			const float g[3] = {gx, gy, gz}, t3[3] = {tgt.x, tgt.y, tgt.z};
			for (int k = 0; k < 3; ++k) {
				float d = -g[k] / uv_pdf;
				if (!a.train_in_linear_colors) {
					const float sd = t3[k] <= 0.04045f ? 1.0f / 12.92f : 2.4f / 1.055f * std::pow((t3[k] + 0.055f) / 1.055f, 1.4f);
					d = d / sd;
				}
				expg[3 * (size_t)i + k] = (128.0f / (float)nrg) * d * es[k] * 0.6931471805599453f;
			}
		}
		cc[i] = c;
	}
	M.ray_compacted.assign(2 * (size_t)R, 0);
	M.loss.assign(R, 0.0f);
	M.ccoords.assign(8 * (size_t)B, 0.0f);
	M.dloss.assign(4 * (size_t)B, 0);
	std::vector<float> cenc((size_t)M.L * B * M.F, 0.0f);
	std::vector<float> ccodes(XD ? NGP_EXTRA_ROW * (size_t)B : 0, 0.0f);  // the compacted samples' latent codes
	const float loss_scale = 128.0f / (float)nrg;
	const float l2r = ract == 3 ? 1e-4f : 0.0f;
	const float l1d = M.mean < 0.01f ? 1e-4f : 0.0f;
	uint32_t ctotal = 0;
	for (uint32_t i = 0; i < R; ++i) ctotal += cc[i];
	uint32_t cdp[2];
	const uint32_t Bl = dp_share(a, ctotal, B, cdp);  // the compaction cap of this rank's share
	uint32_t cbase = 0;
	for (uint32_t i = 0; i < R; ++i) {
		const uint32_t c = cc[i], cb = cbase;
		cbase += c;
		const uint32_t cn = c == 0 ? 0 : std::min(Bl - std::min(Bl, cb), c);
		M.ray_compacted[2 * i] = cn;
		M.ray_compacted[2 * i + 1] = cb;
		if (cn == 0) continue;
		const float* ls = &lstate[8 * (size_t)i];
		M.loss[i] = ls[6] / (float)nrg;
		if (a.exposure_gradient)
			for (int k = 0; k < 3; ++k) a.exposure_gradient[3 * (size_t)ls[7] + k] += expg[3 * (size_t)i + k];
		if (a.error_map) {  // bilinear error deposit (src/testbed_nerf.cu:1028-1054)
			const uint32_t gi = a.ray_index_offset + i;
			Pcg rng;
			rng.state = a.rng_state;
			rng.inc = a.rng_inc;
			rng.advance((int64_t)gi * 16);
			float u, vv;
			const uint32_t img = pick_pixel(a, gi, nrg, rng, &u, &vv, nullptr);
			const ngp_image& im = a.images[img];
			const uint32_t ex = a.error_map_res[0], ey = a.error_map_res[1];
			const float px = std::min(std::max(u * (float)ex - 0.5f, 0.0f), (float)ex - (1.0f + 1e-4f));
			const float py = std::min(std::max(vv * (float)ey - 0.5f, 0.0f), (float)ey - (1.0f + 1e-4f));
			const int ix = (int)px, iy = (int)py;
			const float wx = px - (float)ix, wy = py - (float)iy;
			const int cx = std::min(std::max(ix, 0), (int)im.width - 2), cy = std::min(std::max(iy, 0), (int)im.height - 2);
			float* e = a.error_map + (size_t)img * ex * ey;
			float ml = ls[6];
			const V3 hp = ray_hit[i];
			if (sharp_on && box.contains(hp)) {
				const uint32_t srx = a.sharpness_res[0], sry = a.sharpness_res[1];
				const int sx = std::min(std::max((int)(u * (float)srx), 0), (int)srx - 1);
				const int sy = std::min(std::max((int)(vv * (float)sry), 0), (int)sry - 1);
				const float sharp = a.sharpness_data[((size_t)img * sry + sy) * srx + sx] + 1e-6f;
				const uint32_t mip = mip_pos(hp, a.max_cascade);
				float& cell = a.sharpness_grid[(size_t)mip * CELLS + grid_idx(hp, mip)];
				const float old = cell;
				cell = std::max(old, sharp);
				ml *= std::max(sharp / std::max(sharp, old), 0.01f);
			}
			e[cy * ex + cx] += (1.0f - wx) * (1.0f - wy) * ml;
			e[cy * ex + cx + 1] += wx * (1.0f - wy) * ml;
			e[(cy + 1) * ex + cx] += (1.0f - wx) * wy * ml;
			e[(cy + 1) * ex + cx + 1] += wx * wy * ml;
		}
		const uint32_t b0 = M.ray_numsteps[2 * i + 1];
		const V3 o = ro[i];
		float T = 1.0f, r2 = 0, g2 = 0, b2 = 0, d2 = 0;
		for (uint32_t j = 0; j < cn; ++j) {
			const size_t s = b0 + j, dst = cb + j;
			for (int k = 0; k < 8; ++k) M.ccoords[8 * dst + k] = M.coords[8 * s + k];
			for (uint32_t k = 0; k < (XD ? (uint32_t)NGP_EXTRA_ROW : 0u); ++k) ccodes[NGP_EXTRA_ROW * dst + k] = scodes[NGP_EXTRA_ROW * s + k];
			for (uint32_t l = 0; l < M.L; ++l)
				for (uint32_t f = 0; f < M.F; ++f) cenc[((size_t)l * B + dst) * M.F + f] = enc[((size_t)l * S + s) * M.F + f];
			const float* cw = &M.coords[8 * s];
			const V3 pos = box.mn + v(cw[0] * (box.mx.x - box.mn.x), cw[1] * (box.mx.y - box.mn.y), cw[2] * (box.mx.z - box.mn.z));
			const float depth = len(pos - o);
			const float dt = unwarp_dt(cw[3]);
			const float* ob = &out[4 * s];
			const float rgb[3] = {to_rgb(ob[0], ract), to_rgb(ob[1], ract), to_rgb(ob[2], ract)};
			const float alpha = 1.0f - std::exp(-to_density(ob[3], dact) * dt);
			const float w = alpha * T;
			r2 += w * rgb[0]; g2 += w * rgb[1]; b2 += w * rgb[2];
			T *= 1.0f - alpha;
			const float suf[3] = {ls[3] - r2, ls[4] - g2, ls[5] - b2};
			uint16_t* dl = &M.dloss[4 * dst];
			for (int k = 0; k < 3; ++k) dl[k] = f2h(loss_scale * (w * ls[k] * to_rgb_d(ob[k], ract) + std::max(0.0f, l2r * ob[k])));
			d2 += w * depth;
			const float dsup = ray_dlg[i] * (T * depth - (ray_depth[i] - d2));  // depth_supervision (:1098-1100)
			const float ddm = to_density_d(ob[3], dact) * (dt * (ls[0] * (T * rgb[0] - suf[0]) + ls[1] * (T * rgb[1] - suf[1]) + ls[2] * (T * rgb[2] - suf[2]) + dsup));
			dl[3] = f2h(loss_scale * ddm + (ob[3] < 0.0f ? -l1d : 0.0f) + (ob[3] > -10.0f && depth < a.near_distance ? 1e-4f : 0.0f));
		}
	}
	M.total_compacted = cbase;
	M.loss_sum = 0.0f;
	for (float l : M.loss) M.loss_sum += l;

	// Trainer::training_step on the compacted batch; rollover folded into a multiplicity weight
	// (data parallel: this rank's samples are global samples cdp[0] + j of the global batch of cdp[1])
	const uint32_t C = std::min(cbase, Bl), CG = cdp[1];
	std::vector<float> wts(C), dlf(4 * (size_t)C), denc((size_t)M.L * C * M.F, 0.0f), ce((size_t)M.L * C * M.F);
	for (uint32_t j = 0; j < C; ++j) wts[j] = 1.0f + (float)((B - 1 - (cdp[0] + j)) / CG) * ((float)CG / (float)B);
	for (uint32_t j = 0; j < 4 * C; ++j) dlf[j] = h2f(M.dloss[j]);
	for (uint32_t l = 0; l < M.L; ++l)
		for (uint32_t j = 0; j < C; ++j)
			for (uint32_t f = 0; f < M.F; ++f) ce[((size_t)l * C + j) * M.F + f] = cenc[((size_t)l * B + j) * M.F + f];
	const bool ext = a.cam_pos_gradient && a.cam_rot_gradient;
	const bool dist = a.distortion_map && a.distortion_res[0] && a.distortion_res[1] && a.distortion_gradient &&
	                  a.distortion_gradient_weight;
	const bool cam = ext || dist;
	std::vector<float> dsh(cam ? 16 * (size_t)C : 0), dpos(cam ? 3 * (size_t)C : 0);
	const bool xgrad = XD && a.extra_dims_gradient;
	std::vector<float> dextra(xgrad ? NGP_EXTRA_ROW * (size_t)C : 0);
	mlp_backward(M, M.grads.data(), M.p16.data(), ce.data(), M.ccoords.data(), 8, C, dlf.data(), wts.data(), denc.data(),
	             cam ? dsh.data() : nullptr, XD ? ccodes.data() : nullptr, NGP_EXTRA_ROW, xgrad ? dextra.data() : nullptr);
	if (xgrad) {
		// compute_extra_dims_gradient_train_nerf (src/testbed_nerf.cu:1271-1306): each kept ray's compacted samples'
		// dL/d(code) into its image's gradient
		for (uint32_t i = 0; i < R; ++i) {
			const uint32_t cn = M.ray_compacted[2 * i], cb = M.ray_compacted[2 * i + 1];
			if (cn == 0) continue;
			const uint32_t img = (uint32_t)lstate[8 * (size_t)i + 7];
			for (uint32_t k = 0; k < XD; ++k) {
				float g = 0.0f;
				for (uint32_t j = 0; j < cn; ++j) g += dextra[NGP_EXTRA_ROW * ((size_t)cb + j) + k];
				a.extra_dims_gradient[NGP_EXTRA_ROW * (size_t)img + k] += g;
			}
		}
	}
	const float* cml = ml_on ? M.ccoords.data() + 7 : nullptr;
	if (cam) hg_input_grad(M, M.p16.data(), M.ccoords.data(), 8, C, denc.data(), wts.data(), dpos.data(), cml, 8);
	hg_backward(M, M.ccoords.data(), 8, C, denc.data(), cml, 8);
	if (cam) {
		// compute_cam_gradient_train_nerf (src/testbed_nerf.cu:1163-1269), extrinsics part
		const V3 diag = box.mx - box.mn;
		for (uint32_t i = 0; i < R; ++i) {
			const uint32_t cn = M.ray_compacted[2 * i], cb = M.ray_compacted[2 * i + 1];
			if (cn == 0) continue;
			const V3 o = ro[i], d = rd[i];
			V3 go = v(0, 0, 0), gd = v(0, 0, 0);
			for (uint32_t j = 0; j < cn; ++j) {
				const size_t s2 = (size_t)cb + j;
				const float* c = &M.ccoords[8 * s2];
				const V3 pg = v(dpos[3 * s2] / diag.x, dpos[3 * s2 + 1] / diag.y, dpos[3 * s2 + 2] / diag.z);
				go = go + pg;
				const V3 pos = box.mn + v(c[0] * diag.x, c[1] * diag.y, c[2] * diag.z);
				gd = gd + pg * len(pos - o) + sh4_input_grad(c + 4, &dsh[16 * s2]);
			}
			const uint32_t img = (uint32_t)lstate[8 * (size_t)i + 7];
			const float p = ray_uv_pdf[i];
			if (dist) {
				// the direction gradient orthogonal to the direction, in the camera's frame, splatted
				// bilinearly at the pixel (src/testbed_nerf.cu:1234-1246, deposit_image_gradient
				// common_device.cuh:82-115)
				const V3 og = gd - d * dot(gd, d);
				const V3 ip = inv3_mul(cam_of(a.images[img].xform), og);
				const uint32_t rx = a.distortion_res[0], ry = a.distortion_res[1];
				const float fx = (float)rx * ray_uv[2 * i], fy = (float)ry * ray_uv[2 * i + 1];
				const int px = (int)fx, py = (int)fy;
				const float wx = fx - (float)px, wy = fy - (float)py;
				const float val[2] = {ip.x / p, ip.y / p};
				for (int k = 0; k < 4; ++k) {
					const float w = (k & 1 ? wx : 1.0f - wx) * (k & 2 ? wy : 1.0f - wy);
					const int x = std::min(std::max(px + (k & 1), 0), (int)rx - 1), y = std::min(std::max(py + (k >> 1), 0), (int)ry - 1);
					for (int c = 0; c < 2; ++c) {
						a.distortion_gradient[2 * ((size_t)x + (size_t)y * rx) + c] += val[c] * w;
						a.distortion_gradient_weight[2 * ((size_t)x + (size_t)y * rx) + c] += w;
					}
				}
			}
			if (!ext) continue;
			const V3 aa = v(d.y * gd.z - d.z * gd.y, d.z * gd.x - d.x * gd.z, d.x * gd.y - d.y * gd.x);
			a.cam_pos_gradient[3 * img + 0] += go.x / p;
			a.cam_pos_gradient[3 * img + 1] += go.y / p;
			a.cam_pos_gradient[3 * img + 2] += go.z / p;
			a.cam_rot_gradient[3 * img + 0] += aa.x / p;
			a.cam_rot_gradient[3 * img + 1] += aa.y / p;
			a.cam_rot_gradient[3 * img + 2] += aa.z / p;
		}
	}
	if (!a.defer_optimizer) optimizer(M, a.training_step, a.optimize_mlp, a.optimize_encoding);
}

// ---- occupancy grid (testbed_nerf.cu:74-331, 2271-2379) ------------------------------------
static void mark_untrained(Model& M, const ngp_grid_args& a, uint32_t n_elem) {
	for (uint32_t i = 0; i < n_elem; ++i) {
		const uint32_t level = i / CELLS, pi = i % CELLS;
		const float vs = std::scalbn(1.0f / GRID, (int)level);
		const V3 pos = (v((float)morton_inv(pi), (float)morton_inv(pi >> 1), (float)morton_inv(pi >> 2)) * (1.0f / GRID) - v(0.5f, 0.5f, 0.5f)) * std::scalbn(1.0f, (int)level) + v(0.5f, 0.5f, 0.5f);
		uint32_t count = 0;
		for (uint32_t j = 0; j < a.n_images && count < 1; ++j) {
			const ngp_image& im = a.images[j];
			if (im.lens_mode == 2 || im.lens_mode == 3 || im.lens_mode == 5) { ++count; continue; }
			const Cam x = cam_of(im.xform);
			const V3 A = x.c[0], Bv = x.c[1], Cc = x.c[2];
			const V3 bc = v(Bv.y * Cc.z - Bv.z * Cc.y, Bv.z * Cc.x - Bv.x * Cc.z, Bv.x * Cc.y - Bv.y * Cc.x);
			const V3 ca = v(Cc.y * A.z - Cc.z * A.y, Cc.z * A.x - Cc.x * A.z, Cc.x * A.y - Cc.y * A.x);
			const V3 ab = v(A.y * Bv.z - A.z * Bv.y, A.z * Bv.x - A.x * Bv.z, A.x * Bv.y - A.y * Bv.x);
			const float inv = 1.0f / dot(A, bc);
			for (uint32_t k = 0; k < 8; ++k) {
				const V3 corner = pos + v((k & 1) ? vs : 0, (k & 2) ? vs : 0, (k & 4) ? vs : 0);
				const V3 dir = normalize(corner - x.c[3]);
				if (dot(dir, x.c[2]) < 1e-4f) continue;
				// pos_to_uv (common_device.cuh:497-531) with the lens's distortion, then the uv_to_ray check
				const V3 rel = corner - x.c[3];
				const V3 cd = v(dot(bc * inv, rel), dot(ca * inv, rel), dot(ab * inv, rel));
				float cx = cd.x / cd.z, cy = cd.y / cd.z;
				float du = 0.0f, dv = 0.0f;
				if (im.lens_mode == 1 || im.lens_mode == 4) lens_delta(im.lens_mode, im.lens_params, cx, cy, &du, &dv);
				cx += du;
				cy += dv;
				const float u = cx * im.focal_length[0] / (float)im.width + im.principal_point[0];
				const float vv = cy * im.focal_length[1] / (float)im.height + im.principal_point[1];
				V3 rd;
				lens_dir(u, vv, (float)im.width, (float)im.height, im.focal_length[0], im.focal_length[1], im.principal_point[0],
				         im.principal_point[1], im.lens_mode, im.lens_params, &rd);
				rd = normalize(rot(x, rd));
				if (len(rd - dir) < 1e-3f && u > 0 && vv > 0 && u < 1 && vv < 1) { ++count; break; }
			}
		}
		if (a.clear_visible || (M.grid[i] < 0) != (count < 1)) M.grid[i] = count >= 1 ? 0.0f : -1.0f;
	}
}

static void bitfield_update(Model& M, uint32_t max_cascade) {
	unsigned long long sum = 0;
	for (uint32_t i = 0; i < CELLS; ++i) sum += (unsigned long long)(std::min(std::max(M.grid[i], 0.0f), 65536.0f) * 16777216.0f);
	M.mean = (float)((double)sum / 16777216.0 / (double)CELLS);
	const float thresh = std::min(0.01f, M.mean);
	M.bits.assign(CELLS / 8 * CASCADES, 0);
	for (uint32_t i = 0; i < CELLS / 8 * (max_cascade + 1); ++i) {
		uint8_t b = 0;
		for (uint32_t j = 0; j < 8; ++j) b |= M.grid[i * 8 + j] > thresh ? (uint8_t)(1u << j) : 0;
		M.bits[i] = b;
	}
	for (uint32_t level = 1; level < CASCADES; ++level) {
		const uint8_t* prev = &M.bits[(size_t)(level - 1) * CELLS / 8];
		uint8_t* next = &M.bits[(size_t)level * CELLS / 8];
		for (uint32_t i = 0; i < CELLS / 64; ++i) {
			uint8_t b = 0;
			for (uint32_t j = 0; j < 8; ++j) b |= prev[i * 8 + j] > 0 ? (uint8_t)(1u << j) : 0;
			next[morton(morton_inv(i) + 16, morton_inv(i >> 1) + 16, morton_inv(i >> 2) + 16)] |= b;
		}
	}
}

// Sampling + density evaluation + max-splat into tmp.  Data-parallel form: this rank
// evaluates the contiguous 1/world_size slice of the samples (as density_grid.hip does);
// the caller max-reduces tmp over ranks before grid_finish.
static void grid_evaluate(Model& M, const ngp_grid_args& a) {
	const uint32_t nc = a.max_cascade + 1, ne = CELLS * nc;
	if (M.grid.size() < ne) M.grid.resize(ne, 0.0f);
	if (a.mark_untrained) mark_untrained(M, a, ne);
	M.tmp.assign(ne, 0.0f);
	const Box box{v(a.aabb_min[0], a.aabb_min[1], a.aabb_min[2]), v(a.aabb_max[0], a.aabb_max[1], a.aabb_max[2])};
	Pcg rng;
	rng.state = a.rng_state;
	rng.inc = a.rng_inc;
	const uint32_t ntot = a.n_uniform_samples + a.n_nonuniform_samples;
	std::vector<float> pos(4 * (size_t)ntot);
	std::vector<uint32_t> idxs(ntot);
	for (int pass = 0; pass < 2; ++pass) {
		const uint32_t n = pass == 0 ? a.n_uniform_samples : a.n_nonuniform_samples;
		const float thresh = pass == 0 ? -0.01f : 0.01f;
		const uint32_t first = pass == 0 ? 0 : a.n_uniform_samples;
		for (uint32_t i = 0; i < n; ++i) {
			Pcg r = rng;
			r.advance((int64_t)i * 4);
			const uint32_t level = (uint32_t)(r.nextf() * (float)nc) % nc;
			uint32_t idx = 0;
			for (uint32_t j = 0; j < 10; ++j) {
				idx = ((i + a.ema_step * n) * 56924617u + j * 19349663u + 96925573u) % CELLS;
				idx += level * CELLS;
				if (M.grid[idx] > thresh) break;
			}
			const uint32_t pi = idx % CELLS;
			const float r0 = r.nextf(), r1 = r.nextf(), r2 = r.nextf();
			const V3 p = (v(((float)morton_inv(pi) + r0) / GRID, ((float)morton_inv(pi >> 1) + r1) / GRID, ((float)morton_inv(pi >> 2) + r2) / GRID) - v(0.5f, 0.5f, 0.5f)) * std::scalbn(1.0f, (int)level) + v(0.5f, 0.5f, 0.5f);
			const V3 w = box.rel(p);
			float* q = &pos[4 * (size_t)(first + i)];
			q[0] = w.x; q[1] = w.y; q[2] = w.z; q[3] = warp_dt(MIN_STEP);
			idxs[first + i] = idx;
		}
		rng.advance();
	}
	// density (NerfNetwork::density, training params) and max-splat over this rank's slice
	const uint32_t world = std::max(a.world_size, 1u);
	const uint32_t per = (ntot + world - 1) / world;
	const uint32_t first = std::min(ntot, a.rank * per), cnt = std::min(ntot - first, per);
	const std::vector<uint16_t>& P = a.use_inference_params ? M.inf16 : M.p16;
	std::vector<float> enc((size_t)M.L * ntot * M.F);
	hg_forward(M, P.data(), pos.data(), 4, ntot, enc.data());
	std::vector<float> col(M.E);
	Acts A;
	for (uint32_t i = first; i < first + cnt; ++i) {
		gather_enc(M, enc.data(), ntot, i, col.data());
		// density MLP only
		std::vector<float> x(M.Epad, 0.0f), y;
		for (uint32_t k = 0; k < M.E; ++k) x[k] = col[k];
		for (uint32_t l = 0; l < M.n_density_layers; ++l) {
			layer_fwd(M, P.data(), M.layers[l], x, y, true);
			x = y;
		}
		const float th = to_density(x[0], M.cfg.density_activation) * MIN_STEP;
		M.tmp[idxs[i]] = std::max(M.tmp[idxs[i]], th);
	}
}

// EMA of the grid with tmp + mean/bitfield (ema_grid_samples_nerf, update_density_grid_mean_and_bitfield)
static void grid_finish(Model& M, const ngp_grid_args& a) {
	const uint32_t ne = CELLS * (a.max_cascade + 1);
	for (uint32_t i = 0; i < ne; ++i) {
		const float prev = M.grid[i];
		M.grid[i] = prev < 0.0f ? prev : std::max(prev * a.decay, M.tmp[i]);
	}
	bitfield_update(M, a.max_cascade);
}

// ---- tracer (render_nerf, NerfTracer::trace; per ray, chunking-invariant) ---------------------
// 0: the lattice march (the HIP path's formulation, exact per sample); 1: the reference's literal
// float-chained march (ref_render_ray) -- oref_set_render_literal
static int g_render_literal = 0;
// square2disk_shirley (random_val.cuh:112-128)
static void disk_shirley(float a, float b, float* x, float* y) {
	const float PI = 3.14159265358979323846f;
	float phi, r;
	if (a * a > b * b) {
		r = a;
		phi = (PI / 4.0f) * (b / a);
	} else {
		r = b;
		phi = (PI / 2.0f) - (PI / 4.0f) * (a / b);
	}
	*x = r * std::cos(phi);
	*y = r * std::sin(phi);
}

// d(raw density)/d(warped position) of one sample (network->input_gradient, the Normals mode's input;
// src/testbed_nerf.cu:1715-1717): MLP backward from dL/dout = (0, 0, 0, 1), then the grid's input gradient
static V3 density_gradient(const Model& M, const uint16_t* P, const float* coord, std::vector<float>& gscratch) {
	std::vector<float> enc(M.L * M.F), denc(M.L * M.F);
	hg_forward(M, P, coord, 8, 1, enc.data());
	const float dl[4] = {0.0f, 0.0f, 0.0f, 1.0f};
	mlp_backward(M, gscratch.data(), P, enc.data(), coord, 8, 1, dl, nullptr, denc.data());
	float g[3];
	hg_input_grad(M, P, coord, 8, 1, denc.data(), nullptr, g);
	return v(g[0], g[1], g[2]);
}

// composite_kernel_nerf's glow (src/testbed_nerf.cu:540-628, the active branch): a grid and a cut line
// below glow_y_cutoff added to the colour (replacing it in grid mode); mask_to_alpha scales the weight.
static void glow(const ngp_render_args& a, V3 pos, V3 cam_pos, V3* rgb, float* weight) {
	const int gm = a.glow_mode;
	const bool green_grid = gm & 1, green_cutline = gm & 2, mask_to_alpha = gm & 4, radial_mode = gm & 8, grid_mode = gm & 16;
	float g = 0.0f;
	float dist;
	if (radial_mode) {
		dist = len(pos - cam_pos);
		dist = std::min(dist, (4.5f - pos.y) * 0.333f);
	} else {
		dist = pos.y;
	}
	if (grid_mode) {
		g = 1.0f / std::max(1.0f, dist);
	} else {
		float y = a.glow_y_cutoff - dist;
		float mask = 0.0f;
		if (y > 0.0f) {
			y *= 80.0f;
			mask = std::min(1.0f, y);
			if (green_cutline) g += std::max(0.0f, 1.0f - std::fabs(1.0f - y)) * 4.0f;
			if (y > 1.0f) y = 1.0f - (y - 1.0f) * 0.05f;
			if (green_grid) g += std::max(0.0f, y / std::max(1.0f, dist));
		}
		if (mask_to_alpha) *weight *= mask;
	}
	if (g > 0.0f) {
		const float PI = 3.141592653589793f;
		float line = 0.0f;
		for (float f : {2.0f, 4.0f, 8.0f, 16.0f}) {
			line += std::max(0.0f, std::cos(pos.y * f * PI * 16.0f) - 0.975f);
			line += std::max(0.0f, std::cos(pos.x * f * PI * 16.0f) - 0.975f);
			line += std::max(0.0f, std::cos(pos.z * f * PI * 16.0f) - 0.975f);
		}
		if (grid_mode) {
			g = g * line * 15.0f;
			*rgb = v(g * 0.25f, g, g * 0.5f);
		} else {
			g = g * g * 0.25f + g * line * 15.0f;
			*rgb = v(rgb->x + g * 0.25f, rgb->y + g, rgb->z + g * 0.5f);
		}
	}
}

// uv_to_ray + init_rays_with_payload_kernel_nerf's ray (src/testbed_nerf.cu:1408-1441, common_device.cuh:441-459)
// of pixel (x, y): lens, learned distortion, the pixel's (rolling-shutter) camera, depth of field, near
// distance; the direction is not normalised.  false: the lens has no ray for the pixel.
static bool pixel_camera_ray(const ngp_render_args& a, const Cam& cam, uint32_t x, uint32_t y, float ox, float oy, float aperture,
                             V3* o_out, V3* d_out) {
	const uint32_t idx = x + a.width * y;
	const float u = ((float)x + ox) / (float)a.width, vv = ((float)y + oy) / (float)a.height;
	V3 d;
	if (!lens_dir(u, vv, (float)a.width, (float)a.height, a.focal_length[0], a.focal_length[1], a.screen_center[0],
	              a.screen_center[1], a.lens_mode, a.lens_params, &d))
		return false;
	if (a.distortion_map && a.distortion_res[0] && a.distortion_res[1]) {
		float ddx, ddy;
		distortion_lerp(a.distortion_map, a.distortion_res[0], a.distortion_res[1], u, vv, &ddx, &ddy);
		d.x += ddx;
		d.y += ddy;
	}
	// the pixel's camera (src/testbed_nerf.cu:1416)
	const Cam pc = rs_on(a.rolling_shutter)
	                   ? slerp_cam(cam, cam_of(a.camera_end), a.rolling_shutter[0] + a.rolling_shutter[1] * u + a.rolling_shutter[2] * vv +
	                                                              a.rolling_shutter[3] * ldval(a.sample_index, idx * 72239731u, 0))
	                   : cam;
	d = rot(pc, d);
	V3 o = pc.c[3];
	if (aperture != 0.0f) {  // depth of field (uv_to_ray, common_device.cuh:450-456)
		const V3 lookat = o + d * a.focus_z;
		const uint32_t px = (uint32_t)(int)(u * (float)a.width), py = (uint32_t)(int)(vv * (float)a.height);
		const uint32_t seed = px * 19349663u + py * 96925573u;
		float dx, dy;
		disk_shirley(ldval(a.sample_index, seed, 0) * 2.0f - 1.0f, ldval(a.sample_index, seed, 1) * 2.0f - 1.0f, &dx, &dy);
		o = o + pc.c[0] * (aperture * dx) + pc.c[1] * (aperture * dy);
		d = (lookat - o) * (1.0f / a.focus_z);
	}
	*o_out = o + d * a.near_distance;
	*d_out = d;
	return true;
}

// render_nerf (src/testbed_nerf.cu:1827-1987): per pixel, the NerfTracer march and composite of every
// render mode but Distortion / EncodingVis, then shade_kernel_nerf; Slice evaluates one point per pixel.
static void render(const Model& M, const ngp_render_args& a, float* frame, float* depthbuf) {
	const RBox box = rbox_of(Box{v(a.aabb_min[0], a.aabb_min[1], a.aabb_min[2]), v(a.aabb_max[0], a.aabb_max[1], a.aabb_max[2])},
	                         a.render_aabb_to_local);
	const Box tbox{v(a.train_aabb_min[0], a.train_aabb_min[1], a.train_aabb_min[2]), v(a.train_aabb_max[0], a.train_aabb_max[1], a.train_aabb_max[2])};
	const Cam cam = cam_of(a.camera);
	const uint16_t* P = a.use_inference_params ? M.inf16.data() : M.p16.data();
	const Stepping stp = make_stepping(a.cone_angle_constant);
	const int ract = M.cfg.rgb_activation, dact = M.cfg.density_activation;
	const int mode = a.render_mode;
	const float aperture = mode == NGP_RENDER_MODE_SLICE ? 0.0f : a.aperture_size;
	const uint32_t sc = std::max(a.shard_count, 1u), sr = std::max(a.shard_rows, 1u), si = a.shard_index % sc;
	float ox, oy;
	pixel_offset(a.snap_to_pixel_centers ? 0 : a.sample_index, &ox, &oy);
	// rows are independent (the all-core CPU baseline); dynamic: rows differ in cost
#pragma omp parallel
	{
	std::vector<float> enc(M.L * M.F), col(M.E), out(4), gscratch(mode == NGP_RENDER_MODE_NORMALS ? M.n_mlp : 0);
#pragma omp for schedule(dynamic, 1)
	for (uint32_t y = 0; y < a.height; ++y) {
		if ((y / sr) % sc != si) continue;
		for (uint32_t x = 0; x < a.width; ++x) {
			const uint32_t idx = x + a.width * y;
			float* fb = frame + 4 * (size_t)idx;
			fb[0] = fb[1] = fb[2] = fb[3] = 0.0f;
			depthbuf[idx] = MAXD;
			V3 o, d;
			if (!pixel_camera_ray(a, cam, x, y, ox, oy, aperture, &o, &d)) continue;  // invalid ray: the pixel stays empty
			if (mode == NGP_RENDER_MODE_SLICE) {
				// one point per pixel at camera depth focus_z, compute_nerf_rgba with depth 0.01, shade (Slice)
				const V3 pos = o + d * a.focus_z;
				const V3 dn = normalize(d);
				const V3 w = tbox.rel(pos);
				float coord[8] = {w.x, w.y, w.z, warp_dt(MIN_STEP), (dn.x + 1) * 0.5f, (dn.y + 1) * 0.5f, (dn.z + 1) * 0.5f, 0.0f};
				hg_forward(M, P, coord, 8, 1, enc.data());
				mlp_forward(M, P, enc.data(), coord, 8, 1, out.data(), a.extra_dims, 0);
				const float alpha = std::min(std::max(1.0f - std::exp(-to_density(out[3], dact) * 0.01f), 0.0f), 1.0f);
				float c[4] = {to_rgb(out[0], ract) * alpha, to_rgb(out[1], ract) * alpha, to_rgb(out[2], ract) * alpha, alpha};
				if (!a.train_in_linear_colors) for (int k = 0; k < 3; ++k) c[k] = s2l(c[k]);
				for (int k = 0; k < 4; ++k) fb[k] = c[k];
				depthbuf[idx] = a.focus_z;
				continue;
			}
			d = normalize(d);
			float t0, t1;
			box.b.intersect(box.local(o), box.local(d), &t0, &t1);
			float t = std::max(t0, 0.0f) + 1e-6f;
			if (!box.contains(o + d * t)) continue;
			const V3 idir = v(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
			const float jitter = ldval(a.sample_index, idx * 786433u, 0);
			float c[4] = {0, 0, 0, 0}, maxw = 0.0f, dep = 0.0f;
			float cost = 0.0f;
			uint32_t j = 0;
			const V3 wd = v((d.x + 1) * 0.5f, (d.y + 1) * 0.5f, (d.z + 1) * 0.5f);
			// composite_kernel_nerf for one sample at (t, dt); false once the ray is opaque enough
			auto composite = [&](float ts, float dt) -> bool {
				const V3 w = tbox.rel(o + d * ts);
				float coord[8] = {w.x, w.y, w.z, warp_dt(dt), wd.x, wd.y, wd.z, 0.0f};
				hg_forward(M, P, coord, 8, 1, enc.data());
				mlp_forward(M, P, enc.data(), coord, 8, 1, out.data(), a.extra_dims, 0);
				const V3 pos = tbox.mn + v(coord[0] * (tbox.mx.x - tbox.mn.x), coord[1] * (tbox.mx.y - tbox.mn.y), coord[2] * (tbox.mx.z - tbox.mn.z));
				const float T = 1.0f - c[3];
				const float alpha = 1.0f - std::exp(-to_density(out[3], dact) * unwarp_dt(coord[3]));
				float wgt = alpha * T;
				V3 rgb = v(to_rgb(out[0], ract), to_rgb(out[1], ract), to_rgb(out[2], ract));
				if (a.glow_mode) glow(a, pos, cam.c[3], &rgb, &wgt);
				if (mode == NGP_RENDER_MODE_NORMALS) {
					const V3 g = density_gradient(M, P, coord, gscratch) * -to_density_d(out[3], dact);
					rgb = normalize(g);
				} else if (mode == NGP_RENDER_MODE_POSITIONS) {
					rgb = (pos - 0.5f) * 0.5f + 0.5f;
				} else if (mode == NGP_RENDER_MODE_DEPTH) {
					const float dv = dot(cam.c[2], pos - o) * a.depth_scale;
					rgb = v(dv, dv, dv);
				} else if (mode == NGP_RENDER_MODE_AO) {
					rgb = v(alpha, alpha, alpha);
				}
				if (mode != NGP_RENDER_MODE_COST) {
					c[0] += rgb.x * wgt;
					c[1] += rgb.y * wgt;
					c[2] += rgb.z * wgt;
				}
				c[3] += wgt;
				if (wgt > maxw) { maxw = wgt; dep = dot(cam.c[2], pos - cam.c[3]); }
				if (c[3] > 1.0f - a.min_transmittance) {
					const float inv = 1.0f / c[3];
					if (mode != NGP_RENDER_MODE_COST) for (int k = 0; k < 3; ++k) c[k] *= inv;
					c[3] *= inv;
					return false;
				}
				++j;
				return true;
			};
			if (g_render_literal) {
				// the reference's own float-chained march (ref_render_ray), 8 samples per pass
				if (ref_render_ray(t, jitter, a.cone_angle_constant, o, d, M.bits.data(), a.max_cascade, box, 8, 10000, composite) == 0) continue;
			} else {
				float n = lat_to(stp, t) + jitter;
				if (!next_occupied(&n, stp, o, d, idir, M.bits.data(), a.max_cascade, box)) continue;
				for (uint32_t step = 0; step < 10000; ++step) {
					if (!next_occupied(&n, stp, o, d, idir, M.bits.data(), a.max_cascade, box)) break;
					const float ts = lat_from(stp, n);
					const float dt = lat_from(stp, n + 1.0f) - ts;
					n += 1.0f;
					if (!composite(ts, dt)) break;
				}
			}
			// Cost: the reference's payload.n_steps -- the index of the terminating sample, or every
			// composited sample of a ray that left the volume (src/testbed_nerf.cu:664-667)
			cost = (float)j;
			if (!(c[3] > 0.001f)) continue;  // compact_kernel_nerf drops near-transparent rays
			// shade_kernel_nerf (src/testbed_nerf.cu:1309-1349)
			if (mode == NGP_RENDER_MODE_NORMALS) {
				const V3 nn = normalize(v(c[0], c[1], c[2]));
				c[0] = (0.5f * nn.x + 0.5f) * c[3];
				c[1] = (0.5f * nn.y + 0.5f) * c[3];
				c[2] = (0.5f * nn.z + 0.5f) * c[3];
			} else if (mode == NGP_RENDER_MODE_COST) {
				const float cc = cost / 128.0f;
				c[0] = c[1] = c[2] = cc;
				c[3] = 1.0f;
			} else if (a.gbuffer_hard_edges && mode == NGP_RENDER_MODE_DEPTH) {
				c[0] = c[1] = c[2] = dep * a.depth_scale;
			} else if (a.gbuffer_hard_edges && mode == NGP_RENDER_MODE_POSITIONS) {
				const V3 p3 = cam.c[3] + d * (dep / dot(d, cam.c[2]));
				c[0] = (p3.x - 0.5f) * 0.5f + 0.5f;
				c[1] = (p3.y - 0.5f) * 0.5f + 0.5f;
				c[2] = (p3.z - 0.5f) * 0.5f + 0.5f;
			}
			if (!a.train_in_linear_colors && mode == NGP_RENDER_MODE_SHADE) for (int k = 0; k < 3; ++k) c[k] = s2l(c[k]);
			for (int k = 0; k < 4; ++k) fb[k] = c[k];
			if (c[3] > 0.2f) depthbuf[idx] = dep;
		}
	}
	}
}

}  // namespace oref

using namespace oref;

static thread_local std::string g_err;
template <class F>
static int guard(F&& f) {
	try { f(); return 0; } catch (const std::exception& e) { g_err = e.what(); return 1; }
}

extern "C" {

// threads of the parallel loops (render rows, encoding, inference); 1 by default so the tests
// run the scalar oracle; the bench's all-core CPU baseline raises it
void oref_set_threads(int n) { omp_set_num_threads(n > 0 ? n : 1); }
uint32_t oref_hardware_concurrency(void) { return std::thread::hardware_concurrency(); }

const char* oref_last_error(void) { return g_err.c_str(); }

// Known-answer helpers
void oref_pcg32(uint64_t seed, uint64_t seq, uint32_t n, uint32_t* out) {
	Pcg r;
	r.seed(seed, seq);
	for (uint32_t i = 0; i < n; ++i) out[i] = r.next();
}
void oref_pcg32_floats_advanced(uint64_t state, uint64_t inc, int64_t adv, uint32_t n, float* out) {
	Pcg r;
	r.state = state;
	r.inc = inc;
	r.advance(adv);
	for (uint32_t i = 0; i < n; ++i) out[i] = r.nextf();
}
float oref_ld_random_val(uint32_t index, uint32_t seed, uint32_t dim) { return ldval(index, seed, dim); }

// camera-space direction of a screen position under a lens (uv_to_ray's direction part)
int oref_lens_direction(float u, float v, float rx, float ry, float fx, float fy, float cx, float cy, int mode,
                        const float* params, float* dir3) {
	V3 d;
	const bool ok = lens_dir(u, v, rx, ry, fx, fy, cx, cy, mode, params, &d);
	dir3[0] = d.x;
	dir3[1] = d.y;
	dir3[2] = d.z;
	return ok ? 1 : 0;
}

// the training ray's image and pixel (image_idx + nerf_random_image_pos_training, with the
// error-map CDFs when given) -- exposed for the sampling tests
uint32_t oref_pick_pixel(const ngp_train_args* a, uint32_t gi, float* u, float* v, float* pdf) {
	Pcg rng;
	rng.state = a->rng_state;
	rng.inc = a->rng_inc;
	rng.advance((int64_t)gi * 16);
	return pick_pixel(*a, gi, a->n_rays_global ? a->n_rays_global : a->n_rays, rng, u, v, pdf);
}

// construct_cdf_2d / construct_cdf_1d (src/testbed_nerf.cu:1493-1546), host arrays
void oref_error_map_build_cdf(const float* data, uint32_t n_images, uint32_t rx, uint32_t ry, float* cdf_x_cond_y,
                              float* cdf_y, float* cdf_img) {
	const float MIN_PDF = 0.01f;
	for (uint32_t img = 0; img < n_images; ++img) {
		for (uint32_t y = 0; y < ry; ++y) {
			const size_t off = ((size_t)img * ry + y) * rx;
			float cum = 0.0f;
			for (uint32_t x = 0; x < rx; ++x) {
				cum += data[off + x] + 1e-10f;
				cdf_x_cond_y[off + x] = cum;
			}
			cdf_y[(size_t)img * ry + y] = cum;
			const float norm = 1.0f / cum;
			for (uint32_t x = 0; x < rx; ++x)
				cdf_x_cond_y[off + x] = (1.0f - MIN_PDF) * cdf_x_cond_y[off + x] * norm + MIN_PDF * (float)(x + 1) / (float)rx;
		}
		float* cy = cdf_y + (size_t)img * ry;
		float cum = 0.0f;
		for (uint32_t y = 0; y < ry; ++y) {
			cum += cy[y];
			cy[y] = cum;
		}
		cdf_img[img] = cum;
		const float norm = 1.0f / cum;
		for (uint32_t y = 0; y < ry; ++y) cy[y] = (1.0f - MIN_PDF) * cy[y] * norm + MIN_PDF * (float)(y + 1) / (float)ry;
	}
}
uint32_t oref_sobol(uint32_t index, uint32_t dim) { return sobol(index, dim); }
uint32_t oref_morton3D(uint32_t x, uint32_t y, uint32_t z) { return morton(x, y, z); }
void oref_sh4(const float* wdir, float* out) { sh4(wdir, out); }
uint16_t oref_f2h(float f) { return f2h(f); }
float oref_h2f(uint16_t h) { return h2f(h); }

void* oref_model_create(const ngp_network_config* cfg) {
	auto* M = new Model();
	M->cfg = *cfg;
	build(*M);
	return M;
}
void oref_model_destroy(void* m) { delete static_cast<Model*>(m); }
uint64_t oref_model_n_params(void* m) { return static_cast<Model*>(m)->n; }
uint64_t oref_model_n_mlp_params(void* m) { return static_cast<Model*>(m)->n_mlp; }
void oref_model_level_table(void* m, float* scale, uint32_t* res, uint32_t* offset, uint32_t* size, uint32_t* hashed) {
	Model& M = *static_cast<Model*>(m);
	for (uint32_t l = 0; l < M.L; ++l) {
		scale[l] = M.scale[l]; res[l] = M.res[l]; offset[l] = M.offset[l]; size[l] = M.size[l]; hashed[l] = M.hashed[l];
	}
}
// set fp32 master params; fp16 copies derived; optimizer reset (EMA = params)
void oref_model_set_params(void* m, const float* p) {
	Model& M = *static_cast<Model*>(m);
	for (uint64_t i = 0; i < M.n; ++i) {
		M.p32[i] = p[i];
		M.p16[i] = f2h(p[i]);
		M.ema32[i] = p[i];
		M.inf16[i] = M.p16[i];
		M.m[i] = M.vv[i] = 0.0f;
		M.steps[i] = 0;
		M.grads[i] = 0.0f;
	}
	M.ema_step = 0;
}
// the EMA weights of a trained model: the fp16 inference params (use_inference_params) derived from them
void oref_model_set_inference_params(void* m, const float* ema) {
	Model& M = *static_cast<Model*>(m);
	for (uint64_t i = 0; i < M.n; ++i) {
		M.ema32[i] = ema[i];
		M.inf16[i] = f2h(ema[i]);
	}
}
void oref_model_get(void* m, int kind, void* out) {
	Model& M = *static_cast<Model*>(m);
	switch (kind) {
		case NGP_PARAMS_FP32: std::memcpy(out, M.p32.data(), M.n * 4); break;
		case NGP_PARAMS_FP16: std::memcpy(out, M.p16.data(), M.n * 2); break;
		case NGP_PARAMS_EMA_FP32: std::memcpy(out, M.ema32.data(), M.n * 4); break;
		case NGP_PARAMS_INFER_FP16: std::memcpy(out, M.inf16.data(), M.n * 2); break;
		case NGP_GRADS_FP32: std::memcpy(out, M.grads.data(), M.n * 4); break;
		default: break;
	}
}
void oref_zero_grads(void* m) { auto& M = *static_cast<Model*>(m); std::fill(M.grads.begin(), M.grads.end(), 0.0f); }
void oref_model_set_grads(void* m, const float* g) {
	Model& M = *static_cast<Model*>(m);
	std::memcpy(M.grads.data(), g, M.n * 4);
}

void oref_encode(void* m, const float* pos, uint32_t stride, uint32_t n, float* enc, int use_inf) {
	Model& M = *static_cast<Model*>(m);
	hg_forward(M, use_inf ? M.inf16.data() : M.p16.data(), pos, stride, n, enc);
}
void oref_encode_indices(void* m, const float* pos, uint32_t stride, uint32_t n, uint32_t* idx, float* w) {
	Model& M = *static_cast<Model*>(m);
	for (uint32_t i = 0; i < n; ++i)
		for (uint32_t l = 0; l < M.L; ++l) {
			uint32_t ix[8];
			float ww[8];
			hg_corners(M, l, pos + (size_t)i * stride, ix, ww);
			for (int c = 0; c < 8; ++c) {
				idx[((size_t)i * M.L + l) * 8 + c] = M.offset[l] + ix[c];
				w[((size_t)i * M.L + l) * 8 + c] = ww[c];
			}
		}
}
void oref_infer(void* m, const float* coords, uint32_t fpc, uint32_t n, float* out, int use_inf) {
	Model& M = *static_cast<Model*>(m);
	const uint16_t* P = use_inf ? M.inf16.data() : M.p16.data();
	std::vector<float> enc((size_t)M.L * n * M.F);
	hg_forward(M, P, coords, fpc, n, enc.data());
	// n_extra_dims > 0: the records' extra dims (floats 7 .. 7 + n_extra_dims) are the latent codes
	mlp_forward(M, P, enc.data(), coords, fpc, n, out, M.cfg.n_extra_dims ? coords + 7 : nullptr, fpc);
}
// the reference's padded network output: 16 rows per sample, row 3 = density (extract_density)
void oref_infer_padded(void* m, const float* coords, uint32_t fpc, uint32_t n, float* out16, int use_inf) {
	Model& M = *static_cast<Model*>(m);
	const uint16_t* P = use_inf ? M.inf16.data() : M.p16.data();
	std::vector<float> enc((size_t)M.L * n * M.F), col(M.E);
	hg_forward(M, P, coords, fpc, n, enc.data());
	Acts A;
	const uint32_t NL = (uint32_t)M.layers.size();
	for (uint32_t i = 0; i < n; ++i) {
		gather_enc(M, enc.data(), n, i, col.data());
		mlp_forward_one(M, P, col.data(), coords + (size_t)i * fpc + 4, A, M.cfg.n_extra_dims ? coords + (size_t)i * fpc + 7 : nullptr);
		for (uint32_t r = 0; r < 16; ++r) out16[16 * (size_t)i + r] = A.a[NL][r];
		out16[16 * (size_t)i + 3] = A.a[M.n_density_layers][0];
	}
}
void oref_mlp_forward_enc(void* m, const float* enc, const float* coords, uint32_t fpc, uint32_t n, float* out) {
	Model& M = *static_cast<Model*>(m);
	mlp_forward(M, M.p16.data(), enc, coords, fpc, n, out);
}
void oref_density(void* m, const float* pos, uint32_t stride, uint32_t n, float* out, int use_inf) {
	Model& M = *static_cast<Model*>(m);
	const uint16_t* P = use_inf ? M.inf16.data() : M.p16.data();
	std::vector<float> enc((size_t)M.L * n * M.F), col(M.E);
	hg_forward(M, P, pos, stride, n, enc.data());
	for (uint32_t i = 0; i < n; ++i) {
		gather_enc(M, enc.data(), n, i, col.data());
		std::vector<float> x(M.Epad, 0.0f), y;
		for (uint32_t k = 0; k < M.E; ++k) x[k] = col[k];
		for (uint32_t l = 0; l < M.n_density_layers; ++l) { layer_fwd(M, P, M.layers[l], x, y, true); x = y; }
		out[i] = x[0];
	}
}
// enc [L][n][F] floats (fp16 values), dirs [n][3] warped, dloss [n][4] (fp16 values)
void oref_backward(void* m, const float* enc, const float* dirs, uint32_t n, const float* dloss, const float* weight, float* denc) {
	Model& M = *static_cast<Model*>(m);
	std::vector<float> coords(8 * (size_t)n, 0.0f);
	for (uint32_t i = 0; i < n; ++i) for (int k = 0; k < 3; ++k) coords[8 * i + 4 + k] = dirs[3 * i + k];
	mlp_backward(M, M.grads.data(), M.p16.data(), enc, coords.data(), 8, n, dloss, weight, denc);
}
// the same with latent codes extra [n][NGP_EXTRA_ROW] and their input gradient dextra [n][NGP_EXTRA_ROW] (optional)
void oref_backward_extra(void* m, const float* enc, const float* dirs, const float* extra, uint32_t n, const float* dloss,
                         const float* weight, float* denc, float* dextra) {
	Model& M = *static_cast<Model*>(m);
	std::vector<float> coords(8 * (size_t)n, 0.0f);
	for (uint32_t i = 0; i < n; ++i) for (int k = 0; k < 3; ++k) coords[8 * i + 4 + k] = dirs[3 * i + k];
	mlp_backward(M, M.grads.data(), M.p16.data(), enc, coords.data(), 8, n, dloss, weight, denc, nullptr, extra, NGP_EXTRA_ROW, dextra);
}
void oref_encode_backward(void* m, const float* pos, uint32_t stride, uint32_t n, const float* denc) {
	hg_backward(*static_cast<Model*>(m), pos, stride, n, denc);
}
// Test hook: training ray i's sample parameters -- mode 0: the lattice walk (fast path), as
// stepping-space positions n0 + k; mode 1: the literal transcription of the reference's loop
// (chained t += calc_dt(t), advance_to_next_voxel), as stepping-space positions to(t).
// Returns the sample count (<= cap), writes min(count, cap) values and *n0 (the lattice origin).
uint32_t oref_train_ray_samples(void* m, const ngp_train_args* a, uint32_t i, int mode, float* out, uint32_t cap, float* n0_out) {
	Model& M = *static_cast<Model*>(m);
	const uint32_t nrg = a->n_rays_global ? a->n_rays_global : a->n_rays;
	const Box box{v(a->aabb_min[0], a->aabb_min[1], a->aabb_min[2]), v(a->aabb_max[0], a->aabb_max[1], a->aabb_max[2])};
	const Stepping stp = make_stepping(a->cone_angle_constant);
	V3 o, d;
	float n0, t0, r;
	if (!train_ray(*a, a->ray_index_offset + i, nrg, &o, &d, &n0, &t0, &r)) return 0;
	if (n0_out) *n0_out = n0;
	if (mode == 0)
		return training_walk(stp, box, M.bits.data(), a->max_cascade, o, d, n0, std::min(cap, STEPS),
		                     [&](uint32_t j, uint32_t k, float, float, V3) { out[j] = n0 + (float)k; });
	const float cone = a->cone_angle_constant;
	const V3 idir = v(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
	float t = ref_advance_n_steps(t0, cone, r);
	uint32_t j = 0;
	V3 pos;
	while (box.contains(pos = o + d * t) && j < std::min(cap, STEPS)) {
		const float dt = ref_calc_dt(t, cone);
		const uint32_t mip = mip_dt(dt, pos, a->max_cascade);
		if (occupied(pos, M.bits.data(), mip)) {
			out[j++] = ref_to_stepping_space(t, cone);
			t += dt;
		} else {
			t = ref_advance_to_next_voxel(t, cone, pos, d, idir, mip);
		}
	}
	return j;
}

void oref_set_render_literal(int on) { g_render_literal = on ? 1 : 0; }
// Test hook: the render march of pixel (x, y) -- mode 0: the lattice march render() uses, as stepping-space
// positions n; mode 1: the reference's literal march (ref_render_ray, n_steps samples per pass), as
// to_stepping_space(t).  Both march to the box exit (no composite stop).  Returns the sample count
// (<= cap), writes min(count, cap) values and the lattice origin n0 = to_stepping_space(t_start) + jitter.
// trace_out (mode 1, optional): every point the literal march visits, [k][3] = stepping position, distance
// to the nearest cell face at the mip the point was decided at (in cells), occupied; *trace_n in: capacity,
// out: points written.
uint32_t oref_render_ray_samples(void* m, const ngp_render_args* a, uint32_t x, uint32_t y, int mode, uint32_t n_steps,
                                 float* out, uint32_t cap, float* n0_out, float* trace_out, uint32_t* trace_n) {
	Model& M = *static_cast<Model*>(m);
	const RBox box = rbox_of(Box{v(a->aabb_min[0], a->aabb_min[1], a->aabb_min[2]), v(a->aabb_max[0], a->aabb_max[1], a->aabb_max[2])},
	                         a->render_aabb_to_local);
	const Stepping stp = make_stepping(a->cone_angle_constant);
	float ox, oy;
	pixel_offset(a->snap_to_pixel_centers ? 0 : a->sample_index, &ox, &oy);
	V3 o, d;
	if (!pixel_camera_ray(*a, cam_of(a->camera), x, y, ox, oy, a->aperture_size, &o, &d)) { if (trace_n) *trace_n = 0; return 0; }
	d = normalize(d);
	float t0, t1;
	box.b.intersect(box.local(o), box.local(d), &t0, &t1);
	const float t = std::max(t0, 0.0f) + 1e-6f;
	if (!box.contains(o + d * t)) { if (trace_n) *trace_n = 0; return 0; }
	const float jitter = ldval(a->sample_index, (x + a->width * y) * 786433u, 0);
	if (n0_out) *n0_out = lat_to(stp, t) + jitter;
	if (mode == 1) {
		MarchTrace tr;
		const uint32_t c = ref_render_ray(t, jitter, a->cone_angle_constant, o, d, M.bits.data(), a->max_cascade, box, std::max(n_steps, 1u),
		                                  cap, [&](float ts, float) { *out++ = ref_to_stepping_space(ts, a->cone_angle_constant); return true; },
		                                  trace_out ? &tr : nullptr);
		if (trace_out && trace_n) {
			const size_t nt = std::min<size_t>(tr.n.size(), *trace_n);
			for (size_t k = 0; k < nt; ++k) {
				trace_out[3 * k] = tr.n[k];
				trace_out[3 * k + 1] = tr.face[k];
				trace_out[3 * k + 2] = (float)tr.occ[k];
			}
			*trace_n = (uint32_t)nt;
		}
		return c;
	}
	if (trace_n) *trace_n = 0;
	const V3 idir = v(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
	float n = lat_to(stp, t) + jitter;
	uint32_t count = 0;
	while (count < cap && next_occupied(&n, stp, o, d, idir, M.bits.data(), a->max_cascade, box)) {
		out[count++] = n;
		n += 1.0f;
	}
	return count;
}

int oref_train_step(void* m, const ngp_train_args* a) { return guard([&] { train_step(*static_cast<Model*>(m), *a); }); }
void oref_optimizer_step(void* m, uint32_t step, int opt_mlp, int opt_enc) { optimizer(*static_cast<Model*>(m), step, opt_mlp, opt_enc); }
void oref_train_stats(void* m, ngp_train_stats* s) {
	Model& M = *static_cast<Model*>(m);
	std::memset(s, 0, sizeof(*s));
	s->n_rays = (uint32_t)M.loss.size();
	s->measured_batch_size_before_compaction = M.total_samples;
	s->measured_batch_size = M.total_compacted;
	s->loss = M.loss_sum;
}
// scratch mirrors of ngp_train_scratch (host copies)
size_t oref_train_scratch(void* m, int kind, void* out) {
	Model& M = *static_cast<Model*>(m);
	auto cp = [&](const void* src, size_t bytes) { if (out) std::memcpy(out, src, bytes); return bytes; };
	switch (kind) {
		case NGP_SCRATCH_RAY_NUMSTEPS: return cp(M.ray_numsteps.data(), M.ray_numsteps.size() * 4);
		case NGP_SCRATCH_COORDS: return cp(M.coords.data(), M.coords.size() * 4);
		case NGP_SCRATCH_MLP_OUT: return cp(M.mlp_out.data(), M.mlp_out.size() * 2);
		case NGP_SCRATCH_RAY_COMPACTED: return cp(M.ray_compacted.data(), M.ray_compacted.size() * 4);
		case NGP_SCRATCH_DLOSS: return cp(M.dloss.data(), M.dloss.size() * 2);
		case NGP_SCRATCH_LOSS: return cp(M.loss.data(), M.loss.size() * 4);
		case NGP_SCRATCH_COMPACT_COORDS: return cp(M.ccoords.data(), M.ccoords.size() * 4);
		default: return 0;
	}
}
int oref_density_grid_update(void* m, const ngp_grid_args* a) {
	return guard([&] {
		grid_evaluate(*static_cast<Model*>(m), *a);
		grid_finish(*static_cast<Model*>(m), *a);
	});
}
int oref_density_grid_evaluate(void* m, const ngp_grid_args* a) { return guard([&] { grid_evaluate(*static_cast<Model*>(m), *a); }); }
int oref_density_grid_finish(void* m, const ngp_grid_args* a) { return guard([&] { grid_finish(*static_cast<Model*>(m), *a); }); }
// evaluation buffer (n floats) for the data-parallel max all-reduce
void oref_density_grid_tmp(void* m, float* io, uint32_t n, int write) {
	Model& M = *static_cast<Model*>(m);
	if (write) M.tmp.assign(io, io + n);
	else std::copy(M.tmp.begin(), M.tmp.begin() + std::min<size_t>(n, M.tmp.size()), io);
}
void oref_density_grid_bitfield(void* m, uint32_t max_cascade) { bitfield_update(*static_cast<Model*>(m), max_cascade); }
void oref_density_grid_set(void* m, const float* grid, uint32_t n) {
	Model& M = *static_cast<Model*>(m);
	M.grid.assign(grid, grid + n);
}
void oref_density_grid_get(void* m, float* grid, uint8_t* bits, float* mean) {
	Model& M = *static_cast<Model*>(m);
	if (grid) std::memcpy(grid, M.grid.data(), M.grid.size() * 4);
	if (bits) std::memcpy(bits, M.bits.data(), M.bits.size());
	if (mean) *mean = M.mean;
}
void oref_set_bitfield(void* m, const uint8_t* bits) {
	Model& M = *static_cast<Model*>(m);
	M.bits.assign(bits, bits + CELLS / 8 * CASCADES);
}
int oref_render(void* m, const ngp_render_args* a, float* frame, float* depth) {
	return guard([&] { render(*static_cast<Model*>(m), *a, frame, depth); });
}
// accumulate_kernel + tonemap_kernel for one pixel buffer (render_buffer.cu:232-266,533-565)
void oref_accumulate_tonemap(const float* frame, float* accum, float* out, uint32_t W, uint32_t H, uint32_t spp,
                             int color_space, float exposure, const float* bg_in, int output_srgb) {
	for (size_t i = 0; i < (size_t)W * H; ++i) {
		float c[4], t[4];
		for (int k = 0; k < 4; ++k) { c[k] = frame[4 * i + k]; t[k] = spp == 0 ? 0.0f : accum[4 * i + k]; }
		if (color_space == 1) for (int k = 0; k < 3; ++k) c[k] = l2s(c[k]);
		for (int k = 0; k < 4; ++k) t[k] = (t[k] * (float)spp + c[k]) / ((float)spp + 1.0f);
		for (int k = 0; k < 4; ++k) accum[4 * i + k] = t[k];
		if (!out) continue;
		float bg[4] = {bg_in[0], bg_in[1], bg_in[2], bg_in[3]};
		if (color_space != 1) for (int k = 0; k < 3; ++k) bg[k] = s2l(bg[k]);
		const float w = (1.0f - t[3]) * bg[3];
		for (int k = 0; k < 3; ++k) t[k] += bg[k] * w;
		t[3] += w;
		if (color_space == 1) for (int k = 0; k < 3; ++k) t[k] = s2l(t[k]);
		const float e = std::pow(2.0f, exposure);
		for (int k = 0; k < 3; ++k) t[k] *= e;
		if (output_srgb) for (int k = 0; k < 3; ++k) t[k] = l2s(t[k]);
		for (int k = 0; k < 4; ++k) out[4 * i + k] = t[k];
	}
}


// Testbed::get_density_on_grid (src/testbed_nerf.cu:3026-3075): generate_grid_samples_nerf_uniform (:147-160) places
// lattice point (x, y, z) / (res - 1) of the box, rotated by transpose(render_aabb_to_local) and warped into the
// training aabb; NerfNetwork::density gives the raw output (fp16); grid_samples_half_to_float (:234-250) unwarps
// the position and replaces the value by -10000 where the cascaded density grid at mip_from_pos is below 0.01
// (a point outside the grid reads 0).  grid: [n_cascades][128^3] host floats, null = no masking.
void oref_density_on_grid(void* m, const ngp_grid_query* q, const float* grid, float* out) {
	const uint32_t rx = q->res[0], ry = q->res[1], rz = q->res[2];
	const size_t n = (size_t)rx * ry * rz;
	const Box box{v(q->box_min[0], q->box_min[1], q->box_min[2]), v(q->box_max[0], q->box_max[1], q->box_max[2])};
	const Box train{v(q->aabb_min[0], q->aabb_min[1], q->aabb_min[2]), v(q->aabb_max[0], q->aabb_max[1], q->aabb_max[2])};
	const RBox rb = rbox_of(box, q->box_to_local);
	const V3 den = v((float)(rx - 1), (float)(ry - 1), (float)(rz - 1));
	std::vector<float> rows(4 * n);
	for (size_t i = 0; i < n; ++i) {
		const uint32_t x = (uint32_t)(i % rx), y = (uint32_t)((i / rx) % ry), z = (uint32_t)(i / ((size_t)rx * ry));
		V3 p = v((float)x, (float)y, (float)z) / den;
		p = V3{p.x * (box.mx.x - box.mn.x), p.y * (box.mx.y - box.mn.y), p.z * (box.mx.z - box.mn.z)} + box.mn;
		if (rb.rot) {
			const float* R = rb.R;  // transpose(R) * p
			p = V3{R[0] * p.x + R[3] * p.y + R[6] * p.z, R[1] * p.x + R[4] * p.y + R[7] * p.z, R[2] * p.x + R[5] * p.y + R[8] * p.z};
		}
		const V3 w = train.rel(p);
		rows[4 * i + 0] = w.x;
		rows[4 * i + 1] = w.y;
		rows[4 * i + 2] = w.z;
		rows[4 * i + 3] = warp_dt(MIN_STEP);
	}
	const size_t chunk = 4096;
#pragma omp parallel for schedule(dynamic)
	for (size_t c = 0; c < n; c += chunk) {
		const uint32_t cnt = (uint32_t)std::min(chunk, n - c);
		std::vector<float> raw(cnt);
		oref_density(m, rows.data() + 4 * c, 4, cnt, raw.data(), q->use_inference_params);
		for (uint32_t j = 0; j < cnt; ++j) {
			const size_t i = c + j;
			float val = h2f(f2h(raw[j]));
			if (grid && q->mask_with_grid) {
				const V3 w = v(rows[4 * i], rows[4 * i + 1], rows[4 * i + 2]);
				const V3 pos = V3{w.x * (train.mx.x - train.mn.x), w.y * (train.mx.y - train.mn.y), w.z * (train.mx.z - train.mn.z)} + train.mn;
				const uint32_t mip = mip_pos(pos, q->max_cascade);
				const uint32_t gi = grid_idx(pos, mip);
				const float gd = gi == 0xFFFFFFFFu ? 0.0f : grid[gi + (size_t)CELLS * mip];
				if (gd < 0.01f) val = -10000.0f;
			}
			out[i] = val;
		}
	}
}

// save_density_grid_to_png (src/marching_cubes.cu:957-1020): density [z][y][x] (res3d), mosaic of ceil(rz / ndown) x
// ndown tiles with ndown = floor(sqrt(rz)) (rz, ry swapped when swap_y_z); tile z at column z % nacross, row
// z / nacross; unswapped rows are flipped (y = ry - 1 - v); byte = (uint8)clamp((d - thresh) * 128 / range + 128.5, 0, 255);
// unused tiles are 0.  *w, *h: the mosaic size; out: w * h bytes (null: size only).  The log line's counts
// (:965-996) go to counts[0] (voxels with 1..7 of 8 corners below thresh) and counts[1] (interior points with a
// 6-neighbour on the other side of thresh).
void oref_density_slices_mosaic(const float* d, const int* res3d, float thresh, int swap_y_z, float range, uint8_t* out,
                                int* w, int* h, uint32_t* counts) {
	const int X = res3d[0], Y = res3d[1], Z = res3d[2];
	auto below = [&](int x, int y, int z) { return d[((size_t)z * Y + y) * X + x] < thresh; };
	if (counts) {
		counts[0] = counts[1] = 0;
		for (int z = 1; z + 1 < Z; ++z)
			for (int y = 1; y + 1 < Y; ++y)
				for (int x = 1; x + 1 < X; ++x) {
					int c = 0;
					for (int dz = 0; dz < 2; ++dz)
						for (int dy = 0; dy < 2; ++dy)
							for (int dx = 0; dx < 2; ++dx) c += below(x + dx, y + dy, z + dz);
					counts[0] += (c > 0 && c < 8);
					const bool me = below(x, y, z);
					const bool diff = below(x + 1, y, z) != me || below(x - 1, y, z) != me || below(x, y + 1, z) != me ||
					                  below(x, y - 1, z) != me || below(x, y, z + 1) != me || below(x, y, z - 1) != me;
					counts[1] += diff;
				}
	}
	const int ty = swap_y_z ? Z : Y, tz = swap_y_z ? Y : Z;  // tile height and tile count
	const int ndown = (int)std::sqrt((float)tz), nacross = (tz + ndown - 1) / ndown;
	*w = X * nacross;
	*h = ty * ndown;
	if (!out) return;
	const float scale = 128.0f / range;
	std::memset(out, 0, (size_t)(*w) * (*h));
	for (int t = 0; t < tz; ++t) {
		const int u0 = (t % nacross) * X, v0 = (t / nacross) * ty;
		for (int r = 0; r < ty; ++r)
			for (int x = 0; x < X; ++x) {
				// swapped: image row r of tile t is grid (y = t, z = r); otherwise grid (y = ty - 1 - r, z = t)
				const float val = swap_y_z ? d[((size_t)r * Y + t) * X + x] : d[((size_t)t * Y + (ty - 1 - r)) * X + x];
				float b = (val - thresh) * scale + 128.5f;
				b = b < 0.0f ? 0.0f : (b > 255.0f ? 255.0f : b);
				out[(size_t)(v0 + r) * (*w) + u0 + x] = (uint8_t)b;
			}
	}
}

}  // extern "C"
