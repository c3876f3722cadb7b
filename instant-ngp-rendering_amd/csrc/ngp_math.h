// ngp_math.h — scalar math shared by the gfx950 kernels and the host runtime.
//
// Everything here is __host__ __device__ so the C++ Testbed (g++) and the HIP
// kernels (hipcc, gfx950) agree bit for bit on RNG streams, Morton codes and the
// NeRF stepping rules.  Each helper cites the reference function it restates.
#pragma once

#include <stdint.h>
#include <math.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define NGP_HD __host__ __device__ __forceinline__
#else
#define NGP_HD inline
#endif

namespace ngp {

// ---------------------------------------------------------------------------
// Constants — include/neural-graphics-primitives/nerf_device.cuh:24-42,
// common_device.cuh:32.
// ---------------------------------------------------------------------------
constexpr uint32_t NERF_GRIDSIZE = 128;
constexpr uint32_t NERF_GRID_N_CELLS = NERF_GRIDSIZE * NERF_GRIDSIZE * NERF_GRIDSIZE;
constexpr uint32_t NERF_STEPS = 1024;
constexpr uint32_t NERF_CASCADES = 8;
constexpr float SQRT3 = 1.73205080757f;
constexpr float STEPSIZE = SQRT3 / (float)NERF_STEPS;
constexpr float MIN_CONE_STEPSIZE = STEPSIZE;
constexpr float MAX_CONE_STEPSIZE = STEPSIZE * (float)(1u << (NERF_CASCADES - 1)) * (float)NERF_STEPS / (float)NERF_GRIDSIZE;
constexpr uint32_t N_MAX_RANDOM_SAMPLES_PER_RAY = 16;
constexpr float NERF_MIN_OPTICAL_THICKNESS = 0.01f;
constexpr float MAX_DEPTH = 16384.0f;
constexpr uint32_t BATCH_SIZE_GRANULARITY = 256;

// ---------------------------------------------------------------------------
// Small vector type (the reference uses tcnn::vec3).
// ---------------------------------------------------------------------------
struct v3 {
	float x, y, z;
};
NGP_HD v3 mk3(float x, float y, float z) { v3 r; r.x = x; r.y = y; r.z = z; return r; }
NGP_HD v3 mk3(float s) { return mk3(s, s, s); }
NGP_HD v3 operator+(v3 a, v3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
NGP_HD v3 operator-(v3 a, v3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
NGP_HD v3 operator*(v3 a, v3 b) { return mk3(a.x * b.x, a.y * b.y, a.z * b.z); }
NGP_HD v3 operator/(v3 a, v3 b) { return mk3(a.x / b.x, a.y / b.y, a.z / b.z); }
NGP_HD v3 operator*(v3 a, float s) { return mk3(a.x * s, a.y * s, a.z * s); }
NGP_HD v3 operator*(float s, v3 a) { return mk3(a.x * s, a.y * s, a.z * s); }
NGP_HD v3 operator/(v3 a, float s) { return mk3(a.x / s, a.y / s, a.z / s); }
NGP_HD v3 operator+(v3 a, float s) { return mk3(a.x + s, a.y + s, a.z + s); }
NGP_HD v3 operator-(v3 a, float s) { return mk3(a.x - s, a.y - s, a.z - s); }
NGP_HD float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
NGP_HD float length(v3 a) { return sqrtf(dot(a, a)); }
NGP_HD v3 normalize(v3 a) { return a * (1.0f / length(a)); }
NGP_HD float maxc(v3 a) { return fmaxf(fmaxf(a.x, a.y), a.z); }
NGP_HD v3 absv(v3 a) { return mk3(fabsf(a.x), fabsf(a.y), fabsf(a.z)); }

// Column-major 4x3 camera matrix, columns = right, up, forward, origin
// (tcnn mat4x3 as used by Testbed, common.h TrainingXForm).
struct m43 {
	v3 c[4];
};
NGP_HD v3 rot(const m43& m, v3 d) { return m.c[0] * d.x + m.c[1] * d.y + m.c[2] * d.z; }
// camera_slerp (common_device.cuh:628-631): rotation slerped through quaternions, translation
// mixed.  The quaternion conversions and slerp live in tcnn's vec.h, which is absent from the
// mount; they are restated from glm (quat_cast, slerp with the lerp fallback at cos > 1 - eps,
// mat3_cast), so the interpolated camera is parity-unpinned beyond t = 0 (start returned exactly).
struct q4 {
	float w, x, y, z;
};
NGP_HD q4 quat_from_rot(const m43& m) {
	const float m00 = m.c[0].x, m01 = m.c[0].y, m02 = m.c[0].z, m10 = m.c[1].x, m11 = m.c[1].y, m12 = m.c[1].z;
	const float m20 = m.c[2].x, m21 = m.c[2].y, m22 = m.c[2].z;
	const float fx = m00 - m11 - m22, fy = m11 - m00 - m22, fz = m22 - m00 - m11, fw = m00 + m11 + m22;
	int bi = 0;
	float fb = fw;
	if (fx > fb) { fb = fx; bi = 1; }
	if (fy > fb) { fb = fy; bi = 2; }
	if (fz > fb) { fb = fz; bi = 3; }
	const float bv = sqrtf(fb + 1.0f) * 0.5f, mult = 0.25f / bv;
	q4 q;
	if (bi == 0) q = {bv, (m12 - m21) * mult, (m20 - m02) * mult, (m01 - m10) * mult};
	else if (bi == 1) q = {(m12 - m21) * mult, bv, (m01 + m10) * mult, (m20 + m02) * mult};
	else if (bi == 2) q = {(m20 - m02) * mult, (m01 + m10) * mult, bv, (m12 + m21) * mult};
	else q = {(m01 - m10) * mult, (m20 + m02) * mult, (m12 + m21) * mult, bv};
	return q;
}
NGP_HD q4 quat_slerp(q4 a, q4 b, float t) {
	float c = a.w * b.w + a.x * b.x + a.y * b.y + a.z * b.z;
	if (c < 0.0f) {
		b = {-b.w, -b.x, -b.y, -b.z};
		c = -c;
	}
	if (c > 1.0f - 1.1920928955078125e-7f)
		return {a.w * (1.0f - t) + b.w * t, a.x * (1.0f - t) + b.x * t, a.y * (1.0f - t) + b.y * t, a.z * (1.0f - t) + b.z * t};
	const float ang = acosf(c), s0 = sinf((1.0f - t) * ang), s1 = sinf(t * ang), inv = 1.0f / sinf(ang);
	return {(s0 * a.w + s1 * b.w) * inv, (s0 * a.x + s1 * b.x) * inv, (s0 * a.y + s1 * b.y) * inv, (s0 * a.z + s1 * b.z) * inv};
}
NGP_HD m43 camera_slerp(const m43& a, const m43& b, float t) {
	if (t == 0.0f) return a;
	q4 q = quat_slerp(quat_from_rot(a), quat_from_rot(b), t);
	const float n = sqrtf(q.w * q.w + q.x * q.x + q.y * q.y + q.z * q.z), in = 1.0f / n;
	q = {q.w * in, q.x * in, q.y * in, q.z * in};
	const float xx = q.x * q.x, yy = q.y * q.y, zz = q.z * q.z, xz = q.x * q.z, xy = q.x * q.y, yz = q.y * q.z;
	const float wx = q.w * q.x, wy = q.w * q.y, wz = q.w * q.z;
	m43 r;
	r.c[0] = mk3(1.0f - 2.0f * (yy + zz), 2.0f * (xy + wz), 2.0f * (xz - wy));
	r.c[1] = mk3(2.0f * (xy - wz), 1.0f - 2.0f * (xx + zz), 2.0f * (yz + wx));
	r.c[2] = mk3(2.0f * (xz + wy), 2.0f * (yz - wx), 1.0f - 2.0f * (xx + yy));
	r.c[3] = mk3(a.c[3].x * (1.0f - t) + b.c[3].x * t, a.c[3].y * (1.0f - t) + b.c[3].y * t, a.c[3].z * (1.0f - t) + b.c[3].z * t);
	return r;
}
// get_xform_given_rolling_shutter (common_device.cuh:633-636): pixel time A + B u + C v + D motionblur_time
NGP_HD m43 xform_given_rolling_shutter(const m43& start, const m43& end, const float* rs, float u, float v, float mb) {
	return camera_slerp(start, end, rs[0] + rs[1] * u + rs[2] * v + rs[3] * mb);
}

// inverse(mat3(m)) * g with glm's adjugate / determinant inverse (column-major m[c][r])
NGP_HD v3 inverse3_mul(const m43& m, v3 g) {
	const float m00 = m.c[0].x, m01 = m.c[0].y, m02 = m.c[0].z;
	const float m10 = m.c[1].x, m11 = m.c[1].y, m12 = m.c[1].z;
	const float m20 = m.c[2].x, m21 = m.c[2].y, m22 = m.c[2].z;
	const float inv_det = 1.0f / (m00 * (m11 * m22 - m21 * m12) - m10 * (m01 * m22 - m21 * m02) + m20 * (m01 * m12 - m11 * m02));
	const float i00 = (m11 * m22 - m21 * m12) * inv_det, i10 = -(m10 * m22 - m20 * m12) * inv_det, i20 = (m10 * m21 - m20 * m11) * inv_det;
	const float i01 = -(m01 * m22 - m21 * m02) * inv_det, i11 = (m00 * m22 - m20 * m02) * inv_det, i21 = -(m00 * m21 - m20 * m01) * inv_det;
	const float i02 = (m01 * m12 - m11 * m02) * inv_det, i12 = -(m00 * m12 - m10 * m02) * inv_det, i22 = (m00 * m11 - m10 * m01) * inv_det;
	return mk3(i00 * g.x + i10 * g.y + i20 * g.z, i01 * g.x + i11 * g.y + i21 * g.z, i02 * g.x + i12 * g.y + i22 * g.z);
}

// ---------------------------------------------------------------------------
// Camera lenses — uv_to_ray's direction part (common_device.cuh:248-460).  Modes follow
// ELensMode (common.h:188-195): 0 Perspective, 1 OpenCV, 2 FTheta, 3 LatLong,
// 4 OpenCVFisheye, 5 Equirectangular.  params[7]: k1 k2 p1 p2 (OpenCV), k1 k2 k3 k4
// (fisheye), r0..r4 w h (F-Theta).
// ---------------------------------------------------------------------------
enum LensMode : int { LENS_PERSPECTIVE = 0, LENS_OPENCV = 1, LENS_FTHETA = 2, LENS_LATLONG = 3, LENS_OPENCV_FISHEYE = 4,
                      LENS_EQUIRECTANGULAR = 5 };
constexpr float NGP_PI = 3.14159265358979323846f;

NGP_HD void opencv_delta(const float* k, float u, float v, float* du, float* dv) {
	const float u2 = u * u, uv = u * v, v2 = v * v, r2 = u2 + v2;
	const float radial = k[0] * r2 + k[1] * r2 * r2;
	*du = u * radial + 2.0f * k[2] * uv + k[3] * (r2 + 2.0f * u2);
	*dv = v * radial + 2.0f * k[3] * uv + k[2] * (r2 + 2.0f * v2);
}
NGP_HD void opencv_fisheye_delta(const float* k, float u, float v, float* du, float* dv) {
	const float r = sqrtf(u * u + v * v);
	if (r > 2.220446049250313e-16f) {  // numeric_limits<double>::epsilon() as float
		const float theta = atanf(r), t2 = theta * theta, t4 = t2 * t2, t6 = t4 * t2, t8 = t4 * t4;
		const float thetad = theta * (1.0f + k[0] * t2 + k[1] * t4 + k[2] * t6 + k[3] * t8);
		*du = u * thetad / r - u;
		*dv = v * thetad / r - v;
	} else {
		*du = 0.0f;
		*dv = 0.0f;
	}
}
// iterative_lens_undistortion: Newton with a central-difference Jacobian, <= 100 steps
template <int MODE>
NGP_HD void iterative_undistortion(const float* k, float* u, float* v) {
	const float x0 = *u, y0 = *v;
	float x = x0, y = y0;
	for (uint32_t i = 0; i < 100; ++i) {
		const float s0 = fmaxf(1.1920929e-7f, fabsf(1e-6f * x)), s1 = fmaxf(1.1920929e-7f, fabsf(1e-6f * y));
		float dx, dy, a0, b0, a1, b1, c0, d0, c1, d1;
		auto f = [&](float px, float py, float* ox, float* oy) {
			if (MODE == LENS_OPENCV) opencv_delta(k, px, py, ox, oy);
			else opencv_fisheye_delta(k, px, py, ox, oy);
		};
		f(x, y, &dx, &dy);
		f(x - s0, y, &a0, &b0);
		f(x + s0, y, &a1, &b1);
		f(x, y - s1, &c0, &d0);
		f(x, y + s1, &c1, &d1);
		// J (column-major as in the reference): J[0][0] = d(x+dx)/dx, J[1][0] = d(x+dx)/dy, ...
		const float j00 = 1.0f + (a1 - a0) / (2.0f * s0), j10 = (c1 - c0) / (2.0f * s1);
		const float j01 = (b1 - b0) / (2.0f * s0), j11 = 1.0f + (d1 - d0) / (2.0f * s1);
		const float rx = x + dx - x0, ry = y + dy - y0;
		// inverse(J) * r with glm's mat2 inverse: 1/det * [[j11, -j01], [-j10, j00]] (columns)
		const float det = j00 * j11 - j10 * j01;
		const float inv = 1.0f / det;
		const float sx = (j11 * inv) * rx + (-j10 * inv) * ry;
		const float sy = (-j01 * inv) * rx + (j00 * inv) * ry;
		x -= sx;
		y -= sy;
		if (sx * sx + sy * sy < 1e-10f) break;
	}
	*u = x;
	*v = y;
}
// Camera-space ray direction of screen position uv (not normalised); false: no ray (F-Theta
// beyond its field of view -- the sampler then uses the camera axis, as the reference does)
// Buffer2DView<const vec2>::at_lerp (common.h:249-266) of the learned distortion map
// ([res_y][res_x][2] f32) at uv: bilinear between the texels around res * uv, clamped to the edge
// (uv_to_ray adds it to the camera-space direction's xy, common_device.cuh:441-443).
NGP_HD void distortion_at_lerp(const float* map, uint32_t rx, uint32_t ry, float u, float v, float* dx, float* dy) {
	const float fx = (float)rx * u, fy = (float)ry * v;
	const int px = (int)fx, py = (int)fy;
	const float wx = fx - (float)px, wy = fy - (float)py;
	const int x0 = px < 0 ? 0 : (px > (int)rx - 1 ? (int)rx - 1 : px), x1 = px + 1 < 0 ? 0 : (px + 1 > (int)rx - 1 ? (int)rx - 1 : px + 1);
	const int y0 = py < 0 ? 0 : (py > (int)ry - 1 ? (int)ry - 1 : py), y1 = py + 1 < 0 ? 0 : (py + 1 > (int)ry - 1 ? (int)ry - 1 : py + 1);
	const float w00 = (1.0f - wx) * (1.0f - wy), w10 = wx * (1.0f - wy), w01 = (1.0f - wx) * wy, w11 = wx * wy;
	const float* a = map + 2 * ((size_t)y0 * rx + x0);
	const float* b = map + 2 * ((size_t)y0 * rx + x1);
	const float* c = map + 2 * ((size_t)y1 * rx + x0);
	const float* d = map + 2 * ((size_t)y1 * rx + x1);
	*dx = w00 * a[0] + w10 * b[0] + w01 * c[0] + w11 * d[0];
	*dy = w00 * a[1] + w10 * b[1] + w01 * c[1] + w11 * d[1];
}

NGP_HD bool lens_direction(float u, float v, float res_x, float res_y, float fx, float fy, float cx, float cy, int mode,
                           const float* k, v3* dir) {
	if (mode == LENS_FTHETA) {
		const float xpix = (u - cx) * k[5], ypix = (v - cy) * k[6];
		const float norm = sqrtf(xpix * xpix + ypix * ypix);
		const float alpha = k[0] + norm * (k[1] + norm * (k[2] + norm * (k[3] + norm * k[4])));
		float sa = sinf(alpha), ca = cosf(alpha);
		if (ca <= 1.17549435e-38f || norm == 0.0f) return false;
		sa *= 1.0f / norm;
		*dir = mk3(sa * xpix, sa * ypix, ca);
		return true;
	}
	if (mode == LENS_LATLONG) {
		const float theta = (v - 0.5f) * NGP_PI, phi = (u - 0.5f) * NGP_PI * 2.0f;
		const float st = sinf(theta), ct = cosf(theta), sp = sinf(phi), cp = cosf(phi);
		*dir = mk3(sp * ct, st, cp * ct);
		return true;
	}
	if (mode == LENS_EQUIRECTANGULAR) {
		const float ct = (v - 0.5f) * 2.0f, st = sqrtf(fmaxf(1.0f - ct * ct, 0.0f)), phi = (u - 0.5f) * NGP_PI * 2.0f;
		*dir = mk3(sinf(phi) * st, ct, cosf(phi) * st);
		return true;
	}
	float x = (u - cx) * res_x / fx, y = (v - cy) * res_y / fy;
	if (mode == LENS_OPENCV) iterative_undistortion<LENS_OPENCV>(k, &x, &y);
	else if (mode == LENS_OPENCV_FISHEYE) iterative_undistortion<LENS_OPENCV_FISHEYE>(k, &x, &y);
	*dir = mk3(x, y, 1.0f);
	return true;
}

// ---------------------------------------------------------------------------
// PCG32 (tiny-cuda-nn `pcg32`, W. Jakob's pcg32.h); default_rng_t in
// include/neural-graphics-primitives/random_val.cuh:26.
// ---------------------------------------------------------------------------
struct pcg32 {
	uint64_t state, inc;
	NGP_HD pcg32() : state(0x853c49e6748fea9bULL), inc(0xda3e39cb94b95bdbULL) {}
	NGP_HD explicit pcg32(uint64_t initstate, uint64_t initseq = 1u) { seed(initstate, initseq); }
	NGP_HD void seed(uint64_t initstate, uint64_t initseq = 1u) {
		state = 0u;
		inc = (initseq << 1u) | 1u;
		next_uint();
		state += initstate;
		next_uint();
	}
	NGP_HD uint32_t next_uint() {
		uint64_t oldstate = state;
		state = oldstate * 0x5851f42d4c957f2dULL + inc;
		uint32_t xorshifted = (uint32_t)(((oldstate >> 18u) ^ oldstate) >> 27u);
		uint32_t r = (uint32_t)(oldstate >> 59u);
		return (xorshifted >> r) | (xorshifted << ((~r + 1u) & 31));
	}
	NGP_HD float next_float() {
		union { uint32_t u; float f; } x;
		x.u = (next_uint() >> 9) | 0x3f800000u;
		return x.f - 1.0f;
	}
	NGP_HD void advance(int64_t delta_ = (1ll << 32)) {
		uint64_t cur_mult = 0x5851f42d4c957f2dULL, cur_plus = inc, acc_mult = 1u, acc_plus = 0u;
		uint64_t delta = (uint64_t)delta_;
		while (delta > 0) {
			if (delta & 1) {
				acc_mult *= cur_mult;
				acc_plus = acc_plus * cur_mult + cur_plus;
			}
			cur_plus = (cur_mult + 1) * cur_plus;
			cur_mult *= cur_mult;
			delta /= 2;
		}
		state = acc_mult * state + acc_plus;
	}
};

// ---------------------------------------------------------------------------
// tcnn ExponentialDecay (configs/nerf/base.json:9-14) in closed form: the learning rate is
// multiplied by decay_base at decay_start, decay_start + interval, ... for optimizer steps below
// decay_end.  PARITY UNPINNED: tcnn's optimizer source is not in the reference mount, so the exact
// step a decay lands on (first at decay_start, none at or after decay_end) is the restated spec
// (SURVEY App. C 6), shared by the network optimizer, the distortion map and the camera updates.
// ---------------------------------------------------------------------------
NGP_HD float exp_decay_learning_rate(float lr, float decay_base, uint32_t decay_start, uint32_t decay_interval,
                                     uint32_t decay_end, uint32_t step) {
	if (decay_interval == 0 || step < decay_start || decay_end <= decay_start) return lr;
	const uint32_t s = step < decay_end ? step : decay_end - 1;
	return lr * powf(decay_base, (float)((s - decay_start) / decay_interval + 1));
}

// ---------------------------------------------------------------------------
// Morton codes (tcnn morton3D / morton3D_invert), used at nerf_device.cuh:327,
// src/testbed_nerf.cu:86-88,206-208,326-330.
// ---------------------------------------------------------------------------
NGP_HD uint32_t expand_bits(uint32_t v) {
	v = (v * 0x00010001u) & 0xFF0000FFu;
	v = (v * 0x00000101u) & 0x0F00F00Fu;
	v = (v * 0x00000011u) & 0xC30C30C3u;
	v = (v * 0x00000005u) & 0x49249249u;
	return v;
}
NGP_HD uint32_t morton3D(uint32_t x, uint32_t y, uint32_t z) {
	return (expand_bits(x)) | (expand_bits(y) << 1) | (expand_bits(z) << 2);
}
NGP_HD uint32_t morton3D_invert(uint32_t x) {
	x = x & 0x49249249u;
	x = (x | (x >> 2)) & 0xc30c30c3u;
	x = (x | (x >> 4)) & 0x0f00f00fu;
	x = (x | (x >> 8)) & 0xff0000ffu;
	x = (x | (x >> 16)) & 0x0000ffffu;
	return x;
}

// ---------------------------------------------------------------------------
// Low-discrepancy sequence — random_val.cuh:162-325 (Burley 2019 scrambled Sobol).
// Only the dimensions the NeRF path uses (0 and 1) are needed.
// ---------------------------------------------------------------------------
NGP_HD uint32_t sobol_dim(uint32_t index, uint32_t dim) {
	// dim 0: van der Corput (bit reversal); dim 1: direction numbers of
	// random_val.cuh:176-179 (0x80000000, 0xc0000000, 0xa0000000, ...), which are
	// the Pascal-triangle-mod-2 matrix: v_k = v_{k-1} ^ (v_{k-1} >> 1).
	uint32_t X = 0;
	uint32_t v = 0x80000000u;
	for (uint32_t bit = 0; bit < 32; ++bit) {
		uint32_t dirn = dim == 0 ? (0x80000000u >> bit) : v;
		if ((index >> bit) & 1u) X ^= dirn;
		v = v ^ (v >> 1);
	}
	return X;
}
NGP_HD uint32_t hash_combine(uint32_t seed, uint32_t v) { return seed ^ (v + (seed << 6) + (seed >> 2)); }
NGP_HD uint32_t reverse_bits(uint32_t x) {
	x = (((x & 0xaaaaaaaau) >> 1) | ((x & 0x55555555u) << 1));
	x = (((x & 0xccccccccu) >> 2) | ((x & 0x33333333u) << 2));
	x = (((x & 0xf0f0f0f0u) >> 4) | ((x & 0x0f0f0f0fu) << 4));
	x = (((x & 0xff00ff00u) >> 8) | ((x & 0x00ff00ffu) << 8));
	return ((x >> 16) | (x << 16));
}
NGP_HD uint32_t laine_karras_permutation(uint32_t x, uint32_t seed) {
	x += seed;
	x ^= x * 0x6c50b47cu;
	x ^= x * 0xb82f1e52u;
	x ^= x * 0xc7afe638u;
	x ^= x * 0x8d22f6e6u;
	return x;
}
NGP_HD uint32_t nested_uniform_scramble_base2(uint32_t x, uint32_t seed) {
	return reverse_bits(laine_karras_permutation(reverse_bits(x), seed));
}
// ld_random_val (random_val.cuh:287-291)
NGP_HD float ld_random_val(uint32_t index, uint32_t seed, uint32_t dim = 0) {
	const float S = (float)(1.0 / (double)(1ull << 32));
	index = nested_uniform_scramble_base2(index, seed);
	return (float)nested_uniform_scramble_base2(sobol_dim(index, dim), hash_combine(seed, dim)) * S;
}
// ld_random_val_2d (random_val.cuh:266-285)
NGP_HD void ld_random_val_2d(uint32_t index, uint32_t seed, float* x, float* y) {
	const float S = (float)(1.0 / (double)(1ull << 32));
	index = nested_uniform_scramble_base2(index, seed);
	*x = (float)nested_uniform_scramble_base2(sobol_dim(index, 0), hash_combine(seed, 0)) * S;
	*y = (float)nested_uniform_scramble_base2(sobol_dim(index, 1), hash_combine(seed, 1)) * S;
}
NGP_HD float fractf(float x) { return x - floorf(x); }
// ld_random_pixel_offset (random_val.cuh:320-325)
NGP_HD void ld_random_pixel_offset(uint32_t spp, float* ox, float* oy) {
	float ax, ay, bx, by;
	ld_random_val_2d(0, 0xdeadbeefu, &ax, &ay);
	ld_random_val_2d(spp, 0xdeadbeefu, &bx, &by);
	*ox = fractf(0.5f - ax + bx);
	*oy = fractf(0.5f - ay + by);
}

// ---------------------------------------------------------------------------
// Colour helpers — common_device.cuh:34-80.
// ---------------------------------------------------------------------------
// srgb_to_linear_derivative (common_device.cuh:46-52)
NGP_HD float srgb_to_linear_derivative(float srgb) {
	return srgb <= 0.04045f ? 1.0f / 12.92f : 2.4f / 1.055f * powf((srgb + 0.055f) / 1.055f, 1.4f);
}
NGP_HD float srgb_to_linear(float srgb) {
	return srgb <= 0.04045f ? srgb / 12.92f : powf((srgb + 0.055f) / 1.055f, 2.4f);
}
NGP_HD float linear_to_srgb(float lin) {
	return lin < 0.0031308f ? 12.92f * lin : 1.055f * powf(lin, 0.41666f) - 0.055f;
}
NGP_HD float logistic(float x) { return 1.0f / (1.0f + expf(-x)); }

// ---------------------------------------------------------------------------
// Axis-aligned box — bounding_box.cuh:95-97,172-230.
// ---------------------------------------------------------------------------
struct aabb3 {
	v3 min, max;
};
NGP_HD bool aabb_contains(const aabb3& b, v3 p) {
	return p.x >= b.min.x && p.x <= b.max.x && p.y >= b.min.y && p.y <= b.max.y && p.z >= b.min.z && p.z <= b.max.z;
}
NGP_HD v3 aabb_relative(const aabb3& b, v3 p) { return (p - b.min) / (b.max - b.min); }
NGP_HD void ray_intersect(const aabb3& b, v3 pos, v3 dir, float* t0, float* t1) {
	const float FMAX = 3.402823466e+38f;
	float tmin = (b.min.x - pos.x) / dir.x, tmax = (b.max.x - pos.x) / dir.x;
	if (tmin > tmax) { float t = tmin; tmin = tmax; tmax = t; }
	float tymin = (b.min.y - pos.y) / dir.y, tymax = (b.max.y - pos.y) / dir.y;
	if (tymin > tymax) { float t = tymin; tymin = tymax; tymax = t; }
	if (tmin > tymax || tymin > tmax) { *t0 = FMAX; *t1 = FMAX; return; }
	if (tymin > tmin) tmin = tymin;
	if (tymax < tmax) tmax = tymax;
	float tzmin = (b.min.z - pos.z) / dir.z, tzmax = (b.max.z - pos.z) / dir.z;
	if (tzmin > tzmax) { float t = tzmin; tzmin = tzmax; tzmax = t; }
	if (tmin > tzmax || tzmin > tmax) { *t0 = FMAX; *t1 = FMAX; return; }
	if (tzmin > tmin) tmin = tzmin;
	if (tzmax < tmax) tmax = tzmax;
	*t0 = tmin;
	*t1 = tmax;
}

// The render crop box (Testbed::m_render_aabb + m_render_aabb_to_local): positions are tested in
// the box's local frame, local = R * world (nerf_device.cuh:475, src/testbed_nerf.cu:1467-1469).
struct RenderBox {
	aabb3 box;
	float R[9];  // row-major
	int rot;     // 0: R is the identity
};
NGP_HD v3 rbox_local(const RenderBox& b, v3 p) {
	if (!b.rot) return p;
	return mk3(b.R[0] * p.x + b.R[1] * p.y + b.R[2] * p.z, b.R[3] * p.x + b.R[4] * p.y + b.R[5] * p.z,
	           b.R[6] * p.x + b.R[7] * p.y + b.R[8] * p.z);
}
NGP_HD bool rbox_contains(const RenderBox& b, v3 p) { return aabb_contains(b.box, rbox_local(b, p)); }
inline RenderBox make_render_box(const aabb3& box, const float* R) {
	RenderBox b;
	b.box = box;
	bool any = false, ident = true;
	for (int k = 0; k < 9; ++k) {
		b.R[k] = R ? R[k] : 0.0f;
		any |= b.R[k] != 0.0f;
		ident &= b.R[k] == ((k % 4 == 0) ? 1.0f : 0.0f);
	}
	b.rot = any && !ident;
	if (!b.rot)
		for (int k = 0; k < 9; ++k) b.R[k] = (k % 4 == 0) ? 1.0f : 0.0f;
	return b;
}

// ---------------------------------------------------------------------------
// Warps — nerf_device.cuh:265-314.
// ---------------------------------------------------------------------------
NGP_HD v3 warp_direction(v3 d) { return (d + 1.0f) * 0.5f; }
NGP_HD float warp_dt(float dt) {
	float max_stepsize = MIN_CONE_STEPSIZE * (float)(1u << (NERF_CASCADES - 1));
	return (dt - MIN_CONE_STEPSIZE) / (max_stepsize - MIN_CONE_STEPSIZE);
}
NGP_HD float unwarp_dt(float dt) {
	float max_stepsize = MIN_CONE_STEPSIZE * (float)(1u << (NERF_CASCADES - 1));
	return dt * (max_stepsize - MIN_CONE_STEPSIZE) + MIN_CONE_STEPSIZE;
}
NGP_HD v3 unwarp_position(v3 p, const aabb3& b) { return b.min + p * (b.max - b.min); }

// ---------------------------------------------------------------------------
// Occupancy grid — nerf_device.cuh:316-357.
// ---------------------------------------------------------------------------
NGP_HD uint32_t cascaded_grid_idx_at(v3 pos, uint32_t mip) {
	float mip_scale = scalbnf(1.0f, -(int)mip);
	pos = pos - 0.5f;
	pos = pos * mip_scale;
	pos = pos + 0.5f;
	int ix = (int)(pos.x * (float)NERF_GRIDSIZE);
	int iy = (int)(pos.y * (float)NERF_GRIDSIZE);
	int iz = (int)(pos.z * (float)NERF_GRIDSIZE);
	if (ix < 0 || ix >= (int)NERF_GRIDSIZE || iy < 0 || iy >= (int)NERF_GRIDSIZE || iz < 0 || iz >= (int)NERF_GRIDSIZE) {
		return 0xFFFFFFFFu;
	}
	return morton3D((uint32_t)ix, (uint32_t)iy, (uint32_t)iz);
}
NGP_HD bool density_grid_occupied_at(v3 pos, const uint8_t* bitfield, uint32_t mip) {
	uint32_t idx = cascaded_grid_idx_at(pos, mip);
	if (idx == 0xFFFFFFFFu) return false;
	return bitfield[idx / 8 + (NERF_GRID_N_CELLS / 8) * mip] & (1u << (idx % 8));
}

NGP_HD float signf_(float x) { return x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f); }

// ---------------------------------------------------------------------------
// Stepping lattice.  A ray's candidate samples sit at n0 + k (k = 0, 1, ...) in the
// reference's "stepping space" (uniform steps of MIN_CONE_STEPSIZE for cone_angle 0,
// geometric steps otherwise; nerf_device.cuh:359-459).  A lattice point is a sample
// when it lies in the AABB and its occupancy cell is set.  The reference reaches the
// same points by chaining t += calc_dt(t) and advance_to_next_voxel(); defining them
// as n0 + k lets a wave test 64 lattice points of one ray at once (training sampler)
// and lets the render skip an empty cell in one jump whose exactness is verified.
// Division by constants is a multiply by the reciprocal (the reference is built
// with --use_fast_math, CMakeLists.txt:82); the log-regime constants are resolved
// once per launch (make_stepping) instead of per call.
// ---------------------------------------------------------------------------
constexpr float INV_MIN_CONE_STEPSIZE = 1.0f / MIN_CONE_STEPSIZE;
constexpr float INV_MAX_CONE_STEPSIZE = 1.0f / MAX_CONE_STEPSIZE;
struct Stepping {
	float cone, l, inv_l, a, b, at, bt;
};
inline Stepping make_stepping(float cone) {
	Stepping s;
	s.cone = cone;
	if (cone <= 1e-5f) {
		s.l = s.inv_l = s.a = s.b = s.at = s.bt = 0.0f;
		return s;
	}
	s.l = logf(1.0f + cone);
	s.inv_l = 1.0f / s.l;
	s.a = (logf(MIN_CONE_STEPSIZE) - logf(s.l)) * s.inv_l;
	s.b = (logf(MAX_CONE_STEPSIZE) - logf(s.l)) * s.inv_l;
	s.at = expf(s.a * s.l);
	s.bt = expf(s.b * s.l);
	return s;
}
NGP_HD float step_to(const Stepping& s, float t) {
	if (s.cone <= 1e-5f) return t * INV_MIN_CONE_STEPSIZE;
	if (t <= s.at) return (t - s.at) * INV_MIN_CONE_STEPSIZE + s.a;
	if (t <= s.bt) return logf(t) * s.inv_l;
	return (t - s.bt) * INV_MAX_CONE_STEPSIZE + s.b;
}
NGP_HD float step_from(const Stepping& s, float n) {
	if (s.cone <= 1e-5f) return n * MIN_CONE_STEPSIZE;
	if (n <= s.a) return (n - s.a) * MIN_CONE_STEPSIZE + s.at;
	if (n <= s.b) return expf(n * s.l);
	return (n - s.b) * MAX_CONE_STEPSIZE + s.bt;
}
// distance to the boundary of the current cell at resolution 128 * 2^-mip (power-of-two scales: exact)
NGP_HD float distance_to_next_cell(v3 pos, v3 dir, v3 idir, uint32_t mip) {
	const float res = scalbnf((float)NERF_GRIDSIZE, -(int)mip), inv_res = scalbnf(1.0f / (float)NERF_GRIDSIZE, (int)mip);
	const v3 p = (pos - 0.5f) * res;
	const float tx = (floorf(p.x + 0.5f + 0.5f * signf_(dir.x)) - p.x) * idir.x;
	const float ty = (floorf(p.y + 0.5f + 0.5f * signf_(dir.y)) - p.y) * idir.y;
	const float tz = (floorf(p.z + 0.5f + 0.5f * signf_(dir.z)) - p.z) * idir.z;
	return fmaxf(fminf(fminf(tx, ty), tz) * inv_res, 0.0f);
}

NGP_HD uint32_t mip_from_pos(v3 pos, uint32_t max_cascade = NERF_CASCADES - 1) {
	int exponent;
	float maxval = maxc(absv(pos - 0.5f));
	frexpf(maxval, &exponent);
	int m = exponent + 1;
	m = m < 0 ? 0 : (m > (int)max_cascade ? (int)max_cascade : m);
	return (uint32_t)m;
}
NGP_HD uint32_t mip_from_dt(float dt, v3 pos, uint32_t max_cascade = NERF_CASCADES - 1) {
	uint32_t mip = mip_from_pos(pos, max_cascade);
	dt *= 2.0f * (float)NERF_GRIDSIZE;
	if (dt < 1.0f) return mip;
	int exponent;
	frexpf(dt, &exponent);
	int m = exponent < (int)mip ? (int)mip : exponent;   // clamp((int)mip, exponent, max)
	m = m > (int)max_cascade ? (int)max_cascade : m;
	return (uint32_t)m;
}

// Render march (if_unoccupied_advance_to_next_occupied_voxel, nerf_device.cuh:461-494, on the
// lattice): a lattice point is a sample when it lies in the AABB and its cell at clamp(mip_from_pos,
// 0, max_mip) is occupied; an empty cell is left in one jump past the far faces of the empty box
// the octant distance fields give for it (at the coarsest empty mip, as the reference climbs).
// The jump is taken only if the lattice point just before the landing point is still inside the
// skipped box (or already outside the AABB), so every skipped point lies in empty space or outside
// the volume and the result equals testing the points one by one.
enum LatticeStep : int { LATTICE_OCCUPIED = 0, LATTICE_SKIPPED = 1, LATTICE_EXIT = 2 };

// Octant distance fields (render.hip k_df_*): for each mip, ray octant o (bit k set = the
// direction's component k is negative) and cell c, D = the Chebyshev distance from c to the
// nearest occupied cell of that mip lying in the octant's closed orthant from c (0 = c is
// occupied).  The box of cells c + s*[0, D-1]^3 (s = the octant's signs) is then empty, and a
// ray heading into octant o leaves it only through its far faces.  Cells beyond the grid count
// as occupied below max_mip (the next mip takes over there) and as empty at max_mip (outside
// the AABB).  Layout: [mip][octant][z][y][x] bytes, 255 = capped.
constexpr uint32_t DF_BYTES_PER_FIELD = NERF_GRID_N_CELLS;
NGP_HD uint32_t ray_octant(v3 d) { return (d.x < 0.0f ? 1u : 0u) | (d.y < 0.0f ? 2u : 0u) | (d.z < 0.0f ? 4u : 0u); }
// integer cell coordinates of pos at `mip` (cascaded_grid_idx_at without the Morton code)
NGP_HD bool cascaded_cell_at(v3 pos, uint32_t mip, int* ix, int* iy, int* iz) {
	const float mip_scale = scalbnf(1.0f, -(int)mip);
	const v3 q = (pos - 0.5f) * mip_scale + 0.5f;
	*ix = (int)(q.x * (float)NERF_GRIDSIZE);
	*iy = (int)(q.y * (float)NERF_GRIDSIZE);
	*iz = (int)(q.z * (float)NERF_GRIDSIZE);
	return *ix >= 0 && *ix < (int)NERF_GRIDSIZE && *iy >= 0 && *iy < (int)NERF_GRIDSIZE && *iz >= 0 && *iz < (int)NERF_GRIDSIZE;
}
NGP_HD uint32_t df_index(uint32_t mip, uint32_t oct, int ix, int iy, int iz) {
	return (mip * 8u + oct) * DF_BYTES_PER_FIELD + ((uint32_t)iz * NERF_GRIDSIZE + (uint32_t)iy) * NERF_GRIDSIZE + (uint32_t)ix;
}
// lattice_step through the octant distance fields: same result as lattice_step (the point is
// occupied iff D = 0 at its mip; the coarsest empty mip is climbed as the reference does), but
// an empty cell is left through the far faces of its empty D-box in one verified jump.
template <bool PARALLEL_CLIMB = false>
NGP_HD int lattice_step_df(float* n_io, const Stepping& st, v3 o, v3 d, v3 idir, uint32_t oct, const uint8_t* df,
                           uint32_t max_mip, const RenderBox& aabb) {
	const float n = *n_io;
	const float t = step_from(st, n);
	const v3 pos = o + d * t;
	if (t >= MAX_DEPTH || !rbox_contains(aabb, pos)) return LATTICE_EXIT;
	uint32_t mip = mip_from_pos(pos);
	mip = mip > max_mip ? max_mip : mip;
	int cx, cy, cz;
	if (!cascaded_cell_at(pos, mip, &cx, &cy, &cz)) {
		*n_io = n + 1.0f;
		return LATTICE_SKIPPED;
	}
	uint32_t D = df[df_index(mip, oct, cx, cy, cz)];
	if (PARALLEL_CLIMB) {
		// coarsest empty mip, as the reference climbs, with every mip's distance fetched at once -- this mip's and the
		// coarser ones' (their cells depend on the position only) -- and climbed in registers: one load latency per
		// lattice step instead of one per mip visited.  Used by k_render_init, whose skip to the first sample crosses
		// config E's seven cascades; the march kernels run at 64 VGPRs, where these registers spill, and keep the
		// serial climb below.  The chosen mip's cell is recomputed.
		constexpr uint32_t MAXQ = NERF_CASCADES - 1;
		uint32_t Du[MAXQ], inmask = 0;
#pragma unroll
		for (uint32_t q = 0; q < MAXQ; ++q) {
			const uint32_t mq = mip + 1u + q;
			int ux, uy, uz;
			const bool in = mq <= max_mip && cascaded_cell_at(pos, mq, &ux, &uy, &uz);
			inmask |= (in ? 1u : 0u) << q;
			Du[q] = in ? df[df_index(mq, oct, ux, uy, uz)] : 0u;
		}
		if (D == 0u) return LATTICE_OCCUPIED;
		uint32_t top = mip;
#pragma unroll
		for (uint32_t q = 0; q < MAXQ; ++q) {
			if (!((inmask >> q) & 1u) || Du[q] == 0u) break;
			top = mip + 1u + q;
			D = Du[q];
		}
		if (top != mip) {
			mip = top;
			cascaded_cell_at(pos, mip, &cx, &cy, &cz);
		}
	}
	if (D == 0u) return LATTICE_OCCUPIED;
	while (!PARALLEL_CLIMB && mip < max_mip) {  // coarsest empty mip, as the reference climbs
		int ux, uy, uz;
		if (!cascaded_cell_at(pos, mip + 1, &ux, &uy, &uz)) break;
		const uint32_t Du = df[df_index(mip + 1, oct, ux, uy, uz)];
		if (Du == 0u) break;
		++mip;
		D = Du;
		cx = ux;
		cy = uy;
		cz = uz;
	}
	const float res = scalbnf((float)NERF_GRIDSIZE, -(int)mip), inv_res = scalbnf(1.0f / (float)NERF_GRIDSIZE, (int)mip);
	const v3 p = (pos - 0.5f) * res;  // cell coordinates - 64
	const float fd = (float)D;
	const float fx = d.x < 0.0f ? (float)(cx - 64) + 1.0f - fd : (float)(cx - 64) + fd;
	const float fy = d.y < 0.0f ? (float)(cy - 64) + 1.0f - fd : (float)(cy - 64) + fd;
	const float fz = d.z < 0.0f ? (float)(cz - 64) + 1.0f - fd : (float)(cz - 64) + fd;
	const float exit = fmaxf(fminf(fminf((fx - p.x) * idir.x, (fy - p.y) * idir.y), (fz - p.z) * idir.z) * inv_res, 0.0f);
	const float n_far = step_to(st, t + exit);
	float nn = n + ceilf(fmaxf(n_far - n, 0.5f));
	if (nn - n > 1.0f) {
		// the jump stands if the point before the landing point is still in the empty box, or
		// already outside the AABB (the box is convex: every point in between is in it too)
		const v3 last = o + d * step_from(st, nn - 1.0f);
		if (rbox_contains(aabb, last)) {
			int qx, qy, qz;
			const bool in_grid = cascaded_cell_at(last, mip, &qx, &qy, &qz);
			const int ex = d.x < 0.0f ? cx - qx : qx - cx, ey = d.y < 0.0f ? cy - qy : qy - cy,
			          ez = d.z < 0.0f ? cz - qz : qz - cz;
			const int lim = (int)D - 1;
			if (!in_grid || ex < 0 || ex > lim || ey < 0 || ey > lim || ez < 0 || ez > lim) nn = n + 1.0f;
		}
	}
	*n_io = nn;
	return LATTICE_SKIPPED;
}

// The training sampler's walk through the octant distance fields, for aabb_scale 1 (one mip: there
// the reference's advance_to_next_voxel chain, src/testbed_nerf.cu:779-795, samples exactly the
// occupied lattice points inside the AABB, since a jump only ever leaves an empty cell).  Lattice
// point n0 + k with k an integer offset, so sample positions are step_from(n0 + k) bit for bit as the
// chain walk computes them: occupied -> OCCUPIED; outside the AABB -> EXIT; empty -> SKIPPED with *k
// moved past the far faces of the cell's empty D-box, the jump verified (as in lattice_step_df) on
// the exact lattice point before the landing one.
NGP_HD int train_step_df(uint32_t* k_io, float n0, const Stepping& st, v3 o, v3 d, v3 idir, uint32_t oct, const uint8_t* df,
                         const aabb3& aabb) {
	const uint32_t k = *k_io;
	const float n = n0 + (float)k;
	const float t = step_from(st, n);
	const v3 pos = o + d * t;
	if (!aabb_contains(aabb, pos)) return LATTICE_EXIT;
	int cx, cy, cz;
	if (!cascaded_cell_at(pos, 0, &cx, &cy, &cz)) {
		*k_io = k + 1u;
		return LATTICE_SKIPPED;
	}
	const uint32_t D = df[df_index(0, oct, cx, cy, cz)];
	if (D == 0u) return LATTICE_OCCUPIED;
	const float res = (float)NERF_GRIDSIZE, inv_res = 1.0f / (float)NERF_GRIDSIZE;
	const v3 p = (pos - 0.5f) * res;  // cell coordinates - 64
	const float fd = (float)D;
	const float fx = d.x < 0.0f ? (float)(cx - 64) + 1.0f - fd : (float)(cx - 64) + fd;
	const float fy = d.y < 0.0f ? (float)(cy - 64) + 1.0f - fd : (float)(cy - 64) + fd;
	const float fz = d.z < 0.0f ? (float)(cz - 64) + 1.0f - fd : (float)(cz - 64) + fd;
	const float exit = fmaxf(fminf(fminf((fx - p.x) * idir.x, (fy - p.y) * idir.y), (fz - p.z) * idir.z) * inv_res, 0.0f);
	const float n_far = step_to(st, t + exit);
	uint32_t c = (uint32_t)fminf(ceilf(fmaxf(n_far - n, 0.5f)), 1048576.0f);
	if (c > 1u) {
		const v3 last = o + d * step_from(st, n0 + (float)(k + c - 1u));
		if (aabb_contains(aabb, last)) {
			int qx, qy, qz;
			const bool in_grid = cascaded_cell_at(last, 0, &qx, &qy, &qz);
			const int ex = d.x < 0.0f ? cx - qx : qx - cx, ey = d.y < 0.0f ? cy - qy : qy - cy, ez = d.z < 0.0f ? cz - qz : qz - cz;
			const int lim = (int)D - 1;
			if (!in_grid || ex < 0 || ex > lim || ey < 0 || ey > lim || ez < 0 || ez > lim) c = 1u;
		}
	}
	*k_io = k + c;
	return LATTICE_SKIPPED;
}

// ---------------------------------------------------------------------------
// Image sampling helpers — nerf_device.cuh:552-598, common_device.cuh:730-806.
// ---------------------------------------------------------------------------
NGP_HD uint32_t image_idx(uint32_t base_idx, uint32_t n_rays, uint32_t n_training_images) {
	return (uint32_t)((((uint64_t)base_idx) * n_training_images) / n_rays) % n_training_images;
}

// binary_search (common.h:207-230): first index with data[i] >= val, clamped to length-1.
NGP_HD uint32_t cdf_search(float val, const float* data, uint32_t length) {
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
	return first < length - 1 ? first : length - 1;
}

// Error-map importance sampling (nerf_device.cuh:495-525, 577-593).
struct ErrorCdf {
	const float* x_cond_y;  // [img][ry][rx]
	const float* y;         // [img][ry]
	const float* img;       // [n_images]
	uint32_t rx, ry;
};
constexpr float UNIFORM_SAMPLING_FRACTION = 0.5f;
constexpr float MIN_PDF = 0.01f;  // construct_cdf_2d/1d mixing (src/testbed_nerf.cu:1491)
constexpr float MIN_PMF = 0.1f;   // image CDF mixing (src/testbed_nerf.cu:2563)
// sample_cdf_2d: half the samples stay uniform, the rest follow the image's error CDF
// (*pdf is left untouched on the uniform half, as in the reference)
NGP_HD void sample_cdf_2d(float* u, float* v, uint32_t img, const ErrorCdf& c, float* pdf) {
	if (*u < UNIFORM_SAMPLING_FRACTION) {
		*u = *u * (1.0f / UNIFORM_SAMPLING_FRACTION);
		return;
	}
	const float su = (*u - UNIFORM_SAMPLING_FRACTION) * (1.0f / (1.0f - UNIFORM_SAMPLING_FRACTION));
	const float* cy = c.y + (size_t)img * c.ry;
	const uint32_t y = cdf_search(*v, cy, c.ry);
	float prev = y > 0 ? cy[y - 1] : 0.0f;
	const float sv = (*v - prev) / (cy[y] - prev);
	const float* cx = c.x_cond_y + ((size_t)img * c.ry + y) * c.rx;
	const uint32_t x = cdf_search(su, cx, c.rx);
	prev = x > 0 ? cx[x - 1] : 0.0f;
	const float pmf_x = cx[x] - prev;
	const float sx = (su - prev) / pmf_x;
	*pdf = pmf_x * (cy[y] - (y > 0 ? cy[y - 1] : 0.0f)) * (float)(c.rx * c.ry);
	*u = ((float)x + sx) / (float)c.rx;
	*v = ((float)y + sv) / (float)c.ry;
}

// Loss (nerf_device.cuh:74-142,600-615). loss_type matches ELossType (common.h:79-87).
enum LossType : int { LOSS_L2 = 0, LOSS_L1 = 1, LOSS_MAPE = 2, LOSS_SMAPE = 3, LOSS_HUBER = 4, LOSS_LOGL1 = 5, LOSS_RELL2 = 6 };
NGP_HD void loss_and_gradient(float target, float pred, int loss_type, float* loss, float* grad) {
	float diff = pred - target;
	switch (loss_type) {
		case LOSS_RELL2: { float den = pred * pred + 1e-2f; *loss = diff * diff / den; *grad = 2.0f * diff / den; } break;
		case LOSS_L1: { *loss = fabsf(diff); *grad = copysignf(1.0f, diff); } break;
		case LOSS_MAPE: { float den = fabsf(pred) + 1e-2f; *loss = fabsf(diff) / den; *grad = copysignf(1.0f / den, diff); } break;
		case LOSS_SMAPE: { float den = 0.5f * (fabsf(pred) + fabsf(target)) + 1e-2f; *loss = fabsf(diff) / den; *grad = copysignf(1.0f / den, diff); } break;
		case LOSS_HUBER: {
			const float alpha = 0.1f;
			float ad = fabsf(diff);
			float sq = 0.5f / alpha * diff * diff;
			*loss = (ad > alpha ? (ad - 0.5f * alpha) : sq) / 5.0f;
			*grad = (ad > alpha ? (diff > 0 ? 1.0f : -1.0f) : (diff / alpha)) / 5.0f;
		} break;
		case LOSS_LOGL1: { float dv = fabsf(diff) + 1.0f; *loss = logf(dv); *grad = copysignf(1.0f / dv, diff); } break;
		default: { *loss = diff * diff; *grad = 2.0f * diff; } break;
	}
}

// Activations (nerf_device.cuh:203-254). ENerfActivation: None, ReLU, Logistic, Exponential.
enum Activation : int { ACT_NONE = 0, ACT_RELU = 1, ACT_LOGISTIC = 2, ACT_EXP = 3 };
NGP_HD float network_to_rgb(float v, int act) {
	switch (act) {
		case ACT_RELU: return v > 0.0f ? v : 0.0f;
		case ACT_LOGISTIC: return logistic(v);
		case ACT_EXP: return expf(fminf(fmaxf(v, -10.0f), 10.0f));
		default: return v;
	}
}
NGP_HD float network_to_rgb_derivative(float v, int act) {
	switch (act) {
		case ACT_RELU: return v > 0.0f ? 1.0f : 0.0f;
		case ACT_LOGISTIC: { float d = logistic(v); return d * (1 - d); }
		case ACT_EXP: return expf(fminf(fmaxf(v, -10.0f), 10.0f));
		default: return 1.0f;
	}
}
NGP_HD float network_to_density(float v, int act) {
	switch (act) {
		case ACT_RELU: return v > 0.0f ? v : 0.0f;
		case ACT_LOGISTIC: return logistic(v);
		case ACT_EXP: return expf(v);
		default: return v;
	}
}
NGP_HD float network_to_density_derivative(float v, int act) {
	switch (act) {
		case ACT_RELU: return v > 0.0f ? 1.0f : 0.0f;
		case ACT_LOGISTIC: { float d = logistic(v); return d * (1 - d); }
		case ACT_EXP: return expf(fminf(fmaxf(v, -15.0f), 15.0f));
		default: return 1.0f;
	}
}

}  // namespace ngp
