// encode_device.h -- the hash encoder's per-(sample, level) device code (tcnn GridEncoding forward,
// grid.h: pos_fract, grid_index with the CoherentPrime hash, trilinear interpolation), shared by the
// encoder kernels (hashgrid.hip) and the fused render network (mlp.hip k_mlp_infer_rf with ENC).
#pragma once

#include "ngp_internal.h"

namespace ngp {

struct Corner {
	float px, py, pz;
	uint32_t gx, gy, gz;
};

__device__ __forceinline__ void pos_fract(float input, float scale, float* frac, uint32_t* grid) {
	// tcnn pos_fract: pos = fmaf(scale, x, 0.5); grid = floor; frac = pos - floor
	float p = fmaf(scale, input, 0.5f);
	float f = floorf(p);
	*grid = (uint32_t)(int)f;
	*frac = p - f;
}

// tcnn grid_index: CoherentPrime hash for hashed levels, dense stride otherwise, modulo the
// level size.  Hashed levels have size 2^T (a mask); a dense index is below 2*size (corner
// coordinates reach res, so res + res^2 + res^3 < 2 res^3 <= 2 size), so the modulo is
// one conditional subtraction -- same value as idx % size, no integer division.
__device__ __forceinline__ uint32_t grid_index(uint32_t hashed, uint32_t size, uint32_t res, uint32_t x, uint32_t y,
                                               uint32_t z) {
	if (hashed) return ((x * 1u) ^ (y * 2654435761u) ^ (z * 805459861u)) & (size - 1u);
	const uint32_t idx = x + y * res + z * res * res;
	// tcnn: index % size.  Positions in [0, 1] overshoot by less than one table size (the
	// +1 corners), so one subtraction suffices; the modulo keeps any other input in range.
	if (idx < size) return idx;
	return idx - size < size ? idx - size : idx % size;
}

template <uint32_t F>
struct FeatVec;
template <>
struct FeatVec<1> { using T = __half; };
template <>
struct FeatVec<2> { using T = uint32_t; };
template <>
struct FeatVec<4> { using T = uint2; };
template <>
struct FeatVec<8> { using T = uint4; };

// Two consecutive table entries (an aligned pair), used to fetch the x / x+1 corners with
// one load when they share it (dense index even, or hashed with x even: index ^ 1).
template <uint32_t F>
struct PairVec;
template <>
struct PairVec<1> { using T = uint32_t; };
template <>
struct PairVec<2> { using T = uint2; };
template <>
struct PairVec<4> { using T = uint4; };

template <uint32_t F>
__device__ __forceinline__ void unpack(const typename FeatVec<F>::T& v, float* out) {
	const __half* h = reinterpret_cast<const __half*>(&v);
#pragma unroll
	for (uint32_t f = 0; f < F; ++f) out[f] = __half2float(h[f]);
}

template <bool HASHED>
__device__ __forceinline__ uint32_t corner_index(uint32_t size, uint32_t res, uint32_t x, uint32_t y, uint32_t z) {
	if (HASHED) return ((x * 1u) ^ (y * 2654435761u) ^ (z * 805459861u)) & (size - 1u);
	const uint32_t idx = x + y * res + z * res * res;
	// tcnn: index % size.  Positions in [0, 1] overshoot by less than one table size (the
	// +1 corners), so one subtraction suffices; the modulo keeps any other input in range.
	if (idx < size) return idx;
	return idx - size < size ? idx - size : idx % size;
}

// The 8 corner entries of a cell, all loads issued before any is consumed.  The x / x+1
// corners share one aligned load when both fall in it: a 16-B quad of entries (F = 2;
// the x+1 corner is in it unless x (hashed) or the index (dense) is 3 mod 4), else a pair
// (dense index even, or hashed with x even: index ^ 1); only the other lanes issue the
// second corner's own load.  The encoder is bound by the texture addresser (TA busy ~87 %
// of a render launch): fewer lanes in the lone-corner loads is what makes it faster.
__device__ __forceinline__ uint32_t quad_pick(const uint4& v, uint32_t k) {
	return k == 0 ? v.x : (k == 1 ? v.y : (k == 2 ? v.z : v.w));
}

template <uint32_t F, bool HASHED, bool QUAD = false>
__device__ __forceinline__ void gather_corners(const typename FeatVec<F>::T* __restrict__ tab, uint32_t size, uint32_t res,
                                               uint32_t gx, uint32_t gy, uint32_t gz, typename FeatVec<F>::T* vals) {
	using VT = typename FeatVec<F>::T;
	uint32_t i0[4], i1[4];
#pragma unroll
	for (uint32_t q = 0; q < 4; ++q) {
		const uint32_t yy = gy + (q & 1u), zz = gz + (q >> 1);
		i0[q] = corner_index<HASHED>(size, res, gx, yy, zz);
		i1[q] = corner_index<HASHED>(size, res, gx + 1u, yy, zz);
	}
	if constexpr (QUAD && F == 2 && !HASHED) {
		// dense level: the x+1 corner is the next entry (unless the index wraps at the level's
		// end), so one 8-B load at the x corner's entry fetches both -- 4 load instructions per
		// level instead of 4 quads + 4 masked lone loads (the encoder is bound by the texture
		// addresser's work per load instruction).  4-B aligned 8-B global loads are legal on
		// gfx950 (the compiler emits them for 4-B aligned memcpy).
		bool adj = true;
#pragma unroll
		for (uint32_t q = 0; q < 4; ++q) adj &= i1[q] == i0[q] + 1u;
		uint2 pr[4];
		if (adj) {
#pragma unroll
			for (uint32_t q = 0; q < 4; ++q) __builtin_memcpy(&pr[q], tab + i0[q], sizeof(uint2));
		}
		if (__ballot(!adj)) {  // a wrapped index (at most a few lanes, rarely any)
			if (!adj) {
#pragma unroll
				for (uint32_t q = 0; q < 4; ++q) pr[q] = make_uint2(tab[i0[q]], tab[i1[q]]);
			}
		}
#pragma unroll
		for (uint32_t q = 0; q < 4; ++q) {
			vals[2 * q] = pr[q].x;
			vals[2 * q + 1] = pr[q].y;
		}
	} else if constexpr (QUAD && F == 2) {
		// aligned 16-B quads of entries: the x+1 corner shares the x corner's quad unless x
		// (hashed) or the index (dense) is 3 mod 4 -- a quarter of the lanes load it alone
		const uint4* qtab = reinterpret_cast<const uint4*>(tab);
		uint4 qd[4];
		uint32_t lone[4];
#pragma unroll
		for (uint32_t q = 0; q < 4; ++q) qd[q] = qtab[i0[q] >> 2];
#pragma unroll
		for (uint32_t q = 0; q < 4; ++q)
			if ((i1[q] >> 2) != (i0[q] >> 2)) lone[q] = tab[i1[q]];
#pragma unroll
		for (uint32_t q = 0; q < 4; ++q) {
			vals[2 * q] = quad_pick(qd[q], i0[q] & 3u);
			vals[2 * q + 1] = (i1[q] >> 2) != (i0[q] >> 2) ? lone[q] : quad_pick(qd[q], i1[q] & 3u);
		}
	} else if constexpr (F <= 4) {
		using PT = typename PairVec<F>::T;
		const PT* ptab = reinterpret_cast<const PT*>(tab);
		PT pr[4];
		VT lone[4];
#pragma unroll
		for (uint32_t q = 0; q < 4; ++q) pr[q] = ptab[i0[q] >> 1];
#pragma unroll
		for (uint32_t q = 0; q < 4; ++q)
			if ((i1[q] ^ i0[q]) != 1u) lone[q] = tab[i1[q]];
#pragma unroll
		for (uint32_t q = 0; q < 4; ++q) {
			const VT* pv = reinterpret_cast<const VT*>(&pr[q]);
			const VT a = pv[0], b = pv[1];
			vals[2 * q] = (i0[q] & 1u) ? b : a;
			vals[2 * q + 1] = (i1[q] ^ i0[q]) != 1u ? lone[q] : ((i1[q] & 1u) ? b : a);
		}
	} else {
#pragma unroll
		for (uint32_t q = 0; q < 4; ++q) {
			vals[2 * q] = tab[i0[q]];
			vals[2 * q + 1] = tab[i1[q]];
		}
	}
}

template <uint32_t F, bool QUAD>
__device__ __forceinline__ typename FeatVec<F>::T encode_one(uint32_t level, float px, float py, float pz,
                                                             const __half* __restrict__ table, const LevelTable& lt) {
	const float scale = lt.scale[level];
	const uint32_t res = lt.res[level], size = lt.size[level], hashed = lt.hashed[level];
	using VT = typename FeatVec<F>::T;
	const VT* tab = reinterpret_cast<const VT*>(table + (size_t)lt.offset[level] * F);

	float fx, fy, fz;
	uint32_t gx, gy, gz;
	pos_fract(px, scale, &fx, &gx);
	pos_fract(py, scale, &fy, &gy);
	pos_fract(pz, scale, &fz, &gz);

	VT vals[8];
	if (hashed) {
		gather_corners<F, true, QUAD>(tab, size, res, gx, gy, gz, vals);
	} else if constexpr (F == 2) {
		// dense level with corner records (render site): two 16-B loads fetch the 8 corners
		// (the cell's z and z + 1 records) instead of four 8-B pairs -- the encoder is bound by
		// the texture addresser's work per load instruction.  Corners outside [0, res) (only
		// positions outside the unit cube) take the table path.
		if (lt.rec && gx < res && gy < res && gz < res) {
			const uint4* r = lt.rec + lt.rec_off[level] + gx + res * (gy + res * gz);
			const uint4 a = r[0], b = r[res * res];
			vals[0] = a.x; vals[1] = a.y; vals[2] = a.z; vals[3] = a.w;
			vals[4] = b.x; vals[5] = b.y; vals[6] = b.z; vals[7] = b.w;
		} else {
			gather_corners<F, false, QUAD>(tab, size, res, gx, gy, gz, vals);
		}
	} else {
		gather_corners<F, false, QUAD>(tab, size, res, gx, gy, gz, vals);
	}
	float acc[F];
#pragma unroll
	for (uint32_t f = 0; f < F; ++f) acc[f] = 0.0f;
#pragma unroll
	for (uint32_t c = 0; c < 8; ++c) {
		float w = 1.0f;
		w *= (c & 1u) ? fx : 1.0f - fx;
		w *= (c & 2u) ? fy : 1.0f - fy;
		w *= (c & 4u) ? fz : 1.0f - fz;
		float v[F];
		unpack<F>(vals[c], v);
#pragma unroll
		for (uint32_t f = 0; f < F; ++f) acc[f] = fmaf(w, v[f], acc[f]);
	}
	VT o;
	__half* oh = reinterpret_cast<__half*>(&o);
#pragma unroll
	for (uint32_t f = 0; f < F; ++f) {
		// round to fp32 first, then to fp16, as tcnn and the oracle do: without the barrier the
		// last fmaf and the conversion fold into v_fma_mixlo_f16 (one rounding), which differs
		// from the two roundings when the fp32 sum lies on an fp16 tie
		__asm__("" : "+v"(acc[f]));
		oh[f] = __float2half_rn(acc[f]);
	}
	return o;
}

}  // namespace ngp
