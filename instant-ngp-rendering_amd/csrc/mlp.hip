// mlp.hip — fused NeRF MLPs (density MLP + SH + rgb MLP) on gfx950 fp16 MFMA.
//
// Restates tiny-cuda-nn FullyFusedMLP<half, W> as composed by NerfNetwork
// (include/neural-graphics-primitives/nerf_network.h:81-139 forward, :189-268
// backward): enc --density MLP--> [density_out(16) | SH4(dir)(16)] --rgb MLP--> rgb.
//
// MI355X design
//  * v_mfma_f32_16x16x32_f16: A = weights (16 output rows x 32 inputs), B =
//    activations (32 inputs x 16 samples), C = 16 rows x 16 samples, fp32
//    accumulation (tcnn accumulates in fp16 WMMA fragments).
//  * inference (k_mlp_infer_rf: render, training forward, density grid) is
//    register-resident: a layer's C tiles are the next layer's B operands once
//    k_pack has permuted its K order, so activations never leave the VGPRs;
//    weight fragments live in LDS (one copy per workgroup).
//  * training (k_mlp_train: fwd + dgrad + wgrad in one persistent launch, 8
//    waves x 16 samples per 128-sample chunk): activations and deltas live in
//    LDS images [sample][row] (row stride padded by 16 B: conflict-free
//    ds_read_b128); weight gradients are sum_s delta[s][m] * a[s][k] with both
//    operands read sample-major through ds_read_b64_tr_b16 (hardware
//    transpose), accumulated in registers over the loop and written once per
//    workgroup as a row of partials that k_mlp_reduce sums in a fixed order.
#include <algorithm>

#include <cstring>

#include "encode_device.h"
#include "ngp_internal.h"

namespace ngp {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef short s4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef unsigned int v2u __attribute__((ext_vector_type(2)));

constexpr int SPW = 32;         // samples per wave
constexpr int CT = SPW / 16;    // 16-sample column tiles per wave
constexpr int WAVES = 4;
constexpr int BLOCK = WAVES * 64;
constexpr int SAMPLES_PER_BLOCK = WAVES * SPW;
constexpr int FRAG_HALVES = 512;  // 64 lanes x 8 halves
// the training kernel: 8 waves x 16 samples per workgroup (the same 128-sample chunk and
// 146 KiB LDS images as 4 x 32, but two waves per SIMD to hide the LDS round trips)
constexpr int TWAVES = 8;
constexpr int TSPW = 16;
constexpr int TCT = TSPW / 16;
constexpr int TBLOCK = TWAVES * 64;
static_assert(TWAVES * TSPW == SAMPLES_PER_BLOCK, "the training images hold one chunk");

// XE = 2: n_extra_dims 17..32 fill rows 32..63 (both K steps whole; the training images keep 64 rows).
// XE = 1: the rgb network's input carries the per-image latent code (NerfNetwork's n_extra_dims <= 16, the
// dir encoding's Identity part): [density out 16 | SH 16 | extra 16] = 48 rows, read as two 32-row K steps whose
// last 16 rows meet zero weights.  The training images then keep the rgb input segment last in a sample's row,
// 48 rows long: the second K step's rows 48..63 are the row's zeroed pad and the next row's first halves
// (finite values times zero weights), so the 160 KiB LDS budget holds.
template <int W_, int DH_, int RH_, int KE_, int XE_ = 0>
struct Net {
	static constexpr int W = W_, DH = DH_, RH = RH_, KE = KE_, XE = XE_;
	static constexpr int Wp = (W + 31) / 32 * 32;
	static constexpr int NL = DH + RH + 2;
	static constexpr int ENC_ROWS = 32 * KE;
	static constexpr int XROWS = XE == 2 ? 64 : (XE ? 48 : 32);  // rgb input rows kept in the training images
	static constexpr int out_dim(int l) { return (l == DH || l == NL - 1) ? 16 : W; }
	static constexpr int in_rows(int l) { return l == 0 ? ENC_ROWS : (l == DH + 1 ? (XE ? 64 : 32) : Wp); }
	static constexpr bool relu_out(int l) { return !(l == DH || l == NL - 1); }
	static constexpr bool relu_in(int l) { return !(l == 0 || l == DH + 1); }
	static constexpr int Mt(int l) { return out_dim(l) / 16; }
	static constexpr int Ks(int l) { return in_rows(l) / 32; }
	static constexpr int Ms(int l) { return (out_dim(l) + 31) / 32; }
	static constexpr int Kt(int l) { return in_rows(l) / 16; }
	// LDS image layouts (rows per sample); TRAIN keeps every activation for wgrad.
	template <bool TRAIN>
	static constexpr int rows() { return TRAIN ? ENC_ROWS + (DH + RH) * Wp + XROWS : ENC_ROWS + 2 * Wp + 32; }
	template <bool TRAIN>
	static constexpr int x_seg() { return TRAIN ? (XE ? ENC_ROWS + (DH + RH) * Wp : ENC_ROWS + DH * Wp) : ENC_ROWS + 2 * Wp; }
	template <bool TRAIN>
	static constexpr int dens_hidden(int h) { return TRAIN ? ENC_ROWS + h * Wp : ENC_ROWS + (h % 2) * Wp; }
	template <bool TRAIN>
	static constexpr int rgb_hidden(int r) {
		return TRAIN ? ENC_ROWS + DH * Wp + (XE ? 0 : 32) + r * Wp : ENC_ROWS + (r % 2) * Wp;
	}
	template <bool TRAIN>
	static constexpr int seg_in(int l) {
		return l == 0 ? 0 : (l <= DH ? dens_hidden<TRAIN>(l - 1) : (l == DH + 1 ? x_seg<TRAIN>() : rgb_hidden<TRAIN>(l - DH - 2)));
	}
	template <bool TRAIN>
	static constexpr int seg_out(int l) {
		return l < DH ? dens_hidden<TRAIN>(l) : (l == DH ? x_seg<TRAIN>() : (l < NL - 1 ? rgb_hidden<TRAIN>(l - DH - 1) : -1));
	}
	template <bool TRAIN>
	static constexpr int stride() { return rows<TRAIN>() + 8; }  // halves; +16 B breaks bank aliasing
	static constexpr int fwd_frags_upto(int L) {
		int s = 0;
		for (int l = 0; l < L; ++l) s += Mt(l) * Ks(l);
		return s;
	}
	static constexpr int fwd_frags() { return fwd_frags_upto(NL); }
	static constexpr int bwd_frags() {
		int s = 0;
		for (int l = 0; l < NL; ++l) s += Kt(l) * Ms(l);
		return s;
	}
	static constexpr int fwd_off(int l) { return fwd_frags_upto(l) * FRAG_HALVES; }
	// register-resident inference fragments (k_mlp_infer_rf): the forward fragments again,
	// with the K order of every layer after the first permuted to the C-register layout
	static constexpr int rfwd_off(int l) { return (fwd_frags() + bwd_frags() + fwd_frags_upto(l)) * FRAG_HALVES; }
	static constexpr int all_frags() { return 2 * fwd_frags() + bwd_frags(); }
	static constexpr int bwd_off(int l) {
		int s = fwd_frags();
		for (int i = 0; i < l; ++i) s += Kt(i) * Ms(i);
		return s * FRAG_HALVES;
	}
	// weight-gradient 16x16 tiles per layer of the [out][in] matrix
	static constexpr int KT16(int l) { return in_rows(l) / 16; }
	static constexpr int gtiles(int l) { return Mt(l) * KT16(l); }
	static constexpr int gtile_base(int l) {
		int s = 0;
		for (int i = 0; i < l; ++i) s += gtiles(i);
		return s;
	}
	static constexpr int tile_layer(int t) {
		int l = 0;
		while (l + 1 < NL && t >= gtile_base(l + 1)) ++l;
		return l;
	}
	static constexpr int slots() { return (gtile_base(NL) + WAVES - 1) / WAVES; }
	static constexpr int tslots() { return (gtile_base(NL) + TWAVES - 1) / TWAVES; }
	static constexpr int drows() { return Wp > 32 ? Wp : 32; }
	static constexpr int dstride() { return 2 * drows() + 8; }
	static constexpr size_t lds_train() {
		return (size_t)(fwd_frags() + bwd_frags()) * FRAG_HALVES * 2 + (size_t)WAVES * SPW * stride<true>() * 2 +
		       (size_t)WAVES * SPW * dstride() * 2;
	}
};

struct MlpArgs {
	const __half* frags;
	const __half* enc;
	uint32_t enc_plane;
	uint32_t enc_lsh, enc_gsh;  // EncLayout{enc_plane, enc_lsh, enc_gsh} of enc (denc: level-major)
	const float* coords;
	uint32_t coord_stride;
	uint32_t n;
	uint32_t E;        // encoding width (L*F)
	uint32_t F;
	uint32_t enc_pad;  // param input width of the first density layer (multiple of 16)
	__half* out;
	const __half* dloss;
	const float* weight;
	float* grads;
	__half* denc;
	uint64_t param_off[MAX_LAYERS];
	uint32_t param_in[MAX_LAYERS];
	const uint32_t* n_dev;  // optional device-side sample count (<= n)
	float* dsh;             // optional [n][16] dL/d(SH inputs) (camera gradients)
	uint32_t enc_bytes, coord_bytes, sh_bytes;  // buffer-resource extents (register-resident inference)
	uint32_t dir_offset;              // float offset of the direction in a coords record
	const __half* sh;                 // optional [rays][16] precomputed SH inputs (renderer), instead of directions,
	const uint32_t* sh_ray;           //   row of sample i: sh_ray[i] (the samples of a ray share its row)
	uint32_t out_mode, out_stride;    // 0: out [n][4]; 1 / 2: the reference's 16-row output, column- / row-major
	float* partials;                  // k_mlp_train: [workgroup][n_mlp_params] weight-gradient partials
	uint32_t n_mlp;                   // MLP parameter count (partials row pitch)
	uint32_t skip_unfilled;           // SH-row inference: skip column tiles whose rows are all NO_SH_ROW
	uint32_t prio;                    // SH-row inference (renderer): wave issue priority (ngp_tuning.render_priority bits 2-3)
	// Net::XE (n_extra_dims > 0): the latent codes, fp32 rows of NGP_EXTRA_ROW (zero past n_extra_dims); sample i reads row
	// sample_img[i] (training: the sample's image), or row 0 without sample_img (rendering: the rendering code)
	const float* extra;
	const uint32_t* sample_img;
	float* dextra;  // optional [n][NGP_EXTRA_ROW] dL/d(latent code) of each sample's own row (the extra dims' gradient)
};

__device__ __forceinline__ f4 mfma(h8 a, h8 b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0); }
__device__ __forceinline__ h8 lds_h8(const _Float16* p) { return *reinterpret_cast<const h8*>(p); }
__device__ __forceinline__ void lds_st_h4(_Float16* p, h4 v) { *reinterpret_cast<h4*>(p) = v; }
__device__ __forceinline__ void lds_st_h8(_Float16* p, h8 v) { *reinterpret_cast<h8*>(p) = v; }
__device__ __forceinline__ h4 tr_read(const _Float16* p) {
	s4 r = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(p));
	return __builtin_bit_cast(h4, r);
}
__device__ __forceinline__ _Float16 u16h(uint32_t u) { return __builtin_bit_cast(_Float16, (uint16_t)(u & 0xffffu)); }
__device__ __forceinline__ uint32_t n_chunks_of(uint32_t n) { return (n + SAMPLES_PER_BLOCK - 1) / SAMPLES_PER_BLOCK; }

// This wave's SPW samples of the encoding (EncLayout) -> image rows [0, ENC_ROWS).
template <class N, int STRIDE, int SPW_ = SPW>
__device__ __forceinline__ void load_encoding(const MlpArgs& a, _Float16* img, uint32_t base, int lane) {
	constexpr int CHUNKS = N::ENC_ROWS / 8;
	for (int t = lane; t < SPW_ * CHUNKS; t += 64) {
		const int smp = t % SPW_, chunk = t / SPW_;
		const uint32_t i = base + smp;
		const uint32_t k0 = chunk * 8;
		h8 v = {0, 0, 0, 0, 0, 0, 0, 0};
		if (i < a.n && k0 < a.E) {
			const EncLayout lay{a.enc_plane, a.enc_lsh, a.enc_gsh};
			if (a.F == 2 && k0 + 8 <= a.E) {
				const uint32_t* e = reinterpret_cast<const uint32_t*>(a.enc);
#pragma unroll
				for (int q = 0; q < 4; ++q) {
					const uint32_t u = e[lay.vec(k0 / 2 + q, i)];
					v[2 * q] = u16h(u);
					v[2 * q + 1] = u16h(u >> 16);
				}
			} else if (a.F == 4 && k0 + 8 <= a.E) {
				const uint2* e = reinterpret_cast<const uint2*>(a.enc);
#pragma unroll
				for (int q = 0; q < 2; ++q) {
					const uint2 u = e[lay.vec(k0 / 4 + q, i)];
					v[4 * q + 0] = u16h(u.x);
					v[4 * q + 1] = u16h(u.x >> 16);
					v[4 * q + 2] = u16h(u.y);
					v[4 * q + 3] = u16h(u.y >> 16);
				}
			} else {
				const uint16_t* e = reinterpret_cast<const uint16_t*>(a.enc);
				for (int j = 0; j < 8; ++j) {
					const uint32_t k = k0 + j;
					if (k < a.E) {
						const uint32_t lvl = k / a.F, f = k % a.F;
						v[j] = __builtin_bit_cast(_Float16, e[lay.vec(lvl, i) * a.F + f]);
					}
				}
			}
		}
		lds_st_h8(img + smp * STRIDE + k0, v);
	}
}

// Spherical harmonics, degree 4, of the warped direction (tcnn SphericalHarmonicsEncoding;
// configs/nerf/base.json:37-49) into rows [x_seg+16, x_seg+32).
template <int STRIDE, int SPW_ = SPW>
__device__ __forceinline__ void load_sh(const MlpArgs& a, _Float16* img, int x_seg, uint32_t base, int lane) {
	for (int t = lane; t < SPW_ * 2; t += 64) {
		const int smp = t % SPW_, half = t / SPW_;
		const uint32_t i = base + smp;
		h8 v = {0, 0, 0, 0, 0, 0, 0, 0};
		if (i < a.n) {
			const float* c = a.coords ? a.coords + (size_t)i * a.coord_stride : nullptr;
			const float x = c ? c[4] * 2.0f - 1.0f : 0.0f, y = c ? c[5] * 2.0f - 1.0f : 0.0f, z = c ? c[6] * 2.0f - 1.0f : 0.0f;
			const float xy = x * y, xz = x * z, yz = y * z, x2 = x * x, y2 = y * y, z2 = z * z;
			if (half == 0) {
				v[0] = (_Float16)(0.28209479177387814f);
				v[1] = (_Float16)(-0.48860251190291987f * y);
				v[2] = (_Float16)(0.48860251190291987f * z);
				v[3] = (_Float16)(-0.48860251190291987f * x);
				v[4] = (_Float16)(1.0925484305920792f * xy);
				v[5] = (_Float16)(-1.0925484305920792f * yz);
				v[6] = (_Float16)(0.94617469575755997f * z2 - 0.31539156525251999f);
				v[7] = (_Float16)(-1.0925484305920792f * xz);
			} else {
				v[0] = (_Float16)(0.54627421529603959f * x2 - 0.54627421529603959f * y2);
				v[1] = (_Float16)(0.59004358992664352f * y * (-3.0f * x2 + y2));
				v[2] = (_Float16)(2.8906114426405538f * xy * z);
				v[3] = (_Float16)(0.45704579946446572f * y * (1.0f - 5.0f * z2));
				v[4] = (_Float16)(0.3731763325901154f * z * (5.0f * z2 - 3.0f));
				v[5] = (_Float16)(0.45704579946446572f * x * (1.0f - 5.0f * z2));
				v[6] = (_Float16)(1.4453057213202769f * z * (x2 - y2));
				v[7] = (_Float16)(0.59004358992664352f * x * (-x2 + 3.0f * y2));
			}
		}
		lds_st_h8(img + smp * STRIDE + x_seg + 16 + 8 * half, v);
	}
}

// One forward layer for this wave's CT column tiles.  Output rows go to LDS
// segment seg_out, or (final rgb layer) are returned in `res`.
template <class N, bool TRAIN, int l, int CT_ = CT>
__device__ __forceinline__ void fwd_layer(const _Float16* frags, _Float16* img, int lane, f4 (&res)[CT_]) {
	constexpr int STRIDE = N::template stride<TRAIN>();
	constexpr int MT = N::Mt(l), KS = N::Ks(l);
	constexpr int SIN = N::template seg_in<TRAIN>(l), SOUT = N::template seg_out<TRAIN>(l);
	const int g = lane >> 4, n = lane & 15;
	h8 b[CT_][KS];
#pragma unroll
	for (int c = 0; c < CT_; ++c)
#pragma unroll
		for (int s = 0; s < KS; ++s) b[c][s] = lds_h8(img + (16 * c + n) * STRIDE + SIN + 32 * s + 8 * g);
	const _Float16* fr = frags + N::fwd_off(l);
#pragma unroll
	for (int mt = 0; mt < MT; ++mt) {
		h8 a[KS];
#pragma unroll
		for (int s = 0; s < KS; ++s) a[s] = lds_h8(fr + ((mt * KS + s) * 64 + lane) * 8);
#pragma unroll
		for (int c = 0; c < CT_; ++c) {
			f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
			for (int s = 0; s < KS; ++s) acc = mfma(a[s], b[c][s], acc);
			if constexpr (N::relu_out(l)) {
#pragma unroll
				for (int r = 0; r < 4; ++r) acc[r] = fmaxf(acc[r], 0.0f);
			}
			if constexpr (SOUT >= 0) {
				h4 o = {(_Float16)acc[0], (_Float16)acc[1], (_Float16)acc[2], (_Float16)acc[3]};
				lds_st_h4(img + (16 * c + n) * STRIDE + SOUT + 16 * mt + 4 * g, o);
			} else {
				res[c] = acc;
			}
		}
	}
}

template <class N, bool TRAIN, int l, int END, int CT_ = CT>
__device__ __forceinline__ void fwd_range(const _Float16* frags, _Float16* img, int lane, f4 (&res)[CT_]) {
	if constexpr (l < END) {
		fwd_layer<N, TRAIN, l, CT_>(frags, img, lane, res);
		fwd_range<N, TRAIN, l + 1, END, CT_>(frags, img, lane, res);
	}
}

// ---------------------------------------------------------------------------
// Register-resident inference (no LDS).  For v_mfma_f32_16x16x32_f16 lane (g, n) holds
// C[4g + r][n] (r < 4) of a 16-row output tile and B[8g + j][n] (j < 8) of a 32-row
// input step.  Two consecutive output tiles 2s, 2s+1 therefore ARE the next layer's
// K-step s once the K order is permuted: position 8g + j <-> input row
// 32s + (j < 4 ? 4g + j : 16 + 4g + j - 4).  k_pack applies that permutation to the
// weights (rfwd fragments), so a layer's fp32 accumulators become the next layer's
// fp16 B operands in place, and all weight fragments live in VGPRs for the whole
// persistent loop.  Each wave streams tiles of 16*CT samples and prefetches the next
// tile's encoding and direction while the current one runs through the MFMAs.
// ---------------------------------------------------------------------------
template <class N, int CT_>
struct RawTile {
	uint32_t e[CT_][8 * N::KE];  // encoding halves of this lane's K slots, packed in pairs where F >= 2
	float d[CT_][3];             // warped direction, or
	uint32_t h[CT_][2];          // SH inputs 4g .. 4g+3 (precomputed rows)
	uint32_t ri[CT_];            // SHIN: the samples' SH row indices
	uint32_t x[CT_][N::XE == 2 ? 4 : 2];  // Net::XE: latent-code components 4g .. 4g+3 (and 16 + 4g .. +3: XE 2), fp16 pairs
};

// Buffer resource over a device array (raw buffer, 32-bit byte offsets; reads past
// num_records return 0).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, uint32_t bytes) {
	return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

// Loads this lane's share of a tile: encoding features 32s + 8g .. +7 of sample
// base + 16c + n and its direction.  FF: 2 / 4 = F of a level-major encoding (one load per
// level), 12 / 14 = F = 2 / 4 in four-level planes (EncLayout lsh = 2: one 16-B load per
// K step; the K order is then the planes' and k_pack permutes the first layer to match),
// 0 = any layout, element by element.  SHIN: the direction inputs are precomputed per-ray SH
// rows (8 B per lane group) instead of a direction the lane expands itself: this loads the
// samples' row indices (first, so a later wait for them leaves the encoding loads in flight);
// sh_load fetches the rows one ring stage later.
// the SH rows of a ring slot whose row indices were loaded one stage earlier
template <class N, int CT_>
__device__ __forceinline__ void sh_load(__amdgpu_buffer_rsrc_t sh_rs, int g, RawTile<N, CT_>& r) {
#pragma unroll
	for (int c = 0; c < CT_; ++c) {
		const auto v = __builtin_amdgcn_raw_buffer_load_b64(sh_rs, 32 * r.ri[c] + 8 * g, 0, 0);
		r.h[c][0] = v[0];
		r.h[c][1] = v[1];
	}
}

template <class N, int CT_, int FF, bool SHIN>
__device__ __forceinline__ void rf_load(const MlpArgs& a, __amdgpu_buffer_rsrc_t enc_rs, __amdgpu_buffer_rsrc_t crd_rs,
                                        uint32_t base, int g, int n, RawTile<N, CT_>& r, bool want_dir) {
	if (want_dir && SHIN) {
#pragma unroll
		for (int c = 0; c < CT_; ++c) r.ri[c] = __builtin_amdgcn_raw_buffer_load_b32(crd_rs, 4 * (base + 16 * c + n), 0, 0);
	}
#pragma unroll
	for (int c = 0; c < CT_; ++c) {
		const uint32_t i = base + 16 * c + n;
#pragma unroll
		for (int s = 0; s < N::KE; ++s) {
			const uint32_t k0 = 32 * s + 8 * g;
			if constexpr (FF == 12) {
				// K positions 32s + 8g .. +7 = plane 4s + g (levels 4s + g + qG, q < 4); planes past
				// the encoding lie past the buffer's extent: the load returns 0
				const auto v = __builtin_amdgcn_raw_buffer_load_b128(enc_rs, 16 * ((4 * s + g) * a.enc_plane + i), 0, 0);
#pragma unroll
				for (int q = 0; q < 4; ++q) r.e[c][4 * s + q] = v[q];
			} else if constexpr (FF == 14) {
				// K positions 32s + 8g .. +7 = half g & 1 of plane 2s + g/2
				const uint32_t o = 32 * ((2 * s + (g >> 1)) * a.enc_plane + i) + 16 * (g & 1);
				const auto v = __builtin_amdgcn_raw_buffer_load_b128(enc_rs, o, 0, 0);
#pragma unroll
				for (int q = 0; q < 4; ++q) r.e[c][4 * s + q] = v[q];
			} else if constexpr (FF == 2) {
#pragma unroll
				for (int q = 0; q < 4; ++q) {
					// levels past the encoding lie past the buffer's extent: the load returns 0
					const uint32_t lvl = k0 / 2 + q;
					r.e[c][4 * s + q] = __builtin_amdgcn_raw_buffer_load_b32(enc_rs, 4 * (lvl * a.enc_plane + i), 0, 0);
				}
			} else if constexpr (FF == 4) {
#pragma unroll
				for (int q = 0; q < 2; ++q) {
					const uint32_t lvl = k0 / 4 + q;
					const auto v = __builtin_amdgcn_raw_buffer_load_b64(enc_rs, 8 * (lvl * a.enc_plane + i), 0, 0);
					r.e[c][4 * s + 2 * q] = v[0];
					r.e[c][4 * s + 2 * q + 1] = v[1];
				}
			} else {
				const uint16_t* e = reinterpret_cast<const uint16_t*>(a.enc);
				const EncLayout lay{a.enc_plane, a.enc_lsh, a.enc_gsh};
#pragma unroll
				for (int q = 0; q < 4; ++q) {
					uint32_t pair = 0;
#pragma unroll
					for (int h = 0; h < 2; ++h) {
						const uint32_t k = k0 + 2 * q + h;
						if (i < a.n && k < a.E) {
							const uint32_t lvl = k / a.F, f = k % a.F;
							pair |= (uint32_t)e[lay.vec(lvl, i) * a.F + f] << (16 * h);
						}
					}
					r.e[c][4 * s + q] = pair;
				}
			}
		}
		if constexpr (N::XE) {
			if (want_dir) {
				const uint32_t row = a.sample_img && i < a.n ? a.sample_img[i] : 0u;
#pragma unroll
				for (int hh = 0; hh < N::XE; ++hh) {
					const float4 v = *reinterpret_cast<const float4*>(a.extra + (size_t)row * NGP_EXTRA_ROW + 16 * hh + 4 * g);
					const h4 hv = {(_Float16)v.x, (_Float16)v.y, (_Float16)v.z, (_Float16)v.w};
					const uint2 u = __builtin_bit_cast(uint2, hv);
					r.x[c][2 * hh] = u.x;
					r.x[c][2 * hh + 1] = u.y;
				}
			}
		}
		if (want_dir && SHIN) {
		} else if (want_dir) {
			const uint32_t o = 4 * (i * a.coord_stride + a.dir_offset);
			r.d[c][0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(crd_rs, o, 0, 0));
			r.d[c][1] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(crd_rs, o + 4, 0, 0));
			r.d[c][2] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(crd_rs, o + 8, 0, 0));
		}
	}
}

__device__ __forceinline__ h8 pack_h8(uint32_t u0, uint32_t u1, uint32_t u2, uint32_t u3) {
	const uint4 v = make_uint4(u0, u1, u2, u3);
	return __builtin_bit_cast(h8, v);
}
__device__ __forceinline__ h8 c_to_b(const f4& lo, const f4& hi) {
	return h8{(_Float16)lo[0], (_Float16)lo[1], (_Float16)lo[2], (_Float16)lo[3],
	          (_Float16)hi[0], (_Float16)hi[1], (_Float16)hi[2], (_Float16)hi[3]};
}

// SH degree 4 components 4g .. 4g+3 of the warped direction (same formulas as load_sh).
// The compiler turns the g-select into four short divergent paths, which measured
// cheaper than computing all 16 components and blending.
__device__ __forceinline__ void sh4_slice(const float* dw, int g, float (&o)[4]) {
	float v[16];
	sh_deg4(dw[0], dw[1], dw[2], v);
#pragma unroll
	for (int r = 0; r < 4; ++r) o[r] = g == 0 ? v[r] : g == 1 ? v[4 + r] : g == 2 ? v[8 + r] : v[12 + r];
}

// one layer: B operands in (KS steps) -> C tiles out (MT tiles), weights w[frag].  Every weight fragment
// is read from LDS once and feeds the CT column tiles' MFMAs; there is no per-tile branch (a branch
// around each MFMA keeps the compiler from sharing the fragment reads: one LDS round trip per MFMA)
template <class N, int l, int CT_>
__device__ __forceinline__ void rf_layer(const h8* w, const h8 (&bin)[CT_][2], f4 (&cout)[CT_][4]) {
	constexpr int MT = N::Mt(l), KS = N::Ks(l), F0 = N::fwd_frags_upto(l);
	h8 a[MT][KS];
#pragma unroll
	for (int mt = 0; mt < MT; ++mt)
#pragma unroll
		for (int s = 0; s < KS; ++s) a[mt][s] = w[(F0 + mt * KS + s) * 64];
#pragma unroll
	for (int mt = 0; mt < MT; ++mt)
#pragma unroll
		for (int c = 0; c < CT_; ++c) {
			f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
			for (int s = 0; s < KS; ++s) acc = mfma(a[mt][s], bin[c][s], acc);
			cout[c][mt] = acc;  // ReLU (hidden layers) is applied by rf_chain on the packed halves
		}
}

// C tiles of a hidden layer -> ReLU'd B operands of the next layer (missing tiles are
// zero).  ReLU commutes with the rounding to fp16, so it runs on the packed halves.
template <int MT, int CT_>
__device__ __forceinline__ void rf_chain(const f4 (&cin)[CT_][4], h8 (&bout)[CT_][2]) {
	const f4 z = {0.f, 0.f, 0.f, 0.f};
	typedef _Float16 h2v __attribute__((ext_vector_type(2)));
#pragma unroll
	for (int c = 0; c < CT_; ++c)
#pragma unroll
		for (int s = 0; s < 2; ++s)
			if (2 * s < MT) {
				h8 v = c_to_b(cin[c][2 * s], 2 * s + 1 < MT ? cin[c][2 * s + 1] : z);
#pragma unroll
				for (int q = 0; q < 4; ++q) {
					h2v p = {v[2 * q], v[2 * q + 1]};
					p = __builtin_elementwise_max(p, h2v{(_Float16)0, (_Float16)0});
					v[2 * q] = p[0];
					v[2 * q + 1] = p[1];
				}
				bout[c][s] = v;
			}
}

template <class N, int l, int END, int CT_>
__device__ __forceinline__ void rf_hidden_range(const h8* w, h8 (&b)[CT_][2], f4 (&c)[CT_][4]) {
	if constexpr (l < END) {
		rf_layer<N, l, CT_>(w, b, c);
		rf_chain<N::Mt(l), CT_>(c, b);
		rf_hidden_range<N, l + 1, END, CT_>(w, b, c);
	}
}

// The tile pipeline is PF deep: every wave keeps PF tiles' loads in flight (register
// ring, statically indexed by unrolling the loop PF times) -- the kernel is bound by
// memory latency x bytes in flight, not by the MFMAs (20 per 16 samples).  Weight
// fragments are read from LDS (one copy per workgroup) to leave the VGPRs to the ring.
template <class N, int CT_, int PF, bool DENSITY_ONLY, bool SHIN>
__device__ __forceinline__ void rf_tile(const MlpArgs& a, const h8* w, const RawTile<N, CT_>& cur, uint32_t base, int g,
                                        int n, int32_t live_pre = -1) {
	h8 b[CT_][2];
	f4 c[CT_][4];
#pragma unroll
	for (int cc = 0; cc < CT_; ++cc)
#pragma unroll
		for (int s = 0; s < N::KE; ++s)
			b[cc][s] = pack_h8(cur.e[cc][4 * s], cur.e[cc][4 * s + 1], cur.e[cc][4 * s + 2], cur.e[cc][4 * s + 3]);
	// SH-row inputs (renderer): a wave step whose slots no ray filled (k_generate marks them with row
	// NO_SH_ROW) is not computed -- k_composite reads a ray's filled samples only.  A step with any filled
	// slot computes all its tiles (branch-free MFMA chains)
	uint32_t live = (1u << CT_) - 1u;
	if constexpr (SHIN && !DENSITY_ONLY) {
		if (a.skip_unfilled) {
			if (live_pre >= 0) {
				live = (uint32_t)live_pre;  // computed when the tile's SH rows were fetched (k_mlp_infer_sh)
			} else {
				live = 0;
#pragma unroll
				for (int cc = 0; cc < CT_; ++cc) live |= (__ballot(cur.ri[cc] != NO_SH_ROW) != 0ull ? 1u : 0u) << cc;
			}
			if (live == 0) return;
		}
	}
	rf_hidden_range<N, 0, N::DH, CT_>(w, b, c);
	rf_layer<N, N::DH, CT_>(w, b, c);
	if constexpr (DENSITY_ONLY) {
		if (g == 0) {
#pragma unroll
			for (int cc = 0; cc < CT_; ++cc) {
				const uint32_t i = base + 16 * cc + n;
				if (i < a.n) a.out[i] = __builtin_bit_cast(__half, (_Float16)c[cc][0][0]);
			}
		}
	} else {
		_Float16 dens[CT_];
#pragma unroll
		for (int cc = 0; cc < CT_; ++cc) {
			dens[cc] = (_Float16)c[cc][0][0];
			if constexpr (SHIN) {
				const h4 lo = {(_Float16)c[cc][0][0], (_Float16)c[cc][0][1], (_Float16)c[cc][0][2], (_Float16)c[cc][0][3]};
				const uint2 lu = __builtin_bit_cast(uint2, lo);
				b[cc][0] = pack_h8(lu.x, lu.y, cur.h[cc][0], cur.h[cc][1]);  // rgb input: [density out 16 | SH 16]
			} else {
				float sh[4];
				sh4_slice(cur.d[cc], g, sh);
				const f4 shv = {sh[0], sh[1], sh[2], sh[3]};
				b[cc][0] = c_to_b(c[cc][0], shv);  // rgb input: [density out 16 | SH 16]
			}
			// the latent code (rgb input rows 32..47; the K permutation puts rows 32 + 4g .. +3 in slots 0..3)
			if constexpr (N::XE == 1) b[cc][1] = pack_h8(cur.x[cc][0], cur.x[cc][1], 0u, 0u);
			// XE 2: slots 4..7 of the second K step are rgb input rows 48 + 4g .. +3 = code components 16 + 4g .. +3
			if constexpr (N::XE == 2) b[cc][1] = pack_h8(cur.x[cc][0], cur.x[cc][1], cur.x[cc][2], cur.x[cc][3]);
		}
		rf_hidden_range<N, N::DH + 1, N::NL - 1, CT_>(w, b, c);
		rf_layer<N, N::NL - 1, CT_>(w, b, c);
		if (a.out_mode == 0) {
			if (g == 0) {
#pragma unroll
				for (int cc = 0; cc < CT_; ++cc) {
					const uint32_t i = base + 16 * cc + n;
					if (i < a.n && ((live >> cc) & 1u)) {
						const h4 o = {(_Float16)c[cc][0][0], (_Float16)c[cc][0][1], (_Float16)c[cc][0][2], dens[cc]};
						*reinterpret_cast<h4*>(a.out + (size_t)i * 4) = o;
					}
				}
			}
		} else {
			// all 16 output rows: lane group g holds rows 4g .. 4g+3; row 3 is the density (extract_density)
#pragma unroll
			for (int cc = 0; cc < CT_; ++cc) {
				const uint32_t i = base + 16 * cc + n;
				if (i >= a.n) continue;
				h4 o = {(_Float16)c[cc][0][0], (_Float16)c[cc][0][1], (_Float16)c[cc][0][2], (_Float16)c[cc][0][3]};
				if (g == 0) o[3] = dens[cc];
				if (a.out_mode == 1) {
					*reinterpret_cast<h4*>(a.out + (size_t)i * a.out_stride + 4 * g) = o;
				} else {
#pragma unroll
					for (int r = 0; r < 4; ++r) {
							const _Float16 v = o[r];  // (a bit_cast of the vector element itself read element 0)
							a.out[(size_t)(4 * g + r) * a.out_stride + i] = __builtin_bit_cast(__half, v);
						}
				}
			}
		}
	}
}

template <class N, int CT_, int PF, bool DENSITY_ONLY, int FF, bool SHIN = false>
__global__ void __launch_bounds__(BLOCK) k_mlp_infer_rf(MlpArgs a) {
	static_assert(N::KE <= 2 && N::Wp <= 64, "register layout assumes <= 2 K-steps per layer");
	if (a.n_dev) a.n = min(a.n, *a.n_dev);
	if constexpr (SHIN) set_wave_priority(a.prio);
	constexpr int NF = DENSITY_ONLY ? N::fwd_frags_upto(N::DH + 1) : N::fwd_frags();
	extern __shared__ __attribute__((aligned(16))) char smem[];
	h8* w = reinterpret_cast<h8*>(smem);  // [frag][lane]
	{
		const h8* src = reinterpret_cast<const h8*>(a.frags + N::rfwd_off(0));
		for (int t = threadIdx.x; t < NF * 64; t += BLOCK) w[t] = src[t];
	}
	__syncthreads();
	const int lane = threadIdx.x & 63, g = lane >> 4, n = lane & 15;
	const h8* wl = w + lane;  // fragment f of this lane: wl[f * 64]
	constexpr uint32_t TS = 16 * CT_;
	const uint32_t n_tiles = (a.n + TS - 1) / TS;
	const uint32_t stride = gridDim.x * WAVES;
	// wave-uniform tile index (scalar registers: the ring's guards are scalar branches)
	const uint32_t t0 = __builtin_amdgcn_readfirstlane(blockIdx.x * WAVES + (threadIdx.x >> 6));
	const __amdgpu_buffer_rsrc_t enc_rs = make_rsrc(a.enc, a.enc_bytes);
	const __amdgpu_buffer_rsrc_t crd_rs = make_rsrc(SHIN ? (const void*)a.sh_ray : (const void*)a.coords, DENSITY_ONLY ? 0u : a.coord_bytes);
	const __amdgpu_buffer_rsrc_t sh_rs = make_rsrc(a.sh, SHIN && !DENSITY_ONLY ? a.sh_bytes : 0u);
	constexpr bool SHR = SHIN && !DENSITY_ONLY;
	// PF tiles' loads in flight in a ring of PF + 1 slots, the loop unrolled PF + 1 times so every slot
	// index is static: step q consumes slot q and loads tile t + PF stride into the slot step q - 1
	// consumed -- no register copies between the ring and the tile being computed
	constexpr int R = PF + 1;
	RawTile<N, CT_> ring[R];
	// The ring's loads are issued unconditionally (k_mlp_infer_sh, round 6): a branch around them made the compiler's
	// s_waitcnt bookkeeping fall back at the merges -- each step waited for the loads it had just issued (the
	// training forward and the density-grid evaluation: vmcnt(1) right after the next tile's direction and
	// encoding loads).  A tile past the end reads through descriptors of zero extent (no traffic; zeros) and is
	// never computed.  FF 0 / 2 / 4 (the element-wise and level-major loads) keep their own guards.
	const __amdgpu_buffer_rsrc_t none_rs = make_rsrc(a.enc, 0u);
#pragma unroll
	for (int q = 0; q < PF; ++q) {
		const uint32_t t = t0 + q * stride;
		rf_load<N, CT_, FF, SHIN>(a, t < n_tiles ? enc_rs : none_rs, t < n_tiles ? crd_rs : none_rs, t * TS, g, n, ring[q],
		                          !DENSITY_ONLY);
	}
	if constexpr (SHR) sh_load<N, CT_>(sh_rs, g, ring[0]);
	for (uint32_t tb = t0; tb < n_tiles; tb += R * stride) {
#pragma unroll
		for (int q = 0; q < R; ++q) {
			const uint32_t t = tb + q * stride;
			if (t >= n_tiles) break;
			const uint32_t tn = t + PF * stride;
			rf_load<N, CT_, FF, SHIN>(a, tn < n_tiles ? enc_rs : none_rs, tn < n_tiles ? crd_rs : none_rs, tn * TS, g, n,
			                          ring[(q + PF) % R], !DENSITY_ONLY);
			if constexpr (SHR) {
				// SH rows of the next tile to consume (its row indices were issued with its encoding; with
				// PF = 1 that is the tile just loaded)
				sh_load<N, CT_>(sh_rs, g, ring[(q + 1) % R]);
			}
			rf_tile<N, CT_, PF, DENSITY_ONLY, SHIN>(a, wl, ring[q], t * TS, g, n);
		}
	}
}

// ---------------------------------------------------------------------------
// The renderer's network call with a decoupled load pipeline (ngp_tuning.render_mlp_pipeline 2 / 3).
// k_mlp_infer_rf's SH-row path fetches a tile's SH rows right after issuing its row indices, so every wave
// step waits one full memory latency for the indices before it computes (round 5: the waves were parked at
// s_waitcnt 55 % of their cycles in the standalone 2^21-sample microbench, profiles/r06_mlp_microbench_*).
// Here every load a step waits for was issued at least one step earlier: at the step computing tile t a
// wave issues the SH rows of tile t+1 (their row indices came PF steps earlier), the row indices of tile
// t+PF+1 and the encodings of tile t+PF, then computes tile t.  A tile's live mask (column tiles holding a
// filled slot) is taken when its SH rows are fetched, so its row-index registers are free for the indices
// of the tile PF+1 steps ahead.  Same arithmetic as k_mlp_infer_rf (bit-identical outputs).
// ---------------------------------------------------------------------------
template <class N, int CT_>
__device__ __forceinline__ void ri_load(__amdgpu_buffer_rsrc_t crd_rs, uint32_t base, int n, RawTile<N, CT_>& r) {
#pragma unroll
	for (int c = 0; c < CT_; ++c) r.ri[c] = __builtin_amdgcn_raw_buffer_load_b32(crd_rs, 4 * (base + 16 * c + n), 0, 0);
}

template <class N, int CT_>
__device__ __forceinline__ uint32_t sh_load_live(__amdgpu_buffer_rsrc_t sh_rs, int g, RawTile<N, CT_>& r, bool skip) {
	sh_load<N, CT_>(sh_rs, g, r);
	uint32_t live = (1u << CT_) - 1u;
	if (skip) {
		live = 0;
#pragma unroll
		for (int cc = 0; cc < CT_; ++cc) live |= (__ballot(r.ri[cc] != NO_SH_ROW) != 0ull ? 1u : 0u) << cc;
	}
	return __builtin_amdgcn_readfirstlane(live);
}

// One wave step of k_mlp_infer_sh: rf_tile's SH-row path with the renderer's [n][4] output only, stored through a
// buffer resource whose extent is the device-side sample count (the stores past it are dropped by the hardware:
// no per-sample compare, 32-bit offsets instead of 64-bit address arithmetic per column tile)
template <class N, int CT_>
__device__ __forceinline__ void sh_tile(const h8* w, const RawTile<N, CT_>& cur, __amdgpu_buffer_rsrc_t out_rs, uint32_t base,
                                        int g, int n, uint32_t live) {
	if (live == 0) return;
	h8 b[CT_][2];
	f4 c[CT_][4];
#pragma unroll
	for (int cc = 0; cc < CT_; ++cc)
#pragma unroll
		for (int s = 0; s < N::KE; ++s)
			b[cc][s] = pack_h8(cur.e[cc][4 * s], cur.e[cc][4 * s + 1], cur.e[cc][4 * s + 2], cur.e[cc][4 * s + 3]);
	rf_hidden_range<N, 0, N::DH, CT_>(w, b, c);
	rf_layer<N, N::DH, CT_>(w, b, c);
	h4 dens[CT_];
#pragma unroll
	for (int cc = 0; cc < CT_; ++cc) {
		dens[cc] = h4{(_Float16)c[cc][0][0], (_Float16)c[cc][0][1], (_Float16)c[cc][0][2], (_Float16)c[cc][0][3]};
		const uint2 lu = __builtin_bit_cast(uint2, dens[cc]);
		b[cc][0] = pack_h8(lu.x, lu.y, cur.h[cc][0], cur.h[cc][1]);  // rgb input: [density out 16 | SH 16]
	}
	rf_hidden_range<N, N::DH + 1, N::NL - 1, CT_>(w, b, c);
	rf_layer<N, N::NL - 1, CT_>(w, b, c);
	if (g == 0) {
#pragma unroll
		for (int cc = 0; cc < CT_; ++cc) {
			if ((live >> cc) & 1u) {
				const h4 o = {(_Float16)c[cc][0][0], (_Float16)c[cc][0][1], (_Float16)c[cc][0][2], dens[cc][0]};
				const uint2 u = __builtin_bit_cast(uint2, o);
				__builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, u), out_rs, 8 * (base + 16 * cc + n), 0, 0);
			}
		}
	}
}

template <class N, int CT_, int PF, int FF>
__global__ void __launch_bounds__(BLOCK) k_mlp_infer_sh(MlpArgs a) {
	static_assert(N::KE <= 2 && N::Wp <= 64 && N::XE == 0, "register layout assumes <= 2 K-steps per layer, no extra dims");
	if (a.n_dev) a.n = min(a.n, *a.n_dev);
	set_wave_priority(a.prio);
	constexpr int NF = N::fwd_frags();
	extern __shared__ __attribute__((aligned(16))) char smem[];
	h8* w = reinterpret_cast<h8*>(smem);  // [frag][lane]
	{
		const h8* src = reinterpret_cast<const h8*>(a.frags + N::rfwd_off(0));
		for (int t = threadIdx.x; t < NF * 64; t += BLOCK) w[t] = src[t];
	}
	__syncthreads();
	const int lane = threadIdx.x & 63, g = lane >> 4, n = lane & 15;
	const h8* wl = w + lane;
	constexpr uint32_t TS = 16 * CT_;
	const uint32_t n_tiles = (a.n + TS - 1) / TS;
	const uint32_t stride = gridDim.x * WAVES;
	const uint32_t t0 = __builtin_amdgcn_readfirstlane(blockIdx.x * WAVES + (threadIdx.x >> 6));
	const __amdgpu_buffer_rsrc_t enc_rs = make_rsrc(a.enc, a.enc_bytes);
	const __amdgpu_buffer_rsrc_t crd_rs = make_rsrc(a.sh_ray, a.coord_bytes);
	const __amdgpu_buffer_rsrc_t sh_rs = make_rsrc(a.sh, a.sh_bytes);
	const bool skip = a.skip_unfilled != 0;
	const __amdgpu_buffer_rsrc_t out_rs = make_rsrc(a.out, 8u * a.n);  // a.n: the device-side count
	// slot of tile t0 + k * stride: k % R (the loop is unrolled R times, so every slot index is static)
	constexpr int R = PF + 1;
	RawTile<N, CT_> ring[R];
	uint32_t live[R];
	// The loads are issued unconditionally: a tile past the end reads past the buffers' extents (the raw
	// buffer loads return 0; a row index of 0 fetches SH row 0) and is never computed.  Guarding them with
	// branches made the compiler's s_waitcnt bookkeeping conservative at the merges (vmcnt(0) before every
	// SH fetch and every tile: the pipeline drained each step)
	// (a tile past the end reads through an empty descriptor: its encoding loads would otherwise land in the next
	// plane's rows -- real traffic, 17 MB per launch at 4 workgroups per CU, a quarter of a surface-scene pass)
	const __amdgpu_buffer_rsrc_t none_rs = make_rsrc(a.enc, 0u);
#pragma unroll
	for (int k = 0; k <= PF; ++k) ri_load<N, CT_>(crd_rs, (t0 + k * stride) * TS, n, ring[k % R]);
#pragma unroll
	for (int k = 0; k < PF; ++k)
		rf_load<N, CT_, FF, true>(a, t0 + k * stride < n_tiles ? enc_rs : none_rs, crd_rs, (t0 + k * stride) * TS, g, n, ring[k], false);
	live[0] = sh_load_live<N, CT_>(sh_rs, g, ring[0], skip);
	for (uint32_t tb = t0; tb < n_tiles; tb += R * stride) {
#pragma unroll
		for (int q = 0; q < R; ++q) {
			const uint32_t t = tb + q * stride;
			if (t >= n_tiles) break;
			live[(q + 1) % R] = sh_load_live<N, CT_>(sh_rs, g, ring[(q + 1) % R], skip);
			ri_load<N, CT_>(crd_rs, (t + (PF + 1) * stride) * TS, n, ring[q]);
			rf_load<N, CT_, FF, true>(a, t + PF * stride < n_tiles ? enc_rs : none_rs, crd_rs, (t + PF * stride) * TS, g, n,
			                          ring[(q + PF) % R], false);
			sh_tile<N, CT_>(wl, ring[q], out_rs, t * TS, g, n, live[q]);
		}
	}
}

// ---------------------------------------------------------------------------
// Training: forward (activations kept), dgrad chain, wgrad via transposed reads.
// ---------------------------------------------------------------------------
template <class N, int l>
__device__ __forceinline__ void wgrad_layer(const _Float16* imgs, const _Float16* dimgs, int wave, int lane,
                                            f4 (&acc)[N::tslots()], uint32_t enc_pad) {
	constexpr int STRIDE = N::template stride<true>();
	constexpr int DS = N::dstride();
	constexpr int DCUR = ((N::NL - 1 - l) % 2) * N::drows();
	constexpr int SIN = N::template seg_in<true>(l);
	constexpr int KTN = N::KT16(l);
	const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
#pragma unroll
	for (int t = 0; t < N::gtiles(l); ++t) {
		constexpr int dummy = 0;
		(void)dummy;
		const int gt = N::gtile_base(l) + t;
		const int mt = t / KTN, kt = t % KTN;
		if (gt % TWAVES != wave) continue;
		if (l == 0 && (uint32_t)(16 * kt) >= enc_pad) continue;
		if (N::XE == 1 && l == N::DH + 1 && kt == 3) continue;  // the latent code's zero padding rows
		const int slot = gt / TWAVES;
		f4 c = acc[slot];
#pragma unroll
		for (int w2 = 0; w2 < TWAVES * TSPW / 32; ++w2) {  // K = 32 consecutive samples of the chunk per MFMA
			const _Float16* ds = dimgs + w2 * 32 * DS + DCUR + 16 * mt + 4 * p;
			const _Float16* as = imgs + w2 * 32 * STRIDE + SIN + 16 * kt + 4 * p;
			const h4 a0 = tr_read(ds + (8 * g + q) * DS), a1 = tr_read(ds + (8 * g + 4 + q) * DS);
			const h4 b0 = tr_read(as + (8 * g + q) * STRIDE), b1 = tr_read(as + (8 * g + 4 + q) * STRIDE);
			const h8 A = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
			const h8 B = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
			c = mfma(A, B, c);
		}
		acc[slot] = c;
	}
}

template <class N, int l, int CT_ = TCT>
__device__ __forceinline__ void dgrad_layer(const MlpArgs& a, const _Float16* frags, const _Float16* img,
                                            _Float16* dimg, int lane, uint32_t base) {
	constexpr int STRIDE = N::template stride<true>();
	constexpr int DS = N::dstride();
	constexpr int DCUR = ((N::NL - 1 - l) % 2) * N::drows();
	constexpr int DNXT = (1 - (N::NL - 1 - l) % 2) * N::drows();
	constexpr int SIN = N::template seg_in<true>(l);
	constexpr int MS = N::Ms(l);
	// the rgb network's input: the 16 density-output rows, then (for the camera gradients) the 16 SH rows
	constexpr int KT = N::Kt(l);
	const int g = lane >> 4, n = lane & 15;
	h8 b[CT_][MS];
#pragma unroll
	for (int c = 0; c < CT_; ++c)
#pragma unroll
		for (int s = 0; s < MS; ++s) b[c][s] = lds_h8(dimg + (16 * c + n) * DS + DCUR + 32 * s + 8 * g);
	const _Float16* fr = frags + N::bwd_off(l);
#pragma unroll
	for (int mt = 0; mt < KT; ++mt) {
		// rgb input rows: 16..31 SH (camera gradients), 32..47 the latent code (extra dims), 48..63 padding
		if (l == N::DH + 1 && mt == 1 && !a.dsh) continue;
		if (l == N::DH + 1 && mt >= 2 && !a.dextra) continue;
		if (l == N::DH + 1 && mt >= 2 + N::XE) continue;  // XE 1: rows 48..63 are padding
		h8 af[MS];
#pragma unroll
		for (int s = 0; s < MS; ++s) af[s] = lds_h8(fr + ((mt * MS + s) * 64 + lane) * 8);
#pragma unroll
		for (int c = 0; c < CT_; ++c) {
			f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
			for (int s = 0; s < MS; ++s) acc = mfma(af[s], b[c][s], acc);
			const int smp = 16 * c + n;
			const uint32_t i = base + smp;
			if constexpr (N::relu_in(l)) {
				const h4 act = *reinterpret_cast<const h4*>(img + smp * STRIDE + SIN + 16 * mt + 4 * g);
#pragma unroll
				for (int r = 0; r < 4; ++r) acc[r] = act[r] > (_Float16)0 ? acc[r] : 0.0f;
			}
			if constexpr (l == N::DH + 1) {
				// add_density_gradient (nerf_network.h:63-74): dL/d(density raw) joins row 0
				if (mt == 0 && g == 0 && i < a.n) {
					const float w = a.weight ? a.weight[i] : 1.0f;
					acc[0] += (float)__half2float(a.dloss[(size_t)i * 4 + 3]) * w;
				}
			}
			if (l == N::DH + 1 && mt >= 1) {
				// dL/d(SH) or dL/d(latent code) of the sample's own row: the deltas carry its rollover weight
				if (i < a.n) {
					const float inv = a.weight ? 1.0f / a.weight[i] : 1.0f;
					float* dst = mt == 1 ? a.dsh + (size_t)i * 16 : a.dextra + (size_t)i * NGP_EXTRA_ROW + 16 * (mt - 2);
					*reinterpret_cast<float4*>(dst + 4 * g) = make_float4(acc[0] * inv, acc[1] * inv, acc[2] * inv, acc[3] * inv);
				}
			} else if constexpr (l > 0) {
				h4 o = {(_Float16)acc[0], (_Float16)acc[1], (_Float16)acc[2], (_Float16)acc[3]};
				lds_st_h4(dimg + smp * DS + DNXT + 16 * mt + 4 * g, o);
			} else {
				if (i < a.n) {
					const uint32_t k0 = 16 * mt + 4 * g;
					if (a.F == 2 && k0 + 4 <= a.E) {
						// F = 2: rows k0, k0+1 and k0+2, k0+3 are the two features of two levels: one
						// 4-B store per level (level-major dL/denc), values as the element path
#pragma unroll
						for (int q = 0; q < 2; ++q) {
							const __half2 v = __halves2half2(__float2half_rn(acc[2 * q]), __float2half_rn(acc[2 * q + 1]));
							*reinterpret_cast<__half2*>(a.denc + ((size_t)(k0 / 2 + q) * a.enc_plane + i) * 2) = v;
						}
					} else {
#pragma unroll
						for (int r = 0; r < 4; ++r) {
							const uint32_t k = k0 + r;
							if (k < a.E) {
								const uint32_t lvl = k / a.F, f = k % a.F;
								a.denc[((size_t)lvl * a.enc_plane + i) * a.F + f] = __float2half_rn(acc[r]);  // level-major
							}
						}
					}
				}
			}
		}
	}
	if constexpr (l == N::DH + 1) {
		// density-output delta has 16 rows; rows 16..31 of the next k-step must be zero
#pragma unroll
		for (int c = 0; c < CT_; ++c) lds_st_h4(dimg + (16 * c + n) * DS + DNXT + 16 + 4 * g, h4{0, 0, 0, 0});
	}
}

template <class N, int l>
__device__ __forceinline__ void bwd_range(const MlpArgs& a, const _Float16* frags, const _Float16* imgs,
                                          _Float16* dimgs, int wave, int lane, uint32_t base,
                                          f4 (&acc)[N::tslots()]) {
	if constexpr (l >= 0) {
		constexpr int STRIDE = N::template stride<true>();
		constexpr int DS = N::dstride();
		__syncthreads();  // every wave's delta for layer l is in LDS
		if (a.grads) wgrad_layer<N, l>(imgs, dimgs, wave, lane, acc, a.enc_pad);
		dgrad_layer<N, l>(a, frags, imgs + wave * TSPW * STRIDE, dimgs + wave * TSPW * DS, lane, base);
		bwd_range<N, l - 1>(a, frags, imgs, dimgs, wave, lane, base, acc);
	}
}

// The workgroup's weight gradients -> its row of the partials (plain stores: every weight is
// in exactly one tile); k_mlp_reduce sums the rows in a fixed order.  Replaces one fp32 atomic
// per weight and workgroup onto the same 10k addresses (256-way contention at the L2).
template <class N, int l>
__device__ __forceinline__ void flush_range(const MlpArgs& a, int wave, int lane, const f4 (&acc)[N::tslots()]) {
	if constexpr (l < N::NL) {
		constexpr int KTN = N::KT16(l);
		const int g = lane >> 4, n = lane & 15;
		const uint32_t pin = a.param_in[l];
		float* gl = a.partials + (size_t)blockIdx.x * a.n_mlp + a.param_off[l];
#pragma unroll
		for (int t = 0; t < N::gtiles(l); ++t) {
			const int gt = N::gtile_base(l) + t;
			if (gt % TWAVES != wave) continue;
			const int mt = t / KTN, kt = t % KTN;
			const uint32_t col = 16 * kt + n;
			if (col >= pin) continue;
			const f4 c = acc[gt / TWAVES];
#pragma unroll
			for (int r = 0; r < 4; ++r) {
				const uint32_t row = 16 * mt + 4 * g + r;
				if (row < (uint32_t)N::out_dim(l)) gl[(size_t)row * pin + col] = c[r];
			}
		}
		flush_range<N, l + 1>(a, wave, lane, acc);
	}
}

// Sum of the workgroups' partials into the fp32 MLP gradients: 16 lanes per weight, each
// adding 1/16 of the rows, then a shuffle reduction -- a fixed order, so the MLP gradients are
// deterministic.
__global__ void __launch_bounds__(256) k_mlp_reduce(const float* __restrict__ partials, uint32_t rows, uint32_t n,
                                                    float* __restrict__ grads) {
	const uint32_t t = blockIdx.x * 256u + threadIdx.x;
	const uint32_t j = t >> 4, q = t & 15u;
	float s = 0.0f;
	if (j < n) {
#pragma unroll 4
		for (uint32_t r = q; r < rows; r += 16) s += partials[(size_t)r * n + j];
	}
#pragma unroll
	for (uint32_t o = 8; o > 0; o >>= 1) s += __shfl_xor(s, o, 16);
	if (j < n && q == 0) grads[j] += s;
}

// Next chunk's global inputs, fetched into registers while the current chunk runs (F = 2
// encodings with whole 8-half K chunks; other shapes load directly): the raw encoding words,
// the warped direction and the loss gradient of this lane's rows.
struct TrainPrefetch {
	uint32_t e[2][4];
	float d[3];
	uint2 dl;
	float w;
	float4 x[4];  // Net::XE: latent-code components 8h .. 8h + 7 (XE 1) / 16h .. 16h + 15 (XE 2), h = lane / SPW - 2
};

// the latent code of sample i (Net::XE), components 4Q h .. 4Q h + 4Q - 1 (Q float4s) as fp32 -- converted to fp16
// (tcnn's Identity encoding: the float input in the network's half type) by extra_h8; zeros past the batch
template <int Q, int NX>
__device__ __forceinline__ void load_extra(const MlpArgs& a, uint32_t i, int h, float4 (&x)[NX]) {
#pragma unroll
	for (int q = 0; q < Q; ++q) x[q] = make_float4(0.f, 0.f, 0.f, 0.f);
	if (i >= a.n) return;
	const uint32_t row = a.sample_img ? a.sample_img[i] : 0u;
	const float4* src = reinterpret_cast<const float4*>(a.extra + (size_t)row * NGP_EXTRA_ROW + 4 * Q * h);
#pragma unroll
	for (int q = 0; q < Q; ++q) x[q] = src[q];
}
__device__ __forceinline__ void load_extra8(const MlpArgs& a, uint32_t i, int h, float4 (&x)[2]) { load_extra<2>(a, i, h, x); }
__device__ __forceinline__ h8 extra_h8(const float4 (&x)[2]) {
	return h8{(_Float16)x[0].x, (_Float16)x[0].y, (_Float16)x[0].z, (_Float16)x[0].w,
	          (_Float16)x[1].x, (_Float16)x[1].y, (_Float16)x[1].z, (_Float16)x[1].w};
}

template <class N, int SPW_ = TSPW>
__device__ __forceinline__ void train_fetch(const MlpArgs& a, uint32_t base, int lane, TrainPrefetch& p) {
	constexpr int CHUNKS = N::ENC_ROWS / 8;
	const EncLayout lay{a.enc_plane, a.enc_lsh, a.enc_gsh};
	const uint32_t* e = reinterpret_cast<const uint32_t*>(a.enc);
#pragma unroll
	for (int it = 0; it < 2; ++it) {
		const int t = lane + 64 * it, smp = t % SPW_, chunk = t / SPW_;
		const uint32_t i = base + smp, k0 = chunk * 8;
		const bool ok = t < SPW_ * CHUNKS && i < a.n && k0 < a.E;
#pragma unroll
		for (int q = 0; q < 4; ++q) p.e[it][q] = ok ? e[lay.vec(k0 / 2 + q, i)] : 0u;
	}
	const uint32_t i = base + (lane % SPW_);
	const bool in = i < a.n && a.coords;  // no coordinates (input gradients only): the zero direction
	const float* c = a.coords + (size_t)(in ? i : 0) * a.coord_stride;
#pragma unroll
	for (int k = 0; k < 3; ++k) p.d[k] = in ? c[4 + k] : 0.5f;
	if constexpr (N::XE) {
		if (lane >= 2 * SPW_ && lane < 4 * SPW_) load_extra<2 * N::XE>(a, i, lane / SPW_ - 2, p.x);
	}
	p.dl = make_uint2(0u, 0u);
	p.w = 1.0f;
	if (lane < SPW_ && in) {
		p.dl = *reinterpret_cast<const uint2*>(a.dloss + (size_t)i * 4);
		if (a.weight) p.w = a.weight[i];
	}
}

// The prefetched inputs -> this wave's LDS images (encoding rows, SH rows, output-layer delta),
// the same values load_encoding / load_sh / the delta loop store.
template <class N, int STRIDE, int DS, int SPW_ = TSPW>
__device__ __forceinline__ void train_commit(const MlpArgs& a, const TrainPrefetch& p, _Float16* img, _Float16* dimg,
                                             int x_seg, uint32_t base, int lane) {
	constexpr int CHUNKS = N::ENC_ROWS / 8;
#pragma unroll
	for (int it = 0; it < 2; ++it) {
		const int t = lane + 64 * it;
		if (t < SPW_ * CHUNKS) {
			const int smp = t % SPW_, chunk = t / SPW_;
			h8 v;
#pragma unroll
			for (int q = 0; q < 4; ++q) {
				v[2 * q] = u16h(p.e[it][q]);
				v[2 * q + 1] = u16h(p.e[it][q] >> 16);
			}
			lds_st_h8(img + smp * STRIDE + chunk * 8, v);
		}
	}
	{
		// lane = half * SPW_ + sample: SH components 8 half .. 8 half + 7 of the warped direction
		const int smp = lane % SPW_, half = lane / SPW_;
		const bool in = base + smp < a.n;
		float v[16];
		sh_deg4(p.d[0], p.d[1], p.d[2], v);
		h8 o;
#pragma unroll
		for (int k = 0; k < 8; ++k) o[k] = in ? (_Float16)(half ? v[8 + k] : v[k]) : (_Float16)0;
		if (half < 2) lds_st_h8(img + smp * STRIDE + x_seg + 16 + 8 * half, o);
		if constexpr (N::XE) {
			// the latent code: rgb input rows 32..47 (XE 2: 32..63, 16 per lane)
			if (half >= 2 && half < 4) {
				const float4 x0[2] = {p.x[0], p.x[1]};
				lds_st_h8(img + smp * STRIDE + x_seg + 32 + 8 * N::XE * (half - 2), extra_h8(x0));
				if constexpr (N::XE == 2) {
					const float4 x1[2] = {p.x[2], p.x[3]};
					lds_st_h8(img + smp * STRIDE + x_seg + 32 + 16 * (half - 2) + 8, extra_h8(x1));
				}
			}
		}
	}
	for (int t = lane; t < SPW_ * 4; t += 64) {
		const int smp = t % SPW_, ch = t / SPW_;
		h8 v = {0, 0, 0, 0, 0, 0, 0, 0};
		const uint2 dl = make_uint2(__shfl(p.dl.x, smp, 64), __shfl(p.dl.y, smp, 64));
		const float w = __shfl(p.w, smp, 64);
		if (ch == 0) {
			const __half* d = reinterpret_cast<const __half*>(&dl);
			v[0] = (_Float16)(__half2float(d[0]) * w);
			v[1] = (_Float16)(__half2float(d[1]) * w);
			v[2] = (_Float16)(__half2float(d[2]) * w);
		}
		lds_st_h8(dimg + smp * DS + 8 * ch, v);  // layer NL-1 uses buffer 0
	}
}

template <class N>
__global__ void __launch_bounds__(TBLOCK) k_mlp_train(MlpArgs a) {
	if (a.n_dev) a.n = min(a.n, *a.n_dev);
	extern __shared__ __attribute__((aligned(16))) char smem[];
	constexpr int STRIDE = N::template stride<true>();
	constexpr int DS = N::dstride();
	constexpr int FH = (N::fwd_frags() + N::bwd_frags()) * FRAG_HALVES;
	_Float16* frags = reinterpret_cast<_Float16*>(smem);
	_Float16* imgs = frags + FH;
	_Float16* dimgs = imgs + WAVES * SPW * STRIDE;
	const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
	_Float16* img = imgs + wave * TSPW * STRIDE;
	_Float16* dimg = dimgs + wave * TSPW * DS;

	for (int t = threadIdx.x; t < FH / 8; t += TBLOCK)
		reinterpret_cast<h8*>(frags)[t] = reinterpret_cast<const h8*>(a.frags)[t];
	for (int t = lane; t < TSPW * STRIDE / 8; t += 64) reinterpret_cast<h8*>(img)[t] = h8{0, 0, 0, 0, 0, 0, 0, 0};
	for (int t = lane; t < TSPW * DS / 8; t += 64) reinterpret_cast<h8*>(dimg)[t] = h8{0, 0, 0, 0, 0, 0, 0, 0};

	f4 acc[N::tslots()];
#pragma unroll
	for (int s = 0; s < N::tslots(); ++s) acc[s] = f4{0.f, 0.f, 0.f, 0.f};

	const uint32_t n_chunks = n_chunks_of(a.n);
	// F = 2 with whole K chunks: the next chunk's inputs are fetched during the current one
	const bool pref = a.F == 2 && (a.E % 8) == 0 && N::ENC_ROWS / 8 * TSPW <= 128;
	TrainPrefetch pf;
	if (pref && blockIdx.x < n_chunks) train_fetch<N>(a, blockIdx.x * SAMPLES_PER_BLOCK + wave * TSPW, lane, pf);
	for (uint32_t chunk = blockIdx.x; chunk < n_chunks; chunk += gridDim.x) {
		__syncthreads();  // previous chunk's wgrad reads of every image are done
		const uint32_t base = chunk * SAMPLES_PER_BLOCK + wave * TSPW;
		if (pref) {
			train_commit<N, STRIDE, DS>(a, pf, img, dimg, N::template x_seg<true>(), base, lane);
			const uint32_t nxt = chunk + gridDim.x;
			if (nxt < n_chunks) train_fetch<N>(a, nxt * SAMPLES_PER_BLOCK + wave * TSPW, lane, pf);
		} else {
			load_encoding<N, STRIDE, TSPW>(a, img, base, lane);
			load_sh<STRIDE, TSPW>(a, img, N::template x_seg<true>(), base, lane);
			if constexpr (N::XE) {
				for (int t = lane; t < TSPW * 2 * N::XE; t += 64) {
					float4 x[2];
					load_extra8(a, base + t % TSPW, t / TSPW, x);
					lds_st_h8(img + (t % TSPW) * STRIDE + N::template x_seg<true>() + 32 + 8 * (t / TSPW), extra_h8(x));
				}
			}
			// delta of the rgb output layer: rows 0..2 = dL/drgb_raw (loss-scaled, rollover-weighted)
			for (int t = lane; t < TSPW * 4; t += 64) {
				const int smp = t % TSPW, ch = t / TSPW;
				const uint32_t i = base + smp;
				h8 v = {0, 0, 0, 0, 0, 0, 0, 0};
				if (ch == 0 && i < a.n) {
					const float w = a.weight ? a.weight[i] : 1.0f;
					const __half* d = a.dloss + (size_t)i * 4;
					v[0] = (_Float16)(__half2float(d[0]) * w);
					v[1] = (_Float16)(__half2float(d[1]) * w);
					v[2] = (_Float16)(__half2float(d[2]) * w);
				}
				lds_st_h8(dimg + smp * DS + 8 * ch, v);  // layer NL-1 uses buffer 0
			}
		}
		f4 res[TCT];
		fwd_range<N, true, 0, N::NL - 1, TCT>(frags, img, lane, res);
		bwd_range<N, N::NL - 1>(a, frags, imgs, dimgs, wave, lane, base, acc);
	}
	if (a.grads) flush_range<N, 0>(a, wave, lane, acc);
}

// ---------------------------------------------------------------------------
// Weight packing: row-major fp16 params -> per-lane MFMA fragments.
// ---------------------------------------------------------------------------
struct PackLayer {
	uint64_t param_off;
	uint32_t out, in;         // param dims
	uint32_t mt, ks, fwd_off; // forward: [mt][ks] fragments
	uint32_t kt, ms, bwd_off; // backward (transposed): [kt][ms] fragments
	uint32_t rfwd_off;        // register-resident forward: [mt][ks], K permuted for l > 0
};
struct PackArgs {
	PackLayer L[MAX_LAYERS];
	uint32_t n_layers;
	uint32_t total_frags;
	uint32_t plane_f, gsh;  // first-layer K order of the register-resident path: planes (F = 2 / 4) or natural (0)
};

// Input column of K position k of the first layer for k_mlp_infer_rf's plane loads
// (EncLayout lsh = 2, G = 2^gsh planes; plane p holds levels p + qG): F = 2: k = 32s + 8g + 2q
// + f reads plane 4s + g slot q; F = 4: k = 32s + 8g + 4r + f reads plane 2s + g/2 slot
// 2(g & 1) + r.  ~0u: no such plane (the load returns 0; the weight is 0).
__device__ __forceinline__ uint32_t plane_col(uint32_t k, uint32_t F, uint32_t gsh) {
	const uint32_t s = k / 32, g = (k % 32) / 8, G = 1u << gsh;
	uint32_t p, slot, f;
	if (F == 2) {
		p = 4 * s + g;
		slot = (k % 8) / 2;
		f = k % 2;
	} else {
		p = 2 * s + g / 2;
		slot = 2 * (g & 1) + (k % 8) / 4;
		f = k % 4;
	}
	if (p >= G) return ~0u;
	return (p + slot * G) * F + f;
}

__global__ void k_pack(const __half* __restrict__ params, __half* __restrict__ out, PackArgs p) {
	const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
	const uint32_t frag = t / 64, lane = t % 64;
	if (frag >= p.total_frags) return;
	const uint32_t g = lane >> 4, m = lane & 15;
	// find the layer and direction of this fragment
	for (uint32_t l = 0; l < p.n_layers; ++l) {
		const PackLayer& L = p.L[l];
		const uint32_t f0 = L.fwd_off / FRAG_HALVES, nf = L.mt * L.ks;
		const uint32_t b0 = L.bwd_off / FRAG_HALVES, nb = L.kt * L.ms;
		const __half* W = params + L.param_off;
		if (frag >= f0 && frag < f0 + nf) {
			const uint32_t idx = frag - f0, mt = idx / L.ks, s = idx % L.ks;
			const uint32_t row = 16 * mt + m;
			for (uint32_t j = 0; j < 8; ++j) {
				const uint32_t col = 32 * s + 8 * g + j;
				out[(size_t)t * 8 + j] = (row < L.out && col < L.in) ? W[(size_t)row * L.in + col] : __float2half(0.0f);
			}
			return;
		}
		const uint32_t r0 = L.rfwd_off / FRAG_HALVES;
		if (frag >= r0 && frag < r0 + nf) {
			const uint32_t idx = frag - r0, mt = idx / L.ks, s = idx % L.ks;
			const uint32_t row = 16 * mt + m;
			for (uint32_t j = 0; j < 8; ++j) {
				uint32_t col = 32 * s + (l == 0 ? 8 * g + j : (j < 4 ? 4 * g + j : 16 + 4 * g + (j - 4)));
				if (l == 0 && p.plane_f) col = plane_col(col, p.plane_f, p.gsh);
				out[(size_t)t * 8 + j] = (row < L.out && col < L.in) ? W[(size_t)row * L.in + col] : __float2half(0.0f);
			}
			return;
		}
		if (frag >= b0 && frag < b0 + nb) {
			const uint32_t idx = frag - b0, mt = idx / L.ms, s = idx % L.ms;
			const uint32_t col = 16 * mt + m;  // input neuron (row of W^T)
			for (uint32_t j = 0; j < 8; ++j) {
				const uint32_t row = 32 * s + 8 * g + j;  // output neuron
				out[(size_t)t * 8 + j] = (row < L.out && col < L.in) ? W[(size_t)row * L.in + col] : __float2half(0.0f);
			}
			return;
		}
	}
}

// ---------------------------------------------------------------------------
// Host side: variant dispatch.
// ---------------------------------------------------------------------------
using V0 = Net<64, 1, 2, 1>;  // lego / base.json (enc 32)
using V1 = Net<64, 1, 2, 2>;  // enc 48..64
using V2 = Net<16, 1, 2, 1>;  // config A
using V3 = Net<32, 1, 2, 1>;
using V4 = Net<64, 2, 2, 1>;
using V5 = Net<64, 1, 1, 1>;
using V6 = Net<64, 1, 3, 1>;
using V7 = Net<64, 1, 2, 1, 1>;  // lego / base.json with per-image latent codes (n_extra_dims 1..16)
using V8 = Net<64, 1, 2, 1, 2>;  // the same with n_extra_dims 17..32 (light directions + a 16-wide code)

int mlp_variant_for(uint32_t width, uint32_t dh, uint32_t rh, uint32_t enc_pad, uint32_t n_extra_dims) {
	const uint32_t ke = enc_pad <= 32 ? 1 : (enc_pad <= 64 ? 2 : 0);
	if (n_extra_dims) return width == 64 && dh == 1 && rh == 2 && ke == 1 && n_extra_dims <= 32 ? (n_extra_dims <= 16 ? 7 : 8) : -1;
	if (width == 64 && dh == 1 && rh == 2 && ke == 1) return 0;
	if (width == 64 && dh == 1 && rh == 2 && ke == 2) return 1;
	if (width == 16 && dh == 1 && rh == 2 && ke == 1) return 2;
	if (width == 32 && dh == 1 && rh == 2 && ke == 1) return 3;
	if (width == 64 && dh == 2 && rh == 2 && ke == 1) return 4;
	if (width == 64 && dh == 1 && rh == 1 && ke == 1) return 5;
	if (width == 64 && dh == 1 && rh == 3 && ke == 1) return 6;
	return -1;
}

template <class N>
static void layer_geometry(const ngp_model* m, PackArgs& p) {
	p.n_layers = N::NL;
	for (int l = 0; l < N::NL; ++l) {
		PackLayer& L = p.L[l];
		L.param_off = m->layers[l].param_offset;
		L.out = m->layers[l].out;
		L.in = m->layers[l].in;
		L.mt = N::Mt(l);
		L.ks = N::Ks(l);
		L.fwd_off = N::fwd_off(l);
		L.kt = N::Kt(l);
		L.ms = N::Ms(l);
		L.bwd_off = N::bwd_off(l);
		L.rfwd_off = N::rfwd_off(l);
	}
	p.total_frags = N::all_frags();
}

#define NGP_DISPATCH(variant, ...)                      \
	switch (variant) {                                   \
		case 0: { using N = V0; __VA_ARGS__; } break;           \
		case 1: { using N = V1; __VA_ARGS__; } break;           \
		case 2: { using N = V2; __VA_ARGS__; } break;           \
		case 3: { using N = V3; __VA_ARGS__; } break;           \
		case 4: { using N = V4; __VA_ARGS__; } break;           \
		case 5: { using N = V5; __VA_ARGS__; } break;           \
		case 6: { using N = V6; __VA_ARGS__; } break;           \
		case 7: { using N = V7; __VA_ARGS__; } break;           \
		case 8: { using N = V8; __VA_ARGS__; } break;           \
		default: throw std::runtime_error("unsupported MLP configuration"); \
	}

uint32_t mlp_frag_halves(const ngp_model* m) {
	uint32_t r = 0;
	NGP_DISPATCH(m->mlp_variant, r = N::all_frags() * FRAG_HALVES);
	return r;
}

void pack_mlp_fragments(const ngp_model* m, const __half* params16, __half* frags, hipStream_t s) {
	PackArgs p{};
	NGP_DISPATCH(m->mlp_variant, layer_geometry<N>(m, p));
	p.plane_f = m->enc_lsh == 2 && (m->lt.F == 2 || m->lt.F == 4) ? m->lt.F : 0u;
	p.gsh = m->enc_gsh;
	const uint32_t threads = p.total_frags * 64;
	k_pack<<<div_up(threads, 256), 256, 0, s>>>(params16, frags, p);
	NGP_HIP_CHECK(hipGetLastError());
}

int cu_count() {
	static int n = 0;
	if (n == 0) {
		int dev = 0;
		NGP_HIP_CHECK(hipGetDevice(&dev));
		NGP_HIP_CHECK(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
		if (n <= 0) n = 256;
	}
	return n;
}

static MlpArgs base_args(const ngp_model* m) {
	MlpArgs a{};
	a.E = m->enc_width;
	a.F = m->lt.F;
	a.enc_pad = m->enc_pad;
	for (uint32_t l = 0; l < m->n_layers; ++l) {
		a.param_off[l] = m->layers[l].param_offset;
		a.param_in[l] = m->layers[l].in;
	}
	return a;
}

template <class N, class K>
static void set_lds(K kernel, size_t bytes) {
	NGP_HIP_CHECK(hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
}

void launch_mlp_infer(const ngp_model* m, const __half* frags, const __half* enc, EncLayout enc_layout,
                      const float* coords, uint32_t coord_stride, uint32_t n, __half* out, hipStream_t s,
                      const uint32_t* n_dev, uint32_t dir_offset, const __half* sh, uint32_t out_mode, uint32_t out_stride,
                      const uint32_t* sh_ray, uint32_t sh_rows, bool skip_unfilled, const MlpExtra& x) {
	if (n == 0) return;
	if (enc_layout.lsh != m->enc_lsh) throw std::runtime_error("encoding layout differs from the packed first layer's");
	MlpArgs a = base_args(m);
	a.frags = frags;
	a.enc = enc;
	a.enc_plane = enc_layout.plane;
	a.enc_lsh = enc_layout.lsh;
	a.enc_gsh = enc_layout.gsh;
	a.coords = coords;
	a.coord_stride = coord_stride;
	a.n = n;
	a.out = out;
	a.n_dev = n_dev;
	a.enc_bytes = (uint32_t)std::min<uint64_t>((uint64_t)m->enc_width * enc_layout.plane * 2, 0xffffffffu);
	a.coord_bytes = (uint32_t)std::min<uint64_t>((uint64_t)n * (sh ? 1 : coord_stride) * 4, 0xffffffffu);
	a.dir_offset = dir_offset;
	if (sh && !sh_ray) throw std::runtime_error("launch_mlp_infer: SH rows need their per-sample row indices");
	a.sh = sh;
	a.sh_ray = sh_ray;
	a.sh_bytes = (uint32_t)std::min<uint64_t>((uint64_t)sh_rows * 32, 0xffffffffu);
	a.out_mode = out_mode;
	a.out_stride = out_stride;
	a.skip_unfilled = skip_unfilled && sh_ray && out_mode == 0;
	a.prio = sh_ray ? (m->tuning.render_priority >> 2) & 3u : 0u;
	a.extra = x.extra ? x.extra : m->zero_extra.ptr;
	a.sample_img = x.extra ? x.sample_img : nullptr;
	NGP_DISPATCH(m->mlp_variant, {
		const size_t lds = (size_t)N::fwd_frags() * FRAG_HALVES * 2;
		// workgroups per CU (ngp_tuning.mlp_workgroups_per_cu; 8 measured 0.6 % faster per frame than
		// 5 = the occupancy with fixed weights, +4 % bench value on one box; the other pipeline's
		// encoder launches then share the CUs longer, which lowers their measured per-launch rate)
		const uint32_t wg_per_cu = m->tuning.mlp_workgroups_per_cu ? m->tuning.mlp_workgroups_per_cu : 8u;
		const uint32_t grid = std::min<uint32_t>(div_up(n, 16 * WAVES), cu_count() * wg_per_cu);
		const bool pl = a.enc_lsh == 2;
		// the renderer's path.  Wave steps of 16 * CT samples: the CT column tiles share each weight fragment
		// read from LDS (16-sample steps were LDS-bandwidth bound, 20 ds_read_b128 per 20 MFMAs).  64-sample
		// steps (CT = 4, -4 % frame time against 16 in round 3) hold 194 VGPRs: 2 waves per SIMD, MFMA busy
		// 0.40 of the CU cycles (profiles/r04_pmc_mlp.txt); 32-sample steps (CT = 2) 110 VGPRs: 4 waves per
		// SIMD, MFMA busy 0.46.  With two ray pipelines the other pipeline's encoder shares the CUs and the
		// 64-sample steps measured 0-2 % faster per frame; with one (surface scenes) the 32-sample steps 1-2 %
		// (profiles/r04_mlp_tile_ab.txt): the renderer picks per frame (RenderScratch::mlp_tile)
		// (the network alone, ngp_model_infer_sh_rows: 32-sample steps, see the decoupled pipeline below)
		const uint32_t tile = m->tuning.render_mlp_tile ? m->tuning.render_mlp_tile : (x.standalone ? 2u : m->rs.mlp_tile);
		// the 64-sample steps beside the other pipeline's encoder: 6 workgroups per CU (13.60 vs 13.67 ms per fire frame
		// against 8 with 6 M passes; profiles/r05_schedule_sweep.txt)
		const uint32_t wg_render = m->tuning.mlp_workgroups_per_cu ? m->tuning.mlp_workgroups_per_cu : 6u;
		// the decoupled load pipeline (k_mlp_infer_sh, ngp_tuning.render_mlp_pipeline 2 / 3; 1 = the round-5 ring)
		// alone on the GPU the two-tile-deep ring (3) at 32-sample steps and 4 workgroups per CU measured best (0.40 of
		// the fp16 peak vs 0.39 for 2; in frame 3 is 0.5 % slower per fire frame: profiles/r06_mlp_microbench_wg_sweep.txt,
		// r06_render_mlp_pipeline_ab.txt)
		const uint32_t pipe = m->tuning.render_mlp_pipeline ? m->tuning.render_mlp_pipeline : (x.standalone ? 3u : 2u);
		bool done = false;
		if constexpr (N::XE == 0) {
			if (sh && a.F == 2 && pl && pipe >= 2 && out_mode == 0) {
				// workgroups per CU = the resident ones (64-sample steps: 174 VGPRs, 2 waves per SIMD = 2 workgroups;
				// 32-sample steps: 96 VGPRs, 4 workgroups): no second round of workgroups reloading the weights
				// (standalone 0.34 -> 0.38 and 0.37 -> 0.39 of the peak, profiles/r06_mlp_microbench_pipelines.txt;
				// fire frame 13.23 -> 13.18 ms, profiles/r06_render_mlp_pipeline_ab.txt)
				const uint32_t wg = m->tuning.mlp_workgroups_per_cu ? m->tuning.mlp_workgroups_per_cu : (tile == 4 ? 2u : tile == 2 ? 4u : 8u);
				const uint32_t ts = 16 * (tile == 4 ? 4 : tile == 2 ? 2 : 1);
				const uint32_t grid_sh = std::min<uint32_t>(div_up(n, ts * WAVES), cu_count() * wg);
				if (tile == 4 && pipe == 2) launch_timed(k_mlp_infer_sh<N, 4, 1, 12>, grid_sh, BLOCK, lds, s, a);
				else if (tile == 4) launch_timed(k_mlp_infer_sh<N, 4, 2, 12>, grid_sh, BLOCK, lds, s, a);
				else if (tile == 2 && pipe == 2) launch_timed(k_mlp_infer_sh<N, 2, 1, 12>, grid_sh, BLOCK, lds, s, a);
				else if (tile == 2) launch_timed(k_mlp_infer_sh<N, 2, 2, 12>, grid_sh, BLOCK, lds, s, a);
				else if (pipe == 2) launch_timed(k_mlp_infer_sh<N, 1, 2, 12>, grid_sh, BLOCK, lds, s, a);
				else launch_timed(k_mlp_infer_sh<N, 1, 3, 12>, grid_sh, BLOCK, lds, s, a);
				done = true;
			}
		}
		if (done) {
		} else if (sh && a.F == 2 && pl && tile == 4)
			launch_timed(k_mlp_infer_rf<N, 4, 1, false, 12, true>, std::min<uint32_t>(div_up(n, 64 * WAVES), cu_count() * wg_render), BLOCK, lds, s, a);
		else if (sh && a.F == 2 && pl && tile == 2)
			launch_timed(k_mlp_infer_rf<N, 2, 1, false, 12, true>, std::min<uint32_t>(div_up(n, 32 * WAVES), cu_count() * wg_per_cu), BLOCK, lds, s, a);
		else if (sh && a.F == 2 && pl) launch_timed(k_mlp_infer_rf<N, 1, 2, false, 12, true>, grid, BLOCK, lds, s, a);
		else if (sh && a.F == 4 && pl) launch_timed(k_mlp_infer_rf<N, 1, 2, false, 14, true>, grid, BLOCK, lds, s, a);
		// element-wise loads read K in natural order: only valid where k_pack did not permute the
		// first layer to the plane order (plane_f == 0)
		else if (sh) launch_timed(k_mlp_infer_rf<N, 1, 2, false, 0, true>, grid, BLOCK, lds, s, a);
		else if (a.F == 2 && pl) launch_timed(k_mlp_infer_rf<N, 1, 2, false, 12>, grid, BLOCK, lds, s, a);
		else if (a.F == 4 && pl) launch_timed(k_mlp_infer_rf<N, 1, 2, false, 14>, grid, BLOCK, lds, s, a);
		else if (a.F == 2 && !pl) launch_timed(k_mlp_infer_rf<N, 1, 2, false, 2>, grid, BLOCK, lds, s, a);
		else if (a.F == 4 && !pl) launch_timed(k_mlp_infer_rf<N, 1, 2, false, 4>, grid, BLOCK, lds, s, a);
		else launch_timed(k_mlp_infer_rf<N, 1, 2, false, 0>, grid, BLOCK, lds, s, a);
	});
	NGP_HIP_CHECK(hipGetLastError());
}

void launch_mlp_density(const ngp_model* m, const __half* frags, const __half* enc, EncLayout enc_layout, uint32_t n,
                        __half* out, hipStream_t s, const uint32_t* n_dev) {
	if (n == 0) return;
	if (enc_layout.lsh != m->enc_lsh) throw std::runtime_error("encoding layout differs from the packed first layer's");
	MlpArgs a = base_args(m);
	a.frags = frags;
	a.enc = enc;
	a.enc_plane = enc_layout.plane;
	a.enc_lsh = enc_layout.lsh;
	a.enc_gsh = enc_layout.gsh;
	a.n = n;
	a.out = out;
	a.n_dev = n_dev;
	a.enc_bytes = (uint32_t)std::min<uint64_t>((uint64_t)m->enc_width * enc_layout.plane * 2, 0xffffffffu);
	NGP_DISPATCH(m->mlp_variant, {
		const size_t lds = (size_t)N::fwd_frags_upto(N::DH + 1) * FRAG_HALVES * 2;
		// workgroups per CU (ngp_tuning.mlp_workgroups_per_cu; 8 measured 0.6 % faster per frame than
		// 5 = the occupancy with fixed weights, +4 % bench value on one box; the other pipeline's
		// encoder launches then share the CUs longer, which lowers their measured per-launch rate)
		const uint32_t wg_per_cu = m->tuning.mlp_workgroups_per_cu ? m->tuning.mlp_workgroups_per_cu : 8u;
		const uint32_t grid = std::min<uint32_t>(div_up(n, 16 * WAVES), cu_count() * wg_per_cu);
		const bool pl = a.enc_lsh == 2;
		if (a.F == 2 && pl) k_mlp_infer_rf<N, 1, 2, true, 12><<<grid, BLOCK, lds, s>>>(a);
		else if (a.F == 4 && pl) k_mlp_infer_rf<N, 1, 2, true, 14><<<grid, BLOCK, lds, s>>>(a);
		else if (a.F == 2 && !pl) k_mlp_infer_rf<N, 1, 2, true, 2><<<grid, BLOCK, lds, s>>>(a);
		else if (a.F == 4 && !pl) k_mlp_infer_rf<N, 1, 2, true, 4><<<grid, BLOCK, lds, s>>>(a);
		else k_mlp_infer_rf<N, 1, 2, true, 0><<<grid, BLOCK, lds, s>>>(a);
	});
	NGP_HIP_CHECK(hipGetLastError());
}

void launch_mlp_train(const ngp_model* m, const __half* frags, const __half* enc, EncLayout enc_layout,
                      const float* coords, uint32_t coord_stride, uint32_t n, const __half* dloss,
                      const float* weight, float* grads_mlp, __half* denc, hipStream_t s,
                      const uint32_t* n_dev, float* dsh, const MlpExtra& x) {
	if (n == 0) return;
	MlpArgs a = base_args(m);
	a.dsh = dsh;
	a.extra = x.extra ? x.extra : m->zero_extra.ptr;
	a.sample_img = x.extra ? x.sample_img : nullptr;
	a.dextra = m->cfg.n_extra_dims ? x.dextra : nullptr;
	a.frags = frags;
	a.enc = enc;
	a.enc_plane = enc_layout.plane;
	a.enc_lsh = enc_layout.lsh;
	a.enc_gsh = enc_layout.gsh;
	a.coords = coords;
	a.coord_stride = coord_stride;
	a.n = n;
	a.dloss = dloss;
	a.weight = weight;
	a.grads = grads_mlp;
	a.denc = denc;
	a.n_dev = n_dev;
	NGP_DISPATCH(m->mlp_variant, {
		const size_t lds = N::lds_train();
		if (lds > 160 * 1024) throw std::runtime_error("MLP training LDS footprint exceeds 160 KiB");
		const uint32_t grid = std::min<uint32_t>(div_up(n, SAMPLES_PER_BLOCK), cu_count());
		if (grads_mlp) {
			m->mlp_partials.reserve((size_t)cu_count() * m->n_mlp_params);
			a.partials = m->mlp_partials.ptr;
			a.n_mlp = m->n_mlp_params;
		}
		set_lds<N>(k_mlp_train<N>, lds);
		launch_timed(k_mlp_train<N>, grid, TBLOCK, lds, s, a);
		if (grads_mlp) k_mlp_reduce<<<div_up(16 * m->n_mlp_params, 256), 256, 0, s>>>(m->mlp_partials.ptr, grid, m->n_mlp_params, grads_mlp);
	});
	NGP_HIP_CHECK(hipGetLastError());
}

}  // namespace ngp
