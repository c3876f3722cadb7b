// Texture-addresser / L1 throughput calibration for the hash encoder's access shapes (diagnostic).
//
// The render encoder is bound by its load instructions (TA_BUSY ~ 87 %).  This program measures
// what one wave load instruction costs as a function of its width, its active lanes and how many
// distinct cache lines its lanes touch, on tables that stay cache resident (2 MiB: L2; 24 MiB: the
// lego hash table's size, Infinity Cache).  Every thread issues ITER loads (8 independent ones in
// flight) and XORs the data into a sink.  Output: per shape, wave instructions, lane loads and bytes
// per CU clock.  Usage: tools/ta_calib   (GPU box)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                            \
	do {                                                                                 \
		hipError_t e_ = (x);                                                             \
		if (e_ != hipSuccess) {                                                          \
			fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
			exit(1);                                                                     \
		}                                                                                \
	} while (0)

__device__ __forceinline__ uint32_t mix(uint32_t x) {
	x ^= x >> 16;
	x *= 0x7feb352du;
	x ^= x >> 15;
	x *= 0x846ca68bu;
	x ^= x >> 16;
	return x;
}

constexpr int ITER = 64;

// W: 4, 8 or 16 bytes per lane.  MODE 0: random lines; 1: lanes in groups of 16 share a 64-B line
// (consecutive words); 2: fully coalesced (a wave reads one contiguous span).  ACTIVE: lanes of 64
// that issue the load (the rest are masked off, as the encoder's lone corner loads).
template <int W, int MODE, int ACTIVE>
__global__ void __launch_bounds__(256) k_gather(const uint4* __restrict__ tab, uint32_t mask16, uint32_t* __restrict__ sink) {
	const uint32_t tid = blockIdx.x * 256u + threadIdx.x;
	const uint32_t lane = threadIdx.x & 63u;
	uint32_t acc = 0;
	const bool on = lane < (uint32_t)ACTIVE;
	const char* base = reinterpret_cast<const char*>(tab);
#pragma unroll 1
	for (int it = 0; it < ITER; it += 8) {
		uint32_t off[8];
#pragma unroll
		for (int u = 0; u < 8; ++u) {
			const uint32_t h = mix(tid * 131u + (uint32_t)(it + u) * 0x9e3779b9u);
			uint32_t slot16;  // 16-B slot index
			if (MODE == 0) slot16 = h & mask16;
			else if (MODE == 1) slot16 = ((mix((tid >> 4) * 977u + (uint32_t)(it + u)) & mask16) & ~(uint32_t)(W - 1)) + ((lane & 15u) * W) / 16u;
			else slot16 = ((mix((tid >> 6) * 977u + (uint32_t)(it + u)) & mask16) & ~(uint32_t)(4 * W - 1)) + (lane * W) / 16u;
			off[u] = slot16 * 16u + (MODE == 0 ? 0u : ((lane * W) % 16u));
		}
		if (on) {
#pragma unroll
			for (int u = 0; u < 8; ++u) {
				if constexpr (W == 16) {
					const uint4 v = *reinterpret_cast<const uint4*>(base + off[u]);
					acc ^= v.x ^ v.y ^ v.z ^ v.w;
				} else if constexpr (W == 8) {
					const uint2 v = *reinterpret_cast<const uint2*>(base + off[u]);
					acc ^= v.x ^ v.y;
				} else {
					acc ^= *reinterpret_cast<const uint32_t*>(base + off[u]);
				}
			}
		}
	}
	if (acc == 0x12345678u) sink[0] = acc;
}

// XCD of every workgroup (HW_REG_XCC_ID, bits 3:0): checks the round-robin placement the encoders assume
__global__ void k_xcc(uint32_t* __restrict__ out) {
	if (threadIdx.x == 0) out[blockIdx.x] = (uint32_t)__builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 15u;
}

template <int W, int MODE, int ACTIVE>
static void run(const char* name, const uint4* tab, size_t tab_bytes, uint32_t* sink, int cus, double clk_hz) {
	const uint32_t mask16 = (uint32_t)(tab_bytes / 16 - 1);
	const uint32_t blocks = cus * 64;
	hipEvent_t a, b;
	CK(hipEventCreate(&a));
	CK(hipEventCreate(&b));
	k_gather<W, MODE, ACTIVE><<<blocks, 256>>>(tab, mask16, sink);
	CK(hipEventRecord(a));
	const int reps = 5;
	for (int r = 0; r < reps; ++r) k_gather<W, MODE, ACTIVE><<<blocks, 256>>>(tab, mask16, sink);
	CK(hipEventRecord(b));
	CK(hipEventSynchronize(b));
	float ms;
	CK(hipEventElapsedTime(&ms, a, b));
	const double s = ms / 1e3 / reps;
	const double waves = (double)blocks * 4, instr = waves * ITER, lanes = instr * ACTIVE;
	const double cu_clk = s * clk_hz * cus;
	printf("%-34s table %5.1f MiB: %8.1f us  instr/CU/clk %.4f  lane-loads/CU/clk %.3f  bytes/CU/clk %.2f\n", name,
	       tab_bytes / 1048576.0, s * 1e6, instr / cu_clk, lanes / cu_clk, lanes * W / cu_clk);
	CK(hipEventDestroy(a));
	CK(hipEventDestroy(b));
}

int main() {
	int dev = 0, cus = 0, khz = 0;
	CK(hipSetDevice(dev));
	CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
	CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeClockRate, dev));
	const double clk = khz * 1e3;
	printf("CUs %d clock %.0f MHz\n", cus, clk / 1e6);
	uint4* tab;
	uint32_t* sink;
	const size_t big = 32ull << 20;
	CK(hipMalloc(&tab, big));
	CK(hipMalloc(&sink, 64));
	CK(hipMemset(tab, 1, big));
	{
		const int nb = 8192;
		uint32_t* xd;
		CK(hipMalloc(&xd, nb * 4));
		k_xcc<<<nb, 64>>>(xd);
		uint32_t h[nb];
		CK(hipMemcpy(h, xd, sizeof(h), hipMemcpyDeviceToHost));
		CK(hipFree(xd));
		int same = 0;  // blocks b, b + 8 on one XCD
		for (int b = 0; b + 8 < nb; ++b) same += h[b] == h[b + 8];
		printf("xcc of blocks 0..15:");
		for (int b = 0; b < 16; ++b) printf(" %u", h[b]);
		printf("   blocks b, b+8 on the same XCD: %d of %d\n", same, nb - 8);
	}
	for (size_t tb : {2ull << 20, 32ull << 20}) {
		run<4, 0, 64>("gather  4B random, 64 lanes", tab, tb, sink, cus, clk);
		run<8, 0, 64>("gather  8B random, 64 lanes", tab, tb, sink, cus, clk);
		run<16, 0, 64>("gather 16B random, 64 lanes", tab, tb, sink, cus, clk);
		run<4, 0, 16>("gather  4B random, 16 lanes", tab, tb, sink, cus, clk);
		run<16, 0, 16>("gather 16B random, 16 lanes", tab, tb, sink, cus, clk);
		run<4, 0, 4>("gather  4B random,  4 lanes", tab, tb, sink, cus, clk);
		run<4, 1, 64>("gather  4B 16 lanes/line, 64 l", tab, tb, sink, cus, clk);
		run<16, 1, 64>("gather 16B 4 lanes/64B, 64 l", tab, tb, sink, cus, clk);
		run<4, 2, 64>("coalesced  4B, 64 lanes", tab, tb, sink, cus, clk);
		run<16, 2, 64>("coalesced 16B, 64 lanes", tab, tb, sink, cus, clk);
	}
	CK(hipFree(tab));
	CK(hipFree(sink));
	return 0;
}
