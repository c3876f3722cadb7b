// FETCH_SIZE calibration for the access shapes of this repository's kernels (diagnostic).
//
// rocprofv3 --pmc FETCH_SIZE counts the L2's memory-side read requests; MI355X_MICROARCH.md
// documents that on gfx950 it reports half the bytes of a wide coalesced 16-B-per-lane stream,
// and calls other widths uncalibrated.  This program issues each access shape the kernels use on
// a 1 GiB buffer (4x the Infinity Cache, so reads go to HBM) with a known byte count:
//   k_stream16  16 B per lane, coalesced (optimizer / copies)
//   k_stream4    4 B per lane, coalesced (row copies of 4-B records)
//   k_gather4    4 B per lane at random 4-B-aligned addresses (hash-grid lone corners)
//   k_gather16  16 B per lane at random 16-B-aligned addresses (hash-grid quads)
//   k_table4     4 B random gathers into a 16 MiB table re-read 16 times (about the lego hash
//                table's 24 MB: Infinity-Cache resident -- does FETCH_SIZE see the re-reads?)
// tools/fetch_calib.sh runs it under one --pmc FETCH_SIZE pass and tools/fetch_calib.py turns the
// per-dispatch counters into measured bytes / issued bytes per shape.
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

__global__ void k_stream16(const uint4* __restrict__ a, size_t n, uint32_t* __restrict__ sink) {
	uint32_t acc = 0;
	for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
		const uint4 v = a[i];
		acc ^= v.x ^ v.y ^ v.z ^ v.w;
	}
	if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void k_stream4(const uint32_t* __restrict__ a, size_t n, uint32_t* __restrict__ sink) {
	uint32_t acc = 0;
	for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) acc ^= a[i];
	if (acc == 0x12345678u) sink[0] = acc;
}

// n_reads random reads, each lane one per iteration; `mask` = element count - 1 (power of two)
__global__ void k_gather4(const uint32_t* __restrict__ a, uint32_t mask, uint32_t n_reads, uint32_t* __restrict__ sink) {
	uint32_t acc = 0;
	for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n_reads; i += gridDim.x * blockDim.x) acc ^= a[mix(i) & mask];
	if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void k_gather16(const uint4* __restrict__ a, uint32_t mask, uint32_t n_reads, uint32_t* __restrict__ sink) {
	uint32_t acc = 0;
	for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n_reads; i += gridDim.x * blockDim.x) {
		const uint4 v = a[mix(i) & mask];
		acc ^= v.x ^ v.y ^ v.z ^ v.w;
	}
	if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void k_table4(const uint32_t* __restrict__ a, uint32_t mask, uint32_t n_reads, uint32_t* __restrict__ sink) {
	uint32_t acc = 0;
	for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n_reads; i += gridDim.x * blockDim.x) acc ^= a[mix(i) & mask];
	if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
	const size_t bytes = (size_t)1 << 30;
	void* buf = nullptr;
	uint32_t* sink = nullptr;
	CK(hipMalloc(&buf, bytes));
	CK(hipMalloc((void**)&sink, 64));
	CK(hipMemset(buf, 1, bytes));
	const uint32_t n_gather = 1u << 24;            // 16 M reads
	const int grid = 256 * 8, block = 256;
	for (int rep = 0; rep < 2; ++rep) {
		k_stream16<<<grid, block>>>((const uint4*)buf, bytes / 16, sink);
		k_stream4<<<grid, block>>>((const uint32_t*)buf, bytes / 4, sink);
		k_gather4<<<grid, block>>>((const uint32_t*)buf, (uint32_t)(bytes / 4 - 1), n_gather, sink);
		k_gather16<<<grid, block>>>((const uint4*)buf, (uint32_t)(bytes / 16 - 1), n_gather, sink);
		// warm the table, then re-read it: 16 M reads over 16 MiB = 16 passes
		k_table4<<<grid, block>>>((const uint32_t*)buf, (1u << 22) - 1, n_gather, sink);
	}
	CK(hipDeviceSynchronize());
	printf("{\"stream16_bytes\": %zu, \"stream4_bytes\": %zu, \"gather4_reads\": %u, \"gather16_reads\": %u, "
	       "\"table4_reads\": %u, \"table_bytes\": %u}\n",
	       bytes, bytes, n_gather, n_gather, n_gather, (1u << 22) * 4u);
	CK(hipFree(buf));
	CK(hipFree(sink));
	return 0;
}
