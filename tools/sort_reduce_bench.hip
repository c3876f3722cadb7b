// Sort-and-reduce alternative to the hash-grid backward's atomics (SURVEY 7 hard part 1; diagnostic).
//
// The training step's k_hashgrid_bwd scatters, per hashed level, the 8 corner gradients of each of the
// ~2^18 compacted samples with packed fp16 atomics (after merging runs of equal indices across the
// lanes of a wave).  The alternative sorts the (corner index, gradient) pairs of a level by index,
// reduces the runs and writes each touched entry once.  This program times the parts of that
// alternative on the bench's sizes with hipCUB: the pair construction (one store per corner), the
// radix sort over the level's 19 index bits, and the run-length reduction (ReduceByKey), for 11
// hashed levels -- the cost the alternative cannot go below -- next to a packed-fp16 atomic scatter
// of the same pairs.  Usage: tools/sort_reduce_bench  (GPU box)
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                            \
	do {                                                                                 \
		hipError_t e_ = (x);                                                             \
		if (e_ != hipSuccess) {                                                          \
			fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
			exit(1);                                                                     \
		}                                                                                \
	} while (0)

constexpr uint32_t LOG2_T = 19, SAMPLES = 1u << 18, CORNERS = 8, LEVELS = 11;

__device__ __forceinline__ uint32_t mix(uint32_t x) {
	x ^= x >> 16;
	x *= 0x7feb352du;
	x ^= x >> 15;
	x *= 0x846ca68bu;
	x ^= x >> 16;
	return x;
}

// (index, gradient) of corner c of sample s at a fine level: samples are consecutive points along rays,
// so consecutive samples land in nearby cells (x advances by ~3 cells per sample at res 2048)
__global__ void k_pairs(uint32_t level, uint32_t* __restrict__ keys, uint32_t* __restrict__ vals) {
	const uint32_t t = blockIdx.x * 256u + threadIdx.x;
	if (t >= SAMPLES * CORNERS) return;
	const uint32_t s = t / CORNERS, c = t % CORNERS;
	const uint32_t ray = s / 16, k = s % 16;
	const uint32_t x = (mix(ray * 3u + level) & 2047u) + 3u * k + (c & 1u), y = (mix(ray * 5u + level) & 2047u) + ((c >> 1) & 1u),
	               z = (mix(ray * 7u + level) & 2047u) + (c >> 2);
	keys[t] = (x ^ (y * 2654435761u) ^ (z * 805459861u)) & ((1u << LOG2_T) - 1u);
	const _Float16 g0 = (_Float16)((float)(mix(t) & 1023u) * 1e-6f), g1 = (_Float16)((float)(mix(t + 1u) & 1023u) * 1e-6f);
	vals[t] = (uint32_t)__builtin_bit_cast(uint16_t, g0) | ((uint32_t)__builtin_bit_cast(uint16_t, g1) << 16);
}

typedef _Float16 half2_vec __attribute__((ext_vector_type(2)));
__global__ void k_atomic(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ vals, __half* grad) {
	const uint32_t t = blockIdx.x * 256u + threadIdx.x;
	if (t >= SAMPLES * CORNERS) return;
	const half2_vec v = __builtin_bit_cast(half2_vec, vals[t]);
	__builtin_amdgcn_global_atomic_fadd_v2f16((__attribute__((address_space(1))) half2_vec*)(grad + 2 * (size_t)keys[t]), v);
}

struct Half2Sum {
	__device__ __forceinline__ uint32_t operator()(uint32_t a, uint32_t b) const {
		const half2_vec x = __builtin_bit_cast(half2_vec, a), y = __builtin_bit_cast(half2_vec, b);
		return __builtin_bit_cast(uint32_t, x + y);
	}
};

__global__ void k_apply(const uint32_t* __restrict__ ukeys, const uint32_t* __restrict__ sums, const uint32_t* __restrict__ n_runs,
                        uint32_t* __restrict__ grad) {
	const uint32_t t = blockIdx.x * 256u + threadIdx.x;
	if (t >= *n_runs) return;
	const half2_vec a = __builtin_bit_cast(half2_vec, grad[ukeys[t]]), b = __builtin_bit_cast(half2_vec, sums[t]);
	grad[ukeys[t]] = __builtin_bit_cast(uint32_t, a + b);  // every touched entry once: a plain read-modify-write
}

int main() {
	const uint32_t N = SAMPLES * CORNERS;
	uint32_t *keys, *vals, *skeys, *svals, *ukeys, *sums, *nruns;
	__half* grad;
	CK(hipMalloc(&keys, N * 4));
	CK(hipMalloc(&vals, N * 4));
	CK(hipMalloc(&skeys, N * 4));
	CK(hipMalloc(&svals, N * 4));
	CK(hipMalloc(&ukeys, N * 4));
	CK(hipMalloc(&sums, N * 4));
	CK(hipMalloc(&nruns, 4));
	CK(hipMalloc(&grad, (size_t)LEVELS << LOG2_T << 2));
	CK(hipMemset(grad, 0, (size_t)LEVELS << LOG2_T << 2));
	size_t sort_bytes = 0, rbk_bytes = 0;
	CK(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, keys, skeys, vals, svals, (int)N, 0, (int)LOG2_T));
	CK(hipcub::DeviceReduce::ReduceByKey(nullptr, rbk_bytes, skeys, ukeys, svals, sums, nruns, Half2Sum(), (int)N));
	void* tmp;
	CK(hipMalloc(&tmp, std::max(sort_bytes, rbk_bytes)));
	hipEvent_t e[5];
	for (auto& x : e) CK(hipEventCreate(&x));
	float t_pairs = 0, t_sort = 0, t_rbk = 0, t_apply = 0, t_atomic = 0;
	const int reps = 5;
	for (int rep = 0; rep <= reps; ++rep) {
		float a = 0, b = 0, c = 0, d = 0, f = 0;
		for (uint32_t l = 0; l < LEVELS; ++l) {
			uint32_t* g = reinterpret_cast<uint32_t*>(grad) + ((size_t)l << LOG2_T);
			CK(hipEventRecord(e[0]));
			k_pairs<<<N / 256, 256>>>(l, keys, vals);
			CK(hipEventRecord(e[1]));
			CK(hipcub::DeviceRadixSort::SortPairs(tmp, sort_bytes, keys, skeys, vals, svals, (int)N, 0, (int)LOG2_T));
			CK(hipEventRecord(e[2]));
			CK(hipcub::DeviceReduce::ReduceByKey(tmp, rbk_bytes, skeys, ukeys, svals, sums, nruns, Half2Sum(), (int)N));
			CK(hipEventRecord(e[3]));
			k_apply<<<N / 256, 256>>>(ukeys, sums, nruns, g);
			CK(hipEventRecord(e[4]));
			CK(hipEventSynchronize(e[4]));
			float x;
			CK(hipEventElapsedTime(&x, e[0], e[1])); a += x;
			CK(hipEventElapsedTime(&x, e[1], e[2])); b += x;
			CK(hipEventElapsedTime(&x, e[2], e[3])); c += x;
			CK(hipEventElapsedTime(&x, e[3], e[4])); d += x;
			CK(hipEventRecord(e[0]));
			k_atomic<<<N / 256, 256>>>(keys, vals, reinterpret_cast<__half*>(g));
			CK(hipEventRecord(e[1]));
			CK(hipEventSynchronize(e[1]));
			CK(hipEventElapsedTime(&x, e[0], e[1])); f += x;
		}
		if (rep == 0) continue;  // warm-up
		t_pairs += a; t_sort += b; t_rbk += c; t_apply += d; t_atomic += f;
	}
	uint32_t runs = 0;
	CK(hipMemcpy(&runs, nruns, 4, hipMemcpyDeviceToHost));
	printf("per training step (%u hashed levels x %u samples x %u corners):\n", LEVELS, SAMPLES, CORNERS);
	printf("  pair construction  %8.1f us\n", 1e3 * t_pairs / reps);
	printf("  radix sort (19 b)  %8.1f us\n", 1e3 * t_sort / reps);
	printf("  reduce by key      %8.1f us   (%u runs of %u pairs in the last level)\n", 1e3 * t_rbk / reps, runs, N);
	printf("  apply runs         %8.1f us\n", 1e3 * t_apply / reps);
	printf("  sort-and-reduce    %8.1f us total\n", 1e3 * (t_pairs + t_sort + t_rbk + t_apply) / reps);
	printf("  packed fp16 atomics of the same pairs (no run merging) %8.1f us\n", 1e3 * t_atomic / reps);
	return 0;
}
