// Issue rate of 32-bit integer multiplies on gfx950: 8 independent chains per lane of v_mul_lo_u32, v_mul_u32_u24
// and v_add_u32 (reference), 1024 blocks x 256 threads; prints ns per wave-instruction per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int OP>
__global__ void k(unsigned* out, unsigned seed, int iters) {
  unsigned x[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) x[c] = seed + threadIdx.x * 8 + c;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      if constexpr (OP == 0) x[c] = x[c] * 0x21f0aaadu;
      else if constexpr (OP == 1) x[c] = __umul24(x[c], 0x9e3b4du);
      else x[c] = x[c] + 0x21f0aaadu + (x[c] >> 3);
    }
  }
  unsigned s = 0;
#pragma unroll
  for (int c = 0; c < 8; ++c) s ^= x[c];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
int main() {
  unsigned* out;
  hipMalloc(&out, 1024 * 256 * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int iters = 4096;
  const char* names[3] = {"v_mul_lo_u32", "v_mul_u32_u24", "v_add+shift (2 ops)"};
  for (int rep = 0; rep < 2; ++rep)
    for (int op = 0; op < 3; ++op) {
      hipEventRecord(a);
      if (op == 0) k<0><<<1024, 256>>>(out, 1, iters);
      if (op == 1) k<1><<<1024, 256>>>(out, 1, iters);
      if (op == 2) k<2><<<1024, 256>>>(out, 1, iters);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      // wave-instructions per SIMD: 1024 blocks x 4 waves / 1024 SIMDs x iters x 8
      const double per_simd = 1024.0 * 4 / 1024 * iters * 8;
      printf("%-22s %.3f ms  %.3f ns per wave-instruction per SIMD\n", names[op], ms, ms * 1e6 / per_simd);
    }
  return 0;
}
