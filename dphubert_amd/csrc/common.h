// Shared device helpers for the DPHuBERT gfx950 kernel library.
//
// Conventions (see include/dphubert_hip.h):
//   * activations are bf16 (stored as raw uint16_t), statistics and
//     accumulation are fp32, master weights / gradients are fp32;
//   * every entry point takes an explicit hipStream_t and never allocates;
//   * errors are returned as negative DPH_E* codes with a thread-local
//     message retrievable through dph_last_error().
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/dphubert_hip.h"

typedef uint16_t bf16_t;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(4))) short s16x4_t;
typedef __attribute__((ext_vector_type(8))) short s16x8_t;

namespace dph {

void set_error(const char* fmt, ...);
int check_launch(const char* what);
// deterministic mode (runtime.hip, dph_set_deterministic): fixed-order cross-block reductions instead of float atomics
bool deterministic();
// deferred fixed-order column reductions (runtime.hip, dph_defer_reductions): while deferring, a slab reduction
// out[j] += sum_r ws[r * ld + j] (j < n) is queued by colred_push and launched with the rest by dph_flush_reductions
bool colred_deferring();
int colred_push(const float* ws, int64_t nrows, int64_t ld, int64_t n, float* out, hipStream_t stream);
// norm.hip: o_q[c] += sum_r ws[r][q * seg + c] over the column segments q of a [nrows][ncols] fp32 partial slab (NULL
// outputs skipped); fixed order in deterministic mode, row groups + one atomic per column per group otherwise
int slab_reduce_cols(const float* ws, int64_t nrows, int64_t ncols, int64_t seg, float* o0, float* o1, float* o2,
                      hipStream_t stream);
// norm.hip: out[0] += sum of n partials, in order (one wave)
void sdot_reduce(const float* part, int64_t n, float* out, hipStream_t stream);

// propagate a non-OK DPH_* code from a host-side helper (its error text is already set)
#define DPH_TRY(expr)                       \
  do {                                      \
    const int dph_try_rc_ = (expr);         \
    if (dph_try_rc_ != DPH_OK) return dph_try_rc_; \
  } while (0)

#define DPH_REQUIRE(cond, ...)              \
  do {                                      \
    if (!(cond)) {                          \
      ::dph::set_error(__VA_ARGS__);        \
      return DPH_EINVAL;                    \
    }                                       \
  } while (0)

__device__ __forceinline__ float bf2f(bf16_t h) { return __uint_as_float(((uint32_t)h) << 16); }

// round-to-nearest-even f32 -> bf16 (NaN stays NaN via the hardware cvt)
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 h = (__bf16)f;
  return __builtin_bit_cast(bf16_t, h);
}

// two floats -> packed bf16 pair by ONE v_cvt_pk_bf16_f32 (the scalar form compiled to two converts
// plus a shift / or repack)
typedef float dph_f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 dph_bf16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack2bf(float a, float b) {
  const dph_bf16x2_t h = __builtin_convertvector((dph_f32x2_t){a, b}, dph_bf16x2_t);
  return __builtin_bit_cast(uint32_t, h);
}

// 8 consecutive bf16 -> fp32 (16-B vector load when the row is 8-aligned; masked tail otherwise)
__device__ __forceinline__ void load_bf16x8(const bf16_t* p, int64_t c0, int64_t C, float (&v)[8]) {
  if (c0 + 8 <= C && (C & 7) == 0) {
    const uint4 r = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);
      v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (c0 + i < C) ? bf2f(p[i]) : 0.f;
  }
}

// Exact-erf GELU (torch default, components.py:110,331,734).  Phi(x) is evaluated through
// erfc(z) = t*P5(t)*exp(-z^2), t = 1/(1 + 0.3275911 z) (Abramowitz & Stegun 7.1.26, absolute
// error <= 1.5e-7 for z >= 0): branch-free, one rcp + one exp + 7 VALU ops (the exp(-z^2) is
// shared with phi(x) for GELU'), no cancellation for negative x.  The error is ~1e-7 absolute
// on Phi, GELU and GELU' -- far below the bf16 step (3.9e-3 relative) of every stored output.
// (The Numerical-Recipes Chebyshev erfc used before cost a second exp and 5 more FMAs per
// element: the GELU epilogues of the conv / FFN GEMMs are VALU-bound on it.)
__device__ __forceinline__ float erfc_pos(float z, float& e_minus_z2) {
  // z >= 0; returns erfc(z) and exp(-z^2)
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));   // 1 ulp, no IEEE divide sequence
  const float p = t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f +
                  t * 1.061405429f))));
  e_minus_z2 = __expf(-z * z);
  return p * e_minus_z2;
}

__device__ __forceinline__ float norm_cdf(float x, float& pdf) {
  float e;
  const float r = erfc_pos(fabsf(x) * 0.70710678118654752f, e);
  pdf = 0.39894228040143268f * e;   // phi(x) = exp(-x^2/2)/sqrt(2 pi)
  return x >= 0.f ? 1.0f - 0.5f * r : 0.5f * r;
}

__device__ __forceinline__ float gelu_f(float x) {
  float pdf;
  return x * norm_cdf(x, pdf);
}

__device__ __forceinline__ float gelu_grad_f(float x) {
  float pdf;
  const float cdf = norm_cdf(x, pdf);
  return cdf + x * pdf;
}

// gelu and gelu' together (one erfc evaluation)
__device__ __forceinline__ void gelu_and_grad(float x, float& g, float& dg) {
  float pdf;
  const float cdf = norm_cdf(x, pdf);
  g = x * cdf;
  dg = cdf + x * pdf;
}

// Counter-based RNG: two rounds of a 32-bit avalanche hash (Wellons' low-bias constants) over the
// folded (seed, element index).  The same (seed, index) always gives the same bits, so forward
// and backward kernels regenerate identical dropout / HardConcrete noise without storing masks.
// 32-bit arithmetic only: the previous splitmix64 finaliser (3 64-bit multiplies per element)
// cost 60 % of the attention forward at p = 0.1, where every score element draws a number.
__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x21f0aaadu;
  x ^= x >> 15;
  x *= 0x735a2d97u;
  x ^= x >> 15;
  return x;
}

__device__ __forceinline__ uint32_t rand_u32(uint64_t seed, uint64_t idx) {
  uint32_t x = (uint32_t)idx ^ ((uint32_t)(idx >> 32) * 0x9E3779B9u) ^ (uint32_t)seed;
  x = hash32(x);
  return hash32(x ^ (uint32_t)(seed >> 32));
}

// uniform in [0,1) with 24 random bits
__device__ __forceinline__ float rand_uniform(uint64_t seed, uint64_t idx) {
  return (float)(rand_u32(seed, idx) >> 8) * (1.0f / 16777216.0f);
}

// Dropout bits: ONE hash32 per PAIR of consecutive elements (element idx uses the low / high 16
// bits of pair idx >> 1), compared against a 16-bit threshold.  Half the hash work of a per-element
// draw and a quarter of rand_u32's (v_mul_lo_u32 is a quarter-rate op: the per-element double
// hash cost ~64 cycles per element in the GEMM epilogues).  p is quantised to 1/65536.
__device__ __forceinline__ uint32_t drop_thr(float p) { return (uint32_t)(p * 65536.0f + 0.5f); }

__device__ __forceinline__ uint32_t drop_bits2(uint64_t seed, uint64_t pair) {
  const uint32_t hi = (uint32_t)(pair >> 32) * 0x9E3779B9u + (uint32_t)(seed >> 32) * 0x85EBCA6Bu;
  return hash32((uint32_t)pair ^ (uint32_t)seed ^ hi);
}

// dropout keep factor: 0 or 1/(1-p); p == 0 -> 1
__device__ __forceinline__ float dropout_scale(uint64_t seed, uint64_t idx, float p, float inv_keep) {
  if (p <= 0.f) return 1.0f;
  const uint32_t bits = drop_bits2(seed, idx >> 1);
  const uint32_t u = (idx & 1) ? (bits >> 16) : (bits & 0xffffu);
  return u >= drop_thr(p) ? inv_keep : 0.0f;
}

// keep factors (0 or 1/(1-p)) of the 4 consecutive elements idx0..idx0+3: the same bits as four
// dropout_scale calls, from 2 hashes (idx0 even) or 3 (odd)
__device__ __forceinline__ void dropout_scale4(uint64_t seed, uint64_t idx0, float p, float inv_keep, float (&z)[4]) {
  if (p <= 0.f) {
#pragma unroll
    for (int i = 0; i < 4; ++i) z[i] = 1.0f;
    return;
  }
  const uint32_t thr = drop_thr(p);
  const uint64_t pr = idx0 >> 1;
  const uint32_t b0 = drop_bits2(seed, pr), b1 = drop_bits2(seed, pr + 1);
  uint32_t u[4];
  if ((idx0 & 1) == 0) {
    u[0] = b0 & 0xffffu; u[1] = b0 >> 16; u[2] = b1 & 0xffffu; u[3] = b1 >> 16;
  } else {
    const uint32_t b2 = drop_bits2(seed, pr + 2);
    u[0] = b0 >> 16; u[1] = b1 & 0xffffu; u[2] = b1 >> 16; u[3] = b2 & 0xffffu;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) z[i] = u[i] >= thr ? inv_keep : 0.0f;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

__host__ __device__ __forceinline__ int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// ---- zero fill as a KERNEL node -------------------------------------------------------------
// The library zeroes its scratch with this kernel, never with hipMemsetAsync: inside a stream capture
// that also carries the hand-added event-record nodes of the live GEMM timing (runtime.hip), a memset
// node is the one node kind whose ordering we cannot check, and an accumulator zeroed out of order
// reads whatever tensor owned the block earlier in the capture.
namespace {
__global__ void __launch_bounds__(256) zero_words_kernel(uint32_t* __restrict__ p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) p[i] = 0u;
}
// bytes must be a multiple of 4 (every caller zeroes fp32 / uint32 words)
inline void zero_async(void* p, int64_t bytes, hipStream_t stream) {
  const int64_t n = bytes / 4;
  if (n <= 0) return;
  const int64_t nb = cdiv(n, 256) < 1024 ? cdiv(n, 256) : 1024;
  hipLaunchKernelGGL(zero_words_kernel, dim3((unsigned)nb), dim3(256), 0, stream, reinterpret_cast<uint32_t*>(p), n);
}

// out[0] = sum of n partials part[i * stride + k] ... fixed order (one wave, lane-strided then a shuffle tree):
// a deterministic replacement for same-address float atomics
__device__ __forceinline__ float sum_partials_wave(const float* __restrict__ part, int64_t n, int64_t stride) {
  const int lane = threadIdx.x & 63;
  float s = 0.f;
  for (int64_t i = lane; i < n; i += 64) s += part[i * stride];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  return s;
}

// Deterministic-mode column reduction (dph_set_deterministic): a block of 32 x DET_PH threads sums 32 columns of a
// [nrows][ld] fp32 partial slab over ALL its rows in a fixed order -- thread (column tx, phase ph) takes rows ph,
// ph + DET_PH, ... into four chains (added in chain order), the DET_PH phase totals are added in phase order -- so the
// result does not depend on scheduling.  `p` points at row 0 of the thread's column (NULL: 0).  Every thread of the
// block must call it (it synchronises); the total is returned to the threads with ph == 0.
constexpr int DET_PH = 32;
__device__ __forceinline__ float det_column_total(const float* __restrict__ p, int64_t nrows, int64_t ld,
                                                  float (*red)[33]) {
  const int tx = threadIdx.x & 31, ph = threadIdx.x >> 5;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (p) {
    int64_t r = ph;
    for (; r + 3 * DET_PH < nrows; r += 4 * DET_PH) {
      s0 += p[r * ld];
      s1 += p[(r + DET_PH) * ld];
      s2 += p[(r + 2 * DET_PH) * ld];
      s3 += p[(r + 3 * DET_PH) * ld];
    }
    if (r < nrows) s0 += p[r * ld];
    if (r + DET_PH < nrows) s1 += p[(r + DET_PH) * ld];
    if (r + 2 * DET_PH < nrows) s2 += p[(r + 2 * DET_PH) * ld];
  }
  red[ph][tx] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  float t = 0.f;
  if (ph == 0) {
#pragma unroll 8
    for (int i = 0; i < DET_PH; ++i) t += red[i][tx];
  }
  __syncthreads();
  return t;
}
}  // namespace

// ---- per-step RNG epoch ---------------------------------------------------------------------
// Every kernel that draws dropout / HardConcrete noise mixes a device-resident epoch word into
// its seed at entry.  The trainer advances that word with a stream-ordered op once per step, so a
// captured HIP graph (fixed kernel arguments) still draws fresh noise on every replay, and the
// backward kernels of a step regenerate exactly the forward's masks.  Each translation unit has
// its own pointer variable (no -fgpu-rdc); dph_set_rng_epoch() sets all of them.
void register_epoch_setter(int (*fn)(const uint64_t*));
namespace {
__device__ const uint64_t* g_rng_epoch = nullptr;
int set_epoch_tu(const uint64_t* p) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_rng_epoch), &p, sizeof(p)) == hipSuccess ? 0 : -1;
}
struct EpochReg {
  EpochReg() { register_epoch_setter(&set_epoch_tu); }
};
EpochReg g_epoch_reg;
}  // namespace

__device__ __forceinline__ uint64_t epoch_seed(uint64_t seed) {
  const uint64_t* e = g_rng_epoch;
  return e ? seed + (*e) * 0x9E3779B97F4A7C15ull : seed;
}

}  // namespace dph
