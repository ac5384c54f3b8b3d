// HardConcrete L0 gates (hardconcrete.py:76-116) and the differentiable
// expected parameter count (model.py:109-113 + the get_num_params chain of
// components.py) used by the Lagrangian sparsity regulariser
// (lightning.py:267-273).
//
// The reference launches ~31-55 tiny kernels per step for the gates and ~100
// scalar ops for the expected size.  Here the expected size is a polynomial in
// the per-module l0 norms, evaluated (and differentiated analytically) by two
// kernels whose term table the host builds once from the model config.
#include "common.h"

namespace dph {
namespace {

__global__ void hc_fwd_kernel(const float* __restrict__ la, const float* __restrict__ u_in, float* __restrict__ u_out,
                              float* __restrict__ mask, int64_t n, uint64_t seed, float beta, float lo, float hi,
                              float eps) {
  seed = epoch_seed(seed);   // per-step RNG epoch (graph replays)
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  // u ~ U(eps, 1-eps)   (hardconcrete.py:96)
  const float u = u_in ? u_in[i] : eps + (1.0f - 2.0f * eps) * rand_uniform(seed, (uint64_t)i);
  if (u_out) u_out[i] = u;
  const float s = 1.0f / (1.0f + __expf(-((__logf(u / (1.0f - u)) + la[i]) / beta)));
  const float v = s * (hi - lo) + lo;
  mask[i] = v == 0.0f ? __int_as_float(1) : fminf(fmaxf(v, 0.0f), 1.0f);   // (see hc_bank_fwd_kernel)
}

__global__ void hc_bwd_kernel(const float* __restrict__ la, const float* __restrict__ u, const float* __restrict__ dm,
                              float* __restrict__ dla, int64_t n, float beta, float lo, float hi) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float s = 1.0f / (1.0f + __expf(-((__logf(u[i] / (1.0f - u[i])) + la[i]) / beta)));
  const float v = s * (hi - lo) + lo;
  // clamp backward passes the gradient on the closed interval [0, 1] (torch semantics)
  const float pass = (v >= 0.0f && v <= 1.0f) ? 1.0f : 0.0f;
  dla[i] += dm[i] * pass * (hi - lo) * s * (1.0f - s) / beta;
}

// ---- batched gates: every HardConcrete module of a model in one launch (forward) / one launch
// (backward), instead of one pair of launches per module (31 per step for HuBERT-Base conv,head,interm).
// The entry table travels BY VALUE in the kernel arguments, so a captured HIP graph replays it with
// no device-side table; DPH_HC_BANK_CHUNK entries per launch.
constexpr int kBankChunk = DPH_HC_BANK_CHUNK;
struct BankArgs {
  const float* la[kBankChunk];
  const float* uin[kBankChunk];   // fwd: injected u (NULL: draw); bwd: unused
  float* dst[kBankChunk];          // fwd: unused (mask at mask_flat + off); bwd: dlog_alpha (+=)
  const float* dm[kBankChunk];     // bwd: dmask (NULL: no gradient reached this gate)
  int64_t off[kBankChunk];         // offset of the entry in the flat u / mask buffers
  int32_t n[kBankChunk];
};

__device__ __forceinline__ float hc_s(float u, float la, float beta) {
  return 1.0f / (1.0f + __expf(-((__logf(u / (1.0f - u)) + la) / beta)));
}

// grid (ceil(max n / 256), entries)
__global__ void __launch_bounds__(256) hc_bank_fwd_kernel(BankArgs a, float* __restrict__ u_flat,
                                                          float* __restrict__ mask_flat, uint64_t seed, float beta,
                                                          float lo, float hi, float eps) {
  seed = epoch_seed(seed);
  const int e = blockIdx.y;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= a.n[e]) return;
  const int64_t f = a.off[e] + i;
  // u ~ U(eps, 1-eps) (hardconcrete.py:96), counter = flat index over the whole bank
  const float u = a.uin[e] ? a.uin[e][i] : eps + (1.0f - 2.0f * eps) * rand_uniform(seed, (uint64_t)f);
  u_flat[f] = u;
  const float v = hc_s(u, a.la[e][i], beta) * (hi - lo) + lo;
  // (a pre-clamp value of exactly 0 still passes the clamp's gradient (closed interval, below): its mask is the
  // smallest subnormal instead of 0, so "mask == 0" means "no gradient through this gate" and the attention
  // kernels may skip such a head entirely)
  mask_flat[f] = v == 0.0f ? __int_as_float(1) : fminf(fmaxf(v, 0.0f), 1.0f);
}

__global__ void __launch_bounds__(256) hc_bank_bwd_kernel(BankArgs a, const float* __restrict__ u_flat, float beta,
                                                          float lo, float hi) {
  const int e = blockIdx.y;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= a.n[e] || a.dm[e] == nullptr) return;
  const float s = hc_s(u_flat[a.off[e] + i], a.la[e][i], beta);
  const float v = s * (hi - lo) + lo;
  const float pass = (v >= 0.0f && v <= 1.0f) ? 1.0f : 0.0f;   // clamp backward on the closed interval
  a.dst[e][i] += a.dm[e][i] * pass * (hi - lo) * s * (1.0f - s) / beta;
}

// l0[g] = sum_i sigmoid(la_g[i] + bias), one block per group
__global__ void __launch_bounds__(256) l0_kernel(const float* const* __restrict__ ptrs,
                                                 const int64_t* __restrict__ sizes, float bias,
                                                 float* __restrict__ l0) {
  __shared__ float red[4];
  const int64_t g = blockIdx.x;
  const float* p = ptrs[g];
  const int64_t n = sizes[g];
  float s = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += 256) s += 1.0f / (1.0f + __expf(-(p[i] + bias)));
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) l0[g] = red[0] + red[1] + red[2] + red[3];
}

__device__ double term_value(const double* coef, const int32_t* idx, int64_t t, const float* l0, int skip_slot) {
  double v = coef[t];
  for (int a = 0; a < 3; ++a) {
    const int k = idx[t * 3 + a];
    if (k >= 0 && a != skip_slot) v *= (double)l0[k];
  }
  return v;
}

__global__ void poly_kernel(const double* __restrict__ coef, const int32_t* __restrict__ idx, int64_t n_terms,
                            double constant, const float* __restrict__ l0, float* __restrict__ out) {
  __shared__ double red[256];
  double s = 0.0;
  for (int64_t t = threadIdx.x; t < n_terms; t += blockDim.x) s += term_value(coef, idx, t, l0, -1);
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = (float)(red[0] + constant);
}

// grad: one block per group g: dE/dl0[g] (product rule over the terms), then
// dla[i] += dout * dE/dl0[g] * sigmoid'(la + bias)
__global__ void __launch_bounds__(256) poly_bwd_kernel(const float* const* __restrict__ ptrs,
                                                       float* __restrict__ gflat,
                                                       const int64_t* __restrict__ goff,
                                                       const int64_t* __restrict__ sizes,
                                                       const double* __restrict__ coef,
                                                       const int32_t* __restrict__ idx, int64_t n_terms,
                                                       const float* __restrict__ l0, const float* __restrict__ dout,
                                                       float bias) {
  __shared__ double red[256];
  const int g = blockIdx.x;
  double s = 0.0;
  for (int64_t t = threadIdx.x; t < n_terms; t += blockDim.x)
    for (int a = 0; a < 3; ++a)
      if (idx[t * 3 + a] == g) s += term_value(coef, idx, t, l0, a);
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  const float dl0 = (float)red[0] * (dout ? *dout : 1.0f);
  const float* p = ptrs[g];
  float* gp = gflat + goff[g];
  const int64_t n = sizes[g];
  for (int64_t i = threadIdx.x; i < n; i += 256) {
    const float sg = 1.0f / (1.0f + __expf(-(p[i] + bias)));
    gp[i] += dl0 * sg * (1.0f - sg);
  }
}

}  // namespace
}  // namespace dph

using namespace dph;

extern "C" int dph_hc_sample_fwd(const float* log_alpha, const float* u_in, float* u_out, float* mask, int64_t n,
                                 uint64_t seed, float beta, float limit_l, float limit_r, float eps,
                                 hipStream_t stream) {
  DPH_REQUIRE(log_alpha && mask && n > 0, "dph_hc_sample_fwd: bad args");
  hipLaunchKernelGGL(hc_fwd_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, stream, log_alpha, u_in, u_out, mask,
                     n, seed, beta, limit_l, limit_r, eps);
  return check_launch("dph_hc_sample_fwd");
}

extern "C" int dph_hc_sample_bwd(const float* log_alpha, const float* u, const float* dmask, float* dlog_alpha,
                                 int64_t n, float beta, float limit_l, float limit_r, hipStream_t stream) {
  DPH_REQUIRE(log_alpha && u && dmask && dlog_alpha && n > 0, "dph_hc_sample_bwd: bad args");
  hipLaunchKernelGGL(hc_bwd_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, stream, log_alpha, u, dmask,
                     dlog_alpha, n, beta, limit_l, limit_r);
  return check_launch("dph_hc_sample_bwd");
}

static int bank_launch(bool fwd, const DphHcEntry* entries, int64_t n_entries, float* u_flat, float* mask_flat,
                       uint64_t seed, float beta, float lo, float hi, float eps, hipStream_t stream) {
  for (int64_t c0 = 0; c0 < n_entries; c0 += kBankChunk) {
    const int ne = (int)std::min<int64_t>(kBankChunk, n_entries - c0);
    BankArgs a = {};
    int64_t nmax = 0;
    for (int e = 0; e < ne; ++e) {
      const DphHcEntry& x = entries[c0 + e];
      DPH_REQUIRE(x.log_alpha && x.n > 0 && x.n < (1ll << 31) && x.offset >= 0, "dph_hc_bank: bad entry %lld",
                  (long long)(c0 + e));
      DPH_REQUIRE(fwd || x.dmask == nullptr || x.dlog_alpha, "dph_hc_bank_bwd: entry %lld has a dmask but no "
                  "dlog_alpha", (long long)(c0 + e));
      a.la[e] = x.log_alpha;
      a.uin[e] = x.u_in;
      a.dst[e] = x.dlog_alpha;
      a.dm[e] = x.dmask;
      a.off[e] = x.offset;
      a.n[e] = (int32_t)x.n;
      nmax = std::max<int64_t>(nmax, x.n);
    }
    const dim3 grid((unsigned)cdiv(nmax, 256), (unsigned)ne);
    if (fwd)
      hipLaunchKernelGGL(hc_bank_fwd_kernel, grid, dim3(256), 0, stream, a, u_flat, mask_flat, seed, beta, lo, hi, eps);
    else
      hipLaunchKernelGGL(hc_bank_bwd_kernel, grid, dim3(256), 0, stream, a, (const float*)u_flat, beta, lo, hi);
  }
  return check_launch(fwd ? "dph_hc_bank_fwd" : "dph_hc_bank_bwd");
}

extern "C" int dph_hc_bank_fwd(const DphHcEntry* entries, int64_t n_entries, float* u_flat, float* mask_flat,
                               uint64_t seed, float beta, float limit_l, float limit_r, float eps, hipStream_t stream) {
  DPH_REQUIRE(entries && n_entries > 0 && u_flat && mask_flat, "dph_hc_bank_fwd: bad args");
  return bank_launch(true, entries, n_entries, u_flat, mask_flat, seed, beta, limit_l, limit_r, eps, stream);
}

extern "C" int dph_hc_bank_bwd(const DphHcEntry* entries, int64_t n_entries, const float* u_flat, float beta,
                               float limit_l, float limit_r, hipStream_t stream) {
  DPH_REQUIRE(entries && n_entries > 0 && u_flat, "dph_hc_bank_bwd: bad args");
  return bank_launch(false, entries, n_entries, const_cast<float*>(u_flat), nullptr, 0, beta, limit_l, limit_r, 0.f,
                     stream);
}

extern "C" int dph_expected_params_fwd(const float* const* la_ptrs, const int64_t* la_sizes, int64_t n_groups,
                                       const double* coef, const int32_t* idx, int64_t n_terms, double constant,
                                       float hc_bias, float* l0, float* out, hipStream_t stream) {
  DPH_REQUIRE(out && l0 && (n_groups == 0 || (la_ptrs && la_sizes)) && (n_terms == 0 || (coef && idx)),
              "dph_expected_params_fwd: bad args");
  if (n_groups > 0)
    hipLaunchKernelGGL(l0_kernel, dim3((unsigned)n_groups), dim3(256), 0, stream, la_ptrs, la_sizes, hc_bias, l0);
  hipLaunchKernelGGL(poly_kernel, dim3(1), dim3(256), 0, stream, coef, idx, n_terms, constant, l0, out);
  return check_launch("dph_expected_params_fwd");
}

extern "C" int dph_expected_params_bwd(const float* const* la_ptrs, float* grad_flat, const int64_t* grad_offsets,
                                       const int64_t* la_sizes, int64_t n_groups, const double* coef,
                                       const int32_t* idx, int64_t n_terms, const float* l0, const float* dout,
                                       float hc_bias, hipStream_t stream) {
  DPH_REQUIRE(n_groups >= 0, "dph_expected_params_bwd: bad args");
  if (n_groups == 0) return DPH_OK;
  DPH_REQUIRE(la_ptrs && grad_flat && grad_offsets && la_sizes && coef && idx && l0,
              "dph_expected_params_bwd: null pointer");
  hipLaunchKernelGGL(poly_bwd_kernel, dim3((unsigned)n_groups), dim3(256), 0, stream, la_ptrs, grad_flat, grad_offsets,
                     la_sizes,
                     coef, idx, n_terms, l0, dout, hc_bias);
  return check_launch("dph_expected_params_bwd");
}
