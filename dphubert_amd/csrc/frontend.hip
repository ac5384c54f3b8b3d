// Waveform frontend of the FeatureExtractor and the positional-conv weight norm.
//
// conv0 (1 -> C channels, kernel k0, stride s0, no bias) + GroupNorm(C, C) +
// exact GELU + HardConcrete channel mask  (components.py:81-87,107-114,
// 1071-1076).  conv0 has a single input channel, so it is NOT a GEMM: each
// output is a k0-tap FIR of the waveform.  The waveform tile sits in LDS and
// every tap is an LDS broadcast read; conv0 is recomputed (10 FMAs/output)
// instead of ever storing its pre-norm output, so the only HBM traffic is the
// bf16 layer output (and its gradient in backward).
//
// Statistics: per (utterance, channel) over L0 = floor((S-k0)/s0)+1 steps, in closed form
// from the waveform's per-utterance tap sums and 10 x 10 Gram matrix (fp64, conv0_gram_reduce):
// biased variance, eps = 1e-5, as torch.group_norm.
//
// Weight norm (components.py:306, dim=2): w = g * v / ||v||_(dims 0,1).
#include "common.h"

#ifndef DPH_C0_ABL
#define DPH_C0_ABL 0   // diagnostic builds only: 1 = conv0 GELU / GELU' replaced by a cheap stand-in (timing ablation)
#endif

namespace dph {
namespace {
#if DPH_C0_ABL
__device__ __forceinline__ float c0_gelu(float x) { return x * 0.5f; }
__device__ __forceinline__ void c0_gelu_and_grad(float x, float& g, float& d) { g = 0.5f * x; d = 0.5f; }
#else
__device__ __forceinline__ float c0_gelu(float x) { return gelu_f(x); }
__device__ __forceinline__ void c0_gelu_and_grad(float x, float& g, float& d) { gelu_and_grad(x, g, d); }
#endif

// conv0 of every wav2vec2 / HuBERT / WavLM config is (512, 10, 5): compile-time taps and stride let
// each thread keep a sliding window of the waveform in registers (k0 = 2*s0: consecutive rows share
// half their taps), so a row costs s0 LDS broadcast reads instead of k0.
constexpr int K0 = 10;
constexpr int S0 = 5;
static_assert(K0 == 2 * S0, "sliding window assumes k0 = 2*s0");
constexpr int APPLY_ROWS = 256;  // time steps per apply block
constexpr int BWD_ROWS = 512;    // time steps per backward block

struct Conv0 {
  int64_t B, S, C, L0;
};

// thread layout shared by the conv0 kernels: TPR threads per time row (CPT channels each), RPP
// thread-rows per block, each owning a CONTIGUOUS range of nper time steps (sliding window)
template <int CPT>
struct RowLayout {
  int tpr, rpp;
  __device__ RowLayout(int64_t C) {
    tpr = (int)((C + CPT - 1) / CPT);
    rpp = max(1, 256 / tpr);
  }
};

__device__ __forceinline__ void win_load(float (&x)[K0], const float* xs, int t) {
#pragma unroll
  for (int j = 0; j < K0; ++j) x[j] = xs[t * S0 + j];
}

// window of row t -> window of row t+1
__device__ __forceinline__ void win_advance(float (&x)[K0], const float* xs, int t) {
#pragma unroll
  for (int j = 0; j < S0; ++j) x[j] = x[j + S0];
#pragma unroll
  for (int j = 0; j < S0; ++j) x[S0 + j] = xs[(t + 1) * S0 + S0 + j];
}

template <int CPT>
__device__ __forceinline__ void fir(const float (&wr)[CPT][K0], const float (&x)[K0], float (&v)[CPT]) {
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    float a = 0.f;
#pragma unroll
    for (int j = 0; j < K0; ++j) a = fmaf(wr[i][j], x[j], a);
    v[i] = a;
  }
}

template <int CPT>
__device__ __forceinline__ void load_taps(float (&wr)[CPT][K0], const float* w, int64_t c0, int64_t C, bool active) {
#pragma unroll
  for (int i = 0; i < CPT; ++i)
#pragma unroll
    for (int j = 0; j < K0; ++j) wr[i][j] = (active && c0 + i < C) ? w[(c0 + i) * K0 + j] : 0.f;
}

// stage the waveform samples of time steps [t0, t0+nt) in LDS
__device__ __forceinline__ int stage_wave(float* xs, const float* wave, const Conv0& p, int64_t b, int64_t t0,
                                          int nt) {
  const int nsamp = (nt - 1) * S0 + K0;
  const float* xw = wave + b * p.S + t0 * S0;
  for (int i = threadIdx.x; i < nsamp; i += blockDim.x) xs[i] = xw[i];
  __syncthreads();
  return nsamp;
}

// VEC: C % 8 == 0, every thread's 8 channels one 16-byte store (no per-row branch)
template <bool GN, bool VEC>
__global__ void __launch_bounds__(256) conv0_apply_kernel(const float* __restrict__ wave, const float* __restrict__ w,
                                                          const float* __restrict__ bias, Conv0 p,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ beta,
                                                          const float* __restrict__ mask,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ rstd, bf16_t* __restrict__ y) {
  constexpr int CPT = 8;
  __shared__ float xs[APPLY_ROWS * S0 + K0];
  const int64_t b = blockIdx.y;
  const int64_t t0 = (int64_t)blockIdx.x * APPLY_ROWS;
  const int nt = (int)min<int64_t>(APPLY_ROWS, p.L0 - t0);
  stage_wave(xs, wave, p, b, t0, nt);
  RowLayout<CPT> L(p.C);
  const int tid = threadIdx.x;
  if (tid >= L.tpr * L.rpp) return;
  const int64_t c0 = (int64_t)(tid % L.tpr) * CPT;
  const int r0 = tid / L.tpr;
  float wr[CPT][K0], sc[CPT], sh[CPT], mk[CPT];
  load_taps<CPT>(wr, w, c0, p.C, true);
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int64_t c = c0 + i;
    const bool ok = c < p.C;
    if (GN) {
      const float rs = ok ? rstd[b * p.C + c] : 0.f;
      const float g = ok ? gamma[c] : 0.f;
      sc[i] = g * rs;
      sh[i] = ok ? beta[c] - mean[b * p.C + c] * g * rs : 0.f;
    } else {
      sc[i] = 1.f;
      sh[i] = (ok && bias) ? bias[c] : 0.f;
    }
    mk[i] = (ok && mask) ? mask[c] : 1.f;
  }
  const int nper = (nt + L.rpp - 1) / L.rpp;
  const int ta = r0 * nper;
  const int tb = min(nt, ta + nper);
  if (ta >= tb) return;
  float x[K0];
  win_load(x, xs, ta);
  // (the window advance past the last row reads xs within its K0 - S0 slack, never used)
  for (int t = ta; t < tb; ++t) {
    float o[CPT];
    fir<CPT>(wr, x, o);
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const float v = fmaf(o[i], sc[i], sh[i]);
      o[i] = GN ? c0_gelu(v) * mk[i] : v;
    }
    bf16_t* yp = y + ((b * p.L0) + t0 + t) * p.C + c0;
    if (VEC) {
      *reinterpret_cast<uint4*>(yp) = make_uint4(pack2bf(o[0], o[1]), pack2bf(o[2], o[3]), pack2bf(o[4], o[5]),
                                                 pack2bf(o[6], o[7]));
    } else {
#pragma unroll
      for (int i = 0; i < CPT; ++i)
        if (c0 + i < p.C) yp[i] = f2bf(o[i]);
    }
    win_advance(x, xs, t);
  }
}

// CPT consecutive bf16 channels of one dy row -> fp32 (one 4/8/16-byte load when aligned)
// (VEC: the caller guarantees C % CPT == 0, every row a whole vector -- no per-load branch)
template <int CPT, bool VEC = false>
__device__ __forceinline__ void load_dyc(const bf16_t* dyp, int64_t c0, int64_t C, float (&d)[CPT]) {
  if (VEC || (c0 + CPT <= C && (C % CPT) == 0)) {
    uint32_t r[CPT / 2];
    if constexpr (CPT == 2) {
      r[0] = *reinterpret_cast<const uint32_t*>(dyp);
    } else if constexpr (CPT == 4) {
      const uint2 v = *reinterpret_cast<const uint2*>(dyp);
      r[0] = v.x; r[1] = v.y;
    } else {
      static_assert(CPT == 8, "CPT");
      const uint4 v = *reinterpret_cast<const uint4*>(dyp);
      r[0] = v.x; r[1] = v.y; r[2] = v.z; r[3] = v.w;
    }
#pragma unroll
    for (int i = 0; i < CPT / 2; ++i) {
      d[2 * i] = __uint_as_float(r[i] << 16);
      d[2 * i + 1] = __uint_as_float(r[i] & 0xffff0000u);
    }
  } else {
#pragma unroll
    for (int i = 0; i < CPT; ++i) d[i] = (c0 + i < C) ? bf2f(dyp[i]) : 0.f;
  }
}

// Backward in ONE pass over dy (components.py:107-114 backward: GroupNorm(C groups) + GELU + mask).
// With g = gamma*xh + beta, dg = dy*mask*GELU'(g), dxh = dg*gamma, the GroupNorm input gradient is
// dconv = rstd*(dxh - A/N - xh*Bv/N) (A = sum_t dxh, Bv = sum_t dxh*xh), and the conv0 weight
// gradient dw[c][j] = sum_t dconv[t]*x_j[t] (x_j[t] = wave[s0*t+j]) is LINEAR in per-(b,c) sums:
//   dw[c][j] = sum_b rstd*(P_j - (A/N)*S_j - (Bv/N)*Q_j),
//   P_j = sum_t dxh*x_j (accumulated here), S_j = sum_t x_j and
//   Q_j = sum_t xh*x_j = rstd*(sum_k w[c][k]*G[k][j] - mean*S_j) from the per-utterance Gram matrix
//   G[k][j] = sum_t x_k*x_j of the waveform (conv0_gram_part_kernel + conv0_gram_reduce).
// So the old second pass (recompute conv0 + GELU' + dconv) disappears.  Per (b, c) the blocks add
// their 15 partial sums (P[10], A, Bv, dgamma, dbeta, dmask) into ws with fp32 atomics (63 time
// blocks per address), conv0_bwd_finalize combines them.  dy is prefetched 4 time steps ahead.
constexpr int NQ = 15;
typedef float f32x2_t __attribute__((ext_vector_type(2)));

template <int CPT, int PF, bool VEC>
__global__ void __launch_bounds__(256) conv0_gn_bwd_kernel(const float* __restrict__ wave,
                                                           const float* __restrict__ w, Conv0 p,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta,
                                                           const float* __restrict__ mask,
                                                           const float* __restrict__ mean,
                                                           const float* __restrict__ rstd,
                                                           const bf16_t* __restrict__ dy, float* __restrict__ sums,
                                                           int rows, float* __restrict__ part) {
  __shared__ float xs[BWD_ROWS * S0 + K0];
  __shared__ float red[256 * CPT];
  const int64_t b = blockIdx.y;
  const int64_t t0 = (int64_t)blockIdx.x * rows;
  const int nt = (int)min<int64_t>(rows, p.L0 - t0);
  stage_wave(xs, wave, p, b, t0, nt);
  RowLayout<CPT> L(p.C);
  const int tid = threadIdx.x;
  const bool active = tid < L.tpr * L.rpp;
  const int64_t c0 = active ? (int64_t)(tid % L.tpr) * CPT : 0;
  const int r0 = active ? tid / L.tpr : 0;
  float wr[CPT][K0], mu[CPT], rs[CPT], ga[CPT], be[CPT], mk[CPT];
  load_taps<CPT>(wr, w, c0, p.C, active);
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int64_t c = c0 + i;
    const bool ok = active && c < p.C;
    mu[i] = ok ? mean[b * p.C + c] : 0.f;
    rs[i] = ok ? rstd[b * p.C + c] : 0.f;
    ga[i] = ok ? gamma[c] : 0.f;
    be[i] = ok ? beta[c] : 0.f;
    mk[i] = (ok && mask) ? mask[c] : 1.f;
  }
  float acc[CPT][NQ];
#pragma unroll
  for (int i = 0; i < CPT; ++i)
#pragma unroll
    for (int q = 0; q < NQ; ++q) acc[i][q] = 0.f;
  f32x2_t acc2[CPT / 2 > 0 ? CPT / 2 : 1][NQ];      // (CPT even: the packed accumulators)
#pragma unroll
  for (int i = 0; i < (CPT / 2 > 0 ? CPT / 2 : 1); ++i)
#pragma unroll
    for (int q = 0; q < NQ; ++q) acc2[i][q] = f32x2_t{0.f, 0.f};
  const int nper = (nt + L.rpp - 1) / L.rpp;
  const int ta = r0 * nper;
  const int tb = min(nt, ta + nper);
  // one time step of one thread's CPT channels (d: its dy row)
  auto step = [&](const float (&x)[K0], const float (&d)[CPT]) {
    if constexpr (CPT % 2 == 0) {
      // channel pairs in packed fp32 (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32: two lanes' worth of the
      // FIR, the 10 tap sums and the 5 statistics per instruction); the same operations and rounding as the
      // scalar path, only GELU / GELU' stay per channel
#pragma unroll
      for (int pi = 0; pi < CPT / 2; ++pi) {
        const int i0 = 2 * pi, i1 = 2 * pi + 1;
        f32x2_t v = {0.f, 0.f};
#pragma unroll
        for (int j = 0; j < K0; ++j) v = __builtin_elementwise_fma(f32x2_t{wr[i0][j], wr[i1][j]}, f32x2_t{x[j], x[j]}, v);
        const f32x2_t xh = (v - f32x2_t{mu[i0], mu[i1]}) * f32x2_t{rs[i0], rs[i1]};
        const f32x2_t g = __builtin_elementwise_fma(f32x2_t{ga[i0], ga[i1]}, xh, f32x2_t{be[i0], be[i1]});
        float gl0, gd0, gl1, gd1;
        c0_gelu_and_grad(g.x, gl0, gd0);
        c0_gelu_and_grad(g.y, gl1, gd1);
        const f32x2_t cu = {d[i0], d[i1]};
        // dg' = dy GELU'(g): the channel's mask and gamma are factored out of every sum (applied per block)
        const f32x2_t dgp = cu * f32x2_t{gd0, gd1};
#pragma unroll
        for (int j = 0; j < K0; ++j) acc2[pi][j] = __builtin_elementwise_fma(dgp, f32x2_t{x[j], x[j]}, acc2[pi][j]);
        acc2[pi][10] += dgp;
        acc2[pi][11] = __builtin_elementwise_fma(dgp, xh, acc2[pi][11]);
        acc2[pi][14] = __builtin_elementwise_fma(cu, f32x2_t{gl0, gl1}, acc2[pi][14]);
      }
    } else {
      float v[CPT];
      fir<CPT>(wr, x, v);
#pragma unroll
      for (int i = 0; i < CPT; ++i) {
        const float xh = (v[i] - mu[i]) * rs[i];
        const float g = fmaf(ga[i], xh, be[i]);
        float gl, gd;
        c0_gelu_and_grad(g, gl, gd);
        const float dgp = d[i] * gd;
#pragma unroll
        for (int j = 0; j < K0; ++j) acc[i][j] = fmaf(dgp, x[j], acc[i][j]);
        acc[i][10] += dgp;
        acc[i][11] = fmaf(dgp, xh, acc[i][11]);
        acc[i][14] = fmaf(d[i], gl, acc[i][14]);
      }
    }
  };
  if (active && ta < tb) {
    const bf16_t* dyrow = dy + ((b * p.L0) + t0) * p.C + c0;
    float x[K0];
    win_load(x, xs, ta);
    // dy rows prefetched PF steps ahead; a row past tb is clamped to tb - 1 (loaded, never used) so the loads
    // carry no branch.  The window advance past the last row reads xs within its K0 - S0 slack (never used).
    float cur[PF][CPT], nxt[PF][CPT];
#pragma unroll
    for (int u = 0; u < PF; ++u) load_dyc<CPT, VEC>(dyrow + (int64_t)min(ta + u, tb - 1) * p.C, c0, p.C, cur[u]);
    int tg = ta;
    for (; tg + PF <= tb; tg += PF) {
#pragma unroll
      for (int u = 0; u < PF; ++u)
        load_dyc<CPT, VEC>(dyrow + (int64_t)min(tg + PF + u, tb - 1) * p.C, c0, p.C, nxt[u]);
#pragma unroll
      for (int u = 0; u < PF; ++u) {
        step(x, cur[u]);
        win_advance(x, xs, tg + u);
      }
#pragma unroll
      for (int u = 0; u < PF; ++u)
#pragma unroll
        for (int i = 0; i < CPT; ++i) cur[u][i] = nxt[u][i];
    }
    // ragged tail (< PF steps): its rows are already in cur
#pragma unroll
    for (int u = 0; u < PF - 1; ++u) {
      if (tg + u < tb) {
        step(x, cur[u]);
        win_advance(x, xs, tg + u);
      }
    }
  }
  if constexpr (CPT % 2 == 0) {
#pragma unroll
    for (int pi = 0; pi < CPT / 2; ++pi)
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        acc[2 * pi][q] = acc2[pi][q].x;
        acc[2 * pi + 1][q] = acc2[pi][q].y;
      }
  }
  // reduce over the rpp thread-rows sharing the same channels, then one atomic per (b, c, q) per block
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    if (q == 12 || q == 13) continue;   // derived from 10 / 11 below
#pragma unroll
    for (int i = 0; i < CPT; ++i) red[tid * CPT + i] = acc[i][q];
    __syncthreads();
    if (active && r0 == 0) {
#pragma unroll
      for (int i = 0; i < CPT; ++i) {
        float s = 0.f;
        for (int r = 0; r < L.rpp; ++r) s += red[(r * L.tpr + (tid % L.tpr)) * CPT + i];
        const int64_t c = c0 + i;
        // acc q: 0-9 sum dg' x_j, 10 sum dg', 11 sum dg' xh, 14 sum dy GELU(g) (12, 13 unused) -> the 15 sums
        // conv0_bwd_finalize reads: P_j = ga mk (0-9), A = ga mk S1, Bv = ga mk T2, dgamma = mk T2,
        // dbeta = mk S1, dmask
        if (c < p.C && q != 12 && q != 13 && part) {
          // deterministic mode: this block's 15 sums as its own slab entry, added in time-block order by
          // conv0_part_reduce
          const float gm = ga[i] * mk[i];
          float* o = part + ((b * gridDim.x + blockIdx.x) * p.C + c) * NQ;
          if (q < 10) {
            o[q] = gm * s;
          } else if (q == 10) {
            o[10] = gm * s;
            o[13] = mk[i] * s;
          } else if (q == 11) {
            o[11] = gm * s;
            o[12] = mk[i] * s;
          } else {
            o[14] = s;
          }
        } else if (c < p.C && q != 12 && q != 13) {
          const float gm = ga[i] * mk[i];
          float* o = sums + (b * p.C + c) * NQ;
          if (q < 10) {
            atomicAdd(o + q, gm * s);
          } else if (q == 10) {
            atomicAdd(o + 10, gm * s);
            atomicAdd(o + 13, mk[i] * s);
          } else if (q == 11) {
            atomicAdd(o + 11, gm * s);
            atomicAdd(o + 12, mk[i] * s);
          } else {
            atomicAdd(o + 14, s);
          }
        }
      }
    }
    __syncthreads();
  }
}

// Backward of the plain conv0 (layer_norm-mode extractors, components.py:107 conv with optional
// bias, its LayerNorm / GELU / mask backward already applied to dz): dw[c][j] += sum_{b,t} dz*x_j,
// dbias[c] += sum_{b,t} dz.  Same thread layout as the GN backward; one atomic per (c, tap) per block.
template <int CPT>
__global__ void __launch_bounds__(256) conv0_plain_bwd_kernel(const float* __restrict__ wave, Conv0 p,
                                                              const bf16_t* __restrict__ dz, float* __restrict__ dw,
                                                              float* __restrict__ dbias, float* __restrict__ part) {
  constexpr int NA = K0 + 1;
  __shared__ float xs[BWD_ROWS * S0 + K0];
  __shared__ float red[256 * CPT];
  const int64_t b = blockIdx.y;
  const int64_t t0 = (int64_t)blockIdx.x * BWD_ROWS;
  const int nt = (int)min<int64_t>(BWD_ROWS, p.L0 - t0);
  stage_wave(xs, wave, p, b, t0, nt);
  RowLayout<CPT> L(p.C);
  const int tid = threadIdx.x;
  const bool active = tid < L.tpr * L.rpp;
  const int64_t c0 = active ? (int64_t)(tid % L.tpr) * CPT : 0;
  const int r0 = active ? tid / L.tpr : 0;
  float acc[CPT][NA];
#pragma unroll
  for (int i = 0; i < CPT; ++i)
#pragma unroll
    for (int q = 0; q < NA; ++q) acc[i][q] = 0.f;
  const int nper = (nt + L.rpp - 1) / L.rpp;
  const int ta = r0 * nper;
  const int tb = min(nt, ta + nper);
  if (active && ta < tb) {
    const bf16_t* dzrow = dz + ((b * p.L0) + t0) * p.C + c0;
    float x[K0];
    win_load(x, xs, ta);
    for (int t = ta; t < tb; ++t) {
      float d[CPT];
      load_dyc<CPT>(dzrow + (int64_t)t * p.C, c0, p.C, d);
#pragma unroll
      for (int i = 0; i < CPT; ++i) {
#pragma unroll
        for (int j = 0; j < K0; ++j) acc[i][j] = fmaf(d[i], x[j], acc[i][j]);
        acc[i][K0] += d[i];
      }
      if (t + 1 < tb) win_advance(x, xs, t);
    }
  }
#pragma unroll
  for (int q = 0; q < NA; ++q) {
#pragma unroll
    for (int i = 0; i < CPT; ++i) red[tid * CPT + i] = acc[i][q];
    __syncthreads();
    if (active && r0 == 0) {
#pragma unroll
      for (int i = 0; i < CPT; ++i) {
        float sm = 0.f;
        for (int r = 0; r < L.rpp; ++r) sm += red[(r * L.tpr + (tid % L.tpr)) * CPT + i];
        const int64_t c = c0 + i;
        if (c < p.C && part) {
          // deterministic mode: this block's entry of the [b][time block][C][11] slab (conv0_plain_part_reduce)
          part[((b * gridDim.x + blockIdx.x) * p.C + c) * NA + q] = sm;
        } else if (c < p.C) {
          if (q < K0) atomicAdd(dw + c * K0 + q, sm);
          else if (dbias) atomicAdd(dbias + c, sm);
        }
      }
    }
    __syncthreads();
  }
}

// per utterance: S[j] = sum_t x_j[t], G[k][j] = sum_t x_k[t] x_j[t] (x_j[t] = wave[s0*t + j], t < L0),
// fp64, packed: gram[b][0..9] = S, gram[b][10 + j*(j+1)/2 + k] = G[k][j] (k <= j).
constexpr int NG = K0 + K0 * (K0 + 1) / 2;   // 65
constexpr int GRAM_CHUNKS = 16;   // fixed split of an utterance's steps (the workspace size does not depend on S)

__device__ __forceinline__ int gram_idx(int k, int j) {   // symmetric
  return k <= j ? K0 + j * (j + 1) / 2 + k : K0 + k * (k + 1) / 2 + j;
}

// Block (chunk, b) of a fixed GRAM_CHUNKS-way split of utterance b's steps writes its partial sums to
// gpart[(b * GRAM_CHUNKS + chunk) * NG + q]; conv0_gram_reduce adds them in chunk order (no atomics: the forward's
// GroupNorm statistics below are bitwise reproducible).
__global__ void __launch_bounds__(256) conv0_gram_part_kernel(const float* __restrict__ wave, Conv0 p,
                                                              double* __restrict__ gpart) {
  __shared__ double red[4][NG];
  const int64_t b = blockIdx.y;
  const float* xw = wave + b * p.S;
  const int64_t per = cdiv(p.L0, (int64_t)GRAM_CHUNKS);
  const int64_t t1 = min<int64_t>(p.L0, (int64_t)(blockIdx.x + 1) * per);
  double acc[NG];
#pragma unroll
  for (int q = 0; q < NG; ++q) acc[q] = 0.0;
  for (int64_t t = (int64_t)blockIdx.x * per + threadIdx.x; t < t1; t += 256) {
    float x[K0];
#pragma unroll
    for (int j = 0; j < K0; ++j) x[j] = xw[t * S0 + j];
#pragma unroll
    for (int j = 0; j < K0; ++j) {
      acc[j] += x[j];
#pragma unroll
      for (int k = 0; k <= j; ++k) acc[K0 + j * (j + 1) / 2 + k] += (double)x[k] * (double)x[j];
    }
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int q = 0; q < NG; ++q) {
    double v = acc[q];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) red[wv][q] = v;
  }
  __syncthreads();
  for (int q = threadIdx.x; q < NG; q += 256)
    gpart[(b * GRAM_CHUNKS + blockIdx.x) * NG + q] = (red[0][q] + red[1][q]) + (red[2][q] + red[3][q]);
}

// One block per utterance: gram[b] = the chunk partials summed in order (optional output), and -- with mean / rstd
// given -- the GroupNorm(C, C) statistics of conv0's output in closed form.  Channel c's conv value at step t is
// v = sum_j w[c][j] x_j[t], so over the N = L0 steps (the whole padded sequence, as torch.group_norm takes it)
//   mean = sum_j w_j S_j / N,   E[v^2] = sum_jk w_j w_k G_jk / N,   var = E[v^2] - mean^2   (biased, fp64)
// from the waveform's per-utterance sums S_j and Gram matrix G_jk: no pass over the B x L0 x C conv outputs.
__global__ void __launch_bounds__(256) conv0_gram_reduce(const double* __restrict__ gpart, const float* __restrict__ w,
                                                         Conv0 p, double* __restrict__ gram, float* __restrict__ mean,
                                                         float* __restrict__ rstd, float eps) {
  __shared__ double g[NG];
  const int64_t b = blockIdx.x;
  for (int q = threadIdx.x; q < NG; q += 256) {
    double v = 0.0;
    for (int ch = 0; ch < GRAM_CHUNKS; ++ch) v += gpart[(b * GRAM_CHUNKS + ch) * NG + q];
    g[q] = v;
    if (gram) gram[b * NG + q] = v;
  }
  __syncthreads();
  if (!mean) return;
  const double N = (double)p.L0;
  for (int64_t c = threadIdx.x; c < p.C; c += 256) {
    double wj[K0];
#pragma unroll
    for (int j = 0; j < K0; ++j) wj[j] = (double)w[c * K0 + j];
    double m = 0.0, e2 = 0.0;
#pragma unroll
    for (int j = 0; j < K0; ++j) {
      m = fma(wj[j], g[j], m);
      double r = 0.0;
#pragma unroll
      for (int k = 0; k < j; ++k) r = fma(wj[k], g[K0 + j * (j + 1) / 2 + k], r);
      e2 = fma(wj[j], fma(2.0, r, wj[j] * g[K0 + j * (j + 1) / 2 + j]), e2);
    }
    m /= N;
    const double var = fmax(e2 / N - m * m, 0.0);
    mean[b * p.C + c] = (float)m;
    rstd[b * p.C + c] = (float)(1.0 / sqrt(var + (double)eps));
  }
}

// deterministic mode: sums[b][c][q] = the time blocks' partials of utterance b added in block order (four chains)
__global__ void __launch_bounds__(256) conv0_part_reduce(const float* __restrict__ part, int64_t nblk, int64_t per_b,
                                                         int64_t B, float* __restrict__ sums) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= B * per_b) return;
  const int64_t b = i / per_b, j = i % per_b;
  const float* p = part + b * nblk * per_b + j;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int64_t k = 0;
  for (; k + 3 < nblk; k += 4) {
    s0 += p[k * per_b];
    s1 += p[(k + 1) * per_b];
    s2 += p[(k + 2) * per_b];
    s3 += p[(k + 3) * per_b];
  }
  for (; k < nblk; ++k) s0 += p[k * per_b];
  sums[i] = (s0 + s1) + (s2 + s3);
}

// deterministic mode of the plain conv0 backward: dw[c][j] / dbias[c] += the [b][time block][C][11] partials summed
// over (b, time block) in order, one thread per (c, q)
__global__ void __launch_bounds__(256) conv0_plain_part_reduce(const float* __restrict__ part, int64_t nbt, int64_t C,
                                                               float* __restrict__ dw, float* __restrict__ dbias) {
  constexpr int NA = K0 + 1;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= C * NA) return;
  const int64_t c = i / NA, q = i % NA;
  const float* p = part + i;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int64_t k = 0;
  for (; k + 3 < nbt; k += 4) {
    s0 += p[k * C * NA];
    s1 += p[(k + 1) * C * NA];
    s2 += p[(k + 2) * C * NA];
    s3 += p[(k + 3) * C * NA];
  }
  for (; k < nbt; ++k) s0 += p[k * C * NA];
  const float t = (s0 + s1) + (s2 + s3);
  if (q < K0) dw[c * K0 + q] += t;
  else if (dbias) dbias[c] += t;
}

// one thread per channel: combine the per-(b,c) sums into dw[c][j], dgamma, dbeta, dmask (accumulate)
__global__ void conv0_bwd_finalize(const float* __restrict__ sums, const double* __restrict__ gram,
                                   const float* __restrict__ w, const float* __restrict__ mean,
                                   const float* __restrict__ rstd, Conv0 p, float* __restrict__ dw,
                                   float* __restrict__ dgamma, float* __restrict__ dbeta, float* __restrict__ dmask) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= p.C) return;
  const double N = (double)p.L0;
  double wc[K0], dwc[K0];
#pragma unroll
  for (int j = 0; j < K0; ++j) {
    wc[j] = w[c * K0 + j];
    dwc[j] = 0.0;
  }
  double dga = 0.0, dbe = 0.0, dma = 0.0;
  for (int64_t b = 0; b < p.B; ++b) {
    const float* sm = sums + (b * p.C + c) * NQ;
    const double* gb = gram + b * NG;
    const double mu = mean[b * p.C + c], r = rstd[b * p.C + c];
    const double A = sm[10], Bv = sm[11];
#pragma unroll
    for (int j = 0; j < K0; ++j) {
      double cg = 0.0;
#pragma unroll
      for (int k = 0; k < K0; ++k) cg += wc[k] * gb[gram_idx(k, j)];
      const double Q = r * (cg - mu * gb[j]);
      dwc[j] += r * ((double)sm[j] - (A / N) * gb[j] - (Bv / N) * Q);
    }
    dga += sm[12];
    dbe += sm[13];
    dma += sm[14];
  }
#pragma unroll
  for (int j = 0; j < K0; ++j) dw[c * K0 + j] += (float)dwc[j];
  if (dgamma) dgamma[c] += (float)dga;
  if (dbeta) dbeta[c] += (float)dbe;
  if (dmask) dmask[c] += (float)dma;
}

// ---- weight norm -----------------------------------------------------------
// per-tap dot products over dims (0,1), deterministic two-stage reduction (no atomics, so the
// forward pass is bitwise reproducible): x [R][K] (R = Cout*Cin_g)
//   stage 1: part[blk][j] = sum_{r in blk} a[r][j]*b[r][j]
//   stage 2: out[j] = sum_blk part[blk][j]  (fixed order)
// 256 threads: with K <= 256, PH = 256 / K row phases per tap (thread (phase, tap) takes rows r0 + phase, + PH, ...
// into four chains, loads of four rows in flight), the phases added in order through LDS -- a fixed order, so
// deterministic.  (The round-4 form, one thread per tap walking its 64 rows one dependent load after the other
// over 128-thread blocks, ran 30 us for the positional conv's 19 MB.)
__global__ void __launch_bounds__(256) tap_dot_partial_kernel(const float* __restrict__ a,
                                                              const float* __restrict__ bb, int64_t R, int64_t K,
                                                              float* __restrict__ part, int64_t rows_per_block) {
  __shared__ float red[256];
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(R, r0 + rows_per_block);
  const int PH = K <= 256 ? (int)(256 / K) : 1;
  const int ph = (int)(threadIdx.x / (K <= 256 ? K : 256));
  for (int64_t j = threadIdx.x % (K <= 256 ? K : 256); j < K; j += 256) {
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    int64_t r = r0 + ph;
    if (ph < PH) {
      for (; r + 3 * PH < r1; r += 4 * PH) {
        s0 = fmaf(a[r * K + j], bb[r * K + j], s0);
        s1 = fmaf(a[(r + PH) * K + j], bb[(r + PH) * K + j], s1);
        s2 = fmaf(a[(r + 2 * PH) * K + j], bb[(r + 2 * PH) * K + j], s2);
        s3 = fmaf(a[(r + 3 * PH) * K + j], bb[(r + 3 * PH) * K + j], s3);
      }
      for (; r < r1; r += PH) s0 = fmaf(a[r * K + j], bb[r * K + j], s0);
    }
    const float s = (s0 + s1) + (s2 + s3);
    if (PH == 1) {
      part[(int64_t)blockIdx.x * K + j] = s;
    } else {
      red[threadIdx.x] = s;
      __syncthreads();
      if (ph == 0) {
        float t = 0.f;
        for (int q = 0; q < PH; ++q) t += red[q * K + j];
        part[(int64_t)blockIdx.x * K + j] = t;
      }
    }
  }
}

// one block per tap; fixed strided partition + fixed-shape tree (deterministic)
__global__ void __launch_bounds__(256) tap_dot_finalize_kernel(const float* __restrict__ part, int64_t nblk,
                                                               int64_t K, float* __restrict__ out) {
  __shared__ float red[4];
  const int64_t j = blockIdx.x;
  float s = 0.f;
  for (int64_t b = threadIdx.x; b < nblk; b += 256) s += part[b * K + j];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[j] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ void weight_norm_apply_kernel(const float* __restrict__ g, const float* __restrict__ v,
                                         const float* __restrict__ nsq, float* __restrict__ norm_out, int64_t Cout,
                                         int64_t Cin, int64_t K, int64_t G, float* __restrict__ w,
                                         bf16_t* __restrict__ wk, bf16_t* __restrict__ wt) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n = Cout * Cin * K;
  if (i < K && norm_out) norm_out[i] = sqrtf(nsq[i]);
  if (i >= n) return;
  const int64_t j = i % K;
  const int64_t c = (i / K) % Cin;
  const int64_t o = i / (K * Cin);
  const float val = g[j] * v[i] / sqrtf(nsq[j]);
  if (w) w[i] = val;
  const int64_t Cg = Cout / G;
  const int64_t grp = o / Cg;
  const int64_t oo = o % Cg;
  if (wk) wk[(grp * Cg + oo) * (K * Cin) + j * Cin + c] = f2bf(val);
  if (wt) wt[(grp * Cin + c) * (K * Cg) + (K - 1 - j) * Cg + oo] = f2bf(val);
}

// dw from the GEMM image layout [G][Cg][K*Cin] (index j*Cin + c) into [Cout][Cin][K]
__global__ void img_to_weight_kernel(const float* __restrict__ img, float* __restrict__ dw, int64_t Cout, int64_t Cin,
                                     int64_t K, int64_t G) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= Cout * Cin * K) return;
  const int64_t j = i % K;
  const int64_t c = (i / K) % Cin;
  const int64_t o = i / (K * Cin);
  const int64_t Cg = Cout / G;
  dw[i] = img[((o / Cg) * Cg + o % Cg) * (K * Cin) + j * Cin + c];
}

__global__ void weight_norm_bwd_kernel(const float* __restrict__ dw, const float* __restrict__ g,
                                       const float* __restrict__ v, const float* __restrict__ norm,
                                       const float* __restrict__ S, int64_t n, int64_t K, float* __restrict__ dg,
                                       float* __restrict__ dv) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < K && dg) dg[i] = S[i] / norm[i];
  if (i >= n) return;
  const int64_t j = i % K;
  const float nj = norm[j];
  dv[i] = g[j] / nj * dw[i] - g[j] * S[j] / (nj * nj * nj) * v[i];
}

}  // namespace
}  // namespace dph

using namespace dph;

static Conv0 make_conv0(int64_t B, int64_t S, int64_t C) {
  Conv0 p;
  p.B = B;
  p.S = S;
  p.C = C;
  p.L0 = (S - K0) / S0 + 1;
  return p;
}

extern "C" int dph_conv0_gn_fwd(const float* wave, int64_t B, int64_t S, const float* w, int64_t C, int64_t k0,
                                int64_t s0, const float* gamma, const float* beta, const float* mask, void* y,
                                float* mean, float* rstd, float* ws, int64_t ws_bytes, hipStream_t stream) {
  DPH_REQUIRE(wave && w && gamma && beta && y && mean && rstd && ws, "dph_conv0_gn_fwd: null pointer");
  if (k0 != K0 || s0 != S0) {
    set_error("dph_conv0_gn_fwd: conv0 kernel/stride (%lld,%lld) unsupported (only (10,5))", (long long)k0,
              (long long)s0);
    return DPH_EUNSUPPORTED;
  }
  DPH_REQUIRE(S >= K0 && C <= 2048, "dph_conv0_gn_fwd: unsupported S=%lld C=%lld", (long long)S, (long long)C);
  Conv0 p = make_conv0(B, S, C);
  DPH_REQUIRE(ws_bytes >= (int64_t)B * GRAM_CHUNKS * NG * 8, "dph_conv0_gn_fwd: workspace too small (%lld < %lld)",
              (long long)ws_bytes, (long long)(B * GRAM_CHUNKS * NG * 8));
  double* gpart = reinterpret_cast<double*>(ws);
  hipLaunchKernelGGL(conv0_gram_part_kernel, dim3(GRAM_CHUNKS, (unsigned)B), dim3(256), 0, stream, wave, p, gpart);
  hipLaunchKernelGGL(conv0_gram_reduce, dim3((unsigned)B), dim3(256), 0, stream, gpart, w, p, (double*)nullptr, mean,
                     rstd, 1e-5f);
  const dim3 grid((unsigned)cdiv(p.L0, APPLY_ROWS), (unsigned)B);
  if (C % 8 == 0)
    hipLaunchKernelGGL((conv0_apply_kernel<true, true>), grid, dim3(256), 0, stream, wave, w, (const float*)nullptr, p,
                       gamma, beta, mask, mean, rstd, reinterpret_cast<bf16_t*>(y));
  else
    hipLaunchKernelGGL((conv0_apply_kernel<true, false>), grid, dim3(256), 0, stream, wave, w, (const float*)nullptr, p,
                       gamma, beta, mask, mean, rstd, reinterpret_cast<bf16_t*>(y));
  return check_launch("dph_conv0_gn_fwd");
}

extern "C" int dph_conv0_fwd(const float* wave, int64_t B, int64_t S, const float* w, const float* bias, int64_t C,
                             int64_t k0, int64_t s0, void* y, hipStream_t stream) {
  DPH_REQUIRE(wave && w && y, "dph_conv0_fwd: null pointer");
  if (k0 != K0 || s0 != S0) {
    set_error("dph_conv0_fwd: conv0 kernel/stride (%lld,%lld) unsupported (only (10,5))", (long long)k0,
              (long long)s0);
    return DPH_EUNSUPPORTED;
  }
  DPH_REQUIRE(S >= K0 && C <= 2048, "dph_conv0_fwd: unsupported");
  Conv0 p = make_conv0(B, S, C);
  const dim3 grid((unsigned)cdiv(p.L0, APPLY_ROWS), (unsigned)B);
  const float* nul = nullptr;
  if (C % 8 == 0)
    hipLaunchKernelGGL((conv0_apply_kernel<false, true>), grid, dim3(256), 0, stream, wave, w, bias, p, nul, nul, nul,
                       nul, nul, reinterpret_cast<bf16_t*>(y));
  else
    hipLaunchKernelGGL((conv0_apply_kernel<false, false>), grid, dim3(256), 0, stream, wave, w, bias, p, nul, nul, nul,
                       nul, nul, reinterpret_cast<bf16_t*>(y));
  return check_launch("dph_conv0_fwd");
}

// workspace (bytes) of dph_conv0_bwd: the per-(utterance, time block) partial slab of deterministic mode
extern "C" int64_t dph_conv0_bwd_workspace(int64_t B, int64_t S, int64_t C) {
  if (B <= 0 || S < K0 || C <= 0) return 0;
  const int64_t L0 = (S - K0) / S0 + 1;
  return B * cdiv(L0, (int64_t)BWD_ROWS) * C * (K0 + 1) * 4;
}

extern "C" int dph_conv0_bwd(const float* wave, int64_t B, int64_t S, int64_t C, int64_t k0, int64_t s0,
                             const void* dz, float* dw, float* dbias, float* ws, int64_t ws_bytes,
                             hipStream_t stream) {
  DPH_REQUIRE(wave && dz && dw, "dph_conv0_bwd: null pointer");
  if (k0 != K0 || s0 != S0) {
    set_error("dph_conv0_bwd: conv0 kernel/stride (%lld,%lld) unsupported (only (10,5))", (long long)k0,
              (long long)s0);
    return DPH_EUNSUPPORTED;
  }
  DPH_REQUIRE(S >= K0 && C <= 1024, "dph_conv0_bwd: unsupported (C > 1024)");
  const bool det = deterministic();
  DPH_REQUIRE(!det || (ws && ws_bytes >= dph_conv0_bwd_workspace(B, S, C)),
              "dph_conv0_bwd: deterministic mode needs dph_conv0_bwd_workspace(B, S, C) bytes of workspace");
  Conv0 p = make_conv0(B, S, C);
  const int64_t nblk = cdiv(p.L0, (int64_t)BWD_ROWS);
  hipLaunchKernelGGL(conv0_plain_bwd_kernel<4>, dim3((unsigned)nblk, (unsigned)B), dim3(256), 0,
                     stream, wave, p, reinterpret_cast<const bf16_t*>(dz), dw, dbias, det ? ws : nullptr);
  if (det)
    hipLaunchKernelGGL(conv0_plain_part_reduce, dim3((unsigned)cdiv(C * (K0 + 1), 256)), dim3(256), 0, stream, ws,
                       B * nblk, C, dw, dbias);
  return check_launch("dph_conv0_bwd");
}

// (the smallest GroupNorm-backward time block is BWD_ROWS / 2 rows: DPH_C0B_VARIANT=3)
static int64_t conv0_gn_part_floats(int64_t B, int64_t S, int64_t C) {
  const int64_t L0 = S >= K0 ? (S - K0) / S0 + 1 : 0;
  return B * cdiv(L0, (int64_t)(BWD_ROWS / 2)) * C * NQ;
}

extern "C" int64_t dph_conv0_gn_bwd_workspace(int64_t B, int64_t S, int64_t C) {
  return cdiv(B * C * NQ * 4, 64) * 64 + B * NG * 8 + B * GRAM_CHUNKS * NG * 8 + conv0_gn_part_floats(B, S, C) * 4;
}

extern "C" int dph_conv0_gn_bwd(const float* wave, int64_t B, int64_t S, const float* w, int64_t C, int64_t k0,
                                int64_t s0, const float* gamma, const float* beta, const float* mask,
                                const float* mean, const float* rstd, const void* dy, float* dw, float* dgamma,
                                float* dbeta, float* dmask, float* ws, int64_t ws_bytes, hipStream_t stream) {
  DPH_REQUIRE(wave && w && gamma && beta && mean && rstd && dy && dw && ws, "dph_conv0_gn_bwd: null pointer");
  if (k0 != K0 || s0 != S0) {
    set_error("dph_conv0_gn_bwd: conv0 kernel/stride (%lld,%lld) unsupported (only (10,5))", (long long)k0,
              (long long)s0);
    return DPH_EUNSUPPORTED;
  }
  DPH_REQUIRE(S >= K0 && C <= 1024, "dph_conv0_gn_bwd: unsupported (C > 1024)");   // 256 threads x 4 channels
  DPH_REQUIRE(ws_bytes >= dph_conv0_gn_bwd_workspace(B, S, C), "dph_conv0_gn_bwd: workspace too small (%lld < %lld)",
              (long long)ws_bytes, (long long)dph_conv0_gn_bwd_workspace(B, S, C));
  Conv0 p = make_conv0(B, S, C);
  float* sums = ws;
  const int64_t sums_bytes = cdiv(B * C * NQ * 4, 64) * 64;
  double* gram = reinterpret_cast<double*>(reinterpret_cast<char*>(ws) + sums_bytes);
  double* gpart = gram + B * NG;
  // deterministic mode: per-(utterance, time block) partials after the Gram partials, reduced in order into sums
  const bool det = deterministic();
  float* part = det ? reinterpret_cast<float*>(gpart + B * GRAM_CHUNKS * NG) : nullptr;
  if (!det) zero_async(ws, sums_bytes, stream);
  hipLaunchKernelGGL(conv0_gram_part_kernel, dim3(GRAM_CHUNKS, (unsigned)B), dim3(256), 0, stream, wave, p, gpart);
  hipLaunchKernelGGL(conv0_gram_reduce, dim3((unsigned)B), dim3(256), 0, stream, gpart, w, p, gram, (float*)nullptr,
                     (float*)nullptr, 0.f);
  // DPH_C0B_VARIANT (tuning knob): 0 = 4 channels/thread, 4-row dy prefetch, 512 rows/block; 1 = 2 ch/thread;
  // 2 = 4 ch, 1-row prefetch; 3 = 4 ch, 256 rows/block
  static const int var = [] {
    const char* e = getenv("DPH_C0B_VARIANT");
    return e ? atoi(e) : 0;
  }();
  const int rows = var == 3 ? BWD_ROWS / 2 : BWD_ROWS;
  dim3 grid((unsigned)cdiv(p.L0, rows), (unsigned)B);
  const bf16_t* dyb = reinterpret_cast<const bf16_t*>(dy);
  const bool vec = C % 4 == 0;
  if (var == 1 && C <= 512 && vec)
    hipLaunchKernelGGL((conv0_gn_bwd_kernel<2, 4, true>), grid, dim3(256), 0, stream, wave, w, p, gamma, beta, mask, mean,
                       rstd, dyb, sums, rows, part);
  else if (var == 1 && C <= 512)
    hipLaunchKernelGGL((conv0_gn_bwd_kernel<2, 4, false>), grid, dim3(256), 0, stream, wave, w, p, gamma, beta, mask, mean,
                       rstd, dyb, sums, rows, part);
  else if (var == 2)
    hipLaunchKernelGGL((conv0_gn_bwd_kernel<4, 1, false>), grid, dim3(256), 0, stream, wave, w, p, gamma, beta, mask, mean,
                       rstd, dyb, sums, rows, part);
  else if (vec)
    hipLaunchKernelGGL((conv0_gn_bwd_kernel<4, 4, true>), grid, dim3(256), 0, stream, wave, w, p, gamma, beta, mask,
                       mean, rstd, dyb, sums, rows, part);
  else
    hipLaunchKernelGGL((conv0_gn_bwd_kernel<4, 4, false>), grid, dim3(256), 0, stream, wave, w, p, gamma, beta, mask,
                       mean, rstd, dyb, sums, rows, part);
  if (det)
    hipLaunchKernelGGL(conv0_part_reduce, dim3((unsigned)cdiv(B * C * NQ, 256)), dim3(256), 0, stream, part,
                       (int64_t)grid.x, C * NQ, B, sums);
  hipLaunchKernelGGL(conv0_bwd_finalize, dim3((unsigned)cdiv(C, 64)), dim3(64), 0, stream, sums, gram, w, mean, rstd,
                     p, dw, dgamma, dbeta, dmask);
  return check_launch("dph_conv0_gn_bwd");
}

static constexpr int64_t TAP_ROWS = 64;

static int tap_dot(const float* a, const float* b, int64_t R, int64_t K, float* out, float* ws, int64_t ws_bytes,
                   hipStream_t stream) {
  const int64_t nblk = cdiv(R, TAP_ROWS);
  DPH_REQUIRE(ws && ws_bytes >= nblk * K * 4, "weight norm: workspace too small (%lld bytes needed)",
              (long long)(nblk * K * 4));
  hipLaunchKernelGGL(tap_dot_partial_kernel, dim3((unsigned)nblk), dim3(256), 0, stream, a, b, R, K, ws, TAP_ROWS);
  hipLaunchKernelGGL(tap_dot_finalize_kernel, dim3((unsigned)K), dim3(256), 0, stream, ws, nblk, K, out);
  return DPH_OK;
}

extern "C" int dph_weight_norm_fwd(const float* g, const float* v, int64_t Cout, int64_t Cin_g, int64_t K, int64_t G,
                                   float* w, float* norm, void* wk, void* wt, float* ws, int64_t ws_bytes,
                                   hipStream_t stream) {
  DPH_REQUIRE(g && v && norm && Cout % G == 0 && K <= 4096, "dph_weight_norm_fwd: bad args");
  // norm holds the per-tap sum of squares until the final pass takes the sqrt
  float* nsq = norm;
  const int64_t R = Cout * Cin_g;
  int rc = tap_dot(v, v, R, K, nsq, ws, ws_bytes, stream);
  if (rc != DPH_OK) return rc;
  const int64_t n = Cout * Cin_g * K;
  // apply reads nsq; the norms are written in a separate, final pass (no read/write race)
  hipLaunchKernelGGL(weight_norm_apply_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, stream, g, v, nsq,
                     (float*)nullptr, Cout, Cin_g, K, G, w, reinterpret_cast<bf16_t*>(wk),
                     reinterpret_cast<bf16_t*>(wt));
  hipLaunchKernelGGL(weight_norm_apply_kernel, dim3((unsigned)cdiv(K, 256)), dim3(256), 0, stream, g, v, nsq, norm,
                     (int64_t)0, Cin_g, K, G, (float*)nullptr, (bf16_t*)nullptr, (bf16_t*)nullptr);
  return check_launch("dph_weight_norm_fwd");
}

extern "C" int dph_weight_norm_bwd(const float* dw_img, const float* g, const float* v, const float* norm,
                                   int64_t Cout, int64_t Cin_g, int64_t K, int64_t G, float* dg, float* dv, float* ws,
                                   int64_t ws_bytes, hipStream_t stream) {
  DPH_REQUIRE(dw_img && g && v && norm && dg && dv && Cout % G == 0, "dph_weight_norm_bwd: bad args");
  const int64_t n = Cout * Cin_g * K;
  // dv doubles as the [Cout][Cin][K] copy of dw, S (K floats) lives in dg until the final pass
  hipLaunchKernelGGL(img_to_weight_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, stream, dw_img, dv, Cout, Cin_g,
                     K, G);
  int rc = tap_dot(dv, v, Cout * Cin_g, K, dg, ws, ws_bytes, stream);
  if (rc != DPH_OK) return rc;
  // dv_out = (g/n) dw - g S/n^3 v  computed in place (each element reads only its own dv)
  hipLaunchKernelGGL(weight_norm_bwd_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, stream, dv, g, v, norm, dg,
                     n, K, (float*)nullptr, dv);
  // dg = S / n  (separate pass: S is read above)
  hipLaunchKernelGGL(weight_norm_bwd_kernel, dim3((unsigned)cdiv(K, 256)), dim3(256), 0, stream, dv, g, v, norm, dg,
                     (int64_t)0, K, dg, dv);
  return check_launch("dph_weight_norm_bwd");
}
