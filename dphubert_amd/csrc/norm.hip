// LayerNorm forward/backward over the last dim (one wave per row) and column
// sums (bias gradients).  fp32 statistics, bf16 storage.
//
// Reference call sites: nn.LayerNorm in FeatureProjection (components.py:271),
// EncoderLayer (:839,:850,:853,:856), Transformer._preprocess (:889) and the
// channel LayerNorm of layer_norm-mode extractors (:54-61).  torch semantics:
// biased variance, eps inside the sqrt.
#include "common.h"
#include <initializer_list>

namespace dph {
namespace {

constexpr int LN_MAXV = 4;   // up to 4 x (64 lanes x 4 elements) = 1024 columns
#ifndef DPH_LN_FWD_RPW
#define DPH_LN_FWD_RPW 2
#endif
#ifndef DPH_LN_BWD_RPW
#define DPH_LN_BWD_RPW 2
#endif
#ifndef DPH_LN_BWD_WAVES
#define DPH_LN_BWD_WAVES 8
#endif
constexpr int LN_FWD_RPW = DPH_LN_FWD_RPW;     // rows per wave, forward (all rows' loads issued before any math)
constexpr int LN_BWD_RPW = DPH_LN_BWD_RPW;     // rows per wave, backward
constexpr int LN_BWD_WAVES = DPH_LN_BWD_WAVES; // backward block: LN_BWD_WAVES x LN_BWD_RPW rows share one column reduction

__device__ __forceinline__ void unpack4(uint2 r, float (&o)[4]) {
  o[0] = __uint_as_float(r.x << 16);
  o[1] = __uint_as_float(r.x & 0xffff0000u);
  o[2] = __uint_as_float(r.y << 16);
  o[3] = __uint_as_float(r.y & 0xffff0000u);
}

// LayerNorm inputs are bf16, or fp32 for the layer_norm-mode conv layers (pre-LN conv outputs kept
// in fp32: 7 stacked bf16 roundings of the pre-LN values measured 1.02e-2 hidden rel-L2 vs the fp32
// reference, over the 1e-2 bar)
template <typename XT> struct XRaw;
template <> struct XRaw<bf16_t> { using T = uint2; };
template <> struct XRaw<float> { using T = float4; };
__device__ __forceinline__ uint2 ldx4(const bf16_t* p) { return *reinterpret_cast<const uint2*>(p); }
__device__ __forceinline__ float4 ldx4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void unpack4(float4 r, float (&o)[4]) {
  o[0] = r.x; o[1] = r.y; o[2] = r.z; o[3] = r.w;
}
// 4-element load / store of a bf16 or fp32 row segment (the pre-norm residual stream's gradient is fp32)
__device__ __forceinline__ void ld4(const bf16_t* p, float (&o)[4]) { unpack4(*reinterpret_cast<const uint2*>(p), o); }
__device__ __forceinline__ void ld4(const float* p, float (&o)[4]) { unpack4(*reinterpret_cast<const float4*>(p), o); }
__device__ __forceinline__ void st4(bf16_t* p, const float (&v)[4]) {
  *reinterpret_cast<uint2*>(p) = make_uint2(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]));
}
__device__ __forceinline__ void st4(float* p, const float (&v)[4]) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
}

// per-column vector (gamma / beta / scale) for the NV 4-column chunks a lane owns; 0 past D
template <int NV>
__device__ __forceinline__ void load_cols(const float* __restrict__ v, int D, int lane, float fill, float (&o)[NV][4]) {
#pragma unroll
  for (int c = 0; c < NV; ++c) {
    const int col = (c * 64 + lane) * 4;
    if (v && col + 4 <= D && (D & 3) == 0) {
      const float4 t = *reinterpret_cast<const float4*>(v + col);
      o[c][0] = t.x; o[c][1] = t.y; o[c][2] = t.z; o[c][3] = t.w;
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) o[c][i] = (col + i < D) ? (v ? v[col + i] : fill) : 0.f;
    }
  }
}

// Forward: one wave owns LN_FWD_RPW rows; gamma/beta live in registers, all row loads are issued
// first (latency of the HBM reads overlaps across rows), fp32 two-pass statistics in registers.
// Rows have stride ld >= D (ld % 4 == 0); columns [D, ld) are row padding: read as 0, written as 0.
// GM: also y2 = GELU(LN(x)) * gm_mask[c] from the fp32 normalised value (layer_norm-mode conv
// layers, components.py:54-61 + :110-114); y (the bf16 LN output, kept for the GELU backward) may be NULL.
template <int NV, bool GM = false, typename XT = bf16_t>
__global__ void __launch_bounds__(256) ln_fwd_kernel(const XT* __restrict__ x, const float* __restrict__ xscale,
                                                     const float* __restrict__ gamma, const float* __restrict__ beta,
                                                     bf16_t* __restrict__ y, float* __restrict__ mean_out,
                                                     float* __restrict__ rstd_out, int64_t rows, int D, int ld,
                                                     float eps, float drop_p, uint64_t seed,
                                                     const float* __restrict__ gm_mask = nullptr,
                                                     bf16_t* __restrict__ y2 = nullptr) {
  seed = epoch_seed(seed);   // per-step RNG epoch (graph replays)
  const int lane = threadIdx.x & 63;
  const int64_t r0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * LN_FWD_RPW;
  if (r0 >= rows) return;
  typename XRaw<XT>::T raw[LN_FWD_RPW][NV];
#pragma unroll
  for (int r = 0; r < LN_FWD_RPW; ++r)
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      const int col = (c * 64 + lane) * 4;
      raw[r][c] = (r0 + r < rows && col < D) ? ldx4(x + (r0 + r) * ld + col) : typename XRaw<XT>::T{};
    }
  float ga[NV][4], be[NV][4], xs[NV][4];
  load_cols<NV>(gamma, D, lane, 1.f, ga);
  load_cols<NV>(beta, D, lane, 0.f, be);
  load_cols<NV>(xscale, D, lane, 1.f, xs);
  const float inv_keep = drop_p > 0.f ? 1.f / (1.f - drop_p) : 1.f;
  const float invD = 1.0f / (float)D;
#pragma unroll
  for (int r = 0; r < LN_FWD_RPW; ++r) {
    const int64_t row = r0 + r;
    if (row >= rows) break;
    float v[NV][4];
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      const int col = (c * 64 + lane) * 4;
      unpack4(raw[r][c], v[c]);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[c][i] = (col + i < D) ? v[c][i] * xs[c][i] : 0.f;
        s += v[c][i];
      }
    }
    const float mean = wave_sum(s) * invD;
    float q = 0.f;
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      const int col = (c * 64 + lane) * 4;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float d = v[c][i] - mean;
        q += (col + i < D) ? d * d : 0.f;
      }
    }
    const float rstd = rsqrtf(wave_sum(q) * invD + eps);
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      const int col = (c * 64 + lane) * 4;
      if (col < ld) {
        float z[4];
        dropout_scale4(seed, (uint64_t)row * D + col, drop_p, inv_keep, z);
        float o[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = (col + i < D) ? ((v[c][i] - mean) * rstd * ga[c][i] + be[c][i]) * z[i] : 0.f;
        if (!GM || y) *reinterpret_cast<uint2*>(y + row * ld + col) = make_uint2(pack2bf(o[0], o[1]), pack2bf(o[2], o[3]));
        if constexpr (GM) {
          float g[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) g[i] = (col + i < D) ? gelu_f(o[i]) * (gm_mask ? gm_mask[col + i] : 1.f) : 0.f;
          *reinterpret_cast<uint2*>(y2 + row * ld + col) = make_uint2(pack2bf(g[0], g[1]), pack2bf(g[2], g[3]));
        }
      }
    }
    if (lane == 0) {
      mean_out[row] = mean;
      rstd_out[row] = rstd;
    }
  }
}

// Backward: 8 waves x LN_BWD_RPW rows per block, every row load issued before the math.  Per-column
// partials (dgamma, dbeta, branch column sums) are summed in registers over the wave's rows, then
// across the block's waves with LDS atomics, and written as one slab row per block; slab_reduce
// adds the columns into the outputs.  (One global atomic per column per block -- ~500 blocks onto
// the same 2304 addresses -- measured 0.09 TB/s: same-address atomics serialise at the memory side.)
// XT: the LN input's type; DT: dx / dx_add (fp32 for the pre-norm residual stream, components.py:846-850)
template <int NV, typename XT = bf16_t, typename DT = bf16_t>
__global__ void __launch_bounds__(64 * LN_BWD_WAVES) ln_bwd_kernel(
    const bf16_t* __restrict__ dy, const XT* __restrict__ x, const float* __restrict__ xscale,
    const float* __restrict__ gamma, const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
    DT* __restrict__ dx, float* __restrict__ dgamma, float* __restrict__ dbeta, int64_t rows, int D, int ld,
    float drop_p, uint64_t seed, bf16_t* __restrict__ branch, float branch_p, uint64_t branch_seed,
    const float* __restrict__ branch_smask, float* __restrict__ branch_colsum, const bf16_t* __restrict__ branch_pre,
    float* __restrict__ branch_sdot, const DT* __restrict__ dx_add, float* __restrict__ ws,
    float* __restrict__ sdot_part) {
  seed = epoch_seed(seed); branch_seed = epoch_seed(branch_seed);   // per-step RNG epoch (graph replays)
  __shared__ float4 red[LN_BWD_WAVES][NV * 64];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int64_t r0 = ((int64_t)blockIdx.x * LN_BWD_WAVES + wave) * LN_BWD_RPW;
  typename XRaw<XT>::T rx[LN_BWD_RPW][NV];
  uint2 rd[LN_BWD_RPW][NV];
#pragma unroll
  for (int r = 0; r < LN_BWD_RPW; ++r)
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      const int col = (c * 64 + lane) * 4;
      const bool ok = r0 + r < rows && col < D;
      rx[r][c] = ok ? ldx4(x + (r0 + r) * ld + col) : typename XRaw<XT>::T{};
      rd[r][c] = ok ? *reinterpret_cast<const uint2*>(dy + (r0 + r) * ld + col) : make_uint2(0, 0);
    }
  float ga[NV][4], xs[NV][4];
  load_cols<NV>(gamma, D, lane, 1.f, ga);
  load_cols<NV>(xscale, D, lane, 1.f, xs);
  const float inv_keep = drop_p > 0.f ? 1.f / (1.f - drop_p) : 1.f;
  const float binv_keep = branch_p > 0.f ? 1.f / (1.f - branch_p) : 1.f;
  const float bsm = branch_smask ? *branch_smask : 1.0f;
  const float invD = 1.0f / (float)D;
  float pg[NV][4], pb[NV][4], pc[NV][4];
#pragma unroll
  for (int c = 0; c < NV; ++c)
#pragma unroll
    for (int i = 0; i < 4; ++i) pg[c][i] = pb[c][i] = pc[c][i] = 0.f;
  float sdot = 0.f;
#pragma unroll
  for (int r = 0; r < LN_BWD_RPW; ++r) {
    const int64_t row = r0 + r;
    if (row >= rows) break;
    const float mean = mean_in[row];
    const float rstd = rstd_in[row];
    float xh[NV][4], g[NV][4], dyv[NV][4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      const int col = (c * 64 + lane) * 4;
      float xv[4], dv[4], z[4];
      unpack4(rx[r][c], xv);
      unpack4(rd[r][c], dv);
      dropout_scale4(seed, (uint64_t)row * D + col, drop_p, inv_keep, z);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bool ok = col + i < D;
        xh[c][i] = ok ? (xv[i] * xs[c][i] - mean) * rstd : 0.f;
        dyv[c][i] = ok ? dv[i] * z[i] : 0.f;
        g[c][i] = dyv[c][i] * ga[c][i];
        s1 += g[c][i];
        s2 += g[c][i] * xh[c][i];
        pg[c][i] += dyv[c][i] * xh[c][i];
        pb[c][i] += dyv[c][i];
      }
    }
    s1 = wave_sum(s1) * invD;
    s2 = wave_sum(s2) * invD;
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      const int col = (c * 64 + lane) * 4;
      if (col >= ld) continue;
      float o[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] = (col + i < D) ? rstd * (g[c][i] - s1 - xh[c][i] * s2) * xs[c][i] : 0.f;
      if (dx_add) {
        // other gradient paths into the LN input (pre-norm residual); the branch output below
        // stays the LN-path gradient only
        float ad[4];
        ld4(dx_add + row * ld + col, ad);
        const float s[4] = {o[0] + ad[0], o[1] + ad[1], o[2] + ad[2], o[3] + ad[3]};
        st4(dx + row * ld + col, s);
      } else {
        st4(dx + row * ld + col, o);
      }
      if (branch) {
        float pre[4] = {0.f, 0.f, 0.f, 0.f}, z[4], bo[4];
        if (branch_sdot) unpack4(*reinterpret_cast<const uint2*>(branch_pre + row * ld + col), pre);
        dropout_scale4(branch_seed, (uint64_t)row * D + col, branch_p, binv_keep, z);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float zz = (col + i < D) ? o[i] * z[i] : 0.f;
          sdot += zz * pre[i];
          bo[i] = zz * bsm;
          pc[c][i] += bo[i];
        }
        *reinterpret_cast<uint2*>(branch + row * ld + col) = make_uint2(pack2bf(bo[0], bo[1]), pack2bf(bo[2], bo[3]));
      }
    }
  }
  // cross-wave column reduction, one quantity at a time: plain float4 LDS stores of every wave's
  // partials, then each thread sums the 8 waves for its column quads and writes the block's slab
  // row ws[block][3][D] (LDS float atomics with the 16-B lane stride ran 4-way bank-conflicted:
  // +35 us per launch)
  float* wrow = ws + (int64_t)blockIdx.x * 3 * D;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const bool want = q == 0 ? dgamma != nullptr : (q == 1 ? dbeta != nullptr : branch_colsum != nullptr);
    if (!want) continue;
    __syncthreads();
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      const float(&pq)[NV][4] = q == 0 ? pg : (q == 1 ? pb : pc);
      red[wave][c * 64 + lane] = make_float4(pq[c][0], pq[c][1], pq[c][2], pq[c][3]);
    }
    __syncthreads();
    for (int j = threadIdx.x; j < NV * 64; j += 64 * LN_BWD_WAVES) {
      float4 t = red[0][j];
#pragma unroll
      for (int w = 1; w < LN_BWD_WAVES; ++w) {
        const float4 u = red[w][j];
        t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
      }
      const int col = j * 4;
      const float tv[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (col + i < D) wrow[q * D + col + i] = tv[i];
    }
  }
  if (branch_sdot) {
    // one same-address atomic per BLOCK (per wave: 66 us for a 7984 x 768 launch, profiles/r4_s28_ln_ab.txt)
    __shared__ float sdot_s[16];
    sdot = wave_sum(sdot);
    if (lane == 0) sdot_s[wave] = sdot;
    __syncthreads();
    if (threadIdx.x == 0) {
      float t = 0.f;
      for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += sdot_s[w];
      // deterministic mode: the block's partial, summed in block order by sdot_reduce_kernel
      if (sdot_part) sdot_part[blockIdx.x] = t;
      else atomicAdd(branch_sdot, t);
    }
  }
}

// Per-utterance waveform LayerNorm (model.py:96-103, wav2vec2-Large normalize_waveform): each
// row's first len samples -> (x - mean) * rsqrt(var + eps) (no affine, biased variance), the
// rest -> 0.  One 1024-thread block per utterance; fp64 sums (S = 160 000 samples).
__global__ void __launch_bounds__(1024) wave_norm_kernel(const float* __restrict__ x,
                                                         const int64_t* __restrict__ lengths, int64_t S, float eps,
                                                         float* __restrict__ y) {
  __shared__ double red[2][16];
  const int64_t b = blockIdx.x;
  const int64_t L = lengths ? min<int64_t>(max<int64_t>(lengths[b], 0), S) : S;
  const float* xr = x + b * S;
  double s1 = 0.0, s2 = 0.0;
  for (int64_t i = threadIdx.x; i < L; i += blockDim.x) {
    const double v = xr[i];
    s1 += v;
    s2 += v * v;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s1 += __shfl_xor(s1, o, 64);
    s2 += __shfl_xor(s2, o, 64);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][w] = s1;
    red[1][w] = s2;
  }
  __syncthreads();
  double t1 = 0.0, t2 = 0.0;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) {
    t1 += red[0][i];
    t2 += red[1][i];
  }
  const double n = L > 0 ? (double)L : 1.0;
  const double mean = t1 / n;
  const double var = max(t2 / n - mean * mean, 0.0);
  const float m = (float)mean;
  const float r = (float)(1.0 / sqrt(var + (double)eps));
  float* yr = y + b * S;
  for (int64_t i = threadIdx.x; i < S; i += blockDim.x) yr[i] = i < L ? (xr[i] - m) * r : 0.f;
}

// column partial sums of x [rows][cols] bf16: block (blockIdx.x: 512-column chunk, blockIdx.y: range of
// rows_per_block rows) = 64 x 4 threads, 8 columns per thread -> ws[blockIdx.y][cols].  ld: x's row stride;
// logical column c reads physical column c + (c >= skip0 ? skipn : 0) (dph_colsum3 without its middle segment:
// the q / v bias gradients read 2/3 of the fused dqkv rows, skip0 and skipn multiples of 8)
__global__ void __launch_bounds__(256) colsum_kernel(const bf16_t* __restrict__ x, float* __restrict__ ws,
                                                     int64_t rows, int64_t cols, int64_t rows_per_block, int64_t ld,
                                                     int64_t skip0, int64_t skipn) {
  __shared__ float red[4][512];
  const int tx = threadIdx.x & 63;
  const int ty = threadIdx.x >> 6;
  const int64_t c0 = (int64_t)blockIdx.x * 512 + tx * 8;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_block;
  const int64_t r1 = min(rows, r0 + rows_per_block);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const bool vec = (c0 + 8 <= cols) && (cols % 8 == 0) && (ld % 8 == 0);
  const int64_t pc0 = c0 + (c0 >= skip0 ? skipn : 0);
#pragma unroll 4
  for (int64_t r = r0 + ty; r < r1; r += 4) {
    const bf16_t* p = x + r * ld + pc0;
    if (vec) {
      uint4 raw = *reinterpret_cast<const uint4*>(p);
      uint32_t w[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        acc[2 * i] += __uint_as_float(w[i] << 16);
        acc[2 * i + 1] += __uint_as_float(w[i] & 0xffff0000u);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (c0 + i < cols) acc[i] += bf2f(p[i]);
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) red[ty][tx * 8 + i] = acc[i];
  __syncthreads();
  for (int c = threadIdx.x; c < 512; c += 256) {
    const int64_t col = (int64_t)blockIdx.x * 512 + c;
    if (col < cols) ws[(int64_t)blockIdx.y * cols + col] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
  }
}

// out[n] += s(n) * sum_r a[r][n] * b[r][n] (dph_colprod): block = 64 x 4 threads, 8 columns per thread over a
// range of rows, the 4 row phases summed in LDS, one atomic per column per block
__global__ void __launch_bounds__(256) colprod_kernel(const bf16_t* __restrict__ a, int64_t lda,
                                                      const float* __restrict__ b, int64_t ldb,
                                                      const float* __restrict__ colmask, float* __restrict__ out,
                                                      int64_t R, int64_t N, int64_t rows_per_block) {
  __shared__ float red[4][512];
  const int tx = threadIdx.x & 63;
  const int ty = threadIdx.x >> 6;
  const int64_t c0 = (int64_t)blockIdx.x * 512 + tx * 8;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_block;
  const int64_t r1 = min(R, r0 + rows_per_block);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const bool vec = c0 + 8 <= N && (lda % 8) == 0 && (ldb % 4) == 0;
  for (int64_t r = r0 + ty; r < r1; r += 4) {
    const bf16_t* pa = a + r * lda + c0;
    const float* pb = b + r * ldb + c0;
    if (vec) {
      const uint4 ra = *reinterpret_cast<const uint4*>(pa);
      const float4 b0 = *reinterpret_cast<const float4*>(pb);
      const float4 b1 = *reinterpret_cast<const float4*>(pb + 4);
      const uint32_t w[4] = {ra.x, ra.y, ra.z, ra.w};
      const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        acc[2 * i] = fmaf(__uint_as_float(w[i] << 16), bv[2 * i], acc[2 * i]);
        acc[2 * i + 1] = fmaf(__uint_as_float(w[i] & 0xffff0000u), bv[2 * i + 1], acc[2 * i + 1]);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (c0 + i < N) acc[i] = fmaf(bf2f(pa[i]), pb[i], acc[i]);
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) red[ty][tx * 8 + i] = acc[i];
  __syncthreads();
  for (int c = threadIdx.x; c < 512; c += 256) {
    const int64_t col = (int64_t)blockIdx.x * 512 + c;
    if (col >= N) continue;
    float sc = 1.f;
    if (colmask) {
      const float m = colmask[col];
      sc = m != 0.f ? 1.0f / m : 0.f;
    }
    atomicAdd(out + col, sc * (red[0][c] + red[1][c] + red[2][c] + red[3][c]));
  }
}

// deterministic mode: the same contraction with every column's rows in a fixed order, one block per 32 columns (thread
// (column, phase) takes rows phase, phase + DET_PH, ... in four chains, the phases added in order; no atomics)
__global__ void __launch_bounds__(32 * DET_PH) colprod_det_kernel(const bf16_t* __restrict__ a, int64_t lda,
                                                                  const float* __restrict__ b, int64_t ldb,
                                                                  const float* __restrict__ colmask,
                                                                  float* __restrict__ out, int64_t R, int64_t N) {
  __shared__ float red[DET_PH][33];
  const int tx = threadIdx.x & 31, ph = threadIdx.x >> 5;
  const int64_t col = (int64_t)blockIdx.x * 32 + tx;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (col < N) {
    int64_t r = ph;
    for (; r + 3 * DET_PH < R; r += 4 * DET_PH) {
      s0 = fmaf(bf2f(a[r * lda + col]), b[r * ldb + col], s0);
      s1 = fmaf(bf2f(a[(r + DET_PH) * lda + col]), b[(r + DET_PH) * ldb + col], s1);
      s2 = fmaf(bf2f(a[(r + 2 * DET_PH) * lda + col]), b[(r + 2 * DET_PH) * ldb + col], s2);
      s3 = fmaf(bf2f(a[(r + 3 * DET_PH) * lda + col]), b[(r + 3 * DET_PH) * ldb + col], s3);
    }
    if (r < R) s0 = fmaf(bf2f(a[r * lda + col]), b[r * ldb + col], s0);
    if (r + DET_PH < R) s1 = fmaf(bf2f(a[(r + DET_PH) * lda + col]), b[(r + DET_PH) * ldb + col], s1);
    if (r + 2 * DET_PH < R) s2 = fmaf(bf2f(a[(r + 2 * DET_PH) * lda + col]), b[(r + 2 * DET_PH) * ldb + col], s2);
  }
  red[ph][tx] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (ph == 0 && col < N) {
    float t = 0.f;
#pragma unroll 8
    for (int i = 0; i < DET_PH; ++i) t += red[i][tx];
    float sc = 1.f;
    if (colmask) {
      const float m = colmask[col];
      sc = m != 0.f ? 1.0f / m : 0.f;
    }
    out[col] += sc * t;
  }
}

// out_q[c] += sum_r ws[r][q * seg + c] for the (up to 3) column segments q of width seg (null outputs
// skipped).  Block = 64 columns x 4 row phases over one of gridDim.y row groups; one atomic per column
// per group (a handful of adders per address).
__global__ void __launch_bounds__(256) slab_reduce_kernel(const float* __restrict__ ws, int64_t nrows, int64_t ncols,
                                                          int64_t seg, float* __restrict__ o0, float* __restrict__ o1,
                                                          float* __restrict__ o2) {
  __shared__ float red[4][64];
  const int tx = threadIdx.x & 63;
  const int ty = threadIdx.x >> 6;
  const int64_t col = (int64_t)blockIdx.x * 64 + tx;
  const int64_t per = cdiv(nrows, (int64_t)gridDim.y);
  const int64_t ra = (int64_t)blockIdx.y * per;
  const int64_t rb = min(nrows, ra + per);
  const int q = col < ncols ? (int)(col / seg) : 0;
  float* out = q == 0 ? o0 : (q == 1 ? o1 : o2);
  float s = 0.f;
  if (col < ncols && out) {
    int64_t r = ra + ty;
    float s1 = 0.f, s2 = 0.f, s3 = 0.f;
    for (; r + 12 < rb; r += 16) {
      s += ws[r * ncols + col];
      s1 += ws[(r + 4) * ncols + col];
      s2 += ws[(r + 8) * ncols + col];
      s3 += ws[(r + 12) * ncols + col];
    }
    for (; r < rb; r += 4) s += ws[r * ncols + col];
    s += (s1 + s2) + s3;
  }
  red[ty][tx] = s;
  __syncthreads();
  if (ty == 0 && col < ncols && out) atomicAdd(out + (col - (int64_t)q * seg), red[0][tx] + red[1][tx] + red[2][tx] + red[3][tx]);
}

// row groups of a slab reduction: >= 32 rows (8 per thread phase) per group, up to 32 groups (one atomic per column
// per group)
int64_t slab_groups(int64_t nrows) { return std::max<int64_t>(1, std::min<int64_t>(32, cdiv(nrows, 32))); }

// deterministic mode: the same sums with every column's rows added in a fixed order by one block (32 columns each)
__global__ void __launch_bounds__(32 * DET_PH) slab_reduce_det_kernel(const float* __restrict__ ws, int64_t nrows,
                                                                      int64_t ncols, int64_t seg, float* __restrict__ o0,
                                                                      float* __restrict__ o1, float* __restrict__ o2) {
  __shared__ float red[DET_PH][33];
  const int64_t col = (int64_t)blockIdx.x * 32 + (threadIdx.x & 31);
  const int q = col < ncols ? (int)(col / seg) : 0;
  float* out = q == 0 ? o0 : (q == 1 ? o1 : o2);
  const bool live = col < ncols && out != nullptr;
  const float t = det_column_total(live ? ws + col : nullptr, nrows, ncols, red);
  if ((threadIdx.x >> 5) == 0 && live) out[col - (int64_t)q * seg] += t;
}

// out[0] += sum of n per-block partials, in block order (one wave)
__global__ void __launch_bounds__(64) sdot_reduce_kernel(const float* __restrict__ part, int64_t n,
                                                         float* __restrict__ out) {
  const float s = sum_partials_wave(part, n, 1);
  if (threadIdx.x == 0) out[0] += s;
}

int slab_reduce_launch(const float* ws, int64_t nrows, int64_t ncols, int64_t seg, float* o0, float* o1, float* o2,
                       hipStream_t stream) {
  if (colred_deferring()) {
    float* outs[3] = {o0, o1, o2};
    for (int q = 0; q < 3 && q * seg < ncols; ++q) {
      const int rc = colred_push(ws + q * seg, nrows, ncols, std::min<int64_t>(seg, ncols - q * seg), outs[q], stream);
      if (rc != DPH_OK) return rc;
    }
    return DPH_OK;
  }
  if (deterministic())
    hipLaunchKernelGGL(slab_reduce_det_kernel, dim3((unsigned)cdiv(ncols, 32)), dim3(32 * DET_PH), 0, stream, ws,
                       nrows, ncols, seg, o0, o1, o2);
  else
    hipLaunchKernelGGL(slab_reduce_kernel, dim3((unsigned)cdiv(ncols, 64), (unsigned)slab_groups(nrows)), dim3(256), 0,
                       stream, ws, nrows, ncols, seg, o0, o1, o2);
  return DPH_OK;
}

int64_t colsum_rpb(int64_t rows) { return std::max<int64_t>(64, cdiv(cdiv(rows, 8192), 4) * 4); }

// Forward, the common case (bf16 rows of D = 256 * k <= 1024 with no row padding, no input scale, no dropout --
// every post-norm encoder LayerNorm, components.py:853,856): a HALF wave per row, 16-byte loads and stores
// (NE = D / 32 elements per lane: NE / 8 vector accesses), sums over the 32 lanes of the half.  Half the memory
// instructions of ln_fwd_kernel's 8-byte quads; otherwise the same fp32 two-pass statistics per row.
__device__ __forceinline__ void ld8(const bf16_t* p, float (&o)[8]) {
  const uint4 r = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    o[2 * i] = __uint_as_float(w[i] << 16);
    o[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ void ld8(const float* p, float (&o)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w;
  o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}
__device__ __forceinline__ void st8(bf16_t* p, const float (&o)[8]) {
  *reinterpret_cast<uint4*>(p) =
      make_uint4(pack2bf(o[0], o[1]), pack2bf(o[2], o[3]), pack2bf(o[4], o[5]), pack2bf(o[6], o[7]));
}
__device__ __forceinline__ void st8(float* p, const float (&o)[8]) {
  *reinterpret_cast<float4*>(p) = make_float4(o[0], o[1], o[2], o[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(o[4], o[5], o[6], o[7]);
}

// Forward, the common case (rows of D = 256 * k <= 1024 with no row padding, no input scale, no dropout -- every
// post-norm encoder LayerNorm, components.py:853,856, with bf16 x, and the pre-norm layers' LN1 / LN2 over the fp32
// residual stream, components.py:846-850): a HALF wave per row, 16-byte loads and stores (NE = D / 32 elements per
// lane: NE / 8 vector accesses of bf16, twice that of fp32), sums over the 32 lanes of the half.  Half the memory
// instructions of ln_fwd_kernel's 8-byte quads; otherwise the same fp32 two-pass statistics per row.
template <int NE, typename XT = bf16_t>
__global__ void __launch_bounds__(256) ln_fwd16_kernel(const XT* __restrict__ x, const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, bf16_t* __restrict__ y,
                                                       float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                       int64_t rows, float eps) {
  constexpr int NC = NE / 8;                 // 8-element chunks per lane
  constexpr int D = NE * 32;
  const int lane = threadIdx.x & 63;
  const int hl = lane & 31;
  const int64_t row = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 2 + (lane >> 5);
  const bool ok = row < rows;
  float v[NC][8];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    if (ok) {
      ld8(x + row * D + (c * 32 + hl) * 8, v[c]);
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) v[c][i] = 0.f;
    }
  }
  // gamma / beta issued with the row loads (after the statistics they were one more dependent load latency of a
  // one-round grid)
  float4 gb[NC][4];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int col = (c * 32 + hl) * 8;
    gb[c][0] = *reinterpret_cast<const float4*>(gamma + col);
    gb[c][1] = *reinterpret_cast<const float4*>(gamma + col + 4);
    gb[c][2] = *reinterpret_cast<const float4*>(beta + col);
    gb[c][3] = *reinterpret_cast<const float4*>(beta + col + 4);
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int i = 0; i < 8; ++i) s += v[c][i];
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  const float mean = s * (1.0f / (float)D);
  float q = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float d = v[c][i] - mean;
      q += d * d;
    }
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
  const float rstd = rsqrtf(q * (1.0f / (float)D) + eps);
  if (!ok) return;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int col = (c * 32 + hl) * 8;
    const float4 g0 = gb[c][0], g1 = gb[c][1], b0 = gb[c][2], b1 = gb[c][3];
    const float ga[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
    const float be[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
    float o[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (v[c][i] - mean) * rstd * ga[i] + be[i];
    st8(y + row * D + col, o);
  }
  if (hl == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// Backward, the common case (bf16 dy of D = 256 * k <= 1024, no row padding, no input scale, no dropout on the LN
// input): the post-norm layers (bf16 x / dx; the branch gradient -- dropout, layer mask, its column sums and
// mask-gradient dot -- as ln_bwd_kernel) and the pre-norm layers (fp32 x / dx / dx_add, the residual stream,
// components.py:846-850): a HALF wave per row with 16-byte accesses, 8 waves x 2 rows per block and the same
// per-block slab row ws[block][3][D] for slab_reduce.  The two halves of a wave (two rows, same columns) combine
// their column partials with one lane ^ 32 exchange before the cross-wave LDS sum.
template <int NE, typename XT = bf16_t, typename DT = bf16_t>
__global__ void __launch_bounds__(512, 4) ln_bwd16_kernel(
    const bf16_t* __restrict__ dy, const XT* __restrict__ x, const float* __restrict__ gamma,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in, DT* __restrict__ dx,
    float* __restrict__ dgamma, float* __restrict__ dbeta, int64_t rows, bf16_t* __restrict__ branch, float branch_p,
    uint64_t branch_seed, const float* __restrict__ branch_smask, float* __restrict__ branch_colsum,
    const bf16_t* __restrict__ branch_pre, float* __restrict__ branch_sdot, const DT* __restrict__ dx_add,
    float* __restrict__ ws, float* __restrict__ sdot_part) {
  constexpr int NC = NE / 8;
  constexpr int D = NE * 32;
  static_assert(LN_BWD_WAVES == 8 && LN_BWD_RPW == 2, "ln_bwd16: the slab layout assumes 16 rows per block");
  branch_seed = epoch_seed(branch_seed);
  __shared__ float4 red[3][8][NC * 32][2];
  const int lane = threadIdx.x & 63;
  const int hl = lane & 31;
  const int wave = threadIdx.x >> 6;
  const int64_t row = ((int64_t)blockIdx.x * 8 + wave) * 2 + (lane >> 5);
  const bool ok = row < rows;
  float xh[NC][8], g[NC][8], dyv[NC][8], ga[NC][8];
  const float mean = ok ? mean_in[row] : 0.f;
  const float rstd = ok ? rstd_in[row] : 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int64_t off = row * D + (c * 32 + hl) * 8;
    if (ok) {
      ld8(x + off, xh[c]);
      ld8(dy + off, dyv[c]);
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) xh[c][i] = dyv[c][i] = 0.f;
    }
  }
  float4 gq[NC][2];   // gamma, issued with the row loads
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int col = (c * 32 + hl) * 8;
    gq[c][0] = *reinterpret_cast<const float4*>(gamma + col);
    gq[c][1] = *reinterpret_cast<const float4*>(gamma + col + 4);
  }
  // the branch's pre-mask output (layer-mask gradient dot), also issued with the row loads: read after the dx
  // stores it was a second dependent HBM round trip per row
  // (post-norm bf16 rows only: the fp32 residual-stream variants have no registers to spare)
  constexpr bool EARLY_PRE = std::is_same<XT, bf16_t>::value && std::is_same<DT, bf16_t>::value;
  uint4 prer[NC];
  const bool want_pre = branch != nullptr && branch_sdot != nullptr && ok;
#pragma unroll
  for (int c = 0; c < NC; ++c)
    prer[c] = (EARLY_PRE && want_pre) ? *reinterpret_cast<const uint4*>(branch_pre + row * D + (c * 32 + hl) * 8)
                                      : make_uint4(0u, 0u, 0u, 0u);
  const float binv_keep = branch_p > 0.f ? 1.f / (1.f - branch_p) : 1.f;
  const float bsm = branch_smask ? *branch_smask : 1.0f;
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const float4 g0 = gq[c][0], g1 = gq[c][1];
    ga[c][0] = g0.x; ga[c][1] = g0.y; ga[c][2] = g0.z; ga[c][3] = g0.w;
    ga[c][4] = g1.x; ga[c][5] = g1.y; ga[c][6] = g1.z; ga[c][7] = g1.w;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      xh[c][i] = (xh[c][i] - mean) * rstd;
      g[c][i] = dyv[c][i] * ga[c][i];
      s1 += g[c][i];
      s2 += g[c][i] * xh[c][i];
    }
  }
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) {
    s1 += __shfl_xor(s1, o, 64);
    s2 += __shfl_xor(s2, o, 64);
  }
  s1 *= 1.0f / (float)D;
  s2 *= 1.0f / (float)D;
  float sdot = 0.f;
  float pc[NC][8];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int col = (c * 32 + hl) * 8;
    float o[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = rstd * (g[c][i] - s1 - xh[c][i] * s2);
    if (ok) {
      if (dx_add) {
        // other gradient paths into the LN input (pre-norm residual); the branch below stays the LN-path gradient
        float ad[8], sm[8];
        ld8(dx_add + row * D + col, ad);
#pragma unroll
        for (int i = 0; i < 8; ++i) sm[i] = o[i] + ad[i];
        st8(dx + row * D + col, sm);
      } else {
        st8(dx + row * D + col, o);
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) pc[c][i] = 0.f;
    if (branch) {
      float pre[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, z[8], bo[8];
      if (branch_sdot && ok) {
        const uint4 rp = EARLY_PRE ? prer[c] : *reinterpret_cast<const uint4*>(branch_pre + row * D + col);
        const uint32_t wp[4] = {rp.x, rp.y, rp.z, rp.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          pre[2 * i] = __uint_as_float(wp[i] << 16);
          pre[2 * i + 1] = __uint_as_float(wp[i] & 0xffff0000u);
        }
      }
      float z0[4], z1[4];
      dropout_scale4(branch_seed, (uint64_t)row * D + col, branch_p, binv_keep, z0);
      dropout_scale4(branch_seed, (uint64_t)row * D + col + 4, branch_p, binv_keep, z1);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        z[i] = z0[i];
        z[4 + i] = z1[i];
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float zz = ok ? o[i] * z[i] : 0.f;
        sdot += zz * pre[i];
        bo[i] = zz * bsm;
        pc[c][i] = bo[i];
      }
      if (ok)
        *reinterpret_cast<uint4*>(branch + row * D + col) =
            make_uint4(pack2bf(bo[0], bo[1]), pack2bf(bo[2], bo[3]), pack2bf(bo[4], bo[5]), pack2bf(bo[6], bo[7]));
    }
  }
  // column partials of this row: dgamma = dy * xh, dbeta = dy, branch colsum = bo (rows past `rows` are zero), all
  // three staged in ONE LDS pass (one pair of barriers instead of three)
  float* wrow = ws + (int64_t)blockIdx.x * 3 * D;
  const bool want[3] = {dgamma != nullptr, dbeta != nullptr, branch_colsum != nullptr};
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    if (!want[q]) continue;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      float t[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float vq = q == 0 ? (ok ? dyv[c][i] * xh[c][i] : 0.f) : (q == 1 ? (ok ? dyv[c][i] : 0.f) : pc[c][i]);
        t[i] = vq + __shfl_xor(vq, 32, 64);
      }
      if (lane < 32) {
        red[q][wave][c * 32 + hl][0] = make_float4(t[0], t[1], t[2], t[3]);
        red[q][wave][c * 32 + hl][1] = make_float4(t[4], t[5], t[6], t[7]);
      }
    }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < 3 * NC * 32 * 2; j += 512) {
    const int q = j / (NC * 32 * 2), jj = j % (NC * 32 * 2);
    if (!want[q]) continue;
    const int cj = jj >> 1, hh = jj & 1;
    float4 acc = red[q][0][cj][hh];
#pragma unroll
    for (int w = 1; w < 8; ++w) {
      const float4 u = red[q][w][cj][hh];
      acc.x += u.x; acc.y += u.y; acc.z += u.z; acc.w += u.w;
    }
    // (cj = c * 32 + hl owns columns (c * 32 + hl) * 8 .. + 7; hh picks the half)
    *reinterpret_cast<float4*>(wrow + q * D + cj * 8 + hh * 4) = acc;
  }
  if (branch_sdot) {
    // one same-address atomic per BLOCK (per wave: 66 us for a 7984 x 768 launch, profiles/r4_s28_ln_ab.txt)
    __shared__ float sdot_s[16];
    sdot = wave_sum(sdot);
    if (lane == 0) sdot_s[wave] = sdot;
    __syncthreads();
    if (threadIdx.x == 0) {
      float t = 0.f;
      for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += sdot_s[w];
      // deterministic mode: the block's partial, summed in block order by sdot_reduce_kernel
      if (sdot_part) sdot_part[blockIdx.x] = t;
      else atomicAdd(branch_sdot, t);
    }
  }
}

}  // namespace

// (shared with the other translation units: common.h)
int slab_reduce_cols(const float* ws, int64_t nrows, int64_t ncols, int64_t seg, float* o0, float* o1, float* o2,
                     hipStream_t stream) {
  return slab_reduce_launch(ws, nrows, ncols, seg, o0, o1, o2, stream);
}
void sdot_reduce(const float* part, int64_t n, float* out, hipStream_t stream) {
  hipLaunchKernelGGL(sdot_reduce_kernel, dim3(1), dim3(64), 0, stream, part, n, out);
}
}  // namespace dph

using namespace dph;

extern "C" int dph_layernorm_fwd_ld(const void* x, const float* xscale, const float* gamma, const float* beta,
                                    void* y, float* mean, float* rstd, int64_t rows, int64_t D, int64_t ld, float eps,
                                    float dropout_p, uint64_t seed, hipStream_t stream) {
  DPH_REQUIRE(x && gamma && beta && y && mean && rstd, "dph_layernorm_fwd: null pointer");
  if (ld == 0) ld = D;
  DPH_REQUIRE(D >= 1 && ld >= D && ld % 4 == 0 && ld <= LN_MAXV * 256 && rows > 0,
              "dph_layernorm_fwd: unsupported D=%lld ld=%lld", (long long)D, (long long)ld);
  static const bool ln16 = [] {
    const char* e = getenv("DPH_LN_FWD16");
    return !(e && e[0] == '0');
  }();
  if (ln16 && !xscale && dropout_p <= 0.f && ld == D && D % 256 == 0 && D <= 1024 &&
      (reinterpret_cast<uintptr_t>(x) & 15) == 0 && (reinterpret_cast<uintptr_t>(y) & 15) == 0 &&
      (reinterpret_cast<uintptr_t>(gamma) & 15) == 0 && (reinterpret_cast<uintptr_t>(beta) & 15) == 0) {
    const dim3 g16((unsigned)cdiv(rows, 8));
    const bf16_t* xb = reinterpret_cast<const bf16_t*>(x);
    bf16_t* yb = reinterpret_cast<bf16_t*>(y);
    switch (D / 256) {
      case 1: hipLaunchKernelGGL(ln_fwd16_kernel<8>, g16, dim3(256), 0, stream, xb, gamma, beta, yb, mean, rstd, rows, eps); break;
      case 2: hipLaunchKernelGGL(ln_fwd16_kernel<16>, g16, dim3(256), 0, stream, xb, gamma, beta, yb, mean, rstd, rows, eps); break;
      case 3: hipLaunchKernelGGL(ln_fwd16_kernel<24>, g16, dim3(256), 0, stream, xb, gamma, beta, yb, mean, rstd, rows, eps); break;
      default: hipLaunchKernelGGL(ln_fwd16_kernel<32>, g16, dim3(256), 0, stream, xb, gamma, beta, yb, mean, rstd, rows, eps); break;
    }
    return check_launch("dph_layernorm_fwd");
  }
  const dim3 grid((unsigned)cdiv(rows, 4 * LN_FWD_RPW));
#define LN_FWD_LAUNCH(NV)                                                                                    \
  hipLaunchKernelGGL(ln_fwd_kernel<NV>, grid, dim3(256), 0, stream, reinterpret_cast<const bf16_t*>(x), xscale, \
                     gamma, beta, reinterpret_cast<bf16_t*>(y), mean, rstd, rows, (int)D, (int)ld, eps, dropout_p, seed)
  switch (cdiv(ld, 256)) {
    case 1: LN_FWD_LAUNCH(1); break;
    case 2: LN_FWD_LAUNCH(2); break;
    case 3: LN_FWD_LAUNCH(3); break;
    default: LN_FWD_LAUNCH(4); break;
  }
#undef LN_FWD_LAUNCH
  return check_launch("dph_layernorm_fwd");
}

extern "C" int dph_layernorm_gelu_fwd(const void* x, int x_f32, const float* gamma, const float* beta, void* h,
                                      const float* mask, void* y, float* mean, float* rstd, int64_t rows, int64_t D,
                                      float eps, hipStream_t stream) {
  DPH_REQUIRE(x && gamma && beta && y && mean && rstd, "dph_layernorm_gelu_fwd: null pointer");
  DPH_REQUIRE(D >= 1 && D % 4 == 0 && D <= LN_MAXV * 256 && rows > 0, "dph_layernorm_gelu_fwd: unsupported D=%lld",
              (long long)D);
  const dim3 grid((unsigned)cdiv(rows, 4 * LN_FWD_RPW));
#define LNG_LAUNCH(NV)                                                                                           \
  if (x_f32)                                                                                                     \
    hipLaunchKernelGGL((ln_fwd_kernel<NV, true, float>), grid, dim3(256), 0, stream,                              \
                       reinterpret_cast<const float*>(x), (const float*)nullptr, gamma, beta,                      \
                       reinterpret_cast<bf16_t*>(h), mean, rstd, rows, (int)D, (int)D, eps, 0.f, (uint64_t)0, mask, \
                       reinterpret_cast<bf16_t*>(y));                                                             \
  else                                                                                                           \
    hipLaunchKernelGGL((ln_fwd_kernel<NV, true>), grid, dim3(256), 0, stream, reinterpret_cast<const bf16_t*>(x), \
                       (const float*)nullptr, gamma, beta, reinterpret_cast<bf16_t*>(h), mean, rstd, rows, (int)D, \
                       (int)D, eps, 0.f, (uint64_t)0, mask, reinterpret_cast<bf16_t*>(y))
  switch (cdiv(D, 256)) {
    case 1: LNG_LAUNCH(1); break;
    case 2: LNG_LAUNCH(2); break;
    case 3: LNG_LAUNCH(3); break;
    default: LNG_LAUNCH(4); break;
  }
#undef LNG_LAUNCH
  return check_launch("dph_layernorm_gelu_fwd");
}

extern "C" int dph_layernorm_fwd(const void* x, const float* xscale, const float* gamma, const float* beta, void* y,
                                 float* mean, float* rstd, int64_t rows, int64_t D, float eps, float dropout_p,
                                 uint64_t seed, hipStream_t stream) {
  return dph_layernorm_fwd_ld(x, xscale, gamma, beta, y, mean, rstd, rows, D, D, eps, dropout_p, seed, stream);
}

extern "C" int64_t dph_layernorm_bwd_workspace(int64_t rows, int64_t D) {
  // per-block slab rows [nblk][3][D] + the per-block branch_sdot partials of deterministic mode [nblk]
  const int64_t nblk = cdiv(rows, (int64_t)LN_BWD_WAVES * LN_BWD_RPW);
  return nblk * (3 * D + 1) * 4;
}

namespace {
bool ln16_env(const char* name) {
  const char* e = getenv(name);
  return !(e && e[0] == '0');
}
bool ln16_shape(int64_t D, std::initializer_list<const void*> ps) {
  if (D % 256 != 0 || D > 1024) return false;
  for (const void* q : ps)
    if (q && (reinterpret_cast<uintptr_t>(q) & 15) != 0) return false;
  return true;
}
// the 16-byte backward over fp32 x (XT) with bf16 (x32) or fp32 (res32) dx; no branch outputs
template <typename DT>
void ln_bwd16_f32x(const void* dy, const float* x, const float* gamma, const float* mean, const float* rstd, DT* dx,
                   float* dgamma, float* dbeta, int64_t rows, int64_t D, const DT* dx_add, float* ws, dim3 grid,
                   hipStream_t stream) {
  const bf16_t* dyb = reinterpret_cast<const bf16_t*>(dy);
#define LN_BWD16F_LAUNCH(NE)                                                                                     \
  hipLaunchKernelGGL((ln_bwd16_kernel<NE, float, DT>), grid, dim3(512), 0, stream, dyb, x, gamma, mean, rstd, dx,  \
                     dgamma, dbeta, rows, (bf16_t*)nullptr, 0.f, (uint64_t)0, (const float*)nullptr,              \
                     (float*)nullptr, (const bf16_t*)nullptr, (float*)nullptr, dx_add, ws, (float*)nullptr)
  switch (D / 256) {
    case 1: LN_BWD16F_LAUNCH(8); break;
    case 2: LN_BWD16F_LAUNCH(16); break;
    case 3: LN_BWD16F_LAUNCH(24); break;
    default: LN_BWD16F_LAUNCH(32); break;
  }
#undef LN_BWD16F_LAUNCH
}
}  // namespace

extern "C" int dph_layernorm_bwd_ld(const void* dy, const void* x, const float* xscale, const float* gamma,
                                    const float* mean, const float* rstd, void* dx, float* dgamma, float* dbeta,
                                    int64_t rows, int64_t D, int64_t ld, float dropout_p, uint64_t seed, void* branch,
                                    float branch_p, uint64_t branch_seed, const float* branch_smask,
                                    float* branch_colsum, const void* branch_pre, float* branch_sdot,
                                    const void* dx_add, float* ws, int64_t ws_bytes, hipStream_t stream) {
  DPH_REQUIRE(dy && x && gamma && mean && rstd && dx, "dph_layernorm_bwd: null pointer");
  if (ld == 0) ld = D;
  DPH_REQUIRE(D >= 1 && ld >= D && ld % 4 == 0 && ld <= LN_MAXV * 256 && rows > 0,
              "dph_layernorm_bwd: unsupported D=%lld ld=%lld", (long long)D, (long long)ld);
  DPH_REQUIRE(!branch_sdot || branch_pre, "dph_layernorm_bwd: branch_sdot needs branch_pre");
  DPH_REQUIRE(!(branch_colsum || branch_sdot) || branch, "dph_layernorm_bwd: branch sums need branch output");
  const bool sums = dgamma || dbeta || branch_colsum;
  const bool det_sdot = branch_sdot && deterministic();
  DPH_REQUIRE(!(sums || det_sdot) || (ws && ws_bytes >= dph_layernorm_bwd_workspace(rows, D)),
              "dph_layernorm_bwd: workspace too small (%lld < %lld bytes)", (long long)ws_bytes,
              (long long)dph_layernorm_bwd_workspace(rows, D));
  const dim3 grid((unsigned)cdiv(rows, LN_BWD_WAVES * LN_BWD_RPW));
  float* sdot_part = det_sdot ? ws + (int64_t)grid.x * 3 * D : nullptr;
  static const bool ln16 = [] {
    const char* e = getenv("DPH_LN_BWD16");
    return !(e && e[0] == '0');
  }();
  auto a16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  if (ln16 && !xscale && dropout_p <= 0.f && ld == D && D % 256 == 0 && D <= 1024 && a16(dy) && a16(x) &&
      a16(dx) && a16(gamma) && (!branch || a16(branch)) && (!branch_pre || a16(branch_pre)) &&
      (!dx_add || a16(dx_add))) {
    const bf16_t* dyb = reinterpret_cast<const bf16_t*>(dy);
    const bf16_t* xb = reinterpret_cast<const bf16_t*>(x);
#define LN_BWD16_LAUNCH(NE)                                                                                       \
  hipLaunchKernelGGL(ln_bwd16_kernel<NE>, grid, dim3(512), 0, stream, dyb, xb, gamma, mean, rstd,                 \
                     reinterpret_cast<bf16_t*>(dx), dgamma, dbeta, rows, reinterpret_cast<bf16_t*>(branch), branch_p, \
                     branch_seed, branch_smask, branch_colsum, reinterpret_cast<const bf16_t*>(branch_pre),           \
                     branch_sdot, reinterpret_cast<const bf16_t*>(dx_add), ws, sdot_part)
    switch (D / 256) {
      case 1: LN_BWD16_LAUNCH(8); break;
      case 2: LN_BWD16_LAUNCH(16); break;
      case 3: LN_BWD16_LAUNCH(24); break;
      default: LN_BWD16_LAUNCH(32); break;
    }
#undef LN_BWD16_LAUNCH
  } else {
#define LN_BWD_LAUNCH(NV)                                                                                        \
  hipLaunchKernelGGL(ln_bwd_kernel<NV>, grid, dim3(64 * LN_BWD_WAVES), 0, stream,                                \
                     reinterpret_cast<const bf16_t*>(dy), reinterpret_cast<const bf16_t*>(x), xscale, gamma, mean, \
                     rstd, reinterpret_cast<bf16_t*>(dx), dgamma, dbeta, rows, (int)D, (int)ld, dropout_p, seed,  \
                     reinterpret_cast<bf16_t*>(branch), branch_p, branch_seed, branch_smask, branch_colsum,       \
                     reinterpret_cast<const bf16_t*>(branch_pre), branch_sdot, reinterpret_cast<const bf16_t*>(dx_add), \
                     ws, sdot_part)
  switch (cdiv(ld, 256)) {
    case 1: LN_BWD_LAUNCH(1); break;
    case 2: LN_BWD_LAUNCH(2); break;
    case 3: LN_BWD_LAUNCH(3); break;
    default: LN_BWD_LAUNCH(4); break;
  }
#undef LN_BWD_LAUNCH
  }
  if (sums) DPH_TRY(slab_reduce_launch(ws, grid.x, 3 * D, D, dgamma, dbeta, branch_colsum, stream));
  if (det_sdot) hipLaunchKernelGGL(sdot_reduce_kernel, dim3(1), dim3(64), 0, stream, sdot_part, (int64_t)grid.x, branch_sdot);
  return check_launch("dph_layernorm_bwd");
}

extern "C" int dph_layernorm_bwd_x32(const void* dy, const float* x, const float* gamma, const float* mean,
                                     const float* rstd, void* dx, float* dgamma, float* dbeta, int64_t rows, int64_t D,
                                     float* ws, int64_t ws_bytes, hipStream_t stream) {
  DPH_REQUIRE(dy && x && gamma && mean && rstd && dx, "dph_layernorm_bwd_x32: null pointer");
  DPH_REQUIRE(D >= 1 && D % 4 == 0 && D <= LN_MAXV * 256 && rows > 0, "dph_layernorm_bwd_x32: unsupported D=%lld",
              (long long)D);
  const bool sums = dgamma || dbeta;
  DPH_REQUIRE(!sums || (ws && ws_bytes >= dph_layernorm_bwd_workspace(rows, D)),
              "dph_layernorm_bwd_x32: workspace too small (%lld < %lld bytes)", (long long)ws_bytes,
              (long long)dph_layernorm_bwd_workspace(rows, D));
  const dim3 grid((unsigned)cdiv(rows, LN_BWD_WAVES * LN_BWD_RPW));
  static const bool ln16 = ln16_env("DPH_LN_BWD16");
  if (ln16 && ln16_shape(D, {dy, x, dx, gamma})) {
    ln_bwd16_f32x<bf16_t>(dy, x, gamma, mean, rstd, reinterpret_cast<bf16_t*>(dx), dgamma, dbeta, rows, D,
                          (const bf16_t*)nullptr, ws, grid, stream);
  } else {
#define LN_BWD32_LAUNCH(NV)                                                                                      \
  hipLaunchKernelGGL((ln_bwd_kernel<NV, float>), grid, dim3(64 * LN_BWD_WAVES), 0, stream,                       \
                     reinterpret_cast<const bf16_t*>(dy), x, (const float*)nullptr, gamma, mean, rstd,           \
                     reinterpret_cast<bf16_t*>(dx), dgamma, dbeta, rows, (int)D, (int)D, 0.f, (uint64_t)0,        \
                     (bf16_t*)nullptr, 0.f, (uint64_t)0, (const float*)nullptr, (float*)nullptr,                  \
                     (const bf16_t*)nullptr, (float*)nullptr, (const bf16_t*)nullptr, ws, (float*)nullptr)
  switch (cdiv(D, 256)) {
    case 1: LN_BWD32_LAUNCH(1); break;
    case 2: LN_BWD32_LAUNCH(2); break;
    case 3: LN_BWD32_LAUNCH(3); break;
    default: LN_BWD32_LAUNCH(4); break;
  }
#undef LN_BWD32_LAUNCH
  }
  if (sums) DPH_TRY(slab_reduce_launch(ws, grid.x, 3 * D, D, dgamma, dbeta, nullptr, stream));
  return check_launch("dph_layernorm_bwd_x32");
}

extern "C" int dph_layernorm_fwd_x32(const float* x, const float* gamma, const float* beta, void* y, float* mean,
                                     float* rstd, int64_t rows, int64_t D, float eps, hipStream_t stream) {
  DPH_REQUIRE(x && gamma && beta && y && mean && rstd, "dph_layernorm_fwd_x32: null pointer");
  DPH_REQUIRE(D >= 1 && D % 4 == 0 && D <= LN_MAXV * 256 && rows > 0, "dph_layernorm_fwd_x32: unsupported D=%lld",
              (long long)D);
  static const bool ln16 = ln16_env("DPH_LN_FWD16");
  if (ln16 && ln16_shape(D, {x, y, gamma, beta})) {
    const dim3 g16((unsigned)cdiv(rows, 8));
    bf16_t* yb = reinterpret_cast<bf16_t*>(y);
    switch (D / 256) {
      case 1: hipLaunchKernelGGL((ln_fwd16_kernel<8, float>), g16, dim3(256), 0, stream, x, gamma, beta, yb, mean, rstd, rows, eps); break;
      case 2: hipLaunchKernelGGL((ln_fwd16_kernel<16, float>), g16, dim3(256), 0, stream, x, gamma, beta, yb, mean, rstd, rows, eps); break;
      case 3: hipLaunchKernelGGL((ln_fwd16_kernel<24, float>), g16, dim3(256), 0, stream, x, gamma, beta, yb, mean, rstd, rows, eps); break;
      default: hipLaunchKernelGGL((ln_fwd16_kernel<32, float>), g16, dim3(256), 0, stream, x, gamma, beta, yb, mean, rstd, rows, eps); break;
    }
    return check_launch("dph_layernorm_fwd_x32");
  }
  const dim3 grid((unsigned)cdiv(rows, 4 * LN_FWD_RPW));
#define LN_FWD32_LAUNCH(NV)                                                                                      \
  hipLaunchKernelGGL((ln_fwd_kernel<NV, false, float>), grid, dim3(256), 0, stream, x, (const float*)nullptr,    \
                     gamma, beta, reinterpret_cast<bf16_t*>(y), mean, rstd, rows, (int)D, (int)D, eps, 0.f,       \
                     (uint64_t)0, (const float*)nullptr, (bf16_t*)nullptr)
  switch (cdiv(D, 256)) {
    case 1: LN_FWD32_LAUNCH(1); break;
    case 2: LN_FWD32_LAUNCH(2); break;
    case 3: LN_FWD32_LAUNCH(3); break;
    default: LN_FWD32_LAUNCH(4); break;
  }
#undef LN_FWD32_LAUNCH
  return check_launch("dph_layernorm_fwd_x32");
}

extern "C" int dph_layernorm_bwd_res32(const void* dy, const float* x, const float* gamma, const float* mean,
                                       const float* rstd, float* dx, float* dgamma, float* dbeta, int64_t rows,
                                       int64_t D, const float* dx_add, float* ws, int64_t ws_bytes,
                                       hipStream_t stream) {
  DPH_REQUIRE(dy && x && gamma && mean && rstd && dx, "dph_layernorm_bwd_res32: null pointer");
  DPH_REQUIRE(D >= 1 && D % 4 == 0 && D <= LN_MAXV * 256 && rows > 0, "dph_layernorm_bwd_res32: unsupported D=%lld",
              (long long)D);
  const bool sums = dgamma || dbeta;
  DPH_REQUIRE(!sums || (ws && ws_bytes >= dph_layernorm_bwd_workspace(rows, D)),
              "dph_layernorm_bwd_res32: workspace too small (%lld < %lld bytes)", (long long)ws_bytes,
              (long long)dph_layernorm_bwd_workspace(rows, D));
  const dim3 grid((unsigned)cdiv(rows, LN_BWD_WAVES * LN_BWD_RPW));
  static const bool ln16 = ln16_env("DPH_LN_BWD16");
  if (ln16 && ln16_shape(D, {dy, x, dx, gamma, dx_add})) {
    ln_bwd16_f32x<float>(dy, x, gamma, mean, rstd, dx, dgamma, dbeta, rows, D, dx_add, ws, grid, stream);
  } else {
#define LN_BWDR_LAUNCH(NV)                                                                                       \
  hipLaunchKernelGGL((ln_bwd_kernel<NV, float, float>), grid, dim3(64 * LN_BWD_WAVES), 0, stream,                \
                     reinterpret_cast<const bf16_t*>(dy), x, (const float*)nullptr, gamma, mean, rstd, dx, dgamma, \
                     dbeta, rows, (int)D, (int)D, 0.f, (uint64_t)0, (bf16_t*)nullptr, 0.f, (uint64_t)0,           \
                     (const float*)nullptr, (float*)nullptr, (const bf16_t*)nullptr, (float*)nullptr, dx_add, ws,      \
                     (float*)nullptr)
  switch (cdiv(D, 256)) {
    case 1: LN_BWDR_LAUNCH(1); break;
    case 2: LN_BWDR_LAUNCH(2); break;
    case 3: LN_BWDR_LAUNCH(3); break;
    default: LN_BWDR_LAUNCH(4); break;
  }
#undef LN_BWDR_LAUNCH
  }
  if (sums) DPH_TRY(slab_reduce_launch(ws, grid.x, 3 * D, D, dgamma, dbeta, nullptr, stream));
  return check_launch("dph_layernorm_bwd_res32");
}

extern "C" int dph_wave_layernorm(const float* x, const int64_t* lengths, int64_t B, int64_t S, float eps, float* y,
                                  hipStream_t stream) {
  DPH_REQUIRE(x && y && B > 0 && S > 0, "dph_wave_layernorm: bad args");
  hipLaunchKernelGGL(wave_norm_kernel, dim3((unsigned)B), dim3(1024), 0, stream, x, lengths, S, eps, y);
  return check_launch("dph_wave_layernorm");
}

extern "C" int dph_layernorm_bwd(const void* dy, const void* x, const float* xscale, const float* gamma,
                                 const float* mean, const float* rstd, void* dx, float* dgamma, float* dbeta,
                                 int64_t rows, int64_t D, float dropout_p, uint64_t seed, void* branch,
                                 float branch_p, uint64_t branch_seed, const float* branch_smask,
                                 float* branch_colsum, const void* branch_pre, float* branch_sdot, float* ws,
                                 int64_t ws_bytes, hipStream_t stream) {
  return dph_layernorm_bwd_ld(dy, x, xscale, gamma, mean, rstd, dx, dgamma, dbeta, rows, D, D, dropout_p, seed,
                              branch, branch_p, branch_seed, branch_smask, branch_colsum, branch_pre, branch_sdot,
                              nullptr, ws, ws_bytes, stream);
}

extern "C" int dph_colprod(const void* a, int64_t lda, const float* b, int64_t ldb, const float* colmask, float* out,
                           int64_t R, int64_t N, hipStream_t stream) {
  DPH_REQUIRE(a && b && out && R > 0 && N > 0 && lda >= N && ldb >= N, "dph_colprod: bad args");
  if (deterministic()) {
    hipLaunchKernelGGL(colprod_det_kernel, dim3((unsigned)cdiv(N, 32)), dim3(32 * DET_PH), 0, stream,
                       reinterpret_cast<const bf16_t*>(a), lda, b, ldb, colmask, out, R, N);
    return check_launch("dph_colprod");
  }
  const int64_t rpb = 32;
  dim3 grid((unsigned)cdiv(N, 512), (unsigned)cdiv(R, rpb));
  hipLaunchKernelGGL(colprod_kernel, grid, dim3(256), 0, stream, reinterpret_cast<const bf16_t*>(a), lda, b, ldb,
                     colmask, out, R, N, rpb);
  return check_launch("dph_colprod");
}

extern "C" int64_t dph_colsum_workspace(int64_t rows, int64_t cols) {
  return cdiv(rows, colsum_rpb(rows)) * cols * 4;
}

extern "C" int dph_colsum(const void* x, float* out, int64_t rows, int64_t cols, float* ws, int64_t ws_bytes,
                          hipStream_t stream) {
  DPH_REQUIRE(x && out && rows > 0 && cols > 0, "dph_colsum: bad args");
  DPH_REQUIRE(ws && ws_bytes >= dph_colsum_workspace(rows, cols), "dph_colsum: workspace too small");
  const int64_t rpb = colsum_rpb(rows);
  const int64_t nrb = cdiv(rows, rpb);
  dim3 grid((unsigned)cdiv(cols, 512), (unsigned)nrb);
  hipLaunchKernelGGL(colsum_kernel, grid, dim3(256), 0, stream, reinterpret_cast<const bf16_t*>(x), ws, rows, cols,
                     rpb, cols, cols, (int64_t)0);
  DPH_TRY(slab_reduce_launch(ws, nrb, cols, cols, out, nullptr, nullptr, stream));
  return check_launch("dph_colsum");
}

// Column sums of a [rows][3*seg] matrix into three segment outputs (NULL output: segment skipped).  The fused
// q/k/v projection gradient: the k_proj bias gradient is the column sum of dK, which is exactly zero (each query
// row's scores are shifted by q.b_k for every key, and softmax is shift invariant, components.py:411-417) -- its
// fp32 evaluation is rounding noise that AdamW would turn into +-lr steps, so it is not computed (out1 = NULL).
extern "C" int dph_colsum3(const void* x, float* out0, float* out1, float* out2, int64_t rows, int64_t seg, float* ws,
                           int64_t ws_bytes, hipStream_t stream) {
  const int64_t cols = 3 * seg;
  DPH_REQUIRE(x && rows > 0 && seg > 0, "dph_colsum3: bad args");
  DPH_REQUIRE(ws && ws_bytes >= dph_colsum_workspace(rows, cols), "dph_colsum3: workspace too small");
  const int64_t rpb = colsum_rpb(rows);
  const int64_t nrb = cdiv(rows, rpb);
  if (out1 == nullptr && out0 && out2 && seg % 8 == 0) {
    // the middle segment skipped: only the outer two are read (the slab holds [seg | seg])
    dim3 grid2((unsigned)cdiv(2 * seg, 512), (unsigned)nrb);
    hipLaunchKernelGGL(colsum_kernel, grid2, dim3(256), 0, stream, reinterpret_cast<const bf16_t*>(x), ws, rows,
                       2 * seg, rpb, cols, seg, seg);
    DPH_TRY(slab_reduce_launch(ws, nrb, 2 * seg, seg, out0, out2, nullptr, stream));
    return check_launch("dph_colsum3");
  }
  dim3 grid((unsigned)cdiv(cols, 512), (unsigned)nrb);
  hipLaunchKernelGGL(colsum_kernel, grid, dim3(256), 0, stream, reinterpret_cast<const bf16_t*>(x), ws, rows, cols,
                     rpb, cols, cols, (int64_t)0);
  DPH_TRY(slab_reduce_launch(ws, nrb, cols, seg, out0, out1, out2, stream));
  return check_launch("dph_colsum3");
}
