// LayerNorm forward/backward over the last dim (one wave per row) and column
// sums (bias gradients).  fp32 statistics, bf16 storage.
//
// Reference call sites: nn.LayerNorm in FeatureProjection (components.py:271),
// EncoderLayer (:839,:850,:853,:856), Transformer._preprocess (:889) and the
// channel LayerNorm of layer_norm-mode extractors (:54-61).  torch semantics:
// biased variance, eps inside the sqrt.
#include "common.h"

namespace dph {
namespace {

constexpr int LN_MAXV = 4;   // up to 4 x (64 lanes x 4 elements) = 1024 columns

__global__ void __launch_bounds__(256) ln_fwd_kernel(const bf16_t* __restrict__ x, const float* __restrict__ xscale,
                                                     const float* __restrict__ gamma, const float* __restrict__ beta,
                                                     bf16_t* __restrict__ y, float* __restrict__ mean_out,
                                                     float* __restrict__ rstd_out, int64_t rows, int D, int ld,
                                                     float eps, float drop_p, uint64_t seed) {
  seed = epoch_seed(seed);   // per-step RNG epoch (graph replays)
  // rows have stride ld >= D (ld % 4 == 0); columns [D, ld) are row padding: read as 0, written as 0
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const bf16_t* xr = x + row * ld;
  float v[LN_MAXV][4];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < LN_MAXV; ++c) {
    const int col = (c * 64 + lane) * 4;
    if (col < D) {
      uint2 raw = *reinterpret_cast<const uint2*>(xr + col);
      v[c][0] = __uint_as_float(raw.x << 16);
      v[c][1] = __uint_as_float(raw.x & 0xffff0000u);
      v[c][2] = __uint_as_float(raw.y << 16);
      v[c][3] = __uint_as_float(raw.y & 0xffff0000u);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (col + i >= D) v[c][i] = 0.f;
        else if (xscale) v[c][i] *= xscale[col + i];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) s += v[c][i];
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) v[c][i] = 0.f;
    }
  }
  const float mean = wave_sum(s) / D;
  float q = 0.f;
#pragma unroll
  for (int c = 0; c < LN_MAXV; ++c) {
    const int col = (c * 64 + lane) * 4;
    if (col < D) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float d = v[c][i] - mean;
        if (col + i < D) q += d * d;
      }
    }
  }
  const float var = wave_sum(q) / D;
  const float rstd = rsqrtf(var + eps);
  const float inv_keep = drop_p > 0.f ? 1.f / (1.f - drop_p) : 1.f;
#pragma unroll
  for (int c = 0; c < LN_MAXV; ++c) {
    const int col = (c * 64 + lane) * 4;
    if (col < ld) {
      float o[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (col + i < D) {
          o[i] = (v[c][i] - mean) * rstd * gamma[col + i] + beta[col + i];
          o[i] *= dropout_scale(seed, (uint64_t)row * D + col + i, drop_p, inv_keep);
        } else {
          o[i] = 0.f;
        }
      }
      *reinterpret_cast<uint2*>(y + row * ld + col) = make_uint2(pack2bf(o[0], o[1]), pack2bf(o[2], o[3]));
    }
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// Backward.  Each wave walks rows with a grid stride; per-column partials
// (dgamma, dbeta, branch column sums) stay in registers, are reduced across
// the block's 4 waves through LDS and land with one atomic per column.
__global__ void __launch_bounds__(256) ln_bwd_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x, const float* __restrict__ xscale,
    const float* __restrict__ gamma, const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
    bf16_t* __restrict__ dx, float* __restrict__ dgamma, float* __restrict__ dbeta, int64_t rows, int D, int ld,
    float drop_p,
    uint64_t seed, bf16_t* __restrict__ branch, float branch_p, uint64_t branch_seed,
    const float* __restrict__ branch_smask, float* __restrict__ branch_colsum, const bf16_t* __restrict__ branch_pre,
    float* __restrict__ branch_sdot, const bf16_t* __restrict__ dx_add) {
  seed = epoch_seed(seed); branch_seed = epoch_seed(branch_seed);   // per-step RNG epoch (graph replays)
  __shared__ float red[4][3][LN_MAXV * 256];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const float inv_keep = drop_p > 0.f ? 1.f / (1.f - drop_p) : 1.f;
  const float binv_keep = branch_p > 0.f ? 1.f / (1.f - branch_p) : 1.f;
  const float bsm = branch_smask ? *branch_smask : 1.0f;
  float pg[LN_MAXV][4], pb[LN_MAXV][4], pc[LN_MAXV][4];
#pragma unroll
  for (int c = 0; c < LN_MAXV; ++c)
#pragma unroll
    for (int i = 0; i < 4; ++i) pg[c][i] = pb[c][i] = pc[c][i] = 0.f;
  float sdot = 0.f;

  for (int64_t row = (int64_t)blockIdx.x * 4 + wave; row < rows; row += (int64_t)gridDim.x * 4) {
    const float mean = mean_in[row];
    const float rstd = rstd_in[row];
    float xh[LN_MAXV][4], g[LN_MAXV][4], dyv[LN_MAXV][4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < LN_MAXV; ++c) {
      const int col = (c * 64 + lane) * 4;
      if (col < D) {
        uint2 rx = *reinterpret_cast<const uint2*>(x + row * ld + col);
        uint2 rd = *reinterpret_cast<const uint2*>(dy + row * ld + col);
        float xv[4] = {__uint_as_float(rx.x << 16), __uint_as_float(rx.x & 0xffff0000u),
                       __uint_as_float(rx.y << 16), __uint_as_float(rx.y & 0xffff0000u)};
        float dv[4] = {__uint_as_float(rd.x << 16), __uint_as_float(rd.x & 0xffff0000u),
                       __uint_as_float(rd.y << 16), __uint_as_float(rd.y & 0xffff0000u)};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const bool ok = col + i < D;
          float xs = (xscale && ok) ? xv[i] * xscale[col + i] : xv[i];
          xh[c][i] = ok ? (xs - mean) * rstd : 0.f;
          dyv[c][i] = ok ? dv[i] * dropout_scale(seed, (uint64_t)row * D + col + i, drop_p, inv_keep) : 0.f;
          g[c][i] = ok ? dyv[c][i] * gamma[col + i] : 0.f;
          s1 += g[c][i];
          s2 += g[c][i] * xh[c][i];
          pg[c][i] += dyv[c][i] * xh[c][i];
          pb[c][i] += dyv[c][i];
        }
      }
    }
    s1 = wave_sum(s1) / D;
    s2 = wave_sum(s2) / D;
#pragma unroll
    for (int c = 0; c < LN_MAXV; ++c) {
      const int col = (c * 64 + lane) * 4;
      if (col < ld) {
        float o[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const bool ok = col + i < D;
          o[i] = ok ? rstd * (g[c][i] - s1 - xh[c][i] * s2) : 0.f;
          if (xscale && ok) o[i] *= xscale[col + i];
        }
        if (dx_add) {
          // other gradient paths into the LN input (pre-norm residual); the branch output below
          // stays the LN-path gradient only
          const uint2 ra = *reinterpret_cast<const uint2*>(dx_add + row * ld + col);
          const float ad[4] = {__uint_as_float(ra.x << 16), __uint_as_float(ra.x & 0xffff0000u),
                               __uint_as_float(ra.y << 16), __uint_as_float(ra.y & 0xffff0000u)};
          *reinterpret_cast<uint2*>(dx + row * ld + col) =
              make_uint2(pack2bf(o[0] + ad[0], o[1] + ad[1]), pack2bf(o[2] + ad[2], o[3] + ad[3]));
        } else {
          *reinterpret_cast<uint2*>(dx + row * ld + col) = make_uint2(pack2bf(o[0], o[1]), pack2bf(o[2], o[3]));
        }
        if (branch) {
          float bo[4];
          float pre[4] = {0.f, 0.f, 0.f, 0.f};
          if (branch_sdot) {
            uint2 rp = *reinterpret_cast<const uint2*>(branch_pre + row * ld + col);
            pre[0] = __uint_as_float(rp.x << 16);
            pre[1] = __uint_as_float(rp.x & 0xffff0000u);
            pre[2] = __uint_as_float(rp.y << 16);
            pre[3] = __uint_as_float(rp.y & 0xffff0000u);
          }
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float z = (col + i < D) ? o[i] * dropout_scale(branch_seed, (uint64_t)row * D + col + i, branch_p,
                                                                 binv_keep) : 0.f;
            sdot += z * pre[i];
            bo[i] = z * bsm;
            pc[c][i] += bo[i];
          }
          *reinterpret_cast<uint2*>(branch + row * ld + col) = make_uint2(pack2bf(bo[0], bo[1]),
                                                                         pack2bf(bo[2], bo[3]));
        }
      }
    }
  }
  // block reduction of the column partials
#pragma unroll
  for (int c = 0; c < LN_MAXV; ++c)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int col = (c * 64 + lane) * 4 + i;
      red[wave][0][col] = pg[c][i];
      red[wave][1][col] = pb[c][i];
      red[wave][2][col] = pc[c][i];
    }
  __syncthreads();
  for (int col = threadIdx.x; col < D; col += 256) {
    float a = 0.f, b = 0.f, cc = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      a += red[w][0][col];
      b += red[w][1][col];
      cc += red[w][2][col];
    }
    if (dgamma) atomicAdd(dgamma + col, a);
    if (dbeta) atomicAdd(dbeta + col, b);
    if (branch_colsum) atomicAdd(branch_colsum + col, cc);
  }
  if (branch_sdot) {
    sdot = wave_sum(sdot);
    if (lane == 0) atomicAdd(branch_sdot, sdot);
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

// out[n] += sum_m x[m][n]; block = 64 x 4 threads, 8 columns per thread
__global__ void __launch_bounds__(256) colsum_kernel(const bf16_t* __restrict__ x, float* __restrict__ out,
                                                     int64_t rows, int64_t cols, int64_t rows_per_block) {
  __shared__ float red[4][512];
  const int tx = threadIdx.x & 63;
  const int ty = threadIdx.x >> 6;
  const int64_t c0 = (int64_t)blockIdx.x * 512 + tx * 8;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_block;
  const int64_t r1 = min(rows, r0 + rows_per_block);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const bool vec = (c0 + 8 <= cols) && (cols % 8 == 0);
  for (int64_t r = r0 + ty; r < r1; r += 4) {
    const bf16_t* p = x + r * cols + c0;
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
    if (col < cols) atomicAdd(out + col, red[0][c] + red[1][c] + red[2][c] + red[3][c]);
  }
}

}  // namespace
}  // namespace dph

using namespace dph;

extern "C" int dph_layernorm_fwd_ld(const void* x, const float* xscale, const float* gamma, const float* beta,
                                    void* y, float* mean, float* rstd, int64_t rows, int64_t D, int64_t ld, float eps,
                                    float dropout_p, uint64_t seed, hipStream_t stream) {
  DPH_REQUIRE(x && gamma && beta && y && mean && rstd, "dph_layernorm_fwd: null pointer");
  if (ld == 0) ld = D;
  DPH_REQUIRE(D >= 1 && ld >= D && ld % 4 == 0 && ld <= LN_MAXV * 256 && rows > 0,
              "dph_layernorm_fwd: unsupported D=%lld ld=%lld", (long long)D, (long long)ld);
  hipLaunchKernelGGL(ln_fwd_kernel, dim3((unsigned)cdiv(rows, 4)), dim3(256), 0, stream,
                     reinterpret_cast<const bf16_t*>(x), xscale, gamma, beta, reinterpret_cast<bf16_t*>(y), mean, rstd,
                     rows, (int)D, (int)ld, eps, dropout_p, seed);
  return check_launch("dph_layernorm_fwd");
}

extern "C" int dph_layernorm_fwd(const void* x, const float* xscale, const float* gamma, const float* beta, void* y,
                                 float* mean, float* rstd, int64_t rows, int64_t D, float eps, float dropout_p,
                                 uint64_t seed, hipStream_t stream) {
  return dph_layernorm_fwd_ld(x, xscale, gamma, beta, y, mean, rstd, rows, D, D, eps, dropout_p, seed, stream);
}

extern "C" int dph_layernorm_bwd_ld(const void* dy, const void* x, const float* xscale, const float* gamma,
                                    const float* mean, const float* rstd, void* dx, float* dgamma, float* dbeta,
                                    int64_t rows, int64_t D, int64_t ld, float dropout_p, uint64_t seed, void* branch,
                                    float branch_p, uint64_t branch_seed, const float* branch_smask,
                                    float* branch_colsum, const void* branch_pre, float* branch_sdot,
                                    const void* dx_add, hipStream_t stream) {
  DPH_REQUIRE(dy && x && gamma && mean && rstd && dx, "dph_layernorm_bwd: null pointer");
  if (ld == 0) ld = D;
  DPH_REQUIRE(D >= 1 && ld >= D && ld % 4 == 0 && ld <= LN_MAXV * 256 && rows > 0,
              "dph_layernorm_bwd: unsupported D=%lld ld=%lld", (long long)D, (long long)ld);
  DPH_REQUIRE(!branch_sdot || branch_pre, "dph_layernorm_bwd: branch_sdot needs branch_pre");
  DPH_REQUIRE(!(branch_colsum || branch_sdot) || branch, "dph_layernorm_bwd: branch sums need branch output");
  const int64_t blocks = std::min<int64_t>(cdiv(rows, 4 * 8), 1024);
  hipLaunchKernelGGL(ln_bwd_kernel, dim3((unsigned)blocks), dim3(256), 0, stream,
                     reinterpret_cast<const bf16_t*>(dy), reinterpret_cast<const bf16_t*>(x), xscale, gamma, mean,
                     rstd, reinterpret_cast<bf16_t*>(dx), dgamma, dbeta, rows, (int)D, (int)ld, dropout_p, seed,
                     reinterpret_cast<bf16_t*>(branch), branch_p, branch_seed, branch_smask, branch_colsum,
                     reinterpret_cast<const bf16_t*>(branch_pre), branch_sdot,
                     reinterpret_cast<const bf16_t*>(dx_add));
  return check_launch("dph_layernorm_bwd");
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
                                 float* branch_colsum, const void* branch_pre, float* branch_sdot,
                                 hipStream_t stream) {
  return dph_layernorm_bwd_ld(dy, x, xscale, gamma, mean, rstd, dx, dgamma, dbeta, rows, D, D, dropout_p, seed,
                              branch, branch_p, branch_seed, branch_smask, branch_colsum, branch_pre, branch_sdot,
                              nullptr, stream);
}

extern "C" int dph_colsum(const void* x, float* out, int64_t rows, int64_t cols, hipStream_t stream) {
  DPH_REQUIRE(x && out && rows > 0 && cols > 0, "dph_colsum: bad args");
  const int64_t rpb = std::max<int64_t>(64, cdiv(cdiv(rows, 8192), 4) * 4);
  dim3 grid((unsigned)cdiv(cols, 512), (unsigned)cdiv(rows, rpb));
  hipLaunchKernelGGL(colsum_kernel, grid, dim3(256), 0, stream, reinterpret_cast<const bf16_t*>(x), out, rows, cols,
                     rpb);
  return check_launch("dph_colsum");
}
