// Elementwise / layout kernels of the conv frontend and weight handling.
//
//   col2im + GELU/HardConcrete-mask backward of the strided conv layers
//     (components.py:107-114 backward), GELU/mask backward,
//   pos-conv regroup + zero padding (components.py:298-306,327-330 as a
//     batched GEMM over per-group time windows),
//   fp32 master weight -> bf16 GEMM images.
#include "common.h"

#include <algorithm>

namespace dph {
namespace {

// Shared shape: block = 64 x 4 threads; thread handles 8 channels of a row,
// grid.x over 512-channel chunks, grid.y over row ranges.  Column partials
// (mask gradients) are reduced across the 4 row-lanes through LDS.
template <bool COL2IM>
__global__ void __launch_bounds__(256) gelu_mask_bwd_kernel(const bf16_t* __restrict__ src, int64_t Lout,
                                                            int64_t Lin, int64_t C, int k, int s,
                                                            const bf16_t* __restrict__ z_pre,
                                                            const float* __restrict__ mask, bf16_t* __restrict__ out,
                                                            float* __restrict__ dmask, int64_t rows,
                                                            int64_t rows_per_block, float* __restrict__ part) {
  __shared__ float red[4][512];
  const int tx = threadIdx.x & 63;
  const int ty = threadIdx.x >> 6;
  const int64_t c0 = (int64_t)blockIdx.x * 512 + tx * 8;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_block;
  const int64_t r1 = min(rows, r0 + rows_per_block);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float mk[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) mk[i] = (mask && c0 + i < C) ? mask[c0 + i] : 1.0f;
  if (c0 < C) {
    for (int64_t r = r0 + ty; r < r1; r += 4) {
      float dy[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if constexpr (COL2IM) {
        const int64_t b = r / Lin;
        const int64_t tp = r % Lin;
        for (int j = 0; j < k; ++j) {
          const int64_t d = tp - j;
          if (d < 0 || d % s) continue;
          const int64_t t = d / s;
          if (t >= Lout) continue;
          float v[8];
          load_bf16x8(src + ((b * Lout + t) * k + j) * C + c0, c0, C, v);
#pragma unroll
          for (int i = 0; i < 8; ++i) dy[i] += v[i];
        }
      } else {
        load_bf16x8(src + r * C + c0, c0, C, dy);
      }
      float o[8];
      if (z_pre) {
        float z[8];
        load_bf16x8(z_pre + r * C + c0, c0, C, z);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          float g, dg;
          gelu_and_grad(z[i], g, dg);
          acc[i] += dy[i] * g;
          o[i] = dy[i] * mk[i] * dg;
        }
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = dy[i];
      }
      bf16_t* op = out + r * C + c0;
      if (c0 + 8 <= C && C % 8 == 0) {
        *reinterpret_cast<uint4*>(op) = make_uint4(pack2bf(o[0], o[1]), pack2bf(o[2], o[3]), pack2bf(o[4], o[5]),
                                                   pack2bf(o[6], o[7]));
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i)
          if (c0 + i < C) op[i] = f2bf(o[i]);
      }
    }
  }
  if (!dmask) return;
#pragma unroll
  for (int i = 0; i < 8; ++i) red[ty][tx * 8 + i] = acc[i];
  __syncthreads();
  for (int c = threadIdx.x; c < 512; c += 256) {
    const int64_t col = (int64_t)blockIdx.x * 512 + c;
    if (col >= C) continue;
    const float t = red[0][c] + red[1][c] + red[2][c] + red[3][c];
    // deterministic mode: the block's partial row of the [grid.y][C] slab (summed in order after the launch)
    if (part) part[(int64_t)blockIdx.y * C + col] = t;
    else atomicAdd(dmask + col, t);
  }
}

__global__ void regroup_pad_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ xg, int64_t B, int64_t T,
                                   int64_t G, int64_t Cg, int64_t P, int64_t Q) {
  // one thread per 8 elements of xg [B][G][P+T+Q][Cg]
  const int64_t Tp = P + T + Q;
  const int64_t n8 = B * G * Tp * Cg / 8;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n8) return;
  const int64_t e = i * 8;
  const int64_t c = e % Cg;
  const int64_t tp = (e / Cg) % Tp;
  const int64_t g = (e / (Cg * Tp)) % G;
  const int64_t b = e / (Cg * Tp * G);
  const int64_t t = tp - P;
  uint4 v = make_uint4(0, 0, 0, 0);
  if (t >= 0 && t < T) v = *reinterpret_cast<const uint4*>(x + (b * T + t) * (G * Cg) + g * Cg + c);
  *reinterpret_cast<uint4*>(xg + e) = v;
}

__global__ void cast_bf16_kernel(const float* __restrict__ src, bf16_t* __restrict__ dst, int64_t n) {
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i + 4 <= n) {
    float4 v = *reinterpret_cast<const float4*>(src + i);
    *reinterpret_cast<uint2*>(dst + i) = make_uint2(pack2bf(v.x, v.y), pack2bf(v.z, v.w));
  } else {
    for (int64_t j = i; j < n; ++j) dst[j] = f2bf(src[j]);
  }
}

// w [O][C][k] fp32 -> dst [Op][k*Cp] bf16 (index j*Cp + c); zero padding rows / channels
__global__ void conv_pack_kernel(const float* __restrict__ w, bf16_t* __restrict__ dst, int64_t O, int64_t C,
                                 int64_t k, int64_t Op, int64_t Cp) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= Op * Cp * k) return;
  const int64_t c = i % Cp;
  const int64_t j = (i / Cp) % k;
  const int64_t o = i / (Cp * k);
  dst[i] = (o < O && c < C) ? f2bf(w[(o * C + c) * k + j]) : (bf16_t)0;
}

// g [>=O][k*Cp] fp32 -> dst [O][C][k]
__global__ void conv_unpack_kernel(const float* __restrict__ g, float* __restrict__ dst, int64_t O, int64_t C,
                                   int64_t k, int64_t Cp, int accum) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= O * C * k) return;
  const int64_t j = i % k;
  const int64_t c = (i / k) % C;
  const int64_t o = i / (C * k);
  const float v = g[o * k * Cp + j * Cp + c];
  dst[i] = accum ? dst[i] + v : v;
}

__global__ void add_bf16_kernel(const bf16_t* __restrict__ a, const bf16_t* __restrict__ b, bf16_t* __restrict__ o,
                                int64_t n) {
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8;
  if (i + 8 <= n) {
    uint4 va = *reinterpret_cast<const uint4*>(a + i);
    uint4 vb = *reinterpret_cast<const uint4*>(b + i);
    uint32_t wa[4] = {va.x, va.y, va.z, va.w}, wb[4] = {vb.x, vb.y, vb.z, vb.w}, wo[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float lo = __uint_as_float(wa[q] << 16) + __uint_as_float(wb[q] << 16);
      const float hi = __uint_as_float(wa[q] & 0xffff0000u) + __uint_as_float(wb[q] & 0xffff0000u);
      wo[q] = pack2bf(lo, hi);
    }
    *reinterpret_cast<uint4*>(o + i) = make_uint4(wo[0], wo[1], wo[2], wo[3]);
  } else {
    for (int64_t j = i; j < n; ++j) o[j] = f2bf(bf2f(a[j]) + bf2f(b[j]));
  }
}

// out = dy * drop(p, seed, m*cols+n) * (*smask), rows with (m % len_rows) >= row_len[m / len_rows] zeroed;
// colsum[n] += out; sdot += sum dy*drop*pre
// DyT / OT: bf16, or fp32 for the pre-norm residual stream (its gradient / the pos-conv output, components.py:846-850)
__device__ __forceinline__ float to_f(bf16_t v) { return bf2f(v); }
__device__ __forceinline__ float to_f(float v) { return v; }
template <typename DyT, typename OT>
__global__ void __launch_bounds__(256) branch_bwd_kernel(const DyT* __restrict__ dy, OT* __restrict__ out,
                                                         int64_t rows, int64_t cols, float p, uint64_t seed,
                                                         const float* __restrict__ smask,
                                                         const int64_t* __restrict__ row_len, int64_t len_rows,
                                                         float* __restrict__ colsum, const bf16_t* __restrict__ pre,
                                                         float* __restrict__ sdot, int64_t rows_per_block,
                                                         float* __restrict__ part) {
  seed = epoch_seed(seed);   // per-step RNG epoch (graph replays)
  __shared__ float red[4][512];
  __shared__ float sred[4];
  const int tx = threadIdx.x & 63;
  const int ty = threadIdx.x >> 6;
  const int64_t c0 = (int64_t)blockIdx.x * 512 + tx * 8;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_block;
  const int64_t r1 = min(rows, r0 + rows_per_block);
  const float inv_keep = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const float sm = smask ? *smask : 1.0f;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float sd = 0.f;
  if (c0 < cols) {
    for (int64_t r = r0 + ty; r < r1; r += 4) {
      const bool zero = row_len && ((r % len_rows) >= row_len[r / len_rows]);
      float o[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int64_t c = c0 + i;
        float v = 0.f;
        if (c < cols && !zero) {
          v = to_f(dy[r * cols + c]) * dropout_scale(seed, (uint64_t)r * cols + c, p, inv_keep);
          if (pre) sd += v * bf2f(pre[r * cols + c]);
          v *= sm;
        }
        o[i] = v;
        acc[i] += v;
      }
      OT* op = out + r * cols + c0;
      if constexpr (sizeof(OT) == 4) {
        if (c0 + 8 <= cols && cols % 8 == 0) {
          *reinterpret_cast<float4*>(op) = make_float4(o[0], o[1], o[2], o[3]);
          *reinterpret_cast<float4*>(op + 4) = make_float4(o[4], o[5], o[6], o[7]);
        } else {
#pragma unroll
          for (int i = 0; i < 8; ++i)
            if (c0 + i < cols) op[i] = o[i];
        }
      } else if (c0 + 8 <= cols && cols % 8 == 0) {
        *reinterpret_cast<uint4*>(op) = make_uint4(pack2bf(o[0], o[1]), pack2bf(o[2], o[3]), pack2bf(o[4], o[5]),
                                                   pack2bf(o[6], o[7]));
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i)
          if (c0 + i < cols) op[i] = f2bf(o[i]);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) red[ty][tx * 8 + i] = acc[i];
  sd = wave_sum(sd);
  if (tx == 0) sred[ty] = sd;
  __syncthreads();
  // deterministic mode (part != NULL): the block's column partials as row blockIdx.y of a [grid.y][cols] slab and its
  // sdot partial after the slab (index y * grid.x + x), both summed in order after the launch
  if (colsum) {
    for (int c = threadIdx.x; c < 512; c += 256) {
      const int64_t col = (int64_t)blockIdx.x * 512 + c;
      if (col >= cols) continue;
      const float t = red[0][c] + red[1][c] + red[2][c] + red[3][c];
      if (part) part[(int64_t)blockIdx.y * cols + col] = t;
      else atomicAdd(colsum + col, t);
    }
  }
  if (sdot && threadIdx.x == 0) {
    const float t = sred[0] + sred[1] + sred[2] + sred[3];
    if (part) part[(int64_t)gridDim.y * cols + (int64_t)blockIdx.y * gridDim.x + blockIdx.x] = t;
    else atomicAdd(sdot, t);
  }
}

int64_t rows_per_block_for(int64_t rows) { return std::max<int64_t>(16, cdiv(cdiv(rows, 4096), 4) * 4); }
// deterministic mode: at most ~512 row blocks (the fixed-order slab reduction then sums <= 512 rows per column)
int64_t rows_per_block_det(int64_t rows) {
  return std::max<int64_t>(rows_per_block_for(rows), cdiv(cdiv(rows, 512), 4) * 4);
}

}  // namespace
}  // namespace dph

using namespace dph;

// Workspace (bytes) of the row-block column reductions below (dph_col2im_gelu_bwd / dph_gelu_mask_bwd over rows x C,
// dph_branch_bwd(_f32) over rows x cols): the per-row-block partial slab + sdot partials of deterministic mode
extern "C" int64_t dph_rowblock_workspace(int64_t rows, int64_t cols) {
  if (rows <= 0 || cols <= 0) return 0;
  const int64_t nrb = cdiv(rows, rows_per_block_det(rows));
  return (nrb * cols + nrb * cdiv(cols, 512)) * 4;
}

namespace {
// deterministic mode needs the workspace whenever a column sum / sdot is requested
int rowblock_plan(int64_t rows, int64_t cols, bool sums, float* ws, int64_t ws_bytes, int64_t& rpb, float*& part,
                  const char* who) {
  part = nullptr;
  rpb = rows_per_block_for(rows);
  if (sums && deterministic()) {
    DPH_REQUIRE(ws && ws_bytes >= dph_rowblock_workspace(rows, cols),
                "%s: deterministic mode needs dph_rowblock_workspace(rows, cols) bytes of workspace", who);
    rpb = rows_per_block_det(rows);
    part = ws;
  }
  return DPH_OK;
}
}  // namespace

extern "C" int dph_col2im_gelu_bwd(const void* dcols, int64_t B, int64_t Lout, int64_t Lin, int64_t C, int64_t k,
                                   int64_t s, const void* z_pre, const float* mask, void* out, float* dmask, float* ws,
                                   int64_t ws_bytes, hipStream_t stream) {
  DPH_REQUIRE(dcols && out && B > 0 && Lout > 0 && Lin >= Lout && C > 0 && k > 0 && s > 0,
              "dph_col2im_gelu_bwd: bad args");
  DPH_REQUIRE(!dmask || z_pre, "dph_col2im_gelu_bwd: dmask needs z_pre");
  const int64_t rows = B * Lin;
  int64_t rpb;
  float* part;
  if (int rc = rowblock_plan(rows, C, dmask != nullptr, ws, ws_bytes, rpb, part, "dph_col2im_gelu_bwd")) return rc;
  const int64_t nrb = cdiv(rows, rpb);
  dim3 grid((unsigned)cdiv(C, 512), (unsigned)nrb);
  hipLaunchKernelGGL(gelu_mask_bwd_kernel<true>, grid, dim3(256), 0, stream, reinterpret_cast<const bf16_t*>(dcols),
                     Lout, Lin, C, (int)k, (int)s, reinterpret_cast<const bf16_t*>(z_pre), mask,
                     reinterpret_cast<bf16_t*>(out), dmask, rows, rpb, part);
  if (part) DPH_TRY(slab_reduce_cols(part, nrb, C, C, dmask, nullptr, nullptr, stream));
  return check_launch("dph_col2im_gelu_bwd");
}

extern "C" int dph_gelu_mask_bwd(const void* dy, const void* z_pre, const float* mask, void* out, float* dmask,
                                 int64_t rows, int64_t C, float* ws, int64_t ws_bytes, hipStream_t stream) {
  DPH_REQUIRE(dy && z_pre && out && rows > 0 && C > 0, "dph_gelu_mask_bwd: bad args");
  int64_t rpb;
  float* part;
  if (int rc = rowblock_plan(rows, C, dmask != nullptr, ws, ws_bytes, rpb, part, "dph_gelu_mask_bwd")) return rc;
  const int64_t nrb = cdiv(rows, rpb);
  dim3 grid((unsigned)cdiv(C, 512), (unsigned)nrb);
  hipLaunchKernelGGL(gelu_mask_bwd_kernel<false>, grid, dim3(256), 0, stream, reinterpret_cast<const bf16_t*>(dy),
                     (int64_t)1, (int64_t)1, C, 1, 1, reinterpret_cast<const bf16_t*>(z_pre), mask,
                     reinterpret_cast<bf16_t*>(out), dmask, rows, rpb, part);
  if (part) DPH_TRY(slab_reduce_cols(part, nrb, C, C, dmask, nullptr, nullptr, stream));
  return check_launch("dph_gelu_mask_bwd");
}

extern "C" int dph_regroup_pad(const void* x, void* xg, int64_t B, int64_t T, int64_t G, int64_t Cg,
                               int64_t pad_front, int64_t pad_back, hipStream_t stream) {
  DPH_REQUIRE(x && xg && Cg % 8 == 0 && B > 0 && T > 0 && G > 0, "dph_regroup_pad: bad args (Cg %% 8 == 0)");
  const int64_t n8 = B * G * (pad_front + T + pad_back) * Cg / 8;
  hipLaunchKernelGGL(regroup_pad_kernel, dim3((unsigned)cdiv(n8, 256)), dim3(256), 0, stream,
                     reinterpret_cast<const bf16_t*>(x), reinterpret_cast<bf16_t*>(xg), B, T, G, Cg, pad_front,
                     pad_back);
  return check_launch("dph_regroup_pad");
}

namespace dph {
namespace {
// bf16 [R][C] -> [C][R] through a 64x64 LDS tile (16-B loads and stores; R, C multiples of 8).
// Makes the k-contiguous image W^T of a weight for the input-gradient GEMM dx = dy @ W, so that
// GEMM stages both operands with the LDS-DMA ring instead of hardware-transposed LDS reads.
__global__ void __launch_bounds__(256) transpose_bf16_kernel(const bf16_t* __restrict__ src, int64_t R, int64_t C,
                                                             bf16_t* __restrict__ dst) {
  __shared__ uint16_t t[64][72];
  const int64_t r0 = (int64_t)blockIdx.y * 64, c0 = (int64_t)blockIdx.x * 64;
  const int tid = threadIdx.x;
  const int c8 = (tid & 7) * 8;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int r = (tid >> 3) + 32 * h;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (r0 + r < R && c0 + c8 < C) v = *reinterpret_cast<const uint4*>(src + (r0 + r) * C + c0 + c8);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      t[r][c8 + 2 * q] = (uint16_t)(w[q] & 0xffffu);
      t[r][c8 + 2 * q + 1] = (uint16_t)(w[q] >> 16);
    }
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int c = (tid >> 3) + 32 * h;      // output row (source column)
    if (c0 + c >= C || r0 + c8 >= R) continue;
    uint32_t w[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) w[q] = (uint32_t)t[c8 + 2 * q][c] | ((uint32_t)t[c8 + 2 * q + 1][c] << 16);
    *reinterpret_cast<uint4*>(dst + (c0 + c) * R + r0 + c8) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}
}  // namespace
}  // namespace dph

extern "C" int dph_transpose_bf16(const void* src, int64_t R, int64_t C, void* dst, hipStream_t stream) {
  DPH_REQUIRE(src && dst && R > 0 && C > 0 && R % 8 == 0 && C % 8 == 0,
              "dph_transpose_bf16: bad args (R=%lld C=%lld must be multiples of 8)", (long long)R, (long long)C);
  DPH_REQUIRE(cdiv(R, 64) < 65536, "dph_transpose_bf16: too many rows");
  hipLaunchKernelGGL(dph::transpose_bf16_kernel, dim3((unsigned)cdiv(C, 64), (unsigned)cdiv(R, 64)), dim3(256), 0,
                     stream, reinterpret_cast<const bf16_t*>(src), R, C, reinterpret_cast<bf16_t*>(dst));
  return check_launch("dph_transpose_bf16");
}

namespace dph {
namespace {
// Batched image refresh after the optimizer step (one launch each instead of ~85 casts + ~50
// transposes of 1-2 M elements, each a few-us launch):
//   cast:      tab[e] = {src fp32*, dst bf16*, n}; grid (blocks, entries), grid-stride per entry
//   transpose: tab[e] = {src bf16*, dst bf16*, R, C}; grid (blocks, entries), 64x64 tiles
__global__ void __launch_bounds__(256) cast_bf16_multi_kernel(const int64_t* __restrict__ tab) {
  const int64_t* e = tab + 3 * blockIdx.y;
  const float* src = reinterpret_cast<const float*>(e[0]);
  bf16_t* dst = reinterpret_cast<bf16_t*>(e[1]);
  const int64_t n = e[2];
  for (int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4; i < n; i += (int64_t)gridDim.x * 1024) {
    if (i + 4 <= n) {
      const float4 v = *reinterpret_cast<const float4*>(src + i);
      *reinterpret_cast<uint2*>(dst + i) = make_uint2(pack2bf(v.x, v.y), pack2bf(v.z, v.w));
    } else {
      for (int64_t j = i; j < n; ++j) dst[j] = f2bf(src[j]);
    }
  }
}

//   copy:      tab[e] = {src fp32* (0: write zeros), dst fp32*, n}; grid (blocks, entries)
__global__ void __launch_bounds__(256) copy_f32_multi_kernel(const int64_t* __restrict__ tab) {
  const int64_t* e = tab + 3 * blockIdx.y;
  const float* src = reinterpret_cast<const float*>(e[0]);
  float* dst = reinterpret_cast<float*>(e[1]);
  const int64_t n = e[2];
  const bool vec = ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0;
  for (int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4; i < n; i += (int64_t)gridDim.x * 1024) {
    if (vec && i + 4 <= n) {
      *reinterpret_cast<float4*>(dst + i) = src ? *reinterpret_cast<const float4*>(src + i) : make_float4(0.f, 0.f, 0.f, 0.f);
    } else {
      for (int64_t j = i; j < n && j < i + 4; ++j) dst[j] = src ? src[j] : 0.f;
    }
  }
}

__global__ void __launch_bounds__(256) transpose_bf16_multi_kernel(const int64_t* __restrict__ tab) {
  __shared__ uint16_t t[64][72];
  const int64_t* e = tab + 4 * blockIdx.y;
  const bf16_t* src = reinterpret_cast<const bf16_t*>(e[0]);
  bf16_t* dst = reinterpret_cast<bf16_t*>(e[1]);
  const int64_t R = e[2], C = e[3];
  const int64_t ctiles = (C + 63) / 64, ntiles = ((R + 63) / 64) * ctiles;
  const int tid = threadIdx.x;
  const int c8 = (tid & 7) * 8;
  for (int64_t tt = blockIdx.x; tt < ntiles; tt += gridDim.x) {
    const int64_t r0 = (tt / ctiles) * 64, c0 = (tt % ctiles) * 64;
    __syncthreads();   // previous tile's reads done
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = (tid >> 3) + 32 * h;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (r0 + r < R && c0 + c8 < C) v = *reinterpret_cast<const uint4*>(src + (r0 + r) * C + c0 + c8);
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        t[r][c8 + 2 * q] = (uint16_t)(w[q] & 0xffffu);
        t[r][c8 + 2 * q + 1] = (uint16_t)(w[q] >> 16);
      }
    }
    __syncthreads();
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = (tid >> 3) + 32 * h;
      if (c0 + c >= C || r0 + c8 >= R) continue;
      uint32_t w[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) w[q] = (uint32_t)t[c8 + 2 * q][c] | ((uint32_t)t[c8 + 2 * q + 1][c] << 16);
      *reinterpret_cast<uint4*>(dst + (c0 + c) * R + r0 + c8) = make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
}
}  // namespace
}  // namespace dph

extern "C" int dph_cast_bf16_multi(const int64_t* table, int64_t n_entries, hipStream_t stream) {
  DPH_REQUIRE(table && n_entries > 0 && n_entries < 65536, "dph_cast_bf16_multi: bad args");
  hipLaunchKernelGGL(dph::cast_bf16_multi_kernel, dim3(64, (unsigned)n_entries), dim3(256), 0, stream, table);
  return check_launch("dph_cast_bf16_multi");
}

extern "C" int dph_copy_f32_multi(const int64_t* table, int64_t n_entries, int64_t max_n, hipStream_t stream) {
  DPH_REQUIRE(table && n_entries > 0 && n_entries < 65536 && max_n > 0, "dph_copy_f32_multi: bad args");
  const int64_t blocks = std::min<int64_t>(std::max<int64_t>(cdiv(max_n, 1024), 1), 2048);
  hipLaunchKernelGGL(dph::copy_f32_multi_kernel, dim3((unsigned)blocks, (unsigned)n_entries), dim3(256), 0, stream,
                     table);
  return check_launch("dph_copy_f32_multi");
}

extern "C" int dph_transpose_bf16_multi(const int64_t* table, int64_t n_entries, hipStream_t stream) {
  DPH_REQUIRE(table && n_entries > 0 && n_entries < 65536, "dph_transpose_bf16_multi: bad args");
  hipLaunchKernelGGL(dph::transpose_bf16_multi_kernel, dim3(128, (unsigned)n_entries), dim3(256), 0, stream, table);
  return check_launch("dph_transpose_bf16_multi");
}

namespace dph {
namespace {
struct ConvGeom {
  int32_t k[16], s[16];
  int32_t n;
};
// frame lengths through the conv stack (components.py:179-181 per layer:
// L = max(0, floor((L - k) / s) + 1)), all layers in one launch
__global__ void conv_lengths_kernel(const int64_t* __restrict__ in, int64_t* __restrict__ out, int64_t n, ConvGeom g) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int64_t L = in[i];
  for (int l = 0; l < g.n; ++l) {
    const int64_t d = L - g.k[l];
    const int64_t q = d >= 0 ? d / g.s[l] : -((-d + g.s[l] - 1) / g.s[l]);   // floor division
    L = q + 1 > 0 ? q + 1 : 0;
  }
  out[i] = L;
}
}  // namespace
}  // namespace dph

extern "C" int dph_conv_lengths(const int64_t* len_in, int64_t* len_out, int64_t n, int64_t n_layers,
                                const int32_t* kernel_sizes, const int32_t* strides, hipStream_t stream) {
  DPH_REQUIRE(len_in && len_out && n > 0 && n_layers > 0 && n_layers <= 16 && kernel_sizes && strides,
              "dph_conv_lengths: bad args");
  dph::ConvGeom g{};
  for (int64_t l = 0; l < n_layers; ++l) {
    DPH_REQUIRE(strides[l] > 0, "dph_conv_lengths: stride must be > 0");
    g.k[l] = kernel_sizes[l];
    g.s[l] = strides[l];
  }
  g.n = (int32_t)n_layers;
  hipLaunchKernelGGL(dph::conv_lengths_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, stream, len_in, len_out, n, g);
  return check_launch("dph_conv_lengths");
}

namespace dph {
namespace {
// y = GELU(h) * mask[c] over a dense [rows][C] bf16 tensor (layer_norm-mode conv layers,
// components.py:110-114 after the LayerNorm); 8 columns per thread
__global__ void __launch_bounds__(256) gelu_mask_fwd_kernel(const bf16_t* __restrict__ h, const float* __restrict__ mask,
                                                            bf16_t* __restrict__ y, int64_t rows, int64_t C) {
  const int64_t c8n = C / 8;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * c8n) return;
  const int64_t c0 = (i % c8n) * 8;
  const uint4 v = *reinterpret_cast<const uint4*>(h + i * 8);
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t o[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float a = gelu_f(__uint_as_float(w[q] << 16)) * (mask ? mask[c0 + 2 * q] : 1.f);
    const float b = gelu_f(__uint_as_float(w[q] & 0xffff0000u)) * (mask ? mask[c0 + 2 * q + 1] : 1.f);
    o[q] = pack2bf(a, b);
  }
  *reinterpret_cast<uint4*>(y + i * 8) = make_uint4(o[0], o[1], o[2], o[3]);
}
}  // namespace
}  // namespace dph

extern "C" int dph_gelu_mask_fwd(const void* h, const float* mask, void* y, int64_t rows, int64_t C,
                                 hipStream_t stream) {
  DPH_REQUIRE(h && y && rows > 0 && C > 0 && C % 8 == 0, "dph_gelu_mask_fwd: bad args (C %% 8 == 0 required)");
  hipLaunchKernelGGL(dph::gelu_mask_fwd_kernel, dim3((unsigned)cdiv(rows * (C / 8), 256)), dim3(256), 0, stream,
                     reinterpret_cast<const bf16_t*>(h), mask, reinterpret_cast<bf16_t*>(y), rows, C);
  return check_launch("dph_gelu_mask_fwd");
}

extern "C" int dph_cast_bf16(const float* src, void* dst, int64_t n, hipStream_t stream) {
  DPH_REQUIRE(src && dst && n > 0, "dph_cast_bf16: bad args");
  hipLaunchKernelGGL(cast_bf16_kernel, dim3((unsigned)cdiv(cdiv(n, 4), 256)), dim3(256), 0, stream, src,
                     reinterpret_cast<bf16_t*>(dst), n);
  return check_launch("dph_cast_bf16");
}

extern "C" int dph_conv_weight_pack(const float* w, void* dst, int64_t O, int64_t C, int64_t k, int64_t Op,
                                    int64_t Cp, hipStream_t stream) {
  DPH_REQUIRE(w && dst && O > 0 && C > 0 && k > 0 && Op >= O && Cp >= C, "dph_conv_weight_pack: bad args");
  hipLaunchKernelGGL(conv_pack_kernel, dim3((unsigned)cdiv(Op * Cp * k, 256)), dim3(256), 0, stream, w,
                     reinterpret_cast<bf16_t*>(dst), O, C, k, Op, Cp);
  return check_launch("dph_conv_weight_pack");
}

extern "C" int dph_conv_weight_unpack_grad(const float* g, float* dst, int64_t O, int64_t C, int64_t k, int64_t Cp,
                                           int accum, hipStream_t stream) {
  DPH_REQUIRE(g && dst && O > 0 && C > 0 && k > 0 && Cp >= C, "dph_conv_weight_unpack_grad: bad args");
  hipLaunchKernelGGL(conv_unpack_kernel, dim3((unsigned)cdiv(O * C * k, 256)), dim3(256), 0, stream, g, dst, O, C, k,
                     Cp, accum);
  return check_launch("dph_conv_weight_unpack_grad");
}

extern "C" int dph_add_bf16(const void* a, const void* b, void* out, int64_t n, hipStream_t stream) {
  DPH_REQUIRE(a && b && out && n > 0, "dph_add_bf16: bad args");
  hipLaunchKernelGGL(add_bf16_kernel, dim3((unsigned)cdiv(cdiv(n, 8), 256)), dim3(256), 0, stream,
                     reinterpret_cast<const bf16_t*>(a), reinterpret_cast<const bf16_t*>(b),
                     reinterpret_cast<bf16_t*>(out), n);
  return check_launch("dph_add_bf16");
}

extern "C" int dph_branch_bwd(const void* dy, void* out, int64_t rows, int64_t cols, float p, uint64_t seed,
                              const float* smask, const int64_t* row_len, int64_t len_rows, float* colsum,
                              const void* pre, float* sdot, float* ws, int64_t ws_bytes, hipStream_t stream) {
  DPH_REQUIRE(dy && out && rows > 0 && cols > 0, "dph_branch_bwd: bad args");
  DPH_REQUIRE(!row_len || len_rows > 0, "dph_branch_bwd: row_len needs len_rows");
  DPH_REQUIRE(!sdot || pre, "dph_branch_bwd: sdot needs pre");
  int64_t rpb;
  float* part;
  if (int rc = rowblock_plan(rows, cols, colsum || sdot, ws, ws_bytes, rpb, part, "dph_branch_bwd")) return rc;
  const int64_t nrb = cdiv(rows, rpb);
  dim3 grid((unsigned)cdiv(cols, 512), (unsigned)nrb);
  hipLaunchKernelGGL((branch_bwd_kernel<bf16_t, bf16_t>), grid, dim3(256), 0, stream,
                     reinterpret_cast<const bf16_t*>(dy), reinterpret_cast<bf16_t*>(out), rows, cols, p, seed, smask,
                     row_len, len_rows, colsum, reinterpret_cast<const bf16_t*>(pre), sdot, rpb, part);
  if (part && colsum) DPH_TRY(slab_reduce_cols(part, nrb, cols, cols, colsum, nullptr, nullptr, stream));
  if (part && sdot) sdot_reduce(part + nrb * cols, nrb * (int64_t)grid.x, sdot, stream);
  return check_launch("dph_branch_bwd");
}

extern "C" int dph_branch_bwd_f32(const float* dy, void* out, int out_f32, int64_t rows, int64_t cols, float p,
                                  uint64_t seed, const float* smask, const int64_t* row_len, int64_t len_rows,
                                  float* colsum, const void* pre, float* sdot, float* ws, int64_t ws_bytes,
                                  hipStream_t stream) {
  DPH_REQUIRE(dy && out && rows > 0 && cols > 0, "dph_branch_bwd_f32: bad args");
  DPH_REQUIRE(!row_len || len_rows > 0, "dph_branch_bwd_f32: row_len needs len_rows");
  DPH_REQUIRE(!sdot || pre, "dph_branch_bwd_f32: sdot needs pre");
  int64_t rpb;
  float* part;
  if (int rc = rowblock_plan(rows, cols, colsum || sdot, ws, ws_bytes, rpb, part, "dph_branch_bwd_f32")) return rc;
  const int64_t nrb = cdiv(rows, rpb);
  dim3 grid((unsigned)cdiv(cols, 512), (unsigned)nrb);
  if (out_f32)
    hipLaunchKernelGGL((branch_bwd_kernel<float, float>), grid, dim3(256), 0, stream, dy,
                       reinterpret_cast<float*>(out), rows, cols, p, seed, smask, row_len, len_rows, colsum,
                       reinterpret_cast<const bf16_t*>(pre), sdot, rpb, part);
  else
    hipLaunchKernelGGL((branch_bwd_kernel<float, bf16_t>), grid, dim3(256), 0, stream, dy,
                       reinterpret_cast<bf16_t*>(out), rows, cols, p, seed, smask, row_len, len_rows, colsum,
                       reinterpret_cast<const bf16_t*>(pre), sdot, rpb, part);
  if (part && colsum) DPH_TRY(slab_reduce_cols(part, nrb, cols, cols, colsum, nullptr, nullptr, stream));
  if (part && sdot) sdot_reduce(part + nrb * cols, nrb * (int64_t)grid.x, sdot, stream);
  return check_launch("dph_branch_bwd_f32");
}
