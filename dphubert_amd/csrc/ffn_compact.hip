// FFN intermediate units with an exactly-zero HardConcrete mask (hardconcrete.py:99 clamps the stretched sample
// to [0, 1]): such a unit contributes nothing to the layer output and gets no gradient through its mask
// (components.py:733-741 forward: f = gelu(x W1^T + b1) * mask).  The encoder layer then runs its FFN GEMMs over
// the ACTIVE units only, packed to the front of [Fc]-wide images, with device-side extents: the step graph is
// captured once, so the active count never reaches the host -- the GEMMs read it (DphGemmArgs.dyn_ext) and skip
// the tiles / K-tiles past it.
//
//   dph_ffn_compact   mask [F] -> idx [Fc] (active units in order), ext = the GEMM extents:
//                     ext[0..2] = {0, keff, 0} (N dynamic), ext[3..5] = {0, 0, keff} (K dynamic),
//                     ext[6..8] = {keff, 0, 0} (M dynamic), ext[9] = n_active;
//                     keff = max(128, n_active rounded up to 64) <= Fc (the packed images are zero past n_active,
//                     so the padding K-tiles and columns contribute exactly 0)
//   gathers           W1 rows, W2 columns (and the transposed images), b1 / mask  -> packed, zero padded
//   scatters          dW1 rows, dW2 columns, db1 / dmask of the packed units -> the full-width gradients
#include "common.h"

#include <algorithm>

namespace dph {
namespace {

constexpr int CT = 1024;   // compaction block (F <= 8 * CT)

__global__ void __launch_bounds__(CT) ffn_compact_kernel(const float* __restrict__ mask, int F, int Fc,
                                                         int32_t* __restrict__ idx, int32_t* __restrict__ ext) {
  __shared__ int wsum[CT / 64];
  __shared__ int base_s;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (tid == 0) base_s = 0;
  __syncthreads();
  for (int c0 = 0; c0 < F; c0 += CT) {
    const int i = c0 + tid;
    const bool act = i < F && mask[i] != 0.f;
    const uint64_t bal = __ballot(act);
    const int pre = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) wsum[w] = __popcll(bal);
    __syncthreads();
    int off = base_s;
    for (int k = 0; k < w; ++k) off += wsum[k];
    if (act) idx[off + pre] = i;
    __syncthreads();
    if (tid == 0) {
      int t = 0;
      for (int k = 0; k < CT / 64; ++k) t += wsum[k];
      base_s += t;
    }
    __syncthreads();
  }
  const int n = base_s;
  for (int j = n + tid; j < Fc; j += CT) idx[j] = -1;
  if (tid == 0) {
    int keff = ((n + 63) / 64) * 64;
    keff = keff < 128 ? 128 : keff;
    keff = keff > Fc ? Fc : keff;
    ext[0] = 0; ext[1] = keff; ext[2] = 0;
    ext[3] = 0; ext[4] = 0; ext[5] = keff;
    ext[6] = keff; ext[7] = 0; ext[8] = 0;
    ext[9] = n;
  }
}

// dst[j][0:cols] = src[idx[j]][0:cols] (bf16, 16-B chunks), zero rows past n_active
__global__ void __launch_bounds__(256) gather_rows_bf16_kernel(const bf16_t* __restrict__ src, int64_t ld_src,
                                                               const int32_t* __restrict__ idx, bf16_t* __restrict__ dst,
                                                               int64_t rows, int64_t cols) {
  const int64_t c8 = cols / 8;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= rows * c8) return;
  const int64_t j = e / c8, c = (e - j * c8) * 8;
  const int32_t r = idx[j];
  uint4 v = make_uint4(0, 0, 0, 0);
  if (r >= 0) v = *reinterpret_cast<const uint4*>(src + (int64_t)r * ld_src + c);
  *reinterpret_cast<uint4*>(dst + j * cols + c) = v;
}

// dst[r][j] = src[r][idx[j]] (bf16), zero columns past n_active; one thread per 2 output columns
__global__ void __launch_bounds__(256) gather_cols_bf16_kernel(const bf16_t* __restrict__ src, int64_t ld_src,
                                                               const int32_t* __restrict__ idx, bf16_t* __restrict__ dst,
                                                               int64_t rows, int64_t Fc) {
  const int64_t h = Fc / 2;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= rows * h) return;
  const int64_t r = e / h, j = (e - r * h) * 2;
  const int32_t i0 = idx[j], i1 = idx[j + 1];
  const bf16_t* s = src + r * ld_src;
  const uint32_t lo = i0 >= 0 ? (uint32_t)reinterpret_cast<const uint16_t*>(s)[i0] : 0u;
  const uint32_t hi = i1 >= 0 ? (uint32_t)reinterpret_cast<const uint16_t*>(s)[i1] : 0u;
  *reinterpret_cast<uint32_t*>(dst + r * Fc + j) = lo | (hi << 16);
}

__global__ void __launch_bounds__(256) gather_vec_f32_kernel(const float* __restrict__ src,
                                                             const int32_t* __restrict__ idx, float* __restrict__ dst,
                                                             int64_t Fc) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= Fc) return;
  const int32_t i = idx[j];
  dst[j] = (i >= 0 && src) ? src[i] : 0.f;
}

// dst[idx[j]][0:cols] (+)= src[j][0:cols] (fp32; active units are distinct: no atomics)
__global__ void __launch_bounds__(256) scatter_rows_f32_kernel(const float* __restrict__ src,
                                                               const int32_t* __restrict__ idx, float* __restrict__ dst,
                                                               int64_t ld_dst, int64_t rows, int64_t cols, int accum) {
  const int64_t c4 = cols / 4;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= rows * c4) return;
  const int64_t j = e / c4, c = (e - j * c4) * 4;
  const int32_t r = idx[j];
  if (r < 0) return;
  float4 v = *reinterpret_cast<const float4*>(src + j * cols + c);
  float4* d = reinterpret_cast<float4*>(dst + (int64_t)r * ld_dst + c);
  if (accum) {
    const float4 o = *d;
    v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
  }
  *d = v;
}

// dst[r][idx[j]] (+)= src[r][j] (fp32)
__global__ void __launch_bounds__(256) scatter_cols_f32_kernel(const float* __restrict__ src,
                                                               const int32_t* __restrict__ idx, float* __restrict__ dst,
                                                               int64_t ld_dst, int64_t rows, int64_t Fc, int accum) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= rows * Fc) return;
  const int64_t r = e / Fc, j = e - r * Fc;
  const int32_t i = idx[j];
  if (i < 0) return;
  const float v = src[r * Fc + j];
  float* d = dst + r * ld_dst + i;
  *d = accum ? *d + v : v;
}

// All packed images of a layer in ONE launch (blockIdx.y = job, grid-stride over blockIdx.x): the FFN GEMM
// operands of the forward AND the backward (W1 rows, W2 columns, W2^T rows, W1^T columns, b1 / mask), built
// once per forward -- one launch instead of six (each small gather cost a launch's worth of GPU time).
struct FfnPack {
  const bf16_t *w1, *w2, *w2t, *w1t;   // [Fp][D], [D][Fp], [Fp][D], [D][Fp] (w2t / w1t may be null)
  const float *b1, *mask;              // [Fp] (b1 may be null: zeros)
  bf16_t *w1g, *w2g, *w2gt, *w1gt;     // [Fc][D], [D][Fc], [Fc][D], [D][Fc]
  float *b1g, *mg;                     // [Fc]
  int64_t Fp, Fc, D;
};

__global__ void __launch_bounds__(256) ffn_pack_kernel(const FfnPack p, const int32_t* __restrict__ idx) {
  const int job = blockIdx.y;
  const int64_t stride = (int64_t)gridDim.x * 256;
  const int64_t t0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (job == 0 || job == 2) {                       // row gathers, 16-B chunks
    const bf16_t* src = job == 0 ? p.w1 : p.w2t;
    bf16_t* dst = job == 0 ? p.w1g : p.w2gt;
    if (!src) return;
    const int64_t c8 = p.D / 8, n = p.Fc * c8;
    for (int64_t e = t0; e < n; e += stride) {
      const int64_t j = e / c8, c = (e - j * c8) * 8;
      const int32_t r = idx[j];
      uint4 v = make_uint4(0, 0, 0, 0);
      if (r >= 0) v = *reinterpret_cast<const uint4*>(src + (int64_t)r * p.D + c);
      *reinterpret_cast<uint4*>(dst + j * p.D + c) = v;
    }
  } else if (job == 1 || job == 3) {                // column gathers, 2 columns per thread
    const bf16_t* src = job == 1 ? p.w2 : p.w1t;
    bf16_t* dst = job == 1 ? p.w2g : p.w1gt;
    if (!src) return;
    const int64_t h = p.Fc / 2, n = p.D * h;
    for (int64_t e = t0; e < n; e += stride) {
      const int64_t r = e / h, j = (e - r * h) * 2;
      const int32_t i0 = idx[j], i1 = idx[j + 1];
      const uint16_t* srow = reinterpret_cast<const uint16_t*>(src + r * p.Fp);
      const uint32_t lo = i0 >= 0 ? (uint32_t)srow[i0] : 0u, hi = i1 >= 0 ? (uint32_t)srow[i1] : 0u;
      *reinterpret_cast<uint32_t*>(dst + r * p.Fc + j) = lo | (hi << 16);
    }
  } else {                                          // vectors
    for (int64_t j = t0; j < p.Fc; j += stride) {
      const int32_t i = idx[j];
      p.b1g[j] = (i >= 0 && p.b1) ? p.b1[i] : 0.f;
      p.mg[j] = i >= 0 ? p.mask[i] : 0.f;
    }
  }
}

// The packed gradients back to the full-width ones, one launch: dW2 columns, dW1 rows, db1, dmask (accumulate)
struct FfnUnpack {
  const float *dw2g, *dw1g, *db1g, *dmg;   // [D][Fc], [Fc][D], [Fc], [Fc]
  float *dw2, *dw1, *db1, *dm;             // [D][F] (row stride ld2), [F][D], [F], [F]
  int64_t ld2, Fc, D;
};

__global__ void __launch_bounds__(256) ffn_unpack_kernel(const FfnUnpack p, const int32_t* __restrict__ idx) {
  const int job = blockIdx.y;
  const int64_t stride = (int64_t)gridDim.x * 256;
  const int64_t t0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (job == 0) {
    const int64_t n = p.D * p.Fc;
    for (int64_t e = t0; e < n; e += stride) {
      const int64_t r = e / p.Fc, j = e - r * p.Fc;
      const int32_t i = idx[j];
      if (i >= 0) p.dw2[r * p.ld2 + i] += p.dw2g[e];
    }
  } else if (job == 1) {
    const int64_t c4 = p.D / 4, n = p.Fc * c4;
    for (int64_t e = t0; e < n; e += stride) {
      const int64_t j = e / c4, c = (e - j * c4) * 4;
      const int32_t r = idx[j];
      if (r < 0) continue;
      const float4 v = *reinterpret_cast<const float4*>(p.dw1g + j * p.D + c);
      float4* d = reinterpret_cast<float4*>(p.dw1 + (int64_t)r * p.D + c);
      float4 o = *d;
      o.x += v.x; o.y += v.y; o.z += v.z; o.w += v.w;
      *d = o;
    }
  } else {
    for (int64_t j = t0; j < p.Fc; j += stride) {
      const int32_t i = idx[j];
      if (i < 0) continue;
      if (p.db1) p.db1[i] += p.db1g[j];
      if (p.dm) p.dm[i] += p.dmg[j];
    }
  }
}

}  // namespace
}  // namespace dph

using namespace dph;

extern "C" int dph_ffn_pack(const void* w1, const void* w2, const void* w2t, const void* w1t, const float* b1,
                            const float* mask, const int32_t* idx, void* w1g, void* w2g, void* w2gt, void* w1gt,
                            float* b1g, float* mg, int64_t Fp, int64_t Fc, int64_t D, hipStream_t stream) {
  DPH_REQUIRE(w1 && w2 && mask && idx && w1g && w2g && b1g && mg && (!w2t || w2gt) && (!w1t || w1gt),
              "dph_ffn_pack: null pointer");
  DPH_REQUIRE(D % 8 == 0 && Fc % 64 == 0 && Fc >= Fp && Fp % 2 == 0, "dph_ffn_pack: D=%lld Fp=%lld Fc=%lld",
              (long long)D, (long long)Fp, (long long)Fc);
  const FfnPack p{reinterpret_cast<const bf16_t*>(w1), reinterpret_cast<const bf16_t*>(w2),
                  reinterpret_cast<const bf16_t*>(w2t), reinterpret_cast<const bf16_t*>(w1t), b1, mask,
                  reinterpret_cast<bf16_t*>(w1g), reinterpret_cast<bf16_t*>(w2g), reinterpret_cast<bf16_t*>(w2gt),
                  reinterpret_cast<bf16_t*>(w1gt), b1g, mg, Fp, Fc, D};
  const int64_t work = std::max<int64_t>(Fc * (D / 8), D * (Fc / 2));
  const unsigned gx = (unsigned)std::min<int64_t>(cdiv(work, 256), 1024);
  hipLaunchKernelGGL(ffn_pack_kernel, dim3(gx, 5), dim3(256), 0, stream, p, idx);
  return check_launch("dph_ffn_pack");
}

extern "C" int dph_ffn_unpack_grads(const float* dw2g, const float* dw1g, const float* db1g, const float* dmg,
                                    const int32_t* idx, float* dw2, int64_t ld2, float* dw1, float* db1, float* dm,
                                    int64_t Fc, int64_t D, hipStream_t stream) {
  DPH_REQUIRE(dw2g && dw1g && db1g && dmg && idx && dw2 && dw1 && D % 4 == 0,
              "dph_ffn_unpack_grads: null pointer or D %% 4 != 0");
  const FfnUnpack p{dw2g, dw1g, db1g, dmg, dw2, dw1, db1, dm, ld2, Fc, D};
  const unsigned gx = (unsigned)std::min<int64_t>(cdiv(D * Fc, 256), 1024);
  hipLaunchKernelGGL(ffn_unpack_kernel, dim3(gx, 3), dim3(256), 0, stream, p, idx);
  return check_launch("dph_ffn_unpack_grads");
}

extern "C" int dph_ffn_compact(const float* mask, int64_t F, int64_t Fc, int32_t* idx, int32_t* ext,
                               hipStream_t stream) {
  DPH_REQUIRE(mask && idx && ext, "dph_ffn_compact: null pointer");
  DPH_REQUIRE(F > 0 && F <= 8 * CT && Fc >= F && Fc % 64 == 0 && Fc >= 128,
              "dph_ffn_compact: F=%lld Fc=%lld (Fc % 64 == 0, Fc >= max(F, 128), F <= %d)", (long long)F,
              (long long)Fc, 8 * CT);
  hipLaunchKernelGGL(ffn_compact_kernel, dim3(1), dim3(CT), 0, stream, mask, (int)F, (int)Fc, idx, ext);
  return check_launch("dph_ffn_compact");
}

extern "C" int dph_gather_rows_bf16(const void* src, int64_t ld_src, const int32_t* idx, void* dst, int64_t rows,
                                    int64_t cols, hipStream_t stream) {
  DPH_REQUIRE(src && idx && dst && cols % 8 == 0 && ld_src % 8 == 0 && rows > 0,
              "dph_gather_rows_bf16: cols=%lld ld=%lld (multiples of 8)", (long long)cols, (long long)ld_src);
  const int64_t n = rows * (cols / 8);
  hipLaunchKernelGGL(gather_rows_bf16_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, stream,
                     reinterpret_cast<const bf16_t*>(src), ld_src, idx, reinterpret_cast<bf16_t*>(dst), rows, cols);
  return check_launch("dph_gather_rows_bf16");
}

extern "C" int dph_gather_cols_bf16(const void* src, int64_t ld_src, const int32_t* idx, void* dst, int64_t rows,
                                    int64_t Fc, hipStream_t stream) {
  DPH_REQUIRE(src && idx && dst && Fc % 2 == 0 && rows > 0, "dph_gather_cols_bf16: Fc=%lld (even)", (long long)Fc);
  const int64_t n = rows * (Fc / 2);
  hipLaunchKernelGGL(gather_cols_bf16_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, stream,
                     reinterpret_cast<const bf16_t*>(src), ld_src, idx, reinterpret_cast<bf16_t*>(dst), rows, Fc);
  return check_launch("dph_gather_cols_bf16");
}

extern "C" int dph_gather_vec_f32(const float* src, const int32_t* idx, float* dst, int64_t Fc, hipStream_t stream) {
  DPH_REQUIRE(idx && dst && Fc > 0, "dph_gather_vec_f32: null pointer");
  hipLaunchKernelGGL(gather_vec_f32_kernel, dim3((unsigned)cdiv(Fc, 256)), dim3(256), 0, stream, src, idx, dst, Fc);
  return check_launch("dph_gather_vec_f32");
}

extern "C" int dph_scatter_rows_f32(const float* src, const int32_t* idx, float* dst, int64_t ld_dst, int64_t rows,
                                    int64_t cols, int accumulate, hipStream_t stream) {
  DPH_REQUIRE(src && idx && dst && cols % 4 == 0 && ld_dst % 4 == 0 && rows > 0,
              "dph_scatter_rows_f32: cols=%lld ld=%lld (multiples of 4)", (long long)cols, (long long)ld_dst);
  const int64_t n = rows * (cols / 4);
  hipLaunchKernelGGL(scatter_rows_f32_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, stream, src, idx, dst,
                     ld_dst, rows, cols, accumulate);
  return check_launch("dph_scatter_rows_f32");
}

extern "C" int dph_scatter_cols_f32(const float* src, const int32_t* idx, float* dst, int64_t ld_dst, int64_t rows,
                                    int64_t Fc, int accumulate, hipStream_t stream) {
  DPH_REQUIRE(src && idx && dst && rows > 0 && Fc > 0, "dph_scatter_cols_f32: null pointer");
  const int64_t n = rows * Fc;
  hipLaunchKernelGGL(scatter_cols_f32_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, stream, src, idx, dst,
                     ld_dst, rows, Fc, accumulate);
  return check_launch("dph_scatter_cols_f32");
}
