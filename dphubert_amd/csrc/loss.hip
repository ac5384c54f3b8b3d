// Layer-wise distillation loss (lightning.py:116-139) forward + backward.
//
// s: student projections, fp32, layer-major [L][B][T][D] (the rows of
//    torch.stack(dim=1) of lightning.py:263 in another order; the loss is a
//    mean over rows, so the order does not matter);
// t: teacher hidden states, bf16, L separate [B][T][D] buffers
//    (= torch.stack of lightning.py:250-252 without the copy).
// loss = l2w*mean((s-t)^2) + l1w*mean|s-t| + cosw*(-mean cos)            (raw)
//                                          + cosw*(-mean log sigmoid(cos)) (log_sig)
// cos = s.t / (max(|s|,eps) * max(|t|,eps)), eps = 1e-8 (nn.CosineSimilarity).
// One wave per (b, l, t) row; row statistics are kept for the backward.
#include "common.h"

namespace dph {
namespace {

// teacher layer l is bf16, or fp32 when bit l of f32 is set (the fp32 residual stream of pre-norm encoders)
struct TPtrs {
  const void* p[DPH_MAX_DISTILL_LAYERS];
  uint32_t f32;
};

__device__ __forceinline__ void load_t4(const TPtrs& tp, int64_t l, int64_t off, float (&o)[4]) {
  if ((tp.f32 >> l) & 1u) {
    const float4 v = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(tp.p[l]) + off);
    o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
  } else {
    const uint2 v = *reinterpret_cast<const uint2*>(reinterpret_cast<const bf16_t*>(tp.p[l]) + off);
    o[0] = __uint_as_float(v.x << 16); o[1] = __uint_as_float(v.x & 0xffff0000u);
    o[2] = __uint_as_float(v.y << 16); o[3] = __uint_as_float(v.y & 0xffff0000u);
  }
}

constexpr float COS_EPS = 1e-8f;

__device__ __forceinline__ float log_sigmoid(float x) { return x >= 0.f ? -log1pf(__expf(-x)) : x - log1pf(__expf(x)); }

__global__ void __launch_bounds__(256) loss_fwd_kernel(const float* __restrict__ s, TPtrs tp, int64_t B, int64_t L,
                                                       int64_t T, int64_t D, int cos_logsig,
                                                       float* __restrict__ rowstats, float* __restrict__ partial) {
  __shared__ float red[4][3];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int64_t rows = B * L * T;
  float l1 = 0.f, l2 = 0.f, cterm = 0.f;
  for (int64_t row = (int64_t)blockIdx.x * 4 + wave; row < rows; row += (int64_t)gridDim.x * 4) {
    const int64_t t = row % T;
    const int64_t b = (row / T) % B;
    const int64_t l = row / (T * B);
    const float* sr = s + row * D;
    const int64_t toff = (b * T + t) * D;
    float dot = 0.f, ns = 0.f, nt = 0.f;
    for (int64_t c = lane * 4; c < D; c += 256) {
      const float4 sv = *reinterpret_cast<const float4*>(sr + c);
      const float a[4] = {sv.x, sv.y, sv.z, sv.w};
      float bb[4];
      load_t4(tp, l, toff + c, bb);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float d = a[i] - bb[i];
        l1 += fabsf(d);
        l2 += d * d;
        dot += a[i] * bb[i];
        ns += a[i] * a[i];
        nt += bb[i] * bb[i];
      }
    }
    dot = wave_sum(dot);
    ns = wave_sum(ns);
    nt = wave_sum(nt);
    const float cs = dot / (fmaxf(sqrtf(ns), COS_EPS) * fmaxf(sqrtf(nt), COS_EPS));
    cterm += cos_logsig ? log_sigmoid(cs) : cs;
    if (lane == 0) {
      rowstats[row * 3 + 0] = dot;
      rowstats[row * 3 + 1] = ns;
      rowstats[row * 3 + 2] = nt;
    }
  }
  l1 = wave_sum(l1);
  l2 = wave_sum(l2);
  if (lane == 0) {
    red[wave][0] = l1;
    red[wave][1] = l2;
    red[wave][2] = cterm;
  }
  __syncthreads();
  // one partial triple per block (no atomics: the finalize kernel sums them in a fixed order)
  if (threadIdx.x < 3)
    partial[blockIdx.x * 3 + threadIdx.x] =
        red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
}

// one wave: sums the nblk partial triples in a fixed order
__global__ void __launch_bounds__(64) loss_finalize_kernel(const float* __restrict__ partial, int64_t nblk, int64_t rows,
                                                           int64_t nel, float l2w, float l1w, float cosw,
                                                           float* __restrict__ out) {
  const float s_l1 = sum_partials_wave(partial + 0, nblk, 3);
  const float s_l2 = sum_partials_wave(partial + 1, nblk, 3);
  const float s_c = sum_partials_wave(partial + 2, nblk, 3);
  if (threadIdx.x != 0) return;
  const float mse = s_l2 / (float)nel;
  const float l1 = s_l1 / (float)nel;
  const float cos = -s_c / (float)rows;
  out[1] = l2w != 0.f ? mse : 0.f;
  out[2] = l1w != 0.f ? l1 : 0.f;
  out[3] = cosw != 0.f ? cos : 0.f;
  out[0] = l2w * out[1] + l1w * out[2] + cosw * out[3];
}

__global__ void __launch_bounds__(256) loss_bwd_kernel(const float* __restrict__ s, TPtrs tp,
                                                       const float* __restrict__ rowstats,
                                                       const float* __restrict__ dloss, int64_t B, int64_t L,
                                                       int64_t T, int64_t D, float l2w, float l1w, float cosw,
                                                       int cos_logsig, bf16_t* __restrict__ ds) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int64_t rows = B * L * T;
  const int64_t row = (int64_t)blockIdx.x * 4 + wave;
  if (row >= rows) return;
  const int64_t t = row % T;
  const int64_t b = (row / T) % B;
  const int64_t l = row / (T * B);
  const float g = dloss ? *dloss : 1.0f;
  const float nel = (float)(rows * D);
  const float dot = rowstats[row * 3 + 0];
  const float ns_ = fmaxf(sqrtf(rowstats[row * 3 + 1]), COS_EPS);
  const float nt_ = fmaxf(sqrtf(rowstats[row * 3 + 2]), COS_EPS);
  const float cs = dot / (ns_ * nt_);
  // d(-mean f(cos))/dcos
  float fc = -1.0f / (float)rows;
  if (cos_logsig) fc *= 1.0f / (1.0f + __expf(cs));   // d log sigmoid(x)/dx = sigmoid(-x)
  fc *= cosw;
  const float ca = fc / (ns_ * nt_);          // coefficient of t
  const float cb = fc * cs / (ns_ * ns_);     // coefficient of s
  const float* sr = s + row * D;
  const int64_t toff = (b * T + t) * D;
  bf16_t* dr = ds + row * D;
  for (int64_t c = lane * 4; c < D; c += 256) {
    const float4 sv = *reinterpret_cast<const float4*>(sr + c);
    const float a[4] = {sv.x, sv.y, sv.z, sv.w};
    float bb[4];
    load_t4(tp, l, toff + c, bb);
    float o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float d = a[i] - bb[i];
      const float sg = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
      o[i] = g * (l2w * 2.f * d / nel + l1w * sg / nel + ca * bb[i] - cb * a[i]);
    }
    *reinterpret_cast<uint2*>(dr + c) = make_uint2(pack2bf(o[0], o[1]), pack2bf(o[2], o[3]));
  }
}

}  // namespace
}  // namespace dph

using namespace dph;

extern "C" int dph_distill_loss_fwd_ex(const float* s, const void* const* t_layers, uint32_t t_f32_mask, int64_t B,
                                       int64_t L, int64_t T, int64_t D, float l2w, float l1w, float cosw,
                                       int cos_logsig, float* rowstats, float* partial, float* out,
                                       hipStream_t stream) {
  DPH_REQUIRE(s && t_layers && rowstats && partial && out, "dph_distill_loss_fwd: null pointer");
  DPH_REQUIRE(L >= 1 && L <= DPH_MAX_DISTILL_LAYERS && D % 4 == 0 && B > 0 && T > 0,
              "dph_distill_loss_fwd: unsupported L=%lld D=%lld", (long long)L, (long long)D);
  TPtrs tp;
  for (int i = 0; i < DPH_MAX_DISTILL_LAYERS; ++i) tp.p[i] = i < L ? t_layers[i] : nullptr;
  tp.f32 = t_f32_mask;
  const int64_t rows = B * L * T;
  const int64_t nblk = std::min<int64_t>(cdiv(rows, 4), DPH_LOSS_PARTIAL_FLOATS / 3);
  hipLaunchKernelGGL(loss_fwd_kernel, dim3((unsigned)nblk), dim3(256), 0, stream, s, tp, B, L, T, D, cos_logsig, rowstats,
                     partial);
  hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(64), 0, stream, partial, nblk, rows, rows * D, l2w, l1w, cosw,
                     out);
  return check_launch("dph_distill_loss_fwd");
}

extern "C" int dph_distill_loss_fwd(const float* s, const void* const* t_layers, int64_t B, int64_t L, int64_t T,
                                    int64_t D, float l2w, float l1w, float cosw, int cos_logsig, float* rowstats,
                                    float* partial, float* out, hipStream_t stream) {
  return dph_distill_loss_fwd_ex(s, t_layers, 0u, B, L, T, D, l2w, l1w, cosw, cos_logsig, rowstats, partial, out,
                                 stream);
}

extern "C" int dph_distill_loss_bwd_ex(const float* s, const void* const* t_layers, uint32_t t_f32_mask,
                                       const float* rowstats, const float* dloss, int64_t B, int64_t L, int64_t T,
                                       int64_t D, float l2w, float l1w, float cosw, int cos_logsig, void* ds,
                                       hipStream_t stream) {
  DPH_REQUIRE(s && t_layers && rowstats && ds, "dph_distill_loss_bwd: null pointer");
  DPH_REQUIRE(L >= 1 && L <= DPH_MAX_DISTILL_LAYERS && D % 4 == 0, "dph_distill_loss_bwd: unsupported");
  TPtrs tp;
  for (int i = 0; i < DPH_MAX_DISTILL_LAYERS; ++i) tp.p[i] = i < L ? t_layers[i] : nullptr;
  tp.f32 = t_f32_mask;
  const int64_t rows = B * L * T;
  hipLaunchKernelGGL(loss_bwd_kernel, dim3((unsigned)cdiv(rows, 4)), dim3(256), 0, stream, s, tp, rowstats, dloss, B, L,
                     T, D, l2w, l1w, cosw, cos_logsig, reinterpret_cast<bf16_t*>(ds));
  return check_launch("dph_distill_loss_bwd");
}

extern "C" int dph_distill_loss_bwd(const float* s, const void* const* t_layers, const float* rowstats,
                                    const float* dloss, int64_t B, int64_t L, int64_t T, int64_t D, float l2w,
                                    float l1w, float cosw, int cos_logsig, void* ds, hipStream_t stream) {
  return dph_distill_loss_bwd_ex(s, t_layers, 0u, rowstats, dloss, B, L, T, D, l2w, l1w, cosw, cos_logsig, ds,
                                 stream);
}

namespace dph {
namespace {
// ---- Lagrangian sparsity regulariser + total loss (lightning.py:221-229) ----------------------------------
// es = 1 - num / orig, d = es - target, reg = lambda1 * d + lambda2 * d^2, loss = distill + reg: one thread,
// the fp32 operations in the reference's order (replaces ~10 one-element ATen launches forward and ~12 backward).
__global__ void reg_fwd_kernel(const float* distill, const float* num, const float* l1, const float* l2,
                               const float* tgt_dev, float tgt, float orig, float* out) {
  const float t = tgt_dev ? *tgt_dev : tgt;
  const float es = 1.0f - *num / orig;
  const float d = es - t;
  const float reg = *l1 * d + *l2 * (d * d);
  out[0] = *distill + reg;
  out[1] = reg;
  out[2] = es;
}

// grads[0..2] = d/dnum, d/dlambda1, d/dlambda2 of (gL * loss + greg * reg + ges * es); the distill loss's
// gradient is gL itself (the host passes it through)
__global__ void reg_bwd_kernel(const float* gL, const float* greg, const float* ges, const float* num, const float* l1,
                               const float* l2, const float* tgt_dev, float tgt, float orig, float* grads,
                               float* sink_l1, float* sink_l2) {
  const float t = tgt_dev ? *tgt_dev : tgt;
  const float es = 1.0f - *num / orig;
  const float d = es - t;
  const float gr = (gL ? *gL : 0.0f) + (greg ? *greg : 0.0f);
  const float gd = gr * *l1 + gr * *l2 * 2.0f * d;
  const float g_es = gd + (ges ? *ges : 0.0f);
  grads[0] = -g_es / orig;
  grads[1] = gr * d;
  grads[2] = gr * (d * d);
  if (sink_l1) *sink_l1 += grads[1];
  if (sink_l2) *sink_l2 += grads[2];
}
}  // namespace
}  // namespace dph

extern "C" int dph_reg_loss_fwd(const float* distill, const float* num, const float* lambda1, const float* lambda2,
                                const float* target_dev, float target, float orig_params, float* out,
                                hipStream_t stream) {
  DPH_REQUIRE(distill && num && lambda1 && lambda2 && out && orig_params > 0.f, "dph_reg_loss_fwd: bad args");
  hipLaunchKernelGGL(reg_fwd_kernel, dim3(1), dim3(1), 0, stream, distill, num, lambda1, lambda2, target_dev, target,
                     orig_params, out);
  return check_launch("dph_reg_loss_fwd");
}

extern "C" int dph_reg_loss_bwd(const float* g_loss, const float* g_reg, const float* g_es, const float* num,
                                const float* lambda1, const float* lambda2, const float* target_dev, float target,
                                float orig_params, float* grads, float* sink_l1, float* sink_l2,
                                hipStream_t stream) {
  DPH_REQUIRE(num && lambda1 && lambda2 && grads && orig_params > 0.f, "dph_reg_loss_bwd: bad args");
  hipLaunchKernelGGL(reg_bwd_kernel, dim3(1), dim3(1), 0, stream, g_loss, g_reg, g_es, num, lambda1, lambda2,
                     target_dev, target, orig_params, grads, sink_l1, sink_l2);
  return check_launch("dph_reg_loss_bwd");
}
