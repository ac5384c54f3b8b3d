// Fused multi-tensor AdamW with global-norm gradient clipping.
//
// Reference: torch.optim.AdamW over three param groups (main / log_alpha /
// lambda with negative lr) built in lightning.py:200-228, gradient clipping
// Trainer(gradient_clip_val=clip_norm) (distill.py:48) = clip_grad_norm_(all
// params, max_norm, norm_type=2): coef = max_norm / (||g|| + 1e-6), grads *=
// min(coef, 1).  The clip coefficient stays on the device (no host sync).
//
// Work is split into fixed-size chunks (slot, start) prepared once on the
// host, so one launch walks ~95.6 M parameters spread over ~400 tensors.
#include "common.h"

namespace dph {
namespace {

constexpr int64_t CHUNK = 8192;
constexpr int MAX_GROUPS = 4;

struct Groups {
  DphAdamGroup g[MAX_GROUPS];
};

// ||g||^2 over every chunk: a fixed grid of at most SUMSQ_BLOCKS blocks walks the chunks, sums in
// registers (16-B loads where the tensor is 16-B aligned) and writes ONE partial per block (out[1 + b]);
// a one-wave kernel sums the partials in a fixed order into out[0] (deterministic clip norm, no memset).
// (One block per 8192-element chunk with a same-address float atomic each meant ~11.7 k atomics per step:
// they serialise at the memory side, ~16 ns each -- 0.19 ms for a 382 MB read.)
constexpr int SUMSQ_BLOCKS = DPH_SUMSQ_FLOATS - 1;

__global__ void __launch_bounds__(256) sumsq_kernel(const DphTensorSlot* __restrict__ slots,
                                                    const int64_t* __restrict__ cslot,
                                                    const int64_t* __restrict__ cstart, int64_t n_chunks,
                                                    float* __restrict__ out) {
  __shared__ float red[4];
  // four independent accumulators: a full chunk's eight float4 loads per thread are issued four at a time (one
  // dependent add chain and one load per trip ran the 382 MB read at ~5.4 TB/s)
  float s = 0.f, sa = 0.f, sb = 0.f, sc = 0.f;
  auto sq = [](float4 v) { return v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w; };
  for (int64_t c = blockIdx.x; c < n_chunks; c += gridDim.x) {
    const DphTensorSlot sl = slots[cslot[c]];
    if (!sl.grad) continue;
    const int64_t s0 = cstart[c];
    const int64_t s1 = min(sl.n, s0 + CHUNK);
    int64_t i = s0;
    if ((reinterpret_cast<uintptr_t>(sl.grad + s0) & 15) == 0) {
      const int64_t n4 = (s1 - s0) >> 2;
      const float4* g4 = reinterpret_cast<const float4*>(sl.grad + s0);
      int64_t j = threadIdx.x;
      for (; j + 768 < n4; j += 1024) {
        const float4 v0 = g4[j], v1 = g4[j + 256], v2 = g4[j + 512], v3 = g4[j + 768];
        s += sq(v0);
        sa += sq(v1);
        sb += sq(v2);
        sc += sq(v3);
      }
      for (; j < n4; j += 256) s += sq(g4[j]);
      i = s0 + 4 * n4;
    }
    for (i += threadIdx.x; i < s1; i += 256) s += sl.grad[i] * sl.grad[i];
  }
  s = (s + sa) + (sb + sc);
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[1 + blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ void __launch_bounds__(64) sumsq_finalize_kernel(float* __restrict__ out, int64_t nb) {
  const float s = sum_partials_wave(out + 1, nb, 1);
  if (threadIdx.x == 0) out[0] = s;
}

__global__ void __launch_bounds__(256) adamw_kernel(const DphTensorSlot* __restrict__ slots,
                                                    const int64_t* __restrict__ cslot,
                                                    const int64_t* __restrict__ cstart, Groups G, float step,
                                                    const DphAdamDyn* __restrict__ dyn,
                                                    const float* __restrict__ sumsq, float max_norm,
                                                    const uint64_t* __restrict__ img) {
  const int64_t c = blockIdx.x;
  const DphTensorSlot sl = slots[cslot[c]];
  if (!sl.grad) return;
  // the parameter's place in its bf16 GEMM image (0: none): the updated master is cast there too
  bf16_t* const im = img ? reinterpret_cast<bf16_t*>(img[cslot[c]]) : nullptr;
  // device-resident lr / step (HIP-graph replays) or the launch-time values
  const DphAdamGroup gr = dyn ? dyn->g[sl.group] : G.g[sl.group];
  if (dyn) step = dyn->step;
  float clip = 1.0f;
  if (sumsq && max_norm > 0.f) clip = fminf(max_norm / (sqrtf(*sumsq) + 1e-6f), 1.0f);
  const float bc1 = 1.0f - powf(gr.beta1, step);
  const float bc2 = 1.0f - powf(gr.beta2, step);
  const float step_size = gr.lr / bc1;
  const float bc2_sqrt = sqrtf(bc2);
  const float decay = 1.0f - gr.lr * gr.weight_decay;
  const int64_t s0 = cstart[c];
  const int64_t s1 = min(sl.n, s0 + CHUNK);
  const float b1c = 1.0f - gr.beta1, b2c = 1.0f - gr.beta2;
  auto upd = [&](float gi, float& p, float& m, float& v, float& go) {
    const float g = gi * clip;
    p *= decay;
    m = m + (g - m) * b1c;
    v = v * gr.beta2 + b2c * g * g;
    const float denom = sqrtf(v) / bc2_sqrt + gr.eps;
    p = p - step_size * m / denom;
    go = g;
  };
  int64_t i0 = s0;
  // 16-B path over the chunk's whole quads when all four streams are 16-B aligned there
  const uintptr_t al = reinterpret_cast<uintptr_t>(sl.grad + s0) | reinterpret_cast<uintptr_t>(sl.param + s0) |
                       reinterpret_cast<uintptr_t>(sl.exp_avg + s0) | reinterpret_cast<uintptr_t>(sl.exp_avg_sq + s0) |
                       (im ? 2 * reinterpret_cast<uintptr_t>(im + s0) : 0);   // (8-B image stores)
  if ((al & 15) == 0) {
    const int64_t n4 = (s1 - s0) >> 2;
    float4* g4 = reinterpret_cast<float4*>(sl.grad + s0);
    float4* p4 = reinterpret_cast<float4*>(sl.param + s0);
    float4* m4 = reinterpret_cast<float4*>(sl.exp_avg + s0);
    float4* v4 = reinterpret_cast<float4*>(sl.exp_avg_sq + s0);
    // (two quads per trip -- eight loads before the first store -- measured slower: 84 VGPRs, 5 waves per SIMD,
    // 467 -> 532 us per step for the 95 M-parameter student, profiles/r6_optim_ab.txt)
    for (int64_t j = threadIdx.x; j < n4; j += 256) {
      float4 g = g4[j], p = p4[j], m = m4[j], v = v4[j];
      upd(g.x, p.x, m.x, v.x, g.x);
      upd(g.y, p.y, m.y, v.y, g.y);
      upd(g.z, p.z, m.z, v.z, g.z);
      upd(g.w, p.w, m.w, v.w, g.w);
      p4[j] = p;
      m4[j] = m;
      v4[j] = v;
      if (clip < 1.0f) g4[j] = g;   // (clip_grad_norm_ scales .grad in place; unscaled, it is already there)
      if (im) *reinterpret_cast<uint2*>(im + s0 + 4 * j) = make_uint2(pack2bf(p.x, p.y), pack2bf(p.z, p.w));
    }
    i0 = s0 + 4 * n4;
  }
  for (int64_t i = i0 + threadIdx.x; i < s1; i += 256) {
    float p = sl.param[i], m = sl.exp_avg[i], v = sl.exp_avg_sq[i], g;
    upd(sl.grad[i], p, m, v, g);
    sl.param[i] = p;
    sl.exp_avg[i] = m;
    sl.exp_avg_sq[i] = v;
    if (clip < 1.0f) sl.grad[i] = g;
    if (im) im[i] = f2bf(p);
  }
}

}  // namespace
}  // namespace dph

using namespace dph;

extern "C" int dph_grad_sumsq(const DphTensorSlot* slots, int64_t n_slots, const int64_t* chunk_slot,
                              const int64_t* chunk_start, int64_t n_chunks, float* sumsq, hipStream_t stream) {
  DPH_REQUIRE(slots && chunk_slot && chunk_start && sumsq && n_slots > 0 && n_chunks > 0, "dph_grad_sumsq: bad args");
  const int64_t nb = n_chunks < SUMSQ_BLOCKS ? n_chunks : SUMSQ_BLOCKS;
  hipLaunchKernelGGL(sumsq_kernel, dim3((unsigned)nb), dim3(256), 0, stream, slots, chunk_slot, chunk_start, n_chunks,
                     sumsq);
  hipLaunchKernelGGL(sumsq_finalize_kernel, dim3(1), dim3(64), 0, stream, sumsq, nb);
  return check_launch("dph_grad_sumsq");
}

extern "C" int dph_adamw_step(const DphTensorSlot* slots, int64_t n_slots, const int64_t* chunk_slot,
                              const int64_t* chunk_start, int64_t n_chunks, const DphAdamGroup* groups,
                              int64_t n_groups, int64_t step, const float* sumsq, float max_norm,
                              hipStream_t stream) {
  DPH_REQUIRE(slots && chunk_slot && chunk_start && groups && n_chunks > 0, "dph_adamw_step: bad args");
  DPH_REQUIRE(n_groups >= 1 && n_groups <= MAX_GROUPS && step >= 1, "dph_adamw_step: bad groups/step");
  Groups G;
  for (int i = 0; i < MAX_GROUPS; ++i) G.g[i] = groups[i < n_groups ? i : 0];
  hipLaunchKernelGGL(adamw_kernel, dim3((unsigned)n_chunks), dim3(256), 0, stream, slots, chunk_slot, chunk_start, G,
                     (float)step, (const DphAdamDyn*)nullptr, sumsq, max_norm, (const uint64_t*)nullptr);
  return check_launch("dph_adamw_step");
}

extern "C" int dph_adamw_step_dev(const DphTensorSlot* slots, int64_t n_slots, const int64_t* chunk_slot,
                                  const int64_t* chunk_start, int64_t n_chunks, const DphAdamDyn* dyn,
                                  const float* sumsq, float max_norm, hipStream_t stream) {
  DPH_REQUIRE(slots && chunk_slot && chunk_start && dyn && n_chunks > 0, "dph_adamw_step_dev: bad args");
  Groups G = {};
  hipLaunchKernelGGL(adamw_kernel, dim3((unsigned)n_chunks), dim3(256), 0, stream, slots, chunk_slot, chunk_start, G,
                     1.0f, dyn, sumsq, max_norm, (const uint64_t*)nullptr);
  return check_launch("dph_adamw_step_dev");
}

extern "C" int dph_adamw_step_img(const DphTensorSlot* slots, int64_t n_slots, const int64_t* chunk_slot,
                                  const int64_t* chunk_start, int64_t n_chunks, const DphAdamDyn* dyn,
                                  const DphAdamGroup* groups, int64_t n_groups, int64_t step, const float* sumsq,
                                  float max_norm, const uint64_t* img, hipStream_t stream) {
  DPH_REQUIRE(slots && chunk_slot && chunk_start && n_chunks > 0, "dph_adamw_step_img: bad args");
  DPH_REQUIRE(dyn || (groups && n_groups >= 1 && n_groups <= MAX_GROUPS && step >= 1),
              "dph_adamw_step_img: need dyn or groups/step");
  Groups G = {};
  if (!dyn)
    for (int i = 0; i < MAX_GROUPS; ++i) G.g[i] = groups[i < n_groups ? i : 0];
  hipLaunchKernelGGL(adamw_kernel, dim3((unsigned)n_chunks), dim3(256), 0, stream, slots, chunk_slot, chunk_start, G,
                     dyn ? 1.0f : (float)step, dyn, sumsq, max_norm, img);
  return check_launch("dph_adamw_step_img");
}
