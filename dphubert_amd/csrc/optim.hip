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

__global__ void __launch_bounds__(256) sumsq_kernel(const DphTensorSlot* __restrict__ slots,
                                                    const int64_t* __restrict__ cslot,
                                                    const int64_t* __restrict__ cstart, float* __restrict__ out) {
  __shared__ float red[4];
  const int64_t c = blockIdx.x;
  const DphTensorSlot sl = slots[cslot[c]];
  const int64_t s0 = cstart[c];
  const int64_t s1 = min(sl.n, s0 + CHUNK);
  float s = 0.f;
  if (sl.grad)
    for (int64_t i = s0 + threadIdx.x; i < s1; i += 256) s += sl.grad[i] * sl.grad[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(out, red[0] + red[1] + red[2] + red[3]);
}

__global__ void __launch_bounds__(256) adamw_kernel(const DphTensorSlot* __restrict__ slots,
                                                    const int64_t* __restrict__ cslot,
                                                    const int64_t* __restrict__ cstart, Groups G, float step,
                                                    const DphAdamDyn* __restrict__ dyn,
                                                    const float* __restrict__ sumsq, float max_norm) {
  const int64_t c = blockIdx.x;
  const DphTensorSlot sl = slots[cslot[c]];
  if (!sl.grad) return;
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
  for (int64_t i = s0 + threadIdx.x; i < s1; i += 256) {
    const float g = sl.grad[i] * clip;
    float p = sl.param[i] * decay;
    float m = sl.exp_avg[i];
    float v = sl.exp_avg_sq[i];
    m = m + (g - m) * (1.0f - gr.beta1);
    v = v * gr.beta2 + (1.0f - gr.beta2) * g * g;
    const float denom = sqrtf(v) / bc2_sqrt + gr.eps;
    p = p - step_size * m / denom;
    sl.param[i] = p;
    sl.exp_avg[i] = m;
    sl.exp_avg_sq[i] = v;
    sl.grad[i] = g;
  }
}

}  // namespace
}  // namespace dph

using namespace dph;

extern "C" int dph_grad_sumsq(const DphTensorSlot* slots, int64_t n_slots, const int64_t* chunk_slot,
                              const int64_t* chunk_start, int64_t n_chunks, float* sumsq, hipStream_t stream) {
  DPH_REQUIRE(slots && chunk_slot && chunk_start && sumsq && n_slots > 0 && n_chunks > 0, "dph_grad_sumsq: bad args");
  if (hipMemsetAsync(sumsq, 0, sizeof(float), stream) != hipSuccess) return check_launch("dph_grad_sumsq memset");
  hipLaunchKernelGGL(sumsq_kernel, dim3((unsigned)n_chunks), dim3(256), 0, stream, slots, chunk_slot, chunk_start,
                     sumsq);
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
                     (float)step, (const DphAdamDyn*)nullptr, sumsq, max_norm);
  return check_launch("dph_adamw_step");
}

extern "C" int dph_adamw_step_dev(const DphTensorSlot* slots, int64_t n_slots, const int64_t* chunk_slot,
                                  const int64_t* chunk_start, int64_t n_chunks, const DphAdamDyn* dyn,
                                  const float* sumsq, float max_norm, hipStream_t stream) {
  DPH_REQUIRE(slots && chunk_slot && chunk_start && dyn && n_chunks > 0, "dph_adamw_step_dev: bad args");
  Groups G = {};
  hipLaunchKernelGGL(adamw_kernel, dim3((unsigned)n_chunks), dim3(256), 0, stream, slots, chunk_slot, chunk_start, G,
                     1.0f, dyn, sumsq, max_norm);
  return check_launch("dph_adamw_step_dev");
}
