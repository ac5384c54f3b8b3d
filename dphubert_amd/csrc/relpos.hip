// WavLM relative-position bias and its GRU-style gate (WavLMSelfAttention, components.py:486-659).
//
// The reference materialises position_bias (B*H, T, T) fp32 from an Embedding lookup of bucketed offsets and
// multiplies it by a per-(b, h, q) gate before adding it to the scores.  Here nothing of size T x T exists:
//   * dph_relpos_table  -> tab[h][r] = embed[bucket(r - (T-1))][head[h]], r in [0, 2T-1) (one diagonal per r);
//     the attention kernels add gate[b,h,q] * tab[h][k - q + T - 1] to each score in registers.
//   * dph_wavlm_gate_fwd -> gate[b][h][t] from the attention input x (Linear(head_dim, 8), 2 groups of 4 summed,
//     sigmoid, gate = ga * (gb * c[h] - 1) + 2), components.py:637-643.
//   * backward: the attention dQ kernel emits dgate (row sums of dS * tab) and dtab (diagonal sums of dS * gate);
//     dph_relpos_table_bwd folds dtab into the embedding gradient, dph_wavlm_gate_bwd turns dgate into
//     d(gate weights, bias, const) and adds the input gradient into dx.
#include <cmath>

#include "common.h"

namespace dph {
namespace {

// components.py:563-600, bidirectional: evaluated in fp32 exactly as the reference (log of the fp32 ratio,
// divided by log(max_distance / max_exact) rounded to fp32, times (num_buckets - max_exact), truncated).
__device__ __forceinline__ int relpos_bucket(int rel, int num_buckets, int max_distance, float log_ratio) {
  const int nb = num_buckets / 2;
  int out = rel > 0 ? nb : 0;
  const int r = rel < 0 ? -rel : rel;
  const int max_exact = nb / 2;
  if (r < max_exact) return out + r;
  const float lr = logf((float)r / (float)max_exact);
  int large = max_exact + (int)((lr / log_ratio) * (float)(nb - max_exact));
  large = min(large, nb - 1);
  return out + large;
}

__global__ void relpos_table_kernel(const float* __restrict__ embed, const int64_t* __restrict__ heads,
                                    float* __restrict__ tab, int64_t* __restrict__ buckets, int T, int H, int Htot,
                                    int num_buckets, int max_distance, float log_ratio) {
  const int R = 2 * T - 1;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= R * H) return;
  const int h = i / R, r = i % R;
  const int bk = relpos_bucket(r - (T - 1), num_buckets, max_distance, log_ratio);
  const int hh = heads ? (int)heads[h] : h;
  if (tab) tab[i] = embed[(int64_t)bk * Htot + hh];
  if (buckets && h == 0) buckets[r] = bk;
}

__global__ void relpos_table_bwd_kernel(const float* __restrict__ dtab, const int64_t* __restrict__ heads,
                                        float* __restrict__ dembed, int T, int H, int Htot, int num_buckets,
                                        int max_distance, float log_ratio) {
  const int R = 2 * T - 1;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= R * H) return;
  const int h = i / R, r = i % R;
  const float v = dtab[i];
  if (v == 0.f) return;
  const int bk = relpos_bucket(r - (T - 1), num_buckets, max_distance, log_ratio);
  const int hh = heads ? (int)heads[h] : h;
  atomicAdd(dembed + (int64_t)bk * Htot + hh, v);
}

// deterministic mode: the diagonals r of one bucket form ONE contiguous run (the bucket is monotone in |k - q| on
// each side of the main diagonal, and the two sides use disjoint bucket ranges), so the thread at a run's first
// diagonal sums the run in order and is the only writer of its embedding entry
__global__ void relpos_table_bwd_det_kernel(const float* __restrict__ dtab, const int64_t* __restrict__ heads,
                                            float* __restrict__ dembed, int T, int H, int Htot, int num_buckets,
                                            int max_distance, float log_ratio) {
  const int R = 2 * T - 1;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= R * H) return;
  const int h = i / R, r = i % R;
  const int bk = relpos_bucket(r - (T - 1), num_buckets, max_distance, log_ratio);
  if (r > 0 && relpos_bucket(r - 1 - (T - 1), num_buckets, max_distance, log_ratio) == bk) return;
  float acc = 0.f;
  for (int j = r; j < R && relpos_bucket(j - (T - 1), num_buckets, max_distance, log_ratio) == bk; ++j)
    acc += dtab[h * R + j];
  const int hh = heads ? (int)heads[h] : h;
  dembed[(int64_t)bk * Htot + hh] += acc;
}

constexpr int HDG = 64;   // gate head dim

struct GateArgs {
  const bf16_t* x;         // [B*T][ldx], head hh occupies columns hh*64 .. +63
  int64_t ldx;
  const float* w;          // [8][64]
  const float* bias;       // [8]
  const float* gconst;     // [Htot]
  const int64_t* heads;    // [H] total-head index of each remaining head (null = identity)
  int64_t B, T, H;
};

// The 4 logits of a group are only ever summed (components.py:639 .view(..., 2, 4).sum(-1)), so each group is
// ONE dot product with the group's summed weight row: w_s = [wa[64] | wb[64] | ba | bb] built per block.
__device__ __forceinline__ void load_group_weights(const GateArgs& a, float* w_s) {
  const int t = threadIdx.x;
  if (t < 2 * HDG) {
    const int grp = t / HDG, d = t % HDG;
    float v = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) v += a.w[(4 * grp + j) * HDG + d];
    w_s[t] = v;
  } else if (t < 2 * HDG + 2) {
    const int grp = t - 2 * HDG;
    w_s[t] = a.bias[4 * grp] + a.bias[4 * grp + 1] + a.bias[4 * grp + 2] + a.bias[4 * grp + 3];
  }
}

// group sums (za, zb) of (b, t, head hh) and their sigmoids
__device__ __forceinline__ void gate_logits(const GateArgs& a, const float* w_s, int64_t bt, int hh, float& ga,
                                            float& gb) {
  const bf16_t* xp = a.x + bt * a.ldx + (int64_t)hh * HDG;
  float za = w_s[2 * HDG], zb = w_s[2 * HDG + 1];
#pragma unroll
  for (int k = 0; k < HDG; k += 8) {
    const uint4 v = *reinterpret_cast<const uint4*>(xp + k);
    const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
    const float4 a0 = *reinterpret_cast<const float4*>(w_s + k), a1 = *reinterpret_cast<const float4*>(w_s + k + 4);
    const float4 b0 = *reinterpret_cast<const float4*>(w_s + HDG + k);
    const float4 b1 = *reinterpret_cast<const float4*>(w_s + HDG + k + 4);
    const float wa[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
    const float wb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float x0 = __uint_as_float(wv[q] << 16), x1 = __uint_as_float(wv[q] & 0xffff0000u);
      za += wa[2 * q] * x0 + wa[2 * q + 1] * x1;
      zb += wb[2 * q] * x0 + wb[2 * q + 1] * x1;
    }
  }
  ga = 1.f / (1.f + __expf(-za));
  gb = 1.f / (1.f + __expf(-zb));
}

// one thread per (b, t, h); threads of a block share (b, t) rows of consecutive heads
__global__ void __launch_bounds__(256) wavlm_gate_fwd_kernel(GateArgs a, float* __restrict__ gate) {
  __shared__ __attribute__((aligned(16))) float w_s[2 * HDG + 4];
  load_group_weights(a, w_s);
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= a.B * a.T * a.H) return;
  const int h = (int)(i % a.H);
  const int64_t bt = i / a.H;
  const int hh = a.heads ? (int)a.heads[h] : h;
  float ga, gb;
  gate_logits(a, w_s, bt, hh, ga, gb);
  const int64_t b = bt / a.T, t = bt % a.T;
  gate[(b * a.H + h) * a.T + t] = ga * (gb * a.gconst[hh] - 1.f) + 2.f;
}

// backward, pass 1: per (b, t, h): group gradients dza, dzb (each of a group's 4 logits gets it), dx += dza wa +
// dzb wb, db, dconst; (dza, dzb) -> scratch for the weight gradient
__global__ void __launch_bounds__(256) wavlm_gate_bwd_kernel(GateArgs a, const float* __restrict__ dgate,
                                                             bf16_t* __restrict__ dx, int64_t lddx,
                                                             float* __restrict__ dz_out, float* __restrict__ db,
                                                             float* __restrict__ dconst, float* __restrict__ dc_out) {
  __shared__ __attribute__((aligned(16))) float w_s[2 * HDG + 4];
  __shared__ float dc_s[64];   // per-block dconst partials (total heads <= 64)
  load_group_weights(a, w_s);
  if (threadIdx.x < 64) dc_s[threadIdx.x] = 0.f;
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const bool live = i < a.B * a.T * a.H;
  float dza = 0.f, dzb = 0.f, dc = 0.f;
  int hh = 0;
  if (live) {
    const int h = (int)(i % a.H);
    const int64_t bt = i / a.H;
    hh = a.heads ? (int)a.heads[h] : h;
    float ga, gb;
    gate_logits(a, w_s, bt, hh, ga, gb);
    const int64_t b = bt / a.T, t = bt % a.T;
    const float dg = dgate[(b * a.H + h) * a.T + t];
    const float c = a.gconst[hh];
    const float dga = dg * (gb * c - 1.f);
    const float dgb = dg * ga * c;
    dc = dg * ga * gb;
    dza = dga * ga * (1.f - ga);
    dzb = dgb * gb * (1.f - gb);
    dz_out[i * 2] = dza;
    dz_out[i * 2 + 1] = dzb;
    if (dc_out) dc_out[i] = dc;
    // dx[d] += dza wa[d] + dzb wb[d]  (read-modify-write of this head's 64 bf16; heads of a row are disjoint)
    bf16_t* xp = dx + bt * lddx + (int64_t)hh * HDG;
#pragma unroll
    for (int k = 0; k < HDG; k += 8) {
      uint4 v = *reinterpret_cast<const uint4*>(xp + k);
      uint32_t wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int d = k + 2 * q;
        const float a0 = dza * w_s[d] + dzb * w_s[HDG + d];
        const float a1 = dza * w_s[d + 1] + dzb * w_s[HDG + d + 1];
        wv[q] = pack2bf(__uint_as_float(wv[q] << 16) + a0, __uint_as_float(wv[q] & 0xffff0000u) + a1);
      }
      *reinterpret_cast<uint4*>(xp + k) = make_uint4(wv[0], wv[1], wv[2], wv[3]);
    }
  }
  // deterministic mode (dc_out): db / dconst are summed in a fixed order by the weight-gradient / finish kernels
  if (dc_out) return;
  // db[j] = sum dz_j (j < 4: dza, else dzb): wave sums -> one atomic pair per block; dconst[hh] += dc
  __shared__ float red[2][4];
  const float sa = wave_sum(dza), sb = wave_sum(dzb);
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = sa;
    red[1][threadIdx.x >> 6] = sb;
  }
  if (live) atomicAdd(&dc_s[hh], dc);
  __syncthreads();
  if (threadIdx.x < 64 && dc_s[threadIdx.x] != 0.f) atomicAdd(dconst + threadIdx.x, dc_s[threadIdx.x]);
  if (threadIdx.x == 0) {
    atomicAdd(db + 0, red[0][0] + red[0][1] + red[0][2] + red[0][3]);
    atomicAdd(db + 4, red[1][0] + red[1][1] + red[1][2] + red[1][3]);
  }
}

// backward, pass 2: dW[j][d] = sum_n dz[n][j/4] x[n][d]; block = 256 rows n, thread (jg = t>>6 in {0..3}, d = t&63)
// sums a quarter of the rows for both groups, LDS-combined, then atomics (db rows 1-3, 5-7 copied at the end).
__global__ void __launch_bounds__(256) wavlm_gate_wgrad_kernel(GateArgs a, const float* __restrict__ dz,
                                                               float* __restrict__ dw, const float* __restrict__ dc,
                                                               float* __restrict__ part2) {
  __shared__ float red[4][2][HDG];
  const int d = threadIdx.x & 63;
  const int part = threadIdx.x >> 6;
  const int64_t N = a.B * a.T * a.H;
  const int64_t n0 = (int64_t)blockIdx.x * 256;
  float acc_a = 0.f, acc_b = 0.f;
  for (int r = part; r < 256; r += 4) {
    const int64_t n = n0 + r;
    if (n >= N) break;
    const int h = (int)(n % a.H);
    const int64_t bt = n / a.H;
    const int hh = a.heads ? (int)a.heads[h] : h;
    const float xv = bf2f(a.x[bt * a.ldx + (int64_t)hh * HDG + d]);
    acc_a += dz[n * 2] * xv;
    acc_b += dz[n * 2 + 1] * xv;
  }
  red[part][0][d] = acc_a;
  red[part][1][d] = acc_b;
  __syncthreads();
  if (part < 2) {
    // the 4 logits of a group share the same gradient: one partial row per group and block (no atomics: ~1500
    // blocks' atomics on 128 addresses serialised), summed over blocks by wavlm_gate_finish_kernel
    dw[((int64_t)blockIdx.x * 2 + part) * HDG + d] = red[0][part][d] + red[1][part][d] + red[2][part][d] + red[3][part][d];
  }
  if (part2) {
    // deterministic mode: this block's dconst per total head (thread t < 64) and the two group sums of dz
    // (threads 64, 65) over its 256 rows in row order -> part2[block][66]
    const int t = threadIdx.x;
    if (t < 66) {
      float acc = 0.f;
      for (int r = 0; r < 256; ++r) {
        const int64_t n = n0 + r;
        if (n >= N) break;
        if (t < 64) {
          const int h = (int)(n % a.H);
          const int hh = a.heads ? (int)a.heads[h] : h;
          if (hh == t) acc += dc[n];
        } else {
          acc += dz[n * 2 + (t - 64)];
        }
      }
      part2[(int64_t)blockIdx.x * 66 + t] = acc;
    }
  }
}

// deterministic mode: the per-block partial rows summed in block order (det_column_total) -- blocks 0..3: the 128
// dW group columns (each added to its group's 4 rows); blocks 4..6: part2's 66 columns (dconst per head, then the
// two db group sums, each added to its group's 4 bias entries)
__global__ void __launch_bounds__(32 * DET_PH) wavlm_gate_finish_det_kernel(float* __restrict__ dw, float* __restrict__ db,
                                                                           float* __restrict__ dconst,
                                                                           const float* __restrict__ part,
                                                                           const float* __restrict__ part2, int nblk) {
  __shared__ float red[DET_PH][33];
  const int tx = threadIdx.x & 31, ph = threadIdx.x >> 5;
  if (blockIdx.x < 4) {
    const int col = blockIdx.x * 32 + tx;   // (group, d) = (col / 64, col % 64)
    const float t = det_column_total(part + col, nblk, 2 * HDG, red);
    if (ph == 0) {
      const int grp = col / HDG, d = col % HDG;
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) dw[(grp * 4 + jj) * HDG + d] += t;
    }
  } else {
    const int col = (blockIdx.x - 4) * 32 + tx;
    const float t = det_column_total(col < 66 ? part2 + col : nullptr, nblk, 66, red);
    if (ph == 0 && col < 66) {
      if (col < 64) {
        if (t != 0.f) dconst[col] += t;     // (heads past Htot have no rows: their sum is 0 and is not written)
      } else {
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) db[(col - 64) * 4 + jj] += t;
      }
    }
  }
}

// dW / db rows of one group are identical (each logit of a group gets the group's gradient): sum the per-block
// partial rows, 32 blocks' partials per finishing block, and add them to all 4 rows of the group
constexpr int FIN_CHUNK = 32;
__global__ void __launch_bounds__(128) wavlm_gate_finish_kernel(float* __restrict__ dw, float* __restrict__ db,
                                                                const float* __restrict__ part, int nblk,
                                                                const float* __restrict__ db0) {
  const int t = threadIdx.x;   // 128 threads: (group, d)
  const int grp = t >> 6, d = t & 63;
  const int k0 = blockIdx.x * FIN_CHUNK;
  const int k1 = min(k0 + FIN_CHUNK, nblk);
  float acc = 0.f;
  for (int k = k0; k < k1; ++k) acc += part[((int64_t)k * 2 + grp) * HDG + d];
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) atomicAdd(dw + (grp * 4 + jj) * HDG + d, acc);
  if (blockIdx.x == 0 && d == 0)
    for (int jj = 0; jj < 4; ++jj) db[grp * 4 + jj] += db0[grp * 4];
}

}  // namespace
}  // namespace dph

using namespace dph;

static float relpos_log_ratio(int64_t num_buckets, int64_t max_distance) {
  const int64_t max_exact = (num_buckets / 2) / 2;
  // python float math.log(max_distance / max_exact), rounded to fp32 when it meets the fp32 tensor
  return (float)std::log((double)max_distance / (double)max_exact);
}

extern "C" int dph_relpos_table(const float* embed, const int64_t* heads, float* tab, int64_t* buckets, int64_t T,
                                int64_t H, int64_t Htot, int64_t num_buckets, int64_t max_distance,
                                hipStream_t stream) {
  DPH_REQUIRE((tab ? embed != nullptr : true) && (tab || buckets) && T > 0 && T <= 4096 && H > 0 && Htot >= H &&
                  num_buckets >= 4 && max_distance > num_buckets / 4,
              "dph_relpos_table: bad args");
  const int n = (int)((2 * T - 1) * H);
  hipLaunchKernelGGL(relpos_table_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, stream, embed, heads, tab,
                     buckets, (int)T, (int)H, (int)Htot, (int)num_buckets, (int)max_distance,
                     relpos_log_ratio(num_buckets, max_distance));
  return check_launch("dph_relpos_table");
}

extern "C" int dph_relpos_table_bwd(const float* dtab, const int64_t* heads, float* dembed, int64_t T, int64_t H,
                                    int64_t Htot, int64_t num_buckets, int64_t max_distance, hipStream_t stream) {
  DPH_REQUIRE(dtab && dembed && T > 0 && T <= 4096 && H > 0 && Htot >= H && num_buckets >= 4 &&
                  max_distance > num_buckets / 4,
              "dph_relpos_table_bwd: bad args");
  const int n = (int)((2 * T - 1) * H);
  if (deterministic())
    hipLaunchKernelGGL(relpos_table_bwd_det_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, stream, dtab, heads,
                       dembed, (int)T, (int)H, (int)Htot, (int)num_buckets, (int)max_distance,
                       relpos_log_ratio(num_buckets, max_distance));
  else
    hipLaunchKernelGGL(relpos_table_bwd_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, stream, dtab, heads,
                       dembed, (int)T, (int)H, (int)Htot, (int)num_buckets, (int)max_distance,
                       relpos_log_ratio(num_buckets, max_distance));
  return check_launch("dph_relpos_table_bwd");
}

extern "C" int dph_wavlm_gate_fwd(const void* x, int64_t ldx, const float* w, const float* bias, const float* gconst,
                                  const int64_t* heads, float* gate, int64_t B, int64_t T, int64_t H, int64_t head_dim,
                                  hipStream_t stream) {
  DPH_REQUIRE(x && w && bias && gconst && gate && B > 0 && T > 0 && H > 0 && head_dim == HDG && ldx % 8 == 0,
              "dph_wavlm_gate_fwd: bad args (head_dim 64, ldx % 8 == 0)");
  GateArgs a{reinterpret_cast<const bf16_t*>(x), ldx, w, bias, gconst, heads, B, T, H};
  hipLaunchKernelGGL(wavlm_gate_fwd_kernel, dim3((unsigned)cdiv(B * T * H, 256)), dim3(256), 0, stream, a, gate);
  return check_launch("dph_wavlm_gate_fwd");
}

// workspace (bytes) of dph_wavlm_gate_bwd, either mode: dz [N][2], dc [N], db0 [8], the per-block dW group rows
// [nblk][2][64] and (deterministic mode) the per-block dconst / db rows [nblk][66]; N = B*T*H, nblk = ceil(N / 256)
extern "C" int64_t dph_wavlm_gate_bwd_workspace(int64_t B, int64_t T, int64_t H) {
  const int64_t N = B * T * H, nblk = cdiv(N, 256);
  return (3 * N + 8 + nblk * (2 * HDG + 66)) * 4;
}

// dx (bf16, ld lddx) is ADDED to; dw [8][64], db [8], dconst [Htot] accumulate
extern "C" int dph_wavlm_gate_bwd(const void* x, int64_t ldx, const float* w, const float* bias, const float* gconst,
                                  const int64_t* heads, const float* dgate, void* dx, int64_t lddx, float* dw,
                                  float* db, float* dconst, float* ws, int64_t ws_bytes, int64_t B, int64_t T,
                                  int64_t H, int64_t head_dim, hipStream_t stream) {
  DPH_REQUIRE(x && w && bias && gconst && dgate && dx && dw && db && dconst && ws && B > 0 && T > 0 && H > 0 &&
                  head_dim == HDG && ldx % 8 == 0 && lddx % 8 == 0 && ldx / HDG <= 64,
              "dph_wavlm_gate_bwd: bad args (head_dim 64, <= 64 heads)");
  DPH_REQUIRE(ws_bytes >= dph_wavlm_gate_bwd_workspace(B, T, H), "dph_wavlm_gate_bwd: workspace too small");
  GateArgs a{reinterpret_cast<const bf16_t*>(x), ldx, w, bias, gconst, heads, B, T, H};
  const int64_t N = B * T * H;
  const int nblk = (int)cdiv(N, 256);
  const bool det = deterministic();
  float* dz = ws;
  float* dc = ws + 2 * N;           // [N] (deterministic mode)
  float* db0 = dc + N;              // [8] (entries 0 and 4 used)
  float* part = db0 + 8;            // [nblk][2][64] per-block group rows of dW
  float* part2 = part + (int64_t)nblk * 2 * HDG;   // [nblk][66] (deterministic mode)
  if (!det) zero_async(db0, 8 * sizeof(float), stream);
  hipLaunchKernelGGL(wavlm_gate_bwd_kernel, dim3((unsigned)cdiv(N, 256)), dim3(256), 0, stream, a, dgate,
                     reinterpret_cast<bf16_t*>(dx), lddx, dz, db0, dconst, det ? dc : nullptr);
  hipLaunchKernelGGL(wavlm_gate_wgrad_kernel, dim3((unsigned)nblk), dim3(256), 0, stream, a, dz, part,
                     (const float*)dc, det ? part2 : nullptr);
  if (det)
    hipLaunchKernelGGL(wavlm_gate_finish_det_kernel, dim3(7), dim3(32 * DET_PH), 0, stream, dw, db, dconst, part,
                       part2, nblk);
  else
    hipLaunchKernelGGL(wavlm_gate_finish_kernel, dim3((unsigned)cdiv(nblk, FIN_CHUNK)), dim3(128), 0, stream, dw, db,
                       part, nblk, db0);
  return check_launch("dph_wavlm_gate_bwd");
}
