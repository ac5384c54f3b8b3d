// Fused multi-head self-attention (head dim 64) for gfx950, forward + backward.
//
// Reference: SelfAttention.forward, components.py:405-426:
//   w = (scaling*q) @ k^T + mask(-1e4 on padded keys); w -= rowmax; softmax;
//   dropout(p); out = w @ v; out *= head_mask[h].
// Nothing of size T x T is ever written to HBM: scores live in MFMA
// accumulators, the forward keeps a running (max, sum) per query row and saves
// only LSE = max + log(sum); the backward recomputes P from LSE.
//
// q, k, v are read straight from the fused QKV projection output
// [B*T][3*H*64] (q | k | v blocks), gradients are written into the same
// layout, so no (B,H,T,hd) permute copies exist.
//
// MFMA: v_mfma_f32_16x16x32_bf16.  "Swapped" products put the key index in
// the accumulator rows, so a P/dS tile feeds the next product directly as the
// B operand (the k permutation of the accumulator rows is matched by the
// transposed LDS read ds_read_b64_tr_b16 of V / K / dO / Q tiles).
#include "common.h"

#include <type_traits>

namespace dph {
namespace {

constexpr int HD = 64;
constexpr int KT = 64;        // keys per tile (fwd / dQ), keys per block (dKV)
constexpr int QT = 64;        // query rows per block (fwd / dQ)
constexpr int QT_BWD = 32;    // query rows per step of the dKV kernel
constexpr int PADROW = 72;    // padded row (elements) for b128-only tiles

typedef __attribute__((address_space(3))) s16x4_t lds_s16x4;

// 128-byte rows (64 bf16), 32-B units XOR-swizzled by (row>>1)&3: conflict-free
// for both the 16-B row reads and the 8-row transposed reads.
__device__ __forceinline__ int swz128(int r, int col) { return r * 128 + ((((col >> 4) ^ (r >> 1)) & 3) * 32) + (col & 15) * 2; }

__device__ __forceinline__ bf16x8_t lds_b128(const char* lds, int byte) {
  return *reinterpret_cast<const bf16x8_t*>(lds + byte);
}

// transposed fragment: lane (g=l>>4, i=l&15, q=i>>2, p=i&3) gets X[rows r0(g)+0..3][col c0+i] and
// X[rows r1(g)+0..3][c0+i] from a swizzled [rows][64] tile
__device__ __forceinline__ bf16x8_t tr_frag(const char* lds, int r0, int r1, int c0, int lane) {
  const int i = lane & 15;
  const int q = i >> 2;
  const int p = i & 3;
  s16x4_t v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + swz128(r0 + q, c0 + 4 * p)));
  s16x4_t v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + swz128(r1 + q, c0 + 4 * p)));
  s16x8_t v = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
  return __builtin_bit_cast(bf16x8_t, v);
}

// (one v_cvt_pk_bf16_f32 per element pair; element-wise casts came out as packs of mismatched pairs plus
// v_alignbit / v_pk_mov shuffles)
__device__ __forceinline__ bf16x8_t pack_frag(const f32x4_t& a, const f32x4_t& b) {
  return __builtin_bit_cast(bf16x8_t, make_uint4(pack2bf(a[0], a[1]), pack2bf(a[2], a[3]), pack2bf(b[0], b[1]),
                                                 pack2bf(b[2], b[3])));
}

__device__ __forceinline__ uint4 scale_bf16x8(uint4 v, float s) {
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) w[k] = pack2bf(__uint_as_float(w[k] << 16) * s, __uint_as_float(w[k] & 0xffff0000u) * s);
  return make_uint4(w[0], w[1], w[2], w[3]);
}

struct AttnShape {
  int64_t B, T, H, RS;  // RS = row stride of qkv (3*H*64)
};

// WavLM gated relative-position bias (components.py:629-651): score[b,h,q,k] += gate[b,h,q] * tab[h][k-q+T-1].
// tab holds the bucketed embedding already gathered per remaining head (dph_relpos_table), gate the per-query
// GRU gate (dph_wavlm_gate_fwd).  Backward: dgate[b,h,q] = sum_k dS*tab (row sums, written), dtab[h][r] +=
// sum over the diagonal r of dS*gate (LDS histogram per block, then global atomics).
struct RelBias {
  const float* tab;    // [H][2T-1]
  const float* gate;   // [B][H][T]
  float* dgate;        // [B][H][T]
  float* dtab;         // [H][2T-1], accumulated
  // deterministic mode: per-wave LDS histograms and each dQ block's diagonal sums as one row of this slab
  // [B][H][query blocks][T + RB - 1], added into dtab in a fixed order by relpos_dtab_reduce (NULL: float atomics)
  float* dtab_part;
};

// clamped diagonal index: rows / keys past T (masked to 0 probability) read a valid entry
__device__ __forceinline__ int rel_idx(int key, int q, int T32) {
  return min(key, T32 - 1) - min(q, T32 - 1) + T32 - 1;
}

// A block of RB query rows (or RB keys) over all T keys (queries) touches T + RB - 1 consecutive diagonals,
// starting at `off`: stage that window of the head's table in LDS (dynamic shared memory) once per block.
constexpr int RBW = 128;   // == RB (defined below), rows / keys per block
__device__ __forceinline__ void stage_tab_window(float* tw, const float* tab_h, int off, int T32) {
  for (int j = threadIdx.x; j < T32 + RBW - 1; j += 256) {
    const int gi = j + off;
    tw[j] = (gi >= 0 && gi < 2 * T32 - 1) ? tab_h[gi] : 0.f;
  }
}

// Dropout of the attention probabilities: element (row = (b*H+h)*T + q, key) draws 16 bits from ONE
// 32-bit hash per (row, key pair) -- rows padded to an even key count, so the 4 consecutive keys a
// lane holds in the forward / dQ kernels cost 2 hashes, and in the dK/dV kernel (4 queries of one
// key per lane) neighbouring lanes (keys 2m, 2m+1) split the hashing and swap halves.
__device__ __forceinline__ uint32_t attn_hash(uint64_t seed, uint64_t row, int64_t key, uint64_t half_tp) {
  return drop_bits2(seed, row * half_tp + (uint64_t)(key >> 1));
}

// drop_bits2 for pair indices below 2^32 (every attention shape: B*H*T*ceil(T/2) < 2^32 is checked on the
// host): the seed's high-word product is a per-launch constant, so a pair costs one xor + hash32
__device__ __forceinline__ uint32_t seed_mix(uint64_t seed) {
  return (uint32_t)seed ^ ((uint32_t)(seed >> 32) * 0x85EBCA6Bu);
}
__device__ __forceinline__ uint32_t attn_hash32(uint32_t mix, uint32_t pair) { return hash32(pair ^ mix); }

// packed-16 dropout test of one pair hash: 0xffff in each half whose 16 bits are below thr (dropped), else 0.
// (bits ^ 0x8000) - (thr - 0x8000) is the signed difference bits - thr shifted into int16 range; the saturating
// subtract keeps its sign, the arithmetic shift spreads it.  thr <= 65535 (p < 1).
typedef short s16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ s16x2_t drop_thr2(uint32_t thr) {
  const short t = (short)((int)min(thr, 65535u) - 32768);
  return s16x2_t{t, t};
}
__device__ __forceinline__ uint32_t drop_mask2(uint32_t bits, s16x2_t thr2) {
  const s16x2_t d = __builtin_elementwise_sub_sat(__builtin_bit_cast(s16x2_t, bits ^ 0x80008000u), thr2);
  return __builtin_bit_cast(uint32_t, d >> (short)15);
}

// Stored keep bits (forward -> backward): uint16 word (row, key tile kt, lane group g) holds the keep bit of
// key kt*64 + 16 s + 4 g + i at bit 4 s + i -- exactly the 16 keys lane group g of a row owns in the forward
// and dQ MFMA layouts, so those kernels move one aligned uint16 per row and tile, and the dK/dV kernel reads
// the row's whole 64-bit tile word.
constexpr float L2E = 1.4426950408889634f;

__device__ __forceinline__ float attn_keep(uint32_t bits, bool odd_key, uint32_t thr, float inv_keep) {
  return ((odd_key ? (bits >> 16) : (bits & 0xffffu)) >= thr) ? inv_keep : 0.f;
}

// (the select form: the WavLM dQ body, where the asm form's constant-bit SGPRs pushed the kernel into spills)
__device__ __forceinline__ float keep_scale_x(uint32_t word, int bit, float inv_keep) {
  return ((word >> bit) & 1u) ? inv_keep : 0.f;
}
// stored keep bit `bit` of `word` -> inv_keep (kept) or 0 (dropped): the bit sign-extended (v_bfe_i32) masks
// inv_keep's bits -- two VALU ops instead of an and / compare / select.  In asm: for a constant bit the compiler
// turns the builtin's bfe + and back into and / compare / select.  keep_scale: bit per lane (VGPR); keep_scale_u:
// bit uniform (SGPR, s_mov'd constants in the unrolled dQ loop).
__device__ __forceinline__ float keep_scale(uint32_t word, int bit, float inv_keep) {
  uint32_t r;
  asm("v_bfe_i32 %0, %1, %2, 1\n\tv_and_b32 %0, %3, %0" : "=&v"(r) : "v"(word), "v"(bit), "s"(inv_keep));
  return __uint_as_float(r);
}
__device__ __forceinline__ float keep_scale_u(uint32_t word, int bit, float inv_keep) {
  uint32_t r;
  asm("v_bfe_i32 %0, %1, %2, 1\n\tv_and_b32 %0, %3, %0" : "=&v"(r) : "v"(word), "s"(bit), "s"(inv_keep));
  return __uint_as_float(r);
}

// stage a [rows][64] bf16 tile (rows from row0, clamped to T) from column block col0 into LDS.
// swizzled: swz128 layout; else padded [rows][72].
template <int ROWS, bool SWZ>
__device__ __forceinline__ void stage_load(uint4 (&reg)[ROWS / 32], const bf16_t* base, int64_t row0, int64_t T,
                                           int64_t RS, float scale, int tid) {
#pragma unroll
  for (int i = 0; i < ROWS / 32; ++i) {
    const int c = tid + 256 * i;
    const int r = c >> 3;
    const int c8 = (c & 7) * 8;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (row0 + r < T) v = *reinterpret_cast<const uint4*>(base + (row0 + r) * RS + c8);
    if (scale != 1.0f) v = scale_bf16x8(v, scale);
    reg[i] = v;
  }
}

template <int ROWS, bool SWZ>
__device__ __forceinline__ void stage_store(char* lds, const uint4 (&reg)[ROWS / 32], int tid) {
#pragma unroll
  for (int i = 0; i < ROWS / 32; ++i) {
    const int c = tid + 256 * i;
    const int r = c >> 3;
    const int c8 = (c & 7) * 8;
    const int byte = SWZ ? swz128(r, c8) : (r * PADROW + c8) * 2;
    *reinterpret_cast<uint4*>(lds + byte) = reg[i];
  }
}

constexpr int KTILE_PAD_BYTES = KT * PADROW * 2;   // 9216
constexpr int TILE_SWZ_BYTES = KT * 128;           // 8192

// Each wave owns NG = 2 groups of 16 rows (queries in the forward / dQ kernels, keys in dK/dV), so
// every K / V (resp. Q / dO) fragment read from LDS feeds NG MFMAs: with one group per wave the
// fragment reads alone filled the CU's LDS bandwidth (~1 KB per 16-cycle MFMA per wave).
constexpr int NG = 2;
constexpr int RB = 4 * 16 * NG;   // rows per block: 128
static_assert(RB == RBW, "table window width");

// ---------------------------------------------------------------------------
// forward: block = (128 query rows, head h, utterance b), 4 waves x 2 x 16 rows.
// DROP is a template parameter and the key masks are selects on 32-bit key indices, so a tile is
// one basic block (runtime `if`s split it and kept hipcc from overlapping one query group's
// softmax with the other group's MFMAs).
// ---------------------------------------------------------------------------
template <bool DROP, bool BIAS, bool PREC>
__global__ void __launch_bounds__(256, 2) attn_fwd_kernel(const bf16_t* __restrict__ qkv, float* __restrict__ o_u,
                                                          bf16_t* __restrict__ o_m, float* __restrict__ lse,
                                                          const float* __restrict__ head_mask,
                                                          const int64_t* __restrict__ key_len, AttnShape sh,
                                                          float scale, float drop_p, uint64_t seed, RelBias rb,
                                                          uint16_t* __restrict__ keep_out) {
  seed = epoch_seed(seed);   // per-step RNG epoch (graph replays)
  const uint32_t mix = seed_mix(seed);
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * TILE_SWZ_BYTES];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int g = lane >> 4;
  const int64_t b = blockIdx.z;
  const int64_t h = blockIdx.y;
  const int64_t T = sh.T, H = sh.H, RS = sh.RS;
  const int T32 = (int)T;
  const int64_t q0 = (int64_t)blockIdx.x * RB + wave * 16 * NG;
  const bf16_t* rowbase = qkv + b * T * RS;
  const int klen = (int)(key_len ? key_len[b] : T);
  const uint64_t half_tp = (uint64_t)(T + 1) >> 1;
  int64_t qme[NG];
  uint64_t hrow[NG];   // dropout pair index of (row, key 0)
#pragma unroll
  for (int u = 0; u < NG; ++u) {
    qme[u] = q0 + 16 * u + (lane & 15);
    hrow[u] = ((uint64_t)(b * H + h) * T + (uint64_t)qme[u]) * half_tp;
  }
  extern __shared__ float tw[];   // BIAS: [T + RB - 1] table window of this block's diagonals
  const int toff = T32 - 1 - ((int)blockIdx.x * RB + RB - 1);
  if constexpr (BIAS) stage_tab_window(tw, rb.tab + h * (2 * T - 1), toff, T32);   // ordered by the first barrier
  float gq[NG];
#pragma unroll
  for (int u = 0; u < NG; ++u) gq[u] = (BIAS && qme[u] < T) ? rb.gate[(b * H + h) * T + qme[u]] : 0.f;

  // Q' = scale*q fragments (B operand of S^T = K Q'^T): Q'[q = lane&15][hd = 32ks + 8g + j]
  bf16x8_t qf[NG][2];
#pragma unroll
  for (int u = 0; u < NG; ++u)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      uint4 v = make_uint4(0, 0, 0, 0);
      if (qme[u] < T) v = *reinterpret_cast<const uint4*>(rowbase + qme[u] * RS + h * HD + ks * 32 + 8 * g);
      qf[u][ks] = __builtin_bit_cast(bf16x8_t, scale_bf16x8(v, scale));
    }

  f32x4_t oacc[NG][4];
  float m_run[NG], l_run[NG];
#pragma unroll
  for (int u = 0; u < NG; ++u) {
    m_run[u] = -INFINITY;
    l_run[u] = 0.f;
#pragma unroll
    for (int d = 0; d < 4; ++d) oacc[u][d] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  }
  const float inv_keep = DROP ? 1.f / (1.f - drop_p) : 1.f;
  const uint32_t thr = drop_thr(drop_p);

  const int nkt = (int)cdiv(T, KT);
  uint4 rk[2], rv[2];
  auto ldsK = [&](int buf) { return smem + buf * 2 * TILE_SWZ_BYTES; };
  auto ldsV = [&](int buf) { return smem + buf * 2 * TILE_SWZ_BYTES + TILE_SWZ_BYTES; };
  stage_load<KT, true>(rk, rowbase + (H + h) * HD, 0, T, RS, 1.0f, tid);
  stage_load<KT, true>(rv, rowbase + (2 * H + h) * HD, 0, T, RS, 1.0f, tid);
  stage_store<KT, true>(ldsK(0), rk, tid);
  stage_store<KT, true>(ldsV(0), rv, tid);
  __syncthreads();

  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nkt;
    if (more) {
      stage_load<KT, true>(rk, rowbase + (H + h) * HD, (int64_t)(kt + 1) * KT, T, RS, 1.0f, tid);
      stage_load<KT, true>(rv, rowbase + (2 * H + h) * HD, (int64_t)(kt + 1) * KT, T, RS, 1.0f, tid);
    }
    const char* K_ = ldsK(cur);
    const char* V_ = ldsV(cur);
    // S^T[key = 16s + 4g + i][q = lane&15] per query group
    f32x4_t sacc[NG][4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
#pragma unroll
      for (int u = 0; u < NG; ++u) sacc[u][s] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8_t kf = lds_b128(K_, swz128(16 * s + (lane & 15), ks * 32 + 8 * g));
#pragma unroll
        for (int u = 0; u < NG; ++u) sacc[u][s] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[u][ks], sacc[u][s], 0, 0, 0);
      }
    }
    const int kb = kt * KT + 4 * g;   // key of (s = 0, i = 0) for this lane
    // Softmax + dropout + PV of one tile.  MASKED: the tile holds padded (>= klen) or missing (>= T) keys;
    // every other tile skips the per-element compares (block-uniform choice).  exp via exp2 with log2(e)
    // folded into one fma per element: p = 2^(s*log2e - m*log2e).
    auto tile = [&](auto masked_c) {
      constexpr bool MASKED = decltype(masked_c)::value;
#pragma unroll
      for (int u = 0; u < NG; ++u) {
        float mt = -INFINITY;
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int key = kb + 16 * s + i;
            float v = sacc[u][s][i];
            if constexpr (BIAS) v += gq[u] * tw[rel_idx(key, (int)qme[u], T32) - toff];
            if constexpr (MASKED) {
              v = key >= klen ? v - 10000.0f : v;
              v = key >= T32 ? -INFINITY : v;
            }
            sacc[u][s][i] = v;
            mt = fmaxf(mt, v);
          }
        mt = fmaxf(mt, __shfl_xor(mt, 16, 64));
        mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
        const float m_new = fmaxf(m_run[u], mt);
        const float alpha = __builtin_amdgcn_exp2f((m_run[u] - m_new) * L2E);
        const float ml = m_new * L2E;
        float ls = 0.f;
        uint32_t kbits = 0;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          uint32_t hb[2] = {0u, 0u};
          if constexpr (DROP) {
            const uint32_t pr = (uint32_t)(hrow[u] + (uint64_t)((kb + 16 * s) >> 1));
            hb[0] = attn_hash32(mix, pr);
            hb[1] = attn_hash32(mix, pr + 1);
          }
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float p = __builtin_amdgcn_exp2f(fmaf(sacc[u][s][i], L2E, -ml));
            ls += p;
            if constexpr (DROP) {
              const bool keep = ((i & 1) ? (hb[i >> 1] >> 16) : (hb[i >> 1] & 0xffffu)) >= thr;
              kbits |= (keep ? 1u : 0u) << (4 * s + i);
              sacc[u][s][i] = keep ? p * inv_keep : 0.f;
            } else {
              sacc[u][s][i] = p;
            }
          }
        }
        if constexpr (DROP) {
          if (keep_out != nullptr && qme[u] < T)
            keep_out[((b * H + h) * T + qme[u]) * (nkt * 4) + kt * 4 + g] = (uint16_t)kbits;
        }
        ls += __shfl_xor(ls, 16, 64);
        ls += __shfl_xor(ls, 32, 64);
        l_run[u] = l_run[u] * alpha + ls;
        m_run[u] = m_new;
#pragma unroll
        for (int d = 0; d < 4; ++d)
#pragma unroll
          for (int i = 0; i < 4; ++i) oacc[u][d][i] *= alpha;
        // O^T[d][q] += V^T[d][key] P^T[key][q]; k index of step kk: key(g,j) = 16(2kk + j/4) + 4g + j%4
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const bf16x8_t pf = pack_frag(sacc[u][2 * kk], sacc[u][2 * kk + 1]);
          bf16x8_t pl;   // PREC: residuals p - bf16(p) (see launch_fwd)
          if constexpr (PREC) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              pl[j] = (__bf16)(sacc[u][2 * kk][j] - (float)pf[j]);
              pl[4 + j] = (__bf16)(sacc[u][2 * kk + 1][j] - (float)pf[4 + j]);
            }
          }
#pragma unroll
          for (int d = 0; d < 4; ++d) {
            const bf16x8_t vf = tr_frag(V_, 32 * kk + 4 * g, 32 * kk + 16 + 4 * g, 16 * d, lane);
            oacc[u][d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf, oacc[u][d], 0, 0, 0);
            if constexpr (PREC) oacc[u][d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pl, oacc[u][d], 0, 0, 0);
          }
        }
      }
    };
    // (the WavLM-bias instantiations keep one masked body: a second copy spills registers there)
    if (!BIAS && (kt + 1) * KT <= klen && (kt + 1) * KT <= T32) tile(std::integral_constant<bool, BIAS>());
    else tile(std::integral_constant<bool, true>());
    if (more) {
      stage_store<KT, true>(ldsK(cur ^ 1), rk, tid);
      stage_store<KT, true>(ldsV(cur ^ 1), rv, tid);
    }
    __syncthreads();
  }

  const float hm = head_mask ? head_mask[h] : 1.0f;
#pragma unroll
  for (int u = 0; u < NG; ++u) {
    if (qme[u] >= T) continue;
    const float inv_l = 1.0f / l_run[u];
    const int64_t obase = (b * T + qme[u]) * (H * HD) + h * HD;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const int col = 16 * d + 4 * g;
      float v[4] = {oacc[u][d][0] * inv_l, oacc[u][d][1] * inv_l, oacc[u][d][2] * inv_l, oacc[u][d][3] * inv_l};
      // fp32: the backward's D = rowsum(dO * O) must cancel against sum_j P_j dP_j to fp32 accuracy (a bf16 O
      // leaves 2^-9 |dO||v| of noise in every dS, which dominates dQ / dK where the softmax saturates)
      if (o_u) *reinterpret_cast<float4*>(o_u + obase + col) = make_float4(v[0], v[1], v[2], v[3]);
      *reinterpret_cast<uint2*>(o_m + obase + col) =
          make_uint2(pack2bf(v[0] * hm, v[1] * hm), pack2bf(v[2] * hm, v[3] * hm));
    }
    if (g == 0 && lse) lse[(b * H + h) * T + qme[u]] = m_run[u] + __logf(l_run[u]);
  }
}

// ---------------------------------------------------------------------------
// forward on v_mfma_f32_32x32x16_bf16 (HuBERT / wav2vec2: no relative-position bias).  Each wave owns 32
// query rows as the N side of S^T = K Q'^T (a 32 x 32 accumulator: lane l holds query q = l & 31 and keys
// 8 (r >> 2) + 4 (l >> 5) + (r & 3) of a 32-key subtile), so a row's softmax is in-lane plus one
// exchange with lane l ^ 32.  The P accumulator registers 8e..8e+7 ARE the B operand of the k-step e of
// O^T += V^T P^T once the k index is read as that key permutation; the V^T A operand follows it with
// two transposed LDS reads (rows base + 4 hi + 0..3 and base + 8 + 4 hi + 0..3).  Against the 16 x 16 x 32
// form: the same MFMA cycles, 16 instead of 24 KB of LDS fragment reads per wave and 64-key tile (V is
// read once, not once per 16-row group), half the MFMA instructions.
// LDS: K rows of 128 B with 16-B chunk c at position c ^ ((r >> 1) & 7) (the 32 rows x 2 chunks of a
// b128 K-fragment read are bank-conflict free), V in the vswz image of its transposed reads.
// ---------------------------------------------------------------------------
typedef __attribute__((ext_vector_type(16))) float f32x16_t;
constexpr float RESCALE_TH = 8.0f;   // deferred-max threshold of the 32 x 32 forward (score units)

__device__ __forceinline__ int kswz(int r, int chunk) { return r * 128 + ((chunk ^ ((r >> 1) & 7)) << 4); }

// V image of the 32 x 32 forward: 32-B unit u of row r at u ^ (2 ((r >> 1) & 1)).  A transposed A-operand read
// puts, per half-wave, rows r0..r0+3 (r0 % 4 == 0) x units {2d, 2d+1} in one LDS cycle: these 8 segments land
// on 8 distinct (row parity, unit) bank groups.  (swz128, the 16 x 16 kernels' image, maps two of them onto
// one group: 65 % of the LDS cycles were conflict cycles, SQ_LDS_BANK_CONFLICT.)
__device__ __forceinline__ int vswz(int r, int col) {
  return r * 128 + ((((col >> 4) ^ (((r >> 1) & 1) << 1)) & 3) * 32) + (col & 15) * 2;
}

__device__ __forceinline__ bf16x8_t tr_frag_v(const char* lds, int r0, int r1, int c0, int lane) {
  const int i = lane & 15;
  const int q = i >> 2;
  const int p = i & 3;
  s16x4_t v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + vswz(r0 + q, c0 + 4 * p)));
  s16x4_t v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + vswz(r1 + q, c0 + 4 * p)));
  s16x8_t v = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
  return __builtin_bit_cast(bf16x8_t, v);
}

__device__ __forceinline__ bf16x8_t pack8(const f32x16_t& a, int base) {
  uint4 w;
  w.x = pack2bf(a[base + 0], a[base + 1]);
  w.y = pack2bf(a[base + 2], a[base + 3]);
  w.z = pack2bf(a[base + 4], a[base + 5]);
  w.w = pack2bf(a[base + 6], a[base + 7]);
  return __builtin_bit_cast(bf16x8_t, w);
}

template <bool DROP>
__global__ void __launch_bounds__(256, 2) attn_fwd32_kernel(const bf16_t* __restrict__ qkv, float* __restrict__ o_u,
                                                           bf16_t* __restrict__ o_m, float* __restrict__ lse,
                                                           const float* __restrict__ head_mask,
                                                           const int64_t* __restrict__ key_len, AttnShape sh,
                                                           float scale, float drop_p, uint64_t seed,
                                                           uint16_t* __restrict__ keep_out) {
  seed = epoch_seed(seed);
  const uint32_t mix = seed_mix(seed);
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * TILE_SWZ_BYTES];   // [buf][K | V][64 rows x 128 B]
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int hi = lane >> 5;
  const int b = blockIdx.z;
  const int h = blockIdx.y;
  const int T32 = (int)sh.T, H = (int)sh.H;
  const int64_t RS = sh.RS;
  const int q = (int)blockIdx.x * RB + wave * 32 + (lane & 31);
  const bf16_t* rowbase = qkv + (int64_t)b * sh.T * RS;
  const int klen = (int)(key_len ? key_len[b] : sh.T);
  const uint32_t half_tp = (uint32_t)(T32 + 1) >> 1;
  const uint32_t hrow = ((uint32_t)(b * H + h) * (uint32_t)T32 + (uint32_t)q) * half_tp;
  // a head whose sampled HardConcrete mask is exactly 0 (clamped, hardconcrete.py:99) contributes nothing and gets no
  // gradient through its mask: the masked output is 0 and nothing else of it is read (the backward skips it too)
  if (head_mask != nullptr && head_mask[h] == 0.f) {
    if (q < T32) {
      bf16_t* orow = o_m + ((int64_t)b * T32 + q) * (H * HD) + h * HD + 32 * hi;
#pragma unroll
      for (int c = 0; c < 4; ++c) *reinterpret_cast<uint4*>(orow + 8 * c) = make_uint4(0, 0, 0, 0);
    }
    return;
  }
  // Q' = scale * q as the B operand: qf[t] = Q'[q][16 t + 8 hi + 0..7]
  bf16x8_t qf[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    uint4 v = make_uint4(0, 0, 0, 0);
    if (q < T32) v = *reinterpret_cast<const uint4*>(rowbase + (int64_t)q * RS + h * HD + 16 * t + 8 * hi);
    qf[t] = __builtin_bit_cast(bf16x8_t, scale_bf16x8(v, scale));
  }
  f32x16_t oacc[2];
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) oacc[d][r] = 0.f;
  float m_run = -INFINITY, l_run = 0.f;
  const float inv_keep = DROP ? 1.f / (1.f - drop_p) : 1.f;
  const uint32_t thr = drop_thr(drop_p);
  const int nkt = (T32 + KT - 1) / KT;
  uint4 rk[2], rv[2];
  auto ldsK = [&](int buf) { return smem + buf * 2 * TILE_SWZ_BYTES; };
  auto ldsV = [&](int buf) { return smem + buf * 2 * TILE_SWZ_BYTES + TILE_SWZ_BYTES; };
  auto store_kv = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + 256 * i;
      const int r = c >> 3;
      *reinterpret_cast<uint4*>(ldsK(buf) + kswz(r, c & 7)) = rk[i];
      *reinterpret_cast<uint4*>(ldsV(buf) + vswz(r, (c & 7) * 8)) = rv[i];
    }
  };
  stage_load<KT, false>(rk, rowbase + (H + h) * HD, 0, sh.T, RS, 1.0f, tid);
  stage_load<KT, true>(rv, rowbase + (2 * H + h) * HD, 0, sh.T, RS, 1.0f, tid);
  store_kv(0);
  __syncthreads();

  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nkt;
    if (more) {
      stage_load<KT, false>(rk, rowbase + (H + h) * HD, (int64_t)(kt + 1) * KT, sh.T, RS, 1.0f, tid);
      stage_load<KT, true>(rv, rowbase + (2 * H + h) * HD, (int64_t)(kt + 1) * KT, sh.T, RS, 1.0f, tid);
    }
    const char* K_ = ldsK(cur);
    const char* V_ = ldsV(cur);
    f32x16_t sacc[2];
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const bf16x8_t kf = lds_b128(K_, kswz(32 * k2 + (lane & 31), 2 * t + hi));
        // (t = 0: the zero accumulator as the MFMA's inline-constant C operand, no register zeroing)
        sacc[k2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[t], t == 0 ? f32x16_t{} : sacc[k2], 0, 0, 0);
      }
    }
    const int kb = kt * KT + 4 * hi;   // key of (k2 = 0, r = 0) in this lane
    auto tile = [&](auto masked_c) {
      constexpr bool MASKED = decltype(masked_c)::value;
      float mt = -INFINITY;
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float v = sacc[k2][r];
          if constexpr (MASKED) {
            const int key = kb + 32 * k2 + 8 * (r >> 2) + (r & 3);
            v = key >= klen ? v - 10000.0f : v;
            v = key >= T32 ? -INFINITY : v;
          }
          sacc[k2][r] = v;
          mt = fmaxf(mt, v);
        }
      mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
      // deferred rescale: the running max moves only when a row's tile max exceeds it by more than
      // RESCALE_TH (p <= e^8 meanwhile: no overflow, the same relative bf16 rounding), and the 32 O
      // rescale multiplies run only when some row of the wave moved (wave-uniform branch)
      const bool move = mt > m_run + RESCALE_TH;
      if (__any(move)) {
        const float m_new = move ? mt : m_run;
        const float alpha = __builtin_amdgcn_exp2f((m_run - m_new) * L2E);
        l_run *= alpha;
        m_run = m_new;
#pragma unroll
        for (int d = 0; d < 2; ++d)
#pragma unroll
          for (int r = 0; r < 16; ++r) oacc[d][r] *= alpha;
      }
      const float ml = m_run * L2E;
      float ls = 0.f;
      uint32_t kw[2] = {0u, 0u};   // stored keep words hi and 2 + hi of this row and tile
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2)
#pragma unroll
        for (int rq = 0; rq < 4; ++rq) {
          uint32_t hb[2] = {0u, 0u};
          if constexpr (DROP) {
            const uint32_t pr = hrow + (uint32_t)((kb + 32 * k2 + 8 * rq) >> 1);
            hb[0] = attn_hash32(mix, pr);
            hb[1] = attn_hash32(mix, pr + 1);
          }
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int r = 4 * rq + i;
            const float p = __builtin_amdgcn_exp2f(fmaf(sacc[k2][r], L2E, -ml));
            ls += p;
            if constexpr (DROP) {
              const bool keep = ((i & 1) ? (hb[i >> 1] >> 16) : (hb[i >> 1] & 0xffffu)) >= thr;
              kw[rq & 1] |= (keep ? 1u : 0u) << (4 * (2 * k2 + (rq >> 1)) + i);
              sacc[k2][r] = keep ? p : 0.f;   // (1 / (1 - p) applied once to O at the end)
            } else {
              sacc[k2][r] = p;
            }
          }
        }
      if constexpr (DROP) {
        if (keep_out != nullptr && q < T32) {
          uint16_t* kp = keep_out + ((int64_t)(b * H + h) * T32 + q) * (nkt * 4) + kt * 4;
          kp[hi] = (uint16_t)kw[0];
          kp[2 + hi] = (uint16_t)kw[1];
        }
      }
      ls += __shfl_xor(ls, 32, 64);
      l_run += ls;
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2)
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const bf16x8_t pf = pack8(sacc[k2], 8 * e);
          const int base = 32 * k2 + 16 * e + 4 * hi;
#pragma unroll
          for (int d = 0; d < 2; ++d) {
            const bf16x8_t vf = tr_frag_v(V_, base, base + 8, 32 * d + 16 * ((lane >> 4) & 1), lane);
            oacc[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf, oacc[d], 0, 0, 0);
          }
        }
    };
    if ((kt + 1) * KT <= klen && (kt + 1) * KT <= T32) tile(std::integral_constant<bool, false>());
    else tile(std::integral_constant<bool, true>());
    if (more) store_kv(cur ^ 1);
    __syncthreads();
  }

  if (q >= T32) return;
  const float hm = head_mask ? head_mask[h] : 1.0f;
  const float inv_l = inv_keep / l_run;
  const int64_t obase = ((int64_t)b * T32 + q) * (H * HD) + h * HD;
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int rq = 0; rq < 4; ++rq) {
      const int col = 32 * d + 8 * rq + 4 * hi;
      float v[4] = {oacc[d][4 * rq] * inv_l, oacc[d][4 * rq + 1] * inv_l, oacc[d][4 * rq + 2] * inv_l,
                    oacc[d][4 * rq + 3] * inv_l};
      if (o_u) *reinterpret_cast<float4*>(o_u + obase + col) = make_float4(v[0], v[1], v[2], v[3]);
      *reinterpret_cast<uint2*>(o_m + obase + col) =
          make_uint2(pack2bf(v[0] * hm, v[1] * hm), pack2bf(v[2] * hm, v[3] * hm));
    }
  if (hi == 0 && lse) lse[(int64_t)(b * H + h) * T32 + q] = m_run + __logf(l_run);
}

// ---------------------------------------------------------------------------
// The 32 x 32 forward, restructured for VALU issue (PMC, profiles/r4_s2_pmcattn_summary.txt: 18.4 VALU
// instructions per MFMA at p = 0, 34.6 at p = 0.1, MFMA busy 10-13 %: the kernel is VALU-issue bound):
//  * key tiles that need no mask run in a loop of their own and the masked tile(s) after it, so the O
//    accumulators flow straight from one loop into the next (the old single loop with a masked / unmasked
//    branch inside compiled to 32 v_mov_b64 phi copies of the accumulators per tile);
//  * tiles wholly past the key length are skipped: their scores carry the -1e4 key mask
//    (components.py:411-415) and exp2 of (s - 1e4 - max) * log2(e) is exactly 0 in fp32, so they add
//    nothing to O or to the row sum (when every key is masked -- key_len 0 -- all tiles run masked);
//  * K / V tile loads clamp their rows to T - 1 instead of branching per row (rows past T only feed keys
//    the mask zeroes);
//  * the eight K fragments of a tile are read before its first MFMA (the compiler otherwise waited
//    lgkmcnt(0) on each read in front of its MFMA);
//  * the row sum is four interleaved chains instead of one 32-deep dependent chain;
//  * P is packed to bf16 pairs as soon as it is computed and the dropout is applied to the packed word
//    (drop_mask2: three packed-16 ops per hashed key pair, 41 -> 40.8 us with stored keep bits);
//  * the staged K / V rows live in four named registers (as an array captured by the lambdas they were
//    demoted to 80 B per lane of scratch: 47.4 -> 31.1 us at p = 0, profiles/r4_s4_attn_fwd_ab.txt).
// Where the rest goes (B = 16, T = 499, p = 0, profiles/r4_s6_attn_fwd_breakdown.txt, knobs since removed):
// without the fp32 o_u store 27.2 us, without any output store 24.2, without the K / V loads past the first
// tile 27.9, with exp2 replaced by its argument 29.1, with all of these 20.3 -- the MFMA work alone is 4.9 us.
// Same arithmetic per score as attn_fwd32_kernel; keep bits in the same layout (tiles past the key length
// are not written: their probabilities are 0 and the backward multiplies whatever it reads there by 0).
// ---------------------------------------------------------------------------
// STAGE: the epilogue goes through LDS (the K / V tiles' space, free after the loop's last barrier): each wave writes
// its 32 x 64 normalised O rows there and re-reads them row-contiguous, so every global store instruction writes
// whole rows (o_u: 4 rows of 256 B, o_m: 4 rows of 128 B per wave instruction) instead of 16-B / 8-B pieces of 32
// rows (the store tail of a one-round grid: guide T21, MI355X_MICROARCH 'attention epilogue store tail')
template <bool DROP, bool STAGE, bool PREC>
__global__ void __launch_bounds__(256, 3) attn_fwd32v2_kernel(const bf16_t* __restrict__ qkv, float* __restrict__ o_u,
                                                             bf16_t* __restrict__ o_m, float* __restrict__ lse,
                                                             const float* __restrict__ head_mask,
                                                             const int64_t* __restrict__ key_len, AttnShape sh,
                                                             float scale, float drop_p, uint64_t seed,
                                                             uint16_t* __restrict__ keep_out) {
  seed = epoch_seed(seed);
  const uint32_t mix = seed_mix(seed);
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * TILE_SWZ_BYTES];   // [buf][K | V][64 rows x 128 B]
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int hi = lane >> 5;
  const int b = blockIdx.z;
  const int h = blockIdx.y;
  const int T32 = (int)sh.T, H = (int)sh.H;
  const int64_t RS = sh.RS;
  const int q = (int)blockIdx.x * RB + wave * 32 + (lane & 31);
  const bf16_t* rowbase = qkv + (int64_t)b * sh.T * RS;
  const int klen = (int)(key_len ? key_len[b] : sh.T);
  const uint32_t half_tp = (uint32_t)(T32 + 1) >> 1;
  const uint32_t hrow = ((uint32_t)(b * H + h) * (uint32_t)T32 + (uint32_t)q) * half_tp;
  if (head_mask != nullptr && head_mask[h] == 0.f) {
    if (q < T32) {
      bf16_t* orow = o_m + ((int64_t)b * T32 + q) * (H * HD) + h * HD + 32 * hi;
#pragma unroll
      for (int c = 0; c < 4; ++c) *reinterpret_cast<uint4*>(orow + 8 * c) = make_uint4(0, 0, 0, 0);
    }
    return;
  }
  bf16x8_t qf[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    uint4 v = make_uint4(0, 0, 0, 0);
    if (q < T32) v = *reinterpret_cast<const uint4*>(rowbase + (int64_t)q * RS + h * HD + 16 * t + 8 * hi);
    qf[t] = __builtin_bit_cast(bf16x8_t, scale_bf16x8(v, scale));
  }
  f32x16_t oacc[2];
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) oacc[d][r] = 0.f;
  float m_run = -INFINITY, l_run = 0.f;
  const float inv_keep = DROP ? 1.f / (1.f - drop_p) : 1.f;
  const uint32_t thr = drop_thr(drop_p);
  const s16x2_t thr2 = drop_thr2(thr);
  const int nkt = (T32 + KT - 1) / KT;                      // keep-word stride (layout of every tile)
  const int kend = (klen >= 1 && klen < T32) ? klen : T32;  // keys that can carry probability
  const int ntile = (kend + KT - 1) / KT;
  const int nfull = klen >= 1 ? kend / KT : 0;              // tiles with no masked key
  // staged K / V rows as four named registers (an array of them, captured by the lambdas, was demoted to
  // scratch memory: 80 bytes per lane of scratch stores and loads per tile)
  uint4 rk0, rk1, rv0, rv1;
  auto ldsK = [&](int buf) { return smem + buf * 2 * TILE_SWZ_BYTES; };
  auto ldsV = [&](int buf) { return smem + buf * 2 * TILE_SWZ_BYTES + TILE_SWZ_BYTES; };
  // K / V rows of key tile kt (rows clamped to T - 1: no per-row branch)
  const int c8 = (tid & 7) * 8;
  auto load_kv = [&](int kt) {
    const int r0 = min(kt * KT + (tid >> 3), T32 - 1);
    const int r1 = min(kt * KT + 32 + (tid >> 3), T32 - 1);
    const bf16_t* kb0 = rowbase + (int64_t)r0 * RS + (H + h) * HD + c8;
    const bf16_t* kb1 = rowbase + (int64_t)r1 * RS + (H + h) * HD + c8;
    rk0 = *reinterpret_cast<const uint4*>(kb0);
    rk1 = *reinterpret_cast<const uint4*>(kb1);
    rv0 = *reinterpret_cast<const uint4*>(kb0 + H * HD);
    rv1 = *reinterpret_cast<const uint4*>(kb1 + H * HD);
  };
  auto store_kv = [&](int buf) {
    const int r = tid >> 3;
    *reinterpret_cast<uint4*>(ldsK(buf) + kswz(r, tid & 7)) = rk0;
    *reinterpret_cast<uint4*>(ldsV(buf) + vswz(r, c8)) = rv0;
    *reinterpret_cast<uint4*>(ldsK(buf) + kswz(r + 32, tid & 7)) = rk1;
    *reinterpret_cast<uint4*>(ldsV(buf) + vswz(r + 32, c8)) = rv1;
  };
  load_kv(0);
  store_kv(0);
  __syncthreads();

  auto body = [&](int kt, auto masked_c) {
    constexpr bool MASKED = decltype(masked_c)::value;
    const int cur = kt & 1;
    const bool more = kt + 1 < ntile;
    if (more) load_kv(kt + 1);
    const char* K_ = ldsK(cur);
    const char* V_ = ldsV(cur);
    bf16x8_t kf[2][4];
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2)
#pragma unroll
      for (int t = 0; t < 4; ++t) kf[k2][t] = lds_b128(K_, kswz(32 * k2 + (lane & 31), 2 * t + hi));
    f32x16_t sacc[2];
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2)
#pragma unroll
      for (int t = 0; t < 4; ++t)
        sacc[k2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[k2][t], qf[t], t == 0 ? f32x16_t{} : sacc[k2], 0, 0, 0);
    const int kb = kt * KT + 4 * hi;   // key of (k2 = 0, r = 0) in this lane
    float mt = -INFINITY;
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float v = sacc[k2][r];
        if constexpr (MASKED) {
          const int key = kb + 32 * k2 + 8 * (r >> 2) + (r & 3);
          v = key >= klen ? v - 10000.0f : v;
          v = key >= T32 ? -INFINITY : v;
          sacc[k2][r] = v;
        }
        mt = fmaxf(mt, v);
      }
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
    const bool move = mt > m_run + RESCALE_TH;
    if (__any(move)) {
      const float m_new = move ? mt : m_run;
      const float alpha = __builtin_amdgcn_exp2f((m_run - m_new) * L2E);
      l_run *= alpha;
      m_run = m_new;
#pragma unroll
      for (int d = 0; d < 2; ++d)
#pragma unroll
        for (int r = 0; r < 16; ++r) oacc[d][r] *= alpha;
    }
    const float ml = m_run * L2E;
    float ls[4] = {0.f, 0.f, 0.f, 0.f};
    // P packed to bf16 pairs right away (keys 2m, 2m+1 -- the pair one hash draws for), the dropout applied
    // to the packed word: per 16-bit half, (bits ^ 0x8000) - (thr - 0x8000) saturating is negative exactly when
    // bits < thr, and its arithmetic shift by 15 is the half's drop mask.  Three packed-16 ops and two bitops
    // per PAIR instead of an extract / compare / select / bit-insert per score.
    uint32_t pw[2][4][2];
    uint32_t pl[2][4][2];        // PREC: bf16 residual words p - bf16(p)
    uint32_t kd[2] = {0u, 0u};   // DROP bits of the rq-even / rq-odd stored words: even key low half, odd high
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2)
#pragma unroll
      for (int rq = 0; rq < 4; ++rq) {
        float pv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 4 * rq + i;
          pv[i] = __builtin_amdgcn_exp2f(fmaf(sacc[k2][r], L2E, -ml));
          ls[i] += pv[i];
        }
#pragma unroll
        for (int pi = 0; pi < 2; ++pi) {
          uint32_t w = pack2bf(pv[2 * pi], pv[2 * pi + 1]);
          if constexpr (PREC)
            pl[k2][rq][pi] = pack2bf(pv[2 * pi] - __uint_as_float(w << 16),
                                     pv[2 * pi + 1] - __uint_as_float(w & 0xffff0000u));
          if constexpr (DROP) {
            const uint32_t hsh = attn_hash32(mix, hrow + (uint32_t)((kb + 32 * k2 + 8 * rq) >> 1) + pi);
            const uint32_t m = drop_mask2(hsh, thr2);
            w &= ~m;
            if constexpr (PREC) pl[k2][rq][pi] &= ~m;
            const int bt = 4 * (2 * k2 + (rq >> 1)) + 2 * pi;
            kd[rq & 1] |= m & ((1u << bt) | (1u << (17 + bt)));
          }
          pw[k2][rq][pi] = w;
        }
      }
    if constexpr (DROP) {
      if (keep_out != nullptr && q < T32) {
        uint16_t* kp = keep_out + ((int64_t)(b * H + h) * T32 + q) * (nkt * 4) + kt * 4;
        kp[hi] = (uint16_t)~(kd[0] | (kd[0] >> 16));
        kp[2 + hi] = (uint16_t)~(kd[1] | (kd[1] >> 16));
      }
    }
    float lsum = (ls[0] + ls[1]) + (ls[2] + ls[3]);
    lsum += __shfl_xor(lsum, 32, 64);
    l_run += lsum;
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const uint4 pq = make_uint4(pw[k2][2 * e][0], pw[k2][2 * e][1], pw[k2][2 * e + 1][0], pw[k2][2 * e + 1][1]);
        const bf16x8_t pf = __builtin_bit_cast(bf16x8_t, pq);
        const int base = 32 * k2 + 16 * e + 4 * hi;
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          const bf16x8_t vf = tr_frag_v(V_, base, base + 8, 32 * d + 16 * ((lane >> 4) & 1), lane);
          oacc[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf, oacc[d], 0, 0, 0);
          if constexpr (PREC) {
            const uint4 lq = make_uint4(pl[k2][2 * e][0], pl[k2][2 * e][1], pl[k2][2 * e + 1][0], pl[k2][2 * e + 1][1]);
            oacc[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, __builtin_bit_cast(bf16x8_t, lq), oacc[d], 0, 0, 0);
          }
        }
      }
    if (more) store_kv(cur ^ 1);
    __syncthreads();
  };
  int kt = 0;
  for (; kt < nfull; ++kt) body(kt, std::integral_constant<bool, false>());
  for (; kt < ntile; ++kt) body(kt, std::integral_constant<bool, true>());

  const float hm = head_mask ? head_mask[h] : 1.0f;
  const float inv_l = inv_keep / l_run;
  if constexpr (STAGE) {
    // (every wave passed the last tile's barrier: the 32 KB of K / V buffers are free; 4 waves x 32 rows x 68
    // floats = 34 KB would not fit, so each wave stages its rows in two halves of 16 rows)
    constexpr int OST = 68;                              // padded row (floats)
    float* ob = reinterpret_cast<float*>(smem) + wave * (16 * OST);
    const int r = lane & 31;
    const int qb = (int)blockIdx.x * RB + wave * 32;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      if ((r >> 4) == half) {
#pragma unroll
        for (int d = 0; d < 2; ++d)
#pragma unroll
          for (int rq = 0; rq < 4; ++rq) {
            const int col = 32 * d + 8 * rq + 4 * hi;
            *reinterpret_cast<float4*>(ob + (r & 15) * OST + col) =
                make_float4(oacc[d][4 * rq] * inv_l, oacc[d][4 * rq + 1] * inv_l, oacc[d][4 * rq + 2] * inv_l,
                            oacc[d][4 * rq + 3] * inv_l);
          }
      }
      __syncthreads();
      // 16 lanes per row (16 B each), 4 rows per wave instruction
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int rr = 4 * i + (lane >> 4);
        const int cc = (lane & 15) * 4;
        const int qr = qb + 16 * half + rr;
        const float4 v = *reinterpret_cast<const float4*>(ob + rr * OST + cc);
        if (qr < T32) {
          const int64_t ob2 = ((int64_t)b * T32 + qr) * (H * HD) + h * HD + cc;
          if (o_u) *reinterpret_cast<float4*>(o_u + ob2) = v;
          *reinterpret_cast<uint2*>(o_m + ob2) = make_uint2(pack2bf(v.x * hm, v.y * hm), pack2bf(v.z * hm, v.w * hm));
        }
      }
      if (half == 0) __syncthreads();
    }
    if (hi == 0 && lse && q < T32) lse[(int64_t)(b * H + h) * T32 + q] = m_run + __logf(l_run);
    return;
  }
  if (q >= T32) return;
  const int64_t obase = ((int64_t)b * T32 + q) * (H * HD) + h * HD;
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int rq = 0; rq < 4; ++rq) {
      const int col = 32 * d + 8 * rq + 4 * hi;
      float v[4] = {oacc[d][4 * rq] * inv_l, oacc[d][4 * rq + 1] * inv_l, oacc[d][4 * rq + 2] * inv_l,
                    oacc[d][4 * rq + 3] * inv_l};
      if (o_u) *reinterpret_cast<float4*>(o_u + obase + col) = make_float4(v[0], v[1], v[2], v[3]);
      *reinterpret_cast<uint2*>(o_m + obase + col) =
          make_uint2(pack2bf(v[0] * hm, v[1] * hm), pack2bf(v[2] * hm, v[3] * hm));
    }
  if (hi == 0 && lse) lse[(int64_t)(b * H + h) * T32 + q] = m_run + __logf(l_run);
}

// ---------------------------------------------------------------------------
// backward prep: D[b][h][t] = rowdot = sum_d dO_m * O_u ; dhm[h] += sum rowdot
// Eight lanes per (row, head), 8 columns each: consecutive lanes read consecutive 16 B of dO_m and 32 B of O_u
// (the row's H heads are contiguous), so a wave's loads are whole cache lines; the 8 partials meet in three xor
// steps.  (One thread per (row, head) -- each lane 384 B of its own rows, 64 rows per load instruction -- ran at
// 2.3 TB/s: 15.8 us per 7984 x 768 launch.)  Block = PREP_IT groups of rpb rows x all heads.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int prep_rpb(int64_t H) { return H <= 32 ? 4 : 1; }
constexpr int PREP_IT = 8;   // row groups per block (all loads issued first): 32 rows per block at H <= 32

__global__ void __launch_bounds__(1024) attn_bwd_prep_kernel(const bf16_t* __restrict__ dom,
                                                             const float* __restrict__ ou,
                                                             const float* __restrict__ head_mask,
                                                             float* __restrict__ Dv, float* __restrict__ dhm,
                                                             int64_t B, int64_t T, int64_t H,
                                                             float* __restrict__ part) {
  __shared__ float red[4 * 128];   // [row of the group][head] (H <= 128)
  const int rpb = prep_rpb(H);
  const int per_row = (int)H * 8;
  const int r = (int)threadIdx.x / per_row;
  const int ci = (int)threadIdx.x % per_row;   // 16-B chunk of dO_m within the row
  const int64_t h = ci >> 3;
  const float hmh = head_mask ? head_mask[h] : 1.0f;
  int64_t bt[PREP_IT];
  uint4 va[PREP_IT];
  float4 c0[PREP_IT], c1[PREP_IT];
#pragma unroll
  for (int it = 0; it < PREP_IT; ++it) {
    bt[it] = ((int64_t)blockIdx.x * PREP_IT + it) * rpb + r;   // each row group: rpb consecutive rows
    va[it] = make_uint4(0u, 0u, 0u, 0u);
    c0[it] = c1[it] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (bt[it] < B * T && hmh != 0.f) {   // (a skipped head's unmasked output was never written: D = 0)
      va[it] = *reinterpret_cast<const uint4*>(dom + bt[it] * H * HD + ci * 8);
      c0[it] = *reinterpret_cast<const float4*>(ou + bt[it] * H * HD + ci * 8);
      c1[it] = *reinterpret_cast<const float4*>(ou + bt[it] * H * HD + ci * 8 + 4);
    }
  }
  float hsum = 0.f;   // this (row slot, head)'s rowdots over the row groups, in group order
#pragma unroll
  for (int it = 0; it < PREP_IT; ++it) {
    const float wc[8] = {c0[it].x, c0[it].y, c0[it].z, c0[it].w, c1[it].x, c1[it].y, c1[it].z, c1[it].w};
    const uint32_t wa[4] = {va[it].x, va[it].y, va[it].z, va[it].w};
    float rd = 0.f;   // rowdot(dO_m, O_u): D and the head-mask gradient
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      rd += __uint_as_float(wa[q] << 16) * wc[2 * q];
      rd += __uint_as_float(wa[q] & 0xffff0000u) * wc[2 * q + 1];
    }
    // (the 8 lanes of a head group are aligned: per_row is a multiple of 8)
    rd += __shfl_xor(rd, 1, 64);
    rd += __shfl_xor(rd, 2, 64);
    rd += __shfl_xor(rd, 4, 64);
    // D = rowdot(dO_m, O_u): the dK / dV and dQ kernels form dP from the same bf16 dO_m (the head mask factors
    // out of dP, D and dS and is applied to their fp32 outputs), so D = sum_j P_j dP_j holds for THOSE dP_j --
    // with a D from another rounding of dO than dP's, dS = P (dP - D) keeps a row sum that the O-weighted key
    // sums of dQ / dK multiply by the keys' common component (a 0.99 head mask put the 12-layer fixture's
    // last-layer dW_q off by 50 % before round 5)
    if (bt[it] < B * T && (ci & 7) == 0) {
      const int64_t bb = bt[it] / T, t = bt[it] % T;
      Dv[(bb * H + h) * T + t] = rd;
    }
    hsum += rd;   // rows past B*T read nothing: rd = 0
  }
  if (!dhm) return;
  if ((ci & 7) == 0) red[r * 128 + h] = hsum;
  __syncthreads();
  if ((int)threadIdx.x < H) {
    float t = red[threadIdx.x];
    for (int j = 1; j < rpb; ++j) t += red[j * 128 + threadIdx.x];
    // deterministic mode: slab [block][H], summed in block order after the launch
    if (part) part[(int64_t)blockIdx.x * H + threadIdx.x] = t;
    else atomicAdd(dhm + threadIdx.x, t);
  }
}

// ---------------------------------------------------------------------------
// backward dK, dV: block = (128 keys, h, b), wave w owns keys k0 = 128*bx + 32w + 16u + (0..15),
// u < NG.  Loops over query steps of 32 rows; Q' and dO' (= hm*dO_m) tiles staged in LDS.
// ---------------------------------------------------------------------------
template <bool DROP, bool BIAS, bool KEEP>
__device__ __forceinline__ void attn_bwd_dkv_body(const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ dom,
                                                  const float* __restrict__ head_mask, const float* __restrict__ lse,
                                                  const float* __restrict__ Dv, bf16_t* __restrict__ dqkv,
                                                  const int64_t* __restrict__ key_len, AttnShape sh, float scale,
                                                  float drop_p, uint64_t seed, RelBias rb,
                                                  const uint16_t* __restrict__ keep_in, float* __restrict__ bpart,
                                                  int bx, int64_t h, int64_t b) {
  seed = epoch_seed(seed);   // per-step RNG epoch (graph replays)
  const uint32_t mix = seed_mix(seed);
  constexpr int TB = QT_BWD * 128;   // 4096 B per tile
  // + stored keep words: [2 bufs][2 key tiles of this block][32 query rows] x 64 bit
  __shared__ __attribute__((aligned(16))) char smem[2 * (2 * TB) + 3 * 2 * QT_BWD * 4 + 2 * 2 * QT_BWD * 8];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int g = lane >> 4;
  const int64_t T = sh.T, H = sh.H, RS = sh.RS;
  const int64_t k0 = (int64_t)bx * RB + wave * 16 * NG;
  const bf16_t* rowbase = qkv + b * T * RS;
  const bf16_t* dobase = dom + b * T * (H * HD) + h * HD;
  const int64_t klen = key_len ? key_len[b] : T;
  const float hm = head_mask ? head_mask[h] : 1.0f;
  const float inv_keep = drop_p > 0.f ? 1.f / (1.f - drop_p) : 1.f;
  const uint32_t thr = drop_thr(drop_p);
  const uint64_t half_tp = (uint64_t)(T + 1) >> 1;
  const bool odd_key = (lane & 1) != 0;     // key parity (k0 is a multiple of 16)
  // A power-of-two softmax scale (64-wide heads: 1/8) is folded out of the staged Q tiles: S = Q K^T unscaled,
  // its scale applied in the exp2 argument (L2E * scale) or the bias fma, dK = scale * dS^T Q at the store.  Each
  // of these is exact (a power-of-two factor commutes with every rounding), so the results are bitwise those of
  // staging bf16(scale * Q) -- without the per-tile unpack / multiply / repack of every Q element.
  const bool fold = (__float_as_uint(scale) & 0x807fffffu) == 0u && scale != 0.f;
  const float s_mul = fold ? scale : 1.f;          // applied to S (exp2 argument / bias fma) and to dK
  const float q_scale = fold ? 1.f : scale;        // applied to the staged Q tile
  const float l2s = L2E * s_mul;
  // the head mask factors out: dP, D (dph_attention_bwd_prep) and dS are formed from dO_m itself and dK, dV are
  // multiplied by hm in fp32 at the store (no per-tile rounding of hm * dO_m to bf16)
  const float dk_mul = s_mul * hm;
  int64_t kme[NG];
  bool kpad[NG], kout[NG];   // key padded (masked -1e4) / past T
  const int T32 = (int)T;
  float kmask[NG];   // additive key mask in log2 units (-1e4 * log2 e on padded keys)
  bool anypad = false;
#pragma unroll
  for (int u = 0; u < NG; ++u) {
    kme[u] = k0 + 16 * u + (lane & 15);
    kpad[u] = kme[u] >= klen;
    kout[u] = kme[u] >= T;
    kmask[u] = kpad[u] ? -10000.0f * L2E : 0.f;
    anypad = anypad || kpad[u];
  }
  const bool wpad = __any(anypad);   // wave-uniform

  // K[key = lane&15][hd 32ks+8g+j], V[...]: B operands of S = Q' K^T and dP = dO V^T
  bf16x8_t kf[NG][2], vf[NG][2];
#pragma unroll
  for (int u = 0; u < NG; ++u)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      uint4 x = make_uint4(0, 0, 0, 0), c = make_uint4(0, 0, 0, 0);
      if (kme[u] < T) {
        x = *reinterpret_cast<const uint4*>(rowbase + kme[u] * RS + (H + h) * HD + ks * 32 + 8 * g);
        c = *reinterpret_cast<const uint4*>(rowbase + kme[u] * RS + (2 * H + h) * HD + ks * 32 + 8 * g);
      }
      kf[u][ks] = __builtin_bit_cast(bf16x8_t, x);
      vf[u][ks] = __builtin_bit_cast(bf16x8_t, c);
    }
  f32x4_t dk[NG][4], dv[NG][4];
#pragma unroll
  for (int u = 0; u < NG; ++u)
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      dk[u][d] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      dv[u][d] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    }
  auto ldsQ = [&](int buf) { return smem + buf * 2 * TB; };
  auto ldsO = [&](int buf) { return smem + buf * 2 * TB + TB; };
  float* lse_s = reinterpret_cast<float*>(smem + 4 * TB);        // [2][32]
  float* dv_s = reinterpret_cast<float*>(smem + 4 * TB + 2 * QT_BWD * 4);
  float* g_s = reinterpret_cast<float*>(smem + 4 * TB + 4 * QT_BWD * 4);   // [2][32] gates (BIAS)
  // keep words [2 bufs][2 key tiles][2 halves][32 query rows]: the 4 consecutive query rows a lane's MFMA layout
  // holds for one key are one 16-B read (a word per row and (row, half) pair as [2][32][2] cost one ds_read_b32 and
  // two address ops per score)
  uint32_t* kw_s = reinterpret_cast<uint32_t*>(smem + 4 * TB + 6 * QT_BWD * 4);
  const int nkt = (int)cdiv(T, KT);
  constexpr bool use_keep = DROP && KEEP;   // KEEP: read the forward's stored keep bits (else re-hash)
  // this lane's key inside its 64-key tile: word half and bit of the stored keep word (forward layout)
  int kt_loc[NG], kbit[NG], khalf[NG];
#pragma unroll
  for (int u = 0; u < NG; ++u) {
    const int key = (int)kme[u];
    kt_loc[u] = (key >> 6) - 2 * bx;
    const int bit = 16 * ((key >> 2) & 3) + 4 * ((key >> 4) & 3) + (key & 3);
    khalf[u] = bit >> 5;
    kbit[u] = bit & 31;
  }
  extern __shared__ float tw[];   // BIAS: [T + RB - 1] table window (diagonals of this block's keys)
  const int toff = bx * RB;
  if constexpr (BIAS) stage_tab_window(tw, rb.tab + h * (2 * T - 1), toff, (int)T);   // ordered by the first barrier

  const int nqt = (int)cdiv(T, QT_BWD);
  // the next query tile's rows AND its per-row words (lse, D, gate, keep bits) are loaded into registers at the
  // top of an iteration and written to LDS at its end: every global load is a whole iteration of MFMAs ahead of
  // the barrier that publishes it (the per-row words used to be loaded inside the store step, right before the
  // barrier, so the block waited one global-load latency per 32-query tile)
  uint4 rq[1], ro[1];
  float lse_r = 0.f, dv_r = 0.f, g_r = 0.f;
  uint2 kw_r = make_uint2(0u, 0u);
  auto load_tiles = [&](int qt) {
    stage_load<QT_BWD, true>(rq, rowbase + h * HD, (int64_t)qt * QT_BWD, T, RS, q_scale, tid);
    stage_load<QT_BWD, true>(ro, dobase, (int64_t)qt * QT_BWD, T, H * HD, 1.0f, tid);   // dO_m as is
    if (tid < QT_BWD) {
      const int64_t q = (int64_t)qt * QT_BWD + tid;
      lse_r = q < T ? -(lse[(b * H + h) * T + q] * L2E) : 0.f;   // -lse, log2 units
      dv_r = q < T ? Dv[(b * H + h) * T + q] : 0.f;
      if constexpr (BIAS) g_r = q < T ? rb.gate[(b * H + h) * T + q] : 0.f;
    }
    if (use_keep && tid >= 64 && tid < 128) {   // (constexpr-false unless KEEP)
      const int r = tid & 31, lt = (tid >> 5) & 1;
      const int64_t q = (int64_t)qt * QT_BWD + r;
      const int ktile = 2 * bx + lt;
      kw_r = make_uint2(0u, 0u);
      if (q < T && ktile < nkt)
        kw_r = *reinterpret_cast<const uint2*>(keep_in + ((b * H + h) * T + q) * (nkt * 4) + ktile * 4);
    }
  };
  auto store_tiles = [&](int buf, int qt) {
    (void)qt;
    stage_store<QT_BWD, true>(ldsQ(buf), rq, tid);
    stage_store<QT_BWD, true>(ldsO(buf), ro, tid);
    if (tid < QT_BWD) {
      lse_s[buf * QT_BWD + tid] = lse_r;
      dv_s[buf * QT_BWD + tid] = dv_r;
      if constexpr (BIAS) g_s[buf * QT_BWD + tid] = g_r;
    }
    if (use_keep && tid >= 64 && tid < 128) {
      const int r = tid & 31, lt = (tid >> 5) & 1;
      kw_s[((buf * 2 + lt) * 2 + 0) * QT_BWD + r] = kw_r.x;
      kw_s[((buf * 2 + lt) * 2 + 1) * QT_BWD + r] = kw_r.y;
    }
  };
  load_tiles(0);
  store_tiles(0, 0);
  __syncthreads();
  for (int qt = 0; qt < nqt; ++qt) {
    const int cur = qt & 1;
    const bool more = qt + 1 < nqt;
    if (more) load_tiles(qt + 1);
    const char* Q_ = ldsQ(cur);
    const char* O_ = ldsO(cur);
    // S[q = 16w + 4g + i][key = lane&15], dP likewise (w: query sub-step, u: key group)
    f32x4_t sacc[NG][2], pacc[NG][2];
#pragma unroll
    for (int w = 0; w < 2; ++w) {
#pragma unroll
      for (int u = 0; u < NG; ++u) {
        sacc[u][w] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        pacc[u][w] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8_t qa = lds_b128(Q_, swz128(16 * w + (lane & 15), ks * 32 + 8 * g));
        const bf16x8_t oa = lds_b128(O_, swz128(16 * w + (lane & 15), ks * 32 + 8 * g));
#pragma unroll
        for (int u = 0; u < NG; ++u) {
          sacc[u][w] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa, kf[u][ks], sacc[u][w], 0, 0, 0);
          pacc[u][w] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(oa, vf[u][ks], pacc[u][w], 0, 0, 0);
        }
      }
    }
    bf16x8_t pzf[NG], dsf[NG];
    // PAD: this wave holds padded keys (>= klen; the -1e4 key mask joins the exp2 argument's constant).  Without
    // them the constant is the staged -lse itself, no add per score.
    auto softmax_bwd = [&](auto pad_c) {
    constexpr bool PAD = decltype(pad_c)::value || BIAS;
#pragma unroll
    for (int u = 0; u < NG; ++u) {
      f32x4_t pz[2], ds[2];
#pragma unroll
      for (int w = 0; w < 2; ++w) {
        uint4 kwv = make_uint4(0u, 0u, 0u, 0u);
        if constexpr (use_keep)
          kwv = *reinterpret_cast<const uint4*>(kw_s + ((cur * 2 + kt_loc[u]) * 2 + khalf[u]) * QT_BWD + 16 * w + 4 * g);
        uint32_t hb[4] = {0u, 0u, 0u, 0u};
        if constexpr (DROP) {
          if constexpr (!use_keep) {
            // this lane hashes queries ia, ia+1 of its key pair; the neighbour (key ^ 1) the other two
            const int ia = odd_key ? 2 : 0;
            const uint64_t qa = (uint64_t)(b * H + h) * T + (uint64_t)(qt * QT_BWD + 16 * w + 4 * g + ia);
            const uint32_t h0 = attn_hash32(mix, (uint32_t)(qa * half_tp + (uint64_t)(kme[u] >> 1)));
            const uint32_t h1 = attn_hash32(mix, (uint32_t)((qa + 1) * half_tp + (uint64_t)(kme[u] >> 1)));
            const uint32_t o0 = (uint32_t)__shfl_xor((int)h0, 1, 64);
            const uint32_t o1 = (uint32_t)__shfl_xor((int)h1, 1, 64);
            hb[0] = odd_key ? o0 : h0;
            hb[1] = odd_key ? o1 : h1;
            hb[2] = odd_key ? h0 : o0;
            hb[3] = odd_key ? h1 : o1;
          }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int ql = 16 * w + 4 * g + i;
          float sv = sacc[u][w][i];   // unscaled when fold
          float p;
          // padded keys (>= klen) get the -1e4 of the key mask; keys past T and queries past T have zero K / V / Q /
          // dO / D rows, so their p never reaches a stored dK / dV row or a nonzero product
          const float nl = lse_s[cur * QT_BWD + ql];   // -lse (log2 units)
          const float c = PAD ? kmask[u] + nl : nl;
          if constexpr (BIAS) {
            sv = fmaf(sv, s_mul, g_s[cur * QT_BWD + ql] * tw[rel_idx((int)kme[u], qt * QT_BWD + ql, T32) - toff]);
            p = __builtin_amdgcn_exp2f(fmaf(sv, L2E, c));
          } else {
            p = __builtin_amdgcn_exp2f(fmaf(sv, l2s, c));
          }
          float z = 1.f;
          if constexpr (DROP) {
            if constexpr (use_keep) {
              // the keep bit sign-extended to an all-ones / zero mask over inv_keep's bits: z in {inv_keep, 0}
              const uint32_t wd = (&kwv.x)[i];
              z = keep_scale(wd, kbit[u], inv_keep);
            } else {
              z = attn_keep(hb[i], odd_key, thr, 1.f) != 0.f ? inv_keep : 0.f;
            }
          }
          pz[w][i] = p * z;
          ds[w][i] = p * (pacc[u][w][i] * z - dv_s[cur * QT_BWD + ql]);
        }
      }
      pzf[u] = pack_frag(pz[0], pz[1]);
      dsf[u] = pack_frag(ds[0], ds[1]);
    }
    };
    if (BIAS || wpad) softmax_bwd(std::integral_constant<bool, true>());
    else softmax_bwd(std::integral_constant<bool, false>());
    // dV[key][d] += sum_q PZ[q][key] dO'[q][d] ; dK[key][d] += sum_q dS[q][key] Q'[q][d]
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const bf16x8_t of = tr_frag(O_, 4 * g, 16 + 4 * g, 16 * d, lane);
      const bf16x8_t qf = tr_frag(Q_, 4 * g, 16 + 4 * g, 16 * d, lane);
#pragma unroll
      for (int u = 0; u < NG; ++u) {
        dv[u][d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pzf[u], of, dv[u][d], 0, 0, 0);
        dk[u][d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(dsf[u], qf, dk[u][d], 0, 0, 0);
      }
    }
    if (more) store_tiles(cur ^ 1, qt + 1);
    __syncthreads();
  }
  if (bpart != nullptr) {
    // v_proj bias gradient (the column sums of dV, components.py:365 v_proj): this wave's partial over its keys
    // < T, in a fixed order (keys in-lane, then the four lane groups g), into its row of the [waves][2 * H * 64]
    // slab (q half | v half) that the host reduces over the rows -- no second pass over dqkv
    float cs[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      cs[d] = 0.f;
#pragma unroll
      for (int u = 0; u < NG; ++u)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (k0 + 16 * u + 4 * g + i < T) cs[d] += dv[u][d][i];
      cs[d] += __shfl_xor(cs[d], 16, 64);
      cs[d] += __shfl_xor(cs[d], 32, 64);
    }
    // the four waves' partials meet in LDS (the per-row word area: every wave left the loop's last barrier) and
    // wave 0 adds them in wave order after the barrier below: one slab row per block
    float* bred = reinterpret_cast<float*>(smem + 4 * TB);
    if (g == 0) {
#pragma unroll
      for (int d = 0; d < 4; ++d) bred[wave * HD + 16 * d + (lane & 15)] = cs[d];
    }
  }
  // lane holds dK[key = k0 + 16u + 4g + i][d = 16dd + (lane&15)]: stage the wave's [32 keys][64] bf16
  // tile in LDS and store whole 128-B key rows with 16-B stores (4 per lane per tensor instead of 32
  // scattered 2-byte stores)
  __syncthreads();   // every wave is done with the Q / dO tiles
  if (bpart != nullptr && wave == 0) {
    const float* bred = reinterpret_cast<const float*>(smem + 4 * TB);
    const float t = ((bred[lane] + bred[HD + lane]) + bred[2 * HD + lane]) + bred[3 * HD + lane];
    bpart[((int64_t)b * gridDim.x + bx) * (2 * H * HD) + (H + h) * HD + lane] = t * hm;
  }
  uint16_t* st = reinterpret_cast<uint16_t*>(smem) + wave * (16 * NG * HD);
#pragma unroll
  for (int tsel = 0; tsel < 2; ++tsel) {
#pragma unroll
    for (int u = 0; u < NG; ++u)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int d = 0; d < 4; ++d)
          st[(16 * u + 4 * g + i) * HD + 16 * d + (lane & 15)] = f2bf(tsel == 0 ? dk[u][d][i] * dk_mul : dv[u][d][i] * hm);
    __syncthreads();
#pragma unroll
    for (int ps = 0; ps < 16 * NG / 8; ++ps) {
      const int r = (lane >> 3) + 8 * ps;
      const int64_t key = k0 + r;
      const uint4 v = *reinterpret_cast<const uint4*>(st + r * HD + (lane & 7) * 8);
      if (key < T)
        *reinterpret_cast<uint4*>(dqkv + (b * T + key) * RS + ((tsel + 1) * H + h) * HD + (lane & 7) * 8) = v;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// backward dQ: block = (128 query rows, h, b), 4 waves x 2 x 16 rows; loops over key tiles.
// ---------------------------------------------------------------------------
template <bool DROP, bool BIAS, bool KEEP>
__device__ __forceinline__ void attn_bwd_dq_body(const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ dom,
                                                 const float* __restrict__ head_mask, const float* __restrict__ lse,
                                                 const float* __restrict__ Dv, bf16_t* __restrict__ dqkv,
                                                 const int64_t* __restrict__ key_len, AttnShape sh, float scale,
                                                 float drop_p, uint64_t seed, RelBias rb,
                                                 const uint16_t* __restrict__ keep_in, float* __restrict__ bpart,
                                                 int bx, int64_t h, int64_t b) {
  extern __shared__ float dyn[];   // BIAS: hist [T + RB - 1] (diagonal sums of dS * gate) | table window [T + RB - 1]
  seed = epoch_seed(seed);   // per-step RNG epoch (graph replays)
  const uint32_t mix = seed_mix(seed);
  // K and V tiles both in the swz128 image: the 16-B row reads of a ds_read_b128 lane group (rows 0-3 / 12-15 of
  // one k-chunk + rows 4-11 of the next) hit 16 distinct 16-B bank groups; the padded [64][72] V image put them
  // 2-way on 8 of them (SQ_LDS_BANK_CONFLICT 26-32 % of the backward's LDS cycles)
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * TILE_SWZ_BYTES];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int g = lane >> 4;
  const int64_t T = sh.T, H = sh.H, RS = sh.RS;
  const int64_t q0 = (int64_t)bx * RB + wave * 16 * NG;
  const bf16_t* rowbase = qkv + b * T * RS;
  const int64_t klen = key_len ? key_len[b] : T;
  const float hm = head_mask ? head_mask[h] : 1.0f;
  const float dq_mul = scale * hm;   // dQ = scale * hm * dS_m K (dS_m from dO_m)
  const float inv_keep = drop_p > 0.f ? 1.f / (1.f - drop_p) : 1.f;
  int64_t qme[NG];
  uint64_t hrow[NG];
  bool qout[NG];
  bf16x8_t qf[NG][2], of[NG][2];
  float my_lse[NG], my_D[NG];
  f32x4_t dq[NG][4];
  const int T32 = (int)T, klen32 = (int)klen;
  const uint64_t half_tp0 = (uint64_t)(T + 1) >> 1;
#pragma unroll
  for (int u = 0; u < NG; ++u) {
    qme[u] = q0 + 16 * u + (lane & 15);
    qout[u] = qme[u] >= T;
    hrow[u] = ((uint64_t)(b * H + h) * T + (uint64_t)qme[u]) * half_tp0;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      uint4 x = make_uint4(0, 0, 0, 0), c = make_uint4(0, 0, 0, 0);
      if (qme[u] < T) {
        x = *reinterpret_cast<const uint4*>(rowbase + qme[u] * RS + h * HD + ks * 32 + 8 * g);
        c = *reinterpret_cast<const uint4*>(dom + (b * T + qme[u]) * (H * HD) + h * HD + ks * 32 + 8 * g);
      }
      qf[u][ks] = __builtin_bit_cast(bf16x8_t, scale_bf16x8(x, scale));
      of[u][ks] = __builtin_bit_cast(bf16x8_t, c);   // dO_m: hm is applied to dQ (and the bias gradients) at the end
    }
    my_lse[u] = qme[u] < T ? lse[(b * H + h) * T + qme[u]] * L2E : 0.f;   // log2 units: p = 2^(s log2e - lse')
    my_D[u] = qme[u] < T ? Dv[(b * H + h) * T + qme[u]] : 0.f;
#pragma unroll
    for (int d = 0; d < 4; ++d) dq[u][d] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  }
  // deterministic mode: one histogram per wave (a wave's LDS adds run in program order, its lanes' addresses in
  // one add are distinct), summed in wave order at the end
  const int HW = T32 + RB - 1;
  const bool det_h = BIAS && rb.dtab_part != nullptr;
  float* hist = dyn + (det_h ? wave * HW : 0);
  float* tw = dyn + (det_h ? 4 : 1) * HW;
  const int qb0 = bx * RB;
  const int toff = T32 - 1 - (qb0 + RB - 1);
  float gq[NG], dg[NG];
#pragma unroll
  for (int u = 0; u < NG; ++u) {
    gq[u] = (BIAS && qme[u] < T) ? rb.gate[(b * H + h) * T + qme[u]] : 0.f;
    dg[u] = 0.f;
  }
  if constexpr (BIAS) {
    for (int i = tid; i < (det_h ? 4 : 1) * HW; i += 256) dyn[i] = 0.f;   // ordered before use by the first barrier
    stage_tab_window(tw, rb.tab + h * (2 * T - 1), toff, T32);
  }

  auto ldsK = [&](int buf) { return smem + buf * 2 * TILE_SWZ_BYTES; };
  auto ldsV = [&](int buf) { return smem + buf * 2 * TILE_SWZ_BYTES + TILE_SWZ_BYTES; };
  const int nkt = (int)cdiv(T, KT);
  uint4 rk[2], rv[2];
  stage_load<KT, true>(rk, rowbase + (H + h) * HD, 0, T, RS, 1.0f, tid);
  stage_load<KT, true>(rv, rowbase + (2 * H + h) * HD, 0, T, RS, 1.0f, tid);
  stage_store<KT, true>(ldsK(0), rk, tid);
  stage_store<KT, true>(ldsV(0), rv, tid);
  __syncthreads();
  const uint32_t thr = drop_thr(drop_p);
  const uint64_t half_tp = (uint64_t)(T + 1) >> 1;
  uint32_t kw_next[NG];
#pragma unroll
  for (int u = 0; u < NG; ++u)
    kw_next[u] = (DROP && KEEP && !qout[u]) ? keep_in[((b * H + h) * T + qme[u]) * (nkt * 4) + g] : 0u;
  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nkt;
    if (more) {
      stage_load<KT, true>(rk, rowbase + (H + h) * HD, (int64_t)(kt + 1) * KT, T, RS, 1.0f, tid);
      stage_load<KT, true>(rv, rowbase + (2 * H + h) * HD, (int64_t)(kt + 1) * KT, T, RS, 1.0f, tid);
    }
    const char* K_ = ldsK(cur);
    const char* V_ = ldsV(cur);
    f32x4_t ds[NG][4];
    // stored keep bits of this key tile (16 per lane and row; loaded one tile ahead), or the in-kernel hash
    uint32_t kw[NG];
#pragma unroll
    for (int u = 0; u < NG; ++u) {
      kw[u] = kw_next[u];
      if (DROP && KEEP && more && !qout[u])
        kw_next[u] = keep_in[((b * H + h) * T + qme[u]) * (nkt * 4) + (kt + 1) * 4 + g];
    }
    // MASKED: the tile holds padded (>= klen) or missing (>= T) keys.  Elsewhere no per-element compare: rows
    // past T have zero dO and D, so their dS is exactly 0 whatever p is.
    auto tile = [&](auto masked_c) {
      constexpr bool MASKED = decltype(masked_c)::value;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        f32x4_t sa[NG], pa[NG];
#pragma unroll
        for (int u = 0; u < NG; ++u) {
          sa[u] = f32x4_t{0.f, 0.f, 0.f, 0.f};
          pa[u] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const bf16x8_t ka = lds_b128(K_, swz128(16 * s + (lane & 15), ks * 32 + 8 * g));
          const bf16x8_t va = lds_b128(V_, swz128(16 * s + (lane & 15), ks * 32 + 8 * g));
#pragma unroll
          for (int u = 0; u < NG; ++u) {
            sa[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka, qf[u][ks], sa[u], 0, 0, 0);
            pa[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va, of[u][ks], pa[u], 0, 0, 0);
          }
        }
        const int kb = kt * KT + 16 * s + 4 * g;
#pragma unroll
        for (int u = 0; u < NG; ++u) {
          uint32_t hb[2] = {0u, 0u};
          if constexpr (DROP && !KEEP) {
            const uint32_t pr = (uint32_t)(hrow[u] + (uint64_t)(kb >> 1));
            hb[0] = attn_hash32(mix, pr);
            hb[1] = attn_hash32(mix, pr + 1);
          }
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int key = kb + i;
            float sv = sa[u][i];
            float tv = 0.f;
            if constexpr (BIAS) {
              tv = tw[rel_idx(key, (int)qme[u], T32) - toff];
              sv += gq[u] * tv;
            }
            if constexpr (MASKED) sv = key >= klen32 ? sv - 10000.0f : sv;
            float p = __builtin_amdgcn_exp2f(fmaf(sv, L2E, -my_lse[u]));
            if constexpr (MASKED) p = (key >= T32 || qout[u]) ? 0.f : p;
            float z = 1.f;
            if constexpr (DROP) {
              if constexpr (KEEP) z = BIAS ? keep_scale_x(kw[u], 4 * s + i, inv_keep) : keep_scale_u(kw[u], 4 * s + i, inv_keep);
              else z = attn_keep(hb[i >> 1], i & 1, thr, 1.f) != 0.f ? inv_keep : 0.f;
            }
            const float dsv = p * (pa[u][i] * z - my_D[u]);
            ds[u][s][i] = dsv;
            if constexpr (BIAS) dg[u] += dsv * tv;
          }
        }
      }
    };
    if (!BIAS && (kt + 1) * KT <= klen32 && (kt + 1) * KT <= T32) tile(std::integral_constant<bool, BIAS>());
    else tile(std::integral_constant<bool, true>());
    if constexpr (BIAS) {
      // diagonal sums of dS * gate: element (u, s, i) sits on diagonal kt*64 + 16(s-u) + 4g + i - (q - qb0 - ...)
      // of this block's histogram, so the query groups u meeting on the same s-u are added first (NG + 3
      // diagonals x 4 instead of NG x 4 x 4 LDS atomics); masked elements are exactly 0 and skipped
      const int l = lane & 15;
      const int base = kt * KT + 4 * g - wave * 16 * NG - l + RB - 1;
#pragma unroll
      for (int dd = -(NG - 1); dd < 4; ++dd) {
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          v[i] = 0.f;
#pragma unroll
          for (int u = 0; u < NG; ++u) {
            const int s = dd + u;
            if (s >= 0 && s < 4) v[i] += ds[u][s][i] * gq[u];
          }
        }
        // element (l, i) and (l + 1, i + 1) share a diagonal: fold each chain (l, 0), (l+1, 1), (l+2, 2),
        // (l+3, 3) into its first cell -- heads are then (l, 0) for every lane plus (0, i > 0)
        const float a1 = __shfl_down(v[1], 1, 64), a2 = __shfl_down(v[2], 1, 64), a3 = __shfl_down(v[3], 1, 64);
        if (l <= 14) {
          v[0] += a1;
          v[1] += a2;
          v[2] += a3;
        }
        const float b2 = __shfl_down(v[2], 2, 64), b3 = __shfl_down(v[3], 2, 64);
        if (l <= 13) {
          v[0] += b2;
          v[1] += b3;
        }
        // the (l = 0, i > 0) heads ride on lanes l = 1..3 of the same g in a second atomic
        const float e1 = __shfl(v[1], lane & 48, 64), e2 = __shfl(v[2], lane & 48, 64), e3 = __shfl(v[3], lane & 48, 64);
        const float ex = l == 1 ? e1 : (l == 2 ? e2 : e3);
        // lanes (g, l), (g+1, l+4), (g+2, l+8), (g+3, l+12) share the i = 0 diagonal: fold along g as well
        float w = v[0];
        const float w1 = __shfl(w, (lane + 20) & 63, 64);
        w += (g <= 2 && l <= 11) ? w1 : 0.f;
        const float w2 = __shfl(w, (lane + 40) & 63, 64);
        w += (g <= 1 && l <= 7) ? w2 : 0.f;
        const int idx = base + 16 * dd;
        if ((g == 0 || l < 4) && w != 0.f && idx >= 0 && idx < T32 + RB - 1) atomicAdd(&hist[idx], w);
        const int idx2 = base + 2 * l + 16 * dd;   // diagonal of head (g, 0, i = l)
        if (l >= 1 && l <= 3 && ex != 0.f && idx2 >= 0 && idx2 < T32 + RB - 1) atomicAdd(&hist[idx2], ex);
      }
    }
    // dQ'^T[d][q] += K^T[d][key] dS^T[key][q]
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8_t dsf[NG];
#pragma unroll
      for (int u = 0; u < NG; ++u) dsf[u] = pack_frag(ds[u][2 * kk], ds[u][2 * kk + 1]);
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const bf16x8_t kt_f = tr_frag(K_, 32 * kk + 4 * g, 32 * kk + 16 + 4 * g, 16 * d, lane);
#pragma unroll
        for (int u = 0; u < NG; ++u) dq[u][d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kt_f, dsf[u], dq[u][d], 0, 0, 0);
      }
    }
    if (more) {
      stage_store<KT, true>(ldsK(cur ^ 1), rk, tid);
      stage_store<KT, true>(ldsV(cur ^ 1), rv, tid);
    }
    __syncthreads();
  }
  if constexpr (BIAS) {
#pragma unroll
    for (int u = 0; u < NG; ++u) {
      float v = dg[u];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (g == 0 && qme[u] < T) rb.dgate[(b * H + h) * T + qme[u]] = v * hm;
    }
    __syncthreads();   // all histogram adds of the block are done
    if (det_h) {
      float* prow = rb.dtab_part + (((int64_t)b * H + h) * cdiv(T, (int64_t)RB) + bx) * HW;
      for (int i = tid; i < HW; i += 256) prow[i] = (((dyn[i] + dyn[HW + i]) + dyn[2 * HW + i]) + dyn[3 * HW + i]) * hm;
    } else {
      float* dt = rb.dtab + h * (2 * T - 1);
      const int off = T32 - 1 - (qb0 + RB - 1);   // global diagonal index of hist[0]
      for (int i = tid; i < T32 + RB - 1; i += 256) {
        const int gi = i + off;
        const float v = hist[i];
        if (gi >= 0 && gi < 2 * T32 - 1 && v != 0.f) atomicAdd(dt + gi, v * hm);
      }
    }
  }
  if (bpart != nullptr) {
    // q_proj bias gradient (the column sums of dQ): lane holds dQ[q0 + 16u + (lane&15)][16d + 4g + j]; summed over
    // u in-lane, then over the 16 row lanes, in a fixed order (rows past T hold exactly 0 and are skipped anyway)
    f32x4_t cs[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      cs[d] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < NG; ++u)
        if (qme[u] < T) cs[d] += dq[u][d];
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int m = 1; m < 16; m <<= 1) cs[d][j] += __shfl_xor(cs[d][j], m, 64);
    }
    // the four waves' partials meet in LDS (the K / V tile area, free after the loop's last barrier); wave 0 adds
    // them in wave order: one slab row per block
    float* bred = reinterpret_cast<float*>(smem);
    if ((lane & 15) == 0) {
#pragma unroll
      for (int d = 0; d < 4; ++d) *reinterpret_cast<f32x4_t*>(bred + wave * HD + 16 * d + 4 * g) = cs[d];
    }
    __syncthreads();
    if (wave == 0) {
      const float t = ((bred[lane] + bred[HD + lane]) + bred[2 * HD + lane]) + bred[3 * HD + lane];
      bpart[((int64_t)b * gridDim.x + bx) * (2 * H * HD) + h * HD + lane] = t * dq_mul;
    }
  }
#pragma unroll
  for (int u = 0; u < NG; ++u) {
    if (qme[u] >= T) continue;
    bf16_t* rowp = dqkv + (b * T + qme[u]) * RS + h * HD;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const int col = 16 * d + 4 * g;
      *reinterpret_cast<uint2*>(rowp + col) = make_uint2(pack2bf(dq[u][d][0] * dq_mul, dq[u][d][1] * dq_mul),
                                                         pack2bf(dq[u][d][2] * dq_mul, dq[u][d][3] * dq_mul));
    }
  }
}


// ---------------------------------------------------------------------------
// backward launch: the dK/dV blocks (z < nbz) and the dQ blocks (z >= nbz) of one layer in ONE grid.  Each
// kernel alone is 768 blocks at the distill shape (B=16, H=12, T=499) against 512 resident slots (2 per CU),
// so each ran 1.5 rounds with the last one half empty; in one grid the dQ blocks (about half the work of a
// dK/dV block) fill the CUs the dK/dV blocks free, longest first (dispatch follows z).
// mode 1 / 2: dK/dV only / dQ only (A/B timing, DPH_ATTN_SPLIT=1).
// ---------------------------------------------------------------------------
template <bool DROP, bool BIAS, bool KEEP>
__global__ void __launch_bounds__(256, 2) attn_bwd_kernel(const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ dom,
                                                       const float* __restrict__ head_mask,
                                                       const float* __restrict__ lse, const float* __restrict__ Dv,
                                                       bf16_t* __restrict__ dqkv, const int64_t* __restrict__ key_len,
                                                       AttnShape sh, float scale, float drop_p, uint64_t seed,
                                                       RelBias rb, const uint16_t* __restrict__ keep_in,
                                                       float* __restrict__ bpart, int nbz, int mode) {
  const int z = (int)blockIdx.z;
  const bool kv = mode == 1 || (mode == 0 && z < nbz);
  if constexpr (!BIAS) {
    // head with an exactly-zero mask (skipped by the forward): its q / k / v gradients are 0
    const int64_t h = blockIdx.y;
    if (head_mask != nullptr && head_mask[h] == 0.f) {
      const int64_t T = sh.T, H = sh.H, RS = sh.RS;
      const int64_t b = kv ? z : (mode == 0 ? z - nbz : z);
      const int64_t r0 = (int64_t)blockIdx.x * RB;
      for (int c = threadIdx.x; c < RB * 8 * (kv ? 2 : 1); c += 256) {
        const int64_t r = r0 + (c >> 3) % RB;
        const int sel = kv ? 1 + (c >> 3) / RB : 0;
        if (r < T)
          *reinterpret_cast<uint4*>(dqkv + (b * T + r) * RS + (sel * H + h) * HD + (c & 7) * 8) = make_uint4(0, 0, 0, 0);
      }
      if (bpart != nullptr && threadIdx.x < HD)   // this head's q (dQ blocks) / v (dK/dV blocks) bias partial row
        bpart[((int64_t)b * gridDim.x + blockIdx.x) * (2 * H * HD) + ((kv ? H : 0) + h) * HD + threadIdx.x] = 0.f;
      return;
    }
  }
  if (kv)
    attn_bwd_dkv_body<DROP, BIAS, KEEP>(qkv, dom, head_mask, lse, Dv, dqkv, key_len, sh, scale, drop_p, seed, rb,
                                        keep_in, bpart, (int)blockIdx.x, blockIdx.y, z);
  else
    attn_bwd_dq_body<DROP, BIAS, KEEP>(qkv, dom, head_mask, lse, Dv, dqkv, key_len, sh, scale, drop_p, seed, rb,
                                       keep_in, bpart, (int)blockIdx.x, blockIdx.y, mode == 0 ? z - nbz : z);
}

// deterministic mode: dtab[h][gi] += the dQ blocks' diagonal sums (relpos dtab_part slab) over (b, query block) in
// order; one thread per (h, diagonal)
__global__ void __launch_bounds__(256) relpos_dtab_reduce(const float* __restrict__ part, int64_t B, int64_t H,
                                                          int64_t T, float* __restrict__ dtab) {
  const int64_t R = 2 * T - 1, HW = T + RB - 1, nqb = cdiv(T, (int64_t)RB);
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= H * R) return;
  const int64_t h = i / R, gi = i % R;
  float s = 0.f;
  for (int64_t b = 0; b < B; ++b)
    for (int64_t bx = 0; bx < nqb; ++bx) {
      const int64_t j = gi - (T - 1 - (bx * RB + RB - 1));
      if (j >= 0 && j < HW) s += part[((b * H + h) * nqb + bx) * HW + j];
    }
  dtab[i] += s;
}

}  // namespace
}  // namespace dph

using namespace dph;

namespace {

// DPH_ATTN_FWD=2: the 16 x 16 x 32 forward for every shape (A/B; the WavLM bias always takes it); =1: the first
// 32 x 32 forward (attn_fwd32_kernel, A/B against the restructured attn_fwd32v2_kernel, the default).  Measured
// and dropped: the 32 x 32 x 16 forward at three waves per SIMD (K / V by LDS-DMA, Q' staged in LDS, 168
// VGPRs with 14-20 spilled) ran 46 / 58 us against 38 / 51 us at two waves per SIMD.
static int fwd32_mode() {
  const char* e = getenv("DPH_ATTN_FWD");
  return (e && e[0] == '2') ? 0 : ((e && e[0] == '1') ? 1 : 2);
}

template <bool DROP, bool BIAS>
void launch_fwd(dim3 grid, hipStream_t stream, const void* qkv, void* o_u, void* o_m, float* lse, const float* hm,
                const int64_t* key_len, AttnShape sh, float scale, float p, uint64_t seed, RelBias rb, void* keep) {
  const int mode = BIAS ? 0 : fwd32_mode();
  static const bool prec_env = [] {
    const char* e = getenv("DPH_ATTN_PREC");
    return !(e && e[0] == '0');
  }();
  const bool prec = prec_env && o_u != nullptr;
  if (mode == 2) {
    // DPH_ATTN_EPI=0: the per-lane scattered epilogue stores (A/B).  PREC (a forward whose O_u feeds a backward,
    // unless DPH_ATTN_PREC=0): O accumulates P as bf16(P) + bf16(P - bf16(P)), so D = dO . O_u equals
    // sum_j P_j dP_j to ~2^-17 and dS = P (dP - D) keeps its row sums near zero on saturated rows
    static const bool staged = [] {
      const char* e = getenv("DPH_ATTN_EPI");
      return !(e && e[0] == '0');
    }();
    auto go = [&](auto kern) {
      hipLaunchKernelGGL(kern, grid, dim3(256), 0, stream, reinterpret_cast<const bf16_t*>(qkv),
                         reinterpret_cast<float*>(o_u), reinterpret_cast<bf16_t*>(o_m), lse, hm, key_len, sh, scale,
                         p, seed, reinterpret_cast<uint16_t*>(keep));
    };
    if (staged) {
      if (prec) go(attn_fwd32v2_kernel<DROP, true, true>);
      else go(attn_fwd32v2_kernel<DROP, true, false>);
    } else {
      if (prec) go(attn_fwd32v2_kernel<DROP, false, true>);
      else go(attn_fwd32v2_kernel<DROP, false, false>);
    }
    return;
  }
  if (mode == 1) {
    hipLaunchKernelGGL((attn_fwd32_kernel<DROP>), grid, dim3(256), 0, stream, reinterpret_cast<const bf16_t*>(qkv),
                       reinterpret_cast<float*>(o_u), reinterpret_cast<bf16_t*>(o_m), lse, hm, key_len, sh, scale, p,
                       seed, reinterpret_cast<uint16_t*>(keep));
    return;
  }
  const size_t tw_bytes = BIAS ? (size_t)(sh.T + RB - 1) * sizeof(float) : 0;
  auto go16 = [&](auto kern) {
    hipLaunchKernelGGL(kern, grid, dim3(256), tw_bytes, stream, reinterpret_cast<const bf16_t*>(qkv),
                       reinterpret_cast<float*>(o_u), reinterpret_cast<bf16_t*>(o_m), lse, hm, key_len, sh, scale, p,
                       seed, rb, reinterpret_cast<uint16_t*>(keep));
  };
  if (prec) go16(attn_fwd_kernel<DROP, BIAS, true>);
  else go16(attn_fwd_kernel<DROP, BIAS, false>);
}

template <bool DROP, bool BIAS, bool KEEP>
void launch_bwd_k(dim3 grid, hipStream_t stream, const void* qkv, const void* dom, const float* hm, const float* lse,
                  const float* Dvec, void* dqkv, const int64_t* key_len, AttnShape sh, float scale, float p,
                  uint64_t seed, RelBias rb, const void* keep, float* bpart) {
  const size_t tw_bytes = BIAS ? (size_t)(sh.T + RB - 1) * sizeof(float) : 0;
  // dynamic LDS: the table window + one diagonal histogram (four, per wave, in deterministic mode)
  const size_t dyn_bytes = (rb.dtab_part != nullptr ? 5 : 2) * tw_bytes;
  const char* e = getenv("DPH_ATTN_SPLIT");
  const int nbz = (int)grid.z;
  if (e && e[0] == '1') {
    for (int mode = 1; mode <= 2; ++mode)
      hipLaunchKernelGGL((attn_bwd_kernel<DROP, BIAS, KEEP>), grid, dim3(256), dyn_bytes, stream,
                         reinterpret_cast<const bf16_t*>(qkv), reinterpret_cast<const bf16_t*>(dom), hm, lse, Dvec,
                         reinterpret_cast<bf16_t*>(dqkv), key_len, sh, scale, p, seed, rb,
                         reinterpret_cast<const uint16_t*>(keep), bpart, nbz, mode);
    return;
  }
  const dim3 g2(grid.x, grid.y, 2 * grid.z);
  hipLaunchKernelGGL((attn_bwd_kernel<DROP, BIAS, KEEP>), g2, dim3(256), dyn_bytes, stream,
                     reinterpret_cast<const bf16_t*>(qkv), reinterpret_cast<const bf16_t*>(dom), hm, lse, Dvec,
                     reinterpret_cast<bf16_t*>(dqkv), key_len, sh, scale, p, seed, rb,
                     reinterpret_cast<const uint16_t*>(keep), bpart, nbz, 0);
}

template <bool DROP, bool BIAS>
void launch_bwd(dim3 grid, hipStream_t stream, const void* qkv, const void* dom, const float* hm, const float* lse,
                const float* Dvec, void* dqkv, const int64_t* key_len, AttnShape sh, float scale, float p,
                uint64_t seed, RelBias rb, const void* keep, float* bpart) {
  if (DROP && keep != nullptr)
    launch_bwd_k<DROP, BIAS, true>(grid, stream, qkv, dom, hm, lse, Dvec, dqkv, key_len, sh, scale, p, seed, rb, keep,
                                   bpart);
  else
    launch_bwd_k<DROP, BIAS, false>(grid, stream, qkv, dom, hm, lse, Dvec, dqkv, key_len, sh, scale, p, seed, rb, keep,
                                    bpart);
}

}  // namespace

// dropout pair indices (row * ceil(T/2) + key/2) must fit 32 bits (the kernels' hoisted seed mix)
static bool pairs_fit(int64_t B, int64_t T, int64_t H) { return B * H * T * ((T + 1) / 2) < ((int64_t)1 << 32); }

extern "C" int64_t dph_attention_keep_bytes(int64_t B, int64_t T, int64_t H) { return B * H * T * cdiv(T, KT) * 8; }

static int attention_fwd(const void* qkv, void* o_unmasked, void* o_masked, float* lse, const float* head_mask,
                         const int64_t* key_len, int64_t B, int64_t T, int64_t H, float scale, float dropout_p,
                         uint64_t seed, RelBias rb, void* keep, hipStream_t stream) {
  AttnShape sh{B, T, H, 3 * H * HD};
  dim3 grid((unsigned)cdiv(T, RB), (unsigned)H, (unsigned)B);
  const bool bias = rb.tab != nullptr;
  DPH_REQUIRE(dropout_p <= 0.f || pairs_fit(B, T, H), "dph_attention_fwd: B*H*T*ceil(T/2) >= 2^32 dropout pairs");
  DPH_REQUIRE(keep == nullptr || (reinterpret_cast<uintptr_t>(keep) & 7) == 0, "dph_attention_fwd: keep bits not 8-B aligned");
  if (dropout_p > 0.f) {
    if (bias) launch_fwd<true, true>(grid, stream, qkv, o_unmasked, o_masked, lse, head_mask, key_len, sh, scale, dropout_p, seed, rb, keep);
    else launch_fwd<true, false>(grid, stream, qkv, o_unmasked, o_masked, lse, head_mask, key_len, sh, scale, dropout_p, seed, rb, keep);
  } else {
    if (bias) launch_fwd<false, true>(grid, stream, qkv, o_unmasked, o_masked, lse, head_mask, key_len, sh, scale, dropout_p, seed, rb, nullptr);
    else launch_fwd<false, false>(grid, stream, qkv, o_unmasked, o_masked, lse, head_mask, key_len, sh, scale, dropout_p, seed, rb, nullptr);
  }
  return check_launch("dph_attention_fwd");
}

static int attention_bwd(const void* qkv, const void* do_masked, const float* head_mask, const float* lse,
                         const float* Dvec, void* dqkv, const int64_t* key_len, int64_t B, int64_t T, int64_t H,
                         float scale, float dropout_p, uint64_t seed, RelBias rb, const void* keep, hipStream_t stream,
                         float* dbq = nullptr, float* dbv = nullptr, float* bws = nullptr) {
  AttnShape sh{B, T, H, 3 * H * HD};
  dim3 grid((unsigned)cdiv(T, RB), (unsigned)H, (unsigned)B);
  const bool bias = rb.tab != nullptr;
  float* bpart = dbq != nullptr ? bws : nullptr;
  DPH_REQUIRE(dropout_p <= 0.f || pairs_fit(B, T, H), "dph_attention_bwd: B*H*T*ceil(T/2) >= 2^32 dropout pairs");
  DPH_REQUIRE(keep == nullptr || (reinterpret_cast<uintptr_t>(keep) & 7) == 0, "dph_attention_bwd: keep bits not 8-B aligned");
  DPH_REQUIRE(2 * B < 65536 && H < 65536, "dph_attention_bwd: grid too large (B=%lld H=%lld)", (long long)B, (long long)H);
  if (dropout_p > 0.f) {
    if (bias) launch_bwd<true, true>(grid, stream, qkv, do_masked, head_mask, lse, Dvec, dqkv, key_len, sh, scale, dropout_p, seed, rb, keep, bpart);
    else launch_bwd<true, false>(grid, stream, qkv, do_masked, head_mask, lse, Dvec, dqkv, key_len, sh, scale, dropout_p, seed, rb, keep, bpart);
  } else {
    if (bias) launch_bwd<false, true>(grid, stream, qkv, do_masked, head_mask, lse, Dvec, dqkv, key_len, sh, scale, dropout_p, seed, rb, nullptr, bpart);
    else launch_bwd<false, false>(grid, stream, qkv, do_masked, head_mask, lse, Dvec, dqkv, key_len, sh, scale, dropout_p, seed, rb, nullptr, bpart);
  }
  DPH_TRY(check_launch("dph_attention_bwd"));
  // q / v bias gradients: the wave-row slab summed over its rows in order (queued in a deferred-reduction block)
  if (bpart != nullptr) DPH_TRY(slab_reduce_cols(bpart, B * grid.x, 2 * H * HD, H * HD, dbq, dbv, nullptr, stream));
  return check_launch("dph_attention_bwd");
}

// the q / v bias-gradient slab of dph_attention_bwd_qv / dph_attention_bwd_relpos_qv: one fp32 row of [q | v] columns
// (2 * H * 64) per 128-row block of the backward grid (B * ceil(T / 128) rows)
extern "C" int64_t dph_attention_bwd_qv_workspace(int64_t B, int64_t T, int64_t H) {
  return B * cdiv(T, (int64_t)RB) * 2 * H * HD * 4;
}

extern "C" int dph_attention_fwd(const void* qkv, void* o_unmasked, void* o_masked, float* lse,
                                 const float* head_mask, const int64_t* key_len, int64_t B, int64_t T, int64_t H,
                                 float scale, float dropout_p, uint64_t seed, void* keep_bits, hipStream_t stream) {
  DPH_REQUIRE(qkv && o_masked && B > 0 && T > 0 && H > 0, "dph_attention_fwd: bad args");
  return attention_fwd(qkv, o_unmasked, o_masked, lse, head_mask, key_len, B, T, H, scale, dropout_p, seed,
                       RelBias{nullptr, nullptr, nullptr, nullptr}, keep_bits, stream);
}

extern "C" int dph_attention_fwd_relpos(const void* qkv, void* o_unmasked, void* o_masked, float* lse,
                                        const float* head_mask, const int64_t* key_len, const float* rel_tab,
                                        const float* gate, int64_t B, int64_t T, int64_t H, float scale,
                                        float dropout_p, uint64_t seed, void* keep_bits, hipStream_t stream) {
  DPH_REQUIRE(qkv && o_masked && rel_tab && gate && B > 0 && T > 0 && T <= 3584 && H > 0,
              "dph_attention_fwd_relpos: bad args (T <= 3584)");
  return attention_fwd(qkv, o_unmasked, o_masked, lse, head_mask, key_len, B, T, H, scale, dropout_p, seed,
                       RelBias{rel_tab, gate, nullptr, nullptr}, keep_bits, stream);
}

static int64_t prep_rpb_host(int64_t H) { return H <= 32 ? 4 : 1; }

extern "C" int64_t dph_attention_bwd_prep_workspace(int64_t B, int64_t T, int64_t H) {
  return cdiv(B * T, prep_rpb_host(H) * PREP_IT) * H * 4;
}

extern "C" int dph_attention_bwd_prep(const void* do_masked, const void* o_unmasked, const float* head_mask,
                                      float* Dvec, float* dhead_mask, int64_t B, int64_t T, int64_t H, float* ws,
                                      int64_t ws_bytes, hipStream_t stream) {
  DPH_REQUIRE(do_masked && o_unmasked && Dvec && B > 0 && T > 0 && H > 0, "dph_attention_bwd_prep: bad args");
  const bool det = dhead_mask && deterministic();
  DPH_REQUIRE(!det || (ws && ws_bytes >= dph_attention_bwd_prep_workspace(B, T, H)),
              "dph_attention_bwd_prep: deterministic mode needs dph_attention_bwd_prep_workspace bytes");
  DPH_REQUIRE(H <= 128, "dph_attention_bwd_prep: H=%lld > 128", (long long)H);
  const int64_t rpb = prep_rpb_host(H);
  dim3 grid((unsigned)cdiv(B * T, rpb * PREP_IT));
  hipLaunchKernelGGL(attn_bwd_prep_kernel, grid, dim3((unsigned)(rpb * H * 8)), 0, stream,
                     reinterpret_cast<const bf16_t*>(do_masked),
                     reinterpret_cast<const float*>(o_unmasked), head_mask, Dvec, dhead_mask, B, T, H,
                     det ? ws : nullptr);
  if (det) DPH_TRY(slab_reduce_cols(ws, grid.x, H, H, dhead_mask, nullptr, nullptr, stream));
  return check_launch("dph_attention_bwd_prep");
}

extern "C" int dph_attention_bwd(const void* qkv, const void* do_masked, const float* head_mask, const float* lse,
                                 const float* Dvec, void* dqkv, const int64_t* key_len, int64_t B, int64_t T,
                                 int64_t H, float scale, float dropout_p, uint64_t seed, const void* keep_bits,
                                 hipStream_t stream) {
  DPH_REQUIRE(qkv && do_masked && lse && Dvec && dqkv && B > 0 && T > 0 && H > 0, "dph_attention_bwd: bad args");
  return attention_bwd(qkv, do_masked, head_mask, lse, Dvec, dqkv, key_len, B, T, H, scale, dropout_p, seed,
                       RelBias{nullptr, nullptr, nullptr, nullptr}, keep_bits, stream);
}

extern "C" int dph_attention_bwd_qv(const void* qkv, const void* do_masked, const float* head_mask, const float* lse,
                                    const float* Dvec, void* dqkv, const int64_t* key_len, int64_t B, int64_t T,
                                    int64_t H, float scale, float dropout_p, uint64_t seed, const void* keep_bits,
                                    float* dbq, float* dbv, float* ws, int64_t ws_bytes, hipStream_t stream) {
  DPH_REQUIRE(qkv && do_masked && lse && Dvec && dqkv && dbq && dbv && B > 0 && T > 0 && H > 0,
              "dph_attention_bwd_qv: bad args");
  DPH_REQUIRE(ws && ws_bytes >= dph_attention_bwd_qv_workspace(B, T, H) && (reinterpret_cast<uintptr_t>(ws) & 15) == 0,
              "dph_attention_bwd_qv: needs dph_attention_bwd_qv_workspace bytes (16-B aligned)");
  return attention_bwd(qkv, do_masked, head_mask, lse, Dvec, dqkv, key_len, B, T, H, scale, dropout_p, seed,
                       RelBias{nullptr, nullptr, nullptr, nullptr}, keep_bits, stream, dbq, dbv, ws);
}

// deterministic mode: the dQ blocks' diagonal-sum slab [B][H][ceil(T/128)][T + 127] fp32
extern "C" int64_t dph_attention_bwd_relpos_workspace(int64_t B, int64_t T, int64_t H) {
  return B * H * cdiv(T, (int64_t)RB) * (T + RB - 1) * 4;
}

static int attention_bwd_relpos(const void* qkv, const void* do_masked, const float* head_mask, const float* lse,
                                const float* Dvec, void* dqkv, const int64_t* key_len, const float* rel_tab,
                                const float* gate, float* dgate, float* drel_tab, int64_t B, int64_t T, int64_t H,
                                float scale, float dropout_p, uint64_t seed, const void* keep_bits, float* ws,
                                int64_t ws_bytes, hipStream_t stream, float* dbq, float* dbv, float* bws) {
  DPH_REQUIRE(qkv && do_masked && lse && Dvec && dqkv && rel_tab && gate && dgate && drel_tab && B > 0 && T > 0 &&
                  T <= 3584 && H > 0,
              "dph_attention_bwd_relpos: bad args (T <= 3584: the [T+127] fp32 table window, in deterministic mode plus four "
              "per-wave [T+127] diagonal histograms -- <= 74 KB of dynamic LDS beside 34 KB of tiles)");
  const bool det = deterministic();
  DPH_REQUIRE(!det || (ws && ws_bytes >= dph_attention_bwd_relpos_workspace(B, T, H)),
              "dph_attention_bwd_relpos: deterministic mode needs dph_attention_bwd_relpos_workspace bytes");
  const int rc = attention_bwd(qkv, do_masked, head_mask, lse, Dvec, dqkv, key_len, B, T, H, scale, dropout_p, seed,
                               RelBias{rel_tab, gate, dgate, drel_tab, det ? ws : nullptr}, keep_bits, stream, dbq,
                               dbv, bws);
  if (rc || !det) return rc;
  hipLaunchKernelGGL(relpos_dtab_reduce, dim3((unsigned)cdiv(H * (2 * T - 1), 256)), dim3(256), 0, stream, ws, B, H, T,
                     drel_tab);
  return check_launch("dph_attention_bwd_relpos dtab reduce");
}

extern "C" int dph_attention_bwd_relpos(const void* qkv, const void* do_masked, const float* head_mask,
                                        const float* lse, const float* Dvec, void* dqkv, const int64_t* key_len,
                                        const float* rel_tab, const float* gate, float* dgate, float* drel_tab,
                                        int64_t B, int64_t T, int64_t H, float scale, float dropout_p, uint64_t seed,
                                        const void* keep_bits, float* ws, int64_t ws_bytes, hipStream_t stream) {
  return attention_bwd_relpos(qkv, do_masked, head_mask, lse, Dvec, dqkv, key_len, rel_tab, gate, dgate, drel_tab, B,
                              T, H, scale, dropout_p, seed, keep_bits, ws, ws_bytes, stream, nullptr, nullptr,
                              nullptr);
}

extern "C" int dph_attention_bwd_relpos_qv(const void* qkv, const void* do_masked, const float* head_mask,
                                           const float* lse, const float* Dvec, void* dqkv, const int64_t* key_len,
                                           const float* rel_tab, const float* gate, float* dgate, float* drel_tab,
                                           int64_t B, int64_t T, int64_t H, float scale, float dropout_p,
                                           uint64_t seed, const void* keep_bits, float* ws, int64_t ws_bytes,
                                           float* dbq, float* dbv, float* bws, int64_t bws_bytes,
                                           hipStream_t stream) {
  DPH_REQUIRE(dbq && dbv && bws && bws_bytes >= dph_attention_bwd_qv_workspace(B, T, H) &&
                  (reinterpret_cast<uintptr_t>(bws) & 15) == 0,
              "dph_attention_bwd_relpos_qv: needs dph_attention_bwd_qv_workspace bytes (16-B aligned)");
  return attention_bwd_relpos(qkv, do_masked, head_mask, lse, Dvec, dqkv, key_len, rel_tab, gate, dgate, drel_tab, B,
                              T, H, scale, dropout_p, seed, keep_bits, ws, ws_bytes, stream, dbq, dbv, bws);
}
