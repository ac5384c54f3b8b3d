// Generic bf16 MFMA GEMM for gfx950 with fused epilogues.
//
//   C[z][m][n] = epi( alpha * sum_k A[z][m][k] * B[z][k][n] )
//
// One kernel serves every matmul of the DPHuBERT hot path (forward, input
// gradient and weight gradient of nn.Linear, the strided conv1..6 as an
// implicit GEMM over channels-last activations, the grouped positional conv
// as a batched GEMM) -- see include/dphubert_hip.h for the call sites.
//
// Tiling: 128x128x64 block tile, 256 threads = 4 waves (2x2), each wave a
// 64x64 output tile = 4x4 v_mfma_f32_16x16x32_bf16 accumulators.  Both
// operands are staged global -> registers -> LDS with a double-buffered LDS
// ring and ONE barrier per K-step.  Operand layouts:
//   k-contiguous  ([rows][K]): LDS image [128][64], 16-B chunk p of row r holds
//                 k-chunk p ^ ((r>>1)&7) (conflict free for the 16-lane
//                 ds_read_b128 groups and the 2-row ds_write_b128 groups; the
//                 padded [128][72] image measured 33 % bank-conflict cycles),
//                 fragments by ds_read_b128.
//   mn-contiguous ([K][rows]): LDS image [64][128] with a 32-B XOR swizzle
//                 (unit ^= (k&3)|((k>>3)&1)<<2, conflict free for the two
//                 8-row halves of a transposed read), fragments by the gfx950
//                 hardware transpose read ds_read_b64_tr_b16 -- no explicit
//                 transposes of activations or weights anywhere.
// The MFMA is issued "swapped" (B-tile fragment as the A operand) so each
// lane ends up holding 4 CONSECUTIVE output columns of one row: 8-B (bf16)
// or 16-B (fp32) stores and cheap per-column epilogue vectors.
#include "gemm_core.h"

#include <type_traits>

#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

namespace dph {

namespace {
constexpr int BM = 128;
constexpr int BN = 128;
constexpr int BK = 64;
constexpr int NTHREADS = 256;                 // 4 waves: 2 (M) x 2 (N), each a 64x64 output tile
constexpr int CHUNKS = (128 * BK / 8) / NTHREADS;   // 16-B chunks per thread per operand tile
constexpr int WTN = 64;                       // wave tile width (N)
constexpr int NJ = WTN / 16;                  // accumulator tiles per wave along N
constexpr int LDS_KC = 128 * BK * 2;          // bytes, k-contig tile [128][64], 16-B chunk XOR swizzle
constexpr int LDS_MN = BK * 128 * 2;          // bytes, mn-contig tile

template <bool KC>
struct TileBytes {
  static constexpr int v = KC ? LDS_KC : LDS_MN;
};


__device__ __forceinline__ int swz(int k) { return (k & 3) | (((k >> 3) & 1) << 2); }

// ---- staging: global -> registers ----------------------------------------
template <bool KC, int NT = NTHREADS>
struct Stager {
  static constexpr int CH = (128 * BK / 8) / NT;   // 16-B chunks per thread per operand tile
  const bf16_t* base;   // operand base incl. batch offset
  int64_t roff[CH];  // k-contig: per-chunk row offsets (fixed per block)
  bool rvalid[CH];
  int64_t r0;           // first row/col of the tile (M or N index)
  int64_t R;            // rows (M or N)
  DphMat d;

  __device__ __forceinline__ void init(const DphMat& dm, const bf16_t* b, int64_t tile0, int64_t Rn, int tid) {
    d = dm;
    base = b;
    r0 = tile0;
    R = Rn;
    if constexpr (KC) {
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        int c = tid + NT * i;
        int64_t r = tile0 + (c >> 3);
        rvalid[i] = r < Rn;
        roff[i] = row_addr(dm, rvalid[i] ? r : Rn - 1);
      }
    }
  }

  // Loads are unconditional (addresses clamped into the operand) so hipcc can keep several
  // tiles in flight with counted vmcnt; out-of-range chunks are zeroed at store time.
  __device__ __forceinline__ void load(uint4 (&reg)[CH], int64_t k0, int64_t kend, int tid) const {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      int c = tid + NT * i;
      if constexpr (KC) {
        int64_t k = min(k0 + (c & 7) * 8, kend - 8);
        reg[i] = *reinterpret_cast<const uint4*>(base + roff[i] + k);
      } else {
        int64_t k = min(k0 + (c >> 4), kend - 1);
        int64_t col = min(r0 + (c & 15) * 8, ((R + 7) & ~(int64_t)7) - 8);   // padded rows: see dph_gemm
        reg[i] = *reinterpret_cast<const uint4*>(base + row_addr(d, k) + col);
      }
    }
  }

  __device__ __forceinline__ void store(char* lds, const uint4 (&reg)[CH], int64_t k0, int64_t kend, int tid) const {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      int c = tid + NT * i;
      int byte;
      bool ok;
      if constexpr (KC) {
        byte = (c >> 3) * 128 + (((c & 7) ^ (((c >> 3) >> 1) & 7)) * 16);
        ok = rvalid[i] && (k0 + (c & 7) * 8 < kend);
      } else {
        int kr = c >> 4;
        int col8 = c & 15;
        int u = (col8 >> 1) ^ swz(kr);
        byte = kr * 256 + u * 32 + (col8 & 1) * 16;
        ok = (k0 + kr < kend) && (r0 + col8 * 8 < R);
      }
      *reinterpret_cast<uint4*>(lds + byte) = ok ? reg[i] : make_uint4(0, 0, 0, 0);
    }
  }
};

// ---- fragments: LDS -> registers --------------------------------------------
// Returns the MFMA operand fragment for rows [rb, rb+16) of the tile and
// k-substep ks: lane l holds X[row rb + (l&15)][k = ks*32 + 8*(l>>4) + j].
template <bool KC>
__device__ __forceinline__ bf16x8_t frag(const char* lds, int rb, int ks, int lane) {
  if constexpr (KC) {
    const int row = rb + (lane & 15);
    const int phys = (ks * 4 + (lane >> 4)) ^ ((row >> 1) & 7);
    return *reinterpret_cast<const bf16x8_t*>(lds + row * 128 + phys * 16);
  } else {
    const int g = lane >> 4;
    const int i = lane & 15;
    const int q = i >> 2;
    const int p = i & 3;
    const int k0 = ks * 32 + 8 * g + q;
    const int u = rb >> 4;
    const int b0 = k0 * 256 + ((u ^ swz(k0)) * 32) + 8 * p;
    const int k1 = k0 + 4;
    const int b1 = k1 * 256 + ((u ^ swz(k1)) * 32) + 8 * p;
    typedef __attribute__((address_space(3))) s16x4_t lds_s16x4;
    s16x4_t v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + b0));
    s16x4_t v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + b1));
    s16x8_t v = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
    return __builtin_bit_cast(bf16x8_t, v);
  }
}

// ---- epilogue ---------------------------------------------------------------
// Row-contiguous epilogue: one thread handles 8 consecutive columns [n, n+8) of row m, so
// every global access (bias / mask vectors, residual / aux inputs, pre-activation and C
// outputs) is a 16-byte vector access and a wave covers whole 256-B row segments.
struct Cs8 {
  float out[8];
  float aux[8];
};

__device__ __forceinline__ void load8_bf16(const bf16_t* p, bool vec, int nv, float (&o)[8]) {
  if (vec) {
    const uint4 r = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      o[2 * q] = __uint_as_float(w[q] << 16);
      o[2 * q + 1] = __uint_as_float(w[q] & 0xffff0000u);
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (i < nv) ? bf2f(p[i]) : 0.f;
  }
}

__device__ __forceinline__ void load8_f32(const float* p, bool vec, int nv, float (&o)[8]) {
  if (vec) {
    const float4 a = *reinterpret_cast<const float4*>(p);
    const float4 b = *reinterpret_cast<const float4*>(p + 4);
    o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w;
    o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (i < nv) ? p[i] : 0.f;
  }
}

__device__ __forceinline__ void store8_bf16(bf16_t* p, bool vec, int nv, const float (&v)[8]) {
  if (vec) {
    *reinterpret_cast<uint4*>(p) = make_uint4(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]), pack2bf(v[4], v[5]),
                                              pack2bf(v[6], v[7]));
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (i < nv) p[i] = f2bf(v[i]);
  }
}

__device__ __forceinline__ void epilogue8(const DphGemmArgs& a, int64_t z, int64_t m, int64_t n, float (&v)[8],
                                          Cs8& cs) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    cs.out[i] = 0.f;
    cs.aux[i] = 0.f;
  }
  if (m >= a.M || n >= a.N) return;
  const int64_t voff = (a.C.z_div > 0 ? (z % a.C.z_div) : z) * a.vec_z_inner;
  const int64_t coff = z_addr(a.C, z) + row_addr(a.C, m) + n;
  const int nv = (int)min<int64_t>(8, a.N - n);
  // 16-B vector path needs 8 valid columns and 16-B aligned rows (all strides multiples of 8)
  const bool vec = (nv == 8) && ((coff & 7) == 0);
  const bool vvec = (nv == 8) && (((voff + n) & 3) == 0);
  const float inv_keep = a.dropout_p > 0.f ? 1.0f / (1.0f - a.dropout_p) : 1.0f;
  const uint64_t seed = a.dropout_p > 0.f ? epoch_seed(a.seed) : 0;
  const uint64_t drow = ((uint64_t)(z * a.M + a.drop_row_offset + m)) * (uint64_t)a.N;
  bool zero_row = false;
  if (a.row_len) zero_row = (m % a.len_rows) >= a.row_len[m / a.len_rows];
  float bias[8], cm[8], aux[8], res[8];
  if (a.bias) load8_f32(a.bias + voff + n, vvec, nv, bias);
  if (a.colmask) load8_f32(a.colmask + voff + n, vvec, nv, cm);
  if (a.aux_in) load8_bf16(reinterpret_cast<const bf16_t*>(a.aux_in) + coff, vec, nv, aux);
  if (a.residual) {
    if (a.flags & DPH_GEMM_RESID_F32)   // fp32 residual stream (pre-norm layers)
      load8_f32(reinterpret_cast<const float*>(a.residual) + coff,
                (nv == 8) && ((coff & 3) == 0) && ((reinterpret_cast<uintptr_t>(a.residual) & 15) == 0), nv, res);
    else
      load8_bf16(reinterpret_cast<const bf16_t*>(a.residual) + coff, vec, nv, res);
  }
  const float sm = a.smask ? *a.smask : 1.0f;
  float pre[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    float x = v[i] * a.alpha;
    if (a.bias) x += bias[i];
    pre[i] = x;
    const float dz = dropout_scale(seed, drow + n + i, a.dropout_p, inv_keep);
    const float c = a.colmask ? cm[i] : 1.0f;
    float ax = 0.f;
    if (a.act == DPH_ACT_GELU) {
      x = gelu_f(x) * dz * c;
    } else if (a.act == DPH_ACT_GELU_BWD) {
      const float gz = x * dz;
      float g, dg;
      gelu_and_grad(aux[i], g, dg);
      ax = gz * g;
      x = gz * dg * c;
    } else {
      x = x * dz * c;
    }
    x = x * sm;
    if (a.residual) x += res[i];
    if (zero_row) x = 0.f;
    v[i] = x;
    cs.out[i] = (i < nv) ? x : 0.f;
    cs.aux[i] = (i < nv) ? ax : 0.f;
  }
  if (a.pre_out) store8_bf16(reinterpret_cast<bf16_t*>(a.pre_out) + coff, vec, nv, pre);
  if (a.c_dtype == DPH_OUT_BF16) {
    store8_bf16(reinterpret_cast<bf16_t*>(a.C.ptr) + coff, vec, nv, v);
  } else {
    float* p = reinterpret_cast<float*>(a.C.ptr) + coff;
    const bool fvec = (nv == 8) && ((coff & 3) == 0);
    if (a.c_dtype == DPH_OUT_F32_ACCUM) {
      float old[8];
      load8_f32(p, fvec, nv, old);
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] += old[i];
    }
    if (fvec) {
      *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
      *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (i < nv) p[i] = v[i];
    }
  }
}

// ---- fast tile epilogue ----------------------------------------------------------------------
// A thread owns the 8 columns [n, n+8) of the P rows m = mrow0 + RPP*p + (p/JP)*JUMP of a staged
// fp32 tile (LDS row mrow0-relative RPP*p).
// gfx9 counts stores in vmcnt, so a global load issued after a store makes its s_waitcnt wait
// for that store's write acknowledgement: the per-row generic epilogue8 (conditional loads
// between stores, each behind an s_waitcnt vmcnt(0)) measured 15 us per round of 128x128 tiles,
// as long as the whole K=768 main loop.  Here every global input (bias / colmask once, then the
// per-row aux / residual / old-C / row-length values of all P rows) is issued first, retired by
// one wait, and the stores follow with no load behind them.  Preconditions (tile_epi_ok): full
// 8-column groups and 16-B aligned rows of C and of the vectors.
__device__ __forceinline__ bool tile_epi_ok(const DphGemmArgs& a, int64_t n) {
  const int64_t calign = a.C.row_stride | a.C.batch_stride | a.C.z_outer | a.C.z_inner;
  const uintptr_t palign = reinterpret_cast<uintptr_t>(a.C.ptr) | reinterpret_cast<uintptr_t>(a.pre_out) |
                           reinterpret_cast<uintptr_t>(a.aux_in) | reinterpret_cast<uintptr_t>(a.residual);
  const uintptr_t valign = reinterpret_cast<uintptr_t>(a.bias) | reinterpret_cast<uintptr_t>(a.colmask);
  // one per-row bf16 input (aux_in OR residual) and a plain (non-accumulating) output
  // (an fp32 residual takes the generic epilogue8)
  return n + 8 <= a.N && (calign & 7) == 0 && (palign & 15) == 0 && (valign & 15) == 0 &&
         (a.vec_z_inner & 3) == 0 && !(a.aux_in && a.residual) && a.c_dtype != DPH_OUT_F32_ACCUM &&
         (a.N & 1) == 0 && !(a.flags & DPH_GEMM_RESID_F32);
}

__device__ __forceinline__ void unpack_bf16x8(const uint4 r, float (&o)[8]) {
  const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    o[2 * q] = __uint_as_float(w[q] << 16);
    o[2 * q + 1] = __uint_as_float(w[q] & 0xffff0000u);
  }
}

__device__ __forceinline__ void load_f32x8(const float* p, float (&o)[8]) {
  const float4 u = *reinterpret_cast<const float4*>(p);
  const float4 v = *reinterpret_cast<const float4*>(p + 4);
  o[0] = u.x; o[1] = u.y; o[2] = u.z; o[3] = u.w;
  o[4] = v.x; o[5] = v.y; o[6] = v.z; o[7] = v.w;
}

// Rolled row loop (small code: the executed epilogue is fetched once into the instruction cache;
// fully unrolled variants measured 1.6x slower per tile purely with code size), the row-dependent
// input of row p+1 is loaded before row p's stores, so its wait never covers a store.
template <int P, int RPP, int JP, int JUMP, int ACT, bool DROP>
__device__ __forceinline__ void tile_epi_rows(const DphGemmArgs& a, int64_t z, int64_t mrow0, int64_t n,
                                              const float* lds, int lds_stride, float (&cso)[8], float (&csa)[8]) {
  const int64_t voff = (a.C.z_div > 0 ? (z % a.C.z_div) : z) * a.vec_z_inner + n;
  const int64_t cz = z_addr(a.C, z) + n;
  // (arithmetic select of the two pointer VALUES: a `?:` over the fields becomes a select of field
  // addresses, which forces the whole kernel-argument struct into scratch)
  const uintptr_t ax_p = reinterpret_cast<uintptr_t>(a.aux_in), rs_p = reinterpret_cast<uintptr_t>(a.residual);
  const bf16_t* inp = reinterpret_cast<const bf16_t*>(ax_p | (rs_p & (uintptr_t)(-(intptr_t)(ax_p == 0))));
  const bool has_in = inp != nullptr, has_res = has_in && ax_p == 0;
  const bool has_len = a.row_len != nullptr, has_pre = a.pre_out != nullptr, out_bf16 = a.c_dtype == DPH_OUT_BF16;
  const bool colsum = a.colsum_out || a.colsum_aux;
  float bias[8], csm[8], kc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    bias[i] = 0.f;
    csm[i] = 1.f;
  }
  if (a.bias) load_f32x8(a.bias + voff, bias);
  if (a.colmask) load_f32x8(a.colmask + voff, csm);
  // per-column factors fixed for the thread: csm = colmask * layer mask, kc = csm / (1 - p)
  const float sm = a.smask ? *a.smask : 1.0f;
  const float inv_keep = DROP ? 1.0f / (1.0f - a.dropout_p) : 1.0f;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    csm[i] *= sm;
    kc[i] = csm[i] * inv_keep;
  }
  const uint32_t thr = DROP ? drop_thr(a.dropout_p) : 0u;
  const uint64_t seed = DROP ? epoch_seed(a.seed) : 0;
  const uint32_t lr = has_len ? (uint32_t)a.len_rows : 1u;
  auto row_of = [&](int p) -> int64_t { return mrow0 + RPP * p + (p / JP) * JUMP; };
  uint4 nxt = make_uint4(0, 0, 0, 0);
  if (has_in && row_of(0) < a.M) nxt = *reinterpret_cast<const uint4*>(inp + cz + row_addr(a.C, row_of(0)));
#pragma unroll 1
  for (int p = 0; p < P; ++p) {
    const int64_t m = row_of(p);
    const uint4 cur = nxt;
    if (has_in && p + 1 < P && row_of(p + 1) < a.M)
      nxt = *reinterpret_cast<const uint4*>(inp + cz + row_addr(a.C, row_of(p + 1)));
    if (m >= a.M) continue;
    const int64_t coff = cz + row_addr(a.C, m);
    bool zero_row = false;
    if (has_len) {
      const uint32_t seg = (uint32_t)m / lr;
      zero_row = (uint32_t)m >= (uint32_t)a.row_len[seg] + seg * lr;
    }
    float v[8], in[8], pre[8], ax[8];
    load_f32x8(lds + p * RPP * lds_stride, v);
    unpack_bf16x8(cur, in);
    uint32_t keep = 0xffu;                     // bit i: element i kept
    if constexpr (DROP) {
      const uint64_t pair0 = (((uint64_t)(z * a.M + a.drop_row_offset + m)) * (uint64_t)a.N + (uint64_t)n) >> 1;
      keep = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t bits = drop_bits2(seed, pair0 + j);
        keep |= ((bits & 0xffffu) >= thr ? 1u : 0u) << (2 * j);
        keep |= ((bits >> 16) >= thr ? 1u : 0u) << (2 * j + 1);
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      pre[i] = fmaf(v[i], a.alpha, bias[i]);
      const bool k = (keep >> i) & 1u;
      if constexpr (ACT == DPH_ACT_GELU) {
        v[i] = k ? gelu_f(pre[i]) * kc[i] : 0.f;
      } else if constexpr (ACT == DPH_ACT_GELU_BWD) {
        const float gz = DROP ? (k ? pre[i] * inv_keep : 0.f) : pre[i];
        float g, dg;
        gelu_and_grad(in[i], g, dg);
        ax[i] = gz * g;
        v[i] = gz * dg * csm[i];
      } else {
        v[i] = DROP ? (k ? pre[i] * kc[i] : 0.f) : pre[i] * csm[i];
      }
    }
    if (has_res) {
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] += in[i];
    }
    if (zero_row) {
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = 0.f;
    }
    if (colsum) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        cso[i] += v[i];
        if constexpr (ACT == DPH_ACT_GELU_BWD) csa[i] += ax[i];
      }
    }
#ifdef DPH_EPI_NOSTORE
    if (v[0] != 1.2345e-30f) continue;   // timing diagnostic: no global stores (results kept live)
#endif
    if (has_pre)
      *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(a.pre_out) + coff) =
          make_uint4(pack2bf(pre[0], pre[1]), pack2bf(pre[2], pre[3]), pack2bf(pre[4], pre[5]), pack2bf(pre[6], pre[7]));
    if (out_bf16) {
      *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(a.C.ptr) + coff) =
          make_uint4(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]), pack2bf(v[4], v[5]), pack2bf(v[6], v[7]));
    } else {
      float* q = reinterpret_cast<float*>(a.C.ptr) + coff;
      *reinterpret_cast<float4*>(q) = make_float4(v[0], v[1], v[2], v[3]);
      *reinterpret_cast<float4*>(q + 4) = make_float4(v[4], v[5], v[6], v[7]);
    }
  }
}

// The activation and dropout are template parameters: with runtime switches hipcc if-converts the
// branches and evaluates BOTH erfc-GELU forms and the dropout hash for every element (measured
// 32k cycles per 128x128 tile with every feature off, vs 2.5k for a bare copy-out).
template <int P, int RPP, int JP = P, int JUMP = 0>
__device__ __forceinline__ void tile_epi(const DphGemmArgs& a, int64_t z, int64_t mrow0, int64_t n, const float* lds,
                                         int lds_stride, float (&cso)[8], float (&csa)[8]) {
  const bool drop = a.dropout_p > 0.f;
  if (a.act == DPH_ACT_GELU) {
    if (drop) tile_epi_rows<P, RPP, JP, JUMP, DPH_ACT_GELU, true>(a, z, mrow0, n, lds, lds_stride, cso, csa);
    else tile_epi_rows<P, RPP, JP, JUMP, DPH_ACT_GELU, false>(a, z, mrow0, n, lds, lds_stride, cso, csa);
  } else if (a.act == DPH_ACT_GELU_BWD) {
    if (drop) tile_epi_rows<P, RPP, JP, JUMP, DPH_ACT_GELU_BWD, true>(a, z, mrow0, n, lds, lds_stride, cso, csa);
    else tile_epi_rows<P, RPP, JP, JUMP, DPH_ACT_GELU_BWD, false>(a, z, mrow0, n, lds, lds_stride, cso, csa);
  } else {
    if (drop) tile_epi_rows<P, RPP, JP, JUMP, DPH_ACT_NONE, true>(a, z, mrow0, n, lds, lds_stride, cso, csa);
    else tile_epi_rows<P, RPP, JP, JUMP, DPH_ACT_NONE, false>(a, z, mrow0, n, lds, lds_stride, cso, csa);
  }
}

// LDS staging of the fp32 accumulator tile for the row-contiguous epilogue
constexpr int CROW = BN + 4;                       // padded fp32 row
constexpr int LDS_C = BM * CROW * 4;               // 67,584 B

template <bool AK, bool BKc, int NT = NTHREADS>
__global__ void __launch_bounds__(NT, 2) gemm_kernel(const DphGemmArgs a, int64_t kchunk,
                                                     unsigned* __restrict__ tile_cnt = nullptr) {
  constexpr int PIPE = 2 * (TileBytes<AK>::v + TileBytes<BKc>::v);
  __shared__ __attribute__((aligned(16))) char smem[PIPE > LDS_C ? PIPE : LDS_C];
  char* const ldsA0 = smem;
  char* const ldsB0 = smem + 2 * TileBytes<AK>::v;
#define LDSA(buf) (ldsA0 + (buf) * TileBytes<AK>::v)
#define LDSB(buf) (ldsB0 + (buf) * TileBytes<BKc>::v)

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  // NT = 256: 4 waves 2 (M) x 2 (N) of 64x64; NT = 512: 8 waves 2 x 4 of 64x32 (two waves per SIMD
  // per block: one wave's fragment reads / barrier wait overlap the other's MFMAs)
  constexpr int NWN = NT / 128;            // waves along N
  constexpr int KWTN = BN / NWN;           // wave tile width
  constexpr int KNJ = KWTN / 16;
  const int wm = wave / NWN;
  const int wn = wave % NWN;

  const int64_t zz = blockIdx.z;
  const int64_t split = zz % a.splits;
  const int64_t z = zz / a.splits;
  // XCD-aware grouped tile order (guide T1): blocks are dealt round-robin over the 8 XCDs, so
  // give every XCD a contiguous range of tiles, and walk that range in GROUP_M-tall column
  // strips so the ~64 co-resident blocks of an XCD cover an 8x8 tile square and share their
  // A/B panels in that XCD's private L2.
  int64_t tm, tn;
  {
    const int64_t ntm = gridDim.y, ntn = gridDim.x;
    const int64_t nt = ntm * ntn;
    const int64_t bid = (int64_t)blockIdx.y * ntn + blockIdx.x;
    const int64_t q = nt / 8, r = nt % 8;
    const int64_t xcd = bid % 8, loc = bid / 8;
    const int64_t t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
    constexpr int64_t GM = 8;
    const int64_t gsz = GM * ntn;
    const int64_t grp = t / gsz;
    const int64_t gm0 = grp * GM;
    const int64_t gh = min(GM, ntm - gm0);
    const int64_t l = t % gsz;
    tm = gm0 + l % gh;
    tn = l / gh;
  }
  const int64_t m0 = tm * BM;
  const int64_t n0 = tn * BN;
  const int64_t kbeg = split * kchunk;
  const int64_t kend = min(a.K, kbeg + kchunk);

  Stager<AK, NT> sa;
  Stager<BKc, NT> sb;
  sa.init(a.A, reinterpret_cast<const bf16_t*>(a.A.ptr) + z_addr(a.A, z), m0, a.M, tid);
  sb.init(a.B, reinterpret_cast<const bf16_t*>(a.B.ptr) + z_addr(a.B, z), n0, a.N, tid);

  f32x4_t acc[4][KNJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < KNJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // Pipeline: LDS double buffer + one register stage.  Tile t+1 is issued into registers at the
  // top of step t (unconditional loads: counted vmcnt), tile t is computed from LDS, then tile
  // t+1 is written to the other LDS buffer behind one barrier.  Two co-resident blocks per CU
  // (73 KB LDS, <=256 VGPR) overlap each other's load latency.
  uint4 ra[Stager<AK, NT>::CH], rb[Stager<BKc, NT>::CH];
  const int nk = (int)cdiv(max<int64_t>(kend - kbeg, 0), BK);
  auto kof = [&](int t) { return kbeg + (int64_t)t * BK; };
  if (nk > 0) {
    sa.load(ra, kof(0), kend, tid);
    sb.load(rb, kof(0), kend, tid);
    sa.store(LDSA(0), ra, kof(0), kend, tid);
    sb.store(LDSB(0), rb, kof(0), kend, tid);
  }
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    const int cur = t & 1;
    const bool more = (t + 1) < nk;
    if (more) {
      sa.load(ra, kof(t + 1), kend, tid);
      sb.load(rb, kof(t + 1), kend, tid);
    }
    const char* LA = LDSA(cur);
    const char* LB = LDSB(cur);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8_t af[4], bfr[KNJ];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = frag<AK>(LA, wm * 64 + 16 * i, ks, lane);
#pragma unroll
      for (int j = 0; j < KNJ; ++j) bfr[j] = frag<BKc>(LB, wn * KWTN + 16 * j, ks, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < KNJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
    if (more) {
      sa.store(LDSA(cur ^ 1), ra, kof(t + 1), kend, tid);
      sb.store(LDSB(cur ^ 1), rb, kof(t + 1), kend, tid);
    }
    __syncthreads();
  }

#undef LDSA
#undef LDSB
  // ---- accumulators -> LDS (lane holds C[rowbase + (lane&15)][colbase + 4*(lane>>4) + r]) ----
  float* ct = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = wm * 64 + 16 * i + (lane & 15);
#pragma unroll
    for (int j = 0; j < KNJ; ++j) {
      const int c = wn * KWTN + 16 * j + 4 * (lane >> 4);
      *reinterpret_cast<float4*>(ct + r * CROW + c) = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2],
                                                                   acc[i][j][3]);
    }
  }
  __syncthreads();
  // ---- row-contiguous epilogue: thread = 8 columns x 8 rows (rows r0 + 16 p) ----
  const int c8 = (tid & 15) * 8;
  const int r0 = tid >> 4;
  if (a.splits > 1) {
    float* ws = reinterpret_cast<float*>(a.workspace) + (zz * a.M) * a.N;
#pragma unroll 2
    for (int p = 0; p < BM * BN / 8 / NT; ++p) {
      const int r = r0 + (NT / 16) * p;
      const int64_t m = m0 + r;
      const int64_t n = n0 + c8;
      if (m >= a.M || n >= a.N) continue;
      const float* src = ct + r * CROW + c8;
      float* dst = ws + m * a.N + n;
      if (n + 8 <= a.N && (a.N & 3) == 0) {
        *reinterpret_cast<float4*>(dst) = *reinterpret_cast<const float4*>(src);
        *reinterpret_cast<float4*>(dst + 4) = *reinterpret_cast<const float4*>(src + 4);
      } else {
        for (int q = 0; q < 8 && n + q < a.N; ++q) dst[q] = src[q];
      }
    }
    if (tile_cnt == nullptr) return;   // a separate splitk_reduce_kernel combines the slices
    // In-launch split-K combine (guide: "Projection GEMM at M = 256", item 2): publish this slice
    // (stores drained, agent-scope release, then the ticket), and the block that draws the last
    // ticket of the tile acquires, sums every slice's slab and runs the epilogue.  No block waits on
    // another, so any placement of a tile's slices over XCDs / CUs is correct.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    unsigned* flag = reinterpret_cast<unsigned*>(smem);
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int64_t tile = z * ((int64_t)gridDim.x * gridDim.y) + tm * gridDim.x + tn;
      const unsigned old = __hip_atomic_fetch_add(tile_cnt + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const bool last = old == (unsigned)(a.splits - 1);
      if (last) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        tile_cnt[tile] = 0u;   // ready for the next launch on the same counters
      }
      flag[0] = last ? 1u : 0u;
    }
    __syncthreads();
    if (flag[0] == 0u) return;
    const float* ws0 = reinterpret_cast<const float*>(a.workspace) + ((z * a.splits) * a.M) * a.N;
    const int64_t sstride = a.M * a.N;
#pragma unroll 1
    for (int p = 0; p < BM * BN / 8 / NT; ++p) {
      const int r = r0 + (NT / 16) * p;
      const int64_t m = m0 + r;
      const int64_t n = n0 + c8;
      if (m >= a.M || n >= a.N) continue;
      float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      const bool vec = n + 8 <= a.N && (a.N & 3) == 0;
      for (int sp = 0; sp < a.splits; ++sp) {
        float t[8];
        load8_f32(ws0 + sp * sstride + m * a.N + n, vec, (int)min<int64_t>(8, a.N - n), t);
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] += t[q];
      }
      Cs8 cs;
      epilogue8(a, z, m, n, v, cs);
    }
    return;
  }
  float cso[8], csa[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    cso[q] = 0.f;
    csa[q] = 0.f;
  }
  if (tile_epi_ok(a, n0 + c8)) {
    tile_epi<BM * BN / 8 / NT, NT / 16>(a, z, m0 + r0, n0 + c8, ct + r0 * CROW + c8, CROW, cso, csa);
  } else {
#pragma unroll 1
  for (int p = 0; p < BM * BN / 8 / NT; ++p) {
    const int r = r0 + (NT / 16) * p;
    const float* src = ct + r * CROW + c8;
    float v[8];
    const float4 x0 = *reinterpret_cast<const float4*>(src);
    const float4 x1 = *reinterpret_cast<const float4*>(src + 4);
    v[0] = x0.x; v[1] = x0.y; v[2] = x0.z; v[3] = x0.w;
    v[4] = x1.x; v[5] = x1.y; v[6] = x1.z; v[7] = x1.w;
    Cs8 cs;
    epilogue8(a, z, m0 + r, n0 + c8, v, cs);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      cso[q] += cs.out[q];
      csa[q] += cs.aux[q];
    }
  }
  }
  if ((a.colsum_out != nullptr) || (a.colsum_aux != nullptr)) {
    // lanes l, l^16, l^32, l^48 share columns inside a wave; then 4 waves through LDS
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      cso[q] += __shfl_xor(cso[q], 16, 64);
      cso[q] += __shfl_xor(cso[q], 32, 64);
      csa[q] += __shfl_xor(csa[q], 16, 64);
      csa[q] += __shfl_xor(csa[q], 32, 64);
    }
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);   // [waves][2][128]
    if (lane < 16) {   // (NT / 16 rows per pass: lanes l, l^16, ... share columns)
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        red[(wave * 2 + 0) * 128 + c8 + q] = cso[q];
        red[(wave * 2 + 1) * 128 + c8 + q] = csa[q];
      }
    }
    __syncthreads();
    if (tid < 128) {
      const int64_t n = n0 + tid;
      if (n < a.N) {
        const int64_t voff = (a.C.z_div > 0 ? (z % a.C.z_div) : z) * a.vec_z_inner;
        const int64_t csn = a.colsum_n > 0 ? a.colsum_n : a.N;
        float so = 0.f, sx = 0.f;
#pragma unroll
        for (int w = 0; w < NT / 64; ++w) {
          so += red[(w * 2 + 0) * 128 + tid];
          sx += red[(w * 2 + 1) * 128 + tid];
        }
        if (a.flags & GEMM_COLSUM_SLAB) {
          // one slab row per 128-row M tile and grid batch (dph_gemm sums the slab in a fixed order: deterministic
          // mode; batches share one output vector there)
          const int64_t ns = cdiv(a.M, (int64_t)BM);
          float* wo = reinterpret_cast<float*>(a.workspace) + (z * ns + m0 / BM) * a.N;
          if (n < csn) {
            wo[n] = so;
            wo[a.batch * ns * a.N + n] = sx;
          }
        } else {
          if (a.colsum_out && n < csn) atomicAdd(a.colsum_out + voff + n, so);
          if (a.colsum_aux && n < csn) atomicAdd(a.colsum_aux + voff + n, sx);
        }
      }
    }
  }
}

// =============================================================================================
// LDS-DMA ring kernels (both operands k-contiguous, K % 32 == 0), one template, two shapes:
//   RingCfg<256,256,128,64>: 256x256 tile, 8 waves (2 M x 4 N) of 128x64, one block per CU;
//   RingCfg<128,128,64,64>:  128x128 tile, 4 waves (2 x 2) of 64x64, two blocks per CU.
//
// Staging: a ring of 4 LDS slots, each one 32-deep k-slice of both operands ([rows][32 k] bf16),
// filled by the LDS-DMA (global_load_lds_dwordx4: no VGPR round trip, no ds_write, which at
// ~79 B/clk/CU would cost more LDS time than the ds_read_b128 fragment reads at 256 B/clk).
// k-slice i+4 is issued into slot i%4 as soon as slice i is in registers, so three slices (96 k)
// are always in flight behind the one being multiplied; waits are counted (`s_waitcnt vmcnt(8)`:
// 2 slices x 4 DMA per thread may stay pending) behind a raw s_barrier -- never vmcnt(0) in the
// loop.  Within a wave, the fragments of slice i+1 are read while the MFMAs of slice i run (two
// fragment register sets).  One barrier per slice certifies both that slice i+1 landed for every
// wave (RAW) and that every wave finished reading the slot being restaged (WAR).
//
// LDS image of an operand slice: 64-B rows; 16-B chunk p of row r holds logical k-chunk
// p ^ swz_chunk(r), conflict free for the real ds_read_b128 lane groups (each 16-lane group spans
// 16 rows and two k-chunks; the naive (r>>2)&3 measured 50 % bank-conflict cycles).  The swizzle
// is applied on the DMA SOURCE address since an LDS-DMA writes its 1 KB lane-linearly.
// =============================================================================================
#ifndef DPH_DIRECT_EPI
#define DPH_DIRECT_EPI 1    // 0: every ring tile takes the LDS-staged epilogue (A/B builds)
#endif
#ifndef DPH_ABLATE
#define DPH_ABLATE 0        // timing ablations of the ring loop (tools/ablate_gemm.py); 0 = production
#endif
#ifndef DPH_MID8_MINB
#define DPH_MID8_MINB 2     // blocks per CU of the 8-wave 128 x 128 tile (A/B builds: 1)
#endif
// internal DphGemmArgs.flags bit set by dph_gemm: the register epilogue writes its per-wave column sums to a
// workspace slab [2][cdiv(M, WTM)][N] (summed by colsum_slab_reduce_kernel) instead of one same-address float
// atomic per column per wave (126 -- 2000 adders per address on the FFN / conv input-gradient GEMMs: the
// atomics, not the MFMAs or the GELU', set those launches' time)
// (GEMM_COLSUM_SLAB: defined at the top of the file)
// internal flags bit set by dph_gemm / dph_gemm_grouped on ppw launches with gridDim.z > 1 (problems / split-K
// slices): the XCD-aware tile order runs over the whole (z, tile) space, so each XCD takes a contiguous range
// of one slice's / problem's tiles (their shared operand panels stay in that XCD's L2).  DPH_PPW_ZMAP=0: per-z order
constexpr int64_t GEMM_PPW_ZMAP = (int64_t)1 << 21;
namespace ring {
constexpr int KS = 32;      // k per slice
constexpr int NSLOT = 4;

// found by exhaustive search over 2-bit XOR swizzles of the row bits
__device__ __forceinline__ int swz_chunk(int r) { return ((r & 1) * 3) ^ (((r >> 2) & 1) << 1); }


// MFMA operand fragment: rows rb..rb+15 of a [rows][32] slice image; lane l gets
// X[rb + (l&15)][k = 8*(l>>4) .. +7]
__device__ __forceinline__ bf16x8_t frag(const char* lds, int rb, int lane) {
  const int row = rb + (lane & 15);
  const int phys = (lane >> 4) ^ swz_chunk(row);
  return *reinterpret_cast<const bf16x8_t*>(lds + row * 64 + phys * 16);
}

// mn-contiguous slice image: [KS k-rows][R] bf16 (rows of R*2 bytes); the 32-B unit u of k-row k holds
// logical unit u ^ swz(k) (the register-staged kernel's swizzle, conflict free for the transposed
// reads of a half-wave: k-rows {0..3, 8..11} + 16h).  Fragment: lane l gets X[rb + (l&15)][k = 8(l>>4)+j]
// by two hardware-transposed ds_read_b64_tr_b16.
__device__ __forceinline__ bf16x8_t frag_mn(const char* lds, int rb, int lane, int rbytes) {
  const int g = lane >> 4;
  const int i = lane & 15;
  const int q = i >> 2;
  const int p = i & 3;
  const int k0 = 8 * g + q;
  const int u = rb >> 4;
  const int b0 = k0 * rbytes + ((u ^ swz(k0)) * 32) + 8 * p;
  const int k1 = k0 + 4;
  const int b1 = k1 * rbytes + ((u ^ swz(k1)) * 32) + 8 * p;
  typedef __attribute__((address_space(3))) s16x4_t lds_s16x4;
  s16x4_t v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + b0));
  s16x4_t v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + b1));
  s16x8_t v = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
  return __builtin_bit_cast(bf16x8_t, v);
}

template <int BM_, int BN_, int WTM_, int WTN_>
struct Cfg {
  static constexpr int BM = BM_, BN = BN_, WTM = WTM_, WTN = WTN_;
  static constexpr int WGM = BM / WTM, WGN = BN / WTN;     // wave grid
  static constexpr int NW = WGM * WGN;
  static constexpr int NT = 64 * NW;
  static constexpr int FM = WTM / 16, FN = WTN / 16;       // accumulator tiles per wave
  static_assert(FM >= FN, "the ring step deals fragment reads over FM chunks");
  static constexpr int HALF_A = BM * KS * 2, HALF_B = BN * KS * 2;
  static constexpr int SLOT = HALF_A + HALF_B;
  static constexpr int PIPE = NSLOT * SLOT;
  static constexpr int DMA_A = BM * 64 / (NT * 16);          // DMA instructions per thread per slice
  static constexpr int DMA_B = BN * 64 / (NT * 16);
  static constexpr int DMA = DMA_A + DMA_B;                   // per thread per slice
  static_assert(DMA == 2 || DMA == 3 || DMA == 4 || DMA == 5 || DMA == 8,
                "vmcnt immediates exist for 2, 3, 4, 5 or 8 DMA per thread per slice");
  static constexpr int EROWS = BM % 128 == 0 ? (BM > 128 ? 128 : BM) : BM / 2;   // epilogue staging rows per pass
  static constexpr int CROW = BN + 4;
  static constexpr int EPI = EROWS * CROW * 4;
  static constexpr int LDS = PIPE > EPI ? PIPE : EPI;
  // blocks per CU (the 192-row tile: one, its shapes have about one tile per CU; the persistent loop needs
  // more than 256 registers for its 96 accumulators + two fragment sets)
  static constexpr int MINB = (BM % 128 != 0 || (NW >= 8 && BM * BN > 128 * 128)) ? 1
                             : (NW >= 8 && BM * BN == 128 * 128) ? DPH_MID8_MINB : (BM * BN <= 128 * 64 ? 3 : 2);
  // HIP's second __launch_bounds__ argument is the minimum number of WAVES PER SIMD (not blocks per CU):
  // MINB blocks of NW waves over the 4 SIMDs (caps the VGPRs at 512 / WPE)
  static constexpr int WPE = (MINB * NW + 3) / 4;
};
using Big = Cfg<256, 256, 128, 64>;
using Mid = Cfg<128, 128, 64, 64>;
// narrow-N shapes (the grouped positional conv: N = 48 output channels per group, M = T, K = 6144):
// 256 x 64 tile, 4 waves of 128 x 32, two blocks per CU (2 x 80 KB LDS)
using Tall = Cfg<256, 64, 128, 32>;
// N = 768 shapes with few 128x128 tiles (< 2 per CU): 128 x 64 tile, 4 waves of 64 x 32, 48 KB LDS
using Half = Cfg<128, 64, 64, 32>;
// 128 x 128 tile with 8 waves of 64 x 32 (two waves per SIMD per block): experiment
using Mid8 = Cfg<128, 128, 64, 32>;
// 256 x 128 / 128 x 256 tiles, 8 waves of 64 x 64 (16 MFMAs per wave per slice, 512 B of fragment reads
// per MFMA; half the L2->LDS bytes per flop of the 128 x 128 tile), one block per CU
using Wide = Cfg<256, 128, 64, 64>;
using Flat = Cfg<128, 256, 64, 64>;
// 192 x 128 tile, 4 waves of 96 x 64 (24 MFMAs per wave per slice, 0.42 fragment reads per MFMA): the
// M = B*T, N = 768 projections (out-proj / FFN2 forward, QKV / FFN1 / out-proj input gradients) have 189
// 128 x 256 tiles for 256 CUs (74 % of the chip busy, each CU a full 32 K-output tile); 192 x 128 gives
// 252 tiles of 24 K outputs (98 % busy, 25 % less work on the critical CU)
using Tri = Cfg<192, 128, 96, 64>;

// the ring kernel finishes a tile in the register epilogue (direct_epi: per-wave column-sum slab rows of WTM) when
// the config allows it and the args do (splits == 1 && direct_epi_ok), else in the LDS-staged one (rows of BM)
template <class C>
constexpr bool direct_cfg() {
  return DPH_DIRECT_EPI && (C::FM * C::FN <= 16 || C::NW == 4) && C::WPE <= 3;
}

// s_waitcnt vmcnt(n * DMA): at most n slices' DMAs still in flight
template <int DMA, int n>
__device__ __forceinline__ void wait_slices() {
  if constexpr (DMA * n == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (DMA * n == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if constexpr (DMA * n == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  else if constexpr (DMA * n == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (DMA * n == 9) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
  else if constexpr (DMA * n == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (DMA * n == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  else if constexpr (DMA * n == 10) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  else if constexpr (DMA * n == 15) asm volatile("s_waitcnt vmcnt(15)" ::: "memory");
  else if constexpr (DMA * n == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (DMA * n == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if constexpr (DMA * n == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if constexpr (DMA * n == 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  else static_assert(DMA * n < 0, "no vmcnt immediate");
}

template <class C>
struct Frags {
  bf16x8_t a[C::FM];
  bf16x8_t b[C::FN];
};

template <class C, bool AK, bool BK>
__device__ __forceinline__ void read_frags(Frags<C>& f, const char* slot, int wr, int wc, int lane) {
#pragma unroll
  for (int j = 0; j < C::FN; ++j)
    f.b[j] = BK ? frag(slot + C::HALF_A, wc * C::WTN + 16 * j, lane)
                : frag_mn(slot + C::HALF_A, wc * C::WTN + 16 * j, lane, C::BN * 2);
#pragma unroll
  for (int i = 0; i < C::FM; ++i)
    f.a[i] = AK ? frag(slot, wr * C::WTM + 16 * i, lane) : frag_mn(slot, wr * C::WTM + 16 * i, lane, C::BM * 2);
}

// LDS-DMA source of one 16-B chunk per lane for an operand slice.
//   k-contiguous ([rows][K]): row fixed per DMA, k advances by KS per slice (precomputed offset).
//   mn-contiguous ([K][rows]): k-row kl of the slice fixed per DMA, the operand row index
//     k = kbeg + KS*i + kl advances by KS per slice: tracked as (batch, row-in-batch) for
//     rows_per_batch layouts (rpb >= KS: at most one carry per slice); rows past kend read row
//     kend-1 (finite data; the A operand's tail rows are zeroed in LDS before use).
template <bool KC, int DMAN>
struct DmaSrc {
  int64_t off[DMAN];   // KC: element offset incl. kbeg; MN: column offset within a row
  int32_t kb[DMAN], kr[DMAN], kk[DMAN];   // MN: k-row as (batch, row in batch) and its absolute index
};

template <bool KC, int N, int NW, int R>
__device__ __forceinline__ void dma_setup(DmaSrc<KC, N>& ds, const DphMat& d, int64_t r0, int64_t Rtot, int64_t kbeg,
                                          int wave, int lane) {
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const int c = (j * NW + wave) * 64 + lane;
    if constexpr (KC) {
      const int r = c >> 2;
      ds.off[j] = row_addr(d, min(r0 + r, Rtot - 1)) + ((c & 3) ^ swz_chunk(r)) * 8 + kbeg;
    } else {
      constexpr int CPR = R / 8;                      // 16-B chunks per k-row
      const int kl = c / CPR, pc = c % CPR;
      const int lu = (pc >> 1) ^ swz(kl);
      ds.off[j] = min(r0 + lu * 16 + (pc & 1) * 8, ((Rtot + 7) & ~(int64_t)7) - 8);
      const int64_t k = kbeg + kl;
      ds.kk[j] = (int32_t)k;
      if (d.rows_per_batch > 0) {
        ds.kb[j] = (int32_t)(k / d.rows_per_batch);
        ds.kr[j] = (int32_t)(k % d.rows_per_batch);
      } else {
        ds.kb[j] = 0;
        ds.kr[j] = (int32_t)k;
      }
    }
  }
}


template <class C>
__device__ __forceinline__ void mfma_slice(f32x4_t (&acc)[C::FM][C::FN], const Frags<C>& f) {
#pragma unroll
  for (int i = 0; i < C::FM; ++i)
#pragma unroll
    for (int j = 0; j < C::FN; ++j)
      acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.b[j], f.a[i], acc[i][j], 0, 0, 0);
}


template <class C>
__device__ __forceinline__ void direct_epi(const DphGemmArgs& a, int64_t z, int64_t mw, int64_t nw, int lane,
                                           const f32x4_t (&acc)[C::FM][C::FN]) {
  const bool drop = a.dropout_p > 0.f;
  if (a.act == DPH_ACT_GELU) {
    if (drop) direct_epi_t<C, DPH_ACT_GELU, true>(a, z, mw, nw, lane, acc);
    else direct_epi_t<C, DPH_ACT_GELU, false>(a, z, mw, nw, lane, acc);
  } else if (a.act == DPH_ACT_GELU_BWD) {
    if (drop) direct_epi_t<C, DPH_ACT_GELU_BWD, true>(a, z, mw, nw, lane, acc);
    else direct_epi_t<C, DPH_ACT_GELU_BWD, false>(a, z, mw, nw, lane, acc);
  } else {
    if (drop) direct_epi_t<C, DPH_ACT_NONE, true>(a, z, mw, nw, lane, acc);
    else direct_epi_t<C, DPH_ACT_NONE, false>(a, z, mw, nw, lane, acc);
  }
}
}  // namespace ring

template <class C, bool AK, bool BK>
__global__ void __launch_bounds__(C::NT, C::WPE) ring_gemm_kernel(const DphGemmArgs a, int64_t kchunk) {
  __shared__ __attribute__((aligned(1024))) char smem[C::LDS];
#ifdef DPH_STAGGER
  // timing experiment: the second block of each CU in the first dispatch round (linear ids 256..511,
  // placed breadth-first) starts late, so co-resident blocks run out of phase
  if (C::MINB >= 2) {
    const int64_t nb = (int64_t)gridDim.x * gridDim.y * gridDim.z;
    const int64_t lb = ((int64_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
    if (nb >= 768 && lb >= 256 && lb < 512)
      for (int r = 0; r < DPH_STAGGER; ++r) __builtin_amdgcn_s_sleep(127);
  }
#endif
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wr = wave / C::WGN;
  const int wc = wave % C::WGN;

  const int64_t zz = blockIdx.z;
  const int64_t split = zz % a.splits;
  const int64_t z = zz / a.splits;
  int64_t tm, tn;
  {
    const int64_t ntm = gridDim.y, ntn = gridDim.x;
    const int64_t nt = ntm * ntn;
    const int64_t bid = (int64_t)blockIdx.y * ntn + blockIdx.x;
    const int64_t q = nt / 8, r = nt % 8;
    const int64_t xcd = bid % 8, loc = bid / 8;
    const int64_t t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
    constexpr int64_t GM = C::BM > 128 ? 4 : 8;
    const int64_t gsz = GM * ntn;
    const int64_t grp = t / gsz;
    const int64_t gm0 = grp * GM;
    const int64_t gh = min(GM, ntm - gm0);
    const int64_t l = t % gsz;
    tm = gm0 + l % gh;
    tn = l / gh;
  }
  const int64_t m0 = tm * C::BM;
  const int64_t n0 = tn * C::BN;
  const int64_t kbeg = split * kchunk;
  const int64_t kend = min(a.K, kbeg + kchunk);
  // k-slices (whole slices unless both operands are mn-contiguous: then the last one may be partial)
  const int H = DPH_ABLATE == 6 ? 0 : (int)cdiv(max<int64_t>(kend - kbeg, 0), ring::KS);
  const int ktail = (int)((kend - kbeg) - (int64_t)(H - 1) * ring::KS);   // valid k-rows of slice H-1
  unsigned long long st0 = 0, st1 = 0, st2 = 0, st3 = 0, sA = 0, sB = 0, sC = 0;
  DPH_TSTAMP(st0);

  // DMA sources: instruction j of wave w fills bytes [(j*NW+w)*1024, +1024) of the operand's slot
  // half (lane-linear), i.e. chunk c = (j*NW+w)*64 + lane.  k-contiguous: slice row c/4, physical
  // chunk c%4 <- logical chunk (c%4) ^ swz(row).  mn-contiguous: k-row c/(R/8), physical chunk
  // c%(R/8) of that k-row <- logical 32-B unit ((c%(R/8))>>1) ^ swz(k-row).
  const bf16_t* Ab = reinterpret_cast<const bf16_t*>(a.A.ptr) + z_addr(a.A, z);
  const bf16_t* Bb = reinterpret_cast<const bf16_t*>(a.B.ptr) + z_addr(a.B, z);
  ring::DmaSrc<AK, C::DMA_A> da;
  ring::DmaSrc<BK, C::DMA_B> db;
  ring::dma_setup<AK, C::DMA_A, C::NW, C::BM>(da, a.A, m0, a.M, kbeg, wave, lane);
  ring::dma_setup<BK, C::DMA_B, C::NW, C::BN>(db, a.B, n0, a.N, kbeg, wave, lane);
  const int64_t a_tail = AK ? 0 : row_addr(a.A, max<int64_t>(kend - 1, 0));
  const int64_t b_tail = BK ? 0 : row_addr(a.B, max<int64_t>(kend - 1, 0));
  // source element offset of DMA j for slice i (mn: advances the k-row state by KS)
  auto src_mn = [&](auto& ds, const DphMat& d, int64_t tail, int j) -> int64_t {
    const int64_t o = ds.kk[j] < kend ? (int64_t)ds.kb[j] * d.batch_stride + (int64_t)ds.kr[j] * d.row_stride + ds.off[j]
                                      : tail + ds.off[j];
    ds.kk[j] += ring::KS;
    ds.kr[j] += ring::KS;
    if (d.rows_per_batch > 0 && ds.kr[j] >= d.rows_per_batch) {
      ds.kr[j] -= d.rows_per_batch;
      ds.kb[j] += 1;
    }
    return o;
  };
  // DMA j of k-slice i -> slot i % 4 (j < DMA_A: operand A, else B); slices are issued in order
  auto issue_one = [&](int i, int j) {
    char* la = smem + (i & (ring::NSLOT - 1)) * C::SLOT;
    const int64_t ko = (int64_t)i * ring::KS;
    if (j < C::DMA_A) {
      ring::dma16(Ab + (AK ? da.off[j] + ko : src_mn(da, a.A, a_tail, j)), la + (j * C::NW + wave) * 1024);
    } else {
      const int jb = j - C::DMA_A;
      ring::dma16(Bb + (BK ? db.off[jb] + ko : src_mn(db, a.B, b_tail, jb)),
                  la + C::HALF_A + (jb * C::NW + wave) * 1024);
    }
  };
  auto issue = [&](int i) {
#pragma unroll
    for (int j = 0; j < C::DMA; ++j) issue_one(i, j);
  };
  // both operands mn-contiguous and K not a multiple of KS: zero the A operand's k-rows past kend in
  // the last slice (its B rows repeat row kend-1: finite, multiplied by 0).  Runs after the slice's
  // DMA landed for every wave (vmcnt(0) + barrier) and before any fragment read of it.
  auto zero_tail = [&](int i) {
    char* la = smem + (i & (ring::NSLOT - 1)) * C::SLOT;
    const int nb = (ring::KS - ktail) * C::BM * 2;
    for (int o = tid * 16; o < nb; o += C::NT * 16)
      *reinterpret_cast<uint4*>(la + ktail * C::BM * 2 + o) = make_uint4(0, 0, 0, 0);
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  const bool has_tail = !AK && ktail < ring::KS;
  auto slot = [&](int i) -> const char* { return smem + (i & (ring::NSLOT - 1)) * C::SLOT; };

  f32x4_t acc[C::FM][C::FN];
#pragma unroll
  for (int i = 0; i < C::FM; ++i)
#pragma unroll
    for (int j = 0; j < C::FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // one pipeline step: slice i is in registers (cur); wait for slice i+1, restage slot i%4 with
  // slice i+4, read slice i+1 into nxt while multiplying cur.  The step is cut into FM chunks
  // (one accumulator row of MFMAs each) and the DMAs and fragment reads are dealt over them: an
  // LDS-DMA costs its wave ~60-180 issue cycles, which hide behind the MFMAs of the chunk instead
  // of stalling the wave in front of them (measured: the loop spent ~3x its MFMA time per slice
  // with the DMAs issued as one block after the barrier).
  auto step = [&](int i, ring::Frags<C>& cur, ring::Frags<C>& nxt) {
    if (i + 3 < H) {
      ring::wait_slices<C::DMA, 2>();
    } else if (i + 2 < H) {
      ring::wait_slices<C::DMA, 1>();
    } else {
      ring::wait_slices<C::DMA, 0>();
    }
    __builtin_amdgcn_sched_barrier(0);
    if (DPH_ABLATE != 3) __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    const bool restage = i + 4 < H && DPH_ABLATE != 1;
    const bool rd = i + 1 < H && DPH_ABLATE != 4;
    if (has_tail && i + 2 == H) zero_tail(i + 1);
    const char* sn = slot(i + 1);
#pragma unroll
    for (int q = 0; q < C::FM; ++q) {
#pragma unroll
      for (int j = q; j < C::DMA; j += C::FM)
        if (restage) issue_one(i + 4, j);
      if (rd) {
        if (q < C::FN)
          nxt.b[q] = BK ? ring::frag(sn + C::HALF_A, wc * C::WTN + 16 * q, lane)
                        : ring::frag_mn(sn + C::HALF_A, wc * C::WTN + 16 * q, lane, C::BN * 2);
        nxt.a[q] = AK ? ring::frag(sn, wr * C::WTM + 16 * q, lane) : ring::frag_mn(sn, wr * C::WTM + 16 * q, lane, C::BM * 2);
      }
      if (DPH_ABLATE != 2) {
#pragma unroll
        for (int jj = 0; jj < C::FN; ++jj)
          acc[q][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur.b[jj], cur.a[q], acc[q][jj], 0, 0, 0);
      } else {
        asm volatile("" ::"v"(cur.a[q]));
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (DPH_ABLATE == 2) {
#pragma unroll
      for (int q = 0; q < C::FN; ++q) asm volatile("" ::"v"(cur.b[q]));
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): nxt landed (and slot i+1 reads retired)
    __builtin_amdgcn_sched_barrier(0);
  };
  // Steady-state step (i + 5 < H): always restages slot i%4 with slice i+4 and reads slice i+1, waits for
  // at most 2 slices in flight.  No runtime condition is left in the body, so the MFMAs, DMAs and fragment
  // reads of a slice form one basic block (the generic step's per-chunk `if`s compiled to ~25 scalar
  // compare / branch instructions per slice that split the MFMAs into blocks of FN).
  auto step_fast = [&](int i, ring::Frags<C>& cur, ring::Frags<C>& nxt) {
    ring::wait_slices<C::DMA, 2>();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    const char* sn = slot(i + 1);
#pragma unroll
    for (int q = 0; q < C::FM; ++q) {
#pragma unroll
      for (int j = q; j < C::DMA; j += C::FM) issue_one(i + 4, j);
      if (q < C::FN)
        nxt.b[q] = BK ? ring::frag(sn + C::HALF_A, wc * C::WTN + 16 * q, lane)
                      : ring::frag_mn(sn + C::HALF_A, wc * C::WTN + 16 * q, lane, C::BN * 2);
      nxt.a[q] = AK ? ring::frag(sn, wr * C::WTM + 16 * q, lane) : ring::frag_mn(sn, wr * C::WTM + 16 * q, lane, C::BM * 2);
#pragma unroll
      for (int jj = 0; jj < C::FN; ++jj)
        acc[q][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur.b[jj], cur.a[q], acc[q][jj], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_sched_barrier(0);
  };

  if (H > 0) {
#pragma unroll
    for (int i = 0; i < ring::NSLOT; ++i)
      if (i < H) issue(i);
    // slice 0: wait until at most the later slices' DMAs remain
    if (H >= 4) {
      ring::wait_slices<C::DMA, 3>();
    } else if (H == 3) {
      ring::wait_slices<C::DMA, 2>();
    } else if (H == 2) {
      ring::wait_slices<C::DMA, 1>();
    } else {
      ring::wait_slices<C::DMA, 0>();
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    ring::Frags<C> f0, f1;
    if (has_tail && H == 1) zero_tail(0);
    ring::read_frags<C, AK, BK>(f0, slot(0), wr, wc, lane);
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_sched_barrier(0);
    DPH_TSTAMP(st1);
    int i = 0;
    if (DPH_ABLATE == 0) {
      for (; i + 6 <= H; i += 2) {       // both steps of the pair have i + 5 < H
        step_fast(i, f0, f1);
        step_fast(i + 1, f1, f0);
      }
    }
    for (; i + 1 < H; i += 2) {
      step(i, f0, f1);
      step(i + 1, f1, f0);
    }
    if (i < H) step(i, f0, f1);
  }
  DPH_TSTAMP(st2);

  if (DPH_ABLATE == 5) {   // timing ablation: no epilogue (accumulators kept live)
#pragma unroll
    for (int i = 0; i < C::FM; ++i)
#pragma unroll
      for (int j = 0; j < C::FN; ++j) asm volatile("" ::"v"(acc[i][j]));
    return;
  }
  // ---- epilogue: straight from the accumulators when the layout allows ----
  auto write_stamps = [&]() {
    __syncthreads();
    DPH_TSTAMP(st3);
    if (tid == 0) {
      unsigned hw, xcc;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
      unsigned long long* o = reinterpret_cast<unsigned long long*>(a.workspace) +
                              16 * ((int64_t)blockIdx.y * gridDim.x + blockIdx.x);
      o[0] = st0; o[1] = st1; o[2] = st2; o[3] = st3; o[4] = hw; o[5] = xcc; o[6] = sA; o[7] = sB; o[8] = sC;
    }
  };
  // (not the 256 x 256 tile: its 128 accumulators leave no room for the epilogue inputs; not the 8-wave
  // 128 x 128 tile: at 4 waves per SIMD its 128-VGPR budget spilled 50 registers)
  if constexpr (ring::direct_cfg<C>()) {
    if (a.splits == 1 && ring::direct_epi_ok(a)) {
      DPH_TSTAMP(sA);
      sB = sA;
#ifdef DPH_EPI_TWICE
      ring::direct_epi<C>(a, z, m0 + wr * C::WTM, n0 + wc * C::WTN, lane, acc);   // timing: cold, then warm code
      DPH_TSTAMP(sB);
#endif
      ring::direct_epi<C>(a, z, m0 + wr * C::WTM, n0 + wc * C::WTN, lane, acc);
      DPH_TSTAMP(sC);
      if (DPH_STAMP) write_stamps();
      return;
    }
  }
  // ---- staged epilogue, EROWS rows at a time: accumulators -> LDS fp32 -> row-contiguous ----
  constexpr int TPR = C::BN / 8;              // threads per output row (8 columns each)
  constexpr int RPP = C::NT / TPR;            // rows per pass
  float* ct = reinterpret_cast<float*>(smem);
  const int c8 = (tid % TPR) * 8;
  const int r0 = tid / TPR;
  float cso[8], csa[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    cso[q] = 0.f;
    csa[q] = 0.f;
  }
  // Pass h stages accumulator rows i in [h*FMH, (h+1)*FMH) of every wave, so the registers of
  // the staged rows die before the next pass (the Big tile cannot hold its 128 accumulator VGPRs
  // and the epilogue's prefetched inputs at once).  LDS row r holds tile row
  // (r / SEG) * WTM + h * SEG + r % SEG.
  constexpr int NPASS = C::BM / C::EROWS;
  constexpr int FMH = C::FM / NPASS;
  constexpr int SEG = C::WTM / NPASS;
  constexpr int JP = SEG / RPP;                // passes p per SEG run of rows
  static_assert(SEG % RPP == 0 && C::FM % NPASS == 0, "epilogue row map");
  auto trow = [&](int h, int r) { return (r / SEG) * C::WTM + h * SEG + r % SEG; };
#pragma unroll
  for (int h = 0; h < NPASS; ++h) {
    __syncthreads();
    if (h == 0) DPH_TSTAMP(sA);
#pragma unroll
    for (int ii = 0; ii < FMH; ++ii) {
      const int i = h * FMH + ii;
      const int r = wr * SEG + 16 * ii + (lane & 15);
#pragma unroll
      for (int j = 0; j < C::FN; ++j) {
        const int c = wc * C::WTN + 16 * j + 4 * (lane >> 4);
        *reinterpret_cast<float4*>(ct + r * C::CROW + c) =
            make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
      }
    }
    __syncthreads();
    if (h == 0) DPH_TSTAMP(sB);
    if (a.splits > 1) {
      float* ws = reinterpret_cast<float*>(a.workspace) + (zz * a.M) * a.N;
#pragma unroll 2
      for (int p = 0; p < C::EROWS / RPP; ++p) {
        const int r = r0 + RPP * p;
        const int64_t m = m0 + trow(h, r);
        const int64_t n = n0 + c8;
        if (m >= a.M || n >= a.N) continue;
        const float* src = ct + r * C::CROW + c8;
        float* dst = ws + m * a.N + n;
        if (n + 8 <= a.N && (a.N & 3) == 0) {
          *reinterpret_cast<float4*>(dst) = *reinterpret_cast<const float4*>(src);
          *reinterpret_cast<float4*>(dst + 4) = *reinterpret_cast<const float4*>(src + 4);
        } else {
          for (int q = 0; q < 8 && n + q < a.N; ++q) dst[q] = src[q];
        }
      }
      continue;
    }
    // (the 8-wave Big tile keeps the per-row epilogue: the prefetching one pushes its main loop into
    // scratch spills at the 256-VGPR cap)
    if constexpr (C::NW < 8 || C::FM * C::FN <= 16) {
      if (tile_epi_ok(a, n0 + c8)) {
        tile_epi<C::EROWS / RPP, RPP, JP, C::WTM - SEG>(a, z, m0 + trow(h, r0), n0 + c8, ct + r0 * C::CROW + c8,
                                                        C::CROW, cso, csa);
        if (h == 0) DPH_TSTAMP(sC);
        continue;
      }
    }
#pragma unroll 1
    for (int p = 0; p < C::EROWS / RPP; ++p) {
      const int r = r0 + RPP * p;
      const float* src = ct + r * C::CROW + c8;
      float v[8];
      const float4 x0 = *reinterpret_cast<const float4*>(src);
      const float4 x1 = *reinterpret_cast<const float4*>(src + 4);
      v[0] = x0.x; v[1] = x0.y; v[2] = x0.z; v[3] = x0.w;
      v[4] = x1.x; v[5] = x1.y; v[6] = x1.z; v[7] = x1.w;
      Cs8 cs;
      epilogue8(a, z, m0 + trow(h, r), n0 + c8, v, cs);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        cso[q] += cs.out[q];
        csa[q] += cs.aux[q];
      }
    }
  }
  if (DPH_STAMP) {
    write_stamps();
    return;
  }
  if (a.splits == 1 && ((a.colsum_out != nullptr) || (a.colsum_aux != nullptr))) {
    // lanes sharing columns inside a wave (lane ^ TPR, ...), then the waves through LDS
#pragma unroll
    for (int q = 0; q < 8; ++q) {
#pragma unroll
      for (int o = TPR; o < 64; o <<= 1) {
        cso[q] += __shfl_xor(cso[q], o, 64);
        csa[q] += __shfl_xor(csa[q], o, 64);
      }
    }
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);   // [NW][2][BN]
    if (lane < TPR) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        red[(wave * 2 + 0) * C::BN + c8 + q] = cso[q];
        red[(wave * 2 + 1) * C::BN + c8 + q] = csa[q];
      }
    }
    __syncthreads();
    if (tid < C::BN) {
      const int64_t n = n0 + tid;
      if (n < a.N) {
        const int64_t voff = (a.C.z_div > 0 ? (z % a.C.z_div) : z) * a.vec_z_inner;
        const int64_t csn = a.colsum_n > 0 ? a.colsum_n : a.N;
        float so = 0.f, sx = 0.f;
#pragma unroll
        for (int w = 0; w < C::NW; ++w) {
          so += red[(w * 2 + 0) * C::BN + tid];
          sx += red[(w * 2 + 1) * C::BN + tid];
        }
        if (a.flags & GEMM_COLSUM_SLAB) {
          // one slab row per BM-row M tile and grid batch (summed in a fixed order by colsum_slab_reduce_kernel)
          const int64_t ns = cdiv(a.M, (int64_t)C::BM);
          float* wo = reinterpret_cast<float*>(a.workspace) + (z * ns + m0 / C::BM) * a.N;
          if (n < csn) {
            wo[n] = so;
            wo[a.batch * ns * a.N + n] = sx;
          }
        } else {
          if (a.colsum_out && n < csn) atomicAdd(a.colsum_out + voff + n, so);
          if (a.colsum_aux && n < csn) atomicAdd(a.colsum_aux + voff + n, sx);
        }
      }
    }
  }
}

// =============================================================================================
// Persistent ring kernel: gridDim.x blocks (the CU slots) walk the tiles t = blockIdx.x + k*gridDim.x;
// the k-slices of a block's consecutive tiles form ONE stream through the 4-slot ring, so the first
// slices of tile k+1 are staged while tile k's last slices are multiplied and while its (direct,
// register-only) epilogue runs: no per-tile pipeline fill (~4-5k cycles measured per 128 x 256 tile)
// and no per-tile block launch.  The per-step schedule, counted waits and slot reuse are the ring
// kernel's; the DMA source pointers switch to the next tile when the issue side crosses into it.
// Both operands k-contiguous, K % 64 == 0 (an even slice count per tile keeps the two fragment
// register sets in phase across tiles), splits == 1, direct-epilogue layouts.  Epilogue stores count in
// vmcnt, which only makes the next steps' counted waits stricter (never looser).
// =============================================================================================
template <class C, int ACT, bool DROP>
__global__ void __launch_bounds__(C::NT, C::WPE) ring_persist_kernel(const DphGemmArgs a, int64_t ntm, int64_t ntn) {
  __shared__ __attribute__((aligned(1024))) char smem[C::PIPE];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wr = wave / C::WGN;
  const int wc = wave % C::WGN;
  const int64_t nt = ntm * ntn;
  const int64_t G = gridDim.x;
  const int64_t ntiles = (nt * a.batch - blockIdx.x + G - 1) / G;
  const int H = (int)(a.K / ring::KS);
  const int64_t S = ntiles * (int64_t)H;
  // tile k of this block -> (z, m0, n0): the ring kernel's XCD-grouped, GM-swizzled order over the
  // virtual block id v (gridDim.x % 8 == 0 or a single round, so v % 8 is this block's XCD)
  // (32-bit arithmetic: tile counts < 2^31, checked on the host; 64-bit divisions cost ~40 instructions
  // and their registers each)
  const uint32_t nt32 = (uint32_t)nt, ntm32 = (uint32_t)ntm, ntn32 = (uint32_t)ntn;
  auto tile_of = [&](int64_t k, int64_t& z, int64_t& m0, int64_t& n0) {
    const uint32_t v = (uint32_t)blockIdx.x + (uint32_t)k * (uint32_t)G;
    const uint32_t zz = v / nt32;
    const uint32_t bid = v - zz * nt32;
    const uint32_t q = nt32 >> 3, r = nt32 & 7;
    const uint32_t xcd = bid & 7, loc = bid >> 3;
    const uint32_t t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
    constexpr uint32_t GM = C::BM > 128 ? 4 : 8;
    const uint32_t gsz = GM * ntn32;
    const uint32_t grp = t / gsz;
    const uint32_t gm0 = grp * GM;
    const uint32_t gh = min(GM, ntm32 - gm0);
    const uint32_t l = t - grp * gsz;
    const uint32_t lq = l / gh;
    z = zz;
    m0 = (int64_t)(gm0 + (l - lq * gh)) * C::BM;
    n0 = (int64_t)lq * C::BN;
  };
  // issue side: DMA sources of the tile being staged (4 slices ahead of the one being multiplied; it
  // switches to tile k+1 when tile k's slice H-4 is multiplied)
  const bf16_t* pa[C::DMA_A];
  const bf16_t* pb[C::DMA_B];
  auto setup = [&](int64_t k) {
    int64_t z, m0, n0;
    tile_of(k, z, m0, n0);
    const bf16_t* Ab = reinterpret_cast<const bf16_t*>(a.A.ptr) + z_addr(a.A, z);
    const bf16_t* Bb = reinterpret_cast<const bf16_t*>(a.B.ptr) + z_addr(a.B, z);
#pragma unroll
    for (int j = 0; j < C::DMA_A; ++j) {
      const int c = (j * C::NW + wave) * 64 + lane;
      const int r = c >> 2;
      pa[j] = Ab + row_addr32(a.A, (uint32_t)min(m0 + r, a.M - 1)) + ((c & 3) ^ ring::swz_chunk(r)) * 8;
    }
#pragma unroll
    for (int j = 0; j < C::DMA_B; ++j) {
      const int c = (j * C::NW + wave) * 64 + lane;
      const int r = c >> 2;
      pb[j] = Bb + row_addr32(a.B, (uint32_t)min(n0 + r, a.N - 1)) + ((c & 3) ^ ring::swz_chunk(r)) * 8;
    }
  };
  setup(0);
  // DMA j of stream slice g = slice `is` of the tile being staged
  auto issue_one = [&](int64_t g, int is, int j) {
    char* la = smem + (g & (ring::NSLOT - 1)) * C::SLOT;
    const int64_t ko = (int64_t)is * ring::KS;
    if (j < C::DMA_A) ring::dma16(pa[j] + ko, la + (j * C::NW + wave) * 1024);
    else ring::dma16(pb[j - C::DMA_A] + ko, la + C::HALF_A + ((j - C::DMA_A) * C::NW + wave) * 1024);
  };
  auto slot = [&](int64_t g) -> const char* { return smem + (g & (ring::NSLOT - 1)) * C::SLOT; };

  f32x4_t acc[C::FM][C::FN];
#pragma unroll
  for (int i = 0; i < C::FM; ++i)
#pragma unroll
    for (int j = 0; j < C::FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  auto step = [&](int64_t g, int is, ring::Frags<C>& cur, ring::Frags<C>& nxt) {
    if (g + 3 < S) {
      ring::wait_slices<C::DMA, 2>();
    } else if (g + 2 < S) {
      ring::wait_slices<C::DMA, 1>();
    } else {
      ring::wait_slices<C::DMA, 0>();
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    const bool restage = g + 4 < S;
    const bool rd = g + 1 < S;
    const char* sn = slot(g + 1);
#pragma unroll
    for (int q = 0; q < C::FM; ++q) {
#pragma unroll
      for (int j = q; j < C::DMA; j += C::FM)
        if (restage) issue_one(g + 4, is, j);
      if (rd) {
        if (q < C::FN) nxt.b[q] = ring::frag(sn + C::HALF_A, wc * C::WTN + 16 * q, lane);
        nxt.a[q] = ring::frag(sn, wr * C::WTM + 16 * q, lane);
      }
#pragma unroll
      for (int jj = 0; jj < C::FN; ++jj)
        acc[q][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur.b[jj], cur.a[q], acc[q][jj], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_sched_barrier(0);
  };
  // After a lean epilogue the wave has FM*FN (or 2*FM*FN) stores outstanding, issued after the DMAs of the
  // next tile's slices 0..2 and before those of slice 3 on: the first three steps of the tile then wait
  // for vmcnt(2*DMA + FM*FN) instead of vmcnt(2*DMA), so the stores drain under those steps' MFMAs
  // instead of being waited for by the first one (vmcnt retires in order: this still waits for the DMA
  // the step needs, and at most for the older half of the stores when pre_out doubles them).
  constexpr int VM_EXTRA = 2 * C::DMA + C::FM * C::FN;
  static_assert(VM_EXTRA < 64, "vmcnt immediate");
  constexpr int WAIT_EXTRA = (VM_EXTRA & 15) | ((VM_EXTRA >> 4) << 14) | 0x70 | 0xF00;
  auto step_fast = [&](int64_t g, int is, ring::Frags<C>& cur, ring::Frags<C>& nxt, bool extra) {
    if (extra) __builtin_amdgcn_s_waitcnt(WAIT_EXTRA);
    else ring::wait_slices<C::DMA, 2>();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    const char* sn = slot(g + 1);
#pragma unroll
    for (int q = 0; q < C::FM; ++q) {
#pragma unroll
      for (int j = q; j < C::DMA; j += C::FM) issue_one(g + 4, is, j);
      if (q < C::FN) nxt.b[q] = ring::frag(sn + C::HALF_A, wc * C::WTN + 16 * q, lane);
      nxt.a[q] = ring::frag(sn, wr * C::WTM + 16 * q, lane);
#pragma unroll
      for (int jj = 0; jj < C::FN; ++jj)
        acc[q][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur.b[jj], cur.a[q], acc[q][jj], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_sched_barrier(0);
  };

  // prologue: stream slices 0..3, wait for slice 0
#pragma unroll
  for (int g = 0; g < ring::NSLOT; ++g)
    if (g < S) {
#pragma unroll
      for (int j = 0; j < C::DMA; ++j) issue_one(g, g, j);
    }
  if (S >= 4) {
    ring::wait_slices<C::DMA, 3>();
  } else if (S == 3) {
    ring::wait_slices<C::DMA, 2>();
  } else if (S == 2) {
    ring::wait_slices<C::DMA, 1>();
  } else {
    ring::wait_slices<C::DMA, 0>();
  }
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  ring::Frags<C> f0, f1;
  ring::read_frags<C, true, true>(f0, slot(0), wr, wc, lane);
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_sched_barrier(0);
  int64_t g = 0;
  bool after_lean = false;
#pragma unroll 1
  for (int64_t k = 0; k < ntiles; ++k) {
    const bool last = k + 1 == ntiles;
    // every pair restages two slices except the stream's last two pairs (generic steps: the counted
    // waits drain and nothing is staged past the end; kept out of the pair loop, whose register
    // allocation they otherwise spoil: 33 spilled VGPRs with them inside, none without)
    const int ifast = last ? H - 4 : H;
#pragma unroll 1
    for (int i = 0; i < ifast; i += 2, g += 2) {
      // slices i+4, i+5 of this tile, or (from i = H-4 on) slices i+4-H, i+5-H of the next one
      int is = i + 4;
      if (is >= H) {
        is -= H;
        if (is == 0) setup(k + 1);
      }
      step_fast(g, is, f0, f1, after_lean && i < 3);
      step_fast(g + 1, is + 1, f1, f0, after_lean && i + 1 < 3);
    }
    if (last) {
      step(g, 0, f0, f1);
      step(g + 1, 0, f1, f0);
      step(g + 2, 0, f0, f1);
      step(g + 3, 0, f1, f0);
      g += 4;
    }
    int64_t z, m0, n0;
    tile_of(k, z, m0, n0);
    // (one epilogue variant per kernel: the activation / dropout dispatch happens on the host -- all six
    // inlined into the tile loop spilled ~1000 VGPRs)
    after_lean = ring::direct_epi_t<C, ACT, DROP>(a, z, m0 + wr * C::WTM, n0 + wc * C::WTN, lane, acc);
#pragma unroll
    for (int i = 0; i < C::FM; ++i)
#pragma unroll
      for (int j = 0; j < C::FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  }
}

// =============================================================================================
// Ping-pong GEMM (both operands k-contiguous, K % 64 == 0, direct-epilogue layouts).
//
// 8 waves = two groups of four (wr = 0 / 1; waves w and w + 4 share a SIMD) that run the SAME phase
// program one barrier interval apart: in every interval one wave of each SIMD multiplies (an MFMA
// cluster between two barriers) while its partner issues the LDS fragment reads and LDS-DMA stages of
// its next phase, so the matrix core and the LDS / memory pipes work at once (the guide's 256^2 8-phase
// structure, cdna_hip_programming.md §5; the ring kernels above run one barrier per 32-deep slice with
// every wave in the same role, and their main loop measured 1.5-1.6x the MFMA time).
//
// Geometry: BM x BN tile, 64-deep K-tiles, waves 2 (M) x 4 (N), each a (BM/2) x (BN/4) output of FM x FN
// 16x16 accumulators.  A K-tile is staged as four HALF-TILES with their own lifetimes:
//   A-lo: the first FM/2 fragment rows of both wave rows   (BM/2 rows)
//   A-hi: the last FM/2                                     (BM/2 rows)
//   B-n0: the first ceil(FN/2) fragment columns of every wave column, B-n1: the rest
// Phase j of K-tile u (buffer u & 1) reads / multiplies:
//   j=0: read A-lo, B-n0 -> MFMA A-lo x B-n0      j=1: read B-n1 -> A-lo x B-n1
//   j=2: read A-hi       -> A-hi x B-n1           j=3: (no reads)  A-hi x B-n0 (B-n0 kept since j=0)
// and issues ONE half-tile: j=0 B-n1(u+1), j=1 A-hi(u+1), j=2 A-lo(u+2), j=3 B-n0(u+2) (Cfg::B0PF: j=2 B-n0(u+2),
// j=3 A-lo(u+2), and B-n0(u+1) read in j=3 into a second register set instead of at j=0 of u+1).  With the two
// groups one interval apart, a stage may overwrite a half-tile two phases after its last read (WAR) and a
// half-tile may be read one phase after the wait that retires it (RAW); the issue order above gives every
// half-tile exactly that and keeps four half-tiles (G DMAs per thread = one K-tile) in flight across the
// barriers: each phase waits vmcnt(G), never 0 in the steady state.
// LDS: two K-tile buffers, each half-tile rows of 128 B whose 16-B chunk p holds k-chunk p ^ ((r>>1)&7)
// (the swizzle goes on the DMA SOURCE address: LDS-DMA writes lane-linear), conflict-free ds_read_b128.
// =============================================================================================
namespace pp {

template <class C, int ACT, bool DROP>
__global__ void __launch_bounds__(C::NT, C::WPE) pp_gemm_kernel(const DphGemmArgs a) {
  __shared__ __attribute__((aligned(1024))) char smem[C::LDS];
  unsigned long long st0 = 0, st1 = 0, st2 = 0, st3 = 0;
  (void)st0; (void)st1; (void)st2; (void)st3;
  DPH_TSTAMP(st0);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  // tile: the ring kernel's XCD-grouped order (blocks b, b+8, ... share an XCD and get neighbouring tiles)
  const int64_t z = blockIdx.z;
  int64_t m0, n0;
  {
    const uint32_t ntm = gridDim.y, ntn = gridDim.x, nt = ntm * ntn;
    const uint32_t bid = blockIdx.y * ntn + blockIdx.x;
    const uint32_t q = nt >> 3, r = nt & 7;
    const uint32_t xcd = bid & 7, loc = bid >> 3;
    const uint32_t t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
    constexpr uint32_t GM = C::BM > 128 ? 4 : 8;
    const uint32_t gsz = GM * ntn;
    const uint32_t grp = t / gsz;
    const uint32_t gm0 = grp * GM;
    const uint32_t gh = min(GM, ntm - gm0);
    const uint32_t l = t - grp * gsz;
    const uint32_t lq = l / gh;
    m0 = (int64_t)(gm0 + (l - lq * gh)) * C::BM;
    n0 = (int64_t)lq * C::BN;
  }
  int nk = (int)(a.K / BK);
  if (a.dyn_ext != nullptr) {
    // device-side extents (packed FFN units): whole blocks past m / n return before any barrier, the K loop
    // stops at k (a multiple of 64, >= 128)
    const int em = __builtin_amdgcn_readfirstlane(a.dyn_ext[0]), en = __builtin_amdgcn_readfirstlane(a.dyn_ext[1]);
    const int ek = __builtin_amdgcn_readfirstlane(a.dyn_ext[2]);
    if ((em > 0 && m0 >= em) || (en > 0 && n0 >= en)) return;
    if (ek > 0 && ek < a.K) nk = ek / BK;
  }
  const bf16_t* Ab = reinterpret_cast<const bf16_t*>(a.A.ptr) + z_addr(a.A, z);
  const bf16_t* Bb = reinterpret_cast<const bf16_t*>(a.B.ptr) + z_addr(a.B, z);
  f32x4_t acc[C::FM][C::FN];
#pragma unroll
  for (int i = 0; i < C::FM; ++i)
#pragma unroll
    for (int j = 0; j < C::FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  mainloop<C>(a, Ab, Bb, m0, n0, nk, acc, smem, wave, lane, st1);
  DPH_TSTAMP(st2);
  ring::direct_epi_t<C, ACT, DROP, true>(a, z, m0 + wr * C::WTM, n0 + wc * C::WTN, lane, acc);
  if (DPH_STAMP) {
    // diagnostic build only (tools/stamp_pp.py): per-block stamps into the workspace, written by lane 0 of wave 0
    __syncthreads();
    DPH_TSTAMP(st3);
    if (tid == 0) {
      unsigned hw, xcc;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
      unsigned long long* o = reinterpret_cast<unsigned long long*>(a.workspace) +
                              8 * ((int64_t)blockIdx.y * gridDim.x + blockIdx.x);
      o[0] = st0; o[1] = st1; o[2] = st2; o[3] = st3; o[4] = hw; o[5] = xcc;
    }
  }
}
}  // namespace pp

// =============================================================================================
// Ping-pong weight-gradient kernel: both operands mn-contiguous (A = [K][M], B = [K][N], K = the B*T frames
// of the batch), split-K over blockIdx.z.  dW = dY^T X of every nn.Linear / conv layer (components.py:107,
// :272, :406-408, :430, :733, :741; lightning.py:258) without transposing an activation: the LDS-DMA stages
// each half-tile as a [64 k][R] image (R = 64 or 128 operand rows, 16-B chunk c of k-row r at c ^ fsw(r)),
// and the MFMA fragments come out of it by ds_read_b64_tr_b16 (two per 16 x 32 fragment; the swizzle puts
// the 8 k-rows x 2 chunks of a half-wave's transposed read on 16 distinct 4-bank groups).  Same 8-wave
// schedule as pp_gemm_kernel (two groups one barrier interval apart, four half-tiles per 64-deep K-tile).
//   * K tail: DMA rows past kend re-read row kend - 1 (finite), the A fragments of the last K-tile zero
//     their k >= kend elements before the MFMAs;
//   * BB: B rows in the batched layout (conv weight gradients: row k = output frame, windows of stride s*C
//     inside each utterance) -- one carry per 64-row tile (rows_per_batch >= 64);
//   * splits > 1: dph_gemm passes epilogue args whose C is the fp32 workspace slab (z = batch * splits +
//     split), summed into dW by splitk_reduce_kernel.
// =============================================================================================
namespace ppw {
using pp::BK;

template <int R>
__device__ __forceinline__ int fsw(int r) { return (2 * ((r >> 1) & 1) + 4 * ((r >> 3) & 1) + 8 * (r & 1)) & (R / 8 - 1); }

// byte offset (k-row 0 .. 3 of the lane's first transposed read, ksub 0) of the fragment with operand rows
// cb .. cb + 15 (cb % 16 == 0) in a [64][R] half-tile image; ksub s adds 64 R bytes, the second read 8 R
template <int R>
__device__ __forceinline__ int tfrag_off(int cb, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int k0 = 8 * g + q;
  const int c = (cb >> 3) + (p >> 1);
  return k0 * (2 * R) + ((c ^ fsw<R>(k0)) << 4) + ((p & 1) << 3);
}

template <int R>
__device__ __forceinline__ bf16x8_t tfrag(const char* ht, int off, int s) {
  typedef __attribute__((address_space(3))) s16x4_t lds_s16x4;
  const char* p0 = ht + off + s * 64 * R;
  const s16x4_t v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p0);
  const s16x4_t v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p0 + 8 * R));
  const s16x8_t v = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
  return __builtin_bit_cast(bf16x8_t, v);
}

// zero the elements k >= n of a lane's 8 consecutive k values (n <= 0: all, n >= 8: none)
__device__ __forceinline__ bf16x8_t kmask(bf16x8_t f, int n) {
  uint4 w = __builtin_bit_cast(uint4, f);
  auto m = [&](int e) -> uint32_t { return n >= e + 2 ? 0xffffffffu : (n == e + 1 ? 0x0000ffffu : 0u); };
  w.x &= m(0);
  w.y &= m(2);
  w.z &= m(4);
  w.w &= m(6);
  return __builtin_bit_cast(bf16x8_t, w);
}

template <class C, bool BB>
__global__ void __launch_bounds__(C::NT, C::WPE) ppw_gemm_kernel(const DphGemmArgs a, int64_t kchunk,
                                                                 const DphGemmGroup grp) {
  __shared__ __attribute__((aligned(1024))) char smem[C::LDS];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  int64_t zz = blockIdx.z;
  int64_t m0, n0;
  {
    const uint32_t ntm = gridDim.y, ntn = gridDim.x, nt = ntm * ntn;
    // blocks reach the XCDs round-robin in dispatch order (x fastest, then y, then z); logical tile t = the
    // block's rank inside its XCD's contiguous share, over one z plane or (ZMAP) over all of them
    const bool zmap = (a.flags & GEMM_PPW_ZMAP) != 0;
    const uint32_t total = zmap ? nt * gridDim.z : nt;
    const uint32_t bid = (zmap ? blockIdx.z * nt : 0u) + blockIdx.y * ntn + blockIdx.x;
    const uint32_t q = total >> 3, r = total & 7;
    const uint32_t xcd = bid & 7, loc = bid >> 3;
    uint32_t t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
    if (zmap) {
      zz = t / nt;
      t -= (uint32_t)zz * nt;
    }
    constexpr uint32_t GM = C::BM > 128 ? 4 : 8;
    const uint32_t gsz = GM * ntn;
    const uint32_t grp = t / gsz;
    const uint32_t gm0 = grp * GM;
    const uint32_t gh = min(GM, ntm - gm0);
    const uint32_t l = t - grp * gsz;
    const uint32_t lq = l / gh;
    m0 = (int64_t)(gm0 + (l - lq * gh)) * C::BM;
    n0 = (int64_t)lq * C::BN;
  }
  zz = __builtin_amdgcn_readfirstlane((int)zz);
  const int64_t z = zz / a.splits;
  const int64_t split = zz - z * a.splits;
  if (a.dyn_ext != nullptr) {   // device-side extents: blocks past m / n return at once (packed FFN units)
    const int em = __builtin_amdgcn_readfirstlane(a.dyn_ext[0]), en = __builtin_amdgcn_readfirstlane(a.dyn_ext[1]);
    if ((em > 0 && m0 >= em) || (en > 0 && n0 >= en)) return;
  }
  const int32_t kbeg = (int32_t)(split * kchunk);
  const int32_t kend = (int32_t)min<int64_t>(a.K, kbeg + kchunk);
  const int nk = (kend - kbeg + BK - 1) / BK;
  // (grouped launch: problem z's operands; the host zeroed their z offsets)
  const bf16_t* Ab = reinterpret_cast<const bf16_t*>(grp.n ? grp.a[z] : a.A.ptr) + z_addr(a.A, z);
  const bf16_t* Bb = reinterpret_cast<const bf16_t*>(grp.n ? grp.b[z] : a.B.ptr) + z_addr(a.B, z);
  const uint32_t rsa = (uint32_t)a.A.row_stride, rsb = (uint32_t)a.B.row_stride;
  // DMA of a [64][R] half-tile: wave instruction gi = jj * 8 + wave fills k-rows gi * (512 / R) ..; lane ->
  // k-row gi * (512 / R) + lane / (R / 8), physical chunk lane % (R / 8) <- logical chunk pc ^ fsw(k-row),
  // i.e. operand rows (columns of the image) 8 lc .. 8 lc + 7, mapped to the tile by the half-tile kind
  constexpr int HA = C::WTM / 2;
  const int64_t mpad = ((a.M + 7) & ~(int64_t)7) - 8, npad = ((a.N + 7) & ~(int64_t)7) - 8;
  uint32_t cal[C::GA], cah[C::GA], cb0[C::GB0], cb1[C::GB1];   // column (operand row) offsets
  uint8_t kal[C::GA], kb0[C::GB0], kb1[C::GB1];                // k-row within the tile
  auto krow_of = [&](int jj, int R) { return (jj * 8 + wave) * (512 / R) + lane / (R / 8); };
#pragma unroll
  for (int jj = 0; jj < C::GA; ++jj) {
    constexpr int R = C::RA;
    const int kr = krow_of(jj, R);
    const int rho = (((lane % (R / 8)) ^ fsw<R>(kr)) * 8);
    const int trow = (rho / HA) * C::WTM + rho % HA;
    kal[jj] = (uint8_t)kr;
    cal[jj] = (uint32_t)min<int64_t>(m0 + trow, mpad);
    cah[jj] = (uint32_t)min<int64_t>(m0 + trow + HA, mpad);
  }
#pragma unroll
  for (int jj = 0; jj < C::GB0; ++jj) {
    constexpr int R = C::RB0;
    const int kr = krow_of(jj, R);
    const int rho = (((lane % (R / 8)) ^ fsw<R>(kr)) * 8);
    const int tcol = (rho / (16 * C::FN0)) * C::WTN + rho % (16 * C::FN0);
    kb0[jj] = (uint8_t)kr;
    cb0[jj] = (uint32_t)min<int64_t>(n0 + tcol, npad);
  }
#pragma unroll
  for (int jj = 0; jj < C::GB1; ++jj) {
    constexpr int R = C::RB1;
    const int kr = krow_of(jj, R);
    const int rho = (((lane % (R / 8)) ^ fsw<R>(kr)) * 8);
    const int tcol = (rho / (16 * C::FN1)) * C::WTN + 16 * C::FN0 + rho % (16 * C::FN1);
    kb1[jj] = (uint8_t)kr;
    cb1[jj] = (uint32_t)min<int64_t>(n0 + tcol, npad);
  }
  // B rows in the batched layout: (utterance, frame) of each kind's next K-tile start, one carry per tile
  const uint32_t rpb = BB ? (uint32_t)a.B.rows_per_batch : 0u;
  const uint32_t bsb = BB ? (uint32_t)a.B.batch_stride : 0u;
  uint32_t bq[2] = {0u, 0u}, br[2] = {0u, 0u};
  uint32_t blast = 0u;
  if constexpr (BB) {
    bq[0] = bq[1] = (uint32_t)kbeg / rpb;
    br[0] = br[1] = (uint32_t)kbeg - bq[0] * rpb;
    const uint32_t kl = (uint32_t)kend - 1u, ql = kl / rpb;
    blast = ql * bsb + (kl - ql * rpb) * rsb;
  }
  auto a_off = [&](int kt, int kr, uint32_t col) -> uint32_t {
    return __umul24((uint32_t)min(kt + kr, kend - 1), rsa) + col;   // (k, row stride < 2^24: checked on the host)
  };
  auto b_off = [&](int kt, int kr, uint32_t col, int kind) -> uint32_t {
    if constexpr (BB) {
      uint32_t r = br[kind] + (uint32_t)kr;
      uint32_t off = bq[kind] * bsb;
      if (r >= rpb) {
        r -= rpb;
        off += bsb;
      }
      off += __umul24(r, rsb) + col;
      return kt + kr < kend ? off : blast + col;
    } else {
      return __umul24((uint32_t)min(kt + kr, kend - 1), rsb) + col;
    }
  };
  auto b_adv = [&](int kind) {
    if constexpr (BB) {
      br[kind] += BK;
      if (br[kind] >= rpb) {
        br[kind] -= rpb;
        ++bq[kind];
      }
    }
  };
  auto buf = [&](int u) -> char* { return smem + (u & 1) * C::BUF; };
  auto st_alo = [&](int u) {
    const int kt = kbeg + u * BK;
#pragma unroll
    for (int jj = 0; jj < C::GA; ++jj) ring::dma16(Ab + a_off(kt, kal[jj], cal[jj]), buf(u) + C::O_ALO + (jj * 8 + wave) * 1024);
  };
  auto st_ahi = [&](int u) {
    const int kt = kbeg + u * BK;
#pragma unroll
    for (int jj = 0; jj < C::GA; ++jj) ring::dma16(Ab + a_off(kt, kal[jj], cah[jj]), buf(u) + C::O_AHI + (jj * 8 + wave) * 1024);
  };
  auto st_b0 = [&](int u) {
    const int kt = kbeg + u * BK;
#pragma unroll
    for (int jj = 0; jj < C::GB0; ++jj) ring::dma16(Bb + b_off(kt, kb0[jj], cb0[jj], 0), buf(u) + C::O_B0 + (jj * 8 + wave) * 1024);
    b_adv(0);
  };
  auto st_b1 = [&](int u) {
    const int kt = kbeg + u * BK;
#pragma unroll
    for (int jj = 0; jj < C::GB1; ++jj) ring::dma16(Bb + b_off(kt, kb1[jj], cb1[jj], 1), buf(u) + C::O_B1 + (jj * 8 + wave) * 1024);
    b_adv(1);
  };

  f32x4_t acc[C::FM][C::FN];
#pragma unroll
  for (int i = 0; i < C::FM; ++i)
#pragma unroll
    for (int j = 0; j < C::FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  bf16x8_t fa[C::FM2][2], fb0[C::FN0][2], fb1[C::FN1][2];
  // fragment byte offsets inside their half-tile images (loop invariant)
  int oa[C::FM2], ob0[C::FN0], ob1[C::FN1];
#pragma unroll
  for (int i = 0; i < C::FM2; ++i) oa[i] = tfrag_off<C::RA>(wr * HA + 16 * i, lane);
#pragma unroll
  for (int j = 0; j < C::FN0; ++j) ob0[j] = tfrag_off<C::RB0>(wc * 16 * C::FN0 + 16 * j, lane);
#pragma unroll
  for (int j = 0; j < C::FN1; ++j) ob1[j] = tfrag_off<C::RB1>(wc * 16 * C::FN1 + 16 * j, lane);

  auto rd_a = [&](const char* ht) {
    if (PP_ABL_READ) return;
#pragma unroll
    for (int i = 0; i < C::FM2; ++i)
#pragma unroll
      for (int s = 0; s < 2; ++s) fa[i][s] = tfrag<C::RA>(ht, oa[i], s);
  };
  auto rd_b0 = [&](const char* bu) {
    if (PP_ABL_READ) return;
#pragma unroll
    for (int j = 0; j < C::FN0; ++j)
#pragma unroll
      for (int s = 0; s < 2; ++s) fb0[j][s] = tfrag<C::RB0>(bu + C::O_B0, ob0[j], s);
  };
  auto rd_b1 = [&](const char* bu) {
    if (PP_ABL_READ) return;
#pragma unroll
    for (int j = 0; j < C::FN1; ++j)
#pragma unroll
      for (int s = 0; s < 2; ++s) fb1[j][s] = tfrag<C::RB1>(bu + C::O_B1, ob1[j], s);
  };
  // the last K-tile's A elements with k >= kend
  const int kv = kend - (kbeg + (nk - 1) * BK);      // valid k-rows of the last K-tile (1 .. 64)
  auto mask_a = [&]() {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int n = kv - 32 * s - 8 * (lane >> 4);
#pragma unroll
      for (int i = 0; i < C::FM2; ++i) fa[i][s] = kmask(fa[i][s], n);
    }
  };
  auto mm0 = [&](int i0) {
    if (PP_ABL_MFMA) return;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < C::FM2; ++i)
#pragma unroll
        for (int j = 0; j < C::FN0; ++j)
          acc[i0 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb0[j][s], fa[i][s], acc[i0 + i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  auto mm1 = [&](int i0) {
    if (PP_ABL_MFMA) return;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < C::FM2; ++i)
#pragma unroll
        for (int j = 0; j < C::FN1; ++j)
          acc[i0 + i][C::FN0 + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb1[j][s], fa[i][s], acc[i0 + i][C::FN0 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  using pp::bar;
  using pp::lgkm0;
  using pp::vm_wait;
  constexpr int G = C::G;
  st_alo(0);
  st_b0(0);
  st_b1(0);
  st_ahi(0);
  st_alo(1);
  st_b0(1);
  vm_wait<G>();
  bar();
  if (wr == 1) bar();
  int u = 0;
#pragma unroll 1
  for (; u + 2 < nk; ++u) {
    const char* bu = buf(u);
    rd_b0(bu);
    rd_a(bu + C::O_ALO);
    st_b1(u + 1);
    vm_wait<G>();
    bar();
    lgkm0();
    __builtin_amdgcn_sched_barrier(0);
    mm0(0);
    bar();
    rd_b1(bu);
    st_ahi(u + 1);
    vm_wait<G>();
    bar();
    lgkm0();
    __builtin_amdgcn_sched_barrier(0);
    mm1(0);
    bar();
    rd_a(bu + C::O_AHI);
    st_alo(u + 2);
    vm_wait<G>();
    bar();
    lgkm0();
    __builtin_amdgcn_sched_barrier(0);
    mm1(C::FM2);
    bar();
    st_b0(u + 2);
    vm_wait<G>();
    bar();
    mm0(C::FM2);
    bar();
  }
#pragma unroll
  for (int t = 0; t < 2; ++t, ++u) {
    const bool second_last = t == 0;
    const bool tail = !second_last && kv < BK;
    const char* bu = buf(u);
    rd_b0(bu);
    rd_a(bu + C::O_ALO);
    if (second_last) {
      st_b1(u + 1);
      vm_wait<G>();
    } else {
      vm_wait<C::GA>();
    }
    bar();
    lgkm0();
    __builtin_amdgcn_sched_barrier(0);
    if (tail) mask_a();
    mm0(0);
    bar();
    rd_b1(bu);
    if (second_last) {
      st_ahi(u + 1);
      vm_wait<G>();
    } else {
      vm_wait<0>();
    }
    bar();
    lgkm0();
    __builtin_amdgcn_sched_barrier(0);
    mm1(0);
    bar();
    rd_a(bu + C::O_AHI);
    if (second_last) vm_wait<G - C::GA>();
    else vm_wait<0>();
    bar();
    lgkm0();
    __builtin_amdgcn_sched_barrier(0);
    if (tail) mask_a();
    mm1(C::FM2);
    bar();
    if (second_last) vm_wait<C::GB1 + C::GA>();
    else vm_wait<0>();
    bar();
    mm0(C::FM2);
    bar();
  }
  if (wr == 0) bar();
  if (grp.n && a.splits == 1) {
    DphGemmArgs e = a;
    e.C.ptr = grp.c[z];
    ring::direct_epi_t<C, DPH_ACT_NONE, false>(e, zz, m0 + wr * C::WTM, n0 + wc * C::WTN, lane, acc);
  } else {
    ring::direct_epi_t<C, DPH_ACT_NONE, false>(a, zz, m0 + wr * C::WTM, n0 + wc * C::WTN, lane, acc);
  }
}
}  // namespace ppw

// out[c] += sum_r slab[r][c] (out) and aux[c] += sum_r slab[nrows + r][c]: 64 columns x 4 row phases per block
// over one of gridDim.y (<= 32) row groups, one atomic per column per group
__global__ void __launch_bounds__(256) colsum_slab_reduce_kernel(const float* __restrict__ slab, int64_t nrows,
                                                                 int64_t ncols, int64_t csn, float* __restrict__ out,
                                                                 float* __restrict__ aux) {
  __shared__ float red[2][4][64];
  const int tx = threadIdx.x & 63;
  const int ty = threadIdx.x >> 6;
  const int64_t col = (int64_t)blockIdx.x * 64 + tx;
  const int64_t per = cdiv(nrows, (int64_t)gridDim.y);
  const int64_t ra = (int64_t)blockIdx.y * per;
  const int64_t rb = min(nrows, ra + per);
  float so = 0.f, sa = 0.f;
  if (col < csn) {
    // four rows' loads in flight per thread (independent partial sums)
    float so1 = 0.f, sa1 = 0.f, so2 = 0.f, sa2 = 0.f, so3 = 0.f, sa3 = 0.f;
    int64_t r = ra + ty;
    for (; r + 12 < rb; r += 16) {
      so += slab[r * ncols + col];
      sa += slab[(nrows + r) * ncols + col];
      so1 += slab[(r + 4) * ncols + col];
      sa1 += slab[(nrows + r + 4) * ncols + col];
      so2 += slab[(r + 8) * ncols + col];
      sa2 += slab[(nrows + r + 8) * ncols + col];
      so3 += slab[(r + 12) * ncols + col];
      sa3 += slab[(nrows + r + 12) * ncols + col];
    }
    for (; r < rb; r += 4) {
      so += slab[r * ncols + col];
      sa += slab[(nrows + r) * ncols + col];
    }
    so += (so1 + so2) + so3;
    sa += (sa1 + sa2) + sa3;
  }
  red[0][ty][tx] = so;
  red[1][ty][tx] = sa;
  __syncthreads();
  if (ty == 0 && col < csn) {
    if (out) atomicAdd(out + col, red[0][0][tx] + red[0][1][tx] + red[0][2][tx] + red[0][3][tx]);
    if (aux) atomicAdd(aux + col, red[1][0][tx] + red[1][1][tx] + red[1][2][tx] + red[1][3][tx]);
  }
}

// deterministic mode: the same sums, every column's slab rows added in a fixed order by one block of 32 columns x
// DET_PH row phases (det_column_total); out and aux each get one writer per column
__global__ void __launch_bounds__(32 * DET_PH) colsum_slab_reduce_det_kernel(const float* __restrict__ slab,
                                                                             int64_t nrows, int64_t ncols, int64_t csn,
                                                                             float* __restrict__ out,
                                                                             float* __restrict__ aux) {
  __shared__ float red[DET_PH][33];
  const int64_t col = (int64_t)blockIdx.x * 32 + (threadIdx.x & 31);
  const bool live = col < csn;
  const float so = det_column_total(live && out ? slab + col : nullptr, nrows, ncols, red);
  const float sa = det_column_total(live && aux ? slab + nrows * ncols + col : nullptr, nrows, ncols, red);
  if ((threadIdx.x >> 5) == 0 && live) {
    if (out) out[col] += so;
    if (aux) aux[col] += sa;
  }
}

// split-K reduction + epilogue: one thread per 8 columns of a row
__global__ void splitk_reduce_kernel(const DphGemmArgs a0, const DphGemmGroup grp) {
  DphGemmArgs a = a0;
  if (grp.n) a.C.ptr = grp.c[blockIdx.z];   // grouped launch: problem z's output (its z offset is 0)
  const int64_t z = blockIdx.z;
  const int64_t n8 = (a.N + 7) / 8;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= a.M * n8) return;
  const int64_t m = idx / n8;
  const int64_t n = (idx % n8) * 8;
  const float* ws = reinterpret_cast<const float*>(a.workspace);
  float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const bool vec = (n + 8 <= a.N) && ((a.N & 3) == 0);
  for (int s = 0; s < a.splits; ++s) {
    const float* p = ws + ((z * a.splits + s) * a.M + m) * a.N + n;
    float t[8];
    load8_f32(p, vec, (int)min<int64_t>(8, a.N - n), t);
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] += t[q];
  }
  Cs8 cs;
  epilogue8(a, z, m, n, v, cs);
}

}  // namespace

}  // namespace dph

using namespace dph;

// register-staged kernel width: 512 threads (8 waves of 64x32) for K chunks <= 8192, where the
// second wave per SIMD hides the per-k-step fragment reads and barrier (wgrad shapes +1-3 %, a
// (k, mn) 7984x3072x768 +14 %); 256 (4 waves of 64x64) for the long-K conv weight gradients (-3 %
// with 8 waves).  DPH_GEMM_SMALL_NT=256|512 forces one.
static int small_nt(int64_t kchunk) {
  static const int v = [] {
    const char* e = getenv("DPH_GEMM_SMALL_NT");
    return e ? atoi(e) : 0;
  }();
  if (v == 256 || v == 512) return v;
  return kchunk <= 8192 ? 512 : 256;
}

// DPH_GEMM_PATH: unset/auto = size-based choice, "small" = 128x128 kernel only, "big" = large-tile
// kernel wherever its layout constraints allow (tests exercise both paths in one process)
static int gemm_path_override() {
  const char* e = getenv("DPH_GEMM_PATH");
  if (!e) return 0;
  return !strcmp(e, "small") ? 1 : !strcmp(e, "big") ? 2 : !strcmp(e, "mid") ? 3 : !strcmp(e, "tall") ? 4 : !strcmp(e, "half") ? 5 : !strcmp(e, "mid8") ? 6 : !strcmp(e, "mid8mn") ? 7 : !strcmp(e, "wide") ? 8 : !strcmp(e, "flat") ? 9 : !strcmp(e, "tri") ? 10 : !strcmp(e, "notri") ? 11 : !strcmp(e, "pp256") ? 12 : !strcmp(e, "pp128x256") ? 13 : !strcmp(e, "pp256x128") ? 14 : !strcmp(e, "pp128x192") ? 15 : !strcmp(e, "pp128") ? 16 : !strcmp(e, "ppw") ? 17 : !strcmp(e, "sk") ? 18 : 0;
}

// the 192 x 128 tile takes the register epilogue only (its staged epilogue is compiled but not routed)
static bool tri_ok(const DphGemmArgs& a) {
  return a.splits == 1 && a.a_kcontig && a.b_kcontig && a.K % ring::KS == 0 && ring::direct_epi_ok(a) &&
         a.act != DPH_ACT_GELU_BWD;
}

static int num_cus();

// the ping-pong kernels: both operands k-contiguous with 16-B aligned rows, whole 64-deep K-tiles (at least
// two: the prologue stages two), register-epilogue layouts, DMA source offsets within 32 bits
static bool pp_ok(const DphGemmArgs& a) {
  if (!(a.splits == 1 && a.a_kcontig && a.b_kcontig && a.K % pp::BK == 0 && a.K >= 2 * pp::BK &&
        ring::direct_epi_ok(a)))
    return false;
  auto op_ok = [&](const DphMat& d, int64_t rows) {
    const int64_t al = d.row_stride | d.batch_stride | d.z_inner | d.z_outer;
    if ((al & 7) != 0 || (reinterpret_cast<uintptr_t>(d.ptr) & 15) != 0) return false;
    const int64_t r = rows - 1;
    const int64_t last = d.rows_per_batch > 0 ? (r / d.rows_per_batch) * d.batch_stride + (r % d.rows_per_batch) * d.row_stride
                                              : r * d.row_stride;
    return last + a.K < ((int64_t)1 << 31) && rows < ((int64_t)1 << 31);
  };
  return op_ok(a.A, a.M) && op_ok(a.B, a.N);
}

// DPH_GEMM_PP=0 keeps every GEMM off the ping-pong kernels (A/B; read per call)
static bool pp_enabled() {
  const char* e = getenv("DPH_GEMM_PP");
  return !(e && e[0] == '0');
}

// Ping-pong tile choice: estimated time = whole rounds of tiles over the CU slots x one tile's MFMA work at the
// tile's measured rate (8192^3 random bf16, tools/gemm_ab.py: 256x256 1514, 128x192 1282, 128x256 1221,
// 256x128 1211, 128x128 1178 TFLOP/s; a 128x128 block shares its CU with a second one).  Picks 256x256 for the
// many-round conv GEMMs and 128x192 for the M = B*T projections (756 / 252 tiles = whole rounds on 256 CUs).
// DPH_PP_B0PF=0: one-round 128 x 192 grids on the plain schedule too (A/B and the bitwise test; read per call)
static bool pp_b0pf() {
  const char* e = getenv("DPH_PP_B0PF");
  return !(e && e[0] == '0');
}

// Multi-round 128 x 192 grids with the plain epilogue (no activation, no dropout: the QKV forward, 756 tiles) on the
// two-blocks-per-CU build (Cfg::M2, <= 128 VGPRs, 20 B of epilogue spill): one block's prologue / epilogue runs
// beside the other's main loop -- QKV forward 41.9 -> 36.1 us (profiles/r6_m2_ab.txt).  The GELU / dropout epilogues
// spill 36-172 B per lane at that cap and measured slower (FFN1 / FFN2-DGK: +3-24 %): they keep one block per CU.
// DPH_PP_M2=0 keeps every 128 x 192 grid on the one-block build, =1 forces M2 for all of them (A/B, read per call).
static bool pp_m2(const DphGemmArgs& a) {
  const char* e = getenv("DPH_PP_M2");
  if (e && e[0] == '0') return false;
  if (e && e[0] == '1') return true;
  return a.act == DPH_ACT_NONE && a.dropout_p <= 0.f && !(a.flags & DPH_GEMM_PRE_DGK);
}

static int pp_pick(const DphGemmArgs& a) {
  struct Opt { int kind, bm, bn, per_cu; double tf; };
  static const Opt opts[] = {{12, 256, 256, 1, 1514.0}, {15, 128, 192, 1, 1282.0}, {13, 128, 256, 1, 1221.0},
                             {14, 256, 128, 1, 1211.0}, {16, 128, 128, 2, 1178.0}};
  const int64_t cus = num_cus();
  // DPH_PP_FORCE=kind (A/B sweeps, read per call): that tile whenever the ping-pong path runs
  if (const char* e = getenv("DPH_PP_FORCE")) {
    const int fk = atoi(e);
    for (const Opt& o : opts)
      if (o.kind == fk) return fk;
  }
  // FFN-width GELU epilogues (the intermediate forward with its stored factor, the DGK input gradient): the
  // epilogue outweighs the 12 K-tiles of MFMA work, and the two-blocks-per-CU 128 x 128 tile runs one block's
  // epilogue beside the other's main loop: 62.5 / 57.6 / 54.3 us vs 70.2 / 64.3 / 61.9 on 128 x 192
  // (student FFN1 / teacher FFN1 / FFN2 DGK dgrad at 7984 x 3072 x 768, profiles/r4_s8_pp_tile_ab.txt)
  // (the Large shape, 5988 x 4096 x 1024, measured the same with and without the rule: 23.21 / 23.23 ms per step,
  // profiles/r4_s33_large_gelu128_ab.txt.)  DPH_PP_GELU128=0 drops the rule (A/B, read per call)
  const char* g128 = getenv("DPH_PP_GELU128");
  if (!(g128 && g128[0] == '0') && a.act != DPH_ACT_NONE && a.N >= 2048 && a.K <= 1024 && a.batch == 1) return 16;
  int best = 12;
  double best_t = 1e300;
  for (const Opt& o : opts) {
    const int64_t tiles = cdiv(a.M, o.bm) * cdiv(a.N, o.bn) * a.batch;
    const int64_t rounds = cdiv(tiles, cus * o.per_cu);
    const double t = (double)rounds * o.per_cu * (double)o.bm * o.bn / o.tf;
    if (t < best_t * 0.999) {
      best_t = t;
      best = o.kind;
    }
  }
  return best;
}

// ---- the weight-gradient ping-pong path (ppw) ----
// DPH_GEMM_PPW=0 keeps the (mn, mn) GEMMs on the register-staged kernel (A/B; read per call)
static bool ppw_enabled() {
  const char* e = getenv("DPH_GEMM_PPW");
  return !(e && e[0] == '0');
}

struct PpwPlan {
  int kind;         // 12 / 13 / 15 / 16 (pp tile ids), 0: none
  int splits;
  int64_t kchunk;   // K per split (whole 64-deep K-tiles)
};

// Tile and split-K choice: whole rounds of (tile, split) blocks over the CU slots x one block's MFMA work at the
// tile's measured ping-pong rate, plus the fp32 slab the splits write and splitk_reduce_kernel reads back
// (~4 TB/s) and that launch.  Each split keeps at least eight K-tiles.  The 128 x 192 and 128 x 128 tiles run two
// blocks per CU here (<= 128 VGPRs, <= 80 KB LDS).  Long-K (conv) shapes: 128 x 192 tiles and ~48 K-tiles per
// split (up to 32 splits).  Sweep behind both rules: profiles/r3_s9_wgrad_sweep.txt (tools/wgrad_sweep.py).
// DPH_PPW_LONGK=0: the round-3 long-K rule (128 x 192, ~48 K-tiles per split) for the conv weight gradients (A/B)
static bool long_k_one_round() {
  static const bool on = [] {
    const char* e = getenv("DPH_PPW_LONGK");
    return !(e && e[0] == '0');
  }();
  return on;
}

// DPH_PPW_GSPLIT=0: the grouped weight gradients on the rounds model alone (A/B)
static bool grouped_two_splits() {
  static const bool on = [] {
    const char* e = getenv("DPH_PPW_GSPLIT");
    return !(e && e[0] == '0');
  }();
  return on;
}

static PpwPlan ppw_plan(int64_t M, int64_t N, int64_t K, int64_t batch, int want_splits) {
  struct Opt { int kind, bm, bn, per_cu; double tf; };
  static const Opt opts[] = {{12, 256, 256, 1, 1514.0}, {15, 128, 192, 2, 1282.0}, {13, 128, 256, 1, 1221.0},
                             {16, 128, 128, 2, 1178.0}};
  const int64_t cus = num_cus();
  const int64_t nkt = cdiv(K, (int64_t)pp::BK);
  constexpr int64_t MIN_KT = 8;
  // DPH_PPW_FORCE="kind:splits" (A/B sweeps, read per call): only that tile, and that split count when free
  int fk = 0, fs = 0;
  if (const char* e = getenv("DPH_PPW_FORCE")) sscanf(e, "%d:%d", &fk, &fs);
  if (want_splits == 0 && fs > 0) want_splits = fs;
  PpwPlan best{0, 0, 0};
  double best_t = 1e300;
  for (const Opt& o : opts) {
    if (fk && o.kind != fk) continue;
    const int64_t tiles = cdiv(M, (int64_t)o.bm) * cdiv(N, (int64_t)o.bn) * batch;
    for (int s = 1; s <= 32; ++s) {
      if (want_splits > 0 && s != want_splits) continue;
      const int64_t kct = cdiv(nkt, (int64_t)s);
      if (kct < 2 || cdiv(nkt, kct) != s || nkt - (s - 1) * kct < 2) continue;
      if (want_splits == 0 && kct < MIN_KT && s > 1) continue;
      double t;
      const int64_t tiles256 = cdiv(M, (int64_t)256) * cdiv(N, (int64_t)256) * batch;
      if (nkt >= 384 && tiles256 <= 32 && want_splits == 0 && long_k_one_round()) {
        // long K over few output tiles (the conv extractor's weight gradients, 512 x k*512 over B*L frames): ONE round
        // of 256 x 256 (tile, split) blocks over the CUs -- 12 tiles x 21 splits: conv1-4 447 / 236 / 129 / 74 us
        // against 529 / 286 / 134 / 82 us on the 128 x 192 / ~48-K-tile rule below (profiles/r4_s40_wgrad_sweep.txt);
        // the nearest feasible split count on that tile, other tiles only as a fallback
        const int64_t s1 = std::max<int64_t>(1, std::min<int64_t>(32, cus / tiles256));
        t = (double)(s > s1 ? s - s1 : s1 - s) + (o.kind == 12 ? 0.0 : 1000.0);
      } else if (batch > 1 && M >= 256 && N >= 256 && tiles256 * 2 <= cus * 3 && nkt >= 32 && want_splits == 0 &&
                 grouped_two_splits()) {
        // grouped weight gradients (n layers' dW of one shape per launch) whose 256 x 256 tiles fill at most 1.5
        // rounds: two K-splits on that tile -- n = 12 QKV (1.27 rounds) 550 -> 478 us, out-proj (0.42) 194 -> 170 us
        // (profiles/r4_s42_wgrad_group_sweep.txt; FFN1 / FFN2 at 1.69 rounds stay on one split)
        t = (o.kind == 12 && s == 2) ? 0.0 : 1000.0 + (double)s;
      } else if (nkt >= 768 && want_splits == 0) {
        // long K: the measured optimum sits at ~48 K-tiles per split on 128 x 192 (conv1 / conv2 at 32 splits)
        if (o.kind != 15) continue;
        t = kct > 48 ? (double)(kct - 48) : (double)(48 - kct);
      } else {
        const int64_t rounds = cdiv(tiles * s, cus * o.per_cu);
        t = (double)rounds * o.per_cu * 2.0 * o.bm * o.bn * (double)(kct * pp::BK) / (o.tf * 1e12 / (double)cus);
        if (s > 1) t += (double)(s + 1) * batch * M * N * 8.0 / 4.0e12 + 3e-6;
      }
      if (t < best_t * 0.999) {
        best_t = t;
        best = PpwPlan{o.kind, s, kct * pp::BK};
      }
    }
  }
  return best;
}

// operands and epilogue the ppw kernels take: (mn, mn), plain epilogue (alpha, fp32 / accumulating output), dense
// A rows, B rows dense or batched with >= 64 rows per batch, 16-B aligned rows, DMA offsets and the 24-bit row
// products within range
static bool ppw_ok(const DphGemmArgs& a) {
  if (a.a_kcontig || a.b_kcontig || a.act != DPH_ACT_NONE || a.bias || a.colmask || a.smask || a.pre_out || a.aux_in ||
      a.residual || a.colsum_out || a.colsum_aux || a.row_len || a.dropout_p != 0.f || a.c_dtype == DPH_OUT_BF16)
    return false;
  if (a.M < 64 || a.N < 64 || a.K < 2 * pp::BK || a.K >= (1 << 24)) return false;
  if (cdiv(a.M, (int64_t)128) >= 65536 || (int64_t)a.batch * a.splits >= 65536) return false;
  auto op_ok = [&](const DphMat& d, int64_t cols, bool batched_ok) {
    const int64_t al = d.row_stride | d.batch_stride | d.z_inner | d.z_outer;
    if ((al & 7) != 0 || (reinterpret_cast<uintptr_t>(d.ptr) & 15) != 0) return false;
    // (rows may overlap -- conv windows, row stride s*C < k*C -- when the extent is whole 16-B chunks; a ragged
    // extent needs rows padded to the chunk, as dph_gemm requires)
    if (d.row_stride >= (1 << 24) || ((cols & 7) != 0 && d.row_stride < ((cols + 7) & ~(int64_t)7))) return false;
    int64_t last;
    if (d.rows_per_batch > 0) {
      if (!batched_ok || d.rows_per_batch < pp::BK || d.rows_per_batch >= (1 << 24)) return false;
      const int64_t r = a.K - 1;
      last = (r / d.rows_per_batch) * d.batch_stride + (d.rows_per_batch - 1) * d.row_stride;
    } else {
      last = (a.K - 1) * d.row_stride;
    }
    return last + cols + 8 < ((int64_t)1 << 31);
  };
  return op_ok(a.A, a.M, false) && op_ok(a.B, a.N, true);
}

// epilogue args of a ppw launch: the real C (splits == 1) or the fp32 slab of the splits (z = batch * splits + split)
static bool ppw_zmap_enabled() {
  const char* e = getenv("DPH_PPW_ZMAP");
  return !(e && e[0] == '0');
}

static DphGemmArgs ppw_epi_args(const DphGemmArgs& a) {
  DphGemmArgs e = a;
  if ((int64_t)a.batch * a.splits > 1 && ppw_zmap_enabled() &&
      cdiv(a.M, (int64_t)64) * cdiv(a.N, (int64_t)64) * a.batch * a.splits < ((int64_t)1 << 31))
    e.flags |= GEMM_PPW_ZMAP;
  if (a.splits > 1) {
    e.C = DphMat{a.workspace, 0, 0, a.N, 0, 0, a.M * a.N};
    e.c_dtype = DPH_OUT_F32;
    e.alpha = 1.0f;
  }
  return e;
}

// the plan dph_gemm runs for an eligible (mn, mn) GEMM with these splits (kind 0: the register-staged kernel)
static PpwPlan ppw_route(const DphGemmArgs& a) {
  // (a forced DPH_GEMM_PATH other than "ppw" keeps the (mn, mn) GEMMs where it points: tests cover both kernels)
  const int path = gemm_path_override();
  if (!ppw_enabled() || (path != 0 && path != 17) || !ppw_ok(a)) return PpwPlan{0, 0, 0};
  const PpwPlan p = ppw_plan(a.M, a.N, a.K, a.batch, a.splits);
  if (p.kind == 0 || !ring::direct_epi_ok(ppw_epi_args(a))) return PpwPlan{0, 0, 0};
  return p;
}

// split-K factor the ppw plan wants for an (mn, mn) weight-gradient shape (0: no plan; the caller's heuristic)
extern "C" int dph_gemm_mn_plan(int64_t M, int64_t N, int64_t K, int64_t batch) {
  if (!ppw_enabled() || M < 64 || N < 64 || K < 2 * pp::BK || batch < 1) return 0;
  return ppw_plan(M, N, K, batch, 0).splits;
}

template <class Cf>
static void launch_ppw(const DphGemmArgs& e, int64_t kchunk, const DphGemmGroup& grp, hipStream_t stream) {
  const dim3 g((unsigned)cdiv(e.N, Cf::BN), (unsigned)cdiv(e.M, Cf::BM), (unsigned)(e.batch * e.splits)), b(Cf::NT);
  if (e.B.rows_per_batch > 0) hipLaunchKernelGGL((ppw::ppw_gemm_kernel<Cf, true>), g, b, 0, stream, e, kchunk, grp);
  else hipLaunchKernelGGL((ppw::ppw_gemm_kernel<Cf, false>), g, b, 0, stream, e, kchunk, grp);
}

// the ppw plan's launch (+ split-K reduce) for args ppw_route accepted
static int run_ppw(const DphGemmArgs& a, const PpwPlan& pw, const DphGemmGroup& grp, hipStream_t stream) {
  const DphGemmArgs e = ppw_epi_args(a);
  if (pw.kind == 12) launch_ppw<pp::P256>(e, pw.kchunk, grp, stream);
  else if (pw.kind == 13) launch_ppw<pp::P128x256>(e, pw.kchunk, grp, stream);
  else if (pw.kind == 15) launch_ppw<pp::P128x192>(e, pw.kchunk, grp, stream);
  else launch_ppw<pp::P128>(e, pw.kchunk, grp, stream);
  int rc = check_launch("dph_gemm (ppw)");
  if (rc || a.splits == 1) return rc;
  const int64_t work = a.M * cdiv(a.N, (int64_t)8);
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)cdiv(work, (int64_t)256), 1, (unsigned)a.batch), dim3(256), 0,
                     stream, a, grp);
  return check_launch("dph_gemm (ppw) splitk_reduce");
}

// only where both tilings are a single round over the CUs (one block per CU) and the 192 x 128 one has
// less area per CU: with several rounds the 128 x 256 tile's two waves per SIMD win (conv1 255984 x 512 x
// 1536: 553 vs 622 us)
static bool tri_better(const DphGemmArgs& a) {
  const int64_t cus = num_cus();
  const int64_t tf = cdiv(a.M, ring::Flat::BM) * cdiv(a.N, ring::Flat::BN) * a.batch;
  const int64_t tt = cdiv(a.M, ring::Tri::BM) * cdiv(a.N, ring::Tri::BN) * a.batch;
  return tf <= cus && tt <= cus && ring::Tri::BM * ring::Tri::BN < ring::Flat::BM * ring::Flat::BN;
}

// an operand the ring kernels can stage: k-contiguous with whole 32-deep k-slices, or mn-contiguous
// (any K: a partial last slice is zero-filled) whose batched row layout carries at most once per slice
static bool ring_operand_ok(bool kcontig, const DphMat& d, int64_t K) {
  if (kcontig) return K % ring::KS == 0;
  if (K >= ((int64_t)1 << 31) - 2 * ring::KS) return false;   // 32-bit k-row state
  return d.rows_per_batch == 0 || d.rows_per_batch >= ring::KS;
}

// 0: 128x128 register-staged kernel, 1: ring Mid (128x128), 2: ring Big (256x256).  The ring kernels
// take (k, k), (k, mn) and (mn, mn) operand layouts; (mn, k) and K-tails beside a k-contiguous
// operand stay on the register-staged kernel.
static int gemm_kind(const DphGemmArgs& a, int64_t kchunk) {
  // mn-contiguous operands on the ring measured slower than the register-staged kernel on every
  // step shape (dgrad 7984x768x3072: 80 vs 73 us, conv1 wgrad 862 vs 642 us: two transposed reads per
  // fragment and a barrier per 32-k slice), so by default they stay there; DPH_GEMM_PATH=mid/big
  // forces the ring (tests cover both)
  const int path0 = gemm_path_override();
  const bool layouts = (a.a_kcontig && a.b_kcontig) || ((path0 == 3 || path0 == 7) && !((!a.a_kcontig) && a.b_kcontig));
  const bool ring_ok = layouts && ring_operand_ok(a.a_kcontig, a.A, a.K) && ring_operand_ok(a.b_kcontig, a.B, a.K) &&
                       (a.splits == 1 || kchunk % ring::KS == 0);
  // the 256x256 tile is k-contiguous only: its 128 accumulators leave no registers for the
  // mn-contiguous k-row state (it spilled 28-100 VGPRs)
  const bool big_ok = ring_ok && a.a_kcontig && a.b_kcontig;
  const int64_t tiles256 = cdiv(a.M, ring::Big::BM) * cdiv(a.N, ring::Big::BN) * a.batch * a.splits;
  int kind = !ring_ok ? 0 : ((big_ok && tiles256 >= 480) ? 2 : 1);
  // N <= 64 (<= 1/4 of a 256 tile, 1/2 of a 128 tile): the 256 x 64 tile
  if (big_ok && a.N <= ring::Tall::BN && a.M > 128) kind = 3;
  // short K (<= 32 slices): the 8-wave 128 x 128 tile (two waves per SIMD per block overlap the
  // fixed per-tile costs; measured +10 % on the K = 768 projections, even at K = 3072)
  // (also instead of the 256 x 256 tile: conv dgrad 255984x1536x512 ran 389 TF/s on it)
  else if ((kind == 1 || kind == 2) && big_ok && kchunk <= 1024) kind = 5;
  // the 128 x 256 tile (8 waves of 64 x 64, persistent grid): long K (the 128 x 128 tiles measured 20 %
  // slower on 7984 x 768 x 3072 / 2304, the 256 x 256 one 10 % on the 1536-deep conv GEMMs) and N <= 1024
  // (few 128 x 128 tiles per CU: 7984 x 768 x 768 -11 %)
  if (big_ok && a.N > ring::Tall::BN && (kchunk >= 1536 || (a.N <= 1024 && kchunk >= 4 * ring::KS))) kind = 8;
  // N <= 1024 on the 192 x 128 tile when it fills the CUs better (whole-chip rounds of tiles x tile area)
  if (kind == 8 && a.N <= 1024 && tri_ok(a) && tri_better(a)) kind = 10;
  // the ping-pong kernels wherever their layout holds (A/B: DPH_GEMM_PP=0; a forced DPH_GEMM_PATH wins)
  if (pp_enabled() && pp_ok(a)) kind = pp_pick(a);
  const int path = gemm_path_override();
  if (path == 1) kind = 0;
  if (path == 2 && big_ok) kind = 2;
  if (path == 3 && ring_ok) kind = 1;
  if (path == 4 && big_ok) kind = 3;
  if (path == 5 && big_ok) kind = 4;
  if (path == 6 && big_ok) kind = 5;
  if (path == 7 && ring_ok && !big_ok) kind = 6;     // 8-wave 128x128 tile with mn-contiguous operands
  if (path == 8 && big_ok) kind = 7;
  if (path == 9 && big_ok) kind = 8;
  if (path == 10 && big_ok && tri_ok(a)) kind = 10;
  if (path == 11 && kind == 10) kind = 8;     // "notri": the 128 x 256 tile where the 192 x 128 one would run
  if (path >= 12 && path <= 16 && pp_ok(a)) kind = path;   // ping-pong tiles (A/B)
  return kind;
}

static int64_t gemm_kchunk(const DphGemmArgs& a) {
  return a.splits > 1 ? cdiv(cdiv(a.K, a.splits), BK) * BK : a.K;
}

static bool persist_ok(const DphGemmArgs& a);

static bool sk_route(const DphGemmArgs& a, SkPlan* p);

extern "C" const char* dph_gemm_variant(const DphGemmArgs* args) {
  if (!args) return "";
  const DphGemmArgs& a = *args;
  {
    SkPlan skp;
    if (a.sk_ws && sk_route(a, &skp)) return sk_variant(a);
  }
  const bool dgk = a.act == DPH_ACT_GELU_BWD_DGK || (a.act == DPH_ACT_GELU && (a.flags & DPH_GEMM_PRE_DGK));
  const PpwPlan pw = ppw_route(a);
  if (pw.kind == 12) return "ppw_gemm_kernel<dph::(anonymous namespace)::pp::Cfg<256, 256>";
  if (pw.kind == 13) return "ppw_gemm_kernel<dph::(anonymous namespace)::pp::Cfg<128, 256>";
  if (pw.kind == 15) return "ppw_gemm_kernel<dph::(anonymous namespace)::pp::Cfg<128, 192>";
  if (pw.kind == 16) return "ppw_gemm_kernel<dph::(anonymous namespace)::pp::Cfg<128, 128>";
  const int kind = dgk ? pp_pick(a) : gemm_kind(a, gemm_kchunk(a));
  if (kind == 12) return "pp_gemm_kernel<dph::(anonymous namespace)::pp::Cfg<256, 256>";
  if (kind == 13) return "pp_gemm_kernel<dph::(anonymous namespace)::pp::Cfg<128, 256>";
  if (kind == 14) return "pp_gemm_kernel<dph::(anonymous namespace)::pp::Cfg<256, 128>";
  if (kind == 15) return "pp_gemm_kernel<dph::(anonymous namespace)::pp::Cfg<128, 192>";
  if (kind == 16) return "pp_gemm_kernel<dph::(anonymous namespace)::pp::Cfg<128, 128>";
  if (kind == 6) return a.a_kcontig ? "ring::Cfg<128, 128, 64, 32>, true, false>" : "ring::Cfg<128, 128, 64, 32>, false, false>";
  if (kind == 10) return persist_ok(a) ? "persist_kernel<dph::(anonymous namespace)::ring::Cfg<192, 128, 96, 64>"
                                       : "ring::Cfg<192, 128, 96, 64>, true, true>";
  if (kind == 8) return persist_ok(a) ? "persist_kernel<dph::(anonymous namespace)::ring::Cfg<128, 256, 64, 64>"
                                      : "ring::Cfg<128, 256, 64, 64>, true, true>";
  if (kind == 7) return persist_ok(a) ? "persist_kernel<dph::(anonymous namespace)::ring::Cfg<256, 128, 64, 64>"
                                      : "ring::Cfg<256, 128, 64, 64>, true, true>";
  if (kind == 5) return "ring::Cfg<128, 128, 64, 32>, true, true>";
  if (kind == 4) return "ring::Cfg<128, 64, 64, 32>, true, true>";
  if (kind == 3) return "ring::Cfg<256, 64, 128, 32>, true, true>";
  if (kind == 2) return "ring::Cfg<256, 256, 128, 64>, true, true>";
  if (kind == 1) {
    if (a.a_kcontig && a.b_kcontig) return "ring::Cfg<128, 128, 64, 64>, true, true>";
    if (a.a_kcontig) return "ring::Cfg<128, 128, 64, 64>, true, false>";
    return "ring::Cfg<128, 128, 64, 64>, false, false>";
  }
  const bool w8 = small_nt(gemm_kchunk(a)) == 512;
  if (a.a_kcontig && a.b_kcontig) return w8 ? "gemm_kernel<true, true, 512>" : "gemm_kernel<true, true>";
  if (a.a_kcontig) return w8 ? "gemm_kernel<true, false, 512>" : "gemm_kernel<true, false>";
  if (a.b_kcontig) return w8 ? "gemm_kernel<false, true, 512>" : "gemm_kernel<false, true>";
  return w8 ? "gemm_kernel<false, false, 512>" : "gemm_kernel<false, false>";
}

template <class Cf, bool MN>
static void launch_ring(const DphGemmArgs& a, int64_t kchunk, hipStream_t stream) {
  dim3 g((unsigned)cdiv(a.N, Cf::BN), (unsigned)cdiv(a.M, Cf::BM), (unsigned)(a.batch * a.splits));
  if constexpr (MN) {
    if (a.a_kcontig)
      hipLaunchKernelGGL((ring_gemm_kernel<Cf, true, false>), g, dim3(Cf::NT), 0, stream, a, kchunk);
    else
      hipLaunchKernelGGL((ring_gemm_kernel<Cf, false, false>), g, dim3(Cf::NT), 0, stream, a, kchunk);
  } else {
    hipLaunchKernelGGL((ring_gemm_kernel<Cf, true, true>), g, dim3(Cf::NT), 0, stream, a, kchunk);
  }
}

template <class Cf>
static void launch_pp(const DphGemmArgs& a, hipStream_t stream) {
  const dim3 g((unsigned)cdiv(a.N, Cf::BN), (unsigned)cdiv(a.M, Cf::BM), (unsigned)a.batch), b(Cf::NT);
  const bool drop = a.dropout_p > 0.f;
  if (a.act == DPH_ACT_GELU_BWD_DGK) {
    hipLaunchKernelGGL((pp::pp_gemm_kernel<Cf, DPH_ACT_GELU_BWD_DGK, false>), g, b, 0, stream, a);
  } else if (a.act == DPH_ACT_GELU && (a.flags & DPH_GEMM_PRE_DGK)) {
    if (drop) hipLaunchKernelGGL((pp::pp_gemm_kernel<Cf, ACT_GELU_DGKPRE, true>), g, b, 0, stream, a);
    else hipLaunchKernelGGL((pp::pp_gemm_kernel<Cf, ACT_GELU_DGKPRE, false>), g, b, 0, stream, a);
  } else if (a.act == DPH_ACT_GELU) {
    if (drop) hipLaunchKernelGGL((pp::pp_gemm_kernel<Cf, DPH_ACT_GELU, true>), g, b, 0, stream, a);
    else hipLaunchKernelGGL((pp::pp_gemm_kernel<Cf, DPH_ACT_GELU, false>), g, b, 0, stream, a);
  } else if (a.act == DPH_ACT_GELU_BWD) {
    if (drop) hipLaunchKernelGGL((pp::pp_gemm_kernel<Cf, DPH_ACT_GELU_BWD, true>), g, b, 0, stream, a);
    else hipLaunchKernelGGL((pp::pp_gemm_kernel<Cf, DPH_ACT_GELU_BWD, false>), g, b, 0, stream, a);
  } else {
    if (drop) hipLaunchKernelGGL((pp::pp_gemm_kernel<Cf, DPH_ACT_NONE, true>), g, b, 0, stream, a);
    else hipLaunchKernelGGL((pp::pp_gemm_kernel<Cf, DPH_ACT_NONE, false>), g, b, 0, stream, a);
  }
}

// CU count of the current device (persistent grids)
static int num_cus() {
  static int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 256;
    return v > 0 ? v : 256;
  }();
  return n;
}

// The persistent stream-K 256 x 256 kernel (gemm_sk.hip) for the wide-N M = B*T projections: taken when the layout
// is the ping-pong one and sk_plan accepts the shape.  GEMMs flagged as sharing the GPU with another stream (the
// concurrent teacher forward) take it too; DPH_GEMM_SK_SHARED=0 keeps those on the tile grids (A/B; read per call).
static bool sk_route(const DphGemmArgs& a, SkPlan* p) {
  // (a forced DPH_GEMM_PATH other than "sk" keeps its tile path: the GEMM tests run every path on the same shapes)
  const int path = gemm_path_override();
  if ((path != 0 && path != 18) || ppw_route(a).kind || !pp_ok(a)) return false;
  if (a.flags & DPH_GEMM_NO_PERSIST) {
    const char* e = getenv("DPH_GEMM_SK_SHARED");
    if (e && e[0] == '0') return false;
  }
  return sk_plan(a, num_cus(), p);
}

// DPH_GEMM_PERSIST=0 keeps the one-tile-per-block ring launch (A/B; read per call like DPH_GEMM_PATH)
static bool persist_enabled() {
  const char* e = getenv("DPH_GEMM_PERSIST");
  return !(e && e[0] == '0');
}

static bool persist_ok(const DphGemmArgs& a) {
  // (not GELU_BWD: its epilogue inside the tile loop spills 40-50 VGPRs)
  return persist_enabled() && !(a.flags & DPH_GEMM_NO_PERSIST) && a.act != DPH_ACT_GELU_BWD && a.splits == 1 &&
         a.a_kcontig && a.b_kcontig &&
         a.K % (2 * ring::KS) == 0 &&
         a.K >= 4 * ring::KS && ring::direct_epi_ok(a) && a.M < ((int64_t)1 << 31) && a.N < ((int64_t)1 << 31) &&
         cdiv(a.M, 128) * cdiv(a.N, 128) * a.batch < ((int64_t)1 << 30);
}

template <class Cf>
static bool launch_ring_persist(const DphGemmArgs& a, hipStream_t stream) {
  if (!persist_ok(a)) return false;
  const int64_t ntm = cdiv(a.M, Cf::BM), ntn = cdiv(a.N, Cf::BN);
  const int64_t total = ntm * ntn * a.batch;
  const int64_t slots = (int64_t)num_cus() * Cf::MINB;
  const int64_t grid = total < slots ? total : slots;
  const dim3 g((unsigned)grid), b(Cf::NT);
  const bool drop = a.dropout_p > 0.f;
  if (a.act == DPH_ACT_GELU) {
    if (drop) hipLaunchKernelGGL((ring_persist_kernel<Cf, DPH_ACT_GELU, true>), g, b, 0, stream, a, ntm, ntn);
    else hipLaunchKernelGGL((ring_persist_kernel<Cf, DPH_ACT_GELU, false>), g, b, 0, stream, a, ntm, ntn);
  } else {
    if (drop) hipLaunchKernelGGL((ring_persist_kernel<Cf, DPH_ACT_NONE, true>), g, b, 0, stream, a, ntm, ntn);
    else hipLaunchKernelGGL((ring_persist_kernel<Cf, DPH_ACT_NONE, false>), g, b, 0, stream, a, ntm, ntn);
  }
  return true;
}

extern "C" int dph_gemm(const DphGemmArgs* args, hipStream_t stream) {
  DPH_REQUIRE(args != nullptr, "dph_gemm: null args");
  const DphGemmArgs& a = *args;
  DPH_REQUIRE(a.M > 0 && a.N > 0 && a.K > 0, "dph_gemm: bad sizes M=%lld N=%lld K=%lld", (long long)a.M,
              (long long)a.N, (long long)a.K);
  DPH_REQUIRE(a.batch >= 1 && a.splits >= 1, "dph_gemm: batch/splits must be >= 1");
  DPH_REQUIRE(a.A.ptr && a.B.ptr && a.C.ptr, "dph_gemm: null operand");
  DPH_REQUIRE(a.K % 8 == 0 || !a.a_kcontig, "dph_gemm: k-contiguous A needs K %% 8 == 0 (K=%lld)", (long long)a.K);
  DPH_REQUIRE(a.K % 8 == 0 || !a.b_kcontig, "dph_gemm: k-contiguous B needs K %% 8 == 0 (K=%lld)", (long long)a.K);
  // an mn-contiguous operand is read in 8-wide 16-B chunks: its extent must be a multiple of 8, or
  // its rows padded to one (row stride % 8 == 0 and >= the rounded-up extent; the padding columns
  // only feed outputs that are never stored)
  DPH_REQUIRE(a.a_kcontig || a.M % 8 == 0 || (a.A.row_stride % 8 == 0 && a.A.row_stride >= (a.M + 7) / 8 * 8),
              "dph_gemm: mn-contiguous A needs M %% 8 == 0 or 8-padded rows");
  DPH_REQUIRE(a.b_kcontig || a.N % 8 == 0 || (a.B.row_stride % 8 == 0 && a.B.row_stride >= (a.N + 7) / 8 * 8),
              "dph_gemm: mn-contiguous B needs N %% 8 == 0 or 8-padded rows");
  DPH_REQUIRE(a.act != DPH_ACT_GELU_BWD || a.aux_in, "dph_gemm: GELU_BWD needs aux_in");
  DPH_REQUIRE(!a.row_len || a.len_rows > 0, "dph_gemm: row_len needs len_rows");
  DPH_REQUIRE(!(a.flags & DPH_GEMM_RESID_F32) ||
                  (a.residual && a.act != DPH_ACT_GELU_BWD && a.act != DPH_ACT_GELU_BWD_DGK),
              "dph_gemm: DPH_GEMM_RESID_F32 needs a residual and a forward (non-GELU-backward) epilogue");
  int64_t kchunk = a.K;
  if (a.splits > 1) {
    DPH_REQUIRE(!a.colsum_out && !a.colsum_aux, "dph_gemm: column sums not supported with split-K");
    kchunk = cdiv(cdiv(a.K, a.splits), BK) * BK;
    const int64_t need = (int64_t)a.batch * a.splits * a.M * a.N * 4;
    DPH_REQUIRE(a.workspace && a.workspace_bytes >= need, "dph_gemm: split-K workspace too small (%lld < %lld)",
                (long long)a.workspace_bytes, (long long)need);
  }
  // (mn, mn) weight gradients: the ping-pong kernel with its own tile / split plan (the caller sized the workspace
  // with dph_gemm_mn_plan's splits; any other split count keeps the register-staged kernel)
  {
    const PpwPlan pw = ppw_route(a);
    if (pw.kind) return run_ppw(a, pw, DphGemmGroup{}, stream);
  }
  // LDS-DMA ring kernels for k-contiguous A and B with whole 32-deep k-slices: the 256x256 tile
  // when there are >= ~2 full rounds of tiles over the 256 CUs at one block per CU, else the
  // 128x128 tile (DPH_GEMM_PATH=small|big|mid forces a path, for tests)
  // the DGK GELU pair (stored gelu' factor / f) exists in the ping-pong kernels' register epilogue only
  const bool dgk = a.act == DPH_ACT_GELU_BWD_DGK || (a.act == DPH_ACT_GELU && (a.flags & DPH_GEMM_PRE_DGK));
  if (dgk) {
    DPH_REQUIRE(pp_ok(a), "dph_gemm: DPH_ACT_GELU_BWD_DGK / DPH_GEMM_PRE_DGK need the ping-pong layout "
                "(k-contiguous A and B, K %% 64 == 0, dense aligned C): M=%lld N=%lld K=%lld act=%d direct=%d "
                "A(rs=%lld ptr%%16=%d) B(rs=%lld ptr%%16=%d) C(rs=%lld ptr%%16=%d) aux%%16=%d res%%16=%d pre%%16=%d",
                (long long)a.M, (long long)a.N, (long long)a.K, a.act, (int)ring::direct_epi_ok(a),
                (long long)a.A.row_stride, (int)(reinterpret_cast<uintptr_t>(a.A.ptr) & 15), (long long)a.B.row_stride,
                (int)(reinterpret_cast<uintptr_t>(a.B.ptr) & 15), (long long)a.C.row_stride,
                (int)(reinterpret_cast<uintptr_t>(a.C.ptr) & 15), (int)(reinterpret_cast<uintptr_t>(a.aux_in) & 15),
                (int)(reinterpret_cast<uintptr_t>(a.residual) & 15), (int)(reinterpret_cast<uintptr_t>(a.pre_out) & 15));
    DPH_REQUIRE(a.act != DPH_ACT_GELU_BWD_DGK || (a.dropout_p == 0.f && !a.smask && !a.pre_out),
                "dph_gemm: DPH_ACT_GELU_BWD_DGK takes no dropout / smask / pre_out");
    DPH_REQUIRE(a.act != DPH_ACT_GELU || a.pre_out, "dph_gemm: DPH_GEMM_PRE_DGK needs pre_out");
  }
  const int kind = dgk ? pp_pick(a) : gemm_kind(a, kchunk);
  SkPlan skp{};
  const bool use_sk = a.sk_ws != nullptr && sk_route(a, &skp);
  // ((mn, mn) weight gradients off the ppw plan compute the full static extent: correct, only slower -- the packed
  // FFN operands are finite wherever a product is stored and read)
  DPH_REQUIRE(!a.dyn_ext || (!a.a_kcontig && !a.b_kcontig) || (kind >= 12 && kind <= 16 && a.splits == 1),
              "dph_gemm: device-side extents (dyn_ext) need a ping-pong layout (k-contiguous A and B, K %% 64 == 0, dense "
              "aligned C) or the (mn, mn) weight-gradient plan: M=%lld N=%lld K=%lld", (long long)a.M, (long long)a.N,
              (long long)a.K);
  // Column sums (bias / mask gradients of the GELU-backward epilogues) go through a workspace slab of per-tile (or
  // per-wave) partial rows when the caller passed one (kernels.py does for batch 1), summed after the GEMM by
  // colsum_slab_reduce_kernel: in row groups with one float atomic per column per group, or -- deterministic mode --
  // by one group in a fixed order.  The slab row granularity is the epilogue's: per wave (WTM rows) in the register
  // epilogues, per M tile (BM rows) in the LDS-staged ones.
  const bool want_cs = (a.colsum_out || a.colsum_aux) != 0;
  int64_t slot_rows = 0;
  if (want_cs) {
    auto ring_rows = [&](int64_t bm, int64_t wtm, bool dcfg) { return (dcfg && ring::direct_epi_ok(a)) ? wtm : bm; };
    switch (use_sk ? 12 : kind) {
      case 12: case 14: slot_rows = 128; break;            // ping-pong register epilogues (and stream-K): per wave
      case 13: case 15: case 16: slot_rows = 64; break;
      case 10: slot_rows = ring_rows(ring::Tri::BM, ring::Tri::WTM, ring::direct_cfg<ring::Tri>()); break;
      case 8: slot_rows = ring_rows(ring::Flat::BM, ring::Flat::WTM, ring::direct_cfg<ring::Flat>()); break;
      case 7: slot_rows = ring_rows(ring::Wide::BM, ring::Wide::WTM, ring::direct_cfg<ring::Wide>()); break;
      case 5: case 6: slot_rows = ring_rows(ring::Mid8::BM, ring::Mid8::WTM, ring::direct_cfg<ring::Mid8>()); break;
      case 4: slot_rows = ring_rows(ring::Half::BM, ring::Half::WTM, ring::direct_cfg<ring::Half>()); break;
      case 3: slot_rows = ring_rows(ring::Tall::BM, ring::Tall::WTM, ring::direct_cfg<ring::Tall>()); break;
      case 2: slot_rows = ring_rows(ring::Big::BM, ring::Big::WTM, ring::direct_cfg<ring::Big>()); break;
      case 1: slot_rows = ring_rows(ring::Mid::BM, ring::Mid::WTM, ring::direct_cfg<ring::Mid>()); break;
      default: slot_rows = BM; break;                      // register-staged kernel: per 128-row M tile
    }
  }
  // (slab rows: grid batch z x per-batch slots; batches > 1 only when they share the output vectors: vec_z_inner 0)
  const int64_t nslots = want_cs ? a.batch * cdiv(a.M, slot_rows) : 0;
  const bool slab = want_cs && (a.batch == 1 || a.vec_z_inner == 0) && a.workspace &&
                    a.workspace_bytes >= 2 * nslots * a.N * 4;
  DPH_REQUIRE(!want_cs || slab || !deterministic(),
              "dph_gemm: deterministic mode needs the column-sum workspace (>= 2 * batch * cdiv(M, 64) * N fp32; batch "
              "> 1 only with shared output vectors, vec_z_inner 0)");
  DphGemmArgs b = a;
  if (slab) b.flags |= GEMM_COLSUM_SLAB;
  if (use_sk) {
    DPH_TRY(sk_launch(b, skp, stream));
  } else if (kind >= 12 && kind <= 16) {
    DPH_REQUIRE(cdiv(a.M, 128) < 65536 && a.batch < 65536, "dph_gemm: grid too large");
    if (kind == 12) launch_pp<pp::P256>(b, stream);
    else if (kind == 13) launch_pp<pp::P128x256>(b, stream);
    else if (kind == 14) launch_pp<pp::P256x128>(b, stream);
    else if (kind == 15) {
      if (pp_b0pf() && cdiv(a.M, 128) * cdiv(a.N, 192) * a.batch <= num_cus()) launch_pp<pp::P128x192::PF>(b, stream);
      else if (pp_m2(a)) launch_pp<pp::P128x192::M2>(b, stream);
      else launch_pp<pp::P128x192>(b, stream);
    } else {
      launch_pp<pp::P128>(b, stream);
    }
  } else if (kind == 10) {
    DPH_REQUIRE(cdiv(a.M, ring::Tri::BM) < 65536 && a.batch * a.splits < 65536, "dph_gemm: grid too large");
    if (!launch_ring_persist<ring::Tri>(b, stream)) launch_ring<ring::Tri, false>(b, kchunk, stream);
  } else if (kind == 8) {
    DPH_REQUIRE(cdiv(a.M, ring::Flat::BM) < 65536 && a.batch * a.splits < 65536, "dph_gemm: grid too large");
    if (!launch_ring_persist<ring::Flat>(b, stream)) launch_ring<ring::Flat, false>(b, kchunk, stream);
  } else if (kind == 7) {
    DPH_REQUIRE(cdiv(a.M, ring::Wide::BM) < 65536 && a.batch * a.splits < 65536, "dph_gemm: grid too large");
    if (!launch_ring_persist<ring::Wide>(b, stream)) launch_ring<ring::Wide, false>(b, kchunk, stream);
  } else if (kind == 6) {
    DPH_REQUIRE(cdiv(a.M, ring::Mid8::BM) < 65536 && a.batch * a.splits < 65536, "dph_gemm: grid too large");
    launch_ring<ring::Mid8, true>(b, kchunk, stream);
  } else if (kind == 5) {
    DPH_REQUIRE(cdiv(a.M, ring::Mid8::BM) < 65536 && a.batch * a.splits < 65536, "dph_gemm: grid too large");
    launch_ring<ring::Mid8, false>(b, kchunk, stream);
  } else if (kind == 4) {
    DPH_REQUIRE(cdiv(a.M, ring::Half::BM) < 65536 && a.batch * a.splits < 65536, "dph_gemm: grid too large");
    launch_ring<ring::Half, false>(b, kchunk, stream);
  } else if (kind == 3) {
    DPH_REQUIRE(cdiv(a.M, ring::Tall::BM) < 65536 && a.batch * a.splits < 65536, "dph_gemm: grid too large");
    launch_ring<ring::Tall, false>(b, kchunk, stream);
  } else if (kind == 2) {
    DPH_REQUIRE(cdiv(a.M, ring::Big::BM) < 65536 && a.batch * a.splits < 65536, "dph_gemm: grid too large");
    launch_ring<ring::Big, false>(b, kchunk, stream);
  } else if (kind == 1) {
    DPH_REQUIRE(cdiv(a.M, ring::Mid::BM) < 65536 && a.batch * a.splits < 65536, "dph_gemm: grid too large");
    if (a.a_kcontig && a.b_kcontig) launch_ring<ring::Mid, false>(b, kchunk, stream);
    else launch_ring<ring::Mid, true>(b, kchunk, stream);
  } else {
  dim3 grid((unsigned)cdiv(a.N, BN), (unsigned)cdiv(a.M, BM), (unsigned)(a.batch * a.splits));
  DPH_REQUIRE(grid.y < 65536 && grid.z < 65536, "dph_gemm: grid too large");
  // split-K on the register-staged kernel: slices are combined inside the launch by the last-arriving
  // block of each tile when the workspace carries the per-tile tickets (zeroed here, reset by the
  // combining block)
  unsigned* cnt = nullptr;
  if (a.splits > 1) {
    const int64_t slab = (int64_t)a.batch * a.splits * a.M * a.N * 4;
    const int64_t tiles = (int64_t)grid.x * grid.y * a.batch;
    if (a.workspace_bytes >= slab + tiles * 4) {
      cnt = reinterpret_cast<unsigned*>(reinterpret_cast<char*>(a.workspace) + slab);
      zero_async(cnt, tiles * 4, stream);
    }
  }
  if (small_nt(kchunk) == 512) {
    if (a.a_kcontig && a.b_kcontig)
      hipLaunchKernelGGL((gemm_kernel<true, true, 512>), grid, dim3(512), 0, stream, b, kchunk, cnt);
    else if (a.a_kcontig && !a.b_kcontig)
      hipLaunchKernelGGL((gemm_kernel<true, false, 512>), grid, dim3(512), 0, stream, b, kchunk, cnt);
    else if (!a.a_kcontig && a.b_kcontig)
      hipLaunchKernelGGL((gemm_kernel<false, true, 512>), grid, dim3(512), 0, stream, b, kchunk, cnt);
    else
      hipLaunchKernelGGL((gemm_kernel<false, false, 512>), grid, dim3(512), 0, stream, b, kchunk, cnt);
  } else {
  if (a.a_kcontig && a.b_kcontig)
    hipLaunchKernelGGL((gemm_kernel<true, true>), grid, dim3(NTHREADS), 0, stream, b, kchunk, cnt);
  else if (a.a_kcontig && !a.b_kcontig)
    hipLaunchKernelGGL((gemm_kernel<true, false>), grid, dim3(NTHREADS), 0, stream, b, kchunk, cnt);
  else if (!a.a_kcontig && a.b_kcontig)
    hipLaunchKernelGGL((gemm_kernel<false, true>), grid, dim3(NTHREADS), 0, stream, b, kchunk, cnt);
  else
    hipLaunchKernelGGL((gemm_kernel<false, false>), grid, dim3(NTHREADS), 0, stream, b, kchunk, cnt);
  }
  if (cnt != nullptr) return check_launch("dph_gemm");
  }
  int rc = check_launch("dph_gemm");
  if (rc) return rc;
  if (slab) {
    const int64_t csn = std::min<int64_t>(a.colsum_n > 0 ? a.colsum_n : a.N, a.N);
    // (>= 16 slab rows per group: a few hundred blocks even at N = 768, each thread's rows in flight together;
    // deterministic mode: each column's rows in a fixed order)
    if (colred_deferring()) {
      const float* sl = reinterpret_cast<const float*>(a.workspace);
      DPH_TRY(colred_push(sl, nslots, a.N, csn, a.colsum_out, stream));
      DPH_TRY(colred_push(sl + nslots * a.N, nslots, a.N, csn, a.colsum_aux, stream));
    } else if (deterministic()) {
      hipLaunchKernelGGL(colsum_slab_reduce_det_kernel, dim3((unsigned)cdiv(csn, 32)), dim3(32 * DET_PH), 0, stream,
                         reinterpret_cast<const float*>(a.workspace), nslots, a.N, csn, a.colsum_out, a.colsum_aux);
    } else {
      const unsigned groups = (unsigned)std::max<int64_t>(1, std::min<int64_t>(32, cdiv(nslots, 16)));
      hipLaunchKernelGGL(colsum_slab_reduce_kernel, dim3((unsigned)cdiv(csn, 64), groups), dim3(256), 0, stream,
                         reinterpret_cast<const float*>(a.workspace), nslots, a.N, csn, a.colsum_out, a.colsum_aux);
    }
    return check_launch("dph_gemm colsum reduce");
  }
  if (a.splits > 1) {
    const int64_t work = a.M * cdiv(a.N, 8);
    dim3 g2((unsigned)cdiv(work, 256), 1, (unsigned)a.batch);
    hipLaunchKernelGGL(splitk_reduce_kernel, g2, dim3(256), 0, stream, a, DphGemmGroup{});
    rc = check_launch("dph_gemm splitk_reduce");
  }
  return rc;
}

extern "C" int dph_gemm_grouped(const DphGemmArgs* args, const DphGemmGroup* group, hipStream_t stream) {
  DPH_REQUIRE(args != nullptr && group != nullptr, "dph_gemm_grouped: null args");
  const DphGemmGroup& g = *group;
  DPH_REQUIRE(g.n >= 1 && g.n <= DPH_GEMM_GROUP_MAX, "dph_gemm_grouped: group size %d outside 1..%d", g.n,
              DPH_GEMM_GROUP_MAX);
  DphGemmArgs a = *args;
  DPH_REQUIRE(a.M > 0 && a.N > 0 && a.K > 0 && a.splits >= 1, "dph_gemm_grouped: bad sizes");
  DPH_REQUIRE(a.batch == g.n, "dph_gemm_grouped: batch (%d) must equal the group size (%d)", a.batch, g.n);
  DPH_REQUIRE(!a.a_kcontig && !a.b_kcontig, "dph_gemm_grouped: (mn, mn) operands only");
  uintptr_t al = 0;
  for (int i = 0; i < g.n; ++i) {
    DPH_REQUIRE(g.a[i] && g.b[i] && g.c[i], "dph_gemm_grouped: null operand of problem %d", i);
    al |= reinterpret_cast<uintptr_t>(g.a[i]) | reinterpret_cast<uintptr_t>(g.b[i]) |
          (a.splits == 1 ? reinterpret_cast<uintptr_t>(g.c[i]) : 0);
  }
  if ((al & 15) != 0) {
    set_error("dph_gemm_grouped: operands not 16-byte aligned");
    return DPH_EUNSUPPORTED;
  }
  for (DphMat* d : {&a.A, &a.B, &a.C}) {
    d->batch_stride = 0;
    d->z_div = 0;
    d->z_outer = 0;
    d->z_inner = 0;
  }
  a.A.ptr = const_cast<void*>(g.a[0]);
  a.B.ptr = const_cast<void*>(g.b[0]);
  a.C.ptr = g.c[0];
  if (a.splits > 1) {
    const int64_t need = (int64_t)a.batch * a.splits * a.M * a.N * 4;
    DPH_REQUIRE(a.workspace && a.workspace_bytes >= need, "dph_gemm_grouped: split-K workspace too small (%lld < %lld)",
                (long long)a.workspace_bytes, (long long)need);
  }
  const PpwPlan pw = ppw_route(a);
  if (!pw.kind || pw.splits != a.splits) {
    set_error("dph_gemm_grouped: no ping-pong weight-gradient plan for these args");
    return DPH_EUNSUPPORTED;
  }
  return run_ppw(a, pw, g, stream);
}

extern "C" int dph_gemm_sk_plan(const DphGemmArgs* args, int64_t* ws_bytes, int64_t* nflags) {
  if (ws_bytes) *ws_bytes = 0;
  if (nflags) *nflags = 0;
  if (!args || args->M <= 0 || args->N <= 0 || args->K <= 0) return 0;
  dph::SkPlan p;
  if (!sk_route(*args, &p)) return 0;
  if (ws_bytes) *ws_bytes = dph::sk_ws_bytes(p);
  if (nflags) *nflags = dph::sk_nflags(p);
  return 1;
}
