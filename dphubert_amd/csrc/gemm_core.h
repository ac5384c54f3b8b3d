// Device-side building blocks shared by the GEMM translation units (gemm.hip: every GEMM path and the host
// dispatch; gemm_sk.hip: the persistent stream-K ping-pong kernel): DphMat addressing, the LDS-DMA helper, the
// register epilogue of the ping-pong / ring kernels and the ping-pong tile configurations.
#pragma once
#include "common.h"

#include <type_traits>

#ifndef DPH_STAMP
#define DPH_STAMP 0         // diagnostic build: per-block s_memtime stamps into a.workspace (tools/stamp_gemm.py)
#endif
#define DPH_TSTAMP(v)                                                                     \
  do {                                                                                    \
    if (DPH_STAMP) {                                                                      \
      __builtin_amdgcn_sched_barrier(0);                                                  \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory");            \
      __builtin_amdgcn_sched_barrier(0);                                                  \
    }                                                                                     \
  } while (0)

namespace dph {
namespace {
// internal DphGemmArgs.flags bit set by dph_gemm: column sums go to a workspace slab of per-tile / per-wave partial
// rows (see the epilogues) instead of float atomics
constexpr int64_t GEMM_COLSUM_SLAB = (int64_t)1 << 20;

// internal epilogue variant: DPH_ACT_GELU under DPH_GEMM_PRE_DGK (pre_out stores gelu'(pre)*mask*keep/(1-p))
constexpr int ACT_GELU_DGKPRE = 16;

__device__ __forceinline__ int64_t row_addr(const DphMat& d, int64_t r) {
  if (d.rows_per_batch > 0) return (r / d.rows_per_batch) * d.batch_stride + (r % d.rows_per_batch) * d.row_stride;
  return r * d.row_stride;
}

// row_addr for row indices < 2^31 (32-bit division: the 64-bit one is a ~40-instruction routine)
__device__ __forceinline__ int64_t row_addr32(const DphMat& d, uint32_t r) {
  if (d.rows_per_batch > 0) {
    const uint32_t q = r / (uint32_t)d.rows_per_batch;
    return (int64_t)q * d.batch_stride + (int64_t)(r - q * (uint32_t)d.rows_per_batch) * d.row_stride;
  }
  return (int64_t)r * d.row_stride;
}

__device__ __forceinline__ int64_t z_addr(const DphMat& d, int64_t z) {
  if (d.z_div > 0) return (z / d.z_div) * d.z_outer + (z % d.z_div) * d.z_inner;
  return z * d.z_inner;
}

namespace ring {
__device__ __forceinline__ void dma16(const bf16_t* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

// ---- direct (register) epilogue -------------------------------------------------------------
// The MFMA is issued B-first, so lane l holds, of accumulator fragment (i, j), the 4 consecutive
// columns n = nw + 16 j + 4 (l >> 4) .. +3 of row m = mw + 16 i + (l & 15).  Each lane finishes and
// stores those values straight from its registers: no LDS staging, no block barrier.  The code is
// kept lean because the epilogue is instruction-issue bound: one 64-bit base per lane, fragment
// offsets i * 16 * row_stride + 16 j (the j part folds into the store's immediate offset), 32-bit
// row-segment arithmetic, column sums over the 16 rows of a lane group by DPP adds (the first
// version -- 64-bit row_addr / row-length divisions and ds_bpermute shuffles -- compiled to ~2900
// instructions per wave and measured 11-13k cycles per 128 x 256 tile, as long as half a K = 768
// main loop).  Every global input (bias / colmask per column group, aux / residual per element) is
// issued before the first store, so the wait on them never covers a store (gfx9 counts stores in
// vmcnt).  Preconditions (direct_epi_ok): N % 4 == 0 (a 4-column group is wholly inside or outside N),
// C rows addressed as m * row_stride or by the batched row layout, 4-element aligned strides, 16-B aligned
// pointers, at most one of aux_in / residual, M * N and the row-length segments within 32 bits.
__host__ __device__ __forceinline__ bool direct_epi_ok(const DphGemmArgs& a) {
  const int64_t calign = a.C.row_stride | a.C.batch_stride | a.C.z_outer | a.C.z_inner | a.N | a.vec_z_inner;
  const uintptr_t palign = reinterpret_cast<uintptr_t>(a.C.ptr) | reinterpret_cast<uintptr_t>(a.pre_out) |
                           reinterpret_cast<uintptr_t>(a.aux_in) | reinterpret_cast<uintptr_t>(a.residual) |
                           reinterpret_cast<uintptr_t>(a.bias) | reinterpret_cast<uintptr_t>(a.colmask);
  const bool dgk = a.act == DPH_ACT_GELU_BWD_DGK;
  return (calign & 3) == 0 && (palign & 15) == 0 && (dgk ? a.aux_in != nullptr : !(a.aux_in && a.residual)) &&
         a.M < ((int64_t)1 << 31) && (!a.row_len || a.len_rows > 0) &&
         (a.act == DPH_ACT_GELU_BWD || dgk || (!a.colsum_out && !a.colsum_aux));   // column sums: GELU backward only
}

__device__ __forceinline__ void unpack_bf16x4(const uint2 r, float (&o)[4]) {
  o[0] = __uint_as_float(r.x << 16);
  o[1] = __uint_as_float(r.x & 0xffff0000u);
  o[2] = __uint_as_float(r.y << 16);
  o[3] = __uint_as_float(r.y & 0xffff0000u);
}

// sum over the 16 lanes of a DPP row (lane bits 0..3); every lane of the row gets the sum
__device__ __forceinline__ float row16_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xb1, 0xf, 0xf, false));    // quad_perm 1,0,3,2
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4e, 0xf, 0xf, false));    // quad_perm 2,3,0,1
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x124, 0xf, 0xf, false));   // row_ror 4
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x128, 0xf, 0xf, false));   // row_ror 8
  return v;
}

// Returns true when the check-free copy ran: then the wave issued exactly FM*FN stores of C (plus FM*FN of
// pre_out when requested) and no other memory operation is left outstanding (the persistent kernel's
// counted waits rely on it).
// WIDE (ping-pong kernels): in the check-free bf16 copy, the 4-column groups of fragment pairs (j, j + 1) are
// exchanged between lane groups g and g ^ 1 (v_permlane16_swap_b32: odd 16-lane rows of the group-j register with
// the even rows of the group-(j+1) register), so each lane stores 8 consecutive columns with one 16-B store
// instead of two 8-B ones (the store tail is issue-bound: guide T21).  Not for the persistent ring kernel, whose
// counted waits assume one store per fragment.
template <class C, int ACT, bool DROP, bool WIDE = false>
__device__ __forceinline__ bool direct_epi_t(const DphGemmArgs& a, int64_t z, int64_t mw, int64_t nw, int lane,
                                             const f32x4_t (&acc)[C::FM][C::FN]) {
  constexpr int FM = C::FM, FN = C::FN;
  const int64_t N = a.N;
  const int32_t M = (int32_t)a.M;
  const int64_t rs = a.C.row_stride;
  const int32_t ml = (int32_t)mw + (lane & 15);
  const int64_t nl = nw + 4 * (lane >> 4);
  const bool nfull = nw + C::WTN <= N;          // wave-uniform: every column group in range
  const bool mfull = mw + C::WTM <= a.M;
  const int64_t voff = (a.C.z_div > 0 ? (z % a.C.z_div) : z) * a.vec_z_inner;
  // element offset of fragment row i (columns nl..): rows m * row_stride, or the batched row layout
  // (b = m / rows_per_batch: the conv input-gradient phase GEMMs write every other row of each utterance)
  const bool rpb = a.C.rows_per_batch > 0;
  const int64_t zb = z_addr(a.C, z) + nl;
  const int64_t rstep = 16 * rs;
  const int64_t r0off = rpb ? 0 : (int64_t)ml * rs;
  // (the lean copy never has a batched row layout: its rows are a plain stride, no division per row)
  auto roff = [&](int i, auto ck) -> int64_t {
    if constexpr (decltype(ck)::value)
      return zb + (rpb ? row_addr32(a.C, (uint32_t)(ml + 16 * i)) : r0off + i * rstep);
    else
      return zb + r0off + i * rstep;
  };
  const int64_t base = zb + r0off;   // (rpb == 0)
  // (arithmetic select of the two pointer VALUES, as in tile_epi_rows)
  const uintptr_t ax_p = reinterpret_cast<uintptr_t>(a.aux_in), rs_p = reinterpret_cast<uintptr_t>(a.residual);
  // an fp32 residual (DPH_GEMM_RESID_F32: the pre-norm residual stream) is read in the checked copy below, not
  // through the bf16 per-element input
  const bool res32 = (a.flags & DPH_GEMM_RESID_F32) != 0;
  const uintptr_t rs_b = rs_p & (uintptr_t)(-(intptr_t)!res32);
  const bf16_t* inp = reinterpret_cast<const bf16_t*>(ax_p | (rs_b & (uintptr_t)(-(intptr_t)(ax_p == 0))));
  const bool has_in = inp != nullptr, has_res = has_in && ax_p == 0;
  // (column sums are compiled for the GELU backward variants only: the only GEMMs that request them)
  constexpr bool BWD = ACT == DPH_ACT_GELU_BWD || ACT == DPH_ACT_GELU_BWD_DGK;
  constexpr bool DGK = ACT == DPH_ACT_GELU_BWD_DGK;
  const bool colsum = BWD && (a.colsum_out || a.colsum_aux);
  // per-column factors: bias, csm = colmask * layer mask
  float bias[FN][4], csm[FN][4];
  const float sm = a.smask ? *a.smask : 1.0f;
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    float4 b = make_float4(0.f, 0.f, 0.f, 0.f), c = make_float4(1.f, 1.f, 1.f, 1.f);
    if (nfull || nl + 16 * j < N) {
      if (a.bias) b = *reinterpret_cast<const float4*>(a.bias + voff + nl + 16 * j);
      if (a.colmask) c = *reinterpret_cast<const float4*>(a.colmask + voff + nl + 16 * j);
    }
    bias[j][0] = b.x; bias[j][1] = b.y; bias[j][2] = b.z; bias[j][3] = b.w;
    csm[j][0] = c.x * sm; csm[j][1] = c.y * sm; csm[j][2] = c.z * sm; csm[j][3] = c.w * sm;
  }
  if constexpr (DGK) {
    // the mask gradient divides the stored forward output by its column mask (f = gelu * mask * keep/(1-p))
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) csm[j][r] = csm[j][r] != 0.f ? 1.0f / csm[j][r] : 0.f;
  }
  const float inv_keep = DROP ? 1.0f / (1.0f - a.dropout_p) : 1.0f;
  const uint32_t thr = DROP ? drop_thr(a.dropout_p) : 0u;
  const uint64_t seed = DROP ? epoch_seed(a.seed) : 0;
  // per-element inputs of every fragment, issued together
  // (loaded two rows ahead inside the fragment loop: at most two rows of inputs are live, 16 VGPRs
  // instead of 32 -- the persistent kernel's GELU_BWD variant spilled with all of them preloaded)
  uint2 in[FM][FN], in2[DGK ? FM : 1][DGK ? FN : 1];
  (void)base;
  const bf16_t* inp2 = reinterpret_cast<const bf16_t*>(rs_p);      // DGK: the forward's output f (optional)
  const bool has_in2 = DGK && inp2 != nullptr;
  auto load_in = [&](int i, auto ck) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      in[i][j] = make_uint2(0, 0);
      if constexpr (DGK) in2[i][j] = make_uint2(0, 0);
      if (has_in && (mfull || ml + 16 * i < M) && (nfull || nl + 16 * j < N)) {
        in[i][j] = *reinterpret_cast<const uint2*>(inp + roff(i, ck) + 16 * j);
        if constexpr (DGK) {
          if (has_in2) in2[i][j] = *reinterpret_cast<const uint2*>(inp2 + roff(i, ck) + 16 * j);
        }
      }
    }
  };
  // rows past their row_len segment store zeros: 32-bit segment / remainder of the first row, stepped by 16
  uint32_t zrow = 0;                                   // bit i: row i is a zero row
  if (a.row_len) {
    const uint32_t L = (uint32_t)a.len_rows;
    uint32_t seg = (uint32_t)ml / L, rem = (uint32_t)ml - seg * L;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      if (i) {
        rem += 16;
        while (rem >= L) rem -= L, ++seg;
      }
      if (ml + 16 * i < M && (int64_t)rem >= a.row_len[seg]) zrow |= 1u << i;
    }
  }
  float cso[FN][4], csa[FN][4];
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) cso[j][r] = csa[j][r] = 0.f;
  const bool out_bf16 = a.c_dtype == DPH_OUT_BF16, accum = a.c_dtype == DPH_OUT_F32_ACCUM;
  char* cb = reinterpret_cast<char*>(a.C.ptr);
  char* pb = reinterpret_cast<char*>(a.pre_out);
  const uint64_t e_base = ((uint64_t)(z * a.M + a.drop_row_offset + ml)) * (uint64_t)N + (uint64_t)nl;
  // CK: bounds and zero-row checks, any output type (edge tiles, row_len, fp32 outputs); interior tiles
  // with a bf16 output run the check-free copy
  // (WIDE: 16-B aligned rows are needed for the widened stores -- row stride % 8 == 0; wave-uniform)
  const bool wide = WIDE && (rs & 7) == 0;
  auto frags = [&](auto ck) {
    constexpr bool CK = decltype(ck)::value;
    const bool obf = !CK || out_bf16;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      uint2 opk[FN], ppk[FN];   // (WIDE, !CK: this row's packed outputs, stored after the column loop)
      if (i == 0) {
        load_in(0, ck);
        if (FM > 1) load_in(1, ck);
      }
      if (i + 2 < FM) load_in(i + 2, ck);
      if (CK && !mfull && ml + 16 * i >= M) continue;
      const bool zero_row = CK && ((zrow >> i) & 1u);
      const int64_t ro = roff(i, ck);
      char* crow = cb + ro * (obf ? 2 : 4);
      char* prow = pb + ro * 2;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        if (CK && !nfull && nl + 16 * j >= N) continue;
        float v[4], pre[4], ax[4], xin[4], xin2[4];
        unpack_bf16x4(in[i][j], xin);
        if constexpr (DGK) unpack_bf16x4(in2[i][j], xin2);
        if constexpr (!BWD && CK) {
          if (res32) {
            const float4 q = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(rs_p) + ro + 16 * j);
            xin[0] += q.x; xin[1] += q.y; xin[2] += q.z; xin[3] += q.w;
          }
        }
        uint32_t keep = 0xfu;
        if constexpr (DROP) {
          // element e_base + 16 i N + 16 j is even (N % 4 == 0, n % 4 == 0): pairs e/2 and e/2 + 1
          const uint64_t pr = (e_base + (uint64_t)(16 * i) * (uint64_t)N + 16 * j) >> 1;
          const uint32_t b0 = drop_bits2(seed, pr), b1 = drop_bits2(seed, pr + 1);
          keep = ((b0 & 0xffffu) >= thr ? 1u : 0u) | ((b0 >> 16) >= thr ? 2u : 0u) |
                 ((b1 & 0xffffu) >= thr ? 4u : 0u) | ((b1 >> 16) >= thr ? 8u : 0u);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          pre[r] = fmaf(acc[i][j][r], a.alpha, bias[j][r]);
          const bool k = (keep >> r) & 1u;
          ax[r] = 0.f;
          if constexpr (ACT == DPH_ACT_GELU) {
            v[r] = k ? gelu_f(pre[r]) * (csm[j][r] * inv_keep) : 0.f;
          } else if constexpr (ACT == ACT_GELU_DGKPRE) {
            // the stored "pre" is the backward's factor gelu'(pre) * mask * keep / (1 - p)
            float g, dg;
            gelu_and_grad(pre[r], g, dg);
            const float kk = k ? csm[j][r] * inv_keep : 0.f;
            v[r] = g * kk;
            pre[r] = dg * kk;
          } else if constexpr (DGK) {
            ax[r] = pre[r] * xin2[r] * csm[j][r];
            v[r] = pre[r] * xin[r];
          } else if constexpr (ACT == DPH_ACT_GELU_BWD) {
            const float gz = DROP ? (k ? pre[r] * inv_keep : 0.f) : pre[r];
            float g, dg;
            gelu_and_grad(xin[r], g, dg);
            ax[r] = gz * g;
            v[r] = gz * dg * csm[j][r];
          } else {
            v[r] = DROP ? (k ? pre[r] * (csm[j][r] * inv_keep) : 0.f) : pre[r] * csm[j][r];
          }
          // residual: xin is zero without one (the backward variants' xin is their aux input, never a residual)
          if constexpr (!BWD) v[r] += xin[r];
          if (CK) v[r] = zero_row ? 0.f : v[r];
        }
        if (colsum) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            cso[j][r] += v[r];
            if constexpr (BWD) csa[j][r] += ax[r];   // (not zeroed on zero rows, as epilogue8)
          }
        }
#ifdef DPH_EPI_NOSTORE
        asm volatile("" ::"v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(pre[0]));
        continue;
#endif
        if (WIDE && !CK && wide) {
          opk[j] = make_uint2(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]));
          if (a.pre_out) ppk[j] = make_uint2(pack2bf(pre[0], pre[1]), pack2bf(pre[2], pre[3]));
          continue;
        }
        if (a.pre_out) *reinterpret_cast<uint2*>(prow + 32 * j) = make_uint2(pack2bf(pre[0], pre[1]), pack2bf(pre[2], pre[3]));
        if (obf) {
          *reinterpret_cast<uint2*>(crow + 32 * j) = make_uint2(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]));
        } else {
          float4* q = reinterpret_cast<float4*>(crow + 64 * j);
          if (accum) {
            const float4 old = *q;
            v[0] += old.x; v[1] += old.y; v[2] += old.z; v[3] += old.w;
          }
          *q = make_float4(v[0], v[1], v[2], v[3]);
        }
      }
#ifndef DPH_EPI_NOSTORE
      if constexpr (WIDE && !CK) {
        if (wide) {
          // lane group g stores columns 16 (j + (g & 1)) + 8 (g >> 1) .. + 7 of the pair (j, j + 1)
          const int g = lane >> 4;
          const int off = 32 * (g & 1) + 16 * (g >> 1) - 8 * g;   // bytes, relative to this lane's column nl
          auto st_pairs = [&](char* rowp, uint2 (&pk)[FN]) {
#pragma unroll
            for (int j = 0; j + 1 < FN; j += 2) {
              const auto rx = __builtin_amdgcn_permlane16_swap(pk[j].x, pk[j + 1].x, false, false);
              const auto ry = __builtin_amdgcn_permlane16_swap(pk[j].y, pk[j + 1].y, false, false);
              *reinterpret_cast<uint4*>(rowp + 32 * j + off) = make_uint4(rx[0], ry[0], rx[1], ry[1]);
            }
            if constexpr (FN % 2 == 1) *reinterpret_cast<uint2*>(rowp + 32 * (FN - 1)) = pk[FN - 1];
          };
          const int64_t ro = roff(i, ck);
          if (a.pre_out) st_pairs(pb + ro * 2, ppk);
          st_pairs(cb + ro * 2, opk);
        }
      }
#endif
    }
  };
  const bool lean = mfull && nfull && !a.row_len && out_bf16 && !rpb && !res32;
  if (lean) frags(std::false_type{});
  else frags(std::true_type{});
  if (colsum) {
    // lanes 0, 16, 32, 48 hold the sums of their 4-column groups: one slab entry (COLSUM_SLAB: slab row
    // mw / WTM, summed by colsum_slab_reduce_kernel) or one atomic per column per wave
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        cso[j][r] = row16_sum(cso[j][r]);
        if constexpr (BWD) csa[j][r] = row16_sum(csa[j][r]);
      }
    if ((lane & 15) == 0 && (a.flags & GEMM_COLSUM_SLAB)) {
      const int64_t csn = min(a.colsum_n > 0 ? a.colsum_n : N, N);
      if (mw < a.M) {
        const int64_t nslots = cdiv(a.M, (int64_t)C::WTM);
        float* wo = reinterpret_cast<float*>(a.workspace) + (z * nslots + mw / C::WTM) * N;
        float* wa = wo + a.batch * nslots * N;
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int64_t n = nl + 16 * j + r;
            if (n >= csn) continue;
            wo[n] = cso[j][r];
            if constexpr (BWD) wa[n] = csa[j][r];
          }
      }
    } else if ((lane & 15) == 0) {
      const int64_t csn = a.colsum_n > 0 ? a.colsum_n : N;
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t n = nl + 16 * j + r;
          if (n >= csn || n >= N) continue;
          if (a.colsum_out) atomicAdd(a.colsum_out + voff + n, cso[j][r]);
          if (BWD && a.colsum_aux) atomicAdd(a.colsum_aux + voff + n, csa[j][r]);
        }
    }
  }
  return lean && !colsum;
}
}  // namespace ring

namespace pp {
constexpr int BK = 64;

template <int BM_, int BN_>
struct Cfg {
  static constexpr int BM = BM_, BN = BN_;
  static constexpr int NW = 8, NT = 512, WGM = 2, WGN = 4;
  static constexpr int WTM = BM / 2, WTN = BN / 4;
  static constexpr int FM = WTM / 16, FN = WTN / 16;
  static constexpr int FM2 = FM / 2, FN0 = (FN + 1) / 2, FN1 = FN / 2;
  static constexpr int RA = BM / 2, RB0 = 64 * FN0, RB1 = 64 * FN1;     // half-tile rows
  static constexpr int GA = RA / 64, GB0 = RB0 / 64, GB1 = RB1 / 64;    // LDS-DMA per thread per half-tile
  static constexpr int G = 2 * GA + GB0 + GB1;                          // per K-tile
  static constexpr int O_ALO = 0, O_AHI = RA * 128, O_B0 = 2 * RA * 128, O_B1 = O_B0 + RB0 * 128;
  static constexpr int BUF = (BM + BN) * 128;
  static constexpr int LDS = 2 * BUF;
  // two blocks per CU only for the small tiles (the 128 x 192 GELU epilogues spilled at the 128-VGPR cap)
  static constexpr int MINB = (LDS <= 80 * 1024 && FM * FN <= 8) ? 2 : 1;
  static constexpr int WPE = MINB * 2;                                  // waves per SIMD
  // the A-lo fragments of K-tile u + 1 read in K-tile u's last interval (pp_gemm_kernel): taken where it measured
  // faster -- the 256-row tiles (8192^3 on 256 x 256: 2382 -> 2124 cycles per K-tile) and 128 x 128; the 128 x 192
  // projection shapes ran 2-3 % slower with it (tools/stamp_pp.py, profiles/r5_pp_loop_stamps.txt)
  static constexpr bool SPLITA = BM_ == 256 || (BM_ == 128 && BN_ == 128);
  // the next K-tile's B-n0 fragments read in the last interval (pp_gemm_kernel): the PF variant below
  static constexpr bool B0PF = false;
  struct PF;
  struct M2;
  static_assert(FM % 2 == 0 && FN >= 2 && RA % 64 == 0 && G < 16, "pp tile geometry");
};
// Cfg::PF: the B-n0 prefetch schedule of pp_gemm_kernel (tiles without the A-lo split).  Taken for ONE-ROUND
// grids: their K-tile loop is the whole launch (7984 x 768 x 3072 on 128 x 192: 44.8 -> 40.3 us), while on
// multi-round grids its extra registers (126 -> 202 VGPRs) keep the second block off the CU (QKV forward
// 35.1 -> 40.0 us, profiles/r5_pp_b0pf_ab.txt)
template <int BM_, int BN_>
struct Cfg<BM_, BN_>::PF : Cfg<BM_, BN_> {
  static_assert(!Cfg<BM_, BN_>::SPLITA, "B-n0 prefetch: tiles without the A-lo split");
  static constexpr bool B0PF = true;
};
// Cfg::M2: two blocks per CU (4 waves per SIMD: <= 128 VGPRs) for a tile that otherwise gets one -- the 128 x 192
// tile on multi-round grids, so one block's prologue / epilogue overlaps the other's main loop (A/B: DPH_PP_M2)
template <int BM_, int BN_>
struct Cfg<BM_, BN_>::M2 : Cfg<BM_, BN_> {
  static_assert(Cfg<BM_, BN_>::LDS <= 80 * 1024, "two blocks per CU: LDS");
  static constexpr int MINB = 2;
  static constexpr int WPE = 4;
};
using P256 = Cfg<256, 256>;
using P128x256 = Cfg<128, 256>;
using P256x128 = Cfg<256, 128>;
using P128x192 = Cfg<128, 192>;
using P128 = Cfg<128, 128>;

template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x70 | 0xF00);
}
__device__ __forceinline__ void lgkm0() { __builtin_amdgcn_s_waitcnt(0xC07F); }
__device__ __forceinline__ void bar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// 16 x 32 operand fragment of ksub s from a half-tile image: rows rb..rb+15 (rb % 16 == 0)
__device__ __forceinline__ bf16x8_t hfrag(const char* ht, int rb, int s, int lane) {
  const int row = rb + (lane & 15);
  const int phys = (s * 4 + (lane >> 4)) ^ ((lane & 15) >> 1);
  return *reinterpret_cast<const bf16x8_t*>(ht + row * 128 + phys * 16);
}

#ifndef DPH_PP_ABL
#define DPH_PP_ABL 0   // diagnostic builds only (tools/stamp_pp.py): 1 = no main-loop DMAs, 2 = no main-loop MFMAs,
#endif              // 3 = no main-loop LDS reads, 4 = no main-loop barriers, 5 = reads + barriers only, 6 = MFMAs +
                    // barriers only (timing ablations: the results are garbage)
#define PP_ABL_DMA (DPH_PP_ABL == 1 || DPH_PP_ABL == 5 || DPH_PP_ABL == 6)
#define PP_ABL_MFMA (DPH_PP_ABL == 2 || DPH_PP_ABL == 5)
#define PP_ABL_READ (DPH_PP_ABL == 3 || DPH_PP_ABL == 6)
#define PP_ABL_BAR (DPH_PP_ABL == 4)
// One ping-pong main loop (see pp_gemm_kernel): K-tiles 0 .. nk - 1 (nk >= 2) of the BM x BN tile at (m0, n0) of the
// operands whose first column is Ab / Bb (the caller applies the batch and K offsets), accumulated into acc.  Starts
// with the prologue's DMAs, ends with the two wave groups re-paired by a barrier: every LDS read of the loop is
// complete, so the caller may stage into either buffer right after it.
template <class C>
__device__ __forceinline__ void mainloop(const DphGemmArgs& a, const bf16_t* Ab, const bf16_t* Bb, int64_t m0,
                                         int64_t n0, int nk, f32x4_t (&acc)[C::FM][C::FN], char* smem, int wave,
                                         int lane, unsigned long long& st1) {
  (void)st1;
  const int wr = wave >> 2, wc = wave & 3;
  // DMA sources (element offsets, < 2^31: checked on the host) of instruction jj of each half-tile kind:
  // wave instruction gi = jj * 8 + wave fills half-tile rows gi*8 .. +7, lane -> row gi*8 + lane/8,
  // physical chunk lane % 8 <- logical k-chunk (lane % 8) ^ ((row >> 1) & 7)
  uint32_t oal[C::GA], oah[C::GA], ob0[C::GB0], ob1[C::GB1];
  constexpr int HA = C::WTM / 2;
#pragma unroll
  for (int jj = 0; jj < C::GA; ++jj) {
    const int rho = (jj * 8 + wave) * 8 + (lane >> 3);
    const int lc = (lane & 7) ^ ((rho >> 1) & 7);
    const int trow = (rho / HA) * C::WTM + rho % HA;
    oal[jj] = (uint32_t)(row_addr32(a.A, (uint32_t)min<int64_t>(m0 + trow, a.M - 1)) + lc * 8);
    oah[jj] = (uint32_t)(row_addr32(a.A, (uint32_t)min<int64_t>(m0 + trow + HA, a.M - 1)) + lc * 8);
  }
#pragma unroll
  for (int jj = 0; jj < C::GB0; ++jj) {
    const int rho = (jj * 8 + wave) * 8 + (lane >> 3);
    const int lc = (lane & 7) ^ ((rho >> 1) & 7);
    const int tcol = (rho / (16 * C::FN0)) * C::WTN + rho % (16 * C::FN0);
    ob0[jj] = (uint32_t)(row_addr32(a.B, (uint32_t)min<int64_t>(n0 + tcol, a.N - 1)) + lc * 8);
  }
#pragma unroll
  for (int jj = 0; jj < C::GB1; ++jj) {
    const int rho = (jj * 8 + wave) * 8 + (lane >> 3);
    const int lc = (lane & 7) ^ ((rho >> 1) & 7);
    const int tcol = (rho / (16 * C::FN1)) * C::WTN + 16 * C::FN0 + rho % (16 * C::FN1);
    ob1[jj] = (uint32_t)(row_addr32(a.B, (uint32_t)min<int64_t>(n0 + tcol, a.N - 1)) + lc * 8);
  }
  auto buf = [&](int u) -> char* { return smem + (u & 1) * C::BUF; };
  // (DPH_PP_ABL == 1: DMAs past the prologue's two K-tiles are not issued -- a timing ablation on stale operands)
  auto dma_on = [&](int u) { return !PP_ABL_DMA || u < 2; };
  auto st_alo = [&](int u) {
    if (!dma_on(u)) return;
#pragma unroll
    for (int jj = 0; jj < C::GA; ++jj) ring::dma16(Ab + oal[jj] + (int64_t)u * BK, buf(u) + C::O_ALO + (jj * 8 + wave) * 1024);
  };
  auto st_ahi = [&](int u) {
    if (!dma_on(u)) return;
#pragma unroll
    for (int jj = 0; jj < C::GA; ++jj) ring::dma16(Ab + oah[jj] + (int64_t)u * BK, buf(u) + C::O_AHI + (jj * 8 + wave) * 1024);
  };
  auto st_b0 = [&](int u) {
    if (!dma_on(u)) return;
#pragma unroll
    for (int jj = 0; jj < C::GB0; ++jj) ring::dma16(Bb + ob0[jj] + (int64_t)u * BK, buf(u) + C::O_B0 + (jj * 8 + wave) * 1024);
  };
  auto st_b1 = [&](int u) {
    if (!dma_on(u)) return;
#pragma unroll
    for (int jj = 0; jj < C::GB1; ++jj) ring::dma16(Bb + ob1[jj] + (int64_t)u * BK, buf(u) + C::O_B1 + (jj * 8 + wave) * 1024);
  };

  // A fragments of the tile's low and high row halves in separate registers: the low half of K-tile u + 1 is read
  // during K-tile u's last (A-high x B-n0) interval -- its half-tile landed two intervals earlier -- so every
  // interval carries at most FM2 * 2 or FN0 * 2 fragment reads (4 / 2 / 4 / 4 on the 128 x 192 tile instead of
  // 8 / 2 / 4 / 0, whose 8-read interval left the next MFMA cluster waiting on its LDS reads)
  bf16x8_t falo[C::FM2][2] = {}, fa_hi_[C::FM2][2] = {}, fb0x[C::FN0][2] = {}, fb0y[C::FN0][2] = {}, fb1[C::FN1][2] = {};
  bf16x8_t (&fahi)[C::FM2][2] = C::SPLITA ? fa_hi_ : falo;   // one A fragment set where the split is not taken
  // Cfg::B0PF: the B-n0 fragments of K-tile u + 1 are read in K-tile u's last interval, beside its A-hi x B-n0
  // cluster (two register sets, alternating per K-tile): its half-tile landed by that interval's counted wait
  // (issued one K-tile earlier), so no wait moves -- the 8-read first interval of a K-tile becomes a 4-read one
  constexpr bool B0PF = C::B0PF;

  auto rd_a = [&](const char* ht, bf16x8_t (&fa)[C::FM2][2]) {
    if (PP_ABL_READ) return;
#pragma unroll
    for (int i = 0; i < C::FM2; ++i)
#pragma unroll
      for (int s = 0; s < 2; ++s) fa[i][s] = hfrag(ht, wr * HA + 16 * i, s, lane);
  };
  auto rd_b0 = [&](const char* bu, bf16x8_t (&fb0)[C::FN0][2]) {
    if (PP_ABL_READ) return;
#pragma unroll
    for (int j = 0; j < C::FN0; ++j)
#pragma unroll
      for (int s = 0; s < 2; ++s) fb0[j][s] = hfrag(bu + C::O_B0, wc * 16 * C::FN0 + 16 * j, s, lane);
  };
  auto rd_b1 = [&](const char* bu) {
    if (PP_ABL_READ) return;
#pragma unroll
    for (int j = 0; j < C::FN1; ++j)
#pragma unroll
      for (int s = 0; s < 2; ++s) fb1[j][s] = hfrag(bu + C::O_B1, wc * 16 * C::FN1 + 16 * j, s, lane);
  };
  // MFMA cluster: rows [i0, i0 + FM2) (fragments fa) x the given B fragment set
  auto mm0 = [&](int i0, const bf16x8_t (&fa)[C::FM2][2], const bf16x8_t (&fb0)[C::FN0][2]) {
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
  auto mm1 = [&](int i0, const bf16x8_t (&fa)[C::FM2][2]) {
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
  constexpr int G = C::G;
  auto lbar = [&]() {
    if (!PP_ABL_BAR) bar();
  };
  // prologue: the half-tiles of "phases" -6 .. -1 (A-lo(0), B-n0(0), B-n1(0), A-hi(0), A-lo(1), B-n0(1)),
  // then wait for A-lo(0) and B-n0(0)
  if constexpr (B0PF) {   // (B-n0 staged before A-lo: see kstep)
    st_b0(0);
    st_alo(0);
    st_b1(0);
    st_ahi(0);
    st_b0(1);
    st_alo(1);
  } else {
    st_alo(0);
    st_b0(0);
    st_b1(0);
    st_ahi(0);
    st_alo(1);
    st_b0(1);
  }
  vm_wait<G>();
  bar();
  DPH_TSTAMP(st1);
  if constexpr (C::SPLITA) rd_a(buf(0) + C::O_ALO, falo);
  if constexpr (B0PF) rd_b0(buf(0), fb0x);
  if (wr == 1) bar();            // group 1 runs one interval behind group 0
  // one K-tile of the main loop; fbc: this tile's B-n0 fragments, fbn: the next tile's (B0PF)
  auto kstep = [&](int u, bf16x8_t (&fbc)[C::FN0][2], bf16x8_t (&fbn)[C::FN0][2]) {
    const char* bu = buf(u);
    // j = 0
    if constexpr (!B0PF) rd_b0(bu, fbc);
    if constexpr (!C::SPLITA) rd_a(bu + C::O_ALO, falo);
    st_b1(u + 1);
    vm_wait<G>();
    lbar();
    lgkm0();
    __builtin_amdgcn_sched_barrier(0);
    mm0(0, falo, fbc);
    lbar();
    // j = 1
    rd_b1(bu);
    st_ahi(u + 1);
    vm_wait<G>();
    lbar();
    lgkm0();
    __builtin_amdgcn_sched_barrier(0);
    mm1(0, falo);
    lbar();
    // j = 2 (B0PF: B-n0(u + 2) here and A-lo(u + 2) at j = 3, so that B-n0(u + 1) is retired by THIS wait -- in
    // both wave groups by the barrier after group 0's j = 3 wait, where group 0 reads it)
    rd_a(bu + C::O_AHI, fahi);
    if constexpr (B0PF) st_b0(u + 2);
    else st_alo(u + 2);
    vm_wait<G>();
    lbar();
    lgkm0();
    __builtin_amdgcn_sched_barrier(0);
    mm1(C::FM2, fahi);
    lbar();
    // j = 3 (SPLITA: A-lo(u + 1) landed by the vm_wait of j = 2, visible after its barrier; not waited for here.
    // B0PF: B-n0(u + 1), issued at j = 2 of K-tile u - 1, retired by both groups' j = 2 waits: group 0 reads it
    // after the barrier that pairs its j = 3 wait with group 1's j = 2 wait, group 1 one interval later)
    if constexpr (C::SPLITA) rd_a(buf(u + 1) + C::O_ALO, falo);
    if constexpr (B0PF) st_alo(u + 2);
    else st_b0(u + 2);
    vm_wait<G>();
    lbar();
    if constexpr (B0PF) {
      rd_b0(buf(u + 1), fbn);
      __builtin_amdgcn_sched_barrier(0);   // (issued ahead of the cluster, not sunk below it)
    }
    mm0(C::FM2, fahi, fbc);
    lbar();
  };
  // the last two K-tiles: nothing staged past nk - 1, the counted waits drain
  auto tail = [&](int u, bf16x8_t (&fbc)[C::FN0][2], bf16x8_t (&fbn)[C::FN0][2]) {
#pragma unroll
    for (int t = 0; t < 2; ++t, ++u) {
      const bool second_last = t == 0;
      const char* bu = buf(u);
      bf16x8_t (&fb)[C::FN0][2] = (B0PF && t == 1) ? fbn : fbc;
      if constexpr (!B0PF) rd_b0(bu, fb);
      if constexpr (!C::SPLITA) rd_a(bu + C::O_ALO, falo);
      if (second_last) {
        st_b1(u + 1);
        vm_wait<G>();
      } else {
        vm_wait<C::GA>();
      }
      lbar();
      lgkm0();
      __builtin_amdgcn_sched_barrier(0);
      mm0(0, falo, fb);
      lbar();
      rd_b1(bu);
      if (second_last) {
        st_ahi(u + 1);
        vm_wait<G>();
      } else {
        vm_wait<0>();
      }
      lbar();
      lgkm0();
      __builtin_amdgcn_sched_barrier(0);
      mm1(0, falo);
      lbar();
      rd_a(bu + C::O_AHI, fahi);
      if (second_last) {
        if constexpr (B0PF) vm_wait<C::GB1 + C::GA>();   // B-n0(u + 1) and A-lo(u + 1) retired
        else vm_wait<G - C::GA>();
      } else {
        vm_wait<0>();
      }
      lbar();
      lgkm0();
      __builtin_amdgcn_sched_barrier(0);
      mm1(C::FM2, fahi);
      lbar();
      if (second_last) {
        if constexpr (C::SPLITA) rd_a(buf(u + 1) + C::O_ALO, falo);   // (landed by the j = 2 wait above)
        vm_wait<C::GB1 + C::GA>();   // (B-n0(u + 1), issued one K-tile earlier, is done)
      } else {
        vm_wait<0>();
      }
      lbar();
      if (B0PF && second_last) {
        rd_b0(buf(u + 1), fbn);
        __builtin_amdgcn_sched_barrier(0);
      }
      mm0(C::FM2, fahi, fb);
      lbar();
    }
  };
  int u = 0;
  if constexpr (B0PF) {
#pragma unroll 1
    for (; u + 3 < nk; u += 2) {
      kstep(u, fb0x, fb0y);
      kstep(u + 1, fb0y, fb0x);
    }
    if (u + 2 < nk) {
      kstep(u, fb0x, fb0y);
      tail(u + 1, fb0y, fb0x);
    } else {
      tail(u, fb0x, fb0y);
    }
  } else {
#pragma unroll 1
    for (; u + 2 < nk; ++u) kstep(u, fb0x, fb0x);
    tail(u, fb0x, fb0x);
  }
  if (wr == 0) bar();            // pairs with group 1's extra barrier
}
}  // namespace pp
}  // namespace
}  // namespace dph

namespace dph {
// stream-K partition (gemm_sk.hip): ntm x ntn tiles of 256 x 256, nk 64-deep K-tiles each (even), nblk blocks;
// block b's iteration range starts at 2 * floor(b * half / nblk), half = ntm * ntn * nk / 2
struct SkPlan {
  int32_t ntm, ntn, nk, nblk;
  int64_t half;
};
bool sk_plan(const DphGemmArgs& a, int cus, SkPlan* out);
int64_t sk_ws_bytes(const SkPlan& p);
int64_t sk_nflags(const SkPlan& p);
int sk_launch(const DphGemmArgs& a, const SkPlan& p, hipStream_t stream);
const char* sk_variant(const DphGemmArgs& a);
}  // namespace dph
