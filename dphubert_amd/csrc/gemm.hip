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
//   k-contiguous  ([rows][K]): LDS image [128][64+8] (16-B row pad, conflict
//                 free for the 16-lane ds_read_b128 groups), fragments by
//                 ds_read_b128.
//   mn-contiguous ([K][rows]): LDS image [64][128] with a 32-B XOR swizzle
//                 (unit ^= (k&3)|((k>>3)&1)<<2, conflict free for the two
//                 8-row halves of a transposed read), fragments by the gfx950
//                 hardware transpose read ds_read_b64_tr_b16 -- no explicit
//                 transposes of activations or weights anywhere.
// The MFMA is issued "swapped" (B-tile fragment as the A operand) so each
// lane ends up holding 4 CONSECUTIVE output columns of one row: 8-B (bf16)
// or 16-B (fp32) stores and cheap per-column epilogue vectors.
#include "common.h"

#include <stdarg.h>
#include <stdio.h>

namespace dph {

namespace {
constexpr int BM = 128;
constexpr int BN = 128;
constexpr int BK = 64;
constexpr int NTHREADS = 256;
constexpr int KROW = BK + 8;                  // k-contig LDS row (elements)
constexpr int LDS_KC = 128 * KROW * 2;        // bytes, k-contig tile
constexpr int LDS_MN = BK * 128 * 2;          // bytes, mn-contig tile

template <bool KC>
struct TileBytes {
  static constexpr int v = KC ? LDS_KC : LDS_MN;
};

__device__ __forceinline__ int64_t row_addr(const DphMat& d, int64_t r) {
  if (d.rows_per_batch > 0) return (r / d.rows_per_batch) * d.batch_stride + (r % d.rows_per_batch) * d.row_stride;
  return r * d.row_stride;
}

__device__ __forceinline__ int64_t z_addr(const DphMat& d, int64_t z) {
  if (d.z_div > 0) return (z / d.z_div) * d.z_outer + (z % d.z_div) * d.z_inner;
  return z * d.z_inner;
}

__device__ __forceinline__ int swz(int k) { return (k & 3) | (((k >> 3) & 1) << 2); }

// ---- staging: global -> registers ----------------------------------------
template <bool KC>
struct Stager {
  const bf16_t* base;   // operand base incl. batch offset
  int64_t roff[4];      // k-contig: per-chunk row offsets (fixed per block)
  bool rvalid[4];
  int64_t r0;           // first row/col of the tile (M or N index)
  int64_t R;            // rows (M or N)
  DphMat d;

  __device__ void init(const DphMat& dm, const bf16_t* b, int64_t tile0, int64_t Rn, int tid) {
    d = dm;
    base = b;
    r0 = tile0;
    R = Rn;
    if constexpr (KC) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        int c = tid + NTHREADS * i;
        int64_t r = tile0 + (c >> 3);
        rvalid[i] = r < Rn;
        roff[i] = rvalid[i] ? row_addr(dm, r) : 0;
      }
    }
  }

  __device__ void load(uint4 (&reg)[4], int64_t k0, int64_t kend, int tid) const {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int c = tid + NTHREADS * i;
      uint4 v = make_uint4(0, 0, 0, 0);
      if constexpr (KC) {
        int64_t k = k0 + (c & 7) * 8;
        if (rvalid[i] && k < kend) v = *reinterpret_cast<const uint4*>(base + roff[i] + k);
      } else {
        int64_t k = k0 + (c >> 4);
        int64_t col = r0 + (c & 15) * 8;
        if (k < kend && col < R) v = *reinterpret_cast<const uint4*>(base + row_addr(d, k) + col);
      }
      reg[i] = v;
    }
  }

  __device__ void store(char* lds, const uint4 (&reg)[4], int tid) const {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int c = tid + NTHREADS * i;
      int byte;
      if constexpr (KC) {
        byte = ((c >> 3) * KROW + (c & 7) * 8) * 2;
      } else {
        int kr = c >> 4;
        int col8 = c & 15;
        int u = (col8 >> 1) ^ swz(kr);
        byte = kr * 256 + u * 32 + (col8 & 1) * 16;
      }
      *reinterpret_cast<uint4*>(lds + byte) = reg[i];
    }
  }
};

// ---- fragments: LDS -> registers --------------------------------------------
// Returns the MFMA operand fragment for rows [rb, rb+16) of the tile and
// k-substep ks: lane l holds X[row rb + (l&15)][k = ks*32 + 8*(l>>4) + j].
template <bool KC>
__device__ __forceinline__ bf16x8_t frag(const char* lds, int rb, int ks, int lane) {
  if constexpr (KC) {
    int row = rb + (lane & 15);
    int col = ks * 32 + 8 * (lane >> 4);
    return *reinterpret_cast<const bf16x8_t*>(lds + (row * KROW + col) * 2);
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
struct EpiAcc {
  float out[4];
  float aux[4];
};

// Apply the epilogue to 4 consecutive columns [n, n+4) of row m (batch z).
// Returns the stored values (for column sums) in acc.out / acc.aux.
__device__ __forceinline__ void epilogue4(const DphGemmArgs& a, int64_t z, int64_t m, int64_t n, float (&v)[4],
                                          EpiAcc& cs) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    cs.out[i] = 0.f;
    cs.aux[i] = 0.f;
  }
  if (m >= a.M || n >= a.N) return;
  const int64_t voff = (a.C.z_div > 0 ? (z % a.C.z_div) : z) * a.vec_z_inner;
  const int64_t coff = z_addr(a.C, z) + row_addr(a.C, m) + n;
  const bool full = (n + 4 <= a.N);
  const int nv = full ? 4 : (int)(a.N - n);
  const float inv_keep = a.dropout_p > 0.f ? 1.0f / (1.0f - a.dropout_p) : 1.0f;
  const uint64_t drow = ((uint64_t)(z * a.M + a.drop_row_offset + m)) * (uint64_t)a.N;
  bool zero_row = false;
  if (a.row_len) {
    int64_t b = m / a.len_rows;
    zero_row = (m % a.len_rows) >= a.row_len[b];
  }
  float pre[4], aux[4] = {0.f, 0.f, 0.f, 0.f}, res[4] = {0.f, 0.f, 0.f, 0.f};
  if (a.aux_in) {
    const bf16_t* p = reinterpret_cast<const bf16_t*>(a.aux_in) + coff;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (i < nv) aux[i] = bf2f(p[i]);
  }
  if (a.residual) {
    const bf16_t* p = reinterpret_cast<const bf16_t*>(a.residual) + coff;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (i < nv) res[i] = bf2f(p[i]);
  }
  const float sm = a.smask ? *a.smask : 1.0f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t nn = (i < nv) ? n + i : n;
    float x = v[i] * a.alpha;
    if (a.bias) x += a.bias[voff + nn];
    pre[i] = x;
    const float dz = dropout_scale(a.seed, drow + nn, a.dropout_p, inv_keep);
    float cm = a.colmask ? a.colmask[voff + nn] : 1.0f;
    float ax = 0.f;
    if (a.act == DPH_ACT_GELU) {
      x = gelu_f(x) * dz * cm;
    } else if (a.act == DPH_ACT_GELU_BWD) {
      const float gz = x * dz;
      ax = gz * gelu_f(aux[i]);
      x = gz * gelu_grad_f(aux[i]) * cm;
    } else {
      x = x * dz * cm;
    }
    x = x * sm + res[i];
    if (zero_row) x = 0.f;
    v[i] = x;
    cs.out[i] = (i < nv) ? x : 0.f;
    cs.aux[i] = (i < nv) ? ax : 0.f;
  }
  if (a.pre_out) {
    bf16_t* p = reinterpret_cast<bf16_t*>(a.pre_out) + coff;
    if (full) {
      *reinterpret_cast<uint2*>(p) = make_uint2(pack2bf(pre[0], pre[1]), pack2bf(pre[2], pre[3]));
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (i < nv) p[i] = f2bf(pre[i]);
    }
  }
  if (a.c_dtype == DPH_OUT_BF16) {
    bf16_t* p = reinterpret_cast<bf16_t*>(a.C.ptr) + coff;
    if (full) {
      *reinterpret_cast<uint2*>(p) = make_uint2(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]));
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (i < nv) p[i] = f2bf(v[i]);
    }
  } else {
    float* p = reinterpret_cast<float*>(a.C.ptr) + coff;
    if (a.c_dtype == DPH_OUT_F32_ACCUM) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (i < nv) p[i] += v[i];
    } else if (full) {
      *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (i < nv) p[i] = v[i];
    }
  }
}

template <bool AK, bool BKc>
__global__ void __launch_bounds__(NTHREADS, 2) gemm_kernel(const DphGemmArgs a, int64_t kchunk) {
  __shared__ __attribute__((aligned(16))) char smem[2 * (TileBytes<AK>::v + TileBytes<BKc>::v)];
  char* const ldsA0 = smem;
  char* const ldsB0 = smem + 2 * TileBytes<AK>::v;
#define LDSA(buf) (ldsA0 + (buf) * TileBytes<AK>::v)
#define LDSB(buf) (ldsB0 + (buf) * TileBytes<BKc>::v)

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1;
  const int wn = wave & 1;

  const int64_t zz = blockIdx.z;
  const int64_t split = zz % a.splits;
  const int64_t z = zz / a.splits;
  const int64_t m0 = (int64_t)blockIdx.y * BM;
  const int64_t n0 = (int64_t)blockIdx.x * BN;
  const int64_t kbeg = split * kchunk;
  const int64_t kend = min(a.K, kbeg + kchunk);

  Stager<AK> sa;
  Stager<BKc> sb;
  sa.init(a.A, reinterpret_cast<const bf16_t*>(a.A.ptr) + z_addr(a.A, z), m0, a.M, tid);
  sb.init(a.B, reinterpret_cast<const bf16_t*>(a.B.ptr) + z_addr(a.B, z), n0, a.N, tid);

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  uint4 ra[4], rb[4];
  const int nk = (int)cdiv(max<int64_t>(kend - kbeg, 0), BK);
  if (nk > 0) {
    sa.load(ra, kbeg, kend, tid);
    sb.load(rb, kbeg, kend, tid);
    sa.store(LDSA(0), ra, tid);
    sb.store(LDSB(0), rb, tid);
  }
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    const int cur = t & 1;
    const bool more = (t + 1) < nk;
    if (more) {
      sa.load(ra, kbeg + (int64_t)(t + 1) * BK, kend, tid);
      sb.load(rb, kbeg + (int64_t)(t + 1) * BK, kend, tid);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8_t af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = frag<AK>(LDSA(cur), wm * 64 + 16 * i, ks, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = frag<BKc>(LDSB(cur), wn * 64 + 16 * j, ks, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
    if (more) {
      sa.store(LDSA(cur ^ 1), ra, tid);
      sb.store(LDSB(cur ^ 1), rb, tid);
    }
    __syncthreads();
  }

#undef LDSA
#undef LDSB
  // lane holds C[m = rowbase + (lane&15)][n = colbase + 4*(lane>>4) + r]
  if (a.splits > 1) {
    float* ws = reinterpret_cast<float*>(a.workspace) + (zz * a.M) * a.N;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t m = m0 + wm * 64 + 16 * i + (lane & 15);
      if (m >= a.M) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t n = n0 + wn * 64 + 16 * j + 4 * (lane >> 4);
        if (n + 4 <= a.N) {
          *reinterpret_cast<float4*>(ws + m * a.N + n) = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2],
                                                                      acc[i][j][3]);
        } else {
          for (int r = 0; r < 4 && n + r < a.N; ++r) ws[m * a.N + n + r] = acc[i][j][r];
        }
      }
    }
    return;
  }

  const bool want_cs = (a.colsum_out != nullptr) || (a.colsum_aux != nullptr);
  float cso[4][4], csa[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      cso[j][r] = 0.f;
      csa[j][r] = 0.f;
    }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t m = m0 + wm * 64 + 16 * i + (lane & 15);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t n = n0 + wn * 64 + 16 * j + 4 * (lane >> 4);
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      EpiAcc cs;
      epilogue4(a, z, m, n, v, cs);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        cso[j][r] += cs.out[r];
        csa[j][r] += cs.aux[r];
      }
    }
  }
  if (want_cs) {
    const int64_t voff = (a.C.z_div > 0 ? (z % a.C.z_div) : z) * a.vec_z_inner;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float so = cso[j][r], sx = csa[j][r];
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          so += __shfl_xor(so, o, 64);
          sx += __shfl_xor(sx, o, 64);
        }
        const int64_t n = n0 + wn * 64 + 16 * j + 4 * (lane >> 4) + r;
        if ((lane & 15) == 0 && n < a.N) {
          if (a.colsum_out) atomicAdd(a.colsum_out + voff + n, so);
          if (a.colsum_aux) atomicAdd(a.colsum_aux + voff + n, sx);
        }
      }
  }
}

// split-K reduction + epilogue: one thread per 4 columns
__global__ void splitk_reduce_kernel(const DphGemmArgs a) {
  const int64_t z = blockIdx.z;
  const int64_t n4 = (a.N + 3) / 4;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= a.M * n4) return;
  const int64_t m = idx / n4;
  const int64_t n = (idx % n4) * 4;
  const float* ws = reinterpret_cast<const float*>(a.workspace);
  float v[4] = {0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < a.splits; ++s) {
    const float* p = ws + ((z * a.splits + s) * a.M + m) * a.N + n;
    for (int r = 0; r < 4; ++r)
      if (n + r < a.N) v[r] += p[r];
  }
  EpiAcc cs;
  epilogue4(a, z, m, n, v, cs);
}

}  // namespace

}  // namespace dph

using namespace dph;

extern "C" int dph_gemm(const DphGemmArgs* args, hipStream_t stream) {
  DPH_REQUIRE(args != nullptr, "dph_gemm: null args");
  const DphGemmArgs& a = *args;
  DPH_REQUIRE(a.M > 0 && a.N > 0 && a.K > 0, "dph_gemm: bad sizes M=%lld N=%lld K=%lld", (long long)a.M,
              (long long)a.N, (long long)a.K);
  DPH_REQUIRE(a.batch >= 1 && a.splits >= 1, "dph_gemm: batch/splits must be >= 1");
  DPH_REQUIRE(a.A.ptr && a.B.ptr && a.C.ptr, "dph_gemm: null operand");
  DPH_REQUIRE(a.K % 8 == 0 || !a.a_kcontig, "dph_gemm: k-contiguous A needs K %% 8 == 0 (K=%lld)", (long long)a.K);
  DPH_REQUIRE(a.K % 8 == 0 || !a.b_kcontig, "dph_gemm: k-contiguous B needs K %% 8 == 0 (K=%lld)", (long long)a.K);
  DPH_REQUIRE(a.a_kcontig || a.M % 8 == 0, "dph_gemm: mn-contiguous A needs M %% 8 == 0");
  DPH_REQUIRE(a.b_kcontig || a.N % 8 == 0, "dph_gemm: mn-contiguous B needs N %% 8 == 0");
  DPH_REQUIRE(a.act != DPH_ACT_GELU_BWD || a.aux_in, "dph_gemm: GELU_BWD needs aux_in");
  DPH_REQUIRE(!a.row_len || a.len_rows > 0, "dph_gemm: row_len needs len_rows");
  int64_t kchunk = a.K;
  if (a.splits > 1) {
    DPH_REQUIRE(!a.colsum_out && !a.colsum_aux, "dph_gemm: column sums not supported with split-K");
    kchunk = cdiv(cdiv(a.K, a.splits), BK) * BK;
    const int64_t need = (int64_t)a.batch * a.splits * a.M * a.N * 4;
    DPH_REQUIRE(a.workspace && a.workspace_bytes >= need, "dph_gemm: split-K workspace too small (%lld < %lld)",
                (long long)a.workspace_bytes, (long long)need);
  }
  dim3 grid((unsigned)cdiv(a.N, BN), (unsigned)cdiv(a.M, BM), (unsigned)(a.batch * a.splits));
  DPH_REQUIRE(grid.y < 65536 && grid.z < 65536, "dph_gemm: grid too large");
  if (a.a_kcontig && a.b_kcontig)
    hipLaunchKernelGGL((gemm_kernel<true, true>), grid, dim3(NTHREADS), 0, stream, a, kchunk);
  else if (a.a_kcontig && !a.b_kcontig)
    hipLaunchKernelGGL((gemm_kernel<true, false>), grid, dim3(NTHREADS), 0, stream, a, kchunk);
  else if (!a.a_kcontig && a.b_kcontig)
    hipLaunchKernelGGL((gemm_kernel<false, true>), grid, dim3(NTHREADS), 0, stream, a, kchunk);
  else
    hipLaunchKernelGGL((gemm_kernel<false, false>), grid, dim3(NTHREADS), 0, stream, a, kchunk);
  int rc = check_launch("dph_gemm");
  if (rc) return rc;
  if (a.splits > 1) {
    const int64_t work = a.M * cdiv(a.N, 4);
    dim3 g2((unsigned)cdiv(work, 256), 1, (unsigned)a.batch);
    hipLaunchKernelGGL(splitk_reduce_kernel, g2, dim3(256), 0, stream, a);
    rc = check_launch("dph_gemm splitk_reduce");
  }
  return rc;
}
