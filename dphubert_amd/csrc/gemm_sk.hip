// Persistent stream-K ping-pong GEMM on 256 x 256 tiles (gfx950).
//
// The M = B*T projections with a wide N -- QKV forward (N = 2304), FFN1 forward and the FFN2 input gradient
// (N = 3072, the GELU / GELU' epilogues), all at K = 768 (components.py:406-408, :733-741) -- have 288 / 384
// 256 x 256 tiles: 1.1 / 1.5 rounds over the 256 CUs, which a one-tile-per-block grid pays as two whole rounds, so
// they ran on the narrower 128 x 192 / 128 x 128 tiles, whose main loops are bound by the L2 -> LDS operand stream
// (40 KB per 128 x 192 K-tile: ~52 B/clk/CU at the MFMA rate).  The 256 x 256 tile streams 32 B/clk/CU and
// runs its main loop at the MFMA rate (2124 cycles per K-tile against 2048 of MFMA work, profiles/r5_pp_loop_stamps.txt).
//
// Stream-K: the tiles' 64-deep K-tiles form one iteration space (tile-major), cut into nblk equal ranges at even
// K-tile indices (every piece of a tile holds >= 2 K-tiles, as the ping-pong prologue / tail need); one block per CU
// walks its range.  A range therefore starts with the LAST K-tiles of a tile (a "tail" piece) and ends with the FIRST
// K-tiles of another (a "head" piece), with whole tiles between.
//   * whole tile: main loop, register epilogue (bias / GELU / dropout / GELU' factor / column-sum slab rows).
//   * tail piece (a block's first segment, k0 > 0): its fp32 partial goes to the block's slot of the hand-off buffer
//     by write-through (sc1) stores; every wave drains them (vmcnt 0), the block meets at a barrier, one lane sets the
//     block's flag by an agent-scope atomic store (cdna_hip_programming.md 6, Guideline 16, R1).
//   * head piece (k0 == 0, the block's LAST segment): the tile's owner.  The tail pieces of its tile are the FIRST
//     segments of the following blocks, so they finished long before; the owner polls each flag (one lane, relaxed,
//     bounded spin), reads each partial with sc1 loads (every load of a handed-off byte, no acquire fence needed) and
//     adds them in block order -- a fixed order, so the result is deterministic -- then runs the epilogue.
// Producers never wait, so the grid cannot deadlock whatever the dispatch order or the CUs another stream holds (the
// concurrent teacher forward): an owner only ever waits for a block that, once running, finishes its tail piece
// without waiting.  The flags come zeroed from the caller (ops zero arena: a fresh slice per call, re-zeroed by the
// graph's fill node on every replay), so no in-kernel reset is needed.
// Logical block b of physical block id: XCD-major (ids x, x + 8, ... run on XCD x and take consecutive ranges, so a
// tail piece's producer and its owner usually share an XCD; placement is a speed hint only -- the hand-off protocol
// does not depend on it).
#include "gemm_core.h"

#include <string.h>

namespace dph {
namespace {
namespace sk {
using C = pp::P256;
constexpr int TILE_F = C::BM * C::BN;       // floats per partial slot
constexpr int NACC = C::FM * C::FN;         // f32x4 accumulators per lane

typedef int v4i_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) int32_t gi32;

__host__ __device__ __forceinline__ int64_t seg_start(const SkPlan& p, int64_t b) {
  return 2 * ((b * p.half) / p.nblk);
}

// tile t (0 .. ntm*ntn-1) -> output origin: groups of GM = 4 M tiles walked N-major (the pp kernels' order)
__device__ __forceinline__ void tile_mn(const SkPlan& p, uint32_t t, int64_t& m0, int64_t& n0) {
  constexpr uint32_t GM = 4;
  const uint32_t ntm = (uint32_t)p.ntm, ntn = (uint32_t)p.ntn;
  const uint32_t gsz = GM * ntn;
  const uint32_t grp = t / gsz;
  const uint32_t gm0 = grp * GM;
  const uint32_t gh = min(GM, ntm - gm0);
  const uint32_t l = t - grp * gsz;
  const uint32_t lq = l / gh;
  m0 = (int64_t)(gm0 + (l - lq * gh)) * C::BM;
  n0 = (int64_t)lq * C::BN;
}

template <int ACT, bool DROP>
__global__ void __launch_bounds__(C::NT, C::WPE) sk_gemm_kernel(const DphGemmArgs a, const SkPlan p) {
  __shared__ __attribute__((aligned(1024))) char smem[C::LDS];
  const int tid = threadIdx.x;
  const int lane0 = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int bid = (int)blockIdx.x;
  const int b = (p.nblk % 8 == 0) ? (bid & 7) * (p.nblk >> 3) + (bid >> 3) : bid;
  int64_t it = seg_start(p, b);
  const int64_t end = seg_start(p, b + 1);
  gi32* flags = (gi32*)(a.sk_flags);
  // (lofs: this lane's byte offset inside a partial slot -- accumulator s of wave w at ((w * NACC + s) * 64 + lane)
  // * 16, so each store / load instruction moves one contiguous KB)
  unsigned long long st1 = 0;
  // DPH_STAMP diagnostic build (tools/stamp_sk.py): per logical block 16 int64 slots in a.workspace -- [0] start,
  // per segment s < 5: [1 + 3s] main loop entry (after a head piece's wait), [2 + 3s] loop done, [3 + 3s] segment done
  int nseg = 0;
  unsigned long long stv = 0;
  auto stamp = [&](int slot) {
    DPH_TSTAMP(stv);
    if (DPH_STAMP && tid == 0 && slot < 16) reinterpret_cast<unsigned long long*>(a.workspace)[b * 16 + slot] = stv;
  };
  stamp(0);
#pragma unroll 1
  while (it < end) {
    // (lane made opaque per segment: keeps the compiler from hoisting lane-derived DMA offsets and epilogue
    // addresses out of the segment loop, where they would stay live across the main loop and spill)
    int lane = lane0;
    asm volatile("" : "+v"(lane));
    const int lofs = (wave * NACC * 64 + lane) * 16;
    const int64_t t = it / p.nk;
    const int k0 = (int)(it - t * p.nk);
    const int k1 = (int)min<int64_t>(p.nk, (int64_t)k0 + (end - it));
    int64_t m0, n0;
    tile_mn(p, (uint32_t)t, m0, n0);
    f32x4_t acc[C::FM][C::FN];
    if (k0 == 0 && k1 < p.nk) {
      // head piece: the accumulators start from the tile's tail piece -- the first segment of block b + 1 (sk_plan
      // gives every block at least nk + 2 K-tiles, so a tile is cut at most once), finished long before this block
      // reaches its last segment.  Loaded before the main loop rather than added after it: the accumulators then
      // have one definition at the loop entry (an add after the loop made the register allocator spill the tail).
      const int q = b + 1;
      if (tid == 0) {
        uint32_t spins = 0;
        while (__hip_atomic_load(flags + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
          __builtin_amdgcn_s_sleep(2);
          if (++spins == (1u << 22)) {   // ~0.5 s: a lost producer -- flag the launch and go on (no hang)
            __hip_atomic_store(flags + p.nblk, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      __syncthreads();
      const auto rs = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<float*>(a.sk_ws) + (int64_t)q * TILE_F,
                                                        (short)0, TILE_F * 4, 0x00020000);
#pragma unroll
      for (int i = 0; i < C::FM; ++i)
#pragma unroll
        for (int j = 0; j < C::FN; ++j)
          acc[i][j] = __builtin_bit_cast(f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(
                                                      rs, lofs + (i * C::FN + j) * 1024, 0, 16 /* sc1 */));
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (the main loop's counted waits assume no older loads)
    } else {
#pragma unroll
      for (int i = 0; i < C::FM; ++i)
#pragma unroll
        for (int j = 0; j < C::FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    }
    stamp(1 + 3 * nseg);
    const bf16_t* Ab = reinterpret_cast<const bf16_t*>(a.A.ptr) + (int64_t)k0 * pp::BK;
    const bf16_t* Bb = reinterpret_cast<const bf16_t*>(a.B.ptr) + (int64_t)k0 * pp::BK;
    pp::mainloop<C>(a, Ab, Bb, m0, n0, k1 - k0, acc, smem, wave, lane, st1);
    // (compiler-only memory barrier: the epilogue's bias / mask / input loads must not be hoisted above the main loop,
    // where their registers would be live beside the fragments and accumulators)
    asm volatile("" ::: "memory");
    stamp(2 + 3 * nseg);
    if (k0 > 0) {
      // tail piece -> slot b (write-through), drained by every wave, then the flag
      const auto rs = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<float*>(a.sk_ws) + (int64_t)b * TILE_F,
                                                        (short)0, TILE_F * 4, 0x00020000);
#pragma unroll
      for (int i = 0; i < C::FM; ++i)
#pragma unroll
        for (int j = 0; j < C::FN; ++j)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i_t, acc[i][j]), rs,
                                                 lofs + (i * C::FN + j) * 1024, 0, 16 /* sc1 */);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) __hip_atomic_store(flags + b, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      ring::direct_epi_t<C, ACT, DROP, true>(a, 0, m0 + wr * C::WTM, n0 + wc * C::WTN, lane, acc);
    }
    stamp(3 + 3 * nseg);
    ++nseg;
    it += k1 - k0;
  }
}
}  // namespace sk
}  // namespace

// ---- host side (declared in gemm_core.h; called by dph_gemm / dph_gemm_sk_plan in gemm.hip) ----
// The stream-K route: k-contiguous operands on the ping-pong layout (pp_ok), one batch, no split-K / device-side
// extents, K a multiple of 128 (an even K-tile count), a wide N (>= 2048: the shapes above), at least one 256 x 256
// tile per block pair.  OFF by default -- DPH_GEMM_SK=1 (plain epilogues) / all (every epilogue) turn it on, read
// per call: on the step's shapes it measured slower than the tile kernels (QKV forward 53.0 vs 39.8 us, teacher FFN1
// 76.5 vs 57.1 us, profiles/r6_sk_ab.txt).  The stamps (tools/stamp_sk.py, profiles/r6_sk_stamps.txt) show why: at
// one 8-wave block per CU nothing overlaps a 256 x 256 epilogue (11 k ticks plain, 20 k with GELU, every block
// bursting its stores at the same two phase points) nor a segment's prologue fill (12 K-tiles take 36.6 k ticks
// against 28-30 k in a long loop), and a head piece waits / loads 256 KB of fp32 partial (entry gap up to 16 k).
// The two-blocks-per-CU 128 x 128 / 128 x 192 tiles hide their epilogue VALU and stores under the other block's MFMAs.
bool sk_plan(const DphGemmArgs& a, int cus, SkPlan* out) {
  const char* e = getenv("DPH_GEMM_SK");
  if (!e || e[0] == '0') return false;
  if (a.batch != 1 || a.splits != 1 || a.dyn_ext || a.K % 128 != 0 || a.K < 256 || a.N < 2048) return false;
  if (!(a.act == DPH_ACT_NONE || a.act == DPH_ACT_GELU || a.act == DPH_ACT_GELU_BWD_DGK)) return false;
  // the epilogues whose working set beside 128 accumulator registers spills (dropout, the stored GELU' factor, the
  // DGK pair: 120-720 B of scratch per lane) stay on the tile kernels unless DPH_GEMM_SK=all (A/B)
  const bool all = e && !strcmp(e, "all");
  const bool heavy = a.dropout_p > 0.f || a.act == DPH_ACT_GELU_BWD_DGK || (a.flags & DPH_GEMM_PRE_DGK);
  if (heavy && !all) return false;
  if (a.c_dtype != DPH_OUT_BF16) return false;
  SkPlan p{};
  p.ntm = (int32_t)cdiv(a.M, (int64_t)sk::C::BM);
  p.ntn = (int32_t)cdiv(a.N, (int64_t)sk::C::BN);
  p.nk = (int32_t)(a.K / pp::BK);
  const int64_t tiles = (int64_t)p.ntm * p.ntn;
  if (tiles >= ((int64_t)1 << 24)) return false;
  p.half = tiles * p.nk / 2;
  // every block's range spans at least nk + 2 K-tiles (ranges are 2 * (floor((b+1) h / n) - floor(b h / n)) >=
  // 2 * floor(h / n)), so a tile is cut at most once: one tail piece per head piece (the kernel's hand-off is
  // one-to-one).  The QKV shape (288 tiles x 12 K-tiles) therefore runs on 240 blocks rather than 256.
  int64_t nb = std::min<int64_t>({(int64_t)cus, p.half, p.half / (p.nk / 2 + 1)});
  if (nb >= 8) nb &= ~(int64_t)7;
  if (nb < 1) return false;
  p.nblk = (int32_t)nb;
  if (p.half / p.nblk < p.nk / 2 + 1) return false;
  *out = p;
  return true;
}

int64_t sk_ws_bytes(const SkPlan& p) { return (int64_t)p.nblk * sk::TILE_F * 4; }
int64_t sk_nflags(const SkPlan& p) { return (int64_t)p.nblk + 1; }

int sk_launch(const DphGemmArgs& a, const SkPlan& p, hipStream_t stream) {
  DPH_REQUIRE(a.sk_ws && a.sk_flags && a.sk_ws_bytes >= sk_ws_bytes(p) && a.sk_nflags >= sk_nflags(p),
              "dph_gemm: stream-K scratch too small (%lld B, %lld flags; need %lld B, %lld flags)",
              (long long)a.sk_ws_bytes, (long long)a.sk_nflags, (long long)sk_ws_bytes(p), (long long)sk_nflags(p));
  const dim3 grid((unsigned)p.nblk), block(sk::C::NT);
  const bool drop = a.dropout_p > 0.f;
  const bool dgkpre = a.act == DPH_ACT_GELU && (a.flags & DPH_GEMM_PRE_DGK);
  if (a.act == DPH_ACT_GELU_BWD_DGK) {
    hipLaunchKernelGGL((sk::sk_gemm_kernel<DPH_ACT_GELU_BWD_DGK, false>), grid, block, 0, stream, a, p);
  } else if (dgkpre) {
    if (drop) hipLaunchKernelGGL((sk::sk_gemm_kernel<ACT_GELU_DGKPRE, true>), grid, block, 0, stream, a, p);
    else hipLaunchKernelGGL((sk::sk_gemm_kernel<ACT_GELU_DGKPRE, false>), grid, block, 0, stream, a, p);
  } else if (a.act == DPH_ACT_GELU) {
    if (drop) hipLaunchKernelGGL((sk::sk_gemm_kernel<DPH_ACT_GELU, true>), grid, block, 0, stream, a, p);
    else hipLaunchKernelGGL((sk::sk_gemm_kernel<DPH_ACT_GELU, false>), grid, block, 0, stream, a, p);
  } else {
    if (drop) hipLaunchKernelGGL((sk::sk_gemm_kernel<DPH_ACT_NONE, true>), grid, block, 0, stream, a, p);
    else hipLaunchKernelGGL((sk::sk_gemm_kernel<DPH_ACT_NONE, false>), grid, block, 0, stream, a, p);
  }
  return check_launch("dph_gemm (stream-K)");
}

const char* sk_variant(const DphGemmArgs& a) {
  const bool drop = a.dropout_p > 0.f;
  if (a.act == DPH_ACT_GELU_BWD_DGK) return "sk_gemm_kernel<3, false>";
  if (a.act == DPH_ACT_GELU && (a.flags & DPH_GEMM_PRE_DGK)) return drop ? "sk_gemm_kernel<16, true>" : "sk_gemm_kernel<16, false>";
  if (a.act == DPH_ACT_GELU) return drop ? "sk_gemm_kernel<1, true>" : "sk_gemm_kernel<1, false>";
  return drop ? "sk_gemm_kernel<0, true>" : "sk_gemm_kernel<0, false>";
}
}  // namespace dph
