// Error reporting and ABI version for the DPHuBERT gfx950 kernel library.
#include "common.h"

#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

namespace dph {
namespace {
thread_local char g_err[1024] = {0};
constexpr int MAX_TU = 32;
int (*g_epoch_setters[MAX_TU])(const uint64_t*);
int g_n_epoch_setters = 0;
}

void register_epoch_setter(int (*fn)(const uint64_t*)) {
  if (g_n_epoch_setters < MAX_TU) g_epoch_setters[g_n_epoch_setters++] = fn;
}

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return DPH_ELAUNCH;
  }
  return DPH_OK;
}

// ---- deterministic mode ----------------------------------------------------------------------
// Process-wide switch read by the launch code of every kernel that reduces float partials across blocks
// (bias / LayerNorm-affine column sums, mask gradients, conv0 sums, head-mask sums, WavLM diagonal sums): on, they
// write per-block partial slabs summed in a fixed order instead of same-address float atomics, so two runs of a
// step (eager or a HIP-graph replay) give bitwise identical gradients.  Initial value: DPH_DETERMINISTIC (default
// on); set before a graph capture (a captured graph keeps the kernels it recorded).
namespace {
int g_det = -1;
}
bool deterministic() {
  if (g_det < 0) {
    const char* e = getenv("DPH_DETERMINISTIC");
    g_det = (e && e[0] == '0') ? 0 : 1;
  }
  return g_det != 0;
}

// ---- deferred column reductions (deterministic mode) -------------------------------------------
// Between dph_defer_reductions(1) and (0) the fixed-order partial-slab column reductions (LayerNorm affine / branch
// bias gradients, dph_colsum*, GEMM epilogue column sums) are queued instead of launched -- each is a ~4 us launch
// of a 32-column x DET_PH-phase grid -- and dph_flush_reductions launches the queue as ONE grid (up to RED_MAXP
// problems per launch), each problem summed exactly as its own launch would (det_column_total), so the results are
// bitwise those of the immediate launches.  The caller keeps every queued slab alive and its outputs unread until
// the flush; two queued problems never write overlapping outputs (an overlapping one flushes the queue first).
namespace {
struct ColRed {
  const float* ws;   // row 0 of the problem's first column
  float* out;        // out[j] += sum_r ws[r * ld + j], j < n
  int32_t nrows, ld, n, pad;
};
constexpr int RED_MAXP = 96;
struct ColRedBatch {
  int32_t np;
  int32_t pre[RED_MAXP + 1];   // first 32-column block of each problem
  ColRed p[RED_MAXP];
};
static_assert(sizeof(ColRedBatch) <= 4096, "kernel argument limit");

__global__ void __launch_bounds__(32 * DET_PH) colred_batch_kernel(const ColRedBatch b) {
  __shared__ float red[DET_PH][33];
  const int bx = (int)blockIdx.x;
  int k = 0;
  while (k + 1 < b.np && b.pre[k + 1] <= bx) ++k;
  const float* ws = b.p[k].ws;
  float* out = b.p[k].out;
  const int64_t col = (int64_t)(bx - b.pre[k]) * 32 + (threadIdx.x & 31);
  const bool live = col < b.p[k].n;
  const float t = det_column_total(live ? ws + col : nullptr, b.p[k].nrows, b.p[k].ld, red);
  if ((threadIdx.x >> 5) == 0 && live) out[col] += t;
}

bool g_defer = false;
std::vector<ColRed> g_redq;
int64_t g_redq_pushed = 0;   // every problem ever queued (dph_reductions_pushed)
hipStream_t g_redq_stream = nullptr;

int flush_redq() {
  size_t i = 0;
  while (i < g_redq.size()) {
    ColRedBatch b{};
    int blocks = 0;
    while (i < g_redq.size() && b.np < RED_MAXP) {
      b.pre[b.np] = blocks;
      b.p[b.np] = g_redq[i++];
      blocks += (int)cdiv(b.p[b.np].n, 32);
      ++b.np;
    }
    b.pre[b.np] = blocks;
    hipLaunchKernelGGL(colred_batch_kernel, dim3((unsigned)blocks), dim3(32 * DET_PH), 0, g_redq_stream, b);
    const int rc = check_launch("dph_flush_reductions");
    if (rc != DPH_OK) {
      g_redq.clear();
      return rc;
    }
  }
  g_redq.clear();
  return DPH_OK;
}
}  // namespace

bool colred_deferring() { return g_defer && deterministic(); }

// (a queue flushed on a clash that fails to launch is dropped: its error code is returned, and the caller passes it
// on, so the reductions it held are never silently lost)
int colred_push(const float* ws, int64_t nrows, int64_t ld, int64_t n, float* out, hipStream_t stream) {
  if (n <= 0 || out == nullptr) return DPH_OK;
  bool clash = !g_redq.empty() && stream != g_redq_stream;
  for (const ColRed& q : g_redq)
    if (out < q.out + q.n && q.out < out + n) clash = true;
  if (clash) {
    const int rc = flush_redq();
    if (rc != DPH_OK) return rc;
  }
  g_redq.push_back(ColRed{ws, out, (int32_t)nrows, (int32_t)ld, (int32_t)n, 0});
  g_redq_stream = stream;
  ++g_redq_pushed;
  return DPH_OK;
}
}  // namespace dph

extern "C" int dph_defer_reductions(int on) {
  dph::g_defer = on != 0;
  return DPH_OK;
}
extern "C" int64_t dph_deferred_reductions(void) { return (int64_t)dph::g_redq.size(); }
extern "C" int64_t dph_reductions_pushed(void) { return dph::g_redq_pushed; }
// Drop the queued reductions without launching them (the error path of a deferred block: their slabs may no longer
// be alive, so launching them would read freed memory and add garbage into the sinks).  Returns how many were dropped.
extern "C" int64_t dph_discard_reductions(void) {
  const int64_t n = (int64_t)dph::g_redq.size();
  dph::g_redq.clear();
  dph::g_redq_stream = nullptr;
  return n;
}
extern "C" int dph_flush_reductions(hipStream_t stream) {
  if (dph::g_redq.empty()) return DPH_OK;
  DPH_REQUIRE(stream == dph::g_redq_stream, "dph_flush_reductions: the queued reductions were issued on another stream");
  return dph::flush_redq();
}

extern "C" const char* dph_last_error(void) { return dph::g_err; }
extern "C" int dph_abi_version(void) { return 24; }
extern "C" int dph_set_deterministic(int on) {
  dph::g_det = on ? 1 : 0;
  return DPH_OK;
}
extern "C" int dph_get_deterministic(void) { return dph::deterministic() ? 1 : 0; }

// Point every kernel's RNG epoch at the device word `epoch` (uint64, device memory) on the current
// device, or detach it (NULL: seeds are used as passed).  Not stream-ordered: call outside any
// capture, before the kernels that should see it.
extern "C" int dph_set_rng_epoch(const uint64_t* epoch) {
  for (int i = 0; i < dph::g_n_epoch_setters; ++i)
    if (dph::g_epoch_setters[i](epoch) != 0) {
      dph::set_error("dph_set_rng_epoch: hipMemcpyToSymbol failed");
      return DPH_ELAUNCH;
    }
  return DPH_OK;
}

// ---- timing events (bench.py's live per-kernel timing) ----------------------------------------
// Recorded with hipEventRecordExternal so that, inside a stream capture, they become event-record
// nodes of the graph whose timestamps are readable after each replay (torch refuses external
// events on ROCm).  Outside a capture the flag is a plain record.
extern "C" int dph_event_create(void** ev) {
  hipEvent_t e = nullptr;
  if (!ev || hipEventCreateWithFlags(&e, hipEventDefault) != hipSuccess) {
    dph::set_error("dph_event_create failed");
    return DPH_ELAUNCH;
  }
  *ev = reinterpret_cast<void*>(e);
  return DPH_OK;
}

extern "C" int dph_event_record(void* ev, hipStream_t stream) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  unsigned long long cid = 0;
  hipGraph_t graph = nullptr;
  const hipGraphNode_t* deps = nullptr;
  size_t ndeps = 0;
  hipError_t e = hipStreamGetCaptureInfo_v2(stream, &st, &cid, &graph, &deps, &ndeps);
  if (e == hipSuccess && st == hipStreamCaptureStatusActive) {
    // capturing: append an event-record node after the stream's current capture frontier and make
    // it the new frontier (hipEventRecordWithFlags(external) is rejected by this ROCm)
    hipGraphNode_t node = nullptr;
    e = hipGraphAddEventRecordNode(&node, graph, deps, ndeps, reinterpret_cast<hipEvent_t>(ev));
    if (e == hipSuccess) e = hipStreamUpdateCaptureDependencies(stream, &node, 1, hipStreamSetCaptureDependencies);
  } else if (e == hipSuccess) {
    e = hipEventRecord(reinterpret_cast<hipEvent_t>(ev), stream);
  }
  if (e != hipSuccess) {
    dph::set_error("dph_event_record (capturing=%d): %s", (int)(st == hipStreamCaptureStatusActive),
                   hipGetErrorString(e));
    return DPH_ELAUNCH;
  }
  return DPH_OK;
}

extern "C" int dph_event_elapsed_ms(void* start, void* stop, float* ms) {
  if (hipEventSynchronize(reinterpret_cast<hipEvent_t>(stop)) != hipSuccess ||
      hipEventElapsedTime(ms, reinterpret_cast<hipEvent_t>(start), reinterpret_cast<hipEvent_t>(stop)) != hipSuccess) {
    dph::set_error("dph_event_elapsed_ms failed");
    return DPH_ELAUNCH;
  }
  return DPH_OK;
}

extern "C" int dph_event_destroy(void* ev) {
  return hipEventDestroy(reinterpret_cast<hipEvent_t>(ev)) == hipSuccess ? DPH_OK : DPH_ELAUNCH;
}
