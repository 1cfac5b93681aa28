// Per-kernel device timing with HIP events on the launch stream (diagnostics for bench.py).
//
// While enabled, every launch wrapped in DPZ_TIMED records a start/end event pair on its own
// stream; dpz_timing_read() waits for the pending pairs and returns the summed durations per
// kernel id.  Launches into a capturing stream are never timed (HIP refuses event records inside
// stream capture).  The state is process-global and not thread-safe: it is a measurement
// facility, not part of the codec.
#include <vector>

#include "dpz_common.h"

namespace dpz {
namespace {

struct Pair {
  hipEvent_t a, b;
  int id;
};

struct TimingState {
  bool on = false;
  std::vector<Pair> pending;
  std::vector<Pair> free_pairs;
  double ms[DPZ_KT_COUNT] = {};
  long long cnt[DPZ_KT_COUNT] = {};
};

TimingState& T() {
  static TimingState s;
  return s;
}

void drain(size_t upto) {
  TimingState& s = T();
  size_t i = 0;
  for (; i < upto && i < s.pending.size(); ++i) {
    Pair& p = s.pending[i];
    float ms = 0.f;
    if (hipEventSynchronize(p.b) == hipSuccess && hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
      s.ms[p.id] += ms;
      s.cnt[p.id] += 1;
    }
    s.free_pairs.push_back(p);
  }
  s.pending.erase(s.pending.begin(), s.pending.begin() + i);
}

}  // namespace

int timing_begin(int id, hipStream_t st) {
  TimingState& s = T();
  if (!s.on || id < 0 || id >= DPZ_KT_COUNT) return -1;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) {
    (void)hipGetLastError();  // never leak a timing-side error into the codec's launch checks
    return -1;
  }
  if (s.pending.size() >= 4096) drain(2048);
  Pair p;
  if (!s.free_pairs.empty()) {
    p = s.free_pairs.back();
    s.free_pairs.pop_back();
  } else {
    if (hipEventCreate(&p.a) != hipSuccess) return -1;
    if (hipEventCreate(&p.b) != hipSuccess) return -1;
  }
  p.id = id;
  if (hipEventRecord(p.a, st) != hipSuccess) {
    (void)hipGetLastError();
    s.free_pairs.push_back(p);
    return -1;
  }
  s.pending.push_back(p);
  return (int)s.pending.size() - 1;
}

void timing_end(int slot, hipStream_t st) {
  if (slot < 0) return;
  TimingState& s = T();
  if ((size_t)slot < s.pending.size() && hipEventRecord(s.pending[slot].b, st) != hipSuccess)
    (void)hipGetLastError();
}

}  // namespace dpz

using namespace dpz;

static const char* const kNames[DPZ_KT_COUNT] = {
    "topk_sample", "topk_filter", "topk_select", "topk_resolve", "topk_compact",
    "topk_exact_hist", "topk_exact_resolve", "topk_exact_count", "topk_exact_scan",
    "topk_exact_write", "topk_accumulate", "fold_offsets", "fold", "dwt", "idwt",
    "elias_count", "elias_scan", "elias_pack", "elias_spec", "elias_resolve", "elias_write",
    "fp16", "scatter_fill", "fpz_size", "fpz_scan", "fpz_pack", "fpz_decode", "cplx",
    "fft_scale", "haar", "lz4", "counter_flush", "fft"};

extern "C" const char* dpz_kernel_name(int id) {
  return (id >= 0 && id < DPZ_KT_COUNT) ? kNames[id] : nullptr;
}

extern "C" int dpz_timing_enable(int on) {
  TimingState& s = T();
  drain(s.pending.size());
  for (int i = 0; i < DPZ_KT_COUNT; ++i) {
    s.ms[i] = 0.0;
    s.cnt[i] = 0;
  }
  s.on = on != 0;
  return DPZ_OK;
}

extern "C" int dpz_timing_read(double* ms_sum, int64_t* count, int max_ids) {
  TimingState& s = T();
  drain(s.pending.size());
  const int m = max_ids < DPZ_KT_COUNT ? max_ids : DPZ_KT_COUNT;
  for (int i = 0; i < m; ++i) {
    if (ms_sum) ms_sum[i] = s.ms[i];
    if (count) count[i] = s.cnt[i];
  }
  return DPZ_KT_COUNT;
}
