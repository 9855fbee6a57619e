// Native gradient-readiness tracker: the bookkeeping core of the DDP reducer and of the ZeRO
// engine's gradient reduction (the role of torch's C++ Reducer in the reference's DDP path,
// SURVEY.md D3 / reference data_parallel_training.py:44, and of DeepSpeed's IPG bucket logic,
// D10 / zero_dp_training.py:40-43).
//
// Parameters are numbered 0..n-1 in flat-buffer order; each belongs to one bucket (a contiguous
// slice of the flat gradient buffer).  Per accumulation window the tracker counts the gradient
// contributions each parameter still expects (fused modules announce every use in forward; a
// tied weight is used twice), marks a parameter ready when its last contribution lands (an
// autograd AccumulateGrad contribution is always final), and decides which buckets may start
// their collective now:
//   * "ordered" buckets launch in bucket-index order only (every rank issues the same collective
//     sequence, whatever the local gradient-ready order),
//   * "eager" buckets (ZeRO-3 units) launch as soon as they are complete.
// The Python side issues the RCCL collectives; everything here is plain host code (no HIP), so
// the same library serves the CPU (gloo) tests and the GPU path.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

#define RT_EXPORT extern "C" __attribute__((visibility("default")))

namespace {

struct Tracker {
  int n = 0, nb = 0;
  std::vector<int> bucket_of;      // param -> bucket
  std::vector<int> bucket_params;  // bucket -> number of params
  std::vector<uint8_t> ordered;    // bucket -> 1: in-order chain, 0: launch when complete
  std::vector<int> pending;        // param -> expected contributions still to come
  std::vector<uint8_t> ready;      // param -> ready in this window
  std::vector<int> ready_count;    // bucket -> ready params
  std::vector<uint8_t> launched;   // bucket -> collective issued in this window
  int next = 0;                    // first ordered bucket not launched yet
  long long windows = 0, launches = 0;

  void reset() {
    std::fill(pending.begin(), pending.end(), 0);
    std::fill(ready.begin(), ready.end(), 0);
    std::fill(ready_count.begin(), ready_count.end(), 0);
    std::fill(launched.begin(), launched.end(), 0);
    next = 0;
    ++windows;
  }

  bool complete(int b) const { return ready_count[b] >= bucket_params[b]; }

  // launchable buckets (marked launched) appended to out[0..cap); returns the count
  int collect(int touched_bucket, int* out, int cap) {
    int k = 0;
    if (touched_bucket >= 0 && !ordered[touched_bucket]) {
      if (!launched[touched_bucket] && complete(touched_bucket) && k < cap) {
        launched[touched_bucket] = 1;
        out[k++] = touched_bucket;
      }
      launches += k;
      return k;
    }
    while (next < nb && k < cap) {
      if (!ordered[next] || launched[next]) {
        ++next;
        continue;
      }
      if (!complete(next)) break;
      launched[next] = 1;
      out[k++] = next++;
    }
    launches += k;
    return k;
  }
};

}  // namespace

RT_EXPORT void* dtd_tracker_create(int nparams, const int* bucket_of, int nbuckets, const uint8_t* ordered) {
  if (nparams <= 0 || nbuckets <= 0) return nullptr;
  auto* t = new Tracker();
  t->n = nparams;
  t->nb = nbuckets;
  t->bucket_of.assign(bucket_of, bucket_of + nparams);
  t->bucket_params.assign(nbuckets, 0);
  for (int p = 0; p < nparams; ++p) {
    const int b = bucket_of[p];
    if (b < 0 || b >= nbuckets) {
      delete t;
      return nullptr;
    }
    t->bucket_params[b]++;
  }
  t->ordered.assign(nbuckets, 1);
  if (ordered) t->ordered.assign(ordered, ordered + nbuckets);
  t->pending.assign(nparams, 0);
  t->ready.assign(nparams, 0);
  t->ready_count.assign(nbuckets, 0);
  t->launched.assign(nbuckets, 0);
  return t;
}

RT_EXPORT void dtd_tracker_destroy(void* h) { delete static_cast<Tracker*>(h); }

RT_EXPORT void dtd_tracker_reset(void* h) { static_cast<Tracker*>(h)->reset(); }

// one more contribution of parameter p is expected in the coming backward (fused-module use)
RT_EXPORT int dtd_tracker_expect(void* h, int p) {
  auto* t = static_cast<Tracker*>(h);
  if (p < 0 || p >= t->n) return -1;
  return ++t->pending[p];
}

// A contribution of p landed.  Returns -1 on a bad index, 0 if p still waits for more, else
// 1 + the number of launchable buckets written to out (when allow_launch; 1 = ready, nothing
// to launch yet).  Readiness is idempotent within a window.
RT_EXPORT int dtd_tracker_contribute(void* h, int p, int autograd, int allow_launch, int* out, int cap) {
  auto* t = static_cast<Tracker*>(h);
  if (p < 0 || p >= t->n) return -1;
  if (!autograd && t->pending[p] > 0) {
    if (--t->pending[p] > 0) return 0;
  }
  const int b = t->bucket_of[p];
  if (!t->ready[p]) {
    t->ready[p] = 1;
    t->ready_count[b]++;
  }
  if (!allow_launch) return 1;
  return 1 + t->collect(b, out, cap);
}

// every bucket not launched yet, in index order (end of backward: unused parameters contribute
// zeros); marks them launched
RT_EXPORT int dtd_tracker_drain(void* h, int* out, int cap) {
  auto* t = static_cast<Tracker*>(h);
  int k = 0;
  for (int b = 0; b < t->nb && k < cap; ++b) {
    if (!t->launched[b]) {
      t->launched[b] = 1;
      out[k++] = b;
    }
  }
  t->next = t->nb;
  t->launches += k;
  return k;
}

RT_EXPORT int dtd_tracker_is_ready(void* h, int p) {
  auto* t = static_cast<Tracker*>(h);
  return (p >= 0 && p < t->n) ? t->ready[p] : -1;
}
RT_EXPORT int dtd_tracker_is_launched(void* h, int b) {
  auto* t = static_cast<Tracker*>(h);
  return (b >= 0 && b < t->nb) ? t->launched[b] : -1;
}
RT_EXPORT int dtd_tracker_ready_count(void* h, int b) {
  auto* t = static_cast<Tracker*>(h);
  return (b >= 0 && b < t->nb) ? t->ready_count[b] : -1;
}
RT_EXPORT long long dtd_tracker_stat(void* h, int which) {
  auto* t = static_cast<Tracker*>(h);
  return which == 0 ? t->windows : t->launches;
}

// Greedy bucket assignment of consecutive parameters (flat-buffer order) under a capacity in
// elements: a new bucket starts when adding the next parameter would exceed the cap and the
// current bucket is not empty (an oversize parameter gets a bucket of its own).  offsets[i] is
// the parameter's aligned start in the flat buffer, total the buffer length.  Writes
// bucket_of[n] and the bucket [start, end) element ranges; returns the bucket count (or -1 when
// more than max_buckets would be needed).
RT_EXPORT int dtd_bucket_assign(int n, const long long* offsets, const long long* numels, long long total,
                                long long cap, int* bucket_of, long long* starts, long long* ends, int max_buckets) {
  if (n <= 0) return 0;
  int nb = 0;
  long long start = 0;
  int count = 0;
  for (int i = 0; i < n; ++i) {
    const long long s = offsets[i];
    if (count > 0 && (s - start) + numels[i] > cap) {
      if (nb >= max_buckets) return -1;
      starts[nb] = start;
      ends[nb] = s;
      ++nb;
      start = s;
      count = 0;
    }
    bucket_of[i] = nb;
    ++count;
  }
  if (nb >= max_buckets) return -1;
  starts[nb] = start;
  ends[nb] = total;
  return nb + 1;
}
