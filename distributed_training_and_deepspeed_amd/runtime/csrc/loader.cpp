// Native host data path: a worker pool that builds training batches straight into pinned host
// buffers, so the Python loop only issues the H2D copy (the reference's
// util.load_wikitext + DataCollatorForLanguageModeling + torch DataLoader; there is no network on
// the MI355X boxes, hence synthetic rows with the reference's schema and masking law).
//
//  * dtd_loader_gather: rows of a host dataset selected by sampler indices, copied by all workers
//    (one contiguous row per memcpy) into a destination buffer.
//  * dtd_loader_synth_mlm: synthetic BERT rows [CLS] x ... x [SEP] with the HF static MLM law
//    (p = 0.15 over non-special tokens; of those 80 % -> [MASK], 10 % -> a random token, 10 %
//    kept; unmasked labels -100), or causal rows (labels = ids).  Every token and decision is a
//    pure function of (seed, global row, position, draw) through a counter-based hash, so a row is
//    identical whichever worker, rank or batch produces it (resumable, rank-shardable).
//  * jobs run asynchronously (submit -> slot id, wait(slot)): the next batch is produced while
//    the current one trains.
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#define RT_EXPORT extern "C" __attribute__((visibility("default")))

namespace {

inline uint64_t mix64(uint64_t z) {   // splitmix64 finaliser
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
inline uint64_t draw(uint64_t seed, uint64_t row, uint32_t pos, uint32_t k) {
  return mix64(mix64(seed ^ (row * 0xD1B54A32D192ED03ull)) ^ ((uint64_t)pos << 8) ^ k);
}
inline double unit(uint64_t h) { return (h >> 11) * (1.0 / 9007199254740992.0); }   // [0, 1)

struct Pool {
  std::vector<std::thread> threads;
  std::mutex mu;
  std::condition_variable cv, done_cv;
  std::deque<std::function<void()>> tasks;
  std::vector<int> pending_per_job;   // indexed by job id (ring)
  std::atomic<bool> stop{false};
  int next_job = 0;

  explicit Pool(int n) : pending_per_job(256, 0) {
    for (int i = 0; i < n; ++i) threads.emplace_back([this] { run(); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(mu);
      stop = true;
    }
    cv.notify_all();
    for (auto& t : threads) t.join();
  }
  void run() {
    for (;;) {
      std::function<void()> f;
      {
        std::unique_lock<std::mutex> l(mu);
        cv.wait(l, [this] { return stop || !tasks.empty(); });
        if (stop && tasks.empty()) return;
        f = std::move(tasks.front());
        tasks.pop_front();
      }
      f();
    }
  }
  // split [0, n) into chunks over the workers; returns the job id (wait() on it).  Ids are slots
  // of a ring: a submit that lands on a slot whose job is still running first waits for it, so
  // that job's finishing tasks can never count down the new job (callers keep a few jobs in
  // flight, far below the ring size, so this wait does not happen in practice).
  int submit(int64_t n, const std::function<void(int64_t, int64_t)>& body) {
    const int nt = std::max<int>(1, (int)threads.size());
    const int64_t chunks = std::min<int64_t>(n, nt * 4);
    std::unique_lock<std::mutex> g(mu);
    const int job = next_job;
    next_job = (next_job + 1) % (int)pending_per_job.size();
    done_cv.wait(g, [this, job] { return pending_per_job[job] <= 0; });
    pending_per_job[job] = (int)std::max<int64_t>(chunks, 0);
    for (int64_t c = 0; c < chunks; ++c) {
      const int64_t a = n * c / chunks, b = n * (c + 1) / chunks;
      tasks.emplace_back([this, body, a, b, job] {
        body(a, b);
        std::lock_guard<std::mutex> g2(mu);
        if (--pending_per_job[job] == 0) done_cv.notify_all();
      });
    }
    cv.notify_all();
    return job;
  }
  void wait(int job) {
    std::unique_lock<std::mutex> l(mu);
    done_cv.wait(l, [this, job] { return pending_per_job[job] <= 0; });
  }
};

}  // namespace

RT_EXPORT void* dtd_loader_create(int nthreads) {
  if (nthreads <= 0) nthreads = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  return new Pool(nthreads);
}

RT_EXPORT void dtd_loader_destroy(void* h) { delete static_cast<Pool*>(h); }

RT_EXPORT int dtd_loader_threads(void* h) { return (int)static_cast<Pool*>(h)->threads.size(); }

RT_EXPORT void dtd_loader_wait(void* h, int job) { static_cast<Pool*>(h)->wait(job); }

// dst[i] = src[idx[i]] for n rows of row_bytes; asynchronous (returns the job id)
RT_EXPORT int dtd_loader_gather(void* h, const void* src, int64_t src_rows, int64_t row_bytes, const int64_t* idx,
                                int64_t n, void* dst) {
  auto* pool = static_cast<Pool*>(h);
  for (int64_t i = 0; i < n; ++i)
    if (idx[i] < 0 || idx[i] >= src_rows) return -1;
  std::vector<int64_t> ix(idx, idx + n);   // the caller's index array may go away
  const char* s = static_cast<const char*>(src);
  char* d = static_cast<char*>(dst);
  return pool->submit(n, [=](int64_t a, int64_t b) {
    for (int64_t i = a; i < b; ++i) std::memcpy(d + i * row_bytes, s + ix[i] * row_bytes, row_bytes);
  });
}

struct SynthSpec {
  uint64_t seed;
  int64_t row0, nrows;    // global rows row0 .. row0 + nrows - 1
  int32_t seq, vocab;
  int32_t lo;             // first non-special id drawn for body tokens
  int32_t cls, sep;       // BERT framing ids (-1: none)
  int32_t mask_id;        // [MASK] (MLM)
  int32_t mlm;            // 1: masked-LM rows, 0: causal rows (labels = ids)
  float mlm_p;            // 0.15
  int32_t nspecial;
  int32_t special[8];     // ids never masked
};

// ids / labels: int64 [nrows, seq]; asynchronous (returns the job id)
RT_EXPORT int dtd_loader_synth(void* h, const SynthSpec* spec, int64_t* ids, int64_t* labels) {
  auto* pool = static_cast<Pool*>(h);
  const SynthSpec sp = *spec;
  if (sp.seq <= 0 || sp.vocab <= sp.lo || sp.nspecial < 0 || sp.nspecial > 8) return -1;
  return pool->submit(sp.nrows, [=](int64_t a, int64_t b) {
    for (int64_t r = a; r < b; ++r) {
      const uint64_t grow = (uint64_t)(sp.row0 + r);
      int64_t* id = ids + r * sp.seq;
      int64_t* lab = labels + r * sp.seq;
      for (int j = 0; j < sp.seq; ++j) {
        int64_t tok = sp.lo + (int64_t)(draw(sp.seed, grow, j, 0) % (uint64_t)(sp.vocab - sp.lo));
        if (sp.cls >= 0 && j == 0) tok = sp.cls;
        if (sp.sep >= 0 && j == sp.seq - 1) tok = sp.sep;
        if (!sp.mlm) {
          id[j] = tok;
          lab[j] = tok;
          continue;
        }
        bool special = false;
        for (int s = 0; s < sp.nspecial; ++s) special |= tok == sp.special[s];
        if (special || unit(draw(sp.seed, grow, j, 1)) >= sp.mlm_p) {
          id[j] = tok;
          lab[j] = -100;
          continue;
        }
        lab[j] = tok;
        if (unit(draw(sp.seed, grow, j, 2)) < 0.8) {
          id[j] = sp.mask_id;
        } else if (unit(draw(sp.seed, grow, j, 3)) < 0.5) {
          id[j] = (int64_t)(draw(sp.seed, grow, j, 4) % (uint64_t)sp.vocab);
        } else {
          id[j] = tok;
        }
      }
    }
  });
}
