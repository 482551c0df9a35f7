// slot_collector.h -- the batching policy shared by the MI355X channel-processor plug-ins (pusch_processor_hip,
// pdsch_processor_hip): process() calls of the reference's upper PHY (one per PDU, from any thread) are queued,
// and one collector thread hands the pending PDUs of a slot to the GPU as one batch when
//   * flush() is called (the slot boundary),
//   * a PDU of another slot arrives (the pending slot is complete),
//   * max_batch PDUs are pending, or
//   * the oldest pending PDU has waited max_wait_us (0: no timer).
// A batch never spans a slot boundary: every slot change is remembered, and each batch ends at the first one.
// The batch callback runs on the collector thread and calls each PDU's notifier.  wait_idle() blocks until every
// PDU queued so far has been processed.  Destruction processes what is still pending, then joins the thread.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace srsran {
namespace hip {

template <typename Entry>
class slot_collector
{
public:
  /// process(batch) returns the number of PDUs it reported as failed.
  using batch_function = std::function<unsigned(std::vector<Entry>&)>;

  struct counters {
    uint64_t nof_pdus = 0, nof_batches = 0, nof_errors = 0;
  };

  slot_collector(unsigned max_batch_, unsigned max_wait_us_, batch_function process_) :
    max_batch(max_batch_ == 0 ? 1 : max_batch_), max_wait(max_wait_us_), process(std::move(process_))
  {
    worker = std::thread([this] { run(); });
  }

  ~slot_collector()
  {
    {
      std::lock_guard<std::mutex> lock(mtx);
      stop      = true;
      flush_req = true;
    }
    cv.notify_all();
    worker.join();
  }

  slot_collector(const slot_collector&)            = delete;
  slot_collector& operator=(const slot_collector&) = delete;

  /// Queues one PDU of slot `slot_key` (any value that differs between slots).
  void enqueue(Entry&& e, uint64_t slot_key)
  {
    {
      std::lock_guard<std::mutex> lock(mtx);
      const uint64_t seq = head_seq + queue.size();
      if (!queue.empty() && slot_key != last_key) {
        boundaries.push_back(seq); // the slot before seq is complete
      }
      last_key = slot_key;
      queue.push_back(item{std::move(e), std::chrono::steady_clock::now()});
      ++in_flight;
    }
    cv.notify_all();
  }

  void flush()
  {
    {
      std::lock_guard<std::mutex> lock(mtx);
      flush_req = true;
    }
    cv.notify_all();
  }

  void wait_idle()
  {
    flush();
    std::unique_lock<std::mutex> lock(mtx);
    idle_cv.wait(lock, [this] { return in_flight == 0; });
  }

  counters get_counters() const
  {
    std::lock_guard<std::mutex> lock(mtx);
    return stats;
  }

private:
  struct item {
    Entry                                 e;
    std::chrono::steady_clock::time_point t; // enqueue time
  };

  void run()
  {
    std::unique_lock<std::mutex> lock(mtx);
    while (true) {
      const auto wait  = std::chrono::microseconds(max_wait);
      auto       ready = [&] {
        return !queue.empty() && (flush_req || stop || !boundaries.empty() || queue.size() >= max_batch ||
                                  (max_wait != 0 && std::chrono::steady_clock::now() - queue.front().t >= wait));
      };
      if (queue.empty() && stop) {
        break;
      }
      if (!ready()) {
        if (max_wait != 0 && !queue.empty()) {
          cv.wait_until(lock, queue.front().t + wait); // the oldest pending PDU's deadline
        } else {
          cv.wait(lock);
        }
        continue;
      }
      // the oldest slot (up to its first boundary), or everything pending, at most max_batch PDUs: a batch never
      // spans a slot boundary
      const size_t       upto = boundaries.empty() ? queue.size() : static_cast<size_t>(boundaries.front() - head_seq);
      const size_t       n    = std::min<size_t>(upto, max_batch);
      std::vector<Entry> batch;
      batch.reserve(n);
      for (size_t i = 0; i != n; ++i) {
        batch.push_back(std::move(queue.front().e));
        queue.pop_front();
      }
      head_seq += n;
      while (!boundaries.empty() && boundaries.front() <= head_seq) {
        boundaries.pop_front();
      }
      flush_req = flush_req && !queue.empty();
      lock.unlock();
      const unsigned errors = process(batch);
      lock.lock();
      stats.nof_pdus += batch.size();
      stats.nof_batches += 1;
      stats.nof_errors += errors;
      in_flight -= batch.size();
      if (in_flight == 0) {
        idle_cv.notify_all();
      }
    }
  }

  const unsigned                        max_batch;
  const unsigned                        max_wait;
  batch_function                        process;
  mutable std::mutex                    mtx;
  std::condition_variable               cv, idle_cv;
  std::deque<item>                      queue;
  uint64_t                              head_seq = 0;   // sequence number of queue.front()
  std::deque<uint64_t>                  boundaries;     // sequence numbers that start a new slot (ascending)
  uint64_t                              last_key = 0;   // slot of the newest queued PDU
  bool                                  flush_req = false, stop = false;
  size_t                                in_flight = 0;
  counters                              stats;
  std::thread                           worker;
};

/// A fixed pool of worker threads for the host-side row copies of a batch (grid staging, grid merging): run(n, fn)
/// calls fn(i) for every i < n on the workers and the calling thread and returns when all calls are done.
class row_pool
{
public:
  explicit row_pool(unsigned nof_threads)
  {
    for (unsigned t = 0; t < nof_threads; ++t) {
      threads.emplace_back([this] { work(); });
    }
  }
  ~row_pool()
  {
    {
      std::lock_guard<std::mutex> lock(mtx);
      stop = true;
    }
    cv.notify_all();
    for (auto& t : threads) {
      t.join();
    }
  }
  row_pool(const row_pool&)            = delete;
  row_pool& operator=(const row_pool&) = delete;

  void run(size_t n, const std::function<void(size_t)>& fn)
  {
    if (n == 0) {
      return;
    }
    if (threads.empty() || n == 1) {
      for (size_t i = 0; i != n; ++i) {
        fn(i);
      }
      return;
    }
    std::unique_lock<std::mutex> lock(run_mtx); // one run at a time
    {
      std::lock_guard<std::mutex> g(mtx);
      job   = &fn;
      count = n;
      next.store(0);
      done.store(0);
      ++generation;
    }
    cv.notify_all();
    drain();
    // every item done AND every worker out of drain(): a worker still inside could otherwise fetch an index of the
    // next run (after its reset of `next`) and count it against the wrong run
    std::unique_lock<std::mutex> g(mtx);
    done_cv.wait(g, [&] { return done.load() == count && active == 0; });
    job = nullptr;
  }

private:
  void drain()
  {
    for (size_t i = next.fetch_add(1); i < count; i = next.fetch_add(1)) {
      (*job)(i);
      if (done.fetch_add(1) + 1 == count) {
        std::lock_guard<std::mutex> g(mtx);
        done_cv.notify_all();
      }
    }
  }
  void work()
  {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lock(mtx);
        cv.wait(lock, [&] { return stop || (generation != seen && job != nullptr); });
        if (stop) {
          return;
        }
        seen = generation;
        ++active; // under the lock that run() resets the counters with: this worker drains this run only
      }
      drain();
      {
        std::lock_guard<std::mutex> lock(mtx);
        --active;
      }
      done_cv.notify_all();
    }
  }
  std::vector<std::thread>                  threads;
  std::mutex                                mtx, run_mtx;
  std::condition_variable                   cv, done_cv;
  const std::function<void(size_t)>*        job   = nullptr;
  size_t                                    count = 0;
  std::atomic<size_t>                       next{0}, done{0};
  uint64_t                                  generation = 0;
  unsigned                                  active     = 0; // workers inside drain()
  bool                                      stop       = false;
};

/// Device buffer + pinned host mirror, grown on demand (contents not preserved).
struct hip_mirrored_buffer {
  uint8_t* d = nullptr;
  uint8_t* h = nullptr;
  size_t   n = 0;
  hip_mirrored_buffer() = default;
  hip_mirrored_buffer(const hip_mirrored_buffer&)            = delete;
  hip_mirrored_buffer& operator=(const hip_mirrored_buffer&) = delete;
  ~hip_mirrored_buffer()
  {
    (void)hipFree(d);
    (void)hipHostFree(h);
  }
  bool ensure(size_t bytes)
  {
    if (bytes <= n) {
      return true;
    }
    const size_t cap = std::max(bytes, n * 2);
    (void)hipFree(d);
    (void)hipHostFree(h);
    d = h = nullptr;
    n     = 0;
    if (hipMalloc(&d, cap) != hipSuccess || hipHostMalloc(&h, cap, hipHostMallocDefault) != hipSuccess) {
      return false;
    }
    n = cap;
    return true;
  }
};

} // namespace hip
} // namespace srsran
