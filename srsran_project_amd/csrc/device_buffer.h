// device_buffer.h -- grow-only device scratch allocation used by the C-ABI objects.
#pragma once

#include <cstdio>
#include <cstdlib>

#include <hip/hip_runtime.h>

#include <cstddef>

namespace srs_amd {

struct device_buffer {
  void*  ptr  = nullptr;
  size_t size = 0;
  device_buffer() = default;
  device_buffer(const device_buffer&) = delete;
  device_buffer& operator=(const device_buffer&) = delete;
  ~device_buffer() { (void)hipFree(ptr); }
  // Grows to at least n bytes (contents are not preserved).
  hipError_t ensure(size_t n)
  {
    if (n <= size) {
      return hipSuccess;
    }
    (void)hipFree(ptr);
    ptr        = nullptr;
    size       = 0;
    hipError_t e = hipMalloc(&ptr, n);
    if (e == hipSuccess) {
      size = n;
    }
    return e;
  }
  // ensure(n), the bytes zeroed whenever the buffer is (re)allocated
  hipError_t ensure_zeroed(size_t n)
  {
    if (n <= size) {
      return hipSuccess;
    }
    hipError_t e = ensure(n);
    return e == hipSuccess ? hipMemset(ptr, 0, size) : e;
  }
  template <typename T>
  T* as() const
  {
    return static_cast<T*>(ptr);
  }
};

// Remembers the geometry last written into a device array by a generator kernel (the per-codeblock
// rate-matching lengths / offsets of rm_arrays_kernel): a call with the same geometry on the same buffer
// skips the launch.  The buffer is written only by that kernel, and stream_order makes a call wait for the
// previous call's completion, so the skipped launch's contents are in place.
struct geometry_cache {
  const void* ptr = nullptr;
  uint32_t    key[8] = {};
  bool        valid  = false;
  // true when the generator must run for (p, k[0..n)); records the new state
  bool stale(const void* p, const uint32_t* k, int n)
  {
    bool same = valid && p == ptr;
    for (int i = 0; i < n && same; ++i) {
      same = key[i] == k[i];
    }
    if (same) {
      return false;
    }
    ptr   = p;
    valid = true;
    for (int i = 0; i < n; ++i) {
      key[i] = k[i];
    }
    return true;
  }
  void invalidate() { valid = false; }
};

// Host wait for an event by polling hipEventQuery: the staging buffers of the slot forms wait here once per call for
// their previous upload, which has normally completed or is about to; hipEventSynchronize could fall back to an
// interrupt-driven wait whose wake-up occasionally took ~7 ms (one such step in twenty, tools/gpu_r04_bimodal.sh).
inline hipError_t event_wait_spin(hipEvent_t ev)
{
  for (;;) {
    const hipError_t e = hipEventQuery(ev);
    if (e != hipErrorNotReady) {
      return e;
    }
  }
}

// Orders the reuse of an object's device scratch across the caller's streams: a batch call on stream s
// first waits for the previous call's completion event when that call ran on another stream, so two
// calls on different streams never overwrite each other's in-flight scratch.
struct stream_order {
  hipEvent_t  done = nullptr;
  hipStream_t last = nullptr;
  bool        used = false;
  stream_order() = default;
  stream_order(const stream_order&) = delete;
  stream_order& operator=(const stream_order&) = delete;
  ~stream_order()
  {
    if (done) {
      (void)hipEventDestroy(done);
    }
  }
  hipError_t begin(hipStream_t s) const { return (used && s != last) ? hipStreamWaitEvent(s, done, 0) : hipSuccess; }
  hipError_t end(hipStream_t s)
  {
    if (done == nullptr) {
      hipError_t e = hipEventCreateWithFlags(&done, hipEventDisableTiming);
      if (e != hipSuccess) {
        return e;
      }
    }
    last = s;
    used = true;
    return hipEventRecord(done, s);
  }
};

// Fans independent launches of one call out over up to FAN_STREAMS helper streams and joins them back into
// the caller's stream (events only, no host synchronisation): the small per-bucket LDPC launches of a
// heterogeneous slot run concurrently instead of one after the other on a mostly idle GPU.
// Lanes of the fan: the helper streams, then (with_main) the caller's stream itself.  Configuration (read once):
// SRSRAN_AMD_FAN_STREAMS helpers (0..4, default 1), SRSRAN_AMD_FAN_MAIN=0 keeps the caller's stream out of the
// fan (default: it is a lane), SRSRAN_AMD_FAN_PRIORITY=1 helpers at the highest stream priority.  Measured on the
// 64-cell sch_slot step (tools/gpu_r04_fan.sh, three processes each): one helper + the caller's stream 0.844-0.849
// ms; four helpers 1.05-1.12 ms (the helpers' hardware queues are assigned per process and collide); no helper
// 1.00 ms; high-priority helpers 1.39-1.65 ms.
// n bytes from pinned host memory h (hipHostMalloc) to device memory d on stream s, by a copy kernel (not the SDMA
// engine; stream_probe.hip)
hipError_t upload_pinned(void* d, const void* h, size_t n, hipStream_t s);

// true when kernels of streams a and b overlap (two spin kernels, host-synchronous; stream_probe.hip)
hipError_t streams_run_concurrently(hipStream_t a, hipStream_t b, bool& concurrent);

struct stream_fan {
  static constexpr int FAN_STREAMS = 4;
  static constexpr int SPARES      = 6; // helpers found on the caller's queue, kept so the next one lands elsewhere
  struct config {
    int  helpers;
    bool with_main, high_priority;
  };
  static const config& cfg()
  {
    static const config c = [] {
      auto env = [](const char* k, int dflt) {
        const char* e = std::getenv(k);
        return e != nullptr ? std::atoi(e) : dflt;
      };
      config r{};
      const int h     = env("SRSRAN_AMD_FAN_STREAMS", 1);
      r.helpers       = h < 0 ? 0 : (h > FAN_STREAMS ? FAN_STREAMS : h);
      r.with_main     = env("SRSRAN_AMD_FAN_MAIN", 1) != 0;
      r.high_priority = env("SRSRAN_AMD_FAN_PRIORITY", 0) != 0;
      return r;
    }();
    return c;
  }
  hipStream_t s[FAN_STREAMS]    = {};
  hipEvent_t  join[FAN_STREAMS] = {};
  hipEvent_t  fork              = nullptr;
  int         n                 = 0;     // helpers of the open fan
  bool        main_lane         = false; // the caller's stream is lane n
  hipStream_t probed[FAN_STREAMS] = {};  // the caller's stream helper i was found concurrent with ...
  bool        probe_done[FAN_STREAMS] = {}; // ... once probed (the caller's stream may be the null stream)
  hipStream_t spare[SPARES]       = {};
  int         nof_spares          = 0;
  stream_fan()                             = default;
  stream_fan(const stream_fan&)            = delete;
  stream_fan& operator=(const stream_fan&) = delete;
  ~stream_fan()
  {
    for (int i = 0; i < FAN_STREAMS; ++i) {
      if (s[i]) {
        (void)hipStreamSynchronize(s[i]);
        (void)hipStreamDestroy(s[i]);
      }
      if (join[i]) {
        (void)hipEventDestroy(join[i]);
      }
    }
    if (fork) {
      (void)hipEventDestroy(fork);
    }
    for (int i = 0; i < nof_spares; ++i) {
      (void)hipStreamDestroy(spare[i]);
    }
  }
  // A helper that runs concurrently with `main`: probed once per (helper, caller stream) -- a helper found on the
  // caller's hardware queue is kept aside (so the next stream created lands on another queue) and replaced, up to
  // SPARES times.  Not while `main` is being captured into a graph (the probe synchronizes).
  hipError_t ensure_concurrent(hipStream_t main, int i, bool high_priority)
  {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if ((probe_done[i] && probed[i] == main) || hipStreamIsCapturing(main, &cs) != hipSuccess ||
        cs != hipStreamCaptureStatusNone) {
      return hipSuccess;
    }
    for (;;) {
      bool       conc = true;
      hipError_t e    = streams_run_concurrently(main, s[i], conc);
      if (e != hipSuccess) {
        return e;
      }
      if (std::getenv("SRSRAN_AMD_FAN_DEBUG") != nullptr) {
        std::fprintf(stderr, "stream_fan: helper %d %s the caller's stream (%d set aside)\n", i,
                     conc ? "runs beside" : "serializes with", nof_spares);
      }
      if (conc || nof_spares == SPARES) {
        probed[i]     = main;
        probe_done[i] = true;
        return hipSuccess;
      }
      spare[nof_spares++] = s[i];
      int lo = 0, hi = 0;
      if (high_priority && hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess) {
        e = hipStreamCreateWithPriority(&s[i], hipStreamNonBlocking, hi);
      } else {
        e = hipStreamCreateWithFlags(&s[i], hipStreamNonBlocking);
      }
      if (e != hipSuccess) {
        s[i] = spare[--nof_spares];
        return e;
      }
    }
  }
  // Lanes of the open fan (>= 1): launches i = 0 .. count-1 go to stream(main, i % width()).
  int width() const { return n + (main_lane || n == 0 ? 1 : 0); }
  hipError_t begin(hipStream_t main, int count)
  {
    const config& c = cfg();
    main_lane       = c.with_main;
    const int want  = count - (main_lane ? 1 : 0); // helpers worth opening
    n               = count <= 1 ? 0 : (want < c.helpers ? want : c.helpers);
    n               = n < 0 ? 0 : n;
    hipError_t e    = hipSuccess;
    if (n > 0 && fork == nullptr) {
      e = hipEventCreateWithFlags(&fork, hipEventDisableTiming);
    }
    for (int i = 0; i < n && e == hipSuccess; ++i) {
      if (s[i] == nullptr) {
        int lo = 0, hi = 0;
        if (c.high_priority && hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess) {
          e = hipStreamCreateWithPriority(&s[i], hipStreamNonBlocking, hi);
        } else {
          e = hipStreamCreateWithFlags(&s[i], hipStreamNonBlocking);
        }
        if (e == hipSuccess) {
          e = hipEventCreateWithFlags(&join[i], hipEventDisableTiming);
        }
      }
      if (e == hipSuccess && main_lane) {
        e = ensure_concurrent(main, i, c.high_priority);
      }
    }
    if (n > 0 && e == hipSuccess) {
      e = hipEventRecord(fork, main);
    }
    for (int i = 0; i < n && e == hipSuccess; ++i) {
      e = hipStreamWaitEvent(s[i], fork, 0);
    }
    return e;
  }
  hipStream_t stream(hipStream_t main, int i) const
  {
    const int w = width();
    const int k = i % w;
    return k < n ? s[k] : main;
  }
  hipError_t end(hipStream_t main)
  {
    hipError_t e = hipSuccess;
    for (int i = 0; i < n && e == hipSuccess; ++i) {
      e = hipEventRecord(join[i], s[i]);
      if (e == hipSuccess) {
        e = hipStreamWaitEvent(main, join[i], 0);
      }
    }
    n = 0;
    return e;
  }
};

// Closes a call begun with stream_order::begin on every exit path, errors included: a pending fan-out is
// joined back into the caller's stream and the completion event recorded, so an early return never leaves
// helper streams forked (still using the scratch) while the next call waits on a stale event.
struct call_scope {
  stream_order& order;
  stream_fan*   fan;
  hipStream_t   s;
  bool          open = true;
  call_scope(stream_order& o, stream_fan* f, hipStream_t st) : order(o), fan(f), s(st) {}
  call_scope(const call_scope&)            = delete;
  call_scope& operator=(const call_scope&) = delete;
  hipError_t close()
  {
    open               = false;
    const hipError_t e = fan != nullptr ? fan->end(s) : hipSuccess;
    const hipError_t o = order.end(s);
    return e != hipSuccess ? e : o;
  }
  ~call_scope()
  {
    if (open) {
      (void)close();
    }
  }
};

// Host-built launch descriptors (per-item argument blocks of a slot call) staged in pinned memory and
// uploaded on the call's stream: the buffer is rewritten only once its previous upload has completed.
// Pinned host staging for per-call descriptor uploads: a ring of RING buffers, each rewritten only once its previous
// upload has completed, so a call can stage its descriptors while up to RING - 1 earlier calls' uploads still wait
// behind their stream's work (r06: the slot forms of consecutive batches no longer wait for each other on the host).
struct pinned_stage {
  static constexpr int RING = 3;
  struct slot {
    void*      h    = nullptr;
    size_t     size = 0;
    hipEvent_t done = nullptr;
    bool       used = false;
  };
  slot ring[RING];
  int  cur = 0;
  pinned_stage()                               = default;
  pinned_stage(const pinned_stage&)            = delete;
  pinned_stage& operator=(const pinned_stage&) = delete;
  ~pinned_stage()
  {
    for (slot& b : ring) {
      if (b.done) {
        (void)hipEventSynchronize(b.done);
        (void)hipEventDestroy(b.done);
      }
      (void)hipHostFree(b.h);
    }
  }
  // Moves to the next buffer of the ring, waits for its previous upload and grows it to n bytes; the host pointer is
  // then writable.
  hipError_t acquire(size_t n)
  {
    cur          = (cur + 1) % RING;
    slot&      b = ring[cur];
    hipError_t e = b.used ? event_wait_spin(b.done) : hipSuccess;
    b.used       = false;
    if (e == hipSuccess && b.done == nullptr) {
      e = hipEventCreateWithFlags(&b.done, hipEventDisableTiming);
    }
    if (e == hipSuccess && b.size < n) {
      (void)hipHostFree(b.h);
      b.h    = nullptr;
      b.size = 0;
      e      = hipHostMalloc(&b.h, n, hipHostMallocDefault);
      b.size = e == hipSuccess ? n : 0;
    }
    return e;
  }
  template <typename T>
  T* at(size_t offset) const
  {
    return reinterpret_cast<T*>(static_cast<unsigned char*>(ring[cur].h) + offset);
  }
  // Copies the first n bytes to device memory d on stream s.
  hipError_t upload(void* d, size_t n, hipStream_t s)
  {
    slot&      b = ring[cur];
    hipError_t e = upload_pinned(d, b.h, n, s);
    if (e == hipSuccess) {
      e = hipEventRecord(b.done, s);
    }
    b.used = e == hipSuccess;
    return e;
  }
  // Copies rows of `width` bytes (consecutive in the stage) to device rows dpitch bytes apart.
  hipError_t upload_rows(void* d, size_t dpitch, size_t width, size_t rows, hipStream_t s)
  {
    slot&      b = ring[cur];
    hipError_t e = hipMemcpy2DAsync(d, dpitch, b.h, width, width, rows, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) {
      e = hipEventRecord(b.done, s);
    }
    b.used = e == hipSuccess;
    return e;
  }
};

inline size_t align_up(size_t n, size_t a)
{
  return (n + a - 1) / a * a;
}

} // namespace srs_amd
