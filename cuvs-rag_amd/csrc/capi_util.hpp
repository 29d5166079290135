// Shared plumbing of the C-ABI translation units (capi.cpp, comm.cpp): the thread-local error
// channel behind mivs_last_error(), HIP status -> MIVS_ERR_* mapping, owning device buffers.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdlib>
#include <chrono>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/mivs.h"

namespace mivs_capi {

inline thread_local std::string g_err;
inline std::atomic<int> g_profiling{0};

struct MivsError : std::runtime_error {
  int code;
  MivsError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

inline void hipchk(hipError_t e, const char* what) {
  if (e == hipSuccess) return;
  (void)hipGetLastError();
  const int code = e == hipErrorOutOfMemory ? MIVS_ERR_OOM : MIVS_ERR_HIP;
  int dev = -1;
  (void)hipGetDevice(&dev);
  throw MivsError(code, std::string(what) + ": " + hipGetErrorString(e) + " (device " + std::to_string(dev) + ")");
}
#define HIPCHK(x) hipchk((x), #x)

inline void require(bool ok, const std::string& msg, int code = MIVS_ERR_INVALID) {
  if (!ok) throw MivsError(code, msg);
}

template <class F>
int32_t guarded(F&& f) {
  try {
    f();
    return MIVS_OK;
  } catch (const MivsError& e) {
    g_err = e.what();
    return e.code;
  } catch (const std::bad_alloc&) {
    g_err = "host allocation failed";
    return MIVS_ERR_OOM;
  } catch (const std::exception& e) {
    g_err = e.what();
    return MIVS_ERR_HIP;
  }
}

// The stream the current C-ABI call enqueues on (set by StreamScope for the call's duration), and whether the
// releasing thread has already waited for every stream that used the buffers it is about to release
// (mivs_index_free after the index's done-events). Buf::release uses them to order a cached block's reuse after
// the work still reading or writing it.
inline thread_local hipStream_t tl_stream = nullptr;
inline thread_local bool tl_stream_set = false;
inline thread_local bool tl_release_synced = false;

struct StreamScope {
  hipStream_t prev;
  bool prev_set;
  explicit StreamScope(hipStream_t s) : prev(tl_stream), prev_set(tl_stream_set) {
    tl_stream = s;
    tl_stream_set = true;
  }
  ~StreamScope() {
    tl_stream = prev;
    tl_stream_set = prev_set;
  }
};

// Large device blocks released by Bufs, kept for reuse by later Bufs of the process. OPT-IN: the
// limit is 0 per device until mivs_set_block_cache_limit (or MIVS_BLOCK_CACHE_MB at load) raises it, so by default a
// released block goes straight back to the driver and torch.cuda.mem_get_info sees it free. Why it exists: a fresh
// hipMalloc of tens of GB can stall for seconds while the pages are cleared -- a timed 10M build after an untimed
// one spent 5.4 s in its first allocations once in four runs (profiles/r05_variants_build.txt) -- whereas a block
// this process freed is handed out again as it is. Blocks of at least kCacheMin bytes are cached up to the device's
// limit; a request takes the smallest cached block of its device within 1/8 above its size; an allocation that fails
// for memory frees the device's cached blocks and tries again; mivs_release_cached_memory hands everything back (the
// drop-ins call it from the reference's cleanup and OOM paths). A cached block carries an event recorded on the
// stream of the call that released it (no device-wide sync); take() waits for that event before reuse.
struct BlockCache {
  static constexpr size_t kCacheMin = (size_t)64 << 20;
  static constexpr int kMaxDev = 64;
  struct Blk {
    void* p;
    size_t n;
    int dev;
    hipEvent_t ev;  // nullptr: nothing in flight (the releaser waited)
  };
  std::mutex mu;
  std::vector<Blk> blocks;
  size_t limit[kMaxDev];
  BlockCache() {
    const char* e = getenv("MIVS_BLOCK_CACHE_MB");
    const size_t l = e && e[0] ? (size_t)std::max(0LL, atoll(e)) << 20 : 0;
    for (size_t& v : limit) v = l;
  }
  static BlockCache& get() {
    static BlockCache* c = new BlockCache;  // (never destroyed: Bufs may be released during process exit)
    return *c;
  }
  size_t limit_of(int dev) {
    std::lock_guard<std::mutex> g(mu);
    return dev >= 0 && dev < kMaxDev ? limit[dev] : 0;
  }
  void set_limit(int dev, size_t bytes) {
    {
      std::lock_guard<std::mutex> g(mu);
      for (int d = 0; d < kMaxDev; ++d)
        if (dev < 0 || d == dev) limit[d] = bytes;
    }
    trim(dev);
  }
  void* take(size_t want, int dev, size_t* got) {
    Blk b{};
    {
      std::lock_guard<std::mutex> g(mu);
      int best = -1;
      for (int i = 0; i < (int)blocks.size(); ++i)
        if (blocks[i].dev == dev && blocks[i].n >= want && blocks[i].n - want <= want / 8 &&
            (best < 0 || blocks[i].n < blocks[best].n))
          best = i;
      if (best < 0) return nullptr;
      b = blocks[best];
      blocks.erase(blocks.begin() + best);
    }
    if (b.ev) {
      (void)hipEventSynchronize(b.ev);
      (void)hipEventDestroy(b.ev);
    }
    *got = b.n;
    return b.p;
  }
  // keep the block if the device's limit allows (true), else the caller frees it
  bool put(void* p, size_t n, int dev, hipEvent_t ev) {
    std::lock_guard<std::mutex> g(mu);
    size_t t = 0;
    for (const Blk& b : blocks)
      if (b.dev == dev) t += b.n;
    if (dev < 0 || dev >= kMaxDev || t + n > limit[dev]) return false;
    blocks.push_back(Blk{p, n, dev, ev});
    return true;
  }
  // free the device's cached blocks beyond its limit (all of them at limit 0; dev < 0: every device); bytes freed
  size_t trim(int dev) {
    std::vector<Blk> out;
    {
      std::lock_guard<std::mutex> g(mu);
      for (int d = 0; d < kMaxDev; ++d) {
        if (dev >= 0 && d != dev) continue;
        size_t t = 0;
        for (size_t i = 0; i < blocks.size();) {
          if (blocks[i].dev == d && t + blocks[i].n > limit[d]) {
            out.push_back(blocks[i]);
            blocks.erase(blocks.begin() + i);
          } else {
            if (blocks[i].dev == d) t += blocks[i].n;
            ++i;
          }
        }
      }
    }
    return free_blocks(out);
  }
  // free every cached block of `dev` (dev < 0: of every device); bytes freed
  size_t flush(int dev) {
    std::vector<Blk> out;
    {
      std::lock_guard<std::mutex> g(mu);
      for (size_t i = 0; i < blocks.size();) {
        if (dev < 0 || blocks[i].dev == dev) {
          out.push_back(blocks[i]);
          blocks.erase(blocks.begin() + i);
        } else {
          ++i;
        }
      }
    }
    return free_blocks(out);
  }
  size_t cached(int dev) {
    std::lock_guard<std::mutex> g(mu);
    size_t t = 0;
    for (const Blk& b : blocks)
      if (dev < 0 || b.dev == dev) t += b.n;
    return t;
  }

 private:
  static size_t free_blocks(std::vector<Blk>& v) {
    size_t t = 0;
    int cur = -1;
    (void)hipGetDevice(&cur);
    for (Blk& b : v) {
      (void)hipSetDevice(b.dev);
      if (b.ev) {
        (void)hipEventSynchronize(b.ev);
        (void)hipEventDestroy(b.ev);
      }
      (void)hipFree(b.p);
      t += b.n;
    }
    if (cur >= 0 && !v.empty()) (void)hipSetDevice(cur);
    return t;
  }
};

// owning device buffer (grow-only when reused as workspace)
struct Buf {
  void* p = nullptr;
  size_t n = 0;    // bytes asked for (what the index footprint reports)
  size_t cap = 0;  // bytes of the block (a cached block may be up to 1/8 larger)
  int dev = -1;
  Buf() = default;
  Buf(const Buf&) = delete;
  Buf& operator=(const Buf&) = delete;
  ~Buf() { release(); }
  void release() {
    if (p) {
      if (cap >= BlockCache::kCacheMin && BlockCache::get().limit_of(dev) > 0) {
        // a cached block may be handed out at once: order its reuse after the work that may still use it -- an
        // event on the releasing call's stream, nothing if the releaser already waited (index free), a device sync
        // only when neither is known
        int cur = -1;
        (void)hipGetDevice(&cur);
        if (cur != dev) (void)hipSetDevice(dev);
        hipEvent_t ev = nullptr;
        if (!tl_release_synced) {
          if (tl_stream_set && hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess) {
            if (hipEventRecord(ev, tl_stream) != hipSuccess) {
              (void)hipEventDestroy(ev);
              ev = nullptr;
              (void)hipDeviceSynchronize();
            }
          } else {
            (void)hipDeviceSynchronize();
          }
        }
        if (!BlockCache::get().put(p, cap, dev, ev)) {
          if (ev) (void)hipEventDestroy(ev);
          (void)hipFree(p);
        }
        if (cur != dev) (void)hipSetDevice(cur);
      } else {
        (void)hipFree(p);
      }
    }
    p = nullptr;
    n = 0;
    cap = 0;
  }
  void reserve(size_t bytes) {
    if (p && bytes <= cap) {
      if (bytes > n) n = bytes;
      return;
    }
    if (p) HIPCHK(hipDeviceSynchronize());  // in-flight work may still use the old workspace
    release();
    int d = 0;
    HIPCHK(hipGetDevice(&d));
    const size_t want = bytes > 0 ? bytes : 16;
    size_t got = 0;
    if (want >= BlockCache::kCacheMin) p = BlockCache::get().take(want, d, &got);
    if (!p) {
      hipError_t e = hipMalloc(&p, want);
      if (e == hipErrorOutOfMemory) {
        (void)hipGetLastError();
        BlockCache::get().flush(d);
        e = hipMalloc(&p, want);
      }
      if (e != hipSuccess) p = nullptr;
      HIPCHK(e);
      got = want;
    }
    n = want;
    cap = got;
    dev = d;
  }
  template <class T>
  T* as() const { return static_cast<T*>(p); }
};

// an integer engine setting from the environment (timing / diagnostic flags, workspace sizes), read at the call
inline int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e && e[0] ? atoi(e) : dflt;
}

// pinned host memory for the search's small device-to-host reads (hipHostMalloc: the copy is a DMA the host
// can poll for, not a staged pageable copy)
struct HostBuf {
  void* p = nullptr;
  size_t n = 0;
  HostBuf() = default;
  HostBuf(const HostBuf&) = delete;
  HostBuf& operator=(const HostBuf&) = delete;
  ~HostBuf() {
    if (p) (void)hipHostFree(p);
  }
  void reserve(size_t bytes) {
    if (bytes <= n && p) return;
    if (p) {
      HIPCHK(hipDeviceSynchronize());
      (void)hipHostFree(p);
    }
    p = nullptr;
    HIPCHK(hipHostMalloc(&p, bytes > 0 ? bytes : 16, hipHostMallocDefault));
    n = bytes;
  }
  template <class T>
  T* as() const { return static_cast<T*>(p); }
};

// Wait for the stream by polling it: the search's one host sync (the fallback size) sits on the step's critical
// path, and a blocking wait's wake-up adds tens of microseconds to every batch
// host-side timeline of a search (MIVS_HOST_TRACE=1: stderr per call; diagnostics only)
struct HostTrace {
  bool on = false;
  std::chrono::steady_clock::time_point t0, t_first, t_wait0, t_wait1;
  int n_wait = 0;
};
inline HostTrace& host_trace() {
  static thread_local HostTrace t;
  return t;
}

inline void spin_wait(hipStream_t s) {
  HostTrace& ht = host_trace();
  if (ht.on && ht.n_wait++ == 0) ht.t_wait0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t e = hipStreamQuery(s);
    if (e == hipSuccess) break;
    if (e != hipErrorNotReady) HIPCHK(e);
  }
  if (ht.on) ht.t_wait1 = std::chrono::steady_clock::now();
}

inline int cu_count(int device) {
  static std::mutex mu;
  static std::vector<int> cache;
  std::lock_guard<std::mutex> g(mu);
  if ((int)cache.size() <= device) cache.resize(device + 1, 0);
  if (cache[device] == 0) {
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, device));
    cache[device] = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
  }
  return cache[device];
}

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    HIPCHK(hipGetDevice(&prev));
    if (prev != dev) HIPCHK(hipSetDevice(dev));
  }
  ~DeviceGuard() {
    int cur = -1;
    if (hipGetDevice(&cur) == hipSuccess && cur != prev && prev >= 0) (void)hipSetDevice(prev);
  }
};

}  // namespace mivs_capi
