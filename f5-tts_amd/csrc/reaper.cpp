// Reaper thread for the deferred release of device resources (reaper.h).
#include "reaper.h"

#include <cerrno>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <system_error>
#include <thread>

#include "../../include/f5h.h"

namespace f5h {

void UseLog::note(hipStream_t st) {
  std::lock_guard<std::mutex> lk(m);
  hipEvent_t e = nullptr;
  for (auto& p : ev)
    if (p.first == st) e = p.second;
  if (!e) {
    // a new stream: first drop the entries whose last use has completed (a caller that makes a stream per
    // request would otherwise grow the list, and this scan, for the object's lifetime); one completed event
    // is reused for the new stream instead of creating one
    for (size_t i = 0; i < ev.size();) {
      if (hipEventQuery(ev[i].second) == hipSuccess) {
        if (!e)
          e = ev[i].second;
        else
          (void)hipEventDestroy(ev[i].second);
        ev[i] = ev.back();
        ev.pop_back();
      } else {
        (void)hipGetLastError();  // hipErrorNotReady
        ++i;
      }
    }
    if (!e && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
      (void)hipGetLastError();
      return;
    }
    ev.emplace_back(st, e);
  }
  if (hipEventRecord(e, st) != hipSuccess) (void)hipGetLastError();
}

std::vector<hipEvent_t> UseLog::take() {
  std::lock_guard<std::mutex> lk(m);
  std::vector<hipEvent_t> out;
  for (auto& p : ev) out.push_back(p.second);
  ev.clear();
  return out;
}

namespace {
std::mutex g_pool_m;
std::vector<std::pair<int, hipMemPool_t>> g_pools;

hipMemPool_t pool_of(int dev) {
  std::lock_guard<std::mutex> lk(g_pool_m);
  for (auto& p : g_pools)
    if (p.first == dev) return p.second;
  hipMemPoolProps props{};
  props.allocType = hipMemAllocationTypePinned;
  props.handleTypes = hipMemHandleTypeNone;
  props.location.type = hipMemLocationTypeDevice;
  props.location.id = dev;
  hipMemPool_t pool = nullptr;
  if (hipMemPoolCreate(&pool, &props) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  // Default: never trimmed implicitly (a trim at a synchronisation point frees memory, and that waits for the
  // device). Released memory then stays reserved for this process's next engine / Vocos / log-mel object:
  // f5h_release_pending(2) (Python: f5_tts_amd.release_memory()) returns it; F5H_POOL_KEEP_MB=<n> caps what
  // the pool keeps past a synchronisation point instead (memory).
  uint64_t keep = ~0ull;
  if (const char* kv = getenv("F5H_POOL_KEEP_MB")) {
    // applied only when the whole value is a number of MB: anything else ("", "off", "inf", "12x") would parse as
    // 0 and trim the pool at every synchronisation point, the opposite of the default
    char* end = nullptr;
    errno = 0;
    const unsigned long long mb = strtoull(kv, &end, 10);
    if (*kv && end && *end == '\0' && errno == 0 && mb < (1ull << 44))
      keep = (uint64_t)mb << 20;
    else
      std::fprintf(stderr, "[f5h] F5H_POOL_KEEP_MB=\"%s\" is not a number of MB: ignored (the pool keeps all)\n", kv);
  }
  (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
  g_pools.emplace_back(dev, pool);
  return pool;
}
}  // namespace

void* dev_alloc(int dev, size_t bytes, hipStream_t st) {
  hipMemPool_t pool = pool_of(dev);
  if (!pool) return nullptr;
  void* p = nullptr;
  if (hipMallocFromPoolAsync(&p, bytes, pool, st) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return p;
}

void dev_free(void* p, hipStream_t st) {
  if (p && hipFreeAsync(p, st) != hipSuccess) (void)hipGetLastError();
}

void pool_trim() {
  std::lock_guard<std::mutex> lk(g_pool_m);
  for (auto& p : g_pools) {
    (void)hipSetDevice(p.first);
    (void)hipDeviceSynchronize();
    (void)hipMemPoolTrimTo(p.second, 0);
  }
}

namespace {
struct Reaper {
  std::mutex m;
  std::condition_variable work, idle;
  std::deque<std::pair<int, std::function<void()>>> q;
  int running = 0;
  bool started = false;
};
// never destroyed: the thread is detached and may outlive static destruction order
Reaper& R() {
  static Reaper* r = new Reaper();
  return *r;
}

void loop() {
  Reaper& r = R();
  std::unique_lock<std::mutex> lk(r.m);
  for (;;) {
    r.work.wait(lk, [&] { return !r.q.empty(); });
    auto item = std::move(r.q.front());
    r.q.pop_front();
    ++r.running;
    lk.unlock();
    (void)hipSetDevice(item.first);
    item.second();
    (void)hipGetLastError();
    lk.lock();
    --r.running;
    if (r.q.empty() && r.running == 0) r.idle.notify_all();
  }
}

// exit(): run what was retired before the HIP runtime's own teardown (registered after the runtime was
// initialised, so it runs before the runtime's static destructors)
void drain_at_exit() { (void)reaper_pending(true); }
}  // namespace

void retire(int dev, std::function<void()> job) {
  Reaper& r = R();
  {
    std::lock_guard<std::mutex> lk(r.m);
    if (!r.started) {
      try {
        std::thread(loop).detach();
        r.started = true;
        std::atexit(drain_at_exit);
      } catch (const std::system_error&) {
      }
    }
    if (r.started) {
      r.q.emplace_back(dev, std::move(job));
      r.work.notify_one();
      return;
    }
  }
  (void)hipSetDevice(dev);  // no thread: release inline (waits on the object's own events only)
  job();
}

int reaper_pending(bool wait) {
  Reaper& r = R();
  std::unique_lock<std::mutex> lk(r.m);
  if (wait && r.started) r.idle.wait(lk, [&] { return r.q.empty() && r.running == 0; });
  return (int)r.q.size() + r.running;
}

}  // namespace f5h

extern "C" int f5h_release_pending(int32_t wait) {
  const int n = f5h::reaper_pending(wait != 0);
  if (wait == 2 && n == 0) f5h::pool_trim();
  return n;
}
