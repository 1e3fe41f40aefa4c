// tas_pool.h — the persistent host worker pool shared by the host layer
// (tas_host.cpp) and the device layer's per-batch host work (tas_device.hip).
// One pool per process (HostPool::get is an inline function: one instance
// across translation units).  Not part of the public ABI.
#pragma once
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <pthread.h>
#include <sched.h>
#include <cstdio>
#include <string>
#include <thread>
#include <vector>

namespace ktas_pool {

// Persistent host workers for per-batch loops that are independent per
// workload.  Two modes:
//  * run(n, grain, fn): chunks of `grain` items taken by whoever is free; the
//    calling thread takes chunks too and only waits for chunks already taken,
//    so a worker still asleep never delays a call;
//  * run_static(n, fn): the same contiguous part [t*n/T, (t+1)*n/T) always
//    goes to the same thread t (t = 0: the caller), so the phases of one
//    batch that touch the same workloads (compile, batch assembly, device
//    records, decode) find them in that core's cache instead of pulling them
//    across cores.
// Idle workers spin briefly for the next job (steps follow each other within
// a millisecond), then sleep after 2 ms.  KUEUE_TAS_HOST_THREADS sets the
// worker count (0: inline).
class HostPool {
 public:
  static HostPool& get() {
    static HostPool pool;
    return pool;
  }
  size_t workers() const { return threads_.size(); }
  size_t parts() const { return threads_.size() + 1; }
  // fn(begin, end) over [0, n) in chunks of `grain`; one job at a time
  template <class F>
  void run(size_t n, size_t grain, F&& fn) {
    if (inline_only() || n <= grain) {
      if (n) fn(size_t(0), n);
      return;
    }
    std::function<void(size_t, size_t)> f(std::ref(fn));
    submit(n, grain, &f, false);
  }
  // fn(begin, end) over the parts() static parts of [0, n)
  template <class F>
  void run_static(size_t n, F&& fn) {
    if (inline_only() || n < 2 * parts()) {  // the same parts, one after the other
      for (size_t t = 0; t < parts(); t++)
        if (part_begin(n, t, parts()) < part_begin(n, t + 1, parts())) fn(part_begin(n, t, parts()), part_begin(n, t + 1, parts()));
      return;
    }
    std::function<void(size_t, size_t)> f(std::ref(fn));
    submit(n, 0, &f, true);
  }
  // the static part of [0, n) that thread t runs
  static size_t part_begin(size_t n, size_t t, size_t T) { return n * t / T; }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
      epoch_.fetch_add(1);
    }
    cv_.notify_all();
    for (auto& t : threads_) t.join();
  }

 private:
  static constexpr size_t kMaxParts = 64;
  struct Job {
    std::function<void(size_t, size_t)>* fn = nullptr;
    size_t n = 0, grain = 1, chunks = 0;
    bool fixed = false;  // run_static: chunk t is thread t's part
    std::atomic<size_t> next{0}, done{0};
    // run_static: a part is run by whoever claims it first — its own thread,
    // or the caller once its part is done and the owner has not started (a
    // worker the OS has not scheduled yet, e.g. after its core ran another
    // task, does not hold the whole job up)
    std::atomic<uint8_t> claimed[kMaxParts] = {};
    std::mutex errMu;
    std::exception_ptr err;  // the first exception a chunk threw, rethrown on the caller
  };
  void submit(size_t n, size_t grain, std::function<void(size_t, size_t)>* f, bool fixed) {
    std::lock_guard<std::mutex> one(callMu_);
    auto job = std::make_shared<Job>();
    job->fn = f;
    job->n = n;
    job->grain = grain;
    job->fixed = fixed;
    job->chunks = fixed ? parts() : (n + grain - 1) / grain;
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_ = job;
      epoch_.fetch_add(1, std::memory_order_release);
    }
    cv_.notify_all();
    work(*job, 0);
    if (fixed)  // parts whose owner has not started yet
      for (size_t t = 1; t < job->chunks; t++) run_part(*job, t);
    // every chunk has finished (thrown or not) before `f` — on the caller's
    // stack — goes out of scope
    while (job->done.load(std::memory_order_acquire) != job->chunks) std::this_thread::yield();
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_.reset();  // late workers keep their reference; its chunks are exhausted
    }
    if (job->err) std::rethrow_exception(job->err);
  }
  static void call(Job& j, size_t b, size_t e) {
    try {
      (*j.fn)(b, e);
    } catch (...) {
      std::lock_guard<std::mutex> lk(j.errMu);
      if (!j.err) j.err = std::current_exception();
    }
  }
  // CPUs near the creating thread (the caller of every job: part 0): the
  // other cores of its last-level cache, one SMT thread each, so a static
  // part's data moves between cores of one L3 at most (a worker on the other
  // socket of a two-socket host reads the caller's records across it).
  // KUEUE_TAS_HOST_PIN=0 leaves placement to the OS.
  static std::vector<int> near_cpus(size_t want) {
    std::vector<int> out;
    const int self = sched_getcpu();
    if (self < 0) return out;
    auto read_list = [](const std::string& path) {
      std::vector<int> v;
      FILE* f = fopen(path.c_str(), "r");
      if (!f) return v;
      char buf[4096] = {};
      const size_t k = fread(buf, 1, sizeof buf - 1, f);
      fclose(f);
      buf[k] = 0;
      for (char* p = buf; *p;) {  // "a-b,c,d-e"
        char* q = nullptr;
        const long a = strtol(p, &q, 10);
        if (q == p) break;
        long b = a;
        if (*q == '-') b = strtol(q + 1, &q, 10);
        for (long x = a; x <= b; x++) v.push_back(int(x));
        p = *q == ',' ? q + 1 : q;
        if (*p == '\n') break;
      }
      return v;
    };
    const std::string base = "/sys/devices/system/cpu/cpu";
    const std::vector<int> l3 = read_list(base + std::to_string(self) + "/cache/index3/shared_cpu_list");
    cpu_set_t allowed;
    CPU_ZERO(&allowed);
    if (sched_getaffinity(0, sizeof allowed, &allowed) != 0) return out;
    std::vector<int> used = read_list(base + std::to_string(self) + "/topology/thread_siblings_list");
    for (int c : l3) {
      if (out.size() >= want) break;
      if (!CPU_ISSET(c, &allowed) || std::find(used.begin(), used.end(), c) != used.end()) continue;
      out.push_back(c);
      for (int sib : read_list(base + std::to_string(c) + "/topology/thread_siblings_list")) used.push_back(sib);
    }
    if (out.size() < want) out.clear();  // not enough cores in the L3: leave placement to the OS
    return out;
  }
  HostPool() {
    size_t n = std::min<size_t>(4, std::max<unsigned>(2, std::thread::hardware_concurrency()) - 1);
    if (const char* e = getenv("KUEUE_TAS_HOST_THREADS")) n = size_t(std::max(0, atoi(e)));
    n = std::min(n, kMaxParts - 1);
    const char* pin_env = getenv("KUEUE_TAS_HOST_PIN");
    const std::vector<int> cpus = (pin_env && atoi(pin_env) == 0) ? std::vector<int>() : near_cpus(n);
    // every worker starts from the epoch before any job: a static job posted
    // before a worker first runs is still seen by it (it owns a part)
    const uint64_t e0 = epoch_.load();
    for (size_t i = 0; i < n; i++)
      threads_.emplace_back([this, i, e0, cpu = cpus.empty() ? -1 : cpus[i]] {
        if (cpu >= 0) {
          cpu_set_t set;
          CPU_ZERO(&set);
          CPU_SET(cpu, &set);
          (void)pthread_setaffinity_np(pthread_self(), sizeof set, &set);
        }
        loop(i + 1, e0);
      });
    // a child forked without exec has none of the workers: it runs inline
    pthread_atfork(nullptr, nullptr, [] { forked_child() = true; });
  }
  static bool& forked_child() {
    static bool f = false;
    return f;
  }
  bool inline_only() const { return threads_.empty() || forked_child(); }
  static void run_part(Job& j, size_t t) {
    if (j.claimed[t].exchange(1, std::memory_order_acq_rel)) return;  // its owner (or the caller) has it
    const size_t T = j.chunks;
    call(j, part_begin(j.n, t, T), part_begin(j.n, t + 1, T));
    j.done.fetch_add(1, std::memory_order_release);
  }
  void work(Job& j, size_t self) {
    if (j.fixed) {  // this thread's own part only
      run_part(j, self);
      return;
    }
    for (;;) {
      const size_t c = j.next.fetch_add(1, std::memory_order_relaxed);
      if (c >= j.chunks) return;
      const size_t b = c * j.grain;
      call(j, b, std::min(j.n, b + j.grain));
      j.done.fetch_add(1, std::memory_order_release);
    }
  }
  void loop(size_t self, uint64_t seen) {
    for (;;) {
      const auto spin_until = std::chrono::steady_clock::now() + std::chrono::microseconds(2000);
      while (epoch_.load(std::memory_order_acquire) == seen && std::chrono::steady_clock::now() < spin_until)
        std::this_thread::yield();
      std::shared_ptr<Job> job;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || epoch_.load() != seen; });
        if (stop_) return;
        seen = epoch_.load();
        job = job_;
      }
      if (job) work(*job, self);
    }
  }
  std::vector<std::thread> threads_;
  std::mutex mu_, callMu_;
  std::condition_variable cv_;
  std::atomic<uint64_t> epoch_{0};
  std::shared_ptr<Job> job_;
  bool stop_ = false;
};

}  // namespace ktas_pool
