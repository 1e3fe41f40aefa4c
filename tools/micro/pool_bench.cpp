// Host pool job round trip (run_static over 1,024 trivial items) of the
// product pool (tas_pool.h) and the pause-spinning variant (pool_spin.h),
// measured on the GPU box host.
// Build: g++ -O2 -std=c++17 -pthread pool_bench.cpp -o pool_bench
#include <cstdio>
#include "../../kueue_oss_amd/csrc/tas_pool.h"
#include "pool_spin.h"

template <class P>
void bench(const char* name, P& p) {
  std::vector<int> v(1024);
  for (int rep = 0; rep < 3; rep++) {
    auto t0 = std::chrono::steady_clock::now();
    const int K = 20000;
    for (int k = 0; k < K; k++) p.run_static(1024, [&](size_t b, size_t e) { for (size_t i = b; i < e; i++) v[i] += 1; });
    auto t1 = std::chrono::steady_clock::now();
    printf("%s run_static round trip: %.2f us (parts %zu)\n", name,
           std::chrono::duration<double, std::micro>(t1 - t0).count() / K, p.parts());
  }
}

int main() {
  bench("product", ktas_pool::HostPool::get());
  std::this_thread::sleep_for(std::chrono::milliseconds(20));  // the product workers fall asleep
  bench("spin", ktas_pool3::HostPool::get());
}
