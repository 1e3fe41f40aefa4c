// Host-side cost of the HIP runtime calls one evaluation batch issues
// (kernel launches, event records, cross-stream waits, small async copies),
// measured on the GPU box: informs how much of the batch's "enqueue" time is
// API overhead.  Build: hipcc --offload-arch=gfx950 -O2 api_cost.hip -o api_cost
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>

__global__ void empty_kernel(int* p) {
  if (p && threadIdx.x == 1024) p[0] = 1;
}
struct Big {
  char pad[1024];
};
__global__ void big_arg_kernel(Big b, int* p) {
  if (p && threadIdx.x == 1024) p[0] = b.pad[3];
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  hipStream_t s1, s2;
  hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  hipEvent_t ev;
  hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  int* d = nullptr;
  hipMalloc(&d, 1 << 20);
  void* h = nullptr;
  hipHostMalloc(&h, 1 << 20, 0);
  const int N = 2000;
  Big big{};
  auto bench = [&](const char* name, auto fn) {
    for (int i = 0; i < 50; i++) fn();
    hipDeviceSynchronize();
    const double t0 = now_us();
    for (int i = 0; i < N; i++) fn();
    const double t1 = now_us();
    hipDeviceSynchronize();
    printf("%-40s %.2f us/call\n", name, (t1 - t0) / N);
  };
  bench("hipLaunchKernelGGL empty (8 B arg)", [&] { hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s1, d); });
  bench("hipLaunchKernelGGL 1 KB arg", [&] { hipLaunchKernelGGL(big_arg_kernel, dim3(1), dim3(64), 0, s1, big, d); });
  bench("hipLaunchKernelGGL 2048 blocks", [&] { hipLaunchKernelGGL(empty_kernel, dim3(2048), dim3(256), 0, s1, d); });
  bench("hipEventRecord", [&] { hipEventRecord(ev, s1); });
  bench("hipStreamWaitEvent", [&] { hipStreamWaitEvent(s2, ev, 0); });
  bench("hipMemcpyAsync H2D 64 KB pinned", [&] { hipMemcpyAsync(d, h, 65536, hipMemcpyHostToDevice, s1); });
  bench("hipMemcpyAsync D2H 16 KB pinned", [&] { hipMemcpyAsync(h, d, 16384, hipMemcpyDeviceToHost, s1); });
  bench("launch + hipStreamSynchronize", [&] {
    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s1, d);
    hipStreamSynchronize(s1);
  });
  // a graph of 12 empty kernels over two streams vs 12 launches
  hipGraph_t g;
  hipGraphExec_t ge;
  hipStreamBeginCapture(s1, hipStreamCaptureModeGlobal);
  for (int i = 0; i < 12; i++) hipLaunchKernelGGL(empty_kernel, dim3(64), dim3(256), 0, s1, d);
  hipStreamEndCapture(s1, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  bench("hipGraphLaunch (12 kernels)", [&] { hipGraphLaunch(ge, s1); });
  bench("12 x hipLaunchKernelGGL", [&] {
    for (int i = 0; i < 12; i++) hipLaunchKernelGGL(empty_kernel, dim3(64), dim3(256), 0, s1, d);
  });
  bench("12 launches + sync (round trip)", [&] {
    for (int i = 0; i < 12; i++) hipLaunchKernelGGL(empty_kernel, dim3(64), dim3(256), 0, s1, d);
    hipStreamSynchronize(s1);
  });
  bench("graph (12) + sync (round trip)", [&] {
    hipGraphLaunch(ge, s1);
    hipStreamSynchronize(s1);
  });
  return 0;
}
