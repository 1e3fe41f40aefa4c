// Device-side gaps the evaluation batch pays between its kernels and at its
// final synchronization, measured on the GPU box: the round trip of a launch
// + hipStreamSynchronize under the default and the spin scheduling flags, the
// per-kernel cost of a chain of dependent small kernels on one stream, and a
// cross-stream event hand-off.  Build: hipcc --offload-arch=gfx950 -O2
// sync_cost.hip -o sync_cost ; run: ./sync_cost [spin]
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>

__global__ void tiny_kernel(int* p, int v) {
  if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += v;
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  if (argc > 1 && !strcmp(argv[1], "spin")) hipSetDeviceFlags(hipDeviceScheduleSpin);
  if (argc > 1 && !strcmp(argv[1], "yield")) hipSetDeviceFlags(hipDeviceScheduleYield);
  hipStream_t s1, s2;
  hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  hipEvent_t ev, a, b;
  hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  hipEventCreate(&a);
  hipEventCreate(&b);
  int* d = nullptr;
  hipMalloc(&d, 4096);
  hipMemset(d, 0, 4096);
  int* h = nullptr;
  hipHostMalloc(&h, 4096, 0);
  const int N = 2000;
  auto bench = [&](const char* name, auto fn) {
    for (int i = 0; i < 50; i++) fn();
    hipDeviceSynchronize();
    const double t0 = now_us();
    for (int i = 0; i < N; i++) fn();
    hipDeviceSynchronize();
    const double t1 = now_us();
    printf("%-48s %.2f us\n", name, (t1 - t0) / N);
  };
  bench("launch + hipStreamSynchronize", [&] {
    hipLaunchKernelGGL(tiny_kernel, dim3(1), dim3(64), 0, s1, d, 1);
    hipStreamSynchronize(s1);
  });
  bench("launch + D2H 4 B + hipStreamSynchronize", [&] {
    hipLaunchKernelGGL(tiny_kernel, dim3(1), dim3(64), 0, s1, d, 1);
    hipMemcpyAsync(h, d, 4, hipMemcpyDeviceToHost, s1);
    hipStreamSynchronize(s1);
  });
  bench("launch + event + hipEventSynchronize", [&] {
    hipLaunchKernelGGL(tiny_kernel, dim3(1), dim3(64), 0, s1, d, 1);
    hipEventRecord(ev, s1);
    hipEventSynchronize(ev);
  });
  // device time per kernel of a dependent chain (events around 64 kernels)
  for (int k : {1, 16, 64}) {
    float best = 1e9f;
    for (int r = 0; r < 20; r++) {
      hipEventRecord(a, s1);
      for (int i = 0; i < k; i++) hipLaunchKernelGGL(tiny_kernel, dim3(256), dim3(256), 0, s1, d, 1);
      hipEventRecord(b, s1);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      best = ms < best ? ms : best;
    }
    printf("chain of %2d kernels: device %.2f us per kernel\n", k, best * 1000.f / k);
  }
  // an event record between two kernels of one stream, by event flags
  {
    struct {
      const char* name;
      unsigned flags;
    } kinds[] = {{"default", hipEventDefault},
                 {"disable-timing", hipEventDisableTiming},
                 {"disable-system-fence", hipEventDisableSystemFence},
                 {"disable-timing|system-fence", hipEventDisableTiming | hipEventDisableSystemFence}};
    for (auto& k : kinds) {
      hipEvent_t mid;
      hipEventCreateWithFlags(&mid, k.flags);
      float best = 1e9f;
      for (int r = 0; r < 30; r++) {
        hipEventRecord(a, s1);
        for (int i = 0; i < 16; i++) {
          hipLaunchKernelGGL(tiny_kernel, dim3(256), dim3(256), 0, s1, d, 1);
          hipEventRecord(mid, s1);
        }
        hipEventRecord(b, s1);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        best = ms < best ? ms : best;
      }
      printf("kernel + event record (%s): device %.2f us per pair\n", k.name, best * 1000.f / 16);
      // cross-stream hand-off through this kind of event
      float best2 = 1e9f;
      for (int r = 0; r < 50; r++) {
        hipEventRecord(a, s1);
        hipLaunchKernelGGL(tiny_kernel, dim3(1), dim3(64), 0, s1, d, 1);
        hipEventRecord(mid, s1);
        hipStreamWaitEvent(s2, mid, 0);
        hipLaunchKernelGGL(tiny_kernel, dim3(1), dim3(64), 0, s2, d, 1);
        hipEventRecord(b, s2);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        best2 = ms < best2 ? ms : best2;
      }
      printf("  s1 kernel -> %s event -> s2 kernel: device %.2f us\n", k.name, best2 * 1000.f);
      hipEventDestroy(mid);
    }
  }
  // cross-stream hand-off: s1 kernel -> event -> s2 kernel, timed on s1/s2 events
  {
    float best = 1e9f;
    for (int r = 0; r < 50; r++) {
      hipEventRecord(a, s1);
      hipLaunchKernelGGL(tiny_kernel, dim3(1), dim3(64), 0, s1, d, 1);
      hipEventRecord(ev, s1);
      hipStreamWaitEvent(s2, ev, 0);
      hipLaunchKernelGGL(tiny_kernel, dim3(1), dim3(64), 0, s2, d, 1);
      hipEventRecord(b, s2);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      best = ms < best ? ms : best;
    }
    printf("s1 kernel -> event -> s2 kernel: device %.2f us\n", best * 1000.f);
  }
  return 0;
}
