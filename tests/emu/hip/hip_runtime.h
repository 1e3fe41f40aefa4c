// TEST INFRASTRUCTURE: a CPU SIMT emulator standing in for <hip/hip_runtime.h>
// so that the UNMODIFIED kernel sources (kueue_oss_amd/csrc/tas_kernels.hip,
// tas_device.hip) can be compiled with g++ and parity-tested on a machine
// without a GPU (tests/emu/build_emu.sh).  Never linked into the product.
//
// Model: every GPU thread is a fiber (ucontext); a block's fibers run on one
// OS thread, round-robin; blocks run sequentially.  Wave-level primitives
// (__shfl*, __ballot, wave barriers, fences) synchronize the 64 lanes of a
// wave; __syncthreads synchronizes the block.  __shared__ locals become
// function statics, per OS thread (one block of a stream runs at a time).
#pragma once
#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <cstdio>
#include <functional>
#include <tuple>
#include <vector>

#define KTAS_WAVES_PER_EU(n)  // occupancy hint: meaningless on the CPU
#define __global__
#define __device__
#define __host__
#define __forceinline__ inline
#define __launch_bounds__(...)
#define __shared__ static thread_local
#define __constant__
#define HIP_SYMBOL(x) (&(x))

struct dim3 {
  unsigned x, y, z;
  dim3(unsigned a = 1, unsigned b = 1, unsigned c = 1) : x(a), y(b), z(c) {}
};

namespace emu {
struct Ctx {
  dim3 tid, bid, bdim, gdim;
};
Ctx* cur();
void wave_barrier();
void block_barrier();
uint64_t wave_exchange(uint64_t v, int src);       // value of lane `src`
uint64_t wave_ballot(bool p);
void* dynamic_lds();
void launch(dim3 grid, dim3 block, size_t shmem, const std::function<void()>& fn);

// Streams are DEFERRED queues: nothing a stream holds runs until something
// needs it — hipStreamSynchronize of that stream, a hipStreamWaitEvent
// executed by another stream (which drains the recording stream up to the
// event), or a synchronous API (hipMemcpy, hipFree, ...: all streams).  So a
// side stream's work runs as late as its dependencies allow, and a missing
// event dependency shows up as a wrong result instead of passing by luck.
struct Stream;
struct Event {
  Stream* stream = nullptr;
  size_t pos = 0;  // ops of `stream` that precede the record
};
struct Stream {
  std::vector<std::function<void()>> ops;
  size_t done = 0;
  void run_until(size_t n) {
    while (done < n && done < ops.size()) {
      auto op = std::move(ops[done]);
      done++;  // before running: a wait inside may re-enter this stream's drain
      op();
    }
  }
  void drain() { run_until(ops.size()); }
};
std::vector<Stream*>& streams();
inline void drain_all() {
  for (bool again = true; again;) {
    again = false;
    for (Stream* s : streams())
      if (s->done < s->ops.size()) {
        s->drain();
        again = true;
      }
  }
}
}  // namespace emu

#define threadIdx (emu::cur()->tid)
#define blockIdx (emu::cur()->bid)
#define blockDim (emu::cur()->bdim)
#define gridDim (emu::cur()->gdim)

inline void __syncthreads() { emu::block_barrier(); }
#define __builtin_amdgcn_fence(order, scope) emu::wave_barrier()
#define __builtin_amdgcn_wave_barrier() emu::wave_barrier()
#define __builtin_amdgcn_s_waitcnt(x) ((void)(x))  // the emulator's memory is sequentially consistent

inline int __lane_of_cur() { return int(emu::cur()->tid.x & 63u); }
template <typename T>
inline T __shfl(T v, int src, int width = 64) {
  (void)width;
  uint64_t bits = 0;
  memcpy(&bits, &v, sizeof(T));
  uint64_t r = emu::wave_exchange(bits, src & 63);
  T out;
  memcpy(&out, &r, sizeof(T));
  return out;
}
// DPP / swizzle lane permutations (the controls the kernels use)
inline int __builtin_amdgcn_update_dpp(int old, int v, int ctrl, int row_mask, int, bool bound_ctrl) {
  const int l = __lane_of_cur();
  const int row = l >> 4;
  int src = l;
  bool ok = true;
  if (ctrl < 0x100) src = (l & ~3) | ((ctrl >> (2 * (l & 3))) & 3);  // quad_perm
  else if (ctrl == 0x140) src = (l & ~15) | (15 - (l & 15));          // row_mirror
  else if (ctrl == 0x141) src = (l & ~7) | (7 - (l & 7));             // row_half_mirror
  else if (ctrl > 0x110 && ctrl <= 0x11F) {                           // row_shr:n
    src = l - (ctrl - 0x110);
    ok = src >= 0 && (src >> 4) == row;
  } else if (ctrl == 0x142) {  // row_bcast:15: lane 15 of the previous row
    src = row * 16 - 1;
    ok = row > 0;
  } else if (ctrl == 0x143) {  // row_bcast:31: lane 31 to rows 2 and 3
    src = 31;
    ok = row >= 2;
  } else {
    abort();
  }
  const int r = int(emu::wave_exchange(uint64_t(uint32_t(v)), ok ? src : l));  // collective: every lane calls
  if (!((row_mask >> row) & 1)) return old;  // disabled row: not written
  if (!ok) return bound_ctrl ? 0 : old;
  return r;
}
// v_readlane takes its lane from an SGPR: a lane index that differs across
// the wave is a kernel bug (hardware would use one lane's index for all)
inline int __builtin_amdgcn_readlane(int v, int lane) {
  const int lane0 = int(emu::wave_exchange(uint64_t(uint32_t(lane)), 0));
  if (emu::wave_ballot(lane != lane0) != 0) {
    fprintf(stderr, "emu: __builtin_amdgcn_readlane with a non-uniform lane index\n");
    abort();
  }
  return int(emu::wave_exchange(uint64_t(uint32_t(v)), lane & 63));
}
inline int __builtin_amdgcn_ds_swizzle(int v, int pattern) {
  if (pattern & 0x8000) abort();  // bit mode only
  const int l = __lane_of_cur();
  const int and_m = pattern & 31, or_m = (pattern >> 5) & 31, xor_m = (pattern >> 10) & 31;
  const int src = (l & ~31) | ((((l & 31) & and_m) | or_m) ^ xor_m);
  return int(emu::wave_exchange(uint64_t(uint32_t(v)), src));
}
// gfx950 v_permlane16_swap / v_permlane32_swap with vdst = old, vsrc = src:
// the odd 16-lane rows (upper 32-lane half) of vdst trade places with the
// even rows (lower half) of vsrc; returns {vdst', vsrc'}
struct emu_u32x2 {
  uint32_t v[2];
  uint32_t operator[](int i) const { return v[i]; }
};
inline emu_u32x2 emu_permlane_swap(uint32_t old, uint32_t src, int span) {
  const int l = __lane_of_cur();
  const uint32_t o = uint32_t(emu::wave_exchange(uint64_t(old), l ^ span));
  const uint32_t s = uint32_t(emu::wave_exchange(uint64_t(src), l ^ span));
  if (l & span) return {{s, src}};  // vdst' = src of the partner row, vsrc' keeps its own
  return {{old, o}};                // vdst' keeps its own, vsrc' = old of the partner row
}
inline emu_u32x2 __builtin_amdgcn_permlane16_swap(uint32_t old, uint32_t src, bool, bool) {
  return emu_permlane_swap(old, src, 16);
}
inline emu_u32x2 __builtin_amdgcn_permlane32_swap(uint32_t old, uint32_t src, bool, bool) {
  return emu_permlane_swap(old, src, 32);
}
template <typename T>
inline T __shfl_xor(T v, int mask, int width = 64) {
  (void)width;
  return __shfl(v, __lane_of_cur() ^ mask, 64);
}
inline unsigned long long __ballot(int p) { return emu::wave_ballot(p != 0); }
inline int __popcll(unsigned long long x) { return __builtin_popcountll(x); }
inline int __ffsll(unsigned long long x) { return __builtin_ffsll((long long)x); }
inline int __ffsll(long long x) { return __builtin_ffsll(x); }
inline uint64_t __umul64hi(uint64_t a, uint64_t b) { return uint64_t(((unsigned __int128)a * b) >> 64); }
// fibers of one block share one OS thread: plain read-modify-write is atomic
inline int atomicAdd(int* p, int v) { int o = *p; *p = o + v; return o; }
inline unsigned atomicAdd(unsigned* p, unsigned v) { unsigned o = *p; *p = o + v; return o; }
inline unsigned long long atomicAdd(unsigned long long* p, unsigned long long v) {
  unsigned long long o = *p;
  *p = o + v;
  return o;
}
inline unsigned long long atomicCAS(unsigned long long* p, unsigned long long cmp, unsigned long long v) {
  unsigned long long o = *p;
  if (o == cmp) *p = v;
  return o;
}
inline unsigned atomicOr(unsigned* p, unsigned v) { unsigned o = *p; *p = o | v; return o; }
inline int atomicOr(int* p, int v) { int o = *p; *p = o | v; return o; }
inline int atomicMax(int* p, int v) { int o = *p; if (v > o) *p = v; return o; }
inline int atomicAnd(int* p, int v) { int o = *p; *p = o & v; return o; }
inline int atomicMin(int* p, int v) { int o = *p; *p = v < o ? v : o; return o; }
inline unsigned atomicAnd(unsigned* p, unsigned v) { unsigned o = *p; *p = o & v; return o; }
inline void __threadfence() {}
inline void __threadfence_block() {}
// device-scope loads that bypass L1 on hardware; plain loads here
#define __HIP_MEMORY_SCOPE_AGENT 3
template <class T>
inline T __hip_atomic_load(const T* p, int, int) { return *p; }
using std::max;
using std::min;

// ---- runtime API subset ----
typedef int hipError_t;
constexpr hipError_t hipSuccess = 0;
constexpr hipError_t hipErrorInvalidValue = 1;
typedef emu::Stream* hipStream_t;
typedef emu::Event* hipEvent_t;
enum hipMemcpyKind { hipMemcpyHostToDevice = 1, hipMemcpyDeviceToHost = 2, hipMemcpyDeviceToDevice = 3 };
constexpr unsigned hipStreamNonBlocking = 1;
constexpr unsigned hipHostMallocDefault = 0;
constexpr unsigned hipHostMallocMapped = 2;
constexpr unsigned hipHostMallocCoherent = 0x40000000;
inline const char* hipGetErrorString(hipError_t) { return "emu error"; }
inline hipError_t hipGetDeviceCount(int* n) { *n = 1; return hipSuccess; }
inline hipError_t hipSetDevice(int) { return hipSuccess; }
inline hipError_t hipGetLastError() { return hipSuccess; }
template <typename T>
inline hipError_t hipMalloc(T** p, size_t bytes) {
  *p = static_cast<T*>(calloc(1, bytes));
  return *p ? hipSuccess : 2;
}
inline hipError_t hipFree(void* p) {
  emu::drain_all();
  free(p);
  return hipSuccess;
}
template <typename T>
inline hipError_t hipHostMalloc(T** p, size_t bytes, unsigned) {
  *p = static_cast<T*>(calloc(1, bytes));
  return *p ? hipSuccess : 2;
}
inline hipError_t hipHostFree(void* p) {
  emu::drain_all();
  free(p);
  return hipSuccess;
}
inline hipError_t hipHostGetDevicePointer(void** d, void* h, unsigned) { *d = h; return hipSuccess; }
// every pointer is "device" memory to the emulated kernels (they run on the host)
enum hipMemoryType { hipMemoryTypeUnregistered = 0, hipMemoryTypeHost = 1, hipMemoryTypeDevice = 2 };
struct hipPointerAttribute_t {
  hipMemoryType type;
  int device;
};
inline hipError_t hipPointerGetAttributes(hipPointerAttribute_t* a, const void*) {
  a->type = hipMemoryTypeDevice;
  a->device = 0;
  return hipSuccess;
}
inline hipError_t hipMemcpyAsync(void* d, const void* s, size_t n, hipMemcpyKind, hipStream_t st) {
  if (n) st->ops.push_back([=]() { memmove(d, s, n); });
  return hipSuccess;
}
inline hipError_t hipMemcpyToSymbolAsync(const void* sym, const void* s, size_t n, size_t off, hipMemcpyKind k,
                                         hipStream_t st) {
  return hipMemcpyAsync(static_cast<char*>(const_cast<void*>(sym)) + off, s, n, k, st);
}
inline hipError_t hipMemcpy(void* d, const void* s, size_t n, hipMemcpyKind) {
  emu::drain_all();
  if (n) memmove(d, s, n);
  return hipSuccess;
}
struct int4 {
  int x, y, z, w;
};
struct int2 {
  int x, y;
};
inline int2 make_int2(int x, int y) { return int2{x, y}; }
inline int4 make_int4(int x, int y, int z, int w) { return int4{x, y, z, w}; }
inline hipError_t hipMemsetAsync(void* d, int v, size_t n, hipStream_t st) {
  st->ops.push_back([=]() { memset(d, v, n); });
  return hipSuccess;
}
inline hipError_t hipStreamCreateWithFlags(hipStream_t* s, unsigned) {
  *s = new emu::Stream();
  emu::streams().push_back(*s);
  return hipSuccess;
}
inline hipError_t hipStreamCreateWithPriority(hipStream_t* s, unsigned flags, int) {
  return hipStreamCreateWithFlags(s, flags);  // priorities only order the hardware dispatcher
}
inline hipError_t hipDeviceGetStreamPriorityRange(int* lo, int* hi) {
  *lo = 0;
  *hi = -1;
  return hipSuccess;
}
inline hipError_t hipStreamSynchronize(hipStream_t s) {
  s->drain();
  return hipSuccess;
}
inline hipError_t hipStreamDestroy(hipStream_t s) {
  emu::drain_all();
  auto& v = emu::streams();
  v.erase(std::find(v.begin(), v.end(), s));
  delete s;
  return hipSuccess;
}
inline hipError_t hipEventCreate(hipEvent_t* e) {
  *e = new emu::Event();
  return hipSuccess;
}
inline hipError_t hipEventRecord(hipEvent_t e, hipStream_t s) {
  e->stream = s;
  e->pos = s->ops.size();
  return hipSuccess;
}
inline hipError_t hipStreamWaitEvent(hipStream_t s, hipEvent_t e, unsigned) {
  emu::Stream* src = e->stream;
  const size_t pos = e->pos;
  if (src && src != s) s->ops.push_back([=]() { src->run_until(pos); });
  return hipSuccess;
}
inline hipError_t hipEventElapsedTime(float* ms, hipEvent_t, hipEvent_t) { *ms = 0.f; return hipSuccess; }
constexpr unsigned hipEventDisableTiming = 2;
constexpr unsigned hipEventDisableSystemFence = 0x20000000;
inline hipError_t hipEventCreateWithFlags(hipEvent_t* e, unsigned) { return hipEventCreate(e); }
inline hipError_t hipEventSynchronize(hipEvent_t e) {  // the recording stream up to the event
  if (e->stream) e->stream->run_until(e->pos);
  return hipSuccess;
}
enum hipFuncAttribute { hipFuncAttributeMaxDynamicSharedMemorySize = 8 };
inline hipError_t hipFuncSetAttribute(const void*, hipFuncAttribute, int) { return hipSuccess; }  // LDS is host memory here
struct hipFuncAttributes {
  size_t sharedSizeBytes;
};
// static LDS: the hardware's budget is what the kernels' checks reason about (a fixed figure here)
inline hipError_t hipFuncGetAttributes(hipFuncAttributes* a, const void*) {
  a->sharedSizeBytes = 8 * 1024;
  return hipSuccess;
}
inline hipError_t hipEventDestroy(hipEvent_t e) { delete e; return hipSuccess; }

// kernel arguments are captured by value: the launch may run after the caller's locals are gone
#define hipLaunchKernelGGL(kernel, grid, block, shmem, stream, ...)                                              \
  do {                                                                                                            \
    const dim3 emu_g_ = dim3(grid), emu_b_ = dim3(block);                                                         \
    const size_t emu_sh_ = size_t(shmem);                                                                         \
    auto emu_a_ = std::make_tuple(__VA_ARGS__); /* arguments bind at the launch, as on the device */            \
    (stream)->ops.push_back(                                                                                      \
        [=]() { emu::launch(emu_g_, emu_b_, emu_sh_, [=]() { std::apply(kernel, emu_a_); }); });                 \
  } while (0)

// every lane holds the same value where the kernels use it (wave-uniform data)
#define __builtin_amdgcn_readfirstlane(v) (v)
inline uint64_t wall_clock64() { return 0; }
inline int __popc(unsigned x) { return __builtin_popcount(x); }
