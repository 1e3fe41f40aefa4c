// TEST INFRASTRUCTURE: fiber-based SIMT emulator runtime (see hip/hip_runtime.h).
#include <ucontext.h>

#include <cstdio>
#include <vector>

#include "hip/hip_runtime.h"

namespace emu {
std::vector<Stream*>& streams() {
  static std::vector<Stream*> v;
  return v;
}
namespace {
enum Wait { kNone = 0, kWave = 1, kBlock = 2 };
struct Fiber {
  ucontext_t ctx;
  Ctx c;
  int wave = 0, lane = 0;
  bool done = false;
  int wait = kNone;
  uint64_t wait_gen = 0;
  std::vector<char> stack;
};
struct WaveSt {
  int alive = 0, arrived = 0;
  uint64_t gen = 0;
  uint64_t slots[64];
};
struct BlockSt {
  int alive = 0, arrived = 0;
  uint64_t gen = 0;
};
Fiber* g_cur = nullptr;
ucontext_t g_sched;
std::vector<Fiber> g_fibers;
std::vector<WaveSt> g_waves;
BlockSt g_block;
const std::function<void()>* g_fn = nullptr;
std::vector<char> g_lds;

void yield_to_scheduler() { swapcontext(&g_cur->ctx, &g_sched); }

void fiber_main() {
  (*g_fn)();
  Fiber* f = g_cur;
  f->done = true;
  WaveSt& w = g_waves[f->wave];
  w.alive--;
  if (w.arrived > 0 && w.arrived >= w.alive) {
    w.arrived = 0;
    w.gen++;
  }
  g_block.alive--;
  if (g_block.arrived > 0 && g_block.arrived >= g_block.alive) {
    g_block.arrived = 0;
    g_block.gen++;
  }
  // uc_link returns to the scheduler
}
}  // namespace

Ctx* cur() { return &g_cur->c; }
void* dynamic_lds() { return g_lds.data(); }

void wave_barrier() {
  WaveSt& w = g_waves[g_cur->wave];
  uint64_t gen = w.gen;
  if (++w.arrived >= w.alive) {
    w.arrived = 0;
    w.gen++;
    return;
  }
  g_cur->wait = kWave;
  g_cur->wait_gen = gen;
  yield_to_scheduler();
}

void block_barrier() {
  uint64_t gen = g_block.gen;
  if (++g_block.arrived >= g_block.alive) {
    g_block.arrived = 0;
    g_block.gen++;
    return;
  }
  g_cur->wait = kBlock;
  g_cur->wait_gen = gen;
  yield_to_scheduler();
}

uint64_t wave_exchange(uint64_t v, int src) {
  WaveSt& w = g_waves[g_cur->wave];
  w.slots[g_cur->lane] = v;
  wave_barrier();
  uint64_t r = g_waves[g_cur->wave].slots[src];
  wave_barrier();
  return r;
}

uint64_t wave_ballot(bool p) {
  WaveSt& w = g_waves[g_cur->wave];
  w.slots[g_cur->lane] = p ? 1 : 0;
  wave_barrier();
  uint64_t m = 0;
  for (int i = 0; i < 64; i++)
    if (g_waves[g_cur->wave].slots[i]) m |= 1ull << i;
  wave_barrier();
  return m;
}

void launch(dim3 grid, dim3 block, size_t shmem, const std::function<void()>& fn) {
  const int T = int(block.x * block.y * block.z);
  if (T % 64 != 0) {
    fprintf(stderr, "emu: block size must be a multiple of 64\n");
    abort();
  }
  g_fn = &fn;
  g_lds.assign(shmem + 16, 0);
  if (int(g_fibers.size()) < T) g_fibers.resize(T);  // never shrink: stacks are reused across launches
  for (int t = 0; t < T; t++)
    if (g_fibers[t].stack.size() != (256u << 10)) g_fibers[t].stack.assign(256u << 10, 0);
  for (unsigned bz = 0; bz < grid.z; bz++)
    for (unsigned by = 0; by < grid.y; by++)
      for (unsigned bx = 0; bx < grid.x; bx++) {
        g_waves.assign(T / 64, WaveSt{});
        for (auto& w : g_waves) w.alive = 64;
        g_block = BlockSt{};
        g_block.alive = T;
        for (int t = 0; t < T; t++) {
          Fiber& f = g_fibers[t];
          f.c.tid = dim3(unsigned(t), 0, 0);
          f.c.bid = dim3(bx, by, bz);
          f.c.bdim = block;
          f.c.gdim = grid;
          f.wave = t / 64;
          f.lane = t % 64;
          f.done = false;
          f.wait = kNone;
          getcontext(&f.ctx);
          f.ctx.uc_stack.ss_sp = f.stack.data();
          f.ctx.uc_stack.ss_size = f.stack.size();
          f.ctx.uc_link = &g_sched;
          makecontext(&f.ctx, fiber_main, 0);
        }
        int remaining = T;
        while (remaining > 0) {
          bool progress = false;
          for (int t = 0; t < T; t++) {
            Fiber& f = g_fibers[t];
            if (f.done) continue;
            if (f.wait == kWave && g_waves[f.wave].gen == f.wait_gen) continue;
            if (f.wait == kBlock && g_block.gen == f.wait_gen) continue;
            f.wait = kNone;
            g_cur = &f;
            swapcontext(&g_sched, &f.ctx);
            g_cur = nullptr;
            progress = true;
            if (f.done) remaining--;
          }
          if (!progress) {
            fprintf(stderr, "emu: deadlock in block (%u,%u,%u)\n", bx, by, bz);
            abort();
          }
        }
      }
}
}  // namespace emu
