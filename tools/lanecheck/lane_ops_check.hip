// Hardware check of the wave primitives in tas_kernels.hip (butterfly
// reductions over DPP / permlane swaps, the DPP scan, readlane broadcasts):
// one wave per test pattern, results compared with a host computation.
#include "../../kueue_oss_amd/csrc/tas_kernels.hip"

#include <cstdio>
#include <vector>

namespace ktas {
__global__ void lane_ops_kernel(const int32_t* in, int32_t* out) {
  const int lane = lane_id();
  const int32_t v = in[blockIdx.x * 64 + lane];
  int32_t* o = out + blockIdx.x * 64 * 16;
  int k = 0;
  for (int F = 2; F <= 64; F <<= 1) o[(k++) * 64 + lane] = group_reduce(v, F, OpWAdd());  // 6 rows
  o[(k++) * 64 + lane] = group_reduce(v, 64, OpMin());
  o[(k++) * 64 + lane] = group_reduce(v, 64, OpMax());
  int tot = 0;
  o[(k++) * 64 + lane] = wave_excl_scan(v, &tot);
  o[(k++) * 64 + lane] = tot;
  uint64_t av = uint64_t(uint32_t(v) & 7u);
  int32_t ai = lane;
  wave_argmin(av, ai);
  o[(k++) * 64 + lane] = ai;
  const Key key = wave_min_key(Key{uint64_t(uint32_t(v) & 3u), uint64_t(63 - lane)});
  o[(k++) * 64 + lane] = int32_t(key.lo);
  o[(k++) * 64 + lane] = bcast(v, 37);
  o[(k++) * 64 + lane] = int32_t(bfly<16>(uint32_t(v)));
  o[(k++) * 64 + lane] = int32_t(bfly<32>(uint32_t(v)));
  o[(k++) * 64 + lane] = int32_t(wave_min_u64(uint64_t(uint32_t(v)) << 20));
}
// raw semantics, printed: permlane swaps of (lane, 100 + lane), row_bcast:15/31, row_shr:1
__global__ void lane_raw_kernel(int32_t* out) {
  const int lane = lane_id();
  const auto r16 = __builtin_amdgcn_permlane16_swap(uint32_t(lane), uint32_t(100 + lane), false, false);
  const auto r32 = __builtin_amdgcn_permlane32_swap(uint32_t(lane), uint32_t(100 + lane), false, false);
  out[0 * 64 + lane] = int32_t(r16[0]);
  out[1 * 64 + lane] = int32_t(r16[1]);
  out[2 * 64 + lane] = int32_t(r32[0]);
  out[3 * 64 + lane] = int32_t(r32[1]);
  out[4 * 64 + lane] = __builtin_amdgcn_update_dpp(-1, lane, 0x142, 0xF, 0xF, false);
  out[5 * 64 + lane] = __builtin_amdgcn_update_dpp(-1, lane, 0x143, 0xF, 0xF, false);
  out[6 * 64 + lane] = __builtin_amdgcn_update_dpp(-1, lane, 0x111, 0xF, 0xF, false);
  out[7 * 64 + lane] = __builtin_amdgcn_update_dpp(-1, lane, 0x141, 0xF, 0xF, false);
}
}  // namespace ktas

int main() {
  const int nb = 4;
  std::vector<int32_t> in(nb * 64), out(nb * 64 * 16, 0);
  uint32_t x = 12345;
  for (auto& v : in) {
    x = x * 1103515245u + 12345u;
    v = int32_t((x >> 8) & 0xffff) - 30000;
  }
  int32_t *din, *dout;
  if (hipMalloc(&din, in.size() * 4) || hipMalloc(&dout, out.size() * 4)) return 2;
  (void)hipMemcpy(din, in.data(), in.size() * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(ktas::lane_ops_kernel, dim3(nb), dim3(64), 0, 0, din, dout);
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  (void)hipMemcpy(out.data(), dout, out.size() * 4, hipMemcpyDeviceToHost);
  int bad = 0;
  const char* names[] = {"sum2", "sum4", "sum8", "sum16", "sum32", "sum64", "min", "max", "excl_scan", "total",
                         "argmin", "min_key", "bcast37", "bfly16", "bfly32", "min_u64"};
  for (int b = 0; b < nb; b++) {
    const int32_t* v = in.data() + b * 64;
    for (int lane = 0; lane < 64; lane++) {
      int32_t want[16];
      int k = 0;
      for (int F = 2; F <= 64; F <<= 1) {
        uint32_t s = 0;
        for (int j = lane & ~(F - 1); j < (lane & ~(F - 1)) + F; j++) s += uint32_t(v[j]);
        want[k++] = int32_t(s);
      }
      int32_t mn = v[0], mx = v[0], ex = 0, tot = 0;
      for (int j = 0; j < 64; j++) {
        mn = std::min(mn, v[j]);
        mx = std::max(mx, v[j]);
        if (j < lane) ex += v[j];
        tot += v[j];
      }
      want[k++] = mn;
      want[k++] = mx;
      want[k++] = ex;
      want[k++] = tot;
      int am = 0;
      for (int j = 1; j < 64; j++)
        if ((uint32_t(v[j]) & 7u) < (uint32_t(v[am]) & 7u)) am = j;
      want[k++] = am;
      int km = 0;  // min (v & 3, 63 - lane)
      for (int j = 1; j < 64; j++) {
        const uint32_t a = uint32_t(v[j]) & 3u, c = uint32_t(v[km]) & 3u;
        if (a < c || (a == c && 63 - j < 63 - km)) km = j;
      }
      want[k++] = 63 - km;
      want[k++] = v[37];
      want[k++] = v[lane ^ 16];
      want[k++] = v[lane ^ 32];
      uint64_t m64 = ~0ull;
      for (int j = 0; j < 64; j++) m64 = std::min(m64, uint64_t(uint32_t(v[j])) << 20);
      want[k++] = int32_t(uint32_t(m64));
      for (int t = 0; t < k; t++) {
        const int32_t got = out[(b * 16 + t) * 64 + lane];
        if (got != want[t] && bad++ < 40) printf("block %d lane %d %s: got %d want %d\n", b, lane, names[t], got, want[t]);
      }
    }
  }
  {
    std::vector<int32_t> raw(8 * 64);
    hipLaunchKernelGGL(ktas::lane_raw_kernel, dim3(1), dim3(64), 0, 0, dout);
    if (hipDeviceSynchronize() != hipSuccess) return 3;
    (void)hipMemcpy(raw.data(), dout, raw.size() * 4, hipMemcpyDeviceToHost);
    const char* rn[] = {"p16[0]", "p16[1]", "p32[0]", "p32[1]", "bcast15", "bcast31", "shr1", "hmirror"};
    for (int r = 0; r < 8; r++) {
      printf("%-8s", rn[r]);
      for (int l = 0; l < 64; l++) printf(" %d", raw[r * 64 + l]);
      printf("\n");
    }
  }
  printf("lane ops: %d mismatches\n", bad);
  return bad ? 1 : 0;
}
