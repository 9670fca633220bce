// LDS-DMA (global_load_lds_dwordx4) semantics check on gfx950: lane i's 16 bytes land at pf[i]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__global__ void k(const uint4* __restrict__ src, uint4* out, uint32_t n) {
  __shared__ __attribute__((aligned(16))) uint4 pf[64];
  __shared__ uint32_t other[64];
  const uint32_t lane = threadIdx.x;
  pf[lane] = make_uint4(0xdead, 0xdead, 0xdead, 0xdead);
  other[lane] = lane;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_s_waitcnt(0);
  if (lane < n)
    __builtin_amdgcn_global_load_lds((const void*)(src + 3 + lane), (__attribute__((address_space(3))) void*)pf, 16, 0, 0);
  uint32_t acc = other[(lane + 5) & 63];
  __builtin_amdgcn_wave_barrier();
  const uint4 v = pf[lane];
  out[lane] = make_uint4(v.x, v.y, v.z, v.w + acc * 0);
}
int main() {
  std::vector<uint4> h(128);
  for (int i = 0; i < 128; ++i) h[i] = make_uint4(i, i * 2, i * 3, i * 5);
  uint4 *d, *o;
  hipMalloc(&d, 128 * 16);
  hipMalloc(&o, 64 * 16);
  hipMemcpy(d, h.data(), 128 * 16, hipMemcpyHostToDevice);
  int bad = 0;
  for (uint32_t n : {64u, 37u, 1u, 0u}) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, o, n);
    std::vector<uint4> r(64);
    hipMemcpy(r.data(), o, 64 * 16, hipMemcpyDeviceToHost);
    for (uint32_t i = 0; i < 64; ++i) {
      const uint4 w = i < n ? h[3 + i] : make_uint4(0xdead, 0xdead, 0xdead, 0xdead);
      if (r[i].x != w.x || r[i].y != w.y || r[i].z != w.z || r[i].w != w.w) {
        if (bad < 8) printf("n=%u lane %u: got %x %x %x %x want %x %x %x %x\n", n, i, r[i].x, r[i].y, r[i].z, r[i].w, w.x, w.y, w.z, w.w);
        ++bad;
      }
    }
  }
  printf(bad ? "LDS-DMA FAIL %d\n" : "LDS-DMA OK\n", bad);
  return bad != 0;
}
