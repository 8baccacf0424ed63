// Development probe (not product code): how fast a kernel reads one trial's packed rows (1 MB
// at C4) from pinned host memory, by allocation kind and access shape -- the scatter of
// DESIGN.md §10.3b reads 16 B per thread from coherent (fine-grained) host memory at ~7 GB/s.
// For each kind it also rewrites the buffer between launches and checks that every launch
// reads the new contents (a coarse-grained kind must not return stale lines).
//   hipcc --offload-arch=gfx950 -O3 -o hostread_probe hostread_probe.hip && ./hostread_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <vector>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr size_t BYTES = 1u << 20;

// each thread reads PER consecutive 16-B words (the block's words contiguous), sums them into out
template <int PER>
__global__ void __launch_bounds__(256) rd(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16) {
  const size_t base = ((size_t)blockIdx.x * 256) * PER;
  uint4 v[PER];
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const size_t i = base + (size_t)k * 256 + threadIdx.x;
    v[k] = i < n16 ? src[i] : make_uint4(0, 0, 0, 0);
  }
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const size_t i = base + (size_t)k * 256 + threadIdx.x;
    if (i < n16) dst[i] = v[k];
  }
}

template <int PER>
static double time_kernel(const uint4* src, uint4* dst, hipStream_t s, int reps, unsigned* stale, unsigned char* host,
                          std::vector<uint4>& back) {
  const size_t n16 = BYTES / 16;
  const int grid = (int)((n16 + 256 * PER - 1) / (256 * PER));
  hipEvent_t a, b;
  CHK(hipEventCreate(&a)); CHK(hipEventCreate(&b));
  std::vector<float> t;
  for (int r = 0; r < reps; r++) {
    memset(host, (r * 37 + 11) & 0xFF, BYTES);  // new contents every launch
    CHK(hipEventRecord(a, s));
    hipLaunchKernelGGL(rd<PER>, dim3(grid), dim3(256), 0, s, src, dst, n16);
    CHK(hipEventRecord(b, s));
    CHK(hipEventSynchronize(b));
    float ms; CHK(hipEventElapsedTime(&ms, a, b)); t.push_back(ms);
    CHK(hipMemcpy(back.data(), dst, BYTES, hipMemcpyDeviceToHost));
    const unsigned char want = (unsigned char)((r * 37 + 11) & 0xFF);
    const unsigned char* p = reinterpret_cast<const unsigned char*>(back.data());
    for (size_t i = 0; i < BYTES; i += 4093) if (p[i] != want) { (*stale)++; break; }
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2] * 1e3;  // median us
}

int main() {
  hipStream_t s; CHK(hipStreamCreate(&s));
  uint4* dst; CHK(hipMalloc(&dst, BYTES));
  std::vector<uint4> back(BYTES / 16);
  struct Kind { const char* name; unsigned char* p; } kinds[4];
  unsigned char *coh, *nc, *reg;
  CHK(hipHostMalloc((void**)&coh, BYTES, hipHostMallocCoherent | hipHostMallocMapped | hipHostMallocPortable));
  CHK(hipHostMalloc((void**)&nc, BYTES, hipHostMallocNonCoherent | hipHostMallocMapped | hipHostMallocPortable));
  reg = (unsigned char*)aligned_alloc(4096, BYTES);
  CHK(hipHostRegister(reg, BYTES, hipHostRegisterPortable | hipHostRegisterMapped));
  kinds[0] = {"hipHostMalloc coherent (today's staging)", coh};
  kinds[1] = {"hipHostMalloc non-coherent", nc};
  kinds[2] = {"malloc + hipHostRegister", reg};
  int nk = 3;
  const int reps = 60;
  for (int k = 0; k < nk; k++) {
    unsigned stale = 0;
    const uint4* src = reinterpret_cast<const uint4*>(kinds[k].p);
    const double t1 = time_kernel<1>(src, dst, s, reps, &stale, kinds[k].p, back);
    const double t4 = time_kernel<4>(src, dst, s, reps, &stale, kinds[k].p, back);
    const double t16 = time_kernel<16>(src, dst, s, reps, &stale, kinds[k].p, back);
    printf("%-42s 16B/thread %7.1f us (%5.1f GB/s) | 4x16B %7.1f us (%5.1f GB/s) | 16x16B %7.1f us (%5.1f GB/s) | stale launches %u of %d\n",
           kinds[k].name, t1, BYTES / t1 / 1e3, t4, BYTES / t4 / 1e3, t16, BYTES / t16 / 1e3, stale, 3 * reps);
  }
  {  // the copy engine, for reference
    hipEvent_t a, b; CHK(hipEventCreate(&a)); CHK(hipEventCreate(&b));
    std::vector<float> t;
    for (int r = 0; r < reps; r++) {
      CHK(hipEventRecord(a, s));
      CHK(hipMemcpyAsync(dst, coh, BYTES, hipMemcpyHostToDevice, s));
      CHK(hipEventRecord(b, s));
      CHK(hipEventSynchronize(b));
      float ms; CHK(hipEventElapsedTime(&ms, a, b)); t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    printf("%-42s %7.1f us (%5.1f GB/s)\n", "hipMemcpyAsync H2D from coherent pinned", t[t.size() / 2] * 1e3,
           BYTES / (t[t.size() / 2] * 1e3) / 1e3);
  }
  return 0;
}
