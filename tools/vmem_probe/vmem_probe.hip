// Development probe (not product code): cost of the vector-memory access shapes of the term
// loop on gfx950, every CU busy (512 workgroups x 768 threads, 4 independent loads in flight
// per lane).  Prints the time per wave-instruction per CU for each shape; run it under
// rocprofv3 --pmc TA_BUSY_avr TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE for
// the data-path cycles of each (one kernel instance per shape).
//   hipcc --offload-arch=gfx950 -O3 -o vmem_probe vmem_probe.hip && ./vmem_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

constexpr int WG = 768;
constexpr int U = 4;
constexpr uint32_t TAB_BYTES = 4u << 20;   // L2-resident table
constexpr int ROWS = 201;                  // C4's device rows
constexpr int PLANE = ROWS * 16;           // one coefficient plane of one interval

extern __shared__ __attribute__((aligned(16))) char dyn[];

__device__ __forceinline__ uint32_t lcg(uint32_t& h) { h = h * 1664525u + 1013904223u; return h >> 8; }

// PAT: 0 coalesced dwordx2 | 1 dwordx2, lanes 32 B apart | 2 dwordx4, random rows of one 3.2 KB plane
//      3 dwordx4, every lane the same address | 4 dwordx2 random over 512 KB | 5 dwordx4, 16 rows (16-lane groups)
//      6 ds_read_b128 random rows of one plane (LDS) | 7 ds_read_b64 random over 64 KB (LDS)
//      8 dwordx4 coalesced | 9 dwordx2, lanes 16 B apart
//      10 / 11 / 12: as 2 with 1/4, 1/2, 1/8 of the lanes active (the rest skip the load)
//      13 ds_read_b128 random 16-B blocks over 64 KB | 14 dwordx2 lanes 64 B apart
//      15 dwordx4 random rows of 20 planes (128 KB) | 16 as 10 but lanes active by a uniform-random mask per wave
template <int PAT>
__global__ void __launch_bounds__(WG) probe(const char* __restrict__ tab, int iters, double* sink) {
  const int lane = threadIdx.x & 63;
  const uint32_t gw = blockIdx.x * (WG / 64) + (threadIdx.x >> 6);
  uint32_t h = (blockIdx.x * WG + threadIdx.x) * 2654435761u + 12345u;
  double acc = 0.0;
  if constexpr ((PAT >= 6 && PAT <= 7) || PAT == 13) {
    for (int e = threadIdx.x; e < 65536 / 16; e += WG)
      reinterpret_cast<double2*>(dyn)[e] = reinterpret_cast<const double2*>(tab)[e];
    __syncthreads();
  }
  for (int j = 0; j < iters; j++) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t k = (uint32_t)j * U + u;
      uint32_t off;
      if constexpr (PAT == 0) off = ((gw * 4096u + k) * 64u + lane) * 8u;
      else if constexpr (PAT == 1) off = ((gw * 4096u + k) * 256u + lane * 4u) * 8u;
      else if constexpr (PAT == 2 || PAT == 6) off = (k % 200u) * (2u * PLANE) + (lcg(h) % ROWS) * 16u;
      else if constexpr (PAT == 3) off = (k % 200u) * (2u * PLANE) + ((gw + k) % ROWS) * 16u;
      else if constexpr (PAT == 4) off = (lcg(h) % 65536u) * 8u;
      else if constexpr (PAT == 5) off = (k % 200u) * (2u * PLANE) + (((gw + k) * 16u + (lane >> 2)) % ROWS) * 16u;
      else if constexpr (PAT == 7) off = (lcg(h) % 8192u) * 8u;
      else if constexpr (PAT == 8) off = ((gw * 4096u + k) * 64u + lane) * 16u;
      else if constexpr (PAT >= 10 && PAT <= 12) off = (k % 200u) * (2u * PLANE) + (lcg(h) % ROWS) * 16u;
      else if constexpr (PAT == 13) off = (lcg(h) % 4096u) * 16u;
      else if constexpr (PAT == 14) off = ((gw * 4096u + k) * 512u + lane * 8u) * 8u;
      else if constexpr (PAT == 15) off = ((k + (lcg(h) & 15u)) % 200u) * (2u * PLANE) + (lcg(h) % ROWS) * 16u;
      else if constexpr (PAT == 16) off = (k % 200u) * (2u * PLANE) + (lcg(h) % ROWS) * 16u;
      else off = ((gw * 4096u + k) * 128u + lane * 2u) * 8u;
      if constexpr (PAT >= 10 && PAT <= 12) {
        constexpr uint32_t M = PAT == 10 ? 3u : (PAT == 11 ? 1u : 7u);
        if (((h >> 20) & M) == 0) {
          const double2 v = *reinterpret_cast<const double2*>(tab + (off % TAB_BYTES));
          acc += v.x + v.y;
        }
      } else if constexpr (PAT == 16) {
        if ((((h >> 20) ^ k) & 3u) == 0) {
          const double2 v = *reinterpret_cast<const double2*>(tab + (off % TAB_BYTES));
          acc += v.x + v.y;
        }
      } else if constexpr (PAT == 13) {
        const double2 v = *reinterpret_cast<const double2*>(dyn + off);
        acc += v.x + v.y;
      } else if constexpr (PAT == 6) {
        const double2 v = *reinterpret_cast<const double2*>(dyn + (off % PLANE));
        acc += v.x + v.y;
      } else if constexpr (PAT == 7) {
        acc += *reinterpret_cast<const double*>(dyn + off);
      } else if constexpr (PAT == 2 || PAT == 3 || PAT == 5 || PAT == 8 || PAT == 15) {
        const double2 v = *reinterpret_cast<const double2*>(tab + (off % TAB_BYTES));
        acc += v.x + v.y;
      } else {
        acc += *reinterpret_cast<const double*>(tab + (off % TAB_BYTES));
      }
    }
  }
  if (acc == 1.2345) sink[0] = acc;  // never: keeps the loads
}

template <int PAT>
static int run(const char* tab, double* sink, const char* name) {
  const int blocks = 512, iters = 2048;
  const size_t lds = (PAT == 6 || PAT == 7 || PAT == 13) ? 65536 : 0;
  hipEvent_t a, b;
  CHK(hipEventCreate(&a)); CHK(hipEventCreate(&b));
  hipLaunchKernelGGL(probe<PAT>, dim3(blocks), dim3(WG), lds, 0, tab, 64, sink);  // warm
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(a, 0));
  hipLaunchKernelGGL(probe<PAT>, dim3(blocks), dim3(WG), lds, 0, tab, iters, sink);
  CHK(hipEventRecord(b, 0));
  CHK(hipEventSynchronize(b));
  float ms = 0.f;
  CHK(hipEventElapsedTime(&ms, a, b));
  const double winst = (double)blocks * (WG / 64) * iters * U;  // wave-instructions
  const double ns_per = ms * 1e6 * 256.0 / winst;                 // per CU
  printf("%-44s %8.3f ms  %7.2f ns (%6.1f cycles at 2.4 GHz) per wave-instruction per CU\n", name, ms, ns_per,
         ns_per * 2.4);
  return 0;
}

int main() {
  char* tab;
  double* sink;
  CHK(hipMalloc(&tab, TAB_BYTES + 65536));
  CHK(hipMemset(tab, 0, TAB_BYTES + 65536));
  CHK(hipMalloc(&sink, 8));
  run<0>(tab, sink, "0 dwordx2 coalesced (512 B)");
  run<9>(tab, sink, "9 dwordx2 lanes 16 B apart (1 KB)");
  run<1>(tab, sink, "1 dwordx2 lanes 32 B apart (2 KB)");
  run<4>(tab, sink, "4 dwordx2 random over 512 KB");
  run<8>(tab, sink, "8 dwordx4 coalesced (1 KB)");
  run<3>(tab, sink, "3 dwordx4 one address");
  run<5>(tab, sink, "5 dwordx4 16 rows (4 lanes per row)");
  run<2>(tab, sink, "2 dwordx4 random rows of a 3.2 KB plane");
  run<6>(tab, sink, "6 ds_read_b128 random rows of a plane");
  run<7>(tab, sink, "7 ds_read_b64 random over 64 KB");
  run<11>(tab, sink, "11 as 2, 1/2 of the lanes");
  run<10>(tab, sink, "10 as 2, 1/4 of the lanes");
  run<12>(tab, sink, "12 as 2, 1/8 of the lanes");
  run<16>(tab, sink, "16 as 2, 1/4 of the lanes (mask varies)");
  run<13>(tab, sink, "13 ds_read_b128 random over 64 KB");
  run<14>(tab, sink, "14 dwordx2 lanes 64 B apart (4 KB)");
  run<15>(tab, sink, "15 dwordx4 random rows of 16 planes");
  return 0;
}
