// Development probe: do kernels on two streams run concurrently on this box, and which
// kernel properties (scratch, large dynamic LDS, 768-thread groups) or stream operations
// (async copies, cross-stream event waits) serialise them?  Each kernel: 64 workgroups that
// spin ~20 ms of wall clock; two concurrent kernels take ~20 ms, serialised ~40.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <chrono>

extern __shared__ char dyn[];

template <int MODE>
__global__ void __launch_bounds__(768) spin(long long ticks, int* sink, int idx) {
  const long long t0 = wall_clock64();
  volatile int scratch[64];
  if constexpr (MODE == 1) {  // scratch
    for (int i = 0; i < 64; i++) scratch[i] = i + idx;
  }
  if constexpr (MODE == 2) dyn[threadIdx.x] = 1;
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(10);
  if (threadIdx.x == 0 && blockIdx.x == 0) atomicAdd(sink, MODE == 1 ? scratch[idx & 63] : 1);
}

template <int MODE>
static double run(hipStream_t a, hipStream_t b, long long ticks, int* sink, int what, void* dbuf, void* hbuf,
                  hipEvent_t ev) {
  hipDeviceSynchronize();
  const int thr = MODE == 0 ? 256 : 768;
  const size_t lds = MODE == 2 ? 81920 : 0;
  auto t0 = std::chrono::steady_clock::now();
  if (what == 1) hipMemcpyAsync(dbuf, hbuf, 1 << 20, hipMemcpyHostToDevice, a);
  hipLaunchKernelGGL(spin<MODE>, dim3(64), dim3(thr), lds, a, ticks, sink, 3);
  if (what == 1) hipMemcpyAsync(hbuf, dbuf, 1 << 20, hipMemcpyDeviceToHost, a);
  if (what == 2) { hipEventRecord(ev, a); }
  if (what == 1) hipMemcpyAsync((char*)dbuf + (1 << 20), (char*)hbuf + (1 << 20), 1 << 20, hipMemcpyHostToDevice, b);
  hipLaunchKernelGGL(spin<MODE>, dim3(64), dim3(thr), lds, b, ticks, sink, 3);
  if (what == 1) hipMemcpyAsync((char*)hbuf + (1 << 20), (char*)dbuf + (1 << 20), 1 << 20, hipMemcpyDeviceToHost, b);
  hipDeviceSynchronize();
  auto t1 = std::chrono::steady_clock::now();
  return std::chrono::duration<double, std::milli>(t1 - t0).count();
}

int main() {
  int* sink; hipMalloc(&sink, 4);
  void *dbuf, *hbuf;
  hipMalloc(&dbuf, 4 << 20);
  hipHostMalloc(&hbuf, 4 << 20, hipHostMallocDefault);
  hipFuncSetAttribute(reinterpret_cast<const void*>(&spin<2>), hipFuncAttributeMaxDynamicSharedMemorySize, 81920);
  int rate = 0; hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, 0);  // kHz
  const long long ticks = (long long)rate * 20;  // 20 ms
  int lo, hi; hipDeviceGetStreamPriorityRange(&lo, &hi);
  hipStream_t a, b, u;
  hipStreamCreateWithPriority(&a, hipStreamNonBlocking, hi);
  hipStreamCreateWithPriority(&b, hipStreamNonBlocking, lo);
  hipStreamCreateWithPriority(&u, hipStreamNonBlocking, lo);
  hipEvent_t ev; hipEventCreate(&ev);
  run<0>(a, b, ticks, sink, 0, dbuf, hbuf, ev);
  printf("plain 256-thread kernels            %6.1f ms\n", run<0>(a, b, ticks, sink, 0, dbuf, hbuf, ev));
  printf("768 threads + scratch               %6.1f ms\n", run<1>(a, b, ticks, sink, 0, dbuf, hbuf, ev));
  printf("768 threads + 80 KB dynamic LDS     %6.1f ms\n", run<2>(a, b, ticks, sink, 0, dbuf, hbuf, ev));
  printf("plain + async copies around         %6.1f ms\n", run<0>(a, b, ticks, sink, 1, dbuf, hbuf, ev));
  printf("scratch + async copies around       %6.1f ms\n", run<1>(b, u, ticks, sink, 1, dbuf, hbuf, ev));
  printf("LDS + async copies, lo+lo           %6.1f ms\n", run<2>(b, u, ticks, sink, 1, dbuf, hbuf, ev));
  return 0;
}
