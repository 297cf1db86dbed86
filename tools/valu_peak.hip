// VALU issue-rate probe: how many wave64 vector instructions per cycle a CU retires
// for the instruction classes the C3 cluster kernel is made of (32-bit integer ALU,
// v_mul_lo_u32, v_bcnt_u32_b32) against f32 FMA, every SIMD holding 8 waves of
// independent chains. Prints one JSON line per class: wave-instructions per cycle per
// CU (the C3 roofline's peak = that x CUs x clock). Build + run:
//   hipcc --offload-arch=gfx950 -O3 -o tools/valu_peak tools/valu_peak.hip && tools/valu_peak
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

constexpr int kIters = 16384;
constexpr int kChains = 8;   // independent accumulators per lane
constexpr int kUnroll = 4;   // chain steps per loop iteration

template <int OP>
__device__ __forceinline__ void step(uint32_t& a, uint32_t b) {
  if constexpr (OP == 0) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a) : "v"(b));
  else if constexpr (OP == 1) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a) : "v"(b));
  else if constexpr (OP == 2) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a) : "v"(b));
  else if constexpr (OP == 3) asm volatile("v_bcnt_u32_b32 %0, %0, %1" : "+v"(a) : "v"(b));
  else asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a) : "v"(b));
}

// cycles[wave] = s_memtime ticks of the wave's loop (per-wave timing; the grid is sized
// so every wave is resident at once: 8 per SIMD)
template <int OP>
__global__ __launch_bounds__(256) void probe(uint32_t seed, uint32_t* out, unsigned long long* cycles) {
  uint32_t a[kChains];
#pragma unroll
  for (int k = 0; k < kChains; k++) a[k] = seed + threadIdx.x * 7u + (uint32_t)k;
  const uint32_t b = seed | 1u;
  __syncthreads();
  const unsigned long long t0 = clock64();
  for (int i = 0; i < kIters; i++) {
#pragma unroll
    for (int u = 0; u < kUnroll; u++)
#pragma unroll
      for (int k = 0; k < kChains; k++) step<OP>(a[k], b);
  }
  const unsigned long long t1 = clock64();
  uint32_t x = 0;
#pragma unroll
  for (int k = 0; k < kChains; k++) x ^= a[k];
  out[blockIdx.x * 256 + threadIdx.x] = x;  // keeps the chains live (vector store)
  if ((threadIdx.x & 63) == 0) cycles[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int OP>
int run(const char* name, int cus, uint32_t* out, unsigned long long* cyc_dev, unsigned long long* cyc_host) {
  const int grid = cus * 8;  // 8 workgroups of 4 waves per CU: 8 waves per SIMD
  hipLaunchKernelGGL(probe<OP>, dim3(grid), dim3(256), 0, 0, 1u, out, cyc_dev);  // warm-up
  CHK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  CHK(hipEventRecord(e0));
  hipLaunchKernelGGL(probe<OP>, dim3(grid), dim3(256), 0, 0, 3u, out, cyc_dev);
  CHK(hipEventRecord(e1));
  CHK(hipEventSynchronize(e1));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, e0, e1));
  CHK(hipMemcpy(cyc_host, cyc_dev, (size_t)grid * 4 * 8, hipMemcpyDeviceToHost));
  double mean = 0;
  for (int w = 0; w < grid * 4; w++) mean += (double)cyc_host[w];
  mean /= grid * 4;
  const double per_wave = (double)kIters * kUnroll * kChains;  // instructions per wave in the timed loop
  // per SIMD 8 waves ran their loops concurrently over ~mean cycles
  const double per_simd_cycle = 8.0 * per_wave / mean;
  std::printf("{\"op\": \"%s\", \"wave_instr_per_cycle_per_simd\": %.4f, \"cycles_per_wave_instr\": %.3f, "
              "\"wave_instr_per_cycle_per_cu\": %.3f, \"kernel_ms\": %.3f, \"clock_ghz_est\": %.3f}\n",
              name, per_simd_cycle, 1.0 / per_simd_cycle, 4.0 * per_simd_cycle, ms, mean / (ms * 1e6));
  return 0;
}

int main() {
  hipDeviceProp_t p;
  CHK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  std::printf("{\"device\": \"%s\", \"cus\": %d}\n", p.gcnArchName, cus);
  uint32_t* out;
  unsigned long long* cyc;
  CHK(hipMalloc(&out, (size_t)cus * 8 * 256 * 4));
  CHK(hipMalloc(&cyc, (size_t)cus * 8 * 4 * 8));
  unsigned long long* host = new unsigned long long[(size_t)cus * 8 * 4];
  int rc = run<0>("v_xor_b32", cus, out, cyc, host) || run<1>("v_add_u32", cus, out, cyc, host) ||
           run<2>("v_mul_lo_u32", cus, out, cyc, host) || run<3>("v_bcnt_u32_b32", cus, out, cyc, host) ||
           run<4>("v_fma_f32", cus, out, cyc, host);
  delete[] host;
  (void)hipFree(out);
  (void)hipFree(cyc);
  return rc;
}
