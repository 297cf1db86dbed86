// Back-to-back launch floor on one stream: 200 launches of an empty kernel and of a kernel
// that writes 1 MiB (the 1M-slot sweep's output volume), at the 1M sweep's grid (256
// workgroups of 128 threads), timed by HIP events. Run under rocprofv3 --kernel-trace to
// read the per-kernel durations the profiler reports for the same launches.
//   hipcc --offload-arch=gfx950 -O3 -o tools/launch_floor tools/launch_floor.hip && tools/launch_floor
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void empty_kernel(uint32_t* out) {
  if (out == nullptr) out[threadIdx.x] = 1;  // never taken: keeps the argument
}

__global__ void write_kernel(uint4* out, uint32_t n16) {  // 1 MiB: 65,536 16-B stores
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += gridDim.x * blockDim.x)
    out[i] = make_uint4(i, i, i, i);
}

int main() {
  uint32_t* buf;
  CHK(hipMalloc(&buf, 1 << 20));
  hipStream_t s;
  CHK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  for (int variant = 0; variant < 2; variant++) {
    for (int rep = 0; rep < 3; rep++) {
      CHK(hipEventRecord(e0, s));
      for (int k = 0; k < 200; k++) {
        if (variant == 0) hipLaunchKernelGGL(empty_kernel, dim3(256), dim3(128), 0, s, buf);
        else hipLaunchKernelGGL(write_kernel, dim3(256), dim3(128), 0, s, reinterpret_cast<uint4*>(buf), (1u << 20) / 16);
      }
      CHK(hipEventRecord(e1, s));
      CHK(hipEventSynchronize(e1));
      float ms = 0;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      if (rep == 2)
        std::printf("{\"kernel\": \"%s\", \"grid\": 256, \"block\": 128, \"us_per_launch\": %.3f}\n",
                    variant ? "write_1MiB" : "empty", ms * 1000.0 / 200);
    }
  }
  (void)hipFree(buf);
  return 0;
}
