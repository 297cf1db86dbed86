// rg_shard.hip — launchers of the sharded-REF step kernels (one engine over a
// window split across GPUs; the kernels and their fix-up are in rg_kernels.h).
// Kept in a translation unit of its own so the 16 replica counts x 3 tile shapes
// compile in parallel with rabia_gpu.hip.
#include "rg_kernels.h"

namespace rg {

namespace {
template <int N>
void launch_n(int block, int words, uint32_t grid, hipStream_t s, const StepParams& p) {
  const dim3 g(grid, p.n_win > 1 ? p.n_win : 1);  // grid.y: windows of a multi-window launch (tiled kernel)
  constexpr int WM = N <= 5 ? 4 : (N <= 10 ? 2 : 1);
  if (block <= 0) {  // the lag kernel (n <= 10, step_impl): -1 one WG per CU (2048-word tiles as 512 x 4),
                     // -2 the same over the tickets of every window (multi-window launch), 0 two 512-thread
                     // WGs per CU (512 x (n <= 5 ? 2 : 1))
    if constexpr (N <= 10) {
      constexpr int W2 = N <= 5 ? 2 : 1;
      if (block == -2) hipLaunchKernelGGL((ref_lag_kernel<N, 4, 512, true, 2, true>), dim3(grid), dim3(512), 0, s, p);
      else if (block < 0) hipLaunchKernelGGL((ref_lag_kernel<N, 4, 512, true, 2>), dim3(grid), dim3(512), 0, s, p);
      else hipLaunchKernelGGL((ref_lag_kernel<N, W2, 512, true>), dim3(grid), dim3(512), 0, s, p);
    }
  } else if (block == 512) hipLaunchKernelGGL((ref_step_kernel<N, WM, 512, true>), g, dim3(512), 0, s, p);
  else if (block == 256) hipLaunchKernelGGL((ref_step_kernel<N, WM, 256, true>), g, dim3(256), 0, s, p);
  else hipLaunchKernelGGL((ref_step_kernel<N, 1, 128, true>), g, dim3(128), 0, s, p);
  (void)words;
}
using Launch = void (*)(int, int, uint32_t, hipStream_t, const StepParams&);
const Launch kTable[17] = {nullptr,      &launch_n<1>,  &launch_n<2>,  &launch_n<3>,  &launch_n<4>,  &launch_n<5>,
                           &launch_n<6>,  &launch_n<7>,  &launch_n<8>,  &launch_n<9>,  &launch_n<10>, &launch_n<11>,
                           &launch_n<12>, &launch_n<13>, &launch_n<14>, &launch_n<15>, &launch_n<16>};
}  // namespace

// block/words must be one of the shapes rabia_gpu.hip picks: {512, wmax}, {256, wmax}, {128, 1};
// block <= 0 = the persistent lag kernel (tiles by ticket, grid = resident workgroups; -1: one workgroup
// per CU, 512 x 4; -2: the same over several windows; 0: two 512-thread workgroups per CU, 512 x (n <= 5 ? 2 : 1)).
void launch_ref_shard(int n, int block, int words, uint32_t grid, hipStream_t s, const StepParams& p) {
  kTable[n](block, words, grid, s, p);
}

}  // namespace rg
