/*
 * rabia_gpu_debug.h — diagnostic entry points of librabia_gpu.so (not part of
 * the drop-in boundary; used by tools/ablate.py to find where a step's time goes).
 */
#ifndef RABIA_GPU_DEBUG_H
#define RABIA_GPU_DEBUG_H
#include <stdint.h>
#include "rabia_gpu.h"
#ifdef __cplusplus
extern "C" {
#endif
/* diag bits: 1 skip the look-back wait (wrong draws), 2 skip per-tile statistics
 * and the step result, 4 record per-tile s_memrealtime stamps (100 MHz);
 * bits 8-10: tiled kernel shape, 0 = automatic, 1 big (512 x W), 2 mid (256 x W), 3 small (128 x 1);
 * bit 20: large REF launches keep the tiled kernel instead of the persistent lag kernel;
 * bit 21: the lag kernel at any launch size;
 * bit 22: the lag kernel as two 512-thread workgroups per CU (the shape of launches of < 2
 *         1024-thread tiles per CU; A/B on large ones);
 * bits 24-31: lag-kernel grid (0 = one workgroup per CU, two in the 512-thread shape). */
int rg_debug_set(rg_ctx* ctx, uint32_t diag);
/* The phase-step launch the context issued last (what step_impl picked), 6 words:
 * kind (0 tiled REF kernel, 1 persistent lag REF kernel, 2 tiled WMVC kernel), shard (0/1),
 * threads per workgroup, words per thread, grid (tiled: tiles per window; lag: workgroups),
 * windows (grid.y of a multi-window shard launch). */
int rg_debug_last_launch(const rg_ctx* ctx, uint32_t* out6);
int rg_debug_stamps(rg_ctx* ctx, uint64_t* host_out, uint64_t n_words);
/* REF kernel memory pattern (20 in-planes, 8 out-planes, 16 B/lane) without protocol.
 * tile_words = 0: planar planes `stride` words apart; > 0: slot-tiled layout
 * (21 in-planes / 8 out-planes of each tile_words-word slot tile back to back).
 * nt != 0: non-temporal loads and stores. */
int rg_debug_stream_probe(const uint32_t* in_dev, uint32_t* out_dev, uint64_t n_words,
                          uint64_t stride, uint32_t tile_words, uint32_t nt, void* stream);
#ifdef __cplusplus
}
#endif
#endif
