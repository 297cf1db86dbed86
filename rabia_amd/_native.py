"""ctypes binding of the C ABI in include/rabia_gpu.h (rabia_amd/lib/librabia_gpu.so).

There is no fallback: if the library cannot be loaded, or no gfx950 device is
present, the calls raise. torch (when importable) is imported BEFORE the library
so both share one HIP runtime: torch's wheel bundles libamdhip64.so.7 and the
loader then resolves our NEEDED entry to that already-loaded copy, which lets
torch tensors / streams be handed to the library directly.
"""
from __future__ import annotations

import ctypes
import os
import re

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
LIB_PATH = os.environ.get("RABIA_GPU_LIB") or os.path.join(PKG, "lib", "librabia_gpu.so")  # override: A/B runs
HEADER = os.path.join(ROOT, "include", "rabia_gpu.h")
HEADERS = [HEADER] + [os.path.join(ROOT, "include", h) for h in ("rabia_kv.h", "rabia_ingest.h")]

u32, u64, i32, vp = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int32, ctypes.c_void_p

RG_OK, RG_EINVAL, RG_EHIP, RG_ENOMEM, RG_ENODEV, RG_ESTATE = 0, -1, -2, -3, -4, -5
RG_MODE_REF, RG_MODE_WMVC = 0, 1
RG_TRACE_UNIFORM, RG_TRACE_AGREE90, RG_TRACE_SPLIT = 0, 1, 2
OUT_PLANES = 8


class RgConfig(ctypes.Structure):
    _fields_ = [("n_replicas", u32), ("quorum", u32), ("decide_threshold", u32),
                ("self_lane", i32), ("mode", u32), ("device", i32), ("seed", u64),
                ("coin_seed", u64), ("epoch", u64), ("tile_words", u32), ("reserved", u32)]


RESULT_FIELDS = ["n_slots", "n_decided", "n_v1", "n_pending_r1", "n_draws",
                 "last_committed_max", "first_undecided", "rng_next", "commit_watermark", "flags"]


class RgStepResult(ctypes.Structure):
    _fields_ = [(f, u64) for f in RESULT_FIELDS]

    def as_dict(self):
        return {f: int(getattr(self, f)) for f in RESULT_FIELDS}


class RgEngineState(ctypes.Structure):
    _fields_ = [("rng_next", u64), ("last_committed", u64), ("commit_watermark", u64),
                ("steps", u64)]


class RgIngestConfig(ctypes.Structure):
    _fields_ = [("n_replicas", u32), ("tile_words", u32), ("device", i32), ("reserved", u32),
                ("members", (ctypes.c_uint8 * 16) * 16)]


INGEST_STATS = ["r1", "r2", "superseded", "other", "outside", "invalid", "sender", "malformed"]


class RgKvConfig(ctypes.Structure):
    _fields_ = [("max_keys", u64), ("max_value_size", u64), ("enable_notifications", u32),
                ("device", i32), ("table_slots", u64), ("heap_bytes", u64), ("hash_bits", u32),
                ("bucket_bits", u32)]


KV_STATS_FIELDS = ["live_keys", "version", "total_operations", "occupied_slots", "heap_used",
                   "batches", "ordered_batches", "flags", "last_path"]


class RgKvStats(ctypes.Structure):
    _fields_ = [(f, u64) for f in KV_STATS_FIELDS]

    def as_dict(self):
        return {f: int(getattr(self, f)) for f in KV_STATS_FIELDS}


_SIGS = {
    "rg_abi_version": (ctypes.c_int, []),
    "rg_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    "rg_plane_stride": (u64, [u64]),
    "rg_create": (ctypes.c_int, [ctypes.POINTER(vp), ctypes.POINTER(RgConfig)]),
    "rg_destroy": (ctypes.c_int, [vp]),
    "rg_last_error": (ctypes.c_char_p, [vp]),
    "rg_get_config": (ctypes.c_int, [vp, ctypes.POINTER(RgConfig)]),
    "rg_reserve": (ctypes.c_int, [vp, u64, u32]),
    "rg_set_state": (ctypes.c_int, [vp, ctypes.POINTER(RgEngineState)]),
    "rg_get_state": (ctypes.c_int, [vp, ctypes.POINTER(RgEngineState)]),
    "rg_phase_step_async": (ctypes.c_int, [vp, vp, vp, u64, u64, u64, u64, u64, vp, vp]),
    "rg_record_window_words": (u64, [u64, u64]),
    "rg_phase_step": (ctypes.c_int, [vp, vp, vp, u64, u64, u64, u64, u64, ctypes.POINTER(RgStepResult)]),
    "rg_phase_step_shard_async": (ctypes.c_int, [vp, vp, vp, u64, u64, u64, u64, vp, u64, vp, vp]),
    "rg_phase_step_shard_windows_async": (ctypes.c_int, [vp, u32, vp, u64, vp, u64, u64, u64, u64, u64, u64, vp, u64,
                                                         vp, vp]),
    "rg_shard_fixup_async": (ctypes.c_int, [vp, vp, u64, u64, u64, u64, vp, u64, vp, u32, u32, vp, vp]),
    "rg_shard_fixup_windows_async": (ctypes.c_int, [vp, u32, vp, u64, u64, u64, u64, u64, u64, vp, u64, vp, u32, u32,
                                                    vp, vp]),
    "rg_shard_commit_windows_async": (ctypes.c_int, [vp, u32, vp, u32, u64, u64, vp, vp]),
    "rg_decision_bitmap_windows_async": (ctypes.c_int, [vp, u32, vp, u64, u64, u64, vp, vp, u64, vp]),
    "rg_decision_lists_windows_async": (ctypes.c_int, [vp, u32, vp, u64, u64, u64, vp, u32, vp, u64, vp]),
    "rg_shard_commit_async": (ctypes.c_int, [vp, vp, u32, u64, u64, vp, vp]),
    "rg_last_result": (ctypes.c_int, [vp, ctypes.POINTER(RgStepResult)]),
    "rg_last_stage_result": (ctypes.c_int, [vp, ctypes.c_int, ctypes.POINTER(RgStepResult)]),
    "rg_digest_majority_async": (ctypes.c_int, [vp, vp, u64, vp, u64, vp]),
    "rg_coin_async": (ctypes.c_int, [vp, u64, u64, u64, vp, vp]),
    "rg_ref_draws_async": (ctypes.c_int, [vp, u64, u64, vp, vp]),
    "rg_decision_bitmap_async": (ctypes.c_int, [vp, vp, u64, u64, vp, vp, vp]),
    "rg_round1_votes_async": (ctypes.c_int, [vp, vp, vp, u64, vp, u64, u64, u64, u32, vp, vp]),
    "rg_trace_generate_async": (ctypes.c_int, [vp, ctypes.c_int, u64, u64, u64, u64, vp, vp]),
    "rg_digest_trace_async": (ctypes.c_int, [vp, u64, u64, u64, u64, vp, vp]),
    "rg_wmvc_cluster_async": (ctypes.c_int, [vp, vp, u64, u64, u64, u64, u32, vp, vp, vp]),
    "rg_cluster_trace_async": (ctypes.c_int, [vp, u64, u64, u64, u64, vp, vp]),
    "rg_wmvc_cluster_bitmaps_async": (ctypes.c_int, [vp, vp, u64, u64, u64, u64, u32, vp, vp, vp, vp, vp]),
    "rg_cluster_bitmap_async": (ctypes.c_int, [vp, vp, u64, vp, vp, vp]),
    "rg_stream_sync": (ctypes.c_int, [vp, vp]),
    "rg_pack_codes": (ctypes.c_int, [vp, u32, u64, u64, vp]),
    "rg_unpack_planes": (ctypes.c_int, [vp, u32, u64, u64, vp]),
    "rg_planar_to_tiled": (ctypes.c_int, [vp, u32, u64, u64, u32, vp]),
    "rg_tiled_to_planar": (ctypes.c_int, [vp, u32, u64, u32, u64, vp]),
    # multi-GPU exchange over RCCL (include/rabia_gpu.h)
    "rg_comm_unique_id": (ctypes.c_int, [vp]),
    "rg_comm_create": (ctypes.c_int, [vp, vp, ctypes.c_int, ctypes.c_int]),
    "rg_comm_destroy": (ctypes.c_int, [vp]),
    "rg_comm_rank": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    "rg_comm_reserve": (ctypes.c_int, [vp, u32, u64, u32]),
    "rg_comm_allgather_async": (ctypes.c_int, [vp, vp, vp, u64, vp]),
    "rg_shard_exchange_windows_async": (ctypes.c_int, [vp, u32, vp, u64, u64, u64, u64, u64, u64, u64, vp, u64, vp,
                                                       vp, vp, vp]),
    "rg_shard_exchange_decisions_async": (ctypes.c_int, [vp, u32, vp, u64, u64, u64, u64, u64, u64, u64, vp, u64,
                                                         vp, vp, u32, u32, vp, vp]),
    "rg_comm_barrier": (ctypes.c_int, [vp]),
    "rg_comm_max_f64": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_double), u32]),
    # kvstore apply (include/rabia_kv.h)
    "rg_kv_create": (ctypes.c_int, [ctypes.POINTER(vp), ctypes.POINTER(RgKvConfig)]),
    "rg_kv_destroy": (ctypes.c_int, [vp]),
    "rg_kv_last_error": (ctypes.c_char_p, [vp]),
    "rg_kv_mark_applied_async": (ctypes.c_int, [vp, vp, u64, u32, u64, u64, vp, vp, vp, vp]),
    "rg_follower_commit_async": (ctypes.c_int, [vp, vp, u64, u64, u64, u64, vp, vp, vp, vp]),
    "rg_kv_apply_async": (ctypes.c_int, [vp, vp, vp, u64, vp, vp, vp]),
    "rg_kv_get_stats": (ctypes.c_int, [vp, ctypes.POINTER(RgKvStats)]),
    "rg_kv_dump": (ctypes.c_int, [vp, vp, vp, vp, u64]),
    "rg_kv_table_slots": (ctypes.c_int, [vp, ctypes.POINTER(u64)]),
    "rg_kv_trace_async": (ctypes.c_int, [vp, u64, u64, u64, vp, u64, vp, vp]),
    "rg_kv_sync": (ctypes.c_int, [vp, vp]),
    # vote ingestion (include/rabia_ingest.h)
    "rg_ingest_create": (ctypes.c_int, [ctypes.POINTER(vp), ctypes.POINTER(RgIngestConfig)]),
    "rg_ingest_destroy": (ctypes.c_int, [vp]),
    "rg_ingest_last_error": (ctypes.c_char_p, [vp]),
    "rg_ingest_votes_async": (ctypes.c_int, [vp, vp, vp, vp, u64, u64, vp, u64, u64, u64, vp, vp]),
    # diagnostics (include/rabia_gpu_debug.h)
    "rg_debug_set": (ctypes.c_int, [vp, u32]),
    "rg_debug_stamps": (ctypes.c_int, [vp, vp, u64]),
    "rg_debug_last_launch": (ctypes.c_int, [vp, vp]),
    "rg_debug_stream_probe": (ctypes.c_int, [vp, vp, u64, u64, u32, u32, vp]),
}

_lib = None


def header_symbols() -> list[str]:
    """Every function declared in include/rabia_gpu.h and include/rabia_kv.h."""
    names = set()
    for h in HEADERS:
        with open(h) as f:
            text = f.read()
        names |= set(re.findall(r"^\s*(?:[\w\s\*]+?)\b(rg_\w+)\s*\(", text, re.M))
    return sorted(names)


def load():
    """Load librabia_gpu.so (building it first if it is missing)."""
    global _lib
    if _lib is not None:
        return _lib
    try:  # share torch's HIP runtime when torch is present (see module doc)
        import torch  # noqa: F401
    except Exception:  # pragma: no cover - torch is optional for the binding itself
        pass
    if LIB_PATH == os.path.join(PKG, "lib", "librabia_gpu.so"):
        from . import build as _build
        if _build.needs_build():  # missing, or older than one of its sources
            _build.build()
    elif not os.path.exists(LIB_PATH):
        raise FileNotFoundError(f"RABIA_GPU_LIB={LIB_PATH} does not exist")
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


class RabiaGpuError(RuntimeError):
    """Error returned by the C ABI (maps onto the reference's RabiaError variants:
    RG_EINVAL/RG_EHIP/RG_ENOMEM/RG_ENODEV -> Internal, RG_ESTATE -> Consensus)."""

    def __init__(self, code: int, message: str):
        super().__init__(f"[{code}] {message}")
        self.code = code
        self.message = message


def check(rc: int, ctx=None):
    if rc != RG_OK:
        msg = load().rg_last_error(ctx)
        raise RabiaGpuError(rc, msg.decode() if msg else "")
    return rc


def check_ingest(rc: int, h=None):
    if rc != RG_OK:
        msg = load().rg_ingest_last_error(h)
        raise RabiaGpuError(rc, msg.decode() if msg else "")
    return rc


def check_kv(rc: int, kv=None):
    if rc != RG_OK:
        msg = load().rg_kv_last_error(kv)
        raise RabiaGpuError(rc, msg.decode() if msg else "")
    return rc
