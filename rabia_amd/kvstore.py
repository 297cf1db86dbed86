"""Host mirror of the kvstore_smr state machine over the device apply (include/rabia_kv.h).

Mirrors the reference interface the engine's apply step calls for the kvstore
example: KVOperation / KVResult (examples/kvstore_smr/src/operations.rs:10-63),
KVStoreConfig (store.rs:17-42) and KVStoreSMR::apply_command(s) / get_state
(smr_impl.rs:66-131). Commands travel as their Command.data bytes (bincode 1.3.3
of KVOperation); the store itself lives in HBM and is only read back by
`get_state()` (a snapshot, like get_all_data).

The device path is the only path: without the native library or a gfx950 device
the constructor raises (no CPU fallback).
"""
from __future__ import annotations

import ctypes
import struct
from dataclasses import dataclass
from enum import IntEnum

import numpy as np

from . import _native as N


class KVResult(IntEnum):
    """Per-command result codes (include/rabia_kv.h)."""
    SUCCESS = 0
    NOT_FOUND = 1
    ERR_KEY_EMPTY = 2      # Error("Invalid key: Key cannot be empty")
    ERR_KEY_TOO_LONG = 3   # Error("Invalid key: Key too long")
    ERR_VALUE_TOO_LARGE = 4
    ERR_STORE_FULL = 5
    ERR_DECODE = 6         # Command.data is not a bincode KVOperation
    NOT_APPLIED = 7        # slot not decided V1
    ERR_CAPACITY = 8       # the store's table / heap could not hold the batch: refused whole

    def is_success(self):
        return self == KVResult.SUCCESS

    def is_not_found(self):
        return self == KVResult.NOT_FOUND

    def is_error(self):
        return self not in (KVResult.SUCCESS, KVResult.NOT_FOUND, KVResult.NOT_APPLIED)


class KVOperation:
    """bincode 1.3.3 encoding of the KVOperation enum (operations.rs:10-19):
    u32 variant index, then each String as u64 length + UTF-8 bytes."""
    SET, GET, DELETE, EXISTS = 0, 1, 2, 3

    @staticmethod
    def _s(x) -> bytes:
        b = x.encode("utf-8") if isinstance(x, str) else bytes(x)
        return struct.pack("<Q", len(b)) + b

    @classmethod
    def set(cls, key, value) -> bytes:
        return struct.pack("<I", cls.SET) + cls._s(key) + cls._s(value)

    @classmethod
    def get(cls, key) -> bytes:
        return struct.pack("<I", cls.GET) + cls._s(key)

    @classmethod
    def delete(cls, key) -> bytes:
        return struct.pack("<I", cls.DELETE) + cls._s(key)

    @classmethod
    def exists(cls, key) -> bytes:
        return struct.pack("<I", cls.EXISTS) + cls._s(key)


@dataclass
class KVStoreConfig:
    max_keys: int = 1_000_000          # store.rs:35
    max_value_size: int = 1024 * 1024  # store.rs:39
    enable_notifications: bool = True  # store.rs:36
    table_slots: int = 0               # 0 => next pow2 >= 2 * max_keys
    heap_bytes: int = 0                # 0 => 64 * table_slots
    hash_bits: int = 0                 # test hook: truncated key hashes force collision runs
    bucket_bits: int = 0               # test hook: narrow sort buckets mix distinct hashes in a run


def pack_commands(blobs):
    """Concatenate command bytes -> (data u8[], offsets u64[n+1])."""
    offs = np.zeros(len(blobs) + 1, np.uint64)
    if blobs:
        offs[1:] = np.cumsum([len(b) for b in blobs], dtype=np.uint64)
    data = np.frombuffer(b"".join(blobs), np.uint8) if blobs else np.zeros(0, np.uint8)
    return data, offs


class DeviceKVStore:
    """KVStoreSMR whose store is resident in HBM."""

    def __init__(self, config: KVStoreConfig | None = None, device: int = 0):
        self.lib = N.load()
        self.config = config or KVStoreConfig()
        c = N.RgKvConfig(self.config.max_keys, self.config.max_value_size,
                         1 if self.config.enable_notifications else 0, device,
                         self.config.table_slots, self.config.heap_bytes, self.config.hash_bits,
                         self.config.bucket_bits)
        h = ctypes.c_void_p()
        N.check_kv(self.lib.rg_kv_create(ctypes.byref(h), ctypes.byref(c)))
        self.kv = h
        self.device = device

    def close(self):
        if getattr(self, "kv", None):
            self.lib.rg_kv_destroy(self.kv)
            self.kv = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ---- device-pointer entry points (stream-ordered) ----
    def apply_async(self, data_ptr, off_ptr, n_cmds, mask_ptr, results_ptr, stream=0):
        N.check_kv(self.lib.rg_kv_apply_async(self.kv, data_ptr, off_ptr, n_cmds, mask_ptr or None,
                                              results_ptr, stream or None), self.kv)

    def mark_applied_async(self, out_ptr, stride_words, tile_words, n_slots, slot_cmd_off_ptr, mask_ptr,
                           stream=0, slot_base=1, gate_ptr=0):
        """gate_ptr = 0: proposer (every V1 slot); else a device u64 last_committed:
        follower (V1 slots with PhaseId above it, engine.rs:723-728)."""
        N.check_kv(self.lib.rg_kv_mark_applied_async(self.kv, out_ptr, stride_words, tile_words, n_slots,
                                                     slot_base, gate_ptr or None, slot_cmd_off_ptr, mask_ptr,
                                                     stream or None), self.kv)

    def trace_async(self, seed, n_cmds, key_space, data_ptr, data_cap, off_ptr, stream=0):
        N.check_kv(self.lib.rg_kv_trace_async(self.kv, seed, n_cmds, key_space, data_ptr, data_cap, off_ptr,
                                              stream or None), self.kv)

    def sync(self, stream=0):
        N.check_kv(self.lib.rg_kv_sync(self.kv, stream or None), self.kv)

    # ---- host convenience (KVStoreSMR::apply_commands, smr_impl.rs:120-127) ----
    def apply_commands(self, blobs, mask=None) -> list:
        """Synchronous: uploads, applies on the store's own stream, waits, returns
        one KVResult per command."""
        import torch
        data, offs = pack_commands(list(blobs))
        n = len(offs) - 1
        if n == 0:
            return []
        dev = torch.device("cuda", self.device)
        d = torch.from_numpy(data.copy() if data.size else np.zeros(1, np.uint8)).to(dev)
        o = torch.from_numpy(offs.view(np.int64)).to(dev)
        m = torch.from_numpy(np.asarray(mask, np.uint8)).to(dev) if mask is not None else None
        r = torch.empty(n, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize(dev)  # the store's stream does not order after torch's
        flags0 = self.stats()["flags"]
        self.apply_async(d.data_ptr(), o.data_ptr(), n, m.data_ptr() if m is not None else None,
                         r.data_ptr(), None)
        self.sync()
        st = self.stats()
        if st["flags"] & 4:  # a fault inside a commit pass (include/rabia_kv.h): sticky, later batches refused
            if flags0 & 4:
                raise N.RabiaGpuError(N.RG_ESTATE, f"kvstore lost by an earlier faulted batch (flags {st['flags']}): "
                                                   f"this batch of {n} commands was refused and wrote nothing")
            raise N.RabiaGpuError(N.RG_ESTATE, f"kvstore capacity fault during the commit (flags {st['flags']}): "
                                               f"the batch of {n} commands is partially written; the store is lost")
        if st["last_path"] == 2 or st["flags"] != flags0:
            raise N.RabiaGpuError(N.RG_ESTATE, f"kvstore capacity exceeded (flags {st['flags']}): the batch of "
                                               f"{n} commands was refused and changed nothing")
        return [KVResult(int(x)) for x in r.cpu().numpy()]

    def apply_command(self, blob) -> KVResult:
        return self.apply_commands([blob])[0]

    def stats(self) -> dict:
        st = N.RgKvStats()
        N.check_kv(self.lib.rg_kv_get_stats(self.kv, ctypes.byref(st)), self.kv)
        return st.as_dict()

    def get_state(self) -> dict:
        """KVStoreState (smr_impl.rs:14-18) without the wall-clock fields:
        {"data": {key bytes: (value bytes, entry version)}, "version": KVStore.version}."""
        st = self.stats()
        slots = ctypes.c_uint64()
        N.check_kv(self.lib.rg_kv_table_slots(self.kv, ctypes.byref(slots)), self.kv)
        n = int(slots.value)
        hashes = np.zeros(n, np.uint64)
        ent = np.zeros((n, 4), np.uint64)
        heap = np.zeros(max(1, st["heap_used"]), np.uint8)
        N.check_kv(self.lib.rg_kv_dump(self.kv, hashes.ctypes.data, ent.ctypes.data, heap.ctypes.data,
                                       heap.size), self.kv)
        data = {}
        for s in np.nonzero((hashes != 0) & (ent[:, 2] != 0))[0]:
            ko, vo, ver, lens = (int(x) for x in ent[s])
            kl, vl = lens & 0xFFFFFFFF, lens >> 32
            data[heap[ko:ko + kl].tobytes()] = (heap[vo:vo + vl].tobytes(), ver)
        return {"data": data, "version": st["version"]}
