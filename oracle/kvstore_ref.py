"""CPU restatement of the kvstore_smr apply path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker; the product path (rabia_amd/kvstore.py over
rabia_amd/csrc/rg_kv.hip) never calls it.

What it restates (reference @ /root/reference, read as text):
  KVOperation / KVResult / StoreError     examples/kvstore_smr/src/operations.rs:10-19, 55-63, 97-108
  KVStoreSMR::apply_command(s)            examples/kvstore_smr/src/smr_impl.rs:72-127
  KVStore::set / get / delete / exists    examples/kvstore_smr/src/store.rs:144-189, 191-201, 217-251, 254-262
  validate_key / validate_value           store.rs:463-478   (key: non-empty, <= 256 bytes;
                                                              value: <= max_value_size bytes)
  ValueEntry::new / update                store.rs:55-80     (version 1, +1 per update)
  KVStore.version via get_version()       store.rs:486-489   (fetch_add per notification:
                                                              every successful SET, every DELETE
                                                              that removed a key, when
                                                              enable_notifications)
  KVStoreConfig::default                  store.rs:32-42     (max_keys 1,000,000; 1 MiB values)
and the wire form of a command's data (Command.data, rabia-core/src/types.rs:321-326):
bincode 1.3.3 (Cargo.lock) default options = little-endian fixed-width integers, enum
variant as u32, String as u64 length + UTF-8 bytes, trailing bytes allowed.

Result codes (shared with include/rabia_kv.h):
  0 Success, 1 NotFound, 2 Error(InvalidKey "Key cannot be empty"),
  3 Error(InvalidKey "Key too long"), 4 Error(ValueTooLarge), 5 Error(StoreFull),
  6 decode error (Command.data is not a bincode KVOperation), 7 not applied
  (the command's slot was not decided V1).
Wall-clock fields of ValueEntry (created_at/updated_at, store.rs:45-80) are
nondeterministic in the reference and are not part of the compared state.
"""
from __future__ import annotations

import struct

SET, GET, DELETE, EXISTS = 0, 1, 2, 3
OK, NOT_FOUND, E_KEY_EMPTY, E_KEY_LONG, E_VALUE_LARGE, E_FULL, E_DECODE, NOT_APPLIED = range(8)
RESULT_NAMES = ["Success", "NotFound", "Error(Invalid key: Key cannot be empty)",
                "Error(Invalid key: Key too long)", "Error(Value too large)", "Error(Store is full)",
                "DecodeError", "NotApplied"]
MAX_KEY_LEN = 256                 # store.rs:467
DEFAULT_MAX_KEYS = 1_000_000      # store.rs:35
DEFAULT_MAX_VALUE = 1024 * 1024   # store.rs:39


# ---- bincode 1.3.3 wire form of KVOperation (operations.rs:10-19) ------------
def encode_op(kind: int, key: bytes, value: bytes = b"") -> bytes:
    out = struct.pack("<IQ", kind, len(key)) + key
    if kind == SET:
        out += struct.pack("<Q", len(value)) + value
    return out


def decode_op(data: bytes):
    """-> (kind, key, value) or None when bincode::deserialize would fail: short
    input, variant > 3, or a String that is not UTF-8 (serde's String visitor)."""
    if len(data) < 12:
        return None
    kind, klen = struct.unpack_from("<IQ", data, 0)
    if kind > 3 or 12 + klen > len(data):
        return None
    key = data[12:12 + klen]
    value = b""
    pos = 12 + klen
    if kind == SET:
        if pos + 8 > len(data):
            return None
        (vlen,) = struct.unpack_from("<Q", data, pos)
        if pos + 8 + vlen > len(data):
            return None
        value = data[pos + 8:pos + 8 + vlen]
    try:
        key.decode("utf-8")
        value.decode("utf-8")
    except UnicodeDecodeError:
        return None
    return kind, key, value


class KVStoreRef:
    """Sequential KVStoreSMR (smr_impl.rs:66-131) over KVStore (store.rs)."""

    def __init__(self, max_keys: int = DEFAULT_MAX_KEYS, max_value_size: int = DEFAULT_MAX_VALUE,
                 enable_notifications: bool = True):
        self.max_keys = max_keys
        self.max_value_size = max_value_size
        self.notify = enable_notifications
        self.data: dict[bytes, list] = {}   # key -> [value, entry version]
        self.version = 0                    # KVStore.version (store.rs:486-489)
        self.total_operations = 0           # StoreStats.total_operations (store.rs:480-484)

    def _validate_key(self, key: bytes):    # store.rs:463-471
        if len(key) == 0:
            return E_KEY_EMPTY
        if len(key) > MAX_KEY_LEN:
            return E_KEY_LONG
        return None

    def apply(self, kind: int, key: bytes, value: bytes = b"") -> int:
        err = self._validate_key(key)
        if err is not None:
            return err
        if kind == SET:                      # store.rs:144-189
            if len(value) > self.max_value_size:
                return E_VALUE_LARGE
            e = self.data.get(key)
            if e is not None:
                e[0] = value
                e[1] += 1
            else:
                if len(self.data) >= self.max_keys:
                    return E_FULL
                self.data[key] = [value, 1]
            self.total_operations += 1
            if self.notify:
                self.version += 1
            return OK
        if kind in (GET, EXISTS):            # store.rs:191-201, 254-262; smr_impl.rs:79-94
            self.total_operations += 1
            return OK if key in self.data else NOT_FOUND
        if kind == DELETE:                   # store.rs:217-251
            existed = self.data.pop(key, None) is not None
            self.total_operations += 1
            if existed and self.notify:
                self.version += 1
            return OK if existed else NOT_FOUND
        raise ValueError(kind)

    def apply_data(self, data: bytes) -> int:
        op = decode_op(data)
        if op is None:
            return E_DECODE
        return self.apply(*op)

    def apply_commands(self, blobs) -> list:  # smr_impl.rs:120-127: in order, one response each
        return [self.apply_data(b) for b in blobs]

    def state(self) -> dict:
        """Compared state: key -> (value, entry version), plus the store version."""
        return {"data": {k: (v[0], v[1]) for k, v in self.data.items()}, "version": self.version}


def apply_decided(store: KVStoreRef, blobs, slot_cmd_off, applied_slots):
    """Engine-side apply (engine.rs:646-655 / 727-735): the batches of V1-decided
    slots, in ascending slot order; commands of other slots get NOT_APPLIED."""
    res = [NOT_APPLIED] * len(blobs)
    for s in applied_slots:
        for c in range(int(slot_cmd_off[s]), int(slot_cmd_off[s + 1])):
            res[c] = store.apply_data(blobs[c])
    return res
