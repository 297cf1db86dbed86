"""Per-step checkpoint of the device engine state.

The reference persists after EVERY V1 commit (engine.rs:652-655 -> save_state,
engine.rs:156-182): serde_json of rabia_core::persistence::EngineState
{current_phase, last_committed_phase, snapshot} (rabia-core/src/persistence.rs:9-42),
written as temp file + rename (rabia-persistence/src/file_system.rs:62-76), read
back by initialize (engine.rs:238-261). With a window of 10^5-10^8 slots per step
that is one JSON write per decided slot; here one checkpoint is taken per step:

  * `engine_state_json` produces the reference's EngineState bytes exactly as
    serde_json::to_vec would (compact, declaration order; PhaseId newtypes as
    numbers; Snapshot.data (bytes::Bytes) as an array of numbers; checksum =
    crc32fast::hash(data) = CRC-32/IEEE), so a reference node can restore from it;
  * `Checkpoint` adds what the batched engine needs to resume bit-exactly: the
    StdRng position, the contiguous commit watermark and the window's decided /
    V1 bitmaps (rg_decision_bitmap_async), in a little-endian binary record with a
    CRC-32 trailer, saved by the same temp-file + rename discipline.
Byte-level parity of the JSON is by construction (the reference holds no
serialized fixture): "parity unpinned" for the JSON bytes.
"""
from __future__ import annotations

import json
import os
import struct
import zlib
from dataclasses import dataclass, field

import numpy as np

MAGIC = b"RGCK"
VERSION = 1
_HDR = struct.Struct("<4sIQQQQQQQQ")  # magic, version, slot_base, n_slots, current_phase,
                                     # last_committed, commit_watermark, rng_next, steps, n_words


def engine_state_json(current_phase: int, last_committed_phase: int, snapshot=None) -> bytes:
    """serde_json::to_vec(&EngineState) (persistence.rs:9-35). snapshot = None or
    (version, data bytes): Snapshot::new computes the checksum (state_machine.rs:14-24)."""
    snap = None
    if snapshot is not None:
        version, data = snapshot
        snap = {"version": int(version), "data": list(bytes(data)), "checksum": zlib.crc32(bytes(data))}
    obj = {"current_phase": int(current_phase), "last_committed_phase": int(last_committed_phase),
           "snapshot": snap}
    return json.dumps(obj, separators=(",", ":")).encode()


def parse_engine_state_json(data: bytes) -> dict:
    """EngineState::from_bytes (persistence.rs:37-42) + Snapshot::verify_checksum."""
    obj = json.loads(data)
    snap = obj.get("snapshot")
    if snap is not None and zlib.crc32(bytes(snap["data"])) != snap["checksum"]:
        raise ValueError("snapshot checksum mismatch (RabiaError::ChecksumMismatch)")
    return obj


@dataclass
class Checkpoint:
    slot_base: int
    n_slots: int
    current_phase: int
    last_committed: int
    commit_watermark: int
    rng_next: int
    steps: int
    committed: np.ndarray = field(default_factory=lambda: np.zeros(0, np.uint32))
    v1: np.ndarray = field(default_factory=lambda: np.zeros(0, np.uint32))

    def to_bytes(self) -> bytes:
        nw = (self.n_slots + 31) // 32
        c = np.ascontiguousarray(self.committed, np.uint32)
        v = np.ascontiguousarray(self.v1, np.uint32)
        if c.size != nw or v.size != nw:
            raise ValueError("bitmaps must hold ceil(n_slots/32) words")
        body = _HDR.pack(MAGIC, VERSION, self.slot_base, self.n_slots, self.current_phase, self.last_committed,
                         self.commit_watermark, self.rng_next, self.steps, nw) + c.tobytes() + v.tobytes()
        return body + struct.pack("<I", zlib.crc32(body))

    @classmethod
    def from_bytes(cls, data: bytes) -> "Checkpoint":
        if len(data) < _HDR.size + 4:
            raise ValueError("checkpoint truncated")
        body, (crc,) = data[:-4], struct.unpack("<I", data[-4:])
        if zlib.crc32(body) != crc:
            raise ValueError("checkpoint CRC mismatch")
        magic, ver, sb, ns, cp, lc, wm, rn, st, nw = _HDR.unpack_from(body)
        if magic != MAGIC or ver != VERSION or nw != (ns + 31) // 32 or len(body) != _HDR.size + 8 * nw:
            raise ValueError("not a checkpoint of this format")
        words = np.frombuffer(body, np.uint32, 2 * nw, _HDR.size)
        return cls(sb, ns, cp, lc, wm, rn, st, words[:nw].copy(), words[nw:].copy())

    def engine_state_json(self, snapshot=None) -> bytes:
        return engine_state_json(self.current_phase, self.last_committed, snapshot)

    # -- files (rabia-persistence/src/file_system.rs:62-76: temp file + rename) --
    def save(self, path: str) -> None:
        tmp = path + ".tmp"
        with open(tmp, "wb") as f:
            f.write(self.to_bytes())
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, path)

    @classmethod
    def load(cls, path: str):
        if not os.path.exists(path):
            return None  # first start (load_state -> Ok(None))
        with open(path, "rb") as f:
            return cls.from_bytes(f.read())


def capture(evaluator, out_ptr: int, n_slots: int, stride: int, slot_base: int, current_phase: int,
            stream=None) -> Checkpoint:
    """Checkpoint after a step: device engine state (rg_get_state) + the step's
    decided / V1 bitmaps (rg_decision_bitmap_async) of the output buffer."""
    import torch
    nw = (n_slots + 31) // 32
    cm = torch.empty(nw, dtype=torch.int32, device="cuda")
    v1 = torch.empty(nw, dtype=torch.int32, device="cuda")
    evaluator.decision_bitmap_async(out_ptr, n_slots, stride, cm.data_ptr(), v1.data_ptr(), stream or 0)
    evaluator.sync(stream or 0)
    st = evaluator.get_state()
    return Checkpoint(slot_base, n_slots, current_phase, st["last_committed"], st["commit_watermark"],
                      st["rng_next"], st["steps"], cm.cpu().numpy().view(np.uint32).copy(),
                      v1.cpu().numpy().view(np.uint32).copy())


def restore(evaluator, ckpt: Checkpoint) -> None:
    """initialize (engine.rs:238-261) for the batched engine: rg_set_state."""
    evaluator.set_state(rng_next=ckpt.rng_next, last_committed=ckpt.last_committed,
                        commit_watermark=ckpt.commit_watermark, steps=ckpt.steps)
