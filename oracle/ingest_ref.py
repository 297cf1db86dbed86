"""CPU restatement of vote ingestion — TEST INFRASTRUCTURE ONLY.

Only tests/ may import this module, as the checker of rabia_amd/csrc/rg_ingest.hip
(include/rabia_ingest.h); the product path never calls it.

Restates, for wire messages (TCP MessageFrame payloads, rabia-engine/src/network/tcp.rs:114-176):
  bincode::deserialize::<ProtocolMessage>        tcp.rs:583-596 (undecodable frames are dropped)
  ProtocolMessage / MessageType / VoteRound{1,2}  rabia-core/src/messages.rs:7-13, 59-94
  ProtocolMessage::validate                       rabia-core/src/validation.rs:30-81
                                                  (timestamp skew 60 s ahead / 600 s behind;
                                                  VoteRound2 needs a non-empty round1_votes)
  handle_message sender check                     rabia-engine/src/engine.rs:350-368
  add_round{1,2}_vote(from, vote)                 engine.rs:490-492, 620-622; messages.rs:169-175
                                                  (keyed by SENDER; HashMap insert = last wins)
Wire encoding (bincode 1.3.3, uuid 1.18.0 with serde, Cargo.lock): little-endian
fixed-width integers; Uuid as serialize_bytes = u64 length (16) + 16 bytes; newtypes
(PhaseId, NodeId, BatchId) transparent; enums as u32 variant index; Option as a u8
tag; HashMap as u64 count + (key, value) pairs. Parity of the byte layout is pinned
by construction only: the reference holds no serialized message fixtures and its
crates cannot be built here — "parity unpinned" for the exact bytes.
"""
from __future__ import annotations

import struct

VOTE_R1, VOTE_R2 = 1, 2
CATS = ["r1", "r2", "superseded", "other", "outside", "invalid", "sender", "malformed"]
SKEW_MS = 60_000


def uuid_bytes(u: bytes) -> bytes:
    assert len(u) == 16
    return struct.pack("<Q", 16) + u


def encode_message(msg_id: bytes, sender: bytes, to, timestamp: int, variant: int, body: bytes) -> bytes:
    out = uuid_bytes(msg_id) + uuid_bytes(sender)
    out += b"\x00" if to is None else b"\x01" + uuid_bytes(to)
    return out + struct.pack("<QI", timestamp, variant) + body


def vote_body(phase: int, batch_id: bytes, vote: int, voter: bytes, round1_votes=None) -> bytes:
    body = struct.pack("<Q", phase) + uuid_bytes(batch_id) + struct.pack("<I", vote) + uuid_bytes(voter)
    if round1_votes is not None:
        body += struct.pack("<Q", len(round1_votes))
        for node, v in round1_votes:
            body += uuid_bytes(node) + struct.pack("<I", v)
    return body


class _R:
    def __init__(self, b: bytes):
        self.b, self.pos = b, 0

    def take(self, k):
        if self.pos + k > len(self.b):
            raise ValueError("eof")
        v = self.b[self.pos:self.pos + k]
        self.pos += k
        return v

    def u64(self):
        return struct.unpack("<Q", self.take(8))[0]

    def u32(self):
        return struct.unpack("<I", self.take(4))[0]

    def uuid(self):
        if self.u64() != 16:
            raise ValueError("uuid length")
        return self.take(16)


def parse(b: bytes):
    """-> ("other",) | ("vote", variant, sender, ts, phase, vote, n_round1) ; raises on malformed."""
    r = _R(b)
    r.uuid()
    sender = r.uuid()
    tag = r.take(1)[0]
    if tag > 1:
        raise ValueError("option tag")
    if tag == 1:
        r.uuid()
    ts = r.u64()
    variant = r.u32()
    if variant > 8:
        raise ValueError("variant")
    if variant not in (VOTE_R1, VOTE_R2):
        return ("other",)
    phase = r.u64()
    r.uuid()
    vote = r.u32()
    r.uuid()
    if vote > 2:
        raise ValueError("StateValue")
    count = 0
    if variant == VOTE_R2:
        count = r.u64()
        for _ in range(count):
            r.uuid()
            if r.u32() > 2:
                raise ValueError("StateValue")
    return ("vote", variant, sender, ts, phase, vote, count)


def ingest(msgs, senders, members, now_ms, slot_base, codes_r1, codes_r2, stats=None):
    """Apply messages in order to codes_r{1,2}[lane][slot_off] (3 = absent);
    senders[m] = transport sender lane or None. Returns the stats dict."""
    st = stats if stats is not None else {c: 0 for c in CATS}
    n_slots = codes_r1.shape[1]
    last = {}
    for m, b in enumerate(msgs):
        try:
            p = parse(b)
        except (ValueError, struct.error):
            st["malformed"] += 1
            continue
        if p[0] == "other":
            st["other"] += 1
            continue
        _, variant, sender, ts, phase, vote, count = p
        if ts > now_ms + SKEW_MS or (now_ms > ts and now_ms - ts > 10 * SKEW_MS) or \
                (variant == VOTE_R2 and count == 0):
            st["invalid"] += 1
            continue
        lane = members.index(sender) if sender in members else -1
        if lane < 0 or (senders is not None and senders[m] is not None and senders[m] != lane):
            st["sender"] += 1
            continue
        if not slot_base <= phase < slot_base + n_slots:
            st["outside"] += 1
            continue
        key = (variant, lane, phase - slot_base)
        if key in last:
            st["superseded"] += 1
        else:
            st["r1" if variant == VOTE_R1 else "r2"] += 1
        last[key] = vote
    for (variant, lane, s), v in last.items():
        (codes_r1 if variant == VOTE_R1 else codes_r2)[lane, s] = v
    return st
