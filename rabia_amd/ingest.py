"""Host mirror of vote ingestion (include/rabia_ingest.h): received ProtocolMessage
frames -> the window's packed vote planes, on the device.

Stands in for the per-message path of the reference (tcp.rs reader task ->
RabiaEngine::handle_message -> handle_vote_round{1,2} -> PhaseData::add_round{1,2}_vote,
rabia-engine/src/network/tcp.rs:583-596, engine.rs:350-368, 483-492, 613-622).
No CPU fallback: without the native library or a gfx950 device the constructor raises.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native as N


def pack_messages(msgs):
    offs = np.zeros(len(msgs) + 1, np.uint64)
    if msgs:
        offs[1:] = np.cumsum([len(m) for m in msgs], dtype=np.uint64)
    data = np.frombuffer(b"".join(msgs), np.uint8) if msgs else np.zeros(0, np.uint8)
    return data, offs


class VoteIngestor:
    def __init__(self, members, tile_words: int = 0, device: int = 0):
        """members: NodeId UUID bytes (16 each) in lane order (sorted membership)."""
        if not 1 <= len(members) <= 16 or any(len(m) != 16 for m in members):
            raise ValueError("members must be 1..16 UUIDs of 16 bytes")
        self.lib = N.load()
        self.n = len(members)
        self.members = [bytes(m) for m in members]
        self.tile_words = tile_words
        self.device = device
        c = N.RgIngestConfig()
        c.n_replicas, c.tile_words, c.device = self.n, tile_words, device
        for lane, m in enumerate(self.members):
            for i, b in enumerate(m):
                c.members[lane][i] = b
        h = ctypes.c_void_p()
        N.check_ingest(self.lib.rg_ingest_create(ctypes.byref(h), ctypes.byref(c)))
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            self.lib.rg_ingest_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def ingest_async(self, msgs_ptr, off_ptr, sender_ptr, n_msgs, now_ms, votes_ptr, n_slots, stride_words,
                     slot_base, stats_ptr, stream=0):
        N.check_ingest(self.lib.rg_ingest_votes_async(self.h, msgs_ptr, off_ptr, sender_ptr or None, n_msgs,
                                                      now_ms, votes_ptr, n_slots, stride_words, slot_base,
                                                      stats_ptr, stream or None), self.h)

    def ingest(self, msgs, senders, now_ms, votes_dev, n_slots, stride_words, slot_base, stats_dev):
        """Synchronous convenience: uploads `msgs` (list of bytes) and `senders` (lane
        per message or None) and records them into the device planes `votes_dev`
        (a torch tensor); stats_dev = torch int64 tensor of 8 counters."""
        import torch
        data, offs = pack_messages(list(msgs))
        if len(msgs) == 0:
            return
        dev = torch.device("cuda", self.device)
        d = torch.from_numpy(data.copy()).to(dev)
        o = torch.from_numpy(offs.view(np.int64)).to(dev)
        s = torch.from_numpy(np.asarray(senders, np.uint8)).to(dev) if senders is not None else None
        torch.cuda.synchronize(dev)
        self.ingest_async(d.data_ptr(), o.data_ptr(), s.data_ptr() if s is not None else None, len(msgs), now_ms,
                          votes_dev.data_ptr(), n_slots, stride_words, slot_base, stats_dev.data_ptr(), None)
        torch.cuda.synchronize(dev)
