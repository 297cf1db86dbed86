"""Host-side mirror of the reference's phase-evaluation interface, over the C ABI.

Names follow rabia-rs so a maintainer finds the same concepts:
  StateValue (rabia-core/src/types.rs:286-294), NodeId::from(u32) (types.rs:49-75),
  ClusterConfig.quorum_size (rabia-core/src/network.rs:13-21),
  PhaseData::add_round{1,2}_vote / has_round{1,2}_majority (rabia-core/src/messages.rs:169-183)
  -> PhaseWindow (a window of PhaseData as SoA bit planes),
  EngineState.last_committed_phase / commit_phase (rabia-engine/src/state.rs:55-103)
  -> PhaseEvaluator.state.

Every evaluation runs on the GPU through librabia_gpu.so; there is no CPU path.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from enum import IntEnum

import numpy as np

from . import _native as N


class StateValue(IntEnum):
    V0 = 0
    V1 = 1
    VQuestion = 2


ABSENT = 3  # voter not in the HashMap / None / pending


def node_id_from_u32(value: int) -> bytes:
    """NodeId::from(u32): the 4 big-endian bytes repeated 4 times (types.rs:49-75)."""
    return bytes([(value >> 24) & 255, (value >> 16) & 255, (value >> 8) & 255, value & 255] * 4)


@dataclass
class ClusterConfig:
    """rabia-core/src/network.rs:7-21. Lane j = j-th NodeId in sorted order."""
    node_id: bytes
    all_nodes: list

    @property
    def quorum_size(self) -> int:
        return len(self.all_nodes) // 2 + 1

    def lane_of(self, node: bytes) -> int:
        return sorted(self.all_nodes).index(node)

    def total_nodes(self) -> int:
        return len(self.all_nodes)


def record_window_words(n_slots: int, records_cap: int) -> int:
    """u32 words of one window's draw-record region of the sharded step (include/rabia_gpu.h
    rg_record_window_words): the segment table (one word per 2^24 slots + 1, rounded up to
    4), then records_cap 4-B records."""
    return ((((n_slots + 0xFFFFFF) >> 24) + 1 + 3) & ~3) + records_cap


def plane_stride(n_slots: int) -> int:
    return ((n_slots + 127) // 128) * 4


def unpack_bits(plane: np.ndarray, n_slots: int) -> np.ndarray:
    """One bit plane (uint32 words) -> uint8 per slot."""
    return np.unpackbits(np.ascontiguousarray(plane).view(np.uint8), bitorder="little")[:n_slots]


def decode_outputs(out: np.ndarray, n_slots: int) -> dict:
    """8 output planes -> per-slot arrays (codes: V0=0, V1=1, VQ=2, none=3)."""
    b = [unpack_bits(out[i], n_slots) for i in range(N.OUT_PLANES)]
    return {
        "r1": b[0] | (b[1] << 1),
        "r2own": b[2] | (b[3] << 1),
        "dec": b[4] | (b[5] << 1),
        "committed": b[6],
        "value": b[7],
    }


def to_tiled(planar: np.ndarray, n_words: int, tile_words: int) -> np.ndarray:
    """Planar planes [P][stride] -> slot-tiled buffer (include/rabia_gpu.h layout)."""
    planar = np.ascontiguousarray(planar, np.uint32)
    P, stride = planar.shape
    tiles = (n_words + tile_words - 1) // tile_words
    out = np.zeros(tiles * P * tile_words, np.uint32)
    N.check(N.load().rg_planar_to_tiled(planar.ctypes.data, P, n_words, stride, tile_words, out.ctypes.data))
    return out


def from_tiled(tiled: np.ndarray, n_planes: int, n_words: int, tile_words: int, stride: int) -> np.ndarray:
    tiled = np.ascontiguousarray(tiled, np.uint32)
    out = np.zeros((n_planes, stride), np.uint32)
    N.check(N.load().rg_tiled_to_planar(tiled.ctypes.data, n_planes, n_words, tile_words, stride,
                                        out.ctypes.data))
    return out


class PhaseWindow:
    """A window of `n_slots` consecutive phases' vote sets, packed as the device
    layout: (4n+1) planes of uint32 words (R1 lanes, R2 lanes, own state)."""

    def __init__(self, n_replicas: int, n_slots: int, slot_base: int = 1):
        self.n = int(n_replicas)
        self.n_slots = int(n_slots)
        self.slot_base = int(slot_base)
        self.stride = plane_stride(n_slots)
        self.planes = np.zeros((4 * self.n + 1, self.stride), np.uint32)
        # every voter starts absent (empty HashMaps, messages.rs:152-166)
        self.planes[: 4 * self.n] = 0xFFFFFFFF
        self._mask_tail()

    def _mask_tail(self):
        if self.n_slots % 32:
            w = self.n_slots // 32
            self.planes[:, w] &= np.uint32((1 << (self.n_slots % 32)) - 1)
            self.planes[:, w + 1:] = 0
        else:
            self.planes[:, self.n_slots // 32:] = 0

    @classmethod
    def from_codes(cls, r1: np.ndarray, r2: np.ndarray, state=None, slot_base: int = 1):
        r1 = np.ascontiguousarray(r1, np.uint8)
        r2 = np.ascontiguousarray(r2, np.uint8)
        S, n = r1.shape
        w = cls(n, S, slot_base)
        lib = N.load()
        N.check(lib.rg_pack_codes(r1.ctypes.data, n, S, w.stride, w.planes[: 2 * n].ctypes.data))
        N.check(lib.rg_pack_codes(r2.ctypes.data, n, S, w.stride, w.planes[2 * n: 4 * n].ctypes.data))
        w.planes[4 * n] = 0
        if state is not None:
            st = np.ascontiguousarray(state, np.uint8) & 1
            packed = np.packbits(st, bitorder="little")
            buf = np.zeros(w.stride * 4, np.uint8)
            buf[: packed.size] = packed
            w.planes[4 * n] = buf.view(np.uint32)
        return w

    def _set(self, base_plane: int, phase_id: int, lane: int, vote: int):
        s = phase_id - self.slot_base
        if not (0 <= s < self.n_slots) or not (0 <= lane < self.n):
            raise IndexError(f"phase {phase_id} / lane {lane} outside window")
        wd, bit = s // 32, np.uint32(1 << (s % 32))
        for b in range(2):
            p = self.planes[base_plane + 2 * lane + b]
            if (int(vote) >> b) & 1:
                p[wd] |= bit
            else:
                p[wd] &= ~bit

    def add_round1_vote(self, phase_id: int, lane: int, vote: StateValue):
        """PhaseData::add_round1_vote (messages.rs:169-171): last write wins."""
        self._set(0, phase_id, lane, int(vote))

    def add_round2_vote(self, phase_id: int, lane: int, vote: StateValue):
        """PhaseData::add_round2_vote (messages.rs:173-175)."""
        self._set(2 * self.n, phase_id, lane, int(vote))

    def set_state(self, phase_id: int, bit: int):
        s = phase_id - self.slot_base
        wd, m = s // 32, np.uint32(1 << (s % 32))
        if bit:
            self.planes[4 * self.n, wd] |= m
        else:
            self.planes[4 * self.n, wd] &= ~m


def _current_device() -> int:
    """torch's current device when torch has initialised the GPU in this process, else 0
    (no GPU initialisation here)."""
    import sys
    torch = sys.modules.get("torch")
    try:
        if torch is not None and torch.cuda.is_initialized():
            return int(torch.cuda.current_device())
    except Exception:
        pass
    return 0


class PhaseEvaluator:
    """Owns one rg_ctx (device state: StdRng position, last_committed_phase,
    commit watermark). Not thread-safe, like the single &mut engine task
    (engine.rs:184)."""

    def __init__(self, n_replicas: int, *, quorum: int = 0, decide_threshold: int = 0,
                 self_lane: int = -1, mode: str = "ref", seed: int = 0, coin_seed=None,
                 epoch: int = 0, device=None, tile_words: int = 0):
        self.lib = N.load()
        if device is None:  # the caller's current device (a rank's GPU after torch.cuda.set_device), else 0
            device = _current_device()
        self.n = int(n_replicas)
        self.mode = mode
        cfg = N.RgConfig(n_replicas=self.n, quorum=quorum, decide_threshold=decide_threshold,
                         self_lane=self_lane, mode=N.RG_MODE_WMVC if mode == "wmvc" else N.RG_MODE_REF,
                         device=device, seed=seed & (2 ** 64 - 1),
                         coin_seed=(seed if coin_seed is None else coin_seed) & (2 ** 64 - 1),
                         epoch=epoch, tile_words=tile_words)
        ctx = ctypes.c_void_p()
        N.check(self.lib.rg_create(ctypes.byref(ctx), ctypes.byref(cfg)))
        self.ctx = ctx
        got = N.RgConfig()
        N.check(self.lib.rg_get_config(self.ctx, ctypes.byref(got)), self.ctx)
        self.quorum = got.quorum
        self.decide_threshold = got.decide_threshold
        self.tile_words = got.tile_words

    @classmethod
    def from_configs(cls, cluster: ClusterConfig, seed: int, mode: str = "ref", **kw):
        return cls(cluster.total_nodes(), quorum=cluster.quorum_size,
                   self_lane=cluster.lane_of(cluster.node_id), mode=mode, seed=seed, **kw)

    def close(self):
        if getattr(self, "ctx", None):
            self.lib.rg_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def reserve(self, max_slots: int, max_windows: int = 1):
        """rg_reserve: size the context's scratch for calls of up to max_slots slots (all
        windows of one call) and max_windows windows. Synchronous; the _async calls never
        allocate and raise RG_EINVAL past the reservation (rg_create reserves 2^32 / 128)."""
        N.check(self.lib.rg_reserve(self.ctx, int(max_slots), int(max_windows)), self.ctx)

    # -- engine state -----------------------------------------------------
    def get_state(self) -> dict:
        st = N.RgEngineState()
        N.check(self.lib.rg_get_state(self.ctx, ctypes.byref(st)), self.ctx)
        return {"rng_next": st.rng_next, "last_committed": st.last_committed,
                "commit_watermark": st.commit_watermark, "steps": st.steps}

    def set_state(self, rng_next=0, last_committed=0, commit_watermark=1, steps=0):
        st = N.RgEngineState(rng_next, last_committed, commit_watermark, steps)
        N.check(self.lib.rg_set_state(self.ctx, ctypes.byref(st)), self.ctx)

    def last_result(self) -> dict:
        r = N.RgStepResult()
        N.check(self.lib.rg_last_result(self.ctx, ctypes.byref(r)), self.ctx)
        return r.as_dict()

    def last_stage_result(self, stage: int) -> dict:
        """The latest shard fix-up (0), shard commit (1) or follower commit (2) result."""
        r = N.RgStepResult()
        N.check(self.lib.rg_last_stage_result(self.ctx, stage, ctypes.byref(r)), self.ctx)
        return r.as_dict()

    # -- steps ---------------------------------------------------------------
    def phase_step_host(self, window: PhaseWindow, phase: int = 1, max_phase: int = 0):
        """Synchronous step over host planes: returns (out planes, result dict)."""
        if window.n != self.n:
            raise ValueError("window replica count does not match the evaluator")
        out = np.zeros((N.OUT_PLANES, window.stride), np.uint32)
        votes = np.ascontiguousarray(window.planes)
        r = N.RgStepResult()
        if not self.tile_words:
            N.check(self.lib.rg_phase_step(self.ctx, votes.ctypes.data, out.ctypes.data, window.n_slots,
                                           window.stride, window.slot_base, phase, max_phase,
                                           ctypes.byref(r)), self.ctx)
            return out, r.as_dict()
        T = self.tile_words
        nw = (window.n_slots + 31) // 32
        tiles = (nw + T - 1) // T
        tv = to_tiled(votes, nw, T)
        to = np.zeros(tiles * N.OUT_PLANES * T, np.uint32)
        N.check(self.lib.rg_phase_step(self.ctx, tv.ctypes.data, to.ctypes.data, window.n_slots, T,
                                       window.slot_base, phase, max_phase, ctypes.byref(r)), self.ctx)
        return from_tiled(to, N.OUT_PLANES, nw, T, window.stride), r.as_dict()

    def phase_step_async(self, votes_ptr: int, out_ptr: int, n_slots: int, stride: int,
                         slot_base: int = 1, phase: int = 1, max_phase: int = 0,
                         result_ptr: int = 0, stream: int = 0):
        """Device-pointer step enqueued on `stream` (a hipStream_t handle, 0 = own)."""
        N.check(self.lib.rg_phase_step_async(self.ctx, votes_ptr, out_ptr, n_slots, stride, slot_base,
                                             phase, max_phase, result_ptr or None, stream or None),
                self.ctx)

    # -- sharded REF: one engine over a window split across GPUs (shard.py) -----
    def phase_step_shard_async(self, votes_ptr, out_ptr, n_slots, stride, slot_base, records_ptr, records_cap,
                               row_ptr=0, max_phase=0, stream=0):
        """Stage 1: this shard's slots at a provisional stream position + draw records."""
        N.check(self.lib.rg_phase_step_shard_async(self.ctx, votes_ptr, out_ptr, n_slots, stride, slot_base,
                                                   max_phase, records_ptr, records_cap, row_ptr or None,
                                                   stream or None), self.ctx)

    def phase_step_shard_windows_async(self, n_windows, votes_ptr, votes_pitch, out_ptr, out_pitch, n_slots, stride,
                                       slot_base, window_stride, records_ptr, records_cap, rows_ptr, max_phase=0,
                                       stream=0):
        """Stage 1 for n_windows consecutive windows of this shard in one launch (pitches
        in 32-bit words; window w's record region at records_ptr + 4 * w * record_window_words(n_slots,
        records_cap), its row
        at rows_ptr + 80 * w)."""
        N.check(self.lib.rg_phase_step_shard_windows_async(self.ctx, n_windows, votes_ptr, votes_pitch, out_ptr,
                                                           out_pitch, n_slots, stride, slot_base, window_stride,
                                                           max_phase, records_ptr, records_cap, rows_ptr,
                                                           stream or None), self.ctx)

    def shard_fixup_async(self, out_ptr, n_slots, stride, slot_base, records_ptr, records_cap, rows_ptr, shard,
                          n_shards, row_ptr=0, max_phase=0, stream=0):
        """Stage 3: re-draw this shard's VQ slots at their global stream positions."""
        N.check(self.lib.rg_shard_fixup_async(self.ctx, out_ptr, n_slots, stride, slot_base, max_phase, records_ptr,
                                              records_cap, rows_ptr, shard, n_shards, row_ptr or None,
                                              stream or None), self.ctx)

    def shard_fixup_windows_async(self, n_windows, out_ptr, out_pitch, n_slots, stride, slot_base, window_stride,
                                  records_ptr, records_cap, rows_ptr, shard, n_shards, rows_out_ptr=0, max_phase=0,
                                  stream=0):
        """Stage 3 for n_windows windows (rows [n_shards][n_windows], rank-major)."""
        N.check(self.lib.rg_shard_fixup_windows_async(self.ctx, n_windows, out_ptr, out_pitch, n_slots, stride,
                                                      slot_base, window_stride, max_phase, records_ptr, records_cap,
                                                      rows_ptr, shard, n_shards, rows_out_ptr or None,
                                                      stream or None), self.ctx)

    def shard_commit_windows_async(self, n_windows, rows_ptr, n_shards, window_base, window_slots, results_ptr=0,
                                   stream=0):
        """Stage 4 for n_windows consecutive windows (rows [n_shards][n_windows])."""
        N.check(self.lib.rg_shard_commit_windows_async(self.ctx, n_windows, rows_ptr, n_shards, window_base,
                                                       window_slots, results_ptr or None, stream or None), self.ctx)

    def shard_commit_async(self, rows_ptr, n_shards, window_base, window_slots, result_ptr=0, stream=0):
        """Stage 4: fold every shard's final row into this context's engine state."""
        N.check(self.lib.rg_shard_commit_async(self.ctx, rows_ptr, n_shards, window_base, window_slots,
                                               result_ptr or None, stream or None), self.ctx)

    # -- multi-GPU exchange over RCCL (include/rabia_gpu.h, rabia_amd/csrc/rg_comm.hip) --
    @staticmethod
    def comm_unique_id() -> bytes:
        """Rank 0: a fresh 128-byte RCCL id, to be carried to every rank by the host."""
        lib = N.load()
        buf = (ctypes.c_uint8 * 128)()
        N.check(lib.rg_comm_unique_id(buf))
        return bytes(buf)

    def comm_create(self, uid: bytes, rank: int, world: int):
        """Collective over the `world` ranks: attach an RCCL communicator to this context."""
        if len(uid) != 128:
            raise ValueError("the RCCL id is 128 bytes")
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(uid)
        N.check(self.lib.rg_comm_create(self.ctx, buf, rank, world), self.ctx)

    def comm_destroy(self):
        N.check(self.lib.rg_comm_destroy(self.ctx), self.ctx)

    def comm_rank(self):
        r, w = ctypes.c_int(), ctypes.c_int()
        N.check(self.lib.rg_comm_rank(self.ctx, ctypes.byref(r), ctypes.byref(w)), self.ctx)
        return r.value, w.value

    def comm_reserve(self, max_windows: int, max_slots: int, undecided_cap: int = 0):
        """rg_comm_reserve: the exchange scratch for up to max_windows windows of up to
        max_slots-slot shards (and undecided lists of up to undecided_cap entries)."""
        N.check(self.lib.rg_comm_reserve(self.ctx, int(max_windows), int(max_slots), int(undecided_cap)), self.ctx)

    def comm_allgather_async(self, send_ptr, recv_ptr, nbytes, stream=0):
        N.check(self.lib.rg_comm_allgather_async(self.ctx, send_ptr, recv_ptr, nbytes, stream or None), self.ctx)

    def shard_exchange_windows_async(self, n_windows, out_ptr, out_pitch, n_slots, stride, slot_base, window_base,
                                     window_slots, records_ptr, records_cap, rows_ptr, results_ptr, bitmaps_all_ptr=0,
                                     max_phase=0, stream=0):
        """Stages 2-4 (+ bitmaps) of the sharded pipeline through the context's communicator:
        rows all-gathered, fix-up, final rows all-gathered, commit into results_ptr[K]."""
        N.check(self.lib.rg_shard_exchange_windows_async(self.ctx, n_windows, out_ptr, out_pitch, n_slots, stride,
                                                         slot_base, window_base, window_slots, max_phase, records_ptr,
                                                         records_cap, rows_ptr, results_ptr, bitmaps_all_ptr or None,
                                                         stream or None), self.ctx)

    def shard_exchange_decisions_async(self, n_windows, out_ptr, out_pitch, n_slots, stride, slot_base, window_base,
                                       window_slots, records_ptr, records_cap, rows_ptr, results_ptr, undecided_cap,
                                       decisions_all_ptr, with_v1=True, max_phase=0, stream=0):
        """Stages 2-4 with the compact decided-slot payload: every rank's undecided lists
        (+ V1 bitmaps) all-gathered into decisions_all_ptr ([world][P] u32, include/rabia_gpu.h)."""
        N.check(self.lib.rg_shard_exchange_decisions_async(self.ctx, n_windows, out_ptr, out_pitch, n_slots, stride,
                                                           slot_base, window_base, window_slots, max_phase,
                                                           records_ptr, records_cap, rows_ptr, results_ptr,
                                                           undecided_cap, 1 if with_v1 else 0, decisions_all_ptr,
                                                           stream or None), self.ctx)

    def comm_barrier(self):
        N.check(self.lib.rg_comm_barrier(self.ctx), self.ctx)

    def comm_max(self, values):
        """Element-wise max over ranks of a few host floats."""
        arr = (ctypes.c_double * len(values))(*[float(v) for v in values])
        N.check(self.lib.rg_comm_max_f64(self.ctx, arr, len(values)), self.ctx)
        return list(arr)

    def follower_commit_async(self, out_ptr, n_slots, stride, slot_base, applied_ptr=0, gate_ptr=0, result_ptr=0,
                              max_phase=0, stream=0):
        """handle_decision over a decided window (engine.rs:708-746): applied = V1 slots
        above last_committed; last_committed / watermark advance."""
        N.check(self.lib.rg_follower_commit_async(self.ctx, out_ptr, n_slots, stride, slot_base, max_phase,
                                                  applied_ptr or None, gate_ptr or None, result_ptr or None,
                                                  stream or None), self.ctx)

    def digest_majority_async(self, digests_ptr, digest_stride, state_ptr, n_slots, stream=0):
        N.check(self.lib.rg_digest_majority_async(self.ctx, digests_ptr, digest_stride, state_ptr,
                                                  n_slots, stream or None), self.ctx)

    def coin_async(self, slot_base, n_slots, phase, out_ptr, stream=0):
        N.check(self.lib.rg_coin_async(self.ctx, slot_base, n_slots, phase, out_ptr, stream or None),
                self.ctx)

    def round1_votes_async(self, phase_ids_ptr, values_ptr, n_props, proposed_ptr, stride, n_slots, slot_base,
                           track, votes_ptr, stream=0):
        """Own round-1 votes for received proposals (determine_round1_vote, engine.rs:424-481)."""
        N.check(self.lib.rg_round1_votes_async(self.ctx, phase_ids_ptr, values_ptr, n_props, proposed_ptr or None,
                                               stride, n_slots, slot_base, 1 if track else 0, votes_ptr,
                                               stream or None), self.ctx)

    def decision_bitmap_async(self, out_ptr, n_slots, stride, committed_ptr, v1_ptr, stream=0):
        N.check(self.lib.rg_decision_bitmap_async(self.ctx, out_ptr, n_slots, stride, committed_ptr, v1_ptr,
                                                  stream or None), self.ctx)

    def decision_bitmap_windows_async(self, n_windows, out_ptr, out_pitch, n_slots, stride, committed_ptr, v1_ptr,
                                      bitmap_pitch, stream=0):
        N.check(self.lib.rg_decision_bitmap_windows_async(self.ctx, n_windows, out_ptr, out_pitch, n_slots, stride,
                                                          committed_ptr, v1_ptr, bitmap_pitch, stream or None),
                self.ctx)

    def decision_lists_windows_async(self, n_windows, out_ptr, out_pitch, n_slots, stride, lists_ptr, cap, v1_ptr=0,
                                     v1_pitch=0, stream=0):
        """Undecided-slot lists ([n_windows][1 + cap] u32: count, then ascending offsets)
        and optional V1 bitmaps of n_windows windows (rg_decision_lists_windows_async)."""
        N.check(self.lib.rg_decision_lists_windows_async(self.ctx, n_windows, out_ptr, out_pitch, n_slots, stride,
                                                         lists_ptr, cap, v1_ptr or None, v1_pitch, stream or None),
                self.ctx)

    def ref_draws_async(self, first, count, out_ptr, stream=0):
        N.check(self.lib.rg_ref_draws_async(self.ctx, first, count, out_ptr, stream or None), self.ctx)

    def trace_generate_async(self, kind, seed, slot_base, n_slots, stride, votes_ptr, stream=0):
        N.check(self.lib.rg_trace_generate_async(self.ctx, kind, seed, slot_base, n_slots, stride,
                                                 votes_ptr, stream or None), self.ctx)

    def digest_trace_async(self, seed, slot_base, n_slots, digest_stride, digests_ptr, stream=0):
        N.check(self.lib.rg_digest_trace_async(self.ctx, seed, slot_base, n_slots, digest_stride,
                                               digests_ptr, stream or None), self.ctx)

    def wmvc_cluster_async(self, states_ptr, stride, n_slots, slot_base, delivery_seed, max_phases,
                           info_ptr, stats_ptr=0, stream=0):
        N.check(self.lib.rg_wmvc_cluster_async(self.ctx, states_ptr, stride, n_slots, slot_base, delivery_seed,
                                               max_phases, info_ptr, stats_ptr or None, stream or None), self.ctx)

    def wmvc_cluster_bitmaps_async(self, states_ptr, stride, n_slots, slot_base, delivery_seed, max_phases,
                                   info_ptr, decided_ptr, v1_ptr, stats_ptr=0, stream=0):
        N.check(self.lib.rg_wmvc_cluster_bitmaps_async(self.ctx, states_ptr, stride, n_slots, slot_base,
                                                       delivery_seed, max_phases, info_ptr, stats_ptr or None,
                                                       decided_ptr, v1_ptr, stream or None), self.ctx)

    def cluster_bitmap_async(self, info_ptr, n_slots, decided_ptr, v1_ptr, stream=0):
        N.check(self.lib.rg_cluster_bitmap_async(self.ctx, info_ptr, n_slots, decided_ptr, v1_ptr, stream or None),
                self.ctx)

    def cluster_trace_async(self, seed, slot_base, n_slots, stride, states_ptr, stream=0):
        N.check(self.lib.rg_cluster_trace_async(self.ctx, seed, slot_base, n_slots, stride, states_ptr,
                                                stream or None), self.ctx)

    # -- diagnostics (include/rabia_gpu_debug.h) --------------------------------
    def debug_set(self, diag: int):
        N.check(self.lib.rg_debug_set(self.ctx, diag), self.ctx)

    def last_launch(self) -> dict:
        """The kernel shape the last phase step launched (step_impl's pick)."""
        buf = (ctypes.c_uint32 * 6)()
        N.check(self.lib.rg_debug_last_launch(self.ctx, buf), self.ctx)
        kind = ("tiled", "lag", "wmvc")[buf[0]]
        return {"kernel": kind, "shard": bool(buf[1]), "block": buf[2], "words": buf[3], "grid": buf[4],
                "windows": buf[5]}

    def sync(self, stream=0):
        N.check(self.lib.rg_stream_sync(self.ctx, stream or None), self.ctx)
