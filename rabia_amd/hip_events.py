"""HIP events with a device-scope release, for the benchmark's stream ordering.

torch.cuda.Event records with HIP's default system-scope release: on this part the
recording queue then pays a full system-scope fence after the kernel it follows (about
7 us per event behind a 2^30-slot step; tools/gap_probe.py). Cross-stream ordering on one
device needs only a device-scope release (hipEventReleaseToDevice), which is what these
events record with. The runtime is the one torch loaded (same soname), so torch streams
are used directly."""
from __future__ import annotations

import ctypes

hipEventDisableTiming = 0x2
hipEventReleaseToDevice = 0x40000000

_hip = None


def _rt():
    global _hip
    if _hip is None:
        import torch  # noqa: F401  (loads the runtime this module must share)
        _hip = ctypes.CDLL("libamdhip64.so.7")
        for fn, args in (("hipEventCreateWithFlags", [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]),
                         ("hipEventRecord", [ctypes.c_void_p, ctypes.c_void_p]),
                         ("hipStreamWaitEvent", [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint]),
                         ("hipEventElapsedTime", [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p]),
                         ("hipEventSynchronize", [ctypes.c_void_p]),
                         ("hipEventQuery", [ctypes.c_void_p]),
                         ("hipEventDestroy", [ctypes.c_void_p])):
            f = getattr(_hip, fn)
            f.argtypes = args
            f.restype = ctypes.c_int
    return _hip


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed (hipError {rc})")


def _stream_ptr(stream) -> ctypes.c_void_p:
    return ctypes.c_void_p(stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream))


class DevEvent:
    """A HIP event recorded with a device-scope release (timing optional)."""

    def __init__(self, timing: bool = False):
        rt = _rt()
        self.h = ctypes.c_void_p()
        flags = hipEventReleaseToDevice | (0 if timing else hipEventDisableTiming)
        _check(rt.hipEventCreateWithFlags(ctypes.byref(self.h), flags), "hipEventCreateWithFlags")

    def record(self, stream) -> None:
        _check(_rt().hipEventRecord(self.h, _stream_ptr(stream)), "hipEventRecord")

    def wait(self, stream) -> None:
        """Make `stream` wait for this event (device side)."""
        _check(_rt().hipStreamWaitEvent(_stream_ptr(stream), self.h, 0), "hipStreamWaitEvent")

    def synchronize(self) -> None:
        _check(_rt().hipEventSynchronize(self.h), "hipEventSynchronize")

    def query(self) -> bool:
        return _rt().hipEventQuery(self.h) == 0

    def elapsed_ms(self, end: "DevEvent") -> float:
        ms = ctypes.c_float()
        _check(_rt().hipEventElapsedTime(ctypes.byref(ms), self.h, end.h), "hipEventElapsedTime")
        return float(ms.value)

    def __del__(self):
        if _hip is not None and self.h:
            _hip.hipEventDestroy(self.h)
            self.h = ctypes.c_void_p()
