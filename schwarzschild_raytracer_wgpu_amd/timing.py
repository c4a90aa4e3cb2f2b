"""HIP event timing without the system-scope release of a default
hipEventRecord (hipEventDisableSystemFence): per-frame event pairs cost
~7 us/frame on the GPU timeline with torch.cuda.Event (tools/ubench/gap_probe.py).

Binds the HIP runtime already loaded in the process (torch's, via the
libamdhip64.so.7 soname) so events live on the same runtime as the streams.
"""
from __future__ import annotations

import ctypes

import torch  # noqa: F401  (loads the HIP runtime first)

_hip = ctypes.CDLL("libamdhip64.so.7")
_hip.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
_hip.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
_hip.hipEventSynchronize.argtypes = [ctypes.c_void_p]
_hip.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p]
_hip.hipEventDestroy.argtypes = [ctypes.c_void_p]
_hip.hipStreamWaitEvent.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint]

hipEventDefault = 0x0
hipEventDisableSystemFence = 0x20000000


class HipEvent:
    def __init__(self, flags: int = hipEventDisableSystemFence):
        self.h = ctypes.c_void_p()
        rc = _hip.hipEventCreateWithFlags(ctypes.byref(self.h), flags)
        if rc != 0:
            raise RuntimeError(f"hipEventCreateWithFlags: {rc}")

    def record(self, stream=None) -> None:
        s = torch.cuda.current_stream().cuda_stream if stream is None else stream
        rc = _hip.hipEventRecord(self.h, ctypes.c_void_p(s))
        if rc != 0:
            raise RuntimeError(f"hipEventRecord: {rc}")

    def elapsed_time(self, end: "HipEvent") -> float:
        """milliseconds from this event to `end` (both recorded, end completed)."""
        _hip.hipEventSynchronize(end.h)
        ms = ctypes.c_float()
        rc = _hip.hipEventElapsedTime(ctypes.byref(ms), self.h, end.h)
        if rc != 0:
            raise RuntimeError(f"hipEventElapsedTime: {rc}")
        return ms.value

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and h.value and _hip is not None:
            try:
                _hip.hipEventDestroy(h)
            except Exception:  # interpreter shutdown
                pass
            self.h = None
