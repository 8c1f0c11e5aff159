"""BPEEngine — device bring-up over the C-ABI (replaces src/bpe/engine.js).

Constants mirror engine.js:10-13.  ``pipelines`` stays a name-keyed mapping
(bpe-worker.js logs its length) whose values are the native kernel names.
"""
from __future__ import annotations

import ctypes as C

from . import _lib

WORKGROUP_SIZE = 256
TABLE_SIZE = 2_097_152
INVALID_TOKEN = 0xFFFF_FFFF
MAX_WG_DIM = 65_535


class BPEEngine:
    def __init__(self, device: int = 0):
        self._device = device
        self._ctx = None
        self._limits = None
        self._pipelines = None

    def init(self) -> "BPEEngine":
        if self._ctx is not None:
            return self
        lib = _lib.load()
        ctx = C.c_void_p()
        rc = lib.gbpe_ctx_create(self._device, C.byref(ctx))
        if rc != _lib.GBPE_OK:
            raise _lib.GpuBpeError(rc, f"no usable HIP device {self._device} (gbpe_ctx_create status {rc})")
        self._ctx = ctx
        mb = C.c_uint64()
        _lib.check(lib.gbpe_ctx_limits(ctx, C.byref(mb)), ctx, "limits")
        self._limits = {"maxBufferSize": int(mb.value)}
        self._pipelines = {lib.gbpe_kernel_name(i).decode(): lib.gbpe_kernel_name(i).decode()
                           for i in range(lib.gbpe_kernel_count())}
        return self

    def _assert(self):
        if self._ctx is None:
            raise RuntimeError("BPEEngine not initialized — call engine.init() first")

    @property
    def device(self):
        self._assert()
        return self._ctx

    @property
    def pipelines(self) -> dict:
        self._assert()
        return self._pipelines

    @property
    def limits(self) -> dict:
        self._assert()
        return self._limits

    def close(self):
        if self._ctx is not None:
            _lib.load().gbpe_ctx_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
