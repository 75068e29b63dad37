"""Device-resident pipeline: torch tensors hold the inputs in HBM (PyTorch is
plumbing here: device memory, streams, torch.distributed), libtsg.so runs the
gfx950 kernels on them through the tsg_dev_* C ABI.  No CPU fallback: every
call raises TsgError when the HIP library or device is unavailable.
"""
import ctypes as C

import numpy as np

from ._lib import DevCSR, Stats, check, lib


class DeviceCSR:
    """A CSR matrix resident on a HIP device (torch tensors own the memory)."""

    def __init__(self, m, n, rowptr, col, val):
        self.m, self.n = int(m), int(n)
        self.rowptr, self.col, self.val = rowptr, col, val
        self.nnz = int(col.numel())

    @classmethod
    def from_host(cls, m, n, rowptr, col, val, device="cuda"):
        import torch
        rp = torch.from_numpy(np.ascontiguousarray(rowptr, dtype=np.int32)).to(device)
        ci = torch.from_numpy(np.ascontiguousarray(col, dtype=np.int32)).to(device)
        vv = torch.from_numpy(np.ascontiguousarray(val, dtype=np.float64)).to(device)
        return cls(m, n, rp, ci, vv)

    def struct(self):
        # (built once: the tensors are fixed for the object's life, and a timing
        # loop should not pay for three data_ptr() calls and a ctypes struct per call)
        s = getattr(self, "_struct", None)
        if s is None:
            s = self._struct = DevCSR(self.m, self.n, self.nnz, self.rowpointer_ptr(), self.col.data_ptr(),
                                      self.val.data_ptr())
        return s

    def rowpointer_ptr(self):
        return self.rowptr.data_ptr()

    def to_host(self):
        return (self.m, self.n, self.rowptr.cpu().numpy(), self.col.cpu().numpy(), self.val.cpu().numpy())


class Context:
    """Owns a tsg_context (device, caching allocator, outputs of the last call)."""

    def __init__(self, device=0):
        self.ptr = C.c_void_p()
        check("tsg_context_create", lib().tsg_context_create(device, C.byref(self.ptr)))
        self.device = device

    def close(self):
        if self.ptr:
            lib().tsg_context_destroy(self.ptr)
            self.ptr = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self):
        check("tsg_context_reset", lib().tsg_context_reset(self.ptr))

    def spgemm(self, A, B, tile_m=16, tile_n=16, stream=None, b_sorted=False, raw=False):
        """C = A*B device CSR in -> device CSR out.  Returns (DevCSR struct with
        context-owned pointers, stats dict).  Valid until the next reset().
        b_sorted=True: the caller found B's rows column-sorted (rows_sorted) and B
        has not changed since -- the per-call check is skipped
        (tsg_dev_spgemm_sorted_b).  raw=True: the stats as the tsg_stats struct
        (its as_dict() later: a timing loop keeps the conversion out)."""
        a, b, c, st = A.struct(), B.struct(), DevCSR(), Stats()
        s = C.c_void_p(stream) if stream else None
        if b_sorted:
            check("tsg_dev_spgemm_sorted_b", lib().tsg_dev_spgemm_sorted_b(
                self.ptr, C.byref(a), C.byref(b), 1, tile_m, tile_n, s, C.byref(c), C.byref(st)))
        else:
            check("tsg_dev_spgemm", lib().tsg_dev_spgemm(self.ptr, C.byref(a), C.byref(b), tile_m, tile_n, s,
                                                         C.byref(c), C.byref(st)))
        return c, (st if raw else st.as_dict())

    def rows_sorted(self, M, stream=None):
        """whether every row of the device CSR M is strictly column-sorted"""
        m, out = M.struct(), C.c_int(0)
        s = C.c_void_p(stream) if stream else None
        check("tsg_dev_csr_rows_sorted", lib().tsg_dev_csr_rows_sorted(self.ptr, C.byref(m), s, C.byref(out)))
        return bool(out.value)

    def transpose(self, A, stream=None):
        a, c = A.struct(), DevCSR()
        check("tsg_dev_transpose", lib().tsg_dev_transpose(self.ptr, C.byref(a), stream, C.byref(c)))
        return c

    def to_torch(self, c, device="cuda", stream=None):
        """Copy a context-owned DevCSR into torch tensors (D2D)."""
        import torch
        rp = torch.empty(c.m + 1, dtype=torch.int32, device=device)
        ci = torch.empty(max(c.nnz, 1), dtype=torch.int32, device=device)
        vv = torch.empty(max(c.nnz, 1), dtype=torch.float64, device=device)
        L = lib()
        check("tsg_memcpy_d2d", L.tsg_memcpy_d2d(self.ptr, rp.data_ptr(), c.rowpointer, 4 * (c.m + 1), stream))
        if c.nnz:
            check("tsg_memcpy_d2d", L.tsg_memcpy_d2d(self.ptr, ci.data_ptr(), c.columnindex, 4 * c.nnz, stream))
            check("tsg_memcpy_d2d", L.tsg_memcpy_d2d(self.ptr, vv.data_ptr(), c.value, 8 * c.nnz, stream))
        return DeviceCSR(c.m, c.n, rp, ci[: c.nnz], vv[: c.nnz])

    def view_torch(self, c):
        """Zero-copy torch views of a context-owned DevCSR (valid until the next
        reset of this context), via __cuda_array_interface__."""
        import torch

        class _Buf:
            def __init__(self, ptr, n, typestr):
                self.__cuda_array_interface__ = {"shape": (n,), "typestr": typestr, "data": (ptr or 0, False),
                                                 "version": 2, "strides": None}

        dev = torch.device("cuda", torch.cuda.current_device())
        rp = torch.as_tensor(_Buf(c.rowpointer, c.m + 1, "<i4"), device=dev)
        if c.nnz:
            ci = torch.as_tensor(_Buf(c.columnindex, c.nnz, "<i4"), device=dev)
            vv = torch.as_tensor(_Buf(c.value, c.nnz, "<f8"), device=dev)
        else:
            ci = torch.empty(0, dtype=torch.int32, device=dev)
            vv = torch.empty(0, dtype=torch.float64, device=dev)
        return DeviceCSR(c.m, c.n, rp, ci, vv)

    def to_host(self, c, stream=None):
        rp = np.empty(c.m + 1, dtype=np.int32)
        ci = np.empty(max(c.nnz, 1), dtype=np.int32)
        vv = np.empty(max(c.nnz, 1), dtype=np.float64)
        L = lib()
        check("tsg_memcpy_d2h", L.tsg_memcpy_d2h(self.ptr, rp.ctypes.data, c.rowpointer, 4 * (c.m + 1), stream))
        if c.nnz:
            check("tsg_memcpy_d2h", L.tsg_memcpy_d2h(self.ptr, ci.ctypes.data, c.columnindex, 4 * c.nnz, stream))
            check("tsg_memcpy_d2h", L.tsg_memcpy_d2h(self.ptr, vv.ctypes.data, c.value, 8 * c.nnz, stream))
        return c.m, c.n, rp, ci[: c.nnz], vv[: c.nnz]
