"""ctypes wrapper of tools/libwalgen.so (config-5 WAL image generator; bench infra)."""
import ctypes
import os
import subprocess

import numpy as np

_DIR = os.path.dirname(os.path.abspath(__file__))
_L = None


def lib():
    global _L
    if _L is None:
        path = os.path.join(_DIR, "libwalgen.so")
        if not os.path.exists(path):
            subprocess.check_call(["make", "-s", "-C", _DIR, "libwalgen.so"])
        L = ctypes.CDLL(path)
        P, U32, U64, I = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
        L.wg_record_sizes.argtypes = [U64, U64, U32, U32, P]
        L.wg_record_sizes.restype = None
        L.wg_plan.argtypes = [P, U64, U32, P, P, P, P, U64, P]
        L.wg_plan.restype = U64
        L.wg_render.argtypes = [U64, P, U64, U32, P, P, P, P, U64, U64, P, I, I]
        L.wg_render.restype = None
        _L = L
    return _L


class WalPlan:
    """Framing plan of `nrec` records (sizes log-uniform in [lo, hi]) into bs-byte blocks."""

    def __init__(self, seed, nrec=None, sizes=None, lo=64, hi=65536, bs=4096):
        L = lib()
        self.seed, self.bs = seed, bs
        if sizes is None:
            sizes = np.zeros(nrec, dtype=np.uint32)
            L.wg_record_sizes(seed, nrec, lo, hi, sizes.ctypes.data)
        self.sizes = np.ascontiguousarray(sizes, dtype=np.uint32)
        n = len(self.sizes)
        self.rec_block = np.zeros(n, dtype=np.uint32)
        self.rec_off = np.zeros(n, dtype=np.uint16)
        self.rec_kind = np.zeros(n, dtype=np.uint8)
        maxp = bs - 21
        cap = int(np.sum((self.sizes.astype(np.uint64) + 17 + maxp - 1) // maxp)) + 2 * n + 2
        self.first_rec = np.zeros(cap, dtype=np.uint32)
        ref = ctypes.c_uint64(0)
        self.nblocks = int(L.wg_plan(self.sizes.ctypes.data, n, bs, self.rec_block.ctypes.data,
                                     self.rec_off.ctypes.data, self.rec_kind.ctypes.data,
                                     self.first_rec.ctypes.data, cap, ctypes.byref(ref)))
        assert self.nblocks <= cap
        self.refused = ref.value

    def render(self, b0, b1, out=None, threads=16, stamp=True):
        if out is None:
            out = np.empty((b1 - b0) * self.bs, dtype=np.uint8)
        assert out.nbytes >= (b1 - b0) * self.bs and out.flags.c_contiguous
        lib().wg_render(self.seed, self.sizes.ctypes.data, len(self.sizes), self.bs,
                        self.rec_block.ctypes.data, self.rec_off.ctypes.data, self.rec_kind.ctypes.data,
                        self.first_rec.ctypes.data, b0, b1, out.ctypes.data, 1 if stamp else 0, threads)
        return out
