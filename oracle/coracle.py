"""ctypes binding of the C oracle (oracle/liboracle.so) — TEST INFRASTRUCTURE ONLY.

See framesum_oracle.c for what the oracle restates and how it is pinned.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_DIR = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_DIR, "liboracle.so")
DIGEST_DTYPE = np.dtype([("crc32", "<u4"), ("ip_csum", "<u2"), ("l4_csum", "<u2")])

_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _DIR], check=True)
    return LIB


def load() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB):
        build()
    lib = ctypes.CDLL(LIB)
    vp, u8p = ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint8)
    sz, u16, u32 = ctypes.c_size_t, ctypes.c_uint16, ctypes.c_uint32
    lib.oracle_crc32_bitwise.restype = u32
    lib.oracle_crc32_bitwise.argtypes = [vp, sz]
    lib.oracle_crc32_zlib.restype = u32
    lib.oracle_crc32_zlib.argtypes = [vp, sz]
    lib.oracle_ipv4_checksum.restype = u16
    lib.oracle_ipv4_checksum.argtypes = [vp]
    lib.oracle_udp_checksum.restype = u16
    lib.oracle_udp_checksum.argtypes = [vp, vp, vp, sz]
    lib.oracle_tcp_checksum.restype = u16
    lib.oracle_tcp_checksum.argtypes = [vp, vp, vp, sz, vp, sz]
    lib.oracle_recv_eth.restype = ctypes.c_uint8
    lib.oracle_recv_eth.argtypes = [vp, sz, u32, ctypes.POINTER(u16), ctypes.POINTER(u16)]
    lib.oracle_digest_batch.restype = None
    lib.oracle_digest_batch.argtypes = [vp, vp, vp, u32, u32, ctypes.c_int, ctypes.c_int, vp, vp]
    lib.oracle_fill_batch.argtypes = [vp, vp, vp, u32, u32, u32, vp, vp]
    lib.oracle_fill_batch.restype = None
    lib.oracle_digest_fcs_batch.argtypes = [vp, vp, vp, u32, u32, ctypes.c_int, vp, vp]
    lib.oracle_digest_fcs_batch.restype = None
    lib.oracle_crc791_reset.argtypes = [vp]
    lib.oracle_crc791_write.restype = sz
    lib.oracle_crc791_write.argtypes = [vp, vp, sz]
    lib.oracle_crc791_add_u16.argtypes = [vp, u16]
    lib.oracle_crc791_add_u32.argtypes = [vp, u32]
    lib.oracle_crc791_add_u8.argtypes = [vp, ctypes.c_uint8]
    lib.oracle_crc791_sum16.restype = u16
    lib.oracle_crc791_sum16.argtypes = [vp]
    del u8p
    _lib = lib
    return lib


def _buf(b: bytes):
    a = np.frombuffer(bytes(b) + b"\0", dtype=np.uint8)
    return a, a.ctypes.data_as(ctypes.c_void_p)


def crc32_bitwise(b: bytes) -> int:
    a, p = _buf(b)
    return int(load().oracle_crc32_bitwise(p, len(b)))


def crc32_zlib(b: bytes) -> int:
    a, p = _buf(b)
    return int(load().oracle_crc32_zlib(p, len(b)))


def ipv4_checksum(hdr20: bytes) -> int:
    a, p = _buf(hdr20)
    return int(load().oracle_ipv4_checksum(p))


def recv_eth(frame: bytes, mtu: int = 0) -> tuple[int, int, int]:
    a, p = _buf(frame)
    ipc, l4c = ctypes.c_uint16(), ctypes.c_uint16()
    v = load().oracle_recv_eth(p, len(frame), mtu, ctypes.byref(ipc), ctypes.byref(l4c))
    return int(v), int(ipc.value), int(l4c.value)


class CRC791:
    """ctypes view of the C oracle's CRC791 state machine (eth/crc.go:13-84)."""

    def __init__(self):
        self._st = ctypes.create_string_buffer(8)
        load().oracle_crc791_reset(self._st)

    def write(self, b: bytes) -> int:
        a, p = _buf(b)
        return int(load().oracle_crc791_write(self._st, p, len(b)))

    def add_uint16(self, v: int) -> None:
        load().oracle_crc791_add_u16(self._st, v)

    def add_uint32(self, v: int) -> None:
        load().oracle_crc791_add_u32(self._st, v)

    def add_uint8(self, v: int) -> None:
        load().oracle_crc791_add_u8(self._st, v)

    def sum16(self) -> int:
        return int(load().oracle_crc791_sum16(self._st))


FILL_CSUM = 1
FCS_APPEND = 2
FS_ERR_FCS = 14


def digest_batch(buf: np.ndarray, offsets: np.ndarray, lengths: np.ndarray, mtu: int = 0,
                 use_zlib: bool = True, nthreads: int = 1):
    """Oracle digests for a packed batch: returns (digests[DIGEST_DTYPE], status u8)."""
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    lengths = np.ascontiguousarray(lengths, dtype=np.uint32)
    n = int(lengths.size)
    out = np.zeros(n, dtype=DIGEST_DTYPE)
    st = np.zeros(n, dtype=np.uint8)
    load().oracle_digest_batch(
        buf.ctypes.data_as(ctypes.c_void_p), offsets.ctypes.data_as(ctypes.c_void_p),
        lengths.ctypes.data_as(ctypes.c_void_p), n, mtu, 1 if use_zlib else 0, nthreads,
        out.ctypes.data_as(ctypes.c_void_p), st.ctypes.data_as(ctypes.c_void_p))
    return out, st


def fill_batch(buf: np.ndarray, offsets: np.ndarray, lengths: np.ndarray, mtu: int = 0, flags: int = FILL_CSUM):
    """Oracle TX fill IN PLACE on `buf` (a writable uint8 array): checksums into the frames
    (FILL_CSUM) and/or the FCS after each frame (FCS_APPEND). Returns (digests, status) of
    the frames as they are afterwards."""
    assert buf.dtype == np.uint8 and buf.flags["C_CONTIGUOUS"] and buf.flags["WRITEABLE"]
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    lengths = np.ascontiguousarray(lengths, dtype=np.uint32)
    n = int(lengths.size)
    out = np.zeros(n, dtype=DIGEST_DTYPE)
    st = np.zeros(n, dtype=np.uint8)
    load().oracle_fill_batch(
        buf.ctypes.data_as(ctypes.c_void_p), offsets.ctypes.data_as(ctypes.c_void_p),
        lengths.ctypes.data_as(ctypes.c_void_p), n, mtu, flags,
        out.ctypes.data_as(ctypes.c_void_p), st.ctypes.data_as(ctypes.c_void_p))
    return out, st


def digest_fcs_batch(buf: np.ndarray, offsets: np.ndarray, lengths: np.ndarray, mtu: int = 0, nthreads: int = 1):
    """Oracle RX digests of wire frames that carry a trailing 4-byte FCS (lengths include it)."""
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    lengths = np.ascontiguousarray(lengths, dtype=np.uint32)
    n = int(lengths.size)
    out = np.zeros(n, dtype=DIGEST_DTYPE)
    st = np.zeros(n, dtype=np.uint8)
    load().oracle_digest_fcs_batch(
        buf.ctypes.data_as(ctypes.c_void_p), offsets.ctypes.data_as(ctypes.c_void_p),
        lengths.ctypes.data_as(ctypes.c_void_p), n, mtu, nthreads,
        out.ctypes.data_as(ctypes.c_void_p), st.ctypes.data_as(ctypes.c_void_p))
    return out, st
