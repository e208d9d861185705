"""Host-side binding of the framesum C ABI (include/framesum.h).

This is the Python mirror of the reference's batch surface: `digest_batch`
plays the role of running `stacks.PortStack.RecvEth`'s checksum gates plus
`eth.(*IPv4Header).CalculateChecksum` / `(*UDPHeader|*TCPHeader).CalculateChecksumIPv4`
(eth/headers.go:333, :382, :510) over many frames at once, and
`recv_eth_batch` returns the per-frame RecvEth error class
(stacks/portstack.go:120-142). All digests are computed by the gfx950 kernel
in seqs_amd/lib/libframesum.so; there is no CPU fallback — if the library or a
gfx950 device is missing, the calls raise.

torch is used only as device-memory / stream plumbing.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

_LIB_PATH = os.environ.get("FRAMESUM_LIB") or os.path.join(
    os.path.dirname(os.path.abspath(__file__)), "lib", "libframesum.so")

FS_SUCCESS = 0
FS_E_INVALID = -1
FS_E_HIP = -2
FS_E_NOMEM = -3
FS_E_NODEVICE = -4

# fs_verdict (include/framesum.h) — RecvEth error classes (stacks/portstack.go:120-142).
VERDICTS = {
    0: "OK",
    1: "errPacketSmol",
    2: "errPacketExceedsMTU",
    3: "ignored (not IPv4/ARP)",
    4: "ARP",
    5: "errIPVersion",
    6: "errInvalidIHL",
    7: "errBadIPTotalLenOrIHL",
    8: "errUnknownIPProto",
    9: "errTooShortTCPOrUDP",
    10: "errZeroPort",
    11: "errBadUDPLength",
    12: "errBadTCPOffset",
    13: "ErrChecksumTCPorUDP",
    14: "FCS missing or wrong (fs_digest_batch_fcs)",
}

# fs_fill_batch flags
FILL_CSUM = 1
FCS_APPEND = 2
FS_ERR_FCS = 14

# Every symbol include/framesum.h declares (checked by tests/test_abi.py).
EXPORTED_SYMBOLS = (
    "fs_abi_version",
    "fs_device_count",
    "fs_ctx_create",
    "fs_ctx_destroy",
    "fs_last_error",
    "fs_digest_batch",
    "fs_digest_batch_host",
    "fs_fill_batch",
    "fs_fill_batch_host",
    "fs_digest_batch_fcs",
    "fs_digest_batch_multi",
    "fs_ctx_set_kernel",
    "fs_ctx_set_workgroups",
    "fs_ctx_last_kernel",
    "fs_host_alloc",
    "fs_host_free",
    "fs_group_create",
    "fs_group_destroy",
    "fs_group_last_error",
    "fs_shard_count",
    "fs_shard_slab_bytes",
    "fs_digest_batch_sharded",
    "fs_deinterleave",
)

DIGEST_DTYPE = np.dtype([("crc32", "<u4"), ("ip_csum", "<u2"), ("l4_csum", "<u2")])


class FramesumError(RuntimeError):
    pass


_lib = None
_libs: dict = {}

# The test library: the same sources built with -DFS_TEST_HOOKS (seqs_amd/csrc/Makefile), which adds
# the fault-injection setters fs_test_set_fault / fs_test_group_set_fault. Only tests load it; the
# product library has no such hook (and reads no environment variable for one).
TEST_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "test", "libframesum_test.so")


def lib_path() -> str:
    return _LIB_PATH


def load_library(path: Optional[str] = None) -> ctypes.CDLL:
    """Load libframesum.so (raises if it was not built: no fallback path exists). `path`: another
    build of the same ABI (the test library, TEST_LIB_PATH)."""
    global _lib
    if path is None and _lib is not None:
        return _lib
    p = path or _LIB_PATH
    if p in _libs:
        return _libs[p]
    if not os.path.exists(p):
        raise FramesumError(f"{p} is missing — run __graft_entry__.build() (or make -C seqs_amd/csrc)")
    lib = ctypes.CDLL(p)
    vp, u32, u64, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int32
    lib.fs_abi_version.restype = u32
    lib.fs_abi_version.argtypes = []
    lib.fs_device_count.restype = ctypes.c_int
    lib.fs_device_count.argtypes = []
    lib.fs_ctx_create.restype = i32
    lib.fs_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
    lib.fs_ctx_destroy.restype = i32
    lib.fs_ctx_destroy.argtypes = [vp]
    lib.fs_last_error.restype = ctypes.c_char_p
    lib.fs_last_error.argtypes = [vp]
    lib.fs_digest_batch.restype = i32
    lib.fs_digest_batch.argtypes = [vp, vp, vp, vp, u32, u32, vp, vp, vp]
    lib.fs_digest_batch_host.restype = i32
    lib.fs_digest_batch_host.argtypes = [vp, vp, u64, vp, vp, u32, u32, vp, vp]
    lib.fs_ctx_set_kernel.restype = i32
    lib.fs_fill_batch.argtypes = [vp, vp, vp, vp, u32, u32, u32, vp, vp, vp]
    lib.fs_fill_batch.restype = ctypes.c_int32
    lib.fs_fill_batch_host.argtypes = [vp, vp, u64, vp, vp, u32, u32, u32, vp, vp]
    lib.fs_fill_batch_host.restype = ctypes.c_int32
    lib.fs_digest_batch_fcs.argtypes = [vp, vp, vp, vp, u32, u32, vp, vp, vp]
    lib.fs_digest_batch_fcs.restype = ctypes.c_int32
    lib.fs_ctx_set_kernel.argtypes = [vp, ctypes.c_int]
    if hasattr(lib, "fs_ctx_set_workgroups"):  # (absent from builds before round 4: same-box A/B runs)
        lib.fs_ctx_set_workgroups.restype = i32
        lib.fs_ctx_set_workgroups.argtypes = [vp, ctypes.c_int]
    lib.fs_ctx_last_kernel.argtypes = [vp]
    lib.fs_ctx_last_kernel.restype = ctypes.c_int
    lib.fs_digest_batch_multi.restype = i32
    lib.fs_digest_batch_multi.argtypes = [ctypes.POINTER(vp), ctypes.c_int, vp, u64, vp, vp, u32, u32, vp, vp]
    lib.fs_host_alloc.restype = i32
    lib.fs_host_alloc.argtypes = [vp, u64, ctypes.POINTER(vp)]
    lib.fs_host_free.restype = i32
    lib.fs_host_free.argtypes = [vp, vp]
    lib.fs_group_create.restype = i32
    lib.fs_group_create.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.POINTER(vp)]
    lib.fs_group_destroy.restype = i32
    lib.fs_group_destroy.argtypes = [vp]
    lib.fs_group_last_error.restype = ctypes.c_char_p
    lib.fs_group_last_error.argtypes = [vp]
    lib.fs_shard_count.restype = u64
    lib.fs_shard_count.argtypes = [u64, u32, u32]
    lib.fs_shard_slab_bytes.restype = u64
    lib.fs_shard_slab_bytes.argtypes = [u64, u32]
    lib.fs_digest_batch_sharded.restype = i32
    lib.fs_digest_batch_sharded.argtypes = [vp, ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(vp), u64, u32,
                                            vp, vp]
    lib.fs_deinterleave.restype = i32
    lib.fs_deinterleave.argtypes = [vp, vp, u32, u64, vp, vp, vp]
    if hasattr(lib, "fs_test_set_fault"):  # test library only
        lib.fs_test_set_fault.restype = i32
        lib.fs_test_set_fault.argtypes = [vp, ctypes.c_long]
        lib.fs_test_group_set_fault.restype = i32
        lib.fs_test_group_set_fault.argtypes = [vp, ctypes.c_long]
        lib.fs_test_group_set_fault_gather.restype = i32
        lib.fs_test_group_set_fault_gather.argtypes = [vp, ctypes.c_long]
        lib.fs_test_set_kernel_exact.restype = i32
        lib.fs_test_set_kernel_exact.argtypes = [vp, ctypes.c_int]
        lib.fs_test_last_host_path.restype = ctypes.c_int
        lib.fs_test_last_host_path.argtypes = [vp]
    _libs[p] = lib
    if path is None:
        _lib = lib
    return lib


@dataclass
class Digest:
    """One frame's results (fs_digest + verdict)."""

    crc32: int
    ip_csum: int
    l4_csum: int
    verdict: int

    @property
    def err(self) -> Optional[str]:
        return None if self.verdict == 0 else VERDICTS.get(self.verdict, f"verdict {self.verdict}")


class Engine:
    """One framesum context on one GPU (fs_ctx). Not thread-safe, like the C ctx."""

    def __init__(self, device: int = 0, lib_path: Optional[str] = None):
        self.lib = load_library(lib_path)
        self.device = device
        ctx = ctypes.c_void_p()
        st = self.lib.fs_ctx_create(device, ctypes.byref(ctx))
        if st != FS_SUCCESS:
            raise FramesumError(f"fs_ctx_create({device}) failed ({st}): {self.lib.fs_last_error(None).decode()}")
        self._ctx = ctx
        self._pinned: set[int] = set()

    def close(self) -> None:
        if getattr(self, "_ctx", None):
            for addr in list(self._pinned):
                self.lib.fs_host_free(self._ctx, ctypes.c_void_p(addr))
            self._pinned.clear()
            self.lib.fs_ctx_destroy(self._ctx)
            self._ctx = None

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass

    def _check(self, st: int, what: str) -> None:
        if st != FS_SUCCESS:
            raise FramesumError(f"{what} failed ({st}): {self.lib.fs_last_error(self._ctx).decode()}")

    # kernel variants (fs_ctx_set_kernel): results are identical, only the speed differs
    KERNEL_AUTO, KERNEL_MIXED, KERNEL_SEGMENTS, KERNEL_ONE_PASS, KERNEL_SMALL = 0, 2, 3, 4, 8

    def set_kernel(self, variant: int) -> None:
        """0 (KERNEL_AUTO): automatic (the mixed-length kernel after a batch that had mixed-length
        tiles, the one-pass kernel otherwise, the small-frame kernel for short-frame traffic); 2 (KERNEL_MIXED): the
        mixed-length kernel, which splits the long frames of mixed-length tiles into pieces; 3 (KERNEL_SEGMENTS):
        the segment kernel (a tile's frames cut into equal chunks, one per 4-lane group; slower on C3,
        DESIGN.md §3.14); 4 (KERNEL_ONE_PASS): the one-pass kernel (block-aligned rows); 8 (KERNEL_SMALL): the small-frame kernel (one lane per frame) preferred: it runs until a
        launch reports a frame over 128 B, then the automatic choice until short traffic resumes.
        The automatic choice itself moves to the small-frame kernel after 16 launches seen to run
        with no frame over 128 B (include/framesum.h). A TX fill never runs the small-frame kernel.
        Any other value raises."""
        self._check(self.lib.fs_ctx_set_kernel(self._ctx, int(variant)), "fs_ctx_set_kernel")

    def set_workgroups(self, workgroups: int) -> None:
        """fs_ctx_set_workgroups: 0 (default) one 16-wave workgroup per CU; k > 0 at most k
        workgroups per launch, each wave then streams several tiles back to back."""
        self._check(self.lib.fs_ctx_set_workgroups(self._ctx, int(workgroups)), "fs_ctx_set_workgroups")

    def last_kernel(self) -> int:
        """The variant (2, 3, 4 or 8) this context's latest launch ran (0 before its first launch). With
        variant 0 the first 16 launches run the mixed-length kernel (2); it stays chosen while its
        batches have mixed-length tiles, uniform traffic then moves to the one-pass kernel (4)."""
        v = self.lib.fs_ctx_last_kernel(self._ctx)
        if v < 0:
            self._check(v, "fs_ctx_last_kernel")
        return int(v)

    # ---- device-resident path (torch tensors as device memory) -------------
    def digest_device(self, frames, offsets, lengths, mtu: int = 0, out=None, status=None, stream=None):
        """Device-resident batch digest.

        frames: uint8 CUDA tensor; offsets: int64 CUDA tensor; lengths: int32
        CUDA tensor. Returns (out, status): out is an int32 tensor of shape
        (n, 2) holding the raw fs_digest words ([:,0] = crc32 bits,
        [:,1] = ip_csum | l4_csum << 16), status a uint8 tensor. Asynchronous
        on `stream` (default: torch's current stream).
        """
        import torch

        n = int(lengths.numel())
        assert frames.is_cuda and offsets.is_cuda and lengths.is_cuda, "device-resident path needs CUDA tensors"
        assert frames.dtype == torch.uint8 and offsets.dtype == torch.int64 and lengths.dtype == torch.int32
        assert offsets.numel() == n and frames.is_contiguous() and offsets.is_contiguous() and lengths.is_contiguous()
        if out is None:
            out = torch.empty((n, 2), dtype=torch.int32, device=frames.device)
        if status is None:
            status = torch.empty((n,), dtype=torch.uint8, device=frames.device)
        if stream is None:
            stream = torch.cuda.current_stream(frames.device)
        st = self.lib.fs_digest_batch(
            self._ctx,
            ctypes.c_void_p(frames.data_ptr()),
            ctypes.c_void_p(offsets.data_ptr()),
            ctypes.c_void_p(lengths.data_ptr()),
            n,
            mtu,
            ctypes.c_void_p(out.data_ptr()),
            ctypes.c_void_p(status.data_ptr()),
            ctypes.c_void_p(stream.cuda_stream),
        )
        self._check(st, "fs_digest_batch")
        return out, status

    def prepare_digest(self, frames, offsets, lengths, mtu: int = 0, out=None, status=None, stream=None, op="digest",
                       flags: int = FILL_CSUM):
        """A prepared digest_device call: the tensors are checked and the C arguments built ONCE,
        and the returned callable enqueues the same fs_digest_batch (op "fcs": fs_digest_batch_fcs;
        op "fill": fs_fill_batch with `flags`) again on every call, with no per-call validation or
        marshalling. For a caller that digests a fixed set of resident batches into fixed result
        slots over and over (a NIC ring's buffers, the bench's rotated batches): the per-call host
        cost is the C call alone. The callable keeps the tensors alive and raises FramesumError on
        a failed call."""
        n, out, status, stream = self._device_args(frames, offsets, lengths, out, status, stream)
        name = {"digest": "fs_digest_batch", "fcs": "fs_digest_batch_fcs", "fill": "fs_fill_batch"}[op]
        fn = self.lib[name]  # a fresh function pointer with no argtypes: the ctypes objects go as built
        vp, u32 = ctypes.c_void_p, ctypes.c_uint32
        mid = (u32(n), u32(mtu), u32(flags)) if op == "fill" else (u32(n), u32(mtu))
        args = (vp(self._ctx.value), vp(frames.data_ptr()), vp(offsets.data_ptr()), vp(lengths.data_ptr()), *mid,
                vp(out.data_ptr()), vp(status.data_ptr()), vp(stream.cuda_stream))
        keep = (frames, offsets, lengths, out, status, stream)

        def call():
            if self._ctx is None:  # (the context was closed: its pointer in `args` is gone)
                raise FramesumError(f"{name}: the engine was closed")
            st = fn(*args)
            if st:
                self._check(st, name)
            return keep[3], keep[4]

        return call

    def _device_args(self, frames, offsets, lengths, out, status, stream):
        import torch

        n = int(lengths.numel())
        assert frames.is_cuda and offsets.is_cuda and lengths.is_cuda, "device-resident path needs CUDA tensors"
        assert frames.dtype == torch.uint8 and offsets.dtype == torch.int64 and lengths.dtype == torch.int32
        assert offsets.numel() == n and frames.is_contiguous() and offsets.is_contiguous() and lengths.is_contiguous()
        if out is None:
            out = torch.empty((n, 2), dtype=torch.int32, device=frames.device)
        if status is None:
            status = torch.empty((n,), dtype=torch.uint8, device=frames.device)
        if stream is None:
            stream = torch.cuda.current_stream(frames.device)
        return n, out, status, stream

    def fill_device(self, frames, offsets, lengths, mtu: int = 0, flags: int = FILL_CSUM, out=None, status=None,
                    stream=None):
        """TX fill IN PLACE on the device tensor `frames` (fs_fill_batch): FILL_CSUM writes the
        IPv4 and TCP/UDP checksums into every frame RecvEth would checksum, FCS_APPEND the
        CRC-32 after each frame (4 spare bytes needed there). Returns (out, status) as
        digest_device would report them for the written frames."""
        n, out, status, stream = self._device_args(frames, offsets, lengths, out, status, stream)
        st = self.lib.fs_fill_batch(
            self._ctx, ctypes.c_void_p(frames.data_ptr()), ctypes.c_void_p(offsets.data_ptr()),
            ctypes.c_void_p(lengths.data_ptr()), n, mtu, flags, ctypes.c_void_p(out.data_ptr()),
            ctypes.c_void_p(status.data_ptr()), ctypes.c_void_p(stream.cuda_stream))
        self._check(st, "fs_fill_batch")
        return out, status

    def digest_fcs_device(self, frames, offsets, lengths, mtu: int = 0, out=None, status=None, stream=None):
        """RX digest of wire frames with a trailing FCS (fs_digest_batch_fcs): lengths include
        the FCS; status FS_ERR_FCS (14) where it is missing or wrong."""
        n, out, status, stream = self._device_args(frames, offsets, lengths, out, status, stream)
        st = self.lib.fs_digest_batch_fcs(
            self._ctx, ctypes.c_void_p(frames.data_ptr()), ctypes.c_void_p(offsets.data_ptr()),
            ctypes.c_void_p(lengths.data_ptr()), n, mtu, ctypes.c_void_p(out.data_ptr()),
            ctypes.c_void_p(status.data_ptr()), ctypes.c_void_p(stream.cuda_stream))
        self._check(st, "fs_digest_batch_fcs")
        return out, status

    def deinterleave_device(self, gathered, nshards: int, n: int, out=None, status=None, stream=None):
        """Global frame order from nshards gathered round-robin slabs (fs_deinterleave):
        `gathered` is a uint8 CUDA tensor of nshards * shard_slab_bytes(n, nshards) bytes, slab k =
        shard k's digests then its verdicts. Returns (out (n, 2) int32, status (n,) uint8)."""
        import torch

        assert gathered.is_cuda and gathered.dtype == torch.uint8 and gathered.is_contiguous()
        assert gathered.numel() >= nshards * shard_slab_bytes(n, nshards)
        if out is None:
            out = torch.empty((n, 2), dtype=torch.int32, device=gathered.device)
        if status is None:
            status = torch.empty((n,), dtype=torch.uint8, device=gathered.device)
        if stream is None:
            stream = torch.cuda.current_stream(gathered.device)
        st = self.lib.fs_deinterleave(self._ctx, ctypes.c_void_p(gathered.data_ptr()), nshards, n,
                                      ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(status.data_ptr()),
                                      ctypes.c_void_p(stream.cuda_stream))
        self._check(st, "fs_deinterleave")
        return out, status

    # ---- host-staged path (numpy in, numpy out) -----------------------------
    def host_empty(self, shape, dtype=np.uint8) -> np.ndarray:
        """A numpy array in pinned host memory (fs_host_alloc), freed with the array."""
        import weakref

        dtype = np.dtype(dtype)
        nbytes = max(1, int(np.prod(shape)) * dtype.itemsize)
        ptr = ctypes.c_void_p()
        self._check(self.lib.fs_host_alloc(self._ctx, ctypes.c_uint64(nbytes), ctypes.byref(ptr)), "fs_host_alloc")
        raw = (ctypes.c_uint8 * nbytes).from_address(ptr.value)
        arr = np.frombuffer(raw, dtype=np.uint8, count=nbytes)[: int(np.prod(shape)) * dtype.itemsize]
        arr = arr.view(dtype).reshape(shape)
        # freed when the array goes away, or by close() (arrays must not outlive the engine)
        self._pinned.add(ptr.value)
        weakref.finalize(raw, Engine._free_pinned, weakref.ref(self), ptr.value)
        return arr

    @staticmethod
    def _free_pinned(engine_ref, addr: int) -> None:
        eng = engine_ref()
        if eng is not None and getattr(eng, "_ctx", None) and addr in eng._pinned:
            eng._pinned.discard(addr)
            eng.lib.fs_host_free(eng._ctx, ctypes.c_void_p(addr))

    def digest_host(self, frames: np.ndarray, offsets: np.ndarray, lengths: np.ndarray, mtu: int = 0,
                    out: Optional[np.ndarray] = None, status: Optional[np.ndarray] = None):
        """Host buffers in, host results out (fs_digest_batch_host): chunked H2D / kernel / D2H
        pipeline over the context's streams. Returns (digests, status)."""
        frames = np.ascontiguousarray(frames, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        lengths = np.ascontiguousarray(lengths, dtype=np.uint32)
        n = int(lengths.size)
        assert offsets.size == n, "offsets and lengths must describe the same frames"
        if out is None:
            out = np.zeros(n, dtype=DIGEST_DTYPE)
        if status is None:
            status = np.zeros(n, dtype=np.uint8)
        assert out.dtype == DIGEST_DTYPE and out.size >= n and status.dtype == np.uint8 and status.size >= n
        assert out.flags["C_CONTIGUOUS"] and status.flags["C_CONTIGUOUS"], "out / status are written in place"
        if n == 0:
            return out, status
        st = self.lib.fs_digest_batch_host(
            self._ctx,
            frames.ctypes.data_as(ctypes.c_void_p),
            frames.nbytes,
            offsets.ctypes.data_as(ctypes.c_void_p),
            lengths.ctypes.data_as(ctypes.c_void_p),
            n,
            mtu,
            out.ctypes.data_as(ctypes.c_void_p),
            status.ctypes.data_as(ctypes.c_void_p),
        )
        self._check(st, "fs_digest_batch_host")
        return out, status

    def fill_host(self, frames: np.ndarray, offsets: np.ndarray, lengths: np.ndarray, mtu: int = 0,
                  flags: int = FILL_CSUM):
        """TX fill IN PLACE on a writable host uint8 array (fs_fill_batch_host). Returns
        (digests, status) of the frames as written."""
        assert isinstance(frames, np.ndarray) and frames.dtype == np.uint8 and frames.flags["C_CONTIGUOUS"]
        assert frames.flags["WRITEABLE"], "fill_host writes into `frames`"
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        lengths = np.ascontiguousarray(lengths, dtype=np.uint32)
        n = int(lengths.size)
        assert offsets.size == n, "offsets and lengths must describe the same frames"
        out = np.zeros(n, dtype=DIGEST_DTYPE)
        status = np.zeros(n, dtype=np.uint8)
        if n == 0:
            return out, status
        st = self.lib.fs_fill_batch_host(
            self._ctx, frames.ctypes.data_as(ctypes.c_void_p), frames.nbytes,
            offsets.ctypes.data_as(ctypes.c_void_p), lengths.ctypes.data_as(ctypes.c_void_p), n, mtu, flags,
            out.ctypes.data_as(ctypes.c_void_p), status.ctypes.data_as(ctypes.c_void_p))
        self._check(st, "fs_fill_batch_host")
        return out, status

    # ---- reference-shaped surface -------------------------------------------
    def digest_batch(self, frames: Sequence[bytes], mtu: int = 0) -> list[Digest]:
        """Batched equivalent of RecvEth's checksum work for each frame (host lists)."""
        buf, offsets, lengths = pack_frames(frames)
        dig, st = self.digest_host(buf, offsets, lengths, mtu)
        return [Digest(int(d["crc32"]), int(d["ip_csum"]), int(d["l4_csum"]), int(s)) for d, s in zip(dig, st)]

    def recv_eth_batch(self, frames: Sequence[bytes], mtu: int = 0) -> list[Optional[str]]:
        """Per-frame RecvEth error class (None = checksum OK), like RecvEth's return."""
        return [d.err for d in self.digest_batch(frames, mtu)]

    def calculate_headers_batch(self, frames: Sequence[bytes], mtu: int = 0, append_fcs: bool = False) -> list[bytes]:
        """The checksum part of the reference's TX header calculation (stacks/port_tcp.go:178,
        :193; dhcp_client.go:479, :486) for many frames: each frame with its IPv4 and TCP/UDP
        checksum fields filled (frames RecvEth would not checksum come back unchanged), and
        with its FCS appended when `append_fcs`."""
        room = 4 if append_fcs else 0
        buf, offsets, lengths = pack_frames([bytes(f) + bytes(room) for f in frames])
        lengths = lengths - np.uint32(room)
        self.fill_host(buf, offsets, lengths, mtu, FILL_CSUM | (FCS_APPEND if append_fcs else 0))
        return [bytes(buf[int(o) : int(o) + int(l) + room]) for o, l in zip(offsets, lengths)]



def digest_host_multi(engines: Sequence["Engine"], frames: np.ndarray, offsets: np.ndarray, lengths: np.ndarray,
                      mtu: int = 0):
    """Host buffers in, host results out, over several contexts at once (fs_digest_batch_multi):
    contiguous byte-balanced blocks of frames, one per engine (one per GPU), each on its own
    host thread and H2D / kernel / D2H pipeline. Returns (digests, status) in batch order."""
    assert len(engines) > 0 and len({id(e) for e in engines}) == len(engines), "engines must be distinct"
    lib = engines[0].lib
    frames = np.ascontiguousarray(frames, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    lengths = np.ascontiguousarray(lengths, dtype=np.uint32)
    n = int(lengths.size)
    assert offsets.size == n
    out = np.zeros(n, dtype=DIGEST_DTYPE)
    status = np.zeros(n, dtype=np.uint8)
    if n == 0:
        return out, status
    ctxs = (ctypes.c_void_p * len(engines))(*[e._ctx for e in engines])
    st = lib.fs_digest_batch_multi(ctxs, len(engines), frames.ctypes.data_as(ctypes.c_void_p), frames.nbytes,
                                   offsets.ctypes.data_as(ctypes.c_void_p), lengths.ctypes.data_as(ctypes.c_void_p),
                                   n, mtu, out.ctypes.data_as(ctypes.c_void_p), status.ctypes.data_as(ctypes.c_void_p))
    if st != FS_SUCCESS:
        # every entry point clears its context's message first: only failing contexts hold one
        msgs = "; ".join(f"ctx {k}: {m}" for k, e in enumerate(engines)
                         if (m := e.lib.fs_last_error(e._ctx).decode()))
        raise FramesumError(f"fs_digest_batch_multi failed ({st}): {msgs}")
    return out, status

def shard_count(n: int, nshards: int, shard: int) -> int:
    """Frames of shard `shard` when n global frames go round-robin over nshards shards (C ABI)."""
    return int(load_library().fs_shard_count(n, nshards, shard))


def shard_slab_bytes(n: int, nshards: int) -> int:
    """Bytes of one shard's gathered slab: ceil(n/N) digests then ceil(n/N) verdicts, 256-B aligned."""
    return int(load_library().fs_shard_slab_bytes(n, nshards))


class Group:
    """One host process driving several GPUs (fs_group): a context, a stream and an RCCL
    communicator per device. `digest_sharded` runs fs_digest_batch_sharded: every device digests
    its round-robin shard chunk by chunk, grouped ncclSend/ncclRecv bring each chunk's digests to
    the first device, a de-interleave kernel restores global order there."""

    def __init__(self, devices: Sequence[int], lib_path: Optional[str] = None):
        self.lib = load_library(lib_path)
        self.devices = [int(d) for d in devices]
        arr = (ctypes.c_int * len(self.devices))(*self.devices)
        g = ctypes.c_void_p()
        st = self.lib.fs_group_create(arr, len(self.devices), ctypes.byref(g))
        if st != FS_SUCCESS:
            raise FramesumError(f"fs_group_create({self.devices}) failed ({st}): "
                                f"{self.lib.fs_group_last_error(None).decode()}")
        self._g = g

    def close(self) -> None:
        if getattr(self, "_g", None):
            self.lib.fs_group_destroy(self._g)
            self._g = None

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass

    def digest_sharded(self, shards, n: int, mtu: int = 0, out=None, status=None):
        """shards[k] = (frames, offsets int64, lengths int32) CUDA tensors on devices[k] holding
        shard k (fs_shard_count(n, N, k) frames). Returns (out (n, 2) int32, status (n,) uint8)
        on devices[0], in global frame order (synchronous)."""
        import torch

        N = len(self.devices)
        assert len(shards) == N
        vp = ctypes.c_void_p
        fr, of, ln = (vp * N)(), (vp * N)(), (vp * N)()
        for k, (f, o, l) in enumerate(shards):
            assert f.dtype == torch.uint8 and o.dtype == torch.int64 and l.dtype == torch.int32
            assert f.is_contiguous() and o.is_contiguous() and l.is_contiguous()
            assert l.numel() == shard_count(n, N, k) and o.numel() == l.numel()
            assert f.device.index == self.devices[k]
            fr[k], of[k], ln[k] = f.data_ptr(), o.data_ptr(), l.data_ptr()
        dev = torch.device("cuda", self.devices[0])
        if out is None:
            out = torch.empty((n, 2), dtype=torch.int32, device=dev)
        if status is None:
            status = torch.empty((n,), dtype=torch.uint8, device=dev)
        st = self.lib.fs_digest_batch_sharded(self._g, fr, of, ln, n, mtu, vp(out.data_ptr()), vp(status.data_ptr()))
        if st != FS_SUCCESS:
            raise FramesumError(f"fs_digest_batch_sharded failed ({st}): {self.lib.fs_group_last_error(self._g).decode()}")
        return out, status


def pack_frames(frames: Sequence[bytes], align: int = 4):
    """Pack a list of frames into one buffer (each frame at an `align`-aligned offset)."""
    lengths = np.fromiter((len(f) for f in frames), dtype=np.uint32, count=len(frames))
    step = (lengths.astype(np.uint64) + np.uint64(align - 1)) // np.uint64(align) * np.uint64(align)
    offsets = np.zeros(len(frames), dtype=np.uint64)
    if len(frames) > 1:
        offsets[1:] = np.cumsum(step[:-1])
    total = int(offsets[-1] + step[-1]) if len(frames) else 0
    buf = np.zeros(total + 16, dtype=np.uint8)
    for f, o in zip(frames, offsets):
        buf[int(o) : int(o) + len(f)] = np.frombuffer(f, dtype=np.uint8)
    return buf, offsets, lengths


def split_digests(out_words: np.ndarray):
    """(n,2) int32 raw digest words -> (crc32 u32, ip_csum u16, l4_csum u16) numpy arrays."""
    w = np.ascontiguousarray(out_words).view(np.uint32).reshape(-1, 2)
    return w[:, 0].copy(), (w[:, 1] & 0xFFFF).astype(np.uint16), (w[:, 1] >> 16).astype(np.uint16)
