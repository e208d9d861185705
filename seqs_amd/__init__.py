"""seqs_amd — MI355X-native frame-checksum engine for the soypat/seqs RecvEth path.

The product is the C-ABI library seqs_amd/lib/libframesum.so (HIP kernels for
gfx950 + include/framesum.h); this package is its Python host binding plus the
synthetic-workload generator used by bench.py.
"""
from .framesum import (  # noqa: F401
    DIGEST_DTYPE,
    EXPORTED_SYMBOLS,
    FCS_APPEND,
    FILL_CSUM,
    FS_ERR_FCS,
    VERDICTS,
    Digest,
    Engine,
    FramesumError,
    Group,
    digest_host_multi,
    lib_path,
    load_library,
    pack_frames,
    shard_count,
    shard_slab_bytes,
    split_digests,
)

__all__ = [
    "DIGEST_DTYPE",
    "EXPORTED_SYMBOLS",
    "FCS_APPEND",
    "FILL_CSUM",
    "FS_ERR_FCS",
    "VERDICTS",
    "Digest",
    "Engine",
    "FramesumError",
    "Group",
    "digest_host_multi",
    "lib_path",
    "load_library",
    "pack_frames",
    "shard_count",
    "shard_slab_bytes",
    "split_digests",
]
