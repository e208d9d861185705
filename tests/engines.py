"""Engines for the GPU parity columns: every kernel variant a caller can choose (fs_ctx_set_kernel
0 / 2 / 3 / 4 / 8) and, through the test library's fs_test_set_kernel_exact, the small-frame kernel for
every launch (16: what the host-staged path runs for short batches; variant 8 itself leaves that
kernel once the reports show long frames, so only this column keeps the small-frame kernel's own
long-frame path under test)."""
SMALL_EXACT = 16
VARIANTS = [4, 2, 3, 0, 8, SMALL_EXACT]
IDS = ["one_pass", "mixed", "segments", "auto", "small", "small_exact"]


def engine_for(variant: int):
    from seqs_amd import Engine
    from seqs_amd.framesum import TEST_LIB_PATH

    if variant == SMALL_EXACT:
        e = Engine(0, lib_path=TEST_LIB_PATH)
        assert e.lib.fs_test_set_kernel_exact(e._ctx, SMALL_EXACT) == 0
        return e
    e = Engine(0)
    e.set_kernel(variant)
    return e
