"""The product library builds, loads and exports exactly the C ABI include/framesum.h declares.
No compute calls here (CPU-only container): only symbol presence, constants and the
no-device error path."""
import ctypes
import os
import re

import pytest

import seqs_amd
from seqs_amd import framesum

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "framesum.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(fs_[a-z_0-9]+)\s*\(", src)))


def test_header_symbols_match_binding():
    assert header_functions() == sorted(framesum.EXPORTED_SYMBOLS)


def test_library_exports_every_header_symbol():
    lib = seqs_amd.load_library()
    for name in header_functions():
        assert hasattr(lib, name), name
    assert lib.fs_abi_version() == 1


def test_nm_exports():
    import subprocess

    out = subprocess.run(["nm", "-D", "--defined-only", seqs_amd.lib_path()], capture_output=True, text=True,
                         check=True).stdout
    syms = {l.split()[-1] for l in out.splitlines() if l.strip()}
    for name in header_functions():
        assert name in syms, name


def test_verdict_codes_match_oracle_header():
    hdr = open(os.path.join(ROOT, "include", "framesum.h")).read()
    orc = open(os.path.join(ROOT, "oracle", "framesum_oracle.h")).read()
    pat = re.compile(r"(FS_[A-Z0-9_]+)\s*=\s*(\d+)")
    a, b = dict(pat.findall(hdr)), dict(pat.findall(orc))
    assert a == b and len(a) == 15
    assert {int(v): k for k, v in a.items()}.keys() == framesum.VERDICTS.keys()


def test_digest_struct_layout():
    assert framesum.DIGEST_DTYPE.itemsize == 8


def test_no_device_error_is_loud():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(framesum.FramesumError):
        framesum.Engine(0)


def test_product_does_not_reference_oracle():
    # the product path must never import, link or call the test oracle
    pat = re.compile(r"(from\s+oracle|import\s+oracle|coracle|pyref|liboracle|oracle_[a-z])")
    for dirpath, _, files in os.walk(os.path.join(ROOT, "seqs_amd")):
        for fn in files:
            if fn.endswith((".py", ".cpp", ".hip", ".h")):
                assert not pat.search(open(os.path.join(dirpath, fn)).read()), fn
    out = __import__("subprocess").run(["nm", "-D", seqs_amd.lib_path()], capture_output=True, text=True).stdout
    assert "oracle_" not in out


def test_multi_rejects_bad_context_lists():
    # argument checks of fs_digest_batch_multi run before any device call
    import ctypes

    lib = framesum.load_library()
    none = ctypes.c_void_p()
    assert lib.fs_digest_batch_multi(None, 1, none, 0, none, none, 1, 0, none, none) == -1
    ctxs = (ctypes.c_void_p * 2)(None, None)
    assert lib.fs_digest_batch_multi(ctxs, 0, none, 0, none, none, 1, 0, none, none) == -1
    assert lib.fs_digest_batch_multi(ctxs, 2, none, 0, none, none, 1, 0, none, none) == -1
