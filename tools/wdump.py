"""Diagnostic: compare the 16-lane kernel's LDS table image (FS_DIAG_W_DUMP build) with the
host tables (FRAMESUM_LIB=seqs_amd/lib/diag/libframesum_wdump.so)."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import kernel_model as km  # noqa: E402
from seqs_amd import Engine, synth  # noqa: E402

e = Engine(0)
e.set_kernel(3)
dev = torch.device("cuda:0")
b, o, l = synth.uniform_batch(65536, 1500, seed=1)
e.digest_device(torch.from_numpy(b).to(dev), torch.from_numpy(o).to(dev), torch.from_numpy(l).to(dev))
torch.cuda.synchronize()
arr = np.zeros((13 * 4096 + 65536) // 4, dtype=np.uint32)
assert e.lib.fs_debug_read_wdump(arr.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(arr.nbytes)) == 0
names = [("z16", 16), ("z32", 32), ("z48", 48), ("z64", 64), ("z128", 128), ("z192", 192), ("z12", 12), ("z8", 8),
         ("z4", 4), ("z3", 3), ("z2", 2), ("z1", 1), ("z1024", 1024)]
for k, (nm, nb) in enumerate(names):
    tab = arr[k * 1024:(k + 1) * 1024].reshape(4, 256)
    ref = np.array(km.op_table(nb), dtype=np.uint32)
    bad = np.argwhere(tab != ref)
    print(nm, "OK" if bad.size == 0 else f"{len(bad)} bad, first {bad[:4].tolist()}")
ra = arr[13 * 1024:].reshape(256, 64)
z256 = np.array(km.op_table(256), dtype=np.uint32)
for bt in range(4):
    for c in range(8):
        col = ra[:, 8 * bt + c]
        bad = np.nonzero(col != z256[bt])[0]
        if bad.size:
            print(f"regionA table {bt} copy {c}: {bad.size} bad entries, first {bad[:8].tolist()} "
                  f"got {[hex(int(col[i])) for i in bad[:3]]} want {[hex(int(z256[bt][i])) for i in bad[:3]]}")
print("done")
