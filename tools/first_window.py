"""what the initial mixed-kernel window costs a fresh context.
Device-resident C2 (uniform 1500 B) and C3 (mixed) batches on a fresh variant-0 context: each of the
first 24 launches timed alone (HIP events around the launch, synchronized between launches), with the
kernel it ran (fs_ctx_last_kernel); then the same for a context forced to the one-pass kernel. Prints
one JSON line per (config, context)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from seqs_amd import Engine, synth  # noqa: E402

dev = torch.device("cuda:0")
for cfg in ("c2", "c3"):
    buf, off, ln = synth.uniform_batch(65536, 1500, seed=1) if cfg == "c2" else synth.mixed_batch(65536, seed=2)
    tb, to, tl = (torch.from_numpy(buf).to(dev), torch.from_numpy(off).to(dev), torch.from_numpy(ln).to(dev))
    for variant in (0, 4, 2, 3):
        e = Engine(0)
        e.set_kernel(variant)
        out = torch.empty((65536, 2), dtype=torch.int32, device=dev)
        st = torch.empty((65536,), dtype=torch.uint8, device=dev)
        us, kinds = [], []
        for i in range(24):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            a.record()
            e.digest_device(tb, to, tl, out=out, status=st)
            b.record()
            torch.cuda.synchronize()
            us.append(round(a.elapsed_time(b) * 1e3, 2))
            kinds.append(e.last_kernel())
        e.close()
        print(json.dumps({"config": cfg, "variant": variant, "us": us, "kernel": kinds,
                          "first16_us": round(sum(us[:16]), 1), "last8_avg_us": round(sum(us[16:]) / 8, 2)}))
