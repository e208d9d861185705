"""CPU oracle for the framesum parity tests — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package, and only as the checker / the timed CPU baseline; the product
(seqs_amd/, libframesum.so) never imports, links or calls it.
"""
