"""Emit kats_gen.h (C arrays) from the KAT fixture tests/golden/kats.json (data only)."""
import json
import sys

d = json.load(open(sys.argv[1]))
fr = d["frames"]
print("/* generated from tests/golden/kats.json by gen_kats.py */")
print(f"#define KAT_N {len(fr)}")
print("static const char* kat_hex[KAT_N] = {" + ", ".join(f'"{f["hex"]}"' for f in fr) + "};")
print("static const uint16_t kat_l4[KAT_N] = {" + ", ".join(str(f["l4_csum"]) for f in fr) + "};")
print("static const uint16_t kat_ip[KAT_N] = {" + ", ".join(str(f["ip_csum"]) for f in fr) + "};")
print("static const uint8_t kat_verdict[KAT_N] = {" + ", ".join(str(f["verdict"]) for f in fr) + "};")
