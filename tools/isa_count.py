"""Static VALU instruction counts of the MD5 hash kernels (k_hash_group<K>)
for bench.py's VALU roofline of the bulk hash (SURVEY.md §8d config 4 asks
MD5 to be reported against the VALU peak as well as HBM).

Compiles das_amd/csrc/hash.hip for gfx950 to assembly and counts the vector
ALU instructions in each k_hash_group<K> body: one thread hashes one
expression (its handle and its composite type, 2 x ceil((33K - 1 + 9) / 64)
MD5 blocks), straight-line code, so the count is the per-expression VALU
work.  Writes profiles/md5_isa.json.

    python tools/isa_count.py
"""
import json
import os
import re
import subprocess
import tempfile
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    with tempfile.TemporaryDirectory() as d:
        asm = os.path.join(d, "hash.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only",
                        "-S", "-o", asm, os.path.join(ROOT, "das_amd", "csrc", "hash.hip")], check=True,
                       capture_output=True)
        s = open(asm).read()
    out = {"what": "VALU instructions per k_hash_group<K> thread (one expression: handle + composite type)",
           "arch": "gfx950", "kernels": {}}
    for m in re.finditer(r"^(_ZN3das12k_hash_groupILi(\d+)EE\w*):", s, re.M):
        k = int(m.group(2))
        body = s[m.end():s.find(".Lfunc_end", m.end())]
        ins = [l.split()[0] for l in body.splitlines() if l.startswith("\t") and not l.strip().startswith((".", ";"))]
        valu = [x for x in ins if x.startswith("v_")]
        blocks = 2 * ((33 * k - 1 + 9 + 63) // 64) if k > 1 else 0
        out["kernels"][f"k_hash_group<{k}>"] = {"valu": len(valu), "salu": sum(x.startswith("s_") for x in ins),
                                               "md5_blocks": blocks,
                                               "valu_per_block": round(len(valu) / blocks, 1) if blocks else None,
                                               "top": Counter(valu).most_common(6)}
    path = os.path.join(ROOT, "profiles", "md5_isa.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")
    print(json.dumps({k: (v["valu"], v["valu_per_block"]) for k, v in out["kernels"].items()}))


if __name__ == "__main__":
    main()
