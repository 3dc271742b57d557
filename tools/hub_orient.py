"""Config-5 H4 = T0(V1,h0) T1(V1,V2) T2(V2,h1) T3(V2,h0) at 10^9 links: the
sizes that decide the filtered walk's orientation -- forward (S1's T1 out-
degrees, filtered by S23) against reverse (S23's T1 in-degrees, filtered by
S1).  Run on the GPU box."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from das_amd import synthetic  # noqa: E402
from das_amd.database.hip_db import HipDB  # noqa: E402
from tests.test_gpu_fullsize import _dev_pairs  # noqa: E402

db = HipDB(device=0)
arrays = synthetic.powerlaw_kb_device(db.ctx, 1 << 27, 1_000_000_000)
base = len(arrays.type_names)
h0, h1 = base, base + 1
pairs = {k: _dev_pairs(arrays, k) for k in range(4)}
src = {k: (p >> 32) for k, p in pairs.items()}
dst = {k: (p & 0xFFFFFFFF) for k, p in pairs.items()}
n = base + (1 << 27)


def member(k, h):
    m = torch.zeros(n, dtype=torch.bool, device="cuda")
    m[src[k][dst[k] == h]] = True
    return m


s1 = member(0, h0)
s23 = member(2, h1) & member(3, h0)
fwd = s1[src[1]]
rev = s23[dst[1]]
print({"S1": int(s1.sum()), "S23": int(s23.sum()), "T1 distinct": int(src[1].numel()),
       "forward virtual (S1 out-degree)": int(fwd.sum()), "reverse virtual (S23 in-degree)": int(rev.sum()),
       "H4 rows": int((fwd & rev).sum())})
deg = torch.bincount(dst[1][rev], minlength=n)
top = torch.topk(deg, 5)
print("largest S23 in-degrees:", top.values.tolist())
