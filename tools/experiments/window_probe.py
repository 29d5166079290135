#!/usr/bin/env python3
"""How many candidates sit just above the k-th neighbour? (sizing the reduced-precision pre-filter)

For the bench corpus (bench.py's mixture), exact top-KW keys of a query sample over the whole corpus
(upper bound for an IVF probe subset), then per window w the count of keys <= key_k + w. Also the
observed |fp16 dot - fp32 dot| / (|x||q|) on those candidates, next to the rigorous bound the
pre-filter uses.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cuvs-rag_amd"))
import numpy as np
import torch

from mivs import ops
from mivs.neighbors import brute_force

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=10_000_000)
ap.add_argument("--queries", type=int, default=1000)
ap.add_argument("--centers", type=int, default=65536)
ap.add_argument("--sigma", type=float, default=0.75)
ap.add_argument("--kw", type=int, default=256)
a = ap.parse_args()
d, k = 768, 10
x = ops.synth_mixture(a.rows, d, 0, n_centers=a.centers, sigma=a.sigma)
q = ops.synth_mixture(a.queries, d, 0, n_centers=a.centers, sigma=a.sigma, row_begin=1 << 40)
bf = brute_force.build(x)
dist, ids = brute_force.search(bf, q, a.kw)
bf.close()
dist = dist.float()
kth = dist[:, k - 1:k]
print(f"rows={a.rows} sigma={a.sigma} centers={a.centers}: key_10 median {kth.median().item():.4f}, "
      f"key_{a.kw} - key_10 median {(dist[:, -1:] - kth).median().item():.4f}", flush=True)
for w in [1e-4, 2.5e-4, 5e-4, 1e-3, 2e-3, 4e-3, 8e-3, 1.6e-2]:
    c = (dist <= kth + w).sum(1).float()
    print(f"window {w:.1e}: survivors mean {c.mean().item():.2f}  p99 {c.quantile(0.99).item():.0f}  "
          f"max {c.max().item():.0f}  (saturated at {a.kw}: {(c >= a.kw).sum().item()})", flush=True)
# observed fp16 / bf16 dot errors on the candidates
xs = x[ids.clamp(min=0)]                          # [Q, KW, d]
e32 = torch.einsum("qkd,qd->qk", xs.double(), q.double())
nrm = xs.double().norm(dim=2) * q.double().norm(dim=1, keepdim=True)
for name, dt in [("fp16", torch.float16), ("bf16", torch.bfloat16)]:
    ea = torch.einsum("qkd,qd->qk", xs.to(dt).double(), q.to(dt).double())
    rel = ((ea - e32).abs() / nrm)
    print(f"{name}: |dot_a - dot|/(|x||q|) max {rel.max().item():.3e} p99.9 {rel.flatten().quantile(0.999).item():.3e}",
          flush=True)
