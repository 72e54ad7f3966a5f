"""Diagnostic: 50 calls of one C3 configuration (B queries, bf16 table,
HHFM) through the default plan — for rocprofv3 --pmc passes."""
import sys

import torch

sys.path.insert(0, ".")

from hhfm_amd import ops

B = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
plan = int(sys.argv[2]) if len(sys.argv) > 2 else 0
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev)
g.manual_seed(2)
nu, ni, k = 957, 4082, 64
M = nu + ni + 12
E = (torch.randn(M, k, generator=g, device=dev) * 0.01).to(torch.bfloat16)
cols = [torch.randint(0, nu, (B,), generator=g, device=dev),
        torch.randint(nu, nu + ni, (B,), generator=g, device=dev)]
off = nu + ni
for c in (7, 2, 3):
    cols.append(torch.randint(off, off + c, (B,), generator=g, device=dev))
    off += c
A = torch.stack(cols, 1).to(torch.int32).contiguous()
for _ in range(50):
    ops.catalog_topk(A, E, ops.MODE_HHFM, 20, nu, ni, 0, None, 0, (2, 5), (0, 0), plan=plan)
torch.cuda.synchronize()
print("ok")
