"""token_wgrad at one shape (default C2 stage-3 fc1: T 16384, N 1536, K 384) x 20, for PMC passes."""
import sys

import torch

sys.path.insert(0, "vision-instance-seg_amd")
from visionseg import ops  # noqa: E402

T, N, K = (int(v) for v in (sys.argv[1:4] if len(sys.argv) >= 4 else (16384, 1536, 384)))
gy = torch.randn(T, N, device="cuda").to(torch.bfloat16)
x = torch.randn(T, K, device="cuda").to(torch.bfloat16)
for _ in range(20):
    ops.token_wgrad(gy, x, torch.bfloat16, bias=True)
torch.cuda.synchronize()
print("ok")
