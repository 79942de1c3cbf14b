"""3x3 stride-4 pixel-decoder conv (C2 shape, bf16 channels-last): MIOpen's default solver
vs benchmark-mode Find (torch.backends.cudnn.benchmark).  Prints fwd / bwd ms."""
import sys
import torch
import torch.nn.functional as F

bench = len(sys.argv) > 1 and sys.argv[1] == "1"
torch.backends.cudnn.benchmark = bench
dev = "cuda"
x = torch.randn(4, 256, 256, 256, device=dev, dtype=torch.bfloat16).to(memory_format=torch.channels_last).requires_grad_()
w = (torch.randn(256, 256, 3, 3, device=dev, dtype=torch.bfloat16) * 0.02).to(memory_format=torch.channels_last).requires_grad_()
g = torch.randn(4, 256, 256, 256, device=dev, dtype=torch.bfloat16).to(memory_format=torch.channels_last)
for _ in range(3):
    y = F.conv2d(x, w, padding=1)
    y.backward(g)
torch.cuda.synchronize()
e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
tf = tb = 0.0
n = 10
for _ in range(n):
    e[0].record()
    y = F.conv2d(x, w, padding=1)
    e[1].record()
    y.backward(g)
    e[2].record()
    torch.cuda.synchronize()
    tf += e[0].elapsed_time(e[1])
    tb += e[1].elapsed_time(e[2])
fl = 2 * 4 * 256 * 256 * 256 * 256 * 9
print(f"benchmark={bench}: fwd {tf / n:.3f} ms ({fl / (tf / n) / 1e9:.0f} TF/s), bwd {tb / n:.3f} ms ({2 * fl / (tb / n) / 1e9:.0f} TF/s)")
