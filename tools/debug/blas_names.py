"""Print the hipBLASLt kernel names torch.mm picks for the Llama-3-8B projection shapes (run under
rocprofv3 --kernel-trace to read macro tile / wave layout / LDS options from the Tensile names)."""
import torch

for m in (1024, 4096):
    for n, k in ((6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)):
        x = torch.randn(m, k, device="cuda").to(torch.bfloat16)
        w = torch.randn(n, k, device="cuda").to(torch.bfloat16)
        for _ in range(3):
            torch.mm(x, w.t())
torch.cuda.synchronize()
