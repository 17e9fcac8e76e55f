"""A tiny fixed workload for checking rocprofv3 counter output formats: one 256 MB fill."""
import torch
x = torch.empty(1 << 26, dtype=torch.int32, device="cuda")
x.fill_(1)
torch.cuda.synchronize()
print("ok")
