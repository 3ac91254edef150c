"""HBM calibration: device-to-device copy of one 8192^2 fp32 buffer (torch
copy kernel) -- the streaming rate a 1-read + 1-write pass can reach."""
import json
import torch
a = torch.rand(8192, 8192, device="cuda")
b = torch.empty_like(a)
c = torch.empty_like(a)
for _ in range(50):
    b.copy_(a); c.copy_(b)
torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(201)]
ev[0].record()
for i in range(100):
    b.copy_(a); ev[2 * i + 1].record()
    a.copy_(b); ev[2 * i + 2].record()
torch.cuda.synchronize()
ms = sorted(ev[i].elapsed_time(ev[i + 1]) for i in range(200))
med = ms[100]
print(json.dumps({"exp": "d2d copy 256 MiB", "ms_med": round(med, 5), "GBs": round(2 * a.numel() * 4 / med / 1e6, 1)}))
