"""Can timing events recorded during HIP graph capture be read after replay?"""
import torch
x = torch.randn(1 << 24, device="cuda")
y = torch.empty_like(x)
evs = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    evs[0].record()
    torch.mul(x, 2.0, out=y)
    evs[1].record()
    torch.add(x, y, out=y)
    evs[2].record()
for _ in range(3):
    g.replay()
torch.cuda.synchronize()
print("mul ms", evs[0].elapsed_time(evs[1]), "add ms", evs[1].elapsed_time(evs[2]))
