"""How fast is the vendor BLAS (torch.mm -> hipBLASLt/rocBLAS) on the D0 1x1-conv GEMM shapes?
Context for the hand-written kernels: wgrad dW[N,K] = dY^T[N,M] A[M,K]; fwd Y[M,N] = A[M,K] W^T."""
import torch
from torch.profiler import ProfilerActivity, profile

def t(fn, reps=20):
    fn(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / reps

shapes = [(2097152, 16, 96), (2097152, 32, 16), (524288, 24, 144), (524288, 144, 24), (131072, 40, 240),
          (131072, 240, 40), (174592, 64, 64), (174592, 64, 729), (32768, 112, 672), (32768, 672, 112),
          (32768, 480, 80), (8192, 1152, 320), (8192, 1152, 192), (8192, 192, 1152), (8192, 672, 192)]
print(f"{'M':>8} {'K':>5} {'N':>5} | wgrad us  GB/s | fwd us  GB/s")
for M, K, N in shapes:
    a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    dy = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    w = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    out = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    uw = t(lambda: torch.mm(dy.t(), a, out=out))
    uf = t(lambda: torch.mm(a, w.t(), out=y))
    b = M * (K + N) * 2
    print(f"{M:8d} {K:5d} {N:5d} | {uw:8.1f} {b/uw/1e3:6.0f} | {uf:7.1f} {b/uf/1e3:6.0f}", flush=True)
