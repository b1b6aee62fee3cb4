"""Calibration: hipBLASLt (torch.matmul) fp16 throughput on conv-equivalent GEMM shapes."""
import torch


def t(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters / 1e3


for (M, K, N) in [(131072, 1728, 192), (131072, 192, 576), (8192, 8192, 8192), (32768, 1728, 192), (524288, 1728, 192)]:
    a = torch.randn(M, K, device="cuda", dtype=torch.float16)
    b = torch.randn(K, N, device="cuda", dtype=torch.float16)
    sec = t(lambda: a @ b)
    print(f"M={M} K={K} N={N}: {sec*1e6:9.1f} us  {2*M*N*K/sec/1e12:7.1f} TF/s", flush=True)
