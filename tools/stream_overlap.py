"""Do two streams' kernels run at once on this GPU (development aid)?  Times N launches of a
small-grid GEMV-like torch op on stream A alone, a large GEMM on stream B alone, and both
enqueued together; prints wall times (overlap shows as together < A + B)."""
import time

import torch

dev = torch.device("cuda:0")
a = torch.randn(64, 512, device=dev)
w = torch.randn(512, 512, device=dev)
x = torch.randn(4096, 4096, device=dev)
y = torch.randn(4096, 4096, device=dev)
sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)


def run_a(n):
    with torch.cuda.stream(sa):
        for _ in range(n):
            torch.mm(a, w)


def run_b(n):
    with torch.cuda.stream(sb):
        for _ in range(n):
            torch.mm(x, y)


def timed(f):
    torch.cuda.synchronize()
    t = time.perf_counter()
    f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) * 1e3


for _ in range(2):
    ta = timed(lambda: run_a(2000))
    tb = timed(lambda: run_b(40))
    tab = timed(lambda: (run_b(40), run_a(2000)))
    print(f"A alone {ta:.2f} ms, B alone {tb:.2f} ms, both {tab:.2f} ms (sum {ta + tb:.2f})",
          flush=True)
