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


g = torch.cuda.CUDAGraph()
with torch.cuda.stream(sa):
    torch.mm(a, w)  # warm
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=sa):
        for _ in range(500):
            torch.mm(a, w)


def run_g(n):
    with torch.cuda.stream(sa):
        for _ in range(n):
            g.replay()


c = torch.randn(64, 512, device=dev)
v = torch.randn(512, 512, device=dev)


def run_c(n):  # small launches on stream B (as a decode beside the graph)
    with torch.cuda.stream(sb):
        for _ in range(n):
            torch.mm(c, v)


for _ in range(2):
    ta = timed(lambda: run_a(2000))
    tb = timed(lambda: run_b(40))
    tab = timed(lambda: (run_b(40), run_a(2000)))
    print(f"A alone {ta:.2f} ms, B alone {tb:.2f} ms, both {tab:.2f} ms (sum {ta + tb:.2f})",
          flush=True)
    tg = timed(lambda: run_g(4))
    tgb = timed(lambda: (run_b(40), run_g(4)))
    print(f"graph A alone {tg:.2f} ms, with B {tgb:.2f} ms (sum {tg + tb:.2f})", flush=True)
    tc = timed(lambda: run_c(2000))
    tgc = timed(lambda: (run_g(4), run_c(2000)))
    tac = timed(lambda: (run_a(2000), run_c(2000)))
    print(f"small C alone {tc:.2f} ms; graph A + C {tgc:.2f} ms (sum {tg + tc:.2f}); "
          f"eager A + C {tac:.2f} ms (sum {ta + tc:.2f})", flush=True)
