"""Does hipGraphLaunch block the host, and does a launch from a second host thread proceed while
it does (development aid)?  A graph of N small GEMMs on stream A: the host time of one replay on
an idle GPU; then the replay from a worker thread while the main thread enqueues small GEMMs on
stream B (their host enqueue time and whether the two streams' work overlaps)."""
import sys
import threading
import time

import torch

dev = torch.device("cuda:0")
N = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
a = torch.randn(64, 512, device=dev)
w = torch.randn(512, 512, device=dev)
c = torch.randn(64, 512, device=dev)
sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
g = torch.cuda.CUDAGraph()
with torch.cuda.stream(sa):
    torch.mm(a, w)
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=sa):
        for _ in range(N):
            torch.mm(a, w)
torch.cuda.synchronize()


def replay():
    with torch.cuda.stream(sa):
        g.replay()


for rep in range(3):
    t = time.perf_counter()
    replay()
    th = time.perf_counter() - t
    torch.cuda.synchronize()
    tg = time.perf_counter() - t
    t = time.perf_counter()
    with torch.cuda.stream(sb):
        for _ in range(200):
            torch.mm(c, w)
    tb_host = time.perf_counter() - t
    torch.cuda.synchronize()
    tb = time.perf_counter() - t
    # main thread enqueues B while a worker thread is inside the replay
    t = time.perf_counter()
    thr = threading.Thread(target=replay)
    thr.start()
    time.sleep(0.0005)
    t1 = time.perf_counter()
    with torch.cuda.stream(sb):
        for _ in range(200):
            torch.mm(c, w)
    tb_host2 = time.perf_counter() - t1
    thr.join()
    tj = time.perf_counter() - t
    torch.cuda.synchronize()
    tboth = time.perf_counter() - t
    # same, one thread: replay, then B
    t = time.perf_counter()
    replay()
    with torch.cuda.stream(sb):
        for _ in range(200):
            torch.mm(c, w)
    torch.cuda.synchronize()
    tser = time.perf_counter() - t
    print(f"N={N}: replay host {th * 1e3:.2f} ms, graph {tg * 1e3:.2f} ms; B host {tb_host * 1e3:.2f}"
          f" / total {tb * 1e3:.2f} ms; threaded: B host {tb_host2 * 1e3:.2f} ms, join at "
          f"{tj * 1e3:.2f}, all {tboth * 1e3:.2f} ms; one thread {tser * 1e3:.2f} ms", flush=True)
