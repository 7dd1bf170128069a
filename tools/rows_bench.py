"""gemm_dec (csrc/decode_gemm.hip) launch times over grouped-decode shapes (development aid): a
captured graph of launches cycling over enough weight copies (> 300 MB) that every launch streams
its weights from HBM, as in a t5-base decode step; hipEvents around the replay.  MPR_DEC_BLOCKS
(read once per process) is swept by running one process per value.

usage: python tools/rows_bench.py [targets...]         (default: 192)
       python tools/rows_bench.py --one M N K mode     (one measurement, us per launch)
"""
import os
import subprocess
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodalpromptretrieval_amd import _lib  # noqa: E402

SHAPES = [("base qkv", 2304, 768, "rms"), ("base o", 768, 768, "res"),
          ("base wi", 3072, 768, "rms"), ("base wo", 768, 3072, "res"),
          ("small qkv", 1536, 512, "rms"), ("small o", 512, 512, "res"),
          ("small wi", 2048, 512, "rms"), ("small wo", 512, 2048, "res")]


def one(M, N, K, mode, iters=60):
    dev = torch.device("cuda:0")
    _lib.ensure_device(dev)
    ncopy = max(2, min(iters, int(300e6 / (N * K * 4)) + 1))
    A = torch.randn(M, K, device=dev)
    Ws = [torch.randn(N, K, device=dev) * 0.03 for _ in range(ncopy)]
    C = torch.empty(M, N, device=dev)
    R = torch.randn(M, N, device=dev)
    w = torch.rand(K, device=dev) + 0.5
    s = torch.cuda.Stream(dev)

    def launch(i):
        _lib.call("mpr_dec_gemm", _lib.ptr(A), K, _lib.ptr(Ws[i % ncopy]), K, _lib.ptr(C), N, M,
                  N, K, _lib.ptr(R) if mode == "res" else None, N, 0,
                  _lib.ptr(w) if mode == "rms" else None, 1e-6, _lib.stream_ptr(dev))
    with torch.cuda.stream(s):
        for i in range(3):
            launch(i)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for i in range(iters):
            launch(i)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--one":
        M, N, K = (int(x) for x in sys.argv[2:5])
        print(f"{one(M, N, K, sys.argv[5]):.2f}")
        sys.exit(0)
    targets = sys.argv[1:] or ["192"]
    for rows in (32, 128, 256):
        for name, N, K, mode in SHAPES:
            cells = []
            for tb in targets:
                env = dict(os.environ, MPR_DEC_BLOCKS=tb)
                out = subprocess.run([sys.executable, __file__, "--one", str(rows), str(N),
                                      str(K), mode], capture_output=True, text=True, env=env)
                txt = out.stdout.strip()
                if txt:
                    tf = 2.0 * rows * N * K / (float(txt) * 1e-6) / 1e12
                    cells.append(f"T{tb}: {txt:>6s} us {tf:5.1f} TF")
                else:
                    cells.append(f"T{tb}: err {out.stderr.strip()[-100:]}")
            print(f"M={rows:3d} {name:10s} N={N:5d} K={K:5d} | " + " | ".join(cells), flush=True)
