"""GPU: the grouped-decode projection kernel (mpr_dec_gemm, csrc/decode_gemm.hip) behind the
decoder projections of decodes of more than 16 rows (architectures/T5VisionModel.py:200-205).

* values vs an fp64 reference of the same op: max|gpu - ref| <= 2e-6 * max_n sum_k |a w| per
  row (the split-bf16 product is fp32-accurate: ~1e-7 of sum |a w|), with and without the
  split-K finishing launch;
* row-count independence: a row's results are bit-identical whatever else shares the launch (the
  same 16 rows inside 32 / 69 / 128 / 256-row launches): a batch's rows give the same bits in a
  128-row serving-loop group and in a 256-row decode.
"""
import ctypes

import pytest
import torch

from multimodalpromptretrieval_amd import _lib

pytestmark = pytest.mark.gpu
VAL_TOL = 2e-6


def _dec_gemm(A, W, R=None, act=0, rms_w=None, eps=1e-6, out=None):
    M, K = A.shape
    N = W.shape[0]
    C = torch.empty((M, N), device=A.device, dtype=torch.float32) if out is None else out
    _lib.call("mpr_dec_gemm", _lib.ptr(A), A.stride(0), _lib.ptr(W), W.stride(0), _lib.ptr(C),
              C.stride(0), M, N, K, _lib.ptr(R) if R is not None else None,
              R.stride(0) if R is not None else 0, act,
              _lib.ptr(rms_w) if rms_w is not None else None, eps, _lib.stream_ptr(A.device))
    torch.cuda.synchronize()
    return C.cpu()


def _ref(A, W, R=None, act=0, rms_w=None, eps=1e-6):
    A64, W64 = A.double().cpu(), W.double().cpu()
    scale = torch.ones(A.shape[0], 1, dtype=torch.float64)
    if rms_w is not None:
        scale = torch.rsqrt(A64.pow(2).mean(1, keepdim=True) + eps)
        A64 = A64 * rms_w.double().cpu()
    out = (A64 @ W64.T) * scale
    bound = (A64.abs() @ W64.abs().T * scale).max(1, keepdim=True).values
    if act == 2:
        out = out.clamp(min=0)
    if R is not None:
        out = out + R.double().cpu()
    return out, bound


@pytest.mark.parametrize("M,N,K", [(17, 512, 512), (32, 512, 512), (37, 1536, 512),
                                   (128, 512, 2048), (128, 3072, 768), (256, 768, 3072),
                                   (200, 1024, 1024), (128, 2304, 768), (64, 256, 128),
                                   (48, 128, 64), (256, 32, 32)])
def test_dec_gemm_values(device, M, N, K):
    g = torch.Generator().manual_seed(M * 7 + N + K)
    A = torch.randn(M, K, generator=g).to(device)
    W = (torch.randn(N, K, generator=g) * K ** -0.5).to(device)
    R = torch.randn(M, N, generator=g).to(device)
    w = (torch.rand(K, generator=g) + 0.5).to(device)
    for kw in (dict(), dict(R=R), dict(act=2), dict(rms_w=w), dict(rms_w=w, act=2)):
        got = _dec_gemm(A, W, **kw).double()
        ref, bound = _ref(A, W, **kw)
        err = ((got - ref).abs() / bound).max().item()
        assert err <= VAL_TOL, (kw.keys(), err)


def test_dec_gemm_residual_in_place(device):
    """R aliasing C (the decode chain's residual stream updated in place), split-K and not."""
    g = torch.Generator().manual_seed(5)
    for M, N, K in ((64, 512, 512), (128, 2304, 256)):
        A = torch.randn(M, K, generator=g).to(device)
        W = (torch.randn(N, K, generator=g) * 0.05).to(device)
        X = torch.randn(M, N, generator=g).to(device)
        want = _dec_gemm(A, W, R=X.clone())
        assert torch.equal(_dec_gemm(A, W, R=X, out=X), want)


def test_dec_gemm_row_count_independent(device):
    """Rows 32..47 inside launches of 48 / 69 / 128 / 256 rows, bit for bit, in every mode the
    decode chain uses (split-K and single-slice shapes)."""
    g = torch.Generator().manual_seed(11)
    for K, N in ((768, 2304), (3072, 768), (512, 2048)):
        big = torch.randn(256, K, generator=g).to(device)
        W = (torch.randn(N, K, generator=g) * K ** -0.5).to(device)
        R = torch.randn(256, N, generator=g).to(device)
        w = (torch.rand(K, generator=g) + 0.5).to(device)
        rows = slice(32, 48)
        for kw in (dict(), dict(act=2), dict(rms_w=w), dict(rms_w=w, act=2)):
            ref = _dec_gemm(big[:48].contiguous(), W, **kw)[rows]
            for M in (69, 128, 256):
                got = _dec_gemm(big[:M].contiguous(), W, **kw)[rows]
                assert torch.equal(got, ref), (K, N, kw.keys(), M)
        ref = _dec_gemm(big[:48].contiguous(), W, R=R[:48].contiguous())[rows]
        assert torch.equal(_dec_gemm(big[:128].contiguous(), W, R=R[:128].contiguous())[rows], ref)
