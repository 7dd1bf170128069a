"""The training step's GEMM forms (csrc/train.hip + gemm.hip) against a torch fp64 product of the
same operands (relative Frobenius error 1e-6: fp32 accumulation over K):

* K whose tile count is not a multiple of the pipeline depth (K = 1936 = 121 16-deep tiles, the
  dW products over B*L = 16 x 121 rows; K = 32 on the 32-deep 128x128 tiles) — the masked-tail
  path, which an unmasked extra tile once corrupted;
* mpr_gemm_f32_splitk — K cut into chunks computed side by side (a strided batch of the
  split-bf16 kernel) and summed in order; deterministic (two runs bitwise equal).
"""
import pytest
import torch

from multimodalpromptretrieval_amd import _lib

pytestmark = pytest.mark.gpu


def _gemm(A, W, splits=1, R=None, act=0):
    M, K = A.shape
    N = W.shape[0]
    C = torch.empty(M, N, device=A.device)
    if splits > 1:
        part = torch.empty(splits * M * N, device=A.device)
        _lib.call("mpr_gemm_f32_splitk", _lib.ptr(A), K, _lib.ptr(W), K, _lib.ptr(C), N, M, N, K,
                  _lib.ptr(R), N if R is not None else 0, act, splits, _lib.ptr(part),
                  _lib.stream_ptr())
    else:
        _lib.call("mpr_gemm_f32", _lib.ptr(A), K, _lib.ptr(W), K, _lib.ptr(C), N, M, N, K,
                  _lib.ptr(R), N if R is not None else 0, act, _lib.stream_ptr())
    torch.cuda.synchronize()
    return C


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / b.norm())


def _operands(M, N, K, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return torch.randn(M, K, generator=g), torch.randn(N, K, generator=g)


@pytest.mark.parametrize("M,N,K", [(512, 512, 1936), (512, 1536, 1936), (1536, 512, 32),
                                   (2048, 1024, 32), (128, 512, 48), (512, 2048, 1936)])
def test_gemm_odd_tile_counts(device, M, N, K):
    A, W = _operands(M, N, K, M + N + K)
    got = _gemm(A.to(device), W.to(device))
    assert _rel(got, A.double() @ W.double().t()) < 1e-6


@pytest.mark.parametrize("M,N,K,splits", [(128, 512, 32104, 16), (512, 512, 1936, 4),
                                          (64, 64, 4096, 8), (96, 160, 1000, 3)])
def test_splitk_matches_fp64_and_is_deterministic(device, M, N, K, splits):
    A, W = _operands(M, N, K, M * 3 + K)
    Ad, Wd = A.to(device), W.to(device)
    got = _gemm(Ad, Wd, splits=splits)
    assert _rel(got, A.double() @ W.double().t()) < 1e-6
    assert torch.equal(got, _gemm(Ad, Wd, splits=splits))


def test_splitk_residual_and_relu(device):
    A, W = _operands(192, 256, 2048, 5)
    R = torch.randn(192, 256)
    got = _gemm(A.to(device), W.to(device), splits=4, R=R.to(device), act=2)
    ref = torch.relu(A.double() @ W.double().t()) + R.double()
    assert _rel(got, ref) < 1e-6


def _packed(W):
    N, K = W.shape
    nb = _lib.c_int64()
    _lib.call("mpr_pack_x3_bytes", N, K, _lib.ctypes.byref(nb))
    img = torch.empty(nb.value, dtype=torch.uint8, device=W.device)
    _lib.call("mpr_pack_x3", _lib.ptr(W), N, K, K, _lib.ptr(img), nb.value, _lib.stream_ptr())
    return img


@pytest.mark.parametrize("M,N,K,act,res", [
    (1600, 2304, 768, 0, False),    # ViT qkv, two batches (128x128 packed tiles)
    (1600, 768, 3072, 0, True),     # ViT fc2 + residual (64x64, four A stages: K >= 2048)
    (300, 512, 2052, 2, True),      # 64x64 four A stages with a K tail, odd K tiles
    (1536, 1536, 512, 0, False),    # T5 encoder qkv (64x64)
    (800, 3072, 768, 2, False),     # ViT fc1 shape, relu
    (77, 200, 52, 0, True),         # ragged: N and K tails, K % 16 != 0
    (1000, 1000, 1000, 2, True),    # odd tile counts
    (1300, 2100, 772, 0, True),     # 128x128 tiles (four A stages) with a K tail, odd K tiles
])
def test_packed_weight_gemm_is_bit_identical(device, M, N, K, act, res):
    """mpr_gemm_f32_packed (W fragments from the pack_x3 image, no LDS staging of W) returns the
    same bits as mpr_gemm_f32 on the same operands: the same split of W and the same summation
    order of every output element."""
    A, W = _operands(M, N, K, 7 * M + N + K)
    Ad, Wd = A.to(device), W.to(device)
    R = torch.randn(M, N, device=device) if res else None
    ref = _gemm(Ad, Wd, R=R, act=act)
    img = _packed(Wd)
    C = torch.empty(M, N, device=device)
    _lib.call("mpr_gemm_f32_packed", _lib.ptr(Ad), K, _lib.ptr(Wd), K, _lib.ptr(img), _lib.ptr(C),
              N, M, N, K, _lib.ptr(R), N if R is not None else 0, act, _lib.stream_ptr())
    torch.cuda.synchronize()
    assert torch.equal(C, ref)
