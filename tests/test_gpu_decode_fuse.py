"""GPU: the decode chain's q|k|v GEMV with the step's self-attention fused into the same launch
(MPR_DECODE_FUSE_ATTN=1, csrc/gemm.hip SKF_ATTN: the last of each head's tile blocks runs that
head's attention after an agent-scope hand-off).  The fused attention is attention_decode_wave
_kernel's arithmetic (csrc/decode_attn.h), which is bit-identical to the block kernel the unfused
16-row chain launches, so the generated tokens must be bit-identical to the unfused chain's
(t5-small and t5-base geometry, 20 steps, masked sources), and G3 stays exact."""
import os

import pytest
import torch

from multimodalpromptretrieval_amd import synthetic as syn

pytestmark = pytest.mark.gpu


@pytest.fixture
def fuse_env():
    old = os.environ.get("MPR_DECODE_FUSE_ATTN")
    yield
    if old is None:
        os.environ.pop("MPR_DECODE_FUSE_ATTN", None)
    else:
        os.environ["MPR_DECODE_FUSE_ATTN"] = old


@pytest.mark.parametrize("cfg,rows", [(syn.T5Config(), 16), (syn.T5Config(), 5),
                                      (syn.T5_BASE, 16)])
def test_fused_self_attention_tokens_bit_identical(device, fuse_env, cfg, rows):
    from multimodalpromptretrieval_amd.t5 import DeviceT5
    sd = syn.t5_state_dict(3, cfg)
    g = torch.Generator().manual_seed(rows)
    L = 37
    emb = (torch.randn((rows, L, cfg.d_model), generator=g) * 0.5).to(device)
    mask = torch.ones((rows, L))
    mask[0, L - 9:] = 0
    mask = mask.to(device)
    os.environ["MPR_DECODE_FUSE_ATTN"] = "0"
    plain = DeviceT5(sd, device).generate_padded(emb, mask, 20).cpu()
    os.environ["MPR_DECODE_FUSE_ATTN"] = "1"
    dev = DeviceT5(sd, device)
    fused = dev.generate_padded(emb, mask, 20).cpu()
    again = dev.generate_padded(emb, mask, 20).cpu()  # graph replay: counters were reset
    assert torch.equal(plain, fused)
    assert torch.equal(fused, again)
