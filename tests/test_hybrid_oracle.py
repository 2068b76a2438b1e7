"""The hybrid-backbone oracle on CPU (parity unpinned: mamba-ssm 2.2.4 is absent, oracle/hybrid_cpu.py).

What can be pinned without the package is pinned here: the scan recurrence equals the published
chunked SSD form (ssd_minimal_discrete); a prefill of S + 1 tokens equals a prefill of S tokens plus
one decode step (Mamba2.forward vs Mamba2.step, the only difference being the bf16 state store);
the generate loop runs end to end.
"""
import torch

from oracle.hybrid_cpu import OracleHybrid, ssd_chunked, ssd_recurrence
from tests.helpers import synthetic_weights
from zonos_vibes_amd.config import tiny_hybrid


def test_scan_recurrence_equals_chunked_ssd():
    g = torch.Generator().manual_seed(0)
    b, l, h, p, n = 2, 77, 3, 8, 16
    x = torch.randn(b, l, h, p, generator=g)
    dt = torch.rand(b, l, h, generator=g) * 0.3
    A = -torch.rand(h, generator=g) * 8 - 1
    B = torch.randn(b, l, n, generator=g)
    C = torch.randn(b, l, n, generator=g)
    y1, s1 = ssd_recurrence(x, dt, A, B, C)
    for chunk in (16, 32, 256):
        y2, s2 = ssd_chunked(x, dt, A, B, C, chunk)
        assert torch.allclose(y1.double(), y2, rtol=1e-4, atol=1e-4)
        assert torch.allclose(s1.double(), s2, rtol=1e-4, atol=1e-4)


def _oracle(cfg, seed=0):
    return OracleHybrid(cfg, synthetic_weights(cfg, seed=seed))


def test_prefill_then_step_equals_longer_prefill():
    cfg = tiny_hybrid()
    o = _oracle(cfg)
    g = torch.Generator().manual_seed(1)
    h = (torch.randn(2, 13, cfg.backbone.d_model, generator=g)).to(torch.bfloat16)
    full = o.backbone(h, o.new_cache(2, 32))
    c = o.new_cache(2, 32)
    o.backbone(h[:, :12], c)
    c["offset"] = 12
    c["lengths"][:] = 12
    last = o.backbone(h[:, 12:], c)
    ref = full[:, 12:].float()
    err = (last.float() - ref).abs().max().item()
    assert err <= 0.05 * ref.abs().max().item(), err


def test_generate_runs_and_is_deterministic():
    cfg = tiny_hybrid()
    o = _oracle(cfg)
    g = torch.Generator().manual_seed(2)
    cond = (torch.randn(2, 6, cfg.backbone.d_model, generator=g)).to(torch.bfloat16)
    a = o.generate(cond, max_new_tokens=12, sampling_params=dict(temperature=0.0))
    b = o.generate(cond, max_new_tokens=12, sampling_params=dict(temperature=0.0))
    assert a.shape[:2] == (1, 9) and torch.equal(a, b)
