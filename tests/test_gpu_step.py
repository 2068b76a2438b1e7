"""Parity of the persistent decode-step kernel (csrc/zmi_step.hip) at the Zonos-v0.1 layer dims
(d 2048, 16/4 heads, ffn 8192): against the CPU oracle (greedy codes, near-tie aware), against the
per-op launch path (first-step logits), determinism and the hand-off epoch (MI355X only)."""
import pytest
import torch

from zonos_vibes_amd.config import transformer_config, zonos_v01_transformer

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _model(cfg, step_kernel, **kw):
    from zonos_vibes_amd.model import Zonos
    return Zonos.synthetic(cfg, DEV, zero_eos=True, step_kernel=step_kernel, **kw)


def _cond(seed, lc, d=2048):
    import numpy as np
    from zonos_vibes_amd import synthetic as syn
    a = syn.synthetic_conditioning_np(seed, 2, lc, d)
    return torch.from_numpy(a.view(np.int16).copy()).view(torch.bfloat16)


def test_step_kernel_is_selected_at_model_dims():
    m = _model(transformer_config(2048, 1, 16, 4, 8192), True, max_seqlen=64, max_prefill=32)
    assert m.engine.step_args is not None
    # any other geometry stays on the per-op launches (never a silent fallback when asked for)
    with pytest.raises(ValueError):
        _model(transformer_config(512, 1, 4, 1, 1024), True, max_seqlen=64, max_prefill=32)


@pytest.mark.parametrize("lc,n", [(20, 24), (90, 30), (330, 16)])
def test_step_kernel_greedy_matches_oracle(lc, n):
    """2 full-width layers; lc spans 1, 3 and 11 cached positions per attention CU (32 per unit)."""
    from oracle.parity import greedy_divergence
    from oracle.zonos_cpu import OracleZonos
    from tests.helpers import synthetic_weights
    cfg = transformer_config(2048, 2, 16, 4, 8192)
    m = _model(cfg, True, max_seqlen=lc + n + 16, max_prefill=lc + 1)
    cond = _cond(lc, lc)
    m.generate(cond.to(DEV), max_new_tokens=n, sampling_params=dict(temperature=0.0), progress_bar=False)
    om = OracleZonos(cfg, synthetic_weights(cfg, zero_eos=True))
    info = greedy_divergence(m.engine.delayed[0], om, cond, None, n)
    assert info is None or info["step"] > 0, info


def test_step_kernel_logits_match_launch_path_full_model():
    """26 layers: the same decode step (same prefill, same input frame) through the step kernel and
    through the per-op launches. GEMVs are bit-identical by construction; attention sums in a
    different order (fp32), so the logits agree to a small fraction of their range and the greedy
    choices agree wherever the launch path's top-1/top-2 margin is above the bf16 noise floor."""
    from oracle.parity import bf16_ulp
    from zonos_vibes_amd.engine import SamplingParams
    cfg = zonos_v01_transformer()
    outs = []
    for sk in (True, False):
        m = _model(cfg, sk, max_seqlen=256, max_prefill=128)
        e = m.engine
        e.prefill(0, _cond(3, 100).to(DEV), None, 64, SamplingParams(temperature=0.0))
        e.step(1, use_graph=False)
        e.stream.synchronize()
        outs.append(e.logits.clone().cpu())
        del m, e
        torch.cuda.empty_cache()
    ls, ll = outs
    scale = ll.abs().max()
    assert (ls - ll).abs().max() < 2e-2 * scale
    top2 = ll.topk(2, dim=-1).values
    margin = top2[..., 0] - top2[..., 1]
    ulp = torch.tensor([[bf16_ulp(float(v)) for v in row] for row in top2[..., 0]])
    determined = margin > 8 * ulp
    assert determined.any()
    assert torch.equal(ls.argmax(-1)[determined], ll.argmax(-1)[determined])


def test_step_kernel_deterministic_and_epoch_advances():
    cfg = transformer_config(2048, 2, 16, 4, 8192)
    m = _model(cfg, True, max_seqlen=128, max_prefill=64)
    cond = _cond(5, 40).to(DEV)
    e = m.engine
    a = m.generate(cond, max_new_tokens=20, sampling_params=dict(temperature=0.0), progress_bar=False)
    ep0 = int(e.step_ctl[0].item())
    b = m.generate(cond, max_new_tokens=20, sampling_params=dict(temperature=0.0), progress_bar=False)
    assert torch.equal(a, b)
    assert int(e.step_ctl[0].item()) == ep0 + 28   # one epoch per decode step (20 + 8)
    assert int(e.step_ctl[2].item()) == 0
