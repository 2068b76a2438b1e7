"""The persistent layer engine (zmi_layer_engine: attention, out_proj, norm2, fc1 + SwiGLU, fc2 and the next
layer's LayerNorm + QKV / norm_f + heads in one launch per layer) against the launch plan it replaces
(zmi_attn_block / zmi_attention + the zmi_gemv_launch ops): logits, the residual rows, q and the KV caches after
each decode step must be bit-identical (reference zonos/backbone/_torch.py:99-152, zonos/model.py:100-116)."""
import pytest
import torch

from zonos_vibes_amd.config import transformer_config

from zonos_vibes_amd import _lib as _zl  # noqa: E402

# a diagnostic form (include/zonos_diag.h): tested when libzonos_diag.so is built (`build --diag`)
pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not _zl.diag_available(), reason="libzonos_diag.so not built")]
DEV = "cuda"


def _cond(seed, lc, d):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(2, lc, d, generator=g) * 0.5).to(torch.bfloat16)


def _model(n_layer, lc, n_new):
    from zonos_vibes_amd.model import Zonos
    if torch.cuda.get_device_properties(0).multi_processor_count < 256:
        pytest.skip("zmi_layer_engine needs 256 CUs")
    cfg = transformer_config(2048, n_layer, 16, 4, 8192)
    return Zonos.synthetic(cfg, DEV, zero_eos=True, max_seqlen=lc + n_new + 16, max_prefill=lc + 8)


def _state(e):
    return dict(logits=e.logits.clone(), x=e.x.clone(), q=e.q.clone(), kc=e.kc.clone(), vc=e.vc.clone())


@pytest.mark.parametrize("lc,steps", [(6, 4), (590, 3), (1019, 9)])
def test_layer_engine_step_bit_identical(lc, steps):
    """Teacher-forced decode steps from one prefill, engine plan against the launch plan, at positions that
    start a 128-key chunk, cross a 512-key softmax block and pass the fused attention forms' reach (1023)."""
    m = _model(3, lc, 48)
    e = m.engine
    cond = _cond(11, lc, 2048).to(DEV)
    from zonos_vibes_amd.engine import SamplingParams
    params = SamplingParams(temperature=0.0)
    outs = {}
    for use in (False, True):
        e.layer_engine = use
        e._build_plan()
        with torch.cuda.stream(e.stream):  # positions past the prefill must not hold the other run's steps
            e.kc.zero_()
            e.vc.zero_()
        e.prefill(0, cond, None, 40, params)
        states = []
        for _ in range(steps):
            e.step(1, slots=1)
            e.stream.synchronize()
            states.append(_state(e))
        e.check_errors()
        outs[use] = states
        e.release(0)
    for k, (a, b) in enumerate(zip(outs[False], outs[True])):
        for name in a:
            assert torch.equal(a[name], b[name]), (k, name)


def test_layer_engine_generate_codes_equal():
    """generate() with the engine plan (graph-captured, 26 launches + QKV + sampler per step at the full depth is
    covered by the bench; here 4 layers) gives the launch plan's codes."""
    m = _model(4, 40, 80)
    cond = _cond(12, 40, 2048).to(DEV)
    params = dict(temperature=0.0)
    e = m.engine
    e.layer_engine = False
    e._build_plan()
    ref = m.generate(cond, max_new_tokens=80, sampling_params=params, progress_bar=False)
    e.layer_engine = True
    e._build_plan()
    got = m.generate(cond, max_new_tokens=80, sampling_params=params, progress_bar=False)
    assert any(k[1] == "engine" for k in e._graphs), sorted(e._graphs)
    e.layer_engine = False
    e._build_plan()
    assert torch.equal(got, ref)
