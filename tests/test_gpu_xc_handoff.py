"""The fused attention block's chunk-split hand-offs through the XCD's L2 (ZMI_OPT_XC_HANDOFF 0, the default) against
write-through (1): the same granules, so the same codes; and the round-robin workgroup dealing the L2 form relies on
(zmi_xcd_dealing), which the engine checks once per process. An utterance that crosses the 8-chunk -> 24-chunk
boundary at position 1,024 runs both chunk-split forms."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def model():
    from zonos_vibes_amd.config import zonos_v01_transformer
    from zonos_vibes_amd.model import Zonos
    return Zonos.synthetic(zonos_v01_transformer(), DEV, seed=0, zero_eos=True, max_seqlen=1200, max_prefill=170)


def _cond(seed, d, lc):
    import numpy as np

    from zonos_vibes_amd import synthetic as syn
    a = syn.synthetic_conditioning_np(seed, 2, lc, d)
    return torch.from_numpy(a.view(np.int16).copy()).view(torch.bfloat16).to(DEV)


def test_xcd_dealing_is_round_robin(model):
    lib = model.engine.lib
    assert lib.zmi_xcd_dealing(model.engine.sptr) == 1
    assert lib.zmi_get_option(2) == 0  # the engine kept the L2 hand-offs


@pytest.mark.parametrize("lc,n_new", [(160, 899), (40, 200)])
def test_l2_handoffs_decode_the_same_codes_as_write_through(model, lc, n_new):
    from zonos_vibes_amd import _lib
    e = model.engine
    cond = _cond(7, model.config.backbone.d_model, lc)
    out = {}
    try:
        for mode in (1, 0):
            _lib.check(e.lib.zmi_set_option(_lib.OPT_XC_HANDOFF, mode), "set_option")
            e._build_plan()  # graphs hold the launch arguments: capture again
            out[mode] = model.generate(cond, max_new_tokens=n_new, sampling_params=dict(temperature=0.0),
                                       progress_bar=False, chunk=128).cpu()
            e.check_errors()
    finally:
        _lib.check(e.lib.zmi_set_option(_lib.OPT_XC_HANDOFF, 0), "set_option")
        e._build_plan()
    assert out[0].shape[-1] == n_new
    assert torch.equal(out[0], out[1])
