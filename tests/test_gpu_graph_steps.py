"""Multi-step hipGraph replays (engine.graph_steps: k // 16 replays of a 16-step graph, then k % 16 one-step replays)
against one step per replay, at the Zonos-v0.1 dims, batch 1: runs of steps that are not multiples of
16, and an utterance whose positions cross the 8-chunk -> 24-chunk fused-block boundary at position 1,024, so a run
is cut into form segments mid-graph. The codes must be equal: the graphs hold the same launches in the same order."""
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


@pytest.mark.parametrize("lc,n_new,chunk", [(160, 899, 128), (23, 61, 37)])
def test_graph_steps_16_equals_one_step_per_replay(model, lc, n_new, chunk):
    e = model.engine
    cond = _cond(5, model.config.backbone.d_model, lc)
    out = {}
    for gs in (16, 1):
        e.graph_steps = gs
        out[gs] = model.generate(cond, max_new_tokens=n_new, sampling_params=dict(temperature=0.0),
                                 progress_bar=False, chunk=chunk).cpu()
        e.check_errors()
    e.graph_steps = 16
    assert out[16].shape[-1] == n_new
    if lc + 1 + n_new + 8 > 1024:  # the long case really crossed into the 24-chunk form
        assert e.lib.zmi_attn_block_max_pos(8 | 512) == 1023
    assert torch.equal(out[16], out[1])
