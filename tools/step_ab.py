"""A/B of the C2 decode step (live utterance, graph replay, HIP events) across engine plan options.

    python tools/step_ab.py

For each option set: a fresh prefill of the bench conditioning, then bench.time_decode_step's window
of 64 steps around the C2 mean position. Also checks that every option decodes the same codes.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from zonos_vibes_amd import _lib  # noqa: E402
from zonos_vibes_amd.config import zonos_v01_transformer  # noqa: E402
from zonos_vibes_amd.model import Zonos  # noqa: E402

OPTIONS = [dict(prefetch_blocks=0), dict(prefetch_blocks=192, prefetch_fc1_mb=0),
           dict(prefetch_blocks=192, prefetch_fc1_mb=16), dict(prefetch_blocks=192, prefetch_fc1_mb=32),
           dict(prefetch_blocks=192, prefetch_fc1_mb=64), dict(prefetch_blocks=96, prefetch_fc1_mb=32),
           dict(prefetch_blocks=0)]


def main():
    global OPTIONS
    if len(sys.argv) > 1:  # a JSON list of option dicts replaces the default set
        OPTIONS = json.loads(sys.argv[1])
    dev = torch.device("cuda", 0)
    cfg = zonos_v01_transformer()
    m = Zonos.synthetic(cfg, dev, seed=0, zero_eos=True, max_seqlen=bench.LC + bench.N_NEW + 9,
                        max_prefill=bench.LC + 1)
    cond = bench.cond_tensor(1, cfg.backbone.d_model, dev)
    e = m.engine
    ref = None
    for opt in OPTIONS:
        for k, v in opt.items():
            if k.startswith("opt_"):  # library launch knobs: opt_gemv_spread -> zmi_set_option(OPT_GEMV_SPREAD)
                _lib.check(e.lib.zmi_set_option(getattr(_lib, "OPT_" + k[4:].upper()), int(v)), k)
            else:
                setattr(e, k, v)
        e._build_plan()
        at = int(os.environ.get("STEP_AT", "0")) or None  # decode position of the timed window (default: C2's mean)
        bench.time_decode_step(m, cond, steps=16, at=at)  # warm-up (graph capture)
        us, pos = bench.time_decode_step(m, cond, at=at)
        codes = m.generate(cond, max_new_tokens=48, sampling_params=dict(temperature=0.0), progress_bar=False)
        same = None if ref is None else bool(torch.equal(codes, ref))
        ref = codes if ref is None else ref
        e.check_errors()
        print(json.dumps(dict(options=opt, step_us=round(us, 1), pos=pos, codes_equal_first=same)), flush=True)


if __name__ == "__main__":
    main()
