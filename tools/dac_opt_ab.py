"""DAC decode / encode time under library option sets, alternating within one process (one JSON line per case).

    python tools/dac_opt_ab.py '[{"DAC_STAGE": 0}, {"DAC_STAGE": 1}]' [frames ...]
Each case is a dict of zmi_set_option knobs by their _lib.OPT_<name>; every knob a case names is restored to its
default before the next case. The case list runs twice, so drift shows up as disagreement between the rounds."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zonos_vibes_amd import _lib  # noqa: E402
from zonos_vibes_amd.autoencoder import DACAutoencoder  # noqa: E402
from tools.dac_wide_ab import timed  # noqa: E402


def main():
    cases = json.loads(sys.argv[1])
    frames_list = [int(f) for f in sys.argv[2:]] or [861, 5598]
    dev = torch.device("cuda", 0)
    ae = DACAutoencoder(dev)
    lib = _lib.lib()
    names = sorted({k for c in cases for k in c})
    defaults = {k: lib.zmi_get_option(getattr(_lib, "OPT_" + k)) for k in names}
    for frames in frames_list:
        codes = torch.randint(0, 1024, (1, 9, frames), generator=torch.Generator().manual_seed(1)).to(dev)
        wav = (torch.rand(frames * 512, generator=torch.Generator().manual_seed(2)) * 1.6 - 0.8).to(dev)
        lat = torch.empty(frames, 1024, dtype=torch.float32, device=dev)
        for rnd in range(2):
            for case in cases:
                for k in names:
                    _lib.check(lib.zmi_set_option(getattr(_lib, "OPT_" + k), case.get(k, defaults[k])))
                dec = timed(lambda: ae.decode(codes), ae.stream)
                enc = timed(lambda: ae.encode_latents(wav, lat), ae.stream) if frames <= 861 else None
                print(json.dumps(dict(frames=frames, round=rnd, opts=case, decode_ms=round(dec, 3),
                                      encode_ms=None if enc is None else round(enc, 3))), flush=True)
    for k in names:
        lib.zmi_set_option(getattr(_lib, "OPT_" + k), defaults[k])


if __name__ == "__main__":
    main()
