"""DAC decode / encode time on 128-row (ZMI_OPT_DAC_WIDE = 0), 256-row (2) and per-conv (1, threshold
ZMI_OPT_DAC_WIDE_MIN) time tiles, alternating within one process (one JSON line per case)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zonos_vibes_amd import _lib  # noqa: E402
from zonos_vibes_amd.autoencoder import DACAutoencoder  # noqa: E402


def timed(fn, stream, reps=5):
    fn()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(reps):
        st.record(stream)
        fn()
        en.record(stream)
        en.synchronize()
        best = min(best, st.elapsed_time(en))
    return best


def main():
    dev = torch.device("cuda", 0)
    ae = DACAutoencoder(dev)
    lib = _lib.lib()
    cases = [(0, 256), (2, 256), (1, 256), (1, 128), (1, 512), (0, 256), (2, 256)]
    for frames in (861, 5598):
        codes = torch.randint(0, 1024, (1, 9, frames), generator=torch.Generator().manual_seed(1)).to(dev)
        wav = (torch.rand(frames * 512, generator=torch.Generator().manual_seed(2)) * 1.6 - 0.8).to(dev)
        lat = torch.empty(frames, 1024, dtype=torch.float32, device=dev)
        for wide, mn in cases:
            lib.zmi_set_option(_lib.OPT_DAC_WIDE, wide)
            lib.zmi_set_option(_lib.OPT_DAC_WIDE_MIN, mn)
            dec = timed(lambda: ae.decode(codes), ae.stream)
            enc = timed(lambda: ae.encode_latents(wav, lat), ae.stream) if frames <= 861 else None
            print(json.dumps(dict(frames=frames, wide=wide, wide_min=mn, decode_ms=round(dec, 3),
                                  encode_ms=None if enc is None else round(enc, 3))), flush=True)


if __name__ == "__main__":
    main()
