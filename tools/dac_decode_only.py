import sys, os, torch
sys.path.insert(0, os.getcwd())
from zonos_vibes_amd.autoencoder import DACAutoencoder
from zonos_vibes_amd import _lib
# optional knobs: python tools/dac_decode_only.py [NAME=value ...] (NAME of _lib.OPT_<NAME>)
for kv in sys.argv[1:]:
    k, v = kv.split("=")
    _lib.check(_lib.lib().zmi_set_option(getattr(_lib, "OPT_" + k), int(v)))
ae = DACAutoencoder("cuda")
codes = torch.randint(0, 1024, (1, 9, 861), generator=torch.Generator().manual_seed(0)).cuda()
for _ in range(3): ae.decode(codes)
torch.cuda.synchronize()
