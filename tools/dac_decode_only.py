import sys, os, torch
sys.path.insert(0, os.getcwd())
from zonos_vibes_amd.autoencoder import DACAutoencoder
ae = DACAutoencoder("cuda")
codes = torch.randint(0, 1024, (1, 9, 861), generator=torch.Generator().manual_seed(0)).cuda()
for _ in range(3): ae.decode(codes)
torch.cuda.synchronize()
