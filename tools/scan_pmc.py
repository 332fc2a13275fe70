"""Launch the fused value-head scan at the bench size and at a cold large size,
for rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (one counter per pass)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from handyrl_amd.losses import compute_targets_fused

dev = torch.device('cuda', 0)
for B, T, reps, nsets in ((4096, 32, 5, 1), (1 << 18, 32, 5, 3)):
    g = torch.Generator(device=dev).manual_seed(0)
    sets = [(torch.tanh(torch.randn(B, T, 2, 1, device=dev, generator=g)),
             torch.randint(-1, 2, (B, 1, 2, 1), device=dev, generator=g).float(),
             torch.rand(B, T, 1, 1, device=dev, generator=g),
             torch.rand(B, T, 1, 1, device=dev, generator=g)) for _ in range(nsets)]
    torch.cuda.synchronize()
    for i in range(reps):
        v, ret, rho, cs = sets[i % nsets]
        compute_targets_fused('VTRACE', 'UPGO', v, ret, None, 0.7, 1, rho, cs)
    torch.cuda.synchronize()
    print('B=%d T=%d launches=%d' % (B, T, reps), flush=True)
