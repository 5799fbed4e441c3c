"""Encoder2D fwd+bwd with fixed-size conv chunks (one MIOpen problem per layer) and
torch BatchNorm over the full batch: time per new batch size."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reconstruction-of-pde-without-time-label_amd"))
os.environ.pop("MIOPEN_FIND_MODE", None)
import torch
import torch.nn.functional as F
import blindno
os.environ.pop("MIOPEN_FIND_MODE", None)
K = int(os.environ.get("CHUNK", "64"))
enc = blindno.Encoder2D(25, last_kernel=blindno.Encoder2D.kernel_for_grid(128)).cuda().train()
blocks = [enc.convblock1, enc.convblock2_1, enc.convblock2_2, enc.convblock3_1, enc.convblock3_2,
          enc.convblock4_1, enc.convblock4_2, enc.convblock7_1, enc.convblock7_2, enc.convblock7_3]

def fwd(x):
    n = x.shape[0]
    npad = -(-n // K) * K
    x = F.pad(x, (0, 0, 0, 0, 0, 0, 0, npad - n))
    for b in blocks:
        conv, bn = b.layers[0], b.layers[1]
        z = torch.cat([conv(x[i:i + K]) for i in range(0, npad, K)])
        zv = bn(z[:n])
        x = F.leaky_relu(torch.cat([zv, z[n:]]), 0.2)
    return enc.linear(x[:n].flatten(1))

for n in [int(v) for v in sys.argv[1:]]:
    x = torch.randn(n, 1, 128, 128, device="cuda")
    torch.cuda.synchronize(); t = time.perf_counter()
    fwd(x).sum().backward()
    torch.cuda.synchronize()
    print(f"K={K} n={n}: {time.perf_counter() - t:.3f}s", flush=True)
