"""Time Encoder2D fwd+bwd at several batch sizes (MIOpen find/compile cost per new shape)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reconstruction-of-pde-without-time-label_amd"))
import torch
import blindno
print("MIOPEN_FIND_MODE", os.environ.get("MIOPEN_FIND_MODE"), "benchmark", torch.backends.cudnn.benchmark, flush=True)
enc = blindno.Encoder2D(25, last_kernel=blindno.Encoder2D.kernel_for_grid(128)).cuda().train()
for n in [int(v) for v in sys.argv[1:]]:
    x = torch.randn(1, n, 1, 128, 128, device="cuda")
    torch.cuda.synchronize(); t = time.perf_counter()
    enc(x).sum().backward()
    torch.cuda.synchronize()
    print(f"n={n}: {time.perf_counter() - t:.3f}s", flush=True)
