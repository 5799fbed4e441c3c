"""Encoder2D convolution stack fwd+bwd (torch/MIOpen, fixed batch 32 chunks) NCHW vs NHWC."""
import time
import torch
import torch.nn as nn

torch.manual_seed(0)
chs = [(1, 64, (1, 7), (1, 2), (0, 3)), (64, 128, 3, 2, 1), (128, 128, 3, 1, 1), (128, 256, 3, 2, 1),
       (256, 256, 3, 1, 1), (256, 512, 3, 2, 1), (512, 512, 3, 1, 1), (512, 512, 3, 2, 1),
       (512, 512, 3, 2, 1), (512, 512, (4, 2), 1, 0)]
convs = nn.ModuleList([nn.Conv2d(a, b, k, s, p) for a, b, k, s, p in chs]).cuda()


def run(x, cl):
    h = x
    for c in convs:
        h = torch.nn.functional.leaky_relu(c(h), 0.2)
    return h


for cl in (False, True):
    if cl:
        convs.to(memory_format=torch.channels_last)
    x = torch.randn(32, 1, 128, 128, device="cuda", requires_grad=True)
    if cl:
        x = x.detach().to(memory_format=torch.channels_last).requires_grad_(True)
    for _ in range(3):
        run(x, cl).sum().backward()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        run(x, cl).sum().backward()
    torch.cuda.synchronize()
    print(f"channels_last={cl}: {(time.perf_counter() - t0) / 10 * 1e3:.2f} ms per 32-snapshot chunk fwd+bwd", flush=True)
