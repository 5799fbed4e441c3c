"""Host cost of hipGraphLaunch vs node count (small kernels), and GPU time per replay."""
import time
import torch

x = torch.zeros(1024, device="cuda")
s = torch.cuda.Stream()
for n in (10, 50, 150, 300):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        x.add_(1)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            for _ in range(n):
                x.add_(1)
    torch.cuda.synchronize()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    reps = 20
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    th = time.perf_counter() - t0
    torch.cuda.synchronize()
    tw = time.perf_counter() - t0
    print(f"nodes={n:4d} host {th / reps * 1e6:8.1f} us/replay ({th / reps / n * 1e6:5.2f} us/node)  wall {tw / reps * 1e6:8.1f} us/replay", flush=True)
