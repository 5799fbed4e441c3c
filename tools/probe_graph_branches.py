"""Do two parallel branches of a captured graph overlap on this HIP runtime?
Branch = chain of n kernels that each take ~10 us on a few CUs."""
import os
import time
import torch

n = 40
a = torch.zeros(64, 1024, device="cuda")
b = torch.zeros(64, 1024, device="cuda")
main = torch.cuda.Stream()
side = torch.cuda.Stream()


def chain(x):
    for _ in range(n):
        x.mul_(1.0001).add_(0.5).sqrt_()


def build(two):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(main):
        chain(a); chain(b)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=main):
            if two:
                side.wait_stream(main)
                chain(a)
                with torch.cuda.stream(side):
                    chain(b)
                main.wait_stream(side)
            else:
                chain(a)
    return g


for two in (False, True):
    g = build(two)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        g.replay()
    torch.cuda.synchronize()
    print(f"env CAPTURE={os.environ.get('DEBUG_CLR_GRAPH_PACKET_CAPTURE')} QUEUES={os.environ.get('DEBUG_HIP_FORCE_GRAPH_QUEUES')} "
          f"branches={2 if two else 1}: {(time.perf_counter() - t0) / 20 * 1e6:.1f} us/replay", flush=True)
